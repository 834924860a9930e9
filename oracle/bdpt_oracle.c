/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Not part of the product.
 *
 * A plain-C CPU restatement of the reference render path of sim186/gpu_bidirectional_raytracer
 * (src/device.cu, src/MersenneTwister_kernel.cu, src/smallpt_cpu.c, src/display_func.c), used
 * as the parity checker for the HIP kernels in gpu_bidirectional_raytracer_amd/csrc and as the
 * `cpu_baseline` leg of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it; the product never links it.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference itself is unbuildable in this image (it needs
 * the CUDA toolkit/runtime and does not compile as shipped -- SURVEY.md 8(c)), so this
 * restatement is pinned by the known answers the survey recorded from the reference's own
 * kernels (MT607 table hashes and values, the cornell VLP dev_lp[1]) and by glibc rand().
 *
 * Floating-point contract (both here and in the HIP kernels): IEEE fp32 with no contraction
 * (-ffp-contract=off), correctly rounded division and sqrt, the two fp64 steps of the camera
 * ray kept in fp64 (device.cu:565-566,594), and sinf/cosf/powf with correctly-rounded
 * semantics, evaluated as (float)f((double)x).  The reference calls the CUDA float overloads
 * cos/sin/pow (<=2 ulp implementations of the same functions).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/bdpt.h"

typedef bdpt_vec Vec;
typedef bdpt_ray Ray;
typedef bdpt_sphere Sphere;
typedef bdpt_lightpath LightPath;
typedef bdpt_camera Camera;

#define RAND_N      7684096u            /* smallpt_cpu.c:67-69                 */
#define EPSILON     0.01f               /* geom.h:6                            */
#define FLOAT_PI    3.14159265358979323846f /* geom.h:7                        */
#define MT_RNG_COUNT 4096
#define MT_NN 19                        /* MersenneTwister.h:30-39             */
#define MT_MM 9
#define N_PER_RNG 1876

static const float tol = (float)0.0001; /* device.cu:8, cons.h:9              */

/* ---- vec.h macros, restated as functions with the same operation order ---- */
static inline Vec vinit(float a, float b, float c) { Vec v; v.x = a; v.y = b; v.z = c; return v; }
static inline Vec vadd(Vec a, Vec b) { return vinit(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline Vec vsub(Vec a, Vec b) { return vinit(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline Vec vmul(Vec a, Vec b) { return vinit(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline Vec vsmul(float k, Vec b) { return vinit(k * b.x, k * b.y, k * b.z); }
static inline float vdot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline Vec vnorm(Vec v) { float l = 1.f / sqrtf(vdot(v, v)); return vsmul(l, v); }
static inline Vec vxcross(Vec a, Vec b) {
    return vinit(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline int viszero(Vec v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }
static inline float clampf01(float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); }
static inline float o_sinf(float x) { return (float)sin((double)x); }
static inline float o_cosf(float x) { return (float)cos((double)x); }
static inline float o_powf(float x, float y) { return (float)pow((double)x, (double)y); }
static inline int toInt(float x) { return (int)(o_powf(clampf01(x), 1.f / 2.2f) * 255.f + .5f); }

/* ---------------------------------------------------------------------------------------- */
/* MT607 lane generator: RandomGPU MersenneTwister_kernel.cu:63-110, seeded as seedMTGPU :39-51 */
void oracle_mt607(const uint32_t *params /* 4096 x {matrix_a,mask_b,mask_c,seed} */,
                  uint32_t seed, float *out /* RAND_N */)
{
#pragma omp parallel for schedule(static)
    for (int tid = 0; tid < MT_RNG_COUNT; tid++) {
        uint32_t mt[MT_NN];
        const uint32_t matrix_a = params[4 * tid + 0];
        const uint32_t mask_b = params[4 * tid + 1];
        const uint32_t mask_c = params[4 * tid + 2];
        mt[0] = seed;                                   /* seedMTGPU overwrites .seed */
        for (int s = 1; s < MT_NN; s++)
            mt[s] = 1812433253u * (mt[s - 1] ^ (mt[s - 1] >> 30)) + (uint32_t)s;
        int st = 0;
        uint32_t next = mt[0];
        for (int k = 0; k < N_PER_RNG; k++) {
            int s1 = st + 1 >= MT_NN ? st + 1 - MT_NN : st + 1;
            int sm = st + MT_MM >= MT_NN ? st + MT_MM - MT_NN : st + MT_MM;
            uint32_t cur = next;
            next = mt[s1];
            uint32_t y = (cur & 0xFFFFFFFEu) | (next & 0x1u);
            y = mt[sm] ^ (y >> 1) ^ ((y & 1u) ? matrix_a : 0u);
            mt[st] = y;
            st = s1;
            y ^= y >> 12;
            y ^= (y << 7) & mask_b;
            y ^= (y << 15) & mask_c;
            y ^= y >> 18;
            out[tid + k * MT_RNG_COUNT] = ((float)y + 1.0f) / 4294967296.0f;
        }
    }
}

/* ---------------------------------------------------------------------------------------- */
/* Intersection: device.cu:80-154 (closest hit scans from the last sphere down, `<` keeps ties) */
static inline float sphere_intersect(const Sphere *s, const Ray *r)
{
    Vec op = vsub(s->p, r->o);
    float b = vdot(op, r->d);
    float det = b * b - vdot(op, op) + s->rad * s->rad;
    if (det < 0.f) return 0.f;
    det = sqrtf(det);
    float t = b - det;
    if (t > EPSILON) return t;
    t = b + det;
    return t > EPSILON ? t : 0.f;
}

typedef struct { uint64_t segments, closest, shadow, sphere_tests, samples, diffuse, rng_reads, refr; } ostats;

static inline int intersect(const Sphere *sp, unsigned n, const Ray *r, float *t, unsigned *id,
                            ostats *st)
{
    float inf = *t = 1e20f;
    if (st) { st->closest++; st->sphere_tests += n; }
    for (unsigned i = n; i--;) {
        const float d = sphere_intersect(&sp[i], r);
        if (d != 0.f && d < *t) { *t = d; *id = i; }
    }
    return *t < inf;
}

static inline int intersect_p(const Sphere *sp, unsigned n, const Ray *r, float maxt, ostats *st)
{
    if (st) st->shadow++;
    for (unsigned i = n; i--;) {
        if (st) st->sphere_tests++;
        const float d = sphere_intersect(&sp[i], r);
        if (d != 0.f && d < maxt) return 1;
    }
    return 0;
}

static inline int intersect_p_vacuum(const Sphere *sp, unsigned n, const Ray *r, float maxt,
                                     ostats *st)
{
    if (st) st->shadow++;
    for (unsigned i = n; i--;) {
        if (st) st->sphere_tests++;
        const float d = sphere_intersect(&sp[i], r);
        if (d != 0.f && d < maxt && viszero(sp[i].e)) return 1;
    }
    return 0;
}

/* UniformSampleSphereDevice device.cu:157-165 */
static inline Vec uniform_sample_sphere(float u1, float u2)
{
    const float zz = 1.f - 2.f * u1;
    const float q = 1.f - zz * zz;
    const float r = sqrtf(0.f > q ? 0.f : q);
    const float phi = 2.f * FLOAT_PI * u2;
    return vinit(r * o_cosf(phi), r * o_sinf(phi), zz);
}

/* Cosine-weighted hemisphere direction about w (device.cu:190-212, 357-380, 676-699). */
static inline Vec cosine_dir(Vec w, float u_phi, float u_r2)
{
    float r1 = 2.f * FLOAT_PI * u_phi;
    float r2 = u_r2;
    float r2s = sqrtf(r2);
    Vec a = fabsf(w.x) > .1f ? vinit(0.f, 1.f, 0.f) : vinit(1.f, 0.f, 0.f);
    Vec u = vnorm(vxcross(a, w));
    Vec v = vxcross(w, u);
    u = vsmul(o_cosf(r1) * r2s, u);
    v = vsmul(o_sinf(r1) * r2s, v);
    Vec nd = vadd(u, v);
    w = vsmul(sqrtf(1 - r2), w);
    return vadd(nd, w);
}

/* VecMultiply device.cu:10-42 (the light pass only). */
static inline void vec_multiply(Vec *io, Vec m)
{
    float t;
    if (io->x != 0.f && m.x != 0.f) { t = io->x * m.x; if (!(t <= tol || io->x == t)) io->x = t; } else io->x = 0.f;
    if (io->y != 0.f && m.y != 0.f) { t = io->y * m.y; if (!(t <= tol || io->y == t)) io->y = t; } else io->y = 0.f;
    if (io->z != 0.f && m.z != 0.f) { t = io->z * m.z; if (!(t <= tol || io->z == t)) io->z = t; } else io->z = 0.f;
}

/* ---------------------------------------------------------------------------------------- */
/* Light pass: UpdateRendering2 smallpt_cpu.c:311-359 -> GetRayKernel device.cu:167-219 and
 * RadianceLightTracingKernel device.cu:222-455 (DEPTH = 1), for every emitter in order.
 * `rnd` must already hold the MT table for seed current_sample*5 (the kernel is re-run per
 * light with the same seed, so one table serves all lights).  lp[] must be pre-initialised
 * (zeros: survey Appendix A.4); entries a light does not write keep their previous value. */
void oracle_light_pass(const Sphere *sp, unsigned n, const float *rnd, int current_sample,
                       LightPath *lp)
{
    for (unsigned li = 0; li < n; li++) {
        const Sphere light = sp[li];
        if (viszero(light.e)) continue;
#pragma omp parallel for schedule(static)
        for (int ind = 0; ind < BDPT_LIGHT_POINTS; ind++) {
            /* GetRayKernel, seed_id = 0 (smallpt_cpu.c:330) */
            unsigned i = (unsigned)(current_sample * 5 + ind * 4) % (RAND_N - 4u);
            unsigned j = i + 2;
            Vec usp = uniform_sample_sphere(rnd[j], rnd[i]);
            Vec spt = vadd(vsmul(light.rad, usp), light.p);
            Vec normal = vnorm(vsub(spt, light.p));
            Ray ray;
            ray.o = spt;
            ray.d = cosine_dir(normal, rnd[i + 1], rnd[j + 1]);

            /* RadianceLightTracingKernel */
            Vec thr = vsmul(0.25f, light.e);                      /* :248,268 e * (1./4)    */
            float t; unsigned id = 0;
            if (!intersect(sp, n, &ray, &t, &id, NULL)) {         /* escaped: :279-292      */
                Vec nor = vsmul((float)(-1. / light.rad), vsub(ray.o, light.p));
                lp[ind].hp = ray.o;
                lp[ind].rad = vsmul(0.5f, light.e);
                lp[ind].nl = nor;
                continue;
            }
            const Sphere *obj = &sp[id];
            if (!viszero(obj->e)) continue;                       /* :296-298               */
            Vec hit = vadd(ray.o, vsmul(t, ray.d));
            Vec nrm = vnorm(vsub(hit, obj->p));
            const float dp = vdot(nrm, ray.d);
            Vec nl = vsmul(-1.f * (dp > 0 ? 1 : -1), nrm);
            if (obj->refl == BDPT_DIFF) {                         /* :314-337               */
                vec_multiply(&thr, obj->c);
                lp[ind].hp = hit;
                lp[ind].rad = thr;
                lp[ind].nl = nl;
            }
            /* SPEC / REFR: throughput changes but DEPTH=1 ends the loop with no store. */
        }
    }
}

/* ---------------------------------------------------------------------------------------- */
/* Camera terms that RadiancePathTracingKernel recomputes per thread (device.cu:572-592). */
typedef struct { Vec ux, uy, ud; float tx, ty, tz; } campre;

static campre camera_pre(const Camera *c)
{
    campre p;
    p.ux = vnorm(c->x);
    p.uy = vnorm(c->y);
    p.ud = vnorm(c->dir);
    p.tx = vdot(vnorm(vsmul(-1.f, c->x)), c->orig);
    p.ty = vdot(vnorm(vsmul(-1.f, c->y)), c->orig);
    p.tz = vdot(vsmul(-1.f, c->dir), c->orig);        /* :591-592: no vnorm on this one */
    return p;
}

/* SampleLightsDevice device.cu:457-542 (NEE over every emitter + one VLP, blended 1/2). */
static Vec sample_lights(const Sphere *sp, unsigned n, const float *rnd, Vec hit, Vec nl,
                         unsigned nn, const LightPath *lp, int vlp, ostats *st)
{
    Vec result = vinit(0.f, 0.f, 0.f);
    const unsigned dk = nn + 1, dj = nn + 2;
    for (unsigned i = 0; i < n; i++) {
        const Sphere *light = &sp[i];
        if (viszero(light->e)) continue;
        Vec usp = uniform_sample_sphere(rnd[dk], rnd[dj]);
        Vec spt = vadd(vsmul(light->rad, usp), light->p);
        Ray sr; sr.o = hit;
        sr.d = vsub(spt, hit);
        const float len = sqrtf(vdot(sr.d, sr.d));
        sr.d = vsmul(1.f / len, sr.d);
        float wo = vdot(sr.d, usp);
        if (wo > 0.f) continue;
        wo = -wo;
        const float wi = vdot(sr.d, nl);
        if (wi > 0.f && !intersect_p(sp, n, &sr, len - EPSILON, st)) {
            const float s = (4.f * FLOAT_PI * light->rad * light->rad) * wi * wo / (len * len);
            result = vadd(result, vsmul(s, light->e));
        }
    }
    Vec vres = vinit(0.f, 0.f, 0.f);
    {
        const LightPath *v = &lp[vlp];
        Ray sr; sr.o = hit;
        sr.d = vsub(v->hp, hit);
        const float len = sqrtf(vdot(sr.d, sr.d));
        sr.d = vsmul(1.f / len, sr.d);
        float wo = vdot(sr.d, v->nl);
        if (!(wo > 0.f)) {
            wo = -wo;
            const float wi = vdot(sr.d, nl);
            if (wi > 0.f && !intersect_p_vacuum(sp, n, &sr, len - EPSILON, st))
                vres = vadd(vres, vsmul(wi * wo, v->rad));
        }
    }
    vres = vsmul(1.f, vres);                            /* 1./(DEPTH*MAX_VLP) */
    result = vadd(result, vres);
    return vsmul(0.5f, result);
}

static inline int n_lights_of(const Sphere *sp, unsigned n)
{
    int k = 0;
    for (unsigned i = 0; i < n; i++) k += !viszero(sp[i].e);
    return k;
}

/* One eye path (<= 7 segments) of RadiancePathTracingKernel device.cu:553-771. */
static Vec path_sample(const Sphere *sp, unsigned n, const float *rnd, const Camera *cam,
                       const campre *cp, int x, int y, int W, int H, unsigned sid,
                       const LightPath *lp, int vlp, ostats *st)
{
    const float inv_w = (float)(14. / W), inv_h = (float)(10.5 / H);   /* smallpt_cpu.c:411-412 */
    const float fw = (float)W, fh = (float)H;
    const int i = y * W + x;
    const unsigned kk = (26u + (unsigned)(i * 25) + sid) % (RAND_N - 5u);
    const float kx = (float)(((double)((float)x * inv_w) - (double)(inv_w * fw) / 2.)
                             + (double)(rnd[kk] * inv_w));
    const float ky = (float)(((double)((float)y * inv_h) - (double)(inv_h * fh) / 2.)
                             + (double)(rnd[kk + 1] * inv_h));
    const float kz = 10.0f;
    Vec rdir = vinit(0.f, 0.f, 0.f);
    rdir = vadd(rdir, vsmul(kx, cp->ux));
    rdir = vadd(rdir, vsmul(ky, cp->uy));
    rdir = vadd(rdir, vsmul(kz, cp->ud));
    const float w = (cp->tx * kx + cp->ty * ky + cp->tz * kz) + 1;
    rdir = vsmul((float)(1. / w), rdir);
    Ray cur;
    cur.o = vadd(rdir, cam->orig);
    cur.d = vnorm(rdir);

    Vec rad = vinit(0.f, 0.f, 0.f), thr = vinit(1.f, 1.f, 1.f);
    int specular = 1;
    if (st) { st->samples++; st->rng_reads += 2; }            /* d_Rand[kk], d_Rand[kk+1] */
    for (unsigned depth = 0;; ++depth) {
        const unsigned j = (26u + (unsigned)(i * 25) + depth * 5u + sid) % (RAND_N - 5u);
        if (depth > 6) break;
        float t; unsigned id = 0;
        if (st) st->segments++;
        if (!intersect(sp, n, &cur, &t, &id, st)) break;
        const Sphere *obj = &sp[id];
        Vec hit = vadd(cur.o, vsmul(t, cur.d));
        Vec normal = vnorm(vsub(hit, obj->p));
        const float dp = vdot(normal, cur.d);
        Vec nl = vsmul(-1.f * (dp > 0 ? 1 : -1), normal);
        if (!viszero(obj->e)) {
            if (specular) rad = vadd(rad, vmul(thr, vsmul(fabsf(dp), obj->e)));
            break;
        }
        if (obj->refl == BDPT_DIFF) {
            if (st) { st->diffuse++; st->rng_reads += 2 + (n_lights_of(sp, n) ? 2 : 0); }
            specular = 0;
            thr = vmul(thr, obj->c);
            Vec ld = sample_lights(sp, n, rnd, hit, nl, j + 2, lp, vlp, st);
            rad = vadd(rad, vmul(ld, thr));
            cur.o = hit;
            cur.d = cosine_dir(nl, rnd[j], rnd[j + 1]);
        } else if (obj->refl == BDPT_SPEC) {
            specular = 1;
            Vec nd = vsub(cur.d, vsmul(2.f * vdot(normal, cur.d), normal));
            thr = vmul(thr, obj->c);
            cur.o = hit; cur.d = nd;
        } else {
            specular = 1;
            Vec refl = vsub(cur.d, vsmul(2.f * vdot(normal, cur.d), normal));
            const int into = vdot(normal, nl) > 0;
            const float nc = 1.f, nt = 1.5f;
            const float nnt = into ? nc / nt : nt / nc;
            const float ddn = vdot(cur.d, nl);
            const float cos2t = 1.f - nnt * nnt * (1.f - ddn * ddn);
            if (cos2t < 0.f) {
                thr = vmul(thr, obj->c);
                cur.o = hit; cur.d = refl;
                continue;
            }
            if (st) { st->refr++; st->rng_reads += 1; }
            const float kq = (float)(into ? 1 : -1) * (ddn * nnt + sqrtf(cos2t));
            Vec td = vnorm(vsub(vsmul(nnt, cur.d), vsmul(kq, normal)));
            const float a = nt - nc, b = nt + nc;
            const float R0 = a * a / (b * b);
            const float c = 1 - (into ? -ddn : vdot(td, normal));
            const float Re = R0 + (1 - R0) * c * c * c * c * c;
            const float Tr = 1.f - Re;
            const float P = .25f + .5f * Re;
            const float RP = Re / P;
            const float TP = Tr / (1.f - P);
            if (rnd[j + 2] < P) {
                thr = vmul(vsmul(RP, thr), obj->c);
                cur.o = hit; cur.d = refl;
            } else {
                thr = vmul(vsmul(TP, thr), obj->c);
                cur.o = hit; cur.d = td;
            }
        }
    }
    return rad;
}

/* `npass` x RadiancePathTracingKernel (device.cu:544-791) over rows [y0, y1) (all columns),
 * each pixel's passes in order: running mean :774-782, toInt :783-786, counter :787.
 * colors (W*H Vec), counter (W*H), pixels (W*H*4 RGBA) are read-modify-written in place.
 * Returns the statistics of the work done in `stats_out` (8 x uint64) when non-NULL. */
void oracle_path_span(const Sphere *sp, unsigned n, const float *rnd, const Camera *cam,
                      int W, int H, long pix0, long pix1, const LightPath *lp,
                      const unsigned *sid, const int *vlp, int npass,
                      Vec *colors, unsigned *counter, unsigned char *pixels,
                      int nthreads, uint64_t *stats_out);

void oracle_path_passes(const Sphere *sp, unsigned n, const float *rnd, const Camera *cam,
                        int W, int H, int y0, int y1, const LightPath *lp,
                        const unsigned *sid, const int *vlp, int npass,
                        Vec *colors, unsigned *counter, unsigned char *pixels,
                        int nthreads, uint64_t *stats_out)
{
    if (y0 < 0) y0 = 0;
    if (y1 > H) y1 = H;
    oracle_path_span(sp, n, rnd, cam, W, H, (long)y0 * W, (long)y1 * W, lp, sid, vlp, npass,
                     colors, counter, pixels, nthreads, stats_out);
}

/* The same over the row-major pixel range [pix0, pix1) (spot checks of very large frames). */
void oracle_path_span(const Sphere *sp, unsigned n, const float *rnd, const Camera *cam,
                      int W, int H, long pix0, long pix1, const LightPath *lp,
                      const unsigned *sid, const int *vlp, int npass,
                      Vec *colors, unsigned *counter, unsigned char *pixels,
                      int nthreads, uint64_t *stats_out)
{
    const campre cp = camera_pre(cam);
    ostats tot = {0, 0, 0, 0, 0, 0, 0, 0};
    if (pix0 < 0) pix0 = 0;
    if (pix1 > (long)W * H) pix1 = (long)W * H;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        ostats loc = {0, 0, 0, 0, 0, 0, 0, 0};
        ostats *st = stats_out ? &loc : NULL;
#pragma omp for schedule(dynamic, 16)
        for (long pix = pix0; pix < pix1; pix++) {
            const int x = (int)(pix % W), y = (int)(pix / W);
            Vec c = colors[pix];
            unsigned cnt = counter[pix];
            int touched = 0;
            for (int p = 0; p < npass; p++) {
                if (cnt >= BDPT_COUNTER_CAP) break;
                Vec r = path_sample(sp, n, rnd, cam, &cp, x, y, W, H, sid[p], lp,
                                    vlp[p] & (BDPT_LIGHT_POINTS - 1), st);
                if (cnt == 0) c = r;
                else {
                    const float k1 = (float)cnt;
                    const float k2 = 1.f / (k1 + 1.f);
                    c.x = (c.x * k1 + r.x) * k2;
                    c.y = (c.y * k1 + r.y) * k2;
                    c.z = (c.z * k1 + r.z) * k2;
                }
                cnt++;
                touched = 1;
            }
            if (touched) {
                colors[pix] = c;
                counter[pix] = cnt;
                pixels[4 * pix + 0] = (unsigned char)toInt(c.x);
                pixels[4 * pix + 1] = (unsigned char)toInt(c.y);
                pixels[4 * pix + 2] = (unsigned char)toInt(c.z);
                pixels[4 * pix + 3] = 0;
            }
        }
        if (stats_out) {
#pragma omp critical
            {
                tot.segments += loc.segments; tot.closest += loc.closest; tot.shadow += loc.shadow;
                tot.sphere_tests += loc.sphere_tests; tot.samples += loc.samples;
                tot.diffuse += loc.diffuse; tot.rng_reads += loc.rng_reads; tot.refr += loc.refr;
            }
        }
    }
    if (stats_out) {
        stats_out[0] = tot.samples; stats_out[1] = tot.segments; stats_out[2] = tot.closest;
        stats_out[3] = tot.shadow; stats_out[4] = tot.sphere_tests; stats_out[5] = tot.diffuse;
        stats_out[6] = tot.rng_reads; stats_out[7] = tot.refr;
    }
}

/* vnorm (vec.h:22) as it compiles in the reference's host C files (display_func.c is C, so
 * `sqrt` is the double libm sqrt): l = (float)(1.f / sqrt((double)vdot)), one rounding. */
static inline Vec vnorm_host(Vec v) { float l = (float)(1.f / sqrt((double)vdot(v, v))); return vsmul(l, v); }

/* UpdateCamera display_func.c:177-190. */
void oracle_update_camera(Camera *c, int width, int height)
{
    c->dir = vnorm_host(vsub(c->target, c->orig));
    const Vec up = vinit(0.f, 1.f, 0.f);
    const float fov = (float)((M_PI / 180.f) * 45.f);
    c->x = vnorm_host(vxcross(c->dir, up));
    c->x = vsmul(width * fov / height, c->x);
    c->y = vnorm_host(vxcross(c->x, c->dir));
    c->y = vsmul(fov, c->y);
}

/* KeyFunc camera keys display_func.c:276-336 (MOVE_STEP 10.0f).  Returns 1 when the reference
 * calls ReInit(1) for the key (' ' too), 0 otherwise.  The camera is not re-derived here:
 * ReInit -> UpdateCamera does that. */
int oracle_key_camera(Camera *c, int key)
{
    const float step = 10.0f;
    Vec d;
    switch (key) {
    case ' ':
        return 1;
    case 'a':                                            /* :291-298 */
        d = vnorm_host(c->x);
        d = vsmul(-step, d);
        break;
    case 'd':                                            /* :300-307 */
        d = vnorm_host(c->x);
        d = vsmul(step, d);
        break;
    case 'w':                                            /* :309-315 */
        d = vsmul(step, c->dir);
        break;
    case 's':                                            /* :317-323 */
        d = vsmul(-step, c->dir);
        break;
    case 'r':                                            /* :325-329 */
        c->orig.y += step;
        c->target.y += step;
        return 1;
    case 'f':                                            /* :330-334 */
        c->orig.y -= step;
        c->target.y -= step;
        return 1;
    default:
        return 0;
    }
    c->orig = vadd(c->orig, d);
    c->target = vadd(c->target, d);
    return 1;
}

/* SpecialFunc display_func.c:384-433 with GLUT codes (LEFT 100, UP 101, RIGHT 102, DOWN 103,
 * PAGE_UP 104, PAGE_DOWN 105).  ROTATE_STEP = 2.f*M_PI/180.f is a double expression, so the
 * products and sums are double and each assignment rounds to float; the second line reads the
 * component the first one already overwrote (Appendix A.9). */
int oracle_special_key(Camera *c, int key)
{
    const double rs = 2.f * M_PI / 180.f;
    Vec t;
    switch (key) {
    case 101:
    case 103: {                                          /* UP :386-394, DOWN :396-404 */
        const double a = key == 101 ? -rs : rs;
        t = vsub(c->target, c->orig);
        t.y = t.y * cos(a) + t.z * sin(a);
        t.z = -t.y * sin(a) + t.z * cos(a);
        c->target = vadd(t, c->orig);
        return 1;
    }
    case 100:
    case 102: {                                          /* LEFT :406-414, RIGHT :416-424 */
        const double a = key == 100 ? -rs : rs;
        t = vsub(c->target, c->orig);
        t.x = t.x * cos(a) - t.z * sin(a);
        t.z = t.x * sin(a) + t.z * cos(a);
        c->target = vadd(t, c->orig);
        return 1;
    }
    case 104:                                            /* :426-429 */
        c->target.y += 10.0f;
        return 1;
    case 105:                                            /* :430-433 */
        c->target.y -= 10.0f;
        return 1;
    default:
        return 0;
    }
}

/* toInt(vec.h:34) of one value -- lets tests check the product's threshold table. */
int oracle_to_int(float x) { return toInt(x); }

/* FNV-1a 64 over a byte buffer: the digest the survey recorded for the reference's MT tables. */
uint64_t oracle_fnv1a64(const void *data, uint64_t len)
{
    const unsigned char *p = (const unsigned char *)data;
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; i < len; i++) { h ^= p[i]; h *= 0x100000001b3ull; }
    return h;
}

/* FNV-1 64 (multiply, then xor) over a byte buffer: one of the representations tried against the
 * survey's digests (tests/golden/fnv_trials.py). */
uint64_t oracle_fnv1_64(const void *data, uint64_t len)
{
    const unsigned char *p = (const unsigned char *)data;
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; i < len; i++) { h *= 0x100000001b3ull; h ^= p[i]; }
    return h;
}
