// bdpt_cpu.cpp -- the host (CPU) backend of the C-ABI: a render context that runs the reference's
// render path on the CPU cores, selected with device = BDPT_DEVICE_CPU in bdpt_create.  It is the
// product's answer to "smallpt_cpu.c CPU path" configs (BASELINE.json configs[0]) and to a machine
// without a GPU; it is not a fallback -- a GPU context never routes here.
//
// Same floating-point contract as the HIP kernels: IEEE fp32 with no contraction
// (built with -ffp-contract=off), correctly rounded division and sqrt, the fp64 camera steps of
// device.cu:565-566, sin/cos as (float)f((double)x).  So its frames equal the GPU's bit for bit.
// Work is spread over threads by pixel row (each pixel renders its passes in order, as the
// running mean requires).
#include "bdpt_cpu.h"

#include <math.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

namespace {

constexpr float kEps = 0.01f;                              // geom.h:6 EPSILON
constexpr float kPi = 3.14159265358979323846f;             // geom.h:7 FLOAT_PI
constexpr unsigned kRandN = BDPT_RAND_N;

struct V3 {
    float x, y, z;
};
inline V3 v3(float a, float b, float c) { return V3{a, b, c}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator*(float k, V3 b) { return v3(k * b.x, k * b.y, k * b.z); }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline V3 unit(V3 v) { return (1.f / sqrtf(dot(v, v))) * v; }   // vnorm (vec.h:22), fp32 on the device
inline bool zero(V3 v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }
inline V3 of(const bdpt_vec& v) { return v3(v.x, v.y, v.z); }
inline float fsin(float x) { return (float)sin((double)x); }
inline float fcos(float x) { return (float)cos((double)x); }

// Scene in structure-of-arrays form for the traversal loops.
struct Scene {
    unsigned n = 0;
    std::vector<float> px, py, pz, rad;
    std::vector<unsigned char> emissive;
    std::vector<bdpt_sphere> s;
    void load(const bdpt_sphere* sp, unsigned count) {
        n = count;
        s.assign(sp, sp + count);
        px.resize(n); py.resize(n); pz.resize(n); rad.resize(n); emissive.resize(n);
        for (unsigned i = 0; i < n; i++) {
            px[i] = sp[i].p.x; py[i] = sp[i].p.y; pz[i] = sp[i].p.z; rad[i] = sp[i].rad;
            emissive[i] = !zero(of(sp[i].e));
        }
    }
    // SphereIntersectDevice device.cu:80-104: 0 = miss
    float hit(unsigned i, V3 o, V3 d) const {
        const V3 op = v3(px[i], py[i], pz[i]) - o;
        const float b = dot(op, d);
        float det = b * b - dot(op, op) + rad[i] * rad[i];
        if (det < 0.f) return 0.f;
        det = sqrtf(det);
        const float t1 = b - det;
        if (t1 > kEps) return t1;
        const float t2 = b + det;
        return t2 > kEps ? t2 : 0.f;
    }
    // IntersectDevice device.cu:106-124: scan from the last sphere down, `<` keeps ties
    bool closest(V3 o, V3 d, float* t, unsigned* id) const {
        *t = 1e20f;
        for (unsigned i = n; i--;) {
            const float h = hit(i, o, d);
            if (h != 0.f && h < *t) { *t = h; *id = i; }
        }
        return *t < 1e20f;
    }
    // IntersectPDevice / IntersectPVacuumDevice device.cu:126-154
    bool occluded(V3 o, V3 d, float maxt, bool vacuum) const {
        for (unsigned i = n; i--;) {
            const float h = hit(i, o, d);
            if (h != 0.f && h < maxt && !(vacuum && emissive[i])) return true;
        }
        return false;
    }
};

// UniformSampleSphereDevice device.cu:157-165
V3 sphere_point(float u1, float u2) {
    const float zz = 1.f - 2.f * u1;
    const float q = 1.f - zz * zz;
    const float r = sqrtf(0.f > q ? 0.f : q);
    const float phi = 2.f * kPi * u2;
    return v3(r * fcos(phi), r * fsin(phi), zz);
}

// cosine-weighted direction about w (device.cu:190-212, 357-380, 676-699)
V3 cosine_dir(V3 w, float u_phi, float r2) {
    const float r1 = 2.f * kPi * u_phi;
    const float r2s = sqrtf(r2);
    const V3 a = fabsf(w.x) > .1f ? v3(0.f, 1.f, 0.f) : v3(1.f, 0.f, 0.f);
    V3 u = unit(cross(a, w));
    V3 v = cross(w, u);
    u = (fcos(r1) * r2s) * u;
    v = (fsin(r1) * r2s) * v;
    return (u + v) + sqrtf(1 - r2) * w;
}

unsigned to_int8(float v, const float* thr) {                // toInt (vec.h:34) by threshold search
    unsigned k = 0;
    for (unsigned step = 128; step > 0; step >>= 1)
        if (v >= thr[k + step]) k += step;
    return k;
}

int worker_count() {
    if (const char* e = getenv("BDPT_CPU_THREADS")) {
        const int t = atoi(e);
        if (t > 0) return t;
    }
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) return CPU_COUNT(&set) > 0 ? CPU_COUNT(&set) : 1;
    const unsigned h = std::thread::hardware_concurrency();
    return h ? (int)h : 1;
}

template <class F>
void parallel_rows(int y0, int y1, int threads, F body) {
    std::atomic<int> next(y0);
    auto run = [&] {
        for (int y; (y = next.fetch_add(1)) < y1;) body(y);
    };
    const int nt = threads < y1 - y0 ? threads : (y1 - y0 > 0 ? y1 - y0 : 1);
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(run);
    run();
    for (std::thread& t : pool) t.join();
}

}  // namespace

struct bdpt_cpu_ctx {
    int W = 0, H = 0;
    Scene scene;
    bdpt_camera cam{};
    bool cam_set = false, rand_ready = false;
    uint32_t params[4 * BDPT_MT_RNG_COUNT];
    std::vector<float> rnd;
    std::vector<bdpt_lightpath> lp;
    std::vector<bdpt_vec> colors;
    std::vector<unsigned> counter;
    std::vector<unsigned char> pixels;
    float thr[256];
    int shard = 0, nshards = 1, band_rows = 8;
    int threads = 1;
};

extern "C" void bdpt_gamma_thresholds(float thr[256]);

bdpt_cpu_ctx* bdpt_cpu_create(const bdpt_sphere* spheres, unsigned n, int W, int H, const uint32_t* params) {
    bdpt_cpu_ctx* c = new (std::nothrow) bdpt_cpu_ctx();
    if (!c) return nullptr;
    c->W = W; c->H = H;
    c->scene.load(spheres, n);
    memcpy(c->params, params, sizeof c->params);
    const size_t np = (size_t)W * H;
    c->lp.assign(BDPT_LIGHT_POINTS, bdpt_lightpath{});        // zero-initialised (Appendix A.4)
    c->colors.assign(np, bdpt_vec{0.f, 0.f, 0.f});
    c->counter.assign(np, 0u);
    c->pixels.assign(4 * np, 0);
    bdpt_gamma_thresholds(c->thr);
    c->threads = worker_count();
    return c;
}

void bdpt_cpu_destroy(bdpt_cpu_ctx* c) { delete c; }

void bdpt_cpu_set_scene(bdpt_cpu_ctx* c, const bdpt_sphere* spheres, unsigned n) { c->scene.load(spheres, n); }
void bdpt_cpu_set_camera(bdpt_cpu_ctx* c, const bdpt_camera* cam) { c->cam = *cam; c->cam_set = true; }
void bdpt_cpu_reset_accum(bdpt_cpu_ctx* c) { std::fill(c->counter.begin(), c->counter.end(), 0u); }
void bdpt_cpu_set_shard(bdpt_cpu_ctx* c, int shard, int nshards, int band_rows) {
    c->shard = shard; c->nshards = nshards; c->band_rows = band_rows;
}
int bdpt_cpu_threads(const bdpt_cpu_ctx* c) { return c->threads; }

// seedMTGPU(seed) + RandomGPU (MersenneTwister_kernel.cu:39-110): 4096 MT607 lanes, lane-major.
void bdpt_cpu_generate_rand(bdpt_cpu_ctx* c, unsigned seed) {
    c->rnd.resize(kRandN);
    float* out = c->rnd.data();
    const uint32_t* prm = c->params;
    parallel_rows(0, BDPT_MT_RNG_COUNT / 64, c->threads, [&](int blk) {
        for (int tid = blk * 64; tid < blk * 64 + 64; tid++) {
            const uint32_t a = prm[4 * tid], mb = prm[4 * tid + 1], mc = prm[4 * tid + 2];
            uint32_t mt[19];
            mt[0] = seed;
            for (int s = 1; s < 19; s++) mt[s] = 1812433253u * (mt[s - 1] ^ (mt[s - 1] >> 30)) + (uint32_t)s;
            for (int k = 0, s = 0; k < BDPT_N_PER_RNG; k++, s = s == 18 ? 0 : s + 1) {
                const int s1 = s == 18 ? 0 : s + 1, sm = s + 9 >= 19 ? s + 9 - 19 : s + 9;
                uint32_t y = (mt[s] & 0xFFFFFFFEu) | (mt[s1] & 0x1u);
                y = mt[sm] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
                mt[s] = y;
                y ^= y >> 12;
                y ^= (y << 7) & mb;
                y ^= (y << 15) & mc;
                y ^= y >> 18;
                out[tid + k * BDPT_MT_RNG_COUNT] = ((float)y + 1.0f) / 4294967296.0f;
            }
        }
    });
    c->rand_ready = true;
}

// UpdateRendering2 smallpt_cpu.c:311-359: GetRayKernel + RadianceLightTracingKernel per emitter,
// in sphere order (a later light overwrites the VLPs an earlier one wrote).
void bdpt_cpu_light_pass(bdpt_cpu_ctx* c, int current_sample) {
    bdpt_cpu_generate_rand(c, (unsigned)(current_sample * 5));
    const Scene& sc = c->scene;
    const float* rnd = c->rnd.data();
    for (unsigned li = 0; li < sc.n; li++) {
        if (!sc.emissive[li]) continue;
        const bdpt_sphere L = sc.s[li];
        parallel_rows(0, BDPT_LIGHT_POINTS / 64, c->threads, [&](int blk) {
            for (int ind = blk * 64; ind < blk * 64 + 64; ind++) {
                const unsigned i = (unsigned)(current_sample * 5 + ind * 4) % (kRandN - 4u), j = i + 2;
                const V3 spt = L.rad * sphere_point(rnd[j], rnd[i]) + of(L.p);
                const V3 o = spt, d = cosine_dir(unit(spt - of(L.p)), rnd[i + 1], rnd[j + 1]);
                V3 thr = 0.25f * of(L.e);
                float t;
                unsigned id = 0;
                bdpt_lightpath& out = c->lp[ind];
                if (!sc.closest(o, d, &t, &id)) {                      // escaped (:279-292)
                    const V3 nor = (float)(-1. / (double)L.rad) * (o - of(L.p)), hr = 0.5f * of(L.e);
                    out.hp = {o.x, o.y, o.z}; out.rad = {hr.x, hr.y, hr.z}; out.nl = {nor.x, nor.y, nor.z};
                    continue;
                }
                const bdpt_sphere& O = sc.s[id];
                if (sc.emissive[id]) continue;                          // :296-298
                const V3 h = o + t * d;
                const V3 nrm = unit(h - of(O.p));
                const float dp = dot(nrm, d);
                const V3 nl = (-1.f * (float)(dp > 0 ? 1 : -1)) * nrm;
                if (O.refl != BDPT_DIFF) continue;                      // DEPTH = 1: no store
                const float tol = (float)0.0001;                         // VecMultiply :10-42
                float* tv[3] = {&thr.x, &thr.y, &thr.z};
                const float cv[3] = {O.c.x, O.c.y, O.c.z};
                for (int k = 0; k < 3; k++) {
                    if (*tv[k] != 0.f && cv[k] != 0.f) {
                        const float m = *tv[k] * cv[k];
                        if (!(m <= tol || *tv[k] == m)) *tv[k] = m;
                    } else {
                        *tv[k] = 0.f;
                    }
                }
                out.hp = {h.x, h.y, h.z}; out.rad = {thr.x, thr.y, thr.z}; out.nl = {nl.x, nl.y, nl.z};
            }
        });
    }
}

namespace {
// RadiancePathTracingKernel device.cu:553-771 for one (pixel, pass): the radiance of one eye path.
struct PathTracer {
    const Scene& sc;
    const float* rnd;
    const bdpt_lightpath* lp;
    V3 ux, uy, ud, orig;
    float tx, ty, tz, inv_w, inv_h;
    double half_w, half_h;

    PathTracer(const bdpt_cpu_ctx* c) : sc(c->scene), rnd(c->rnd.data()), lp(c->lp.data()) {
        const bdpt_camera& cm = c->cam;
        ux = unit(of(cm.x)); uy = unit(of(cm.y)); ud = unit(of(cm.dir)); orig = of(cm.orig);
        tx = dot(unit(-1.f * of(cm.x)), orig);
        ty = dot(unit(-1.f * of(cm.y)), orig);
        tz = dot(-1.f * of(cm.dir), orig);                      // :591-592, no vnorm
        inv_w = (float)(14. / c->W);                            // smallpt_cpu.c:411-412
        inv_h = (float)(10.5 / c->H);
        half_w = (double)(inv_w * (float)c->W) / 2.;
        half_h = (double)(inv_h * (float)c->H) / 2.;
    }

    // SampleLightsDevice device.cu:457-542: NEE to every emitter + one VLP, blended 1/2
    V3 lights(V3 h, V3 nl, unsigned j, const bdpt_lightpath& v) const {
        V3 res = v3(0.f, 0.f, 0.f);
        for (unsigned i = 0; i < sc.n; i++) {
            if (!sc.emissive[i]) continue;
            const bdpt_sphere& L = sc.s[i];
            const V3 usp = sphere_point(rnd[j + 3], rnd[j + 4]);
            V3 sd = (L.rad * usp + of(L.p)) - h;
            const float len = sqrtf(dot(sd, sd));
            sd = (1.f / len) * sd;
            float wo = dot(sd, usp);
            if (wo > 0.f) continue;
            wo = -wo;
            const float wi = dot(sd, nl);
            if (wi > 0.f && !sc.occluded(h, sd, len - kEps, false))
                res = res + ((4.f * kPi * L.rad * L.rad) * wi * wo / (len * len)) * of(L.e);
        }
        V3 vres = v3(0.f, 0.f, 0.f);
        V3 vd = of(v.hp) - h;
        const float len = sqrtf(dot(vd, vd));
        vd = (1.f / len) * vd;
        float wo = dot(vd, of(v.nl));
        if (!(wo > 0.f)) {
            wo = -wo;
            const float wi = dot(vd, nl);
            if (wi > 0.f && !sc.occluded(h, vd, len - kEps, true)) vres = vres + (wi * wo) * of(v.rad);
        }
        vres = 1.f * vres;
        res = res + vres;
        return 0.5f * res;
    }

    V3 sample(int x, int y, int W, unsigned sid, int vlp) const {
        const unsigned base = 26u + (unsigned)(y * W + x) * 25u;
        const unsigned kk = (base + sid) % (kRandN - 5u);
        const float kx = (float)(((double)((float)x * inv_w) - half_w) + (double)(rnd[kk] * inv_w));
        const float ky = (float)(((double)((float)y * inv_h) - half_h) + (double)(rnd[kk + 1] * inv_h));
        const float kz = 10.0f;
        V3 rdir = v3(0.f, 0.f, 0.f);
        rdir = rdir + kx * ux;
        rdir = rdir + ky * uy;
        rdir = rdir + kz * ud;
        const float w = (tx * kx + ty * ky + tz * kz) + 1;
        rdir = (float)(1. / w) * rdir;
        V3 o = rdir + orig, d = unit(rdir);
        V3 rad = v3(0.f, 0.f, 0.f), thr = v3(1.f, 1.f, 1.f);
        bool specular = true;
        const bdpt_lightpath& v = lp[vlp & (BDPT_LIGHT_POINTS - 1)];
        for (unsigned depth = 0; depth <= 6; ++depth) {
            const unsigned j = (base + depth * 5u + sid) % (kRandN - 5u);
            float t;
            unsigned id = 0;
            if (!sc.closest(o, d, &t, &id)) break;
            const bdpt_sphere& S = sc.s[id];
            const V3 h = o + t * d;
            const V3 normal = unit(h - of(S.p));
            const float dp = dot(normal, d);
            const V3 nl = (-1.f * (float)(dp > 0 ? 1 : -1)) * normal;
            if (sc.emissive[id]) {                                   // :651-661
                if (specular) rad = rad + thr * (fabsf(dp) * of(S.e));
                break;
            }
            if (S.refl == BDPT_DIFF) {                               // :663-703
                specular = false;
                thr = thr * of(S.c);
                rad = rad + lights(h, nl, j, v) * thr;
                o = h;
                d = cosine_dir(nl, rnd[j], rnd[j + 1]);
                continue;
            }
            specular = true;
            const V3 refl = d - (2.f * dot(normal, d)) * normal;
            if (S.refl == BDPT_SPEC) {                               // :704-714
                thr = thr * of(S.c);
                o = h; d = refl;
                continue;
            }
            const bool into = dot(normal, nl) > 0;                   // REFR / LITE :715-770
            const float nc = 1.f, nt = 1.5f, nnt = into ? nc / nt : nt / nc;
            const float ddn = dot(d, nl);
            const float cos2t = 1.f - nnt * nnt * (1.f - ddn * ddn);
            if (cos2t < 0.f) {
                thr = thr * of(S.c);
                o = h; d = refl;
                continue;
            }
            const float kq = (float)(into ? 1 : -1) * (ddn * nnt + sqrtf(cos2t));
            const V3 td = unit(nnt * d - kq * normal);
            const float a = nt - nc, b = nt + nc, R0 = a * a / (b * b);
            const float cc = 1 - (into ? -ddn : dot(td, normal));
            const float Re = R0 + (1 - R0) * cc * cc * cc * cc * cc, Tr = 1.f - Re, P = .25f + .5f * Re;
            if (rnd[j + 2] < P) {
                thr = (Re / P) * thr * of(S.c);
                d = refl;
            } else {
                thr = (Tr / (1.f - P)) * thr * of(S.c);
                d = td;
            }
            o = h;
        }
        return rad;
    }
};
}  // namespace

// npass x UpdateRendering (smallpt_cpu.c:265-297): each pixel of this context's shard renders its
// passes in order with the running mean of device.cu:774-787.
void bdpt_cpu_path_passes(bdpt_cpu_ctx* c, const unsigned* sid, const int* vlp, int npass) {
    const PathTracer pt(c);
    const int W = c->W;
    parallel_rows(0, c->H, c->threads, [&](int y) {
        if (c->nshards > 1 && (y / c->band_rows) % c->nshards != c->shard) return;
        for (int x = 0; x < W; x++) {
            const size_t i = (size_t)y * W + x;
            bdpt_vec col = c->colors[i];
            unsigned cnt = c->counter[i];
            const unsigned cnt0 = cnt;
            for (int p = 0; p < npass && cnt < BDPT_COUNTER_CAP; p++, cnt++) {
                const V3 r = pt.sample(x, y, W, sid[p], vlp[p]);
                if (cnt == 0) {
                    col = {r.x, r.y, r.z};
                } else {
                    const float k1 = (float)cnt, k2 = 1.f / (k1 + 1.f);
                    col.x = (col.x * k1 + r.x) * k2;
                    col.y = (col.y * k1 + r.y) * k2;
                    col.z = (col.z * k1 + r.z) * k2;
                }
            }
            if (cnt == cnt0) continue;
            c->colors[i] = col;
            c->counter[i] = cnt;
            unsigned char* px = &c->pixels[4 * i];
            px[0] = (unsigned char)to_int8(col.x, c->thr);
            px[1] = (unsigned char)to_int8(col.y, c->thr);
            px[2] = (unsigned char)to_int8(col.z, c->thr);
            px[3] = 0;
        }
    });
}

bool bdpt_cpu_rand_ready(const bdpt_cpu_ctx* c) { return c->rand_ready; }
bool bdpt_cpu_camera_set(const bdpt_cpu_ctx* c) { return c->cam_set; }

void bdpt_cpu_read_radiance(const bdpt_cpu_ctx* c, bdpt_vec* colors, unsigned* counter) {
    if (colors) memcpy(colors, c->colors.data(), sizeof(bdpt_vec) * c->colors.size());
    if (counter) memcpy(counter, c->counter.data(), sizeof(unsigned) * c->counter.size());
}
void bdpt_cpu_read_pixels(const bdpt_cpu_ctx* c, unsigned char* rgba) { memcpy(rgba, c->pixels.data(), c->pixels.size()); }
void bdpt_cpu_read_rand(const bdpt_cpu_ctx* c, float* t) { memcpy(t, c->rnd.data(), sizeof(float) * kRandN); }
void bdpt_cpu_read_lightpaths(const bdpt_cpu_ctx* c, bdpt_lightpath* lp) {
    memcpy(lp, c->lp.data(), sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS);
}
void bdpt_cpu_write_lightpaths(bdpt_cpu_ctx* c, const bdpt_lightpath* lp) {
    memcpy(c->lp.data(), lp, sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS);
}
void bdpt_cpu_update_pixels(bdpt_cpu_ctx* c) {
    for (size_t i = 0; i < c->colors.size(); i++) {
        c->pixels[4 * i] = (unsigned char)to_int8(c->colors[i].x, c->thr);
        c->pixels[4 * i + 1] = (unsigned char)to_int8(c->colors[i].y, c->thr);
        c->pixels[4 * i + 2] = (unsigned char)to_int8(c->colors[i].z, c->thr);
        c->pixels[4 * i + 3] = 0;
    }
}
void bdpt_cpu_write_radiance(bdpt_cpu_ctx* c, const bdpt_vec* colors, const unsigned* counter) {
    memcpy(c->colors.data(), colors, sizeof(bdpt_vec) * c->colors.size());
    memcpy(c->counter.data(), counter, sizeof(unsigned) * c->counter.size());
    bdpt_cpu_update_pixels(c);
}
