/*
 * bdpt_util.c -- host-side C pieces of the drop-in that live outside the render kernels:
 * the .scn loader, UpdateCamera, the KeyFunc/SpecialFunc camera and sphere moves, SavePPM,
 * a glibc-compatible rand(), the reference's pass (sid / vlp_index) state machine, and the
 * toInt threshold table the path kernel uses for its 8-bit output.
 * Built with -ffp-contract=off: every float expression keeps the reference's rounding.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/bdpt.h"

static bdpt_vec vinit(float a, float b, float c) { bdpt_vec v; v.x = a; v.y = b; v.z = c; return v; }
static bdpt_vec vadd(bdpt_vec a, bdpt_vec b) { return vinit(a.x + b.x, a.y + b.y, a.z + b.z); }
static bdpt_vec vsub(bdpt_vec a, bdpt_vec b) { return vinit(a.x - b.x, a.y - b.y, a.z - b.z); }
static bdpt_vec vsmul(float k, bdpt_vec b) { return vinit(k * b.x, k * b.y, k * b.z); }
static float vdot(bdpt_vec a, bdpt_vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* vnorm (vec.h:22) as the reference's host C code compiles it: `sqrt` of a float in C is the
 * double libm sqrt, so l = (float)(1.f / sqrt((double)dot)) with one final rounding. */
static bdpt_vec vnorm(bdpt_vec v) { float l = (float)(1.f / sqrt((double)vdot(v, v))); return vsmul(l, v); }
static bdpt_vec vxcross(bdpt_vec a, bdpt_vec b) {
    return vinit(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

/* ReadScene display_func.c:112-175: same fscanf formats, same error conditions. */
int bdpt_read_scene(const char *path, bdpt_camera *cam, bdpt_sphere **out, unsigned *n_out)
{
    if (!path || !cam || !out || !n_out) return BDPT_EINVAL;
    *out = NULL;
    *n_out = 0;
    FILE *f = fopen(path, "r");
    if (!f) {
        fprintf(stderr, "Failed to open file: %s\n", path);
        return BDPT_EIO;
    }
    int c = fscanf(f, "camera %f %f %f  %f %f %f\n", &cam->orig.x, &cam->orig.y, &cam->orig.z,
                   &cam->target.x, &cam->target.y, &cam->target.z);
    if (c != 6) {
        fprintf(stderr, "Failed to read 6 camera parameters: %d\n", c);
        fclose(f);
        return BDPT_EIO;
    }
    unsigned n = 0;
    c = fscanf(f, "size %u\n", &n);
    if (c != 1) {
        fprintf(stderr, "Failed to read sphere count: %d\n", c);
        fclose(f);
        return BDPT_EIO;
    }
    bdpt_sphere *s = (bdpt_sphere *)malloc(sizeof(bdpt_sphere) * (n ? n : 1));
    if (!s) { fclose(f); return BDPT_ENOMEM; }
    for (unsigned i = 0; i < n; i++) {
        int mat = -1;
        c = fscanf(f, "sphere %f  %f %f %f  %f %f %f  %f %f %f  %d\n", &s[i].rad, &s[i].p.x,
                   &s[i].p.y, &s[i].p.z, &s[i].e.x, &s[i].e.y, &s[i].e.z, &s[i].c.x, &s[i].c.y,
                   &s[i].c.z, &mat);
        if (mat < 0 || mat > 3) {
            fprintf(stderr, "Failed to read material type for sphere #%u: %d\n", i, mat);
            free(s);
            fclose(f);
            return BDPT_EIO;
        }
        s[i].refl = mat;                       /* 0..3 -> DIFF, SPEC, REFR, LITE */
        if (c != 11) {
            fprintf(stderr, "Failed to read sphere #%u: %d\n", i, c);
            free(s);
            fclose(f);
            return BDPT_EIO;
        }
    }
    fclose(f);
    *out = s;
    *n_out = n;
    return BDPT_OK;
}

void bdpt_free_scene(bdpt_sphere *s) { free(s); }

/* CornellSpheres scene.h:7-18 and the no-argument camera smallpt_cpu.c:404-405. */
unsigned bdpt_default_scene(bdpt_camera *cam, bdpt_sphere *s)
{
    const float W = 1e4f;
    const bdpt_sphere def[9] = {
        {W, {W + 1.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .25f, .25f}, BDPT_DIFF},
        {W, {-W + 99.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.25f, .25f, .75f}, BDPT_DIFF},
        {W, {50.f, 40.8f, W}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, BDPT_DIFF},
        {W, {50.f, 40.8f, -W + 270.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, BDPT_DIFF},
        {W, {50.f, W, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, BDPT_DIFF},
        {W, {50.f, -W + 81.6f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, BDPT_DIFF},
        {16.5f, {27.f, 16.5f, 47.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, BDPT_SPEC},
        {16.5f, {73.f, 16.5f, 78.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, BDPT_REFR},
        {7.f, {50.f, 81.6f - 15.f, 81.6f}, {12.f, 12.f, 12.f}, {0.f, 0.f, 0.f}, BDPT_REFR},
    };
    if (s) memcpy(s, def, sizeof(def));
    if (cam) {
        memset(cam, 0, sizeof(*cam));
        cam->orig = vinit(50.f, 44.f, 176.f);
        cam->target = vinit(50.f, 44 - 0.042612f, 175.f);
    }
    return 9;
}

/* UpdateCamera display_func.c:177-190. */
void bdpt_update_camera(bdpt_camera *c, int width, int height)
{
    c->dir = vnorm(vsub(c->target, c->orig));
    const bdpt_vec up = vinit(0.f, 1.f, 0.f);
    const float fov = (float)((M_PI / 180.f) * 45.f);
    c->x = vnorm(vxcross(c->dir, up));
    c->x = vsmul(width * fov / height, c->x);
    c->y = vnorm(vxcross(c->x, c->dir));
    c->y = vsmul(fov, c->y);
}

#define MOVE_STEP 10.0f
#define ROTATE_STEP (2.f * M_PI / 180.f)

/* KeyFunc / SpecialFunc camera moves, display_func.c:291-334 and :386-433.  The rotations
 * reuse the already-updated component, exactly as the reference does (survey Appendix A.9). */
int bdpt_camera_key(bdpt_camera *c, int key)
{
    bdpt_vec d, t;
    switch (key) {
    case 'a': d = vsmul(-MOVE_STEP, vnorm(c->x)); break;
    case 'd': d = vsmul(MOVE_STEP, vnorm(c->x)); break;
    case 'w': d = vsmul(MOVE_STEP, c->dir); break;
    case 's': d = vsmul(-MOVE_STEP, c->dir); break;
    case 'r': c->orig.y += MOVE_STEP; c->target.y += MOVE_STEP; return 1;
    case 'f': c->orig.y -= MOVE_STEP; c->target.y -= MOVE_STEP; return 1;
    case ' ': return 1;                                  /* ReInit(1) with no move */
    case BDPT_KEY_PAGE_UP: c->target.y += MOVE_STEP; return 1;
    case BDPT_KEY_PAGE_DOWN: c->target.y -= MOVE_STEP; return 1;
    case BDPT_KEY_UP:
    case BDPT_KEY_DOWN:
        t = vsub(c->target, c->orig);
        {
            const double a = key == BDPT_KEY_UP ? -ROTATE_STEP : ROTATE_STEP;
            t.y = t.y * cos(a) + t.z * sin(a);
            t.z = -t.y * sin(a) + t.z * cos(a);
        }
        c->target = vadd(t, c->orig);
        return 1;
    case BDPT_KEY_LEFT:
    case BDPT_KEY_RIGHT:
        t = vsub(c->target, c->orig);
        {
            const double a = key == BDPT_KEY_LEFT ? -ROTATE_STEP : ROTATE_STEP;
            t.x = t.x * cos(a) - t.z * sin(a);
            t.z = t.x * sin(a) + t.z * cos(a);
        }
        c->target = vadd(t, c->orig);
        return 1;
    default:
        return 0;
    }
    /* vsmul(direction, +-MOVE_STEP, direction); vadd(orig, orig, direction); vadd(target, ...) */
    c->orig = vadd(c->orig, d);
    c->target = vadd(c->target, d);
    return 1;
}

/* KeyFunc sphere edits display_func.c:347-370 (0.5f * MOVE_STEP along one axis). */
int bdpt_sphere_key(bdpt_sphere *s, unsigned n, int cur, int key)
{
    if (!s || cur < 0 || (unsigned)cur >= n) return 0;
    switch (key) {
    case '4': s[cur].p.x -= 0.5f * MOVE_STEP; return 1;
    case '6': s[cur].p.x += 0.5f * MOVE_STEP; return 1;
    case '8': s[cur].p.z -= 0.5f * MOVE_STEP; return 1;
    case '2': s[cur].p.z += 0.5f * MOVE_STEP; return 1;
    case '9': s[cur].p.y += 0.5f * MOVE_STEP; return 1;
    case '3': s[cur].p.y -= 0.5f * MOVE_STEP; return 1;
    default: return 0;
    }
}

/* SavePPM smallpt_cpu.c:239-262: "P3\n%d %d\n%d\n", rows bottom-up, "%d %d %d " per pixel. */
int bdpt_save_ppm(const char *path, const unsigned char *rgba, int w, int h)
{
    if (!path || !rgba || w <= 0 || h <= 0) return BDPT_EINVAL;
    FILE *f = fopen(path, "w");
    if (!f) {
        fprintf(stderr, "Failed to open image file: %s\n", path);
        return BDPT_EIO;
    }
    fprintf(f, "P3\n%d %d\n%d\n", w, h, 255);
    for (int y = h - 1; y >= 0; --y) {
        const unsigned char *p = rgba + 4 * (size_t)y * w;
        for (int x = 0; x < w; ++x, p += 4) fprintf(f, "%d %d %d ", p[0], p[1], p[2]);
    }
    return fclose(f) == 0 ? BDPT_OK : BDPT_EIO;
}

/* Binary variant (P6): same header numbers and bottom-up row order, raw RGB bytes. */
int bdpt_save_ppm_binary(const char *path, const unsigned char *rgba, int w, int h)
{
    if (!path || !rgba || w <= 0 || h <= 0) return BDPT_EINVAL;
    FILE *f = fopen(path, "wb");
    if (!f) {
        fprintf(stderr, "Failed to open image file: %s\n", path);
        return BDPT_EIO;
    }
    fprintf(f, "P6\n%d %d\n%d\n", w, h, 255);
    unsigned char *row = malloc(3 * (size_t)w);
    int ok = row != NULL;
    for (int y = h - 1; ok && y >= 0; --y) {
        const unsigned char *p = rgba + 4 * (size_t)y * w;
        for (int x = 0; x < w; ++x, p += 4) {
            row[3 * x] = p[0]; row[3 * x + 1] = p[1]; row[3 * x + 2] = p[2];
        }
        ok = fwrite(row, 3, (size_t)w, f) == (size_t)w;
    }
    free(row);
    return (fclose(f) == 0 && ok) ? BDPT_OK : BDPT_EIO;
}

/* SavePPM's file name smallpt_cpu.c:245 "max%d_secondi%.3f_exe%d.ppm" (MAX_VLP = 1), bounded
 * (the reference's name[32] overflows once total_time >= 1000 s, Appendix A.10).  Returns the
 * length snprintf reports. */
int bdpt_ppm_name(char *buf, int size, float total_time, int current_sample)
{
    if (!buf || size <= 0) return BDPT_EINVAL;
    return snprintf(buf, (size_t)size, "max%d_secondi%.3f_exe%d.ppm", 1, total_time, current_sample);
}

/* glibc random_r TYPE_3 (x**31 + x**3 + 1), the generator behind rand(). */
void bdpt_srand(bdpt_rand_state *st, unsigned seed)
{
    int *r = st->state;
    if (seed == 0) seed = 1;
    r[0] = (int)seed;
    long word = (long)(int)seed;
    for (int i = 1; i < 31; i++) {
        long hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int)word;
    }
    st->f = 3;
    st->r = 0;
    for (int i = 0; i < 310; i++) (void)bdpt_rand(st);
}

int bdpt_rand(bdpt_rand_state *st)
{
    int *r = st->state;
    unsigned val = (unsigned)r[st->f] + (unsigned)r[st->r];
    r[st->f] = (int)val;
    if (++st->f >= 31) { st->f = 0; ++st->r; }
    else if (++st->r >= 31) st->r = 0;
    return (int)(val >> 1);
}

void bdpt_pass_state_init(bdpt_pass_state *ps)
{
    bdpt_srand(&ps->rng, 1);                     /* rand() never seeded: seed 1 */
    ps->flag = 1;                                /* display_func.c:44 */
    ps->vlp_index = 1;                           /* smallpt_cpu.c:47 MAX_VLP */
}

void bdpt_pass_state_light(bdpt_pass_state *ps) { ps->flag = 2; }   /* smallpt_cpu.c:361 */

void bdpt_pass_state_next(bdpt_pass_state *ps, unsigned *sid, int *vlp)
{
    *sid = (unsigned)bdpt_rand(&ps->rng) % (unsigned)BDPT_RAND_N;        /* :270 */
    *vlp = ps->vlp_index % BDPT_LIGHT_POINTS;
    if (ps->flag == 3) { ps->vlp_index += 1; ps->flag = 1; }            /* :292 MAX_ITER=3 */
    if (ps->flag < 3) ps->flag++;                                        /* :293 */
}

void bdpt_pass_schedule(bdpt_pass_state *ps, int npass, unsigned *sid, int *vlp)
{
    for (int p = 0; p < npass; p++) bdpt_pass_state_next(ps, &sid[p], &vlp[p]);
}

/* toInt vec.h:34 with correctly-rounded powf semantics.  thr[k] (k = 1..255) is the smallest
 * non-negative float x with toInt(x) >= k; toInt is monotone, so the kernel's count of
 * thresholds <= x equals toInt(x) for every float (NaN and negatives give 0). thr[0] = -inf. */
static int to_int_ref(float x)
{
    float c = x < 0.f ? 0.f : (x > 1.f ? 1.f : x);
    float pw = (float)pow((double)c, (double)(1.f / 2.2f));
    return (int)(pw * 255.f + .5f);
}

void bdpt_gamma_thresholds(float thr[256])
{
    thr[0] = -INFINITY;
    for (int k = 1; k < 256; k++) {
        unsigned lo = 0, hi = 0x3f800000u;          /* toInt(1.0f) = 255 >= k */
        while (lo < hi) {
            unsigned mid = lo + (hi - lo) / 2;
            float x;
            memcpy(&x, &mid, 4);
            if (to_int_ref(x) >= k) hi = mid; else lo = mid + 1;
        }
        memcpy(&thr[k], &lo, 4);
    }
}

/* The black-surface exit rule (bdpt_kernels.hip BDPT_ZERO_EXIT, include/bdpt.h).  A hit on a black
 * non-emitter multiplies the reference's throughput by c = 0 (device.cu:665/711/732/758-765), and
 * the path then runs on to its 7th segment (:621), adding thr * term at every later vertex
 * (:656, :671-672).  With thr == +-0 every such addition is +-0 -- and rad + (+-0) == rad -- exactly
 * when every term is finite.  This proves it for the scene, in double arithmetic with margins:
 *  - all scene values finite, every |c| <= 1e3 (then the throughput before the black hit is at
 *    most (4 * 1e3)^7: the refraction weights Re/P and Tr/(1-P) are <= 4, :754-755), and every
 *    sphere radius > 2^-16 * scene scale (a hit point then lies far above rounding from its
 *    sphere's centre, so the normal of :640-641 is not 0/0);
 *  - emission: thr * e * |dp| (:654-656), |dp| <= 1 + eps;
 *  - NEE (:470-505): per emitter e * 4 pi r^2 * wi * wo / len^2 with wi, wo <= 1 + eps; a path
 *    vertex never lies on an emitter (a hit on one ends the path, :652-661) and every emitter keeps
 *    a gap >= max(1, 1e-4 * scale) from every other sphere's surface, so len >= ~1;
 *  - VLP (:510-537): rad * wi * wo, no 1/len^2; a VLP carries e/2 (escaped light ray) or
 *    VecMultiply(e/4, c) (:268, :279-337), so |rad| <= 0.5 * |e| * max(1, |c|); wo uses the
 *    escaped VLP's normal (-(o - p) / r), whose length is within 8 * 2^-24 * (|p| + r) / r of 1;
 *  - the vertex's sum NEE + VLP (:539-540) stays below FLT_MAX: n_lights * max(e * 4 pi r^2) * 1.1
 *    + 0.5 * max|e| * max(1, max|c|) * g < 1e38 (g: the normal-length factor above).
 * Scenes without a black non-emitter return 0 (the exit would only cost a test). */
int bdpt_zero_exit_safe(const bdpt_sphere *s, unsigned n)
{
    if (!s || n == 0) return 0;
    double scale = 0.0, cmax = 0.0, emax = 0.0, nee = 0.0, g = 1.0;
    int black = 0;
    for (unsigned i = 0; i < n; i++) {
        const bdpt_sphere *o = &s[i];
        const double v[10] = {o->rad, o->p.x, o->p.y, o->p.z, o->e.x, o->e.y, o->e.z, o->c.x, o->c.y, o->c.z};
        for (int k = 0; k < 10; k++)
            if (!isfinite(v[k])) return 0;
        const double sc = sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]) + fabs(v[0]);
        if (sc > scale) scale = sc;
        for (int k = 7; k < 10; k++) cmax = fmax(cmax, fabs(v[k]));
        const int emits = !(o->e.x == 0.f && o->e.y == 0.f && o->e.z == 0.f);
        if (!emits && o->c.x == 0.f && o->c.y == 0.f && o->c.z == 0.f) black = 1;
    }
    if (!black || !(cmax <= 1e3)) return 0;
    const double min_gap = fmax(1.0, 1e-4 * scale), min_rad = ldexp(scale, -16);
    for (unsigned i = 0; i < n; i++) {
        const bdpt_sphere *e = &s[i];
        const double re = fabs((double)e->rad);
        if (!(re > min_rad)) return 0;
        if (e->e.x == 0.f && e->e.y == 0.f && e->e.z == 0.f) continue;
        const double em = fmax(fabs(e->e.x), fmax(fabs(e->e.y), fabs(e->e.z)));
        emax = fmax(emax, em);
        nee += em * 4.0 * 3.14159265358979323846 * re * re;
        const double pn = sqrt((double)e->p.x * e->p.x + (double)e->p.y * e->p.y + (double)e->p.z * e->p.z);
        g = fmax(g, 1.0 + 8.0 * ldexp(pn + re, -24) / re);
        for (unsigned k = 0; k < n; k++) {
            if (k == i) continue;
            const bdpt_sphere *o = &s[k];
            const double ro = fabs((double)o->rad);
            const double dx = (double)e->p.x - o->p.x, dy = (double)e->p.y - o->p.y, dz = (double)e->p.z - o->p.z;
            const double d = sqrt(dx * dx + dy * dy + dz * dz);
            const double gap = fmax(d - re - ro, fmax(ro - d - re, re - d - ro));   /* apart / inside */
            if (!(gap >= min_gap)) return 0;
        }
    }
    return nee * 1.1 + 0.5 * emax * fmax(1.0, cmax) * g < 1e38;
}
