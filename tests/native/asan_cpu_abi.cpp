// asan_cpu_abi.cpp -- TEST INFRASTRUCTURE: a HIP-free context layer for the sanitizer build
// (`make asan`).  It implements the context entry points of include/bdpt.h that the C host
// `smallpt` calls, on the product's CPU backend (csrc/bdpt_cpu.cpp) only, so smallpt.c,
// bdpt_util.c and bdpt_cpu.cpp can be built and run under AddressSanitizer + UBSan on a machine
// without a GPU (GPU sanitizers are not available on the MI355X pool).  libbdpt.so's real layer
// (csrc/bdpt_host.cpp) dispatches to the same bdpt_cpu_* functions for BDPT_DEVICE_CPU.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_cpu.h"

struct bdpt_ctx {
    bdpt_cpu_ctx* cpu = nullptr;
    int W = 0, H = 0;
    bool rand_ready = false, cam_set = false;
    unsigned seed = 0;
    bdpt_camera cam{};
    std::vector<bdpt_sphere> spheres;
    char err[256] = {0};
};

static char g_err[256];

static int fail(bdpt_ctx* c, int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(c ? c->err : g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" {

int bdpt_create(bdpt_ctx** out, const bdpt_sphere* s, unsigned n, int W, int H, const char* dat, int device) {
    if (!out) return BDPT_EINVAL;
    *out = nullptr;
    if (device != BDPT_DEVICE_CPU) return fail(nullptr, BDPT_EHIP, "sanitizer build: CPU backend only");
    if (W <= 0 || H <= 0) return fail(nullptr, BDPT_EINVAL, "bad size");
    uint32_t params[4 * BDPT_MT_RNG_COUNT];
    FILE* f = fopen(dat, "rb");
    if (!f) return fail(nullptr, BDPT_EIO, "initMTGPU(): failed to open %s", dat);
    const size_t got = fread(params, sizeof params, 1, f);
    fclose(f);
    if (got != 1) return fail(nullptr, BDPT_EIO, "initMTGPU(): failed to load %s", dat);
    bdpt_ctx* c = new bdpt_ctx();
    c->cpu = bdpt_cpu_create(s, n, W, H, params);
    c->spheres.assign(s, s + n);
    c->W = W;
    c->H = H;
    *out = c;
    return BDPT_OK;
}
int bdpt_create_multi(bdpt_ctx**, const bdpt_sphere*, unsigned, int, int, const char*, const int*, int) {
    return fail(nullptr, BDPT_EINVAL, "sanitizer build: no multi-device contexts");
}
const char* bdpt_create_error(void) { return g_err; }
const char* bdpt_last_error(const bdpt_ctx* c) { return c ? c->err : "null context"; }
void bdpt_destroy(bdpt_ctx* c) {
    if (!c) return;
    bdpt_cpu_destroy(c->cpu);
    delete c;
}
int bdpt_num_devices(const bdpt_ctx*) { return 1; }
const char* bdpt_reduce_backend(const bdpt_ctx*) { return "none"; }
int bdpt_set_scene(bdpt_ctx* c, const bdpt_sphere* s, unsigned n) {
    bdpt_cpu_set_scene(c->cpu, s, n);
    c->spheres.assign(s, s + n);
    return BDPT_OK;
}
int bdpt_set_camera(bdpt_ctx* c, const bdpt_camera* cam) {
    bdpt_cpu_set_camera(c->cpu, cam);
    c->cam = *cam;
    c->cam_set = true;
    return BDPT_OK;
}
int bdpt_get_camera(const bdpt_ctx* c, bdpt_camera* cam) {
    if (!c->cam_set) return BDPT_ESTATE;
    *cam = c->cam;
    return BDPT_OK;
}
int bdpt_get_scene(const bdpt_ctx* c, bdpt_sphere* s, unsigned cap) {
    for (unsigned i = 0; s && i < c->spheres.size() && i < cap; i++) s[i] = c->spheres[i];
    return (int)c->spheres.size();
}
int bdpt_frame_size(const bdpt_ctx* c, int* W, int* H) {
    *W = c->W;
    *H = c->H;
    return BDPT_OK;
}
int bdpt_generate_rand(bdpt_ctx* c, unsigned seed) {
    bdpt_cpu_generate_rand(c->cpu, seed);
    c->rand_ready = true;
    c->seed = seed;
    return BDPT_OK;
}
int bdpt_rand_seed(const bdpt_ctx* c, unsigned* seed) {
    if (!c->rand_ready) return BDPT_ESTATE;
    *seed = c->seed;
    return BDPT_OK;
}
int bdpt_read_lightpaths(bdpt_ctx* c, bdpt_lightpath* lp) { bdpt_cpu_read_lightpaths(c->cpu, lp); return BDPT_OK; }
int bdpt_write_lightpaths(bdpt_ctx* c, const bdpt_lightpath* lp) { bdpt_cpu_write_lightpaths(c->cpu, lp); return BDPT_OK; }
int bdpt_reset_accum(bdpt_ctx* c) { bdpt_cpu_reset_accum(c->cpu); return BDPT_OK; }
int bdpt_set_shard(bdpt_ctx* c, int shard, int nshards, int band) {
    if (nshards < 1 || shard < 0 || shard >= nshards || band < 1) return fail(c, BDPT_EINVAL, "bad shard");
    bdpt_cpu_set_shard(c->cpu, shard, nshards, band);
    return BDPT_OK;
}
int bdpt_light_pass(bdpt_ctx* c, int current_sample) {
    bdpt_cpu_light_pass(c->cpu, current_sample);
    c->rand_ready = true;
    c->seed = (unsigned)(current_sample * 5);
    return BDPT_OK;
}
int bdpt_path_passes(bdpt_ctx* c, const unsigned* sid, const int* vlp, int npass) {
    if (!c->rand_ready || !c->cam_set) return fail(c, BDPT_ESTATE, "light pass / camera missing");
    bdpt_cpu_path_passes(c->cpu, sid, vlp, npass);
    return BDPT_OK;
}
int bdpt_synchronize(bdpt_ctx*) { return BDPT_OK; }
int bdpt_read_pixels(bdpt_ctx* c, unsigned char* rgba) { bdpt_cpu_read_pixels(c->cpu, rgba); return BDPT_OK; }
int bdpt_read_radiance(bdpt_ctx* c, bdpt_vec* col, unsigned* cnt) { bdpt_cpu_read_radiance(c->cpu, col, cnt); return BDPT_OK; }
int bdpt_write_radiance(bdpt_ctx* c, const bdpt_vec* col, const unsigned* cnt) {
    bdpt_cpu_write_radiance(c->cpu, col, cnt);
    return BDPT_OK;
}

// checkpoint / resume: the product's own bdpt_ckpt.c, linked in, over the entry points above
int bdpt__fail(bdpt_ctx* c, int code, const char* msg) { return fail(c, code, "%s", msg); }

}  // extern "C"
