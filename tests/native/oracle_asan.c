/* oracle_asan.c -- TEST INFRASTRUCTURE: driver of the sanitizer build (`make asan`).  Runs the
 * oracle (oracle/bdpt_oracle.c) and the product's CPU backend (csrc/bdpt_cpu.cpp, through the
 * HIP-free layer tests/native/asan_cpu_abi.cpp) on small frames of several scenes under
 * AddressSanitizer + UBSan and checks that both agree bit for bit.  Usage:
 *   oracle_asan <MersenneTwister.dat> <scene.scn>...     exit 0 = clean and equal */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/bdpt.h"

void oracle_mt607(const uint32_t *params, uint32_t seed, float *out);
void oracle_light_pass(const bdpt_sphere *sp, unsigned n, const float *rnd, int current_sample, bdpt_lightpath *lp);
void oracle_path_passes(const bdpt_sphere *sp, unsigned n, const float *rnd, const bdpt_camera *cam, int W, int H,
                        int y0, int y1, const bdpt_lightpath *lp, const unsigned *sid, const int *vlp, int npass,
                        bdpt_vec *colors, unsigned *counter, unsigned char *pixels, int nthreads, uint64_t *stats);

static int run(const char *dat, const char *scene, int W, int H, int npass)
{
    bdpt_camera cam;
    bdpt_sphere *sp = NULL;
    unsigned n = 0;
    if (bdpt_read_scene(scene, &cam, &sp, &n) != BDPT_OK) return 1;
    bdpt_update_camera(&cam, W, H);
    uint32_t *params = malloc(sizeof(uint32_t) * 4 * BDPT_MT_RNG_COUNT);
    FILE *f = fopen(dat, "rb");
    if (!f || fread(params, sizeof(uint32_t) * 4 * BDPT_MT_RNG_COUNT, 1, f) != 1) return 1;
    fclose(f);
    float *rnd = malloc(sizeof(float) * BDPT_RAND_N);
    bdpt_lightpath *lp = calloc(BDPT_LIGHT_POINTS, sizeof *lp);
    for (int i = 0; i < BDPT_MT_RNG_COUNT; i++) params[4 * i + 3] = 0;
    oracle_mt607(params, 0, rnd);
    oracle_light_pass(sp, n, rnd, 0, lp);
    bdpt_pass_state ps;
    bdpt_pass_state_init(&ps);
    bdpt_pass_state_light(&ps);
    unsigned *sid = malloc(sizeof(unsigned) * npass);
    int *vlp = malloc(sizeof(int) * npass);
    bdpt_pass_schedule(&ps, npass, sid, vlp);
    const size_t np = (size_t)W * H;
    bdpt_vec *col = calloc(np, sizeof *col), *col2 = calloc(np, sizeof *col2);
    unsigned *cnt = calloc(np, sizeof *cnt), *cnt2 = calloc(np, sizeof *cnt2);
    unsigned char *px = calloc(4 * np, 1), *px2 = calloc(4 * np, 1);
    oracle_path_passes(sp, n, rnd, &cam, W, H, 0, H, lp, sid, vlp, npass, col, cnt, px, 1, NULL);

    bdpt_ctx *ctx = NULL;
    int rc = bdpt_create(&ctx, sp, n, W, H, dat, BDPT_DEVICE_CPU);
    if (rc == BDPT_OK) rc = bdpt_set_camera(ctx, &cam);
    if (rc == BDPT_OK) rc = bdpt_light_pass(ctx, 0);
    if (rc == BDPT_OK) rc = bdpt_path_passes(ctx, sid, vlp, npass);
    if (rc == BDPT_OK) rc = bdpt_read_radiance(ctx, col2, cnt2);
    if (rc == BDPT_OK) rc = bdpt_read_pixels(ctx, px2);
    const int same = rc == BDPT_OK && !memcmp(col, col2, sizeof *col * np) && !memcmp(cnt, cnt2, sizeof *cnt * np) &&
                     !memcmp(px, px2, 4 * np);
    printf("%s %dx%d x %d: %s\n", scene, W, H, npass, same ? "equal" : "DIFFERENT");
    bdpt_destroy(ctx);
    free(params); free(rnd); free(lp); free(sid); free(vlp);
    free(col); free(col2); free(cnt); free(cnt2); free(px); free(px2);
    bdpt_free_scene(sp);
    return same ? 0 : 1;
}

int main(int argc, char **argv)
{
    if (argc < 3) return 2;
    int bad = 0;
    for (int a = 2; a < argc; a++) bad |= run(argv[1], argv[a], 23, 17, 3);
    return bad;
}
