/*
 * smallpt_app.h -- the host state and the reference's host-side operations shared by the headless
 * host (smallpt.c) and the optional display (smallpt_gl.c): UpdateRendering / UpdateRendering2
 * (smallpt_cpu.c:265-362), ReInit / ReInitScene (:365-387), SavePPM (:238-262) and the
 * KeyFunc / SpecialFunc dispatch (display_func.c:278-437) over the C-ABI of include/bdpt.h.
 */
#ifndef SMALLPT_APP_H
#define SMALLPT_APP_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "../../include/bdpt.h"

static double wall_clock(void)                            /* WallClockTime display_func.c:61 */
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + t.tv_usec / 1000000.0;
}

typedef struct {
    bdpt_ctx *ctx;
    bdpt_camera camera;
    bdpt_sphere *spheres;
    unsigned n;
    int width, height;
    int current_sample, reinit_counter, current_sphere;
    float total_time;
    bdpt_pass_state ps;
} host;

static void report(host *h, int rc, const char *what)
{
    if (rc != BDPT_OK) fprintf(stderr, "%s failed: %s\n", what, bdpt_last_error(h->ctx));
}

/* UpdateRendering2 smallpt_cpu.c:300-362 */
static void update_rendering2(host *h)
{
    printf("UpdateRendering2\n");
    report(h, bdpt_light_pass(h->ctx, h->current_sample), "Kernel Light Tracing");
    bdpt_pass_state_light(&h->ps);
}

/* npass x UpdateRendering smallpt_cpu.c:265-297, fused into one launch */
static void update_rendering(host *h, int npass)
{
    unsigned *sid = malloc(sizeof(unsigned) * npass);
    int *vlp = malloc(sizeof(int) * npass);
    bdpt_pass_schedule(&h->ps, npass, sid, vlp);
    double start = wall_clock();
    int rc = bdpt_path_passes(h->ctx, sid, vlp, npass);
    if (rc == BDPT_OK) rc = bdpt_synchronize(h->ctx);
    report(h, rc, "Kernel RadiancePathTracing");
    h->current_sample += npass;
    const float elapsed = (float)(wall_clock() - start);
    h->total_time += elapsed;
    const float sample_sec = (float)h->height * h->width * npass / elapsed;
    printf("Rendering time %.3f sec (pass %d) Total:%.2f  Sample/sec  %.1fK\n", elapsed,
           h->current_sample, h->total_time, sample_sec / 1000.f);
    free(sid);
    free(vlp);
}

/* ReInit smallpt_cpu.c:373-387 (buffers persist; only the accumulation restarts) */
static void reinit(host *h)
{
    report(h, bdpt_reset_accum(h->ctx), "ReInit");
    h->reinit_counter++;
    bdpt_update_camera(&h->camera, h->width, h->height);
    report(h, bdpt_set_camera(h->ctx, &h->camera), "ReInit camera");
    h->current_sample = 0;
    if (h->reinit_counter % 2 == 0) update_rendering2(h);
    update_rendering(h, 1);
}

/* ReInitScene smallpt_cpu.c:365-371 */
static void reinit_scene(host *h)
{
    h->current_sample = 0;
    report(h, bdpt_reset_accum(h->ctx), "ReInitScene");
    report(h, bdpt_set_scene(h->ctx, h->spheres, h->n), "ReInitScene upload");
    update_rendering2(h);
}

/* SavePPM smallpt_cpu.c:238-262 ('p' in KeyFunc): reference file name, ASCII P3 */
static int save_ppm(host *h, const char *path, int binary)
{
    char name[64];
    if (!path) {
        bdpt_ppm_name(name, (int)sizeof name, h->total_time, h->current_sample);
        path = name;
    }
    unsigned char *rgba = malloc(4 * (size_t)h->width * h->height);
    int rc = rgba ? bdpt_read_pixels(h->ctx, rgba) : BDPT_ENOMEM;
    if (rc == BDPT_OK)
        rc = binary ? bdpt_save_ppm_binary(path, rgba, h->width, h->height)
                    : bdpt_save_ppm(path, rgba, h->width, h->height);
    report(h, rc, "SavePPM");
    free(rgba);
    return rc;
}

/* what a checkpoint carries besides the frame: the pass schedule and the host counters */
typedef struct {
    bdpt_pass_state ps;
    int current_sample, reinit_counter, current_sphere;
    float total_time;
} host_state;

__attribute__((unused)) static void get_state(const host *h, host_state *s)
{
    memset(s, 0, sizeof *s);
    s->ps = h->ps;
    s->current_sample = h->current_sample;
    s->reinit_counter = h->reinit_counter;
    s->current_sphere = h->current_sphere;
    s->total_time = h->total_time;
}

static void key(host *h, int k)
{
    if (k == 'p') {
        (void)save_ppm(h, NULL, 0);
        return;
    }
    int code = k;
    if (k == 'U') code = BDPT_KEY_UP;
    else if (k == 'D') code = BDPT_KEY_DOWN;
    else if (k == 'L') code = BDPT_KEY_LEFT;
    else if (k == 'R') code = BDPT_KEY_RIGHT;
    else if (k == 'P') code = BDPT_KEY_PAGE_UP;
    else if (k == 'Q') code = BDPT_KEY_PAGE_DOWN;
    if (k == '+' || k == '-') {
        h->current_sphere = k == '+' ? (h->current_sphere + 1) % (int)h->n
                                     : (h->current_sphere + ((int)h->n - 1)) % (int)h->n;
        fprintf(stderr, "Selected sphere %d (%f %f %f)\n", h->current_sphere,
                h->spheres[h->current_sphere].p.x, h->spheres[h->current_sphere].p.y,
                h->spheres[h->current_sphere].p.z);
        reinit_scene(h);
    } else if (bdpt_sphere_key(h->spheres, h->n, h->current_sphere, k)) {
        reinit_scene(h);
    } else if (bdpt_camera_key(&h->camera, code)) {
        reinit(h);
    }
}

#endif
