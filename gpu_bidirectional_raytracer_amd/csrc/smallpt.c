/*
 * smallpt.c -- headless C host of the MI355X path tracer: the drop-in for the reference's
 * src/smallpt_cpu.c main()/UpdateRendering*()/ReInit*() and the IdleFunc/KeyFunc loop of
 * src/display_func.c, with GLUT replaced by a scripted key sequence.
 *
 *   smallpt [<width> <height> <scene.scn>] [--spp N] [--batch B] [--keys KEYS] [--out F.ppm]
 *           [--device D | --gpus N | --devices D0,D1,...] [--tile ROWS] [--seed S] [--dat PATH]
 *
 * Without positional arguments the built-in CornellSpheres scene is used (smallpt_cpu.c:400).
 * Like the reference, width/height get +1 (smallpt_cpu.c:409-410).  The first frame runs the
 * light pass (UpdateRendering2) and then path passes; N passes are fused into launches of B.
 * KEYS replays KeyFunc/SpecialFunc: a d w s r f (camera moves), ' ' (re-init), + - (select
 * sphere), 4 6 8 2 9 3 (move the selected sphere), U D L R (arrow keys), P/p (PageUp/Down
 * targets -> here 'P' = PageUp, 'Q' = PageDown), p (SavePPM with the reference's file name);
 * after each key N more passes are rendered.  --p6 writes --out as binary P6.
 * --gpus N (devices 0..N-1) or --devices LIST renders one frame on several GPUs of this process
 * (bdpt_create_multi: pixel bands of --tile rows, default 8, frame assembled by an RCCL reduce);
 * --seed S seeds the pass offsets' rand() (default 1: the reference never calls srand).
 * --checkpoint F saves the accumulation, the pass schedule and the render state (camera, scene,
 * MT table seed, VLPs: keys may have edited them) at the end; --resume F restores all of it after
 * the first light pass, so a run continues exactly where the saved one stopped.
 */
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

static void get_state(const host *h, host_state *s)
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

int main(int argc, char **argv)
{
    host h;
    memset(&h, 0, sizeof(h));
    int spp = 16, batch = 64, device = 0, npos = 0, p6 = 0, ndev = 0, tile = 8;
    int devices[64];
    unsigned seed = 1;
    const char *pos[3] = {0, 0, 0}, *out = NULL, *keys = "", *dat = "assets/data/MersenneTwister.dat";
    const char *ckpt = NULL, *resume = NULL;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--spp") && a + 1 < argc) spp = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--batch") && a + 1 < argc) batch = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--keys") && a + 1 < argc) keys = argv[++a];
        else if (!strcmp(argv[a], "--out") && a + 1 < argc) out = argv[++a];
        else if (!strcmp(argv[a], "--device") && a + 1 < argc) device = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--gpus") && a + 1 < argc) {
            ndev = atoi(argv[++a]);
            if (ndev < 1 || ndev > 64) { fprintf(stderr, "--gpus: 1..64\n"); return 1; }
            for (int k = 0; k < ndev; k++) devices[k] = k;
        } else if (!strcmp(argv[a], "--devices") && a + 1 < argc) {
            ndev = 0;
            for (char *t = strtok(argv[++a], ","); t && ndev < 64; t = strtok(NULL, ",")) devices[ndev++] = atoi(t);
            if (ndev < 1) { fprintf(stderr, "--devices: empty list\n"); return 1; }
        } else if (!strcmp(argv[a], "--tile") && a + 1 < argc) tile = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--seed") && a + 1 < argc) seed = (unsigned)strtoul(argv[++a], NULL, 10);
        else if (!strcmp(argv[a], "--dat") && a + 1 < argc) dat = argv[++a];
        else if (!strcmp(argv[a], "--p6")) p6 = 1;
        else if (!strcmp(argv[a], "--checkpoint") && a + 1 < argc) ckpt = argv[++a];
        else if (!strcmp(argv[a], "--resume") && a + 1 < argc) resume = argv[++a];
        else if (npos < 3) pos[npos++] = argv[a];
        else { fprintf(stderr, "Usage: %s <window width> <window height> <scene file>\n", argv[0]); return -1; }
    }
    fprintf(stderr, "Usage: %s\n", argv[0]);
    fprintf(stderr, "Usage: %s <window width> <window height> <scene file>\n", argv[0]);
    if (npos == 3) {
        h.width = atoi(pos[0]);
        h.height = atoi(pos[1]);
        fprintf(stderr, "Reading scene: %s\n", pos[2]);
        if (bdpt_read_scene(pos[2], &h.camera, &h.spheres, &h.n) != BDPT_OK) exit(-1);
        fprintf(stderr, "Scene size: %u\n", h.n);
    } else if (npos == 0) {
        h.width = 640;                                   /* display_func.c:50-52 defaults */
        h.height = 480;
        h.spheres = malloc(sizeof(bdpt_sphere) * 9);
        h.n = bdpt_default_scene(&h.camera, h.spheres);
    } else {
        exit(-1);
    }
    h.height += 1;
    h.width += 1;
    bdpt_update_camera(&h.camera, h.width, h.height);
    bdpt_pass_state_init(&h.ps);
    if (seed != 1) bdpt_srand(&h.ps.rng, seed);

    fprintf(stderr, "Allocate Buffers\n");
    int rc = ndev ? bdpt_create_multi(&h.ctx, h.spheres, h.n, h.width, h.height, dat, devices, ndev)
                  : bdpt_create(&h.ctx, h.spheres, h.n, h.width, h.height, dat, device);
    if (rc != BDPT_OK) {
        fprintf(stderr, "Unable to allocate GPU data: %s\n", bdpt_create_error());
        return 1;
    }
    if (ndev) {
        report(&h, bdpt_set_shard(h.ctx, 0, 1, tile), "bands");
        fprintf(stderr, "Devices: %d, frame reduce: %s\n", bdpt_num_devices(h.ctx), bdpt_reduce_backend(h.ctx));
    }
    report(&h, bdpt_set_camera(h.ctx, &h.camera), "camera");

    /* IdleFunc display_func.c:192-217: frame 1 = light pass then path pass; then path passes */
    update_rendering2(&h);
    if (resume) {
        host_state st;
        rc = bdpt_load_checkpoint(h.ctx, resume, &st, sizeof st);
        if (rc != BDPT_OK) {
            fprintf(stderr, "Resume failed: %s\n", bdpt_last_error(h.ctx));
            bdpt_destroy(h.ctx);
            return 1;
        }
        h.ps = st.ps;
        h.current_sample = st.current_sample;
        h.reinit_counter = st.reinit_counter;
        h.current_sphere = st.current_sphere;
        h.total_time = st.total_time;
        /* the checkpoint restored the context's camera and scene (edited by keys before the
         * save, perhaps): take them over, so later keys continue from the saved state */
        (void)bdpt_get_camera(h.ctx, &h.camera);
        const int n = bdpt_get_scene(h.ctx, NULL, 0);
        if (n > 0 && (unsigned)n != h.n) {
            bdpt_sphere *sp = malloc(sizeof(bdpt_sphere) * (size_t)n);
            if (!sp) { bdpt_destroy(h.ctx); return 1; }
            if (npos == 3) bdpt_free_scene(h.spheres); else free(h.spheres);
            h.spheres = sp;
            npos = 0;                                          /* now malloc'd here: free() */
        }
        if (n >= 0) h.n = (unsigned)bdpt_get_scene(h.ctx, h.spheres, (unsigned)(n > 0 ? n : 0));
        fprintf(stderr, "Resumed at pass %d\n", h.current_sample);
    }
    for (int done = 0; done < spp; done += batch)
        update_rendering(&h, spp - done < batch ? spp - done : batch);
    for (const char *k = keys; *k; k++) {
        key(&h, (unsigned char)*k);
        for (int done = 0; done < spp; done += batch)
            update_rendering(&h, spp - done < batch ? spp - done : batch);
    }
    if (out) rc = save_ppm(&h, out, p6);
    if (ckpt) {
        host_state st;
        get_state(&h, &st);
        const int crc = bdpt_save_checkpoint(h.ctx, ckpt, &st, sizeof st);
        report(&h, crc, "Checkpoint");
        if (rc == BDPT_OK) rc = crc;
    }
    bdpt_destroy(h.ctx);
    if (npos == 3) bdpt_free_scene(h.spheres); else free(h.spheres);
    return rc == BDPT_OK ? 0 : 1;
}
