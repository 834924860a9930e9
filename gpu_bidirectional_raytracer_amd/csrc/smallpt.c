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
#include "smallpt_app.h"

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
