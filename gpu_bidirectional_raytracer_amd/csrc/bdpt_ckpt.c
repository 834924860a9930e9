/*
 * bdpt_ckpt.c -- checkpoint / resume of a render context (no reference counterpart: the
 * reference keeps its accumulation only in dev_colors / dev_counter, smallpt_cpu.c:153-237;
 * SURVEY.md 5).  Written over the public entry points of include/bdpt.h only, so libbdpt.so and
 * the sanitizer build (tests/native/asan_cpu_abi.cpp) share this one implementation.
 *
 * File layout (little-endian, packed):
 *   header   "BDPTCKP2", int32 W, H, uint32 host_bytes, n_spheres, table seed, flags, 2 x reserved
 *   camera   60 B  (bdpt_camera; zeros if none was set: flags bit 1)
 *   spheres  44 B x n_spheres
 *   VLPs     36 B x 4096 (dev_lp)
 *   colors   12 B x W*H, counter 4 B x W*H
 *   host     host_bytes of caller state (pass schedule, host counters)
 * flags: bit 0 = an MT607 table exists (then `seed` regenerates it), bit 1 = the camera is set.
 *
 * The render state travels with the frame: after KeyFunc edits (ReInit / ReInitScene,
 * display_func.c:278-437) the camera, the spheres, the table and the VLPs differ from what the
 * scene file gives, and a resume must continue with the edited ones or the frame mixes two
 * renders.  The VLPs are stored, not recomputed: entries a light pass does not write keep older
 * values (smallpt_cpu.c:311-342), so they depend on the run's history.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/bdpt.h"

/* provided by the context layer: record `msg` as the context's last error, return `code` */
int bdpt__fail(bdpt_ctx *c, int code, const char *msg);

static const char kMagic[8] = {'B', 'D', 'P', 'T', 'C', 'K', 'P', '2'};
static const char kMagicV1[8] = {'B', 'D', 'P', 'T', 'C', 'K', 'P', '1'};   /* round-2 format */
enum { kHasRand = 1, kHasCamera = 2 };

typedef struct {
    char magic[8];
    int32_t width, height;
    uint32_t host_bytes, n_spheres, seed, flags, reserved[2];
} ckpt_header;

static int failf(bdpt_ctx *c, int code, const char *fmt, const char *a, const char *b)
{
    char msg[8800];
    snprintf(msg, sizeof msg, fmt, a, b);
    return bdpt__fail(c, code, msg);
}

/* Flush a written file to disk; then the rename publishes complete contents. */
static int sync_close(FILE *f)
{
    int ok = fflush(f) == 0;
    ok = fsync(fileno(f)) == 0 && ok;
    return (fclose(f) == 0) && ok;
}

static void sync_dir_of(const char *path)
{
    char dir[4096];
    snprintf(dir, sizeof dir, "%s", path);
    char *slash = strrchr(dir, '/');
    if (slash == dir) slash[1] = 0;
    else if (slash) *slash = 0;
    else snprintf(dir, sizeof dir, ".");
    const int fd = open(dir, O_RDONLY | O_DIRECTORY);
    if (fd >= 0) {
        (void)fsync(fd);
        close(fd);
    }
}

int bdpt_save_checkpoint(bdpt_ctx *c, const char *path, const void *host_state, unsigned host_bytes)
{
    if (!c || !path || (host_bytes && !host_state)) return BDPT_EINVAL;
    bdpt_camera cam;
    memset(&cam, 0, sizeof cam);
    ckpt_header h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, kMagic, 8);
    const int n = bdpt_get_scene(c, NULL, 0);
    if (n < 0) return n;
    if (bdpt_get_camera(c, &cam) == BDPT_OK) h.flags |= kHasCamera;
    if (bdpt_rand_seed(c, &h.seed) == BDPT_OK) h.flags |= kHasRand;
    int W = 0, H = 0;
    if (bdpt_frame_size(c, &W, &H) != BDPT_OK) return BDPT_EINVAL;
    h.width = W;
    h.height = H;
    h.host_bytes = host_bytes;
    h.n_spheres = (uint32_t)n;
    const size_t np = (size_t)W * H;
    bdpt_sphere *sp = malloc(sizeof(bdpt_sphere) * (n ? n : 1));
    bdpt_lightpath *lp = malloc(sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS);
    bdpt_vec *col = malloc(sizeof(bdpt_vec) * np);
    unsigned *cnt = malloc(sizeof(unsigned) * np);
    int rc = (sp && lp && col && cnt) ? BDPT_OK : BDPT_ENOMEM;
    if (rc == BDPT_OK && bdpt_get_scene(c, sp, (unsigned)n) != n) rc = BDPT_ESTATE;
    if (rc == BDPT_OK) rc = bdpt_read_lightpaths(c, lp);
    if (rc == BDPT_OK) rc = bdpt_read_radiance(c, col, cnt);
    if (rc == BDPT_OK) {
        char tmp[4200];
        snprintf(tmp, sizeof tmp, "%s.tmp.%ld", path, (long)getpid());
        FILE *f = fopen(tmp, "wb");
        if (!f) {
            rc = failf(c, BDPT_EIO, "bdpt_save_checkpoint: cannot open %s%s", tmp, "");
        } else {
            int ok = fwrite(&h, sizeof h, 1, f) == 1 && fwrite(&cam, sizeof cam, 1, f) == 1 &&
                     fwrite(sp, sizeof(bdpt_sphere), (size_t)n, f) == (size_t)n &&
                     fwrite(lp, sizeof(bdpt_lightpath), BDPT_LIGHT_POINTS, f) == BDPT_LIGHT_POINTS &&
                     fwrite(col, sizeof(bdpt_vec), np, f) == np && fwrite(cnt, sizeof(unsigned), np, f) == np &&
                     (host_bytes == 0 || fwrite(host_state, 1, host_bytes, f) == host_bytes);
            ok = sync_close(f) && ok;
            if (ok) ok = rename(tmp, path) == 0;
            if (ok) {
                sync_dir_of(path);
            } else {
                unlink(tmp);
                rc = failf(c, BDPT_EIO, "bdpt_save_checkpoint: cannot write %s%s", path, "");
            }
        }
    }
    free(sp); free(lp); free(col); free(cnt);
    return rc;
}

/* The context's own render state, kept so a load that fails half way can put it back. */
typedef struct {
    int n, has_cam, has_rand;
    unsigned seed;
    bdpt_camera cam;
    bdpt_sphere *sp;
    bdpt_lightpath *lp;
    bdpt_vec *col;
    unsigned *cnt;
} ctx_state;

static void state_free(ctx_state *s)
{
    free(s->sp); free(s->lp); free(s->col); free(s->cnt);
}

static int state_save(bdpt_ctx *c, ctx_state *s, size_t np)
{
    memset(s, 0, sizeof *s);
    s->n = bdpt_get_scene(c, NULL, 0);
    if (s->n < 0) return s->n;
    s->has_cam = bdpt_get_camera(c, &s->cam) == BDPT_OK;
    s->has_rand = bdpt_rand_seed(c, &s->seed) == BDPT_OK;
    s->sp = malloc(sizeof(bdpt_sphere) * (s->n ? s->n : 1));
    s->lp = malloc(sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS);
    s->col = malloc(sizeof(bdpt_vec) * np);
    s->cnt = malloc(sizeof(unsigned) * np);
    if (!(s->sp && s->lp && s->col && s->cnt)) return BDPT_ENOMEM;
    if (bdpt_get_scene(c, s->sp, (unsigned)s->n) != s->n) return BDPT_ESTATE;
    int rc = bdpt_read_lightpaths(c, s->lp);
    if (rc == BDPT_OK) rc = bdpt_read_radiance(c, s->col, s->cnt);
    return rc;
}

/* Put the saved state back (best effort: the first failure is the caller's error). */
static void state_restore(bdpt_ctx *c, const ctx_state *s)
{
    if (bdpt_set_scene(c, s->sp, (unsigned)s->n) != BDPT_OK) return;
    if (s->has_cam && bdpt_set_camera(c, &s->cam) != BDPT_OK) return;
    if (s->has_rand && bdpt_generate_rand(c, s->seed) != BDPT_OK) return;
    if (bdpt_write_lightpaths(c, s->lp) != BDPT_OK) return;
    (void)bdpt_write_radiance(c, s->col, s->cnt);
}

int bdpt_load_checkpoint(bdpt_ctx *c, const char *path, void *host_state, unsigned host_bytes)
{
    if (!c || !path || (host_bytes && !host_state)) return BDPT_EINVAL;
    int W = 0, H = 0;
    if (bdpt_frame_size(c, &W, &H) != BDPT_OK) return BDPT_EINVAL;
    FILE *f = fopen(path, "rb");
    if (!f) return failf(c, BDPT_EIO, "bdpt_load_checkpoint: cannot open %s%s", path, "");
    ckpt_header h;
    if (fread(&h, sizeof h, 1, f) != 1) {
        fclose(f);
        return failf(c, BDPT_EIO, "bdpt_load_checkpoint: %s is not a checkpoint%s", path, "");
    }
    if (memcmp(h.magic, kMagicV1, 8) == 0) {
        fclose(f);
        return failf(c, BDPT_EINVAL, "bdpt_load_checkpoint: %s is a version-1 checkpoint (BDPTCKP1: the frame "
                     "without its scene, camera, table and VLPs), which this build cannot resume%s", path, "");
    }
    if (memcmp(h.magic, kMagic, 8) != 0) {
        fclose(f);
        return failf(c, BDPT_EIO, "bdpt_load_checkpoint: %s is not a checkpoint%s", path, "");
    }
    if (h.width != W || h.height != H || h.host_bytes != host_bytes || h.n_spheres > (1u << 20)) {
        char msg[600];
        snprintf(msg, sizeof msg, "bdpt_load_checkpoint: %s holds %dx%d with %u host bytes, not %dx%d with %u",
                 path, h.width, h.height, h.host_bytes, W, H, host_bytes);
        fclose(f);
        return bdpt__fail(c, BDPT_EINVAL, msg);
    }
    const size_t np = (size_t)W * H, n = h.n_spheres;
    bdpt_camera cam;
    bdpt_sphere *sp = malloc(sizeof(bdpt_sphere) * (n ? n : 1));
    bdpt_lightpath *lp = malloc(sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS);
    bdpt_vec *col = malloc(sizeof(bdpt_vec) * np);
    unsigned *cnt = malloc(sizeof(unsigned) * np);
    unsigned char *hs = malloc(host_bytes ? host_bytes : 1);
    int rc = (sp && lp && col && cnt && hs) ? BDPT_OK : BDPT_ENOMEM;
    if (rc == BDPT_OK &&
        !(fread(&cam, sizeof cam, 1, f) == 1 && fread(sp, sizeof(bdpt_sphere), n, f) == n &&
          fread(lp, sizeof(bdpt_lightpath), BDPT_LIGHT_POINTS, f) == BDPT_LIGHT_POINTS &&
          fread(col, sizeof(bdpt_vec), np, f) == np && fread(cnt, sizeof(unsigned), np, f) == np &&
          (host_bytes == 0 || fread(hs, 1, host_bytes, f) == host_bytes)))
        rc = failf(c, BDPT_EIO, "bdpt_load_checkpoint: %s is truncated%s", path, "");
    fclose(f);
    /* the context's state before the load: put back if a restore step fails */
    ctx_state old;
    int saved = 0;
    if (rc == BDPT_OK) {
        rc = state_save(c, &old, np);
        saved = 1;
    }
    /* restore in dependency order: scene (ReInitScene upload, skipped when the context already
     * holds these spheres byte for byte: it would drop the specialised kernels and restart the
     * stream-mode measurement), camera, table, VLPs, frame */
    int step_rc = BDPT_OK;
    if (rc == BDPT_OK && !((size_t)old.n == n && (n == 0 || memcmp(old.sp, sp, sizeof(bdpt_sphere) * n) == 0)))
        rc = step_rc = bdpt_set_scene(c, sp, (unsigned)n);
    if (rc == BDPT_OK && (h.flags & kHasCamera)) rc = step_rc = bdpt_set_camera(c, &cam);
    if (rc == BDPT_OK && (h.flags & kHasRand)) rc = step_rc = bdpt_generate_rand(c, h.seed);
    if (rc == BDPT_OK) rc = step_rc = bdpt_write_lightpaths(c, lp);
    if (rc == BDPT_OK) rc = step_rc = bdpt_write_radiance(c, col, cnt);
    if (step_rc != BDPT_OK) {                   /* a restore step failed: the old state back */
        char msg[512];
        snprintf(msg, sizeof msg, "%s", bdpt_last_error(c));
        state_restore(c, &old);
        (void)bdpt__fail(c, step_rc, msg);
    }
    if (rc == BDPT_OK && host_bytes) memcpy(host_state, hs, host_bytes);
    if (saved) state_free(&old);
    free(sp); free(lp); free(col); free(cnt); free(hs);
    return rc;
}
