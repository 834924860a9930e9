/*
 * bdpt.h -- C-ABI of the MI355X bidirectional path tracer (libbdpt.so).
 *
 * This is the drop-in boundary for the render path of sim186/gpu_bidirectional_raytracer.
 * In the reference the boundary is the set of module globals plus <<<>>> launches inside
 * src/smallpt_cpu.c; every entry point below names the reference function it replaces.
 * Plain C: no torch / HIP types in any signature.  All functions return 0 on success and a
 * negative BDPT_E* code on failure; the message is in bdpt_last_error() (the reference prints
 * cudaGetErrorString() and continues, smallpt_cpu.c:169-233 -- the host does the same with this).
 * One context per GPU; calls on one context must not run concurrently (the reference is single-
 * threaded too); different contexts are independent.
 *
 * Types are layout-compatible with the reference headers (static-asserted in the library):
 *   bdpt_vec       == Vec        include/vec.h:4-6       (12 B)
 *   bdpt_ray       == Ray        include/geom.h:9-11     (24 B)
 *   bdpt_sphere    == Sphere     include/geom.h:23-27    (44 B, enum Refl stored as int)
 *   bdpt_lightpath == LightPath  include/geom.h:29-33    (36 B)
 *   bdpt_camera    == Camera     include/camera.h:7-12   (60 B)
 */
#ifndef BDPT_H
#define BDPT_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } bdpt_vec;
typedef struct { bdpt_vec o, d; } bdpt_ray;
enum { BDPT_DIFF = 0, BDPT_SPEC = 1, BDPT_REFR = 2, BDPT_LITE = 3 }; /* geom.h:18-20 enum Refl */
typedef struct { float rad; bdpt_vec p, e, c; int refl; } bdpt_sphere;
typedef struct { bdpt_vec hp, rad, nl; } bdpt_lightpath;
typedef struct { bdpt_vec orig, target, dir, x, y; } bdpt_camera;

/* Compile-time constants of the reference (cons.h, geom.h, smallpt_cpu.c:67-69). */
#define BDPT_MT_RNG_COUNT 4096              /* MersenneTwister.h:28                         */
#define BDPT_N_PER_RNG    1876              /* AlignUp(DivideRoundUp(7680000,4096),2)       */
#define BDPT_RAND_N       (4096 * 1876)     /* 7,684,096 floats = 30.7 MB                   */
#define BDPT_LIGHT_POINTS 4096              /* geom.h:15 LIGHT_POINTS (DEPTH=1, MAX_VLP=1)  */
#define BDPT_MAX_SEGMENTS 7                 /* device.cu:621 `depth > 6` break               */
#define BDPT_COUNTER_CAP  30000u            /* device.cu:607 `counter[i] < 30000`            */
#define BDPT_MAX_STREAMS  128               /* bdpt_set_streams upper bound                  */

/* Error codes. */
#define BDPT_OK        0
#define BDPT_EINVAL   -1   /* bad argument                                   */
#define BDPT_EIO      -2   /* file could not be read / written               */
#define BDPT_EHIP     -3   /* HIP runtime error                              */
#define BDPT_ENOMEM   -4   /* allocation failed                              */
#define BDPT_ESTATE   -5   /* call out of order (e.g. path pass before RNG)  */

typedef struct bdpt_ctx bdpt_ctx;

/* ---- render-path context (replaces smallpt_cpu.c module globals + AllocateBuffers) ---- */

/* AllocateBuffers smallpt_cpu.c:153-237 + loadMTGPU MersenneTwister_kernel.cu:23-36.
 * W,H are the internal sizes AFTER the reference's +1 (smallpt_cpu.c:409-410).
 * `device` is the HIP ordinal this context renders on, or BDPT_DEVICE_CPU for the host backend
 * (the smallpt_cpu.c CPU path: the same render path on the CPU cores, no GPU needed; identical
 * results; BDPT_CPU_THREADS sets its thread count).  Accumulation starts zeroed. */
#define BDPT_DEVICE_CPU (-1)
int  bdpt_create(bdpt_ctx **out, const bdpt_sphere *spheres, unsigned n_spheres,
                 int width, int height, const char *mt_dat_path, int device);
/* Multi-GPU context (SURVEY.md 8(b) `bdpt_create(..., devices, ndev)`; the reference renders on
 * one device, smallpt_cpu.c:422).  One sub-context per entry of devices[]: device k renders the
 * 8-row pixel bands (y / 8) % ndev == k, every other entry point below applies to all devices,
 * and the read-back entry points (bdpt_read_radiance / _pixels, bdpt_device_buffers,
 * bdpt_update_pixels) return the frame assembled on devices[0] by a sum-reduce: an in-process
 * RCCL ncclReduce over an ncclCommInitAll communicator when the devices are distinct, else peer
 * copies (several shards on one GPU, or BDPT_REDUCE=peer).  The result equals a one-device
 * context's bit for bit.  bdpt_set_shard(ctx, s, n, band) makes the whole group shard s of n
 * groups (multi-node).  bdpt_path_timing / bdpt_kernel_timing report the slowest device. */
int  bdpt_create_multi(bdpt_ctx **out, const bdpt_sphere *spheres, unsigned n_spheres,
                       int width, int height, const char *mt_dat_path, const int *devices, int ndev);
int  bdpt_num_devices(const bdpt_ctx *ctx);
/* "rccl", "peer", or "none" (a one-device context from bdpt_create). */
const char *bdpt_reduce_backend(const bdpt_ctx *ctx);
/* The frame reduce in words, into buf (at most cap bytes, NUL-terminated): for "rccl" the RCCL
 * version, the rank count ncclCommInitAll was given and the device list; for "peer" why RCCL
 * is not used.  Returns the full length, BDPT_EINVAL on bad arguments. */
int  bdpt_reduce_info(const bdpt_ctx *ctx, char *buf, int cap);
/* ncclGetVersion of the librccl this library binds to (e.g. 22606 = 2.26.6), BDPT_ESTATE if it
 * cannot be loaded.  Needs no GPU. */
int  bdpt_rccl_version(void);
/* Assemble the frame now (otherwise done on the first read-back after a change). */
int  bdpt_reduce_frame(bdpt_ctx *ctx);
/* FreeBuffers smallpt_cpu.c:98-110. */
void bdpt_destroy(bdpt_ctx *ctx);
const char *bdpt_last_error(const bdpt_ctx *ctx);
/* Message of the last failed bdpt_create (no context exists then). */
const char *bdpt_create_error(void);

/* ReInitScene smallpt_cpu.c:365-371 (re-upload of dev_spheres, :229). Does not run the light pass. */
int  bdpt_set_scene(bdpt_ctx *ctx, const bdpt_sphere *spheres, unsigned n_spheres);
/* Camera by value, as RadiancePathTracingKernel receives it (device.cu:548). Call after
 * bdpt_update_camera(). */
int  bdpt_set_camera(bdpt_ctx *ctx, const bdpt_camera *camera);
/* counter[] := 0 (ReInit -> AllocateBuffers, smallpt_cpu.c:204); colors/pixels follow on the
 * next pass because counter==0 assigns (device.cu:774). */
int  bdpt_reset_accum(bdpt_ctx *ctx);
/* Multi-GPU sharding: only pixels whose row band (y / band_rows) % nshards == shard are
 * rendered; all other pixels stay zero so a sum-reduce of the frames is exact. Default 0,1,8;
 * band_rows a multiple of 8 (the tile height) launches only the shard's own tile rows. */
int  bdpt_set_shard(bdpt_ctx *ctx, int shard, int nshards, int band_rows);
/* Pass streams (no reference counterpart; results are bit-identical for every S): S lanes per
 * pixel render passes s, s+S, ... into an HBM radiance buffer (12 B per pass and pixel) and an
 * ordered fold applies the running mean of device.cu:774-787 in pass order.
 *   0  = auto (default): the first ten calls of >= 2 passes measure, in this order, the
 *        pass-stream kernel with two passes per lane (S = ceil(passes / 2); one per lane in
 *        launches of < 4 passes or with the BVH), the fused kernel with paired segment loads,
 *        pass streams with four passes per lane (S = ceil(passes / 4), launches of >= 8), two
 *        per lane again, the fused kernel without pairing, four per lane again, twice pass
 *        streams with pixel pools (S = passes, lanes restart on new pixels of their pass;
 *        specialised builds, BDPT_FEAT_POOLS), and twice the ordered in-kernel fold (units of a
 *        tile and 8 passes, running mean in registers, no radiance buffer and no fold kernel;
 *        specialised builds of frames with >= 2 x CUs x 6 tile workgroups, BDPT_FEAT_UNITS);
 *        later calls use the pass-stream variant with the
 *        fastest call, or the faster fused variant if its time per pass (path kernels + a quarter of the fold) beat that by 5 %
 *        (closed scenes with long paths favour pass streams, open scenes with short paths the
 *        fused kernel or pools); re-measured after a scene / shard / traversal change;
 *  -1  = BDPT_STREAMS_PER_LANE: always one pass per lane (S = passes per launch, <= 128);
 *   1  = the fused kernel that keeps the running mean in registers (no buffer);
 *  2..128 = that many streams. */
#define BDPT_STREAMS_PER_LANE (-1)
int  bdpt_set_streams(bdpt_ctx *ctx, int streams);
/* S used by the last bdpt_path_passes call. */
int  bdpt_last_streams(const bdpt_ctx *ctx);
/* The kernel variant the auto stream mode settled on, as BDPT_CHOICE_* bits (0 while it is still
 * measuring, or when the stream mode is not auto).  bdpt_set_stream_choice applies such a choice
 * without measuring (every device of a group); a later scene / shard / traversal / stream-mode
 * change measures again.  No reference counterpart (smallpt_cpu.c:422 renders on one device): a
 * multi-GPU job lets one device measure and gives every device its choice, so all GPUs run the
 * same kernels -- the devices of a bdpt_create_multi group do this by themselves (they follow
 * devices[0]); torchrun ranks pass rank 0's choice along (bench.py). */
#define BDPT_CHOICE_DECIDED 1               /* a choice exists                                */
#define BDPT_CHOICE_FUSED   2               /* the fused S = 1 kernel                         */
#define BDPT_CHOICE_PAIRED  4               /* the fused variant with paired segment loads    */
#define BDPT_CHOICE_QUARTER 8               /* pass streams with four passes per lane         */
#define BDPT_CHOICE_POOLS  16               /* pass streams with pixel pools                  */
#define BDPT_CHOICE_UNITS  32               /* pass streams with the ordered in-kernel fold   */
int  bdpt_stream_choice(const bdpt_ctx *ctx);
int  bdpt_set_stream_choice(bdpt_ctx *ctx, int choice);
/* Device k of a (multi-device) context (0 = devices[0]): S and BDPT_FEAT_* bits of its last
 * bdpt_path_passes call, and its BDPT_CHOICE_* bits. */
int  bdpt_device_mode(bdpt_ctx *ctx, int k, int *last_streams, int *features, int *choice);
/* Scene-specialised kernels (no reference counterpart; results are bit-identical): for scenes of
 * <= 64 spheres (brute-force traversal) the path kernel is compiled at run time (hipRTC, ~1 s, cached on disk) with the
 * sphere geometry folded in as constants.  1 = on (default), 0 = precompiled kernels only.  If
 * hipRTC is unavailable or the compile fails, the precompiled kernel runs. */
int  bdpt_set_specialize(bdpt_ctx *ctx, int on);
/* 1 if the last bdpt_path_passes call ran a specialised kernel; the reason it did not, if not. */
int  bdpt_last_specialized(const bdpt_ctx *ctx);
const char *bdpt_specialize_status(const bdpt_ctx *ctx);
/* Sphere traversal (no reference counterpart; results are bit-identical either way).  The
 * reference tests every sphere per ray (IntersectDevice device.cu:106-124); for scenes with
 * > 16 spheres of which >= 24 are of ordinary size, bdpt_set_scene also builds a BVH over those
 * (walls stay brute force) that skips only spheres that provably cannot change the answer. */
#define BDPT_TRAVERSE_AUTO  0               /* BVH when it has >= 128 spheres                */
#define BDPT_TRAVERSE_BRUTE 1               /* every sphere, like the reference             */
#define BDPT_TRAVERSE_BVH   2               /* BVH whenever the scene has one               */
int  bdpt_set_traversal(bdpt_ctx *ctx, int mode);
int  bdpt_scene_has_bvh(const bdpt_ctx *ctx);
/* BDPT_TRAVERSE_BVH or BDPT_TRAVERSE_BRUTE: what the last bdpt_path_passes call used. */
int  bdpt_last_traversal(const bdpt_ctx *ctx);
/* What the kernel of the last bdpt_path_passes call compiled in (no reference counterpart; none of
 * these changes a result): bit flags below.  The three skips leave out work whose result the
 * reference computes and never uses, so a FLOP model priced on the reference's work counts more
 * than the kernel executes ("reference-equivalent" FLOPs). */
#define BDPT_FEAT_SPECIALIZED 1             /* scene-specialised build (hipRTC)              */
#define BDPT_FEAT_DET_SKIP    2             /* whole-wave skip of sphere tests all lanes miss */
#define BDPT_FEAT_ZERO_EXIT   4             /* paths end at a black non-emitter              */
#define BDPT_FEAT_LAST_SKIP   8             /* no next direction after the 7th segment        */
#define BDPT_FEAT_BVH        16             /* BVH traversal (large scenes)                   */
#define BDPT_FEAT_STREAMS    32             /* pass streams (one pass per lane + ordered fold)*/
#define BDPT_FEAT_POOLS      64             /* pass streams with pixel pools (lanes restart on
                                               new pixels of their pass, claimed in chunks)   */
#define BDPT_FEAT_SCP       256             /* sin/cos planes: the angles' sinf/cosf loaded, not
                                               evaluated (pass streams / units, not pools)     */
#define BDPT_FEAT_UNITS     128             /* pass streams with the ordered fold in the kernel:
                                               units of (tile, range of passes) in range order,
                                               running mean in registers, no radiance buffer   */
int  bdpt_last_kernel_features(const bdpt_ctx *ctx);
/* The black-surface exit rule (BDPT_FEAT_ZERO_EXIT): 1 if ending a path at a black non-emitter is
 * provably exact for this scene -- every term the reference adds after the black hit is finite,
 * so 0 * term = +0 leaves the radiance bit-identical -- else 0.  Pure host function: the
 * specialised build asks it, and tests check it against the Python restatement. */
int  bdpt_zero_exit_safe(const bdpt_sphere *spheres, unsigned n_spheres);

/* UpdateRendering2 smallpt_cpu.c:300-362: for every emitter in sphere order,
 * seedMTGPU(current_sample*5) + RandomGPU (MT607 table), GetRayKernel and
 * RadianceLightTracingKernel (4096 VLPs). */
int  bdpt_light_pass(bdpt_ctx *ctx, int current_sample);
/* Just the MT607 table: seedMTGPU(seed) + RandomGPU<<<32,128>>> (MersenneTwister_kernel.cu:39-110). */
int  bdpt_generate_rand(bdpt_ctx *ctx, unsigned seed);

/* `npass` x UpdateRendering (smallpt_cpu.c:265-297) fused into one launch: pass p uses
 * sid[p] (= rand()%RAND_N, :270) and vlp_index[p] (the :292-293 state machine).
 * Asynchronous on the context's stream (a call only waits for the call issued 4 calls earlier,
 * whose pass-table slot it reuses); bdpt_synchronize() waits for all. */
int  bdpt_path_passes(bdpt_ctx *ctx, const unsigned *sid, const int *vlp_index, int npass);
int  bdpt_synchronize(bdpt_ctx *ctx);
/* Device time (ms, HIP events on the context's stream) of the last bdpt_path_passes call. */
int  bdpt_last_path_ms(bdpt_ctx *ctx, float *ms);
/* Accumulated device time and kernel-launch count of all path-pass calls since the last reset
 * (synchronises first).  reset != 0 zeroes the accumulators after reading them. */
int  bdpt_path_timing(bdpt_ctx *ctx, double *total_ms, long long *launches, int reset);
/* Same accumulation, but only the path kernels' own durations (one HIP event pair around each
 * path-kernel launch, excluding the pass-stream fold): what rocprof reports for that kernel.
 * Overlapped pooled launches (pixel pools, BDPT_FEAT_POOLS): consecutive launches run on two
 * streams and a launch starts while the previous one drains, so their event intervals overlap and
 * bdpt_last_path_ms, bdpt_path_timing and bdpt_kernel_timing add up to MORE than the wall time;
 * divide the wall time of a run by its launches for a per-launch rate (bench.py launch_overlap). */
int  bdpt_kernel_timing(bdpt_ctx *ctx, double *kernel_ms, long long *launches, int reset);
/* Device k of a (multi-device) context, 0 <= k < bdpt_num_devices (0 = devices[0]): its device
 * id (BDPT_DEVICE_CPU for the host backend), its own path-kernel ms and path ms (with the fold)
 * and launches since the last timing reset, and the pixels its shard owns.  Does not reset.
 * New (the reference is single-device, smallpt_cpu.c:422): lets a multi-GPU run report each
 * device's share instead of only the slowest. */
int  bdpt_device_timing(bdpt_ctx *ctx, int k, int *device, double *kernel_ms, double *path_ms,
                        long long *launches, long long *owned_pixels);

/* Read-back.  colors/counter: the float parity artefact (dev_colors / dev_counter);
 * pixels: uchar4 RGBA = pixels_buf (SavePPM, smallpt_cpu.c:241). */
int  bdpt_read_radiance(bdpt_ctx *ctx, bdpt_vec *colors, unsigned *counter);
int  bdpt_read_pixels(bdpt_ctx *ctx, unsigned char *rgba);
int  bdpt_read_rand(bdpt_ctx *ctx, float *rand_table);          /* d_Rand, BDPT_RAND_N */
int  bdpt_read_lightpaths(bdpt_ctx *ctx, bdpt_lightpath *lp);   /* dev_lp, 4096        */
/* Upload all 4096 VLPs (the counterpart of bdpt_read_lightpaths; checkpoint restore). */
int  bdpt_write_lightpaths(bdpt_ctx *ctx, const bdpt_lightpath *lp);
/* The seed of the current MT607 table (current_sample * 5 of the last light pass, or the
 * bdpt_generate_rand argument); BDPT_ESTATE before any table exists. */
int  bdpt_rand_seed(const bdpt_ctx *ctx, unsigned *seed);
/* The context's camera (BDPT_ESTATE if none was set) and scene: bdpt_get_scene copies at most
 * `cap` spheres and returns the scene's sphere count (spheres may be NULL to ask the count). */
int  bdpt_get_camera(const bdpt_ctx *ctx, bdpt_camera *camera);
/* The frame size the context was created with (internal W, H). */
int  bdpt_frame_size(const bdpt_ctx *ctx, int *width, int *height);
int  bdpt_get_scene(const bdpt_ctx *ctx, bdpt_sphere *spheres, unsigned cap);
/* Device pointers for zero-copy collectives (RCCL reduce of the radiance frame).  Path passes
 * run asynchronously on the context's own stream: bdpt_synchronize() before using them.  For a
 * multi-device context: the assembled frame on devices[0]. */
int  bdpt_device_buffers(bdpt_ctx *ctx, void **colors, void **counter, void **pixels);
/* Recompute pixels (toInt gamma) from colors on the device, e.g. after a cross-GPU reduce. */
int  bdpt_update_pixels(bdpt_ctx *ctx);

/* ---- optional display: HIP-GL interop ----
 * The caller owns the window, its OpenGL context (current on the calling thread) and a
 * pixel-unpack buffer of at least 4*W*H bytes (glGenBuffers + glBufferData(GL_PIXEL_UNPACK_BUFFER,
 * 4*W*H, NULL, GL_DYNAMIC_COPY), as CreatePBO smallpt_cpu.c:112-123 makes it).
 * bdpt_gl_register_pbo replaces cudaGLRegisterBufferObject (smallpt_cpu.c:122): BDPT_EINVAL when
 * no GL context is current (GLX or EGL, looked up in the libraries the process has loaded) or on
 * the CPU backend.  bdpt_gl_publish replaces IdleFunc's map / UpdateRendering / unmap bracket
 * (display_func.c:199-215): it maps the buffer, copies the frame's 8-bit pixels into it (the
 * layout of bdpt_read_pixels: RGBA, bottom row first, as glTexSubImage2D takes it; for a
 * multi-device context the assembled frame), unmaps it -- on every path -- and synchronises;
 * BDPT_ESTATE before a register, BDPT_EINVAL when the buffer is smaller than the frame.
 * bdpt_gl_unregister (also done by bdpt_destroy) must run while the GL context still exists. */
int  bdpt_gl_register_pbo(bdpt_ctx *ctx, unsigned int pbo);
int  bdpt_gl_publish(bdpt_ctx *ctx);
int  bdpt_gl_unregister(bdpt_ctx *ctx);

/* ---- checkpoint / resume of the accumulation (no reference counterpart: the reference keeps
 * it only in dev_colors/dev_counter) ---- */
/* Upload colors/counter (W*H each; the counterpart of bdpt_read_radiance); pixels are
 * recomputed.  Rendering then continues from that state bit for bit. */
int  bdpt_write_radiance(bdpt_ctx *ctx, const bdpt_vec *colors, const unsigned *counter);
/* File = header {"BDPTCKP2", W, H, host_bytes, n_spheres, table seed, flags} + camera + spheres +
 * the 4096 VLPs + colors + counter + host_bytes of caller state (e.g. its bdpt_pass_state and
 * current_sample, so the pass schedule resumes too).  The render state travels with the frame: a
 * run whose camera or scene was edited (KeyFunc -> ReInit / ReInitScene) resumes with the edited
 * camera, scene, MT table and VLPs, not the scene file's.  Written to a temporary file, flushed to
 * disk (fsync) and renamed into place.  Load checks W, H and host_bytes against the context, then
 * restores scene, camera, table, VLPs and accumulation (the caller re-reads its own copies with
 * bdpt_get_camera / bdpt_get_scene).  The scene upload is skipped when the context already holds
 * the same spheres byte for byte.  If a restore step fails, the context's previous scene, camera,
 * table, VLPs and accumulation are put back (best effort) and the step's error is returned; a
 * version-1 file ("BDPTCKP1", round 2) is refused with a message that says so. */
int  bdpt_save_checkpoint(bdpt_ctx *ctx, const char *path, const void *host_state, unsigned host_bytes);
int  bdpt_load_checkpoint(bdpt_ctx *ctx, const char *path, void *host_state, unsigned host_bytes);

/* ---- host utilities kept for the drop-in (display_func.c / smallpt_cpu.c) ---- */

/* ReadScene display_func.c:112-175. *spheres is malloc'd; free with bdpt_free_scene. */
int  bdpt_read_scene(const char *path, bdpt_camera *camera, bdpt_sphere **spheres,
                     unsigned *n_spheres);
void bdpt_free_scene(bdpt_sphere *spheres);
/* The built-in CornellSpheres scene (scene.h:7-18) and camera (smallpt_cpu.c:404-405),
 * used when the host is started without arguments. Returns the sphere count (9). */
unsigned bdpt_default_scene(bdpt_camera *camera, bdpt_sphere *spheres_out /* >= 9 */);
/* UpdateCamera display_func.c:177-190 (width/height are the internal sizes). */
void bdpt_update_camera(bdpt_camera *camera, int width, int height);
/* Camera moves of KeyFunc / SpecialFunc (display_func.c:278-437), headless.
 * key: 'a','d','w','s','r','f' or BDPT_KEY_*; returns 1 if the camera moved (caller then
 * does ReInit), 0 for keys that do not move the camera. */
#define BDPT_KEY_UP        0x101
#define BDPT_KEY_DOWN      0x102
#define BDPT_KEY_LEFT      0x103
#define BDPT_KEY_RIGHT     0x104
#define BDPT_KEY_PAGE_UP   0x105
#define BDPT_KEY_PAGE_DOWN 0x106
int  bdpt_camera_key(bdpt_camera *camera, int key);
/* Sphere edits of KeyFunc ('4','6','8','2','9','3': display_func.c:347-370). Returns 1 if moved. */
int  bdpt_sphere_key(bdpt_sphere *spheres, unsigned n_spheres, int current_sphere, int key);
/* SavePPM smallpt_cpu.c:239-262: ASCII P3, rows written bottom-up. */
int  bdpt_save_ppm(const char *path, const unsigned char *rgba, int width, int height);
/* Binary P6 with the same header numbers and bottom-up rows (no reference counterpart). */
int  bdpt_save_ppm_binary(const char *path, const unsigned char *rgba, int width, int height);
/* SavePPM file name smallpt_cpu.c:245, "max1_secondi%.3f_exe%d.ppm", bounded by `size`. */
int  bdpt_ppm_name(char *buf, int size, float total_time, int current_sample);
/* The 256 thresholds behind the kernel's toInt (vec.h:34): thr[k] = smallest float whose
 * toInt is >= k (thr[0] = -inf), with correctly-rounded powf semantics. */
void bdpt_gamma_thresholds(float thr[256]);
/* glibc-compatible rand()/srand() (TYPE_3 additive feedback, 31-word state), so the sid
 * sequence `rand() % RAND_N` (smallpt_cpu.c:270, never srand'd => seed 1) is reproducible
 * independently of the C library in use. */
typedef struct { int state[31]; int f, r; } bdpt_rand_state;
void bdpt_srand(bdpt_rand_state *st, unsigned seed);
int  bdpt_rand(bdpt_rand_state *st);

/* The pass scheduler of the reference: glibc rand() for sid (smallpt_cpu.c:270) and the
 * flag / vlp_index state machine (smallpt_cpu.c:47,292-293,361; display_func.c:44,204-210).
 * Initial state = program start: srand(1), flag = 1, vlp_index = MAX_VLP = 1. */
typedef struct { bdpt_rand_state rng; int flag; int vlp_index; } bdpt_pass_state;
void bdpt_pass_state_init(bdpt_pass_state *ps);
/* UpdateRendering2 epilogue: flag = 2 (smallpt_cpu.c:361). */
void bdpt_pass_state_light(bdpt_pass_state *ps);
/* One UpdateRendering: returns the pass's sid and vlp_index, then applies :292-293.
 * vlp_index is reported modulo LIGHT_POINTS (the reference reads dev_lp out of bounds once it
 * reaches 4096 at ~8191 spp -- survey Appendix A.3; wrapping is the documented fix). */
void bdpt_pass_state_next(bdpt_pass_state *ps, unsigned *sid, int *vlp_index);
/* `npass` consecutive bdpt_pass_state_next calls. */
void bdpt_pass_schedule(bdpt_pass_state *ps, int npass, unsigned *sid, int *vlp_index);

#ifdef __cplusplus
}
#endif
#endif /* BDPT_H */
