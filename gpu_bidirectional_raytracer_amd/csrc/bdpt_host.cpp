// bdpt_host.cpp -- the C-ABI (include/bdpt.h) over the HIP kernels of bdpt_kernels.hip.
//
// Replaces the device-buffer globals and kernel launches of src/smallpt_cpu.c
// (AllocateBuffers :153, FreeBuffers :98, UpdateRendering :265, UpdateRendering2 :300) and
// loadMTGPU/seedMTGPU of src/MersenneTwister_kernel.cu:23-51.  One context = one GPU + one
// HIP stream.  Every HIP call is checked; failures return BDPT_EHIP with the HIP message in
// bdpt_last_error() (the reference prints and continues; the host shell decides).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <hip/hip_gl_interop.h>         // hipGraphicsGLRegisterBuffer (the optional display, 8(f)4)
#include <rccl/rccl.h>                 // types and prototypes only: librccl is opened with dlopen
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
#include <algorithm>
#include <limits>
#include <map>
#include <string>
#include <vector>

#include "../../include/bdpt.h"
#include "bdpt_device.h"
#include "bdpt_bvh.h"
#include "bdpt_cpu.h"
#include <chrono>

static_assert(kBvhEmissive == BDPT_DEV_BVH_EMISSIVE, "BVH id flag");

static_assert(sizeof(bdpt_vec) == 12, "Vec is 12 B (vec.h:4-6)");
static_assert(sizeof(bdpt_ray) == 24, "Ray is 24 B (geom.h:9-11)");
static_assert(sizeof(bdpt_sphere) == 44, "Sphere is 44 B (geom.h:23-27)");
static_assert(sizeof(bdpt_lightpath) == 36, "LightPath is 36 B (geom.h:29-33)");
static_assert(sizeof(bdpt_camera) == 60, "Camera is 60 B (camera.h:7-12)");
static_assert(sizeof(bdpt_dev_lightpath) == sizeof(bdpt_lightpath), "VLP layout");
static_assert(sizeof(bdpt_dev_vec) == sizeof(bdpt_vec), "colour layout");

extern "C" __global__ void bdpt_mt607_kernel(const uint4*, unsigned, float*);
extern "C" __global__ void bdpt_rand_planar_kernel(const float*, float*);
extern "C" __global__ void bdpt_sincos_planar_kernel(const float*, float2*);
extern "C" __global__ void bdpt_light_kernel(const bdpt_dev_sphere*, unsigned, const float*, int,
                                             bdpt_dev_lightpath*);
extern "C" const void* bdpt_path_kernel_table[36];   // [(S > 1) * 18 + (BVH ? 17 : n <= 16 ? n : 0)]
extern "C" __global__ void bdpt_pixels_kernel(const bdpt_dev_vec*, uchar4*, const float*, int);
extern "C" __global__ void bdpt_accum_kernel(bdpt_path_args);
extern "C" __global__ void bdpt_accum_serial_kernel(bdpt_path_args);

extern "C" __global__ void bdpt_frame_add_kernel(float*, const float*, unsigned*, const unsigned*, int);

// gamma thresholds (host, once): see bdpt_util.c
extern "C" void bdpt_gamma_thresholds(float thr[256]);

struct bdpt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // Pass-stream folds (bdpt_accum_kernel) run on their own stream so that a launch's fold
    // overlaps the next launch's path kernel (VALU-bound; the fold is a memory stream); pixel
    // pools fold on `stream` right after their launch instead (bdpt_accum_serial_kernel).  The
    // radiance buffer is double-buffered: launch L writes half L % 2 after the fold of launch L-2
    // has read it.  Everything else that touches colors/counter/pixels runs on `stream` after
    // join_fold() has made it wait for the last concurrent fold.
    hipStream_t fstream = nullptr;
    // Pixel pools with overlapped launches: a pooled launch and its serial fold run on
    // pstream[half of the radiance buffer], so one launch's drain overlaps the next one's start;
    // the folds stay in order through rb_fold_ev.  Everything queued on `stream` that feeds or
    // follows the path kernels joins the last fold first (join_fold).
    hipStream_t pstream[2] = {nullptr, nullptr};
    hipEvent_t amark = nullptr;         // `stream`'s work before a call, for the pstreams to wait on
    bool pool_dirty = false;            // overlapped launches used the claim-counter sets
    unsigned long long* d_prof = nullptr;   // BDPT_PROF=1 (with a -DBDPT_PROF kernel): section cycles
    hipEvent_t rb_path_ev[2] = {nullptr, nullptr};   // path kernel of the half done (stream)
    hipEvent_t rb_fold_ev[2] = {nullptr, nullptr};   // fold of the half done (fstream)
    bool rb_used[2] = {false, false};
    int rb_next = 0, fold_last = 0;
    bool fold_pending = false;          // a fold was issued after the last join_fold
    hipStream_t fold_stream = nullptr;  // the stream of the last fold (fstream or a pstream)
    // Path-pass calls go through a ring of kRing slots, each with its own events, so a call
    // never waits for the GPU except on the call issued kRing calls earlier (the reference's
    // interactive loop issues one pass per call; the pass tables travel in the kernel
    // arguments).  Timing is folded lazily, in call order.
    static constexpr int kRing = 4;
    struct call_slot {
        hipEvent_t ev0 = nullptr, ev1 = nullptr;   // the whole call
        std::vector<hipEvent_t> kev;               // per path-kernel launch {before, after}
        int launches = 0;
        bool pending = false;                      // issued, not folded yet
        bool serial_fold = false;                  // its folds ran after its path kernels, in-stream
    } ring[kRing];
    long long issued = 0, folded = 0;   // calls issued / folded into the accumulators
    double acc_ms = 0.0;         // accumulated device time of finished path-pass calls
    long long acc_launches = 0;
    float last_ms = 0.f;
    double acc_kernel_ms = 0.0;    // path kernels alone (no fold kernel)
    int W = 0, H = 0;
    std::vector<bdpt_sphere> spheres;
    std::vector<int> lights;
    bdpt_camera cam{};
    bool cam_set = false;
    bool rand_ready = false;
    int shard = 0, nshards = 1, band_rows = 8;
    int streams_req = 0;                // bdpt_set_streams: 0 = auto (measured), -1 = one pass per lane
    // auto mode: the first eight calls of >= 2 passes run, in this order, the pass-stream kernels
    // with two passes per lane, the fused S = 1 kernel with paired segment loads (bdpt_kernels.hip
    // BDPT_RNG_PAIR), pass streams with four passes per lane, two per lane again, the fused kernel
    // without pairing, four per lane again, and twice pass streams with pixel pools (specialised
    // builds only, bdpt_kernels.hip BDPT_POOL).  The pass-stream variant kept is the one with the
    // fastest call; the faster fused variant replaces it only if it beats that by kTuneMargin.
    // Calls are compared per pass by path-kernel time plus a quarter of the call's fold: the fold
    // runs on its own stream beside the next call's kernels (fold_timing).  (A cold first call -- clocks still ramping -- no
    // longer decides for the fused kernel.)  tune_phase 0..7: measuring; 8: all issued; 9:
    // decided.  Reset by scene / shard / traversal / specialisation / stream-mode changes.
    // BDPT_STREAMS_TUNE=0: no measurement (two passes per lane).
    // (5 %: open scenes gain >= 10 % from the fused kernel, closed ones lose >= 7 %; with 2 % a
    // one-call measurement once kept the fused kernel for gantz, 7 % slower, profiles/r03_s27_*.
    // Four passes per lane: cornell_glass / cornell_mirror +1.2 %, synthetic64 -2.8 % at 128-pass
    // launches, profiles/r03_s45_ab_passes_per_lane.txt -- so it is measured, not fixed.)
    static constexpr double kTuneMargin = 0.05;
    static constexpr int kTunePhases = 10;
    bool tune_enabled = true;
    int tune_phase = 0;
    bool tune_fused = false;
    bool tune_pair = true;              // the fused variant kept: paired segment loads or not
    bool tune_quarter = false;          // the pass-stream variant kept: four passes per lane
    bool tune_pool = false;             // the pass-stream variant kept: pixel pools
    bool tune_units = false;            // the pass-stream variant kept: the ordered in-kernel fold
    long long tune_call[kTunePhases] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    double tune_ms[kTunePhases] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // whether each tuning call really ran its role's variant: four passes per lane needs launches
    // of >= 8 passes, and the unpaired fused variant exists only as a specialised (JIT) build --
    // otherwise the role repeated another role's kernel and must not decide anything
    bool tune_real[kTunePhases] = {false, false, false, false, false, false, false, false, false, false};
    int tune_npass[kTunePhases] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // multi-device groups: the peers follow the stream mode devices[0] measured (its decision is
    // copied when they reach the decision point), so every device of a group runs the same kernels
    bdpt_ctx* tune_leader = nullptr;
    int last_streams = 1;               // S of the last path-pass launch
    bool last_bvh = false;              // the last path-pass launch traversed the BVH
    int cus = 256;                      // compute units (auto stream count)
    bdpt_dev_vec* d_rbuf = nullptr;     // pass-stream radiance, 2 halves of rbuf_cap: [npass][nloc]
    unsigned* d_rmask = nullptr;        // pixel pools: 4 words per launched pixel (stored passes), 2 halves
    unsigned* d_poolctr = nullptr;      // pixel pools: claimed pixels per pass and eighth, a line each,
                                        // two sets: a pooled launch uses one and zeroes the other
    int pool_set = 0;                   // the set the next pooled launch uses
    unsigned* d_uflags = nullptr;       // ordered in-kernel fold (units): per 8x8 wave tile, epoch << 8 | range
    size_t uflags_cap = 0;
    unsigned uepoch = 0;                // launches of the units kernel (flag tags)
    unsigned* d_uerr = nullptr;         // set by a unit whose handover wait timed out
    bool units_check = false;           // a units launch ran since the last error check
    int traversal = BDPT_TRAVERSE_AUTO; // bdpt_set_traversal
    bool has_bvh = false;               // the scene has a BVH (bdpt_bvh.cpp)
    int bvh_nn = 0, bvh_ns = 0, big_n = 0;
    float bvh_c[3] = {0.f, 0.f, 0.f}, bvh_r = 0.f, bvh_q = 0.f;
    float4 *d_bvh_nodes = nullptr, *d_bvh_geom = nullptr, *d_big_geom = nullptr, *d_mat = nullptr;
    int *d_bvh_ids = nullptr, *d_big_ids = nullptr;
    size_t rbuf_cap = 0;                // elements
    size_t rmask_lanes = 0;             // launched pixels the mask halves hold (4 words each)
    uint4* d_params = nullptr;          // 4096 x {matrix_a, mask_b, mask_c, seed}
    float* d_rand = nullptr;
    float* d_rndp = nullptr;            // planar copy of d_rand (bdpt_rand_planar_kernel)
    float2* d_scp = nullptr;            // {sinf, cosf}(2 pi u) per d_rndp entry (bdpt_sincos_planar_kernel)
    bdpt_dev_lightpath* d_lp = nullptr;
    bdpt_dev_sphere* d_sph = nullptr;
    unsigned sph_cap = 0;
    int* d_lights = nullptr;
    float4* d_geom = nullptr;           // per sphere {p, rad^2}; then the n_vac non-emitters' (VLP-only shadow rounds)
    unsigned n_vac = 0;
    float4* d_lightrec = nullptr;       // per emitter {p, rad}, {e, (4*pi*rad)*rad}
    unsigned emis_mask = 0;
    bdpt_dev_vec* d_colors = nullptr;
    unsigned* d_counter = nullptr;
    uchar4* d_pixels = nullptr;
    float* d_thr = nullptr;
    uint32_t h_params[4 * BDPT_MT_RNG_COUNT];
    // scene-specialised path kernels (hipRTC), by compile options; modules live until destroy
    bool specialize = true;             // bdpt_set_specialize
    bool last_specialized = false;
    std::map<std::string, hipFunction_t> jit_fns;
    std::vector<hipModule_t> jit_mods;
    char jit_err[256] = {0};            // why the last specialisation fell back (diagnostics)
    int jit_waves = 0;                  // waves/SIMD bound of the last specialised build
    bool jit_zero_exit = false;         // the last specialised build has the black-surface exit
    // jit_path_kernel's answer per [fused / pass streams / pools][paired loads] for the current scene, specialise
    // switch and JIT environment (jit_env_key): a call then resolves its kernel without rebuilding the option
    // strings (tens of microseconds per call, which the one-pass-per-call pattern pays every call)
    struct jit_memo_t {
        bool valid = false, zero_exit = false;
        hipFunction_t fn = nullptr;
        int waves = 0;
        std::string flags, err;
    } jit_memo[4][2];
    int last_features = 0;              // BDPT_FEAT_* of the last path-pass launch
    unsigned rand_seed = 0;             // seed of the current MT607 table (rand_ready)
    char err[512] = {0};
    // multi-device context (bdpt_create_multi): this context renders on devices[0] and owns the
    // peer contexts of the other devices; the frame is assembled on devices[0] by a sum-reduce
    bool multi = false;
    std::vector<bdpt_ctx*> peers;
    std::vector<void*> comms;           // ncclComm_t per device when the reduce runs on RCCL
    int reduce_mode = 0;                // kReduce*
    bool frame_stale = true;            // the assembled frame predates the last change
    bdpt_dev_vec* d_fcolors = nullptr;  // assembled frame (devices[0])
    unsigned* d_fcounter = nullptr;
    uchar4* d_fpixels = nullptr;
    bdpt_dev_vec* d_ftmp = nullptr;     // peer-copy staging (kReducePeer)
    unsigned* d_ftmpc = nullptr;
    char reduce_note[256] = {0};        // the RCCL version and communicator, or why RCCL is not used
    bdpt_cpu_ctx* cpu = nullptr;        // device == BDPT_DEVICE_CPU: the host backend (bdpt_cpu.cpp)
    hipGraphicsResource_t gl_res = nullptr;   // registered GL pixel-unpack buffer (bdpt_gl_register_pbo)
    unsigned gl_pbo = 0;
};
enum { kReduceNone = 0, kReduceRccl = 1, kReducePeer = 2 };

static int fail(bdpt_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof(c->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(ctx, call)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((ctx), BDPT_EHIP, "%s: %s", #call, hipGetErrorString(e_));            \
    } while (0)

static int join_fold(bdpt_ctx* c);
static int upload_scene(bdpt_ctx* c) {
    c->tune_phase = 0;                                      // re-measure the stream mode
    for (auto& row : c->jit_memo)                           // the specialised kernels change too
        for (auto& m : row) m.valid = false;
    const unsigned n = (unsigned)c->spheres.size();
    // queued path passes may still read the scene buffers freed / rewritten below (pooled
    // launches on the pstreams: the last fold follows them all)
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<bdpt_dev_sphere> ds(n);
    std::vector<float4> geom(n), lrec;
    std::vector<float4> vgeom;                      // the non-emitters' geometry, ascending index
    c->lights.clear();
    c->emis_mask = 0;
    for (unsigned i = 0; i < n; i++) {
        const bdpt_sphere& s = c->spheres[i];
        bdpt_dev_sphere& d = ds[i];
        d.px = s.p.x; d.py = s.p.y; d.pz = s.p.z;
        d.rr = s.rad * s.rad;                       // the product SphereIntersectDevice forms
        d.ex = s.e.x; d.ey = s.e.y; d.ez = s.e.z;
        d.rad = s.rad;
        d.cx = s.c.x; d.cy = s.c.y; d.cz = s.c.z;
        d.refl = s.refl;
        geom[i] = make_float4(d.px, d.py, d.pz, d.rr);
        if (s.e.x == 0.f && s.e.y == 0.f && s.e.z == 0.f) vgeom.push_back(geom[i]);
        if (!(s.e.x == 0.f && s.e.y == 0.f && s.e.z == 0.f)) {
            c->lights.push_back((int)i);
            if (i < 32) c->emis_mask |= 1u << i;
            const float kPi = 3.14159265358979323846f;
            const float area = 4.f * kPi * s.rad * s.rad;        // device.cu:500, same float ops
            lrec.push_back(make_float4(s.p.x, s.p.y, s.p.z, s.rad));
            lrec.push_back(make_float4(s.e.x, s.e.y, s.e.z, area));
        }
    }
    if (n > c->sph_cap) {
        void* old[] = {c->d_sph, c->d_lights, c->d_geom, c->d_lightrec};
        for (void* b : old)
            if (b) HIPCHK(c, hipFree(b));
        c->d_sph = nullptr; c->d_lights = nullptr; c->d_geom = nullptr; c->d_lightrec = nullptr;
        HIPCHK(c, hipMalloc(&c->d_sph, sizeof(bdpt_dev_sphere) * n));
        HIPCHK(c, hipMalloc(&c->d_lights, sizeof(int) * n));
        HIPCHK(c, hipMalloc(&c->d_geom, 2 * sizeof(float4) * n));   // [n) by index, then the non-emitters
        HIPCHK(c, hipMalloc(&c->d_lightrec, 2 * sizeof(float4) * n));
        c->sph_cap = n;
    }
    if (n) HIPCHK(c, hipMemcpyAsync(c->d_geom, geom.data(), sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    c->n_vac = (unsigned)vgeom.size();
    if (c->n_vac)
        HIPCHK(c, hipMemcpyAsync(c->d_geom + n, vgeom.data(), sizeof(float4) * c->n_vac, hipMemcpyHostToDevice,
                                 c->stream));
    if (!lrec.empty())
        HIPCHK(c, hipMemcpyAsync(c->d_lightrec, lrec.data(), sizeof(float4) * lrec.size(),
                                 hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_sph, ds.data(), sizeof(bdpt_dev_sphere) * n, hipMemcpyHostToDevice, c->stream));
    if (!c->lights.empty())
        HIPCHK(c, hipMemcpyAsync(c->d_lights, c->lights.data(), sizeof(int) * c->lights.size(),
                                 hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));

    // large scenes: BVH over the ordinary spheres + per-sphere material table in HBM
    void* old[] = {c->d_bvh_nodes, c->d_bvh_geom, c->d_big_geom, c->d_mat, c->d_bvh_ids, c->d_big_ids};
    for (void* b : old)
        if (b) HIPCHK(c, hipFree(b));
    c->d_bvh_nodes = c->d_bvh_geom = c->d_big_geom = c->d_mat = nullptr;
    c->d_bvh_ids = c->d_big_ids = nullptr;
    c->has_bvh = false;
    bdpt_bvh bvh;
    if (n > 16 && bdpt_build_bvh(c->spheres.data(), n, &bvh)) {
        std::vector<float4> mat(3 * (size_t)n);
        for (unsigned i = 0; i < n; i++) {
            const bdpt_dev_sphere& d = ds[i];
            const bool emis = !(d.ex == 0.f && d.ey == 0.f && d.ez == 0.f);
            mat[3 * i] = make_float4(d.cx, d.cy, d.cz, bdpt_bits_as_float(d.refl | (emis ? 256 : 0)));
            mat[3 * i + 1] = make_float4(d.ex, d.ey, d.ez, d.rad);
            mat[3 * i + 2] = make_float4(d.px, d.py, d.pz, 0.f);
        }
        c->bvh_nn = (int)bvh.nodes.size() / 2;
        c->bvh_ns = (int)bvh.geom.size();
        c->big_n = (int)bvh.big_geom.size();
        for (int k = 0; k < 3; k++) c->bvh_c[k] = bvh.c_root[k];
        c->bvh_r = bvh.r_root;
        c->bvh_q = bvh.q;
        HIPCHK(c, hipMalloc(&c->d_bvh_nodes, sizeof(float4) * bvh.nodes.size()));
        HIPCHK(c, hipMalloc(&c->d_bvh_geom, sizeof(float4) * bvh.geom.size()));
        HIPCHK(c, hipMalloc(&c->d_bvh_ids, sizeof(int) * bvh.ids.size()));
        HIPCHK(c, hipMalloc(&c->d_mat, sizeof(float4) * mat.size()));
        HIPCHK(c, hipMemcpy(c->d_bvh_nodes, bvh.nodes.data(), sizeof(float4) * bvh.nodes.size(), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_bvh_geom, bvh.geom.data(), sizeof(float4) * bvh.geom.size(), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_bvh_ids, bvh.ids.data(), sizeof(int) * bvh.ids.size(), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_mat, mat.data(), sizeof(float4) * mat.size(), hipMemcpyHostToDevice));
        if (c->big_n) {
            HIPCHK(c, hipMalloc(&c->d_big_geom, sizeof(float4) * bvh.big_geom.size()));
            HIPCHK(c, hipMalloc(&c->d_big_ids, sizeof(int) * bvh.big_ids.size()));
            HIPCHK(c, hipMemcpy(c->d_big_geom, bvh.big_geom.data(), sizeof(float4) * bvh.big_geom.size(),
                                hipMemcpyHostToDevice));
            HIPCHK(c, hipMemcpy(c->d_big_ids, bvh.big_ids.data(), sizeof(int) * bvh.big_ids.size(),
                                hipMemcpyHostToDevice));
        }
        c->has_bvh = true;
    }
    return BDPT_OK;
}

static void release(bdpt_ctx* c) {
    void* bufs[] = {c->d_params, c->d_rand, c->d_rndp, c->d_scp, c->d_lp, c->d_sph, c->d_lights, c->d_geom, c->d_lightrec, c->d_colors,
                    c->d_counter, c->d_pixels, c->d_thr, c->d_rbuf, c->d_rmask, c->d_poolctr, c->d_uflags, c->d_uerr, c->d_bvh_nodes,
                    c->d_bvh_geom, c->d_big_geom, c->d_mat, c->d_bvh_ids, c->d_big_ids,
                    c->d_fcolors, c->d_fcounter, c->d_fpixels, c->d_ftmp, c->d_ftmpc};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& s : c->ring) {
        for (hipEvent_t e : s.kev) (void)hipEventDestroy(e);
        if (s.ev0) (void)hipEventDestroy(s.ev0);
        if (s.ev1) (void)hipEventDestroy(s.ev1);
    }
    for (hipModule_t m : c->jit_mods) (void)hipModuleUnload(m);
    for (int b = 0; b < 2; b++) {
        if (c->rb_path_ev[b]) (void)hipEventDestroy(c->rb_path_ev[b]);
        if (c->rb_fold_ev[b]) (void)hipEventDestroy(c->rb_fold_ev[b]);
    }
    if (c->amark) (void)hipEventDestroy(c->amark);
    for (hipStream_t& ps : c->pstream)
        if (ps) (void)hipStreamDestroy(ps);
    if (c->fstream) (void)hipStreamDestroy(c->fstream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

// ---- scene-specialised path kernels (run-time compiled with hipRTC) -------------------------
// For scenes of <= 64 spheres (not BVH-traversed) the path kernel is recompiled with the scene folded in
// (bdpt_kernels.hip BDPT_JIT): the sphere geometry {p, rad^2} as exact hex-float literals and the
// emitter mask become compile-time constants, so a coordinate difference p - o that several
// spheres share is formed once per ray (cornell's 9 spheres have 15 distinct coordinates, not
// 27) and the scalar scene loads go away: +7 % on cornell.  The float operations are the same in
// the same order, so results are bit-identical to the precompiled kernels
// (tests/test_gpu_specialize.py).  hipRTC is opened with dlopen; when it is missing or a compile
// fails, the precompiled instance runs (bdpt_last_specialized() says which one did).  A build that
// needs scratch (register spills) at 6 waves/SIMD is rebuilt at 5.  Code objects are cached per
// context and on disk ($BDPT_JIT_CACHE, else $HOME/.cache/bdpt-jit), keyed by a hash of the
// sources, the options, the hipRTC version and the device's gfx arch; the cache directory must be
// owned by the user and closed to others (created 0700), else nothing is read from or written to
// disk.  A compile takes ~1 s.
#include "bdpt_jit_src.h"

namespace {
struct rtc_api {
    bool ok = false;
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcAddNameExpression) add_name = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetLoweredName) lowered = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) code = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) log = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    int major = 0, minor = 0;                    // hiprtcVersion (part of the cache key)
};

const rtc_api& rtc() {
    static const rtc_api api = [] {
        rtc_api r;
        const char* libs[] = {"libhiprtc.so.7", "libhiprtc.so", "/opt/rocm/lib/libhiprtc.so.7",
                              "/opt/rocm/lib/libhiprtc.so"};
        void* h = nullptr;
        for (const char* l : libs)
            if ((h = dlopen(l, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) return r;
#define BDPT_RTC_SYM(f, n) r.f = (decltype(r.f))dlsym(h, n)
        BDPT_RTC_SYM(create, "hiprtcCreateProgram");
        BDPT_RTC_SYM(add_name, "hiprtcAddNameExpression");
        BDPT_RTC_SYM(compile, "hiprtcCompileProgram");
        BDPT_RTC_SYM(lowered, "hiprtcGetLoweredName");
        BDPT_RTC_SYM(code_size, "hiprtcGetCodeSize");
        BDPT_RTC_SYM(code, "hiprtcGetCode");
        BDPT_RTC_SYM(log_size, "hiprtcGetProgramLogSize");
        BDPT_RTC_SYM(log, "hiprtcGetProgramLog");
        BDPT_RTC_SYM(destroy, "hiprtcDestroyProgram");
#undef BDPT_RTC_SYM
        auto version = (decltype(&hiprtcVersion))dlsym(h, "hiprtcVersion");
        r.ok = r.create && r.add_name && r.compile && r.lowered && r.code_size && r.code &&
               r.log_size && r.log && r.destroy && version &&
               version(&r.major, &r.minor) == HIPRTC_SUCCESS;
        return r;
    }();
    return api;
}

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

std::string hexf(float v) {                     // exact float literal
    char b[48];
    snprintf(b, sizeof b, "%af", (double)v);
    return b;
}

// The on-disk cache directory, created 0700 if missing; "" (no disk cache) unless it is a
// directory owned by this user that neither group nor others can write.
std::string jit_cache_dir() {
    std::string dir;
    if (const char* d = getenv("BDPT_JIT_CACHE")) dir = d;
    else if (const char* home = getenv("HOME")) dir = std::string(home) + "/.cache/bdpt-jit";
    else return "";
    std::string d;                                           // mkdir -p, 0700
    for (size_t i = 0; i <= dir.size(); i++) {
        if ((i == dir.size() || dir[i] == '/') && !d.empty()) mkdir(d.c_str(), 0700);
        if (i < dir.size()) d += dir[i];
    }
    struct stat st;
    if (stat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != getuid() ||
        (st.st_mode & (S_IWGRP | S_IWOTH)))
        return "";
    return dir;
}

bool read_file(const std::string& path, std::vector<char>& out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    struct stat st;
    if (fstat(fileno(f), &st) != 0 || st.st_uid != getuid() || !S_ISREG(st.st_mode)) {
        fclose(f);
        return false;
    }
    out.resize(st.st_size > 0 ? (size_t)st.st_size : 0);
    const bool ok = st.st_size > 0 && fread(out.data(), 1, out.size(), f) == out.size();
    fclose(f);
    return ok;
}

// Write to a private temporary file and rename it into place only if every byte reached it.
void write_file_atomic(const std::string& path, const std::vector<char>& data) {
    const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    ok = (fflush(f) == 0) && ok;
    ok = (fclose(f) == 0) && ok;
    if (ok) ok = rename(tmp.c_str(), path.c_str()) == 0;
    if (!ok) unlink(tmp.c_str());
}
}  // namespace

// Compile (or fetch from the disk cache) and load one specialised build; nullptr on failure
// (reason in c->jit_err).
static hipFunction_t jit_build(bdpt_ctx* c, const std::string& name, const std::vector<std::string>& opts) {
    const rtc_api& api = rtc();
    std::string key = name;
    for (const std::string& o : opts) key += " " + o;
    const auto it = c->jit_fns.find(key);
    if (it != c->jit_fns.end()) return it->second;

    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
        (void)hipGetLastError();
        snprintf(c->jit_err, sizeof c->jit_err, "hipGetDeviceProperties failed");
        return nullptr;
    }
    uint64_t h = 1469598103934665603ull;
    h = fnv1a(h, kJitMain, sizeof kJitMain);
    for (int i = 0; i < kJitNumHeaders; i++) h = fnv1a(h, kJitHeaders[i], strlen(kJitHeaders[i]));
    h = fnv1a(h, key.data(), key.size());
    const int ver[2] = {api.major, api.minor};
    h = fnv1a(h, ver, sizeof ver);
    h = fnv1a(h, prop.gcnArchName, strnlen(prop.gcnArchName, sizeof prop.gcnArchName));
    char hex[40];
    snprintf(hex, sizeof hex, "%016llx", (unsigned long long)h);
    const std::string dir = jit_cache_dir();
    const std::string path = dir.empty() ? "" : dir + "/path_" + hex + ".hsaco";
    const std::string name_path = path + ".name";
    std::vector<char> code, lowered;
    if (path.empty() || !read_file(path, code) || !read_file(name_path, lowered)) {
        hiprtcProgram prog = nullptr;
        if (api.create(&prog, kJitMain, kJitMainName, kJitNumHeaders, kJitHeaders, kJitHeaderNames) != HIPRTC_SUCCESS) {
            snprintf(c->jit_err, sizeof c->jit_err, "hiprtcCreateProgram failed");
            return nullptr;
        }
        api.add_name(prog, name.c_str());
        std::vector<const char*> o;
        for (const std::string& x : opts) o.push_back(x.c_str());
        const hiprtcResult rc = api.compile(prog, (int)o.size(), o.data());
        const char* low = nullptr;
        size_t sz = 0;
        if (rc != HIPRTC_SUCCESS || api.lowered(prog, name.c_str(), &low) != HIPRTC_SUCCESS || !low ||
            api.code_size(prog, &sz) != HIPRTC_SUCCESS || sz == 0) {
            size_t ls = 0;
            std::string log;
            if (api.log_size(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
                log.resize(ls);
                api.log(prog, &log[0]);
            }
            snprintf(c->jit_err, sizeof c->jit_err, "hipRTC compile failed: %.200s", log.c_str());
            api.destroy(&prog);
            return nullptr;
        }
        code.resize(sz);
        api.code(prog, code.data());
        lowered.assign(low, low + strlen(low) + 1);
        api.destroy(&prog);
        if (!path.empty()) {
            write_file_atomic(path, code);
            write_file_atomic(name_path, lowered);
        }
    }
    if (lowered.empty() || lowered.back() != '\0') lowered.push_back('\0');
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    if (hipModuleLoadData(&mod, code.data()) != hipSuccess ||
        hipModuleGetFunction(&fn, mod, lowered.data()) != hipSuccess) {
        if (mod) (void)hipModuleUnload(mod);
        (void)hipGetLastError();
        snprintf(c->jit_err, sizeof c->jit_err, "loading the specialised code object failed");
        return nullptr;
    }
    c->jit_mods.push_back(mod);
    c->jit_fns[key] = fn;
    return fn;
}

// Passes per launch of the fused S = 1 kernel.  Its workgroups stage a VLP (48 B) and a sid per
// pass of the launch in LDS: 128 passes make 31.5 KB per workgroup.  Measured on caustic8 (one
// session, two rounds, profiles/r03_s1_ab_fused.txt): 64 passes at 5 waves/SIMD (4-KB sincos
// table) 48.8 Gs/s, 64 at 6 (2-KB table) 48.55, 128 at 6 48.2, 128 at 5 (round 2) 47.9.
// BDPT_FUSED_MAX_PASSES overrides.
static int fused_max_passes() {
    static const int cap = [] {
        const char* e = getenv("BDPT_FUSED_MAX_PASSES");
        const int v = e ? atoi(e) : 64;
        return v < 1 ? 1 : (v > 128 ? 128 : v);
    }();
    return cap;
}

// Pixel pools for the pass-stream kernel (bdpt_kernels.hip BDPT_POOL), a specialised build of
// its own launched with one pass per lane slice: the auto stream mode measures it (tuning roles
// 6, 7).  BDPT_POOL: unset = measured, 0 = never, R > 0 = always (streams launches), chunks of
// R x 64 pixels; BDPT_POOL_GRID = G: G x 64 pixels per wave and pass.
static int pool_env() {
    const char* e = getenv("BDPT_POOL");
    if (!e || !*e) return -1;
    const int v = atoi(e);
    return v < 1 ? 0 : (v > 64 ? 64 : v);
}
// Launch shape of a pooled launch of nloc pixels per pass: {chunk R, grid G} (a wave claims R x 64
// pixels at a time; a pass has nloc / (256 G) workgroups).  With the sparse serial fold and
// overlapped launches, larger chunks and grids measured best (profiles/r05_s44_pool_shape.txt,
// r05_s45_*, r05_s46_*, r05_s48_*, r05_s49_*; interleaved rounds, ms per step): whole frame
// (2.08 M) G = 128, R = 64 3.54-3.55 against G = 64, R = 16 3.66-3.68; 1/2 share G = 128, R = 32
// 1.88-1.89 against 1.95-1.96; 1/4 share 0.943-0.954 against 0.956-0.962; 1/8 share (260 K)
// G = 128, R = 16 0.548-0.553 against G = 64, R = 16 0.567-0.568 and G = 128, R = 32 0.576-0.578.
// Launches that are not overlapped (the auto-tuner's calls, BDPT_POOL_OVERLAP=0) keep the shape
// that measured best before the overlap, G = 64, R = 16: a serial launch pays the large shapes'
// drain in full, and with them the tuner's pooled call at the 1/8 share lost to S = 32
// (r05_s50_strong.txt, N = 8 row).
static void pool_shape(long nloc, bool overlap, int* R, int* G) {
    int g = overlap ? 128 : 64;
    int r = !overlap ? 16 : nloc >= 1500000 ? 64 : (nloc >= 400000 ? 32 : 16);
    if (const char* e = getenv("BDPT_POOL_GRID")) {
        const int v = atoi(e);
        if (v >= 1) g = v > 256 ? 256 : v;
    }
    const int pe = pool_env();
    *G = g;
    *R = pe > 0 ? pe : r;
}

// The specialised kernel for the context's scene and pass-stream mode, compiled on first use;
// nullptr = use the precompiled instance (reason in c->jit_err).
// Pass streams with the ordered fold inside the kernel (bdpt_kernels.hip BDPT_UNITS): BDPT_UNITS=P
// forces it with ranges of P passes (experiments; 0 = never).
static constexpr int kUnitPasses = 8;   // passes per unit range in the auto mode (profiles/r05_s5_*)
static int units_env() {
    const char* e = getenv("BDPT_UNITS");
    if (!e || !*e) return -1;
    const int v = atoi(e);
    return v < 1 ? 0 : (v > 128 ? 128 : v);
}

static hipFunction_t jit_path_kernel_build(bdpt_ctx* c, bool streams, bool pair, bool pool, bool units) {
    const unsigned n = (unsigned)c->spheres.size();
    if (!c->specialize || n < 1 || n > 64) return nullptr;          // kJitEmis is 64 bits
    unsigned long long emis = 0;
    for (unsigned i = 0; i < n; i++) {
        const bdpt_vec& e = c->spheres[i].e;
        if (!(e.x == 0.f && e.y == 0.f && e.z == 0.f)) emis |= 1ull << i;
    }
    if (!rtc().ok) {
        snprintf(c->jit_err, sizeof c->jit_err, "hipRTC not found");
        return nullptr;
    }
    std::string geom = "{";
    for (unsigned i = 0; i < n; i++) {
        const bdpt_sphere& sp = c->spheres[i];
        const float rr = sp.rad * sp.rad;                    // as upload_scene forms it
        geom += (i ? ",{" : "{") + hexf(sp.p.x) + "," + hexf(sp.p.y) + "," + hexf(sp.p.z) + "," + hexf(rr) + "}";
    }
    geom += "}";
    // Black-surface exit (bdpt_kernels.hip BDPT_ZERO_EXIT): compiled in only when ending a path at
    // a black non-emitter is provably exact for this scene (bdpt_util.c bdpt_zero_exit_safe).
    const bool zero_exit = bdpt_zero_exit_safe(c->spheres.data(), n) != 0;
    // Waves/SIMD the build targets: 6 for the pass-stream kernel, 5 for the fused S = 1 kernel
    // (at 6 it fits without spills, but then the LDS formula below takes the 2-KB sincos table and
    // caustic8 measured 0.6 % slower than 5 waves with the 4-KB table; fused_max_passes()).
    const char* wenv = getenv(streams ? "BDPT_JIT_WAVES" : "BDPT_JIT_FUSED_WAVES");
    int waves = wenv ? atoi(wenv) : (streams ? 6 : 5);
    const std::string name = "&bdpt_path_kernel_t<" + std::to_string(n) + (streams ? ", true>" : ", false>");
    const char* jflags = getenv("BDPT_JIT_FLAGS");
    const bool user_coarse = jflags && strstr(jflags, "BDPT_SC_COARSE");   // experiments decide
    bool coarse = false;
    for (;; waves--) {
        const std::vector<std::string> opts = {
            "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
            "-fno-gpu-flush-denormals-to-zero", "-DBDPT_JIT=1", "-DBDPT_JIT_N=" + std::to_string(n),
            "-DBDPT_JIT_EMIS=" + std::to_string(emis) + "ull", "-DBDPT_JIT_GEOM=" + geom,
            "-DBDPT_JIT_ZERO_SAFE=" + std::to_string(zero_exit ? 1 : 0),
            "-DBDPT_WAVES_PER_SIMD=" + std::to_string(waves)};
        std::vector<std::string> all = opts;
        if (!streams) all.push_back("-DBDPT_FUSED_WAVES=" + std::to_string(waves));
        if (!streams && !pair) all.push_back("-DBDPT_RNG_PAIR=0");
        if (streams && pool) all.push_back("-DBDPT_POOL=1");
        if (streams && units) all.push_back("-DBDPT_UNITS=1");
        // VLP-only part-full shadow rounds over the non-emitters' list (BDPT_VAC_LIST): only where
        // dropping the emitters saves a lane-group iteration (cornell: 8 of 9 spheres fit 4, 2, 1
        // iterations instead of 5, 3, 2); elsewhere the staging costs (synthetic64 -0.4 %,
        // profiles/r06_s24_ab_vac_list.txt)
        bool vac_list = false;
        for (unsigned k = 1; k <= 3; k++)
            if ((1u << k) <= c->n_vac && (c->n_vac + (1u << k) - 1) >> k < (n + (1u << k) - 1) >> k) vac_list = true;
        if (!vac_list) all.push_back("-DBDPT_VAC_LIST=0");
        if (const char* extra = getenv("BDPT_JIT_FLAGS")) {    // experiments: extra -D options
            std::string tok;
            for (const char* q = extra;; q++) {
                if (*q == ' ' || *q == ',' || *q == 0) {
                    if (!tok.empty()) all.push_back(tok);
                    tok.clear();
                    if (!*q) break;
                } else {
                    tok += *q;
                }
            }
        }
        if (coarse) all.push_back("-DBDPT_SC_COARSE=1");
        hipFunction_t fn = jit_build(c, name, all);
        if (!fn) return nullptr;
        // The 4-KB sincos table costs a workgroup per CU when LDS bounds the count (large
        // scenes: 16 B per sphere; the fused kernel: a VLP and a sid per pass of the launch);
        // then take the 2-KB table of even entries (bdpt_math.h).  Estimated with bdpt_path_passes'
        // smem formula: one pass slot for the pass-stream kernel, fused_max_passes() for the fused.
        int stat = 0;
        if (!coarse && !user_coarse &&
            hipFuncGetAttribute(&stat, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, fn) == hipSuccess) {
            const size_t slots = units ? (size_t)std::max(units_env(), 16) : streams ? 1 : (size_t)fused_max_passes();
            const size_t dyn = sizeof(float4) * (5 * (size_t)n + 3 * slots + 5 + 4 * 128 * 2) + sizeof(unsigned) * slots;
            const size_t lds = 160 * 1024, fine = lds / (dyn + stat), half = lds / (dyn + stat - 2048);
            if (fine < (size_t)waves && half > fine) {
                coarse = true;
                waves++;                                      // same wave count, coarse table
                continue;
            }
        }
        (void)hipGetLastError();
        int scratch = 0;
        if (hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn) != hipSuccess) {
            (void)hipGetLastError();
            scratch = 0;
        }
        // spill-free, or the 5-wave floor (BDPT_JIT_SCRATCH_OK: keep a spilling build; experiments)
        if (scratch == 0 || waves <= 5 || getenv("BDPT_JIT_SCRATCH_OK")) {
            c->jit_err[0] = 0;
            c->jit_waves = waves;
            c->jit_zero_exit = zero_exit;
            return fn;
        }
    }
}

static void jit_forget(bdpt_ctx* c) {                   // the scene or the specialise switch changed
    for (auto& row : c->jit_memo)
        for (auto& m : row) m.valid = false;
}

// Every environment input of jit_path_kernel_build, as one memo key: an in-process A/B that
// changes any of them gets a fresh build (BDPT_FUSED_MAX_PASSES is read once per process).
static std::string jit_env_key() {
    std::string k;
    for (const char* v : {"BDPT_JIT_FLAGS", "BDPT_JIT_WAVES", "BDPT_JIT_FUSED_WAVES", "BDPT_JIT_SCRATCH_OK"}) {
        const char* e = getenv(v);
        k += e ? e : "";
        k += '\x1f';
    }
    return k;
}

static hipFunction_t jit_path_kernel(bdpt_ctx* c, bool streams, bool pair = true, bool pool = false,
                                     bool units = false) {
    const std::string key = jit_env_key();
    bdpt_ctx::jit_memo_t& m = c->jit_memo[streams ? (units ? 3 : pool ? 2 : 1) : 0][pair];
    if (m.valid && m.flags == key) {
        snprintf(c->jit_err, sizeof c->jit_err, "%s", m.err.c_str());
        if (m.fn) { c->jit_waves = m.waves; c->jit_zero_exit = m.zero_exit; }
        return m.fn;
    }
    hipFunction_t fn = jit_path_kernel_build(c, streams, pair, streams && pool, streams && units);
    m.valid = true;
    m.fn = fn;
    m.waves = c->jit_waves;
    m.zero_exit = c->jit_zero_exit;
    m.flags = key;
    m.err = c->jit_err;
    return fn;
}

// Make the context's stream wait for the last pass-stream fold (issued on fstream): call before
// anything on `stream` touches colors/counter/pixels.  Folds run in order on fstream, so the last
// one covers all.
static int join_fold(bdpt_ctx* c) {
    if (c->cpu || !c->fold_pending) return BDPT_OK;
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->rb_fold_ev[c->fold_last], 0));
    c->fold_pending = false;
    return BDPT_OK;
}

// Fold the calls issued before call number `upto` into the accumulators, oldest first (waits
// for each of them to finish).
static int fold_timing(bdpt_ctx* c, long long upto) {
    for (; c->folded < upto && c->folded < c->issued; c->folded++) {
        bdpt_ctx::call_slot& s = c->ring[c->folded % bdpt_ctx::kRing];
        if (!s.pending) continue;
        float ms = 0.f;
        HIPCHK(c, hipEventSynchronize(s.ev1));
        HIPCHK(c, hipEventElapsedTime(&ms, s.ev0, s.ev1));
        c->last_ms = ms;
        c->acc_ms += ms;
        double kms = 0.0;
        for (int k = 0; k < s.launches; k++) {
            float km = 0.f;
            HIPCHK(c, hipEventElapsedTime(&km, s.kev[2 * k], s.kev[2 * k + 1]));
            kms += km;
        }
        c->acc_kernel_ms += kms;
        // the stream mode's measure: the path kernels' time plus a quarter of the rest of the
        // call (a pass-stream call's fold runs on its own stream beside the next call's path
        // kernels and costs about that much of its own time in back-to-back calls: caustic pools
        // 3.79 ms kernels + 1.10 ms fold -> 4.05 ms per call, two passes per lane 4.85 + 0.84 ->
        // 4.95, profiles/r04_s20_*)
        // (a call whose folds ran on its own stream after its path kernels is charged in full)
        for (int r = 0; r < bdpt_ctx::kTunePhases; r++)
            if (c->folded == c->tune_call[r]) c->tune_ms[r] = s.serial_fold ? (double)ms : kms + 0.25 * ((double)ms - kms);
        c->acc_launches += s.launches;
        s.pending = false;
    }
    return BDPT_OK;
}
static int fold_timing(bdpt_ctx* c) { return fold_timing(c, c->issued); }

extern "C" {

const char* bdpt_last_error(const bdpt_ctx* c) { return c ? c->err : "null context"; }

static char g_create_err[512];

int bdpt_create(bdpt_ctx** out, const bdpt_sphere* spheres, unsigned n, int W, int H,
                const char* mt_dat_path, int device) {
    if (!out) return BDPT_EINVAL;
    *out = nullptr;
    bdpt_ctx* c = new (std::nothrow) bdpt_ctx();
    if (!c) return BDPT_ENOMEM;
    int rc = BDPT_OK;
    auto bail = [&](int code) {
        snprintf(g_create_err, sizeof(g_create_err), "%s", c->err);
        release(c);
        delete c;
        return code;
    };
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535 || (long)W * (long)H > (1L << 30) || (n > 0 && !spheres))
        return (fail(c, BDPT_EINVAL, "bdpt_create: bad size %dx%d or spheres", W, H), bail(BDPT_EINVAL));
    c->W = W; c->H = H; c->device = device;
    c->spheres.assign(spheres, spheres + n);
    if (const char* e = getenv("BDPT_SPECIALIZE")) c->specialize = atoi(e) != 0;   // default for new contexts
    // loadMTGPU (MersenneTwister_kernel.cu:23-36): 4096 x 16 B records
    FILE* f = fopen(mt_dat_path ? mt_dat_path : "assets/data/MersenneTwister.dat", "rb");
    if (!f) return (fail(c, BDPT_EIO, "initMTGPU(): failed to open %s", mt_dat_path), bail(BDPT_EIO));
    size_t got = fread(c->h_params, sizeof(c->h_params), 1, f);
    fclose(f);
    if (got != 1) return (fail(c, BDPT_EIO, "initMTGPU(): failed to load %s", mt_dat_path), bail(BDPT_EIO));
    if (device == BDPT_DEVICE_CPU) {                          // the host backend: no HIP at all
        c->cpu = bdpt_cpu_create(spheres, n, W, H, c->h_params);
        if (!c->cpu) return (fail(c, BDPT_ENOMEM, "bdpt_create: CPU backend allocation"), bail(BDPT_ENOMEM));
        for (unsigned i = 0; i < n; i++)
            if (!(spheres[i].e.x == 0.f && spheres[i].e.y == 0.f && spheres[i].e.z == 0.f)) c->lights.push_back((int)i);
        c->specialize = false;
        *out = c;
        return BDPT_OK;
    }
    if (device < 0) return (fail(c, BDPT_EINVAL, "bdpt_create: bad device %d", device), bail(BDPT_EINVAL));

#define CK(call) do { hipError_t e_ = (call); if (e_ != hipSuccess) { \
        fail(c, BDPT_EHIP, "%s: %s", #call, hipGetErrorString(e_)); return bail(BDPT_EHIP); } } while (0)
    CK(hipSetDevice(device));
    CK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (const char* tv = getenv("BDPT_STREAMS_TUNE")) c->tune_enabled = atoi(tv) != 0;
    {
        // BDPT_FOLD_PRIORITY=high|low: the fold stream's priority (experiments; default normal)
        const char* fp = getenv("BDPT_FOLD_PRIORITY");
        int lo = 0, hi = 0;
        if (fp && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
            CK(hipStreamCreateWithPriority(&c->fstream, hipStreamNonBlocking, !strcmp(fp, "high") ? hi : lo));
        else
            CK(hipStreamCreateWithFlags(&c->fstream, hipStreamNonBlocking));
    }
    for (int b = 0; b < 2; b++) {
        CK(hipEventCreateWithFlags(&c->rb_path_ev[b], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&c->rb_fold_ev[b], hipEventDisableTiming));
    }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->cus = cus;
    }
    for (auto& s : c->ring) {
        CK(hipEventCreate(&s.ev0));
        CK(hipEventCreate(&s.ev1));
    }
    const size_t np = (size_t)W * H;
    CK(hipMalloc(&c->d_params, sizeof(c->h_params)));
    CK(hipMalloc(&c->d_rand, sizeof(float) * BDPT_RAND_N));
    CK(hipMalloc(&c->d_rndp, sizeof(float) * BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL));
    CK(hipMalloc(&c->d_scp, sizeof(float2) * BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL));
    CK(hipMalloc(&c->d_lp, sizeof(bdpt_dev_lightpath) * BDPT_LIGHT_POINTS));
    CK(hipMalloc(&c->d_colors, sizeof(bdpt_dev_vec) * np));
    CK(hipMalloc(&c->d_counter, sizeof(unsigned) * np));
    CK(hipMalloc(&c->d_pixels, sizeof(uchar4) * np));
    CK(hipMalloc(&c->d_thr, sizeof(float) * 256));
    CK(hipMemsetAsync(c->d_lp, 0, sizeof(bdpt_dev_lightpath) * BDPT_LIGHT_POINTS, c->stream));
    CK(hipMemsetAsync(c->d_colors, 0, sizeof(bdpt_dev_vec) * np, c->stream));
    CK(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned) * np, c->stream));
    CK(hipMemsetAsync(c->d_pixels, 0, sizeof(uchar4) * np, c->stream));
    float thr[256];
    bdpt_gamma_thresholds(thr);
    CK(hipMemcpyAsync(c->d_thr, thr, sizeof(thr), hipMemcpyHostToDevice, c->stream));
    CK(hipStreamSynchronize(c->stream));
#undef CK
    rc = upload_scene(c);
    if (rc != BDPT_OK) return bail(rc);
    *out = c;
    return BDPT_OK;
}

const char* bdpt_create_error(void) { return g_create_err; }

static void destroy_group(bdpt_ctx* c);

void bdpt_destroy(bdpt_ctx* c) {
    if (!c) return;
    if (c->cpu) {
        bdpt_cpu_destroy(c->cpu);
        delete c;
        return;
    }
    destroy_group(c);
    (void)hipSetDevice(c->device);
    if (c->fstream) (void)hipStreamSynchronize(c->fstream);
    for (hipStream_t ps : c->pstream)
        if (ps) (void)hipStreamSynchronize(ps);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_prof) {                 // section profile of a -DBDPT_PROF kernel (experiments)
        unsigned long long p[24] = {};
        const char* pe = getenv("BDPT_PROF");
        if (pe && !strcmp(pe, "counts") && hipMemcpy(p, c->d_prof, sizeof p, hipMemcpyDeviceToHost) == hipSuccess) {
            fprintf(stderr, "bdpt_counts");        // region counts of a -DBDPT_COUNTS kernel
            for (int q = 0; q < 24; q++) fprintf(stderr, " %llu", p[q]);
            fprintf(stderr, "\n");
        } else if (hipMemcpy(p, c->d_prof, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
            double tot = 0;
            for (int q = 0; q < 6; q++) tot += (double)p[q];
            fprintf(stderr, "bdpt_prof waves=%llu cycles/wave=%.0f", p[7], p[7] ? tot / p[7] : 0.0);
            for (int q = 0; q < 6; q++) fprintf(stderr, " s%d=%.4f", q, tot > 0 ? p[q] / tot : 0.0);
            fprintf(stderr, "\n");
        }
        (void)hipFree(c->d_prof);
    }
    if (c->gl_res) (void)hipGraphicsUnregisterResource(c->gl_res);
    release(c);
    delete c;
}

static int one_set_scene(bdpt_ctx* c, const bdpt_sphere* spheres, unsigned n) {
    if (!c || (n > 0 && !spheres)) return BDPT_EINVAL;
    if (c->cpu) {
        c->spheres.assign(spheres, spheres + n);
        bdpt_cpu_set_scene(c->cpu, spheres, n);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    c->spheres.assign(spheres, spheres + n);
    return upload_scene(c);
}

static int one_set_camera(bdpt_ctx* c, const bdpt_camera* cam) {
    if (!c || !cam) return BDPT_EINVAL;
    if (c->cpu) bdpt_cpu_set_camera(c->cpu, cam);
    c->cam = *cam;
    c->cam_set = true;
    return BDPT_OK;
}

static int one_reset_accum(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_reset_accum(c->cpu);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipMemsetAsync(c->d_counter, 0, sizeof(unsigned) * (size_t)c->W * c->H, c->stream));
    if (c->d_uerr) {                                         // a new frame: no stale handover error
        HIPCHK(c, hipMemsetAsync(c->d_uerr, 0, sizeof(unsigned), c->stream));
        c->units_check = false;
    }
    return BDPT_OK;
}

static int one_set_shard(bdpt_ctx* c, int shard, int nshards, int band_rows) {
    if (!c || nshards < 1 || shard < 0 || shard >= nshards || band_rows < 1)
        return c ? fail(c, BDPT_EINVAL, "bdpt_set_shard: bad shard %d/%d band %d", shard, nshards, band_rows)
                 : BDPT_EINVAL;
    c->shard = shard; c->nshards = nshards; c->band_rows = band_rows;
    c->tune_phase = 0;
    if (c->cpu) bdpt_cpu_set_shard(c->cpu, shard, nshards, band_rows);
    return BDPT_OK;
}

static int one_set_streams(bdpt_ctx* c, int streams) {
    if (!c) return BDPT_EINVAL;
    if (streams < BDPT_STREAMS_PER_LANE || streams > BDPT_MAX_STREAMS)
        return fail(c, BDPT_EINVAL, "bdpt_set_streams: bad stream count %d", streams);
    c->streams_req = streams;
    c->tune_phase = 0;
    return BDPT_OK;
}

int bdpt_last_streams(const bdpt_ctx* c) { return c ? c->last_streams : BDPT_EINVAL; }

static int choice_of(const bdpt_ctx* c) {
    if (c->streams_req != 0 || !c->tune_enabled || c->tune_phase != bdpt_ctx::kTunePhases + 1) return 0;
    return BDPT_CHOICE_DECIDED | (c->tune_fused ? BDPT_CHOICE_FUSED : 0) | (c->tune_pair ? BDPT_CHOICE_PAIRED : 0) |
           (c->tune_quarter ? BDPT_CHOICE_QUARTER : 0) | (c->tune_pool ? BDPT_CHOICE_POOLS : 0) |
           (c->tune_units ? BDPT_CHOICE_UNITS : 0);
}

static int one_set_stream_choice(bdpt_ctx* c, int choice) {
    if (!c) return BDPT_EINVAL;
    if (!(choice & BDPT_CHOICE_DECIDED) || (choice & ~0x3f) ||
        ((choice & BDPT_CHOICE_POOLS) && (choice & BDPT_CHOICE_UNITS)))
        return fail(c, BDPT_EINVAL, "bdpt_set_stream_choice: bad choice 0x%x", choice);
    if (c->streams_req != 0)
        return fail(c, BDPT_ESTATE, "bdpt_set_stream_choice: the stream mode is not auto (%d)", c->streams_req);
    c->tune_fused = (choice & BDPT_CHOICE_FUSED) != 0;
    c->tune_pair = (choice & BDPT_CHOICE_PAIRED) != 0;
    c->tune_quarter = (choice & BDPT_CHOICE_QUARTER) != 0;
    c->tune_pool = (choice & BDPT_CHOICE_POOLS) != 0;
    c->tune_units = (choice & BDPT_CHOICE_UNITS) != 0;
    c->tune_enabled = true;
    c->tune_phase = bdpt_ctx::kTunePhases + 1;
    return BDPT_OK;
}

int bdpt_stream_choice(const bdpt_ctx* c) { return c ? choice_of(c) : BDPT_EINVAL; }

static int one_set_specialize(bdpt_ctx* c, int on) {
    if (!c) return BDPT_EINVAL;
    c->specialize = on != 0;
    jit_forget(c);
    c->tune_phase = 0;
    return BDPT_OK;
}

int bdpt_last_specialized(const bdpt_ctx* c) { return c ? (int)c->last_specialized : BDPT_EINVAL; }

const char* bdpt_specialize_status(const bdpt_ctx* c) { return c ? c->jit_err : "null context"; }

static int one_set_traversal(bdpt_ctx* c, int mode) {
    if (!c) return BDPT_EINVAL;
    if (mode != BDPT_TRAVERSE_AUTO && mode != BDPT_TRAVERSE_BRUTE && mode != BDPT_TRAVERSE_BVH)
        return fail(c, BDPT_EINVAL, "bdpt_set_traversal: bad mode %d", mode);
    c->traversal = mode;
    c->tune_phase = 0;
    return BDPT_OK;
}

int bdpt_scene_has_bvh(const bdpt_ctx* c) { return c ? (int)c->has_bvh : BDPT_EINVAL; }

int bdpt_last_traversal(const bdpt_ctx* c) {
    return c ? (c->last_bvh ? BDPT_TRAVERSE_BVH : BDPT_TRAVERSE_BRUTE) : BDPT_EINVAL;
}

static int one_generate_rand(bdpt_ctx* c, unsigned seed) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_generate_rand(c->cpu, seed);
        c->rand_ready = true;
        c->rand_seed = seed;
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;              // path kernels read the table
    // seedMTGPU(seed): every record's seed field := seed (MersenneTwister_kernel.cu:44-47)
    std::vector<uint32_t> p(c->h_params, c->h_params + 4 * BDPT_MT_RNG_COUNT);
    for (int i = 0; i < BDPT_MT_RNG_COUNT; i++) p[4 * i + 3] = seed;
    HIPCHK(c, hipMemcpyAsync(c->d_params, p.data(), sizeof(uint32_t) * p.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(bdpt_mt607_kernel, dim3(BDPT_MT_RNG_COUNT / 64), dim3(64), 0, c->stream,
                       (const uint4*)c->d_params, seed, c->d_rand);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(bdpt_rand_planar_kernel, dim3((BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL + 255) / 256),
                       dim3(256), 0, c->stream, (const float*)c->d_rand, c->d_rndp);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(bdpt_sincos_planar_kernel, dim3((BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL + 255) / 256),
                       dim3(256), 0, c->stream, (const float*)c->d_rndp, c->d_scp);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->rand_ready = true;
    c->rand_seed = seed;
    return BDPT_OK;
}

static int one_light_pass(bdpt_ctx* c, int current_sample) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_light_pass(c->cpu, current_sample);
        c->rand_ready = true;
        c->rand_seed = (unsigned)(current_sample * 5);
        return BDPT_OK;
    }
    // The reference regenerates the table per light with the same seed (smallpt_cpu.c:321-322):
    // one generation is identical.  With no emitter it launches nothing and the path pass reads
    // an uninitialised d_Rand; we generate the table anyway (the frame is black either way:
    // there is no emission, and dev_lp stays zero) so the run is defined.
    int rc = one_generate_rand(c, (unsigned)(current_sample * 5));
    if (rc) return rc;
    if (c->lights.empty()) return BDPT_OK;
    hipLaunchKernelGGL(bdpt_light_kernel, dim3(BDPT_LIGHT_POINTS / 64), dim3(64), 0, c->stream,
                       (const bdpt_dev_sphere*)c->d_sph, (unsigned)c->spheres.size(),
                       (const float*)c->d_rand, current_sample, c->d_lp);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

// camera terms of device.cu:572-592, with the kernel's float operation order
static void vnorm3(float v[3]) {
    float l = 1.f / sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] = l * v[0]; v[1] = l * v[1]; v[2] = l * v[2];
}

static int one_path_passes(bdpt_ctx* c, const unsigned* sid, const int* vlp, int npass) {
    if (!c) return BDPT_EINVAL;
    if (npass < 0 || (npass > 0 && (!sid || !vlp))) return fail(c, BDPT_EINVAL, "bdpt_path_passes: bad pass list");
    if (npass == 0) return BDPT_OK;
    if (!c->rand_ready) return fail(c, BDPT_ESTATE, "bdpt_path_passes: no random table (run the light pass first)");
    if (!c->cam_set) return fail(c, BDPT_ESTATE, "bdpt_path_passes: camera not set");
    if (c->cpu) {                                           // synchronous; wall-clock timing
        const auto t0 = std::chrono::steady_clock::now();
        bdpt_cpu_path_passes(c->cpu, sid, vlp, npass);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        c->last_ms = (float)ms;
        c->acc_ms += ms;
        c->acc_kernel_ms += ms;
        c->acc_launches += 1;
        c->last_streams = 1;
        c->last_specialized = false;
        c->last_bvh = false;
        c->last_features = 0;
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    // this call's ring slot was last used kRing calls ago: wait for (only) that call
    const int slot = (int)(c->issued % bdpt_ctx::kRing);
    if (int rc = fold_timing(c, c->issued - bdpt_ctx::kRing + 1)) return rc;
    // every launch carries its pass table (<= 128 passes: the launch cap below) in the kernel
    // arguments: no upload, no copy kernel (and its gap) before the path kernel
    static_assert(BDPT_DEV_INLINE_PASSES >= 128, "launches of up to 128 passes");
    bdpt_ctx::call_slot& cs = c->ring[slot];

    bdpt_path_args a;
    memset(&a, 0, sizeof(a));
    a.sph = c->d_sph;
    a.n = (unsigned)c->spheres.size();
    a.n_lights = (unsigned)c->lights.size();
    a.lights = c->d_lights;
    a.lightrec = c->d_lightrec;
    a.geom = c->d_geom;
    a.vgeom = c->d_geom + c->spheres.size();
    a.n_vac = (int)c->n_vac;
    a.emis_mask = c->emis_mask;
    a.rnd = c->d_rand;
    a.rndp = c->d_rndp;
    a.scp = c->d_scp;
    a.lp = c->d_lp;
    a.colors = c->d_colors;
    a.counter = c->d_counter;
    a.pixels = c->d_pixels;
    a.gamma_thr = c->d_thr;
    a.W = c->W; a.H = c->H;
    a.inv_w = (float)(14. / c->W);                       // smallpt_cpu.c:411-412
    a.inv_h = (float)(10.5 / c->H);
    a.half_w = (double)(a.inv_w * (float)c->W) / 2.;      // device.cu:565 inv_width*width/2.
    a.half_h = (double)(a.inv_h * (float)c->H) / 2.;
    const bdpt_camera& cam = c->cam;
    float ux[3] = {cam.x.x, cam.x.y, cam.x.z}, uy[3] = {cam.y.x, cam.y.y, cam.y.z};
    float ud[3] = {cam.dir.x, cam.dir.y, cam.dir.z};
    vnorm3(ux); vnorm3(uy); vnorm3(ud);
    float nx[3] = {-1.f * cam.x.x, -1.f * cam.x.y, -1.f * cam.x.z};
    float ny[3] = {-1.f * cam.y.x, -1.f * cam.y.y, -1.f * cam.y.z};
    float nd[3] = {-1.f * cam.dir.x, -1.f * cam.dir.y, -1.f * cam.dir.z};
    vnorm3(nx); vnorm3(ny);                               // :584-590 (no vnorm on -dir, :591)
    a.tx = nx[0] * cam.orig.x + nx[1] * cam.orig.y + nx[2] * cam.orig.z;
    a.ty = ny[0] * cam.orig.x + ny[1] * cam.orig.y + ny[2] * cam.orig.z;
    a.tz = nd[0] * cam.orig.x + nd[1] * cam.orig.y + nd[2] * cam.orig.z;
    memcpy(a.ux, ux, sizeof(ux)); memcpy(a.uy, uy, sizeof(uy)); memcpy(a.ud, ud, sizeof(ud));
    a.orig[0] = cam.orig.x; a.orig[1] = cam.orig.y; a.orig[2] = cam.orig.z;
    a.shard = c->shard; a.nshards = c->nshards; a.band_rows = c->band_rows;
    if (!c->d_prof && getenv("BDPT_PROF")) {
        HIPCHK(c, hipMalloc(&c->d_prof, 24 * sizeof(unsigned long long)));
        HIPCHK(c, hipMemset(c->d_prof, 0, 24 * sizeof(unsigned long long)));
    }
    a.prof = c->d_prof;

    // Grid rows: every tile row, or (bands a whole number of tile rows) only this shard's bands.
    const int tile_rows = (c->H + BDPT_BTH - 1) / BDPT_BTH;
    int grid_rows = tile_rows;
    a.tiles_per_band = 0;
    if (c->nshards > 1 && c->band_rows % BDPT_BTH == 0) {
        const int tpb = c->band_rows / BDPT_BTH;
        const int nbands = (c->H + c->band_rows - 1) / c->band_rows;
        const int owned = c->shard < nbands ? (nbands - c->shard + c->nshards - 1) / c->nshards : 0;
        a.tiles_per_band = tpb;
        grid_rows = owned * tpb;
        // only the frame's last band can be partial: launch none of its tile rows below the frame
        if (owned > 0) {
            const int last = c->shard + (owned - 1) * c->nshards;          // this shard's last band
            const int tail = (last + 1) * tpb - tile_rows;
            if (tail > 0) grid_rows -= tail;
        }
    }
    // Pass streams: auto = one pass per lane (S = the launch's pass count).  Eye paths are capped
    // at 7 segments and most reach the cap, so single-path lanes keep a wave almost perfectly
    // balanced, while a lane that regenerates through many passes waits for the wave's slowest
    // sum (+11.7 % at 1080p, and it fills the GPU when a shard has few pixels).
    const long lanes = (long)grid_rows * BDPT_BTH * c->W;
    int S = c->streams_req;
    if (S <= 0) S = BDPT_MAX_STREAMS;
    // auto: measure both kernels on the first two calls, then keep the faster
    int tune_role = -1;
    bool pair = true;                                        // fused kernel: paired segment loads
    if (c->streams_req == 0 && c->tune_enabled) {
        const bdpt_ctx* lead = c->tune_leader;
        if (c->tune_phase == bdpt_ctx::kTunePhases && lead && lead->streams_req == 0 &&
            lead->tune_phase == bdpt_ctx::kTunePhases + 1) {  // a group peer: devices[0] decided
            c->tune_fused = lead->tune_fused;
            c->tune_pair = lead->tune_pair;
            c->tune_quarter = lead->tune_quarter;
            c->tune_pool = lead->tune_pool;
            c->tune_units = lead->tune_units;
            c->tune_phase = bdpt_ctx::kTunePhases + 1;
        }
        if (c->tune_phase == bdpt_ctx::kTunePhases) {        // waits for the last measured call
            if (int rc = fold_timing(c, c->tune_call[bdpt_ctx::kTunePhases - 1] + 1)) return rc;
            const double inf = std::numeric_limits<double>::infinity();
            auto per = [&](int r) { return c->tune_real[r] ? c->tune_ms[r] / c->tune_npass[r] : inf; };
            const double half = std::min(per(0), per(3)), quarter = std::min(per(2), per(5));
            const double pooled = std::min(per(6), per(7)), units = std::min(per(8), per(9));
            const double fp = per(1), fn = per(4);
            c->tune_pair = !(fn < fp);                       // the default unless unpaired was measured faster
            c->tune_quarter = quarter < half;
            c->tune_pool = pooled < std::min(half, quarter) && !(units < pooled);
            c->tune_units = units < std::min(std::min(half, quarter), pooled);
            const double fused = c->tune_pair ? fp : fn;
            const double streams = std::min(std::min(std::min(half, quarter), pooled), units);
            c->tune_fused = fused * (1.0 + bdpt_ctx::kTuneMargin) < streams;
            c->tune_phase = bdpt_ctx::kTunePhases + 1;
        }
        if (c->tune_phase < bdpt_ctx::kTunePhases && npass >= 2) {
            tune_role = c->tune_phase;
            if (tune_role == 1 || tune_role == 4) S = 1;
            pair = tune_role != 4;
        } else if (c->tune_phase == bdpt_ctx::kTunePhases + 1 && c->tune_fused) {
            S = 1;
            pair = c->tune_pair;
        }
    }
    a.nloc = (int)lanes;
    dim3 grid((c->W + BDPT_BTW - 1) / BDPT_BTW, grid_rows, 1), block(256);
    // keep single launches bounded (~2^28 samples, <= 128 passes for the LDS pass tables)
    const long per_pass = lanes > 0 ? lanes : 1;
    int chunk = (int)((1L << 28) / per_pass);
    if (chunk < 1) chunk = 1;
    if (chunk > 128) chunk = 128;
    if (const char* mp = getenv("BDPT_MAX_LAUNCH_PASSES")) {   // experiments: smaller launches
        const int m = atoi(mp);
        if (m >= 1 && m < chunk) chunk = m;
    }
    if (S > chunk) S = chunk;
    if (S > npass) S = npass;
    if (S < 1) S = 1;
    if (S == 1 && chunk > fused_max_passes()) chunk = fused_max_passes();   // fused: LDS per pass
    // equal launches: 128 passes over a 4097 x 513-row band (chunk 126) are 2 x 64, not 126 + 2
    if (npass > chunk) {
        const int nch = (npass + chunk - 1) / chunk;
        chunk = (npass + nch - 1) / nch;
        if (S > chunk) S = chunk;
    }
    const bool bvh = c->has_bvh && (c->traversal == BDPT_TRAVERSE_BVH ||
                                    (c->traversal == BDPT_TRAVERSE_AUTO && c->bvh_ns >= kBvhAutoSpheres));
    // auto: the pass-stream kernel renders two passes per lane in launches of >= 4 passes (lanes
    // whose first path ends early start the second in groups, bdpt_kernels.hip BDPT_REGEN_STREAMS):
    // cornell +0.6 %, cornell_glass +1.7 %, cornell_mirror +1.5 %; not for BVH traversal
    // (complex -4.6 %: its lanes' traversal costs differ more than their path lengths)
    // (four passes per lane when the measurement chose them, or to measure them; launches of >= 8)
    bool quarter_ran = false;
    if (c->streams_req == 0 && S >= 4 && !bvh) {
        const bool quarter = tune_role >= 0 ? (tune_role == 2 || tune_role == 5)
                                            : (c->tune_phase == bdpt_ctx::kTunePhases + 1 && c->tune_quarter);
        quarter_ran = quarter && S >= 8;
        S = quarter_ran ? (S + 3) / 4 : (S + 1) / 2;
    }
    // pixel pools: forced by BDPT_POOL=R, or measured (tuning roles 6, 7) and kept
    const int penv = pool_env();
    const bool want_pool = !bvh && S > 1 && penv != 0 &&
                           (penv > 0 || (c->streams_req == 0 &&
                                         (tune_role == 6 || tune_role == 7 ||
                                          (tune_role < 0 && c->tune_phase == bdpt_ctx::kTunePhases + 1 &&
                                           c->tune_pool))));
    if (want_pool) S = chunk < npass ? chunk : npass;        // one pass per lane slice
    // ordered in-kernel fold (units of a tile and a range of passes; no radiance buffer): forced by
    // BDPT_UNITS=P (ranges of P passes), or measured (tuning roles 8, 9) and kept; not for shards
    // whose tile workgroups cannot keep the chip busy with one range per tile (a tile's units run
    // one after another)
    const int uenv = units_env();
    const bool units_fit = (long)((c->W + BDPT_BTW - 1) / BDPT_BTW) * grid_rows >= 2L * c->cus * 6;
    const bool want_units = !bvh && S > 1 && !want_pool && uenv != 0 &&
                            (uenv > 0 || (c->streams_req == 0 && units_fit &&
                                          (tune_role >= 8 || (tune_role < 0 && c->tune_phase == bdpt_ctx::kTunePhases + 1 &&
                                                              c->tune_units))));
    const int unit_passes = uenv > 0 ? uenv : kUnitPasses;
    c->last_streams = S;
    const int kidx = bvh ? 17 : (a.n <= 16 ? (int)a.n : 0);
    if (bvh) {
        a.bvh_nodes = c->d_bvh_nodes; a.bvh_geom = c->d_bvh_geom; a.bvh_ids = c->d_bvh_ids;
        a.big_geom = c->d_big_geom; a.big_ids = c->d_big_ids; a.mat = c->d_mat;
        a.bvh_nn = c->bvh_nn; a.bvh_ns = c->bvh_ns; a.big_n = c->big_n;
        for (int k = 0; k < 3; k++) a.bvh_c[k] = c->bvh_c[k];
        a.bvh_r = c->bvh_r;
        a.bvh_q = c->bvh_q;
    }
    c->last_bvh = bvh;
    if (S > 1 && !want_units) {
        const int cmax = npass < chunk ? npass : chunk;
        const size_t need = (size_t)cmax * (size_t)lanes;
        if (need > c->rbuf_cap || (size_t)lanes > c->rmask_lanes) {
            HIPCHK(c, hipStreamSynchronize(c->stream));     // queued passes and folds may use it
            HIPCHK(c, hipStreamSynchronize(c->fstream));
            for (hipStream_t ps : c->pstream)
                if (ps) HIPCHK(c, hipStreamSynchronize(ps));
            if (c->d_rbuf) HIPCHK(c, hipFree(c->d_rbuf));
            if (c->d_rmask) HIPCHK(c, hipFree(c->d_rmask));
            c->d_rbuf = nullptr;
            c->d_rmask = nullptr;
            c->rbuf_cap = 0;
            c->rb_used[0] = c->rb_used[1] = false;
            if (hipMalloc(&c->d_rbuf, 2 * sizeof(bdpt_dev_vec) * need) != hipSuccess)
                return fail(c, BDPT_ENOMEM, "bdpt_path_passes: pass-stream buffer (2 x %zu B)", sizeof(bdpt_dev_vec) * need);
            if (hipMalloc(&c->d_rmask, 2 * 16 * (size_t)lanes) != hipSuccess)
                return fail(c, BDPT_ENOMEM, "bdpt_path_passes: pass-stream mask (2 x %zu B)", 16 * (size_t)lanes);
            c->rmask_lanes = (size_t)lanes;
            c->rbuf_cap = need;
            // touch every page now (queued before this call's timing event): the first launch
            // would otherwise pay the first-touch cost, and the stream-mode measurement with it
            HIPCHK(c, hipMemsetAsync(c->d_rbuf, 0, 2 * sizeof(bdpt_dev_vec) * need, c->stream));
            HIPCHK(c, hipMemsetAsync(c->d_rmask, 0, 2 * 16 * (size_t)lanes, c->stream));
        }
    }
    const size_t nchunks = grid_rows > 0 ? (size_t)((npass + chunk - 1) / chunk) : 0;
    while (cs.kev.size() < 2 * nchunks) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        cs.kev.push_back(e);
    }
    // resolve the specialised kernels (a compile on first use) before the timed region starts
    hipFunction_t jf_streams = nullptr, jf_fused = nullptr, jf_pool = nullptr, jf_units = nullptr;
    bool any_fused = false, pool_ran = false, units_ran = false;
    for (int p0 = 0; grid_rows > 0 && p0 < npass; p0 += chunk) {
        const int np = npass - p0 < chunk ? npass - p0 : chunk;
        const bool st = (S < np ? S : np) > 1;
        any_fused |= !st;
        if (bvh) continue;
        if (st && want_pool && !jf_pool) jf_pool = jit_path_kernel(c, true, true, true);
        if (st && want_units && !jf_units) jf_units = jit_path_kernel(c, true, true, false, true);
        if (st && !jf_pool && !jf_units && !jf_streams) jf_streams = jit_path_kernel(c, true);
        if (!st && !jf_fused) jf_fused = jit_path_kernel(c, false, pair);
    }
    // Pixel pools fold on the context's stream right after each path kernel (serial fold, over
    // their sparse radiance): the concurrent fold's HBM traffic slowed the next call's pooled path
    // kernel more than the fold costs on its own -- caustic pools 4.10 -> 4.04-4.07 ms per call,
    // path kernel 3.93 -> 3.29-3.31 ms; two passes per lane keep the concurrent fold (cornell
    // S = 64 33.82 -> 33.92 ms serial), profiles/r05_s11_serial_fold.txt.
    const bool serial_fold = jf_pool != nullptr;
    // Pooled launches overlap: each runs (with its fold) on pstream[half], so a launch's drain --
    // ~0.1 ms at its end, when all passes' pools run out together and the last paths finish at
    // falling occupancy -- overlaps the next launch's start (caustic8 +1.1 to +1.7 %, its 1/4 and
    // 1/8 shares +4 to +6 %, profiles/r05_s37_pool_overlap.txt).  Not in the stream mode's tuning
    // calls (measured one at a time, as the other modes); BDPT_POOL_OVERLAP=0 turns it off.
    static const bool overlap_env = !getenv("BDPT_POOL_OVERLAP") || atoi(getenv("BDPT_POOL_OVERLAP")) != 0;
    const bool overlap = serial_fold && overlap_env && tune_role < 0;
    // a fused launch updates colors itself, and a serial fold does so on this stream: they wait
    // for the outstanding concurrent fold, before the call's timing starts (so the stream-mode
    // measurement does not charge that fold to it); overlapped pooled launches order their folds
    // through rb_fold_ev instead
    if (any_fused || jf_units || (serial_fold && !overlap))
        if (int rc = join_fold(c)) return rc;
    if (overlap) {
        if (!c->pstream[0]) {
            for (hipStream_t& ps : c->pstream) HIPCHK(c, hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
            HIPCHK(c, hipEventCreateWithFlags(&c->amark, hipEventDisableTiming));
        }
        HIPCHK(c, hipEventRecord(c->amark, c->stream));  // the pstreams follow `stream`'s earlier work
    }
    bool ev0_done = !overlap;
    if (!overlap) HIPCHK(c, hipEventRecord(cs.ev0, c->stream));
    int launches = 0;
    for (int p0 = 0; grid_rows > 0 && p0 < npass; p0 += chunk, launches++) {
        a.npass = npass - p0 < chunk ? npass - p0 : chunk;
        a.sid = nullptr;
        a.vlp = nullptr;
        for (int q = 0; q < a.npass; q++) {
            a.sid_inl[q] = sid[p0 + q];
            a.vlp_inl[q] = vlp[p0 + q];
        }
        // scene tables (4 per sphere, or the BVH: 2 per node + 1 per sphere) + per-pass VLPs +
        // camera + 4 wave shadow queues (results written over maxt) + sids (+ BVH sphere ids)
#ifdef BDPT_BVH_LDS
        const size_t tree = 2 * (size_t)a.bvh_nn + a.bvh_ns, tree_ids = a.bvh_ns;
#else
        const size_t tree = 0, tree_ids = 0;                 // tree read through L1/L2
#endif
        const size_t tab = bvh ? tree + a.big_n : 4 * (size_t)a.n + (size_t)a.n_vac;   // (bdpt_kernels.hip ntab)
        const size_t ids = bvh ? tree_ids + a.big_n : 0;
        // S per launch: a short last chunk gets no idle stream slices
        const bool st = (S < a.npass ? S : a.npass) > 1;     // the pass-stream kernel
        const bool pooled = st && jf_pool != nullptr;        // its pixel-pool build
        const bool unitsl = st && jf_units != nullptr;       // its ordered in-kernel fold build
        a.streams = S < a.npass ? S : a.npass;
        if (unitsl) a.unit_passes = unit_passes < a.npass ? unit_passes : a.npass;
        // a workgroup stages the VLPs and sids of its own passes only (bdpt_kernels.hip nslot)
        const size_t slots = unitsl ? (size_t)a.unit_passes : ((size_t)a.npass + a.streams - 1) / a.streams;
        size_t smem = sizeof(float4) * (tab + 3 * slots + 5 + 4 * 128 * 2)
                      + sizeof(unsigned) * (slots + ids);
        if (const char* pad = getenv("BDPT_SMEM_PAD"))       // experiments: cap workgroups per CU
            smem += (size_t)atoi(pad);
        if (smem > 160 * 1024)
            return fail(c, BDPT_EINVAL, "bdpt_path_passes: scene too large for LDS (%u spheres)", a.n);
        const void* kern = bdpt_path_kernel_table[st * 18 + kidx];
        const hipFunction_t jf = st ? (pooled ? jf_pool : unitsl ? jf_units : jf_streams) : jf_fused;
        c->last_specialized = jf != nullptr;
        c->last_features = BDPT_FEAT_LAST_SKIP | (bvh ? BDPT_FEAT_BVH : 0) | (st ? BDPT_FEAT_STREAMS : 0) |
                           (pooled ? BDPT_FEAT_POOLS : 0) | (unitsl ? BDPT_FEAT_UNITS : 0) |
                           (st && !pooled ? BDPT_FEAT_SCP : 0) |
                           (jf ? BDPT_FEAT_SPECIALIZED | BDPT_FEAT_DET_SKIP | (c->jit_zero_exit ? BDPT_FEAT_ZERO_EXIT : 0) : 0);
        void* kargs[] = {&a};
        grid.z = a.streams;
        const int half = c->rb_next;
        // the stream of this launch (and of its fold): `stream`, or pstream[half] for an
        // overlapped pooled launch
        hipStream_t ls = c->stream;
        if (pooled && overlap) {
            ls = c->pstream[half];
            HIPCHK(c, hipStreamWaitEvent(ls, c->amark, 0));
        }
        if (!ev0_done) {                                     // the call's time starts here
            HIPCHK(c, hipEventRecord(cs.ev0, ls));
            ev0_done = true;
        }
        if (unitsl) {
            // the units fold in the kernel: no radiance buffer; the previous call's folds were
            // joined above
            a.rbuf = nullptr;
            a.rmask = nullptr;
        } else if (st) {
            // this half was last read by the fold of the launch before the previous one
            if (c->rb_used[half]) HIPCHK(c, hipStreamWaitEvent(ls, c->rb_fold_ev[half], 0));
            a.rbuf = c->d_rbuf + (size_t)half * c->rbuf_cap;
            a.rmask = c->d_rmask + (size_t)half * 4 * c->rmask_lanes;
            // pools mark their stored samples in the mask: cleared first (the fold that read this
            // half ran earlier on this stream)
            if (jf_pool) HIPCHK(c, hipMemsetAsync(a.rmask, 0, 16 * (size_t)lanes, ls));
        } else if (int rc = join_fold(c)) {                  // the fused kernel updates colors itself
            return rc;
        }
        // pixel pools (a specialised pass-stream build with BDPT_POOL): waves of pool x 64 pixels
        dim3 pgrid = grid;
        a.pool = 0;
        a.pool_ctr = nullptr;
        if (pooled) {                                        // per pass 8 counters, a 128-B line each
            if (a.streams != a.npass || a.npass > 128)
                return fail(c, BDPT_EINVAL, "bdpt_path_passes: pixel pools need one pass per stream (%d of %d)",
                            a.streams, a.npass);
            constexpr size_t kSet = 128 * 8 * 32;            // words per set
            if (!c->d_poolctr) {
                HIPCHK(c, hipMalloc(&c->d_poolctr, 2 * kSet * sizeof(unsigned)));
                HIPCHK(c, hipMemsetAsync(c->d_poolctr, 0, 2 * kSet * sizeof(unsigned), c->stream));
                c->pool_set = 0;
            }
            int R = 1, G = 1;
            pool_shape(lanes, overlap, &R, &G);
            a.pool = R;
            if (overlap) {
                // set `half`, cleared on this launch's stream (its previous user, the launch two
                // back, ran earlier on the same stream); the kernel clears no next set
                a.pool_ctr = c->d_poolctr + (size_t)half * kSet;
                a.pool_ctr_next = nullptr;
                HIPCHK(c, hipMemsetAsync(a.pool_ctr, 0, kSet * sizeof(unsigned), ls));
                c->pool_dirty = true;
            } else {
                if (c->pool_dirty) {                         // overlapped launches left both sets used
                    HIPCHK(c, hipMemsetAsync(c->d_poolctr, 0, 2 * kSet * sizeof(unsigned), c->stream));
                    c->pool_dirty = false;
                }
                a.pool_ctr = c->d_poolctr + (size_t)c->pool_set * kSet;
                a.pool_ctr_next = c->d_poolctr + (size_t)(c->pool_set ^ 1) * kSet;
                c->pool_set ^= 1;
            }
            // 1-D, passes interleaved in groups of 8 workgroups (bdpt_kernels.hip s0)
            const long span = 256L * G, per = ((lanes + span - 1) / span + 7) / 8 * 8;
            pgrid = dim3((unsigned)(per * a.streams), 1, 1);
            pool_ran = true;
        }
        if (unitsl) {
            // one workgroup per unit; each claims its unit from its XCD's queue (bdpt_kernels.hip)
            const int wgs = (int)grid.x * grid_rows;
            // the last passes in halving ranges (bdpt_device.h bdpt_unit_range); BDPT_UNITS_TAPER=0 off
            static const int taper = getenv("BDPT_UNITS_TAPER") ? atoi(getenv("BDPT_UNITS_TAPER")) != 0 : 1;
            a.unit_taper = taper;
            const int nranges = bdpt_unit_ranges(a.npass, a.unit_passes, a.unit_taper);
            const size_t nflags = (size_t)wgs * 4;
            if (!c->d_uerr) {                                // error word + 8 queue counters, 128 B apart
                HIPCHK(c, hipMalloc(&c->d_uerr, sizeof(unsigned) * (32 + 8 * 32)));
                HIPCHK(c, hipMemsetAsync(c->d_uerr, 0, sizeof(unsigned), c->stream));
            }
            HIPCHK(c, hipMemsetAsync(c->d_uerr + 32, 0, sizeof(unsigned) * 8 * 32, c->stream));
            if (nflags > c->uflags_cap || ((c->uepoch + 1) & 0xffffffu) == 0) {
                if (nflags > c->uflags_cap) {
                    HIPCHK(c, hipStreamSynchronize(c->stream));
                    if (c->d_uflags) HIPCHK(c, hipFree(c->d_uflags));
                    c->d_uflags = nullptr;
                    HIPCHK(c, hipMalloc(&c->d_uflags, sizeof(unsigned) * nflags));
                    c->uflags_cap = nflags;
                }
                HIPCHK(c, hipMemsetAsync(c->d_uflags, 0, sizeof(unsigned) * c->uflags_cap, c->stream));
                c->uepoch = 0;
            }
            c->uepoch++;                                     // tags never repeat within 2^24 launches
            a.unit_tag = c->uepoch << 8;
            a.unit_flags = c->d_uflags;
            a.unit_err = c->d_uerr;
            a.unit_ctr = c->d_uerr + 32;
            a.unit_wgs = wgs;
            a.gx = (int)grid.x;
            a.gy = grid_rows;
            pgrid = dim3((unsigned)(wgs * nranges), 1, 1);
            c->units_check = true;
            units_ran = true;
        }
        HIPCHK(c, hipEventRecord(cs.kev[2 * launches], ls));
        if (jf)
            HIPCHK(c, hipModuleLaunchKernel(jf, pgrid.x, pgrid.y, pgrid.z, block.x, 1, 1, (unsigned)smem,
                                            ls, kargs, nullptr));
        else
            HIPCHK(c, hipLaunchKernel(kern, grid, block, kargs, smem, ls));
        HIPCHK(c, hipEventRecord(cs.kev[2 * launches + 1], ls));
        const dim3 fgrid((unsigned)((lanes + 255) / 256), 1, 1);   // the fold: 1-D over the launch's rows
        if (st && !unitsl && serial_fold) {                 // the fold after the path kernel
            // (overlapped: after the previous fold too, wherever it ran)
            if (overlap && c->fold_pending) HIPCHK(c, hipStreamWaitEvent(ls, c->rb_fold_ev[c->fold_last], 0));
            HIPCHK(c, hipLaunchKernel((const void*)&bdpt_accum_serial_kernel, fgrid, block, kargs, 0, ls));
            if (overlap) {
                HIPCHK(c, hipEventRecord(c->rb_fold_ev[half], ls));
                c->rb_used[half] = true;
                c->fold_last = half;
                c->fold_pending = true;
                c->fold_stream = ls;
                c->rb_next = half ^ 1;
            }
        } else if (st && !unitsl) {                         // the ordered fold, on fstream
            HIPCHK(c, hipEventRecord(c->rb_path_ev[half], c->stream));
            HIPCHK(c, hipStreamWaitEvent(c->fstream, c->rb_path_ev[half], 0));
            // after the previous fold (an overlapped pooled launch's ran on a pstream)
            if (c->fold_pending && c->fold_stream != c->fstream)
                HIPCHK(c, hipStreamWaitEvent(c->fstream, c->rb_fold_ev[c->fold_last], 0));
            c->fold_stream = c->fstream;
            HIPCHK(c, hipLaunchKernel((const void*)&bdpt_accum_kernel, fgrid, block, kargs, 0, c->fstream));
            HIPCHK(c, hipEventRecord(c->rb_fold_ev[half], c->fstream));
            c->rb_used[half] = true;
            c->fold_last = half;
            c->fold_pending = true;
            c->rb_next = half ^ 1;
        }
    }
    // the call ends with its last fold (fstream, which waited for the path kernels) if one is
    // outstanding, else on the context's stream
    HIPCHK(c, hipEventRecord(cs.ev1, c->fold_pending ? c->fold_stream : c->stream));
    cs.launches = launches;
    cs.pending = true;
    cs.serial_fold = serial_fold;
    if (tune_role >= 0) {
        c->tune_real[tune_role] = tune_role == 2 || tune_role == 5 ? quarter_ran
                                  : tune_role == 1 || tune_role == 4 ? (jf_fused != nullptr || tune_role == 1)
                                  : tune_role == 6 || tune_role == 7 ? pool_ran
                                  : tune_role >= 8 ? units_ran
                                  : true;
        c->tune_call[tune_role] = c->issued;
        c->tune_npass[tune_role] = npass;
        c->tune_phase = tune_role + 1;
    }
    c->issued++;
    return BDPT_OK;
}

// After the stream has drained: did a unit's handover wait time out in a units launch since the
// last check?  Reported once by whichever call looks first (synchronize, the timing calls, the
// read-backs); the error word is then cleared, so later launches report only their own timeouts.
static int units_verdict(bdpt_ctx* c) {
    if (!c->units_check) return BDPT_OK;
    unsigned e = 0;
    HIPCHK(c, hipMemcpy(&e, c->d_uerr, sizeof e, hipMemcpyDeviceToHost));
    c->units_check = false;
    if (!e) return BDPT_OK;
    HIPCHK(c, hipMemset(c->d_uerr, 0, sizeof e));
    return fail(c, BDPT_EHIP, "path kernel: a unit waited too long for its tile's previous range "
                              "(its predecessor did not finish within ~1 s; the frame is not valid)");
}

static int one_synchronize(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) return BDPT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (int rc = units_verdict(c)) return rc;
    return fold_timing(c);
}

int bdpt_last_path_ms(bdpt_ctx* c, float* ms) {
    if (!c || !ms) return BDPT_EINVAL;
    if (int rc = one_synchronize(c)) return rc;
    if (c->acc_launches == 0) return fail(c, BDPT_ESTATE, "bdpt_last_path_ms: no path pass launched");
    *ms = c->last_ms;
    return BDPT_OK;
}

static int one_path_timing(bdpt_ctx* c, double* total_ms, long long* launches, int reset) {
    if (!c) return BDPT_EINVAL;
    if (int rc = one_synchronize(c)) return rc;
    if (total_ms) *total_ms = c->acc_ms;
    if (launches) *launches = c->acc_launches;
    if (reset) { c->acc_ms = 0.0; c->acc_kernel_ms = 0.0; c->acc_launches = 0; }
    return BDPT_OK;
}

static int one_kernel_timing(bdpt_ctx* c, double* kernel_ms, long long* launches, int reset) {
    if (!c) return BDPT_EINVAL;
    if (int rc = one_synchronize(c)) return rc;
    if (kernel_ms) *kernel_ms = c->acc_kernel_ms;
    if (launches) *launches = c->acc_launches;
    if (reset) { c->acc_ms = 0.0; c->acc_kernel_ms = 0.0; c->acc_launches = 0; }
    return BDPT_OK;
}

static int one_read_radiance(bdpt_ctx* c, bdpt_vec* colors, unsigned* counter) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_read_radiance(c->cpu, colors, counter);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    const size_t np = (size_t)c->W * c->H;
    if (colors) HIPCHK(c, hipMemcpyAsync(colors, c->d_colors, sizeof(bdpt_vec) * np, hipMemcpyDeviceToHost, c->stream));
    if (counter) HIPCHK(c, hipMemcpyAsync(counter, c->d_counter, sizeof(unsigned) * np, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return units_verdict(c);                                 // a frame known to be invalid is an error
}

static int one_read_pixels(bdpt_ctx* c, unsigned char* rgba) {
    if (!c || !rgba) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_read_pixels(c->cpu, rgba);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipMemcpyAsync(rgba, c->d_pixels, 4 * (size_t)c->W * c->H, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return units_verdict(c);
}

int bdpt_read_rand(bdpt_ctx* c, float* t) {
    if (!c || !t) return BDPT_EINVAL;
    if (!c->rand_ready) return fail(c, BDPT_ESTATE, "bdpt_read_rand: table not generated");
    if (c->cpu) {
        bdpt_cpu_read_rand(c->cpu, t);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(t, c->d_rand, sizeof(float) * BDPT_RAND_N, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_read_lightpaths(bdpt_ctx* c, bdpt_lightpath* lp) {
    if (!c || !lp) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_read_lightpaths(c->cpu, lp);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(lp, c->d_lp, sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

static int one_write_lightpaths(bdpt_ctx* c, const bdpt_lightpath* lp) {
    if (!c || !lp) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_write_lightpaths(c->cpu, lp);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    // queued passes may still read dev_lp: overlapped pooled launches run on the pstreams, which
    // `stream` follows only through the last fold
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_lp, lp, sizeof(bdpt_lightpath) * BDPT_LIGHT_POINTS, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_rand_seed(const bdpt_ctx* c, unsigned* seed) {
    if (!c || !seed) return BDPT_EINVAL;
    if (!c->rand_ready) return BDPT_ESTATE;
    *seed = c->rand_seed;
    return BDPT_OK;
}

int bdpt_get_camera(const bdpt_ctx* c, bdpt_camera* cam) {
    if (!c || !cam) return BDPT_EINVAL;
    if (!c->cam_set) return BDPT_ESTATE;
    *cam = c->cam;
    return BDPT_OK;
}

int bdpt_get_scene(const bdpt_ctx* c, bdpt_sphere* spheres, unsigned cap) {
    if (!c) return BDPT_EINVAL;
    const unsigned n = (unsigned)c->spheres.size();
    if (spheres)
        for (unsigned i = 0; i < n && i < cap; i++) spheres[i] = c->spheres[i];
    return (int)n;
}

int bdpt_frame_size(const bdpt_ctx* c, int* W, int* H) {
    if (!c || !W || !H) return BDPT_EINVAL;
    *W = c->W;
    *H = c->H;
    return BDPT_OK;
}

int bdpt_last_kernel_features(const bdpt_ctx* c) { return c ? c->last_features : BDPT_EINVAL; }

static int one_device_buffers(bdpt_ctx* c, void** colors, void** counter, void** pixels) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) return fail(c, BDPT_EINVAL, "bdpt_device_buffers: the CPU backend has no device buffers");
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;                   // work queued on the stream follows the fold
    if (colors) *colors = c->d_colors;
    if (counter) *counter = c->d_counter;
    if (pixels) *pixels = c->d_pixels;
    return BDPT_OK;
}

static int one_update_pixels(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) {
        bdpt_cpu_update_pixels(c->cpu);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    const int np = c->W * c->H;
    hipLaunchKernelGGL(bdpt_pixels_kernel, dim3((np + 255) / 256), dim3(256), 0, c->stream,
                       (const bdpt_dev_vec*)c->d_colors, c->d_pixels, (const float*)c->d_thr, np);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

}  // extern "C"

// ---- multi-device contexts (SURVEY.md 8(b) `devices[], ndev`; 5: RCCL in one process) --------
// bdpt_create_multi makes one context per device: the first renders on devices[0] and owns the
// others (peers).  Device k renders the 8-row bands (y / 8) % ndev == k; every other entry point
// applies to all devices (each rebuilds the MT table and the VLPs itself: they are deterministic),
// and the read-back entry points first assemble the frame on devices[0]: an in-process RCCL
// ncclReduce (sum) of the float radiance and the counters over ncclCommInitAll's communicator
// (the sum is exact, each pixel is non-zero on one device only), or, when the devices are not
// distinct (several shards on one GPU) or RCCL is unavailable, peer copies plus an add kernel.
namespace {
struct rccl_api {
    bool ok = false;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    decltype(&ncclGetVersion) version = nullptr;       // optional (reporting only)
};

const rccl_api& rccl() {
    static const rccl_api api = [] {
        rccl_api r;
        // torch (when loaded) has mapped its own librccl.so.1 already: the same SONAME binds to it
        const char* libs[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        void* h = nullptr;
        for (const char* l : libs)
            if ((h = dlopen(l, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) return r;
        r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.reduce = (decltype(r.reduce))dlsym(h, "ncclReduce");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.errstr = (decltype(r.errstr))dlsym(h, "ncclGetErrorString");
        r.version = (decltype(r.version))dlsym(h, "ncclGetVersion");
        r.ok = r.init_all && r.destroy && r.reduce && r.group_start && r.group_end && r.errstr;
        return r;
    }();
    return api;
}

// The group bracket of the in-process frame reduce: every device's two ncclReduce calls between
// one ncclGroupStart and one ncclGroupEnd.  A failed hipSetDevice or ncclReduce stops issuing but
// still closes the group (an open group would make the next RCCL call on the communicators fail
// with an unrelated error); the first error is returned in *he / the result.  Templated on the
// calls so that tests can drive it with injected failures (bdpt__test_reduce_bracket).
template <class Start, class End, class SetDev, class Reduce>
ncclResult_t reduce_bracket(int ndev, Start start, End end, SetDev set_device, Reduce reduce, hipError_t* he) {
    *he = hipSuccess;
    ncclResult_t r = start();
    if (r != ncclSuccess) return r;                   // no group was opened
    for (int k = 0; k < ndev && r == ncclSuccess && *he == hipSuccess; k++) {
        *he = set_device(k);
        if (*he != hipSuccess) break;
        r = reduce(k, 0);                             // colours
        if (r == ncclSuccess) r = reduce(k, 1);       // counters
    }
    const ncclResult_t e = end();                     // always: the group is closed
    return r != ncclSuccess ? r : e;
}
}  // namespace

static void destroy_group(bdpt_ctx* c) {
    if (!c->multi) return;
    for (bdpt_ctx* p : c->peers) {
        (void)hipSetDevice(p->device);
        if (p->fstream) (void)hipStreamSynchronize(p->fstream);
        if (p->stream) (void)hipStreamSynchronize(p->stream);
    }
    if (!c->comms.empty() && rccl().ok)
        for (void* cm : c->comms) (void)rccl().destroy((ncclComm_t)cm);
    c->comms.clear();
    for (bdpt_ctx* p : c->peers) bdpt_destroy(p);
    c->peers.clear();
}

// Apply `f` to every peer; the first failure is reported on the group context.
template <class F>
static int forward(bdpt_ctx* c, F f) {
    for (bdpt_ctx* p : c->peers)
        if (int rc = f(p)) return fail(c, rc, "device %d: %s", p->device, p->err);
    c->frame_stale = true;
    return BDPT_OK;
}

// Group shard layout: device k of a group that is shard `shard` of `nshards` groups renders
// shard shard * ndev + k of nshards * ndev.
static int group_set_shard(bdpt_ctx* c, int shard, int nshards, int band_rows) {
    const int ndev = 1 + (int)c->peers.size();
    if (int rc = one_set_shard(c, shard * ndev, nshards * ndev, band_rows)) return rc;
    for (int k = 1; k < ndev; k++)
        if (int rc = one_set_shard(c->peers[k - 1], shard * ndev + k, nshards * ndev, band_rows))
            return fail(c, rc, "device %d: %s", c->peers[k - 1]->device, c->peers[k - 1]->err);
    c->frame_stale = true;
    return BDPT_OK;
}

// Assemble the frame of a multi-device context on devices[0] (d_fcolors/d_fcounter/d_fpixels).
static int assemble(bdpt_ctx* c) {
    if (!c->multi || !c->frame_stale) return BDPT_OK;
    if (int rc = one_synchronize(c)) return rc;
    for (bdpt_ctx* p : c->peers)
        if (int rc = one_synchronize(p)) return fail(c, rc, "device %d: %s", p->device, p->err);
    const size_t np = (size_t)c->W * c->H;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->d_fcolors) {
        HIPCHK(c, hipMalloc(&c->d_fcolors, sizeof(bdpt_dev_vec) * np));
        HIPCHK(c, hipMalloc(&c->d_fcounter, sizeof(unsigned) * np));
        HIPCHK(c, hipMalloc(&c->d_fpixels, sizeof(uchar4) * np));
    }
    if (c->reduce_mode == kReduceRccl) {
        const rccl_api& api = rccl();
        auto dev = [&](int k) { return k == 0 ? c : c->peers[k - 1]; };
        hipError_t he = hipSuccess;
        const ncclResult_t r = reduce_bracket(
            (int)c->comms.size(), [&] { return api.group_start(); }, [&] { return api.group_end(); },
            [&](int k) { return hipSetDevice(dev(k)->device); },
            [&](int k, int what) {
                bdpt_ctx* d = dev(k);
                return what == 0
                    ? api.reduce(d->d_colors, k == 0 ? (void*)c->d_fcolors : (void*)d->d_colors, 3 * np, ncclFloat32,
                                 ncclSum, 0, (ncclComm_t)c->comms[k], d->stream)
                    : api.reduce(d->d_counter, k == 0 ? (void*)c->d_fcounter : (void*)d->d_counter, np, ncclUint32,
                                 ncclSum, 0, (ncclComm_t)c->comms[k], d->stream);
            },
            &he);
        (void)hipSetDevice(c->device);
        if (he != hipSuccess) return fail(c, BDPT_EHIP, "frame reduce: hipSetDevice: %s", hipGetErrorString(he));
        if (r != ncclSuccess) return fail(c, BDPT_EHIP, "ncclReduce: %s", api.errstr(r));
        for (size_t k = 1; k < c->comms.size(); k++) {
            HIPCHK(c, hipSetDevice(c->peers[k - 1]->device));
            HIPCHK(c, hipStreamSynchronize(c->peers[k - 1]->stream));
        }
        HIPCHK(c, hipSetDevice(c->device));
    } else {
        HIPCHK(c, hipMemcpyAsync(c->d_fcolors, c->d_colors, sizeof(bdpt_dev_vec) * np, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_fcounter, c->d_counter, sizeof(unsigned) * np, hipMemcpyDeviceToDevice, c->stream));
        if (!c->peers.empty() && !c->d_ftmp) {
            HIPCHK(c, hipMalloc(&c->d_ftmp, sizeof(bdpt_dev_vec) * np));
            HIPCHK(c, hipMalloc(&c->d_ftmpc, sizeof(unsigned) * np));
        }
        for (bdpt_ctx* p : c->peers) {
            HIPCHK(c, hipMemcpyPeerAsync(c->d_ftmp, c->device, p->d_colors, p->device, sizeof(bdpt_dev_vec) * np, c->stream));
            HIPCHK(c, hipMemcpyPeerAsync(c->d_ftmpc, c->device, p->d_counter, p->device, sizeof(unsigned) * np, c->stream));
            hipLaunchKernelGGL(bdpt_frame_add_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, c->stream,
                               (float*)c->d_fcolors, (const float*)c->d_ftmp, c->d_fcounter,
                               (const unsigned*)c->d_ftmpc, (int)np);
            HIPCHK(c, hipGetLastError());
        }
    }
    hipLaunchKernelGGL(bdpt_pixels_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, c->stream,
                       (const bdpt_dev_vec*)c->d_fcolors, c->d_fpixels, (const float*)c->d_thr, (int)np);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->frame_stale = false;
    return BDPT_OK;
}

extern "C" {

int bdpt_create_multi(bdpt_ctx** out, const bdpt_sphere* spheres, unsigned n, int W, int H,
                      const char* mt_dat_path, const int* devices, int ndev) {
    if (!out) return BDPT_EINVAL;
    *out = nullptr;
    bool has_cpu = false;
    for (int k = 0; devices && k < ndev && k < 64; k++) has_cpu = has_cpu || devices[k] < 0;
    if (!devices || ndev < 1 || ndev > 64 || has_cpu) {
        snprintf(g_create_err, sizeof g_create_err, "bdpt_create_multi: bad device list (%d devices)", ndev);
        return BDPT_EINVAL;
    }
    bdpt_ctx* c = nullptr;
    if (int rc = bdpt_create(&c, spheres, n, W, H, mt_dat_path, devices[0])) return rc;
    c->multi = true;
    for (int k = 1; k < ndev; k++) {
        bdpt_ctx* p = nullptr;
        if (int rc = bdpt_create(&p, spheres, n, W, H, mt_dat_path, devices[k])) {
            char msg[512];
            snprintf(msg, sizeof msg, "device %d: %s", devices[k], g_create_err);
            bdpt_destroy(c);
            snprintf(g_create_err, sizeof g_create_err, "%s", msg);
            return rc;
        }
        p->tune_leader = c;
        c->peers.push_back(p);
    }
    if (int rc = group_set_shard(c, 0, 1, 8)) {
        snprintf(g_create_err, sizeof g_create_err, "%s", c->err);
        bdpt_destroy(c);
        return rc;
    }
    // RCCL when every device is distinct (a communicator holds each GPU once), else peer copies
    bool distinct = true;
    for (int a = 0; a < ndev; a++)
        for (int b = a + 1; b < ndev; b++) distinct = distinct && devices[a] != devices[b];
    const char* force = getenv("BDPT_REDUCE");
    c->reduce_mode = kReducePeer;
    if (force && !strcmp(force, "peer")) {
        snprintf(c->reduce_note, sizeof c->reduce_note, "BDPT_REDUCE=peer");
    } else if (!distinct) {
        snprintf(c->reduce_note, sizeof c->reduce_note, "devices repeat: peer copies");
    } else if (!rccl().ok) {
        snprintf(c->reduce_note, sizeof c->reduce_note, "librccl not found: peer copies");
    } else {
        std::vector<ncclComm_t> comms(ndev);
        const ncclResult_t r = rccl().init_all(comms.data(), ndev, devices);
        if (r == ncclSuccess) {
            c->comms.assign(comms.begin(), comms.end());
            c->reduce_mode = kReduceRccl;
            const int v = bdpt_rccl_version();
            std::string ids;
            for (int k = 0; k < ndev; k++) ids += (k ? " " : "") + std::to_string(devices[k]);
            snprintf(c->reduce_note, sizeof c->reduce_note, "rccl %d.%d.%d, ncclCommInitAll: %d ranks on devices [%s]",
                     v / 10000, v / 100 % 100, v % 100, ndev, ids.c_str());
        } else {
            snprintf(c->reduce_note, sizeof c->reduce_note, "ncclCommInitAll: %s: peer copies", rccl().errstr(r));
        }
    }
    (void)hipSetDevice(devices[0]);
    *out = c;
    return BDPT_OK;
}

int bdpt_num_devices(const bdpt_ctx* c) { return c ? 1 + (int)c->peers.size() : BDPT_EINVAL; }

int bdpt_rccl_version(void) {
    const rccl_api& api = rccl();
    if (!api.ok) return BDPT_ESTATE;
    int v = 0;
    if (!api.version || api.version(&v) != ncclSuccess) return BDPT_ESTATE;
    return v;
}

int bdpt_reduce_info(const bdpt_ctx* c, char* buf, int cap) {
    if (!c || !buf || cap < 1) return BDPT_EINVAL;
    const char* s = !c->multi ? "none: one device" : c->reduce_note;
    snprintf(buf, (size_t)cap, "%s", s);
    return (int)strlen(s);
}

// Test hook (tests/test_abi_host.py): the reduce bracket driven by fake calls on `ndev` devices,
// hipSetDevice failing on device `fail_dev` and ncclReduce on call `fail_reduce` (-1: never).
// Returns the bracket's ncclResult_t; *open_groups = group starts minus ends afterwards (0: the
// group was closed), *reduces = ncclReduce calls issued, *hip_err = the hipError_t it reported.
int bdpt__test_reduce_bracket(int ndev, int fail_dev, int fail_reduce, int* open_groups, int* reduces,
                              int* hip_err) {
    int open = 0, calls = 0;
    hipError_t he = hipSuccess;
    const ncclResult_t r = reduce_bracket(
        ndev, [&] { open++; return ncclSuccess; }, [&] { open--; return ncclSuccess; },
        [&](int k) { return k == fail_dev ? hipErrorInvalidDevice : hipSuccess; },
        [&](int, int) { return calls++ == fail_reduce ? ncclUnhandledCudaError : ncclSuccess; }, &he);
    if (open_groups) *open_groups = open;
    if (reduces) *reduces = calls;
    if (hip_err) *hip_err = (int)he;
    return (int)r;
}

const char* bdpt_reduce_backend(const bdpt_ctx* c) {
    if (!c) return "null context";
    if (!c->multi) return "none";
    return c->reduce_mode == kReduceRccl ? "rccl" : "peer";
}

int bdpt_reduce_frame(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    return assemble(c);
}

// ---- the entry points: this context, then (multi-device) every peer ------------------------
int bdpt_set_scene(bdpt_ctx* c, const bdpt_sphere* spheres, unsigned n) {
    if (int rc = one_set_scene(c, spheres, n)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_scene(p, spheres, n); });
}
int bdpt_set_camera(bdpt_ctx* c, const bdpt_camera* cam) {
    if (int rc = one_set_camera(c, cam)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_camera(p, cam); });
}
int bdpt_reset_accum(bdpt_ctx* c) {
    if (int rc = one_reset_accum(c)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_reset_accum(p); });
}
int bdpt_set_shard(bdpt_ctx* c, int shard, int nshards, int band_rows) {
    if (!c) return BDPT_EINVAL;
    if (!c->multi) return one_set_shard(c, shard, nshards, band_rows);
    if (nshards < 1 || shard < 0 || shard >= nshards || band_rows < 1)
        return fail(c, BDPT_EINVAL, "bdpt_set_shard: bad shard %d/%d band %d", shard, nshards, band_rows);
    return group_set_shard(c, shard, nshards, band_rows);
}
int bdpt_set_streams(bdpt_ctx* c, int streams) {
    if (int rc = one_set_streams(c, streams)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_streams(p, streams); });
}
int bdpt_set_stream_choice(bdpt_ctx* c, int choice) {
    if (int rc = one_set_stream_choice(c, choice)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_stream_choice(p, choice); });
}
// One device of the group: the kernel its last path-pass call ran and its stream-mode choice.
int bdpt_device_mode(bdpt_ctx* c, int k, int* last_streams, int* features, int* choice) {
    if (!c) return BDPT_EINVAL;
    if (k < 0 || k > (int)c->peers.size())
        return fail(c, BDPT_EINVAL, "bdpt_device_mode: device index %d of %d", k, 1 + (int)c->peers.size());
    const bdpt_ctx* d = k == 0 ? c : c->peers[k - 1];
    if (last_streams) *last_streams = d->last_streams;
    if (features) *features = d->last_features;
    if (choice) *choice = choice_of(d);
    return BDPT_OK;
}
int bdpt_set_specialize(bdpt_ctx* c, int on) {
    if (int rc = one_set_specialize(c, on)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_specialize(p, on); });
}
int bdpt_set_traversal(bdpt_ctx* c, int mode) {
    if (int rc = one_set_traversal(c, mode)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_set_traversal(p, mode); });
}
int bdpt_generate_rand(bdpt_ctx* c, unsigned seed) {
    if (int rc = one_generate_rand(c, seed)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_generate_rand(p, seed); });
}
int bdpt_light_pass(bdpt_ctx* c, int current_sample) {
    if (int rc = one_light_pass(c, current_sample)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_light_pass(p, current_sample); });
}
// Every device's passes are queued before any is waited for: the devices render concurrently.
int bdpt_path_passes(bdpt_ctx* c, const unsigned* sid, const int* vlp, int npass) {
    if (int rc = one_path_passes(c, sid, vlp, npass)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_path_passes(p, sid, vlp, npass); });
}
int bdpt_synchronize(bdpt_ctx* c) {
    if (int rc = one_synchronize(c)) return rc;
    for (bdpt_ctx* p : c->peers)
        if (int rc = one_synchronize(p)) return fail(c, rc, "device %d: %s", p->device, p->err);
    return BDPT_OK;
}
// Multi-device: the slowest device's time (the devices run concurrently); launches of devices[0].
int bdpt_path_timing(bdpt_ctx* c, double* total_ms, long long* launches, int reset) {
    if (int rc = one_path_timing(c, total_ms, launches, reset)) return rc;
    for (bdpt_ctx* p : c->peers) {
        double ms = 0.0;
        if (int rc = one_path_timing(p, &ms, nullptr, reset)) return fail(c, rc, "device %d: %s", p->device, p->err);
        if (total_ms && ms > *total_ms) *total_ms = ms;
    }
    return BDPT_OK;
}
int bdpt_kernel_timing(bdpt_ctx* c, double* kernel_ms, long long* launches, int reset) {
    if (int rc = one_kernel_timing(c, kernel_ms, launches, reset)) return rc;
    for (bdpt_ctx* p : c->peers) {
        double ms = 0.0;
        if (int rc = one_kernel_timing(p, &ms, nullptr, reset)) return fail(c, rc, "device %d: %s", p->device, p->err);
        if (kernel_ms && ms > *kernel_ms) *kernel_ms = ms;
    }
    return BDPT_OK;
}
// One device of the group (k = 0 is devices[0]): its own accumulators, not the maximum, so a
// multi-device run can show load imbalance.  Does not reset.
int bdpt_device_timing(bdpt_ctx* c, int k, int* device, double* kernel_ms, double* path_ms,
                       long long* launches, long long* owned_pixels) {
    if (!c) return BDPT_EINVAL;
    if (k < 0 || k > (int)c->peers.size())
        return fail(c, BDPT_EINVAL, "bdpt_device_timing: device index %d of %d", k, 1 + (int)c->peers.size());
    bdpt_ctx* d = k == 0 ? c : c->peers[k - 1];
    if (int rc = one_synchronize(d)) return d == c ? rc : fail(c, rc, "device %d: %s", d->device, d->err);
    if (device) *device = d->cpu ? BDPT_DEVICE_CPU : d->device;
    if (kernel_ms) *kernel_ms = d->acc_kernel_ms;
    if (path_ms) *path_ms = d->acc_ms;
    if (launches) *launches = d->acc_launches;
    if (owned_pixels) {
        long long rows = 0;
        for (int y = 0; y < d->H; y++) rows += (y / d->band_rows) % d->nshards == d->shard;
        *owned_pixels = rows * d->W;
    }
    return BDPT_OK;
}
// Read-back of a multi-device context reads the assembled frame.
int bdpt_write_lightpaths(bdpt_ctx* c, const bdpt_lightpath* lp) {
    if (int rc = one_write_lightpaths(c, lp)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_write_lightpaths(p, lp); });
}
int bdpt_read_radiance(bdpt_ctx* c, bdpt_vec* colors, unsigned* counter) {
    if (!c) return BDPT_EINVAL;
    if (!c->multi) return one_read_radiance(c, colors, counter);
    if (int rc = assemble(c)) return rc;
    const size_t np = (size_t)c->W * c->H;
    if (colors) HIPCHK(c, hipMemcpyAsync(colors, c->d_fcolors, sizeof(bdpt_vec) * np, hipMemcpyDeviceToHost, c->stream));
    if (counter) HIPCHK(c, hipMemcpyAsync(counter, c->d_fcounter, sizeof(unsigned) * np, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}
int bdpt_read_pixels(bdpt_ctx* c, unsigned char* rgba) {
    if (!c || !rgba) return BDPT_EINVAL;
    if (!c->multi) return one_read_pixels(c, rgba);
    if (int rc = assemble(c)) return rc;
    HIPCHK(c, hipMemcpyAsync(rgba, c->d_fpixels, 4 * (size_t)c->W * c->H, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}
int bdpt_device_buffers(bdpt_ctx* c, void** colors, void** counter, void** pixels) {
    if (!c) return BDPT_EINVAL;
    if (!c->multi) return one_device_buffers(c, colors, counter, pixels);
    if (int rc = assemble(c)) return rc;
    if (colors) *colors = c->d_fcolors;
    if (counter) *counter = c->d_fcounter;
    if (pixels) *pixels = c->d_fpixels;
    return BDPT_OK;
}
int bdpt_update_pixels(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (!c->multi) return one_update_pixels(c);
    return assemble(c);
}

// ---- checkpoint / resume of the accumulation ----------------------------------
// Upload colors/counter (the counterpart of bdpt_read_radiance) and recompute the pixels.  A
// multi-device context gives each device only the pixels of its own bands (zeros elsewhere), so
// the assembled frame is the uploaded one.
static int one_write_radiance(bdpt_ctx* c, const bdpt_vec* colors, const unsigned* counter, bool masked) {
    if (c->cpu) {
        bdpt_cpu_write_radiance(c->cpu, colors, counter);
        return BDPT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = join_fold(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t np = (size_t)c->W * c->H;
    std::vector<bdpt_vec> col;
    std::vector<unsigned> cnt;
    if (masked) {
        col.assign(colors, colors + np);
        cnt.assign(counter, counter + np);
        for (int y = 0; y < c->H; y++) {
            if ((y / c->band_rows) % c->nshards == c->shard) continue;
            memset(&col[(size_t)y * c->W], 0, sizeof(bdpt_vec) * c->W);
            memset(&cnt[(size_t)y * c->W], 0, sizeof(unsigned) * c->W);
        }
        colors = col.data();
        counter = cnt.data();
    }
    HIPCHK(c, hipMemcpyAsync(c->d_colors, colors, sizeof(bdpt_vec) * np, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_counter, counter, sizeof(unsigned) * np, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(bdpt_pixels_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, c->stream,
                       (const bdpt_dev_vec*)c->d_colors, c->d_pixels, (const float*)c->d_thr, (int)np);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_write_radiance(bdpt_ctx* c, const bdpt_vec* colors, const unsigned* counter) {
    if (!c || !colors || !counter) return BDPT_EINVAL;
    if (int rc = one_write_radiance(c, colors, counter, c->multi)) return rc;
    return forward(c, [&](bdpt_ctx* p) { return one_write_radiance(p, colors, counter, true); });
}

// ---- optional display: HIP-GL interop of the window's pixel-unpack buffer ----
// The reference registers its PBO once (cudaGLRegisterBufferObject, smallpt_cpu.c:112-123) and per
// frame maps it, lets the path kernel write pixels_buf = the mapped pointer, and unmaps it
// (IdleFunc, display_func.c:199-215).  Here the kernels keep writing d_pixels (the read-back,
// checkpoint and multi-device paths all read it) and a publish copies the finished frame into the
// mapped buffer on the context's stream: one 4*W*H-byte device copy per displayed frame (8.3 MB
// at 1080p, ~2 us of HBM time), the same bytes in the same bottom-row-first order.
//
// hipGraphicsGLRegisterBuffer needs an OpenGL context current on the calling thread; without one
// it is undefined what the runtime does, so the context is looked up first (GLX, then EGL) in
// libraries the process has already loaded -- libbdpt itself never links or loads OpenGL.
static bool gl_context_current() {
    typedef void* (*cur_fn)(void);
    const char* const libs[2] = {"libGL.so.1", "libEGL.so.1"};
    const char* const syms[2] = {"glXGetCurrentContext", "eglGetCurrentContext"};
    for (int k = 0; k < 2; k++) {
        cur_fn f = (cur_fn)dlsym(RTLD_DEFAULT, syms[k]);
        void* h = nullptr;
        if (!f && (h = dlopen(libs[k], RTLD_LAZY | RTLD_NOLOAD)) != nullptr) f = (cur_fn)dlsym(h, syms[k]);
        const bool cur = f && f() != nullptr;
        if (h) dlclose(h);
        if (cur) return true;
    }
    return false;
}

int bdpt_gl_register_pbo(bdpt_ctx* c, unsigned pbo) {
    if (!c) return BDPT_EINVAL;
    if (c->cpu) return fail(c, BDPT_EINVAL, "bdpt_gl_register_pbo: the CPU backend has no device pixels");
    if (!pbo) return fail(c, BDPT_EINVAL, "bdpt_gl_register_pbo: buffer name 0");
    if (!gl_context_current())
        return fail(c, BDPT_EINVAL, "bdpt_gl_register_pbo: no OpenGL context is current on this thread");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->gl_res) {
        HIPCHK(c, hipGraphicsUnregisterResource(c->gl_res));
        c->gl_res = nullptr;
        c->gl_pbo = 0;
    }
    hipGraphicsResource_t res = nullptr;                        // kept only on success
    HIPCHK(c, hipGraphicsGLRegisterBuffer(&res, pbo, hipGraphicsRegisterFlagsWriteDiscard));
    c->gl_res = res;
    c->gl_pbo = pbo;
    return BDPT_OK;
}

int bdpt_gl_publish(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (!c->gl_res) return fail(c, BDPT_ESTATE, "bdpt_gl_publish: no buffer registered (bdpt_gl_register_pbo)");
    void* pix = nullptr;
    if (int rc = bdpt_device_buffers(c, nullptr, nullptr, &pix)) return rc;   // multi: the assembled frame
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipGraphicsMapResources(1, &c->gl_res, c->stream));
    // from here the buffer is mapped: every path below unmaps it before returning
    const size_t bytes = 4 * (size_t)c->W * c->H;
    void* dst = nullptr;
    size_t size = 0;
    hipError_t e = hipGraphicsResourceGetMappedPointer(&dst, &size, c->gl_res);
    bool small = false;
    if (e == hipSuccess && size < bytes) small = true;
    else if (e == hipSuccess) e = hipMemcpyAsync(dst, pix, bytes, hipMemcpyDeviceToDevice, c->stream);
    const hipError_t u = hipGraphicsUnmapResources(1, &c->gl_res, c->stream);
    if (small)
        return fail(c, BDPT_EINVAL, "bdpt_gl_publish: buffer %u holds %zu bytes, the frame needs %zu",
                    c->gl_pbo, size, bytes);
    if (e != hipSuccess) return fail(c, BDPT_EHIP, "bdpt_gl_publish: mapped copy: %s", hipGetErrorString(e));
    if (u != hipSuccess) return fail(c, BDPT_EHIP, "bdpt_gl_publish: unmap: %s", hipGetErrorString(u));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_gl_unregister(bdpt_ctx* c) {
    if (!c) return BDPT_EINVAL;
    if (!c->gl_res) return BDPT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    hipGraphicsResource_t r = c->gl_res;
    c->gl_res = nullptr;
    c->gl_pbo = 0;
    HIPCHK(c, hipGraphicsUnregisterResource(r));
    return BDPT_OK;
}

// bdpt_save_checkpoint / bdpt_load_checkpoint: bdpt_ckpt.c (over the entry points above)
int bdpt__fail(bdpt_ctx* c, int code, const char* msg) { return fail(c, code, "%s", msg); }

}  // extern "C"


