// bdpt_kernels.hip -- hand-written HIP kernels for gfx950 (MI355X, CDNA4) implementing the render
// path of sim186/gpu_bidirectional_raytracer: the MT607 random table, the light pass (VLP
// creation) and the per-pixel eye-path integrator with NEE + VLP connection.
//
// Numerics contract (shared with the CPU oracle): fp32 with NO contraction
// (built with -ffp-contract=off), correctly rounded fp32 div/sqrt (hipcc default), the fp64 camera
// steps of device.cu:565-566,594 kept in fp64, and sinf/cosf evaluated as (float)sincos((double)x).
// Every float operation below is in the reference's order; reordering any of them changes
// results (SURVEY.md 7 "Hard parts").
#ifndef __HIPCC_RTC__                       // hipRTC provides the HIP runtime itself
#include <hip/hip_runtime.h>
#include <utility>
#endif
#include "bdpt_device.h"
#include "bdpt_math.h"

// Run-time specialised build (bdpt_host.cpp jit_path_kernel, hipRTC): only the path kernel, with
// the scene's sphere geometry {p, rad^2} (exact hex-float literals) and emitter mask as
// compile-time constants, so that every coordinate difference p - o the spheres share is formed
// once per ray and the scalar scene loads disappear.  The float operations are the same, in the
// same order, so the results equal the precompiled instance's bit for bit.
#ifdef BDPT_JIT
struct jit_geom { float x, y, z, w; };
constexpr jit_geom kJitGeom[BDPT_JIT_N] = BDPT_JIT_GEOM;
constexpr unsigned long long kJitEmis = BDPT_JIT_EMIS;
#endif

namespace {

// ---------------------------------------------------------------------------------------------
// small float3 helpers with the reference's operation order (vec.h:12-25)
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float a, float b, float c) { f3 v; v.x = a; v.y = b; v.z = c; return v; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 smul(float k, f3 b) { return mk(k * b.x, k * b.y, k * b.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// 1.f / x, correctly rounded: v_rcp_f32 + one Newton fma is exactly that for |x| in
// [2^-125, 2^125) (all 2^32 inputs checked on gfx950 by tests/native/hw_exact_check.hip); other
// x take the library division on an exec-masked branch.  rcp_rn_inrange: caller proves the range.
__device__ __forceinline__ float rcp_rn_inrange(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.f), r, r);
}
__device__ __forceinline__ float rcp_rn(float x) {
    const float ax = fabsf(x);
    if (__builtin_expect(!(ax >= 0x1p-125f && ax < 0x1p125f), 0)) return 1.f / x;
    return rcp_rn_inrange(x);
}
// 1.f / sqrtf(x) with both operations correctly rounded, one range test for the pair: for x in
// [2^-96, 2^126) the fast sqrt is exact and its root lies in [2^-48, 2^63), inside rcp_rn's range.
__device__ __forceinline__ float rcp_sqrt_rn(float x, float* root) {
    if (__builtin_expect(!(x >= 0x1p-96f && x < 0x1p126f), 0)) {
        *root = sqrtf(x);
        return 1.f / *root;
    }
    *root = bdpt_sqrt_rn_core(x);
    return rcp_rn_inrange(*root);
}

// a / b, correctly rounded, for a = +0 or a, b, a/b and the residual normal: one Markstein step on
// the exact reciprocal, y = RN(1/b), q = RN(a y), r = a - q b (exact by fma), RN(q + r y).  Checked
// on every pair of fp32 significands (2^46 pairs, 0 mismatches, scripts/div_check.hip); correct
// rounding of a quotient of normal numbers depends on the significands only.  The refraction
// weight divides Re or Tr (0 or in [2^-24, 1]: Tr = 1 - Re is a multiple of 2^-24) by P or 1 - P
// (in [1/4, 3/4]), so everything stays normal; a = +0 gives q = r = +0.
__device__ __forceinline__ float div_rn_normal(float a, float b) {
    const float y = rcp_rn_inrange(b);
    const float q = a * y;
    const float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ f3 norm(f3 v) {
    float root;
    return smul(rcp_sqrt_rn(dot(v, v), &root), v);             // one range test (above)
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ bool iszero3(f3 v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }

constexpr float kEps = 0.01f;                              // geom.h:6 EPSILON
constexpr float kPi = 3.14159265358979323846f;             // geom.h:7 FLOAT_PI
constexpr unsigned kRandN = BDPT_DEV_RAND_N;

// the table of bdpt_sincos_tab in device memory (copied to LDS by the path kernel)
__device__ const double bdpt_sincos_table_dev[BDPT_SC_N][2] = BDPT_SINCOS_TABLE_INIT;

// sinf/cosf with correctly-rounded semantics: fp64 sincos rounded once to fp32 (bdpt_math.h),
// table-driven when the caller has the sin(2pi k/N) table in LDS.
// The choice is a template argument, not a null test on `tab`: the compiler cannot prove an
// LDS-derived pointer non-null, and the dead minimax path then kept its fp64 coefficients in
// ~20 VGPRs across the whole path loop.
template <bool TAB>
__device__ __forceinline__ void sincos_cr(float x, float* s, float* c, const double* tab) {
    double sd, cd;
    if constexpr (TAB) bdpt_sincos_tab((double)x, tab, &sd, &cd);
    else bdpt_sincos_dp((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}

// SphereIntersectDevice device.cu:80-104 (g = {p.x, p.y, p.z, rad*rad}), branch-free.
// For 0 <= det < 2^-96 the root is not correctly rounded, but it is < 2^-47: then either
// |b| >= 2^-23 and fl(b -+ root) == b == fl(b -+ sqrtf(det)), or both roots are < EPSILON and the
// test returns 0 -- the result equals the reference's for every det.
__device__ __forceinline__ float sphere_isect(float4 g, f3 o, f3 d) {
    f3 op = mk(g.x - o.x, g.y - o.y, g.z - o.z);
    float b = dot(op, d);
    float det = b * b - dot(op, op) + g.w;
    const float s = bdpt_sqrt_rn_core(det);
    const float t1 = b - s, t2 = b + s;
    const float r = t1 > kEps ? t1 : (t2 > kEps ? t2 : 0.f);
    return det < 0.f ? 0.f : r;
}

// The two roots of the same test, t1 <= t2 (fl is monotone and the root is >= 0; both NaN for a
// negative det).  With r = t1 > EPS ? t1 : t2, the reference's hit (t1 > EPS ? t1 : t2 > EPS ?
// t2 : miss) is "r if t2 > EPS": when t1 > EPS, t2 >= t1 > EPS too.  So the closest-hit update is
// `t2 > EPS && r < t` and the shadow test `t2 > EPS && r < maxt`: one select fewer than with a
// +inf miss encoding (two compares and a select instead of two selects and a compare).
// The reference's `det < 0 -> miss` needs no test of its own (+2.7 % measured): a negative normal
// det gives a NaN root (bdpt_sqrt_rn_core), so t1, t2, r are NaN and t2 > EPS fails; so does a
// generated NaN det.  A negative denormal det may give a root of -0 (v_sqrt_f32 flushes it), so
// r = b -- but then b <= EPS, a miss again: if b > EPS, then fl(b*b) >= 1e-4 and X = fl(b*b - oo)
// is either > 0 (oo < b*b/2; then det >= X > 0) or a multiple of 2^-38 (ulp(oo) >= 2^-38), and
// det = fl(X + r*r) is then >= 0, <= -2^-39, or a nonzero multiple of ulp(r*r) >= 2^-83 -- never
// in (-2^-126, 0).  (det is never -0: fl(b*b) is not -0.)
struct troots { float t1, t2; };
__device__ __forceinline__ troots sphere_roots(float4 g, f3 o, f3 d) {
    f3 op = mk(g.x - o.x, g.y - o.y, g.z - o.z);
    float b = dot(op, d);
    float det = b * b - dot(op, op) + g.w;
    const float s = bdpt_sqrt_rn_core(det);
    return {b - s, b + s};
}
// The same test in two steps, so that a wave can stop after `det` when no lane's det is >= 0 (or
// NaN): every such lane misses (the reference returns 0 for det < 0, device.cu:95), so the root,
// its correction, the two roots and the selects of that sphere are skipped for the whole wave.
// Specialised kernels use it for the non-wall spheres (radius < 1000: for a wall every line hits),
// where most waves' rays all miss the sphere's line.
struct tdet { float b, det; };
__device__ __forceinline__ tdet sphere_det(float4 g, f3 o, f3 d) {
    f3 op = mk(g.x - o.x, g.y - o.y, g.z - o.z);
    float b = dot(op, d);
    return {b, b * b - dot(op, op) + g.w};
}
__device__ __forceinline__ troots roots_of(tdet q) {
    const float s = bdpt_sqrt_rn_core(q.det);
    return {q.b - s, q.b + s};
}
// Hit distances as unsigned keys (BDPT_IKEY; specialised kernels): key(x) = bits(x) - kKeyC mod
// 2^32 with kKeyC = bits(EPSILON) + 1.  For x > EPSILON (+inf included) key(x) <= key(+inf) and
// the key increases with x; every x <= EPSILON (+0 included), every NaN and every negative float
// maps above key(+inf) (the subtraction wraps, or the sign bit survives it).  t1 <= t2 (or both
// NaN), so min(key(t1), key(t2)) is key(t1 > EPS ? t1 : t2) when that value is > EPS and a miss
// key otherwise: the closest-hit update becomes one min3 with the running key (plus the compare
// and select of the index), and the shadow test one unsigned compare against key(maxt) (0 when
// maxt <= EPS or NaN: nothing occludes, as in the float test).
// (The rule is checked on edge values and random roots by tests/test_ikey_rule.py.)  On in the
// scene-specialised kernels: cornell +0.7 to +1.1 %, cornell_glass +0.6 %, synthetic64 +-0.1 %,
// fused caustic / open +0.4 to +1.5 %, simple +3 to +4 % (one session each,
// profiles/r03_s33_ab_ikey.txt); with the min3 written in C the compiler emits two v_min_u32
// and the kernels run 0.5-1 % slower than without keys.
#ifndef BDPT_IKEY
#ifdef BDPT_JIT
#define BDPT_IKEY 1
#else
#define BDPT_IKEY 0
#endif
#endif
constexpr unsigned kKeyC = 0x3C23D70Bu;                      // bits(0.01f) + 1
__device__ __forceinline__ unsigned key_of(float x) { return __float_as_uint(x) - kKeyC; }
__device__ __forceinline__ unsigned umin2(unsigned a, unsigned b) { return a < b ? a : b; }
// one v_min3_u32 (left to itself the compiler compares min(b, c) with a and keeps a separate min:
// two half-rate v_min_u32, and the kernels ran 0.5-1 % slower than without keys)
__device__ __forceinline__ unsigned umin3(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ unsigned maxt_key(float maxt) { return maxt > kEps ? key_of(maxt) : 0u; }

// UniformSampleSphereDevice device.cu:157-165, with s, c = sinf, cosf(2 pi u2) given
__device__ __forceinline__ f3 uniform_sphere_sc(float u1, float s, float c) {
    const float zz = 1.f - 2.f * u1;
    const float q = 1.f - zz * zz;
    const float r = bdpt_sqrt_rn_core(0.f > q ? 0.f : q);   // q is 0 or >= 2^-24: core is exact
    return mk(r * c, r * s, zz);
}
template <bool TAB = false>
__device__ __forceinline__ f3 uniform_sphere(float u1, float u2, const double* tab = nullptr) {
    const float phi = 2.f * kPi * u2;
    float s, c;
    sincos_cr<TAB>(phi, &s, &c, tab);
    return uniform_sphere_sc(u1, s, c);
}

// Cosine-weighted direction about w (device.cu:676-699; also :190-212 and :357-380).
template <bool TAB = false>
__device__ __forceinline__ f3 cosine_dir(f3 w, float u_phi, float u_r2, const double* tab = nullptr) {
    const float r1 = 2.f * kPi * u_phi;
    const float r2 = u_r2;
    const float r2s = bdpt_sqrt_rn_core(r2);                 // r2 = d_Rand value >= 2^-32
    f3 a = fabsf(w.x) > .1f ? mk(0.f, 1.f, 0.f) : mk(1.f, 0.f, 0.f);
    const f3 uc = cross(a, w);                                // |uc|^2 >= 0.01 by the choice of a
    f3 u = smul(rcp_rn_inrange(bdpt_sqrt_rn_core(dot(uc, uc))), uc);   // 0.1 <= |uc| <= 1
    f3 v = cross(w, u);
    float s, c;
    sincos_cr<TAB>(r1, &s, &c, tab);
    u = smul(c * r2s, u);
    v = smul(s * r2s, v);
    f3 nd = add(u, v);
    w = smul(bdpt_sqrt_rn_core(1 - r2), w);                   // 1 - r2 is 0 or >= 2^-24
    return add(nd, w);
}

// The rest of cosine_dir once u = normalize(cross(a, w)) and r2s = sqrt(r2) are known (the path
// kernel computes those two on a path shared with refraction): the same operations in the same
// order as cosine_dir.
// (s, c = sinf, cosf(2 pi u_phi) given: cosine_tail_sc)
__device__ __forceinline__ f3 cosine_tail_sc(f3 w, f3 u, float s, float c, float u_r2, float r2s) {
    f3 v = cross(w, u);
    u = smul(c * r2s, u);
    v = smul(s * r2s, v);
    f3 nd = add(u, v);
    w = smul(bdpt_sqrt_rn_core(1 - u_r2), w);                // 1 - r2 is 0 or >= 2^-24
    return add(nd, w);
}
template <bool TAB = false>
__device__ __forceinline__ f3 cosine_tail(f3 w, f3 u, float u_phi, float u_r2, float r2s,
                                          const double* tab = nullptr) {
    const float r1 = 2.f * kPi * u_phi;
    float s, c;
    sincos_cr<TAB>(r1, &s, &c, tab);
    return cosine_tail_sc(w, u, s, c, u_r2, r2s);
}

// sinf / cosf of 2 pi u for every entry u of the random table, computed once per table
// (bdpt_sincos_planar_kernel, planar like d_rndp) instead of per use (BDPT_SCP, pass-stream
// kernels): the phi of the NEE light sample (u = d_Rand[j + 4], device.cu:162) and of the cosine
// direction (u = d_Rand[j], :677) are both 2 pi u of a table entry, so the per-vertex fp64 sincos
// becomes one 8-B load from the same plane offset as the entry itself.  The stored pair is
// sincos_cr's result for that u, so results are unchanged bit for bit.
#ifndef BDPT_SCP
#define BDPT_SCP 1
#endif
#ifndef BDPT_SCP_LATE
#define BDPT_SCP_LATE 0
#endif
// Shadow rounds whose rays are all VLP rays (IntersectPVacuumDevice, device.cu:141-154, ignores
// emitters) skip the emitters' sphere tests: the NEE rays fill the queue first, so a segment's
// second round is usually VLP rays only.
#ifndef BDPT_VAC_SKIP
#define BDPT_VAC_SKIP 1
#endif
// Lane groups of a part-full shadow round: 2^lg groups for rounds of <= 64 / 2^lg rays (lg <= 5),
// reduced only while fewer groups take as few iterations -- caustic's 3 spheres in 1 iteration
// instead of 2, cornell's 9 in 1 for rounds of <= 4 rays (BDPT_LG_RULE=0: the round-5 rule, lg <= 3,
// reduced while 2^lg exceeds the list)
#ifndef BDPT_LG_RULE
#define BDPT_LG_RULE 1
#endif
// The same rounds when they are part-full (<= 32 rays, traced by lane groups that split the sphere
// list): the groups split the non-emitters' list (bdpt_path_args.vgeom, staged in LDS as GV).
// Not in the pixel-pool build: caustic8 ran 2 % slower with it (profiles/r06_s23_ab_vac_list.txt);
// scene-specialised builds only (the precompiled per-N instances would spill SGPRs from N = 9).
#ifndef BDPT_VAC_LIST
#ifdef BDPT_JIT
#define BDPT_VAC_LIST 1
#else
#define BDPT_VAC_LIST 0
#endif
#endif

// Fused S = 1 kernel: a lane whose path ends parks until at least BDPT_REGEN_K lanes of its wave
// (or all of its live lanes) are parked; then they start their next passes together, so the
// camera-ray and path-start code runs for groups of lanes instead of a few lanes in almost every
// iteration.  1 = restart at once (no parking); 64 = whole-wave lockstep.  One-session A/B
// (profiles/r03_s13_ab_regen.txt): caustic8 48.5 -> 52.3 Gs/s (+7.8 %) at 48, the same within
// 0.5 % for 16..56, 49.1 at 64; open +2 to +3.5 %, simple +1 %, cornell (fused) +10 %.
#ifndef BDPT_REGEN_K
#define BDPT_REGEN_K 48
#endif
// The same grouping for pass-stream lanes that render more than one pass (S < npass; the auto
// stream mode runs two passes per lane, bdpt_host.cpp); then the planar RNG copy is read too (a
// group restarts on one slot, so one sid and depth).  Two passes per lane with grouping against
// one pass per lane, one-session A/B (profiles/r03_s16_ab_regen_streams.txt): cornell +0.7 %,
// cornell_glass +0.8 %, synthetic64 -0.2 %; without grouping two passes per lane cost 3.5-6 %.
// Fused kernel: a parking lane loads its next pass's first-segment randoms at once (it waits at
// least an iteration before it uses them), and its camera randoms a second time into cr0, cr1
// (buffer loads, so the compiler does not merge them with the q0, q1 loads).  caustic8 +1.9 %,
// open +0.3 % in one-session A/B (profiles/r03_s19_ab_park_prefetch.txt); pass streams keep
// loading at release (cornell -1.1 % with it).  An ablation without any table reads runs caustic8
// 37 % faster: the fused kernel's random gathers (20 B per lane and segment at unrelated
// addresses, 6.6 TB/s of L2 fills) are what is left to win on open scenes.
// Fused kernel: the randoms of two segments (depth d even and d + 1) are loaded together, so a
// path's table line is fetched once for both instead of being evicted from L2 between them
// (caustic8 +9 %, open -4 %: the auto stream mode measures the fused kernel with and without it
// and keeps the faster, bdpt_host.cpp; profiles/r03_s22_ab_rng_pair.txt)
#ifndef BDPT_RNG_PAIR
#define BDPT_RNG_PAIR 1
#endif
// pass streams: radiance stores to the fold buffer with the nontemporal (streaming) hint
// pass streams: parked lanes load their next pass's randoms at park time (see the loop)
// pass streams: the segment's randoms settled before the radiance stores (see the loop)
// Pass streams with pixel pools (a build with BDPT_POOL; bdpt_host.cpp launches it with a.pool = R):
// a wave renders ONE pass, and a lane whose path ends takes the next pixel of the wave's pool --
// the lanes stay on one sid, so a restarted group's random gathers stay adjacent in the planar
// copy, unlike lanes that restart on their next pass (another sid each).  The pools are chunks
// of a.pool x 64 consecutive pixels of the launch's rows, claimed with one vector atomic per
// chunk until the pass's pixels are used up, so the waves of a pass finish together instead of
// each waiting on its own last paths.  A pass's pixels are split in 8 parts with a counter each
// (on lines of their own), and a wave claims from the part of its XCD first (one counter word
// saturates near 90 claims/us), then from the others.  (A single queue running through all the
// launch's passes, lanes carrying their pass, measured slower at one GPU: caustic >= 16 %.)
#ifndef BDPT_POOL
#define BDPT_POOL 0
#endif
// Pass streams with the ordered fold inside the kernel (a build with BDPT_UNITS; bdpt_host.cpp
// launches it as a 1-D grid of units, bdpt_path_args.unit_*): no radiance buffer, no fold kernel.
#ifndef BDPT_UNITS
#define BDPT_UNITS 0
#endif
// paired loads: the odd-depth copy of the paired randoms at the point of use (see the loop)
// camera terms: per-lane fp64 base in LDS, kz products formed once per workgroup

}  // namespace

#ifndef BDPT_JIT
// =============================================================================================
// Kernel 1: MT607 table (RandomGPU MersenneTwister_kernel.cu:63-110).  4096 independent twisters,
// lane-major output d_Rand[tid + k*4096].  The 19-word state lives in VGPRs: the recurrence is
// unrolled by its period so every state index is a compile-time constant (no scratch).
// =============================================================================================
template <int S>
__device__ __forceinline__ void mt_step(unsigned (&mt)[19], unsigned a, unsigned mb, unsigned mc,
                                        float* __restrict__ out, int tid, int k) {
    constexpr int S1 = (S + 1) % 19, SM = (S + 9) % 19;
    unsigned y = (mt[S] & 0xFFFFFFFEu) | (mt[S1] & 0x1u);
    y = mt[SM] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
    mt[S] = y;
    y ^= y >> 12;
    y ^= (y << 7) & mb;
    y ^= (y << 15) & mc;
    y ^= y >> 18;
    if (k < BDPT_DEV_N_PER_RNG) out[tid + k * 4096] = ((float)y + 1.0f) / 4294967296.0f;
}

// Planar copy of d_Rand for the pass-stream path kernel: a lane reads d_Rand[j .. j+4] with
// j = 26 + 25 i + 5 depth + sid, so neighbouring pixels are 25 entries apart -- in 25 planes by
// j mod 25 they are adjacent (the 32 pixels of a workgroup row share one 128-B line per plane).
// Planes 25..28 repeat planes 0..3 one entry on, so j + c (c <= 4) is plane (j mod 25) + c at
// j / 25 without a wrap.
extern "C" __global__ __launch_bounds__(256) void bdpt_rand_planar_kernel(const float* __restrict__ rnd,
                                                                        float* __restrict__ rndp) {
    const unsigned o = blockIdx.x * 256u + threadIdx.x;
    if (o >= BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL) return;
    const unsigned p = o / BDPT_DEV_RANDP_PL, q = o - p * BDPT_DEV_RANDP_PL;
    const unsigned src = p < 25u ? 25u * q + p : 25u * (q + 1u) + (p - 25u);
    rndp[o] = src < BDPT_DEV_RAND_N ? rnd[src] : 0.f;
}

// {sinf, cosf}(2 pi u) for every entry u of the planar copy (BDPT_SCP): the path kernel's own
// sincos_cr on the same float argument 2.f * kPi * u, with the 512-entry table (bdpt_math.h), so
// each stored pair is what the path kernel would compute for that entry (a build with the
// 256-entry BDPT_SC_COARSE table computes the same pair: both are the correctly rounded values,
// checked for every float argument by tests/test_math.py).  7.7 M evaluations per table, once per
// bdpt_generate_rand.
extern "C" __global__ __launch_bounds__(256) void bdpt_sincos_planar_kernel(const float* __restrict__ rndp,
                                                                          float2* __restrict__ scp) {
    __shared__ double sct[BDPT_SC_N];
    for (int q = threadIdx.x; q < BDPT_SC_N; q += 256) sct[q] = bdpt_sincos_table_dev[q][0];
    __syncthreads();
    const unsigned o = blockIdx.x * 256u + threadIdx.x;
    if (o >= BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL) return;
    const float x = 2.f * kPi * rndp[o];
    float s, c;
    sincos_cr<true>(x, &s, &c, sct);
    scp[o] = make_float2(s, c);
}

template <int... S>
__device__ __forceinline__ void mt_round(unsigned (&mt)[19], unsigned a, unsigned mb, unsigned mc,
                                         float* __restrict__ out, int tid, int k0,
                                         std::integer_sequence<int, S...>) {
    (mt_step<S>(mt, a, mb, mc, out, tid, k0 + S), ...);
}

extern "C" __global__ __launch_bounds__(64) void bdpt_mt607_kernel(const uint4* __restrict__ params,
                                                                   unsigned seed,
                                                                   float* __restrict__ out) {
    const int tid = blockIdx.x * 64 + threadIdx.x;
    const uint4 p = params[tid];
    unsigned mt[19];
    mt[0] = seed;
#pragma unroll
    for (int s = 1; s < 19; s++) mt[s] = 1812433253u * (mt[s - 1] ^ (mt[s - 1] >> 30)) + (unsigned)s;
    for (int k0 = 0; k0 < BDPT_DEV_N_PER_RNG; k0 += 19)
        mt_round(mt, p.x, p.y, p.z, out, tid, k0, std::make_integer_sequence<int, 19>{});
}

// =============================================================================================
// Kernel 2: light pass -- GetRayKernel (device.cu:167-219) + RadianceLightTracingKernel
// (device.cu:222-455, DEPTH = 1) for every emitter in sphere order, fused: each thread owns
// VLP `ind` and applies the lights in the order the reference launches them (smallpt_cpu.c:311).
// =============================================================================================
extern "C" __global__ __launch_bounds__(64) void bdpt_light_kernel(const bdpt_dev_sphere* __restrict__ sph,
                                                                   unsigned n,
                                                                   const float* __restrict__ rnd,
                                                                   int current_sample,
                                                                   bdpt_dev_lightpath* __restrict__ lp) {
    const int ind = blockIdx.x * 64 + threadIdx.x;
    bdpt_dev_lightpath out = lp[ind];
    for (unsigned li = 0; li < n; li++) {
        const bdpt_dev_sphere L = sph[li];
        const f3 Le = mk(L.ex, L.ey, L.ez), Lp = mk(L.px, L.py, L.pz);
        if (iszero3(Le)) continue;
        // GetRayKernel, seed_id = 0
        const unsigned i = (unsigned)(current_sample * 5 + ind * 4) % (kRandN - 4u);
        const unsigned j = i + 2;
        const f3 usp = uniform_sphere(rnd[j], rnd[i]);
        const f3 spt = add(smul(L.rad, usp), Lp);
        const f3 normal = norm(sub(spt, Lp));
        const f3 ro = spt;
        const f3 rd = cosine_dir(normal, rnd[i + 1], rnd[j + 1]);
        // RadianceLightTracingKernel
        f3 thr = smul(0.25f, Le);
        float t = 1e20f;
        int id = -1;
        for (int s = (int)n - 1; s >= 0; --s) {
            const bdpt_dev_sphere& S = sph[s];
            const float d = sphere_isect(make_float4(S.px, S.py, S.pz, S.rr), ro, rd);
            if (d != 0.f && d < t) { t = d; id = s; }
        }
        if (id < 0) {                                               // escaped (:279-292)
            const f3 nor = smul((float)(-1. / (double)L.rad), sub(ro, Lp));
            const f3 hr = smul(0.5f, Le);
            out.hx = ro.x; out.hy = ro.y; out.hz = ro.z;
            out.rx = hr.x; out.ry = hr.y; out.rz = hr.z;
            out.nx = nor.x; out.ny = nor.y; out.nz = nor.z;
            continue;
        }
        const bdpt_dev_sphere O = sph[id];
        if (!iszero3(mk(O.ex, O.ey, O.ez))) continue;              // :296-298
        const f3 hit = add(ro, smul(t, rd));
        const f3 nrm = norm(sub(hit, mk(O.px, O.py, O.pz)));
        const float dp = dot(nrm, rd);
        const f3 nl = smul(-1.f * (float)(dp > 0 ? 1 : -1), nrm);
        if (O.refl == BDPT_DEV_DIFF) {                              // VecMultiply :10-42, store :330-337
            const float tol = (float)0.0001;
            float tt;
            if (thr.x != 0.f && O.cx != 0.f) { tt = thr.x * O.cx; if (!(tt <= tol || thr.x == tt)) thr.x = tt; } else thr.x = 0.f;
            if (thr.y != 0.f && O.cy != 0.f) { tt = thr.y * O.cy; if (!(tt <= tol || thr.y == tt)) thr.y = tt; } else thr.y = 0.f;
            if (thr.z != 0.f && O.cz != 0.f) { tt = thr.z * O.cz; if (!(tt <= tol || thr.z == tt)) thr.z = tt; } else thr.z = 0.f;
            out.hx = hit.x; out.hy = hit.y; out.hz = hit.z;
            out.rx = thr.x; out.ry = thr.y; out.rz = thr.z;
            out.nx = nl.x; out.ny = nl.y; out.nz = nl.z;
        }
    }
    lp[ind] = out;
}

#endif  // BDPT_JIT

// =============================================================================================
// Kernel 3: the eye-path integrator (RadiancePathTracingKernel device.cu:544-791), `npass`
// passes fused into one launch.
//
//  * One lane = one pixel for the whole launch; the running mean (c*k1 + r)*k2 and the counter
//    stay in VGPRs across passes and are written once, coalesced, at the end (36 B/pixel/launch).
//  * Path regeneration: one loop iteration = one path segment for every live lane; a lane whose
//    path ends accumulates and starts its next pass in the next iteration, so lanes never idle
//    waiting for the longest path of the wave (the reference's 1-spp launch idles them).
//  * Shadow-ray compaction: the NEE and VLP shadow rays of the wave's diffuse vertices
//    (SampleLightsDevice :457-542) are pushed into a per-wave LDS queue at positions given by a
//    ballot + mbcnt prefix count, then traced by all 64 lanes in a wave-uniform pass (1 pass for
//    <= 64 rays, 2 for <= 128) instead of two half-empty divergent loops.  The main loop is
//    wave-uniform (lanes with no work left still serve the queue).
//  * Sphere geometry {p, rad^2}: for N = 1..16 spheres (template) it is read through wave-uniform
//    scalar loads and every traversal loop is fully unrolled; otherwise (N = 0) it is staged in
//    LDS.  Emission / colour / material / centre for the per-lane hit id, the per-pass sid and
//    VLP (dev_lp[vlp_index]) and the camera constants are LDS tables.
//  * The 5 random numbers a segment may consume (d_Rand[j..j+4], j = (26+25i+5*depth+sid) mod
//    (RAND_N-5), device.cu:619) are prefetched one segment ahead.
//  * 256-thread workgroup = 32x8 pixel tile as 4x1 waves of 8x8 pixels; blockIdx.z = pass
//    stream when the launch has fewer pixels than the chip has lanes (multi-GPU shards).
// =============================================================================================
namespace {
constexpr int kQueue = 128;                       // shadow rays per wave and step (<= 2 per lane)

__device__ __forceinline__ int lane_prefix(unsigned long long mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}
// Read-only scene data through the constant address space: wave-uniform indices become scalar
// loads (s_load, scalar cache) that never wait on the vector-memory counter, so the in-flight RNG
// prefetch is not drained by the traversal loops (a plain global load here costs a vmcnt(0)).
__device__ __forceinline__ float4 ld_const(const float4* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const float cfloat;
    const cfloat* q = (const cfloat*)(p + i);
    return make_float4(q[0], q[1], q[2], q[3]);
#else
    return p[i];
#endif
}

// d_Rand[j .. j+4] (device.cu:619): five dword loads, or (BDPT_RAND_X4) one dwordx4 + one dword
// through a 4-byte-aligned vector type.  BDPT_ABL_RNG (ablation, changes results): no loads,
// a hash of j instead -- the cost of the table reads.
__device__ __forceinline__ void load_rand5(const float* __restrict__ rnd, unsigned j, float& q0,
                                           float& q1, float& q2, float& q3, float& q4) {
    q0 = rnd[j]; q1 = rnd[j + 1]; q2 = rnd[j + 2]; q3 = rnd[j + 3]; q4 = rnd[j + 4];
}

// The same five entries through a buffer descriptor with one 32-bit offset register (the fused
// kernel): no 64-bit address temporaries, which the register allocator otherwise
// took from registers a pending load writes -- and then waited for that load right after issuing it.
__device__ __forceinline__ void load_rand5b(__amdgpu_buffer_rsrc_t rs, unsigned j, float& q0,
                                            float& q1, float& q2, float& q3, float& q4) {
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const unsigned vo = j * 4u;
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0);
    q0 = __uint_as_float(v.x); q1 = __uint_as_float(v.y); q2 = __uint_as_float(v.z); q3 = __uint_as_float(v.w);
    q4 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 16, 0));
}

// d_Rand[j .. j+4] from the planar copy: plane j mod 25 + c at j / 25, as buffer loads with the
// plane offsets c * PL in the scalar offset (one address register for all five)
__device__ __forceinline__ void load_rand5p(__amdgpu_buffer_rsrc_t rs, unsigned j, float& q0,
                                            float& q1, float& q2, float& q3, float& q4) {
    const unsigned qd = j / 25u, r = j - qd * 25u;
    const unsigned vo = (r * BDPT_DEV_RANDP_PL + qd) * 4u;
    constexpr unsigned P4 = BDPT_DEV_RANDP_PL * 4u;

    q0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
    q1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, P4, 0));
    q2 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 2 * P4, 0));
    q3 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 3 * P4, 0));
    q4 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 4 * P4, 0));
}

// BDPT_SCP: d_Rand[j .. j+3] and {sinf, cosf}(2 pi d_Rand[j]), {sinf, cosf}(2 pi d_Rand[j+4]) --
// d_Rand[j+4] itself is used only as that angle -- from the planar copies (same plane offsets)
__device__ __forceinline__ void load_rand_scp(__amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rsc,
                                              unsigned j, float& q0, float& q1, float& q2, float& q3,
                                              float& s0, float& c0, float& s4, float& c4) {
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    const unsigned qd = j / 25u, r = j - qd * 25u;
    const unsigned e = r * BDPT_DEV_RANDP_PL + qd, vo = e * 4u, vs = e * 8u;
    constexpr unsigned P4 = BDPT_DEV_RANDP_PL * 4u, P8 = BDPT_DEV_RANDP_PL * 8u;
    q0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
    q1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, P4, 0));
    q2 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 2 * P4, 0));
    q3 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 3 * P4, 0));
    const u2v a = __builtin_amdgcn_raw_buffer_load_b64(rsc, vs, 0, 0);
    const u2v b = __builtin_amdgcn_raw_buffer_load_b64(rsc, vs, 4 * P8, 0);
    s0 = __uint_as_float(a.x); c0 = __uint_as_float(a.y);
    s4 = __uint_as_float(b.x); c4 = __uint_as_float(b.y);
}

// the two parts of load_rand_scp on their own (BDPT_SCP_LATE)
__device__ __forceinline__ void load_rand4p(__amdgpu_buffer_rsrc_t rs, unsigned j, float& q0, float& q1,
                                            float& q2, float& q3) {
    const unsigned qd = j / 25u, r = j - qd * 25u;
    const unsigned vo = (r * BDPT_DEV_RANDP_PL + qd) * 4u;
    constexpr unsigned P4 = BDPT_DEV_RANDP_PL * 4u;
    q0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
    q1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, P4, 0));
    q2 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 2 * P4, 0));
    q3 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 3 * P4, 0));
}
__device__ __forceinline__ void load_sc(__amdgpu_buffer_rsrc_t rsc, unsigned j, float& s0, float& c0,
                                        float& s4, float& c4) {
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    const unsigned qd = j / 25u, r = j - qd * 25u;
    const unsigned vs = (r * BDPT_DEV_RANDP_PL + qd) * 8u;
    constexpr unsigned P8 = BDPT_DEV_RANDP_PL * 8u;
    const u2v a = __builtin_amdgcn_raw_buffer_load_b64(rsc, vs, 0, 0);
    const u2v b = __builtin_amdgcn_raw_buffer_load_b64(rsc, vs, 4 * P8, 0);
    s0 = __uint_as_float(a.x); c0 = __uint_as_float(a.y);
    s4 = __uint_as_float(b.x); c4 = __uint_as_float(b.y);
}

// f(S), f(S-1), ..., f(0) with compile-time indices while f returns true
template <int S, typename F>
__device__ __forceinline__ void unroll_down(F& f) {
    if constexpr (S >= 0) {
        if (f(S)) unroll_down<S - 1>(f);
    }
}

// Handover between the units of a tile (BDPT_UNITS): agent-scope relaxed atomics are coherent
// across XCDs (sc1 loads / stores on gfx950, no L2 invalidation); the producer waits for its data
// stores (s_waitcnt vmcnt(0)) before it stores the flag.  Every value handed over (colours,
// counter, flag) is such an atomic, so no cache maintenance is needed; the C++-model form of the
// same ordering (BDPT_UNITS_FENCE=1: an agent-scope release fence before the flag store and an
// acquire fence after the flag load) compiles to buffer_wbl2 sc1 / buffer_inv sc1 -- a write-back
// and an invalidation of the XCD's whole L2 per unit -- and is kept as a measured variant only
// ("Units").
#ifndef BDPT_UNITS_FENCE
#define BDPT_UNITS_FENCE 0
#endif
__device__ __forceinline__ float ld_coherent(float* p) {
    return __uint_as_float(__hip_atomic_load((unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_coherent(float* p, float v) {
    __hip_atomic_store((unsigned*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait until *f == want.  The unit that sets it was claimed earlier from the same queue, by a
// workgroup that is running (or done); the bound (~1.3 s) turns a broken assumption into an error
// report (*err) instead of a hang.
__device__ __forceinline__ void unit_wait(unsigned* f, unsigned want, unsigned* err) {
    for (unsigned spins = 0;; spins++) {
        const unsigned v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (v == want) break;
        if (spins > (1u << 22)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(10);
    }
#if BDPT_UNITS_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#else
    asm volatile("" ::: "memory");
#endif
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---- BVH traversal (large scenes; tree built by bdpt_bvh.cpp) --------------------------------
// Exactness: a box may be skipped only if no sphere in it can produce a float hit that changes
// the answer.  For the reference's float test t^ = fl(b -+ sqrt(det)) (SphereIntersectDevice),
// with g(t) = |o + t d - p|^2 - r^2 on the same float inputs, expanding g(t^) around the float
// det gives |g(t^)| <= ~50u D^2 (u = 2^-24; det rounding, sqrt rounding, the b error times
// sqrt(det), and |d|^2 - 1 = O(u) from the float vnorm), D >= |op| + r.  So every float hit
// point -- also on an exactly-missed sphere -- lies within 25u D^2 / r of its sphere, hence of
// its box.  Boxes are widened by m = D*(kBvhK + q*D), q = 64u / (smallest BVH radius) (2.6x
// that bound) and kBvhK = 1e-4 (covers the slab test's own ~6u*D rounding ~270x), with
// D = |o - c_root| + r_root; a box is skipped only if entered beyond tmax + m or left before
// -m.  tests/test_bvh_margin.py measures the gap on worst-case rays against m/2.
#ifndef BDPT_BVH_K
#define BDPT_BVH_K 1e-4f
#endif
constexpr float kBvhK = BDPT_BVH_K;
constexpr int kBvhEmissive = BDPT_DEV_BVH_EMISSIVE;
constexpr int kBvhIdMask = BDPT_DEV_BVH_EMISSIVE - 1;

struct bvh_ray {
    f3 olo, ohi, inv;
    float m;
};

__device__ __forceinline__ bvh_ray bvh_setup(const bdpt_path_args& a, f3 o, f3 d) {
    const f3 dc = sub(o, mk(a.bvh_c[0], a.bvh_c[1], a.bvh_c[2]));
    const float D = __builtin_amdgcn_sqrtf(dot(dc, dc) * 1.00001f) * 1.00001f + a.bvh_r;
    bvh_ray r;
    r.m = D * (kBvhK + a.bvh_q * D);
    r.olo = mk(o.x + r.m, o.y + r.m, o.z + r.m);    // lo - (o + m) = (lo - m) - o
    r.ohi = mk(o.x - r.m, o.y - r.m, o.z - r.m);    // hi - (o - m) = (hi + m) - o
    const float e = 1e-20f;
    r.inv = mk(1.f / (fabsf(d.x) > e ? d.x : copysignf(e, d.x)),
               1.f / (fabsf(d.y) > e ? d.y : copysignf(e, d.y)),
               1.f / (fabsf(d.z) > e ? d.z : copysignf(e, d.z)));
    return r;
}

__device__ __forceinline__ bool bvh_box(float4 lo, float4 hi, const bvh_ray& r, float tmax) {
    const float x0 = (lo.x - r.olo.x) * r.inv.x, x1 = (hi.x - r.ohi.x) * r.inv.x;
    const float y0 = (lo.y - r.olo.y) * r.inv.y, y1 = (hi.y - r.ohi.y) * r.inv.y;
    const float z0 = (lo.z - r.olo.z) * r.inv.z, z1 = (hi.z - r.ohi.z) * r.inv.z;
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return tn <= tf && tf >= -r.m && tn <= tmax + r.m;
}
}  // namespace

#ifdef BDPT_STATS
// instrumentation builds only (make variant NAME=stats EXTRA_HIPFLAGS=-DBDPT_STATS; read by
// scripts/shadow_stats.py): [0] shadow steps, [1] shadow rounds, [2] shadow rays, [3] diffuse
// lanes at shadow steps, [4] wave segments, [5] alive lanes at segment starts
__device__ unsigned long long bdpt_dev_stats[8];
extern "C" int bdpt_debug_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bdpt_dev_stats), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(bdpt_dev_stats), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#ifndef BDPT_WAVES_PER_SIMD
#define BDPT_WAVES_PER_SIMD 5
#endif
// (the specialised build is compiled with -DBDPT_WAVES_PER_SIMD=6: folding the scene in frees
// registers, and 6 waves/SIMD measured +3 % over 5 on cornell)
// BVH scenes: 5 waves/SIMD too, although the traversal state spills 10 VGPRs at 96 (measured:
// 4 waves +0 spills is 10-12 % slower, 6 waves spills 27).
#ifndef BDPT_BVH_WAVES
#define BDPT_BVH_WAVES 5
#endif
// The fused S = 1 kernel keeps the running mean and the counter in registers too (4 more live
// values): at 6 waves/SIMD it would spill, so it is bounded at 5 (it is the non-default mode).
#ifndef BDPT_FUSED_WAVES
#define BDPT_FUSED_WAVES (BDPT_WAVES_PER_SIMD < 5 ? BDPT_WAVES_PER_SIMD : 5)
#endif
template <int N, bool STREAMS>
__global__ __launch_bounds__(256, N < 0 ? BDPT_BVH_WAVES : (STREAMS ? BDPT_WAVES_PER_SIMD : BDPT_FUSED_WAVES))
void bdpt_path_kernel_t(bdpt_path_args a) {
    extern __shared__ float4 smem[];
    constexpr bool kBVH = N < 0;      // large scene: walls brute force + BVH (bdpt_bvh.cpp)
    const int n = N > 0 ? N : (int)a.n;
    constexpr int kUnroll = N > 0 ? N : 1;
    constexpr bool kTreeLds = false;  // tree read through L1/L2: 4 workgroups per CU (+10 %)
    const int ntree = kTreeLds ? 2 * a.bvh_nn + a.bvh_ns : 0;
    const int ntab = kBVH ? ntree + a.big_n : 4 * n + a.n_vac;      // (bdpt_host.cpp tab)
    // pass stream: this workgroup's lanes render passes s0, s0+S, s0+2S, ... (slots k = 0, 1, ...)
    // of their pixels (S == 1: all, and each lane keeps the running mean itself; S > 1: radiance
    // goes to rbuf, bdpt_accum_kernel folds it in pass order).  Only the slots' VLPs and sids are
    // staged in LDS (one pass per workgroup with the default S = npass; bdpt_host.cpp sizes it).
    constexpr bool kPool = STREAMS && BDPT_POOL;
    // pixel pools: a 1-D grid with the passes interleaved, so every pass has workgroups from the
    // launch's start to its end and the passes finish together (z-major, the last passes ran at
    // the end on their own workgroups); pass (b / 8) mod S keeps each pass on all 8 XCDs
    // ordered in-kernel fold (BDPT_UNITS builds): a 1-D grid of units (tile, range) in range-major
    // order; a lane renders the range's passes of its pixel in order and keeps the running mean in
    // registers, and the units of a tile follow each other through per-wave-tile flags
    constexpr bool kUnits = STREAMS && BDPT_UNITS && !BDPT_POOL;
    // A workgroup claims its unit from the queue of its XCD (tiles t = xcd mod 8, range-major), or
    // steals from the next queues; so a unit's predecessor (same tile, previous range, same queue)
    // was claimed earlier by a running workgroup, whatever order the hardware dispatches in.  The
    // grid has exactly one workgroup per unit.
    unsigned urange = 0u;
    int vtile = 0;
    if constexpr (kUnits) {
        __shared__ unsigned uclaim[2];
        if (threadIdx.x == 0) {
            const unsigned wgs = (unsigned)a.unit_wgs, nr = (unsigned)bdpt_unit_ranges(a.npass, a.unit_passes, a.unit_taper);
            const unsigned xcd = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;   // XCC_ID
            uclaim[0] = 0xffffffffu;
            for (unsigned k = 0; k < 8u; k++) {
                const unsigned q = (xcd + k) & 7u;
                const unsigned ntq = wgs > q ? (wgs - q + 7u) / 8u : 0u;      // tiles of queue q
                if (ntq == 0u) continue;
                const unsigned u = atomicAdd(a.unit_ctr + q * 32u, 1u);
                if (u < ntq * nr) {
                    uclaim[0] = u / ntq;                                       // range
                    uclaim[1] = q + 8u * (u - (u / ntq) * ntq);                // tile
                    break;
                }
            }
        }
        __syncthreads();
        urange = uclaim[0];
        vtile = (int)uclaim[1];
        if (urange == 0xffffffffu) return;                                     // (cannot happen)
    }
    // the workgroup's tile (vbx, vby) in the tile grid (vgx, vgy)
    const int vbx = kUnits ? vtile % a.gx : (int)blockIdx.x, vby = kUnits ? vtile / a.gx : (int)blockIdx.y;
    const int vgx = kUnits ? a.gx : (int)gridDim.x, vgy = kUnits ? a.gy : (int)gridDim.y;
    const int S = kUnits ? 1 : (STREAMS ? a.streams : 1);
    int ulen = 0;
    const int s0 = kUnits ? bdpt_unit_range(a.npass, a.unit_passes, a.unit_taper, (int)urange, &ulen)
                 : !STREAMS ? 0 : kPool ? (int)((blockIdx.x >> 3) % (unsigned)S) : (int)blockIdx.z;
    const int nslot = kUnits ? ulen : (a.npass - s0 + S - 1) / S;
    const int mslot = kUnits ? a.unit_passes : (a.npass + S - 1) / S;   // slots of the LDS layout (any s0)
    float4* C = smem;                 // {cx, cy, cz, bits(refl | emissive<<8)}
    float4* E = smem + n;             // {ex, ey, ez, rad}
    float4* P = smem + 2 * n;         // {px, py, pz, 0}  (hit normal)
    float4* G = smem + 3 * n;         // {px, py, pz, rad^2}  (N == 0 traversal)
    float4* GV = smem + 4 * n;        // the same for the non-emitters only (VLP-only shadow rounds)
    float4* ND = smem;                // BVH: nodes (2 float4 each)
    float4* SG = ND + 2 * a.bvh_nn;   // BVH: sphere geometry in leaf order
    float4* BG = smem + ntree;        // BVH: brute-force (wall) geometry
    float4* V = smem + ntab;          // per slot: VLP {hx,hy,hz,rx}{ry,rz,nx,ny}{nz,-,-,-}
    float4* K = V + 3 * mslot;        // camera constants (5 float4)
    float4* Q = K + 5;                // shadow queues: 4 waves x kQueue x 2 float4
    // (a ray's occlusion bit is written over its maxt, SQ[idx].w, once the ray is traced)
    unsigned* SID = (unsigned*)(Q + 4 * kQueue * 2);   // per slot sid
    int* SI = (int*)(SID + mslot);    // BVH: sphere ids (| emissive flag), leaf order
    int* BI = SI + (kTreeLds ? a.bvh_ns : 0);   // BVH: wall ids
    const float4* __restrict__ NDt = kTreeLds ? (const float4*)ND : a.bvh_nodes;
    const float4* __restrict__ SGt = kTreeLds ? (const float4*)SG : a.bvh_geom;
    const int* __restrict__ SIt = kTreeLds ? (const int*)SI : a.bvh_ids;
    if constexpr (kBVH) {
        if constexpr (kTreeLds) {
            for (int q = threadIdx.x; q < 2 * a.bvh_nn; q += 256) ND[q] = a.bvh_nodes[q];
            for (int q = threadIdx.x; q < a.bvh_ns; q += 256) {
                SG[q] = a.bvh_geom[q];
                SI[q] = a.bvh_ids[q];
            }
        }
        for (int q = threadIdx.x; q < a.big_n; q += 256) {
            BG[q] = a.big_geom[q];
            BI[q] = a.big_ids[q];
        }
    } else {
        for (int s = threadIdx.x; s < n; s += 256) {
            const bdpt_dev_sphere S = a.sph[s];
            const bool emis = !(S.ex == 0.f && S.ey == 0.f && S.ez == 0.f);
            // bit 8: emitter; bit 9: black non-emitter (c = 0: a hit zeroes the throughput)
            const bool black = !emis && S.cx == 0.f && S.cy == 0.f && S.cz == 0.f;
            C[s] = make_float4(S.cx, S.cy, S.cz, __int_as_float(S.refl | (emis ? 256 : 0) | (black ? 512 : 0)));
            E[s] = make_float4(S.ex, S.ey, S.ez, S.rad);
            P[s] = make_float4(S.px, S.py, S.pz, 0.f);
            G[s] = make_float4(S.px, S.py, S.pz, S.rr);
        }
        if constexpr (BDPT_VAC_LIST && !kPool)
            for (int s = threadIdx.x; s < a.n_vac; s += 256) GV[s] = a.vgeom[s];
    }
    // pixel pools: a workgroup whose pass was drained before it started ends at once (a launch
    // has many more workgroups than fit, and the late ones of a pass find it drained): threads
    // 0..7 read the pass's 8 claim counters in parallel (the claim would try them one after
    // another); the pass is drained when every part is.  caustic +0.3 %, its 1/8 share +1.3 %
    // (profiles/r05_s33_pool_early_exit.txt); a "drained" bitmap instead -- one word for 32
    // passes, set by every wave whose claim failed -- was a contended hot spot (-30 %,
    // r05_s32_pool_skip_bitmap.txt).
    __shared__ unsigned pool_left;
    if constexpr (kPool) {
        // the next pooled launch's counters (the previous launch used them and has finished);
        // before the early exit, so every workgroup does its share.  (Overlapped launches: none,
        // the host clears each launch's set on its stream.)
        if (a.pool_ctr_next)
            for (unsigned w = blockIdx.x * 256u + threadIdx.x; w < 128u * 8u; w += gridDim.x * 256u)
                a.pool_ctr_next[w * 32u] = 0u;
    }
    if (kPool && threadIdx.x == 0) pool_left = 0u;
    __syncthreads();
    if (kPool && threadIdx.x < 8u) {
        const unsigned nl = (unsigned)a.nloc, pt = threadIdx.x;
        const unsigned p0 = (unsigned)(((unsigned long long)nl * pt) >> 3);
        const unsigned p1 = (unsigned)(((unsigned long long)nl * (pt + 1u)) >> 3);
        const unsigned used = __hip_atomic_load(a.pool_ctr + ((unsigned)s0 * 8u + pt) * 32u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        if (p0 + used < p1) atomicOr(&pool_left, 1u);                // LDS
    }
    for (int q = threadIdx.x; q < nslot; q += 256) {
        const int pq = s0 + q * S;
        const bool inl = a.sid == nullptr;                                // uniform
        const int vq = inl ? a.vlp_inl[pq & (BDPT_DEV_INLINE_PASSES - 1)] : a.vlp[pq];
        const bdpt_dev_lightpath L = a.lp[vq & (BDPT_DEV_LIGHT_POINTS - 1)];
        V[3 * q + 0] = make_float4(L.hx, L.hy, L.hz, L.rx);
        V[3 * q + 1] = make_float4(L.ry, L.rz, L.nx, L.ny);
        V[3 * q + 2] = make_float4(L.nz, 0.f, 0.f, 0.f);
        SID[q] = inl ? a.sid_inl[pq & (BDPT_DEV_INLINE_PASSES - 1)] : a.sid[pq];
    }
    if (threadIdx.x == 0) {
        K[0] = make_float4(a.ux[0], a.ux[1], a.ux[2], a.tx);
        K[1] = make_float4(a.uy[0], a.uy[1], a.uy[2], a.ty);
        // kz * ud and tz * kz (kz = 10, device.cu:583-590): the same products, formed once
        K[2] = make_float4(10.0f * a.ud[0], 10.0f * a.ud[1], 10.0f * a.ud[2], a.tz * 10.0f);
        K[3] = make_float4(a.orig[0], a.orig[1], a.orig[2], 0.f);
        K[4] = make_float4(a.inv_w, a.inv_h, 0.f, 0.f);
    }
    // sin(2pi k/N) for the table-driven sincos (bdpt_math.h; cos is entry k + N/4), 4 KB (2 KB
    // with BDPT_SC_COARSE: every other entry)
    // (not with BDPT_SCP: the pass-stream kernels load precomputed pairs -- except the pixel-pool
    // build, whose restarted lanes are bound by their random-table gathers: the two extra gathers
    // per segment cost caustic8 2.5 %, one-session A/B profiles/r06_s8_ab_scp_caustic8.txt)
    constexpr bool kScp = STREAMS && BDPT_SCP && !BDPT_POOL;
    constexpr int kSct = BDPT_SC_N >> BDPT_SC_COARSE;
    const double* SCT = nullptr;
    if constexpr (!kScp) {
        __shared__ double sct[kSct];
        static_assert(kSct % 256 == 0, "table fill");
#pragma unroll
        for (int q = 0; q < kSct; q += 256)
            sct[q + threadIdx.x] = bdpt_sincos_table_dev[(q + threadIdx.x) << BDPT_SC_COARSE][0];
        SCT = sct;
    }
    __syncthreads();
    if (kPool && pool_left == 0u) return;                // uniform: the whole workgroup ends

    auto geom = [&](int s) -> float4 {
#ifdef BDPT_JIT
        if constexpr (N == BDPT_JIT_N) {                        // the scene, folded in
            const jit_geom g = kJitGeom[s];
            return make_float4(g.x, g.y, g.z, g.w);
        }
#endif
        if constexpr (N > 0) return ld_const(a.geom, s); else return G[s];
    };
    auto emissive = [&](int s) -> bool {
#ifdef BDPT_JIT
        if constexpr (N == BDPT_JIT_N) return (kJitEmis >> s) & 1ull;
#endif
        if constexpr (N > 0) return (a.emis_mask >> s) & 1u;
        else return (__float_as_int(C[s].w) & 256) != 0;
    };
    // spheres worth a wave-uniform det test: non-walls of a specialised kernel
    auto small_sphere = [&](int s) -> bool {
#ifdef BDPT_JIT
        if constexpr (N == BDPT_JIT_N) return kJitGeom[s].w < 1e6f;
#endif
        (void)s;
        return false;
    };
    // per-lane hit data: LDS tables, or (BVH scenes, too large for LDS) the global copy
    auto tabC = [&](int s) -> float4 { if constexpr (kBVH) return a.mat[3 * s]; else return C[s]; };
    auto tabE = [&](int s) -> float4 { if constexpr (kBVH) return a.mat[3 * s + 1]; else return E[s]; };
    auto tabP = [&](int s) -> float4 { if constexpr (kBVH) return a.mat[3 * s + 2]; else return P[s]; };

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#ifdef BDPT_PROF
    // section profile (experiments): shader cycles per wave between wave-uniform points, summed
    // per section and added to a.prof by lane 0 at the end (s_memtime waits on lgkmcnt, so the
    // profile perturbs LDS overlap a little)
    unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = __builtin_amdgcn_s_memtime();
#define BDPT_TICK(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pacc[k] += t_ - pt; pt = t_; } while (0)
#else
#define BDPT_TICK(k) do { } while (0)
#endif
#ifdef BDPT_COUNTS
    // region counts (experiments; tools/valu_attrib.py): how often the wave executes each region
    // (the region's condition holds for some lane).  The first active lane counts (inside
    // divergent code a per-lane counter of a fixed lane would miss the events it sits out); the
    // lanes' counts are summed at the end and added to a.prof[0..kCnt).
    constexpr int kCnt = 24;
    unsigned pcnt[kCnt] = {};
    auto first_lane = [&]() { return lane == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true)); };
#define BDPT_CNT(k, cond) do { if (__builtin_amdgcn_ballot_w64(cond) != 0 && first_lane()) pcnt[k]++; } while (0)
#define BDPT_CNTN(k, n) do { const unsigned n_ = (n); if (first_lane()) pcnt[k] += n_; } while (0)
#else
#define BDPT_CNT(k, cond) do { } while (0)
#define BDPT_CNTN(k, n) do { } while (0)
#endif
    int x = vbx * BDPT_BTW + (wave % BDPT_BLOCK_WX) * BDPT_WTW + (lane % BDPT_WTW);
    int ly = vby * BDPT_BTH + (wave / BDPT_BLOCK_WX) * BDPT_WTH + (lane / BDPT_WTW);
    // Frame edges packed into full waves (rows not remapped to shard bands): a frame whose width
    // leaves tw <= 8 columns in the last workgroup column (1921 = 60 x 32 + 1) would give every
    // tile row one wave with tw x 8 live lanes that still runs whole paths; instead those tw x H
    // pixels are dealt out y-major, 256 per workgroup of that column, and likewise the th < 8
    // rows of the last workgroup row (x below the last column, row-major) to the workgroups of
    // that row.  Every pixel is still rendered by exactly one lane.
    if (a.tiles_per_band <= 0) {
        const int gx = vgx, gy = vgy;
        const int xt = (gx - 1) * BDPT_BTW, yt = (gy - 1) * BDPT_BTH;
        const int tw = a.W - xt, th = a.H - yt, wl = (int)threadIdx.x;
        if (tw <= BDPT_WTW && vbx == gx - 1) {
            const int q = vby * 256 + wl;
            x = xt + q % tw;
            ly = q / tw;
        } else if (th < BDPT_BTH && vbx < gx - 1 && vby == gy - 1) {
            const int q = vbx * 256 + wl;
            x = q % xt;
            ly = yt + q / xt;
        }
    }
    const int yoff = (bdpt_dev_tile_row(a, vby) - vby) * BDPT_BTH;   // uniform
    int y = ly + yoff;
    bool active = x < a.W && y < a.H;
    if (active && a.nshards > 1) active = ((y / a.band_rows) % a.nshards) == a.shard;
    // pixel pools: this wave's chunk is [.., pend) of the launch's row-major pixels (local rows:
    // grid row r of the tile grid is tile row bdpt_dev_tile_row(r)), pcur its next unused pixel,
    // lix = the lane's pixel
    unsigned lix = 0, pcur = 0, pend = 0;
    bool drained = false;                              // the pass's pixels are all claimed
    unsigned part = 0, tries = 0;                      // the part claimed from, parts found empty
    if constexpr (kPool) part = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;   // XCC_ID
    auto claim = [&]() -> bool {                       // the next chunk of this wave's pass (uniform)
        const unsigned span = 64u * (unsigned)(a.pool > 1 ? a.pool : 1), nl = (unsigned)a.nloc;   // >= 64: claims advance
        while (tries < 8u) {
            const unsigned p0 = (unsigned)(((unsigned long long)nl * part) >> 3);
            const unsigned p1 = (unsigned)(((unsigned long long)nl * (part + 1u)) >> 3);
            unsigned b = 0;
            if (lane == 0) b = atomicAdd(a.pool_ctr + ((unsigned)s0 * 8u + part) * 32u, span);
            b = p0 + __builtin_amdgcn_readlane(b, 0);
            if (b < p1) {
                pcur = b;
                pend = b + span < p1 ? b + span : p1;
                return true;
            }
            part = (part + 1u) & 7u;
            tries++;
        }
        drained = true;
        return false;
    };
    auto pool_pixel = [&](unsigned q, int& px, int& py) -> bool {
        if (q >= pend) return false;
        // q / W through the fp32 reciprocal (q < 2^28, W < 2^16: the estimate is off by at most
        // one row) and one correction, instead of an integer division
        int lr = (int)((float)q * __builtin_amdgcn_rcpf((float)a.W));
        px = (int)q - lr * a.W;
        if (px < 0) { lr--; px += a.W; } else if (px >= a.W) { lr++; px -= a.W; }
        py = bdpt_dev_tile_row(a, lr / BDPT_BTH) * BDPT_BTH + lr % BDPT_BTH;
        if (py >= a.H) return false;
        return a.nshards <= 1 || a.tiles_per_band > 0 || ((py / a.band_rows) % a.nshards) == a.shard;
    };
    if constexpr (kPool) {
        active = claim();
        lix = pcur + (unsigned)lane;
        pcur += 64u;
        if (active) active = pool_pixel(lix, x, y);
    }
    // Pass p = s0 + k*S (slot k) is rendered iff counter0 + p < 30000 (one increment per pass).
    float4* SQ = Q + wave * kQueue * 2;

    // this lane's camera terms ((double)((float)x * iw) - iw*W/2., same for y) of device.cu:565-566,
    // formed once per launch instead of once per pass
    __shared__ double2 camb[256];
    camb[threadIdx.x] = make_double2((double)((float)x * a.inv_w) - a.half_w,
                                     (double)((float)y * a.inv_h) - a.half_h);
    const int i = active ? y * a.W + x : 0;
    const unsigned ibase = 26u + (unsigned)(i * 25);
    // The pixel coordinates live in one packed register (W, H < 2^16, bdpt_create) and are
    // unpacked where they are used, behind an empty asm the compiler cannot look through: left
    // to itself it hoists (float)x, (float)y and the 64-bit pass-stream store address out of the
    // path loop and then spills them at the 80-VGPR (6 waves/SIMD) bound.
    unsigned xy = ((unsigned)y << 16) | (unsigned)x;
    const float* __restrict__ rnd = a.rnd;
    constexpr unsigned M5 = kRandN - 5u;

    f3 col = mk(0.f, 0.f, 0.f);
    unsigned cnt0 = 0;                // the counter before pass p is cnt0 + p
    // (units: the counter before the unit's slot k is cnt0 + k)
    const unsigned uflag = kUnits ? (unsigned)vtile * 4u + (unsigned)wave : 0u;   // this wave's 8x8 tile
    if constexpr (kUnits) {
        // the previous range of this tile has folded its passes (it was claimed a queue's worth of
        // units earlier: a short wait or none); colours and counter are read at the coherence point
        // (agent-scope relaxed atomics: a stolen unit may have run on another XCD, whose L2 is not ours)
        if (urange > 0) unit_wait(a.unit_flags + uflag, a.unit_tag | urange, a.unit_err);
        if (active) {
            col.x = ld_coherent(&a.colors[i].x);
            col.y = ld_coherent(&a.colors[i].y);
            col.z = ld_coherent(&a.colors[i].z);
            cnt0 = __hip_atomic_load(&a.counter[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (active) {
        if constexpr (!STREAMS) {
            const bdpt_dev_vec cv = a.colors[i];
            col = mk(cv.x, cv.y, cv.z);
        }
        cnt0 = a.counter[i];
    }

    int k = 0;                        // slot: this lane renders pass s0 + k*S next
    unsigned depth = 0;
    unsigned j = (ibase + SID[k]) % M5;
    float q0, q1, q2, q3, q4 = 0.f;
    // one pass per lane (pass streams, S = npass): the lanes of a wave stay on one sid and depth,
    // so their gathers are adjacent in the planar copy (wave-uniform choice)
    // (the fused kernel keeps the linear table: its lanes are on different passes and depths, and
    // planar reads measured -57 % on caustic8, -38 % with whole-wave lockstep groups)
    constexpr bool planar = STREAMS;                 // (the host always passes d_rndp and d_scp)
    constexpr bool kRegen = BDPT_REGEN_K > 1;
    constexpr bool kParkPf = kRegen && !STREAMS;
    // pass streams: a parked lane loads its next pass's first randoms when it parks, with the
    // other lanes' prefetch (loading them at the release instead wrote registers the continuing
    // lanes' prefetch had just targeted, and the compiler waited for that prefetch first)
    constexpr bool kParkLoad = kRegen && STREAMS;
    float cr0 = 0.f, cr1 = 0.f;                     // camera randoms of a released lane (kParkPf)
    // (read through a buffer descriptor: the compiler would otherwise merge them with the q0, q1
    // loads of the same addresses and copy them over behind a vmcnt(0))
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
        (void*)rnd, (short)0, (int)(kRandN * 4u), 0x00020000);
    auto load_cam = [&](unsigned jc) {
        cr0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsl, jc * 4u, 0, 0));
        cr1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsl, jc * 4u, 4, 0));
    };
    // the linear table: plain loads (pass streams) or buffer loads (fused kernel)
    auto load_lin = [&](unsigned jj, float& a0, float& a1, float& a2, float& a3, float& a4) {
        if constexpr (!STREAMS) { load_rand5b(rsl, jj, a0, a1, a2, a3, a4); return; }
        load_rand5(rnd, jj, a0, a1, a2, a3, a4);
    };
    const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.rndp, (short)0, (int)(BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL * 4u), 0x00020000);
    // BDPT_SCP: {sinf, cosf}(2 pi d_Rand[j]) and (2 pi d_Rand[j + 4]) (q4 is not loaded)
    float sn0 = 0.f, cs0 = 0.f, sn4 = 0.f, cs4 = 0.f;
    const __amdgpu_buffer_rsrc_t rss = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.scp, (short)0, (int)(BDPT_DEV_RANDP_PLANES * BDPT_DEV_RANDP_PL * 8u), 0x00020000);
    // BDPT_SCP_LATE (experiment): the pairs loaded at the top of their own segment instead of
    // one segment ahead with d_Rand[j..j+3] (shorter register lifetimes, less time to arrive)
    auto load_plan = [&](unsigned jj) {
        if constexpr (kScp && BDPT_SCP_LATE) load_rand4p(rsp, jj, q0, q1, q2, q3);
        else if constexpr (kScp) load_rand_scp(rsp, rss, jj, q0, q1, q2, q3, sn0, cs0, sn4, cs4);
        else load_rand5p(rsp, jj, q0, q1, q2, q3, q4);
    };
    if (planar) load_plan(j);
    else
    load_lin(j, q0, q1, q2, q3, q4);
    // BDPT_RNG_PAIR: n0..n4 = the next segment's randoms, loaded with q0..q4 at even depths
    constexpr bool kPair = !STREAMS && BDPT_RNG_PAIR;
    float n0 = 0.f, n1 = 0.f, n2 = 0.f, n3 = 0.f, n4 = 0.f;
    auto load_next = [&](unsigned jj) {                 // segment depth + 1: (jj + 5) mod (RAND_N - 5)
        const unsigned jn = jj + 5u < M5 ? jj + 5u : jj + 5u - M5;
        load_lin(jn, n0, n1, n2, n3, n4);
    };
    if constexpr (kPair) load_next(j);
    if constexpr (kParkPf) load_cam(j);
    f3 ro = mk(0.f, 0.f, 0.f), rd = ro, thr = ro, rad = ro, nl = ro;
    bool specular = true, fresh = true, parked = false, want = kPool && !active;
    bool alive = active && nslot > 0 && cnt0 + (unsigned)(kUnits ? k : s0 + k * S) < BDPT_DEV_COUNTER_CAP;

    // (a pool lane without a pixel yet keeps the loop going: it draws one at the iteration's end)
    BDPT_CNTN(14, 1);
    while (__builtin_amdgcn_ballot_w64(alive || (kPool && want)) != 0) {   // wave-uniform loop
        BDPT_CNTN(0, 1);
        BDPT_CNT(1, alive && fresh);
        BDPT_CNT(2, alive);
#ifdef BDPT_STATS
        {
            const unsigned long long ma = __builtin_amdgcn_ballot_w64(alive);
            if (lane == 0) {
                atomicAdd(&bdpt_dev_stats[4], 1ull);
                atomicAdd(&bdpt_dev_stats[5], (unsigned long long)__popcll(ma));
            }
        }
#endif
        bool done = false, diff = false;
        float t = 1e20f;
        int id = -1;
        if constexpr (kScp && BDPT_SCP_LATE) {
            if (alive) load_sc(rss, j, sn0, cs0, sn4, cs4);
        }
        if (alive) {
            if (fresh) {                  // camera ray (:562-600); d_Rand[kk] == q0 (kk == j)
                const float4 c0 = K[0], c1 = K[1], c2 = K[2], c3 = K[3], k4 = K[4];
                // device.cu:565-566: ((float)x*iw - iw*W/2.) + d_Rand[kk]*iw in fp64, then fp32
                const double2 cb = camb[threadIdx.x];
                const float u0 = kParkPf ? cr0 : q0, u1 = kParkPf ? cr1 : q1;
                const float kx = (float)(cb.x + (double)(u0 * k4.x));
                const float ky = (float)(cb.y + (double)(u1 * k4.y));
                f3 rdir = mk(0.f, 0.f, 0.f);
                rdir = add(rdir, smul(kx, mk(c0.x, c0.y, c0.z)));
                rdir = add(rdir, smul(ky, mk(c1.x, c1.y, c1.z)));
                rdir = add(rdir, mk(c2.x, c2.y, c2.z));                       // kz * ud
                const float w = (c0.w * kx + c1.w * ky + c2.w) + 1;           // c2.w = tz * kz
                // (float)(1./(double)w) == 1.f/w: double rounding of a quotient is innocuous
                // when 53 >= 2*24 + 2 (device.cu:594)
                rdir = smul(rcp_rn(w), rdir);
                ro = add(rdir, mk(c3.x, c3.y, c3.z));
                rd = norm(rdir);
                rad = mk(0.f, 0.f, 0.f);
                thr = mk(1.f, 1.f, 1.f);
                specular = true;
                fresh = false;
            }
            // closest hit, scanning from the last sphere down (device.cu:106-124)
            if constexpr (kBVH) {
                // walls by brute force, then the BVH; equal distances go to the higher index,
                // which is what the reference's downward scan with `d < t` yields
                for (int q = a.big_n - 1; q >= 0; --q) {
                    const troots h = sphere_roots(BG[q], ro, rd);
                    const float d = h.t1 > kEps ? h.t1 : h.t2;
                    const int s = BI[q] & kBvhIdMask;
                    if (h.t2 > kEps && (d < t || (d == t && s > id))) { t = d; id = s; }
                }
                const bvh_ray br = bvh_setup(a, ro, rd);
                int node = 0;
                // while-while: walk inner nodes until this lane has a leaf, then test leaves
                while (true) {
                    int info = -1;
                    while (node < a.bvh_nn) {
                        const float4 lo = NDt[2 * node], hi = NDt[2 * node + 1];
                        const int inf = __float_as_int(hi.w);
                        const bool in = bvh_box(lo, hi, br, t);
                        node = (in && inf < 0) ? node + 1 : __float_as_int(lo.w);
                        if (in && inf >= 0) { info = inf; break; }
                    }
                    if (info < 0) break;
                    const int first = info & 0xffffff, end = first + (info >> 24);
                    for (int k = first; k < end; k++) {
                        const troots h = sphere_roots(SGt[k], ro, rd);
                        const float d = h.t1 > kEps ? h.t1 : h.t2;
                        const int s = SIt[k] & kBvhIdMask;
                        if (h.t2 > kEps && (d < t || (d == t && s > id))) { t = d; id = s; }
                    }
                }
            } else {
#ifdef BDPT_JIT
                if constexpr (N == BDPT_JIT_N) {
                    // specialised kernels: integer keys (one v_min3_u32 per sphere) and the
                    // wave-uniform det skip for the non-wall spheres
                    unsigned kt = key_of(t);
                    auto hit = [&](int s) -> bool {
                        const tdet qd = sphere_det(geom(s), ro, rd);
                        if (small_sphere(s) && __builtin_amdgcn_ballot_w64(!(qd.det < 0.f)) == 0) {
                            BDPT_CNTN(10, 1);
                            return true;                          // every lane misses sphere s
                        }
                        const troots q = roots_of(qd);
                        const unsigned nk = umin3(kt, key_of(q.t1), key_of(q.t2));
                        id = nk < kt ? s : id;
                        kt = nk;
                        return true;
                    };
                    unroll_down<N - 1>(hit);
                    t = __uint_as_float(kt + kKeyC);
                } else
#endif
                {
#pragma unroll kUnroll
                    for (int s = n - 1; s >= 0; --s) {
                        const troots q = sphere_roots(geom(s), ro, rd);
                        const float r = q.t1 > kEps ? q.t1 : q.t2;
                        if (q.t2 > kEps && r < t) { t = r; id = s; }
                    }
                }
            }
            done = id < 0;
        }
        BDPT_TICK(0);                 // camera ray + closest hit
        BDPT_CNT(3, alive && !done);
        // paired loads: an odd-depth segment takes the randoms loaded with the previous one --
        // here, after the closest hit and just before the shading uses them, not where the next
        // loads are issued: a copy there made the compiler merge the loaded values through
        // temporaries and wait for the loads it had just issued (s_waitcnt vmcnt(0) right after
        // them), which cancelled the prefetch of every segment; at the top of the loop the wait
        // would not overlap the closest hit.
        if constexpr (kPair) {
            if (alive && (depth & 1u)) { q0 = n0; q1 = n1; q2 = n2; q3 = n3; q4 = n4; }
        }
        if (alive) {
            if (!done) {
                const float4 cm = tabC(id);
                const int mat = __float_as_int(cm.w);
                const float4 pc = tabP(id);
                const f3 hit = add(ro, smul(t, rd));
                const f3 normal = norm(sub(hit, mk(pc.x, pc.y, pc.z)));
                const float dp = dot(normal, rd);
                nl = dp > 0 ? mk(-normal.x, -normal.y, -normal.z) : normal;   // (-1*sign(dp))*n, exact
                if (mat & 256) {                                         // emitter (:651-661)
                    if (specular) {
                        const float4 em = tabE(id);
                        rad = add(rad, mul(thr, smul(fabsf(dp), mk(em.x, em.y, em.z))));
                    }
                    done = true;
#if defined(BDPT_JIT) && BDPT_JIT_ZERO_SAFE
                } else if (N == BDPT_JIT_N && (mat & 512)) {
                    // A black surface (cornell's front wall) makes the throughput exactly 0 (the
                    // reference multiplies it by c = 0 whatever the material), so everything the
                    // path adds from here on -- this vertex's NEE included -- is 0 * (finite) = +0:
                    // the host proved the NEE term finite for this scene (every emitter keeps a gap
                    // >= 1 from every other surface, bdpt_host.cpp).  rad is final: end the path.
                    done = true;
#endif
                } else {
                    // DIFF (:663-703), SPEC (:704-714), REFR (:715-770).  Nearly every wave holds
                    // a few refracting lanes next to its diffuse ones, so the diffuse and the
                    // refraction code both run; their square root (sqrt(r2) | sqrt(cos2t)) and
                    // their normalisation (u | the transmitted direction) are one shared
                    // instruction sequence on lane-selected inputs -- the same float operations
                    // per lane, so the results are unchanged.
                    const bool isdiff = (mat & 255) == BDPT_DEV_DIFF;
                    const f3 cc = mk(cm.x, cm.y, cm.z);
                    BDPT_CNT(4, true);
                    // the path's last segment (depth 6, :621): the next direction and the
                    // specular weights are never used -- a diffuse vertex still weights its NEE
                    if (depth >= 6u) {
                        BDPT_CNT(19, isdiff);
                        if (isdiff) {
                            specular = false;
                            thr = mul(thr, cc);
                            diff = true;
                        }
                    } else {
                    f3 refl = rd;
                    bool refr = false, into = false;
                    float nnt = 0.f, ddn = 0.f, cos2t = 0.f;
                    const float nc = 1.f, nt = 1.5f;
                    BDPT_CNT(17, !isdiff);
                    BDPT_CNT(18, isdiff);
                    if (!isdiff) {
                        specular = true;
                        refl = sub(rd, smul(2.f * dot(normal, rd), normal));
                        if ((mat & 255) == BDPT_DEV_SPEC) {
                            thr = mul(thr, cc);
                            rd = refl;
                        } else {
                            into = dot(normal, nl) > 0;
                            nnt = into ? nc / nt : nt / nc;
                            ddn = dot(rd, nl);
                            cos2t = 1.f - nnt * nnt * (1.f - ddn * ddn);
                            if (cos2t < 0.f) {
                                thr = mul(thr, cc);
                                rd = refl;
                            } else {
                                refr = true;
                            }
                            BDPT_CNT(5, refr);
                        }
                    }
                    if (isdiff || refr) {
                        // r2 = d_Rand value >= 2^-32; cos2t = 1 - X is 0 or >= 2^-24: core exact
                        const float s1 = bdpt_sqrt_rn_core(isdiff ? q1 : cos2t);
                        f3 V;
                        if (isdiff) {
                            const f3 ax = fabsf(nl.x) > .1f ? mk(0.f, 1.f, 0.f) : mk(1.f, 0.f, 0.f);
                            V = cross(ax, nl);                    // |V|^2 >= 0.01 by the choice
                        } else {
                            const float kq = (float)(into ? 1 : -1) * (ddn * nnt + s1);
                            V = sub(smul(nnt, rd), smul(kq, normal));
                        }
                        float root;
                        const f3 U = smul(rcp_sqrt_rn(dot(V, V), &root), V);   // u | td
                        if (isdiff) {
                            specular = false;
                            thr = mul(thr, cc);
                            diff = true;              // shadow rays: below, compacted over the wave
                            if constexpr (kScp) rd = cosine_tail_sc(nl, U, sn0, cs0, q1, s1);
                            else rd = cosine_tail<true>(nl, U, q0, q1, s1, SCT);
                        } else {
                            const float aa = nt - nc, bb = nt + nc;
                            const float R0 = aa * aa / (bb * bb);
                            const float c = 1 - (into ? -ddn : dot(U, normal));
                            const float Re = R0 + (1 - R0) * c * c * c * c * c;
                            const float Tr = 1.f - Re;
                            const float Pp = .25f + .5f * Re;
                            const bool reflect = q2 < Pp;
                            const float k = div_rn_normal(reflect ? Re : Tr, reflect ? Pp : 1.f - Pp);
                            thr = mul(smul(k, thr), cc);
                            rd = reflect ? refl : U;
                        }
                    }
                    }
                    ro = hit;
                }
            }
        }

        BDPT_TICK(1);                 // hit shading
        // ---- SampleLightsDevice (device.cu:457-542) for the diffuse vertices of this segment:
        // NEE towards every emitter (same d_Rand[j+3], d_Rand[j+4] for all) + 1 VLP, blended 1/2.
        if (__builtin_amdgcn_ballot_w64(diff) != 0) {
            f3 res = mk(0.f, 0.f, 0.f), usp = res, vsd = res, vcon = res;
            if (diff) {
                if constexpr (kScp) usp = uniform_sphere_sc(q3, sn4, cs4);
                else usp = uniform_sphere<true>(q3, q4, SCT);
            }
            const int nlights = (int)a.n_lights;
            // the emitters' NEE records {p, rad}, {e, (4*pi*rad)*rad} (bdpt_host.cpp upload_scene)
            // through the constant address space (folding them into the specialised build freed
            // 8 VGPRs but issued 2.5 % more VALU instructions: cornell -1 to -2 % at 5..8 waves)
            auto lrec = [&](int k) -> float4 { return ld_const(a.lightrec, k); };
            const int nsteps = nlights > 0 ? nlights : 1;
            for (int li = 0; li < nsteps; li++) {                         // uniform
                BDPT_CNTN(6, 1);
                bool has_nee = false, has_vlp = false;
                f3 sd = res, con = res;
                float maxt = 0.f, vmaxt = 0.f;
                if (diff && nlights > 0) {
                    const float4 lg = lrec(2 * li);                       // {p, rad}
                    const float4 le = lrec(2 * li + 1);                   // {e, 4*pi*rad*rad}
                    const f3 spt = add(smul(lg.w, usp), mk(lg.x, lg.y, lg.z));
                    sd = sub(spt, ro);
                    float len;
                    sd = smul(rcp_sqrt_rn(dot(sd, sd), &len), sd);
                    float wo = dot(sd, usp);
                    if (!(wo > 0.f)) {
                        wo = -wo;
                        const float wi = dot(sd, nl);
                        if (wi > 0.f) {
                            has_nee = true;
                            maxt = len - kEps;
                            const float na = le.w * wi * wo, nb = len * len;
                            // one Markstein step (div_rn_normal) when a, b lie in [2^-60, 2^60]:
                            // then 1/b, a/b and the residual stay normal; otherwise (grazing
                            // wi * wo) the library division on an exec-masked branch
                            float kq;
                            if (__builtin_expect(na >= 0x1p-60f && na <= 0x1p60f &&
                                                 nb >= 0x1p-60f && nb <= 0x1p60f, 1))
                                kq = div_rn_normal(na, nb);
                            else
                                kq = na / nb;
                            con = smul(kq, mk(le.x, le.y, le.z));
                        }
                    }
                }
                if (diff && li == 0) {                                    // the VLP (:507-537)
                    const float4 v0 = V[3 * k], v1 = V[3 * k + 1], v2 = V[3 * k + 2];
                    // a VLP with zero radiance adds exactly +0 to vres whether it is visible or
                    // not (wi * wo is finite): no ray.  Wave-uniform under pass streams, where a
                    // workgroup renders one pass (zero VLPs: cornell 6 %, cornell_glass 45 %)
                    BDPT_CNT(20, !(v0.w == 0.f && v1.x == 0.f && v1.y == 0.f));
                    if (!(v0.w == 0.f && v1.x == 0.f && v1.y == 0.f)) {
                        vsd = sub(mk(v0.x, v0.y, v0.z), ro);
                        float len;
                        vsd = smul(rcp_sqrt_rn(dot(vsd, vsd), &len), vsd);
                        float wo = dot(vsd, mk(v1.z, v1.w, v2.x));
                        if (!(wo > 0.f)) {
                            wo = -wo;
                            const float wi = dot(vsd, nl);
                            if (wi > 0.f) {
                                has_vlp = true;
                                vmaxt = len - kEps;
                                vcon = smul(wi * wo, mk(v0.w, v1.x, v1.y));
                            }
                        }
                    }
                }
                // compact this step's shadow rays into the wave's queue
                const unsigned long long mn = __builtin_amdgcn_ballot_w64(has_nee);
                const unsigned long long mv = __builtin_amdgcn_ballot_w64(has_vlp);
                const int cn = __popcll(mn);
                const int total = cn + __popcll(mv);
                const int pn = lane_prefix(mn), pv = cn + lane_prefix(mv);
                if (has_nee) {                    // SoA: {o, maxt}[kQueue], {d, vacuum}[kQueue]
                    SQ[pn] = make_float4(ro.x, ro.y, ro.z, maxt);
                    SQ[kQueue + pn] = make_float4(sd.x, sd.y, sd.z, 0.f);
                }
                if (has_vlp) {
                    SQ[pv] = make_float4(ro.x, ro.y, ro.z, vmaxt);
                    SQ[kQueue + pv] = make_float4(vsd.x, vsd.y, vsd.z, 1.f);
                }
                wave_lds_fence();
                BDPT_TICK(2);         // NEE / VLP set-up and queue writes
#ifdef BDPT_STATS
                {
                    const unsigned long long md = __builtin_amdgcn_ballot_w64(diff);
                    if (lane == 0) {
                        atomicAdd(&bdpt_dev_stats[0], 1ull);
                        atomicAdd(&bdpt_dev_stats[1], (unsigned long long)((total + 63) / 64));
                        atomicAdd(&bdpt_dev_stats[2], (unsigned long long)total);
                        atomicAdd(&bdpt_dev_stats[3], (unsigned long long)__popcll(md));
                    }
                }
#endif
                for (int base = 0; base < total; base += 64) {            // uniform
                    // A part-full round (<= 32 rays; typically the second round, ~14 rays for
                    // cornell) is traced by 2^lg lane groups that split the sphere list: ray r
                    // goes to lanes r, r + 64/2^lg, ...; group g tests spheres n-1-g, n-1-g-2^lg,
                    // ...; occlusion is the OR over groups (ballot, folded on the scalar unit).
                    // Each sphere test is the same float sequence, and occlusion is an OR, so the
                    // result is the same in any order.
                    if constexpr (!kBVH) {
                        const int c = total - base;                        // uniform
                        // a round of VLP rays only: the non-emitters' list (IntersectPVacuumDevice
                        // never counts an emitter), which often fits fewer lane-group iterations
                        // (cornell: 8 spheres instead of 9)
                        const bool allvac = BDPT_VAC_LIST && !kPool && base >= cn;   // uniform
                        const int nl = allvac ? a.n_vac : n;
                        const float4* GL = allvac ? GV : G;
#if BDPT_LG_RULE
                        // as many groups as the round's rays allow, down to the fewest that still
                        // take the same number of iterations (ceil(nl / 2^lg)); groups past the
                        // list's end idle
                        int lg = c <= 2 ? 5 : c <= 4 ? 4 : c <= 8 ? 3 : (c <= 16 ? 2 : (c <= 32 ? 1 : 0));
                        while (lg > 0 && (1 << (lg - 1)) >= nl) lg--;
#else
                        int lg = c <= 8 ? 3 : (c <= 16 ? 2 : (c <= 32 ? 1 : 0));
                        while (lg > 0 && (1 << lg) > nl) lg--;
#endif
                        if (lg > 0) {
                            BDPT_CNTN(8, 1);
                            const int rpg = 64 >> lg;
                            const int r = lane & (rpg - 1), g = lane >> (6 - lg);
                            unsigned occ = 0;
                            if (r < c) {
                                const float4 r0 = SQ[base + r], r1 = SQ[kQueue + base + r];
                                const f3 o = mk(r0.x, r0.y, r0.z), d = mk(r1.x, r1.y, r1.z);
                                const bool vac = r1.w != 0.f;
#if BDPT_IKEY
                                const unsigned km = maxt_key(r0.w);
#endif
                                if (allvac) {
                                    for (int s = nl - 1 - g; s >= 0; s -= 1 << lg) {
                                        const troots q = sphere_roots(GL[s], o, d);
#if BDPT_IKEY
                                        if (umin2(key_of(q.t1), key_of(q.t2)) < km) { occ = 1; break; }
#else
                                        const float rr = q.t1 > kEps ? q.t1 : q.t2;
                                        if (q.t2 > kEps && rr < r0.w) { occ = 1; break; }
#endif
                                    }
                                } else
                                for (int s = n - 1 - g; s >= 0; s -= 1 << lg) {
                                    BDPT_CNTN(16, 1);
                                    const troots q = sphere_roots(G[s], o, d);
#if BDPT_IKEY
                                    if (umin2(key_of(q.t1), key_of(q.t2)) < km && !(vac && emissive(s))) { occ = 1; break; }
#else
                                    const float rr = q.t1 > kEps ? q.t1 : q.t2;
                                    if (q.t2 > kEps && rr < r0.w && !(vac && emissive(s))) { occ = 1; break; }
#endif
                                }
                            }
                            unsigned long long m = __builtin_amdgcn_ballot_w64(occ != 0);
                            for (int w = 32; w >= rpg; w >>= 1) m |= m >> w;   // uniform
                            if (lane < c) SQ[base + lane].w = __uint_as_float((unsigned)(m >> lane) & 1u);
                            continue;
                        }
                    }
                    const int idx = base + lane;
                    if (idx < total) {
                        const float4 r0 = SQ[idx], r1 = SQ[kQueue + idx];
                        const f3 o = mk(r0.x, r0.y, r0.z), d = mk(r1.x, r1.y, r1.z);
                        const bool vac = r1.w != 0.f;
                        unsigned occ = 0;
                        if constexpr (kBVH) {                             // IntersectP(Vacuum)Device
                            for (int q = 0; q < a.big_n && !occ; q++) {
                                const troots h = sphere_roots(BG[q], o, d);
                                const float dd = h.t1 > kEps ? h.t1 : h.t2;
                                if (h.t2 > kEps && dd < r0.w && !(vac && (BI[q] & kBvhEmissive))) occ = 1;
                            }
                            const bvh_ray br = bvh_setup(a, o, d);
                            int node = occ ? a.bvh_nn : 0;
                            while (node < a.bvh_nn) {
                                const float4 lo = NDt[2 * node], hi = NDt[2 * node + 1];
                                const int info = __float_as_int(hi.w);
                                if (!bvh_box(lo, hi, br, r0.w)) { node = __float_as_int(lo.w); continue; }
                                if (info < 0) { node++; continue; }
                                const int first = info & 0xffffff, end = first + (info >> 24);
                                for (int k = first; k < end; k++) {
                                    const troots h = sphere_roots(SGt[k], o, d);
                                    const float dd = h.t1 > kEps ? h.t1 : h.t2;
                                    if (h.t2 > kEps && dd < r0.w && !(vac && (SIt[k] & kBvhEmissive))) { occ = 1; break; }
                                }
                                node = occ ? a.bvh_nn : __float_as_int(lo.w);
                            }
                        } else {
                        // occlusion as a wave lane mask (SGPRs): every lane tests every sphere
                        // until all of the round's rays are occluded (one uniform branch per
                        // sphere).  No per-lane break, so no nest of saved exec masks -- for 64
                        // spheres those spilled to VGPR lanes -- and no per-sphere register copy
                        // of the flag; a lane's further tests cannot change its OR.
                        const unsigned long long live = __builtin_amdgcn_ballot_w64(true);
                        const unsigned long long vacm = __builtin_amdgcn_ballot_w64(vac);
                        unsigned long long occm = 0;
#if BDPT_IKEY
                        const unsigned km = maxt_key(r0.w);
#endif
                        BDPT_CNTN(7, 1);
                        auto step = [&](int s) -> bool {                  // IntersectP(Vacuum)Device
                            // a round of VLP rays only (the queue holds the NEE rays first):
                            // IntersectPVacuumDevice never counts an emitter, so its test is skipped
                            if (BDPT_VAC_SKIP && emissive(s) && vacm == live) return true;
                            BDPT_CNTN(9, 1);
                            const tdet qd = sphere_det(geom(s), o, d);
                            if (small_sphere(s) && __builtin_amdgcn_ballot_w64(!(qd.det < 0.f)) == 0) {
                                BDPT_CNTN(12, 1);
                                return true;                          // every ray misses sphere s
                            }
                            const troots q = roots_of(qd);
#if BDPT_IKEY
                            unsigned long long h = __builtin_amdgcn_ballot_w64(
                                umin2(key_of(q.t1), key_of(q.t2)) < km);
#else
                            const float rr = q.t1 > kEps ? q.t1 : q.t2;
                            // two ballots: a ballot of `a && b` is materialised through a VGPR
                            unsigned long long h = __builtin_amdgcn_ballot_w64(q.t2 > kEps) &
                                                   __builtin_amdgcn_ballot_w64(rr < r0.w);
#endif
                            if (emissive(s)) h &= ~vacm;
                            occm |= h;
                            return occm != live;
                        };
                        // spheres n-1 .. 0; unrolled by template recursion (the loop unroller
                        // leaves a loop holding a ballot alone)
                        if constexpr (N > 0) unroll_down<N - 1>(step);
                        else for (int s = n - 1; s >= 0 && step(s); --s) {}
                        occ = (unsigned)(occm >> lane) & 1u;
                        }
                        SQ[idx].w = __uint_as_float(occ);
                    }
                }
                wave_lds_fence();
                BDPT_TICK(3);         // shadow rounds
                if (has_nee && __float_as_uint(SQ[pn].w) == 0) res = add(res, con);
                if (has_vlp && __float_as_uint(SQ[pv].w) != 0) vcon = mk(0.f, 0.f, 0.f);
                if (li == 0 && !has_vlp) vcon = mk(0.f, 0.f, 0.f);
                wave_lds_fence();
            }
            if (diff) {
                f3 vres = mk(0.f, 0.f, 0.f);
                vres = add(vres, vcon);
                vres = smul(1.f, vres);
                res = add(res, vres);
                res = smul(0.5f, res);
                rad = add(rad, mul(res, thr));
            }
        }

        BDPT_TICK(4);                 // shadow results + contribution
        // pass streams: the segment's randoms are settled here, before this iteration's radiance
        // stores.  The loads that refill their registers below then have no earlier load of the
        // same registers to wait for -- the compiler otherwise waits for every outstanding memory
        // operation there, the just-issued stores included (their loads completed long before:
        // the shading used them; the wait appeared on paths that skip the shading).
        if constexpr (kScp) asm volatile("" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3), "v"(sn0), "v"(cs0), "v"(sn4), "v"(cs4));
        else if constexpr (STREAMS) asm volatile("" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3), "v"(q4));
        if (alive) {
            if (!done && ++depth > 6) done = true;                       // :621 7-segment cap
            BDPT_CNT(11, done);
            BDPT_CNTN(15, __popcll(__builtin_amdgcn_ballot_w64(done)));
            if (done) {                                                  // :774-787
                if constexpr (!STREAMS || kUnits) {
                    const unsigned cnt = cnt0 + (unsigned)k;      // S == 1: pass k
                    if (cnt == 0) {
                        col = rad;
                    } else {
                        const float k1 = (float)cnt;
                        const float k2 = rcp_rn_inrange(k1 + 1.f);   // 2 <= k1+1 <= 30000
                        col.x = (col.x * k1 + rad.x) * k2;
                        col.y = (col.y * k1 + rad.y) * k2;
                        col.z = (col.z * k1 + rad.z) * k2;
                    }
                } else {
                    bdpt_dev_vec r;
                    r.x = rad.x; r.y = rad.y; r.z = rad.z;
                    unsigned xyv = xy;
                    asm volatile("" : "+v"(xyv));
                    const int li = kPool ? (int)lix : ((int)(xyv >> 16) - yoff) * a.W + (int)(xyv & 0xffffu);
                    const size_t ri = (size_t)(s0 + k * S) * a.nloc + (size_t)li;
                    if constexpr (kPool) {
                        // sparse radiance: pixel pools serve open scenes, where most samples are
                        // exactly +0 (caustic: 78 % of the samples, half of all 64-pixel runs) --
                        // only the others are stored, each marking its pass in the pixel's mask
                        // (zeroed before the launch), and the fold reads only those (every bit +0
                        // counts as zero, so a -0 component is stored and folded as it is)
                        if ((__float_as_uint(r.x) | __float_as_uint(r.y) | __float_as_uint(r.z)) != 0u) {
                            a.rbuf[ri] = r;
                            const unsigned pq = (unsigned)(s0 + k * S);
                            atomicOr(a.rmask + (size_t)li * 4u + (pq >> 5), 1u << (pq & 31u));
                        }
                    } else {
                        a.rbuf[ri] = r;
                    }
                }
                fresh = true;
                depth = 0;
                if constexpr (kPool) {                // the lane takes a pool pixel below
                    alive = false;
                    want = true;
                } else {
                    k++;
                    const int pn = s0 + k * S;
                    alive = kUnits ? (k < nslot && cnt0 + (unsigned)k < BDPT_DEV_COUNTER_CAP)
                                   : (pn < a.npass && cnt0 + (unsigned)pn < BDPT_DEV_COUNTER_CAP);
                    if constexpr (kRegen) {
                        parked = alive;
                        alive = false;
                    }
                }
            }
            if (!kPool && (alive || ((kParkPf || kParkLoad) && parked))) {   // next segment's randoms (:619)
                // 26 + 25 i and the pass's sid are rebuilt here rather than kept live across the
                // loop (one LDS read and four integer ops per segment, against a spill; keeping j
                // live and adding 5 per segment measured 1 % slower)
                if (kPair && (depth & 1u)) {             // loaded with the previous segment's
                } else {
                unsigned xyv = xy;
                asm volatile("" : "+v"(xyv));
                const unsigned li = (xyv >> 16) * (unsigned)a.W + (xyv & 0xffffu);
                j = (26u + li * 25u + depth * 5u + SID[k]) % M5;
                if (planar) load_plan(j);
                else
                {
                // the camera randoms first: the camera ray waits for them at the top of the loop,
                // and the memory counter drains in issue order, so the segment loads issued after
                // them may stay in flight through the camera ray and the closest hit
                if (kParkPf && parked) load_cam(j);
                load_lin(j, q0, q1, q2, q3, q4);
                if (kPair) load_next(j);
                }
                }
            }
        }
        if constexpr (kPool) {
            // lanes whose path ended take the next pixels of the wave's pool, in lane order (a
            // pixel outside the frame or the shard is passed over: the lane draws again)
            unsigned long long mw = __builtin_amdgcn_ballot_w64(want);
            while (mw != 0 && !drained) {
                if (pcur >= pend && !claim()) break;
                const unsigned q = pcur + (unsigned)lane_prefix(mw);
                pcur += (unsigned)__popcll(mw);
                int px = 0, py = 0;
                if (want && pool_pixel(q, px, py)) {
                    want = false;
                    lix = q;
                    xy = ((unsigned)py << 16) | (unsigned)px;
                    camb[threadIdx.x] = make_double2((double)((float)px * a.inv_w) - a.half_w,
                                                     (double)((float)py * a.inv_h) - a.half_h);
                    parked = true;
                }
                mw = __builtin_amdgcn_ballot_w64(want);
            }
            want = false;                             // the pass's pixels are used up
            // the next segment's randoms (:619) for live lanes and the new pixels' first ones,
            // one load group for both
            if (alive || parked) {
                unsigned xyv = xy;
                asm volatile("" : "+v"(xyv));
                const unsigned li = (xyv >> 16) * (unsigned)a.W + (xyv & 0xffffu);
                j = (26u + li * 25u + depth * 5u + SID[k]) % M5;
                if (planar) load_plan(j);
                else
                load_lin(j, q0, q1, q2, q3, q4);
            }
        }
        if constexpr (kRegen) {
            // release the parked lanes together (wave-uniform decision)
            const unsigned long long mp = __builtin_amdgcn_ballot_w64(parked);
            if (mp != 0 && (__popcll(mp) >= BDPT_REGEN_K || __builtin_amdgcn_ballot_w64(alive) == 0)) {
                BDPT_CNTN(13, 1);
                if (parked) {
                    parked = false;
                    alive = true;
                }
                if (!kParkPf && !kParkLoad && alive && fresh) {   // not loaded at park time: now
                    unsigned xyv = xy;
                    asm volatile("" : "+v"(xyv));
                    const unsigned li = (xyv >> 16) * (unsigned)a.W + (xyv & 0xffffu);
                    const unsigned jr = (26u + li * 25u + SID[k]) % M5;
                    if (planar) load_plan(jr);
                    else
                    load_lin(jr, q0, q1, q2, q3, q4);
                    if (kPair) load_next(jr);
                }
            }
        }
        BDPT_TICK(5);                 // path end / accumulation / RNG prefetch
    }
#ifdef BDPT_PROF
    if (lane == 0 && a.prof) {
        for (int q = 0; q < 6; q++) atomicAdd(&a.prof[q], pacc[q]);
        atomicAdd(&a.prof[7], 1ull);
    }
#endif
#ifdef BDPT_COUNTS
    if (a.prof) {
        const unsigned long long live = __builtin_amdgcn_ballot_w64(true);
        for (int q = 0; q < kCnt; q++) {
            unsigned long long sum = 0;
            for (unsigned long long m = live; m != 0; m &= m - 1)
                sum += (unsigned)__builtin_amdgcn_readlane((int)pcnt[q], __builtin_ctzll(m));
            if (lane == __builtin_ctzll(live) && sum != 0) atomicAdd(&a.prof[q], sum);
        }
    }
#endif
    if constexpr (kUnits) {
        // the unit's result, then this wave tile's flag: the next range's unit may start
        if (active && k > 0) {
            st_coherent(&a.colors[i].x, col.x);
            st_coherent(&a.colors[i].y, col.y);
            st_coherent(&a.colors[i].z, col.z);
            __hip_atomic_store(&a.counter[i], cnt0 + (unsigned)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // pixels once, by the launch's last range: plain stores of several units (on several XCDs,
        // each with its own write-back L2) would reach memory in no defined order
        if (active && s0 + nslot >= a.npass) a.pixels[i] = bdpt_dev_to_rgba(col.x, col.y, col.z, a.gamma_thr);
#if BDPT_UNITS_FENCE
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // the stores above are performed
#endif
        if (lane == 0)
            __hip_atomic_store(a.unit_flags + uflag, a.unit_tag | (urange + 1u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (STREAMS || !active || k == 0) return;                            // nothing rendered
    const unsigned cnt = cnt0 + (unsigned)k;
    bdpt_dev_vec out;
    out.x = col.x; out.y = col.y; out.z = col.z;
    a.colors[i] = out;
    a.counter[i] = cnt;
    a.pixels[i] = bdpt_dev_to_rgba(col.x, col.y, col.z, a.gamma_thr);
}

#ifndef BDPT_JIT
// host-side launch table: [streams * 18 + k], k = sphere count (0 = generic LDS traversal) or 17 = BVH
#define BDPT_K(NN, ST) (const void*)&bdpt_path_kernel_t<NN, ST>
#define BDPT_ROW(ST) BDPT_K(0, ST), BDPT_K(1, ST), BDPT_K(2, ST), BDPT_K(3, ST), BDPT_K(4, ST), \
    BDPT_K(5, ST), BDPT_K(6, ST), BDPT_K(7, ST), BDPT_K(8, ST), BDPT_K(9, ST), BDPT_K(10, ST), \
    BDPT_K(11, ST), BDPT_K(12, ST), BDPT_K(13, ST), BDPT_K(14, ST), BDPT_K(15, ST), BDPT_K(16, ST), \
    BDPT_K(-1, ST)
extern "C" const void* bdpt_path_kernel_table[36] = {BDPT_ROW(false), BDPT_ROW(true)};
#undef BDPT_ROW
#undef BDPT_K

// Ordered fold of pass-stream radiance (S > 1): the running mean of device.cu:774-787 applied
// to rbuf[0..npass) in pass order, so the result is the S == 1 result bit for bit.  Same rows
// (and shard remap) as the path launch; one thread per pixel on a 1-D grid over the launch's
// rows, so a wave reads 768 contiguous bytes per pass (on the path launch's 8x8 wave tiles it
// read 8 runs of 96 B: caustic8 -1.9 to -3.7 %, cornell S = 64 -0.3 %, weak64 +-0.2 %,
// profiles/r05_s16_fold_rows_ab.txt).
template <int U, bool SPARSE>
__device__ __forceinline__ void accum_body(const bdpt_path_args& a) {
    const long l = (long)blockIdx.x * 256 + threadIdx.x;
    if (l >= a.nloc) return;
    const int ly = (int)(l / a.W);
    const int x = (int)(l - (long)ly * a.W);
    const int y = bdpt_dev_tile_row(a, ly / BDPT_BTH) * BDPT_BTH + ly % BDPT_BTH;
    if (y >= a.H) return;
    if (a.nshards > 1 && ((y / a.band_rows) % a.nshards) != a.shard) return;
    const int i = y * a.W + x;
    const size_t li = (size_t)ly * a.W + x;
    const unsigned cnt0 = a.counter[i];
    unsigned cnt = cnt0;
    bdpt_dev_vec col = a.colors[i];
    // passes that count: p < npass with cnt0 + p < 30000 (the path kernel rendered exactly these)
    const int n = cnt0 >= BDPT_DEV_COUNTER_CAP ? 0
                : (int)(BDPT_DEV_COUNTER_CAP - cnt0 < (unsigned)a.npass ? BDPT_DEV_COUNTER_CAP - cnt0 : (unsigned)a.npass);
    const bdpt_dev_vec* __restrict__ rb = a.rbuf + li;
    unsigned m0 = 0u, m1 = 0u, m2 = 0u, m3 = 0u;                 // SPARSE: which passes are stored
    if constexpr (SPARSE) {
        const uint4 mw = reinterpret_cast<const uint4*>(a.rmask)[li];
        m0 = mw.x; m1 = mw.y; m2 = mw.z; m3 = mw.w;
    }
    // (the load under a branch, component by component: `stored ? rb[q] : zero` on the struct
    // became a load through a selected pointer, with `zero` on the stack)
    auto sample = [&](int q, bool stored) -> bdpt_dev_vec {
        bdpt_dev_vec v;
        v.x = v.y = v.z = 0.f;
        if (stored) {
            const bdpt_dev_vec* e = rb + (size_t)q * a.nloc;
            v.x = e->x;
            v.y = e->y;
            v.z = e->z;
        }
        return v;
    };
    auto fold = [&](const bdpt_dev_vec& r) {
        if (cnt == 0) {
            col = r;
        } else {
            const float k1 = (float)cnt;
            const float k2 = rcp_rn_inrange(k1 + 1.f);        // 2 <= k1 + 1 <= 30000: exact
            col.x = (col.x * k1 + r.x) * k2;
            col.y = (col.y * k1 + r.y) * k2;
            col.z = (col.z * k1 + r.z) * k2;
        }
        cnt++;
    };
    // (folds with 8 loads in flight, or with streaming loads, ran faster alone but slowed the
    // concurrent path kernel more: caustic8 -1.3 % (round 2), -4 to -13 % (profiles/r05_s3_*))
    int p = 0;
    if constexpr (U > 1) {                   // U loads in flight (the fold after the path kernel)
        for (; p + U <= n; p += U) {
            bdpt_dev_vec v[U];
            if constexpr (SPARSE) {
                const unsigned w = p < 64 ? (p < 32 ? m0 : m1) : (p < 96 ? m2 : m3);
                const unsigned bits = w >> (p & 31);              // p is a multiple of U = 16
#pragma unroll
                for (int u = 0; u < U; u++) v[u] = sample(p + u, (bits >> u) & 1u);
            } else {
#pragma unroll
                for (int u = 0; u < U; u++) v[u] = sample(p + u, true);
            }
#pragma unroll
            for (int u = 0; u < U; u++) fold(v[u]);
        }
    }
    for (; p < n; p++) {
        const unsigned w = p < 64 ? (p < 32 ? m0 : m1) : (p < 96 ? m2 : m3);
        fold(sample(p, !SPARSE || ((w >> (p & 31)) & 1u)));
    }
    if (cnt == cnt0) return;
    a.colors[i] = col;
    a.counter[i] = cnt;
    a.pixels[i] = bdpt_dev_to_rgba(col.x, col.y, col.z, a.gamma_thr);
}
extern "C" __global__ __launch_bounds__(256) void bdpt_accum_kernel(bdpt_path_args a) { accum_body<1, false>(a); }
// pixel pools: after the path kernel, on its stream, over the sparse radiance
extern "C" __global__ __launch_bounds__(256) void bdpt_accum_serial_kernel(bdpt_path_args a) { accum_body<16, true>(a); }
// (8 or 32 samples in flight per thread measured the same or 0.5 % slower, profiles/r05_s27_fold_u.txt)

// Frame assembly of a multi-device context without RCCL: add a peer's zero-padded frame (exact:
// each pixel is non-zero on one device only, and x + 0 == x).
extern "C" __global__ __launch_bounds__(256) void bdpt_frame_add_kernel(float* __restrict__ col,
                                                                       const float* __restrict__ add_col,
                                                                       unsigned* __restrict__ cnt,
                                                                       const unsigned* __restrict__ add_cnt,
                                                                       int count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    col[3 * i + 0] += add_col[3 * i + 0];
    col[3 * i + 1] += add_col[3 * i + 1];
    col[3 * i + 2] += add_col[3 * i + 2];
    cnt[i] += add_cnt[i];
}

// Recompute pixels from colors (after a cross-GPU reduce of the radiance frame).
extern "C" __global__ __launch_bounds__(256) void bdpt_pixels_kernel(const bdpt_dev_vec* __restrict__ colors,
                                                                     uchar4* __restrict__ pixels,
                                                                     const float* __restrict__ thr,
                                                                     int count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const bdpt_dev_vec c = colors[i];
    pixels[i] = bdpt_dev_to_rgba(c.x, c.y, c.z, thr);
}
#endif  // BDPT_JIT
