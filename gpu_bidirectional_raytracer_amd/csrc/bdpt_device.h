// bdpt_device.h -- device-side data layout shared by the HIP kernels and the host launcher.
//
// HBM layout (one context = one GPU):
//   d_rand    float[7,684,096]      MT607 table, lane-major (tid + k*4096)      30.7 MB
//   d_rndp    float[29][307,364]    the same table in 29 planes (j mod 25)     35.6 MB
//   d_scp     float2[29][307,364]   {sinf, cosf}(2 pi u) of every d_rndp entry 71.3 MB
//   d_lp      bdpt_dev_lightpath[4096]  VLPs {hp, rad, nl}, AoS 36 B            147 KB
//   d_sph     bdpt_dev_sphere[n]    48 B/sphere {p, rad^2, e, rad, c, refl}
//   d_colors  bdpt_dev_vec[W*H]     running-mean radiance, AoS 12 B (== dev_colors)
//   d_counter unsigned[W*H]         samples per pixel (== dev_counter)
//   d_pixels  uchar4[W*H]           gamma-2.2 8-bit RGBA (== pixels_buf)
#ifndef BDPT_DEVICE_H
#define BDPT_DEVICE_H

#ifndef __HIPCC_RTC__                       // hipRTC provides the HIP runtime itself
#include <hip/hip_runtime.h>
#endif

#define BDPT_DEV_RAND_N (4096u * 1876u)
// d_Rand in 25 + 4 planes (bdpt_rand_planar_kernel): plane p < 25 holds d_Rand[25 q + p] at q,
// plane 25 + t holds d_Rand[25 (q + 1) + t]; PL = ceil(RAND_N / 25) entries per plane
#define BDPT_DEV_RANDP_PL 307364u
#define BDPT_DEV_RANDP_PLANES 29u
#define BDPT_DEV_N_PER_RNG 1876
#define BDPT_DEV_LIGHT_POINTS 4096
#define BDPT_DEV_COUNTER_CAP 30000u
#define BDPT_DEV_INLINE_PASSES 128      // launches of <= this many passes carry sid/vlp by value
#define BDPT_DEV_BVH_EMISSIVE (1 << 30)   // BVH sphere id flag (bdpt_bvh.h kBvhEmissive)
#define BDPT_DEV_DIFF 0
#define BDPT_DEV_SPEC 1
#define BDPT_DEV_REFR 2

// Path-kernel tiling: a wave covers BDPT_WTW x (64/BDPT_WTW) pixels, a 256-thread workgroup
// BDPT_BLOCK_WX x (4/BDPT_BLOCK_WX) waves (default 4x1: a 32x8 tile, so 8-row shard bands map to
// whole tile rows).  The host sizes the grid from the same macros.
#ifndef BDPT_WTW
#define BDPT_WTW 8
#endif
#ifndef BDPT_BLOCK_WX
#define BDPT_BLOCK_WX 4
#endif
#define BDPT_WTH (64 / BDPT_WTW)
#define BDPT_BLOCK_WY (4 / BDPT_BLOCK_WX)
#define BDPT_BTW (BDPT_BLOCK_WX * BDPT_WTW)
#define BDPT_BTH (BDPT_BLOCK_WY * BDPT_WTH)

struct bdpt_dev_vec { float x, y, z; };
struct bdpt_dev_lightpath { float hx, hy, hz, rx, ry, rz, nx, ny, nz; };
struct bdpt_dev_sphere {
    float px, py, pz, rr;     // rr = rad*rad (the float product SphereIntersectDevice forms)
    float ex, ey, ez, rad;
    float cx, cy, cz;
    int refl;
};

struct bdpt_path_args {
    const bdpt_dev_sphere* sph;
    unsigned n;
    unsigned n_lights;
    const int* lights;              // indices of emitters (e != 0), ascending
    const float4* lightrec;         // per emitter: {p, rad}, {e, (4*pi*rad)*rad}
    const float4* geom;             // per sphere {p, rad*rad} (SGPR-resident traversal)
    const float4* vgeom;            // the non-emitters' {p, rad*rad}, ascending index (n_vac of them):
    int n_vac;                      // the sphere list of a VLP-only shadow round
    unsigned emis_mask;             // bit s = sphere s is emissive (sphere counts <= 32)
    const float* rnd;
    const float* rndp;              // the planar copy (BDPT_DEV_RANDP_*), pass-stream kernels
    const float2* scp;              // per planar entry u: {sinf, cosf}(2 pi u) (bdpt_sincos_planar_kernel)
    const bdpt_dev_lightpath* lp;
    const unsigned* sid;            // per pass (nullptr: the pass table is sid_inl / vlp_inl)
    const int* vlp;                 // per pass
    int npass;
    // a launch of <= BDPT_DEV_INLINE_PASSES passes (every launch of bdpt_path_passes) carries its
    // pass table in the arguments: no upload, no copy kernel before the path kernel
    unsigned sid_inl[BDPT_DEV_INLINE_PASSES];
    int vlp_inl[BDPT_DEV_INLINE_PASSES];
    bdpt_dev_vec* colors;
    unsigned* counter;
    uchar4* pixels;
    const float* gamma_thr;         // 256 thresholds of toInt (vec.h:34)
    int W, H;
    float inv_w, inv_h;             // (float)(14./W), (float)(10.5/H)
    double half_w, half_h;          // (double)(inv_w*W)/2., (double)(inv_h*H)/2.
    float ux[3], uy[3], ud[3], orig[3];
    float tx, ty, tz;
    int shard, nshards, band_rows;
    int tiles_per_band;             // > 0: grid rows enumerate only this shard's bands
    int streams;                    // pass streams S: lane (pixel, s) renders passes s, s+S, ...
    bdpt_dev_vec* rbuf;             // S > 1: per (pass, launched pixel) radiance, [npass][nloc]
    unsigned* rmask;                // pixel pools: per launched pixel 4 words, bit p set = rbuf holds
                                    // pass p's sample (clear: its radiance is +0, not stored)
    int nloc;                       // launched pixels per pass = tile-grid rows * BDPT_BTH * W
    int pool;                       // > 0 (BDPT_POOL builds): a wave renders one pass, restarting lanes
                                    // on new pixels, claimed in chunks of pool x 64 launched pixels
    unsigned* pool_ctr;             // per pass of the launch and eighth of its pixels: pixels claimed,
                                    // one 128-B line each (zero at the launch's start)
    unsigned* pool_ctr_next;        // the next pooled launch's counters: this launch zeroes them
    // BVH traversal (large scenes, kernel table index 17; see bdpt_bvh.cpp)
    const float4* bvh_nodes;        // 2 per node: {lo, skip}, {hi, leaf first|count<<24 or -1}
    const float4* bvh_geom;         // BVH spheres in leaf order {p, rad^2}
    const int* bvh_ids;             // sphere index | 1<<30 if emissive
    const float4* big_geom;         // brute-force spheres (walls) {p, rad^2}
    const int* big_ids;
    const float4* mat;              // per sphere: {c, refl | emissive<<8}, {e, rad}, {p, 0}
    int bvh_nn, bvh_ns, big_n;
    float bvh_c[3], bvh_r;          // ball around every BVH sphere (per-ray margin)
    float bvh_q;                    // 64u / smallest BVH radius (per-ray margin)
    unsigned long long* prof;       // BDPT_PROF builds: per-section shader cycles (8 counters)
    // Ordered in-kernel fold (BDPT_UNITS builds of the pass-stream kernel): a workgroup claims a
    // unit (tile, range) = passes [range * unit_passes, ...) of a 32x8 tile, one lane per pixel,
    // with the running mean in registers; the units of a tile run in range order (a wave waits for
    // its 8x8 tile's flag to reach epoch << 8 | range).
    int unit_passes;                // passes per range
    int unit_wgs;                   // tile workgroups of the launch (gx * gy)
    int gx, gy;                     // the tile grid the 1-D unit grid enumerates
    unsigned unit_tag;              // this launch's epoch << 8
    unsigned* unit_flags;           // per 8x8 wave tile: epoch << 8 | ranges folded
    unsigned* unit_err;             // non-zero: a handover wait timed out (ordering violated)
    unsigned* unit_ctr;             // per XCD queue: units claimed (8 counters, 128 B apart, zeroed per launch)
    int unit_taper;                 // 1: the launch's last unit_passes passes in halving ranges
};

// Units' pass ranges: unit_passes (P) passes each, except (taper) the launch's last <= P passes,
// which are split in halves -- P = 8: ..., 8, 4, 2, 1, 1 -- so that the launch drains over short
// units (the tiles' last ranges are what runs while the chip empties).  Range r starts at the
// returned pass and holds *len passes; bdpt_unit_ranges counts them.
__host__ __device__ inline int bdpt_unit_range(int npass, int P, int taper, int r, int* len) {
    if (!taper) {
        const int s = r * P;
        *len = npass - s < P ? npass - s : P;
        return s;
    }
    const int nbig = (npass - 1) / P;
    if (r < nbig) {
        *len = P;
        return r * P;
    }
    int s = nbig * P, T = npass - s;
    for (int t = r - nbig; t > 0; t--) {
        const int h = (T + 1) / 2;
        s += h;
        T -= h;
    }
    *len = T > 1 ? (T + 1) / 2 : T;
    return s;
}
__host__ __device__ inline int bdpt_unit_ranges(int npass, int P, int taper) {
    if (!taper) return (npass + P - 1) / P;
    const int nbig = (npass - 1) / P;
    int T = npass - nbig * P, n = nbig;
    while (T > 0) {
        T -= T > 1 ? (T + 1) / 2 : 1;
        n++;
    }
    return n;
}

// Tile row of a workgroup row: identity, or the sub-th tile row of this shard's k-th band.
__device__ __forceinline__ int bdpt_dev_tile_row(const bdpt_path_args& a, int by) {
    if (a.tiles_per_band <= 0) return by;
    if (a.tiles_per_band == 1) return a.shard + by * a.nshards;   // 8-row bands (the default)
    const int k = by / a.tiles_per_band, sub = by - k * a.tiles_per_band;
    return (a.shard + k * a.nshards) * a.tiles_per_band + sub;
}

// toInt (vec.h:34) by threshold search: thr[k] is the smallest float whose toInt is >= k,
// computed on the host with the same pow as the reference semantics; 8 compares per channel.
__device__ __forceinline__ int bdpt_dev_gamma8(float v, const float* __restrict__ thr) {
    int k = 0;
#pragma unroll
    for (int step = 128; step > 0; step >>= 1)
        if (v >= thr[k + step]) k += step;
    return k;
}

__device__ __forceinline__ uchar4 bdpt_dev_to_rgba(float r, float g, float b,
                                                   const float* __restrict__ thr) {
    uchar4 o;
    o.x = (unsigned char)bdpt_dev_gamma8(r, thr);
    o.y = (unsigned char)bdpt_dev_gamma8(g, thr);
    o.z = (unsigned char)bdpt_dev_gamma8(b, thr);
    o.w = 0;
    return o;
}

#endif
