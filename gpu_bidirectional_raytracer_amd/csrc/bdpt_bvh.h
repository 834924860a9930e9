// bdpt_bvh.h -- host BVH builder interface (see bdpt_bvh.cpp) and the constants the path kernel
// shares with it.
#pragma once

#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/bdpt.h"

#ifndef BDPT_BVH_LEAF
#define BDPT_BVH_LEAF 4
#endif
#ifndef BDPT_BVH_MIN
#define BDPT_BVH_MIN 24
#endif
#ifndef BDPT_BVH_AUTO
#define BDPT_BVH_AUTO 128
#endif
constexpr int kBvhLeaf = BDPT_BVH_LEAF;          // spheres per leaf
constexpr int kBvhMinSpheres = BDPT_BVH_MIN;     // fewer BVH spheres: no tree
constexpr int kBvhAutoSpheres = BDPT_BVH_AUTO;   // auto mode: fewer -> brute force (faster on
                                                 // synthetic64's 58, measured)
constexpr int kBvhEmissive = 1 << 30;    // id flag: emissive (IntersectPVacuum skips it)

struct bdpt_bvh {
    // per node 2 float4: {lo.xyz, skip (int bits)}, {hi.xyz, leaf: first | count << 24, else -1}
    std::vector<float4> nodes;
    std::vector<float4> geom;            // BVH spheres in leaf order: {p, rad*rad}
    std::vector<int> ids;                // sphere index | kBvhEmissive
    std::vector<float4> big_geom;        // brute-force list (walls): {p, rad*rad}
    std::vector<int> big_ids;
    float c_root[3] = {0.f, 0.f, 0.f};   // every BVH sphere lies inside the ball (c_root, r_root)
    float r_root = 0.f;
    float q = 0.f;                       // 64 * 2^-24 / smallest BVH sphere radius
};

// host-side reinterpretation of int bits as a float (node / table packing)
inline float bdpt_bits_as_float(int v) {
    float f;
    std::memcpy(&f, &v, sizeof f);
    return f;
}

// Builds the BVH when the scene has at least kBvhMinSpheres ordinary-sized spheres.
bool bdpt_build_bvh(const bdpt_sphere* s, unsigned n, bdpt_bvh* out);
