// bdpt_bvh.cpp -- host-side sphere BVH for large scenes (complex.scn 783,
// mod_cornell.scn 789 spheres).
//
// The reference scans every sphere for every ray (IntersectDevice device.cu:106-124,
// IntersectP(Vacuum)Device :126-154).  The BVH must give exactly the same answer, so it only
// ever *skips* spheres that provably cannot change it (see DESIGN.md "Large scenes"):
//   * spheres much larger than the typical one (the walls, r = 1e4 / 1e5) stay in a brute-force
//     list -- they are hit by almost every ray and would swamp any bounding volume;
//   * the others go into a binary BVH of axis-aligned boxes (surface-area-heuristic splits,
//     <= 4 spheres per leaf), rounded outward to float;
//   * the tree is stored in depth-first order with a skip index per node ("threaded" BVH): a hit
//     inner node continues at node+1 (its first child), a missed node or a finished leaf at its
//     skip index, so a lane traverses without a stack;
//   * the kernel widens every box by a per-ray margin that bounds the float error of the
//     reference's sphere test, and resolves equal distances towards the higher sphere index, so
//     the visiting order is irrelevant.
#include <algorithm>
#include <cmath>
#include <vector>

#include <hip/hip_runtime.h>

#include "bdpt_bvh.h"

namespace {

struct item {
    int id;
    double lo[3], hi[3], c[3];
};

struct builder {
    std::vector<item>& it;
    std::vector<float4>& nodes;
    std::vector<int>& order;

    float down(double v) const {
        float f = (float)v;
        return (double)f > v ? std::nextafter(f, -INFINITY) : f;
    }
    float up(double v) const {
        float f = (float)v;
        return (double)f < v ? std::nextafter(f, INFINITY) : f;
    }

    static double area(const double lo[3], const double hi[3]) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    }

    // Surface-area heuristic: over the three axes and every split of it[b, e) sorted by centroid,
    // minimise area(left) * n_left + area(right) * n_right; leaves it[b, e) sorted along the chosen
    // axis and returns the split index.  Ties keep the lowest axis / split (deterministic).
    int split_sah(int b, int e) {
        const int n = e - b;
        double best = INFINITY;
        int best_ax = 0, best_m = b + n / 2;
        std::vector<double> right(n + 1);
        for (int ax = 0; ax < 3; ax++) {
            std::sort(it.begin() + b, it.begin() + e, [ax](const item& x, const item& y) {
                return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.id < y.id);
            });
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            right[n] = 0.0;
            for (int i = n - 1; i >= 1; i--) {
                for (int a = 0; a < 3; a++) {
                    lo[a] = std::min(lo[a], it[b + i].lo[a]);
                    hi[a] = std::max(hi[a], it[b + i].hi[a]);
                }
                right[i] = area(lo, hi) * (n - i);
            }
            double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = 1; i < n; i++) {
                for (int a = 0; a < 3; a++) {
                    llo[a] = std::min(llo[a], it[b + i - 1].lo[a]);
                    lhi[a] = std::max(lhi[a], it[b + i - 1].hi[a]);
                }
                const double cost = area(llo, lhi) * i + right[i];
                if (cost < best) { best = cost; best_ax = ax; best_m = b + i; }
            }
        }
        std::sort(it.begin() + b, it.begin() + e, [best_ax](const item& x, const item& y) {
            return x.c[best_ax] < y.c[best_ax] || (x.c[best_ax] == y.c[best_ax] && x.id < y.id);
        });
        return best_m;
    }

    // Emits the subtree of it[b, e) at nodes[2*k .. ], returns its node count.
    int build(int b, int e) {
        const int k = (int)nodes.size() / 2;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; i++)
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], it[i].lo[a]);
                hi[a] = std::max(hi[a], it[i].hi[a]);
                clo[a] = std::min(clo[a], it[i].c[a]);
                chi[a] = std::max(chi[a], it[i].c[a]);
            }
        nodes.push_back(make_float4(down(lo[0]), down(lo[1]), down(lo[2]), 0.f));
        nodes.push_back(make_float4(up(hi[0]), up(hi[1]), up(hi[2]), 0.f));
        int count = 1;
        if (e - b <= kBvhLeaf) {
            const int first = (int)order.size();
            for (int i = b; i < e; i++) order.push_back(it[i].id);
            nodes[2 * k + 1].w = bdpt_bits_as_float(first | ((e - b) << 24));
        } else {
#ifdef BDPT_BVH_MEDIAN
            int ax = 0;
            for (int a = 1; a < 3; a++)
                if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
            const int m = (b + e) / 2;
            std::nth_element(it.begin() + b, it.begin() + m, it.begin() + e,
                             [ax](const item& x, const item& y) {
                                 return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.id < y.id);
                             });
#else
            const int m = split_sah(b, e);
#endif
            nodes[2 * k + 1].w = bdpt_bits_as_float(-1);
            count += build(b, m);
            count += build(m, e);
        }
        nodes[2 * k].w = bdpt_bits_as_float(k + count);          // skip: first node after the subtree
        return count;
    }
};

}  // namespace

bool bdpt_build_bvh(const bdpt_sphere* s, unsigned n, bdpt_bvh* out) {
    *out = bdpt_bvh();
    if (n == 0) return false;
    std::vector<float> r(n);
    for (unsigned i = 0; i < n; i++) r[i] = s[i].rad;
    std::vector<float> rs(r);
    std::nth_element(rs.begin(), rs.begin() + n / 2, rs.end());
    const double big = 100.0 * std::fabs((double)rs[n / 2]);
    std::vector<item> it;
    for (unsigned i = 0; i < n; i++) {
        const bool emis = !(s[i].e.x == 0.f && s[i].e.y == 0.f && s[i].e.z == 0.f);
        const int id = (int)i | (emis ? kBvhEmissive : 0);
        const double rad = std::fabs((double)s[i].rad);
        const float rr = s[i].rad * s[i].rad;
        const float4 g = make_float4(s[i].p.x, s[i].p.y, s[i].p.z, rr);
        if (rad > big || !(rad > 0.0) || !std::isfinite(rad)) {      // walls, points
            out->big_geom.push_back(g);
            out->big_ids.push_back(id);
            continue;
        }
        // the sphere test uses rr = fl(rad*rad): bound with the larger of rad and sqrt(rr)
        const double re = std::max(rad, std::sqrt((double)rr)) * (1.0 + 1e-6);
        item t;
        t.id = id;
        const double p[3] = {s[i].p.x, s[i].p.y, s[i].p.z};
        for (int a = 0; a < 3; a++) {
            t.lo[a] = p[a] - re;
            t.hi[a] = p[a] + re;
            t.c[a] = p[a];
        }
        it.push_back(t);
    }
    if ((int)it.size() < kBvhMinSpheres) {
        *out = bdpt_bvh();
        return false;
    }
    // the big list keeps the reference's index order (only the tie rule matters, but keep it tidy)
    std::vector<int> order;
    builder bld{it, out->nodes, order};
    bld.build(0, (int)it.size());
    for (int id : order) {
        const int i = id & ~kBvhEmissive;
        out->geom.push_back(make_float4(s[i].p.x, s[i].p.y, s[i].p.z, s[i].rad * s[i].rad));
        out->ids.push_back(id);
    }
    // root sphere: every BVH sphere lies within r_root of c_root (double, rounded up)
    const float4 lo = out->nodes[0], hi = out->nodes[1];
    const double c[3] = {0.5 * ((double)lo.x + hi.x), 0.5 * ((double)lo.y + hi.y), 0.5 * ((double)lo.z + hi.z)};
    double R = 0.0, rmin = INFINITY;
    for (const item& t : it) {
        const int j = t.id & ~kBvhEmissive;
        rmin = std::min(rmin, std::min(std::fabs((double)s[j].rad),
                                       std::sqrt((double)(s[j].rad * s[j].rad))) * (1.0 - 1e-6));
    }
    out->q = rmin > 0.0 ? (float)(64.0 * 0x1p-24 / rmin * (1.0 + 1e-6)) : INFINITY;
    for (const item& t : it) {
        const int i = t.id & ~kBvhEmissive;
        const double dx = s[i].p.x - c[0], dy = s[i].p.y - c[1], dz = s[i].p.z - c[2];
        R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs((double)s[i].rad));
    }
    for (int a = 0; a < 3; a++) out->c_root[a] = (float)c[a];
    // c_root rounded to float moves the centre by < 1 ulp: absorb it in the radius
    const double dc = std::fabs((double)out->c_root[0] - c[0]) + std::fabs((double)out->c_root[1] - c[1]) +
                      std::fabs((double)out->c_root[2] - c[2]);
    out->r_root = (float)((R + dc) * (1.0 + 1e-6));
    return true;
}
