// CPU check of the BVH traversal (csrc/bdpt_bvh.cpp tree + the kernel's bvh_setup / bvh_box /
// threaded walk, restated here in host float arithmetic) against the reference's every-sphere
// loops (IntersectDevice device.cu:106-124, IntersectPVacuumDevice :141-154).  Rays: camera
// rays, rays from hit points in random directions, and shadow rays towards random points, with
// float directions normalised like the kernel's vnorm.  Prints mismatch counts and work.
//
//   bvh_check <scene.scn> <nrays> <seed>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_bvh.h"

namespace {
struct v3 { float x, y, z; };
v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
v3 norm(v3 v) { float l = 1.f / sqrtf(dot(v, v)); return {l * v.x, l * v.y, l * v.z}; }

float isect(float4 g, v3 o, v3 d) {                      // SphereIntersectDevice, miss = inf
    const v3 op = sub({g.x, g.y, g.z}, o);
    const float b = dot(op, d);
    const float det = b * b - dot(op, op) + g.w;
    if (det < 0.f) return INFINITY;
    const float s = sqrtf(det), t1 = b - s, t2 = b + s;
    const float r = t1 > 0.01f ? t1 : t2;
    return r > 0.01f ? r : INFINITY;
}

int ibits(float f) { int i; memcpy(&i, &f, 4); return i; }

struct bvh_ray { v3 olo, ohi, inv; float m; };

bvh_ray setup(const bdpt_bvh& B, v3 o, v3 d) {
    const v3 dc = sub(o, {B.c_root[0], B.c_root[1], B.c_root[2]});
    const float D = sqrtf(dot(dc, dc) * 1.00001f) * 1.00001f + B.r_root;
    bvh_ray r;
    r.m = D * (1e-4f + B.q * D);
    r.olo = {o.x + r.m, o.y + r.m, o.z + r.m};
    r.ohi = {o.x - r.m, o.y - r.m, o.z - r.m};
    const float e = 1e-20f;
    r.inv = {1.f / (fabsf(d.x) > e ? d.x : copysignf(e, d.x)), 1.f / (fabsf(d.y) > e ? d.y : copysignf(e, d.y)),
             1.f / (fabsf(d.z) > e ? d.z : copysignf(e, d.z))};
    return r;
}

bool box(float4 lo, float4 hi, const bvh_ray& r, float tmax) {
    const float x0 = (lo.x - r.olo.x) * r.inv.x, x1 = (hi.x - r.ohi.x) * r.inv.x;
    const float y0 = (lo.y - r.olo.y) * r.inv.y, y1 = (hi.y - r.ohi.y) * r.inv.y;
    const float z0 = (lo.z - r.olo.z) * r.inv.z, z1 = (hi.z - r.ohi.z) * r.inv.z;
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return tn <= tf && tf >= -r.m && tn <= tmax + r.m;
}

long g_nodes = 0, g_tests = 0;

void closest_bvh(const bdpt_bvh& B, v3 o, v3 d, float& t, int& id) {
    t = 1e20f;
    id = -1;
    for (int q = (int)B.big_geom.size() - 1; q >= 0; --q) {
        const float dd = isect(B.big_geom[q], o, d);
        const int s = B.big_ids[q] & (kBvhEmissive - 1);
        g_tests++;
        if (dd < t || (dd == t && s > id)) { t = dd; id = s; }
    }
    const bvh_ray br = setup(B, o, d);
    const int nn = (int)B.nodes.size() / 2;
    int node = 0;
    while (node < nn) {
        const float4 lo = B.nodes[2 * node], hi = B.nodes[2 * node + 1];
        const int info = ibits(hi.w);
        g_nodes++;
        if (!box(lo, hi, br, t)) { node = ibits(lo.w); continue; }
        if (info < 0) { node++; continue; }
        const int first = info & 0xffffff, end = first + (info >> 24);
        for (int k = first; k < end; k++) {
            const float dd = isect(B.geom[k], o, d);
            const int s = B.ids[k] & (kBvhEmissive - 1);
            g_tests++;
            if (dd < t || (dd == t && s > id)) { t = dd; id = s; }
        }
        node = ibits(lo.w);
    }
}

// Metrics only: closest hit with an explicit stack, nearer child first (by child-box centre
// along the ray), to measure how much ordered traversal would save over the threaded walk.
long g_onodes = 0, g_otests = 0;
void closest_ordered(const bdpt_bvh& B, v3 o, v3 d, float& t, int& id) {
    t = 1e20f;
    id = -1;
    for (int q = (int)B.big_geom.size() - 1; q >= 0; --q) {
        const float dd = isect(B.big_geom[q], o, d);
        const int s = B.big_ids[q] & (kBvhEmissive - 1);
        if (dd < t || (dd == t && s > id)) { t = dd; id = s; }
    }
    const bvh_ray br = setup(B, o, d);
    int stack[64], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const int node = stack[--sp];
        const float4 lo = B.nodes[2 * node], hi = B.nodes[2 * node + 1];
        g_onodes++;
        if (!box(lo, hi, br, t)) continue;
        const int info = ibits(hi.w);
        if (info >= 0) {
            const int first = info & 0xffffff, end = first + (info >> 24);
            for (int k = first; k < end; k++) {
                const float dd = isect(B.geom[k], o, d);
                const int s = B.ids[k] & (kBvhEmissive - 1);
                g_otests++;
                if (dd < t || (dd == t && s > id)) { t = dd; id = s; }
            }
            continue;
        }
        const int l = node + 1, r = ibits(B.nodes[2 * l].w);
        auto centre = [&](int n) {
            const float4 a = B.nodes[2 * n], b = B.nodes[2 * n + 1];
            return (0.5f * (a.x + b.x) - o.x) * d.x + (0.5f * (a.y + b.y) - o.y) * d.y + (0.5f * (a.z + b.z) - o.z) * d.z;
        };
        if (centre(l) <= centre(r)) { stack[sp++] = r; stack[sp++] = l; }
        else { stack[sp++] = l; stack[sp++] = r; }
    }
}

bool occluded_bvh(const bdpt_bvh& B, v3 o, v3 d, float maxt, bool vac) {
    for (size_t q = 0; q < B.big_geom.size(); q++)
        if (isect(B.big_geom[q], o, d) < maxt && !(vac && (B.big_ids[q] & kBvhEmissive))) return true;
    const bvh_ray br = setup(B, o, d);
    const int nn = (int)B.nodes.size() / 2;
    int node = 0;
    while (node < nn) {
        const float4 lo = B.nodes[2 * node], hi = B.nodes[2 * node + 1];
        const int info = ibits(hi.w);
        if (!box(lo, hi, br, maxt)) { node = ibits(lo.w); continue; }
        if (info < 0) { node++; continue; }
        const int first = info & 0xffffff, end = first + (info >> 24);
        for (int k = first; k < end; k++)
            if (isect(B.geom[k], o, d) < maxt && !(vac && (B.ids[k] & kBvhEmissive))) return true;
        node = ibits(lo.w);
    }
    return false;
}
}  // namespace

extern "C" int bdpt_read_scene(const char*, bdpt_camera*, bdpt_sphere**, unsigned*);

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    bdpt_camera cam;
    bdpt_sphere* sp = nullptr;
    unsigned n = 0;
    if (bdpt_read_scene(argv[1], &cam, &sp, &n) != 0) return 3;
    const long nrays = atol(argv[2]);
    std::mt19937 rng((unsigned)atoi(argv[3]));
    std::uniform_real_distribution<float> U(0.f, 1.f);
    bdpt_bvh B;
    if (!bdpt_build_bvh(sp, n, &B)) { printf("{\"bvh\": false}\n"); return 0; }
    std::vector<float4> all(n);
    std::vector<int> emis(n);
    for (unsigned i = 0; i < n; i++) {
        all[i] = make_float4(sp[i].p.x, sp[i].p.y, sp[i].p.z, sp[i].rad * sp[i].rad);
        emis[i] = !(sp[i].e.x == 0.f && sp[i].e.y == 0.f && sp[i].e.z == 0.f);
    }
    long bad_closest = 0, bad_shadow = 0, hits = 0, occl = 0;
    v3 o = {cam.orig.x, cam.orig.y, cam.orig.z};
    for (long k = 0; k < nrays; k++) {
        // 3 in 4 rays aim at a random point of the BVH's root box, the rest go anywhere
        const float4 lo = B.nodes[0], hi = B.nodes[1];
        const v3 tgt = {lo.x + U(rng) * (hi.x - lo.x), lo.y + U(rng) * (hi.y - lo.y), lo.z + U(rng) * (hi.z - lo.z)};
        const v3 d = (k & 3) ? norm(sub(tgt, o)) : norm({U(rng) * 2 - 1, U(rng) * 2 - 1, U(rng) * 2 - 1});
        // brute force, reference order
        float t = 1e20f;
        int id = -1;
        for (int s = (int)n - 1; s >= 0; --s) {
            const float dd = isect(all[s], o, d);
            if (dd < t) { t = dd; id = s; }
        }
        float tb;
        int ib;
        closest_bvh(B, o, d, tb, ib);
        if (ibits(t) != ibits(tb) || id != ib) bad_closest++;
        closest_ordered(B, o, d, tb, ib);
        if (ibits(t) != ibits(tb) || id != ib) bad_closest++;
        // shadow ray from o to a random point (maxt random in [0, 1.2 t])
        const float maxt = U(rng) * 1.2f * (id >= 0 ? t : 300.f);
        const bool vac = (k & 1) != 0;
        bool occ = false;
        for (int s = (int)n - 1; s >= 0 && !occ; --s)
            occ = isect(all[s], o, d) < maxt && !(vac && emis[s]);
        if (occ != occluded_bvh(B, o, d, maxt, vac)) bad_shadow++;
        occl += occ;
        // next origin: the hit point (bounce), or back to the camera
        if (id >= 0 && (k % 8) != 7) {
            hits++;
            o = {o.x + t * d.x, o.y + t * d.y, o.z + t * d.z};
        } else {
            o = {cam.orig.x, cam.orig.y, cam.orig.z};
        }
    }
    printf("{\"bvh\": true, \"nodes\": %zu, \"bvh_spheres\": %zu, \"walls\": %zu, \"rays\": %ld, "
           "\"bad_closest\": %ld, \"bad_shadow\": %ld, \"hits\": %ld, \"occluded\": %ld, "
           "\"node_visits_per_ray\": %.2f, \"sphere_tests_per_ray\": %.2f, "
           "\"ordered_node_visits\": %.2f, \"ordered_sphere_tests\": %.2f}\n",
           B.nodes.size() / 2, B.geom.size(), B.big_geom.size(), nrays, bad_closest, bad_shadow, hits, occl,
           (double)g_nodes / nrays, (double)g_tests / nrays, (double)g_onodes / nrays, (double)g_otests / nrays);
    free(sp);
    return bad_closest || bad_shadow ? 1 : 0;
}
