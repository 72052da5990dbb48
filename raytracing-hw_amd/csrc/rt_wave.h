// rt_wave.h — persistent wave-synchronous path tracer for gfx950 (the default kernel).
//
// Same per-pixel arithmetic as rt_path.h (bit-identical output), scheduled differently:
// instead of one lane running a whole pixel (spp x depth nested loops, where a wave waits
// at every loop exit for its slowest lane), every lane runs a flat state machine
//     IDLE -> (camera ray) -> TRAV -> SHADE -> TRAV ... -> (fold, accumulate) -> IDLE
// and the wave advances all lanes together one phase at a time:
//   (A) lanes without a pixel take one from a per-launch queue (one atomic per wave,
//       lanes ranked by mbcnt over the ballot of requesters);
//   (B) IDLE lanes start their next sample (camera ray, RNG draws);
//   (C) all TRAV lanes step their BVH traversal together, one node / one triangle per step,
//       suspending nothing: a lane that finishes early waits only for this ray, never for a
//       whole path or pixel;
//   (D) SHADE lanes shade, sample the bounce (RNG), record the vertex and either start the
//       next traversal or end the path (backward fold into the pixel sum).
// Lanes that end a path in (D) start a new sample in the next (B), so path-length
// divergence no longer serialises a wave.  Traversal semantics are the reference's exactly
// (per-call local best, near-first order, strict `<`): see closest_hit() in rt_path.h.
#pragma once
#include "rt_path.h"

namespace rtd {

struct Trav {
    NodeRec nd;     // record of the node being processed
    uint32_t cur;
    int phase;      // internal node: 0 = test near child, 1 = test far child
    float acc;      // best t found inside the current node's subtree (reference local best)
    int sp;
    uint32_t k, kend;  // leaf triangles still to test
    Hit best;       // global winner so far (strict <, first of equal t wins)
};

__device__ __forceinline__ void trav_enter(Trav &t, uint32_t id, const NodeRec &n) {
    t.cur = id;
    t.nd = n;
    t.phase = 0;
    t.acc = 1e9f;
    if ((n.b & 3u) == 3u) {
        t.k = n.a;
        t.kend = n.a + (n.b >> 2);
    } else {
        t.k = t.kend = 0;
    }
}

// BVH::intersect (bvh.cpp:239-243): the root box test; false = the ray misses the scene.
template <bool COUNT>
__device__ __forceinline__ bool trav_begin(const DevScene &sc, const Ray &r, Trav &t, Counters &cnt) {
    if (COUNT) { cnt.rays++; cnt.aabb++; }
    t.best.t = 1e9f;
    t.best.prim = -1;
    t.sp = 0;
    NodeRec root = load_node(sc.node, 0);
    float e;
    if (!aabb_hit(root.mn, root.mx, r, e)) return false;
    trav_enter(t, 0, root);
    return true;
}

// Return from a finished subtree: merge its best into the parent's local best (the
// reference's `a.distance < intersection.distance`), skip parents whose both children are
// done, resume the first parent that still has its far child to test.
__device__ __forceinline__ bool trav_pop(const DevScene &sc, Trav &t, uint2 *stk) {
    for (;;) {
        if (t.sp == 0) return false;
        RT_CHECK(t.sp > 0 && t.sp <= kStack, 4, t.sp, t.sp = 1);
        const uint2 f = stk[--t.sp];
        const float pacc = __uint_as_float(f.y);
        t.acc = t.acc < pacc ? t.acc : pacc;
        if (f.x >> 31) {
            t.cur = f.x & 0x7fffffffu;
            RT_CHECK((int)t.cur < sc.n_nodes, 5, t.cur, t.cur = 0);
            t.phase = 1;
            t.nd = load_node(sc.node, t.cur);
            t.k = t.kend = 0;
            return true;
        }
    }
}

// One traversal step (one triangle, or the child tests of one internal node).
// Returns false once the traversal is complete (result in t.best).
template <bool COUNT>
__device__ __forceinline__ bool trav_step(const DevScene &sc, const Ray &r, Trav &t, uint2 *stk, Counters &cnt) {
    if (t.k < t.kend) {
        RT_CHECK((int)t.k < sc.n_tris, 6, t.k, t.k = 0);
        V3 v0, U, V;
        load_tri(sc.tri, (int)t.k, v0, U, V);
        TriHit h;
        if (COUNT) cnt.tri++;
        if (tri_hit(v0, U, V, r, h)) {
            if (h.t < t.acc) t.acc = h.t;
            if (h.t < t.best.t) { t.best.t = h.t; t.best.u = h.u; t.best.v = h.v; t.best.prim = (int)t.k; }
        }
        t.k++;
        if (t.k < t.kend) return true;
        return trav_pop(sc, t, stk);
    }
    uint32_t left = t.nd.a;
    RT_CHECK((int)left + 1 < sc.n_nodes && t.nd.b < 3, 7, ((unsigned long long)t.nd.b << 32) | left, left = 0);
    RT_CHECK(t.sp >= 0 && t.sp < kStack, 8, t.sp, t.sp = 0);
    const float dsplit = t.nd.b == 0 ? r.d.x : (t.nd.b == 1 ? r.d.y : r.d.z);
    const bool left_first = dsplit > 0;
    float e;
    if (t.phase == 0) {
        const uint32_t c0 = left_first ? left : left + 1;
        const NodeRec cn = load_node(sc.node, c0);
        if (COUNT) cnt.aabb++;
        if (aabb_hit(cn.mn, cn.mx, r, e)) {
            stk[t.sp++] = make_uint2(t.cur | (1u << 31), __float_as_uint(t.acc));
            trav_enter(t, c0, cn);
            return true;
        }
    }
    const uint32_t c1 = left_first ? left + 1 : left;
    const NodeRec cn = load_node(sc.node, c1);
    if (COUNT) cnt.aabb++;
    if (aabb_hit(cn.mn, cn.mx, r, e) && !(e > t.acc)) {
        stk[t.sp++] = make_uint2(t.cur, __float_as_uint(t.acc));
        trav_enter(t, c1, cn);
        return true;
    }
    return trav_pop(sc, t, stk);
}

// ------------------------------------------------------------------------ wave lanes
// Pixel-row shard geometry (include/rt_hw.h rt_params): the k-th owned row of rank r is
// the k-th row whose (row / row_block) % world == rank.
struct ShardGeom {
    int width, rank, world, row_block;
    long long n_pixels;
};
__device__ __forceinline__ int shard_row(const ShardGeom &g, int k) {
    const int blk = k / g.row_block;
    return (blk * g.world + g.rank) * g.row_block + (k % g.row_block);
}

enum LaneState { L_IDLE = 0, L_TRAV = 1, L_SHADE = 2 };

// Everything one lane of the wave kernel carries between phases.
struct Lane {
    long long pix;   // owned pixel of the shard, -1 = none
    int s;           // samples done
    int state, power, nv;
    Rng rng;
    V3 sum;
    Ray r;
    Trav t;
    PathRec P;
    uint2 stk[kStack];
};

__device__ __forceinline__ void lane_init(Lane &L) {
    L.pix = -1;
    L.s = 0;
    L.state = L_IDLE;
    L.power = L.nv = 0;
    L.rng = Rng{1u, 0u, 0.f};
    L.sum = V3{0.f, 0.f, 0.f};
    L.t.best.prim = -1;
}

// (A) a new pixel: seed its RNG (scene.cpp:34, random.cpp:12-18; pixel 0 -> state 1)
__device__ __forceinline__ void lane_assign(Lane &L, const DevScene &sc, const ShardGeom &g, long long p) {
    L.pix = p;
    L.s = 0;
    L.sum = V3{0.f, 0.f, 0.f};
    const int k = (int)(p / g.width), i = (int)(p % g.width), j = shard_row(g, k);
    const uint32_t seed = (uint32_t)(j * sc.width + i) % 2147483647u;
    L.rng = Rng{seed == 0 ? 1u : seed, 0u, 0.f};
    L.state = L_IDLE;
}

// (B) start the next sample of the pixel: jittered camera ray (scene.cpp:36-39)
template <bool COUNT>
__device__ __forceinline__ void lane_start_sample(Lane &L, const DevScene &sc, const ShardGeom &g, Counters &cnt) {
    const int k = (int)(L.pix / g.width), i = (int)(L.pix % g.width), j = shard_row(g, k);
    const float ox = rng_offset(L.rng);
    const float oy = rng_offset(L.rng);
    L.r = camera_ray(sc, i, j, ox, oy);
    L.power = sc.ray_depth;
    L.nv = 0;
    L.state = L_SHADE;
    L.t.best.prim = -1;
    if (L.power > 0) {
        L.power -= 1;
        if (trav_begin<COUNT>(sc, L.r, L.t, cnt)) L.state = L_TRAV;
    }
}

// (D) shade the closest hit; bounce or end the path (fold, accumulate, maybe finish the pixel).
template <bool COUNT>
__device__ __forceinline__ void lane_shade(Lane &L, const DevScene &sc, int spp, float *out, Counters &cnt) {
    bool next = false;
    // scene.cpp:85: a hit counts only if closer than max_distance
    if (L.t.best.prim >= 0 && L.t.best.t < sc.max_distance &&
        shade_hit<COUNT>(sc, L.r, L.t.best, L.rng, cnt, L.P, L.nv)) {
        // the recursion continues with the bounce ray while calls remain (scene.cpp:72-75)
        if (L.power > 0) {
            L.power -= 1;
            next = trav_begin<COUNT>(sc, L.r, L.t, cnt);  // false: the child misses the scene
        }
    }
    if (next) {
        L.state = L_TRAV;
        return;
    }
    const V3 c = fold_path(L.P, L.nv);
    L.sum = rtv::add(L.sum, c);
    if (++L.s == spp) {
        RT_CHECK(L.pix >= 0, 9, L.pix, L.pix = 0);
        out[3 * L.pix + 0] = L.sum.x;
        out[3 * L.pix + 1] = L.sum.y;
        out[3 * L.pix + 2] = L.sum.z;
        L.pix = -1;
    }
    L.state = L_IDLE;
}

// trace_sample() with the stepped traversal (host tests check it equals closest_hit()).
template <bool COUNT>
__device__ V3 trace_sample_stepped(const DevScene &sc, Ray r, Rng &rng, Counters &cnt) {
    PathRec P;
    int nv = 0;
    int power = sc.ray_depth;
    uint2 stk[kStack];
    Trav t;
    while (power > 0) {
        power -= 1;
        if (trav_begin<COUNT>(sc, r, t, cnt))
            while (trav_step<COUNT>(sc, r, t, stk, cnt)) {
            }
        if (!(t.best.prim >= 0 && t.best.t < sc.max_distance)) break;
        if (!shade_hit<COUNT>(sc, r, t.best, rng, cnt, P, nv)) break;
    }
    return fold_path(P, nv);
}

}  // namespace rtd
