// rt_trav_wide.h — two-level traversal step: fewer dependent memory round trips per ray.
//
// BVH::intersect (bvh.cpp:177-243) with the reference's visits, counters and winner, as in
// trav_step (rt_wavefront.h), but each iteration of a lane does more of the ray:
//   * at an internal node N it reads N's child pair (L, R) AND the child pair of N's near
//     child X in the same round trip.  X is known before any box is tested: the reference
//     visits L first iff dir[split axis] > 0 (bvh.cpp:196-220), and N's record says where
//     X's children are (rt_bvh_layout.h wide_nodes, word c).  When the step enters X (its
//     box is hit) and X is internal, X's own node step runs in the same iteration from the
//     prefetched pair.  Both steps are the single-level node step of trav_step, in the same
//     order, with the same frames, so the composition changes nothing but the iteration
//     count; the box tests of both levels are computed up front (pure functions of ray and
//     box), so the second level adds little latency;
//   * at a leaf it tests two triangles per iteration (the reference's order, strict <).
// The loads of both phases go through the same 8 x 16 B of registers: a node lane reads two
// 64-B pairs, a leaf lane two 48-B triangles.
// Frames carry the far child's c word too (3 words): popping a far child enters it with
// the prefetch information of a node reached from its parent.
#pragma once
#include "rt_wavefront.h"

// A/B knobs: the second node level (RT_WIDE_NODE) and the second triangle (RT_WIDE_LEAF).
#ifndef RT_WIDE_NODE
#define RT_WIDE_NODE 1
#endif
#ifndef RT_WIDE_LEAF
#define RT_WIDE_LEAF 1
#endif

namespace rtd {

struct TravW {
    uint32_t ab, c;     // TP_NODE: node being entered, its packed (a << 10 | b) and c words
    uint32_t k, kend;   // TP_LEAF: triangles still to test
    float acc;          // best t inside the subtree being traversed (the reference's local best)
    int sp;
    int phase;
    Hit best;           // global winner so far (strict <, first of equal t wins)
};

__device__ __forceinline__ void wenter(TravW &T, uint32_t ab, uint32_t c) {
    const uint32_t a = ab >> 10, b = ab & 1023u;
    T.ab = ab;
    T.c = c;
    T.k = a;
    T.kend = a + (b >> 2);
    T.phase = b < 3u ? TP_NODE : (T.kend > T.k ? TP_LEAF : TP_POP);
}

// BVH::intersect entry (bvh.cpp:239-243): counters, root box result (bit 3 of bits = miss).
template <bool COUNT>
__device__ __forceinline__ bool trav_start_w(uint32_t bits, uint32_t root_ab, uint32_t root_c, TravW &T,
                                             Counters &cnt) {
    if (COUNT) { cnt.rays++; cnt.aabb++; }
    T.best.t = 1e9f;
    T.best.prim = -1;
    T.best.u = T.best.v = 0.f;
    T.sp = 0;
    T.acc = 1e9f;
    wenter(T, root_ab, root_c);
    return (bits & 8u) == 0;
}

// Host / test stack of 3-word frames.
struct ArrayStack3 {
    uint2 *p;
    uint32_t *c;
    __device__ __forceinline__ void put(int i, uint2 v, uint32_t cw) { p[i] = v; c[i] = cw; }
    __device__ __forceinline__ uint2 get(int i) const { return p[i]; }
    __device__ __forceinline__ uint32_t get_c(int i) const { return c[i]; }
};

// Box test results of one child pair, stored order.
struct PairHits {
    float cL[3], cR[3];
    bool inL, inR, hL, hR;
};
__device__ __forceinline__ void pair_hits(const float4 q0, const float4 q1, const float4 q2, const float4 q3, const Ray &r,
                                          PairHits &h) {
    const float mnL[3] = {q0.x, q0.y, q0.z}, mxL[3] = {q0.w, q1.x, q1.y};
    const float mnR[3] = {q2.x, q2.y, q2.z}, mxR[3] = {q2.w, q3.x, q3.y};
    h.hL = box_hit_pt(mnL, mxL, r, h.cL, h.inL);
    h.hR = box_hit_pt(mnR, mxR, r, h.cR, h.inR);
}

// The single-level node step of trav_step on the node being entered (T.ab), given its
// child pair's records (ab, c words) and box results.  Returns true when it entered the
// near child.
template <bool COUNT, class Stack>
__device__ __forceinline__ bool node_substep(TravW &T, uint32_t abL, uint32_t cL_, uint32_t abR, uint32_t cR_,
                                             const PairHits &h, const Ray &r, Stack &stk, Counters &cnt) {
    if (COUNT) cnt.aabb += 2;
    const uint32_t axis = T.ab & 1023u;
    const uint32_t dpos = (r.d.x > 0.f ? 1u : 0u) | (r.d.y > 0.f ? 2u : 0u) | (r.d.z > 0.f ? 4u : 0u);
    const bool lf = (dpos >> axis) & 1u;
    const bool hn = lf ? h.hL : h.hR, hf = lf ? h.hR : h.hL;
    float cF[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) cF[k] = lf ? h.cR[k] : h.cL[k];
    const float ef = box_dist(cF, lf ? h.inR : h.inL, r);
    const uint32_t nab = lf ? abL : abR, nc = lf ? cL_ : cR_;
    const uint32_t fab = lf ? abR : abL, fc = lf ? cR_ : cL_;
    if (hn && hf) {
        RT_CHECK(T.sp < kStack, 11, T.sp, T.sp = 0);
        stk.put(T.sp++, make_uint2(fab, __float_as_uint(ef)), fc);
#ifdef RT_STACK_PROBE
        RT_STACK_PROBE(T.sp);
#endif
    }
    const bool far_only = !hn && hf && !(ef > 1e9f);
    if (hn || far_only) wenter(T, hn ? nab : fab, hn ? nc : fc);
    else T.phase = TP_POP;
    return hn;
}

// One iteration of a lane's traversal (see the header comment).  Returns true once the
// stack is empty (T.best is final).  `node` is the wide node array (DevScene::node_w), `tri`
// the triangle array (padded by one triangle: a leaf lane reads 4 x 16 B per triangle).
template <bool COUNT, class Stack>
__device__ __forceinline__ bool trav_step_w(const DevScene &sc, const Ray &r, TravW &T, Stack &stk, Counters &cnt) {
    const bool at_node = T.phase == TP_NODE, at_leaf = T.phase == TP_LEAF;
    const uint32_t a = T.ab >> 10, axis = T.ab & 1023u;
    // near child X by direction alone, and where its children are
    const uint32_t dpos = (r.d.x > 0.f ? 1u : 0u) | (r.d.y > 0.f ? 2u : 0u) | (r.d.z > 0.f ? 4u : 0u);
    const bool lf = at_node && ((dpos >> axis) & 1u);
    const bool xint = RT_WIDE_NODE && at_node && (((T.c >> (lf ? 0 : 1)) & 1u) != 0u);
    const uint32_t xc = (T.c >> 2) + ((!lf && (T.c & 1u)) ? 2u : 0u);
    const uint32_t k = T.k, k1 = RT_WIDE_LEAF && k + 1 < T.kend ? k + 1 : k;
    const float4 *p0 = at_node ? sc.node_w + 2 * (size_t)a : sc.tri + 3 * (size_t)k;
    const float4 *p1 = at_node ? sc.node_w + 2 * (size_t)(xint ? xc : a) : sc.tri + 3 * (size_t)k1;
    RT_CHECK(!at_node || a + 1 < (uint32_t)sc.n_nodes, 10, a, p0 = sc.node_w);
    RT_CHECK(!at_node || !xint || xc + 1 < (uint32_t)sc.n_nodes, 13, xc, p1 = sc.node_w);
    RT_CHECK(!at_leaf || T.kend <= (uint32_t)sc.n_tris, 12, T.kend, p0 = p1 = sc.tri);
    float4 q[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = p0[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[4 + i] = p1[i];
    if (at_node) {
        PairHits h1, h2;
        pair_hits(q[0], q[1], q[2], q[3], r, h1);
        if (RT_WIDE_NODE) pair_hits(q[4], q[5], q[6], q[7], r, h2);   // X's children (used only if X is entered)
        const bool went_near = node_substep<COUNT>(T, __float_as_uint(q[1].z), __float_as_uint(q[1].w),
                                                   __float_as_uint(q[3].z), __float_as_uint(q[3].w), h1, r, stk, cnt);
        if (went_near && xint)   // T.ab is X now, an internal node: its step from the prefetched pair
            node_substep<COUNT>(T, __float_as_uint(q[5].z), __float_as_uint(q[5].w), __float_as_uint(q[7].z),
                                __float_as_uint(q[7].w), h2, r, stk, cnt);
    } else if (at_leaf) {
        TriHit h0, h1;
        const bool t0 = tri_hit_bl(V3{q[0].x, q[0].y, q[0].z}, V3{q[0].w, q[1].x, q[1].y}, V3{q[1].z, q[1].w, q[2].x}, r, h0);
        const bool t1 = RT_WIDE_LEAF && tri_hit_bl(V3{q[4].x, q[4].y, q[4].z}, V3{q[4].w, q[5].x, q[5].y}, V3{q[5].z, q[5].w, q[6].x}, r, h1);
        if (COUNT) cnt.tri++;
        if (t0) {
            T.acc = h0.t < T.acc ? h0.t : T.acc;
            if (h0.t < T.best.t) { T.best.t = h0.t; T.best.u = h0.u; T.best.v = h0.v; T.best.prim = (int)k; }
        }
        if (k1 != k) {
            if (COUNT) cnt.tri++;
            if (t1) {
                T.acc = h1.t < T.acc ? h1.t : T.acc;
                if (h1.t < T.best.t) { T.best.t = h1.t; T.best.u = h1.u; T.best.v = h1.v; T.best.prim = (int)k1; }
            }
        }
        T.k = k1 + 1;
        if (T.k >= T.kend) T.phase = TP_POP;
    }
    if (T.phase == TP_POP) {
        // return: merge subtree bests upwards until a far child is to be visited
        float acc = T.acc;
        int sp = T.sp;
        for (;;) {
            if (sp == 0) {
                T.sp = 0;
                T.acc = acc;
                return true;
            }
            const uint2 f = stk.get(--sp);
            if (f.x == kFrameAcc) {
                const float p = __uint_as_float(f.y);
                acc = acc < p ? acc : p;
                continue;
            }
            if (!(__uint_as_float(f.y) > acc)) {   // far child survives the near subtree's best
                const uint32_t fc = stk.get_c(sp);
                stk.put(sp++, make_uint2(kFrameAcc, __float_as_uint(acc)), 0u);
                T.sp = sp;
                T.acc = 1e9f;
                wenter(T, f.x, fc);
                return false;
            }
        }
    }
    return false;
}

#ifdef __HIPCC__
// Device stack of 3-word frames: the first kLdsStack in LDS (lane-interleaved as LdsStack),
// deeper ones in scratch.
__shared__ uint32_t wf_lds_stack_c[kLdsStack * 256];
struct LdsStack3 {
    uint2 *spill;
    uint32_t *spill_c;
    __device__ __forceinline__ void put(int i, uint2 v, uint32_t cw) {
        if (i < kLdsStack) {
            wf_lds_stack[i * 256 + threadIdx.x] = v;
            wf_lds_stack_c[i * 256 + threadIdx.x] = cw;
        } else {
            spill[i - kLdsStack] = v;
            spill_c[i - kLdsStack] = cw;
        }
    }
    __device__ __forceinline__ uint2 get(int i) const {
        uint2 v;
        if (i < kLdsStack) {
            v = wf_lds_stack[i * 256 + threadIdx.x];
        } else {
            v = spill[i - kLdsStack];
            asm volatile("" : "+v"(v.x), "+v"(v.y));
        }
        return v;
    }
    __device__ __forceinline__ uint32_t get_c(int i) const {
        uint32_t v;
        if (i < kLdsStack) {
            v = wf_lds_stack_c[i * 256 + threadIdx.x];
        } else {
            v = spill_c[i - kLdsStack];
            asm volatile("" : "+v"(v));
        }
        return v;
    }
};
#endif

}  // namespace rtd
