// rt_team.h — one ray traversed by a whole wave: the tail of a frame.
//
// A pixel's 256 samples are one sequential chain (each sample's RNG state depends on the draws
// of the one before), so once a wave is down to its last pixel — and with ~1 pixel per lane
// (an 8-way split of a 1080p frame) the frame ends on such waves — 63 lanes idle while one
// lane walks the BVH one node pair per iteration.  Here the whole wave walks that lane's ray:
//   * node pairs come in windows: the subtree of RT_TEAM_W pair levels below the current
//     node (2 + 4 + 8 nodes for W = 3), one node per lane, one dependent load per level;
//     every lane tests its own box (box_hit_pt / box_dist: the same operations as trav_step's
//     pair test, primitive.cpp:146-208);
//   * the depth-first walk itself is trav_step's (BVH::intersectHelper, bvh.cpp:177-243):
//     same near/far order, frames, culling and returns, on wave-uniform values, reading the
//     box results of the window instead of testing; a node whose pair is outside the window
//     starts a new window;
//   * a leaf's triangles are tested one per lane and reduced in the reference's order
//     (smallest t; of equal t the first triangle, as the strict < of the sequential loop).
// Visits and the winner are trav_step's; only the counters are not kept (counting renders
// never take this path).  Frames live in the wave's LDS stack columns: frame i at level
// i & 7 of column (owner + (i >> 3)) & 63, so frames 0-7 are the owner's own.
#pragma once
#include "rt_wavefront.h"

#ifndef RT_TEAM_W
#define RT_TEAM_W 3
#endif

namespace rtd {
#ifdef __HIPCC__

constexpr int kTeamSlots = (2 << RT_TEAM_W) - 2;   // window nodes: slot s's children at 2s + 2, 2s + 3
constexpr int kTeamInner = kTeamSlots / 2 - 1;     // slots whose children are in the window
static_assert(kTeamSlots <= 64, "one window node per lane");

__device__ __forceinline__ uint32_t team_u(uint32_t x, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)x, src); }
__device__ __forceinline__ float team_f(float x, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src)); }
__device__ __forceinline__ uint32_t team_first(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

struct TeamStack {
    int base, owner;   // the wave's first thread in the block, the owner's lane
    __device__ __forceinline__ uint2 *slot(int i) const {
        return &wf_lds_stack[(i & (kLdsStack - 1)) * 256 + base + ((owner + i / kLdsStack) & 63)];
    }
    __device__ __forceinline__ void put(int i, uint2 v, int lane) const {
        if (lane == 0) *slot(i) = v;
    }
    __device__ __forceinline__ uint2 get(int i) const {
        const uint2 v = *slot(i);
        return make_uint2(team_first(v.x), team_first(v.y));
    }
};
static_assert((kLdsStack & (kLdsStack - 1)) == 0, "team frames index LDS levels by mask");

// Per lane: window node `lane` (valid when its parent slot is an internal node).
struct TeamWindow {
    uint32_t a0;        // uniform: the child pair at slots 0, 1
    uint32_t na, nb;    // this lane's node: its a, b words
    bool valid, hit;
    float dist;         // entry distance (box_dist: 0 from inside)
};

// Load and test the window below child pair `a0` (RT_TEAM_W dependent loads).
__device__ __forceinline__ void team_window(const DevScene &sc, const Ray &r, uint32_t a0, int lane, TeamWindow &w) {
    w.a0 = a0;
    bool valid = lane < 2;
    uint32_t id = a0 + (uint32_t)(lane & 1);
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) { p = sc.node[2 * (size_t)id]; q = sc.node[2 * (size_t)id + 1]; }
    uint32_t na = __float_as_uint(q.z), nb = __float_as_uint(q.w);
#pragma unroll
    for (int lvl = 2; lvl <= RT_TEAM_W; ++lvl) {
        // slots of this level: [2^lvl - 2, 2^(lvl+1) - 2); parent slot (s - 2) / 2
        const int lo = (1 << lvl) - 2, hi = (2 << lvl) - 2;
        const int par = (lane - 2) >> 1;
        const int src = par < 0 ? 0 : par;
        const uint32_t pa = (uint32_t)__shfl((int)na, src, 64), pb = (uint32_t)__shfl((int)nb, src, 64);
        const bool pv = __shfl((int)valid, src, 64) != 0;
        if (lane >= lo && lane < hi) {
            valid = pv && pb < 3u;
            id = pa + (uint32_t)(lane & 1);
            if (valid) { p = sc.node[2 * (size_t)id]; q = sc.node[2 * (size_t)id + 1]; }
            na = __float_as_uint(q.z);
            nb = __float_as_uint(q.w);
        }
    }
    const float mn[3] = {p.x, p.y, p.z}, mx[3] = {p.w, q.x, q.y};
    float coord[3];
    bool inside;
    w.hit = box_hit_pt(mn, mx, r, coord, inside);
    w.dist = box_dist(coord, inside, r);
    w.na = na;
    w.nb = nb;
    w.valid = valid;
}

// Slot of child pair `a` in the window (its left node), or -1.
__device__ __forceinline__ int team_find(const TeamWindow &w, uint32_t a, int lane) {
    if (a == w.a0) return 0;
    const unsigned long long m = __ballot(lane < kTeamInner && w.valid && w.nb < 3u && w.na == a);
    return m ? 2 * (__ffsll((unsigned long long)m) - 1) + 2 : -1;
}

// The rest of the traversal of `T` (the owner lane's state, made uniform by the caller) by
// the whole wave.  T.sp frames must be in the owner's LDS column (T.sp <= kLdsStack).
__device__ __forceinline__ void trav_team(const DevScene &sc, const Ray &r, TravState &T, const TeamStack &stk,
                                          int lane) {
    const uint32_t dpos = (r.d.x > 0.f ? 1u : 0u) | (r.d.y > 0.f ? 2u : 0u) | (r.d.z > 0.f ? 4u : 0u);
    TeamWindow w;
    w.a0 = 0xffffffffu;
    w.valid = false;
    w.na = w.nb = 0u;
    bool have = false;
    for (;;) {
        if (T.phase == TP_NODE) {
            int ps = have ? team_find(w, T.a, lane) : -1;
            if (ps < 0) {
                team_window(sc, r, T.a, lane, w);
                have = true;
                ps = 0;
            }
            const bool hL = team_u((uint32_t)w.hit, ps) != 0u, hR = team_u((uint32_t)w.hit, ps + 1) != 0u;
            const uint32_t La = team_u(w.na, ps), Lb = team_u(w.nb, ps), Ra = team_u(w.na, ps + 1), Rb = team_u(w.nb, ps + 1);
            const bool lf = (dpos >> T.b) & 1u;
            const float ef = team_f(w.dist, lf ? ps + 1 : ps);   // the far child's entry distance
            const bool hn = lf ? hL : hR, hf = lf ? hR : hL;
            const uint32_t na = lf ? La : Ra, nb = lf ? Lb : Rb, fa = lf ? Ra : La, fb = lf ? Rb : Lb;
            if (hn && hf) stk.put(T.sp++, make_uint2((fa << 10) | fb, __float_as_uint(ef)), lane);
            const bool far_only = !hn && hf && !(ef > 1e9f);
            if (hn || far_only) trav_enter(T, hn ? na : fa, hn ? nb : fb);
            else T.phase = TP_POP;
        } else if (T.phase == TP_LEAF) {
            // triangles k .. kend - 1, one per lane, 64 at a time
            const uint32_t k = T.k + (uint32_t)lane;
            const bool valid = k < T.kend;
            const float4 *t = sc.tri + 3 * (size_t)(valid ? k : T.k);
            const float4 a = t[0], b = t[1], c = t[2];
            TriHit h;
            const bool hit = tri_hit_bl(V3{a.x, a.y, a.z}, V3{a.w, b.x, b.y}, V3{b.z, b.w, c.x}, r, h) & valid;
            // a NaN t passes tri_hit's tests but never updates acc or the best hit
            float key = (hit && h.t == h.t) ? h.t : __builtin_inff();
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const float o = __shfl_xor(key, off, 64);
                key = o < key ? o : key;
            }
            const float tmin = team_f(key, 0);
            if (tmin < __builtin_inff()) {
                const unsigned long long m = __ballot(hit && h.t == tmin);
                const int win = __ffsll((unsigned long long)m) - 1;   // the first of equal t
                T.acc = tmin < T.acc ? tmin : T.acc;
                if (tmin < T.best.t) {
                    T.best.t = tmin;
                    T.best.u = team_f(h.u, win);
                    T.best.v = team_f(h.v, win);
                    T.best.prim = (int)(T.k + (uint32_t)win);
                }
            }
            T.k += 64u;
            if (T.k >= T.kend) T.phase = TP_POP;
        }
        if (T.phase == TP_POP) {
            // trav_pop on the team stack
            float acc = T.acc;
            int sp = T.sp;
            bool done = false;
            for (;;) {
                if (sp == 0) {
                    done = true;
                    break;
                }
                const uint2 f = stk.get(--sp);
                if (f.x == kFrameAcc) {
                    const float pv = __uint_as_float(f.y);
                    acc = acc < pv ? acc : pv;
                    continue;
                }
                if (!(__uint_as_float(f.y) > acc)) {
                    stk.put(sp++, make_uint2(kFrameAcc, __float_as_uint(acc)), lane);
                    T.acc = 1e9f;
                    trav_enter(T, f.x >> 10, f.x & 1023u);
                    break;
                }
            }
            T.sp = sp;
            if (done) {
                T.acc = acc;
                return;
            }
        }
    }
}
#endif

}  // namespace rtd
