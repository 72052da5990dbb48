// rt_mega.h — lane-resident path tracer (kernel 0, the default).
//
// The wavefront (rt_wavefront.h) advances every path one bounce per launch pair, so each
// iteration costs as much as the slowest ray of the whole frame; with few paths per GPU
// (a 1080p frame split over 8 GPUs leaves ~260 k pixels each, about one per lane) the
// frame time becomes the sum over ~1500 iterations of that maximum.  The wavefront is
// kernel 4.  Here every lane owns
// one pixel at a time and runs its whole sample loop (scene.cpp:34-42) itself, so a path
// only ever waits for its own rays:
//   * traversal advances every traversing lane of a wave by one unit per iteration
//     (trav_step: one node pair or one triangle, as in the extend kernel);
//   * lanes whose closest hit is known wait (READY) until `shade_min` lanes of the wave are
//     ready, or no lane is traversing, and are then shaded together (one pass of the long
//     shading code serves many lanes);
//   * a lane whose pixel has all its samples takes the next pixel from a per-launch queue.
// RNG, pixel sum, sample counter and depth budget live in registers; the vertex records go
// to memory (LaneRec, indexed by lane slot).  Same per-pixel arithmetic, so bit-identical output.
#pragma once
#include "rt_wavefront.h"

namespace rtd {

// The lane's slot: its global thread index (the host emulation sets it per lane).
#if defined(__HIPCC__)
__device__ __forceinline__ long long mega_slot() { return (long long)blockIdx.x * blockDim.x + threadIdx.x; }
#else
inline thread_local long long g_mega_slot = 0;
inline long long mega_slot() { return g_mega_slot; }
#endif

using MegaTrav = TravState;
__device__ __forceinline__ const float4 *mega_nodes(const DevScene &sc) { return sc.node; }

// M_LTRAV / M_LREADY: light-pdf walk as its own traversal (light-split kernel, below)
enum MegaState : int { M_IDLE = 0, M_TRAV = 1, M_READY = 2, M_LTRAV = 3, M_LREADY = 4 };

struct MegaLane {
    int pix;         // shard pixel (slot), -1 = none (the host keeps shards below 2^31 pixels)
    uint32_t ctr;    // LaneCtr packed: sample (bits 0-19), depth budget (20-23), vertices (24-28)
    int state;
    // fast mode only (RT_FLAG_FAST): work unit = samples [s, send) of the pixel; its partial
    // sum goes to dst; gpix = j*W+i keys the per-sample Philox seed.  Unused fields of the
    // parity kernel are dropped by the compiler.
    int send;
    uint32_t gpix;
    long long dst;
    unsigned long long work0;   // counting runs: traversal tests before this work unit (its cost)
    Rng rng;
    V3 sum;
    Ray r;
    MegaTrav T;
};

// The lane's pixel sum lives in LDS (3 KB per block) instead of three VGPRs that stay live
// through the shading code; with the RNG state below in LDS too: 30 -> 17 spilled VGPRs at
// the 96-VGPR budget, 1478 -> 1517 Mrays/s at 1080p x256spp, 8-way shard 325 -> 318 ms.
#if defined(__HIPCC__)
__shared__ float mega_lds_sum[3 * 256];
__device__ __forceinline__ V3 lane_sum(const MegaLane &) {
    const int t = threadIdx.x;
    return V3{mega_lds_sum[t], mega_lds_sum[256 + t], mega_lds_sum[512 + t]};
}
__device__ __forceinline__ void lane_sum_set(MegaLane &, V3 v) {
    const int t = threadIdx.x;
    mega_lds_sum[t] = v.x;
    mega_lds_sum[256 + t] = v.y;
    mega_lds_sum[512 + t] = v.z;
}
#else
__device__ __forceinline__ V3 lane_sum(const MegaLane &L) { return L.sum; }
__device__ __forceinline__ void lane_sum_set(MegaLane &L, V3 v) { L.sum = v; }
#endif

// The lane's RNG state (minstd word, normal cache) lives in LDS between its uses (sample
// start, shading), 3 KB per block, instead of three VGPRs held through the traversal.
#if defined(__HIPCC__)
__shared__ uint32_t mega_lds_rng[3 * 256];
__device__ __forceinline__ Rng lane_rng(const MegaLane &) {
    const int t = threadIdx.x;
    return Rng{mega_lds_rng[t], mega_lds_rng[256 + t], __uint_as_float(mega_lds_rng[512 + t])};
}
__device__ __forceinline__ void lane_rng_set(MegaLane &, const Rng &r) {
    const int t = threadIdx.x;
    mega_lds_rng[t] = r.x;
    mega_lds_rng[256 + t] = r.saved_avail;
    mega_lds_rng[512 + t] = __float_as_uint(r.saved);
}
#else
__device__ __forceinline__ Rng lane_rng(const MegaLane &L) { return L.rng; }
__device__ __forceinline__ void lane_rng_set(MegaLane &L, const Rng &r) { L.rng = r; }
#endif

// The lane's sample counter, depth budget and recorded-vertex count, packed in one register
// (samples < 2^20, ray_depth <= 15, vertices <= 16: checked by the host) so the loop state
// that stays live through the shading code is two registers smaller.
struct LaneCtr {
    int s, power, nv;
};
__device__ __forceinline__ LaneCtr lane_ctr(const MegaLane &L) {
    return LaneCtr{(int)(L.ctr & 0xfffffu), (int)((L.ctr >> 20) & 15u), (int)(L.ctr >> 24)};
}
__device__ __forceinline__ void lane_ctr_set(MegaLane &L, const LaneCtr &c) {
    L.ctr = (uint32_t)c.s | (uint32_t)c.power << 20 | (uint32_t)c.nv << 24;
}

// Closest-hit query start for L.r: BVH::intersect's counters and root box (bvh.cpp:239-243).
template <bool COUNT>
__device__ __forceinline__ void mega_begin(MegaLane &L, const NodeRec &root, Counters &cnt) {
    float e;
    const bool hit = box_hit<false>(root.mn, root.mx, L.r, e);
    const uint32_t bits = (L.r.d.x > 0 ? 1u : 0u) | (L.r.d.y > 0 ? 2u : 0u) | (L.r.d.z > 0 ? 4u : 0u) | (hit ? 0u : 8u);
    L.state = trav_start<COUNT>(bits, root.a, root.b, L.T, cnt) ? M_TRAV : M_READY;
}

// Next sample of the lane's pixel: jittered camera ray (scene.cpp:36-39).  Fast mode: the
// sample's own Philox-seeded stream (rt_path.h fast_sample_seed).
template <bool COUNT, bool FAST = false>
__device__ __forceinline__ void mega_sample(MegaLane &L, const DevScene &sc, const ShardGeom &g, const NodeRec &root,
                                            Counters &cnt) {
    LaneCtr c = lane_ctr(L);
    Rng rng = FAST ? Rng{fast_sample_seed(L.gpix, (uint32_t)c.s), 0u, 0.f} : lane_rng(L);
    {   // start_sample (rt_wavefront.h) with 32-bit pixel arithmetic
        const int k = L.pix / g.width, px = L.pix - k * g.width, py = shard_row(g, k);
        const float ox = rng_offset(rng);
        const float oy = rng_offset(rng);
        c.power = sc.ray_depth - 1;
        L.r = camera_ray(sc, px, py, ox, oy);
    }
    lane_rng_set(L, rng);
    c.nv = 0;
    lane_ctr_set(L, c);
    mega_begin<COUNT>(L, root, cnt);
}

// A new pixel: seed its RNG (scene.cpp:34, random.cpp:12-18; pixel 0 -> 1), first sample.
template <bool COUNT>
__device__ __forceinline__ void mega_assign(MegaLane &L, const DevScene &sc, const ShardGeom &g, int p,
                                            const NodeRec &root, Counters &cnt) {
    L.pix = p;
    lane_ctr_set(L, LaneCtr{0, 0, 0});
    lane_sum_set(L, V3{0.f, 0.f, 0.f});
    L.work0 = cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri;
    const int k = p / g.width, px = p - k * g.width, py = shard_row(g, k);
    const uint32_t seed = (uint32_t)(py * sc.width + px) % 2147483647u;
    lane_rng_set(L, Rng{seed == 0 ? 1u : seed, 0u, 0.f});
    mega_sample<COUNT>(L, sc, g, root, cnt);
}

// Fast mode: queue item q = chunk * n_pixels + pixel (every pixel's first chunk, then the
// second, ...: neighbouring lanes take neighbouring pixels); samples [chunk*cs, +cs) of the
// pixel, partial sum to slot q of the chunk-major partial buffer.
template <bool COUNT>
__device__ __forceinline__ void mega_assign_fast(MegaLane &L, const DevScene &sc, const ShardGeom &g, long long q,
                                                 int cs, int spp, const NodeRec &root, Counters &cnt) {
    const long long c = q / g.n_pixels;
    const int p = (int)(q - c * g.n_pixels);
    L.pix = p;
    L.dst = q;
    const int s0 = (int)c * cs;
    lane_ctr_set(L, LaneCtr{s0, 0, 0});
    L.send = s0 + cs < spp ? s0 + cs : spp;
    lane_sum_set(L, V3{0.f, 0.f, 0.f});
    L.work0 = cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri;
    const int k = p / g.width, px = p - k * g.width, py = shard_row(g, k);
    L.gpix = (uint32_t)(py * sc.width + px);
    mega_sample<COUNT, true>(L, sc, g, root, cnt);
}

// Shade the lane's closest hit (one vertex of scene.cpp:85-154); bounce, or end the path:
// fold, accumulate, next sample or pixel done.
template <bool COUNT, bool FAST = false, class Stack>
__device__ __forceinline__ void mega_shade(MegaLane &L, const DevScene &sc, const ShardGeom &g, const WfState &st,
                                           int spp, float *out, unsigned *cost, const NodeRec &root, Stack &stk,
                                           Counters &cnt) {
    LaneRec P{st.rec_ab, st.rec_ab + st.lanes * st.D, st.rec_c, mega_slot(), st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
    const Hit h = L.T.best;
    LaneCtr c = lane_ctr(L);
    bool next = false;
    if (h.prim >= 0 && h.t < sc.max_distance) {
        Rng rng = lane_rng(L);
        const bool cont = shade_hit<COUNT>(sc, L.r, h, rng, cnt, P, c.nv, stk);   // (stack free: T.sp == 0)
        lane_rng_set(L, rng);
        if (cont && c.power > 0) {
            c.power -= 1;
            next = true;
        }
    }
    P.flush_e();
    if (next) {
        lane_ctr_set(L, c);
        mega_begin<COUNT>(L, root, cnt);
        return;
    }
    const V3 sm = rtv::add(lane_sum(L), fold_path(P, c.nv));
    lane_sum_set(L, sm);
    if (++c.s == (FAST ? L.send : spp)) {
        const long long o = FAST ? L.dst : L.pix;
        out[3 * o + 0] = sm.x;
        out[3 * o + 1] = sm.y;
        out[3 * o + 2] = sm.z;
        if (COUNT && cost) cost[L.pix] = (unsigned)(cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri - L.work0);
        L.pix = -1;
        L.state = M_IDLE;
        return;
    }
    lane_ctr_set(L, c);
    mega_sample<COUNT, FAST>(L, sc, g, root, cnt);
}

// ---------------------------------------------------------------- light-split kernel
// ManyLightsDistribution::pdf (random.cpp:179-188) walks the light BVH
// with BVH::intersectAll (bvh.cpp:245-279) at every shading event.  With many emissive
// triangles (C1: 1,152, 21.5 box + 11.5 triangle tests per walk) that walk is a second
// traversal; inline in the shading batch it runs with the batch's lanes in lockstep and
// holds the wave until the longest walk ends.  The light-split kernel runs it as a lane
// state instead: shade_pre, then M_LTRAV (one light-BVH node per iteration, interleaved with
// other lanes' scene traversal), then M_LREADY and shade_post in a later shading batch.
// The shading state that crosses the walk is a lane-slot record (WfState::mid, 5 planes of
// float4): (pos, r2) (N, metallic) (dir, mesh) (incoming dir, tc.x) (tc.y).  The walk reuses
// the lane's traversal stack (empty once its closest hit is known) and TravState: sp, and
// acc as the pdf sum.  Same operations in the same order as light_pdf, so the same bits.

// One node of the walk: pop; a leaf sums its triangles' pdf terms in index order, an
// internal node pushes the children whose boxes the ray hits (right, then left: left is
// visited first).  `dir_rec` holds the un-normalized sample direction (light_pdf's
// `direction`).  Returns true when the stack is empty.
template <bool COUNT, class Stack>
__device__ __forceinline__ bool light_step(const DevScene &sc, const Ray &r, TravState &T, Stack &stk, Counters &cnt,
                                           const float4 *dir_rec) {
    const uint32_t id = stk.get(--T.sp).x;
    const NodeRec nd = load_node(sc.light_node, id);
    if ((nd.b & 3u) == 3u) {
        const uint32_t first = nd.a, count = nd.b >> 2;
        for (uint32_t k = first; k < first + count; ++k) {
            const float4 a = sc.light[4 * k], b = sc.light[4 * k + 1], c = sc.light[4 * k + 2], w = sc.light[4 * k + 3];
            TriHit h;
            if (COUNT) cnt.ltri++;
            if (tri_hit(V3{a.x, a.y, a.z}, V3{a.w, b.x, b.y}, V3{b.z, b.w, c.x}, r, h)) {
                V3 n{c.y, c.z, c.w};
                if (rtv::dot(r.d, n) > 0) n = rtv::neg(n);
                const float4 dq = *dir_rec;
                const float probability = 1.f / w.x;   // 1 / triangle_area (random.cpp:88)
                T.acc += fabsf(probability * (h.t * h.t) / rtv::dot(n, V3{dq.x, dq.y, dq.z}));
            }
        }
    } else {
        const uint32_t left = nd.a;
        float e;
        const NodeRec l = load_node(sc.light_node, left), rr = load_node(sc.light_node, left + 1);
        if (COUNT) cnt.laabb += 2;
        const bool hl = aabb_hit(l.mn, l.mx, r, e);
        const bool hr = aabb_hit(rr.mn, rr.mx, r, e);
        RT_CHECK(T.sp + 2 <= kStack, 13, T.sp, T.sp = 0);
        if (hr) stk.put(T.sp++, make_uint2(left + 1, 0u));
        if (hl) stk.put(T.sp++, make_uint2(left, 0u));
    }
    return T.sp == 0;
}

// Shading of the light-split kernel: a READY lane runs shade_pre and starts its light walk
// (or, without lights, finishes the vertex); an LREADY lane finishes the vertex with the
// walked pdf.  The rest is mega_shade's: bounce, or fold and next sample / pixel.
template <bool COUNT, bool FAST, class Stack>
__device__ __forceinline__ void mega_shade_split(MegaLane &L, const DevScene &sc, const ShardGeom &g,
                                                 const WfState &st, int spp, float *out, unsigned *cost,
                                                 const NodeRec &root, Stack &stk, Counters &cnt) {
    const long long slot = mega_slot();
    LaneRec P{st.rec_ab, st.rec_ab + st.lanes * st.D, st.rec_c, slot, st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
    float4 *mid = st.mid + slot;
    const long long ln = st.lanes;
    LaneCtr c = lane_ctr(L);
    bool next = false;
    if (L.state == M_READY) {
        const Hit h = L.T.best;
        ShadeMid m;
        bool pre = false;
        if (h.prim >= 0 && h.t < sc.max_distance) {
            Rng rng = lane_rng(L);
            pre = shade_pre<COUNT>(sc, L.r, h, rng, cnt, P, c.nv, m);
            lane_rng_set(L, rng);
        }
        if (pre) {
            if (sc.n_lights) {
                P.flush_e();
                mid[0] = make_float4(m.pos.x, m.pos.y, m.pos.z, m.r2);
                mid[ln] = make_float4(m.N.x, m.N.y, m.N.z, m.metallic);
                mid[2 * ln] = make_float4(m.dir.x, m.dir.y, m.dir.z, __int_as_float(m.mesh));
                mid[3 * ln] = make_float4(L.r.d.x, L.r.d.y, L.r.d.z, m.tc.x);
                mid[4 * ln] = make_float4(m.tc.y, 0.f, 0.f, 0.f);
                if (COUNT) cnt.lq++;
                L.r = make_ray(m.pos, m.dir);   // light_pdf's Ray(point, direction)
                L.T.acc = 0.f;
                L.T.sp = 0;
                stk.put(L.T.sp++, make_uint2(0u, 0u));
                L.state = M_LTRAV;
                lane_ctr_set(L, c);
                return;
            }
            next = shade_post(sc, L.r.d, m, scene_pdf_lp(sc, m.N, rtv::neg(L.r.d), m.r2, m.dir, 0.f), P, c.nv, L.r) &&
                   c.power > 0;
        }
    } else {   // M_LREADY
        const float4 q0 = mid[0], q1 = mid[ln], q2 = mid[2 * ln], q3 = mid[3 * ln], q4 = mid[4 * ln];
        ShadeMid m;
        m.pos = V3{q0.x, q0.y, q0.z};
        m.r2 = q0.w;
        m.N = V3{q1.x, q1.y, q1.z};
        m.metallic = q1.w;
        m.dir = V3{q2.x, q2.y, q2.z};
        m.mesh = __float_as_int(q2.w);
        m.tc = V2{q3.w, q4.x};
        const V3 rd{q3.x, q3.y, q3.z};
        P.set_e(c.nv - 1, P.get_e(c.nv - 1));
        const float lp = L.T.acc / (float)sc.n_lights;
        next = shade_post(sc, rd, m, scene_pdf_lp(sc, m.N, rtv::neg(rd), m.r2, m.dir, lp), P, c.nv, L.r) && c.power > 0;
    }
    if (next) c.power -= 1;
    P.flush_e();
    if (next) {
        lane_ctr_set(L, c);
        mega_begin<COUNT>(L, root, cnt);
        return;
    }
    const V3 sm = rtv::add(lane_sum(L), fold_path(P, c.nv));
    lane_sum_set(L, sm);
    if (++c.s == (FAST ? L.send : spp)) {
        const long long o = FAST ? L.dst : L.pix;
        out[3 * o + 0] = sm.x;
        out[3 * o + 1] = sm.y;
        out[3 * o + 2] = sm.z;
        if (COUNT && cost) cost[L.pix] = (unsigned)(cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri - L.work0);
        L.pix = -1;
        L.state = M_IDLE;
        return;
    }
    lane_ctr_set(L, c);
    mega_sample<COUNT, FAST>(L, sc, g, root, cnt);
}

// One iteration of a wave's main loop for one lane, given the wave's decision: shade the
// READY lanes this iteration (shade_now), or step the traversing lanes.
template <bool COUNT, class Stack, class Nodes, bool FAST = false, bool LSPLIT = false>
__device__ __forceinline__ void mega_iterate(MegaLane &L, bool shade_now, const DevScene &sc, const ShardGeom &g,
                                             const WfState &st, int spp, float *out, unsigned *cost,
                                             const NodeRec &root, Stack &stk, const Nodes &nodes, Counters &cnt) {
    if constexpr (LSPLIT) {
        if (shade_now) {
            if (L.state == M_READY || L.state == M_LREADY)
                mega_shade_split<COUNT, FAST>(L, sc, g, st, spp, out, cost, root, stk, cnt);
            return;
        }
        if (L.state == M_LTRAV) {
            if (light_step<COUNT>(sc, L.r, L.T, stk, cnt, st.mid + 2 * st.lanes + mega_slot())) L.state = M_LREADY;
            return;
        }
    }
    if (shade_now) {
        if (L.state == M_READY) mega_shade<COUNT, FAST>(L, sc, g, st, spp, out, cost, root, stk, cnt);
    } else if (L.state == M_TRAV) {
        if (trav_step<COUNT>(sc, L.r, L.T, stk, nodes, cnt)) L.state = M_READY;
    }
}

}  // namespace rtd
