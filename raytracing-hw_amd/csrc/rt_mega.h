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
#if !defined(__HIPCC__)
#include <algorithm>   // (host emulation of wave_order)
#endif

namespace rtd {

// The lane's slot: its global thread index (the host emulation sets it per lane).
#if defined(__HIPCC__)
__device__ __forceinline__ long long mega_slot() { return (long long)blockIdx.x * blockDim.x + threadIdx.x; }
#else
inline thread_local long long g_mega_slot = 0;
inline long long mega_slot() { return g_mega_slot; }
#endif

__device__ __forceinline__ const float4 *mega_nodes(const DevScene &sc) { return sc.node; }

// M_LTRAV / M_LREADY: light-pdf walk as its own traversal (light-split kernel, below).
// M_DONE_NEW / M_DONE: a runahead job whose sample has ended, holding its colour and end
// state until its pixel's frontier reaches it (speculative runahead, below).
enum MegaState : int { M_IDLE = 0, M_TRAV = 1, M_READY = 2, M_LTRAV = 3, M_LREADY = 4, M_DONE_NEW = 5, M_DONE = 6 };
static_assert(M_DONE < 8, "rt_mega_kernel packs a lane's state in 3 bits (RT_PACK_TRAV)");

template <class TS>
struct MegaLaneT {
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
    TS T;
    uint32_t wbase;   // threadIdx.x of the wave's lane 0 (uniform: an SGPR; RT_TID_REMAT)
};
// The runahead kernel's lanes (and the host harness's spec emulation) keep TravState; the
// lane-resident kernel's TravStateU (rt_wavefront.h).
using MegaLane = MegaLaneT<TravState>;
using MegaLaneU = MegaLaneT<TravStateU>;

// The lane's pixel sum lives in LDS (3 KB per block) instead of three VGPRs that stay live
// through the shading code; with the RNG state below in LDS too: 30 -> 17 spilled VGPRs at
// the 96-VGPR budget, 1478 -> 1517 Mrays/s at 1080p x256spp, 8-way shard 325 -> 318 ms.
#if defined(__HIPCC__)
// RT_TID_REMAT: the lane's index in its block is recomputed where it is used (the wave's base
// in an SGPR | mbcnt), not held: the compiler computes threadIdx-based LDS addresses and slot
// indices once at kernel entry and keeps them, per lane, in VGPRs through the whole kernel
// (spilled, as loop invariants, at the register peak of the shading pass).  The mbcnt pair is
// in a volatile asm so that it is neither hoisted nor merged.
#ifndef RT_TID_REMAT
#define RT_TID_REMAT 1   // 0: A/B (profiles/r05n_ab.jsonl: 1074.9-1078.9 ms alone, 1037.9-1040.6 with RT_PACK_TRAV)
#endif
constexpr bool kTidRemat = RT_TID_REMAT != 0;
__device__ __forceinline__ uint32_t lane_id_fresh() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
template <class ML>
__device__ __forceinline__ int lane_tid(const ML &L) {
    if constexpr (kTidRemat) return (int)(L.wbase | lane_id_fresh());
    else return (int)threadIdx.x;
}
template <class ML>
__device__ __forceinline__ long long mega_slot_of(const ML &L) {
    return (long long)blockIdx.x * blockDim.x + lane_tid(L);
}
__shared__ float mega_lds_sum[3 * 256];
template <class ML>
__device__ __forceinline__ V3 lane_sum(const ML &L) {
    const int t = lane_tid(L);
    return V3{mega_lds_sum[t], mega_lds_sum[256 + t], mega_lds_sum[512 + t]};
}
template <class ML>
__device__ __forceinline__ void lane_sum_set(ML &L, V3 v) {
    const int t = lane_tid(L);
    mega_lds_sum[t] = v.x;
    mega_lds_sum[256 + t] = v.y;
    mega_lds_sum[512 + t] = v.z;
}
#else
template <class ML>
inline long long mega_slot_of(const ML &) { return mega_slot(); }
template <class ML>
__device__ __forceinline__ V3 lane_sum(const ML &L) { return L.sum; }
template <class ML>
__device__ __forceinline__ void lane_sum_set(ML &L, V3 v) { L.sum = v; }
#endif

// The lane's RNG state (minstd word, normal cache) lives in LDS between its uses (sample
// start, shading), 2 KB per block, instead of three VGPRs held through the traversal.  The
// minstd word is below 2^31 (modulus 2^31 - 1), so the cache flag (0 or 1) rides in its top
// bit (rt_device_selfcheck 1 checks the round trip): the kilobyte saved, with the computed
// linear texel decode's, pays for a twelfth LDS stack frame.
__device__ __forceinline__ uint32_t rng_word_pack(uint32_t x, uint32_t saved_avail) { return x | saved_avail << 31; }
__device__ __forceinline__ void rng_word_unpack(uint32_t w, uint32_t &x, uint32_t &saved_avail) {
    x = w & 0x7fffffffu;
    saved_avail = w >> 31;
}
#if defined(__HIPCC__)
__shared__ uint32_t mega_lds_rng[2 * 256];
template <class ML>
__device__ __forceinline__ Rng lane_rng(const ML &L) {
    const int t = lane_tid(L);
    Rng r;
    rng_word_unpack(mega_lds_rng[t], r.x, r.saved_avail);
    r.saved = __uint_as_float(mega_lds_rng[256 + t]);
    return r;
}
template <class ML>
__device__ __forceinline__ void lane_rng_set(ML &L, const Rng &r) {
    const int t = lane_tid(L);
    mega_lds_rng[t] = rng_word_pack(r.x, r.saved_avail);
    mega_lds_rng[256 + t] = __float_as_uint(r.saved);
}
#else
template <class ML>
__device__ __forceinline__ Rng lane_rng(const ML &L) { return L.rng; }
template <class ML>
__device__ __forceinline__ void lane_rng_set(ML &L, const Rng &r) { L.rng = r; }
#endif

// The lane's sample counter, depth budget and recorded-vertex count, packed in one register
// (samples < 2^20, ray_depth <= 15, vertices <= 16: checked by the host) so the loop state
// that stays live through the shading code is two registers smaller.
struct LaneCtr {
    int s, power, nv;
};
template <class ML>
__device__ __forceinline__ LaneCtr lane_ctr(const ML &L) {
    return LaneCtr{(int)(L.ctr & 0xfffffu), (int)((L.ctr >> 20) & 15u), (int)(L.ctr >> 24)};
}
template <class ML>
__device__ __forceinline__ void lane_ctr_set(ML &L, const LaneCtr &c) {
    L.ctr = (uint32_t)c.s | (uint32_t)c.power << 20 | (uint32_t)c.nv << 24;
}

// Closest-hit query start for L.r: BVH::intersect's counters and root box (bvh.cpp:239-243).
template <bool COUNT, class ML>
__device__ __forceinline__ void mega_begin(ML &L, const NodeRec &root, Counters &cnt) {
    float e;
    const bool hit = box_hit<false>(root.mn, root.mx, L.r, e);
    const uint32_t bits = (L.r.d.x > 0 ? 1u : 0u) | (L.r.d.y > 0 ? 2u : 0u) | (L.r.d.z > 0 ? 4u : 0u) | (hit ? 0u : 8u);
    L.state = trav_start<COUNT>(bits, root.a, root.b, L.T, cnt) ? M_TRAV : M_READY;
}

// Next sample of the lane's pixel: jittered camera ray (scene.cpp:36-39).  Fast mode: the
// sample's own Philox-seeded stream (rt_path.h fast_sample_seed).
template <bool COUNT, bool FAST = false, class ML>
__device__ __forceinline__ void mega_sample(ML &L, const DevScene &sc, const ShardGeom &g, const NodeRec &root,
                                            Counters &cnt) {
    LaneCtr c = lane_ctr(L);
    Rng rng = FAST ? Rng{fast_sample_seed(L.gpix, (uint32_t)c.s), 0u, 0.f} : lane_rng(L);
    {   // start_sample (rt_wavefront.h) with 32-bit pixel arithmetic
        int px, py;
        shard_xy(g, L.pix, px, py);
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

// A parked pixel: (pixel, next sample, start state of that sample, sum so far)
struct Parked {
    uint32_t pix, s;
    Rng x;
    V3 sum;
};
__device__ __forceinline__ Parked parked(const uint4 *park, long long k) {
    const uint4 a = park[2 * k], b = park[2 * k + 1];
    Parked q;
    q.pix = a.x;
    q.s = a.y;
    rng_word_unpack(a.z, q.x.x, q.x.saved_avail);
    q.x.saved = __uint_as_float(a.w);
    q.sum = V3{__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)};
    return q;
}

// The RNG state shard pixel p's sample 0 starts from: minstd_rand seeded with the pixel
// index (scene.cpp:34, random.cpp:12-18; pixel 0 -> 1).
__device__ __forceinline__ Rng pixel_seed(const DevScene &sc, const ShardGeom &g, int p) {
    int px, py;
    shard_xy(g, p, px, py);
    const uint32_t seed = (uint32_t)(py * sc.width + px) % 2147483647u;
    return Rng{seed == 0 ? 1u : seed, 0u, 0.f};
}

// A new pixel: seed its RNG, first sample.
template <bool COUNT, class ML>
__device__ __forceinline__ void mega_assign(ML &L, const DevScene &sc, const ShardGeom &g, int p,
                                            const NodeRec &root, Counters &cnt) {
    L.pix = p;
    lane_ctr_set(L, LaneCtr{0, 0, 0});
    lane_sum_set(L, V3{0.f, 0.f, 0.f});
    L.work0 = cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri;
    lane_rng_set(L, pixel_seed(sc, g, p));
    mega_sample<COUNT>(L, sc, g, root, cnt);
}

// A parked pixel (hand-off): its next sample from its parked state, onto its parked sum.
template <class ML>
__device__ __forceinline__ void mega_resume(ML &L, const DevScene &sc, const ShardGeom &g, const Parked &q,
                                            const NodeRec &root) {
    L.pix = (int)q.pix;
    lane_ctr_set(L, LaneCtr{(int)q.s, 0, 0});
    lane_sum_set(L, q.sum);
    lane_rng_set(L, q.x);
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    mega_sample<false>(L, sc, g, root, cnt);
}

// Fast mode: queue item q = chunk * n_pixels + pixel (every pixel's first chunk, then the
// second, ...: neighbouring lanes take neighbouring pixels); samples [chunk*cs, +cs) of the
// pixel, partial sum to slot q of the chunk-major partial buffer.
template <bool COUNT, class ML>
__device__ __forceinline__ void mega_assign_fast(ML &L, const DevScene &sc, const ShardGeom &g, long long q,
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
    int px, py;
    shard_xy(g, p, px, py);
    L.gpix = (uint32_t)(py * sc.width + px);
    mega_sample<COUNT, true>(L, sc, g, root, cnt);
}

// Hand-off (rt_device.hip RT_HANDOFF): a pixel whose next sample is s, whose RNG is at the
// state sample s starts from and whose sum holds samples 0 .. s-1, written to the park list
// (one atomic per wave: every lane that parks in the same pass of the wave), and resumed by
// the runahead kernel from exactly that state: its remaining samples run in order from it and
// add to that sum, so the bits do not change.
// The park list: 2 x uint4 per lane slot of the parking launch (pixel, next sample, packed RNG
// word, normal cache | sum, 0); a slot nobody parked in holds pixel 0xffffffff (the host fills
// it so before the launch).  Indexed by slot, not by an atomic count: no ballot or atomic in
// the shading code (that cost the plain kernel 28 more spilled VGPRs).
constexpr uint32_t kNoPark = 0xffffffffu;
__device__ __forceinline__ void park_pixel(uint4 *park, long long slot, int pix, int s, const Rng &r, V3 sum) {
    park[2 * slot] = make_uint4((uint32_t)pix, (uint32_t)s, rng_word_pack(r.x, r.saved_avail), __float_as_uint(r.saved));
    park[2 * slot + 1] = make_uint4(__float_as_uint(sum.x), __float_as_uint(sum.y), __float_as_uint(sum.z), 0u);
}
// Shade the lane's closest hit (one vertex of scene.cpp:85-154); bounce, or end the path:
// fold, accumulate, next sample or pixel done.
// Set when a lane of the wave added its sample itself (spec_job_end): its pixel may take
// runahead jobs again, so the wave runs a management pass when a lane is idle.
#if defined(__HIPCC__)
__shared__ int spec_hint_lds[4];
__device__ __forceinline__ void spec_hint_set() { spec_hint_lds[threadIdx.x >> 6] = 1; }
__device__ __forceinline__ bool spec_hint_take() {
    const bool h = spec_hint_lds[threadIdx.x >> 6] != 0;
    spec_hint_lds[threadIdx.x >> 6] = 0;
    return h;
}
#else
inline thread_local bool g_spec_hint[4096];   // host harness: per emulated wave (mega_slot() / 64)
inline void spec_hint_set() { g_spec_hint[(mega_slot() >> 6) & 4095] = true; }
inline bool spec_hint_take() {
    bool &h = g_spec_hint[(mega_slot() >> 6) & 4095];
    const bool v = h;
    h = false;
    return v;
}
#endif

// End of a runahead job's sample (speculative runahead, below): adds it and starts the next
// sample on this lane when no other job of its pixel is in flight, else waits (M_DONE_NEW).
template <class ML>
__device__ void spec_job_end(ML &L, const DevScene &sc, const ShardGeom &g, const WfState &st, int spp,
                             float *out, const NodeRec &root, V3 color, LaneCtr c);

// `tail` (wave-uniform): the wave runs runahead jobs (spec_manage below); a job's path end
// goes to spec_job_end instead of the pixel sum in the lane.
// `park` (wave-uniform; lane-resident kernel, hand-off): a path end that leaves the pixel
// unfinished stops there (idle, still holding the pixel, for park_pixel) instead of starting
// its next sample.
template <bool COUNT, bool FAST = false, class Stack, class ML>
__device__ __forceinline__ void mega_shade(ML &L, const DevScene &sc, const ShardGeom &g, const WfState &st,
                                           int spp, float *out, unsigned *cost, const NodeRec &root, Stack &stk,
                                           Counters &cnt, bool tail = false, bool park = false) {
    LaneRec P{st.rec_ab, st.rec_c, mega_slot_of(L), st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
    Hit h = L.T.best;
    LaneCtr c = lane_ctr(L);
    bool next = false;
    const bool shaded = h.prim >= 0 && h.t < sc.max_distance;
    if (shaded) {
#if defined(__HIPCC__)
        if constexpr (kUvRecompute) {   // (u, v) of the closest hit (rt_wavefront.h RT_UV_RECOMPUTE)
            RT_CHECK(h.prim < sc.n_tris, 1, h.prim, h.prim = 0);
            hit_uv(sc, L.r, h);
        }
#endif
        Rng rng = lane_rng(L);
        const bool cont = shade_hit<COUNT>(sc, L.r, h, rng, cnt, P, c.nv, stk);   // (stack free: T.sp == 0)
        lane_rng_set(L, rng);
        if (cont && c.power > 0) {
            c.power -= 1;
            next = true;
        }
    }
    // (parity: no flush_e; a continued vertex has its record, and a path that ends at the
    // vertex shaded here folds from its emission in registers.  Fast mode writes it and folds
    // from memory: keeping it live there made that instantiation spill 31 VGPRs instead of 22.)
    if constexpr (FAST) P.flush_e();
    if (next) {
        lane_ctr_set(L, c);
        mega_begin<COUNT>(L, root, cnt);
        return;
    }
    if (!COUNT && !FAST && tail) {   // runahead job: colour of sample c.s, end state in the RNG slot
        spec_job_end(L, sc, g, st, spp, out, root, fold_path(P, c.nv, shaded), c);
        return;
    }
    const V3 sm = rtv::add(lane_sum(L), fold_path(P, c.nv, !FAST && shaded));
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
    if (!COUNT && !FAST && park) {   // (idle, still holding its pixel: the kernel's loop parks it)
        lane_ctr_set(L, c);
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
template <bool COUNT, class Stack, class TS>
__device__ __forceinline__ bool light_step(const DevScene &sc, const Ray &r, TS &T, Stack &stk, Counters &cnt,
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
template <bool COUNT, bool FAST, class Stack, class ML>
__device__ __forceinline__ void mega_shade_split(ML &L, const DevScene &sc, const ShardGeom &g,
                                                 const WfState &st, int spp, float *out, unsigned *cost,
                                                 const NodeRec &root, Stack &stk, Counters &cnt) {
    const long long slot = mega_slot();
    LaneRec P{st.rec_ab, st.rec_c, slot, st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
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
template <bool COUNT, class Stack, class Nodes, bool FAST = false, bool LSPLIT = false, class ML>
__device__ __forceinline__ void mega_iterate(ML &L, bool shade_now, const DevScene &sc, const ShardGeom &g,
                                             const WfState &st, int spp, float *out, unsigned *cost,
                                             const NodeRec &root, Stack &stk, const Nodes &nodes, Counters &cnt,
                                             bool tail = false, bool park = false) {
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
        if (L.state == M_READY) mega_shade<COUNT, FAST>(L, sc, g, st, spp, out, cost, root, stk, cnt, tail, park);
    } else if (L.state == M_TRAV) {
        if (trav_step<COUNT>(sc, L.r, L.T, stk, nodes, cnt)) L.state = M_READY;
    }
}

// ---------------------------------------------------------------- speculative sample runahead
// A pixel's samples form one sequential chain (scene.cpp:34-42): sample t+1 starts from the
// RNG state sample t ends in, and how many draws sample t takes depends on its path.  Once
// the pixel queue is empty, a wave's lanes run out of pixels while the heavy pixels' chains
// go on: the frame then lasts as long as its slowest chain.  Runahead lets the
// idle lanes of the wave run the next samples of those chains before their start state is
// known, and keeps only results whose start state is proven:
//   * A path with v vertices calls SceneDistribution::sample v times, and the draws of one
//     call are decided by the drawn values alone (rt_path.h rng_skip_sample).  So the state
//     sample t ends in is rng_skip_sample(X_t, v_t), and v_t is mostly ray_depth for the
//     pixels whose chains are long (69% of the samples of the heaviest sponza pixels).
//   * Each pixel has a record.  Its frontier f is the first sample not yet added; X_f, the
//     true state sample f starts from, is known once sample f-1 is added.  Jobs f, f+1, ...,
//     nxt-1 are in flight, each on its own lane: job f from X_f, job u+1 from
//     rng_skip_sample(start of job u, ray_depth).  An ended job waits (M_DONE) until it is the
//     frontier.
//   * When the frontier job has ended it is added to the pixel sum (in sample order, so the
//     float sum is the reference's), and its end state E becomes X_{f+1}.  The jobs past it
//     stay only if job f+1 started from E (states compared bit for bit); otherwise the
//     record's epoch ends and the lanes running them are freed.  A result is only ever used
//     when its start state equals the true one, so the pixel sum is bit-identical to the
//     sequential chain's.
// Records live in WfState::mid (the light-split kernel's planes, unused here), indexed by
// the wave's lane that held the pixel when the wave entered its tail: plane 0 (pix, f, nxt,
// epoch), 1 (sum xyz, meta), 2 (X_f, lane table low word), 3 (start state of job nxt-1, lane
// table high word); plane 4 is each lane's job (tag = record | epoch << 6, start state).  A management pass loads them once, works on registers with the wave's
// shuffles and ballots, and stores them back: one memory round trip per pass.  The same
// pass runs on the host test harness (tests/native/kernel_host.cpp) over emulated lanes:
// WArr is one register per lane on the GPU and a 64-entry array on the host.

// Diagnostics build (RT_MEGA_PROF): runahead event counts, printed by the launch.
// [0] management passes [1] their cycles (per wave) [2] frontier jobs issued [3] runahead jobs
// issued [4] jobs added [5] of them runahead jobs [6] invalidations [7] waves that reached a tail
// [8] parked pixels claimed in the tail (hand-off) [9]-[13] unused [14] chain-link time sum
// (pixel completion since its wave's start / spp)
// [15] pixels completed
#if defined(RT_MEGA_PROF) && defined(__HIPCC__)
// (per-block LDS sums, added to g_spec_prof once at the end of the kernel: global atomics on
// eight words from every wave serialised the runahead kernel)
__device__ unsigned long long g_spec_prof[16];
__shared__ unsigned long long spec_prof_lds[16];
#define RT_SPEC_STAT(k, v) atomicAdd(&::rtd::spec_prof_lds[k], (unsigned long long)(v))
// chain links: a pixel's completion time since its wave's start (wall clock, 100 MHz) / spp,
// summed in [14] (count in [15]); the wave's start time is set by the kernel
__shared__ unsigned long long spec_wave_t0_lds[4];
// every chain's completion (wall clock, pixel), for the tail study of the launch's print
constexpr int kChainRec = 1 << 20;
__device__ unsigned long long g_chain_t[kChainRec];
__device__ unsigned int g_chain_pix[kChainRec];
__device__ unsigned int g_chain_n;
#define RT_SPEC_CHAIN_END(spp, pix) \
    RT_SPEC_STAT(14, (wall_clock64() - ::rtd::spec_wave_t0_lds[threadIdx.x >> 6]) / (unsigned long long)(spp)); \
    RT_SPEC_STAT(15, 1); \
    { \
        const unsigned ci_ = atomicAdd(&::rtd::g_chain_n, 1u); \
        if (ci_ < (unsigned)::rtd::kChainRec) { \
            ::rtd::g_chain_t[ci_] = wall_clock64(); \
            ::rtd::g_chain_pix[ci_] = (unsigned)(pix); \
        } \
    }
#elif !defined(__HIPCC__)
inline unsigned long long g_spec_prof[16];   // host test harness
#define RT_SPEC_STAT(k, v) (::rtd::g_spec_prof[k] += (unsigned long long)(v))
#define RT_SPEC_CHAIN_END(spp, pix) do { } while (0)
#else
#define RT_SPEC_STAT(k, v) do { } while (0)
#define RT_SPEC_CHAIN_END(spp, pix) do { } while (0)
#endif

// Record meta (plane 1 .w): bit 0 active, bit 1 X_f known (for a pixel that entered the tail
// past its sample 0: false until the wave's first job of the pixel ends).  Window and issue rate, slowest 8-way shard of the headline frame: with
// the round-3 traversal (inner loop, coop leaves, pop cap) window 3 with both runahead jobs
// issued in one pass 208 ms; window 4 one job per pass 218, two 213, three 211; window 2
// 212-215; window 6 228 (profiles/r03_ab.jsonl r03ad-af).  Fewer speculative jobs in flight
// waste fewer lanes on mispredicted chains and add less divergence to the wave.  (Round 2:
// window 3 307 ms, 4 306, 6 316.)  Windows that adapt to a pixel's prediction hit rate (grow
// on a hit, halve on a miss) measured 384 (round 2): the pixels with long chains lost their
// runahead too.
#ifndef RT_SPEC_WINDOW
#define RT_SPEC_WINDOW 3
#endif
#ifndef RT_SPEC_ISSUE
#define RT_SPEC_ISSUE 2
#endif
constexpr uint32_t kRecActive = 1u;
constexpr uint32_t kRecXf = 2u;
constexpr int kSpecWindow = RT_SPEC_WINDOW;   // jobs in flight per pixel at most, frontier included (<= 10)
// A runahead job whose sample ends while its pixel's frontier is still running waits for the
// next pass (M_DONE) instead of triggering one (M_DONE_NEW): its result is only used once the
// frontier reaches it.  8-way slowest shard 240 vs 243 ms (r03n).  0: every job end triggers a pass.
#ifndef RT_SPEC_LAZY
#define RT_SPEC_LAZY 1
#endif
constexpr bool kSpecLazy = RT_SPEC_LAZY != 0;   // spec_job_end: only frontier ends trigger a pass
constexpr int kSpecIssue = RT_SPEC_ISSUE;     // runahead jobs a pixel gets per management pass
static_assert(kSpecWindow >= 1 && kSpecWindow <= 10, "lane table holds 10 slots");
// The lanes running jobs f, f+1, ...: 6-bit slots of a 64-bit table (planes 2 and 3 .w).
// (Round 5's block-shared runahead, RT_SPEC_SHARE, which ran jobs in other waves of the block
// through an LDS offer board, measured slower, 190.1 vs 187.9 ms, and was
// deleted in round 6.)
constexpr int kTabBits = 6;
constexpr unsigned long long kTabMask = (1ull << kTabBits) - 1ull;
__device__ __forceinline__ int spec_tab(unsigned long long t, int q) { return (int)((t >> (kTabBits * q)) & kTabMask); }
__device__ __forceinline__ unsigned long long spec_tab_set(unsigned long long t, int q, int ln) {
    return (t & ~(kTabMask << (kTabBits * q))) | ((unsigned long long)ln << (kTabBits * q));
}

struct SpecView {
    uint4 *base;        // WfState::mid
    long long lanes;    // plane stride (lane slots)
    long long wbase;    // lane slot of this wave's lane 0
    __device__ __forceinline__ uint4 *w(int plane, int r) const { return base + ((long long)plane * lanes + wbase + r); }
};
__device__ __forceinline__ Rng rng_unpack(uint4 v) { return Rng{v.x, v.y, __uint_as_float(v.z)}; }
__device__ __forceinline__ bool rng_same(const Rng &a, const Rng &b) {
    return a.x == b.x && a.saved_avail == b.saved_avail && __float_as_uint(a.saved) == __float_as_uint(b.saved);
}
__device__ __forceinline__ uint4 v3_pack(V3 v, uint32_t w) {
    return make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), w);
}
__device__ __forceinline__ bool job_state(int s) { return s != M_IDLE; }

// Per-lane values of a wave: this lane's register on the GPU (at(src) = the wave shuffle,
// called by every lane), a 64-entry array on the host.  WAVE_PHASE runs its body for this
// lane (GPU) or for every lane in turn (host); a phase only reads other lanes' values that an
// earlier phase wrote.
#if defined(__HIPCC__)
__device__ __forceinline__ uint32_t wshfl(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
template <class T> struct WArr;
template <> struct WArr<uint32_t> {
    uint32_t v;
    __device__ __forceinline__ uint32_t get(int) const { return v; }
    __device__ __forceinline__ void put(int, uint32_t x) { v = x; }
    __device__ __forceinline__ uint32_t at(int s) const { return wshfl(v, s); }
};
template <> struct WArr<int> {
    int v;
    __device__ __forceinline__ int get(int) const { return v; }
    __device__ __forceinline__ void put(int, int x) { v = x; }
    __device__ __forceinline__ int at(int s) const { return __shfl(v, s, 64); }
};
template <> struct WArr<Rng> {
    Rng v;
    __device__ __forceinline__ Rng get(int) const { return v; }
    __device__ __forceinline__ void put(int, Rng x) { v = x; }
    __device__ __forceinline__ Rng at(int s) const {
        return Rng{wshfl(v.x, s), wshfl(v.saved_avail, s), __uint_as_float(wshfl(__float_as_uint(v.saved), s))};
    }
};
template <> struct WArr<V3> {
    V3 v;
    __device__ __forceinline__ V3 get(int) const { return v; }
    __device__ __forceinline__ void put(int, V3 x) { v = x; }
    __device__ __forceinline__ V3 at(int s) const { return V3{__shfl(v.x, s, 64), __shfl(v.y, s, 64), __shfl(v.z, s, 64)}; }
};
// acc = the wave's ballot of p (acc starts at 0)
#define WBALLOT(acc, lane, p) ((acc) = __ballot(p))
#define WAVE_PHASE(lane, ...)                   \
    {                                            \
        const int lane = (int)(threadIdx.x & 63); \
        __VA_ARGS__                              \
    }
struct SpecLanes {   // the wave's lanes as seen by one lane: its own MegaLane
    MegaLane &L;
    __device__ __forceinline__ MegaLane &operator[](int) const { return L; }
};
#else
template <class T> struct WArr {
    T v[64];
    T get(int l) const { return v[l]; }
    void put(int l, T x) { v[l] = x; }
    T at(int s) const { return v[s]; }
};
#define WBALLOT(acc, lane, p) ((acc) |= (p) ? (1ull << (lane)) : 0ull)
#define WAVE_PHASE(lane, ...) \
    for (int lane = 0; lane < 64; ++lane) { __VA_ARGS__ }
struct SpecLanes {
    MegaLane *W;
    MegaLane &operator[](int l) const { return W[l]; }
};
#endif

// Runahead priority (RT_SPEC_PRIO): the order in which records with room in their window get
// the wave's idle lanes.  0: record (lane) order, which at the tail's start is the pre-pass's
// heaviest-first order (rounds 2-4).  1 (default): fewest samples added first (ties by lane):
// every chain of an 8-way shard starts at the same time, so the chain with the smallest
// frontier is the one furthest behind (remaining time ~ elapsed x (spp - f) / f), and it is
// the one that ends the wave.  Round 5 (profiles/r05e_prio_late_ab.jsonl, one box): the 8
// shards of the 8-way split 186.7-188.5 ms (mean 187.6) against 201.2-205.7 (mean 202.7); the
// one-GPU frame (plain kernel) is unchanged (1135.0 vs 1136.0 ms); bits unchanged.
#ifndef RT_SPEC_PRIO
#define RT_SPEC_PRIO 1
#endif
constexpr bool kSpecPrio = RT_SPEC_PRIO != 0;

// srec[k] = the record at position k of the ascending order of key (keys distinct: the lane
// is in their low 6 bits), rank[r] = the position of record r.  GPU: a bitonic sort over the
// wave's lanes (21 exchange steps), then the inverse permutation by ds_permute.
#if defined(__HIPCC__)
__device__ __forceinline__ void wave_order(const WArr<uint32_t> &key, WArr<int> &srec, WArr<int> &rank) {
    const int lane = (int)(threadIdx.x & 63);
    uint32_t k = key.v;
#pragma unroll
    for (int b = 2; b <= 64; b <<= 1)
#pragma unroll
        for (int j = b >> 1; j > 0; j >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)k, j, 64);
            const bool keep_min = ((lane & j) == 0) == ((lane & b) == 0);
            k = keep_min ? (o < k ? o : k) : (o > k ? o : k);
        }
    srec.v = (int)(k & 63u);
    rank.v = __builtin_amdgcn_ds_permute(srec.v << 2, lane);   // lane srec[k] receives k
}
#else
inline void wave_order(const WArr<uint32_t> &key, WArr<int> &srec, WArr<int> &rank) {
    uint32_t k[64];
    for (int l = 0; l < 64; ++l) k[l] = key.get(l);
    std::sort(k, k + 64);
    for (int p = 0; p < 64; ++p) {
        srec.put(p, (int)(k[p] & 63u));
        rank.put((int)(k[p] & 63u), p);
    }
}
#endif

// Position of the i-th (from 0) set bit of m (m has more than i set bits).
__device__ __forceinline__ int nth_bit(unsigned long long m, int i) {
    int pos = 0;
    for (int w = 32; w > 0; w >>= 1)
        if (__builtin_popcountll(m & ((1ull << (pos + w)) - 1ull)) <= i) pos += w;
    return pos;
}
__device__ __forceinline__ int popc64(unsigned long long m) { return __builtin_popcountll(m); }

// Parked pixels a tail wave may still take (the hand-off's runahead launch, rt_mega_kernel
// `mode`): park-list slot base + c for claim counter value c, below n_items; a wave takes them
// into free record slots while it has fewer than `keep` active records.
struct SpecClaim {
    unsigned long long *queue;
    long long base, n_items;
    const uint4 *resume;   // the park list (rt_mega.h parked)
    int keep;
    bool open;             // the list may still hold slots (wave-uniform)
    const int *ridx;       // item -> park-list slot (the spread of the parked pixels), or null
};
// Item p of the resume launch: the parked pixel in slot ridx[p] (the host's spread: the
// pixels with the most work left dealt one per wave) or, without a map, in slot p.
__device__ __forceinline__ Parked parked_item(const uint4 *park, const int *ridx, long long p) {
    return parked(park, ridx ? (long long)ridx[p] : p);
}
// atomicAdd of the wave (called by every lane; one atomic), its old value in every lane
__device__ __forceinline__ unsigned long long wave_fetch_add(unsigned long long *q, unsigned k) {
#if defined(__HIPCC__)
    unsigned long long b = 0;
    if ((threadIdx.x & 63) == 0) b = atomicAdd(q, (unsigned long long)k);
    return __shfl(b, 0, 64);
#else
    const unsigned long long b = *q;
    *q += k;
    return b;
#endif
}

// The wave enters its tail (queue empty): every lane's pixel gets a record at this lane; its
// sample in flight is the frontier job (table slot 0 = this lane), started from the true
// state X_f.  X_f is known from the start for sample 0 (the pixel's seed) and for a pixel
// just resumed from the park list (`xk`, X), so runahead can begin at once; otherwise only
// once the job ends (the lane's RNG has moved on).
__device__ __forceinline__ void spec_convert(MegaLane &L, const DevScene &sc, const ShardGeom &g, const SpecView &V,
                                             int lane, bool xk = false, Rng Xk = Rng{0u, 0u, 0.f}) {
    if (L.pix >= 0) {
        const LaneCtr c = lane_ctr(L);
        const bool x0 = c.s == 0 || xk;
        const Rng X = xk ? Xk : c.s == 0 ? pixel_seed(sc, g, L.pix) : Rng{0u, 0u, 0.f};
        *V.w(0, lane) = make_uint4((uint32_t)L.pix, (uint32_t)c.s, (uint32_t)c.s + 1u, 0u);
        *V.w(1, lane) = v3_pack(lane_sum(L), x0 ? kRecActive | kRecXf : kRecActive);
        // X_f, table slot 0 (this lane); the start state of job nxt - 1 (= f); this lane's job
        *V.w(2, lane) = make_uint4(X.x, X.saved_avail, __float_as_uint(X.saved), (uint32_t)lane);
        *V.w(3, lane) = make_uint4(X.x, X.saved_avail, __float_as_uint(X.saved), 0u);
        *V.w(4, lane) = make_uint4((uint32_t)lane, X.x, X.saved_avail, __float_as_uint(X.saved));
    } else {
        *V.w(1, lane) = make_uint4(0u, 0u, 0u, 0u);
    }
}

// Start job (record r, sample t, epoch e) on this lane from state Y.
template <class ML>
__device__ __forceinline__ void spec_start(ML &L, const DevScene &sc, const ShardGeom &g, const NodeRec &root,
                                           uint32_t pix, uint32_t t, const Rng &Y) {
    L.pix = (int)pix;
    lane_ctr_set(L, LaneCtr{(int)t, 0, 0});
    lane_rng_set(L, Y);
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    mega_sample<false>(L, sc, g, root, cnt);
}

// A job's sample has ended (path end in a tail wave).  When it is its pixel's frontier and no
// other job of the pixel is in flight, this lane adds it at once and goes on with the next
// sample from its end state, as outside the tail (one record round trip instead of a wait
// for a management pass); the record then shows job f + 1 on this lane.  Otherwise the job
// waits for the next pass with its colour in the lane's sum slot.  Only this lane holds a job
// of the pixel in the first case, and passes never overlap a shading step, so the record
// update is this lane's alone.
template <class ML>
__device__ __forceinline__ void spec_job_end(ML &L, const DevScene &sc, const ShardGeom &g, const WfState &st,
                                             int spp, float *out, const NodeRec &root, V3 color, LaneCtr c) {
    const int lane = (int)(mega_slot() & 63);
    const SpecView V{(uint4 *)st.mid, st.lanes, mega_slot() - lane};
    const uint4 j = *V.w(4, lane);
    const int r = (int)(j.x & 63u);
    const uint4 a = *V.w(0, r), b = *V.w(1, r);
    const uint32_t t = (uint32_t)c.s;
    if ((j.x >> 6) == a.w && t == a.y && a.z == t + 1u && (b.w & kRecActive)) {
        const V3 sum = rtv::add(V3{__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)}, color);
        const Rng E = lane_rng(L);
        const uint32_t m = b.w | kRecXf;
        RT_SPEC_STAT(4, 1);
        if (t + 1u == (uint32_t)spp) {
            const long long o = 3 * (long long)a.x;
            out[o + 0] = sum.x;
            out[o + 1] = sum.y;
            out[o + 2] = sum.z;
            *V.w(0, r) = make_uint4(a.x, t + 1u, t + 1u, a.w);
            *V.w(1, r) = v3_pack(sum, 0u);
            RT_SPEC_CHAIN_END(spp, a.x);
            spec_hint_set();   // (a record slot is free: the next pass may claim a pixel into it)
            L.pix = -1;
            L.state = M_IDLE;
            return;
        }
        *V.w(0, r) = make_uint4(a.x, t + 1u, t + 2u, a.w);
        *V.w(1, r) = v3_pack(sum, m);
        *V.w(2, r) = make_uint4(E.x, E.saved_avail, __float_as_uint(E.saved), (uint32_t)lane);   // X_f; slot 0: here
        *V.w(3, r) = make_uint4(E.x, E.saved_avail, __float_as_uint(E.saved), 0u);   // job nxt-1 starts from E
        *V.w(4, lane) = make_uint4(j.x, E.x, E.saved_avail, __float_as_uint(E.saved));
        c.s = (int)t + 1;
        lane_ctr_set(L, c);
        Counters cnt{0, 0, 0, 0, 0, 0, 0};
        mega_sample<false>(L, sc, g, root, cnt);
        if (kSpecWindow > 1 && t + 2u < (uint32_t)spp) spec_hint_set();
        return;
    }
    lane_sum_set(L, color);
    lane_ctr_set(L, c);
    // A frontier job's end needs a pass (its sample is added there and the chain goes on); a
    // runahead job's result can only be used once the frontier reaches it, so with
    // RT_SPEC_LAZY it waits as M_DONE for the next pass instead of triggering one.
    const bool frontier = (j.x >> 6) == a.w && t == a.y;
    L.state = (!kSpecLazy || frontier) ? M_DONE_NEW : M_DONE;
}

// One management pass of a tail wave: add ended frontier jobs in order, free the lanes of
// added, superseded or invalidated jobs, hand idle lanes new jobs (first a frontier job to
// every pixel without one, then runahead jobs in record order: at the tail's start, lane
// order is heaviest first, rt_order_spread_kernel).  Returns whether a record can still take
// a job (the wave calls again when a lane is idle).
__device__ __forceinline__ bool spec_manage(SpecLanes lanes, const DevScene &sc, const ShardGeom &g,
                                            const SpecView &V, int spp, float *out, const NodeRec &root,
                                            SpecClaim &claim) {
    const int depth = sc.ray_depth;
    // records (this lane as record holder)
    WArr<uint32_t> rp, rf, rn, re, rm, tl, th;   // tl, th: lane table
    WArr<V3> rs;
    WArr<Rng> rx, ry;
    // jobs (this lane as job runner)
    WArr<uint32_t> jt, jsamp;
    WArr<int> js;
    WArr<V3> jc;
    WArr<Rng> je, jy;
    WAVE_PHASE(lane, {
        MegaLane &L = lanes[lane];
        const uint4 a = *V.w(0, lane), b = *V.w(1, lane), c = *V.w(2, lane), d = *V.w(3, lane), j = *V.w(4, lane);
        rp.put(lane, a.x);
        rf.put(lane, a.y);
        rn.put(lane, a.z);
        re.put(lane, a.w);
        rs.put(lane, V3{__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)});
        rm.put(lane, b.w);
        rx.put(lane, rng_unpack(c));
        ry.put(lane, rng_unpack(d));
        tl.put(lane, c.w);
        th.put(lane, d.w);
        jt.put(lane, j.x);
        jy.put(lane, Rng{j.y, j.z, __uint_as_float(j.w)});   // plane 4: (tag, start state)
        js.put(lane, L.state);
        jsamp.put(lane, (uint32_t)lane_ctr(L).s);
        const bool done = L.state == M_DONE_NEW || L.state == M_DONE;
        jc.put(lane, done ? lane_sum(L) : V3{0.f, 0.f, 0.f});
        je.put(lane, done ? lane_rng(L) : Rng{0u, 0u, 0.f});
    })
    constexpr int win = kSpecWindow, issue = kSpecIssue;
    // A. add ended frontier jobs, one per pixel per round, at most `win` rounds
    for (int q = 0; q < win; ++q) {
        WArr<int> prog;
        WAVE_PHASE(lane, {
            const uint32_t m = rm.get(lane);
            const unsigned long long tab = (unsigned long long)th.get(lane) << 32 | tl.get(lane);
            const bool has = (m & kRecActive) && rn.get(lane) > rf.get(lane);
            const int j0 = has ? spec_tab(tab, 0) : lane;
            const int j1 = has && rn.get(lane) > rf.get(lane) + 1u ? spec_tab(tab, 1) : lane;
            // the frontier job's lane and the next job's lane (shuffles: every lane)
            const int s0 = js.at(j0);
            const uint32_t t0 = jt.at(j0), n0 = jsamp.at(j0);
            const V3 c0 = jc.at(j0);
            const Rng e0 = je.at(j0), y1 = jy.at(j1);
            const uint32_t tag = (uint32_t)lane | re.get(lane) << 6;
            const bool done0 = (s0 == M_DONE_NEW || s0 == M_DONE) && t0 == tag && n0 == rf.get(lane);
            int pr = 0;
            if (has && done0) {
                uint32_t f = rf.get(lane) + 1u, n = rn.get(lane), mm = m | kRecXf;
                unsigned long long tb = tab >> kTabBits;   // table slots 1.. -> 0..
                const V3 sum = rtv::add(rs.get(lane), c0);
                const bool keep = (m & kRecXf) && n > f && rng_same(y1, e0);
                RT_SPEC_STAT(5, keep ? 1 : 0);
                RT_SPEC_STAT(4, 1);
                if (!keep && n > f) {   // the runahead past f started from another state
                    re.put(lane, re.get(lane) + 1u);
                    n = f;
                    tb = 0ull;
                    RT_SPEC_STAT(6, 1);
                }
                if (f == (uint32_t)spp) {
                    const long long o = 3 * (long long)rp.get(lane);
                    out[o + 0] = sum.x;
                    out[o + 1] = sum.y;
                    out[o + 2] = sum.z;
                    mm = 0u;
                    RT_SPEC_CHAIN_END(spp, rp.get(lane));
                }
                rf.put(lane, f);
                rn.put(lane, n);
                rm.put(lane, mm);
                tl.put(lane, (uint32_t)tb);
                th.put(lane, (uint32_t)(tb >> 32));
                rs.put(lane, sum);
                rx.put(lane, e0);
                pr = 1;
            }
            prog.put(lane, pr);
        })
        unsigned long long any = 0;
        WAVE_PHASE(lane, { WBALLOT(any, lane, prog.get(lane) != 0); })
        if (!any) break;
    }
    // job lanes: added, superseded or invalidated jobs end; ended runahead jobs wait
    WAVE_PHASE(lane, {
        MegaLane &L = lanes[lane];
        const bool job = job_state(js.get(lane));
        const int r = job ? (int)(jt.get(lane) & 63u) : lane;
        const uint32_t fr = rf.at(r), er = re.at(r);
        if (job) {
            if ((jt.get(lane) >> 6) != er || jsamp.get(lane) < fr) {
                L.state = M_IDLE;
                L.pix = -1;
            } else if (L.state == M_DONE_NEW) {
                L.state = M_DONE;
            }
        }
    })
    // C1. pixels without a frontier job in flight get one, from the true state X_f
    unsigned long long nm = 0, idle = 0;
    WAVE_PHASE(lane, {
        const bool need = (rm.get(lane) & kRecActive) && rn.get(lane) == rf.get(lane);
        WBALLOT(nm, lane, need);
        WBALLOT(idle, lane, lanes[lane].state == M_IDLE);
    })
    const int n_need = popc64(nm), n_idle = popc64(idle);
    WAVE_PHASE(lane, {
        MegaLane &L = lanes[lane];
        const int i = popc64(idle & ((1ull << lane) - 1ull));
        const bool issue = ((idle >> lane) & 1ull) && i < n_need;
        const int r = issue ? nth_bit(nm, i) : lane;
        const uint32_t pix = rp.at(r), f = rf.at(r), e = re.at(r);
        const Rng X = rx.at(r);
        if (issue) {
            spec_start(L, sc, g, root, pix, f, X);
            jt.put(lane, (uint32_t)r | e << 6);
            jy.put(lane, X);
            RT_SPEC_STAT(2, 1);
        }
        // record side: the k-th needing record got the k-th idle lane
        const int k = popc64(nm & ((1ull << lane) - 1ull));
        if (((nm >> lane) & 1ull) && k < n_idle) {
            rn.put(lane, rf.get(lane) + 1u);
            ry.put(lane, rx.get(lane));
            tl.put(lane, (uint32_t)nth_bit(idle, k));   // slot 0 (no other jobs are in flight)
            th.put(lane, 0u);
        }
    })
    // C1b. hand-off: a wave with fewer than claim.keep active records takes parked pixels from
    // the park list into free record slots, one atomic per wave; the frontier job of each
    // starts at once on an idle lane, from the parked state: X_f is known, so the record may
    // take runahead jobs in this same pass.  A pixel's samples still run in order from that
    // state, and its sum is added in sample order: same bits.
    if (claim.open) {
        unsigned long long act = 0, idl = 0;
        WAVE_PHASE(lane, {
            WBALLOT(act, lane, (rm.get(lane) & kRecActive) != 0);
            WBALLOT(idl, lane, lanes[lane].state == M_IDLE);
        })
        int want = claim.keep - popc64(act);
        want = want < popc64(idl) ? want : popc64(idl);
        if (want > 0) {
            const long long first = claim.base + (long long)wave_fetch_add(claim.queue, (unsigned)want);
            const long long left = claim.n_items - first;
            const int got = left <= 0 ? 0 : (left < (long long)want ? (int)left : want);
            if (got < want) claim.open = false;
            const unsigned long long fm = ~act;   // free record slots
            WArr<int> made;   // (a hand-off claim may find an empty park slot: no record, no job)
            WAVE_PHASE(lane, {   // record side: the k-th free slot takes item first + k
                const int k = popc64(fm & ((1ull << lane) - 1ull));
                made.put(lane, 0);
                if (((fm >> lane) & 1ull) && k < got) {
                    const Parked q = parked_item(claim.resume, claim.ridx, first + k);
                    if (q.pix != kNoPark) {   // (an empty slot: nobody parked there)
                        made.put(lane, 1);
                        const Rng X = q.x;
                        rp.put(lane, q.pix);
                        rf.put(lane, q.s);
                        rn.put(lane, q.s + 1u);
                        re.put(lane, re.get(lane) + 1u);   // (a new epoch: no stale job of the slot matches)
                        rs.put(lane, q.sum);
                        rm.put(lane, kRecActive | kRecXf);
                        rx.put(lane, X);
                        ry.put(lane, X);
                        tl.put(lane, (uint32_t)nth_bit(idl, k));   // slot 0: the k-th idle lane
                        th.put(lane, 0u);
                        RT_SPEC_STAT(8, 1);
                    }
                }
            })
            WAVE_PHASE(lane, {   // runner side: the i-th idle lane runs the i-th new record's frontier sample
                MegaLane &L = lanes[lane];
                const int i = popc64(idl & ((1ull << lane) - 1ull));
                const bool run = ((idl >> lane) & 1ull) && i < got;
                const int r = run ? nth_bit(fm, i) : lane;
                const uint32_t pix = rp.at(r), e = re.at(r), f = rf.at(r);
                const Rng X = rx.at(r);
                const int mk = made.at(r);   // (every lane shuffles: a lane that is off in a
                                             // ds_bpermute reads as 0 to the lanes that read it)
                if (run && mk) {
                    spec_start(L, sc, g, root, pix, f, X);
                    jt.put(lane, (uint32_t)r | e << 6);
                    jy.put(lane, X);
                    RT_SPEC_STAT(2, 1);
                }
            })
        }
    }
    // C2. runahead: idle lanes take the next jobs of pixels with room in their window
    WArr<int> room, incl;
    unsigned long long idle2 = 0;
    WAVE_PHASE(lane, {
        int rr = 0;
        const uint32_t m = rm.get(lane);
        if ((m & kRecActive) && (m & kRecXf) && rn.get(lane) > rf.get(lane)) {
            const int w = win - (int)(rn.get(lane) - rf.get(lane)), left = spp - (int)rn.get(lane);
            rr = w < left ? w : left;
            rr = rr < 0 ? 0 : (rr < issue ? rr : issue);
        }
        room.put(lane, rr);
        WBALLOT(idle2, lane, lanes[lane].state == M_IDLE);
    })
    // the order in which records take idle lanes (RT_SPEC_PRIO): position k holds record
    // srec[k]; sroom / incl: room and its inclusive prefix sum in that order
    WArr<int> srec, rank, sroom;
    if constexpr (kSpecPrio) {
        WArr<uint32_t> key;
        WAVE_PHASE(lane, {
            key.put(lane, room.get(lane) > 0 ? (rf.get(lane) << 6 | (uint32_t)lane) : (0xffffffc0u | (uint32_t)lane));
        })
        wave_order(key, srec, rank);
        WAVE_PHASE(lane, { sroom.put(lane, room.at(srec.get(lane))); })
    } else {
        WAVE_PHASE(lane, {
            srec.put(lane, lane);
            rank.put(lane, lane);
            sroom.put(lane, room.get(lane));
        })
    }
#if defined(__HIPCC__)
    {
        int x = sroom.v;
        const int lane = (int)(threadIdx.x & 63);
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, (unsigned)d, 64);
            if (lane >= d) x += y;
        }
        incl.v = x;
    }
#else
    for (int l = 0, t = 0; l < 64; ++l) incl.put(l, t += sroom.get(l));
#endif
    const int total = incl.at(63), n_idle2 = popc64(idle2);
    WAVE_PHASE(lane, {
        MegaLane &L = lanes[lane];
        const int i = ((idle2 >> lane) & 1ull) ? popc64(idle2 & ((1ull << lane) - 1ull)) : (1 << 30);
        int k = 0;   // first position with incl > i
        for (int w = 32; w > 0; w >>= 1)
            if (incl.at(k + w - 1) <= i) k += w;
        const int incl_r = incl.at(k), room_r = sroom.at(k), r = srec.at(k);
        const uint32_t pix = rp.at(r), n = rn.at(r), e = re.at(r);
        Rng Y = ry.at(r);
        if (i < total) {
            const int j = i - (incl_r - room_r);
            for (int q = 0; q <= j; ++q) rng_skip_sample(Y, depth, sc.n_lights);
            spec_start(L, sc, g, root, pix, n + (uint32_t)j, Y);
            jt.put(lane, (uint32_t)r | e << 6);
            jy.put(lane, Y);
            RT_SPEC_STAT(3, 1);
        }
    })
    WAVE_PHASE(lane, {   // record side: its takers are idle lanes excl .. excl + taken - 1
        const int rr = room.get(lane), excl = incl.at(rank.get(lane)) - rr;
        int taken = n_idle2 - excl < rr ? n_idle2 - excl : rr;
        taken = taken < 0 ? 0 : taken;
        const int last = taken > 0 ? nth_bit(idle2, excl + taken - 1) : lane;
        const Rng yl = jy.at(last);
        if (taken > 0) {
            unsigned long long tb = (unsigned long long)th.get(lane) << 32 | tl.get(lane);
            const int base = (int)(rn.get(lane) - rf.get(lane));
            for (int q = 0; q < taken; ++q) tb = spec_tab_set(tb, base + q, nth_bit(idle2, excl + q));
            tl.put(lane, (uint32_t)tb);
            th.put(lane, (uint32_t)(tb >> 32));
            rn.put(lane, rn.get(lane) + (uint32_t)taken);
            ry.put(lane, yl);
        }
    })
    // store the records and the jobs; can a record still take a job?
    unsigned long long roomy = 0;
    WAVE_PHASE(lane, {
        *V.w(0, lane) = make_uint4(rp.get(lane), rf.get(lane), rn.get(lane), re.get(lane));
        *V.w(1, lane) = v3_pack(rs.get(lane), rm.get(lane));
        const Rng x = rx.get(lane), yy = ry.get(lane);
        *V.w(2, lane) = make_uint4(x.x, x.saved_avail, __float_as_uint(x.saved), tl.get(lane));
        *V.w(3, lane) = make_uint4(yy.x, yy.saved_avail, __float_as_uint(yy.saved), th.get(lane));
        const Rng y = jy.get(lane);
        *V.w(4, lane) = make_uint4(jt.get(lane), y.x, y.saved_avail, __float_as_uint(y.saved));
        const uint32_t m = rm.get(lane);
        const uint32_t f = rf.get(lane), n = rn.get(lane);
        const bool rm_room = (m & kRecActive) &&
                             (n == f || ((m & kRecXf) && (int)(n - f) < win && (int)n < spp));
        WBALLOT(roomy, lane, rm_room);
    })
    if (claim.open) {   // a free record slot the next pass may fill
        unsigned long long act = 0;
        WAVE_PHASE(lane, { WBALLOT(act, lane, (rm.get(lane) & kRecActive) != 0); })
        if (popc64(act) < claim.keep) roomy = ~0ull;
    }
    return roomy != 0;
}

}  // namespace rtd
