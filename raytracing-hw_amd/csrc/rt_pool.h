// rt_pool.h — the path-pool schedule of the lane-resident path tracer (GPU only).
//
// In the lane-resident kernel (rt_mega.h) a lane owns one path: once its closest hit is known
// the lane waits (READY) until enough of the wave's lanes are ready to shade together, so a
// traversal iteration runs with about 41 of 64 lanes busy.  Here a wave owns
// a pool of kPool = 64 x kPoolPerLane paths whose state lives in HBM (PoolPlanes), and its lanes
// are traversal slots, not path owners:
//   * a free lane takes the next path of the wave's traversal queue (an LDS ring of path
//     numbers), loads its ray and traverses it (trav_step_coop, as in the lane-resident kernel);
//   * when the closest hit is known the lane stores it with the path, appends the path to the
//     wave's ready ring and takes the next queued path at once;
//   * once kPoolBatch paths are ready (or no lane traverses), lanes 0..n-1 each shade one ready
//     path (one vertex of scene.cpp:85-154; the same shade_hit / fold_path / sample-loop code),
//     write its state back and queue its next ray: the bounce, the next sample's camera ray
//     (scene.cpp:36-41), or the first camera ray of a new pixel from the frame's pixel queue.
// With two paths per lane the queue is never empty while a lane is free (queued + ready +
// traversing = kPool), so every traversal iteration runs with all lanes busy until the frame's
// tail.  Every path keeps its own RNG chain, sample order and vertex records, so the bits are
// the lane-resident kernel's (= the reference's).
//
// Path record of path id p (PoolPlanes, float4 planes of stride `paths`; written only by the
// wave that owns p, so a plain store / load pair of one wave needs no fence):
//   A (origin, root-box miss flag)   B (direction, shard pixel)   C (closest hit: t, u, v, prim)
//   D (pixel sum, RNG word: minstd state | normal-cache flag << 31)   E (normal cache, LaneCtr, 0, 0)
// Vertex records: LaneRec indexed by path id (stride `paths`).
#pragma once
#include "rt_mega.h"

#if defined(__HIPCC__)
namespace rtd {

// Paths per lane of a wave's pool (ring ids are bytes: kPool <= 256).
#ifndef RT_POOL_PER_LANE
#define RT_POOL_PER_LANE 2
#endif
// Free lanes that trigger a refill inside the traversal loop (a refill costs a ring read and a
// ray load for the lanes it serves, whatever their number).
#ifndef RT_POOL_REFILL
#define RT_POOL_REFILL 8
#endif
// Ready paths that end the traversal loop for a shading pass.
#ifndef RT_POOL_BATCH
#define RT_POOL_BATCH 64
#endif
constexpr int kPoolPerLane = RT_POOL_PER_LANE;
constexpr int kPool = 64 * kPoolPerLane;
constexpr int kPoolRefill = RT_POOL_REFILL;
constexpr int kPoolBatch = RT_POOL_BATCH;
static_assert(kPool <= 256, "ring entries are bytes");
static_assert(kPoolBatch >= 1 && kPoolBatch <= 64, "a shading pass shades at most one path per lane");

struct PoolPlanes {
    float4 *base;   // WfState::mid: 5 planes
    long long n;    // plane stride (paths)
    __device__ __forceinline__ float4 *A(long long p) const { return base + p; }
    __device__ __forceinline__ float4 *B(long long p) const { return base + n + p; }
    __device__ __forceinline__ float4 *C(long long p) const { return base + 2 * n + p; }
    __device__ __forceinline__ float4 *D(long long p) const { return base + 3 * n + p; }
    __device__ __forceinline__ float4 *E(long long p) const { return base + 4 * n + p; }
};

// A stack whose frames start above the first `base` ones: the light-pdf walk of a lane that
// shades one path while it holds another path's traversal frames [0, base).
template <class Stack>
struct OffsetStack {
    Stack &s;
    int base;
    __device__ __forceinline__ void put(int i, uint2 v) { s.put(base + i, v); }
    __device__ __forceinline__ uint2 get(int i) const { return s.get(base + i); }
};

// The wave's two rings in LDS: traversal queue and ready list (path numbers 0..kPool-1 of the
// wave).  Head and tail are running counts, the same in every lane.
struct PoolRings {
    uint8_t *q, *r;
    int qh, qt, rh, rt;
};

// Append path number j of every lane with `want` to ring `ring` (tail advanced by their count).
__device__ __forceinline__ void pool_push(uint8_t *ring, int &tail, bool want, int j) {
    const unsigned long long m = __ballot(want);
    if (!m) return;
    const int lane = (int)(threadIdx.x & 63);
    if (want) ring[(unsigned)(tail + __popcll(m & ((1ull << lane) - 1ull))) % (unsigned)kPool] = (uint8_t)j;
    tail += __popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The ray of a queued path as traversal needs it: origin and direction from the record,
// Ray::inv = {1,1,1} / direction (primitive.cpp:12-15) recomputed exactly (rcp_ieee is the IEEE
// quotient), the root-box result the shading pass stored.
__device__ __forceinline__ Ray pool_load_ray(const PoolPlanes &V, long long p, uint32_t &miss) {
    const float4 a = *V.A(p), b = *V.B(p);
    Ray r;
    r.o = V3{a.x, a.y, a.z};
    r.d = V3{b.x, b.y, b.z};
    r.inv = V3{rcp_ieee(b.x), rcp_ieee(b.y), rcp_ieee(b.z)};
    miss = __float_as_uint(a.w);
    return r;
}

// A new ray of path p (bounce or camera ray): BVH::intersect's root box test (bvh.cpp:239-243)
// here, once, and the ray to the record.
__device__ __forceinline__ void pool_store_ray(const PoolPlanes &V, long long p, const Ray &r, const NodeRec &root,
                                               int pix) {
    float e;
    const bool hit = box_hit<false>(root.mn, root.mx, r, e);
    *V.A(p) = make_float4(r.o.x, r.o.y, r.o.z, __uint_as_float(hit ? 0u : 1u));
    *V.B(p) = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(pix));
}

// Sample c.s of pixel `pix` starts: jittered camera ray (scene.cpp:36-39); the first traversal
// consumes one call of the depth budget (scene.cpp:72-75).
__device__ __forceinline__ Ray pool_camera(const DevScene &sc, const ShardGeom &g, int pix, Rng &rng, LaneCtr &c) {
    const int k = pix / g.width, px = pix - k * g.width, py = shard_row(g, k);
    const float ox = rng_offset(rng);
    const float oy = rng_offset(rng);
    c.power = sc.ray_depth - 1;
    c.nv = 0;
    return camera_ray(sc, px, py, ox, oy);
}

__device__ __forceinline__ uint32_t pool_ctr(const LaneCtr &c) {
    return (uint32_t)c.s | (uint32_t)c.power << 20 | (uint32_t)c.nv << 24;
}
__device__ __forceinline__ LaneCtr pool_ctr_unpack(uint32_t w) {
    return LaneCtr{(int)(w & 0xfffffu), (int)((w >> 20) & 15u), (int)(w >> 24)};
}

// Path p takes pixel `pix`: RNG seeded from the pixel (scene.cpp:34, random.cpp:12-18; pixel 0
// -> 1), empty sum, sample 0's camera ray.
__device__ __forceinline__ void pool_assign(const PoolPlanes &V, long long p, const DevScene &sc, const ShardGeom &g,
                                            int pix, const NodeRec &root) {
    const int k = pix / g.width, px = pix - k * g.width, py = shard_row(g, k);
    const uint32_t seed = (uint32_t)(py * sc.width + px) % 2147483647u;
    Rng rng{seed == 0 ? 1u : seed, 0u, 0.f};
    LaneCtr c{0, 0, 0};
    const Ray r = pool_camera(sc, g, pix, rng, c);
    pool_store_ray(V, p, r, root, pix);
    *V.D(p) = make_float4(0.f, 0.f, 0.f, __uint_as_float(rng_word_pack(rng.x, rng.saved_avail)));
    *V.E(p) = make_float4(rng.saved, __uint_as_float(pool_ctr(c)), 0.f, 0.f);
}

// The next pixel for every lane with `need` (one atomic per wave); -1 once the queue is empty.
__device__ __forceinline__ int pool_claim(bool need, unsigned long long *queue, long long n_items, const int *order,
                                          bool &exhausted) {
    const unsigned long long m = __ballot(need && !exhausted);
    if (!m) return -1;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((unsigned long long)m) - 1;
    const unsigned cm = (unsigned)__popcll(m);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(queue, (unsigned long long)cm);
    base = __shfl(base, leader, 64);
    if ((long long)base + cm >= n_items) exhausted = true;
    if (!((m >> lane) & 1ull)) return -1;
    const long long q = (long long)base + __popcll(m & ((1ull << lane) - 1ull));
    return q < n_items ? (order ? order[q] : (int)q) : -1;
}

// Shade one ready path p (the lane-resident kernel's mega_shade on a path record): one vertex
// of Scene::intersect, then the bounce, or the path's end (fold, pixel sum, next sample), or the
// pixel's end (sum out; the path then needs a new pixel: returns true).  `push`: p has a new ray.
template <bool COUNT, class Stack>
__device__ __forceinline__ bool pool_shade(const PoolPlanes &V, long long p, const DevScene &sc, const ShardGeom &g,
                                           const WfState &st, int spp, float *out, const NodeRec &root, Stack &stk,
                                           Counters &cnt, bool &push) {
    const float4 a = *V.A(p), b = *V.B(p), h4 = *V.C(p), d4 = *V.D(p), e4 = *V.E(p);
    Ray r;
    r.o = V3{a.x, a.y, a.z};
    r.d = V3{b.x, b.y, b.z};
    r.inv = V3{0.f, 0.f, 0.f};   // (shading reads o and d only)
    const int pix = __float_as_int(b.w);
    const Hit h{h4.x, h4.y, h4.z, __float_as_int(h4.w)};
    Rng rng;
    rng_word_unpack(__float_as_uint(d4.w), rng.x, rng.saved_avail);
    rng.saved = e4.x;
    LaneCtr c = pool_ctr_unpack(__float_as_uint(e4.y));
    LaneRec P{st.rec_ab, st.rec_c, p, st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
    bool next = false;
    const bool shaded = h.prim >= 0 && h.t < sc.max_distance;
    if (shaded) {
        const bool cont = shade_hit<COUNT>(sc, r, h, rng, cnt, P, c.nv, stk);
        if (cont && c.power > 0) {
            c.power -= 1;
            next = true;
        }
    }
    V3 sum{d4.x, d4.y, d4.z};
    bool need_pixel = false;
    if (!next) {   // the path ends here: fold it into the pixel sum (scene.cpp:41-42)
        sum = rtv::add(sum, fold_path(P, c.nv, shaded));
        if (++c.s == spp) {
            out[3 * (long long)pix + 0] = sum.x;
            out[3 * (long long)pix + 1] = sum.y;
            out[3 * (long long)pix + 2] = sum.z;
            need_pixel = true;
        } else {
            r = pool_camera(sc, g, pix, rng, c);
        }
    }
    push = !need_pixel;
    if (!need_pixel) {
        pool_store_ray(V, p, r, root, pix);
        *V.D(p) = make_float4(sum.x, sum.y, sum.z, __uint_as_float(rng_word_pack(rng.x, rng.saved_avail)));
        *V.E(p) = make_float4(rng.saved, __uint_as_float(pool_ctr(c)), 0.f, 0.f);
    }
    return need_pixel;
}

}  // namespace rtd
#endif
