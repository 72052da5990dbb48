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
//   A (origin, shard pixel)   B (direction, LaneCtr)   D (pixel sum, RNG word: minstd state |
//   normal-cache flag << 31)   E (normal cache, 0, 0, 0)
//   C: while queued, (1 / direction, 0) (Ray::inv, so a refill loads the ray and computes
//      nothing before its first traversal step); once traversed, the closest hit (t, u, v, prim)
// A queued ray always enters the root box: the shading pass resolves a ray that misses it
// (BVH::intersect returns at the root, bvh.cpp:239-243) itself, as a path end.
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

// RT_POOL_NT: path-record loads and stores non-temporal (A/B: keep them from evicting the
// scene's BVH and triangle lines from L2 and the Infinity Cache).
#ifndef RT_POOL_NT
#define RT_POOL_NT 0
#endif
__device__ __forceinline__ float4 pool_ld(const float4 *p) {
#if RT_POOL_NT
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(p));
    return make_float4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ void pool_st(float4 *p, float4 v) {
#if RT_POOL_NT
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4f *>(p));
#else
    *p = v;
#endif
}

struct PoolPlanes {
    float4 *base;   // WfState::mid: 5 planes
    long long n;    // plane stride (paths)
    // a uniform base and a 32-bit byte offset (5 planes x paths x 16 B < 4 GiB)
    __device__ __forceinline__ float4 *at(int plane, long long p) const {
        return (float4 *)((char *)base + (size_t)(((uint32_t)plane * (uint32_t)n + (uint32_t)p) << 4));
    }
    __device__ __forceinline__ float4 *A(long long p) const { return at(0, p); }
    __device__ __forceinline__ float4 *B(long long p) const { return at(1, p); }
    __device__ __forceinline__ float4 *C(long long p) const { return at(2, p); }
    __device__ __forceinline__ float4 *D(long long p) const { return at(3, p); }
    __device__ __forceinline__ float4 *E(long long p) const { return at(4, p); }
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

// The ray of a queued path as traversal needs it (origin, direction, Ray::inv): three loads,
// nothing computed from them before the traversal's first step.
__device__ __forceinline__ Ray pool_load_ray(const PoolPlanes &V, long long p) {
    const float4 a = pool_ld(V.A(p)), b = pool_ld(V.B(p)), c = pool_ld(V.C(p));
    Ray r;
    r.o = V3{a.x, a.y, a.z};
    r.d = V3{b.x, b.y, b.z};
    r.inv = V3{c.x, c.y, c.z};
    return r;
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

// A path in registers during a shading pass.
struct PoolPath {
    Ray r;
    Hit h;       // the closest hit of r (prim -1: none)
    int pix;
    LaneCtr c;
    V3 sum;
    Rng rng;
};

// What a path needs after a shading pass or a new pixel (pool_advance, pool_assign).
enum PoolNext : int { PN_QUEUE = 0, PN_READY = 1, PN_PIXEL = 2 };

// Path P's ray and state to its record.  A ray that enters the root box is queued for
// traversal (C = Ray::inv); one that misses it has no hit (BVH::intersect returns at the root,
// bvh.cpp:239-243: a query with its one box test), so C gets "no hit" and the path goes
// straight to the ready ring.
template <bool COUNT>
__device__ __forceinline__ int pool_store(const PoolPath &Q, const PoolPlanes &V, long long p, const NodeRec &root,
                                          Counters &cnt) {
    float e;
    const bool in = box_hit<false>(root.mn, root.mx, Q.r, e);
    if (COUNT && !in) { cnt.rays++; cnt.aabb++; }
    pool_st(V.A(p), make_float4(Q.r.o.x, Q.r.o.y, Q.r.o.z, __int_as_float(Q.pix)));
    pool_st(V.B(p), make_float4(Q.r.d.x, Q.r.d.y, Q.r.d.z, __uint_as_float(pool_ctr(Q.c))));
    pool_st(V.C(p), in ? make_float4(Q.r.inv.x, Q.r.inv.y, Q.r.inv.z, 0.f) : make_float4(1e9f, 0.f, 0.f, __int_as_float(-1)));
    pool_st(V.D(p), make_float4(Q.sum.x, Q.sum.y, Q.sum.z, __uint_as_float(rng_word_pack(Q.rng.x, Q.rng.saved_avail))));
    pool_st(V.E(p), make_float4(Q.rng.saved, 0.f, 0.f, 0.f));
    return in ? PN_QUEUE : PN_READY;
}

// Path P from its closest hit to its next ray: one vertex of Scene::intersect (scene.cpp:85-154)
// and the bounce, or the path's end (fold into the pixel sum, scene.cpp:41-42) and the next
// sample's camera ray (PN_QUEUE / PN_READY, pool_store), or the pixel's end (its sum written
// out: PN_PIXEL).
template <bool COUNT, class Stack>
__device__ __forceinline__ int pool_advance(PoolPath &Q, const PoolPlanes &V, long long p, const DevScene &sc,
                                            const ShardGeom &g, const WfState &st, int spp, float *out,
                                            const NodeRec &root, Stack &stk, Counters &cnt) {
    LaneRec P{st.rec_ab, st.rec_c, p, st.lanes, V3{0.f, 0.f, 0.f}, 0, false};
    bool next = false;
    const bool shaded = Q.h.prim >= 0 && Q.h.t < sc.max_distance;
    if (shaded) {
        const bool cont = shade_hit<COUNT>(sc, Q.r, Q.h, Q.rng, cnt, P, Q.c.nv, stk);
        if (cont && Q.c.power > 0) {
            Q.c.power -= 1;
            next = true;
        }
    }
    if (!next) {   // the path ends here
        Q.sum = rtv::add(Q.sum, fold_path(P, Q.c.nv, shaded));
        if (++Q.c.s == spp) {
            out[3 * (long long)Q.pix + 0] = Q.sum.x;
            out[3 * (long long)Q.pix + 1] = Q.sum.y;
            out[3 * (long long)Q.pix + 2] = Q.sum.z;
            return PN_PIXEL;
        }
        Q.r = pool_camera(sc, g, Q.pix, Q.rng, Q.c);
    }
    return pool_store<COUNT>(Q, V, p, root, cnt);
}

// Path p takes pixel `pix`: RNG seeded from the pixel (scene.cpp:34, random.cpp:12-18; pixel 0
// -> 1), empty sum, sample 0's camera ray.
template <bool COUNT>
__device__ __forceinline__ int pool_assign(const PoolPlanes &V, long long p, const DevScene &sc, const ShardGeom &g,
                                           int pix, const NodeRec &root, Counters &cnt) {
    const int k = pix / g.width, px = pix - k * g.width, py = shard_row(g, k);
    const uint32_t seed = (uint32_t)(py * sc.width + px) % 2147483647u;
    PoolPath Q;
    Q.pix = pix;
    Q.rng = Rng{seed == 0 ? 1u : seed, 0u, 0.f};
    Q.c = LaneCtr{0, 0, 0};
    Q.sum = V3{0.f, 0.f, 0.f};
    Q.r = pool_camera(sc, g, pix, Q.rng, Q.c);
    return pool_store<COUNT>(Q, V, p, root, cnt);
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

// Shade ready path p (closest hit h4: t, u, v, prim): its record into registers, then
// pool_advance (returns its PoolNext).
template <bool COUNT, class Stack>
__device__ __forceinline__ int pool_shade(const PoolPlanes &V, long long p, const float4 h4, const DevScene &sc,
                                          const ShardGeom &g, const WfState &st, int spp, float *out,
                                          const NodeRec &root, Stack &stk, Counters &cnt) {
    const float4 a = pool_ld(V.A(p)), b = pool_ld(V.B(p)), d4 = pool_ld(V.D(p)), e4 = pool_ld(V.E(p));
    PoolPath Q;
    Q.r.o = V3{a.x, a.y, a.z};
    Q.r.d = V3{b.x, b.y, b.z};
    Q.r.inv = V3{0.f, 0.f, 0.f};   // (shading reads o and d only; a new ray computes its own)
    Q.pix = __float_as_int(a.w);
    Q.c = pool_ctr_unpack(__float_as_uint(b.w));
    Q.h = Hit{h4.x, h4.y, h4.z, __float_as_int(h4.w)};
    rng_word_unpack(__float_as_uint(d4.w), Q.rng.x, Q.rng.saved_avail);
    Q.rng.saved = e4.x;
    Q.sum = V3{d4.x, d4.y, d4.z};
    return pool_advance<COUNT>(Q, V, p, sc, g, st, spp, out, root, stk, cnt);
}

}  // namespace rtd
#endif
