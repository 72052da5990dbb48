// rt_wavefront.h — wavefront path tracer for gfx950 (the default render path).
//
// The per-pixel sample loop (scene.cpp:31-52) is split into three kernels over path
// slots (one slot = one pixel of the shard, carrying its RNG stream, pixel sum and the
// current path's vertex records in structure-of-arrays HBM buffers):
//   wf_init    seed every slot's RNG (pixel index), start its first sample (camera ray);
//   wf_extend  closest-hit BVH traversal for every queued ray — a lean kernel (ray in,
//              hit out, traversal state in registers) so many waves are resident and all
//              lanes run the same traversal code;
//   wf_shade   shade every queued hit (emission, normal map, sampling with the slot's RNG,
//              light pdf, BRDF record); then either queue the bounce ray, or fold the path,
//              add it to the pixel sum and queue the next sample's camera ray.
// Each slot advances one ray per iteration in its own exact order, so the output is
// bit-identical to the reference's per-pixel recursion.  Queues are compacted with one
// atomic per wave (ballot + mbcnt ranks keep lane order).
#pragma once
#include "rt_path.h"

namespace rtd {

// Pixel-row shard geometry (include/rt_hw.h rt_params): the k-th owned row of rank r is
// the k-th row whose (row / row_block) % world == rank.
// Pixel p of the shard is (p % width, shard_row(p / width)).  The two divisions by uniform
// divisors run as multiply-and-shift with host-made constants (div_magic): with a plain `/`
// the compiler computes the divisor's reciprocal on the VALU once and holds it, per lane, in
// a VGPR through the whole lane-resident kernel (two of its spilled VGPRs).
struct ShardGeom {
    int width, rank, world, row_block;
    long long n_pixels;
    uint32_t wm, rbm;   // div_magic constants of width and row_block (shard_geom)
    int ws, rbs;
};
// n / d for 0 <= n < 2^31 and d >= 1 (Granlund-Montgomery with N = 31: l = ceil(log2 d),
// m = ceil(2^(31 + l) / d) < 2^32, s = 31 + l; exact for every such n).  Pixel indices and
// shard rows are below 2^31 (the host rejects larger frames).
__device__ __forceinline__ int div_magic(int n, uint32_t m, int s) {
    return (int)(((unsigned long long)(uint32_t)n * m) >> s);
}
inline void div_magic_make(uint32_t d, uint32_t &m, int &s) {
    int l = 0;
    while ((1ull << l) < d) ++l;
    s = 31 + l;
    m = (uint32_t)(((1ull << s) + d - 1) / d);
}
inline ShardGeom shard_geom(int width, int rank, int world, int row_block, long long n_pixels) {
    ShardGeom g{width, rank, world, row_block, n_pixels, 0u, 0u, 0, 0};
    div_magic_make((uint32_t)width, g.wm, g.ws);
    div_magic_make((uint32_t)row_block, g.rbm, g.rbs);
    return g;
}
__device__ __forceinline__ int shard_row(const ShardGeom &g, int k) {
    const int blk = div_magic(k, g.rbm, g.rbs);
    return (blk * g.world + g.rank) * g.row_block + (k - blk * g.row_block);
}
// Column and frame row of shard pixel p.
__device__ __forceinline__ void shard_xy(const ShardGeom &g, long long p, int &px, int &py) {
    const int k = div_magic((int)p, g.wm, g.ws);
    px = (int)p - k * g.width;
    py = shard_row(g, k);
}

struct WfState {
    long long n;      // path slots (= pixels of the shard)
    int D;            // vertex records per slot (= ray_depth)
    int round_min;    // runahead kernel: trav_step_coop's round_min (host: scene size)
    float4 *st;       // 2 per slot: (rng state bits, normal cache, meta bits, 0), (pixel sum, 0)
    float4 *rec_ab;   // AosRec: 2 per slot and vertex; LaneRec: 2 per vertex and lane slot
    float *rec_c;     //         1 per slot and vertex; LaneRec: alpha per vertex and lane slot
    long long lanes;  // lane-resident kernel: lane slots (LaneRec stride; rt_path.h)
    float4 *mid;      // light-split kernel: shading state across the light walk, 5 per lane slot (rt_mega.h)
};
// meta: samples done (bits 0-19), depth budget left (20-23), vertices recorded (24-27),
// normal cache valid (28)

__device__ __forceinline__ void store_hit(float4 *hits, unsigned p, const Hit &h) {
    hits[p] = make_float4(h.t, h.u, h.v, __int_as_float(h.prim));
}
__device__ __forceinline__ Hit load_hit(const float4 *hits, unsigned p) {
    const float4 a = hits[p];
    return Hit{a.x, a.y, a.z, __float_as_int(a.w)};
}

__device__ __forceinline__ uint32_t meta_pack(int s, int power, int nv, uint32_t saved) {
    return (uint32_t)s | ((uint32_t)power << 20) | ((uint32_t)nv << 24) | (saved << 28);
}

#ifdef __HIPCC__
// Position of this lane's entry in a queue when `want` (else undefined): one atomic per
// wave, lanes keep their order.
__device__ __forceinline__ unsigned queue_slot(bool want, unsigned *count) {
    const unsigned long long m = __ballot(want);
    if (!m) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(count, (unsigned)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
}

template <bool COUNT>
__device__ __forceinline__ void counters_flush(const Counters &c, unsigned long long *out) {
    if (!COUNT) return;
    unsigned long long v[7] = {c.rays, c.aabb, c.tri, c.lq, c.laabb, c.ltri, c.hits};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        unsigned long long x = v[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&out[k], x);
    }
}
#endif

// ---------------------------------------------------------------- extend traversal
// BVH::intersect (bvh.cpp:177-243) for the extend kernel.  Same visits, same counters and
// same winner as closest_hit() in rt_path.h, with less memory traffic per internal node:
//   * both children of a node are fetched together — they are siblings (left, left+1) and
//     the device copy of the node array is offset so every sibling pair is one 64-B line;
//   * both child boxes are tested on arrival.  The reference tests the far box only after
//     the near subtree returns, but the test is a pure function of (ray, box) and is always
//     executed, so computing it early changes nothing; only the cull `dist > near best`
//     has to wait for the near subtree;
//   * frames are 8 bytes and carry the far child itself (its a/b fields and entry distance),
//     so resuming a node never re-reads it:
//       far frame  (a << 10 | b, entry distance)  pushed when both children are hit;
//       best frame (kFrameAcc,  node's near best)  pushed when the far child is entered
//                                                  after a near subtree.
//     No frame is needed when a node has only one child to visit: its local best starts at
//     1e9, so merging it is the identity.
constexpr uint32_t kFrameMaxA = (1u << 22) - 1;
constexpr uint32_t kFrameAcc = 0xffffffffu;

__device__ __forceinline__ void load_pair(const float4 *nodes, uint32_t left, NodeRec &L, NodeRec &R) {
    const float4 p0 = nodes[2 * left], q0 = nodes[2 * left + 1], p1 = nodes[2 * left + 2], q1 = nodes[2 * left + 3];
    L.mn[0] = p0.x; L.mn[1] = p0.y; L.mn[2] = p0.z; L.mx[0] = p0.w; L.mx[1] = q0.x; L.mx[2] = q0.y;
    L.a = __float_as_uint(q0.z); L.b = __float_as_uint(q0.w);
    R.mn[0] = p1.x; R.mn[1] = p1.y; R.mn[2] = p1.z; R.mx[0] = p1.w; R.mx[1] = q1.x; R.mx[2] = q1.y;
    R.a = __float_as_uint(q1.z); R.b = __float_as_uint(q1.w);
}

// aabb_hit() (rt_path.h; AABB::intersect, primitive.cpp:146-208) without branches: every
// lane evaluates the same operations and the early returns become selects, so a wave does
// not serialise on the inside / behind / outside cases.  Identical results; the entry
// distance (a sqrt) only when DIST.
// The test itself; `coord` is the entry point (the inside case leaves it unused).
__device__ __forceinline__ bool box_hit_pt(const float mn[3], const float mx[3], const Ray &r, float coord[3],
                                           bool &inside_out) {
    const float o[3] = {r.o.x, r.o.y, r.o.z};
    const float d[3] = {r.d.x, r.d.y, r.d.z};
    const float inv[3] = {r.inv.x, r.inv.y, r.inv.z};
    // (bitwise & | on the conditions: short-circuit && || would be compiled to branches)
    bool inside = true;
    bool mid[3];
    float cand[3], maxT[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const bool lo = o[i] < mn[i];
        const bool hi = !lo & (o[i] > mx[i]);
        mid[i] = !lo & !hi;
        cand[i] = lo ? mn[i] : (hi ? mx[i] : 0.f);
        inside = inside & mid[i];
        maxT[i] = (!mid[i] & (d[i] != 0.f)) ? (cand[i] - o[i]) * inv[i] : -1.f;
    }
    const bool w1 = maxT[0] < maxT[1];
    const float t01 = w1 ? maxT[1] : maxT[0];
    const bool w2 = t01 < maxT[2];
    const float tw = w2 ? maxT[2] : t01;
    const bool on[3] = {(bool)(!w1 & !w2), (bool)(w1 & !w2), w2};
    bool out = tw < 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float c = o[i] + tw * d[i];
        coord[i] = on[i] ? cand[i] : c;
        out = out | (!on[i] & ((c < mn[i]) | (c > mx[i])));
    }
    inside_out = inside;
    return inside || !out;
}
// Entry distance of a box from box_hit_pt's results (0 from inside).  (Round 4: the root as
// the hardware sqrt plus the residual correction, without the compiler's scaling and class
// handling, and a branch to sqrtf outside [2^-96, max]: exact over every float, but 1143 vs
// 1136 ms: the branch costs more than the selects it saves; profiles/r04f_park_sqrt_ab.jsonl.)
__device__ __forceinline__ float box_dist(const float coord[3], bool inside, const Ray &r) {
    const float l = rtv::length(rtv::sub(V3{coord[0], coord[1], coord[2]}, r.o));
    return inside ? 0.f : l;
}
template <bool DIST>
__device__ __forceinline__ bool box_hit(const float mn[3], const float mx[3], const Ray &r, float &dist) {
    float coord[3];
    bool inside;
    const bool hit = box_hit_pt(mn, mx, r, coord, inside);
    if (DIST) dist = box_dist(coord, inside, r);
    return hit;
}

// Both boxes of a child pair at once: the same operations as box_hit_pt on each, arranged
// for fewer instructions:
//   * the candidate plane is `lo ? min : max`: box_hit_pt's 0 for a Mid axis is never
//     used (a Mid axis has maxT = -1 and only wins when the box is missed);
//   * dir != 0 is tested once for both boxes;
//   * the entry point is selected only for the far box (`lf`: the left box is the near one),
//     the only one whose distance traversal needs.
__device__ __forceinline__ void box_pair_hit(const NodeRec &L, const NodeRec &R, const Ray &r, bool lf, bool &hL, bool &hR,
                                             float coordF[3], bool &insideF) {
    // (the conditions are kept in positive form -- "outside the slab", "off the winning
    // plane" -- so that few of them need a negation: each negation of a wave mask is a
    // scalar instruction)
    const float o[3] = {r.o.x, r.o.y, r.o.z};
    const float d[3] = {r.d.x, r.d.y, r.d.z};
    const float inv[3] = {r.inv.x, r.inv.y, r.inv.z};
    bool anyL = false, anyR = false;   // some axis has the origin outside the slab (not inside)
    float candL[3], candR[3], mtL[3], mtR[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const bool loL = o[i] < L.mn[i], loR = o[i] < R.mn[i];
        const bool outL = loL | (o[i] > L.mx[i]), outR = loR | (o[i] > R.mx[i]);   // quadrant != Mid
        anyL = anyL | outL;
        anyR = anyR | outR;
        candL[i] = loL ? L.mn[i] : L.mx[i];
        candR[i] = loR ? R.mn[i] : R.mx[i];
        const bool dnz = d[i] != 0.f;
        const float tL = (candL[i] - o[i]) * inv[i], tR = (candR[i] - o[i]) * inv[i];
        mtL[i] = (outL & dnz) ? tL : -1.f;
        mtR[i] = (outR & dnz) ? tR : -1.f;
    }
    const bool w1L = mtL[0] < mtL[1], w1R = mtR[0] < mtR[1];
    const float t01L = w1L ? mtL[1] : mtL[0], t01R = w1R ? mtR[1] : mtR[0];
    const bool w2L = t01L < mtL[2], w2R = t01R < mtR[2];
    const float twL = w2L ? mtL[2] : t01L, twR = w2R ? mtR[2] : t01R;
    // off the winning plane (whichPlane != i): axis 0 loses to 1 or 2, axis 1 loses to 0 or 2
    const bool offL[3] = {(bool)(w1L | w2L), (bool)(!w1L | w2L), (bool)!w2L};
    const bool offR[3] = {(bool)(w1R | w2R), (bool)(!w1R | w2R), (bool)!w2R};
    bool missL = twL < 0.f, missR = twR < 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float cL = o[i] + twL * d[i], cR = o[i] + twR * d[i];
        missL = missL | (offL[i] & ((cL < L.mn[i]) | (cL > L.mx[i])));
        missR = missR | (offR[i] & ((cR < R.mn[i]) | (cR > R.mx[i])));
        coordF[i] = lf ? (offR[i] ? cR : candR[i]) : (offL[i] ? cL : candL[i]);
    }
    hL = !(anyL & missL);   // inside, or the entry point lies on the box
    hR = !(anyR & missR);
    insideF = lf ? !anyR : !anyL;
}

// 1.f / x, correctly rounded, in three instructions where that is exact: the hardware
// reciprocal (about 1 ulp) and one fma Newton correction, which rounds correctly for every
// normal x with a normal reciprocal — checked on the device over every such float
// (rt_device_selfcheck 0, tests/test_gpu_parity.py).  Other x (denormal or huge, inf, NaN)
// take the IEEE division in a branch no real triangle reaches.  The host build divides.
__device__ __forceinline__ float rcp_ieee(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float ax = __builtin_fabsf(x);
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y0, 1.f);
    float y = __builtin_fmaf(e, y0, y0);
    if (__builtin_expect(!((ax >= 0x1p-126f) & (ax < 0x1p125f)), 0)) y = 1.f / x;
    return y;
#else
    return 1.f / x;
#endif
}

// tri_hit() (rt_path.h; Primitive::intersect, primitive.cpp:17-57) as selects.
__device__ __forceinline__ bool tri_hit_bl(V3 v0, V3 U, V3 V, const Ray &r, TriHit &h) {
    const V3 p = rtv::cross(r.d, V);
    const float det = rtv::dot(U, p);
    // -1e-6 < (double)det < 1e-6 in float: 0x1.0c6f7cp-20f is the least float above the double
    // 1e-6, so the double compares and |det| < it agree on every float (NaN included)
    const bool ok_det = !(__builtin_fabsf(det) < 0x1.0c6f7cp-20f);
    const float inv_det = rcp_ieee(det);
    const V3 s = rtv::sub(r.o, v0);
    const float u = inv_det * rtv::dot(s, p);
    const V3 q = rtv::cross(s, U);
    const float v = inv_det * rtv::dot(r.d, q);
    const float t = inv_det * rtv::dot(V, q);
    h.t = t;
    h.u = u;
    h.v = v;
    return ok_det & !((u < 0) | (u > 1)) & !((v < 0) | (u + v > 1)) & !(t < 0.f);
}

// Queues hold the rays themselves, 48 bytes per entry, so the extend kernel gets a ray with
// three coalesced 16-byte loads and nothing to recompute:
//   [3q]     (origin, slot bits)
//   [3q + 1] (dir, bits: dir-sign mask (bit i: dir[i] > 0) | root-box miss << 3)
//   [3q + 2] (1 / dir, 0)             -- Ray::Ray's inv_direction, computed once by the producer
// The producer (wf_init / wf_shade) also runs the root box test of BVH::intersect
// (bvh.cpp:239-243), a pure function of the ray, so traversal lanes start at the root's
// children.  Hits are written by queue position, 16 bytes: (t, u, v, prim bits).
constexpr int kQRec = 3;   // float4 per queue entry
__device__ __forceinline__ void store_qray(const DevScene &sc, float4 *q, unsigned p, int slot, const Ray &r) {
    const NodeRec root = load_node(sc.node, 0);
    float e;
    const bool hit = box_hit<false>(root.mn, root.mx, r, e);
    const uint32_t bits = (r.d.x > 0 ? 1u : 0u) | (r.d.y > 0 ? 2u : 0u) | (r.d.z > 0 ? 4u : 0u) | (hit ? 0u : 8u);
    q[kQRec * (size_t)p] = make_float4(r.o.x, r.o.y, r.o.z, __int_as_float(slot));
    q[kQRec * (size_t)p + 1] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(bits));
    q[kQRec * (size_t)p + 2] = make_float4(r.inv.x, r.inv.y, r.inv.z, 0.f);
}
// The ray as the shade kernel needs it (origin, direction).
__device__ __forceinline__ Ray load_qray(const float4 *q, unsigned p, int &slot) {
    const float4 a = q[kQRec * (size_t)p], b = q[kQRec * (size_t)p + 1];
    Ray r;
    r.o = V3{a.x, a.y, a.z};
    r.d = V3{b.x, b.y, b.z};
    r.inv = V3{0.f, 0.f, 0.f};
    slot = __float_as_int(a.w);
    return r;
}
// The ray as the extend kernel needs it (+ inv_direction, dir signs, root-box result).
__device__ __forceinline__ Ray load_qray_trav(const float4 *q, unsigned p, uint32_t &bits, int &slot) {
    const float4 a = q[kQRec * (size_t)p], b = q[kQRec * (size_t)p + 1], c = q[kQRec * (size_t)p + 2];
    Ray r;
    r.o = V3{a.x, a.y, a.z};
    r.d = V3{b.x, b.y, b.z};
    r.inv = V3{c.x, c.y, c.z};
    bits = __float_as_uint(b.w);
    slot = __float_as_int(a.w);
    return r;
}
// Dense-queue entry of a slot that has finished all its samples.
__device__ __forceinline__ void store_qray_inactive(float4 *q, unsigned p) {
    q[kQRec * (size_t)p] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
}

// Leaf triangles tested per traversal step.  A node lane and a leaf lane read through the
// same registers: 4 x 16 B of the child pair, or of triangle k (its 3 x 16 B and the next
// record's first), then 3 x 16 B per further triangle.  Sponza 1080p x256spp, lane-resident
// kernel: 2 is +3.6% at 1 GPU over 1 and -7% on the rank-0 shard of an 8-way split; 3 and 4
// lose at 1 GPU (more registers live across the step).  (Host tests build other values.)
#ifndef RT_LEAF_N
#define RT_LEAF_N 2
#endif

// Resumable traversal state of one ray.  Two layouts: TravState keeps the node fields and
// the leaf range in four registers; TravStateU shares two registers between them (a node
// step never reads k / kend, a leaf step never reads a / b), so a traversing lane holds two
// registers fewer through another lane's shading pass.  The lane-resident kernel uses
// TravStateU: 53 -> 50 spilled VGPRs, 1145 -> 1132 ms (r03s5).  The runahead kernel keeps
// TravState: with the shared layout its 8-way shards measured 0.8% slower (205 vs 203 ms mean).
enum TravPhase : int { TP_NODE = 0, TP_LEAF = 1, TP_POP = 2 };
static_assert(TP_POP < 4 && kStack < 128, "rt_mega_kernel packs phase in 2 bits and sp in 7 (RT_PACK_TRAV)");
template <bool SHARED> struct TravFields;
template <> struct TravFields<false> {
    uint32_t a, b;      // TP_NODE: internal node being entered (b = split axis, a = left child)
    uint32_t k, kend;   // TP_LEAF: triangles still to test
};
template <> struct TravFields<true> {
    union { uint32_t a; uint32_t k; };      // TP_NODE: left child / TP_LEAF: next triangle
    union { uint32_t b; uint32_t kend; };   // TP_NODE: split axis / TP_LEAF: end of the leaf's range
};
template <bool SHARED>
struct TravStateT : TravFields<SHARED> {
    static constexpr bool kShared = SHARED;
    float acc;       // best t inside the subtree being traversed (the reference's local best)
    int sp;
    int phase;
    Hit best;        // global winner so far (strict <, first of equal t wins)
};
using TravState = TravStateT<false>;
using TravStateU = TravStateT<true>;

// Where trav_step reads child pairs from: the breadth-first node array in HBM.
struct GlobalNodes {
    const float4 *node;
    __device__ __forceinline__ const float4 *pair(uint32_t left) const { return node + 2 * (size_t)left; }
    __device__ __forceinline__ void load_pair(uint32_t left, NodeRec &L, NodeRec &R) const {
        rtd::load_pair(node, left, L, R);
    }
};

// Host / test stack: a plain array.
struct ArrayStack {
    uint2 *p;
    __device__ __forceinline__ void put(int i, uint2 v) { p[i] = v; }
    __device__ __forceinline__ uint2 get(int i) const { return p[i]; }
};

// Enter a node given its (a, b) fields: internal -> TP_NODE, leaf -> TP_LEAF (an empty
// leaf returns at once).
template <class TS>
__device__ __forceinline__ void trav_enter(TS &T, uint32_t a, uint32_t b) {
    if constexpr (TS::kShared) {
        const bool node = b < 3u;
        T.a = a;                            // = T.k
        T.b = node ? b : a + (b >> 2);      // = T.kend for a leaf
        T.phase = node ? TP_NODE : ((b >> 2) != 0u ? TP_LEAF : TP_POP);
    } else {
        T.a = a;
        T.b = b;
        T.k = a;
        T.kend = a + (b >> 2);
        T.phase = b < 3u ? TP_NODE : (T.kend > T.k ? TP_LEAF : TP_POP);
    }
}

// BVH::intersect entry (bvh.cpp:239-243) for a queued ray: counters, and the root box
// result the producer stored (bits from load_qray_trav).  False = the ray misses the scene
// (T.best says so).  (root_a, root_b) are the root node's fields.
template <bool COUNT, class TS>
__device__ __forceinline__ bool trav_start(uint32_t bits, uint32_t root_a, uint32_t root_b, TS &T,
                                           Counters &cnt) {
    if (COUNT) { cnt.rays++; cnt.aabb++; }
    T.best.t = 1e9f;
    T.best.prim = -1;
    T.best.u = T.best.v = 0.f;
    T.sp = 0;
    T.acc = 1e9f;
    trav_enter(T, root_a, root_b);
    return (bits & 8u) == 0;
}

// Frames one step pops at most; the rest wait for the lane's next step (T.phase stays
// TP_POP), so a lane that unwinds many frames no longer holds its whole wave in the pop
// loop: sponza 1080p 1280 -> 1148 ms, slowest 8-way shard 246 -> 217 ms, C5 at 16 spp
// 348 -> 308 ms; 1 pop: 1150 / 219 ms, 3: 1164 / 221 (profiles/r03_ab.jsonl r03y).  0: no cap.
#ifndef RT_MAX_POPS
#define RT_MAX_POPS 2
#endif
constexpr int kMaxPops = RT_MAX_POPS;
// The return of trav_step: merge subtree bests upwards until a far child is to be visited
// (enter it: false), the stack is empty (T.best is final: true) or kMaxPops frames are
// popped (false, still TP_POP).
template <class Stack, class TS>
__device__ __forceinline__ bool trav_pop(TS &T, Stack &stk) {
    float acc = T.acc;
    int sp = T.sp;
    for (int n = 0;; ++n) {
        if (sp == 0) {
            T.sp = 0;
            T.acc = acc;
            return true;
        }
        if (kMaxPops > 0 && n == kMaxPops) {   // the rest next step (T.phase stays TP_POP)
            T.sp = sp;
            T.acc = acc;
            return false;
        }
        const uint2 f = stk.get(--sp);
        if (f.x == kFrameAcc) {
            const float p = __uint_as_float(f.y);
            acc = acc < p ? acc : p;
            continue;
        }
        if (!(__uint_as_float(f.y) > acc)) {   // far child survives the near subtree's best
            stk.put(sp++, make_uint2(kFrameAcc, __float_as_uint(acc)));
#ifdef RT_STACK_PROBE
            RT_STACK_PROBE(sp);
#endif
            T.sp = sp;
            T.acc = 1e9f;
            trav_enter(T, f.x >> 10, f.x & 1023u);
            return false;
        }
    }
}

// The node part of a traversal step: the child pair q[0..3] (two 32-B node records) of the
// internal node T is entering; pushes the far child when both are hit, enters the near one
// (or the far one alone, or returns: T.phase = TP_POP).
template <bool COUNT, class Stack, class TS>
__device__ __forceinline__ void node_step(const float4 q[4], const Ray &r, TS &T, Stack &stk, Counters &cnt) {
    NodeRec L, R;
    L.mn[0] = q[0].x; L.mn[1] = q[0].y; L.mn[2] = q[0].z; L.mx[0] = q[0].w; L.mx[1] = q[1].x; L.mx[2] = q[1].y;
    L.a = __float_as_uint(q[1].z); L.b = __float_as_uint(q[1].w);
    R.mn[0] = q[2].x; R.mn[1] = q[2].y; R.mn[2] = q[2].z; R.mx[0] = q[2].w; R.mx[1] = q[3].x; R.mx[2] = q[3].y;
    R.a = __float_as_uint(q[3].z); R.b = __float_as_uint(q[3].w);
    if (COUNT) cnt.aabb += 2;
    // dir[split axis] > 0: left child first (sign bits recomputed: cheaper than a register)
    const uint32_t dpos = (r.d.x > 0.f ? 1u : 0u) | (r.d.y > 0.f ? 2u : 0u) | (r.d.z > 0.f ? 4u : 0u);
    const bool lf = (dpos >> T.b) & 1u;
    // test both boxes as they are stored, then name them near / far
    float cF[3];
    bool hL, hR, inF;
    box_pair_hit(L, R, r, lf, hL, hR, cF, inF);
    const float ef = box_dist(cF, inF, r);   // the far child's entry distance
    const bool hn = lf ? hL : hR, hf = lf ? hR : hL;
    const uint32_t na = lf ? L.a : R.a, nb = lf ? L.b : R.b, fa = lf ? R.a : L.a, fb = lf ? R.b : L.b;
    if (hn && hf) {
        RT_CHECK(T.sp < kStack, 11, T.sp, T.sp = 0);
        stk.put(T.sp++, make_uint2((fa << 10) | fb, __float_as_uint(ef)));
#ifdef RT_STACK_PROBE
        RT_STACK_PROBE(T.sp);
#endif
    }
    // near child; or, the near box missed, the far child unless its entry distance
    // exceeds the node's local best (still 1e9); or return
    const bool far_only = !hn && hf && !(ef > 1e9f);
    if (hn || far_only) trav_enter(T, hn ? na : fa, hn ? nb : fb);
    else T.phase = TP_POP;
}

// One unit of traversal work: the child pair of one internal node, or RT_LEAF_N triangles
// of a leaf, followed (when the subtree is finished) by the return up the frames until a
// far child is to be visited.  Returns true once the stack is empty (T.best is final).  A
// wave's lanes each advance by one unit per call, whatever mix of units they are at.
// A leaf lane tests triangles k .. k + N - 1 in the reference's order (strict <, so the
// first of equal t wins), which is the sequence of N single-triangle steps.
// Both memory reads of the step issue before either test (node lanes and leaf lanes load
// through the same registers), so a wave split between node and leaf steps waits for one
// round trip per iteration, not two.
template <bool COUNT, class Stack, class Nodes, class TS>
__device__ __forceinline__ bool trav_step(const DevScene &sc, const Ray &r, TS &T, Stack &stk,
                                          const Nodes &nodes, Counters &cnt) {
    constexpr int N = RT_LEAF_N;
    const bool at_node = T.phase == TP_NODE, at_leaf = T.phase == TP_LEAF;
    const uint32_t k = T.k, klast = T.kend - 1u;
    RT_CHECK(!at_node || T.a + 1 < (uint32_t)sc.n_nodes, 10, T.a, T.a = 0);
    RT_CHECK(!at_leaf || T.kend <= (uint32_t)sc.n_tris, 12, T.kend, T.k = T.kend = 1);
    float4 q[4 + 3 * (N - 1)];
    {
        const float4 *p0 = at_node ? nodes.pair(T.a) : sc.tri + 3 * (size_t)(at_leaf ? k : 0u);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = p0[i];
#pragma unroll
        for (int j = 1; j < N; ++j) {
            const uint32_t kj = at_leaf ? (k + j < klast ? k + j : klast) : 0u;
            const float4 *pj = sc.tri + 3 * (size_t)kj;
#pragma unroll
            for (int i = 0; i < 3; ++i) q[4 + 3 * (j - 1) + i] = pj[i];
        }
#ifdef __HIPCC__
        // (pin the loads here: otherwise the compiler sinks each into its own branch again)
        asm volatile("" ::"v"(q[0].x), "v"(q[1].y), "v"(q[2].z), "v"(q[3].w));
#endif
    }
    if (at_node) {
        node_step<COUNT>(q, r, T, stk, cnt);
    } else if (at_leaf) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int o = j == 0 ? 0 : 4 + 3 * (j - 1);
            const V3 v0{q[o].x, q[o].y, q[o].z}, U{q[o].w, q[o + 1].x, q[o + 1].y}, V{q[o + 1].z, q[o + 1].w, q[o + 2].x};
            const bool valid = j == 0 || k + j <= klast;
            TriHit h;
            const bool hit = tri_hit_bl(v0, U, V, r, h) & valid;
            if (COUNT && valid) cnt.tri++;
            if (hit) {
                T.acc = h.t < T.acc ? h.t : T.acc;
                if (h.t < T.best.t) { T.best.t = h.t; T.best.u = h.u; T.best.v = h.v; T.best.prim = (int)(k + j); }
            }
        }
        T.k = k + N;
        if (T.k >= T.kend) T.phase = TP_POP;
    }
    if (T.phase == TP_POP) return trav_pop(T, stk);
    return false;
}

#ifdef __HIPCC__
// Device stack: the first K entries in LDS (entry k of thread t at [k * 256 + t], so a
// wave's 64 lanes hit consecutive 8-byte words), deeper entries in scratch.  K = 8 holds
// 96% of all pushes on the sponza frame (tools: RT_STACK_PROBE histogram), yet the scratch
// frames of the other 4% were the largest share of the kernel's HBM writes (scratch lines
// leave L2 before they are read back).  K = 11 fills the lane-resident kernel's block to
// 30 KB of LDS (5 blocks per CU still fit): sponza 1080p x256spp 1401 -> 1364 ms, WRITE_SIZE
// 124 -> 101 B per ray at K = 10; K = 12 (32 KB) drops a block per CU (1544 ms)
// (profiles/r02_lds_stack_ab.jsonl).  Round 3: K = 8 costs 4% (1195 vs 1143 ms, r03s2).  The
// lane-resident kernel's K = 12 fits in the same 31 KB since its RNG words and texel table
// shrank by 1 KB each (rt_mega.h lane_rng, rt_path.h texel_decode).  The runahead kernel runs
// 4 blocks per CU (40 KB each), so it holds RT_SPEC_LDS_STACK frames.  Each kernel has its
// own array (lds_stack_frames<K>).
#ifndef RT_LDS_STACK
#define RT_LDS_STACK 12
#endif
#ifndef RT_SPEC_LDS_STACK
#define RT_SPEC_LDS_STACK 15
#endif
constexpr int kLdsStack = RT_LDS_STACK;   // stack frames per lane in LDS (deeper ones spill to scratch)
constexpr int kLdsStackSpec = RT_SPEC_LDS_STACK;   // the runahead kernel's
constexpr int kLdsStackWf = 11;                    // the wavefront extend kernel's
template <int K>
__device__ __forceinline__ uint2 *lds_stack_frames() {
    __shared__ uint2 frames[K * 256];   // blocks of 256 threads
    return frames;
}
template <int K>
struct LdsStackT {
    static_assert(K >= 1 && K < kStack, "LDS frames");
    uint2 *spill;   // this thread's private overflow array (scratch), kStack - K entries
    __device__ __forceinline__ void put(int i, uint2 v) {
        if (i < K) lds_stack_frames<K>()[i * 256 + threadIdx.x] = v;
        else spill[i - K] = v;
    }
    __device__ __forceinline__ uint2 get(int i) const {
        uint2 v;
        if (i < K) {
            v = lds_stack_frames<K>()[i * 256 + threadIdx.x];
        } else {
            v = spill[i - K];
            // keeps the two loads apart: merged, they become one flat load through a
            // selected pointer instead of a ds_read
            asm volatile("" : "+v"(v.x), "+v"(v.y));
        }
        return v;
    }
};

// Cooperative traversal step (the lane-resident kernel's inner loop, GPU only).  A wave's
// lanes are mostly at internal nodes, a few at leaves, and a per-lane step runs both code
// paths for the whole wave: the leaf path (RT_LEAF_N triangles, ~200 instructions) for a
// sixth of the work.  Here the leaf work is spread over the wave instead: each leaf lane
// (the first kCoopLeaves of them, by lane order) publishes its ray and triangle range in LDS,
// and lanes 4h .. 4h+3 of the wave, whatever their own state, test triangles k .. k+3 of the
// h-th leaf lane, one each.  A quad reduction finds the first of the hits with the least t
// (Primitive::intersect's strict <, bvh.cpp:226-232, in index order), which the leaf lane
// takes; so a leaf of up to 4 triangles is one step, with the reference's winner and local
// best.  Node lanes run node_step as in trav_step.  Every lane of the wave must call this
// (active: the lane is traversing); returns true once the lane's stack is empty.

// RT_UV_RECOMPUTE: the coop leaf step keeps only (t, triangle) of the closest hit; the
// shading pass recomputes (u, v) with the same Moller-Trumbore test of that triangle and ray
// (rt_mega.h mega_shade: same inputs, same operations, same bits), so a traversing lane holds
// two registers fewer through the whole loop and the quad reduction moves two values fewer.
// Round 5 (profiles/r05k_ab.jsonl, with RT_INV_RECOMPUTE): frame 1104-1107 ms vs 1132-1137,
// 8-way shards 184.6 vs 187.0-187.8 ms, WRITE_SIZE 0.372 vs 0.457 TB per frame.  0: A/B.
#ifndef RT_UV_RECOMPUTE
#define RT_UV_RECOMPUTE 1
#endif
constexpr bool kUvRecompute = RT_UV_RECOMPUTE != 0;

// (u, v) of a closest hit whose (t, triangle) the coop leaf step found (RT_UV_RECOMPUTE): the
// same Moller-Trumbore test of the same triangle and ray, so the bits the step would have kept.
__device__ __forceinline__ void hit_uv(const DevScene &sc, const Ray &r, Hit &h) {
    const float4 *t = sc.tri + 3 * (size_t)h.prim;
    const float4 t0 = t[0], t1 = t[1], t2 = t[2];
    TriHit th;
    tri_hit_bl(V3{t0.x, t0.y, t0.z}, V3{t0.w, t1.x, t1.y}, V3{t1.z, t1.w, t2.x}, r, th);
    h.u = th.u;
    h.v = th.v;
}

// One step of the quad reduction: take the partner lane's (t, u, v, index) when its t is
// less, or equal with a lower index.
template <int CTL>
__device__ __forceinline__ void quad_min_step(float &c, float &cu, float &cv, int &cj) {
    const float c2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(c), CTL, 0xF, 0xF, false));
    const int j2 = __builtin_amdgcn_mov_dpp(cj, CTL, 0xF, 0xF, false);
    const bool take = c2 < c || (c2 == c && j2 < cj);
    if (!kUvRecompute) {
        const float u2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(cu), CTL, 0xF, 0xF, false));
        const float v2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(cv), CTL, 0xF, 0xF, false));
        cu = take ? u2 : cu;
        cv = take ? v2 : cv;
    }
    c = take ? c2 : c;
    cj = take ? j2 : cj;
}


// kCoopLeaves: leaf lanes served per round (4 lanes of the wave each); their records take
// 32 B each per wave in LDS (the caller's kernel budget decides: DESIGN.md §6).
// round_min: unserved leaf lanes that start another round of the same step (> 64: one
// round per step).  A wave mostly at leaves (a scene of a few dozen triangles, whose tree
// is a few levels deep) otherwise serves kCoopLeaves of its leaf lanes per step and idles
// the rest (rt_device.hip kCoopRoundMin*).
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
// hook: called by every lane once the step's loads have all arrived (after the leaf rounds,
// before the node test): the pool kernel issues its previous step's hit store there, so that
// no wait of this step's loads also waits for that store (vmcnt counts loads and stores in
// issue order).
// MASK_LOAD: only the node lanes issue the child-pair loads (the others skip them instead of
// loading the root's pair).  Round 5 A/B (profiles/r05_memreq_ab.jsonl, two runs): the plain
// kernel (one GPU, lanes mostly traversing) 1175-1177 vs 1132-1133 ms, the runahead kernel
// (8-way shards, sparser waves) 202.8-202.9 vs 203.8-204.3 ms mean shard; so the runahead
// kernel takes it and the plain kernel does not.  Two other request shapes were measured and
// removed: quad-cooperative pair loads with a DPP transpose (1259 ms, 8-way 233 ms) and 36-B
// triangle loads (1132-1137 ms, 8-way 204 ms: neutral).
// Leaf deferral (both lane-resident kernels pass `leaf_defer`).  A step whose wave has
// fewer than RT_LEAF_DEFER leaf lanes, and some node lanes, leaves its leaf lanes for the next
// step (at most RT_LEAF_DEFER_MAX steps in a row), so that the coop step's three triangle
// loads and its triangle test run for more leaves at once; a leaf lane's triangles, their
// order and its closest hit are unchanged (same bits), it only reaches them a step or two
// later.  8-way shards of the headline frame, slowest / mean (profiles/r06s, r06t, two calls,
// two runs each): below 6 with at most 3 in a row 176.3-176.9 / 174.9-175.4 ms, below 6 with
// at most 2 176.3-177.6 / 175.3-175.5, below 4 / 5 / 7 / 8 / 10 179.2-180.1 / 178.4-179.2 /
// 177.1-178.4 / 177.1-177.9 / 179.0-179.7, against 183.5-184.5 / 181.5-182.3 without; then
// at most 4 in a row with the runahead kernel's shading threshold and coop records re-tuned
// (rt_device.hip RT_SPEC_SHADE_MIN).  The plain kernel (1 GPU) defers below 6 as well
// (RT_PLAIN_LEAF_DEFER): frame 1024.2-1025.3 ms against 1049.1-1051.1, 2-way 567.4-573.3
// against 572.3-576.6 (three runs each, profiles/r06z_plain_leaf_defer_ab.jsonl; below 8
// 1030.2-1033.6); below 2 / 3 it measured 1073 / 1064 ms against 1048, below 4 equal
// (profiles/r06r_leaf_defer_ab.jsonl, with at most 2 deferrals in a row).
#ifndef RT_LEAF_DEFER
#define RT_LEAF_DEFER 6
#endif
#ifndef RT_LEAF_DEFER_MAX
#define RT_LEAF_DEFER_MAX 4
#endif
constexpr int kLeafDefer = RT_LEAF_DEFER, kLeafDeferMax = RT_LEAF_DEFER_MAX;
// (the plain kernel's threshold; 0: it does not defer.  Counting renders do not defer: with it
// the counting kernel took 1508 instead of 1165 ms per frame, r06zz kernel trace)
#ifndef RT_PLAIN_LEAF_DEFER
#define RT_PLAIN_LEAF_DEFER 6
#endif
constexpr int kLeafDeferPlain = RT_PLAIN_LEAF_DEFER;
template <bool COUNT, int kCoopLeaves, bool MASK_LOAD, int DEFER = kLeafDefer, class Stack, class Nodes, class TS,
          class Hook = NoHook>
__device__ __forceinline__ bool trav_step_coop(const DevScene &sc, const Ray &r, TS &T, Stack &stk,
                                               const Nodes &nodes, Counters &cnt, bool active, int round_min,
                                               const Hook &hook = Hook{}, int *leaf_defer = nullptr) {
    static_assert(kCoopLeaves >= 1 && kCoopLeaves <= 16, "4 helper lanes per leaf lane");
    __shared__ float4 wf_coop_rec[4][kCoopLeaves][2];   // per wave: (origin, k), (direction, kend)
    const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
    const bool at_node = active && T.phase == TP_NODE, at_leaf = active && T.phase == TP_LEAF;
    RT_CHECK(!at_node || T.a + 1 < (uint32_t)sc.n_nodes, 10, T.a, T.a = 0);
    RT_CHECK(!at_leaf || T.kend <= (uint32_t)sc.n_tris, 12, T.kend, T.k = T.kend = 1);
    // node lanes: the child pair (issued first; consumed after the leaf exchange)
    float4 q[4];
    if (MASK_LOAD) {
        // (only the node lanes issue the pair loads: the others leave the address unit alone;
        // q is read only by node lanes: no initialisation, which would wait on the registers'
        // last loads)
        if (at_node) {
            const float4 *p0 = nodes.pair(T.a);
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = p0[i];
        }
    } else {
        const float4 *p0 = nodes.pair(at_node ? T.a : 0u);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = p0[i];
    }
    // leaf lanes publish (rank = position among the wave's leaf lanes); round b serves
    // ranks b*kCoopLeaves .. (b+1)*kCoopLeaves-1, and a further round runs while at least
    // round_min leaf lanes are left unserved (a wave mostly at leaves: small scenes)
    const unsigned long long lm = __ballot(at_leaf);
    const int n_leaf = __popcll(lm);
    const int lrank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
    bool skip_leaves = false;   // (wave-uniform)
    if (DEFER > 0 && leaf_defer) {
        if (n_leaf > 0 && n_leaf < DEFER && *leaf_defer < kLeafDeferMax && __ballot(at_node) != 0ull) {
            skip_leaves = true;
            ++*leaf_defer;
        } else {
            *leaf_defer = 0;
        }
    }
    for (int base = 0; !skip_leaves && base < n_leaf; base += kCoopLeaves) {   // (wave-uniform)
        if (base > 0 && n_leaf - base < round_min) break;
        const int rank = lrank - base;
        const bool served = at_leaf && rank >= 0 && rank < kCoopLeaves;
        if (base > 0) __builtin_amdgcn_wave_barrier();   // (the last round's records are read)
        if (served) {
            wf_coop_rec[wave][rank][0] = make_float4(r.o.x, r.o.y, r.o.z, __uint_as_float(T.k));
            wf_coop_rec[wave][rank][1] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(T.kend));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int n_served = n_leaf - base < kCoopLeaves ? n_leaf - base : kCoopLeaves;
        // helper lanes: one triangle each
        const int h = lane >> 2, j = lane & 3;
        float c = __builtin_inff(), cu = 0.f, cv = 0.f;
        if (h < n_served) {
            const float4 a = wf_coop_rec[wave][h][0], b = wf_coop_rec[wave][h][1];
            const uint32_t k = __float_as_uint(a.w) + (uint32_t)j;
            if (k < __float_as_uint(b.w)) {
                const float4 *t = sc.tri + 3 * (size_t)k;
                const float4 t0 = t[0], t1 = t[1], t2 = t[2];
                Ray hr;
                hr.o = V3{a.x, a.y, a.z};
                hr.d = V3{b.x, b.y, b.z};
                TriHit th;
                // (a NaN t never wins a strict < : it becomes "no hit" here)
                if (tri_hit_bl(V3{t0.x, t0.y, t0.z}, V3{t0.w, t1.x, t1.y}, V3{t1.z, t1.w, t2.x}, hr, th) &&
                    th.t == th.t) {
                    c = th.t;
                    cu = th.u;
                    cv = th.v;
                }
            }
        }
        // quad reduction: least t, first triangle of equal t; every lane of the quad ends
        // with it (DPP quad permutes: lane ^ 1, then lane ^ 2)
        int cj = j;
        quad_min_step<0xB1>(c, cu, cv, cj);   // quad_perm [1,0,3,2]: lane ^ 1
        quad_min_step<0x4E>(c, cu, cv, cj);   // quad_perm [2,3,0,1]: lane ^ 2
        const int src = 4 * (served ? rank : 0);
        const float wc = __shfl(c, src, 64);
        const float wu = kUvRecompute ? 0.f : __shfl(cu, src, 64), wv = kUvRecompute ? 0.f : __shfl(cv, src, 64);
        const int wj = __shfl(cj, src, 64);
        if (served) {
            if (COUNT) cnt.tri += (T.kend - T.k < 4u ? T.kend - T.k : 4u);
            if (wc < T.acc) T.acc = wc;
            if (wc < T.best.t) {
                T.best.t = wc;
                if (!kUvRecompute) {
                    T.best.u = wu;
                    T.best.v = wv;
                }
                T.best.prim = (int)(T.k + (uint32_t)wj);
            }
            T.k += 4u;
            if (T.k >= T.kend) T.phase = TP_POP;
        }
    }
    hook();
    // node lanes: the pair test
    if (at_node) node_step<COUNT>(q, r, T, stk, cnt);
    if (active && T.phase == TP_POP) return trav_pop(T, stk);
    return false;
}

#endif

// The whole closest-hit query through a queue record (host tests; the device kernel
// interleaves the steps of many rays).
template <bool COUNT>
__device__ __forceinline__ void closest_hit_wf(const DevScene &sc, const float4 *q, unsigned p, Hit &best, uint2 *stk,
                                               Counters &cnt) {
    uint32_t bits;
    int slot;
    const Ray r = load_qray_trav(q, p, bits, slot);
    const NodeRec root = load_node(sc.node, 0);
    TravState T;
    ArrayStack S{stk};
    const GlobalNodes nodes{sc.node};
    if (trav_start<COUNT>(bits, root.a, root.b, T, cnt))
        while (!trav_step<COUNT>(sc, r, T, S, nodes, cnt)) {
        }
    best = T.best;
}

// Start sample s of slot i: jittered camera ray (scene.cpp:36-39); the first traversal
// consumes one call of the depth budget (scene.cpp:72-75).
__device__ __forceinline__ Ray start_sample(const DevScene &sc, const ShardGeom &g, long long i, Rng &rng, int &power) {
    int px, py;
    shard_xy(g, i, px, py);
    const float ox = rng_offset(rng);
    const float oy = rng_offset(rng);
    power = sc.ray_depth - 1;
    return camera_ray(sc, px, py, ox, oy);
}

// ---------------------------------------------------------------- per-slot bodies
// The three kernels in rt_device.hip are these functions plus queue compaction; the host
// test harness (tests/native/kernel_host.cpp) runs the same functions with a host queue.

// wf_init: seed slot i's RNG from its pixel (scene.cpp:34, random.cpp:12-18; pixel 0 -> 1)
// and start its first sample; returns the camera ray.
__device__ __forceinline__ Ray wf_init_slot(const DevScene &sc, const ShardGeom &g, const WfState &st, long long i) {
    int px, py;
    shard_xy(g, i, px, py);
    const uint32_t seed = (uint32_t)(py * sc.width + px) % 2147483647u;
    Rng rng{seed == 0 ? 1u : seed, 0u, 0.f};
    int power = 0;
    const Ray r = start_sample(sc, g, i, rng, power);
    st.st[2 * i] = make_float4(__uint_as_float(rng.x), rng.saved, __uint_as_float(meta_pack(0, power, 0, rng.saved_avail)), 0.f);
    st.st[2 * i + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    return r;
}

// wf_shade: one vertex of scene.cpp:85-154 for slot i (ray r, its closest hit h), then
// bounce (true: r is the slot's next ray to extend) or end the path: fold it, add it to the
// pixel sum (scene.cpp:41-42) and start the next sample (true, r = its camera ray), or
// write the pixel after the last sample (false).
template <bool COUNT>
__device__ __forceinline__ bool wf_shade_slot(const DevScene &sc, const ShardGeom &g, const WfState &st, int spp,
                                              long long i, Ray &r, const Hit &h, float *out, Counters &cnt) {
    const float4 s0 = st.st[2 * i];
    const uint32_t meta = __float_as_uint(s0.z);
    int s = (int)(meta & 0xfffffu), power = (int)((meta >> 20) & 15u), nv = (int)((meta >> 24) & 15u);
    Rng rng{__float_as_uint(s0.x), (meta >> 28) & 1u, s0.y};
    AosRec P{st.rec_ab, st.rec_c, i, st.D, V3{0.f, 0.f, 0.f}, 0, false};
    bool next = false;
    // the recursion continues with the bounce ray while calls remain (scene.cpp:72-75)
    if (h.prim >= 0 && h.t < sc.max_distance && shade_hit<COUNT>(sc, r, h, rng, cnt, P, nv) && power > 0) {
        power -= 1;
        next = true;
    }
    P.flush_e();
    if (!next) {
        const V3 c = fold_path(P, nv);
        const float4 s1 = st.st[2 * i + 1];
        const float ax = s1.x + c.x, ay = s1.y + c.y, az = s1.z + c.z;
        st.st[2 * i + 1] = make_float4(ax, ay, az, 0.f);
        if (++s == spp) {
            out[3 * i + 0] = ax;
            out[3 * i + 1] = ay;
            out[3 * i + 2] = az;
        } else {
            r = start_sample(sc, g, i, rng, power);
            nv = 0;
            next = true;
        }
    }
    st.st[2 * i] = make_float4(__uint_as_float(rng.x), rng.saved, __uint_as_float(meta_pack(s, power, nv, rng.saved_avail)), 0.f);
    return next;
}

}  // namespace rtd
