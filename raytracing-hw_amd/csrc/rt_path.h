// rt_path.h — device-side restatement of the reference's per-pixel sample loop for gfx950.
//
// One lane = one pixel (the reference's RNG stream is sequential per pixel across all
// samples and bounces, so the pixel is the unit of parallelism: SURVEY.md §0.6).
// Every function cites the reference code it reproduces bit for bit; the file is built
// with -ffp-contract=off, IEEE float division/sqrt and preserved denormals.
#pragma once
#include <cstdint>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
// Host build of the same source, used ONLY by tests/native/kernel_host.cpp to check the
// kernel arithmetic on the CPU before it reaches the GPU (never linked into the product).
#include <cmath>
#include <cstring>
#define __device__
#define __host__
#define __forceinline__ inline
struct float4 { float x, y, z, w; };
struct uint2 { uint32_t x, y; };
struct uint4 { uint32_t x, y, z, w; };
inline uint2 make_uint2(uint32_t a, uint32_t b) { return {a, b}; }
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return {a, b, c, d}; }
inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline int __float_as_int(float f) { int u; std::memcpy(&u, &f, 4); return u; }
inline float __int_as_float(int u) { float f; std::memcpy(&f, &u, 4); return f; }
inline float4 make_float4(float a, float b, float c, float d) { return {a, b, c, d}; }
using std::isnan;
#endif

#include "rt_libm.h"
#include "rt_srgb_lut.h"
#include "rt_vec.h"

// Debug build (make DEBUG_CHECKS=1): index checks that record the first violation in
// rt_debug_word (code << 56 | value) and clamp the index so the kernel completes.
#if defined(RT_DEBUG_CHECKS) && defined(__HIPCC__)
__device__ unsigned long long rt_debug_word;
__device__ int rt_debug_poison;   // rt_debug_set_poison (rt_device.hip)
__device__ unsigned rt_debug_prints;   // device printf budget of the diagnostics
#define RT_CHECK(cond, code, val, fix)                                                                        \
    do {                                                                                                     \
        if (!(cond)) {                                                                                       \
            atomicCAS(&rt_debug_word, 0ull, ((unsigned long long)(code) << 56) | ((unsigned long long)(val) & 0xffffffffffffffull)); \
            fix;                                                                                             \
        }                                                                                                    \
    } while (0)
#else
#define RT_CHECK(cond, code, val, fix) do { } while (0)
#endif

// Diagnostics build (RT_MEGA_PROF): per-block clock64() sums of shading segments, added by
// the first active lane of the shading wave (rt_device.hip zeroes and flushes them).
#if defined(RT_MEGA_PROF) && defined(__HIPCC__)
__shared__ unsigned long long rt_prof_lds[8];
#define RT_PROF_BEGIN long long rt_pt_ = clock64();
#define RT_PROF_SEG(k)                                                                                   \
    do {                                                                                                 \
        const long long t1_ = clock64();                                                                 \
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1)                     \
            atomicAdd(&rt_prof_lds[k], (unsigned long long)(t1_ - rt_pt_));                              \
        rt_pt_ = t1_;                                                                                    \
    } while (0)
#else
#define RT_PROF_BEGIN
#define RT_PROF_SEG(k) do { } while (0)
#endif

namespace rtd {

using rtv::V2;
using rtv::V3;
using rtv::V4;

constexpr int kMaxDepth = 16;      // path vertices kept for the backward fold (ray_depth <= 16)
constexpr int kStack = 64;         // BVH stack frames (host rejects deeper trees)
constexpr float kPiF = 3.14159265358979323846f;     // M_PIf32
constexpr float kInvPiF = 0.318309886183790671538f; // M_1_PIf32
constexpr float kStep = 1e-4f;                      // scene.cpp:11 `const float step = 1e-4`
constexpr float kRoughness2Limit = 0.03f;           // scene.cpp:15

// Decode table for RGBA8 texels: 256 sRGB entries (rt_srgb_lut.h, glibc powf) then 256 linear
// entries (float)(int)b / 255.f, the two decodes of Texture::interpolate_sample
// (primitive.h:172-215).  Lives in the scene blob; kernels may stage it in LDS.
inline void fill_decode_lut(float *lut) {
    for (int b = 0; b < 256; ++b) {
        lut[b] = rtm::kSrgbLut[b];
        lut[256 + b] = (float)b / 255.f;
    }
}

// (float)b / 255.f for a byte b, correctly rounded, in three instructions: b times the float
// nearest 1/255 and one fma Newton correction, which rounds correctly for all 256 bytes
// (checked on the device by rt_device_selfcheck 1 and on the host by tests/test_libm.py).
__device__ __forceinline__ float unorm8(uint32_t b) {
    constexpr float r = 0x1.010102p-8f;   // (float)(1 / 255)
    const float x = (float)b, q = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.f, x), r, q);
}
// A texel byte's decode.  Device: the sRGB half of the table (the lane-resident kernel stages
// only those 256 entries in LDS) and the linear decode computed; host: the whole table.
__device__ __forceinline__ float texel_decode(const float *lut, uint32_t byte, bool srgb) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float s = lut[byte], l = unorm8(byte);
    return srgb ? s : l;
#else
    return lut[(srgb ? 0u : 256u) + byte];
#endif
}

struct DevScene {
    const float4 *tri;        // 3 x float4 / triangle: (v0, U.x) (U.yz, V.xy) (V.z, n_geo)
    const float4 *tri_attr;   // 4 x float4 / triangle: normals, texcoords, mesh id
    const float4 *tri_tan;    // 3 x float4 / triangle: tangents
    const float4 *node;       // 2 x float4 / node: (min, max.x) (max.yz, a, b)
    const float4 *light;      // 4 x float4 / light triangle
    const float4 *light_node;
    const float *mesh_f;      // 12 / mesh
    const int *mesh_tex;      // 4 / mesh
    const double *mesh_nt;    // 16 / mesh
    const uint4 *tex_info;    // texel offset, width, height, channels
    const uint32_t *texels;   // RGBA8
    const float *lut;         // 512: [b] = sRGB decode powf(b / 255.f, 2.2f), [256 + b] = b / 255.f
    int n_lights;
    int n_tris, n_nodes, n_meshes;
    int ray_depth;
    float max_distance;
    int width, height;
    float fwidth, fheight;   // (float)width, (float)height: kernel arguments, so the camera
                             // ray's divisions take them from SGPRs (no per-lane copy)
    float cam_pos[3];
    float cam_axes[9];
    float tan_fov[2];
};

struct Counters {
    uint32_t rays, aabb, tri, lq, laabb, ltri, hits;
};

// ------------------------------------------------------------------------ RNG
// std::minstd_rand (libstdc++ linear_congruential_engine<ulong, 48271, 0, 2^31-1>) with
// the polar normal cache of std::normal_distribution<float>, one per pixel.
struct Rng {
    uint32_t x;
    uint32_t saved_avail;
    float saved;
};

// Fast mode (RT_FLAG_FAST): every (pixel, sample) gets its own stream, so
// a pixel's samples no longer form one sequential chain and can run on any lane in any
// order.  Philox4x32-10 (Salmon et al., SC'11; Random123's constants and round function),
// counter = {sample, 0, 0, 0}, key = {pixel index j*W+i, kFastKey}, word 0 seeds the
// sample's minstd stream the way minstd_rand(seed) does (mod 2^31-1, 0 -> 1); the polar
// normal cache starts empty at every sample.  Draw order and arithmetic inside a sample
// are the parity path's.  Statistically equivalent to the reference, not bit-identical.
constexpr uint32_t kFastKey = 0x5eed2026u;
__host__ __device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y, (uint32_t)p0);
    }
    return c;
}
__host__ __device__ __forceinline__ uint32_t fast_sample_seed(uint32_t pixel, uint32_t sample) {
    const uint32_t w = philox4x32_10(make_uint4(sample, 0u, 0u, 0u), make_uint2(pixel, kFastKey)).x % 2147483647u;
    return w == 0 ? 1u : w;
}

__device__ __forceinline__ uint32_t rng_next(Rng &r) {
    uint64_t t = (uint64_t)r.x * 48271u;                          // < 2^47
    uint32_t v = (uint32_t)(t & 0x7fffffffu) + (uint32_t)(t >> 31); // t mod (2^31 - 1), one fold
    if (v >= 0x7fffffffu) v -= 0x7fffffffu;
    r.x = v;
    return v;
}
// generate_canonical<float, 24> (random.tcc:3348-3380): one engine draw (log2 r = 30 bits).
__device__ __forceinline__ float rng_canonical(Rng &r) {
    float s = (float)(rng_next(r) - 1u);
    float v = s / 2147483648.0f;   // (float)2147483646.0L == 2^31
    if (v >= 1.0f) v = 0x1.fffffep-1f;  // nextafter(1, 0)
    return v;
}
// uniform_real_distribution<float>(a, b): canonical * (b - a) + a
__device__ __forceinline__ float rng_uniform_m11(Rng &r) { return rng_canonical(r) * 2.0f + (-1.0f); }  // uniDist(-1, 1)
__device__ __forceinline__ float rng_offset(Rng &r) { return rng_canonical(r) * 1.0f + (-0.5f); }        // offset(-.5, .5)
// normal_distribution<float>(0, 1) polar method (random.tcc:1802-1833)
__device__ __forceinline__ float rng_normal(Rng &r) {
    float ret;
    if (r.saved_avail) {
        r.saved_avail = 0;
        ret = r.saved;
    } else {
        float x, y, r2;
        do {
            x = 2.0f * rng_canonical(r) - 1.0f;   // (float)(2.0f*u - 1.0): exact in double, one rounding
            y = 2.0f * rng_canonical(r) - 1.0f;
            r2 = x * x + y * y;
        } while (r2 > 1.0f || r2 == 0.0f);
        const float mult = sqrtf(-2.0f * rtm::logf_glibc(r2) / r2);
        r.saved = x * mult;
        r.saved_avail = 1;
        ret = y * mult;
    }
    return ret * 1.0f + 0.0f;   // * stddev + mean
}

// ------------------------------------------------------------------------ rays
struct Ray {
    V3 o, d, inv;
};
// Ray::Ray (primitive.cpp:12-15): normalize direction, inv = {1,1,1} / direction
__device__ __forceinline__ Ray make_ray(V3 p, V3 dir) {
    Ray r;
    r.o = p;
    r.d = rtv::normal(dir);
    r.inv = rtv::divv(V3{1.f, 1.f, 1.f}, r.d);
    return r;
}

// AABB::intersect (primitive.cpp:146-208): Graphics-Gems RayBox (Woo), returns the
// distance to the entry point (0 if the origin is inside) or false.
__device__ __forceinline__ bool aabb_hit(const float mn[3], const float mx[3], const Ray &r, float &dist) {
    const float o[3] = {r.o.x, r.o.y, r.o.z};
    const float d[3] = {r.d.x, r.d.y, r.d.z};
    const float inv[3] = {r.inv.x, r.inv.y, r.inv.z};
    bool inside = true;
    int quad[3];
    float cand[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (o[i] < mn[i]) { quad[i] = 0; cand[i] = mn[i]; inside = false; }
        else if (o[i] > mx[i]) { quad[i] = 2; cand[i] = mx[i]; inside = false; }
        else { quad[i] = 1; cand[i] = 0.f; }
    }
    if (inside) { dist = 0.f; return true; }
    float maxT[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) maxT[i] = (quad[i] != 1 && d[i] != 0.f) ? (cand[i] - o[i]) * inv[i] : -1.f;
    int wp = 0;
    if (maxT[wp] < maxT[1]) wp = 1;
    if (maxT[wp] < maxT[2]) wp = 2;
    const float tw = maxT[wp];
    if (tw < 0.f) return false;
    float coord[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (wp != i) {
            coord[i] = o[i] + tw * d[i];
            if (coord[i] < mn[i] || coord[i] > mx[i]) return false;
        } else {
            coord[i] = cand[i];
        }
    }
    dist = rtv::length(rtv::sub(V3{coord[0], coord[1], coord[2]}, r.o));
    return true;
}

struct TriHit {
    float t, u, v;
};
// Primitive::intersect (primitive.cpp:17-57), Moller-Trumbore on (v0, U, V).
__device__ __forceinline__ bool tri_hit(V3 v0, V3 U, V3 V, const Ray &r, TriHit &h) {
    V3 p = rtv::cross(r.d, V);
    float det = rtv::dot(U, p);
    if (-1e-6 < (double)det && (double)det < 1e-6) return false;
    float inv_det = 1.f / det;
    V3 s = rtv::sub(r.o, v0);
    float u = inv_det * rtv::dot(s, p);
    if (u < 0 || u > 1) return false;
    V3 q = rtv::cross(s, U);
    float v = inv_det * rtv::dot(r.d, q);
    if (v < 0 || u + v > 1) return false;
    float t = inv_det * rtv::dot(V, q);
    if (t < 0.f) return false;
    h.t = t;
    h.u = u;
    h.v = v;
    return true;
}

__device__ __forceinline__ void load_tri(const float4 *tri, int id, V3 &v0, V3 &U, V3 &V) {
    float4 a = tri[3 * id], b = tri[3 * id + 1], c = tri[3 * id + 2];
    v0 = V3{a.x, a.y, a.z};
    U = V3{a.w, b.x, b.y};
    V = V3{b.z, b.w, c.x};
}

struct NodeRec {
    float mn[3], mx[3];
    uint32_t a, b;
};
__device__ __forceinline__ NodeRec load_node(const float4 *nodes, uint32_t id) {
    float4 p = nodes[2 * id], q = nodes[2 * id + 1];
    NodeRec n;
    n.mn[0] = p.x; n.mn[1] = p.y; n.mn[2] = p.z;
    n.mx[0] = p.w; n.mx[1] = q.x; n.mx[2] = q.y;
    n.a = __float_as_uint(q.z);
    n.b = __float_as_uint(q.w);
    return n;
}

struct Hit {
    float t, u, v;
    int prim;
};

// BVH::intersect + intersectHelper (bvh.cpp:177-243), recursion replaced by an explicit
// frame stack with the reference's semantics kept exactly:
//   * root box tested first;
//   * near child first by dir[split_dim] > 0 (left, right) else (right, left);
//   * the far child is entered unless its entry distance is > the best t found inside the
//     NEAR subtree of the same node (the reference's per-call local best), not the global
//     best; a frame carries that local best while the far subtree runs;
//   * leaf triangles in index order, strict `<`, so the first of equal-t hits wins.
// The final winner equals the global strict minimum over all tested triangles in visit
// order, which is what `best` tracks.
template <bool COUNT>
__device__ bool closest_hit(const DevScene &sc, const Ray &r, Hit &best, Counters &cnt) {
    if (COUNT) { cnt.rays++; cnt.aabb++; }
    NodeRec nd = load_node(sc.node, 0);
    float e;
    if (!aabb_hit(nd.mn, nd.mx, r, e)) return false;
    uint2 stk[kStack];
    int sp = 0;
    uint32_t cur = 0;
    int phase = 0;
    float acc = 1e9f;
    best.t = 1e9f;
    best.prim = -1;
    const float dcomp[3] = {r.d.x, r.d.y, r.d.z};
    for (;;) {
        bool descend = false;
        if ((nd.b & 3u) == 3u) {  // leaf
            const uint32_t first = nd.a, count = nd.b >> 2;
            for (uint32_t k = first; k < first + count; ++k) {
                V3 v0, U, V;
                load_tri(sc.tri, (int)k, v0, U, V);
                TriHit h;
                if (COUNT) cnt.tri++;
                if (tri_hit(v0, U, V, r, h)) {
                    if (h.t < acc) acc = h.t;
                    if (h.t < best.t) { best.t = h.t; best.u = h.u; best.v = h.v; best.prim = (int)k; }
                }
            }
        } else {
            const uint32_t left = nd.a;
            const bool left_first = dcomp[nd.b] > 0;
            if (phase == 0) {
                const uint32_t c0 = left_first ? left : left + 1;
                NodeRec cn = load_node(sc.node, c0);
                if (COUNT) cnt.aabb++;
                if (aabb_hit(cn.mn, cn.mx, r, e)) {
                    stk[sp++] = make_uint2(cur | (1u << 31), __float_as_uint(acc));
                    cur = c0; phase = 0; acc = 1e9f; nd = cn;
                    descend = true;
                } else {
                    phase = 1;
                }
            }
            if (!descend && phase == 1) {
                const uint32_t c1 = left_first ? left + 1 : left;
                NodeRec cn = load_node(sc.node, c1);
                if (COUNT) cnt.aabb++;
                if (aabb_hit(cn.mn, cn.mx, r, e) && !(e > acc)) {
                    stk[sp++] = make_uint2(cur, __float_as_uint(acc));  // resume in phase 2
                    cur = c1; phase = 0; acc = 1e9f; nd = cn;
                    descend = true;
                }
            }
        }
        if (descend) continue;
        // return to the parent frame, merging this subtree's best (`a.distance < intersection.distance`)
        if (sp == 0) break;
        uint2 f = stk[--sp];
        const float pacc = __uint_as_float(f.y);
        acc = acc < pacc ? acc : pacc;
        phase = (f.x >> 31) ? 1 : 2;
        cur = f.x & 0x7fffffffu;
        nd = load_node(sc.node, cur);
        if (phase == 2) {
            // both children done: fall through to the return path on the next iteration
            // by marking this frame finished
            // (handled by the loop: an internal node in phase 2 takes neither branch)
        }
    }
    return best.prim >= 0;
}

// ManyLightsDistribution::pdf (random.cpp:179-188) over BVH::intersectAll (bvh.cpp:245-279):
// every emissive triangle hit, left subtree before right, no root test, summed in visit order.
// `stk` holds the walk's node ids (.x); the lane-resident kernel passes the lane's traversal
// stack (LDS), free while its lane shades, instead of a private array in scratch memory.
template <bool COUNT, class Stack>
__device__ float light_pdf(const DevScene &sc, V3 point, V3 direction, Counters &cnt, Stack &stk) {
    if (COUNT) cnt.lq++;
    Ray r = make_ray(point, direction);
    int sp = 0;
    stk.put(sp++, make_uint2(0u, 0u));
    float prob = 0.f;
    while (sp > 0) {
        const uint32_t id = stk.get(--sp).x;
        NodeRec nd = load_node(sc.light_node, id);
        if ((nd.b & 3u) == 3u) {
            const uint32_t first = nd.a, count = nd.b >> 2;
            for (uint32_t k = first; k < first + count; ++k) {
                float4 a = sc.light[4 * k], b = sc.light[4 * k + 1], c = sc.light[4 * k + 2], w = sc.light[4 * k + 3];
                TriHit h;
                if (COUNT) cnt.ltri++;
                if (tri_hit(V3{a.x, a.y, a.z}, V3{a.w, b.x, b.y}, V3{b.z, b.w, c.x}, r, h)) {
                    V3 n{c.y, c.z, c.w};
                    if (rtv::dot(r.d, n) > 0) n = rtv::neg(n);
                    const float probability = 1.f / w.x;  // 1 / triangle_area (random.cpp:88)
                    prob += fabsf(probability * (h.t * h.t) / rtv::dot(n, direction));
                }
            }
        } else {
            const uint32_t left = nd.a;
            float e;
            NodeRec l = load_node(sc.light_node, left), rr = load_node(sc.light_node, left + 1);
            if (COUNT) cnt.laabb += 2;
            const bool hl = aabb_hit(l.mn, l.mx, r, e);
            const bool hr = aabb_hit(rr.mn, rr.mx, r, e);
            RT_CHECK(sp + 2 <= kStack, 13, sp, sp = 0);
            if (hr) stk.put(sp++, make_uint2(left + 1, 0u));
            if (hl) stk.put(sp++, make_uint2(left, 0u));
        }
    }
    return prob / (float)sc.n_lights;
}
// A private stack (host tests, the ray-level entry, the wavefront shade kernel).
struct LocalStack {
    uint32_t id[kStack];
    __device__ __forceinline__ void put(int i, uint2 v) { id[i] = v.x; }
    __device__ __forceinline__ uint2 get(int i) const { return make_uint2(id[i], 0u); }
};
template <bool COUNT>
__device__ float light_pdf(const DevScene &sc, V3 point, V3 direction, Counters &cnt) {
    LocalStack stk;
    return light_pdf<COUNT>(sc, point, direction, cnt, stk);
}

// ------------------------------------------------------------------------ textures
// Texture::interpolate_sample (primitive.h:182-215); RGBA8, four channels always.
__device__ __forceinline__ V4 tex_sample_ti(const DevScene &sc, const uint4 ti, V2 p, bool srgb) {
    const int W = (int)ti.y, H = (int)ti.z;
    p.x -= floorf(p.x);
    p.y -= floorf(p.y);
    p.x *= (float)W;
    p.y *= (float)H;
    const int px = (int)floorf(p.x), py = (int)floorf(p.y);
    const float dx = p.x - floorf(p.x), dy = p.y - floorf(p.y);
    uint32_t texel[4];
    // (px + d) % W without a division: p - floorf(p) is in [0, 1], so px is in [0, W] and
    // px + d in [0, W + 1] <= 2W; two conditional subtractions give the remainder (W = 1
    // included).  NaN coordinates convert to 0 on the device, as they would for %.
    auto wrap = [](int v, int n) {
        v = v >= n ? v - n : v;
        return v >= n ? v - n : v;
    };
#pragma unroll
    for (int ddy = 0; ddy < 2; ++ddy)
#pragma unroll
        for (int ddx = 0; ddx < 2; ++ddx) {
            const int x = wrap(px + ddx, W), y = wrap(py + ddy, H);
#ifdef __HIPCC__
            // device copy: 4x4-texel tiles (rt_device.hip tile_textures)
            const uint32_t idx = (uint32_t)(((y >> 2) * ((W + 3) >> 2) + (x >> 2)) * 16 + (y & 3) * 4 + (x & 3));
#else
            const uint32_t idx = (uint32_t)(y * W + x);   // host view: row-major
#endif
            texel[ddx * 2 + ddy] = sc.texels[ti.x + idx];
        }
    float res[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t byte = (texel[k] >> (8 * c)) & 0xffu;
            v[k] = texel_decode(sc.lut, byte, srgb);   // kSrgbLut[byte] or (float)(int)byte / 255.f
        }
        res[c] = v[0] * (1 - dx) * (1 - dy) + v[1] * (1 - dx) * dy + v[2] * dx * (1 - dy) + v[3] * dx * dy;
    }
    return V4{res[0], res[1], res[2], res[3]};
}
__device__ __forceinline__ V4 tex_sample(const DevScene &sc, int tex, V2 p, bool srgb) {
    return tex_sample_ti(sc, sc.tex_info[tex], p, srgb);
}

// ------------------------------------------------------------------------ sampling
// uniform::sphere (random.cpp:28-31)
__device__ __forceinline__ V3 sphere(Rng &r) {
    float a = rng_normal(r);
    float b = rng_normal(r);
    float c = rng_normal(r);
    return rtv::normal(V3{a, b, c});
}
// cosine_weighted::sample / pdf (random.cpp:48-59)
__device__ __forceinline__ V3 cosine_sample(V3 n, Rng &r) {
    V3 d;
    do {
        d = rtv::add(sphere(r), n);
    } while ((double)rtv::length(d) < 1e-12);
    return rtv::normal(d);
}
__device__ __forceinline__ float cosine_pdf(V3 n, V3 d) { return rtv::smax(0.f, rtv::dot(d, n)) * kInvPiF; }

// The uniform sample on a disc of visible_normal::sample (random.cpp:114-122): pairs of
// uniform(-1, 1) draws until one lies inside the unit circle.
__device__ __forceinline__ void disc_draw(Rng &r, float &ux, float &uy) {
    do {
        ux = rng_uniform_m11(r);
        uy = rng_uniform_m11(r);
    } while (ux * ux + uy * uy > 1.f);
}

// visible_normal::sample (random.cpp:103-134)
__device__ __forceinline__ V3 vndf_sample(V3 n, V3 eye, float alpha, Rng &r) {
    const V3 Z{0.f, 0.f, 1.f};
    V4 rot = rtv::quat_from_two_vectors(n, Z);
    V3 Ve = rtv::rotate(eye, rot);
    V3 Vh = rtv::normal(V3{Ve.x * alpha, Ve.y * alpha, Ve.z});
    float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    V3 T1 = lensq > 0 ? rtv::mul(V3{-Vh.y, Vh.x, 0}, 1.f / sqrtf(lensq)) : V3{1, 0, 0};
    V3 T2 = rtv::cross(Vh, T1);
    float ux, uy;
    disc_draw(r, ux, uy);
    float s = 0.5f + 0.5f * Vh.z;
    float ty = (1.f - s) * sqrtf(1.f - ux * ux) + s * uy;
    V3 Nh = rtv::add(rtv::add(rtv::mul(T1, ux), rtv::mul(T2, ty)),
                     rtv::mul(Vh, sqrtf(rtv::smax(0.f, 1.f - ux * ux - ty * ty))));
    V3 Ne = rtv::normal(V3{alpha * Nh.x, alpha * Nh.y, rtv::smax(0.f, Nh.z)});
    Ne = rtv::rotate(Ne, rtv::conj(rot));
    return rtv::normal(rtv::sub(rtv::mul(rtv::mul(Ne, 2.f), rtv::dot(Ne, eye)), eye));
}
// visible_normal::pdf (random.cpp:136-154)
__device__ __forceinline__ float vndf_pdf(V3 n, V3 eye, float alpha, V3 dir) {
    const V3 Z{0.f, 0.f, 1.f};
    V4 rot = rtv::quat_from_two_vectors(n, Z);
    V3 sn = rtv::normal(rtv::add(dir, eye));
    V3 V = rtv::rotate(eye, rot);
    V3 Ni = rtv::rotate(sn, rot);
    if (rtv::dot(V, Ni) < 0.f) return 0.f;
    float alpha2 = alpha * alpha;
    float q = Ni.x * Ni.x / alpha2 + Ni.y * Ni.y / alpha2 + Ni.z * Ni.z;
    float invD = (float)((double)(kPiF * alpha * alpha) * ((double)q * (double)q));
    float invG1 = 0.5f + 0.5f * sqrtf(1.f + (alpha2 * V.x * V.x + alpha2 * V.y * V.y) / (V.z * V.z));
    return 1.f / (4.f * invD * invG1 * rtv::dot(V, Z));
}
// ManyLightsDistribution::sample + LightDistribution::sample (random.cpp:170-177, :65-81)
__device__ __forceinline__ V3 light_sample(const DevScene &sc, V3 point, Rng &r) {
    int s = (int)floorf((rng_uniform_m11(r) + 1.f) * 0.5f * (float)sc.n_lights);
    if (s == sc.n_lights) s -= 1;
    float4 a = sc.light[4 * s], b = sc.light[4 * s + 1], c = sc.light[4 * s + 2];
    float u = (rng_uniform_m11(r) + 1.f) / 2;
    float v = (rng_uniform_m11(r) + 1.f) / 2;
    if (u + v > 1) { u = 1 - u; v = 1 - v; }
    V3 res = rtv::add(rtv::add(V3{a.x, a.y, a.z}, rtv::mul(V3{a.w, b.x, b.y}, u)), rtv::mul(V3{b.z, b.w, c.x}, v));
    return rtv::normal(rtv::sub(res, point));
}

// ------------------------------------------------------------------------ BRDF helpers (vector.h:433-471)
__device__ __forceinline__ float ggx(float alpha, V3 N, V3 H) {
    float alpha2 = alpha * alpha;
    float NdotH = rtv::dot(N, H);
    return alpha2 * kInvPiF / ((NdotH * NdotH * (alpha2 - 1) + 1) * (NdotH * NdotH * (alpha2 - 1) + 1));
}
__device__ __forceinline__ float smith(float alpha, V3 N, V3 V, V3 L) {
    float alpha2 = alpha * alpha;
    if (rtv::dot(N, L) <= 0 || rtv::dot(N, V) <= 0) return 0;
    float nd[2] = {fabsf(rtv::dot(N, L)), fabsf(rtv::dot(N, V))};
    float res = 1.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) res *= 2 * nd[k] / (nd[k] + sqrtf(alpha2 + (1 - alpha2) * nd[k] * nd[k]));
    return res;
}

// matrix.h:66-86 multiplyVector with matrix4d: float accumulators, each add in double.
__device__ __forceinline__ V3 mul_vector_d(const double *m, V3 t) {
    const float tv[4] = {t.x, t.y, t.z, 0.f};
    float res[3] = {0.f, 0.f, 0.f};
    // column by column (same per-component addition order j = 0..3); not unrolled over j so
    // that only one column of doubles is live at a time (register pressure in shading)
#pragma unroll 1
    for (int j = 0; j < 4; ++j) {
        const double tj = (double)tv[j];
#pragma unroll
        for (int i = 0; i < 3; ++i) res[i] = (float)((double)res[i] + m[4 * j + i] * tj);
    }
    return V3{res[0], res[1], res[2]};
}

// ------------------------------------------------------------------------ path vertices
// Scene::intersect (scene.cpp:71-157) is recursive; the kernels run it as a forward pass
// that records each path vertex, followed by the backward fold
//     c_k = e_k + ((((c_{k+1} * coeff_k) * material_k) * cos_k) * alpha_k)
// which reproduces the recursion's rounding exactly.
struct PathRec {
    V3 e[kMaxDepth], m[kMaxDepth];
    float coeff[kMaxDepth], cosv[kMaxDepth], alpha[kMaxDepth];
    __device__ __forceinline__ void set_e(int k, V3 v) { e[k] = v; }
    __device__ __forceinline__ void set_brdf(int k, V3 mm, float c, float cs, float a) {
        m[k] = mm;
        coeff[k] = c;
        cosv[k] = cs;
        alpha[k] = a;
    }
    __device__ __forceinline__ V3 get_e(int k) const { return e[k]; }
    __device__ __forceinline__ V3 get_m(int k) const { return m[k]; }
    __device__ __forceinline__ float get_coeff(int k) const { return coeff[k]; }
    __device__ __forceinline__ float get_cos(int k) const { return cosv[k]; }
    __device__ __forceinline__ float get_alpha(int k) const { return alpha[k]; }
};

// The same records kept structure-of-arrays in HBM for the wavefront pipeline:
// plane (q * D + k) holds component q of vertex k for every path slot.
struct SoARec {
    float *base;
    long long n;   // slots
    long long i;   // this slot
    int D;         // vertex capacity
    __device__ __forceinline__ float &at(int q, int k) const { return base[((long long)(q * D + k)) * n + i]; }
    __device__ __forceinline__ void set_e(int k, V3 v) const { at(0, k) = v.x; at(1, k) = v.y; at(2, k) = v.z; }
    __device__ __forceinline__ void set_brdf(int k, V3 mm, float c, float cs, float a) const {
        at(3, k) = mm.x; at(4, k) = mm.y; at(5, k) = mm.z;
        at(6, k) = c; at(7, k) = cs; at(8, k) = a;
    }
    __device__ __forceinline__ V3 get_e(int k) const { return V3{at(0, k), at(1, k), at(2, k)}; }
    __device__ __forceinline__ V3 get_m(int k) const { return V3{at(3, k), at(4, k), at(5, k)}; }
    __device__ __forceinline__ float get_coeff(int k) const { return at(6, k); }
    __device__ __forceinline__ float get_cos(int k) const { return at(7, k); }
    __device__ __forceinline__ float get_alpha(int k) const { return at(8, k); }
};

// SceneDistribution::sample (random.cpp:194-208): mixture of cosine, VNDF and light
// sampling chosen by one uniform(-1, 1) draw.
// The mixture draw (random.cpp:196-203): 0 cosine, 1 VNDF, 2 light.
__device__ __forceinline__ int mixture_pick(Rng &rng, int n_lights) {
    float s = (rng_uniform_m11(rng) + 1.f) * 3 * 0.5f;
    if (!n_lights) s /= 1.5f;
    return s <= 1.f ? 0 : (s <= 2.f ? 1 : 2);
}
__device__ __forceinline__ V3 scene_sample(const DevScene &sc, V3 pos, V3 N, V3 eye, float r2, Rng &rng) {
    const int b = mixture_pick(rng, sc.n_lights);
    if (b == 0) return cosine_sample(N, rng);
    if (b == 1) return vndf_sample(N, eye, r2, rng);
    return light_sample(sc, pos, rng);
}

// The RNG draws of one sample (scene.cpp:36-41) whose path calls SceneDistribution::sample
// k times, without the geometry: the two pixel offsets, then per call the mixture draw and
// the chosen sampler's draws (cosine: three polar normals through the cache; VNDF: the disc
// pairs; light: triangle choice + u + v).  Every draw count here is decided by the drawn
// values alone; the one geometric exception (cosine_weighted::sample retries when the
// sphere sample cancels the normal to |d| < 1e-12, random.cpp:50-53) is not modelled, so a
// caller must compare states, not assume them (rt_mega.h spec_manage does).  Used by the
// speculative sample runahead: a pixel's sample t+1 starts from the state sample t ends in,
// and for a path of ray_depth vertices that state is rng_skip_sample(start of t, ray_depth).
// The polar normals' values are not needed to advance the state, except the cached one: the
// state's `saved` is x * mult of the last pair drawn (rng_normal), so only that pair's logf and
// sqrtf are evaluated, once, at the end (same operations, same bits).
__device__ __forceinline__ void rng_normal_skip(Rng &r, bool &gen, float &lx, float &lr2) {
    if (r.saved_avail) {
        r.saved_avail = 0;
        return;
    }
    float x, y, r2;
    do {
        x = 2.0f * rng_canonical(r) - 1.0f;
        y = 2.0f * rng_canonical(r) - 1.0f;
        r2 = x * x + y * y;
    } while (r2 > 1.0f || r2 == 0.0f);
    gen = true;
    lx = x;
    lr2 = r2;
    r.saved_avail = 1;
}
__device__ __forceinline__ void rng_skip_sample(Rng &r, int k, int n_lights) {
    (void)rng_next(r);   // rng_offset x 2: one engine draw each
    (void)rng_next(r);
    bool gen = false;
    float lx = 0.f, lr2 = 1.f;
    for (int v = 0; v < k; ++v) {
        const int b = mixture_pick(r, n_lights);
        if (b == 0) {
            rng_normal_skip(r, gen, lx, lr2);
            rng_normal_skip(r, gen, lx, lr2);
            rng_normal_skip(r, gen, lx, lr2);
        } else if (b == 1) {
            float ux, uy;
            disc_draw(r, ux, uy);
        } else {
            (void)rng_next(r);
            (void)rng_next(r);
            (void)rng_next(r);
        }
    }
    if (gen) {
        const float mult = sqrtf(-2.0f * rtm::logf_glibc(lr2) / lr2);
        r.saved = lx * mult;
    }
}

// SceneDistribution::pdf (random.cpp:210-218)
template <bool COUNT, class Stack>
__device__ __forceinline__ float scene_pdf(const DevScene &sc, V3 pos, V3 N, V3 eye, float r2, V3 dir, Counters &cnt,
                                           Stack &stk) {
    if (!sc.n_lights) return (cosine_pdf(N, dir) + vndf_pdf(N, eye, r2, dir)) / 2;
    return (cosine_pdf(N, dir) + light_pdf<COUNT>(sc, pos, dir, cnt, stk) + vndf_pdf(N, eye, r2, dir)) / 3;
}
template <bool COUNT>
__device__ __forceinline__ float scene_pdf(const DevScene &sc, V3 pos, V3 N, V3 eye, float r2, V3 dir, Counters &cnt) {
    LocalStack stk;
    return scene_pdf<COUNT>(sc, pos, N, eye, r2, dir, cnt, stk);
}

// The records of one path slot in HBM for the wavefront pipeline, vertex-major so a vertex
// is two 16-byte stores and one 4-byte store: ab[2 * (i * D + k)] = (e.xyz, coeff),
// ab[... + 1] = (m.xyz, cos), c[i * D + k] = alpha.  The emission is kept in registers until
// the vertex's BRDF is known (set_brdf) or the path ends there (flush_e).
struct AosRec {
    float4 *ab;
    float *c;
    long long i;
    int D;
    V3 e;
    int ek;
    bool pending;
    __device__ __forceinline__ long long v(int k) const { return i * D + k; }
    __device__ __forceinline__ void set_e(int k, V3 x) { e = x; ek = k; pending = true; }
    __device__ __forceinline__ void set_brdf(int k, V3 mm, float cf, float cs, float a) {
        ab[2 * v(k)] = make_float4(e.x, e.y, e.z, cf);
        ab[2 * v(k) + 1] = make_float4(mm.x, mm.y, mm.z, cs);
        c[v(k)] = a;
        pending = false;
    }
    __device__ __forceinline__ void flush_e() {
        if (pending) ab[2 * v(ek)] = make_float4(e.x, e.y, e.z, 0.f);
        pending = false;
    }
    __device__ __forceinline__ V3 get_e(int k) const { const float4 a = ab[2 * v(k)]; return V3{a.x, a.y, a.z}; }
    __device__ __forceinline__ V3 get_m(int k) const { const float4 b = ab[2 * v(k) + 1]; return V3{b.x, b.y, b.z}; }
    __device__ __forceinline__ float get_coeff(int k) const { return ab[2 * v(k)].w; }
    __device__ __forceinline__ float get_cos(int k) const { return ab[2 * v(k) + 1].w; }
    __device__ __forceinline__ float get_alpha(int k) const { return c[v(k)]; }
};

// Vertex records of the lane-resident kernel, indexed by the lane's slot (its global thread
// index) rather than by pixel, so the footprint is lanes x depth, not pixels x depth.
// Vertex k of slot i is one 32-byte sector, R[2 (k * lanes + i)] = (coeff, m.xyz) and
// R[... + 1] = (cos, e.xyz), written by the lane in two adjacent 16-byte stores; the path's
// last vertex writes only its emission half.  The material alpha (1 for every opaque
// material) is stored in its own plane only where it is not 1, which the sign bit of coeff
// marks (coeff = 1 / pdf > 0, so the bit is free).  Round 2 kept (e, coeff), (m, cos) and
// alpha in three planes: each vertex touched three sectors, and the records were 79% of
// the kernel's HBM writes (profiles/r02e_record_layout_ab.jsonl).
// Record addresses are a uniform base plus a 32-bit byte offset (lanes x depth x 32 B stays
// below 4 GiB: the host sizes the workspace), so a record access is one VGPR of offset on the
// base in SGPRs rather than a 64-bit address per lane.
// RT_REC_NT (A/B builds): the vertex records written and read back non-temporally.
#ifndef RT_REC_NT
#define RT_REC_NT 0
#endif
__device__ __forceinline__ void rec_st(float4 &dst, float4 v) {
#if RT_REC_NT && defined(__HIP_DEVICE_COMPILE__)
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4f *>(&dst));
#else
    dst = v;
#endif
}
__device__ __forceinline__ float4 rec_ld(const float4 &src) {
#if RT_REC_NT && defined(__HIP_DEVICE_COMPILE__)
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(&src));
    return make_float4(x.x, x.y, x.z, x.w);
#else
    return src;
#endif
}
struct LaneRec {
    float4 *R;
    float *al;
    long long i, lanes;
    V3 e;
    int ek;
    bool pending;
    __device__ __forceinline__ uint32_t v(int k) const { return (uint32_t)k * (uint32_t)lanes + (uint32_t)i; }
    __device__ __forceinline__ float4 &rec(uint32_t vk, int half) const {
        return *(float4 *)((char *)R + (size_t)((vk << 5) + (uint32_t)(16 * half)));
    }
    __device__ __forceinline__ float &alp(uint32_t vk) const { return *(float *)((char *)al + (size_t)(vk << 2)); }
    __device__ __forceinline__ void set_e(int k, V3 x) { e = x; ek = k; pending = true; }
    __device__ __forceinline__ void set_brdf(int k, V3 mm, float cf, float cs, float a) {
        const bool one = __float_as_uint(a) == 0x3f800000u;
        rec_st(rec(v(k), 0), make_float4(__uint_as_float(__float_as_uint(cf) | (one ? 0u : 0x80000000u)), mm.x, mm.y, mm.z));
        rec_st(rec(v(k), 1), make_float4(cs, e.x, e.y, e.z));
        if (!one) alp(v(k)) = a;
        pending = false;
    }
    __device__ __forceinline__ void flush_e() {
        if (pending) rec_st(rec(v(ek), 1), make_float4(0.f, e.x, e.y, e.z));
        pending = false;
    }
    __device__ __forceinline__ V3 get_e(int k) const { const float4 b = rec_ld(rec(v(k), 1)); return V3{b.y, b.z, b.w}; }
};
// fold_path over LaneRec: the backward recurrence, records read four vertices at a time
// (alpha only for the vertices that stored one).  last_here: the last vertex was shaded in
// this call, so its emission is still P.e (the path's end never writes it to memory).
__device__ __forceinline__ V3 fold_path(const LaneRec &P, int nv, bool last_here = false) {
    if (nv == 0) return V3{0.f, 0.f, 0.f};
    V3 c = P.e;
    if (!last_here) {
        const float4 last = rec_ld(P.rec(P.v(nv - 1), 1));
        c = V3{last.y, last.z, last.w};
    }
    for (int hi = nv - 2; hi >= 0; hi -= 4) {
        float4 A[4], B[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = hi - j >= 0 ? hi - j : 0;
            A[j] = rec_ld(P.rec(P.v(k), 0));
            B[j] = rec_ld(P.rec(P.v(k), 1));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (hi - j < 0) break;
            const uint32_t cb = __float_as_uint(A[j].x);
            const float alpha = (cb >> 31) ? P.alp(P.v(hi - j)) : 1.f;
            V3 x = rtv::mul(c, __uint_as_float(cb & 0x7fffffffu));
            x = rtv::mulv(x, V3{A[j].y, A[j].z, A[j].w});
            x = rtv::mul(x, B[j].x);
            x = rtv::mul(x, alpha);
            c = rtv::add(V3{B[j].y, B[j].z, B[j].w}, x);
        }
    }
    return c;
}

// One hit of Scene::intersect (scene.cpp:85-154) in two halves around the light pdf, so the
// light-BVH walk can run as its own traversal (rt_mega.h light_step):
//   shade_pre  — emission (vertex nv), shading normal, metallic-roughness, the sampled
//                direction, nv++ and the below-surface test; false where the recursion returns;
//   shade_post — pdf from its parts, BRDF factors of vertex nv-1, the bounce ray; false where
//                pdf <= 0 or NaN.
// ShadeMid is what crosses the split (a lane-slot record in the lane-resident kernel).
struct ShadeMid {
    V3 pos, N, dir;
    V2 tc;
    float r2, metallic;
    int mesh;
};

template <bool COUNT, class Rec>
__device__ __forceinline__ bool shade_pre(const DevScene &sc, const Ray &r, const Hit &hit, Rng &rng, Counters &cnt,
                                          Rec &P, int &nv, ShadeMid &m) {
    RT_PROF_BEGIN
    if (COUNT) cnt.hits++;
    int id = hit.prim;
    RT_CHECK(id >= 0 && id < sc.n_tris, 1, id, id = 0);
    RT_CHECK(nv >= 0 && nv < kMaxDepth - 1, 2, nv, nv = 0);
    const float u = hit.u, v = hit.v;
    const float4 t2 = sc.tri[3 * id + 2];
    V3 ngeo{t2.y, t2.z, t2.w};
    bool inside = false;
    if (rtv::dot(r.d, ngeo) > 0) { inside = true; ngeo = rtv::neg(ngeo); }
    const float4 a0 = sc.tri_attr[4 * id], a1 = sc.tri_attr[4 * id + 1], a2 = sc.tri_attr[4 * id + 2],
                 a3 = sc.tri_attr[4 * id + 3];
    int mesh = __float_as_int(a3.w);
    RT_CHECK(mesh >= 0 && mesh < sc.n_meshes, 3, mesh, mesh = 0);
    const float *mf = sc.mesh_f + 12 * mesh;
    const int *mt = sc.mesh_tex + 4 * mesh;
    // texture descriptors of the emission, normal and metallic-roughness slots, read together
    // (one round trip, not one per texture on the way)
    const int mt_e = mt[3], mt_n = mt[1], mt_mr = mt[2];
    const uint4 ti_e = sc.tex_info[mt_e >= 0 ? mt_e : 0], ti_n = sc.tex_info[mt_n >= 0 ? mt_n : 0],
                ti_mr = sc.tex_info[mt_mr >= 0 ? mt_mr : 0];
#ifdef __HIPCC__
    asm volatile("" ::"v"(ti_e.x), "v"(ti_n.x), "v"(ti_mr.x));   // (keep the reads here, not sunk into the branches)
#endif
    const float w = 1 - u - v;
    const V2 tc{w * a2.y + u * a2.w + v * a3.y, w * a2.z + u * a3.x + v * a3.z};
    // Primitive::get_emission (primitive.cpp:121-129)
    V3 emission{mf[3], mf[4], mf[5]};
    if (mt_e >= 0) emission = rtv::mulv(rtv::reduce(tex_sample_ti(sc, ti_e, tc, true)), emission);
    P.set_e(nv, emission);
    RT_PROF_SEG(0);
    // Primitive::get_shading_normal (primitive.cpp:86-105)
    V3 n0{a0.x, a0.y, a0.z}, n1{a0.w, a1.x, a1.y}, n2{a1.z, a1.w, a2.x};
    V3 lz = rtv::normal(rtv::add(rtv::add(rtv::mul(n0, w), rtv::mul(n1, u)), rtv::mul(n2, v)));
    V3 N = lz;
    if (mt_n >= 0) {
        const float4 g0 = sc.tri_tan[3 * id], g1 = sc.tri_tan[3 * id + 1], g2 = sc.tri_tan[3 * id + 2];
        V3 t0{g0.x, g0.y, g0.z}, t1{g1.x, g1.y, g1.z}, tt2{g2.x, g2.y, g2.z};
        V3 lx = rtv::normal(mul_vector_d(sc.mesh_nt + 16 * mesh,
                                         rtv::normal(rtv::add(rtv::add(rtv::mul(t0, w), rtv::mul(t1, u)), rtv::mul(tt2, v)))));
        V3 ly = rtv::mul(rtv::cross(lz, lx), g0.w);
        V3 s = rtv::reduce(tex_sample_ti(sc, ti_n, tc, false));
        V3 ln = rtv::mul(rtv::addf(s, -0.5f), 2.f);
        N = rtv::normal(rtv::add(rtv::add(rtv::mul(lx, ln.x), rtv::mul(ly, ln.y)), rtv::mul(lz, ln.z)));
    }
    if (inside) N = rtv::neg(N);
    RT_PROF_SEG(1);
    // Primitive::get_metallic_roughness (primitive.cpp:131-140)
    float r2 = mf[7], metallic = mf[6];
    if (mt_mr >= 0) {
        V4 mr = tex_sample_ti(sc, ti_mr, tc, false);
        float rr = mr.y * mr.y;
        r2 = rr * mf[7];
        metallic = mr.z * mf[6];
    }
    r2 = rtv::smax(kRoughness2Limit, r2);
    const V3 pos = rtv::add(r.o, rtv::mul(r.d, hit.t));
    const V3 eye = rtv::neg(r.d);
    RT_PROF_SEG(2);
    const V3 dir = scene_sample(sc, pos, N, eye, r2, rng);
    RT_PROF_SEG(3);
    nv++;
    if (rtv::dot(dir, N) <= 0.f) {
        if (rtv::dot(dir, ngeo) <= 0.f) return false;
        N = ngeo;
    }
    m.pos = pos;
    m.N = N;
    m.dir = dir;
    m.tc = tc;
    m.r2 = r2;
    m.metallic = metallic;
    m.mesh = mesh;
    return true;
}

// SceneDistribution::pdf (random.cpp:210-218) from a light pdf computed elsewhere.
__device__ __forceinline__ float scene_pdf_lp(const DevScene &sc, V3 N, V3 eye, float r2, V3 dir, float lp) {
    if (!sc.n_lights) return (cosine_pdf(N, dir) + vndf_pdf(N, eye, r2, dir)) / 2;
    return (cosine_pdf(N, dir) + lp + vndf_pdf(N, eye, r2, dir)) / 3;
}

template <class Rec>
__device__ __forceinline__ bool shade_post(const DevScene &sc, const V3 rd, const ShadeMid &m, float pdf, Rec &P, int nv,
                                           Ray &r_out) {
    RT_PROF_BEGIN
    if (pdf <= 0.f || isnan(pdf)) return false;
    const V3 pos = m.pos, N = m.N, dir = m.dir, eye = rtv::neg(rd);
    const V2 tc = m.tc;
    const float r2 = m.r2, metallic = m.metallic;
    const float *mf = sc.mesh_f + 12 * m.mesh;
    const int *mt = sc.mesh_tex + 4 * m.mesh;
    // BRDF of this vertex (scene.cpp:134-154): used only if the child ray hits
    const float coeff = 1 / pdf;
    const V3 half = rtv::normal(rtv::sub(dir, rd));
    const float vis = smith(r2, N, eye, dir) * (1.f / (4 * fabsf(rtv::dot(N, rd)) * fabsf(rtv::dot(N, dir))));
    const float spec = ggx(r2, N, half) * vis;
    const float VdotH = fabsf(rtv::dot(eye, half));
    V3 base{mf[0], mf[1], mf[2]};
    if (mt[0] >= 0) base = rtv::mulv(rtv::reduce(tex_sample(sc, mt[0], tc, true)), base);
    const float p5 = rtm::pow5_glibc(1.f - VdotH);
    const V3 fres{base.x + (1.f - base.x) * p5, base.y + (1.f - base.y) * p5, base.z + (1.f - base.z) * p5};
    const V3 metal = rtv::mul(fres, spec);
    const V3 diffuse = rtv::mul(base, kInvPiF);
    const float dsc = 0.04f + (1.f - 0.04f) * p5;
    const V3 dielectric = rtv::add(rtv::mul(diffuse, 1 - dsc), rtv::mul(rtv::mul(V3{1.f, 1.f, 1.f}, spec), dsc));
    P.set_brdf(nv - 1, rtv::add(rtv::mul(dielectric, 1 - metallic), rtv::mul(metal, metallic)), coeff,
               rtv::dot(dir, N), mf[8]);
    r_out = make_ray(rtv::add(pos, rtv::mul(dir, kStep)), dir);
    RT_PROF_SEG(5);
    return true;
}


// The whole vertex in one piece (light pdf walked inline): records vertex nv (its emission
// and, if the path continues, its BRDF factors), advances nv and replaces r by the bounce
// ray.  Returns false where the recursion returns at this vertex (sample below the surface,
// pdf <= 0 or NaN).
// `stk`: the light walk's stack (see light_pdf).
template <bool COUNT, class Rec, class Stack>
__device__ bool shade_hit(const DevScene &sc, Ray &r, const Hit &hit, Rng &rng, Counters &cnt, Rec &P, int &nv,
                          Stack &stk) {
    ShadeMid m;
    if (!shade_pre<COUNT>(sc, r, hit, rng, cnt, P, nv, m)) return false;
    RT_PROF_BEGIN
    const float pdf = scene_pdf<COUNT>(sc, m.pos, m.N, rtv::neg(r.d), m.r2, m.dir, cnt, stk);
    RT_PROF_SEG(4);
    return shade_post(sc, r.d, m, pdf, P, nv, r);
}
template <bool COUNT, class Rec>
__device__ bool shade_hit(const DevScene &sc, Ray &r, const Hit &hit, Rng &rng, Counters &cnt, Rec &P, int &nv) {
    LocalStack stk;
    return shade_hit<COUNT>(sc, r, hit, rng, cnt, P, nv, stk);
}

// Backward fold over the recorded vertices (a primary miss gives bg colour 0).
template <class Rec>
__device__ __forceinline__ V3 fold_path(const Rec &P, int nv) {
    if (nv == 0) return V3{0.f, 0.f, 0.f};
    V3 c = P.get_e(nv - 1);
    for (int k = nv - 2; k >= 0; --k) {
        V3 x = rtv::mul(c, P.get_coeff(k));
        x = rtv::mulv(x, P.get_m(k));
        x = rtv::mul(x, P.get_cos(k));
        x = rtv::mul(x, P.get_alpha(k));
        c = rtv::add(P.get_e(k), x);
    }
    return c;
}

// fold_path over vertex records in memory: the same backward recurrence, with the records
// read four vertices at a time (all loads of a batch issue before the first is used, one
// round trip per batch instead of one per vertex).
__device__ __forceinline__ V3 fold_path(const AosRec &P, int nv) {
    if (nv == 0) return V3{0.f, 0.f, 0.f};
    V3 c = P.get_e(nv - 1);
    for (int hi = nv - 2; hi >= 0; hi -= 4) {
        float4 A[4], B[4];
        float C[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = hi - j >= 0 ? hi - j : 0;
            A[j] = P.ab[2 * P.v(k)];
            B[j] = P.ab[2 * P.v(k) + 1];
            C[j] = P.c[P.v(k)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (hi - j < 0) break;
            V3 x = rtv::mul(c, A[j].w);
            x = rtv::mulv(x, V3{B[j].x, B[j].y, B[j].z});
            x = rtv::mul(x, B[j].w);
            x = rtv::mul(x, C[j]);
            c = rtv::add(V3{A[j].x, A[j].y, A[j].z}, x);
        }
    }
    return c;
}

// One sample: ray_depth traversals at most (the 7th call returns without tracing).
template <bool COUNT>
__device__ V3 trace_sample(const DevScene &sc, Ray r, Rng &rng, Counters &cnt) {
    PathRec P;
    int nv = 0;
    int power = sc.ray_depth;
    while (power > 0) {
        power -= 1;
        Hit hit;
        bool ok = closest_hit<COUNT>(sc, r, hit, cnt);
        if (!(ok && hit.t < sc.max_distance)) break;   // miss: bg colour 0, unsuccessful
        if (!shade_hit<COUNT>(sc, r, hit, rng, cnt, P, nv)) break;
    }
    return fold_path(P, nv);
}

// Camera::cast_in_pixel (camera.cpp:49-62)
__device__ __forceinline__ Ray camera_ray(const DevScene &sc, int px, int py, float ox, float oy) {
    V3 t;
    t.x = (2.f * ((float)px + 0.5f + ox) / sc.fwidth - 1) * sc.tan_fov[0];
    t.y = -(2.f * ((float)py + 0.5f + oy) / sc.fheight - 1) * sc.tan_fov[1];
    t.z = 1;
    V3 d{0.f, 0.f, 0.f};
    const float tv[3] = {t.x, t.y, t.z};
#pragma unroll
    for (int i = 0; i < 3; ++i)
        d = rtv::add(d, rtv::mul(V3{sc.cam_axes[3 * i], sc.cam_axes[3 * i + 1], sc.cam_axes[3 * i + 2]}, tv[i]));
    return make_ray(V3{sc.cam_pos[0], sc.cam_pos[1], sc.cam_pos[2]}, d);
}

// Scene::render body for one pixel (scene.cpp:34-43) with the per-pixel RNG convention.
template <bool COUNT>
__device__ V3 render_pixel(const DevScene &sc, int i, int j, int spp, Counters &cnt) {
    Rng rng;
    uint32_t seed = (uint32_t)(j * sc.width + i) % 2147483647u;
    rng.x = seed == 0 ? 1u : seed;
    rng.saved_avail = 0;
    rng.saved = 0.f;
    V3 sum{0.f, 0.f, 0.f};
    for (int s = 0; s < spp; ++s) {
        float ox = rng_offset(rng);
        float oy = rng_offset(rng);
        Ray r = camera_ray(sc, i, j, ox, oy);
        V3 c = trace_sample<COUNT>(sc, r, rng, cnt);
        sum = rtv::add(sum, c);
    }
    return sum;
}

}  // namespace rtd
