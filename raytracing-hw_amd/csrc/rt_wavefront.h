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
#include "rt_wave.h"

namespace rtd {

struct WfState {
    long long n;      // path slots (= pixels of the shard)
    int D;            // vertex records per slot (= ray_depth)
    float *ox, *oy, *oz, *dx, *dy, *dz;   // current ray (origin, normalised direction)
    float *ht, *hu, *hv;                  // closest hit of the current ray
    int *hprim;                           // -1 = miss
    uint32_t *rng_x;
    float *rng_saved;
    uint32_t *meta;                       // s (bits 0-19), power (20-23), nv (24-27), saved flag (28)
    float *sx, *sy, *sz;                  // pixel sums
    float *rec;                           // 9 * D planes of n floats (SoARec)
};

__device__ __forceinline__ uint32_t meta_pack(int s, int power, int nv, uint32_t saved) {
    return (uint32_t)s | ((uint32_t)power << 20) | ((uint32_t)nv << 24) | (saved << 28);
}

// Appends `slot` to a queue when `want`: one atomic per wave, lanes keep their order.
__device__ __forceinline__ void queue_push(bool want, int slot, int *queue, unsigned *count) {
    const unsigned long long m = __ballot(want);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(count, (unsigned)__popcll(m));
    base = __shfl(base, leader, 64);
    if (want) queue[base + __popcll(m & ((1ull << lane) - 1ull))] = slot;
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

__device__ __forceinline__ void store_ray(const WfState &st, long long i, const Ray &r) {
    st.ox[i] = r.o.x; st.oy[i] = r.o.y; st.oz[i] = r.o.z;
    st.dx[i] = r.d.x; st.dy[i] = r.d.y; st.dz[i] = r.d.z;
}
// Ray::Ray's state from the stored fields: inv_direction = {1,1,1} / direction (exact).
__device__ __forceinline__ Ray load_ray(const WfState &st, long long i) {
    Ray r;
    r.o = V3{st.ox[i], st.oy[i], st.oz[i]};
    r.d = V3{st.dx[i], st.dy[i], st.dz[i]};
    r.inv = rtv::divv(V3{1.f, 1.f, 1.f}, r.d);
    return r;
}

// Start sample s of slot i: jittered camera ray (scene.cpp:36-39); the first traversal
// consumes one call of the depth budget (scene.cpp:72-75).
__device__ __forceinline__ Ray start_sample(const DevScene &sc, const ShardGeom &g, long long i, Rng &rng, int &power) {
    const int k = (int)(i / g.width), px = (int)(i % g.width), py = shard_row(g, k);
    const float ox = rng_offset(rng);
    const float oy = rng_offset(rng);
    power = sc.ray_depth - 1;
    return camera_ray(sc, px, py, ox, oy);
}

}  // namespace rtd
