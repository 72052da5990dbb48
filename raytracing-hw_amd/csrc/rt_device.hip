// rt_device.hip — MI355X (gfx950) render kernels and the device half of the C ABI.
//
// Kernels (SURVEY.md §2 kernel inventory):
//   rt_pixels_kernel      one lane per pixel of the shard, full spp loop in-lane
//                         (replaces Scene::render's OpenMP pixel loop, scene.cpp:31-52)
//   rt_persistent_kernel  persistent lanes pulling pixels from a per-launch atomic
//                         queue (wave-aggregated dequeue), same per-pixel math
// Both write the per-pixel float RGB sum (sample_canvas, scene.cpp:20,42) of the owned
// rows; the result is independent of the kernel, the launch shape and the partition.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_path.h"
#include "rt_scene.h"

using rtd::Counters;
using rtd::DevScene;

struct rt_device_scene {
    int device = -1;
    void *buf = nullptr;         // one allocation holding every array
    DevScene ds{};
    unsigned long long *counters = nullptr;  // 6 x u64
    unsigned int *queue = nullptr;           // persistent kernel work counter
    int cu_count = 0;
};

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return rt_fail(RT_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ------------------------------------------------------------------------ kernels
struct ShardGeom {
    int width, rank, world, row_block;
    long long n_pixels;
};

__device__ __forceinline__ int shard_row(const ShardGeom &g, int k) {
    // k-th owned row: rows whose (row / row_block) % world == rank, ascending
    const int blk = k / g.row_block;
    return (blk * g.world + g.rank) * g.row_block + (k % g.row_block);
}

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const Counters &c, unsigned long long *out) {
    if (!COUNT) return;
    atomicAdd(&out[0], (unsigned long long)c.rays);
    atomicAdd(&out[1], (unsigned long long)c.aabb);
    atomicAdd(&out[2], (unsigned long long)c.tri);
    atomicAdd(&out[3], (unsigned long long)c.lq);
    atomicAdd(&out[4], (unsigned long long)c.laabb);
    atomicAdd(&out[5], (unsigned long long)c.ltri);
    atomicAdd(&out[6], (unsigned long long)c.hits);
}

template <bool COUNT>
__global__ void __launch_bounds__(256) rt_pixels_kernel(DevScene sc, ShardGeom g, int spp, float *out,
                                                         unsigned long long *counters) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= g.n_pixels) return;
    const int k = (int)(p / g.width), i = (int)(p % g.width);
    const int j = shard_row(g, k);
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    rtv::V3 s = rtd::render_pixel<COUNT>(sc, i, j, spp, cnt);
    out[3 * p + 0] = s.x;
    out[3 * p + 1] = s.y;
    out[3 * p + 2] = s.z;
    flush_counters<COUNT>(cnt, counters);
}

// Persistent variant: grid = resident lanes; each wave takes 64 consecutive pixels per
// dequeue (one returning atomic per wave), so lanes that finish early pick up new work
// without waiting for a block-wide barrier.  Exit: every wave leaves when the queue is
// drained, so the grid always drains.
template <bool COUNT>
__global__ void __launch_bounds__(256) rt_persistent_kernel(DevScene sc, ShardGeom g, int spp, float *out,
                                                             unsigned long long *counters, unsigned int *queue) {
    const int lane = threadIdx.x & 63;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    for (;;) {
        unsigned int base = 0;
        if (lane == 0) base = atomicAdd(queue, 64u);
        base = __shfl(base, 0, 64);
        if ((long long)base >= g.n_pixels) break;
        const long long p = (long long)base + lane;
        if (p < g.n_pixels) {
            const int k = (int)(p / g.width), i = (int)(p % g.width);
            const int j = shard_row(g, k);
            rtv::V3 s = rtd::render_pixel<COUNT>(sc, i, j, spp, cnt);
            out[3 * p + 0] = s.x;
            out[3 * p + 1] = s.y;
            out[3 * p + 2] = s.z;
        }
    }
    flush_counters<COUNT>(cnt, counters);
}

// Ray-level entry: BVH::intersect + ManyLightsDistribution::pdf for explicit rays.
__global__ void __launch_bounds__(256) rt_rays_kernel(DevScene sc, long long n, const float *org, const float *dir,
                                                       float *out_f, long long *out_i) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    rtd::Ray r = rtd::make_ray(rtv::V3{org[3 * k], org[3 * k + 1], org[3 * k + 2]},
                               rtv::V3{dir[3 * k], dir[3 * k + 1], dir[3 * k + 2]});
    Counters c1{0, 0, 0, 0, 0, 0, 0}, c2{0, 0, 0, 0, 0, 0, 0};
    rtd::Hit h;
    const bool ok = rtd::closest_hit<true>(sc, r, h, c1);
    const float lp = sc.n_lights ? rtd::light_pdf<true>(sc, r.o, r.d, c2) : 0.f;
    out_f[4 * k + 0] = ok ? h.t : 0.f;
    out_f[4 * k + 1] = ok ? h.u : 0.f;
    out_f[4 * k + 2] = ok ? h.v : 0.f;
    out_f[4 * k + 3] = lp;
    out_i[6 * k + 0] = ok;
    out_i[6 * k + 1] = ok ? h.prim : -1;
    out_i[6 * k + 2] = c1.aabb;
    out_i[6 * k + 3] = c1.tri;
    out_i[6 * k + 4] = c2.laabb;
    out_i[6 * k + 5] = c2.ltri;
}

// ------------------------------------------------------------------------ host side
namespace {

template <class T>
size_t append(std::vector<uint8_t> &blob, const std::vector<T> &v) {
    size_t off = (blob.size() + 255) & ~size_t(255);
    blob.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

int ensure_device_scene(rt_scene *s, int device) {
    if (s->dev && s->dev->device == device) return RT_OK;
    if (s->dev) rt_device_scene_release(s);
    if (s->bvh_depth + 2 >= (uint32_t)rtd::kStack || s->light_bvh_depth + 2 >= (uint32_t)rtd::kStack)
        return rt_fail(RT_ERR_LIMIT, "BVH deeper than the device traversal stack (" + std::to_string(rtd::kStack) + ")");
    if (s->ray_depth > rtd::kMaxDepth) return rt_fail(RT_ERR_LIMIT, "ray_depth exceeds device limit");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return rt_fail(RT_ERR_DEVICE, "no HIP device " + std::to_string(device));
    HIP_TRY(hipSetDevice(device));
    std::vector<uint8_t> blob;
    const size_t o_tri = append(blob, s->tri), o_attr = append(blob, s->tri_attr), o_tan = append(blob, s->tri_tan),
                 o_node = append(blob, s->node), o_light = append(blob, s->light),
                 o_lnode = append(blob, s->light_node), o_mf = append(blob, s->mesh_f),
                 o_mt = append(blob, s->mesh_tex), o_nt = append(blob, s->mesh_nt), o_ti = append(blob, s->tex_info),
                 o_tx = append(blob, s->texels);
    blob.resize(((blob.size() + 255) & ~size_t(255)) + 256);
    rt_device_scene *d = new rt_device_scene();
    d->device = device;
    hipError_t e = hipMalloc(&d->buf, blob.size());
    if (e == hipSuccess) e = hipMemcpy(d->buf, blob.data(), blob.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&d->counters, 8 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void **)&d->queue, 64);
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        if (d->buf) (void)hipFree(d->buf);
        if (d->counters) (void)hipFree(d->counters);
        if (d->queue) (void)hipFree(d->queue);
        delete d;
        return rt_fail(RT_ERR_DEVICE, std::string("scene upload: ") + hipGetErrorString(e));
    }
    d->cu_count = prop.multiProcessorCount;
    uint8_t *b = (uint8_t *)d->buf;
    DevScene &ds = d->ds;
    ds.tri = (const float4 *)(b + o_tri);
    ds.tri_attr = (const float4 *)(b + o_attr);
    ds.tri_tan = (const float4 *)(b + o_tan);
    ds.node = (const float4 *)(b + o_node);
    ds.light = (const float4 *)(b + o_light);
    ds.light_node = (const float4 *)(b + o_lnode);
    ds.mesh_f = (const float *)(b + o_mf);
    ds.mesh_tex = (const int *)(b + o_mt);
    ds.mesh_nt = (const double *)(b + o_nt);
    ds.tex_info = (const uint4 *)(b + o_ti);
    ds.texels = (const uint32_t *)(b + o_tx);
    ds.n_lights = (int)(s->light.size() / 16);
    ds.ray_depth = s->ray_depth;
    ds.max_distance = s->max_distance;
    ds.width = s->width;
    ds.height = s->height;
    std::memcpy(ds.cam_pos, s->cam_pos, sizeof ds.cam_pos);
    std::memcpy(ds.cam_axes, s->cam_axes, sizeof ds.cam_axes);
    std::memcpy(ds.tan_fov, s->tan_half_fov, sizeof ds.tan_fov);
    s->dev = d;
    return RT_OK;
}

int launch(rt_scene *s, const rt_params *p, float *d_out, hipStream_t stream, rt_stats *st) {
    if (!s || !p || !d_out) return rt_fail(RT_ERR_ARG, "rt_render: NULL argument");
    if (!s->dev) return rt_fail(RT_ERR_ARG, "rt_render: scene not uploaded");
    const int world = p->world > 0 ? p->world : 1, rank = p->rank, rb = p->row_block > 0 ? p->row_block : 8;
    const int spp = p->spp > 0 ? p->spp : s->samples;
    const int64_t rows = rt_shard_rows_impl(s->height, rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    ShardGeom g{s->width, rank, world, rb, (long long)rows * s->width};
    rt_device_scene *d = s->dev;
    HIP_TRY(hipSetDevice(d->device));
    const bool count = p->count != 0;
    if (count) HIP_TRY(hipMemsetAsync(d->counters, 0, 8 * sizeof(unsigned long long), stream));
    HIP_TRY(hipMemsetAsync(d->queue, 0, 4, stream));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (st) {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, stream));
    }
    if (g.n_pixels > 0) {
        if (p->kernel == 1) {
            const unsigned blocks = (unsigned)((g.n_pixels + 255) / 256);
            if (count) hipLaunchKernelGGL(rt_pixels_kernel<true>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters);
            else hipLaunchKernelGGL(rt_pixels_kernel<false>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters);
        } else {
            // persistent grid: enough waves to fill every SIMD a few times over
            long long waves = (g.n_pixels + 63) / 64;
            long long want = (long long)d->cu_count * 16;  // 16 waves per CU = 4 blocks of 256
            unsigned blocks = (unsigned)((std::min(waves, want) + 3) / 4);
            if (blocks == 0) blocks = 1;
            if (count) hipLaunchKernelGGL(rt_persistent_kernel<true>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
            else hipLaunchKernelGGL(rt_persistent_kernel<false>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
        }
        HIP_TRY(hipGetLastError());
    }
    if (st) {
        HIP_TRY(hipEventRecord(e1, stream));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        std::memset(st, 0, sizeof *st);
        st->pixels = (uint64_t)g.n_pixels;
        st->samples = (uint64_t)g.n_pixels * (uint64_t)spp;
        st->render_ms = ms;
        if (count) {
            unsigned long long c[8];
            HIP_TRY(hipMemcpy(c, d->counters, sizeof c, hipMemcpyDeviceToHost));
            st->rays = c[0]; st->aabb_tests = c[1]; st->tri_tests = c[2];
            st->light_queries = c[3]; st->light_aabb_tests = c[4]; st->light_tri_tests = c[5];
            st->shading_hits = c[6];
        }
    }
    return RT_OK;
}

}  // namespace

void rt_device_scene_release(rt_scene *s) {
    if (!s || !s->dev) return;
    rt_device_scene *d = s->dev;
    if (hipSetDevice(d->device) == hipSuccess) {
        if (d->buf) (void)hipFree(d->buf);
        if (d->counters) (void)hipFree(d->counters);
        if (d->queue) (void)hipFree(d->queue);
    }
    delete d;
    s->dev = nullptr;
}

extern "C" {

int rt_scene_upload(rt_scene *s, int32_t device) {
    if (!s) return rt_fail(RT_ERR_ARG, "rt_scene_upload: NULL scene");
    return ensure_device_scene(s, device);
}

int rt_render_device(rt_scene *s, const rt_params *p, float *d_out, void *stream, rt_stats *st) {
    return launch(s, p, d_out, (hipStream_t)stream, st);
}

int rt_render(rt_scene *s, const rt_params *p, float *out, rt_stats *st) {
    if (!s || !p || !out) return rt_fail(RT_ERR_ARG, "rt_render: NULL argument");
    if (!s->dev) {
        int rc = ensure_device_scene(s, 0);
        if (rc) return rc;
    }
    const int world = p->world > 0 ? p->world : 1, rb = p->row_block > 0 ? p->row_block : 8;
    const int64_t rows = rt_shard_rows_impl(s->height, p->rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    const size_t bytes = (size_t)rows * s->width * 3 * sizeof(float);
    HIP_TRY(hipSetDevice(s->dev->device));
    float *d_out = nullptr;
    HIP_TRY(hipMalloc(&d_out, bytes ? bytes : 4));
    rt_stats local;
    int rc = launch(s, p, d_out, nullptr, st ? st : &local);
    if (rc == RT_OK) {
        hipError_t e = hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = rt_fail(RT_ERR_DEVICE, std::string("rt_render copy: ") + hipGetErrorString(e));
    }
    (void)hipFree(d_out);
    return rc;
}

int rt_intersect_rays(rt_scene *s, int64_t n, const float *org, const float *dir, float *out_f, int64_t *out_i) {
    if (!s || n < 0 || (n > 0 && (!org || !dir || !out_f || !out_i))) return rt_fail(RT_ERR_ARG, "rt_intersect_rays: bad argument");
    if (n == 0) return RT_OK;
    if (!s->dev) {
        int rc = ensure_device_scene(s, 0);
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(s->dev->device));
    float *d_o = nullptr, *d_d = nullptr, *d_f = nullptr;
    long long *d_i = nullptr;
    const size_t v3 = (size_t)n * 3 * sizeof(float);
    hipError_t e = hipMalloc(&d_o, v3);
    if (e == hipSuccess) e = hipMalloc(&d_d, v3);
    if (e == hipSuccess) e = hipMalloc(&d_f, (size_t)n * 4 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_i, (size_t)n * 6 * sizeof(long long));
    if (e == hipSuccess) e = hipMemcpy(d_o, org, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dir, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rt_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, s->dev->ds, (long long)n,
                           d_o, d_d, d_f, d_i);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_f, d_f, (size_t)n * 4 * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_i, d_i, (size_t)n * 6 * sizeof(long long), hipMemcpyDeviceToHost);
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_f);
    (void)hipFree(d_i);
    if (e != hipSuccess) return rt_fail(RT_ERR_DEVICE, std::string("rt_intersect_rays: ") + hipGetErrorString(e));
    return RT_OK;
}

int32_t rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_device_synchronize(void) {
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

}  // extern "C"
