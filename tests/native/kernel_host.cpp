// kernel_host.cpp — TEST ONLY: compiles the GPU kernel source (raytracing-hw_amd/csrc/rt_path.h)
// for the host so tests can check its arithmetic against the goldens without a GPU.  Not
// part of the product: librt_hw_amd.so has no CPU render path.
#include <cstdint>
#include <cstring>
#include "../../raytracing-hw_amd/csrc/rt_path.h"
#include "../../include/rt_hw.h"

static rtd::DevScene make(const rt_scene_view *v) {
    rtd::DevScene s{};
    s.tri = (const float4 *)v->tri;
    s.tri_attr = (const float4 *)v->tri_attr;
    s.tri_tan = (const float4 *)v->tri_tan;
    s.node = (const float4 *)v->node;
    s.light = (const float4 *)v->light;
    s.light_node = (const float4 *)v->light_node;
    s.mesh_f = v->mesh_f;
    s.mesh_tex = v->mesh_tex;
    s.mesh_nt = v->mesh_normal_transform;
    s.tex_info = (const uint4 *)v->tex_info;
    s.texels = (const uint32_t *)v->texels;
    s.n_lights = (int)v->n_lights;
    s.ray_depth = v->ray_depth;
    s.max_distance = v->max_distance;
    s.width = v->width;
    s.height = v->height;
    std::memcpy(s.cam_pos, v->cam_pos, sizeof s.cam_pos);
    std::memcpy(s.cam_axes, v->cam_axes, sizeof s.cam_axes);
    std::memcpy(s.tan_fov, v->tan_half_fov, sizeof s.tan_fov);
    return s;
}

extern "C" void kh_render(const rt_scene_view *v, int spp, int64_t p0, int64_t p1, float *out, uint64_t *cnt) {
    rtd::DevScene s = make(v);
    uint64_t c[6] = {0, 0, 0, 0, 0, 0};
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : c[:6])
    for (int64_t p = p0; p < p1; ++p) {
        rtd::Counters k{0, 0, 0, 0, 0, 0, 0};
        rtv::V3 r = rtd::render_pixel<true>(s, (int)(p % v->width), (int)(p / v->width), spp, k);
        out[3 * (p - p0)] = r.x;
        out[3 * (p - p0) + 1] = r.y;
        out[3 * (p - p0) + 2] = r.z;
        c[0] += k.rays; c[1] += k.aabb; c[2] += k.tri; c[3] += k.lq; c[4] += k.laabb; c[5] += k.ltri;
    }
    std::memcpy(cnt, c, sizeof c);
}
