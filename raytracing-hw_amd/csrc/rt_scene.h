// rt_scene.h — host-side scene object behind the opaque rt_scene handle (include/rt_hw.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rt_hw.h"

struct rt_device_scene;  // owned by rt_device.hip: one per device the scene is uploaded to
struct rt_device_blob;   // owned by rt_device.hip: the device image of the scene, built once

constexpr int kRtMaxDevices = 64;

struct rt_scene {
    int32_t width = 0, height = 0, samples = 0, ray_depth = 6;
    float max_distance = 1e9f;
    float cam_pos[3] = {0, 0, 0};
    float cam_axes[9] = {0};
    float cam_fov[2] = {0, 0};
    float tan_half_fov[2] = {0, 0};

    std::vector<float> tri, tri_attr, tri_tan, node;
    uint32_t bvh_depth = 0;
    std::vector<float> light, light_node;
    uint32_t light_bvh_depth = 0;
    std::vector<float> mesh_f;
    std::vector<int32_t> mesh_tex;
    std::vector<double> mesh_nt;
    std::vector<uint32_t> tex_info;
    std::vector<uint8_t> texels;

    rt_device_scene *dev[kRtMaxDevices] = {};   // [HIP device id]
    rt_device_blob *blob = nullptr;
};

// error plumbing shared by rt_host.cpp and rt_device.hip
void rt_set_error(const std::string &msg);
int rt_fail(int code, const std::string &msg);

// implemented in rt_device.hip: frees every device copy and the device image
void rt_device_scene_release(rt_scene *s);

// row partition helper (rt_host.cpp)
int64_t rt_shard_rows_impl(int32_t height, int32_t rank, int32_t world, int32_t row_block, int32_t *rows_out);
