// integration/render_mi355x.cpp — the reference-side binding of the MI355X drop-in.
//
// This is the glue a maintainer of Korinin38/raytracing-hw adds to use librt_hw_amd.so
// behind the reference's own host code: src/main.cpp parses the glTF with the reference's
// parse_scene_gltf (scene_parser.cpp:25-350, which also builds the BVH and the light list),
// then, instead of Scene::render (scene.cpp:17-65), calls render_on_mi355x below, which
//   1. flattens the parsed Scene (scene.h:14-38) into rt_scene_view arrays: the BVH-ordered
//      objects, bvh.nodes, the light list + its BVH as ManyLightsDistribution builds them
//      (random.cpp:156-168), materials, textures and the camera (camera.h:22-30);
//   2. hands them to rt_scene_from_view and renders the frame on every GPU of the node with
//      rt_render_frame (row-block shards, one host thread per device; each shard finished to
//      8 bits on its GPU exactly as Scene::render finishes it, scene.cpp:54-64, and gathered
//      device-to-device onto GPU 0);
//   3. writes the 8-bit frame into scene.camera->canvas, so scene.draw_into(output)
//      (canvas.h:76-89) is unchanged.
// Errors come back as status codes and are rethrown as std::runtime_error, the reference's
// convention.  Built against the reference's unmodified headers and objects by
// oracle/Makefile (`make -C oracle integration` -> oracle/_ref/render_mi355x).
//
// The binary is the reference's `solution` with that one call swapped:
//   render_mi355x input.gltf W H spp [output.ppm]        (RT_GPUS=n: use n devices)
//   render_mi355x --view input.gltf W H out.rtd          (the flattened view, for tests)
#include <core/scene.h>
#include <io/scene_parser.h>
#include <utils/random.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_hw.h"
#include "rtdump.h"

namespace {

void check(int rc) {
    if (rc != RT_OK) throw std::runtime_error(rt_last_error());
}

float bits_f(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// Scene::max_distance is private (scene.h:35).  Scene::intersect starts every query from
// distance = max_distance (scene.cpp:76-78) and returns it unchanged for a ray that meets
// nothing, so a ray leaving the scene's bounding box reads it through the public API.
// (A maintainer would rather add `float get_max_distance() const` to Scene; this glue
// builds against the unmodified headers.)
float max_distance_of(const Scene &s) {
    const AABB &box = s.bvh.nodes.at(0).aabb;
    Ray r(vector3f{box.max.x + 1.f, box.max.y + 1.f, box.max.z + 1.f}, vector3f{1.f, 1.f, 1.f});
    r.power = 1;
    Engine e(1u);
    return s.intersect(r, e, true).distance;
}

// BVH nodes (bvh.h:10-17) in the view's 8-float layout: box, then (left, split axis) for
// an internal node (right = left + 1, bvh.cpp builds siblings adjacent), (first, 3 | count << 2)
// for a leaf.
void flatten_nodes(const BVH &b, std::vector<float> &out, uint32_t &depth) {
    out.clear();
    std::vector<uint32_t> level(b.nodes.size(), 0);
    depth = 0;
    for (size_t k = 0; k < b.nodes.size(); ++k) {
        const Node &n = b.nodes[k];
        for (int i = 0; i < 3; ++i) out.push_back(n.aabb.min[i]);
        for (int i = 0; i < 3; ++i) out.push_back(n.aabb.max[i]);
        const bool leaf = n.primitive_count > 0;
        if (!leaf) {
            if (n.right != n.left + 1) throw std::runtime_error("render_mi355x: BVH children not adjacent");
            level[n.left] = level[n.right] = level[k] + 1;
        }
        depth = std::max(depth, level[k]);
        const uint32_t a = (uint32_t)(leaf ? n.first_primitive_id : n.left);
        const uint32_t c = leaf ? (uint32_t)(3u | (n.primitive_count << 2)) : (uint32_t)n.split_dim;
        out.push_back(bits_f(a));
        out.push_back(bits_f(c));
    }
}

struct FlatScene {
    std::vector<float> tri, attr, tan, node, light, light_node, mesh_f;
    std::vector<int32_t> mesh_tex;
    std::vector<double> mesh_nt;
    std::vector<uint32_t> tex_info;
    std::vector<uint8_t> texels;
    rt_scene_view view{};
};

void flatten(const Scene &s, FlatScene &f) {
    rt_scene_view &v = f.view;
    const Camera &cam = *s.camera;
    v.width = cam.canvas.width();
    v.height = cam.canvas.height();
    v.samples = s.samples;
    v.ray_depth = s.ray_depth;
    v.max_distance = max_distance_of(s);
    const vector3f p = cam.get_position();
    for (int k = 0; k < 3; ++k) v.cam_pos[k] = p[k];
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 3; ++k) v.cam_axes[3 * a + k] = cam.get_axis(a)[k];
    const vector2f fov = cam.get_fov();
    v.cam_fov[0] = fov.x;
    v.cam_fov[1] = fov.y;
    v.tan_half_fov[0] = std::tan(fov.x / 2);   // as Camera::cast_in_pixel (camera.cpp:51-52)
    v.tan_half_fov[1] = std::tan(fov.y / 2);
    // triangles in the BVH's order (bvh.cpp:166 reorders objects)
    for (const Primitive &o : s.objects) {
        for (int q = 0; q < 3; ++q)
            for (int k = 0; k < 3; ++k) f.tri.push_back(o.position[q][k]);
        const vector3f g = o.get_geometric_normal();
        for (int k = 0; k < 3; ++k) f.tri.push_back(g[k]);
        for (int q = 0; q < 3; ++q)
            for (int k = 0; k < 3; ++k) f.attr.push_back(o.normal[q][k]);
        for (int q = 0; q < 3; ++q)
            for (int k = 0; k < 2; ++k) f.attr.push_back(o.texcoord[q][k]);
        f.attr.push_back(bits_f((uint32_t)o.mesh_id));
        for (int q = 0; q < 3; ++q)
            for (int k = 0; k < 4; ++k) f.tan.push_back(o.tangent[q][k]);
    }
    flatten_nodes(s.bvh, f.node, v.bvh_depth);
    // light list and light BVH as rng::ManyLightsDistribution builds them (random.cpp:156-168)
    std::vector<Primitive> lights;
    for (const Primitive &o : s.objects)
        if (o.emissive()) lights.push_back(o);
    BVH lbvh;
    if (!lights.empty()) lbvh.buildBVH(lights);
    for (const Primitive &o : lights) {
        for (int q = 0; q < 3; ++q)
            for (int k = 0; k < 3; ++k) f.light.push_back(o.position[q][k]);
        const vector3f g = o.get_geometric_normal();   // fills cache.triangle_area too
        for (int k = 0; k < 3; ++k) f.light.push_back(g[k]);
        f.light.push_back(o.cache.triangle_area);
        f.light.insert(f.light.end(), {0.f, 0.f, 0.f});
    }
    v.light_bvh_depth = 0;
    if (!lights.empty()) flatten_nodes(lbvh, f.light_node, v.light_bvh_depth);
    for (const Mesh &m : s.meshes) {
        const Material &a = m.material;
        const float mf[12] = {a.base_color.x, a.base_color.y, a.base_color.z, a.emission.x, a.emission.y, a.emission.z,
                              a.metallic, a.roughness2, a.alpha, a.ior, 0.f, 0.f};
        f.mesh_f.insert(f.mesh_f.end(), mf, mf + 12);
        f.mesh_tex.insert(f.mesh_tex.end(), {a.base_color_i, a.normal_i, a.metallic_roughness_i, a.emission_i});
        f.mesh_nt.insert(f.mesh_nt.end(), m.normal_transform.data, m.normal_transform.data + 16);
    }
    // textures as RGBA8 (tinygltf decodes with 4 components, tiny_gltf.h:2609)
    for (const Texture &t : s.textures) {
        if (t.channels != 4 || t.bytes_per_channel != 1) throw std::runtime_error("render_mi355x: texture is not RGBA8");
        f.tex_info.insert(f.tex_info.end(), {(uint32_t)(f.texels.size() / 4), (uint32_t)t.width, (uint32_t)t.height, 4u});
        f.texels.insert(f.texels.end(), t.data.begin(), t.data.begin() + (size_t)t.width * t.height * 4);
    }
    v.n_tris = (uint32_t)s.objects.size();
    v.tri = f.tri.data();
    v.tri_attr = f.attr.data();
    v.tri_tan = f.tan.data();
    v.n_nodes = (uint32_t)(f.node.size() / 8);
    v.node = f.node.data();
    v.n_lights = (uint32_t)lights.size();
    v.light = f.light.data();
    v.n_light_nodes = (uint32_t)(f.light_node.size() / 8);
    v.light_node = f.light_node.data();
    v.n_meshes = (uint32_t)s.meshes.size();
    v.mesh_f = f.mesh_f.data();
    v.mesh_tex = f.mesh_tex.data();
    v.mesh_normal_transform = f.mesh_nt.data();
    v.n_textures = (uint32_t)s.textures.size();
    v.tex_info = f.tex_info.data();
    v.texels = f.texels.data();
    v.n_texel_bytes = f.texels.size();
}

// Scene::render on the node's GPUs: same canvas, same bits as the reference's loop with the
// per-pixel RNG convention (include/rt_hw.h).
void render_on_mi355x(Scene &s, int n_gpus, rt_stats *st) {
    FlatScene f;
    flatten(s, f);
    rt_scene *rs = nullptr;
    check(rt_scene_from_view(&f.view, &rs));
    const int W = f.view.width, H = f.view.height;
    rt_params p{};
    p.spp = s.samples;
    p.row_block = 8;
    // the finished 8-bit frame, gathered device-to-device onto GPU 0 (rt_render_frame)
    std::vector<uint8_t> rgb((size_t)W * H * 3);
    int rc = rt_render_frame(rs, &p, n_gpus, nullptr, rgb.data(), nullptr, st);
    rt_scene_free(rs);
    check(rc);
    for (int j = 0; j < H; ++j)
        for (int i = 0; i < W; ++i) {
            const uint8_t *c = &rgb[3 * ((size_t)j * W + i)];
            s.camera->canvas.set({i, j}, vector3si{c[0], c[1], c[2]});
        }
}

void write_view(const Scene &s, const char *path) {
    FlatScene f;
    flatten(s, f);
    rt_scene *rs = nullptr;
    check(rt_scene_from_view(&f.view, &rs));   // the library's own validation and copy ...
    rt_scene_view v{};
    check(rt_scene_get_view(rs, &v));           // ... read back as the kernels will see it
    auto fl = [](const float *p, size_t n) { return std::vector<float>(p, p + n); };
    RtDump d(path);
    d.put("tri", fl(v.tri, 12 * (size_t)v.n_tris), {v.n_tris, 12});
    d.put("tri_attr", fl(v.tri_attr, 16 * (size_t)v.n_tris), {v.n_tris, 16});
    d.put("tri_tan", fl(v.tri_tan, 12 * (size_t)v.n_tris), {v.n_tris, 12});
    d.put("node", fl(v.node, 8 * (size_t)v.n_nodes), {v.n_nodes, 8});
    d.put("light", fl(v.light, 16 * (size_t)v.n_lights), {v.n_lights, 16});
    d.put("light_node", fl(v.light_node, 8 * (size_t)v.n_light_nodes), {v.n_light_nodes, 8});
    d.put("mesh_f", fl(v.mesh_f, 12 * (size_t)v.n_meshes), {v.n_meshes, 12});
    d.put("mesh_tex", std::vector<int32_t>(v.mesh_tex, v.mesh_tex + 4 * (size_t)v.n_meshes), {v.n_meshes, 4});
    d.put("mesh_normal_transform",
          std::vector<double>(v.mesh_normal_transform, v.mesh_normal_transform + 16 * (size_t)v.n_meshes), {v.n_meshes, 16});
    d.put("camera", std::vector<float>{v.cam_pos[0], v.cam_pos[1], v.cam_pos[2], v.cam_axes[0], v.cam_axes[1],
                                       v.cam_axes[2], v.cam_axes[3], v.cam_axes[4], v.cam_axes[5], v.cam_axes[6],
                                       v.cam_axes[7], v.cam_axes[8], v.cam_fov[0], v.cam_fov[1], v.tan_half_fov[0],
                                       v.tan_half_fov[1], v.max_distance});
    d.put("meta", std::vector<int32_t>{v.width, v.height, v.samples, v.ray_depth, (int32_t)v.bvh_depth,
                                       (int32_t)v.light_bvh_depth});
    d.put("texels", std::vector<uint8_t>(v.texels, v.texels + v.n_texel_bytes));
    d.put("tex_info", std::vector<uint32_t>(v.tex_info, v.tex_info + 4 * (size_t)v.n_textures), {v.n_textures, 4});
    d.close();
    rt_scene_free(rs);
}

}  // namespace

int main(int argc, char *argv[]) {
    if (argc == 6 && std::string(argv[1]) == "--view") {
        Scene scene = parse_scene_gltf(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), 1);
        write_view(scene, argv[5]);
        return 0;
    }
    if (argc < 5 || argc > 6) throw std::runtime_error("Invalid arguments - " + std::to_string(argc) + " (expected: 5)");
    const std::string input = argv[1], output = argc == 6 ? argv[5] : "output.ppm";
    const int width = std::atoi(argv[2]), height = std::atoi(argv[3]), samples = std::atoi(argv[4]);
    const char *g = std::getenv("RT_GPUS");
    const int n_gpus = g ? std::atoi(g) : 0;

    std::cout << "Loading scene." << std::endl;
    const auto t0 = std::chrono::steady_clock::now();
    Scene scene = parse_scene_gltf(input, width, height, samples);
    const auto t1 = std::chrono::steady_clock::now();
    std::cout << "Scene loaded: " << std::setprecision(2) << std::chrono::duration<double>(t1 - t0).count()
              << " seconds." << std::endl;
    std::cout << std::setprecision(6) << "Rendering scene." << std::endl;
    rt_stats st{};
    render_on_mi355x(scene, n_gpus, &st);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    std::cout << "      " << sec << " seconds (" << sec * 1000 << " ms) elapsed on " << st.devices
              << " MI355X (render " << st.render_ms << " ms)." << std::endl;
    scene.draw_into(output);
    std::cout << "Frame drawn into " << output << std::endl;
    return 0;
}
