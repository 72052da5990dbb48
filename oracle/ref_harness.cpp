// ref_harness.cpp — golden-vector generator built FROM THE REFERENCE SOURCES where they lie
// (/root/reference/src, compiled by oracle/Makefile into oracle/_ref/; never copied here).
// TEST INFRASTRUCTURE ONLY: it is the checker, never the thing measured or shipped.
//
// The reference's render loop (src/core/scene.cpp:31-52) is not bit-reproducible: the
// polar-normal cache `rng::normDist` is a file-static shared by all OpenMP threads
// (src/utils/random.cpp:22) and pixel 0 is seeded from std::random_device
// (random.cpp:12-18).  This harness textually includes random.cpp with that static made
// thread_local, resets it at the start of every pixel and seeds pixel 0 with Engine(1)
//  — the per-pixel-reset convention every build component follows.
//
// Modes (all print one JSON line on stdout, after the reference's own log lines):
//   sums    <gltf> W H spp out.rtd [threads [out.ppm]]
//                                              per-pixel float RGB sums (scene.cpp:20,42) + counters
//                                              (+ the reference's finished frame of them)
//   time    <gltf> W H spp [rows [stride]]     time Scene::render itself (scene.cpp:17-65)
//   rays    <gltf> W H n out.rtd               closest-hit known answers (bvh.cpp:239-243) + per-ray test counts
//   dump    <gltf> W H out.rtd                 post-BVH scene arrays (bvh.cpp:166 reorders objects)
//   samplers <gltf> W H n out.rtd              SceneDistribution::sample/pdf + RNG known answers
//   pixels  <gltf> W H spp idx.i64 out.rtd [threads]
//                                              per-pixel sums of the listed frame pixels (raw int64
//                                              indices j*W+i) at full spp, + per-pixel test counts
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <memory>
#include <optional>
#include <random>
#include <string>
#include <vector>
#include <omp.h>

#include <utils/vector.h>
#include <utils/matrix.h>
#include <geometry/primitive.h>
#include <core/bvh.h>
#include <utils/random.h>
#include <render/canvas.h>
// random.cpp's two file-statics (uniDist, normDist) become per-thread copies.
#define static static thread_local
#include <utils/random.cpp>
#undef static
#include <core/scene.h>
#include <io/scene_parser.h>

#include "rtdump.h"

// ---------------------------------------------------------------- counting wraps
struct alignas(64) Counters {
    uint64_t rays = 0, aabb = 0, tri = 0, lqueries = 0, laabb = 0, ltri = 0;
};
static Counters g_cnt[512];
static thread_local int t_mode = 0;  // 0: outside queries, 1: scene closest-hit, 2: light all-hits

static inline Counters &cnt() { return g_cnt[omp_get_thread_num()]; }

#ifdef RT_WRAP
extern "C" {
Intersection __real__ZNK3BVH9intersectERKSt6vectorI9PrimitiveSaIS1_EE3Ray(const BVH *, const std::vector<Primitive> &, Ray);
Intersection __wrap__ZNK3BVH9intersectERKSt6vectorI9PrimitiveSaIS1_EE3Ray(const BVH *self, const std::vector<Primitive> &p, Ray r) {
    cnt().rays++;
    int old = t_mode;
    t_mode = 1;
    Intersection res = __real__ZNK3BVH9intersectERKSt6vectorI9PrimitiveSaIS1_EE3Ray(self, p, r);
    t_mode = old;
    return res;
}
std::vector<Intersection> __real__ZNK3BVH12intersectAllERKSt6vectorI9PrimitiveSaIS1_EE3Ray(const BVH *, const std::vector<Primitive> &, Ray);
std::vector<Intersection> __wrap__ZNK3BVH12intersectAllERKSt6vectorI9PrimitiveSaIS1_EE3Ray(const BVH *self, const std::vector<Primitive> &p, Ray r) {
    cnt().lqueries++;
    int old = t_mode;
    t_mode = 2;
    std::vector<Intersection> res = __real__ZNK3BVH12intersectAllERKSt6vectorI9PrimitiveSaIS1_EE3Ray(self, p, r);
    t_mode = old;
    return res;
}
std::optional<float> __real__ZNK4AABB9intersectE3Ray(const AABB *, Ray);
std::optional<float> __wrap__ZNK4AABB9intersectE3Ray(const AABB *self, Ray r) {
    if (t_mode == 1) cnt().aabb++;
    else if (t_mode == 2) cnt().laabb++;
    return __real__ZNK4AABB9intersectE3Ray(self, r);
}
Intersection __real__ZNK9Primitive9intersectE3Ray(const Primitive *, Ray);
Intersection __wrap__ZNK9Primitive9intersectE3Ray(const Primitive *self, Ray r) {
    if (t_mode == 1) cnt().tri++;
    else if (t_mode == 2) cnt().ltri++;
    return __real__ZNK9Primitive9intersectE3Ray(self, r);
}
}
#endif

static Counters total_counters() {
    Counters t;
    for (auto &c : g_cnt) {
        t.rays += c.rays; t.aabb += c.aabb; t.tri += c.tri;
        t.lqueries += c.lqueries; t.laabb += c.laabb; t.ltri += c.ltri;
    }
    return t;
}
static void reset_counters() { for (auto &c : g_cnt) c = Counters(); }

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- per-pixel-reset render
// Restates the body of scene.cpp:33-43 for one pixel, with the per-pixel RNG convention.
static vector3f render_pixel(const Scene &s, int i, int j, int spp) {
    rng::normDist.reset();
    const int W = s.camera->canvas.width();
    size_t seed = (size_t)(j * W + i);
    Engine e = seed ? rng::get_generator(seed) : Engine(1u);
    uniform_float_d offset(-0.5f, 0.5f);
    vector3f sum{0.f, 0.f, 0.f};
    for (int k = 0; k < spp; ++k) {
        vector2f po{offset(e), offset(e)};
        vector2i pp{i, j};
        Ray r = s.camera->cast_in_pixel(pp, po);
        r.power = s.ray_depth;
        auto inter = s.intersect(r, e);
        sum += inter.color;
    }
    return sum;
}

static void print_counts(const char *mode, const Counters &c, double secs, int threads, const char *extra = "") {
    std::printf("{\"mode\": \"%s\", \"rays\": %llu, \"aabb\": %llu, \"tri\": %llu, \"light_queries\": %llu, "
                "\"light_aabb\": %llu, \"light_tri\": %llu, \"seconds\": %.6f, \"threads\": %d%s}\n",
                mode, (unsigned long long)c.rays, (unsigned long long)c.aabb, (unsigned long long)c.tri,
                (unsigned long long)c.lqueries, (unsigned long long)c.laabb, (unsigned long long)c.ltri, secs,
                threads, extra);
}

// Scene::render's frame finish (scene.cpp:54-64) of per-pixel sums into the canvas, then
// Scene::draw_into / Canvas::write_to (canvas.h:76-89).
static void finish_to_ppm(const std::vector<float> &sums, int W, int H, int spp, const char *path) {
    Canvas canvas({W, H});
    const float normalizer = 1.f / (float)spp;
    const float gamma_ = 1.f / 2.2f;   // scene.h:36
    for (int j = 0; j < H; ++j)
        for (int i = 0; i < W; ++i) {
            const size_t o = 3 * ((size_t)j * W + i);
            vector3f color{sums[o], sums[o + 1], sums[o + 2]};
            color *= normalizer;
            color = aces_tonemap(color);
            color = pow(color, gamma_);
            canvas.set({i, j}, normal_to_ch8bit(color));
        }
    canvas.write_to(path);
}

static int mode_sums(int argc, char **argv) {
    if (argc < 7) throw std::runtime_error("sums <gltf> W H spp out.rtd [threads [out.ppm]]");
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]);
    int threads = argc > 7 ? atoi(argv[7]) : omp_get_max_threads();
    Scene s = parse_scene_gltf(argv[2], W, H, spp);
    std::vector<float> out((size_t)W * H * 3);
    reset_counters();
    double t0 = now_s();
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads)
    for (int p = 0; p < W * H; ++p) {
        vector3f c = render_pixel(s, p % W, p / W, spp);
        out[3 * (size_t)p + 0] = c.x;
        out[3 * (size_t)p + 1] = c.y;
        out[3 * (size_t)p + 2] = c.z;
    }
    double t1 = now_s();
    RtDump d(argv[6]);
    d.put("sums", out, {(uint64_t)H, (uint64_t)W, 3});
    Counters c = total_counters();
    std::vector<uint64_t> cv{c.rays, c.aabb, c.tri, c.lqueries, c.laabb, c.ltri};
    d.put("counters", cv);
    d.close();
    if (argc > 8) finish_to_ppm(out, W, H, spp, argv[8]);   // the reference's final image of these sums
    print_counts("sums", c, t1 - t0, threads);
    return 0;
}

// Times the reference's own Scene::render (OpenMP over all pixels; shared RNG statics made
// per-thread, otherwise unchanged).  With `rows` < H only `rows` rows are rendered: rows 0,
// stride, 2 * stride, ... (default stride 1: the first rows), so a bounded sample can span
// the frame; the camera canvas keeps H, so the rays are the full-frame rays.
static int mode_time(int argc, char **argv) {
    if (argc < 6) throw std::runtime_error("time <gltf> W H spp [rows [stride]]");
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]);
    int rows = argc > 6 ? atoi(argv[6]) : H;
    int stride = argc > 7 ? std::max(1, atoi(argv[7])) : 1;
    if ((long long)(rows - 1) * stride >= H) rows = (H - 1) / stride + 1;
    Scene s = parse_scene_gltf(argv[2], W, H, spp);
    reset_counters();
    double t0 = now_s(), t1;
    if (rows >= H) {
        s.render();
        t1 = now_s();
    } else {
        // same loop shape as scene.cpp:31 (guided,16 collapse(2)) over the sampled rows
        uniform_float_d offset(-0.5f, 0.5f);
        std::vector<vector3f> sample_canvas((size_t)W * rows, {0.f, 0.f, 0.f});
#pragma omp parallel for schedule(guided, 16) collapse(2)
        for (int k = 0; k < rows; ++k) {
            for (int i = 0; i < W; ++i) {
                const int j = k * stride;
                Engine rng = rng::get_generator(j * W + i);
                for (int q = 0; q < spp; ++q) {
                    vector2f po{offset(rng), offset(rng)};
                    vector2i pp{i, j};
                    Ray r = s.camera->cast_in_pixel(pp, po);
                    r.power = s.ray_depth;
                    auto inter = s.intersect(r, rng);
                    sample_canvas[(size_t)k * W + i] += inter.color;
                }
            }
        }
        t1 = now_s();
    }
    char extra[128];
    std::snprintf(extra, sizeof extra, ", \"pixels\": %lld, \"spp\": %d, \"stride\": %d", (long long)W * rows, spp, stride);
    print_counts("time", total_counters(), t1 - t0, omp_get_max_threads(), extra);
    return 0;
}

// Listed pixels of a frame at full spp (any W x H x spp, e.g. BASELINE's C3-C5): the same
// per-pixel loop as `sums` (render_pixel) on a subset, with per-pixel counters (the counting
// wraps count per thread and a pixel runs on one thread, so the difference is the pixel's).
static int mode_pixels(int argc, char **argv) {
    if (argc < 8) throw std::runtime_error("pixels <gltf> W H spp idx.i64 out.rtd [threads]");
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]);
    int threads = argc > 8 ? atoi(argv[8]) : omp_get_max_threads();
    std::FILE *f = std::fopen(argv[6], "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + argv[6]);
    std::vector<int64_t> idx;
    int64_t v;
    while (std::fread(&v, sizeof v, 1, f) == 1) idx.push_back(v);
    std::fclose(f);
    for (int64_t p : idx)
        if (p < 0 || p >= (int64_t)W * H) throw std::runtime_error("pixel index out of range");
    Scene s = parse_scene_gltf(argv[2], W, H, spp);
    const size_t n = idx.size();
    std::vector<float> out(n * 3);
    std::vector<uint64_t> pc(n * 6);
    reset_counters();
    double t0 = now_s();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (size_t k = 0; k < n; ++k) {
        const Counters before = cnt();
        vector3f c = render_pixel(s, (int)(idx[k] % W), (int)(idx[k] / W), spp);
        const Counters &after = cnt();
        out[3 * k + 0] = c.x;
        out[3 * k + 1] = c.y;
        out[3 * k + 2] = c.z;
        const uint64_t d[6] = {after.rays - before.rays, after.aabb - before.aabb, after.tri - before.tri,
                               after.lqueries - before.lqueries, after.laabb - before.laabb, after.ltri - before.ltri};
        std::memcpy(&pc[6 * k], d, sizeof d);
    }
    double t1 = now_s();
    RtDump d(argv[7]);
    d.put("index", idx);
    d.put("sums", out, {(uint64_t)n, 3});
    d.put("pixel_counters", pc, {(uint64_t)n, 6});
    d.scalar<int32_t>("width", W);
    d.scalar<int32_t>("height", H);
    d.scalar<int32_t>("spp", spp);
    d.close();
    char extra[96];
    std::snprintf(extra, sizeof extra, ", \"pixels\": %zu, \"spp\": %d", n, spp);
    print_counts("pixels", total_counters(), t1 - t0, threads, extra);
    return 0;
}

// Ray-level known answers: camera rays through jittered pixel positions plus one random
// secondary ray from each camera hit.  Records BVH::intersect's result and the number of
// AABB / triangle tests it made (reference traversal order), and the light-mixture pdf.
static int mode_rays(int argc, char **argv) {
    if (argc < 7) throw std::runtime_error("rays <gltf> W H n out.rtd");
    int W = atoi(argv[3]), H = atoi(argv[4]), n = atoi(argv[5]);
    Scene s = parse_scene_gltf(argv[2], W, H, 1);
    std::mt19937_64 g(20261015);
    std::uniform_real_distribution<float> U01(0.f, 1.f);
    std::vector<float> org, dir, t, uv, nrm;
    std::vector<int32_t> hit, inside;
    std::vector<int64_t> obj;
    std::vector<uint64_t> naabb, ntri;
    std::vector<float> lpdf;
    std::vector<uint64_t> nlaabb, nltri;
    bool has_lights = false;
    for (auto &p : s.objects) has_lights |= p.emissive();
    std::unique_ptr<rng::ManyLightsDistribution> ml;
    if (has_lights) ml = std::make_unique<rng::ManyLightsDistribution>(s.objects);
    // records the ray exactly as handed to Ray::Ray (origin, un-normalised direction)
    auto record = [&](vector3f o, vector3f dd) {
        Ray r(o, dd);
        reset_counters();
        t_mode = 0;
        Intersection it = s.bvh.intersect(s.objects, r);
        Counters c = total_counters();
        for (int k = 0; k < 3; ++k) { org.push_back(o[k]); dir.push_back(dd[k]); }
        hit.push_back(it.successful ? 1 : 0);
        obj.push_back(it.successful ? (int64_t)it.object_id : -1);
        t.push_back(it.successful ? it.distance : 0.f);
        uv.push_back(it.successful ? it.local_coords.x : 0.f);
        uv.push_back(it.successful ? it.local_coords.y : 0.f);
        for (int k = 0; k < 3; ++k) nrm.push_back(it.successful ? it.normal[k] : 0.f);
        inside.push_back(it.successful && it.inside ? 1 : 0);
        naabb.push_back(c.aabb);
        ntri.push_back(c.tri);
        reset_counters();
        float lp = ml ? ml->pdf(r.origin, r.direction) : 0.f;
        Counters c2 = total_counters();
        lpdf.push_back(lp);
        nlaabb.push_back(c2.laabb);
        nltri.push_back(c2.ltri);
        return it;
    };
    for (int k = 0; k < n; ++k) {
        // camera-like ray: same construction as Camera::cast_in_pixel (camera.cpp:49-62)
        vector2f tt{(U01(g) * 2.f - 1.f) * std::tan(s.camera->get_fov().x / 2),
                    (U01(g) * 2.f - 1.f) * std::tan(s.camera->get_fov().y / 2)};
        vector3f d0{};
        d0 = d0 + tt.x * s.camera->get_axis(0);
        d0 = d0 + tt.y * s.camera->get_axis(1);
        d0 = d0 + 1.f * s.camera->get_axis(2);
        vector3f o0 = s.camera->get_position();
        Intersection it = record(o0, d0);
        if (it.successful) {
            Ray r(o0, d0);
            vector3f pos = r.origin + r.direction * it.distance;
            vector3f d{U01(g) * 2.f - 1.f, U01(g) * 2.f - 1.f, U01(g) * 2.f - 1.f};
            record(pos + d * 1e-4f, d);
        }
    }
    RtDump d(argv[6]);
    uint64_t m = hit.size();
    d.put("origin", org, {m, 3});
    d.put("direction", dir, {m, 3});
    d.put("hit", hit);
    d.put("object_id", obj);
    d.put("t", t);
    d.put("uv", uv, {m, 2});
    d.put("normal", nrm, {m, 3});
    d.put("inside", inside);
    d.put("n_aabb", naabb);
    d.put("n_tri", ntri);
    d.put("light_pdf", lpdf);
    d.put("n_light_aabb", nlaabb);
    d.put("n_light_tri", nltri);
    d.close();
    std::printf("{\"mode\": \"rays\", \"rays\": %llu}\n", (unsigned long long)m);
    return 0;
}

static void dump_prims(RtDump &d, const std::string &pre, const std::vector<Primitive> &objs) {
    std::vector<float> pos, nrm, tan, tc, gn, area, box;
    std::vector<int32_t> mesh;
    for (auto &p : objs) {
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) { pos.push_back(p.position[v][k]); nrm.push_back(p.normal[v][k]); }
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 4; ++k) tan.push_back(p.tangent[v][k]);
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 2; ++k) tc.push_back(p.texcoord[v][k]);
        vector3f g = p.get_geometric_normal();
        for (int k = 0; k < 3; ++k) gn.push_back(g[k]);
        area.push_back(p.cache.triangle_area);
        AABB b = p.aabb();
        for (int k = 0; k < 3; ++k) box.push_back(b.min[k]);
        for (int k = 0; k < 3; ++k) box.push_back(b.max[k]);
        mesh.push_back(p.mesh_id);
    }
    uint64_t n = objs.size();
    d.put(pre + "position", pos, {n, 3, 3});
    d.put(pre + "normal", nrm, {n, 3, 3});
    d.put(pre + "tangent", tan, {n, 3, 4});
    d.put(pre + "texcoord", tc, {n, 3, 2});
    d.put(pre + "geo_normal", gn, {n, 3});
    d.put(pre + "area", area);
    d.put(pre + "aabb", box, {n, 6});
    d.put(pre + "mesh_id", mesh);
}

static void dump_nodes(RtDump &d, const std::string &pre, const BVH &b) {
    std::vector<float> box;
    std::vector<uint64_t> meta;
    for (auto &n : b.nodes) {
        for (int k = 0; k < 3; ++k) box.push_back(n.aabb.min[k]);
        for (int k = 0; k < 3; ++k) box.push_back(n.aabb.max[k]);
        meta.push_back(n.left);
        meta.push_back(n.right);
        meta.push_back(n.split_dim);
        meta.push_back(n.first_primitive_id);
        meta.push_back(n.primitive_count);
    }
    uint64_t n = b.nodes.size();
    d.put(pre + "aabb", box, {n, 6});
    d.put(pre + "meta", meta, {n, 5});
}

static int mode_dump(int argc, char **argv) {
    if (argc < 6) throw std::runtime_error("dump <gltf> W H out.rtd");
    int W = atoi(argv[3]), H = atoi(argv[4]);
    Scene s = parse_scene_gltf(argv[2], W, H, 1);
    // get_geometric_normal() fills the cache the way Primitive::intersect does (primitive.cpp:77-84)
    RtDump d(argv[5]);
    dump_prims(d, "obj_", s.objects);
    dump_nodes(d, "node_", s.bvh);
    // light list exactly as rng::ManyLightsDistribution builds it (random.cpp:156-168)
    std::vector<Primitive> lights;
    for (auto &p : s.objects)
        if (p.emissive()) lights.push_back(p);
    BVH lb;
    if (!lights.empty()) lb.buildBVH(lights);
    dump_prims(d, "light_", lights);
    dump_nodes(d, "lnode_", lb);
    std::vector<float> mf;
    std::vector<int32_t> mi;
    std::vector<double> mt;
    for (auto &m : s.meshes) {
        const Material &a = m.material;
        float v[] = {a.ior, a.alpha, a.base_color.x, a.base_color.y, a.base_color.z, a.emission.x, a.emission.y,
                     a.emission.z, a.metallic, a.roughness2};
        mf.insert(mf.end(), v, v + 10);
        int iv[] = {a.base_color_i, a.normal_i, a.metallic_roughness_i, a.emission_i};
        mi.insert(mi.end(), iv, iv + 4);
        mt.insert(mt.end(), m.normal_transform.data, m.normal_transform.data + 16);
    }
    uint64_t nm = s.meshes.size();
    d.put("mesh_f", mf, {nm, 10});
    d.put("mesh_tex", mi, {nm, 4});
    d.put("mesh_normal_transform", mt, {nm, 16});
    std::vector<float> cam;
    vector3f cp = s.camera->get_position();
    for (int k = 0; k < 3; ++k) cam.push_back(cp[k]);
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 3; ++k) cam.push_back(s.camera->get_axis(a)[k]);
    cam.push_back(s.camera->get_fov().x);
    cam.push_back(s.camera->get_fov().y);
    d.put("camera", cam);
    std::vector<int32_t> tdim;
    std::vector<uint64_t> thash;
    for (auto &t : s.textures) {
        tdim.push_back(t.width);
        tdim.push_back(t.height);
        tdim.push_back(t.channels);
        uint64_t h = 1469598103934665603ull;  // FNV-1a over the decoded texels
        for (uint8_t b : t.data) h = (h ^ b) * 1099511628211ull;
        thash.push_back(h);
    }
    d.put("tex_dim", tdim, {(uint64_t)s.textures.size(), 3});
    d.put("tex_fnv1a", thash);
    d.scalar<int32_t>("ray_depth", s.ray_depth);
    d.close();
    std::printf("{\"mode\": \"dump\", \"objects\": %zu, \"nodes\": %zu, \"lights\": %zu, \"light_nodes\": %zu}\n",
                s.objects.size(), s.bvh.nodes.size(), lights.size(), lb.nodes.size());
    return 0;
}

// Sampler known answers: SceneDistribution::sample then ::pdf from random shading frames,
// each with a fresh Engine(seed) and reset normal cache; records the next engine output so
// the number of draws consumed is pinned too.  Also raw RNG sequences.
static int mode_samplers(int argc, char **argv) {
    if (argc < 7) throw std::runtime_error("samplers <gltf> W H n out.rtd");
    int W = atoi(argv[3]), H = atoi(argv[4]), n = atoi(argv[5]);
    Scene s = parse_scene_gltf(argv[2], W, H, 1);
    rng::SceneDistribution sd(s.objects);
    std::mt19937_64 g(777);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> in, outd, outp;
    std::vector<uint32_t> seeds, next;
    for (int k = 0; k < n; ++k) {
        vector3f point{U(g) * 3.f, U(g) * 3.f, U(g) * 3.f};
        vector3f nn = normal(vector3f{U(g), U(g), U(g)});
        vector3f eye = normal(vector3f{U(g), U(g), U(g)});
        if (dot(eye, nn) < 0) eye = -eye;
        float r2 = std::max(0.03f, U(g) * U(g));
        uint32_t seed = (uint32_t)(g() % 2147483646u) + 1u;
        rng::normDist.reset();
        Engine e(seed);
        vector3f d = sd.sample(point, nn, eye, r2, e);
        float pdf = sd.pdf(point, nn, eye, r2, d);
        float v[] = {point.x, point.y, point.z, nn.x, nn.y, nn.z, eye.x, eye.y, eye.z, r2};
        in.insert(in.end(), v, v + 10);
        outd.push_back(d.x); outd.push_back(d.y); outd.push_back(d.z);
        outp.push_back(pdf);
        seeds.push_back(seed);
        next.push_back((uint32_t)e());
    }
    // raw sequences: engine, uniform(-1,1), normal(0,1) for a few seeds
    std::vector<uint32_t> raw;
    std::vector<float> uni, nor;
    for (uint32_t seed : {1u, 2u, 12345u, 2147483646u, 65536u}) {
        Engine e(seed);
        for (int k = 0; k < 8; ++k) raw.push_back((uint32_t)e());
        Engine e2(seed);
        for (int k = 0; k < 8; ++k) uni.push_back(rng::uniform::sample(e2));
        Engine e3(seed);
        rng::normDist.reset();
        for (int k = 0; k < 8; ++k) nor.push_back(rng::normal::sample(e3));
    }
    RtDump d(argv[6]);
    uint64_t m = seeds.size();
    d.put("frame", in, {m, 10});
    d.put("seed", seeds);
    d.put("dir", outd, {m, 3});
    d.put("pdf", outp);
    d.put("next", next);
    d.put("raw_engine", raw, {5, 8});
    d.put("raw_uniform", uni, {5, 8});
    d.put("raw_normal", nor, {5, 8});
    d.close();
    std::printf("{\"mode\": \"samplers\", \"n\": %llu}\n", (unsigned long long)m);
    return 0;
}

// finish <out.rtd> <out.ppm> W H spp: the frame finish of Scene::render (scene.cpp:54-64)
// and Scene::draw_into (Canvas::write_to, canvas.h:76-89) on deterministic synthetic pixel
// sums spanning zero, tiny, mid-range, saturating, negative and NaN/inf values.
static int mode_finish(int argc, char **argv) {
    if (argc < 7) throw std::runtime_error("finish out.rtd out.ppm W H spp");
    const int W = std::atoi(argv[4]), H = std::atoi(argv[5]), spp = std::atoi(argv[6]);
    std::vector<float> sums((size_t)W * H * 3);
    uint32_t x = 12345u;
    for (size_t k = 0; k < sums.size(); ++k) {
        x = x * 1664525u + 1013904223u;
        const float u = (float)(x >> 8) / 16777216.f;
        const int kind = (int)(k % 11);
        float v;
        switch (kind) {
            case 0: v = 0.f; break;
            case 1: v = u * 1e-6f; break;
            case 2: v = u * (float)spp * 4.f; break;
            case 3: v = -u; break;
            case 4: v = (k % 97 == 4) ? NAN : u * (float)spp; break;
            case 5: v = (k % 89 == 5) ? INFINITY : u * (float)spp * 0.25f; break;
            default: v = u * u * (float)spp * 1.5f; break;
        }
        sums[k] = v;
    }
    finish_to_ppm(sums, W, H, spp, argv[3]);
    RtDump d(argv[2]);
    d.put("sums", sums, {(uint64_t)H, (uint64_t)W, 3});
    d.put("spp", std::vector<int32_t>{spp});
    d.close();
    std::printf("{\"mode\": \"finish\", \"width\": %d, \"height\": %d, \"spp\": %d}\n", W, H, spp);
    return 0;
}

int main(int argc, char **argv) {
    try {
        if (argc < 2) throw std::runtime_error("usage: ref_harness sums|time|rays|dump|samplers|finish|pixels ...");
        std::string m = argv[1];
        if (m == "sums") return mode_sums(argc, argv);
        if (m == "time") return mode_time(argc, argv);
        if (m == "rays") return mode_rays(argc, argv);
        if (m == "dump") return mode_dump(argc, argv);
        if (m == "samplers") return mode_samplers(argc, argv);
        if (m == "finish") return mode_finish(argc, argv);
        if (m == "pixels") return mode_pixels(argc, argv);
        throw std::runtime_error("unknown mode " + m);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "ref_harness: %s\n", e.what());
        return 1;
    }
}
