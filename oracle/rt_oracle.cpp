// rt_oracle.cpp — CPU restatement of the reference's per-pixel sample loop.
// TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg as the checker / CPU baseline, never by the product path.
//
// Input: a flattened scene (include/rt_hw.h rt_scene_view, the same arrays the kernels
// read).  The code deliberately follows the reference's own structure — recursive
// BVH::intersectHelper, recursive Scene::intersect, operator-style vector math, the real
// libstdc++ <random> engines and glibc logf/pow/powf — so that it is an independent
// second implementation of the GPU kernels (raytracing-hw_amd/csrc/rt_path.h), not a copy.
// Citations are to /root/reference/src.
//
// Parity convention: per pixel, minstd_rand seeded with j*W+i (pixel 0
// -> Engine(1)) and a fresh normal_distribution (the reference's shared cache reset).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>
#include <omp.h>

#include "rt_hw.h"

namespace {

struct Vec3 {
    float x, y, z;
    float &operator[](int i) { return *(&x + i); }
    float operator[](int i) const { return *(&x + i); }
};
struct Vec2 { float x, y; };
struct Vec4 { float x, y, z, w; };

// vector.h operators, same evaluation order
inline Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(Vec3 a) { return {-a.x, -a.y, -a.z}; }
inline Vec3 operator-(Vec3 a, Vec3 b) { return a + (-b); }
inline Vec3 operator*(Vec3 v, float t) { return {v.x * t, v.y * t, v.z * t}; }
inline Vec3 operator*(float t, Vec3 v) { return v * t; }
inline Vec3 operator*(Vec3 a, Vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline Vec3 &operator+=(Vec3 &a, Vec3 b) { a = a + b; return a; }
inline float dot(Vec3 a, Vec3 b) {
    float s = 0.f;
    for (int i = 0; i < 3; ++i) s += a[i] * b[i];
    return s;
}
inline Vec3 cross(Vec3 a, Vec3 b) { return {a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]}; }
inline float length(Vec3 v) {
    float m = 0.f;
    for (int i = 0; i < 3; ++i) m += v[i] * v[i];
    return std::sqrt(m);
}
inline Vec3 normal(Vec3 v) {
    float m = 1.f / length(v);
    return {v.x * m, v.y * m, v.z * m};
}
inline Vec4 normal4(Vec4 v) {
    float m = 0.f;
    m += v.x * v.x; m += v.y * v.y; m += v.z * v.z; m += v.w * v.w;
    m = 1.f / std::sqrt(m);
    return {v.x * m, v.y * m, v.z * m, v.w * m};
}
inline Vec3 rotate(Vec3 v, Vec4 q) {
    Vec3 u{q.x, q.y, q.z};
    float s = q.w;
    return 2.f * dot(u, v) * u + (s * s - dot(u, u)) * v + 2.f * s * cross(u, v);
}
inline Vec4 quat_from_two_vectors(Vec3 u, Vec3 v) {
    Vec3 w = cross(u, v);
    return normal4({w.x, w.y, w.z, 1.f + dot(u, v)});
}
template <class T> inline T smax(T a, T b) { return std::max(a, b); }
template <class T> inline T smin(T a, T b) { return std::min(a, b); }

typedef std::minstd_rand Engine;
typedef std::uniform_real_distribution<float> UniformF;

struct Ray {
    Vec3 origin, direction, inv_direction;
    int power = 1;
    Ray(Vec3 p, Vec3 d) : origin(p), direction(normal(d)) {
        for (int i = 0; i < 3; ++i) inv_direction[i] = 1.f / direction[i];
    }
};

struct Hit {
    bool ok = false;
    float distance = 0.f;
    Vec3 normal{0, 0, 0};
    Vec2 local{0, 0};
    Vec3 color{0, 0, 0};
    bool inside = false;
    int64_t id = -1;
};

struct Counts {
    uint64_t rays = 0, aabb = 0, tri = 0, lq = 0, laabb = 0, ltri = 0;
};

constexpr float kPiF = 3.14159265358979323846f;      // M_PIf32
constexpr float kInvPiF = 0.318309886183790671538f;  // M_1_PIf32

uint32_t ubits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// Philox4x32-10: 10 rounds of two 32x32->64 multiplies (M0 = 0xD2511F53 on word 0,
// M1 = 0xCD9E8D57 on word 2), output {hi1^c1^k0, lo1, hi0^c3^k1, lo0}; the key is bumped by
// the Weyl constants (0x9E3779B9, 0xBB67AE85) before every round but the first.
void philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]}, k[2] = {key[0], key[1]};
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k[0] += 0x9E3779B9u;
            k[1] += 0xBB67AE85u;
        }
        const uint64_t a = (uint64_t)0xD2511F53u * c[0], b = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(b >> 32) ^ c[1] ^ k[0], n2 = (uint32_t)(a >> 32) ^ c[3] ^ k[1];
        c[0] = n0;
        c[1] = (uint32_t)b;
        c[2] = n2;
        c[3] = (uint32_t)a;
    }
    for (int i = 0; i < 4; ++i) out[i] = c[i];
}
// Fast-mode seed of sample s of pixel pix: Philox word 0 (counter {s,0,0,0}, key {pix,
// 0x5eed2026}), as minstd_rand's constructor takes it (it reduces mod 2^31-1, 0 -> 1).
uint32_t philox_seed(uint32_t pix, uint32_t s) {
    const uint32_t ctr[4] = {s, 0u, 0u, 0u}, key[2] = {pix, 0x5eed2026u};
    uint32_t o[4];
    philox4x32_10(ctr, key, o);
    return o[0];
}

class Oracle {
public:
    explicit Oracle(const rt_scene_view &v) : S(v) {}

    const rt_scene_view &S;
    static thread_local Counts cnt;
    static thread_local std::normal_distribution<float> *normDist;

    // ------------------------------------------------------------ geometry
    Vec3 tri_v(const float *base, int k) const { return {base[k], base[k + 1], base[k + 2]}; }

    // AABB::intersect (primitive.cpp:146-208)
    bool box_hit(const float *nd, const Ray &r, float &dist) const {
        const float *mn = nd, *mx = nd + 3;
        bool inside = true;
        int quadrant[3];
        float cand[3] = {0, 0, 0};
        for (int i = 0; i < 3; ++i) {
            if (r.origin[i] < mn[i]) { quadrant[i] = 0; cand[i] = mn[i]; inside = false; }
            else if (r.origin[i] > mx[i]) { quadrant[i] = 2; cand[i] = mx[i]; inside = false; }
            else quadrant[i] = 1;
        }
        if (inside) { dist = 0.f; return true; }
        float maxT[3];
        for (int i = 0; i < 3; i++)
            maxT[i] = (quadrant[i] != 1 && r.direction[i] != 0.f) ? (cand[i] - r.origin[i]) * r.inv_direction[i] : -1.f;
        int which = 0;
        for (int i = 1; i < 3; ++i)
            if (maxT[which] < maxT[i]) which = i;
        if (maxT[which] < 0.f) return false;
        Vec3 coord{};
        for (int i = 0; i < 3; i++) {
            if (which != i) {
                coord[i] = r.origin[i] + maxT[which] * r.direction[i];
                if (coord[i] < mn[i] || coord[i] > mx[i]) return false;
            } else {
                coord[i] = cand[i];
            }
        }
        dist = length(coord - r.origin);
        return true;
    }

    // Primitive::intersect (primitive.cpp:17-57) on a 12/16-float triangle record
    Hit tri_hit(const float *t, const Ray &ray) const {
        Vec3 o = tri_v(t, 0), U = tri_v(t, 3), V = tri_v(t, 6);
        Vec3 p = cross(ray.direction, V);
        float det = dot(U, p);
        if (-1e-6 < det && det < 1e-6) return {};
        float inv_det = 1.f / det;
        Vec3 s = ray.origin - o;
        float u = inv_det * dot(s, p);
        if (u < 0 || u > 1) return {};
        Vec3 q = cross(s, U);
        float v = inv_det * dot(ray.direction, q);
        if (v < 0 || u + v > 1) return {};
        float dist = inv_det * dot(V, q);
        if (dist < 0.f) return {};
        Hit h;
        h.ok = true;
        h.local = {u, v};
        h.normal = tri_v(t, 9);
        h.distance = dist;
        if (dot(ray.direction, h.normal) > 0) { h.inside = true; h.normal = -h.normal; }
        return h;
    }

    static bool is_leaf(const float *nd) { return (ubits(nd[7]) & 3u) == 3u; }
    static uint32_t field_a(const float *nd) { return ubits(nd[6]); }
    static uint32_t field_b(const float *nd) { return ubits(nd[7]); }

    // BVH::intersectHelper (bvh.cpp:177-237), recursive with the per-call local best
    Hit helper(const Ray &r, uint32_t id) const {
        const float *nd = S.node + 8 * id;
        Hit best;
        best.distance = 1e9f;
        if (!is_leaf(nd)) {
            uint32_t left = field_a(nd), right = left + 1, split = field_b(nd);
            uint32_t first = r.direction[split] > 0 ? left : right, second = first == left ? right : left;
            float e;
            cnt.aabb++;
            if (box_hit(S.node + 8 * first, r, e)) {
                Hit a = helper(r, first);
                if (a.ok && a.distance < best.distance) best = a;
            }
            cnt.aabb++;
            if (box_hit(S.node + 8 * second, r, e)) {
                if (!(e > best.distance)) {
                    Hit a = helper(r, second);
                    if (a.ok && a.distance < best.distance) best = a;
                }
            }
            return best;
        }
        uint32_t first = field_a(nd), count = field_b(nd) >> 2;
        for (uint32_t i = first; i < first + count; ++i) {
            cnt.tri++;
            Hit a = tri_hit(S.tri + 12 * i, r);
            if (a.ok && a.distance < best.distance) {
                best = a;
                best.id = i;
            }
        }
        return best;
    }
    // BVH::intersect (bvh.cpp:239-243)
    Hit closest(const Ray &r) const {
        cnt.rays++;
        float e;
        cnt.aabb++;
        if (!box_hit(S.node, r, e)) return {};
        return helper(r, 0);
    }
    // BVH::intersectAllHelper (bvh.cpp:245-273) over the light BVH
    void all_hits(const Ray &r, uint32_t id, std::vector<Hit> &out) const {
        const float *nd = S.light_node + 8 * id;
        if (!is_leaf(nd)) {
            uint32_t left = field_a(nd);
            float e;
            cnt.laabb++;
            if (box_hit(S.light_node + 8 * left, r, e)) all_hits(r, left, out);
            cnt.laabb++;
            if (box_hit(S.light_node + 8 * (left + 1), r, e)) all_hits(r, left + 1, out);
            return;
        }
        uint32_t first = field_a(nd), count = field_b(nd) >> 2;
        for (uint32_t i = first; i < first + count; ++i) {
            cnt.ltri++;
            Hit a = tri_hit(S.light + 16 * i, r);
            if (a.ok) {
                a.id = i;
                out.push_back(a);
            }
        }
    }

    // ------------------------------------------------------------ materials / textures
    const float *mesh_f(int m) const { return S.mesh_f + 12 * m; }
    int mesh_tex(int m, int k) const { return S.mesh_tex[4 * m + k]; }
    int mesh_of(int64_t id) const { int m; std::memcpy(&m, S.tri_attr + 16 * id + 15, 4); return m; }

    // Texture::interpolate_sample (primitive.h:182-215)
    Vec4 tex_sample(int t, Vec2 p, bool srgb) const {
        const uint32_t *ti = S.tex_info + 4 * t;
        int W = (int)ti[1], H = (int)ti[2], C = (int)ti[3];
        const uint8_t *data = S.texels + 4ull * ti[0];
        p.x -= std::floor(p.x);
        p.y -= std::floor(p.y);
        p.x *= (float)W;
        p.y *= (float)H;
        int px = (int)std::floor(p.x), py = (int)std::floor(p.y);
        float dx = p.x - std::floor(p.x), dy = p.y - std::floor(p.y);
        const uint8_t *ptr[4];
        for (int ddy = 0; ddy < 2; ++ddy)
            for (int ddx = 0; ddx < 2; ++ddx) {
                int x = (px + ddx) % W, y = (py + ddy) % H;
                ptr[ddx * 2 + ddy] = data + (size_t)(y * W + x) * C;
            }
        float res[4] = {0, 0, 0, 0};
        for (int c = 0; c < C; ++c) {
            float v[4];
            for (int k = 0; k < 4; ++k) {
                v[k] = (float)(int)ptr[k][c] / 255.f;
                if (srgb) v[k] = std::pow(v[k], 2.2f);
            }
            res[c] = v[0] * (1 - dx) * (1 - dy) + v[1] * (1 - dx) * dy + v[2] * dx * (1 - dy) + v[3] * dx * dy;
        }
        return {res[0], res[1], res[2], res[3]};
    }
    Vec2 texcoord(int64_t id, Vec2 l) const {
        const float *a = S.tri_attr + 16 * id + 9;
        float w = 1 - l.x - l.y;
        return {a[0] * w + a[2] * l.x + a[4] * l.y, a[1] * w + a[3] * l.x + a[5] * l.y};
    }
    // Primitive::get_shading_normal (primitive.cpp:86-105)
    Vec3 shading_normal(int64_t id, Vec2 l) const {
        const float *a = S.tri_attr + 16 * id;
        float w = 1 - l.x - l.y;
        Vec3 lz = normal(w * tri_v(a, 0) + l.x * tri_v(a, 3) + l.y * tri_v(a, 6));
        int m = mesh_of(id);
        if (mesh_tex(m, 1) == -1) return lz;
        const float *tg = S.tri_tan + 12 * id;
        Vec3 t0 = tri_v(tg, 0), t1 = tri_v(tg, 4), t2 = tri_v(tg, 8);
        Vec3 tv = normal(w * t0 + l.x * t1 + l.y * t2);
        const double *M = S.mesh_normal_transform + 16 * m;
        float res[4] = {0, 0, 0, 0}, in[4] = {tv.x, tv.y, tv.z, 0.f};
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) res[i] += M[4 * j + i] * in[j];
        Vec3 lx = normal(Vec3{res[0], res[1], res[2]});
        Vec3 ly = cross(lz, lx) * tg[3];
        Vec4 s = tex_sample(mesh_tex(m, 1), texcoord(id, l), false);
        Vec3 ln = Vec3{s.x + -0.5f, s.y + -0.5f, s.z + -0.5f} * 2.f;
        return normal(lx * ln.x + ly * ln.y + lz * ln.z);
    }
    Vec3 color(int64_t id, Vec2 l) const {  // get_color (primitive.cpp:111-119)
        int m = mesh_of(id);
        Vec3 f{mesh_f(m)[0], mesh_f(m)[1], mesh_f(m)[2]};
        if (mesh_tex(m, 0) == -1) return f;
        Vec4 c = tex_sample(mesh_tex(m, 0), texcoord(id, l), true);
        return Vec3{c.x, c.y, c.z} * f;
    }
    Vec3 emission(int64_t id, Vec2 l) const {  // get_emission (primitive.cpp:121-129)
        int m = mesh_of(id);
        Vec3 f{mesh_f(m)[3], mesh_f(m)[4], mesh_f(m)[5]};
        if (mesh_tex(m, 3) == -1) return f;
        Vec4 c = tex_sample(mesh_tex(m, 3), texcoord(id, l), true);
        return Vec3{c.x, c.y, c.z} * f;
    }
    void metallic_roughness(int64_t id, Vec2 l, float &r2, float &metal) const {  // primitive.cpp:131-140
        int m = mesh_of(id);
        if (mesh_tex(m, 2) == -1) { r2 = mesh_f(m)[7]; metal = mesh_f(m)[6]; return; }
        Vec4 t = tex_sample(mesh_tex(m, 2), texcoord(id, l), false);
        float rr = t.y * t.y;
        r2 = rr * mesh_f(m)[7];
        metal = t.z * mesh_f(m)[6];
    }

    // ------------------------------------------------------------ sampling (random.cpp)
    float uni(Engine &e) const { static thread_local UniformF d(-1.f, 1.f); return d(e); }
    Vec3 sphere(Engine &e) const { Vec3 a{(*normDist)(e), (*normDist)(e), (*normDist)(e)}; return normal(a); }
    Vec3 cosine_sample(Vec3 n, Engine &e) const {
        Vec3 d{};
        do { d = sphere(e) + n; } while (length(d) < 1e-12);
        return normal(d);
    }
    float cosine_pdf(Vec3 n, Vec3 d) const { return smax(0.f, dot(d, n)) * kInvPiF; }
    Vec3 vndf_sample(Vec3 n, Vec3 eye, float alpha, Engine &e) const {
        Vec3 Z{0.f, 0.f, 1.f};
        Vec4 rot = quat_from_two_vectors(n, Z);
        Vec3 Ve = rotate(eye, rot);
        Vec3 Vh = normal(Vec3{Ve.x * alpha, Ve.y * alpha, Ve.z});
        float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
        Vec3 T1 = lensq > 0 ? Vec3{-Vh.y, Vh.x, 0} * (1.f / std::sqrt(lensq)) : Vec3{1, 0, 0};
        Vec3 T2 = cross(Vh, T1);
        Vec2 t;
        do { t.x = uni(e); t.y = uni(e); } while (t.x * t.x + t.y * t.y > 1.f);
        float s = 0.5f + 0.5f * Vh.z;
        t.y = (1.f - s) * std::sqrt(1.f - t.x * t.x) + s * t.y;
        Vec3 Nh = t.x * T1 + t.y * T2 + std::sqrt(smax(0.f, 1.f - t.x * t.x - t.y * t.y)) * Vh;
        Vec3 Ne = normal(Vec3{alpha * Nh.x, alpha * Nh.y, smax(0.f, Nh.z)});
        Ne = rotate(Ne, Vec4{-rot.x, -rot.y, -rot.z, rot.w});
        return normal(2 * Ne * dot(Ne, eye) - eye);
    }
    float vndf_pdf(Vec3 n, Vec3 eye, float alpha, Vec3 dir) const {
        Vec3 Z{0.f, 0.f, 1.f};
        Vec4 rot = quat_from_two_vectors(n, Z);
        Vec3 sn = normal(dir + eye);
        Vec3 V = rotate(eye, rot), Ni = rotate(sn, rot);
        if (dot(V, Ni) < 0.f) return 0.f;
        float alpha2 = alpha * alpha;
        float invD = kPiF * alpha * alpha * std::pow(Ni.x * Ni.x / alpha2 + Ni.y * Ni.y / alpha2 + Ni.z * Ni.z, 2);
        float invG1 = 0.5f + 0.5f * std::sqrt(1.f + (alpha2 * V.x * V.x + alpha2 * V.y * V.y) / (V.z * V.z));
        return 1.f / (4.f * invD * invG1 * dot(V, Z));
    }
    Vec3 light_sample(Vec3 point, Engine &e) const {
        int n = (int)S.n_lights;
        int k = std::floor((uni(e) + 1.f) * 0.5f * (float)n);
        if (k == n) k -= 1;
        const float *L = S.light + 16 * k;
        float u = (uni(e) + 1.f) / 2, v = (uni(e) + 1.f) / 2;
        if (u + v > 1) { u = 1 - u; v = 1 - v; }
        Vec3 res = tri_v(L, 0) + u * tri_v(L, 3) + v * tri_v(L, 6);
        return normal(res - point);
    }
    float light_pdf(Vec3 point, Vec3 direction) const {
        cnt.lq++;
        std::vector<Hit> hits;
        all_hits(Ray(point, direction), 0, hits);
        float prob = 0.f;
        for (auto &h : hits) {
            float probability = 1.f / S.light[16 * h.id + 12];
            prob += std::abs(probability * (h.distance * h.distance) / dot(h.normal, direction));
        }
        return prob / (float)S.n_lights;
    }
    Vec3 sample(Vec3 point, Vec3 n, Vec3 eye, float r2, Engine &e) const {  // random.cpp:194-208
        float s = (uni(e) + 1.f) * 3 * 0.5f;
        if (!S.n_lights) s /= 1.5f;
        if (s <= 1.f) return cosine_sample(n, e);
        if (s <= 2.f) return vndf_sample(n, eye, r2, e);
        return light_sample(point, e);
    }
    float pdf(Vec3 point, Vec3 n, Vec3 eye, float r2, Vec3 d) const {  // random.cpp:210-218
        if (!S.n_lights) return (cosine_pdf(n, d) + vndf_pdf(n, eye, r2, d)) / 2;
        return (cosine_pdf(n, d) + light_pdf(point, d) + vndf_pdf(n, eye, r2, d)) / 3;
    }

    // ------------------------------------------------------------ Scene::intersect (scene.cpp:71-157)
    Hit shade(Ray r, Engine &rng) const {
        if (r.power <= 0) return {};
        r.power -= 1;
        Hit it;
        it.distance = S.max_distance;
        Hit h = closest(r);
        if (h.ok && h.distance < it.distance) {
            it = h;
            it.color = emission(h.id, h.local);
        }
        if (!it.ok) return it;
        Vec3 pos = r.origin + r.direction * it.distance;
        Vec3 N = shading_normal(it.id, it.local);
        if (it.inside) N = -N;
        float metallic, r2;
        metallic_roughness(it.id, it.local, r2, metallic);
        r2 = smax(0.03f, r2);
        Vec3 dir = sample(pos, N, -r.direction, r2, rng);
        if (dot(dir, N) <= 0.f) {
            if (dot(dir, it.normal) <= 0.f) return it;
            N = it.normal;
        }
        float p = pdf(pos, N, -r.direction, r2, dir);
        if (p <= 0.f || std::isnan(p)) return it;
        Ray child(pos + dir * 1e-4f, dir);
        child.power = r.power;
        Hit c = shade(child, rng);
        if (!c.ok) return it;
        float coeff = 1 / p;
        Vec3 half = normal(dir - r.direction);
        float alpha2 = r2 * r2;
        float smith = 0.f;
        if (!(dot(N, dir) <= 0 || dot(N, -r.direction) <= 0)) {
            float nd[2] = {std::abs(dot(N, dir)), std::abs(dot(N, -r.direction))};
            smith = 1.f;
            for (float x : nd) smith *= 2 * x / (x + std::sqrt(alpha2 + (1 - alpha2) * x * x));
        }
        float vis = smith * (1.f / (4 * std::abs(dot(N, r.direction)) * std::abs(dot(N, dir))));
        float NdotH = dot(N, half);
        float ggx = alpha2 * kInvPiF / ((NdotH * NdotH * (alpha2 - 1) + 1) * (NdotH * NdotH * (alpha2 - 1) + 1));
        float spec = ggx * vis;
        float VdotH = std::abs(dot(-r.direction, half));
        Vec3 base = color(it.id, it.local);
        Vec3 F;
        for (int i = 0; i < 3; ++i) F[i] = base[i] + (1.f - base[i]) * (float)std::pow(1.f - VdotH, 5);
        Vec3 metal = spec * F;
        Vec3 diffuse = base * kInvPiF;
        float dsc = 0.04f + (1.f - 0.04f) * (float)std::pow(1.f - VdotH, 5);
        Vec3 dielectric = diffuse * (1 - dsc) + Vec3{1.f, 1.f, 1.f} * spec * dsc;
        Vec3 material = dielectric * (1 - metallic) + metal * metallic;
        int m = mesh_of(it.id);
        it.color += c.color * coeff * material * dot(dir, N) * mesh_f(m)[8];
        return it;
    }

    // Camera::cast_in_pixel (camera.cpp:49-62) + one pixel of Scene::render (scene.cpp:33-43)
    Ray camera_ray(int px, int py, float ox, float oy) const {
        Vec3 t;
        t.x = (2.f * ((float)px + 0.5f + ox) / (float)S.width - 1) * S.tan_half_fov[0];
        t.y = -(2.f * ((float)py + 0.5f + oy) / (float)S.height - 1) * S.tan_half_fov[1];
        t.z = 1;
        Vec3 d{};
        for (int i = 0; i < 3; ++i) d = d + t[i] * Vec3{S.cam_axes[3 * i], S.cam_axes[3 * i + 1], S.cam_axes[3 * i + 2]};
        return Ray(Vec3{S.cam_pos[0], S.cam_pos[1], S.cam_pos[2]}, d);
    }
    Vec3 render_pixel(int i, int j, int spp) const {
        std::normal_distribution<float> nd(0.f, 1.f);
        normDist = &nd;
        size_t seed = (size_t)(j * S.width + i);
        Engine e(seed ? (Engine::result_type)seed : 1u);
        UniformF offset(-0.5f, 0.5f);
        Vec3 sum{0.f, 0.f, 0.f};
        for (int s = 0; s < spp; ++s) {
            float ox = offset(e);
            float oy = offset(e);
            Ray r = camera_ray(i, j, ox, oy);
            r.power = S.ray_depth;
            sum += shade(r, e).color;
        }
        normDist = nullptr;
        return sum;
    }
    // Fast mode (include/rt_hw.h RT_FLAG_FAST; not the reference's RNG convention): sample s
    // of pixel j*W+i runs minstd_rand seeded by philox_seed(j*W+i, s) with a fresh normal
    // cache; samples summed per chunk of cs in order, chunk partials summed in chunk order.
    Vec3 render_pixel_fast(int i, int j, int spp, int cs) const {
        const uint32_t pix = (uint32_t)(j * S.width + i);
        UniformF offset(-0.5f, 0.5f);
        Vec3 total{0.f, 0.f, 0.f};
        for (int c0 = 0; c0 < spp; c0 += cs) {
            Vec3 part{0.f, 0.f, 0.f};
            for (int s = c0; s < std::min(spp, c0 + cs); ++s) {
                std::normal_distribution<float> nd(0.f, 1.f);
                normDist = &nd;
                Engine e(philox_seed(pix, (uint32_t)s));
                float ox = offset(e);
                float oy = offset(e);
                Ray r = camera_ray(i, j, ox, oy);
                r.power = S.ray_depth;
                part += shade(r, e).color;
            }
            total += part;
        }
        normDist = nullptr;
        return total;
    }
};
thread_local Counts Oracle::cnt;
thread_local std::normal_distribution<float> *Oracle::normDist = nullptr;

}  // namespace

extern "C" {

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123 philox.h constants): the fast
// mode's per-sample seed source.  Pinned by Random123's known-answer vectors (test_oracle.py).
void rt_oracle_philox(const uint32_t *ctr, const uint32_t *key, uint32_t *out) {
    philox4x32_10(ctr, key, out);
}

// Fast-mode render of pixels [p0, p1) (see Oracle::render_pixel_fast); returns wall seconds.
double rt_oracle_render_fast(const rt_scene_view *view, int spp, int chunk, int64_t p0, int64_t p1, int threads,
                             float *out) {
    Oracle o(*view);
    const int W = view->width;
    auto t0 = std::chrono::steady_clock::now();
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for num_threads(nt) schedule(guided, 16)
    for (int64_t p = p0; p < p1; ++p) {
        Vec3 s = o.render_pixel_fast((int)(p % W), (int)(p / W), spp, chunk);
        out[3 * (p - p0) + 0] = s.x;
        out[3 * (p - p0) + 1] = s.y;
        out[3 * (p - p0) + 2] = s.z;
    }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Renders pixels [p0, p1) of the row-major W*H frame (float RGB sums) with `threads`
// OpenMP threads (0 = all).  counters (may be NULL): rays, aabb, tri, light queries,
// light aabb, light tri.  Returns wall seconds.
double rt_oracle_render(const rt_scene_view *view, int spp, int64_t p0, int64_t p1, int threads, float *out,
                        uint64_t *counters) {
    Oracle o(*view);
    const int W = view->width;
    uint64_t c[6] = {0, 0, 0, 0, 0, 0};
    auto t0 = std::chrono::steady_clock::now();
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel num_threads(nt)
    {
        Oracle::cnt = Counts();
#pragma omp for schedule(guided, 16)
        for (int64_t p = p0; p < p1; ++p) {
            Vec3 s = o.render_pixel((int)(p % W), (int)(p / W), spp);
            out[3 * (p - p0) + 0] = s.x;
            out[3 * (p - p0) + 1] = s.y;
            out[3 * (p - p0) + 2] = s.z;
        }
#pragma omp critical
        {
            c[0] += Oracle::cnt.rays; c[1] += Oracle::cnt.aabb; c[2] += Oracle::cnt.tri;
            c[3] += Oracle::cnt.lq; c[4] += Oracle::cnt.laabb; c[5] += Oracle::cnt.ltri;
        }
    }
    if (counters) std::memcpy(counters, c, sizeof c);
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Closest-hit + light-pdf known answers for explicit rays (origins/dirs are normalised
// by the Ray constructor as in the reference).  out_f: t, u, v, light_pdf per ray;
// out_i: hit, object id, n_aabb, n_tri, n_light_aabb, n_light_tri per ray.
void rt_oracle_rays(const rt_scene_view *view, int64_t n, const float *org, const float *dir, float *out_f,
                    int64_t *out_i) {
    Oracle o(*view);
    for (int64_t k = 0; k < n; ++k) {
        Ray r(Vec3{org[3 * k], org[3 * k + 1], org[3 * k + 2]}, Vec3{dir[3 * k], dir[3 * k + 1], dir[3 * k + 2]});
        Oracle::cnt = Counts();
        Hit h = o.closest(r);
        Counts c1 = Oracle::cnt;
        Oracle::cnt = Counts();
        float lp = view->n_lights ? o.light_pdf(r.origin, r.direction) : 0.f;
        Counts c2 = Oracle::cnt;
        out_f[4 * k + 0] = h.ok ? h.distance : 0.f;
        out_f[4 * k + 1] = h.ok ? h.local.x : 0.f;
        out_f[4 * k + 2] = h.ok ? h.local.y : 0.f;
        out_f[4 * k + 3] = lp;
        out_i[6 * k + 0] = h.ok;
        out_i[6 * k + 1] = h.ok ? h.id : -1;
        out_i[6 * k + 2] = (int64_t)c1.aabb;
        out_i[6 * k + 3] = (int64_t)c1.tri;
        out_i[6 * k + 4] = (int64_t)c2.laabb;
        out_i[6 * k + 5] = (int64_t)c2.ltri;
    }
}

}  // extern "C"
