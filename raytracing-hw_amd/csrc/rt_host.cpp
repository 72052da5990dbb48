// rt_host.cpp — host side of the MI355X path-tracing core: glTF ingest, the reference-exact
// BVH build, scene flattening into the HBM layout, frame finish and PPM output.
//
// Every float/double expression below restates the reference op for op (g++ with
// -ffp-contract=off, like the reference binary which contains no FMA), because the GPU
// kernels must see the very same triangles, normals, camera and tree to reproduce the
// reference image bit for bit.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_json.h"
#include "rt_scene.h"
#include "rt_vec.h"

using rtv::V2;
using rtv::V3;
using rtv::V4;

// ------------------------------------------------------------------------ errors
static thread_local std::string g_last_error;

void rt_set_error(const std::string &msg) { g_last_error = msg; }
int rt_fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

namespace {

struct rt_error : std::runtime_error {
    int code;
    rt_error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

std::string read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw rt_error(RT_ERR_IO, "File not found : " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

std::string dir_of(const std::string &path) {
    size_t p = path.find_last_of('/');
    return p == std::string::npos ? std::string() : path.substr(0, p + 1);
}

// ---------------------------------------------------------------- images (PNM -> RGBA8)
// tinygltf decodes every image with stb_image forcing 4 components (tiny_gltf.h:2609);
// this build's fixtures ship binary PNM (P6 RGB / P5 grey), decoded the same way
// (alpha = 255, grey replicated), which is what stbi_load(..., 4) returns for them.
struct Image {
    int w = 0, h = 0;
    std::vector<uint8_t> rgba;
};

Image load_pnm(const std::string &path) {
    std::string d = read_file(path);
    size_t p = 0;
    auto token = [&]() {
        for (;;) {
            while (p < d.size() && isspace((unsigned char)d[p])) ++p;
            if (p < d.size() && d[p] == '#') {
                while (p < d.size() && d[p] != '\n') ++p;
                continue;
            }
            break;
        }
        size_t b = p;
        while (p < d.size() && !isspace((unsigned char)d[p])) ++p;
        return d.substr(b, p - b);
    };
    std::string magic = token();
    if (magic != "P6" && magic != "P5")
        throw rt_error(RT_ERR_FORMAT, "Texture format not supported (need binary PNM): " + path);
    Image im;
    im.w = std::stoi(token());
    im.h = std::stoi(token());
    int maxv = std::stoi(token());
    if (maxv != 255) throw rt_error(RT_ERR_FORMAT, "Texture format not supported: only 8 bit channels are supported");
    ++p;  // single whitespace after maxval
    int comp = magic == "P6" ? 3 : 1;
    size_t need = (size_t)im.w * im.h * comp;
    if (d.size() < p + need) throw rt_error(RT_ERR_FORMAT, "truncated image " + path);
    im.rgba.resize((size_t)im.w * im.h * 4);
    const uint8_t *src = (const uint8_t *)d.data() + p;
    for (size_t i = 0; i < (size_t)im.w * im.h; ++i) {
        uint8_t *o = &im.rgba[4 * i];
        if (comp == 3) { o[0] = src[3 * i]; o[1] = src[3 * i + 1]; o[2] = src[3 * i + 2]; }
        else { o[0] = o[1] = o[2] = src[i]; }
        o[3] = 255;
    }
    return im;
}

// ---------------------------------------------------------------- matrix4<double>
// Column storage data[16] as src/utils/matrix.h:8-43.
struct M4 {
    double d[16] = {0};
};

M4 m4_from(const std::vector<double> &v) {
    M4 m;
    for (size_t i = 0; i < 16 && i < v.size(); ++i) m.d[i] = v[i];
    return m;
}
M4 m4_eye() {
    M4 m;
    m.d[0] = m.d[5] = m.d[10] = m.d[15] = 1.0;
    return m;
}
// matrix4::TRS (matrix.h:28-35): float arithmetic, stored to double.
M4 m4_trs(V3 t, V4 r, V3 s) {
    float v[16] = {
        (1.0f - 2.0f * (r.y * r.y + r.z * r.z)) * s.x, (r.x * r.y + r.z * r.w) * s.x * 2.0f,
        (r.x * r.z - r.y * r.w) * s.x * 2.0f, 0.f,
        (r.x * r.y - r.z * r.w) * s.y * 2.0f, (1.0f - 2.0f * (r.x * r.x + r.z * r.z)) * s.y,
        (r.y * r.z + r.x * r.w) * s.y * 2.0f, 0.f,
        (r.x * r.z + r.y * r.w) * s.z * 2.0f, (r.y * r.z - r.x * r.w) * s.z * 2.0f,
        (1.0f - 2.0f * (r.x * r.x + r.y * r.y)) * s.z, 0.f,
        t.x, t.y, t.z, 1.f};
    M4 m;
    for (int i = 0; i < 16; ++i) m.d[i] = v[i];
    return m;
}
// multiply(a, b) (matrix.h:45-63): dest[4i+j] = sum_k a[4i+k] * b[4k+j], left to right.
M4 m4_mul(const M4 &a, const M4 &b) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.d[4 * i + j] = a.d[4 * i] * b.d[j] + a.d[4 * i + 1] * b.d[4 + j] + a.d[4 * i + 2] * b.d[8 + j] +
                             a.d[4 * i + 3] * b.d[12 + j];
    return r;
}
// multiply(mat, vector4f) (matrix.h:66-72): float accumulators, each add done in double.
V4 m4_mul_v4(const M4 &m, V4 t) {
    float tv[4] = {t.x, t.y, t.z, t.w};
    float res[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) res[i] = (float)((double)res[i] + m.d[4 * j + i] * (double)tv[j]);
    return {res[0], res[1], res[2], res[3]};
}
V3 m4_mul_point(const M4 &m, V3 p) { return rtv::reduce(m4_mul_v4(m, {p.x, p.y, p.z, 1.f})); }
V3 m4_mul_vector(const M4 &m, V3 p) { return rtv::reduce(m4_mul_v4(m, {p.x, p.y, p.z, 0.f})); }

// The same products as the shipped reference binary computes them inside parse_scene_gltf's
// triangle loop (scene_parser.cpp:300-319).  GCC 11 at -O3 (the reference's CMake build)
// SLP-vectorizes that loop and keeps some of multiply()'s float accumulators in double, so a
// component is rounded to float once, after all four products are added, instead of after
// every add (matrix.h:66-72).  Determined against the reference's own dumps built with and
// without -fno-tree-slp-vectorize (oracle/Makefile ref_harness_noslp, tests/test_loader.py):
//   positions:  v0 and v1 - v0 as the source says; v2 - v0 in y and z from once-rounded
//               v2 and v0 (x as the source says);
//   normals:    multiplyVector(normal_transform, n) with x and y rounded once, z per add.
// Meshes whose transforms make every product exact (identity, scale, axis swaps) are the
// same either way.
float m4_dot_once(const M4 &m, int i, V3 p, float w) {
    return (float)(m.d[i] * (double)p.x + m.d[4 + i] * (double)p.y + m.d[8 + i] * (double)p.z + m.d[12 + i] * (double)w);
}
V3 m4_mul_vector_gcc(const M4 &m, V3 p) {
    const V3 r = m4_mul_vector(m, p);
    return {m4_dot_once(m, 0, p, 0.f), m4_dot_once(m, 1, p, 0.f), r.z};
}
M4 m4_transpose(const M4 &m) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.d[4 * i + j] = m.d[4 * j + i];
    return r;
}
// Cofactor inverse (matrix.h:88-217).  Each cofactor is six signed triple products summed
// left to right; the table lists (sign, a, b, c) for inv[k] = sum sign * m[a]*m[b]*m[c].
M4 m4_inverse(const M4 &mat) {
    static const int8_t T[16][6][4] = {
        {{+1, 5, 10, 15}, {-1, 5, 11, 14}, {-1, 9, 6, 15}, {+1, 9, 7, 14}, {+1, 13, 6, 11}, {-1, 13, 7, 10}},
        {{-1, 1, 10, 15}, {+1, 1, 11, 14}, {+1, 9, 2, 15}, {-1, 9, 3, 14}, {-1, 13, 2, 11}, {+1, 13, 3, 10}},
        {{+1, 1, 6, 15}, {-1, 1, 7, 14}, {-1, 5, 2, 15}, {+1, 5, 3, 14}, {+1, 13, 2, 7}, {-1, 13, 3, 6}},
        {{-1, 1, 6, 11}, {+1, 1, 7, 10}, {+1, 5, 2, 11}, {-1, 5, 3, 10}, {-1, 9, 2, 7}, {+1, 9, 3, 6}},
        {{-1, 4, 10, 15}, {+1, 4, 11, 14}, {+1, 8, 6, 15}, {-1, 8, 7, 14}, {-1, 12, 6, 11}, {+1, 12, 7, 10}},
        {{+1, 0, 10, 15}, {-1, 0, 11, 14}, {-1, 8, 2, 15}, {+1, 8, 3, 14}, {+1, 12, 2, 11}, {-1, 12, 3, 10}},
        {{-1, 0, 6, 15}, {+1, 0, 7, 14}, {+1, 4, 2, 15}, {-1, 4, 3, 14}, {-1, 12, 2, 7}, {+1, 12, 3, 6}},
        {{+1, 0, 6, 11}, {-1, 0, 7, 10}, {-1, 4, 2, 11}, {+1, 4, 3, 10}, {+1, 8, 2, 7}, {-1, 8, 3, 6}},
        {{+1, 4, 9, 15}, {-1, 4, 11, 13}, {-1, 8, 5, 15}, {+1, 8, 7, 13}, {+1, 12, 5, 11}, {-1, 12, 7, 9}},
        {{-1, 0, 9, 15}, {+1, 0, 11, 13}, {+1, 8, 1, 15}, {-1, 8, 3, 13}, {-1, 12, 1, 11}, {+1, 12, 3, 9}},
        {{+1, 0, 5, 15}, {-1, 0, 7, 13}, {-1, 4, 1, 15}, {+1, 4, 3, 13}, {+1, 12, 1, 7}, {-1, 12, 3, 5}},
        {{-1, 0, 5, 11}, {+1, 0, 7, 9}, {+1, 4, 1, 11}, {-1, 4, 3, 9}, {-1, 8, 1, 7}, {+1, 8, 3, 5}},
        {{-1, 4, 9, 14}, {+1, 4, 10, 13}, {+1, 8, 5, 14}, {-1, 8, 6, 13}, {-1, 12, 5, 10}, {+1, 12, 6, 9}},
        {{+1, 0, 9, 14}, {-1, 0, 10, 13}, {-1, 8, 1, 14}, {+1, 8, 2, 13}, {+1, 12, 1, 10}, {-1, 12, 2, 9}},
        {{-1, 0, 5, 14}, {+1, 0, 6, 13}, {+1, 4, 1, 14}, {-1, 4, 2, 13}, {-1, 12, 1, 6}, {+1, 12, 2, 5}},
        {{+1, 0, 5, 10}, {-1, 0, 6, 9}, {-1, 4, 1, 10}, {+1, 4, 2, 9}, {+1, 8, 1, 6}, {-1, 8, 2, 5}},
    };
    const double *m = mat.d;
    M4 res;
    for (int k = 0; k < 16; ++k) {
        const int8_t(*t)[4] = T[k];
        double acc = (t[0][0] < 0 ? -m[t[0][1]] : m[t[0][1]]) * m[t[0][2]] * m[t[0][3]];
        for (int q = 1; q < 6; ++q) {
            double p = m[t[q][1]] * m[t[q][2]] * m[t[q][3]];
            acc = t[q][0] < 0 ? acc - p : acc + p;
        }
        res.d[k] = acc;
    }
    double det = m[0] * res.d[0] + m[1] * res.d[4] + m[2] * res.d[8] + m[3] * res.d[12];
    if (det == 0) throw rt_error(RT_ERR_FORMAT, "Zero determinant");
    det = 1.0 / det;
    for (int i = 0; i < 16; ++i) res.d[i] *= det;
    return res;
}

// ---------------------------------------------------------------- primitives and boxes
struct Box {  // AABB (primitive.h:18-63), inverted-infinite when empty
    V3 mn{FLT_MAX, FLT_MAX, FLT_MAX};
    V3 mx{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(V3 p) { mn = rtv::vmin(mn, p); mx = rtv::vmax(mx, p); }
    void grow(const Box &b) { mn = rtv::vmin(mn, b.mn); mx = rtv::vmax(mx, b.mx); }
    V3 size() const { return rtv::sub(mx, mn); }
    V3 center() const { return rtv::add(mn, rtv::mul(size(), 0.5f)); }
    float surface_area() const {
        V3 s = size();
        return 2.f * (s.x * s.y + s.x * s.z + s.y * s.z);
    }
};

struct Prim {  // Primitive (primitive.h:96-134)
    V3 pos[3];  // v0, U, V
    V3 nrm[3];
    V4 tan[3];
    V2 tc[3];
    int mesh_id = 0;
    Box box;   // Primitive::aabb() (primitive.cpp:63-75)
    V3 center;
};

struct MeshRec {
    float base_color[3] = {1.f, 1.f, 1.f};
    float emission[3] = {0.f, 0.f, 0.f};
    float metallic = 1.f, roughness2 = 1.f, alpha = 1.f, ior = 1.f;
    int tex[4] = {-1, -1, -1, -1};  // base_color, normal, metallic_roughness, emission
    M4 normal_transform;
};

// ---------------------------------------------------------------- BVH build
// Reference-exact restatement of BVH::buildBVH / buildNode / buildHelperSAH
// (src/core/bvh.cpp:5-175): widest axis only, full std::sort by centroid (BIN_SIZE 1),
// SAH sweep with strict `<`, std::partition on the split value, leaves of <= 4 or on a
// failed split, children appended as (left, left + 1) and built depth-first LIFO.
// libstdc++'s std::sort / std::partition are driven only by the comparison results, so
// sorting an index array reproduces the reference's permutation of the 208-byte objects.
struct BuildNode {
    Box box;
    int64_t left = -1, right = -1, split = -1, first = -1, count = 0;
};

class BvhBuilder {
public:
    BvhBuilder(const std::vector<Prim> &prims, std::vector<uint32_t> &order) : P(prims), order(order) {}

    std::vector<BuildNode> build() {
        if (order.empty()) throw rt_error(RT_ERR_FORMAT, "No primitives for node 0");
        struct Item { size_t place, first, count; };
        std::vector<Item> q;
        q.push_back({nodes.size(), 0, order.size()});
        nodes.emplace_back();
        while (!q.empty()) {
            Item it = q.back();
            q.pop_back();
            BuildNode &nd = nodes[it.place];
            for (size_t k = it.first; k < it.first + it.count; ++k) nd.box.grow(P[order[k]].box);
            if (it.count <= 4) { leaf(it.place, it.first, it.count); continue; }
            size_t split_dim = 0;
            size_t res = sah(nodes[it.place].box, it.first, it.count, split_dim);
            nodes[it.place].split = (int64_t)split_dim;
            if (res == 0 || res == it.count) { leaf(it.place, it.first, it.count); continue; }
            size_t l = nodes.size();
            nodes[it.place].left = (int64_t)l;
            nodes.emplace_back();
            q.push_back({l, it.first, res});
            nodes[it.place].right = (int64_t)(l + 1);
            nodes.emplace_back();
            q.push_back({l + 1, it.first + res, it.count - res});
        }
        return nodes;
    }

private:
    const std::vector<Prim> &P;
    std::vector<uint32_t> &order;
    std::vector<BuildNode> nodes;

    void leaf(size_t place, size_t first, size_t count) {
        nodes[place].first = (int64_t)first;
        nodes[place].count = (int64_t)count;
    }

    float c(uint32_t id, int dim) const { return rtv::at(P[id].center, dim); }

    size_t sah(const Box &node_box, size_t first, size_t count, size_t &best_dim) {
        uint32_t *begin = order.data() + first, *end = begin + count;
        float best_sah = node_box.surface_area() * (float)count;
        float best_split = (float)((double)c(*begin, 2) - 1e-7);
        best_dim = 2;
        int dim = 0;
        {
            float max_size = node_box.size().x;
            for (int i = 0; i < 3; ++i) {
                if (max_size < rtv::at(node_box.size(), i)) {
                    max_size = rtv::at(node_box.size(), i);
                    dim = i;
                }
            }
        }
        std::sort(begin, end, [&](uint32_t a, uint32_t b) { return c(a, dim) < c(b, dim); });
        std::vector<float> left(count), right(count);
        Box tmp;  // sah_bins[0]: one primitive per bin (BIN_SIZE 1)
        tmp.grow(P[begin[0]].box);
        left[0] = tmp.surface_area();
        for (size_t i = 1; i < count; ++i) {
            tmp.grow(P[begin[i]].box);
            left[i] = tmp.surface_area();
        }
        {
            Box bl;
            bl.grow(P[begin[count - 1]].box);
            tmp = bl;
        }
        right[count - 1] = tmp.surface_area();
        for (long i = (long)count - 2; i >= 0; --i) {
            tmp.grow(P[begin[i]].box);
            right[i] = tmp.surface_area();
        }
        for (size_t i = 0; i + 1 < count; ++i) {
            float ls = left[i], rs = right[i + 1];
            int left_cnt = (int)(i + 1);
            float metric = ls * (float)(left_cnt) + rs * (float)(count - (size_t)left_cnt);
            if (metric < best_sah) {
                best_sah = metric;
                best_dim = (size_t)dim;
                if ((size_t)left_cnt < count) best_split = (c(begin[left_cnt - 1], dim) + c(begin[left_cnt], dim)) * 0.5f;
            }
        }
        const int bd = (int)best_dim;
        const float bs = best_split;
        uint32_t *mid = std::partition(begin, end, [&](uint32_t a) { return c(a, bd) < bs; });
        return (size_t)(mid - begin);
    }
};

float as_f32(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
uint32_t as_u32(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// Flattens a built tree to 8 floats per node; returns the max depth.
uint32_t flatten_nodes(const std::vector<BuildNode> &nodes, std::vector<float> &out) {
    out.resize(nodes.size() * 8);
    std::vector<uint32_t> depth(nodes.size(), 0);
    uint32_t maxd = 0;
    for (size_t i = 0; i < nodes.size(); ++i) {
        const BuildNode &n = nodes[i];
        float *o = &out[8 * i];
        o[0] = n.box.mn.x; o[1] = n.box.mn.y; o[2] = n.box.mn.z;
        o[3] = n.box.mx.x; o[4] = n.box.mx.y; o[5] = n.box.mx.z;
        if (n.count == 0) {
            if (n.right != n.left + 1) throw rt_error(RT_ERR_FORMAT, "internal: right != left + 1");
            o[6] = as_f32((uint32_t)n.left);
            o[7] = as_f32((uint32_t)n.split);
            depth[n.left] = depth[n.right] = depth[i] + 1;  // children always follow parents
        } else {
            o[6] = as_f32((uint32_t)n.first);
            o[7] = as_f32(3u | ((uint32_t)n.count << 2));
        }
        maxd = std::max(maxd, depth[i]);
    }
    return maxd;
}

V3 geometric_normal(const Prim &p, float &area) {  // Primitive::get_geometric_normal (primitive.cpp:77-84)
    V3 n = rtv::cross(p.pos[1], p.pos[2]);
    area = 0.5f * rtv::length(n);
    return rtv::normal(n);
}

// ---------------------------------------------------------------- glTF ingest
struct AccessorView {
    const uint8_t *data = nullptr;
    size_t count = 0;
    int ctype = 0;
    std::string type;
};

struct Loader {
    rtj::Value doc;
    std::string base;
    std::vector<std::string> buffers;

    // Every element of the accessor must lie inside its buffer (tightly packed: byteStride is
    // ignored, as scene_parser.cpp does); a malformed file is RT_ERR_FORMAT, never a read
    // past the end.
    AccessorView view(int idx) {
        if (idx < 0) throw rt_error(RT_ERR_FORMAT, "accessor out of range");
        const rtj::Value &a = doc["accessors"][(size_t)idx];
        if (a.is_null()) throw rt_error(RT_ERR_FORMAT, "accessor out of range");
        const int bvi = a["bufferView"].integer(-1);
        if (bvi < 0) throw rt_error(RT_ERR_FORMAT, "bufferView out of range");
        const rtj::Value &bv = doc["bufferViews"][(size_t)bvi];
        if (bv.is_null()) throw rt_error(RT_ERR_FORMAT, "bufferView out of range");
        int b = bv["buffer"].integer(0);
        if (b < 0 || (size_t)b >= buffers.size()) throw rt_error(RT_ERR_FORMAT, "buffer out of range");
        const double off_d = bv["byteOffset"].number(0) + a["byteOffset"].number(0), count_d = a["count"].number(0);
        if (!(off_d >= 0) || !(count_d >= 0) || off_d > 1e15 || count_d > 1e15)
            throw rt_error(RT_ERR_FORMAT, "accessor offset / count invalid");
        AccessorView v;
        const size_t off = (size_t)off_d;
        v.count = (size_t)count_d;
        v.ctype = a["componentType"].integer(0);
        v.type = a["type"].str;
        const size_t comps = v.type == "SCALAR" ? 1 : v.type == "VEC2" ? 2 : v.type == "VEC3" ? 3 : v.type == "VEC4" ? 4
                           : v.type == "MAT4" ? 16 : 0;
        const size_t cbytes = (v.ctype == 5120 || v.ctype == 5121) ? 1 : (v.ctype == 5122 || v.ctype == 5123) ? 2
                            : (v.ctype == 5125 || v.ctype == 5126) ? 4 : 0;
        const size_t size = buffers[b].size();
        if (off > size || (comps * cbytes > 0 && v.count > (size - off) / (comps * cbytes)))
            throw rt_error(RT_ERR_FORMAT, "accessor beyond buffer");
        v.data = (const uint8_t *)buffers[b].data() + off;
        return v;
    }
};

}  // namespace

// Restates parse_scene_gltf (src/io/scene_parser.cpp:25-350) + Scene::Scene
// (src/core/scene.cpp:197-249) + ManyLightsDistribution (src/utils/random.cpp:156-168).
static void load_gltf(rt_scene &S, const std::string &path, int width, int height, int samples) {
    Loader L;
    std::string text = read_file(path);
    L.doc = rtj::parse(text);
    L.base = dir_of(path);
    const rtj::Value &doc = L.doc;
    for (size_t i = 0; i < doc["buffers"].size(); ++i) {
        const std::string &uri = doc["buffers"][i]["uri"].str;
        if (uri.rfind("data:", 0) == 0) throw rt_error(RT_ERR_FORMAT, "data: URIs are not supported");
        L.buffers.push_back(read_file(L.base + uri));
    }
    // node transforms (scene_parser.cpp:47-97): parents must precede children; one level
    // of propagation, exactly as the reference
    size_t nn = doc["nodes"].size();
    std::vector<std::vector<double>> node_matrix(nn);
    for (size_t i = 0; i < nn; ++i) node_matrix[i] = doc["nodes"][i]["matrix"].numbers();
    int node_with_camera = -1;
    for (size_t i = 0; i < nn; ++i) {
        const rtj::Value &node = doc["nodes"][i];
        if (node.has("camera") && node["camera"].integer(-1) != -1 && node_with_camera == -1) node_with_camera = (int)i;
        std::vector<double> T = node["translation"].numbers(), R = node["rotation"].numbers(), Sc = node["scale"].numbers();
        M4 transform;
        if (T.empty() && R.empty() && Sc.empty()) {
            transform = node_matrix[i].empty() ? m4_eye() : m4_from(node_matrix[i]);
        } else {
            V3 t{0.f, 0.f, 0.f};
            V4 r{0.f, 0.f, 0.f, 1.f};
            V3 s{1.f, 1.f, 1.f};
            if (!T.empty()) t = {(float)T[0], (float)T[1], (float)T[2]};
            if (!R.empty()) r = {(float)R[0], (float)R[1], (float)R[2], (float)R[3]};
            if (!Sc.empty()) s = {(float)Sc[0], (float)Sc[1], (float)Sc[2]};
            transform = m4_trs(t, r, s);
            if (!node_matrix[i].empty()) transform = m4_mul(m4_from(node_matrix[i]), transform);
        }
        node_matrix[i].assign(transform.d, transform.d + 16);
        for (size_t c = 0; c < node["children"].size(); ++c) {
            size_t child = (size_t)node["children"][c].integer(0);
            if (child >= nn) throw rt_error(RT_ERR_FORMAT, "child node out of range");
            M4 sub = transform;
            if (!node_matrix[child].empty()) sub = m4_mul(transform, m4_from(node_matrix[child]));
            node_matrix[child].assign(sub.d, sub.d + 16);
        }
    }
    if (node_with_camera == -1) throw rt_error(RT_ERR_FORMAT, "[gltf check] No camera found");

    // camera (scene_parser.cpp:103-127)
    {
        const rtj::Value &cn = doc["nodes"][(size_t)node_with_camera];
        M4 cm = m4_from(node_matrix[node_with_camera]);
        V3 pos = m4_mul_point(cm, {0.f, 0.f, 0.f});
        std::vector<double> sc = cn["scale"].numbers();
        V3 axes[3];
        for (int i = 0; i < 3; ++i) {
            float dv[4] = {0.f, 0.f, 0.f, 0.f};
            dv[i] = 1.f;
            dv[2] = -dv[2];
            V4 res = m4_mul_v4(cm, {dv[0], dv[1], dv[2], dv[3]});
            if (!sc.empty()) {
                res.x /= (float)sc[0];
                res.y /= (float)sc[1];
                res.z /= (float)sc[2];
            }
            axes[i] = rtv::normal(rtv::reduce(res));
        }
        const rtj::Value &persp = doc["cameras"][(size_t)cn["camera"].integer(0)]["perspective"];
        double zfar = persp["zfar"].number(0.0);
        if (zfar > 0) S.max_distance = (float)zfar;
        float fov_y = (float)persp["yfov"].number(0.0);
        double ar = persp["aspectRatio"].number(0.0);
        float aspect = (ar != 0) ? (float)ar : (float)width / (float)height;
        float fov_x = 2.f * std::atan(std::tan(fov_y * 0.5f) * aspect);
        S.cam_pos[0] = pos.x; S.cam_pos[1] = pos.y; S.cam_pos[2] = pos.z;
        for (int i = 0; i < 3; ++i) {
            S.cam_axes[3 * i] = axes[i].x;
            S.cam_axes[3 * i + 1] = axes[i].y;
            S.cam_axes[3 * i + 2] = axes[i].z;
        }
        S.cam_fov[0] = fov_x;
        S.cam_fov[1] = fov_y;
        S.tan_half_fov[0] = std::tan(fov_x / 2);   // camera.cpp:51
        S.tan_half_fov[1] = std::tan(fov_y / 2);   // camera.cpp:52
    }
    S.width = width;
    S.height = height;
    S.samples = samples;
    S.ray_depth = 6;  // ScenePartial::ray_depth (scene_parser.cpp:17)

    // textures (scene_parser.cpp:131-142)
    for (size_t i = 0; i < doc["images"].size(); ++i) {
        const std::string &uri = doc["images"][i]["uri"].str;
        Image im = load_pnm(L.base + uri);
        S.tex_info.push_back((uint32_t)(S.texels.size() / 4));
        S.tex_info.push_back((uint32_t)im.w);
        S.tex_info.push_back((uint32_t)im.h);
        S.tex_info.push_back(4u);
        S.texels.insert(S.texels.end(), im.rgba.begin(), im.rgba.end());
    }
    auto get_image = [&](const rtj::Value &texinfo) -> int {
        int i = texinfo["index"].integer(-1);
        if (i == -1) return -1;
        return doc["textures"][(size_t)i]["source"].integer(-1);
    };

    // meshes / materials / triangles (scene_parser.cpp:145-346)
    std::vector<MeshRec> meshes;
    std::vector<Prim> prims;
    for (size_t ni = 0; ni < nn; ++ni) {
        const rtj::Value &node = doc["nodes"][ni];
        int mesh_idx = node["mesh"].integer(-1);
        if (mesh_idx == -1) continue;
        const rtj::Value &gmesh = doc["meshes"][(size_t)mesh_idx];
        for (size_t pi = 0; pi < gmesh["primitives"].size(); ++pi) {
            const rtj::Value &p = gmesh["primitives"][pi];
            meshes.emplace_back();
            MeshRec &mesh = meshes.back();
            M4 transform = m4_from(node_matrix[ni]);
            mesh.normal_transform = m4_inverse(m4_transpose(transform));
            int mat = p["material"].integer(-1);
            if (mat != -1) {
                const rtj::Value &gm = doc["materials"][(size_t)mat];
                const rtj::Value &pbr = gm["pbrMetallicRoughness"];
                std::vector<double> bcf = pbr["baseColorFactor"].numbers();
                if (bcf.size() != 4) bcf = {1.0, 1.0, 1.0, 1.0};
                for (int j = 0; j < 3; ++j) mesh.base_color[j] = (float)bcf[j];
                if (bcf[3] < 1.) {
                    mesh.alpha = (float)bcf[3];
                    const rtj::Value &ior = gm["extensions"]["KHR_materials_ior"];
                    mesh.ior = gm["extensions"].has("KHR_materials_ior") ? (float)ior["ior"].number(0.0) : 1.5f;
                }
                mesh.metallic = (float)pbr["metallicFactor"].number(1.0);
                mesh.roughness2 = (float)pbr["roughnessFactor"].number(1.0);
                mesh.roughness2 *= mesh.roughness2;
                std::vector<double> ef = gm["emissiveFactor"].numbers();
                if (ef.size() != 3) ef = {0.0, 0.0, 0.0};
                for (int j = 0; j < 3; ++j) mesh.emission[j] = (float)ef[j];
                if (gm["extensions"].has("KHR_materials_emissive_strength")) {
                    float es = (float)gm["extensions"]["KHR_materials_emissive_strength"]["emissiveStrength"].number(0.0);
                    for (int j = 0; j < 3; ++j) mesh.emission[j] *= es;
                }
                mesh.tex[0] = get_image(pbr["baseColorTexture"]);
                mesh.tex[1] = get_image(gm["normalTexture"]);
                mesh.tex[2] = get_image(pbr["metallicRoughnessTexture"]);
                mesh.tex[3] = get_image(gm["emissiveTexture"]);
            }
            const rtj::Value &attrs = p["attributes"];
            if (!p.has("indices")) throw rt_error(RT_ERR_FORMAT, "Index type not supported");
            AccessorView iv = L.view(p["indices"].integer(0));
            if (iv.type != "SCALAR") throw rt_error(RT_ERR_FORMAT, "Index type not supported");
            AccessorView pv = L.view(attrs["POSITION"].integer(0));
            if (pv.type != "VEC3") throw rt_error(RT_ERR_FORMAT, "Position type not supported");
            if (pv.ctype != 5126) throw rt_error(RT_ERR_FORMAT, "Position component type not supported");
            const float *pos_v = (const float *)pv.data;
            const float *nrm_v = nullptr, *tc_v = nullptr, *tan_v = nullptr;
            size_t n_attr = pv.count;   // vertices every present attribute holds (indices must be below)
            // NB: the reference only reads the index count when NORMAL exists
            // (scene_parser.cpp:233-234); without it its count is indeterminate.  Here the
            // accessor's count is used in both cases.
            size_t indices_count = iv.count;
            int indices_ctype = iv.ctype;
            if (attrs.has("NORMAL")) {
                AccessorView nv = L.view(attrs["NORMAL"].integer(0));
                if (nv.type != "VEC3") throw rt_error(RT_ERR_FORMAT, "Normal type not supported");
                if (nv.ctype != 5126) throw rt_error(RT_ERR_FORMAT, "Normal component type not supported");
                nrm_v = (const float *)nv.data;
                n_attr = std::min(n_attr, nv.count);
            }
            if (attrs.has("TEXCOORD_0")) {
                AccessorView tv = L.view(attrs["TEXCOORD_0"].integer(0));
                if (tv.type != "VEC2") throw rt_error(RT_ERR_FORMAT, "Texcoord type not supported");
                if (tv.ctype != 5126) throw rt_error(RT_ERR_FORMAT, "Texcoord component type not supported");
                tc_v = (const float *)tv.data;
                n_attr = std::min(n_attr, tv.count);
            }
            if (attrs.has("TANGENT")) {
                AccessorView tv = L.view(attrs["TANGENT"].integer(0));
                if (tv.type != "VEC4") throw rt_error(RT_ERR_FORMAT, "Tangent type not supported");
                if (tv.ctype != 5126) throw rt_error(RT_ERR_FORMAT, "Tangent component type not supported");
                tan_v = (const float *)tv.data;
                n_attr = std::min(n_attr, tv.count);
            }
            if (indices_ctype != 5123 && indices_ctype != 5125)
                throw rt_error(RT_ERR_FORMAT, "Index component type not supported");
            const int mesh_id = (int)meshes.size() - 1;
            for (size_t t = 0; t < indices_count / 3; ++t) {
                size_t index[3];
                for (int v = 0; v < 3; ++v) {
                    index[v] = indices_ctype == 5123 ? ((const uint16_t *)iv.data)[t * 3 + v]
                                                     : ((const uint32_t *)iv.data)[t * 3 + v];
                    if (index[v] >= n_attr) throw rt_error(RT_ERR_FORMAT, "vertex index beyond an attribute accessor");
                }
                Prim pr;
                pr.mesh_id = mesh_id;
                V3 q[3];
                for (int v = 0; v < 3; ++v) {
                    q[v] = V3{pos_v[index[v] * 3], pos_v[index[v] * 3 + 1], pos_v[index[v] * 3 + 2]};
                    pr.pos[v] = m4_mul_point(transform, q[v]);
                }
                // (the reference binary's v2 - v0: see m4_mul_vector_gcc)
                const float y0 = m4_dot_once(transform, 1, q[0], 1.f), z0 = m4_dot_once(transform, 2, q[0], 1.f);
                const float y2 = m4_dot_once(transform, 1, q[2], 1.f), z2 = m4_dot_once(transform, 2, q[2], 1.f);
                pr.pos[1] = rtv::sub(pr.pos[1], pr.pos[0]);
                pr.pos[2] = V3{pr.pos[2].x - pr.pos[0].x, y2 - y0, z2 - z0};
                for (int v = 0; v < 3; ++v) {
                    V3 n = nrm_v ? V3{nrm_v[index[v] * 3], nrm_v[index[v] * 3 + 1], nrm_v[index[v] * 3 + 2]}
                                 : V3{0.f, 0.f, 1.f};
                    pr.nrm[v] = rtv::normal(m4_mul_vector_gcc(mesh.normal_transform, n));
                }
                for (int v = 0; v < 3; ++v) {
                    pr.tc[v] = tc_v ? V2{tc_v[index[v] * 2], tc_v[index[v] * 2 + 1]} : V2{0.f, 0.f};
                    pr.tan[v] = tan_v ? V4{tan_v[index[v] * 4], tan_v[index[v] * 4 + 1], tan_v[index[v] * 4 + 2],
                                           tan_v[index[v] * 4 + 3]}
                                      : V4{0.f, 0.f, 0.f, 0.f};
                }
                pr.box.grow(pr.pos[0]);
                pr.box.grow(rtv::add(pr.pos[0], pr.pos[1]));
                pr.box.grow(rtv::add(pr.pos[0], pr.pos[2]));
                pr.center = pr.box.center();
                prims.push_back(pr);
            }
        }
    }

    // scene BVH (scene.cpp:231 -> bvh.cpp:166)
    std::vector<uint32_t> order(prims.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (uint32_t)i;
    std::vector<BuildNode> nodes = BvhBuilder(prims, order).build();
    S.bvh_depth = flatten_nodes(nodes, S.node);

    const size_t nt = order.size();
    S.tri.resize(nt * 12);
    S.tri_attr.resize(nt * 16);
    S.tri_tan.resize(nt * 12);
    std::vector<Prim> lights;
    for (size_t k = 0; k < nt; ++k) {
        const Prim &p = prims[order[k]];
        float area = 0.f;
        V3 g = geometric_normal(p, area);
        float *o = &S.tri[12 * k];
        for (int v = 0; v < 3; ++v) { o[3 * v] = p.pos[v].x; o[3 * v + 1] = p.pos[v].y; o[3 * v + 2] = p.pos[v].z; }
        o[9] = g.x; o[10] = g.y; o[11] = g.z;
        float *a = &S.tri_attr[16 * k];
        for (int v = 0; v < 3; ++v) { a[3 * v] = p.nrm[v].x; a[3 * v + 1] = p.nrm[v].y; a[3 * v + 2] = p.nrm[v].z; }
        for (int v = 0; v < 3; ++v) { a[9 + 2 * v] = p.tc[v].x; a[10 + 2 * v] = p.tc[v].y; }
        a[15] = as_f32((uint32_t)p.mesh_id);
        float *tg = &S.tri_tan[12 * k];
        for (int v = 0; v < 3; ++v) { tg[4 * v] = p.tan[v].x; tg[4 * v + 1] = p.tan[v].y; tg[4 * v + 2] = p.tan[v].z; tg[4 * v + 3] = p.tan[v].w; }
        const MeshRec &m = meshes[p.mesh_id];
        if (!(m.emission[0] == 0 && m.emission[1] == 0 && m.emission[2] == 0)) lights.push_back(p);  // Primitive::emissive
    }
    // light list + light BVH (random.cpp:156-168)
    if (!lights.empty()) {
        std::vector<uint32_t> lorder(lights.size());
        for (size_t i = 0; i < lorder.size(); ++i) lorder[i] = (uint32_t)i;
        std::vector<BuildNode> lnodes = BvhBuilder(lights, lorder).build();
        S.light_bvh_depth = flatten_nodes(lnodes, S.light_node);
        S.light.resize(lights.size() * 16, 0.f);
        for (size_t k = 0; k < lights.size(); ++k) {
            const Prim &p = lights[lorder[k]];
            float area = 0.f;
            V3 g = geometric_normal(p, area);
            float *o = &S.light[16 * k];
            for (int v = 0; v < 3; ++v) { o[3 * v] = p.pos[v].x; o[3 * v + 1] = p.pos[v].y; o[3 * v + 2] = p.pos[v].z; }
            o[9] = g.x; o[10] = g.y; o[11] = g.z;
            o[12] = area;
        }
    }
    for (const MeshRec &m : meshes) {
        float f[12] = {m.base_color[0], m.base_color[1], m.base_color[2], m.emission[0], m.emission[1], m.emission[2],
                       m.metallic, m.roughness2, m.alpha, m.ior, 0.f, 0.f};
        S.mesh_f.insert(S.mesh_f.end(), f, f + 12);
        S.mesh_tex.insert(S.mesh_tex.end(), m.tex, m.tex + 4);
        S.mesh_nt.insert(S.mesh_nt.end(), m.normal_transform.d, m.normal_transform.d + 16);
        for (int t = 0; t < 4; ++t)
            if (m.tex[t] >= (int)(S.tex_info.size() / 4)) throw rt_error(RT_ERR_FORMAT, "texture index out of range");
    }
}

// ------------------------------------------------------------------------ ABI
extern "C" {

int rt_scene_load_gltf(const char *path, int32_t width, int32_t height, int32_t samples, rt_scene **out) {
    if (!path || !out || width <= 0 || height <= 0 || samples < 0) return rt_fail(RT_ERR_ARG, "rt_scene_load_gltf: bad argument");
    *out = nullptr;
    try {
        std::unique_ptr<rt_scene> s(new rt_scene());
        load_gltf(*s, path, width, height, samples);
        *out = s.release();
        return RT_OK;
    } catch (const rt_error &e) {
        return rt_fail(e.code, e.what());
    } catch (const std::exception &e) {
        return rt_fail(RT_ERR_FORMAT, std::string("[gltf] ") + e.what());
    }
}

int rt_scene_from_view(const rt_scene_view *v, rt_scene **out) {
    if (!v || !out) return rt_fail(RT_ERR_ARG, "rt_scene_from_view: NULL");
    *out = nullptr;
    try {
        std::unique_ptr<rt_scene> s(new rt_scene());
        s->width = v->width; s->height = v->height; s->samples = v->samples; s->ray_depth = v->ray_depth;
        s->max_distance = v->max_distance;
        std::memcpy(s->cam_pos, v->cam_pos, sizeof s->cam_pos);
        std::memcpy(s->cam_axes, v->cam_axes, sizeof s->cam_axes);
        std::memcpy(s->cam_fov, v->cam_fov, sizeof s->cam_fov);
        std::memcpy(s->tan_half_fov, v->tan_half_fov, sizeof s->tan_half_fov);
        auto cp = [](auto &dst, const auto *src, size_t n) { dst.assign(src, src + n); };
        cp(s->tri, v->tri, (size_t)v->n_tris * 12);
        cp(s->tri_attr, v->tri_attr, (size_t)v->n_tris * 16);
        cp(s->tri_tan, v->tri_tan, (size_t)v->n_tris * 12);
        cp(s->node, v->node, (size_t)v->n_nodes * 8);
        cp(s->light, v->light, (size_t)v->n_lights * 16);
        cp(s->light_node, v->light_node, (size_t)v->n_light_nodes * 8);
        cp(s->mesh_f, v->mesh_f, (size_t)v->n_meshes * 12);
        cp(s->mesh_tex, v->mesh_tex, (size_t)v->n_meshes * 4);
        cp(s->mesh_nt, v->mesh_normal_transform, (size_t)v->n_meshes * 16);
        cp(s->tex_info, v->tex_info, (size_t)v->n_textures * 4);
        cp(s->texels, v->texels, (size_t)v->n_texel_bytes);
        // validate the trees and recompute their depths (children always follow parents)
        auto depth_of = [](const std::vector<float> &nodes, size_t n_prims, const char *what) {
            size_t nn = nodes.size() / 8;
            std::vector<uint32_t> depth(nn, 0);
            uint32_t maxd = 0;
            for (size_t i = 0; i < nn; ++i) {
                uint32_t a = as_u32(nodes[8 * i + 6]), b = as_u32(nodes[8 * i + 7]);
                if ((b & 3u) == 3u) {
                    if ((size_t)a + (b >> 2) > n_prims) throw rt_error(RT_ERR_ARG, std::string(what) + ": leaf range out of bounds");
                } else {
                    if (b > 2 || a <= i || (size_t)a + 1 >= nn) throw rt_error(RT_ERR_ARG, std::string(what) + ": bad internal node");
                    depth[a] = depth[a + 1] = depth[i] + 1;
                }
                maxd = std::max(maxd, depth[i]);
            }
            return maxd;
        };
        if (s->node.empty()) throw rt_error(RT_ERR_ARG, "scene without BVH nodes");
        s->bvh_depth = depth_of(s->node, v->n_tris, "bvh");
        if (!s->light_node.empty()) s->light_bvh_depth = depth_of(s->light_node, v->n_lights, "light bvh");
        for (uint32_t k = 0; k < v->n_tris; ++k) {
            uint32_t m = as_u32(s->tri_attr[16 * k + 15]);
            if (m >= v->n_meshes) throw rt_error(RT_ERR_ARG, "triangle mesh id out of range");
        }
        for (int32_t t : s->mesh_tex)
            if (t >= (int32_t)v->n_textures) throw rt_error(RT_ERR_ARG, "texture index out of range");
        for (uint32_t t = 0; t < v->n_textures; ++t) {
            const uint32_t *ti = &s->tex_info[4 * t];
            if (ti[3] != 4 || ((uint64_t)ti[0] + (uint64_t)ti[1] * ti[2]) * 4 > s->texels.size())
                throw rt_error(RT_ERR_ARG, "texture outside the texel buffer");
        }
        *out = s.release();
        return RT_OK;
    } catch (const rt_error &e) {
        return rt_fail(e.code, e.what());
    } catch (const std::exception &e) {
        return rt_fail(RT_ERR_ARG, e.what());
    }
}

int rt_scene_get_view(const rt_scene *s, rt_scene_view *v) {
    if (!s || !v) return rt_fail(RT_ERR_ARG, "rt_scene_get_view: NULL");
    std::memset(v, 0, sizeof *v);
    v->width = s->width; v->height = s->height; v->samples = s->samples; v->ray_depth = s->ray_depth;
    v->max_distance = s->max_distance;
    std::memcpy(v->cam_pos, s->cam_pos, sizeof v->cam_pos);
    std::memcpy(v->cam_axes, s->cam_axes, sizeof v->cam_axes);
    std::memcpy(v->cam_fov, s->cam_fov, sizeof v->cam_fov);
    std::memcpy(v->tan_half_fov, s->tan_half_fov, sizeof v->tan_half_fov);
    v->n_tris = (uint32_t)(s->tri.size() / 12);
    v->tri = s->tri.data(); v->tri_attr = s->tri_attr.data(); v->tri_tan = s->tri_tan.data();
    v->n_nodes = (uint32_t)(s->node.size() / 8); v->node = s->node.data(); v->bvh_depth = s->bvh_depth;
    v->n_lights = (uint32_t)(s->light.size() / 16); v->light = s->light.data();
    v->n_light_nodes = (uint32_t)(s->light_node.size() / 8); v->light_node = s->light_node.data();
    v->light_bvh_depth = s->light_bvh_depth;
    v->n_meshes = (uint32_t)(s->mesh_f.size() / 12);
    v->mesh_f = s->mesh_f.data(); v->mesh_tex = s->mesh_tex.data(); v->mesh_normal_transform = s->mesh_nt.data();
    v->n_textures = (uint32_t)(s->tex_info.size() / 4); v->tex_info = s->tex_info.data();
    v->texels = s->texels.data(); v->n_texel_bytes = s->texels.size();
    return RT_OK;
}

void rt_scene_free(rt_scene *s) {
    if (!s) return;
    rt_device_scene_release(s);
    delete s;
}

int64_t rt_shard_rows(int32_t height, int32_t rank, int32_t world, int32_t row_block, int32_t *rows_out) {
    return rt_shard_rows_impl(height, rank, world, row_block, rows_out);
}

// Scene::render frame finish (scene.cpp:54-64): c * (1/spp) -> ACES (vector.h:400-407)
// -> powf(c, 1/2.2f) -> (uint8_t)roundf(clamp(c * 255, 0, 255)) (vector.h:222-233).
int rt_tonemap_u8(const float *sum, int32_t width, int32_t height, int32_t spp, uint8_t *rgb) {
    if (!sum || !rgb || width <= 0 || height <= 0 || spp <= 0) return rt_fail(RT_ERR_ARG, "rt_tonemap_u8: bad argument");
    const float normalizer = 1.f / (float)spp;
    const float gamma = 1.f / 2.2f;
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    for (int64_t p = 0; p < (int64_t)width * height; ++p) {
        for (int k = 0; k < 3; ++k) {
            float x = sum[3 * p + k];
            x *= normalizer;
            float num = x * (x * a + b);
            float den = x * (x * c + d) + e;
            float v = rtv::smax(rtv::smin(num / den, 1.f), 0.f);
            v = std::pow(v, gamma);
            float s = rtv::smax(rtv::smin(v * 255, 255.f), 0.f);
            float r = std::round(s);
            rgb[3 * p + k] = std::isnan(r) ? (uint8_t)0 : (uint8_t)(int)r;
        }
    }
    return RT_OK;
}

int rt_write_ppm(const char *path, const uint8_t *rgb, int32_t width, int32_t height) {
    if (!path || !rgb || width <= 0 || height <= 0) return rt_fail(RT_ERR_ARG, "rt_write_ppm: bad argument");
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return rt_fail(RT_ERR_IO, "File open error");
    std::fprintf(f, "P6\n%d %d\n255\n", width, height);
    size_t n = (size_t)width * height * 3;
    bool ok = std::fwrite(rgb, 1, n, f) == n;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_OK : rt_fail(RT_ERR_IO, "File write error");
}

const char *rt_last_error(void) { return g_last_error.c_str(); }
int32_t rt_abi_version(void) { return RT_ABI_VERSION; }

}  // extern "C"

int64_t rt_shard_rows_impl(int32_t height, int32_t rank, int32_t world, int32_t row_block, int32_t *rows_out) {
    if (height <= 0 || world <= 0 || rank < 0 || rank >= world || row_block <= 0) return rt_fail(RT_ERR_ARG, "rt_shard_rows: bad partition");
    int64_t n = 0;
    for (int32_t r = 0; r < height; ++r)
        if ((r / row_block) % world == rank) {
            if (rows_out) rows_out[n] = r;
            ++n;
        }
    return n;
}
