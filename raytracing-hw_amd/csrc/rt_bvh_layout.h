// rt_bvh_layout.h — host-side builders of the device copies of the scene BVH.
//
// Input: the node array as the loader builds it (BVH::buildBVH order, bvh.cpp:5-175),
// 8 words per node: min.xyz, max.xyz, a, b (internal: a = left child, right = a + 1,
// b = split axis < 3; leaf: a = first triangle, b = count << 2 | 3).
//
//   bfs_nodes   same records renumbered breadth-first: siblings stay adjacent, the top
//               levels become a prefix (rt_wavefront.h LdsNodes), and the children pairs of
//               two sibling internal nodes are adjacent pairs (used by wide_nodes).
//   wide_nodes  the breadth-first records with the two index words repacked so that a
//               node also says where its near child's children are (rt_trav_wide.h):
//                 word 6  ab = a << 10 | b              (the node itself, one word)
//                 word 7  c  = g << 2 | R internal << 1 | L internal
//               g = the child pair of the first internal child among (L, R); by the
//               breadth-first order the right child's pair is g + 2 when both are internal.
// Visits, counters and results do not depend on node numbering.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace rtd {

inline uint32_t node_word(const std::vector<float> &n, size_t id, int w) {
    uint32_t x;
    std::memcpy(&x, &n[8 * id + w], 4);
    return x;
}

inline std::vector<float> bfs_nodes(const std::vector<float> &node) {
    const size_t n = node.size() / 8;
    std::vector<float> out(node.size());
    if (n == 0) return out;
    std::vector<uint32_t> order;   // old ids in new order
    order.reserve(n);
    order.push_back(0);
    std::vector<uint32_t> new_id(n, 0);
    for (size_t h = 0; h < order.size(); ++h) {
        const uint32_t u = order[h];
        if (node_word(node, u, 7) < 3u) {
            const uint32_t a = node_word(node, u, 6);
            new_id[a] = (uint32_t)order.size();
            order.push_back(a);
            new_id[a + 1] = (uint32_t)order.size();
            order.push_back(a + 1);
        }
    }
    for (size_t k = 0; k < order.size(); ++k) {
        const uint32_t u = order[k];
        std::memcpy(&out[8 * k], &node[8 * u], 8 * sizeof(float));
        if (node_word(node, u, 7) < 3u) {
            const uint32_t na = new_id[node_word(node, u, 6)];
            std::memcpy(&out[8 * k + 6], &na, 4);
        }
    }
    return out;
}

// `bfs` must come from bfs_nodes.  Throws std::length_error past the packing limits
// (2^22 nodes / triangles, 255 triangles per leaf: the same limits as the 8-byte frames).
inline std::vector<float> wide_nodes(const std::vector<float> &bfs) {
    const size_t n = bfs.size() / 8;
    std::vector<float> out(bfs);
    for (size_t k = 0; k < n; ++k) {
        const uint32_t a = node_word(bfs, k, 6), b = node_word(bfs, k, 7);
        if (a >= (1u << 22) || b >= 1024u) throw std::length_error("wide_nodes: BVH exceeds the 22/10-bit packing");
        const uint32_t ab = a << 10 | b;
        uint32_t c = 0;
        if (b < 3u) {
            const bool li = node_word(bfs, a, 7) < 3u, ri = node_word(bfs, a + 1, 7) < 3u;
            const uint32_t gl = li ? node_word(bfs, a, 6) : 0u, gr = ri ? node_word(bfs, a + 1, 6) : 0u;
            if (li && ri && gr != gl + 2) throw std::logic_error("wide_nodes: children pairs not adjacent");
            const uint32_t g = li ? gl : gr;
            c = g << 2 | (ri ? 2u : 0u) | (li ? 1u : 0u);
        }
        std::memcpy(&out[8 * k + 6], &ab, 4);
        std::memcpy(&out[8 * k + 7], &c, 4);
    }
    return out;
}

}  // namespace rtd
