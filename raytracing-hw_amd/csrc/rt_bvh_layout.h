// rt_bvh_layout.h — host-side builders of the device copies of the scene BVH.
//
// Input: the node array as the loader builds it (BVH::buildBVH order, bvh.cpp:5-175),
// 8 words per node: min.xyz, max.xyz, a, b (internal: a = left child, right = a + 1,
// b = split axis < 3; leaf: a = first triangle, b = count << 2 | 3).
//
//   bfs_nodes   same records renumbered breadth-first: siblings stay adjacent and the top
//               levels become a prefix (the levels nearly every ray visits share lines).
// Visits, counters and results do not depend on node numbering.
#pragma once
#include <cstdint>
#include <cstring>
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

}  // namespace rtd
