// World-space BVH of the f32 kernel (device_scene.hpp DBvhNode): binned SAH.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "device_scene.hpp"

namespace nrt {

struct WorldBvh {
    std::vector<DBvhNode> nodes;  // f32, boxes rounded outward and padded
    std::vector<uint32_t> order;  // BVH prim slot -> input primitive index
    int32_t root = WBVH_DONE;     // child ref of the root (a leaf for tiny inputs)
    uint32_t depth = 0;           // deepest inner-node level (stack bound)
    std::vector<DBvh4Node> nodes4;  // the same tree collapsed to 4-wide nodes
    std::vector<DBvh4cNode> nodes4c;  // nodes4 in the compact form (empty when a limit is exceeded)
    int32_t root4 = WBVH_DONE;
    uint32_t stack4 = 0;            // deepest per-lane stack the 4-wide traversal can reach
    std::vector<DThreadNode> threaded;  // 8 octant copies of the threaded binary tree (n each)
    uint32_t threaded_n = 0;
    double scale = 0.0;             // largest |coordinate| of the primitives' boxes: boxes are padded by
                                    // 1e-6 of it, which covers the f32 slab error of ray origins
                                    // within that range (the exact world mode's culling, kernel.hpp)
};

// bounds[i] = {lo.x, lo.y, lo.z, hi.x, hi.y, hi.z} of primitive i (world space, f64);
// cost[i] = its intersection cost relative to a box test (SAH weight); leaves hold at most
// leaf_max (<= WBVH_LEAF_MAX) primitives.
WorldBvh build_world_bvh(const std::vector<std::array<double, 6>>& bounds, const std::vector<float>& cost,
                         uint32_t leaf_max = WBVH_LEAF_MAX);

}  // namespace nrt
