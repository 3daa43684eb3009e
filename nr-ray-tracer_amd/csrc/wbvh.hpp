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
    int32_t root4 = WBVH_DONE;
    uint32_t stack4 = 0;            // deepest per-lane stack the 4-wide traversal can reach
};

// bounds[i] = {lo.x, lo.y, lo.z, hi.x, hi.y, hi.z} of primitive i (world space, f64);
// cost[i] = its intersection cost relative to a box test (SAH weight).
WorldBvh build_world_bvh(const std::vector<std::array<double, 6>>& bounds, const std::vector<float>& cost);

}  // namespace nrt
