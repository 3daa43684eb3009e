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
};

// bounds[i] = {lo.x, lo.y, lo.z, hi.x, hi.y, hi.z} of primitive i (world space, f64).
WorldBvh build_world_bvh(const std::vector<std::array<double, 6>>& bounds);

}  // namespace nrt
