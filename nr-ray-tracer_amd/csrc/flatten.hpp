// Host-side flattening of the scene graph into the HBM layout of device_scene.hpp.
#pragma once

#include <string>
#include <vector>

#include "device_scene.hpp"
#include "scene.hpp"
#include "wbvh.hpp"

namespace nrt {

struct FlatScene {
    std::vector<DNode<double>> nodes;       // exact kernel: the reference's BVH node for node
    std::vector<DNode<double>> nodes_fast;  // fast kernel: small prim-only subtrees -> NODE_LIST
    std::vector<DPrimFast<double>> fprims;  // fast kernel primitives, list order
    std::vector<DMatFast> mats_fast;
    std::vector<DInstFast<double>> inst_fast;
    int32_t root_fast = NODE_END;
    std::vector<DPrim<double>> prims;
    std::vector<DXform<double>> xforms;
    std::vector<DInstance> instances;
    std::vector<DMaterial> materials;
    std::vector<DTexture> textures;
    std::vector<uint32_t> texels;  // 32-bit words (device_scene.hpp DTexture: TEXFMT_*, permutation tables)
    uint64_t texel_count = 0;       // image texels over all image textures
    int32_t root = NODE_END;
    int32_t max_depth = 0;
    uint32_t num_trees = 0;
    // World-space primitives in the reference's depth-first candidate order
    // (device_scene.hpp DPrimWorld); world_ok = every primitive qualifies.
    std::vector<DPrimWorld<double>> wprims;
    std::vector<uint32_t> wruns;  // kind | count << WKIND_BITS over world units
    uint64_t world_units = 0;     // primitives + fused boxes: the world list's test count
    uint32_t wflags = 0;          // WFLAG_* of the world list
    bool world_ok = false;
    bool list_ok = true;          // the world list reproduces every coplanar tie (flatten.cpp tie forms)
    uint32_t coplanar_pairs = 0;  // overlapping coplanar primitive pairs (device_scene.hpp WCLASS_*)
    // World BVH over the (unfused) world primitives, for large flattenable scenes.
    WorldBvh wbvh;
    std::vector<DPrimWorld<double>> wbvh_prims;  // BVH leaf order
    bool wbvh_ok = false;      // the tree is built (the exact kernel's culling walk may use it)
    bool wbvh_f32_ok = false;  // ... and the f32 world-BVH kernels may: every sphere anchored within the scene
    // Exact kernel's world-BVH mode: the tree it culls with and the exact reference of each of
    // its slots (device_scene.hpp DExactRef), when every world primitive maps onto the exact
    // tree's depth-first walk (instances not nested).  Scenes whose primitives sit under
    // several instance chains get a tree of their own built with the primitive weight
    // EXACT_SAH_PRIM_COST (an exact test, and the instance switch before it, cost several
    // node visits: Cornell 244 -> 226 ms); otherwise wbvh_x stays empty and wbvh is shared.
    WorldBvh wbvh_x;
    std::vector<DExactRef> wexact;
    std::vector<DPrimWorld<double>> wexact_prims;  // world primitive of each exact-tree slot (prefilter)
    std::vector<uint32_t> wprims_kind;  // kind of each world primitive (depth-first rank)
    const WorldBvh& exact_tree() const { return wbvh_x.order.empty() ? wbvh : wbvh_x; }
};

FlatScene flatten_scene(const ObjectPtr& top_level_bvh);

// Precision conversion for the fast kernel.  Boxes are rounded outward so an
// f32 box always contains the f64 one.
struct FlatScene32 {
    std::vector<DNode<float>> nodes;  // from nodes_fast
    std::vector<DPrim<float>> prims;
    std::vector<DXform<float>> xforms;
    std::vector<DInstFast<float>> inst_fast;
    std::vector<DPrimFast<float>> fprims;
    std::vector<DPrimWorld<float>> wprims;
    std::vector<DPrimWorld<float>> wbvh_prims;
    std::vector<DPrimWorld<float>> wexact_prims;
};
FlatScene32 to_f32(const FlatScene& s);

// Canonical text form of the scene graph (used by the parity tests to compare
// the C++ loader + BVH builder against the oracle's independent build).
std::string dump_graph(const ObjectPtr& root);

}  // namespace nrt
