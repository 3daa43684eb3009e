// Shared launch helper (included by each kernels_*.hip translation unit).
#pragma once

#include <stdexcept>

#include "kernel.hpp"

namespace nrt {

// Scenes whose node/prim/xform/material tables fit stay in LDS for the whole launch.
constexpr uint32_t LDS_SCENE_LIMIT = 64 * 1024;

template <typename R, class G, int MAXD, bool EXACT>
static void launch_one(const RenderParams& p, const DSceneView<R>& v, hipStream_t stream) {
    const uint32_t n = (p.pixel_end - p.pixel_begin) * (G::exact_stream ? 1u : p.split);  // lanes
    const uint32_t blocks = (n + dev::BLOCK - 1) / dev::BLOCK;
    const uint32_t ring = (G::uses_lds ? dev::RING * dev::BLOCK * (uint32_t)sizeof(uint2) : 0) +
                          (MAXD < 0 ? WBVH_STACK * dev::BLOCK * (uint32_t)sizeof(int32_t) : 0);  // + BVH stack
    const uint32_t scene = lds_scene_bytes(v);
    if (p.counters) {  // diagnostic phase profile (nrt_debug_phase_profile)
        if constexpr (MAXD > 1) {
            throw std::runtime_error("phase profile: flat-instance scenes only");
        } else if (scene <= LDS_SCENE_LIMIT) {
            hipLaunchKernelGGL((dev::render_kernel<R, G, MAXD, EXACT, true, true>), dim3(blocks), dim3(dev::BLOCK),
                               ring + scene, stream, p, v);
        } else {
            hipLaunchKernelGGL((dev::render_kernel<R, G, MAXD, EXACT, false, true>), dim3(blocks), dim3(dev::BLOCK),
                               ring, stream, p, v);
        }
    } else if (scene <= LDS_SCENE_LIMIT) {
        hipLaunchKernelGGL((dev::render_kernel<R, G, MAXD, EXACT, true>), dim3(blocks), dim3(dev::BLOCK), ring + scene,
                           stream, p, v);
    } else {
        hipLaunchKernelGGL((dev::render_kernel<R, G, MAXD, EXACT, false>), dim3(blocks), dim3(dev::BLOCK), ring,
                           stream, p, v);
    }
}

}  // namespace nrt
