// Kernel launchers, one translation unit per numeric contract:
//   kernels_exact.hip  (f64, -ffp-contract=off: the reference's un-fused arithmetic)
//   kernels_fast.hip   (f32, -ffp-contract=fast + hardware reciprocals)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "device_scene.hpp"
#include "render_params.hpp"

namespace nrt {

// maxd: instance nesting the kernel supports (1 or MAX_INSTANCE_DEPTH); the
// fast kernel also takes the world-space modes below (DSceneView::wprims).
constexpr int MODE_WORLD_LIST = 0;
constexpr int MODE_WORLD_BVH = -1;
// perlin: the scene has Noise / Marble textures (selects the KF_PERLIN kernel variants);
// flat: no spheres and only solid-colour textures (the KF_FLAT world-list / world-BVH variants)
void launch_exact(const RenderParams& p, const DSceneView<double>& v, uint32_t rng, int maxd, bool perlin,
                  bool planes, hipStream_t stream);
void launch_fast(const RenderParams& p, const DSceneView<float>& v, uint32_t rng, int maxd, bool perlin, bool flat,
                 hipStream_t stream);
// Scenes whose node/prim/xform/material tables fit stay in LDS for the whole launch.
constexpr uint32_t LDS_SCENE_LIMIT = 64 * 1024;

// Scene-specialised f32 kernels (jit.hip; Philox or ChaCha8): render_kernel<targs> built with
// hiprtc, a module function, or nullptr when unavailable (NRT_JIT=0, no hiprtc, a compile
// error); launch_fast_jit enqueues it like launch_fast (maxd: MODE_WORLD_LIST or MODE_WORLD_BVH;
// lds_fixed = the staged scene's bytes, the ChaCha8 ring and the BVH stack are added there).
constexpr size_t JIT_MAX_RUNS = 8;  // world lists with more runs keep the generic loop
struct JitStats {
    uint64_t compiled = 0;    // kernels built by hiprtc in this process
    uint64_t launches = 0;    // renders that used one
    uint64_t failed = 0;      // builds that failed (the generic kernel ran instead)
    uint64_t compile_ns = 0;  // wall time spent in hiprtc + module load
    uint64_t disk_hits = 0;   // code objects read from the on-disk cache instead of compiled
    uint64_t load_retries = 0;  // module loads that failed and were left to a later render
};
void* jit_render_kernel(const std::string& targs, int device);
// throws under NRT_JIT=require (jit.hip): called when jit_render_kernel returned null
void jit_require_failed(const std::string& targs);
JitStats jit_stats();
uint64_t jit_compile_only(const std::string& targs, std::string* log);  // code bytes, 0 on failure (tests)
// stack_entry: bytes per world-BVH stack entry (2 for the compact tree, kernel.hpp StackEntry)
void launch_fast_jit(const RenderParams& p, const DSceneView<float>& v, void* fn, uint32_t lds_fixed, int maxd,
                     uint32_t rng, uint32_t stack_entry, hipStream_t stream);
void launch_rng_probe(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample,
                      unsigned long long* d_out);

}  // namespace nrt
