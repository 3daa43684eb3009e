// Host-side interface to the HIP layer (render.hip).  Plain C++ types only.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "render_params.hpp"

namespace nrt {

struct FlatScene;
struct DeviceScene;

int gpu_device_count();
DeviceScene* gpu_upload_scene(const FlatScene& fs, int device);  // throws std::runtime_error
void gpu_free_scene(DeviceScene* ds);
size_t gpu_scene_bytes(const DeviceScene* ds);
int gpu_scene_device(const DeviceScene* ds);
// Enqueue one render launch on `stream` (nullptr = default stream). p.out is a device pointer.
void gpu_launch_render(const DeviceScene* ds, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                       void* stream);
// f32 kernel mode for nrt_trace `trace`: 0 = world-space list, 1 / MAX_INSTANCE_DEPTH = instance BVH.
int gpu_fast_maxd(const DeviceScene* ds, uint32_t trace);
// First `count` draws of `lanes` consecutive streams starting at stream0 (tests).
struct JitCounts {
    uint64_t compiled, launches, failed, compile_ns;
};
JitCounts gpu_jit_counts();  // scene-specialised kernels (jit.hip)
uint64_t gpu_jit_compile_only(const char* targs, std::string* log);
void gpu_rng_probe(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample, uint64_t* host_out);

}  // namespace nrt
