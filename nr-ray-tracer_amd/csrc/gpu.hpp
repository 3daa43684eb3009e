// Host-side interface to the HIP layer (render.hip).  Plain C++ types only.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "render_params.hpp"

namespace nrt {

struct FlatScene;
struct DeviceScene;
struct MultiRender;

// Multi-GPU render in one process (multi.hip): scenes[d] on device first + d (consecutive), one
// RCCL communicator per device (ncclCommInitAll), rows y = d (mod N) on device d, one ncclGather
// to the first device and a row un-permute there.  p is the full-frame RenderParams.  loopback
// (tests): every scenes[d] is on the first device and the gather is device-to-device copies.
MultiRender* gpu_multi_create(const std::vector<DeviceScene*>& scenes, bool loopback);  // throws
bool gpu_multi_rccl_usable(std::string* why);
void gpu_multi_prepare(MultiRender* m, uint32_t width, uint32_t height);  // shard / staging buffers now  // librccl loadable with ncclGather / ncclCommInitAll
void gpu_multi_free(MultiRender* m);
int gpu_multi_first(const MultiRender* m);
int gpu_multi_count(const MultiRender* m);
// asynchronous: dev_out (first device) is written after `stream`'s prior work, and `stream` waits for it
void gpu_multi_render_device(MultiRender* m, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                             float* dev_out, void* stream);
// synchronous: the frame lands in host memory
void gpu_multi_render_host(MultiRender* m, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                           float* host_out);
// HIP-event times (ms) of the last frame: out[d] = device first + d's render kernel, out[N] = the
// gather + un-permute on the first device, out[N + 1] = the device time per frame since the previous
// call: the first device's render start of the window's first frame to the last frame's completion,
// over the frames (0 with fewer than two); a call that writes out[N + 1] starts a new window; returns N + 2
size_t gpu_multi_timings(MultiRender* m, float* out, size_t n);

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
    uint64_t compiled, launches, failed, compile_ns, disk_hits, load_retries;
};
JitCounts gpu_jit_counts();  // scene-specialised kernels (jit.hip)
uint64_t gpu_jit_compile_only(const char* targs, std::string* log);
void gpu_rng_probe(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample, uint64_t* host_out);

}  // namespace nrt
