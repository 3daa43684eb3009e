// Launch parameters of the path-tracing megakernel (host <-> device POD).
#pragma once

#ifndef __HIPCC_RTC__
#include <cstdint>
#endif

namespace nrt {

constexpr uint32_t QUEUE_HEADS = 8;    // one per XCD
constexpr uint32_t QUEUE_STRIDE = 32;  // words: one 128-B line per head


enum : uint32_t { RNG_CHACHA8 = 0, RNG_PHILOX = 1, RNG_PHILOX2_BLOCK = 2 /* nrt_debug_rng only */ };
// f32 Philox render loop: Philox2x32-10 counter (pixel, sample | step << 24), so
// spp <= 2^24 and steps 0..255 (camera 0, scatters 1..max_bounces, defocus 255).
constexpr uint32_t PHILOX2_STEPS = 256, PHILOX2_MAX_SPP = 1u << 24;
constexpr uint32_t PHILOX2_MAX_BOUNCES = PHILOX2_STEPS - 2u;

namespace dev {
// Kernel variant flags (render_kernel's KFLAGS): KF_PROF = phase-profile stamps (diagnostics),
// KF_PERLIN = the scene has Noise / Marble textures, KF_FLAT = world-mode scene without spheres
// whose materials all have solid colours, KF_PLANES = f64 kernel, no spheres, KF_TEXPAL = every
// texture is a solid colour or a PAL16 image (scene-specialised kernels only) (kernel.hpp).
constexpr int KF_PROF = 1, KF_PERLIN = 2, KF_FLAT = 4, KF_PLANES = 8, KF_TEXPAL = 16;
// Exact kernel, small scenes: at most this many slots of the culling tree are tested in slot order
// instead of walked (EXACT_SIG_SLOTS / EXACT_SIG_SLOTS_PF; host default and launcher share it)
constexpr uint32_t EXACT_SLOTS_MAX = 32;
}  // namespace dev

struct RenderParams {
    // Camera after CameraBuilder::build (camera.rs:205-227), always f64 on the host.
    double top_left[3];
    double pixel_delta_u[3];
    double pixel_delta_v[3];
    double look_from[3];
    double defocus_disk_u[3];
    double defocus_disk_v[3];
    double background[3];
    // The same seven vectors rounded to f32 (in this order: top_left, delta_u,
    // delta_v, look_from, disk_u, disk_v, background) for the f32 kernel, so
    // they stay in SGPRs instead of being converted per lane.
    float camf[7][3];
    uint32_t defocus;  // 0: defocus disk is zero (defocus_angle <= 0), disk draws only feed the origin
    uint32_t wave_wait;  // world-BVH mode: lanes that must finish traversal before a shading round
    // Philox mode: pixels per wave (power of two <= 64, wave_pixels * spp < 2^32) and
    // the 2^k grid each sample's radiance is rounded to before the exact f64 sum.
    uint32_t wave_pixels, wave_pixels_log2;
    double acc_scale, acc_unscale;  // 2^k, 2^-k
    uint32_t groups;                // Philox: pixel groups (of wave_pixels) in this launch
    // Philox: QUEUE_HEADS group-queue heads, QUEUE_STRIDE words apart (device, zeroed
    // before the launch); head x hands out the x-th contiguous eighth of the groups
    // (kernel.hpp, Philox branch).  ChaCha8: word 0 counts the pixels handed out past the
    // grid's first round (persistent lanes).
    unsigned int* queue;
    uint32_t width, height;
    uint32_t spp;
    uint32_t max_bounces;
    // Rows rendered by this launch: y = row_offset + k * row_stride, k in [0, rows).
    uint32_t row_offset, row_stride, rows;
    // Pixel range inside the local (rows x width) buffer handled by this launch.
    uint32_t pixel_begin, pixel_end;
    float* out;  // rows * width * 3 floats, row-major (Rgb32FImage layout)
    // Optional per-launch work counters (nullptr = off): see render.hip.
    unsigned long long* counters;
    // Exact kernel, small scenes: test every primitive of the reference tree in its depth-first
    // order instead of culling with the boxes (every lane walks the same node sequence, so the
    // traversal does not diverge; the closest hit and its tie-break are the reference's).
    uint32_t exact_all;
    // Exact kernel, large scenes with a world BVH whose primitives map onto the exact tree
    // (DSceneView::wexact): the f32 world BVH culls, the reference tests decide (kernel.hpp
    // trace_exact_wbvh).
    uint32_t exact_wbvh;
    // Exact world mode, plane-only scenes (KF_PLANES): an f32 prefilter with error bounds picks
    // the candidates of the world-BVH walk, and only those get the reference tests (kernel.hpp
    // trace_exact_wbvh_pf).
    uint32_t exact_pf;
    // Exact world mode: the stackless threaded walk of the culling tree (kernel.hpp xthread_walk)
    // instead of the 4-wide walk with a private stack.
    uint32_t exact_thread;
    // Exact world mode on the compact tree: its traversal stack in LDS (16-bit entries) and
    // 3 waves per SIMD (default), or a private (scratch) stack at 4 (ExactSig lstack).
    uint32_t exact_lstack;
    // Exact world mode with the prefilter, at most EXACT_SLOTS_MAX slots: the prefilter over every
    // slot in order (scalar loads, no walk) instead of the culling walk (EXACT_SIG_SLOTS_PF).
    uint32_t exact_slots;
    // Persistent lanes (ChaCha8): fewest pixels a wave claims per counter atomic while its queue head
    // has more than one round of the grid's lanes left (then as many as lanes ask); the rest wait in
    // the wave's reservoir (kernel.hpp next_pixel).  0: the host picks (render.hip).
    uint32_t exact_claim;
    // Persistent lanes: a claim's finished pixels staged in LDS and written out as one run (1), or each
    // pixel stored as it ends (0).  The host stages only where the staging LDS leaves the resident
    // workgroups unchanged (launch_impl.hpp).
    uint32_t exact_stage;
    float acc_scale_f;  // acc_scale in f32 (f32 kernels: k in [-126, 127])
    // Philox group sizing (launch_impl.hpp philox_launch): groups per resident wave a launch keeps
    // while groups hold > 512 samples; 0 = NRT_GROUPS_PER_WAVE (4, for streamed launches whose tail the
    // next launch fills: nrt_render_device); nrt_render, a one-shot call, asks for 16 (smaller last
    // groups shorten a lone launch's tail)
    uint32_t groups_per_wave;
};

}  // namespace nrt
