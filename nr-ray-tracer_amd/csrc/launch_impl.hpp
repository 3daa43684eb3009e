// Shared launch helper (included by each kernels_*.hip translation unit).
#pragma once

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <tuple>

#include "kernel.hpp"
#include "launch.hpp"

namespace nrt {


// ChaCha8 persistent lanes: a cap on the grid (knob NRT_CHACHA_GRID, tests: a small grid hands out
// most pixels through the per-XCD counters; the frame must not change).
inline uint64_t chacha_grid_cap() {
    const char* e = std::getenv("NRT_CHACHA_GRID");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return v > 0 ? (uint64_t)v : ~0ull;
}

// Blocks the device keeps resident for a kernel (static or a module function) with `lds_bytes` of
// dynamic LDS, cached per (device, kernel, LDS): the occupancy queries cost the host tens of
// microseconds per launch, which a short launch (a row shard at N = 8) waits for on the GPU.
template <class Query>
static uint64_t cached_resident(const void* kernel, uint32_t lds_bytes, Query&& query) {
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, uint32_t>, uint64_t> cache;
    int dev_id = 0;
    if (hipGetDevice(&dev_id) != hipSuccess) throw std::runtime_error("hipGetDevice failed");
    const auto key = std::make_tuple(dev_id, kernel, lds_bytes);
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int per_cu = 0, cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id) != hipSuccess ||
        !query(&per_cu) || per_cu <= 0 || cus <= 0)
        throw std::runtime_error("occupancy query failed for the render kernel");
    const uint64_t n = (uint64_t)per_cu * (uint64_t)cus;
    std::lock_guard<std::mutex> lock(mu);
    cache[key] = n;
    return n;
}
template <typename K>
static uint64_t resident_blocks(K kernel, uint32_t lds_bytes) {
    return cached_resident((const void*)kernel, lds_bytes, [&](int* per_cu) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kernel, dev::BLOCK, lds_bytes) == hipSuccess;
    });
}

// Philox: persistent waves (as many blocks as stay resident, capped by the group
// count) over groups of P pixels.  Unless fixed (NRT_WAVE_PIXELS), P is the
// smallest power of two with >= 1024 samples per group (a group must outlast the
// longest path in flight for the ring of two to keep lanes busy; small groups keep
// a wave's rays on few pixels), halved while the launch has fewer than two groups
// per resident wave (or fewer than NRT_GROUPS_PER_WAVE while groups keep > 512 samples).
// `resident(lds)` = blocks the device keeps resident with `lds` bytes of dynamic LDS,
// `launch(blocks, lds, params)` enqueues the kernel (a static instantiation or a
// scene-specialised module function, jit.hip).
#ifndef NRT_GROUPS_PER_WAVE
#define NRT_GROUPS_PER_WAVE 4  // (16 before frames were pipelined: with the next launch filling the SIMDs a
                               // launch's last groups leave idle, larger groups win: row shards of C5 at
                               // N = 4 / 8 2.588 -> 2.566 / 1.336 -> 1.333 ms, full frames unchanged)
#endif
template <int MAXD, class Resident, class Launch>
static void philox_launch(const RenderParams& p0, uint32_t lds_fixed, Resident&& resident, Launch&& launch) {
    const uint32_t npix = p0.pixel_end - p0.pixel_begin;
    RenderParams p = p0;
    auto ring_bytes = [](uint32_t wp) { return dev::philox_pool_bytes<MAXD>(wp); };
    uint32_t wp = p.wave_pixels;
    if (!wp) {
        // world-BVH kernels (MAXD < 0) take at least 8 pixels per group: their ring of four slots turns
        // over less often (the teapot at spp 256: 4 / 8 / 16 / 32 pixels 30.87 / 30.00 / 29.93 / 32.04 ms;
        // the spheres at spp 64 keep 16: 32 measured 27.05 against 26.77 ms; world lists keep 1024 samples)
        constexpr uint32_t min_px = MAXD < 0 ? 8u : 1u;
        wp = 1;
        while (wp < 64 && ((uint64_t)wp * p.spp < 1024 || wp < min_px)) wp <<= 1;
        const uint64_t w0 = resident(lds_fixed + ring_bytes(wp)) * (dev::BLOCK / 64);
        // halve while the launch has fewer than two groups per resident wave, or
        // (down to 512 samples per group) fewer than NRT_GROUPS_PER_WAVE: the last groups to
        // finish set the tail of a lone launch (C5 at N = 8 without pipelining: 4.6 -> 9.1
        // groups per wave, -5 % kernel time, round 3); pipelined launches overlap that tail
        auto groups = [&](uint32_t w) { return (uint64_t)(npix + w - 1) / w; };
        uint64_t gpw = p.groups_per_wave ? p.groups_per_wave : NRT_GROUPS_PER_WAVE;  // knob NRT_GROUPS_PER_WAVE (A/B runs)
        if (const char* e = std::getenv("NRT_GROUPS_PER_WAVE")) {
            const long v = std::strtol(e, nullptr, 10);
            if (v >= 1 && v <= 64) gpw = (uint64_t)v;
        }
        while (wp > 1 && (groups(wp) < 2 * w0 || ((uint64_t)wp * p.spp > 512 && groups(wp) < gpw * w0))) wp >>= 1;
    }
    const uint64_t waves_res = resident(lds_fixed + ring_bytes(wp)) * (dev::BLOCK / 64);
    p.wave_pixels = wp;
    p.wave_pixels_log2 = 0;
    while ((1u << p.wave_pixels_log2) < wp) ++p.wave_pixels_log2;
    p.groups = (npix + wp - 1) / wp;
    const uint64_t need = ((uint64_t)p.groups + dev::BLOCK / 64 - 1) / (dev::BLOCK / 64);
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min(waves_res / (dev::BLOCK / 64), need));
    launch(blocks, lds_fixed + ring_bytes(wp), p);
}

// Persistent lanes: the claim staging (RenderParams::exact_stage) only where its LDS leaves the
// resident workgroups unchanged.  C4 f64 (teapot: the 16-bit culling stack in LDS, 3 workgroups per CU)
// lost one workgroup per CU to it: claims of 2 / 4 pixels measured 130.7 -> 153 ms in round 5, the
// occupancy, not the claims.  `lds` includes the staging when p.exact_stage is set; both are updated.
template <class Resident>
static void exact_stage_fit(RenderParams& p, uint32_t& lds, Resident&& resident) {
    const bool dbg = std::getenv("NRT_DEBUG_LAUNCH") != nullptr;  // (diagnostics: the launch's LDS and residency)
    if (p.exact_stage) {
        const uint32_t without = lds - dev::STG_LDS_BYTES;
        const uint64_t with_b = resident(lds), without_b = resident(without);
        if (dbg)
            std::fprintf(stderr, "nrt: persistent lanes: LDS %u B -> %llu blocks resident, without claim staging %u B -> %llu\n",
                         lds, (unsigned long long)with_b, without, (unsigned long long)without_b);
        if (without_b > with_b) {
            p.exact_stage = 0;
            lds = without;
        }
    } else if (dbg) {
        std::fprintf(stderr, "nrt: persistent lanes: LDS %u B -> %llu blocks resident (no claim staging)\n", lds,
                     (unsigned long long)resident(lds));
    }
}

// ChaCha8: one lane per pixel.
template <typename R, class G, int MAXD, bool EXACT, bool LDS_SCENE, int KFLAGS, class SIG = dev::NoSig>
static void launch_variant(const RenderParams& p0, const DSceneView<R>& v, uint32_t lds_fixed, hipStream_t stream) {
    auto kernel = dev::render_kernel<R, G, MAXD, EXACT, LDS_SCENE, KFLAGS, SIG>;
    const uint32_t npix = p0.pixel_end - p0.pixel_begin;
    if constexpr (G::exact_stream) {  // persistent lanes (render_kernel): the resident workgroups at most
        RenderParams p = p0;
        uint32_t lds = lds_fixed;
        exact_stage_fit(p, lds, [&](uint32_t b) { return resident_blocks(kernel, b); });
        const uint64_t need = (npix + dev::BLOCK - 1) / dev::BLOCK;
        const uint64_t blocks = std::max<uint64_t>(1, std::min({need, resident_blocks(kernel, lds), chacha_grid_cap()}));
        hipLaunchKernelGGL(kernel, dim3((uint32_t)blocks), dim3(dev::BLOCK), lds, stream, p, v);
    } else {
        philox_launch<MAXD>(
            p0, lds_fixed, [&](uint32_t lds) { return resident_blocks(kernel, lds); },
            [&](uint32_t blocks, uint32_t lds, const RenderParams& p) {
                hipLaunchKernelGGL(kernel, dim3(blocks), dim3(dev::BLOCK), lds, stream, p, v);
            });
    }
}

template <typename R, class G, int MAXD, bool EXACT>
static void launch_one(const RenderParams& p, const DSceneView<R>& v, bool perlin, hipStream_t stream,
                       bool flat = false, bool planes = false) {
    // dynamic LDS below the staged scene: ChaCha8 ring or Philox group ring (added by
    // launch_variant), then the BVH stack
    const uint32_t ring = (G::uses_lds ? dev::chacha_lds_bytes(p.exact_stage) : 0) +
                          (MAXD < 0 ? (v.wbvh_stack + 1u) * dev::BLOCK * (uint32_t)sizeof(int32_t) : 0);
    const uint32_t scene = lds_scene_bytes(v, MAXD);
    using dev::KF_FLAT;
    using dev::KF_PERLIN;
    using dev::KF_PROF;
    constexpr bool FLAT_MODE = MAXD <= 0 && sizeof(R) == 4;  // KF_FLAT: f32 world list / world BVH
    if constexpr (FLAT_MODE) {
        if (flat && !perlin) {  // the phase profile measures this same variant
            if (p.counters) {
                if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, KF_PROF | KF_FLAT>(p, v, ring + scene, stream);
                else launch_variant<R, G, MAXD, EXACT, false, KF_PROF | KF_FLAT>(p, v, ring, stream);
            } else if (scene <= LDS_SCENE_LIMIT) {
                launch_variant<R, G, MAXD, EXACT, true, KF_FLAT>(p, v, ring + scene, stream);
            } else {
                launch_variant<R, G, MAXD, EXACT, false, KF_FLAT>(p, v, ring, stream);
            }
            return;
        }
    }
    if constexpr (sizeof(R) == 8 && MAXD == 1 && G::exact_stream) {
        if (!planes && !perlin && !p.counters && p.exact_wbvh && p.exact_slots && v.n_wexact <= dev::EXACT_SLOTS_MAX) {
            // small scenes with spheres: the reference tests on every slot, no walk compiled in
            // (the reference node array is never read: not staged)
            DSceneView<R> vw = v;
            vw.n_nodes = 0;
            vw.n_xstage = 0;  // (no walk)
            const uint32_t scene = lds_scene_bytes(vw, MAXD);
            using XS = dev::ExactSig<dev::EXACT_SIG_SLOTS, 0>;
            if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, 0, XS>(p, vw, ring + scene, stream);
            else launch_variant<R, G, MAXD, EXACT, false, 0, XS>(p, vw, ring, stream);
            return;
        }
#ifndef NRT_EXACT_PROF
#define NRT_EXACT_PROF 0  // diagnostic builds: the phase profile (p.counters) of the LDS-stack planes variant
#endif
        if (!planes && !perlin && !p.counters && p.exact_wbvh && !p.exact_all && !p.exact_thread && v.wbvh4c &&
            p.exact_lstack && !(p.exact_slots && v.n_wexact <= dev::EXACT_SLOTS_MAX)) {
            // larger scenes with spheres (spheres.toml): the unfiltered world walk on the compact tree with
            // its stack in LDS (the generic kernel's walk keeps a 32-bit stack in scratch)
            using XW = dev::ExactSig<dev::EXACT_SIG_WORLD, WBVH_COMPACT, true>;
            DSceneView<R> vw = v;
            vw.n_nodes = 0;  // (the world walk never reads the reference node array)
            const uint32_t scene = lds_scene_bytes(vw, MAXD);
            const uint32_t stk = (vw.wbvh_stack + 1u) * dev::BLOCK * (uint32_t)sizeof(uint16_t);
            const char* pe = std::getenv("NRT_EXACT_PERSIST");
            if (!(pe && pe[0] == '0')) {  // the walk kept across shading rounds (XWalkU)
                using XWP = dev::ExactSig<dev::EXACT_SIG_WORLD, WBVH_COMPACT, true, true>;
                RenderParams q = p;
                if (!q.wave_wait) q.wave_wait = 56u;
                if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, 0, XWP>(q, vw, ring + stk + scene, stream);
                else launch_variant<R, G, MAXD, EXACT, false, 0, XWP>(q, vw, ring + stk, stream);
                return;
            }
            if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, 0, XW>(p, vw, ring + stk + scene, stream);
            else launch_variant<R, G, MAXD, EXACT, false, 0, XW>(p, vw, ring + stk, stream);
            return;
        }
        if (planes && !perlin && (!p.counters || NRT_EXACT_PROF)) {  // KF_PLANES: the 4-wave f64 variant
            if (p.exact_wbvh && p.exact_pf && !p.exact_all) {  // the prefiltered world walk only
                // (the world walk never reads the reference node array: not staged, 2.4 KB of
                // LDS for the Cornell box)
                DSceneView<R> vw = v;
                vw.n_nodes = 0;
                const uint32_t scene = lds_scene_bytes(vw, MAXD);
                if (p.exact_thread && vw.xthread) {  // the stackless threaded walk
                    using XT = dev::ExactSig<dev::EXACT_SIG_WORLD_PF, dev::XTHREAD_W>;
                    if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XT>(p, vw, ring + scene, stream);
                    else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XT>(p, vw, ring, stream);
                    return;
                }
                if (p.exact_slots && vw.n_wexact <= dev::EXACT_SLOTS_MAX) {  // small scenes: every slot, no walk
                    // (the slot records arrive by scalar loads from global memory: not staged)
                    vw.n_xstage = 0;
                    const uint32_t scene = lds_scene_bytes(vw, MAXD);
                    using XA = dev::ExactSig<dev::EXACT_SIG_SLOTS_PF, 0>;
                    if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XA>(p, vw, ring + scene, stream);
                    else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XA>(p, vw, ring, stream);
                    return;
                }
                if (vw.wbvh4c && p.exact_lstack) {  // the compact walk's stack in LDS, 3 waves per SIMD
                    using XL = dev::ExactSig<dev::EXACT_SIG_WORLD_PF, WBVH_COMPACT, true>;
                    const uint32_t stk = (vw.wbvh_stack + 1u) * dev::BLOCK * (uint32_t)sizeof(uint16_t);
                    // the walk kept across shading rounds (XWalk; knob NRT_EXACT_PERSIST=0: one walk per segment)
                    const char* pe = std::getenv("NRT_EXACT_PERSIST");
                    const bool persist = !(pe && pe[0] == '0');
                    if (persist) {
                        using XP = dev::ExactSig<dev::EXACT_SIG_WORLD_PF, WBVH_COMPACT, true, true>;
                        // shading rounds at 40 walks done (the teapot: 40 / 48 / 64 measured 132 / 132-133 /
                        // 147 ms, 16 / 32 164 / 145 ms, one walk per segment 169 ms); small staged trees (the
                        // Cornell box: short walks) at 64, a while-while walk in trips (182 vs 186 ms; 48: 190)
                        RenderParams q = p;
                        if (!q.wave_wait) q.wave_wait = vw.n_xstage ? 64u : 40u;
#if NRT_EXACT_PROF
                        if (q.counters) {
                            if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES | KF_PROF, XP>(q, vw, ring + stk + scene, stream);
                            else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES | KF_PROF, XP>(q, vw, ring + stk, stream);
                            return;
                        }
#endif
                        if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XP>(q, vw, ring + stk + scene, stream);
                        else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XP>(q, vw, ring + stk, stream);
                        return;
                    }
#if NRT_EXACT_PROF
                    if (p.counters) {
                        if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES | KF_PROF, XL>(p, vw, ring + stk + scene, stream);
                        else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES | KF_PROF, XL>(p, vw, ring + stk, stream);
                        return;
                    }
#endif
                    if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XL>(p, vw, ring + stk + scene, stream);
                    else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XL>(p, vw, ring + stk, stream);
                    return;
                }
                if (vw.wbvh4c) {  // the compact tree: 16-bit stack entries (half the scratch bytes)
                    using XC = dev::ExactSig<dev::EXACT_SIG_WORLD_PF, WBVH_COMPACT>;
                    if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XC>(p, vw, ring + scene, stream);
                    else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XC>(p, vw, ring, stream);
                    return;
                }
                // (tree width left to the run time: fixing it measured C5 -0.3 %, C4 +2.8 %)
                using XS = dev::ExactSig<dev::EXACT_SIG_WORLD_PF, 0>;
                if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES, XS>(p, vw, ring + scene, stream);
                else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES, XS>(p, vw, ring, stream);
                return;
            }
            if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, dev::KF_PLANES>(p, v, ring + scene, stream);
            else launch_variant<R, G, MAXD, EXACT, false, dev::KF_PLANES>(p, v, ring, stream);
            return;
        }
    }
    if (p.counters) {  // diagnostic phase profile (nrt_debug_phase_profile)
        if constexpr (MAXD > 1) {
            throw std::runtime_error("phase profile: flat-instance scenes only");
        } else if (perlin) {
            throw std::runtime_error("phase profile: scenes without Perlin textures only");
        } else if (scene <= LDS_SCENE_LIMIT) {
            launch_variant<R, G, MAXD, EXACT, true, KF_PROF>(p, v, ring + scene, stream);
        } else {
            launch_variant<R, G, MAXD, EXACT, false, KF_PROF>(p, v, ring, stream);
        }
    } else if (perlin) {
        if (scene <= LDS_SCENE_LIMIT) launch_variant<R, G, MAXD, EXACT, true, KF_PERLIN>(p, v, ring + scene, stream);
        else launch_variant<R, G, MAXD, EXACT, false, KF_PERLIN>(p, v, ring, stream);
    } else if (scene <= LDS_SCENE_LIMIT) {
        launch_variant<R, G, MAXD, EXACT, true, 0>(p, v, ring + scene, stream);
    } else {
        launch_variant<R, G, MAXD, EXACT, false, 0>(p, v, ring, stream);
    }
}

}  // namespace nrt
