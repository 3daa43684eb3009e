// MI355X (gfx950) renderer: kernels live in kernel.hpp; this TU instantiates
// them and holds the host side (device buffers, launches).  No torch types.
#include <hip/hip_runtime.h>

#include <atomic>

#include "launch.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "flatten.hpp"
#include "gpu.hpp"
#include "nrt.h"

// =====================================================================
// Host side: device buffers and launches (no torch types, plain HIP).
// =====================================================================
namespace nrt {

namespace {

void check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

template <typename T>
T* upload(const std::vector<T>& v, const char* what) {
    if (v.empty()) return nullptr;
    T* d = nullptr;
    check(hipMalloc((void**)&d, v.size() * sizeof(T)), what);
    check(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), what);
    return d;
}

}  // namespace

struct DeviceScene {
    int device = -1;
    DSceneView<double> v64{};
    DSceneView<float> v32{};
    std::vector<void*> allocations;
    size_t bytes = 0;
    bool world_ok = false;  // fast kernel may run in world-space mode (v32.wprims)
    bool list_ok = false;   // ... in world-list mode (coplanar ties resolved by order)
    uint64_t world_units = 0;
    bool wbvh_ok = false;   // world BVH available (v32.wbvh + wbvh_prims)
    bool perlin = false;    // Noise / Marble textures present (KF_PERLIN kernel variants)
    bool planes = false;    // no spheres (the f64 kernel's KF_PLANES variant)
    bool flat = false;      // world list without spheres, solid colours only (KF_FLAT variants)
    bool texpal = false;    // every texture a solid colour or a PAL16 image (KF_TEXPAL, scene-specialised kernels)
    const DPrimWorld<float>* wbvh_prims = nullptr;
    uint32_t n_wbvh_prims = 0;
    int wbvh_kinds = 0;  // WPRIMS_* of the world BVH's leaves (the scene-specialised kernel's BvhSig)
    std::vector<uint32_t> wruns;  // the world list's run words (scene-specialised kernel, jit.hip)
    // Philox group-queue heads: each launch takes the next of QUEUE_SLOTS sets of
    // QUEUE_HEADS per-XCD heads and zeroes it on its own stream (up to QUEUE_SLOTS
    // launches may be in flight at once).
    unsigned int* queues = nullptr;
    mutable std::atomic<uint32_t> queue_next{0};
};
constexpr uint32_t QUEUE_SLOTS = 256;

// Makes `device` current for a scope and restores the caller's device afterwards: the
// library never leaves the caller's (e.g. torch's) current device changed, and every
// allocation, memset and launch goes to the device the scene lives on.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (device != prev) check(hipSetDevice(device), "hipSetDevice");
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

int gpu_device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// 4-wide world BVH when the scene has one (its stack bound fits); NRT_WBVH4=0
// keeps the binary tree (diagnostic A/B knob).
static bool use_wbvh4(const FlatScene& fs) {
    if (fs.wbvh.nodes4.empty()) return false;
    const char* e = std::getenv("NRT_WBVH4");
    return !(e && e[0] == '0');
}

DeviceScene* gpu_upload_scene(const FlatScene& fs, int device) {
    DeviceGuard guard(device);
    auto* ds = new DeviceScene();
    ds->device = device;
    try {
        FlatScene32 f32 = to_f32(fs);
        auto track = [&](void* p, size_t n) { if (p) { ds->allocations.push_back(p); ds->bytes += n; } return p; };
        auto* n64 = (DNode<double>*)track(upload(fs.nodes, "nodes"), fs.nodes.size() * sizeof(DNode<double>));
        auto* p64 = (DPrim<double>*)track(upload(fs.prims, "prims"), fs.prims.size() * sizeof(DPrim<double>));
        auto* x64 = (DXform<double>*)track(upload(fs.xforms, "xforms"), fs.xforms.size() * sizeof(DXform<double>));
        auto* n32 = (DNode<float>*)track(upload(f32.nodes, "nodes32"), f32.nodes.size() * sizeof(DNode<float>));
        auto* p32 = (DPrim<float>*)track(upload(f32.prims, "prims32"), f32.prims.size() * sizeof(DPrim<float>));
        auto* x32 = (DXform<float>*)track(upload(f32.xforms, "xforms32"), f32.xforms.size() * sizeof(DXform<float>));
        auto* inst = (DInstance*)track(upload(fs.instances, "instances"), fs.instances.size() * sizeof(DInstance));
        auto* mats = (DMaterial*)track(upload(fs.materials, "materials"), fs.materials.size() * sizeof(DMaterial));
        auto* texs = (DTexture*)track(upload(fs.textures, "textures"), fs.textures.size() * sizeof(DTexture));
        auto* texels = (uint32_t*)track(upload(fs.texels, "texels"), fs.texels.size() * sizeof(uint32_t));
        auto* fpr = (DPrimFast<float>*)track(upload(f32.fprims, "fprims"), f32.fprims.size() * sizeof(DPrimFast<float>));
        auto* ifast = (DInstFast<float>*)track(upload(f32.inst_fast, "inst_fast"),
                                               f32.inst_fast.size() * sizeof(DInstFast<float>));
        auto* mfast = (DMatFast*)track(upload(fs.mats_fast, "mats_fast"), fs.mats_fast.size() * sizeof(DMatFast));
        auto* wpr = (DPrimWorld<float>*)track(upload(f32.wprims, "wprims"), f32.wprims.size() * sizeof(DPrimWorld<float>));
        std::vector<uint32_t> wruns_padded = fs.wruns;  // whole 16-B groups (run words read 4 at a time)
        wruns_padded.resize((fs.wruns.size() + 3) & ~size_t(3), 0u);
        auto* wrn = (uint32_t*)track(upload(wruns_padded, "wruns"), wruns_padded.size() * sizeof(uint32_t));
        auto* wbn = (DBvhNode*)track(upload(fs.wbvh.nodes, "wbvh"), fs.wbvh.nodes.size() * sizeof(DBvhNode));
        auto* wb4 = (DBvh4Node*)track(upload(fs.wbvh.nodes4, "wbvh4"), fs.wbvh.nodes4.size() * sizeof(DBvh4Node));
        auto* wb4c = (DBvh4cNode*)track(upload(fs.wbvh.nodes4c, "wbvh4c"), fs.wbvh.nodes4c.size() * sizeof(DBvh4cNode));
        auto* wbp = (DPrimWorld<float>*)track(upload(f32.wbvh_prims, "wbvh_prims"),
                                              f32.wbvh_prims.size() * sizeof(DPrimWorld<float>));
        const uint32_t np = (uint32_t)fs.prims.size(), nx = (uint32_t)fs.xforms.size(),
                       ni = (uint32_t)fs.instances.size(), nm = (uint32_t)fs.materials.size(),
                       nt = (uint32_t)fs.textures.size();
        // f64 view: the exact node array (reference node for node); f32 view: the
        // list-collapsed array with composed instance transforms.
        const uint32_t wstack = std::max<uint32_t>(1u, use_wbvh4(fs) ? fs.wbvh.stack4 : fs.wbvh.depth);
        // the exact kernel's world-BVH mode culls with the f32 world BVH, or with a tree of its own
        // (FlatScene::wbvh_x) on scenes with several instance chains
        auto* wx = (DExactRef*)track(upload(fs.wexact, "wexact"), fs.wexact.size() * sizeof(DExactRef));
        auto* wxp = (DPrimWorld<float>*)track(upload(f32.wexact_prims, "wexact_prims"),
                                              f32.wexact_prims.size() * sizeof(DPrimWorld<float>));
        const bool wx_ok = !fs.wexact.empty();
        const WorldBvh& xt = fs.exact_tree();
        const DBvhNode* xbn = wbn;
        const DBvh4Node* xb4 = wb4;
        const DBvh4cNode* xb4c = wb4c;
        if (&xt != &fs.wbvh) {
            xbn = (DBvhNode*)track(upload(xt.nodes, "wbvh_x"), xt.nodes.size() * sizeof(DBvhNode));
            xb4 = (DBvh4Node*)track(upload(xt.nodes4, "wbvh4_x"), xt.nodes4.size() * sizeof(DBvh4Node));
            xb4c = (DBvh4cNode*)track(upload(xt.nodes4c, "wbvh4c_x"), xt.nodes4c.size() * sizeof(DBvh4cNode));
        }
        // exact walk on the compact tree (16-bit stack entries) unless NRT_EXACT_COMPACT=0
        const char* xce = std::getenv("NRT_EXACT_COMPACT");
        const bool x4c = !xt.nodes4c.empty() && !(xce && xce[0] == '0');
        const bool x4 = !xt.nodes4.empty() && use_wbvh4(fs);
        auto* xth = (DThreadNode*)track(upload(xt.threaded, "wbvh_threaded"), xt.threaded.size() * sizeof(DThreadNode));
        ds->v64 = DSceneView<double>{n64, p64, x64, inst, mats, texs, texels, fs.root, fs.max_depth,
                                     (uint32_t)fs.nodes.size(), np, nx, ni, nm, nt, nullptr, nullptr, nullptr, 0, 0, 0,
                                     nullptr, 0, nullptr, 0, 0, wx_ok ? xbn : nullptr,
                                     (wx_ok && x4) ? xb4 : nullptr, (wx_ok && x4 && x4c) ? xb4c : nullptr,
                                     xt.root4, xt.root,
                                     wx_ok ? (uint32_t)xt.nodes.size() : 0u,
                                     std::max<uint32_t>(1u, x4 ? xt.stack4 : xt.depth), wx_ok ? xth : nullptr,
                                     wx_ok ? xt.threaded_n : 0u, wx_ok ? wx : nullptr,
                                     wx_ok ? wxp : nullptr, wx_ok ? (uint32_t)fs.wexact.size() : 0u, 0u};
        {  // small culling trees travel into LDS with the scene (knob NRT_EXACT_XSTAGE=0: read from HBM)
            const size_t xb = xt.nodes4c.size() * sizeof(DBvh4cNode) +
                              fs.wexact.size() * (sizeof(DPrimWorld<float>) + sizeof(DExactRef));
            const char* xs = std::getenv("NRT_EXACT_XSTAGE");
            if (wx_ok && x4 && x4c && xb <= XSTAGE_MAX_BYTES && !(xs && xs[0] == '0'))
                ds->v64.n_xstage = (uint32_t)xt.nodes4c.size();
        }
        // the fast kernel reads fast prims only: no f32 DPrim copy in its LDS image
        ds->v32 = DSceneView<float>{n32, p32, x32, inst, mats, texs, texels, fs.root_fast, fs.max_depth,
                                    (uint32_t)f32.nodes.size(), 0, 0, ni, nm, nt, fpr, ifast, mfast,
                                    (uint32_t)f32.fprims.size(), (uint32_t)f32.inst_fast.size(),
                                    (uint32_t)fs.mats_fast.size(), wpr, (uint32_t)f32.wprims.size(), wrn,
                                    (uint32_t)fs.wruns.size(), fs.wflags, wbn, use_wbvh4(fs) ? wb4 : nullptr,
                                    use_wbvh4(fs) ? wb4c : nullptr, fs.wbvh.root4, fs.wbvh.root,
                                    (uint32_t)fs.wbvh.nodes.size(), wstack, nullptr, 0u, nullptr, nullptr, 0u, 0u};
        ds->wbvh_ok = fs.wbvh_ok && fs.wbvh_f32_ok;  // (the f32 world-BVH modes)
        for (const DTexture& t : fs.textures) ds->perlin |= t.kind == TEX_NOISE || t.kind == TEX_MARBLE;
        ds->planes = !fs.prims.empty();
        for (const DPrim<double>& pr : fs.prims) ds->planes &= pr.kind != PRIM_SPHERE;
        ds->flat = !ds->perlin;
        ds->texpal = true;
        for (const DTexture& t : fs.textures)
            ds->texpal &= t.kind == TEX_SOLID || (t.kind == TEX_IMAGE && t.format == TEXFMT_PAL16);
        for (const DMatFast& m : fs.mats_fast) ds->flat &= m.solid != 0;
        // unit kinds from the runs (box / room units also hold header and empty face slots)
        for (uint32_t run : fs.wruns)
            ds->flat &= (run & WRUN_KIND_MASK) != PRIM_SPHERE && (run & WRUN_KIND_MASK) != PRIM_SPHERE32;
        ds->flat &= !fs.wruns.empty();
        ds->wbvh_prims = wbp;
        const size_t qbytes = (size_t)QUEUE_SLOTS * QUEUE_HEADS * QUEUE_STRIDE * sizeof(unsigned int);
        check(hipMalloc((void**)&ds->queues, qbytes), "hipMalloc(queues)");
        track(ds->queues, qbytes);
        check(hipMemset(ds->queues, 0, qbytes), "hipMemset(queues)");
        ds->n_wbvh_prims = (uint32_t)f32.wbvh_prims.size();
        {
            bool tri = false, quad = false, other = false;
            for (const DPrimWorld<float>& w : f32.wbvh_prims) {
                const uint32_t k = w.meta & WKIND_MASK;
                tri |= k == PRIM_TRIANGLE;
                quad |= k == PRIM_QUAD;
                other |= k != PRIM_TRIANGLE && k != PRIM_QUAD;
            }
            ds->wbvh_kinds = other || (tri && quad) ? WPRIMS_ANY : (quad ? WPRIMS_QUADS : WPRIMS_TRIANGLES);
        }
        ds->world_ok = fs.world_ok;
        ds->list_ok = fs.list_ok;
        ds->world_units = fs.world_units;
        ds->wruns = fs.wruns;
    } catch (...) {
        gpu_free_scene(ds);
        throw;
    }
    return ds;
}

void gpu_free_scene(DeviceScene* ds) {
    if (!ds) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(ds->device);
    for (void* p : ds->allocations) (void)hipFree(p);
    (void)hipSetDevice(prev);
    delete ds;
}

size_t gpu_scene_bytes(const DeviceScene* ds) { return ds ? ds->bytes : 0; }
int gpu_scene_device(const DeviceScene* ds) { return ds ? ds->device : -1; }

// Fast kernel traversal mode for `trace` (nrt_render_opts.trace): the world
// list when every primitive could be pulled to world space and the list is
// short enough that testing all of it beats traversal; else the world BVH;
// else (instances that cannot flatten) the instance BVH.
int gpu_fast_maxd(const DeviceScene* ds, uint32_t trace) {
    const int inst_maxd = ds->v64.max_depth > 1 ? MAX_INSTANCE_DEPTH : 1;
    if (trace == NRT_TRACE_BVH) return inst_maxd;
    const bool world = ds->world_ok && ds->list_ok && ds->v32.n_wprims > 0;
    if (trace == NRT_TRACE_WORLD_LIST) {
        if (!ds->world_ok || ds->v32.n_wprims == 0)
            throw std::invalid_argument("trace=world-list: scene has primitives that cannot be flattened to world space");
        if (!ds->list_ok)
            throw std::invalid_argument("trace=world-list: coplanar surfaces whose f32 tie the world list cannot resolve");
        return MODE_WORLD_LIST;
    }
    if (trace == NRT_TRACE_WORLD_BVH) {
        if (!ds->wbvh_ok) throw std::invalid_argument("trace=world-bvh: scene cannot be flattened to world space");
        return MODE_WORLD_BVH;
    }
    if (world && ds->world_units <= NRT_WORLD_LIST_MAX) return MODE_WORLD_LIST;
    return ds->wbvh_ok ? MODE_WORLD_BVH : inst_maxd;
}

void gpu_launch_render(const DeviceScene* ds, const RenderParams& p, uint32_t precision, uint32_t rng,
                       uint32_t trace, void* stream_ptr) {
    if (p.pixel_end <= p.pixel_begin) return;
    if (p.width == 0) throw std::runtime_error("width must be > 0");
    DeviceGuard guard(ds->device);  // memset, occupancy query and launch on the scene's device
    hipStream_t stream = (hipStream_t)stream_ptr;
    RenderParams q = p;
    if (q.wave_wait == 0 && precision != 0)  // if-if trips (KF_FLAT world BVH) shade at 24 finished lanes (C4 34.6 -> 34.3 ms;
        q.wave_wait = ds->flat ? 24u : 48u;  // 32 / 40: 31.2 / 31.3 against 30.9 ms, round 5), the sphere / texture variant at 48
                                             // (spheres.toml 1080p: 27.64 / 27.26 / 26.84 / 26.83 / 33.24 ms at 32 / 40 / 48 / 56 / 64)
                                             // (the exact kernel's persistent walk: its own default, launch_impl.hpp)
    // Persistent lanes: claims of 8 pixels while the head has more than a round of its lanes' pixels
    // left, then of what the lanes ask (kernel.hpp next_pixel).  A claim per finished pixel stalls the
    // wave on the atomic's return (earth f64 spp 16: 6.26 -> 5.87 ms at 8) and writes ~35 B of HBM per
    // atomic; the guided tail keeps a reservoir from holding pixels while other waves idle.  The staging
    // of a claim's pixels in LDS, where it costs no occupancy (launch_impl.hpp exact_stage_fit).
    // Staging only at spp <= 64: at spp 256 it measured C5 f64 169-170 -> 208 ms (claims of 8 either way;
    // long pixels hold the wave's 8 slots) while saving no time at C4 / C5's pixel rates.
    if (q.exact_claim == 0) q.exact_claim = 8u;
    q.exact_stage = q.exact_claim > 1u && q.spp <= 64u ? 1u : 0u;
    if (const char* e = std::getenv("NRT_EXACT_STAGE"))  // A/B knob: 0 = never stage claims in LDS
        if (std::strtol(e, nullptr, 10) == 0) q.exact_stage = 0;
    {  // Philox: group queue heads; ChaCha8: the pixel counter of the persistent lanes (head 0)
        const size_t qwords = (size_t)QUEUE_HEADS * QUEUE_STRIDE;
        q.queue = ds->queues + (ds->queue_next.fetch_add(1) % QUEUE_SLOTS) * qwords;
        check(hipMemsetAsync(q.queue, 0, qwords * sizeof(unsigned int), stream), "hipMemsetAsync(queue)");
    }
    if (precision == 0)
        launch_exact(q, ds->v64, rng, ds->v64.max_depth > 1 ? MAX_INSTANCE_DEPTH : 1, ds->perlin, ds->planes, stream);
    else {
        const int maxd = gpu_fast_maxd(ds, trace);
        DSceneView<float> v = ds->v32;  // stage (LDS) only the tables this mode reads
        if (maxd == MODE_WORLD_LIST) {
            v.n_nodes = v.n_fprims = v.n_inst_fast = v.n_instances = 0;
        } else if (maxd == MODE_WORLD_BVH) {
            v.n_nodes = v.n_fprims = v.n_inst_fast = v.n_instances = 0;
            v.wprims = ds->wbvh_prims;  // records come from the BVH-ordered array
            v.n_wprims = ds->n_wbvh_prims;
            v.wruns = nullptr;
            v.n_wruns = 0;
        } else {
            v.n_wprims = 0;
        }
        // scene-specialised kernel (jit.hip): the world list's run words, or the world BVH's
        // width and tie flag, as template arguments; the same LDS layout as launch_one
        void* jit = nullptr;
        uint32_t stack_entry = 4;  // bytes per world-BVH stack entry of the kernel launched
        const uint32_t scene_lds = lds_scene_bytes(v, maxd);
        const bool staged = scene_lds <= LDS_SCENE_LIMIT;
        const uint32_t lds_fixed = staged ? scene_lds : 0u;  // (+ the BVH stack: launch_fast_jit)
        if ((maxd == MODE_WORLD_LIST || maxd == MODE_WORLD_BVH) && (rng == RNG_PHILOX || rng == RNG_CHACHA8) &&
            !ds->perlin && !q.counters) {
            std::string targs = std::string("float, nrt::dev::") + (rng == RNG_PHILOX ? "Philox, " : "ChaCha8, ") +
                                std::to_string(maxd) + ", false, " +
                                (staged ? "true, " : "false, ") +
                                std::to_string(ds->flat ? dev::KF_FLAT : (ds->texpal ? dev::KF_TEXPAL : 0)) + ", ";
            if (maxd == MODE_WORLD_LIST) {
                // ChaCha8 keeps the generic world-list kernel: its specialised build measured
                // 1.85x slower on C5 (72 -> 133 ms), the Philox one 1.25x faster
                if (rng == RNG_PHILOX && !ds->wruns.empty() && ds->wruns.size() <= JIT_MAX_RUNS) {
                    targs += "nrt::dev::WorldSig<";
                    for (size_t i = 0; i < ds->wruns.size(); ++i) targs += (i ? ", " : "") + std::to_string(ds->wruns[i]) + "u";
                    targs += ">";
                    jit = jit_render_kernel(targs, ds->device);
                    if (!jit) jit_require_failed(targs);
                }
            } else if (ds->flat) {  // (if-if trips: teapot 41.1 -> 40.5 ms; the sphere rounds measured slower)
                // the compact 4-wide tree where the scene has one (knob NRT_WBVH_COMPACT=0: the 64-byte one)
                const char* ce = std::getenv("NRT_WBVH_COMPACT");
                const bool compact = v.wbvh4c && !(ce && ce[0] == '0');
                if (compact) stack_entry = 2;
                targs += std::string("nrt::dev::BvhSig<") + (compact ? "5, " : v.wbvh4 ? "4, " : "2, ") +
                         ((v.wflags & WFLAG_COPLANAR) ? "true, " : "false, ") + std::to_string(ds->wbvh_kinds) + ">";
                jit = jit_render_kernel(targs, ds->device);
                if (!jit) jit_require_failed(targs);
            }
        }
        if (jit) launch_fast_jit(q, v, jit, lds_fixed, maxd, rng, jit ? stack_entry : 4u, stream);
        else launch_fast(q, v, rng, maxd, ds->perlin, ds->flat, stream);
    }
    check(hipGetLastError(), "render kernel launch");
}

uint64_t gpu_jit_compile_only(const char* targs, std::string* log) { return jit_compile_only(targs, log); }

JitCounts gpu_jit_counts() {
    const JitStats s = jit_stats();
    return JitCounts{s.compiled, s.launches, s.failed, s.compile_ns, s.disk_hits, s.load_retries};
}

void gpu_rng_probe(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample, uint64_t* host_out) {
    if (lanes == 0 || lanes > 256u) throw std::runtime_error("lanes must be in [1, 256]");
    unsigned long long* d = nullptr;
    const size_t bytes = (size_t)lanes * count * sizeof(unsigned long long);
    check(hipMalloc((void**)&d, bytes ? bytes : 8), "hipMalloc(rng probe)");
    launch_rng_probe(rng, stream0, lanes, count, sample, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess && bytes) e = hipMemcpy(host_out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    check(e, "rng probe");
}

}  // namespace nrt

namespace nrt {
void* device_alloc(size_t bytes, int device) {
    DeviceGuard guard(device);
    void* p = nullptr;
    check(hipMalloc(&p, bytes ? bytes : 16), "hipMalloc(output)");
    return p;
}
void device_free(void* p, int device) {
    try {
        DeviceGuard guard(device);
        (void)hipFree(p);
    } catch (...) {
    }
}
void device_copy_to_host(void* dst, const void* src, size_t bytes, int device) {
    DeviceGuard guard(device);
    check(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy(output)");
}
void device_zero(void* p, size_t bytes, int device) {
    DeviceGuard guard(device);
    check(hipMemset(p, 0, bytes), "hipMemset");
}
void device_sync(int device) {
    DeviceGuard guard(device);
    check(hipDeviceSynchronize(), "render kernel");
}
}  // namespace nrt

int nrt_current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return 0;
    return d;
}
