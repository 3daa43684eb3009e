// C ABI (include/nrt.h).  Every entry point converts exceptions into status
// codes + a thread-local message; nothing here aborts the process.
#include "../../include/nrt.h"

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "flatten.hpp"
#include "noise.hpp"
#include "gpu.hpp"
#include "scene.hpp"
#include "scene_config.hpp"

using namespace nrt;

struct nrt_scene {
    ObjectPtr graph;     // Scene.objects (top-level BVH)
    FlatScene flat;
    std::mutex mu;
    std::vector<DeviceScene*> per_device;  // index = HIP ordinal
    // multi-GPU renders (nrt_render_opts.gpus): one context per (first device, N, loopback), the last used
    std::map<std::tuple<int, int, bool>, MultiRender*> multi;
    MultiRender* last_multi = nullptr;
    ~nrt_scene() {
        for (auto& kv : multi) gpu_multi_free(kv.second);  // (before the device scenes they render)
        for (DeviceScene* d : per_device) gpu_free_scene(d);
    }
};

struct nrt_builder {
    std::vector<TexturePtr> textures;
    std::vector<MaterialPtr> materials;
    std::vector<ObjectPtr> objects;
};

int nrt_current_device();  // render.hip

namespace {

thread_local std::string g_last_error;

struct UnsupportedError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

template <class F>
int guarded(int fail_code, F&& f) {
    try {
        g_last_error.clear();
        return f();
    } catch (const ParseError& e) {
        return set_error(NRT_E_LOAD, e.what());
    } catch (const std::bad_alloc&) {
        return set_error(NRT_E_DEVICE, "out of memory");
    } catch (const std::invalid_argument& e) {  // a bad argument, whichever call found it
        return set_error(NRT_E_INVALID, e.what());
    } catch (const UnsupportedError& e) {
        return set_error(NRT_E_UNSUPPORTED, e.what());
    } catch (const std::exception& e) {
        std::string m = e.what();
        if (m.find("outside the accelerated path") != std::string::npos) return set_error(NRT_E_UNSUPPORTED, m);
        if (m.rfind("HIP error", 0) == 0) return set_error(NRT_E_DEVICE, m);
        return set_error(fail_code, m);
    } catch (...) {
        return set_error(fail_code, "unknown error");
    }
}

V3 v3of(const double* d) { return v3(d[0], d[1], d[2]); }
void put3(double* d, V3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

CameraBuilder from_c(const nrt_camera_builder& b) {
    CameraBuilder c;
    c.width = b.width;
    c.height = b.height;
    c.background_color = v3of(b.background_color);
    c.look_from = v3of(b.look_from);
    c.look_at = v3of(b.look_at);
    c.view_up = v3of(b.view_up);
    c.defocus_angle = b.defocus_angle;
    c.focus_dist = b.focus_dist;
    c.field_of_view = b.field_of_view;
    c.ray_max_bounces = b.ray_max_bounces;
    c.samples_per_pixel = b.samples_per_pixel;
    return c;
}
void to_c(const CameraBuilder& c, nrt_camera_builder* b) {
    b->width = c.width;
    b->height = c.height;
    put3(b->background_color, c.background_color);
    put3(b->look_from, c.look_from);
    put3(b->look_at, c.look_at);
    put3(b->view_up, c.view_up);
    b->defocus_angle = c.defocus_angle;
    b->focus_dist = c.focus_dist;
    b->field_of_view = c.field_of_view;
    b->ray_max_bounces = c.ray_max_bounces;
    b->samples_per_pixel = c.samples_per_pixel;
}
void to_c(const Camera& c, nrt_camera* o) {
    o->width = c.width;
    o->height = c.height;
    o->samples_per_pixel = c.samples_per_pixel;
    o->ray_max_bounces = c.ray_max_bounces;
    put3(o->background_color, c.background_color);
    put3(o->look_from, c.look_from);
    put3(o->defocus_disk_u, c.defocus_disk_u);
    put3(o->defocus_disk_v, c.defocus_disk_v);
    put3(o->pixel_delta_u, c.pixel_delta_u);
    put3(o->pixel_delta_v, c.pixel_delta_v);
    put3(o->top_left, c.top_left);
}

CameraConfig from_c(const nrt_camera_config& c) {
    CameraConfig o;
    const uint32_t s = c.set;
    if (s & NRT_CC_WIDTH) { o.has_width = true; o.width = c.width; }
    if (s & NRT_CC_HEIGHT) { o.has_height = true; o.height = c.height; }
    if (s & NRT_CC_ASPECT_RATIO) { o.has_aspect_ratio = true; o.aspect_ratio = c.aspect_ratio; }
    if (s & NRT_CC_BACKGROUND_COLOR) { o.has_background_color = true; o.background_color = v3of(c.background_color); }
    if (s & NRT_CC_LOOK_AT) { o.has_look_at = true; o.look_at = v3of(c.look_at); }
    if (s & NRT_CC_LOOK_FROM) { o.has_look_from = true; o.look_from = v3of(c.look_from); }
    if (s & NRT_CC_VIEW_UP) { o.has_view_up = true; o.view_up = v3of(c.view_up); }
    if (s & NRT_CC_FOCAL_LENGTH) { o.has_focal_length = true; o.focal_length = c.focal_length; }
    if (s & NRT_CC_FIELD_OF_VIEW) { o.has_field_of_view = true; o.field_of_view = c.field_of_view; }
    if (s & NRT_CC_DEFOCUS_ANGLE) { o.has_defocus_angle = true; o.defocus_angle = c.defocus_angle; }
    if (s & NRT_CC_FOCUS_DISTANCE) { o.has_focus_distance = true; o.focus_distance = c.focus_distance; }
    if (s & NRT_CC_SAMPLES_PER_PIXEL) { o.has_samples_per_pixel = true; o.samples_per_pixel = c.samples_per_pixel; }
    if (s & NRT_CC_RAY_MAX_BOUNCES) { o.has_ray_max_bounces = true; o.ray_max_bounces = c.ray_max_bounces; }
    return o;
}

uint32_t rows_selected(uint32_t height, const nrt_render_opts* o) {
    const uint32_t off = o ? o->row_offset : 0;
    const uint32_t stride = (o && o->row_stride > 1) ? o->row_stride : 1;
    if (off >= height) return 0;
    return (height - off + stride - 1) / stride;
}

DeviceScene* device_scene(nrt_scene* s, int device) {
    std::lock_guard<std::mutex> lock(s->mu);
    if ((int)s->per_device.size() <= device) s->per_device.resize((size_t)device + 1, nullptr);
    if (!s->per_device[(size_t)device]) s->per_device[(size_t)device] = gpu_upload_scene(s->flat, device);
    return s->per_device[(size_t)device];
}

int resolve_device(const nrt_render_opts* o) {
    int n = gpu_device_count();
    if (n <= 0) throw std::runtime_error("HIP error in device query: no GPU device available");
    int dev = o ? o->device : -1;
    if (dev < 0) {
        dev = nrt_current_device();
    }
    if (dev >= n) throw std::invalid_argument("device ordinal out of range");
    return dev;
}

// Primitive tests of one walk over every node of the exact tree (instances walk their BLAS),
// capped at `cap` + 1: RenderParams::exact_all for scenes whose whole list is cheap.
static uint64_t exact_walk_prims(const FlatScene& f, int32_t node, uint64_t cap, int depth = 0) {
    uint64_t n = 0;
    while (node >= 0 && node < (int32_t)f.nodes.size() && n <= cap) {
        const DNode<double>& d = f.nodes[node];
        const uint32_t kind = d.meta & 3u;
        if (kind == NODE_INNER) {
            ++node;
            continue;
        }
        if (kind == NODE_PRIM) {
            ++n;
        } else if (kind == NODE_INSTANCE) {
            const uint32_t idx = d.meta >> 2;
            if (depth > MAX_INSTANCE_DEPTH || idx >= f.instances.size()) return cap + 1;
            n += exact_walk_prims(f, f.instances[idx].root, cap - std::min(cap, n), depth + 1);
        }
        node = d.skip;
    }
    return n;
}
constexpr uint64_t EXACT_ALL_MAX = 48;  // Cornell box: 18 quads (6 walls + two 6-quad cubes)

// nrt_exact_mode of a scene (RenderParams::exact_all / exact_wbvh; NRT_EXACT_ALL / NRT_EXACT_WBVH
// environment knobs override it for A/B runs).
// World-BVH culling wins wherever the scene has the mapping (C5 Cornell: 245 ms against 280 ms
// for the all-primitives walk, C4 teapot 33 against 157 for the reference tree); the walk is
// the fallback for small scenes without it.
static uint32_t exact_mode(const FlatScene& f) {
    if (!f.wexact.empty()) return NRT_EXACT_WORLD;
    if (exact_walk_prims(f, f.root, EXACT_ALL_MAX) <= EXACT_ALL_MAX) return NRT_EXACT_ALL;
    return NRT_EXACT_BVH;
}

RenderParams make_params(const nrt_camera& c, const nrt_render_opts* o, uint32_t rows, const FlatScene& f) {
    if (c.width == 0 || c.height == 0) throw std::invalid_argument("image width and height must be > 0");
    if (c.width * c.height > 0xFFFFFFFFull) throw std::invalid_argument("image has more than 2^32 pixels");
    if (c.samples_per_pixel > 0xFFFFFFFFull || c.ray_max_bounces > 0xFFFFFFFFull)
        throw std::invalid_argument("samples_per_pixel / ray_max_bounces exceed 2^32-1");
    RenderParams p{};
    for (int k = 0; k < 3; ++k) {
        p.top_left[k] = c.top_left[k];
        p.pixel_delta_u[k] = c.pixel_delta_u[k];
        p.pixel_delta_v[k] = c.pixel_delta_v[k];
        p.look_from[k] = c.look_from[k];
        p.defocus_disk_u[k] = c.defocus_disk_u[k];
        p.defocus_disk_v[k] = c.defocus_disk_v[k];
        p.background[k] = c.background_color[k];
        const double* vs[7] = {c.top_left, c.pixel_delta_u, c.pixel_delta_v, c.look_from, c.defocus_disk_u,
                               c.defocus_disk_v, c.background_color};
        for (int q = 0; q < 7; ++q) p.camf[q][k] = (float)vs[q][k];
        if (c.defocus_disk_u[k] != 0.0 || c.defocus_disk_v[k] != 0.0) p.defocus = 1;
    }
    // world-BVH shading-round threshold (C4 +4 %, C1 +13 % over 8); 0 = chosen per kernel variant
    // in gpu_launch_render (32 for the speculative rounds, 24 for the if-if trips); knob NRT_WAVE_WAIT 1..64
    p.wave_wait = 0;
    if (const char* e = std::getenv("NRT_WAVE_WAIT")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1 && v <= 64) p.wave_wait = (uint32_t)v;
    }
    const uint32_t mode = exact_mode(f);
    p.exact_all = mode == NRT_EXACT_ALL ? 1u : 0u;
    if (const char* e = std::getenv("NRT_EXACT_ALL")) p.exact_all = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
    p.exact_wbvh = (!p.exact_all && mode == NRT_EXACT_WORLD) ? 1u : 0u;
    if (const char* e = std::getenv("NRT_EXACT_WBVH")) p.exact_wbvh = std::strtol(e, nullptr, 10) != 0 && !f.wexact.empty();
    // The world mode's f32 culling is conservative for ray origins near the scene: a slab end
    // (f32, per-ray 1/d and o/d) moves the plane by at most ~2 ulp of (|origin| + |plane|), about
    // 1.2e-7 (|origin| + scale), and the boxes are padded by 1e-6 scale (wbvh.cpp; scale = the
    // largest |coordinate| of the primitives' boxes): safe for |origin| up to ~7 scale.  Secondary
    // rays start on primitives; camera rays on the defocus disk around look_from: a camera beyond
    // 4 scale takes the reference tree or the all-primitives walk instead (also over the knobs:
    // a culled primitive would change the frame).
    if (p.exact_wbvh) {
        double ro = 0.0;
        for (const double* v : {c.look_from, c.defocus_disk_u, c.defocus_disk_v})
            ro += std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!(ro <= 4.0 * f.exact_tree().scale)) {
            p.exact_wbvh = 0;
            p.exact_all = exact_walk_prims(f, f.root, EXACT_ALL_MAX) <= EXACT_ALL_MAX ? 1u : 0u;
        }
    }
    // plane-only scenes: the exact world mode's f32 prefilter (knob NRT_EXACT_PF=0 turns it off;
    // over every slot instead of the walk measured slower on Cornell, 223 against 217 ms)
    p.exact_pf = 1;
    // the stackless threaded walk of the culling tree (no private stack; knob NRT_EXACT_THREAD=1) measured
    // slower than the 4-wide walk with its private stack: C5 f64 spp 64 69.2 vs 57.7 ms, C4 128.3 vs 98.6
    p.exact_thread = 0;
    if (const char* e = std::getenv("NRT_EXACT_THREAD")) p.exact_thread = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
    // the compact walk's stack in LDS at 3 waves per SIMD (no scratch traffic: C5 f64 6.1 GB -> 57 MB
    // of HBM writes at spp 64) rather than in scratch at 4: with persistent lanes the two run even
    // (C5 f64 54.9 / 55.0 ms, C4 15.2 / 14.7 ms); knob NRT_EXACT_LSTACK=0 for the scratch stack
    p.exact_lstack = 1;
    if (const char* e = std::getenv("NRT_EXACT_LSTACK")) p.exact_lstack = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
    // every slot in order instead of the culling walk, for small scenes (<= EXACT_SLOTS_MAX slots):
    // the default with spheres (the reference tests on every slot, EXACT_SIG_SLOTS); plane-only scenes
    // keep the prefiltered walk (over every slot measured slower on the Cornell box, 54.3 -> 54.9 ms at
    // spp 64).  Knob NRT_EXACT_SLOTS=0/1.
    // (the slot variants are not built for Perlin scenes, launch_impl.hpp: the flag stays 0 there)
    bool spheres = false, perlin = false;
    for (const DPrim<double>& pr : f.prims) spheres |= pr.kind == PRIM_SPHERE;
    for (const DTexture& t : f.textures) perlin |= t.kind == TEX_NOISE || t.kind == TEX_MARBLE;
    p.exact_slots = spheres && !perlin && f.wexact.size() <= dev::EXACT_SLOTS_MAX ? 1u : 0u;
    if (const char* e = std::getenv("NRT_EXACT_SLOTS")) p.exact_slots = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
    if (const char* e = std::getenv("NRT_EXACT_PF")) p.exact_pf = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
    // persistent lanes: fewest pixels per counter claim (0: render.hip's pick by spp); knob NRT_EXACT_CLAIM=1..64
    p.exact_claim = 0;
    if (const char* e = std::getenv("NRT_EXACT_CLAIM")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1 && v <= 64) p.exact_claim = (uint32_t)v;
    }
    p.width = (uint32_t)c.width;
    p.height = (uint32_t)c.height;
    p.spp = c.samples_per_pixel < 1 ? 1u : (uint32_t)c.samples_per_pixel;
    p.max_bounces = (uint32_t)c.ray_max_bounces;
    // Philox sample pool: pixels per wave, 0 = chosen per launch (render.hip); tuning
    // knob NRT_WAVE_PIXELS (a power of two 1..128).  ChaCha8 streams are sequential:
    // one lane per pixel.
    p.wave_pixels = 1;
    if (o && o->rng == NRT_RNG_PHILOX) {
        p.wave_pixels = 0;
        if (const char* e = std::getenv("NRT_WAVE_PIXELS")) {
            const long v = std::strtol(e, nullptr, 10);
            if (v >= 1 && v <= 128 && (v & (v - 1)) == 0) p.wave_pixels = (uint32_t)v;
        }
        if (c.width > 0xFFFFu || c.height > 0xFFFFu)
            throw std::invalid_argument("Philox mode: image width and height must be < 65536");
        if ((uint64_t)128 * p.spp >= 0xFFFFFFFFull)
            throw std::invalid_argument("samples_per_pixel too large for the Philox sample pool (< 2^25)");
        if (o->precision == NRT_PRECISION_F32 && (p.spp > PHILOX2_MAX_SPP || p.max_bounces > PHILOX2_MAX_BOUNCES))
            throw std::invalid_argument("f32 Philox mode: samples_per_pixel <= 2^24 and ray_max_bounces <= 254 "
                                        "(Philox2x32 counter (pixel, sample | step << 24))");
    }
    // Radiance grid 2^-k: a sample's radiance is at most max(background, emission) x
    // albedo^bounces; k keeps spp such values below 2^52, so the pixel sums are exact
    // (order-free).  Albedo > 1 is counted over at most 8 bounces: past that the sums
    // round like any f64 sum (still deterministic per lane order, no longer order-free).
    {
        double emit = 0.0, alb = 1.0;
        for (int k = 0; k < 3; ++k) emit = std::fmax(emit, std::fabs(c.background_color[k]));
        double texmax = 1.0;  // image texels and marble are <= 1
        for (const DTexture& t : f.textures) {
            if (t.kind == TEX_SOLID)
                for (int k = 0; k < 3; ++k) texmax = std::fmax(texmax, std::fabs(t.color[k]));
            if (t.kind == TEX_NOISE) {  // |Fbm| <= scale x sum_k |persistence|^k (|perlin| <= 1)
                double amp = 0.0, pk = 1.0;
                for (uint32_t k = 0; k < t.a; ++k, pk *= std::fabs(t.color[2])) amp += pk;
                texmax = std::fmax(texmax, std::fabs(t.scale) * amp);
            }
        }
        for (const DMaterial& m : f.materials) {
            if (m.kind == MAT_DIFFUSE_LIGHT) emit = std::fmax(emit, std::fmax(1.0, std::fabs(m.param)) * texmax);
        }
        alb = texmax;
        double lg = std::log2(std::fmax(emit, 1e-300)) + std::log2((double)p.spp) +
                    std::log2(alb) * (double)std::min<uint32_t>(p.max_bounces, 8u);
        int k = 50 - (int)std::ceil(std::fmax(lg, -100.0));
        k = std::max(-900, std::min(k, 900));
        // f32 kernels scale and round in f32 (exact for a power of two in f32 range): the grid
        // exponent stays in [-126, 127] (only radiance x spp beyond 2^176 or below 2^-77 moves it)
        if (o && o->precision == NRT_PRECISION_F32) k = std::max(-126, std::min(k, 127));
        p.acc_scale = std::ldexp(1.0, k);
        p.acc_unscale = std::ldexp(1.0, -k);
        p.acc_scale_f = std::ldexp(1.0f, k);
    }
    p.row_offset = o ? o->row_offset : 0;
    p.row_stride = (o && o->row_stride > 1) ? o->row_stride : 1;
    p.rows = rows;
    p.pixel_begin = 0;
    p.pixel_end = rows * p.width;
    return p;
}

void check_opts(const nrt_render_opts* o) {
    if (!o) return;
    if (o->precision > NRT_PRECISION_F32) throw std::invalid_argument("unknown precision");
    if (o->rng > NRT_RNG_PHILOX) throw std::invalid_argument("unknown rng");
    if (o->trace > NRT_TRACE_WORLD_BVH) throw std::invalid_argument("unknown trace mode");
    if (o->gpus && (o->row_offset != 0 || o->row_stride > 1))
        throw std::invalid_argument("gpus >= 1 renders the whole frame: row_offset must be 0 and row_stride <= 1");
}

// NRT_MULTI_LOOPBACK=1 (tests only): a gpus = N render runs its N row shards on the first device,
// the gather as device-to-device copies (multi.hip), so the N-GPU code runs on a one-GPU box
// Philox groups per resident wave of a synchronous nrt_render (RenderParams::groups_per_wave): its
// launch's tail is not overlapped by a next one, and smaller last groups shorten it (C5 row shards at
// N = 8 unpipelined: 0.830 of linear with 4, 0.872 with 16, profiles/r05_shard_scaling_c5.json)
constexpr uint32_t ONE_SHOT_GROUPS_PER_WAVE = 16;

bool multi_loopback() {
    const char* e = std::getenv("NRT_MULTI_LOOPBACK");
    return e && *e && std::strcmp(e, "0") != 0;
}

// The multi-GPU context of opts (gpus >= 1): devices first .. first + gpus - 1, each with the
// scene uploaded, one RCCL communicator each (multi.hip).  The context (communicators: seconds) is
// built outside the scene's lock, so other renders of the scene do not wait for it.
MultiRender* multi_render(nrt_scene* s, const nrt_render_opts* o) {
    const int n = gpu_device_count();
    if (n <= 0) throw std::runtime_error("HIP error in device query: no GPU device available");
    const int first = o->device < 0 ? 0 : o->device;
    const bool loop = multi_loopback();
    if (loop ? first >= n : (int64_t)first + (int64_t)o->gpus > (int64_t)n)
        throw std::invalid_argument("gpus = " + std::to_string(o->gpus) + " from device " + std::to_string(first) +
                                    ": only " + std::to_string(n) + " device(s) visible");
    const auto key = std::make_tuple(first, (int)o->gpus, loop);
    {
        std::lock_guard<std::mutex> lock(s->mu);
        auto it = s->multi.find(key);
        if (it != s->multi.end()) {
            s->last_multi = it->second;
            return it->second;
        }
    }
    std::vector<DeviceScene*> scenes;
    for (uint32_t d = 0; d < o->gpus; ++d) scenes.push_back(device_scene(s, loop ? first : first + (int)d));
    MultiRender* made = gpu_multi_create(scenes, loop);
    std::lock_guard<std::mutex> lock(s->mu);
    MultiRender*& m = s->multi[key];
    if (m) {  // another thread built it meanwhile: keep theirs
        gpu_multi_free(made);
    } else {
        m = made;
    }
    s->last_multi = m;
    return m;
}

}  // namespace

// device helpers implemented in device_util.hip
extern "C++" {
namespace nrt {
void* device_alloc(size_t bytes, int device);
void device_free(void* p, int device);
void device_copy_to_host(void* dst, const void* src, size_t bytes, int device);
void device_sync(int device);
void device_zero(void* p, size_t bytes, int device);
}
}

extern "C" {

int nrt_abi_version(void) { return NRT_ABI_VERSION; }

#ifndef NRT_SRC_HASH
#define NRT_SRC_HASH "unknown"
#endif
const char* nrt_build_id(void) { return NRT_SRC_HASH; }

int nrt_debug_jit_compile(const char* targs, uint64_t* code_bytes) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!targs || !code_bytes) throw std::invalid_argument("null argument");
        std::string log;
        *code_bytes = gpu_jit_compile_only(targs, &log);
        if (!*code_bytes) throw std::runtime_error("hiprtc: " + log.substr(0, 2000));
        return NRT_OK;
    });
}

int nrt_jit_stats(uint64_t* out, size_t n) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!out && n) throw std::invalid_argument("null output");
        const JitCounts c = gpu_jit_counts();
        const uint64_t v[6] = {c.compiled, c.launches, c.failed, c.compile_ns, c.disk_hits, c.load_retries};
        for (size_t k = 0; k < n && k < 6; ++k) out[k] = v[k];
        return NRT_OK;
    });
}
const char* nrt_last_error(void) { return g_last_error.c_str(); }
int nrt_device_count(void) { return gpu_device_count(); }

void nrt_camera_builder_default(nrt_camera_builder* out) {
    if (out) to_c(CameraBuilder{}, out);
}

int nrt_camera_build(const nrt_camera_builder* b, nrt_camera* out) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!b || !out) throw std::invalid_argument("null argument");
        to_c(camera_build(from_c(*b)), out);
        return NRT_OK;
    });
}

int nrt_camera_config_apply(const nrt_camera_config* cfg, nrt_camera_builder* b) {
    return guarded(NRT_E_LOAD, [&]() {
        if (!cfg || !b) throw std::invalid_argument("null argument");
        CameraBuilder cb = from_c(*b);
        from_c(*cfg).try_update(cb);
        to_c(cb, b);
        return NRT_OK;
    });
}

int nrt_scene_load(const char* path, const nrt_camera_config* overrides, nrt_scene** out, nrt_camera* camera) {
    return nrt_scene_load_ex(path, overrides, 0u, out, camera);
}

int nrt_scene_load_ex(const char* path, const nrt_camera_config* overrides, uint32_t flags, nrt_scene** out,
                      nrt_camera* camera) {
    if (out) *out = nullptr;
    return guarded(NRT_E_LOAD, [&]() {
        if (!path || !out) throw std::invalid_argument("null argument");
        if (flags & ~(uint32_t)NRT_LOAD_LEGACY_SCHEMA) throw std::invalid_argument("unknown load flags");
        CameraConfig cli;
        if (overrides) cli = from_c(*overrides);
        LoadedScene ls = load_scene_file(path, overrides ? &cli : nullptr, (flags & NRT_LOAD_LEGACY_SCHEMA) != 0);
        auto s = std::make_unique<nrt_scene>();
        s->graph = ls.objects;
        s->flat = flatten_scene(ls.objects);
        if (camera) to_c(ls.camera, camera);
        *out = s.release();
        return NRT_OK;
    });
}

nrt_builder* nrt_builder_new(void) { return new (std::nothrow) nrt_builder(); }
void nrt_builder_free(nrt_builder* b) { delete b; }

static int32_t add_tex(nrt_builder* b, TexturePtr t) {
    b->textures.push_back(std::move(t));
    return (int32_t)b->textures.size() - 1;
}
static int32_t add_mat(nrt_builder* b, MaterialPtr m) {
    b->materials.push_back(std::move(m));
    return (int32_t)b->materials.size() - 1;
}
static int32_t add_obj(nrt_builder* b, ObjectPtr o) {
    b->objects.push_back(std::move(o));
    return (int32_t)b->objects.size() - 1;
}
static TexturePtr tex_at(nrt_builder* b, int32_t id) {
    if (id < 0 || (size_t)id >= b->textures.size()) throw std::invalid_argument("invalid texture handle");
    return b->textures[(size_t)id];
}
static MaterialPtr mat_at(nrt_builder* b, int32_t id) {
    if (id < 0 || (size_t)id >= b->materials.size()) throw std::invalid_argument("invalid material handle");
    return b->materials[(size_t)id];
}
static ObjectPtr obj_at(nrt_builder* b, int32_t id) {
    if (id < 0 || (size_t)id >= b->objects.size()) throw std::invalid_argument("invalid object handle");
    return b->objects[(size_t)id];
}

#define NRT_BUILD(body)                                                   \
    if (!b) return set_error(NRT_E_INVALID, "null builder");               \
    return guarded(NRT_E_INVALID, [&]() -> int { body });

int32_t nrt_texture_solid(nrt_builder* b, const double color[3]) {
    NRT_BUILD(auto t = std::make_shared<Texture>(); t->kind = Texture::Solid; t->color = v3of(color);
              return add_tex(b, t);)
}
int32_t nrt_texture_image(nrt_builder* b, uint32_t w, uint32_t h, const float* rgb) {
    NRT_BUILD(if (!rgb || w == 0 || h == 0) throw std::invalid_argument("empty image");
              auto t = std::make_shared<Texture>(); t->kind = Texture::Image; t->width = w; t->height = h;
              t->texels = std::make_shared<std::vector<float>>(rgb, rgb + 3ull * w * h); return add_tex(b, t);)
}
int32_t nrt_texture_image_file(nrt_builder* b, const char* path) {
    NRT_BUILD(if (!path) throw std::invalid_argument("null path"); DecodedImage img = decode_image_file(path);
              auto t = std::make_shared<Texture>(); t->kind = Texture::Image; t->width = img.width;
              t->height = img.height; t->texels = std::make_shared<std::vector<float>>(std::move(img.rgb));
              return add_tex(b, t);)
}
int32_t nrt_texture_checker(nrt_builder* b, int32_t even, int32_t odd, double scale) {
    NRT_BUILD(auto t = std::make_shared<Texture>(); t->kind = Texture::Checker; t->even = tex_at(b, even);
              t->odd = tex_at(b, odd); t->scale = scale; return add_tex(b, t);)
}
int32_t nrt_texture_noise(nrt_builder* b, uint32_t set, uint32_t seed, uint64_t octaves, double frequency,
                          double lacunarity, double persistence) {
    // PerlinRidgedNoiseBuilder::build (noise.rs:79-101), as the loader's Noise texture (scene_config.cpp)
    NRT_BUILD(if (set & ~0x1Fu) throw std::invalid_argument("unknown NRT_NOISE_* bits"); FbmParams f;
              if (set & NRT_NOISE_SEED) f.seed = seed; if (set & NRT_NOISE_FREQUENCY) f.frequency = frequency;
              if (set & NRT_NOISE_LACUNARITY) f.lacunarity = lacunarity;
              if (set & NRT_NOISE_PERSISTENCE) f.persistence = persistence;
              const uint64_t oct = (set & NRT_NOISE_OCTAVES) ? octaves : 1u; f.octaves = fbm_octaves(oct);
              auto t = std::make_shared<Texture>(); t->kind = Texture::Noise; t->fbm = f; return add_tex(b, t);)
}
int32_t nrt_texture_marble(nrt_builder* b, uint32_t set, uint32_t seed, double frequency) {
    // MarbleBuilder::build (marble.rs:46-60): only seed and frequency; 7 octaves
    NRT_BUILD(if (set & ~(uint32_t)(NRT_NOISE_SEED | NRT_NOISE_FREQUENCY))
                  throw std::invalid_argument("Marble takes only NRT_NOISE_SEED and NRT_NOISE_FREQUENCY");
              FbmParams f; if (set & NRT_NOISE_SEED) f.seed = seed; if (set & NRT_NOISE_FREQUENCY) f.frequency = frequency;
              f.octaves = MARBLE_OCTAVES; auto t = std::make_shared<Texture>(); t->kind = Texture::Marble; t->fbm = f;
              return add_tex(b, t);)
}
int32_t nrt_material_lambertian(nrt_builder* b, int32_t texture) {
    NRT_BUILD(auto m = std::make_shared<Material>(); m->kind = Material::Lambertian; m->texture = tex_at(b, texture);
              return add_mat(b, m);)
}
int32_t nrt_material_metal(nrt_builder* b, double fuzz, int32_t texture) {
    NRT_BUILD(auto m = std::make_shared<Material>(); m->kind = Material::Metal; m->fuzz = fuzz;
              m->texture = tex_at(b, texture); return add_mat(b, m);)
}
int32_t nrt_material_dielectric(nrt_builder* b, double refraction_index) {
    NRT_BUILD(auto m = std::make_shared<Material>(); m->kind = Material::Dielectric;
              m->refraction_index = refraction_index; return add_mat(b, m);)
}
int32_t nrt_material_diffuse_light(nrt_builder* b, double intensity, int32_t texture) {
    NRT_BUILD(auto m = std::make_shared<Material>(); m->kind = Material::DiffuseLight; m->intensity = intensity;
              m->texture = tex_at(b, texture); return add_mat(b, m);)
}
int32_t nrt_object_sphere(nrt_builder* b, const double center[3], double radius, int32_t material) {
    NRT_BUILD(return add_obj(b, make_sphere(v3of(center), radius, mat_at(b, material)));)
}
int32_t nrt_object_sphere_moving(nrt_builder* b, const double center[3], const double speed[3], double radius,
                                 int32_t material) {
    NRT_BUILD(if (!speed) throw std::invalid_argument("null speed"); const V3 sp = v3of(speed);
              return add_obj(b, make_sphere(v3of(center), radius, mat_at(b, material), &sp));)
}
int32_t nrt_object_quad(nrt_builder* b, const double p[3], const double u[3], const double v[3], int32_t material) {
    NRT_BUILD(return add_obj(b, make_plane(Object::Quad, v3of(p), v3of(u), v3of(v), mat_at(b, material)));)
}
int32_t nrt_object_triangle(nrt_builder* b, const double p[3], const double u[3], const double v[3], int32_t material) {
    NRT_BUILD(return add_obj(b, make_plane(Object::Triangle, v3of(p), v3of(u), v3of(v), mat_at(b, material)));)
}
int32_t nrt_object_bvh(nrt_builder* b, const int32_t* objects, size_t count) {
    NRT_BUILD(if (count && !objects) throw std::invalid_argument("null object list"); std::vector<ObjectPtr> list;
              for (size_t k = 0; k < count; ++k) list.push_back(obj_at(b, objects[k]));
              return add_obj(b, make_bvh(list));)
}
int32_t nrt_object_translate(nrt_builder* b, int32_t object, const double offset[3]) {
    NRT_BUILD(return add_obj(b, make_translate(obj_at(b, object), v3of(offset)));)
}
int32_t nrt_object_rotate_x(nrt_builder* b, int32_t object, double angle) {
    NRT_BUILD(return add_obj(b, make_rotate(obj_at(b, object), v3(1, 0, 0), angle));)
}
int32_t nrt_object_rotate_y(nrt_builder* b, int32_t object, double angle) {
    NRT_BUILD(return add_obj(b, make_rotate(obj_at(b, object), v3(0, 1, 0), angle));)
}
int32_t nrt_object_rotate_z(nrt_builder* b, int32_t object, double angle) {
    NRT_BUILD(return add_obj(b, make_rotate(obj_at(b, object), v3(0, 0, 1), angle));)
}
int32_t nrt_object_scale(nrt_builder* b, int32_t object, const double scale[3]) {
    NRT_BUILD(return add_obj(b, make_scale(obj_at(b, object), v3of(scale)));)
}

int nrt_builder_finish(nrt_builder* b, int32_t bvh, nrt_scene** out) {
    if (out) *out = nullptr;
    NRT_BUILD(if (!out) throw std::invalid_argument("null output"); ObjectPtr root = obj_at(b, bvh);
              if (root->kind != Object::BvhNode && root->kind != Object::BvhLeaf && root->kind != Object::BvhEmpty)
                  throw std::invalid_argument("scene root must be a BVH (nrt_object_bvh)");
              auto s = std::make_unique<nrt_scene>(); s->graph = root; s->flat = flatten_scene(root);
              *out = s.release(); return NRT_OK;)
}

uint32_t nrt_rows_selected(uint32_t height, const nrt_render_opts* opts) { return rows_selected(height, opts); }

int nrt_scene_upload(nrt_scene* scene, int32_t device) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!scene) throw std::invalid_argument("null scene");
        nrt_render_opts o{};
        o.device = device;
        device_scene(scene, resolve_device(&o));
        return NRT_OK;
    });
}

int nrt_render_device(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts,
                      float* dev_out_rgb, size_t out_len, void* hip_stream) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!scene || !camera || !dev_out_rgb) throw std::invalid_argument("null argument");
        check_opts(opts);
        const uint32_t rows = rows_selected((uint32_t)camera->height, opts);
        RenderParams p = make_params(*camera, opts, rows, scene->flat);
        if (out_len < (size_t)rows * p.width * 3) throw std::invalid_argument("output buffer too small");
        if (opts && opts->gpus) {
            if (rows == 0) return NRT_OK;
            MultiRender* m = multi_render(const_cast<nrt_scene*>(scene), opts);
            gpu_multi_render_device(m, p, opts->precision, opts->rng, opts->trace, dev_out_rgb, hip_stream);
            return NRT_OK;
        }
        const int dev = resolve_device(opts);
        DeviceScene* ds = device_scene(const_cast<nrt_scene*>(scene), dev);
        p.out = dev_out_rgb;
        gpu_launch_render(ds, p, opts ? opts->precision : 0, opts ? opts->rng : 0, opts ? opts->trace : 0, hip_stream);
        return NRT_OK;
    });
}

int nrt_render(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts, float* out_rgb,
               size_t out_len, nrt_progress_fn progress, void* user) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!scene || !camera || !out_rgb) throw std::invalid_argument("null argument");
        check_opts(opts);
        const uint32_t rows = rows_selected((uint32_t)camera->height, opts);
        RenderParams p = make_params(*camera, opts, rows, scene->flat);
        const size_t n = (size_t)rows * p.width * 3;
        if (out_len < n) throw std::invalid_argument("output buffer too small");
        if (n == 0) return NRT_OK;
        p.groups_per_wave = ONE_SHOT_GROUPS_PER_WAVE;  // a one-shot render: nothing follows to fill its tail
        if (opts && opts->gpus) {  // the whole frame over opts->gpus devices, one RCCL gather
            MultiRender* m = multi_render(const_cast<nrt_scene*>(scene), opts);
            gpu_multi_render_host(m, p, opts->precision, opts->rng, opts->trace, out_rgb);
            if (progress) progress(user, p.pixel_end);
            return NRT_OK;
        }
        const int dev = resolve_device(opts);
        DeviceScene* ds = device_scene(const_cast<nrt_scene*>(scene), dev);
        void* d = device_alloc(n * sizeof(float), dev);
        try {
            p.out = (float*)d;
            const uint32_t total = p.pixel_end;
            const uint32_t chunks = progress ? 16u : 1u;
            const uint32_t per = (total + chunks - 1) / chunks;
            for (uint32_t c = 0; c < chunks; ++c) {
                p.pixel_begin = c * per;
                p.pixel_end = std::min(total, (c + 1) * per);
                if (p.pixel_begin >= p.pixel_end) break;
                gpu_launch_render(ds, p, opts ? opts->precision : 0, opts ? opts->rng : 0, opts ? opts->trace : 0, nullptr);
                if (progress) {
                    device_sync(dev);
                    progress(user, p.pixel_end);
                }
            }
            device_sync(dev);
            device_copy_to_host(out_rgb, d, n * sizeof(float), dev);
        } catch (...) {
            device_free(d, dev);
            throw;
        }
        device_free(d, dev);
        return NRT_OK;
    });
}

int nrt_render_prepare(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!scene || !camera) throw std::invalid_argument("null argument");
        check_opts(opts);
        nrt_scene* s = const_cast<nrt_scene*>(scene);
        if (!opts || !opts->gpus) {
            device_scene(s, resolve_device(opts));
            return NRT_OK;
        }
        std::string why;
        if (opts->gpus > 1 && !multi_loopback() && !gpu_multi_rccl_usable(&why))
            throw UnsupportedError("gpus >= 1 needs RCCL's ncclGather: " + why);
        MultiRender* m = multi_render(s, opts);
        gpu_multi_prepare(m, (uint32_t)camera->width, (uint32_t)camera->height);
        return NRT_OK;
    });
}

int nrt_render_timings(const nrt_scene* scene, float* out, size_t n, size_t* count) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!scene || (!out && n)) throw std::invalid_argument("null argument");
        MultiRender* m = nullptr;
        {
            std::lock_guard<std::mutex> lock(const_cast<nrt_scene*>(scene)->mu);
            m = scene->last_multi;
        }
        if (!m) throw std::invalid_argument("no multi-GPU render (gpus >= 1) of this scene yet");
        const size_t c = gpu_multi_timings(m, out, n);
        if (count) *count = c;
        return NRT_OK;
    });
}

int nrt_scene_stats_get(const nrt_scene* scene, nrt_scene_stats* out) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!scene || !out) throw std::invalid_argument("null argument");
        const FlatScene& f = scene->flat;
        out->nodes = f.nodes.size();
        out->prims = f.prims.size();
        out->instances = f.instances.size();
        out->xforms = f.xforms.size();
        out->materials = f.materials.size();
        out->textures = f.textures.size();
        out->texels = f.texel_count;
        out->trees = f.num_trees;
        out->max_instance_depth = (uint32_t)f.max_depth;
        out->device_bytes = f.nodes.size() * (sizeof(DNode<double>) + sizeof(DNode<float>)) +
                            f.prims.size() * (sizeof(DPrim<double>) + sizeof(DPrim<float>)) +
                            f.xforms.size() * (sizeof(DXform<double>) + sizeof(DXform<float>)) +
                            f.instances.size() * sizeof(DInstance) + f.materials.size() * sizeof(DMaterial) +
                            f.textures.size() * sizeof(DTexture) + f.texels.size() * sizeof(uint32_t) +
                            f.nodes_fast.size() * sizeof(DNode<float>) + f.fprims.size() * sizeof(DPrimFast<float>) +
                            f.inst_fast.size() * sizeof(DInstFast<float>) + f.mats_fast.size() * sizeof(DMatFast) +
                            f.wprims.size() * sizeof(DPrimWorld<float>);
        out->world_prims = f.world_ok ? f.world_units : 0;
        out->coplanar_pairs = f.coplanar_pairs;
        out->world_list_ok = f.world_ok && f.list_ok ? 1u : 0u;
        out->exact_mode = exact_mode(f);
        out->texel_formats = 0;
        for (const DTexture& t : f.textures)
            if (t.kind == TEX_IMAGE) out->texel_formats |= 1u << t.format;
        out->texel_bytes = (uint64_t)f.texels.size() * sizeof(uint32_t);
        return NRT_OK;
    });
}

int nrt_scene_dump(const nrt_scene* scene, char* buf, size_t cap, size_t* needed) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!scene) throw std::invalid_argument("null scene");
        const std::string s = dump_graph(scene->graph);
        if (needed) *needed = s.size() + 1;
        if (buf && cap) {
            const size_t n = std::min(cap - 1, s.size());
            std::memcpy(buf, s.data(), n);
            buf[n] = '\0';
        }
        return NRT_OK;
    });
}

void nrt_scene_destroy(nrt_scene* scene) { delete scene; }

int nrt_image_load(const char* path, uint32_t* width, uint32_t* height, float* rgb, size_t cap) {
    return guarded(NRT_E_LOAD, [&]() {
        if (!path || !width || !height) throw std::invalid_argument("null argument");
        const DecodedImage img = decode_image_file(path);
        *width = img.width;
        *height = img.height;
        if (rgb) {
            if (cap < img.rgb.size()) throw std::invalid_argument("output buffer too small");
            std::memcpy(rgb, img.rgb.data(), img.rgb.size() * sizeof(float));
        }
        return NRT_OK;
    });
}

int nrt_image_to_rgb8(const float* rgb, size_t n, float gamma, uint8_t* out) {
    return guarded(NRT_E_INVALID, [&]() {
        if ((n && !rgb) || (n && !out)) throw std::invalid_argument("null argument");
        for (size_t k = 0; k < n; ++k) {
            const float g = std::pow(rgb[k], gamma);           // gamma_correction: p.powf(gamma)
            const float c = !(g < 1.0f) ? 1.0f : std::fmax(g, 0.0f);  // image crate normalize_float
            out[k] = (uint8_t)std::nearbyint(std::round(c * 255.0f));
        }
        return NRT_OK;
    });
}

int nrt_debug_phase_profile(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts,
                            uint64_t* out, size_t n) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!scene || !camera || !out || n < 5) throw std::invalid_argument("need scene, camera and out[5]");
        check_opts(opts);
        const uint32_t rows = rows_selected((uint32_t)camera->height, opts);
        RenderParams p = make_params(*camera, opts, rows, scene->flat);
        const size_t floats = (size_t)rows * p.width * 3;
        const int dev = resolve_device(opts);
        DeviceScene* ds = device_scene(const_cast<nrt_scene*>(scene), dev);
        void* img = device_alloc(floats * sizeof(float) + 64, dev);
        void* ctr = device_alloc(16 * sizeof(uint64_t), dev);
        try {
            device_zero(ctr, 16 * sizeof(uint64_t), dev);
            p.out = (float*)img;
            p.counters = (unsigned long long*)ctr;
            gpu_launch_render(ds, p, opts ? opts->precision : 0, opts ? opts->rng : 0, opts ? opts->trace : 0, nullptr);
            device_sync(dev);
            uint64_t h[16];
            device_copy_to_host(h, ctr, sizeof h, dev);
            for (size_t k = 0; k < n && k < 16; ++k) out[k] = h[k];
        } catch (...) {
            device_free(img, dev);
            device_free(ctr, dev);
            throw;
        }
        device_free(img, dev);
        device_free(ctr, dev);
        return NRT_OK;
    });
}

int nrt_debug_perlin_permutation(uint32_t seed, uint8_t* out) {
    return guarded(NRT_E_INVALID, [&]() {
        if (!out) throw std::invalid_argument("null output");
        perlin_permutation(seed, out);
        return NRT_OK;
    });
}

int nrt_debug_rng(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample, uint64_t* out) {
    return guarded(NRT_E_DEVICE, [&]() {
        if (!out && lanes && count) throw std::invalid_argument("null output");
        if (rng > RNG_PHILOX2_BLOCK) throw std::invalid_argument("unknown rng");
        if (rng == RNG_CHACHA8 && stream0 + lanes > 0xFFFFFFFFull)  // (pixel streams: make_params caps images below 2^32 pixels)
            throw std::invalid_argument("ChaCha8 probe: streams are pixel indices below 2^32");
        if (rng == RNG_PHILOX2_BLOCK && (count > PHILOX2_STEPS || stream0 + lanes > 0xFFFFFFFFull || sample >= PHILOX2_MAX_SPP))
            throw std::invalid_argument("Philox2x32 block probe: step, pixel or sample out of range");
        gpu_rng_probe(rng, stream0, lanes, count, sample, out);
        return NRT_OK;
    });
}

}  // extern "C"
