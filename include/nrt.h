/*
 * nrt.h — C ABI of the MI355X-native renderer for nr-ray-tracer's per-pixel
 * path-tracing loop.
 *
 * The reference has no FFI: the path sits behind Rust generics/traits
 * (SURVEY.md §8b).  Each entry point below names the reference interface it
 * replaces; a Rust host binds them with one `extern "C"` block
 * (INTEGRATION.md).  Conventions:
 *   - every int-returning call returns NRT_OK (0) or a negative NRT_E_* code and
 *     never aborts the process; nrt_last_error() gives the message (thread-local);
 *   - the caller owns every buffer it passes; the library copies all inputs;
 *   - all structs are plain data; no torch / HIP types appear in signatures
 *     (streams are passed as void*).
 */
#ifndef NRT_H
#define NRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NRT_ABI_VERSION 7

enum {
    NRT_OK = 0,
    NRT_E_INVALID = -1,     /* bad argument */
    NRT_E_LOAD = -2,        /* scene file / config error (anyhow::Error in the reference) */
    NRT_E_DEVICE = -3,      /* HIP error / no device */
    NRT_E_UNSUPPORTED = -4  /* feature outside the accelerated path (reserved; every reference scene feature renders) */
};

enum nrt_precision { NRT_PRECISION_F64 = 0, NRT_PRECISION_F32 = 1 };
enum nrt_rng { NRT_RNG_CHACHA8 = 0, NRT_RNG_PHILOX = 1 };
/* Traversal of the f32 kernel (the f64 kernel always walks the reference's BVH):
 *   BVH        the reference's BVH with instances kept (composed transforms), per lane;
 *   WORLD_LIST instances flattened to world space, every lane tests every primitive
 *              (six quads closing a box count as one slab test);
 *   WORLD_BVH  instances flattened, binned-SAH BVH, nearest-child-first with a per-lane stack.
 * AUTO picks WORLD_LIST when the scene flattens and makes at most NRT_WORLD_LIST_MAX
 * test units (nrt_scene_stats.world_prims), else WORLD_BVH when it flattens, else BVH.
 * The WORLD_* modes fail with NRT_E_INVALID on scenes that cannot flatten. */
enum nrt_trace { NRT_TRACE_AUTO = 0, NRT_TRACE_BVH = 1, NRT_TRACE_WORLD_LIST = 2, NRT_TRACE_WORLD_BVH = 3 };
#define NRT_WORLD_LIST_MAX 48

typedef struct nrt_scene nrt_scene;
typedef struct nrt_builder nrt_builder;

/* CameraConfig (packages/ray-tracer/src/cli.rs:157-270): each field optional,
 * present when its NRT_CC_* bit is set in `set`.  Angles in degrees. */
enum {
    NRT_CC_WIDTH = 1u << 0,
    NRT_CC_HEIGHT = 1u << 1,
    NRT_CC_ASPECT_RATIO = 1u << 2,
    NRT_CC_BACKGROUND_COLOR = 1u << 3,
    NRT_CC_LOOK_AT = 1u << 4,
    NRT_CC_LOOK_FROM = 1u << 5,
    NRT_CC_VIEW_UP = 1u << 6,
    NRT_CC_FOCAL_LENGTH = 1u << 7,
    NRT_CC_FIELD_OF_VIEW = 1u << 8,
    NRT_CC_DEFOCUS_ANGLE = 1u << 9,
    NRT_CC_FOCUS_DISTANCE = 1u << 10,
    NRT_CC_SAMPLES_PER_PIXEL = 1u << 11,
    NRT_CC_RAY_MAX_BOUNCES = 1u << 12
};

typedef struct {
    uint32_t set;
    uint32_t reserved;
    uint64_t width, height;
    double aspect_ratio;
    double background_color[3];
    double look_at[3];
    double look_from[3];
    double view_up[3];
    double focal_length; /* parsed, ignored — as in the reference (cli.rs:229) */
    double field_of_view;
    double defocus_angle;
    double focus_distance;
    uint64_t samples_per_pixel;
    uint64_t ray_max_bounces;
} nrt_camera_config;

/* CameraBuilder (lib/camera.rs:30-41); angles in radians. */
typedef struct {
    uint64_t width, height;
    double background_color[3];
    double look_from[3];
    double look_at[3];
    double view_up[3];
    double defocus_angle;
    double focus_dist;
    double field_of_view;
    uint64_t ray_max_bounces;
    uint64_t samples_per_pixel;
} nrt_camera_builder;

/* Camera after CameraBuilder::build (lib/camera.rs:205-227). */
typedef struct {
    uint64_t width, height;
    uint64_t samples_per_pixel;
    uint64_t ray_max_bounces;
    double background_color[3];
    double look_from[3];
    double defocus_disk_u[3];
    double defocus_disk_v[3];
    double pixel_delta_u[3];
    double pixel_delta_v[3];
    double top_left[3];
} nrt_camera;

typedef struct {
    uint32_t precision;  /* nrt_precision */
    uint32_t rng;        /* nrt_rng */
    int32_t device;      /* HIP device ordinal; -1 = current device (gpus >= 1: -1 = device 0) */
    uint32_t row_offset; /* render image rows y = row_offset + k*row_stride ... */
    uint32_t row_stride; /* ... (0 or 1: every row); output rows are compact */
    uint32_t trace;      /* nrt_trace (f32 kernel only) */
    /* 0: one device (`device`), the rows above.  N >= 1: the whole frame over the N devices
     * device .. device+N-1 of this process (Camera::render's one call over the whole machine,
     * lib/camera.rs:315-316): device first+r renders rows y = r (mod N) into its HBM,
     * one RCCL ncclGather (librccl, dlopen'ed; N = 1: a device copy, nothing to exchange) brings the
     * shards to the first device, which un-permutes them into the frame.  Needs row_offset 0 and row_stride <= 1; the frame is the
     * same bits as gpus = 0 (pixels and their RNG streams do not depend on the device).  The
     * scene owns the communicators and shard buffers (created on first use, freed with it). */
    uint32_t gpus;
    uint32_t reserved;
} nrt_render_opts;

typedef struct {
    uint64_t nodes, prims, instances, xforms, materials, textures, texels; /* texels: of all image textures */
    uint32_t trees, max_instance_depth;
    uint64_t device_bytes; /* HBM bytes of the flattened scene on one device */
    uint64_t world_prims;  /* world-list test units after flattening instances to world space: primitives,
                              with six quads closing a box counted once (0: not flattenable) */
    uint32_t coplanar_pairs; /* overlapping coplanar surface pairs (their hits tie in the reference) */
    uint32_t world_list_ok;  /* 1: the world list resolves every such tie as the reference does
                                (else AUTO takes the world BVH, which compares tie keys) */
    uint32_t exact_mode;     /* traversal of the f64 reference-exact kernel (NRT_EXACT_*) */
    uint32_t texel_formats;  /* image textures' storage formats, bit 1 << f for each format f used:
                                0 RGB32F (12 B per texel), 1 RGBA8 (4), 2 RGB8T (3), 3 PAL16 (2 + palettes) */
    /* HBM bytes of the texel array: image textures as stored (PAL16, the default for file images
     * whose bands fit: a 2-byte palette index per texel in 8 x 8 tiles plus an RGBA8 palette per
     * band; else RGB8T, 3 B per texel in 128-B tiles of 8 x 5; RGBA8 tiles; RGB32F for constructor
     * images with values other than k/255) plus the Perlin permutation tables of Noise / Marble */
    uint64_t texel_bytes;
} nrt_scene_stats;
/* Exact-kernel traversal (same closest hit and tie-break as BVH::hit, object.rs:89-121):
 *   BVH      the reference tree, box by box
 *   ALL      every primitive in the tree's depth-first order, no boxes (at most 48 primitives)
 *   WORLD    the f32 world BVH culls (conservatively), the reference tests decide */
enum nrt_exact_mode { NRT_EXACT_BVH = 0, NRT_EXACT_ALL = 1, NRT_EXACT_WORLD = 2 };

typedef void (*nrt_progress_fn)(void* user, uint64_t pixels_done);

/* ---- library ---------------------------------------------------------- */
int nrt_abi_version(void);
/* sha256 prefix of the library's sources it was built from (build provenance; no reference
 * counterpart) */
const char* nrt_build_id(void);
/* Scene-specialised kernels (built with hiprtc, loaded lazily, when a scene is first rendered
 * in an f32 world mode; NRT_JIT=0 turns them off, NRT_JIT=require makes a failed build an
 * error of the render call instead of a fallback to the generic kernel).  The first such render
 * of a scene pays the compile (0.2-0.5 s) inside the render call, unless the on-disk code-object
 * cache holds it (NRT_JIT_CACHE = a directory, default $XDG_CACHE_HOME/nrt-jit or
 * ~/.cache/nrt-jit; "0" turns it off): keyed by the library's build id, the architecture, the
 * template arguments and the compile options, written atomically and verified on load.
 * out[0] = kernels built by hiprtc in this process, out[1] = renders that used a specialised
 * kernel, out[2] = builds that failed (the generic kernel rendered instead: slower, the same
 * frame bit for bit), out[3] = compile + load wall time in ns, out[4] = code objects taken from
 * the disk cache, out[5] = module loads that failed and were retried; the first min(n, 6) are
 * written.  No reference counterpart. */
int nrt_jit_stats(uint64_t* out, size_t n);
/* Tests: compile render_kernel<targs> with hiprtc from the embedded headers, no GPU needed
 * (nothing is loaded); *code_bytes = the code object's size. */
int nrt_debug_jit_compile(const char* targs, uint64_t* code_bytes);
const char* nrt_last_error(void);   /* thread-local; message text mirrors anyhow's */
int nrt_device_count(void);

/* ---- camera (lib/camera.rs:162-203, 94-159; app cli.rs:316-402) --------- */
void nrt_camera_builder_default(nrt_camera_builder* out);           /* CameraBuilder::default */
int nrt_camera_build(const nrt_camera_builder* b, nrt_camera* out);  /* CameraBuilder::build */
/* CameraConfig::try_update onto a builder (image-size rules, degrees->radians) */
int nrt_camera_config_apply(const nrt_camera_config* cfg, nrt_camera_builder* b);

/* ---- scene from file: SceneConfig::try_load_scene + merge_with + try_build
 *      (app scene_config.rs:475-496, render.rs:107-111).  Relative paths inside
 *      the file (nested scenes, textures) resolve against the process CWD, as in
 *      the reference.  `overrides` may be NULL. */
int nrt_scene_load(const char* path, const nrt_camera_config* overrides, nrt_scene** out, nrt_camera* camera);
/* The same with load flags: NRT_LOAD_LEGACY_SCHEMA also accepts the legacy index schema of
 * scenes/triangles.toml (integer texture / material references, `objects`), mapped onto the
 * current one with ids "0", "1", ... (what `create triangles` writes today, create/triangles.rs).
 * Without it the file fails to load (NRT_E_LOAD), as in the reference. */
enum { NRT_LOAD_LEGACY_SCHEMA = 1u << 0 };
int nrt_scene_load_ex(const char* path, const nrt_camera_config* overrides, uint32_t flags, nrt_scene** out,
                      nrt_camera* camera);

/* ---- scene from the library constructors (the Hitable/Material/Texture
 *      trait surface of nr-ray-tracer-lib).  Handles are small non-negative
 *      integers (negative = error). */
nrt_builder* nrt_builder_new(void);
void nrt_builder_free(nrt_builder* b);
int32_t nrt_texture_solid(nrt_builder* b, const double color[3]);                      /* SolidColor::new */
int32_t nrt_texture_image(nrt_builder* b, uint32_t w, uint32_t h, const float* rgb);   /* Image (Rgb32F texels) */
int32_t nrt_texture_image_file(nrt_builder* b, const char* path);                      /* Image::try_from_path */
int32_t nrt_texture_checker(nrt_builder* b, int32_t even, int32_t odd, double scale);  /* CheckerBuilder */
/* PerlinRidgedNoiseBuilder (lib/textures/noise.rs:30-101) and MarbleBuilder (lib/textures/marble.rs:24-60):
 * each builder field is an Option, present when its NRT_NOISE_* bit is set in `set`; absent fields take the
 * builder's defaults (seed 0; octaves 1, clamped to [1, 32] by Fbm::set_octaves; frequency 1; lacunarity
 * 2*pi/3; persistence 0.5; Marble: 7 octaves and the default lacunarity / persistence, only seed and
 * frequency read).  get_color: |Fbm<Perlin>|(p) (Noise), (1 + sin(frequency * p.z + 10 |Fbm|(p))) / 2
 * (Marble), grey, at the world-space hit point. */
enum {
    NRT_NOISE_SEED = 1u << 0,
    NRT_NOISE_OCTAVES = 1u << 1,
    NRT_NOISE_FREQUENCY = 1u << 2,
    NRT_NOISE_LACUNARITY = 1u << 3,
    NRT_NOISE_PERSISTENCE = 1u << 4
};
int32_t nrt_texture_noise(nrt_builder* b, uint32_t set, uint32_t seed, uint64_t octaves, double frequency,
                          double lacunarity, double persistence);
int32_t nrt_texture_marble(nrt_builder* b, uint32_t set, uint32_t seed, double frequency);
int32_t nrt_material_lambertian(nrt_builder* b, int32_t texture);                       /* Lambertian::with_texture */
int32_t nrt_material_metal(nrt_builder* b, double fuzz, int32_t texture);               /* MetalBuilder */
int32_t nrt_material_dielectric(nrt_builder* b, double refraction_index);               /* Dielectric::new */
int32_t nrt_material_diffuse_light(nrt_builder* b, double intensity, int32_t texture);  /* DiffuseLightBuilder */
int32_t nrt_object_sphere(nrt_builder* b, const double center[3], double radius, int32_t material); /* SphereBuilder */
/* SphereBuilder::with_speed (lib/objects/sphere.rs:45-50): centre(time) = center + time * speed for the
 * ray's time in [0, 1) (sphere.rs:110-111, camera.rs:264); the box spans both end positions (sphere.rs:72-84) */
int32_t nrt_object_sphere_moving(nrt_builder* b, const double center[3], const double speed[3], double radius,
                                 int32_t material);
int32_t nrt_object_quad(nrt_builder* b, const double p[3], const double u[3], const double v[3], int32_t material);
int32_t nrt_object_triangle(nrt_builder* b, const double p[3], const double u[3], const double v[3], int32_t material);
int32_t nrt_object_bvh(nrt_builder* b, const int32_t* objects, size_t count);          /* BVH::from */
int32_t nrt_object_translate(nrt_builder* b, int32_t object, const double offset[3]);  /* Translate::new */
int32_t nrt_object_rotate_x(nrt_builder* b, int32_t object, double angle);             /* Rotate::axis_x */
int32_t nrt_object_rotate_y(nrt_builder* b, int32_t object, double angle);             /* Rotate::axis_y */
int32_t nrt_object_rotate_z(nrt_builder* b, int32_t object, double angle);             /* Rotate::axis_z */
int32_t nrt_object_scale(nrt_builder* b, int32_t object, const double scale[3]);       /* Scale::new */
/* Scene { objects: BVH } (lib/scene.rs:6-10); `bvh` must come from nrt_object_bvh. */
int nrt_builder_finish(nrt_builder* b, int32_t bvh, nrt_scene** out);

/* ---- render: Scene::render / Camera::render (lib/scene.rs:13-18, lib/camera.rs:302-343)
 * out_rgb: caller-owned, rows*width*3 f32, row-major (Rgb32FImage layout), where
 * rows = the rows selected by opts (all rows by default).  Synchronous.
 * progress (may be NULL) is called from the calling thread with the number of
 * pixels finished so far, at launch granularity. */
int nrt_render(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts, float* out_rgb,
               size_t out_len, nrt_progress_fn progress, void* user);
/* Same, into device memory on `hip_stream` (hipStream_t, NULL = default stream);
 * asynchronous: returns after enqueueing. */
int nrt_render_device(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts,
                      float* dev_out_rgb, size_t out_len, void* hip_stream);
/* With opts->gpus = N >= 1: dev_out_rgb (W*H*3 f32) and hip_stream belong to the first device
 * (a stream of another device: NRT_E_INVALID); every device's render and the gather are enqueued
 * and the call returns.  The first device's gather and the un-permute run on hip_stream itself,
 * after its prior work, so the library adds only its render streams to the caller's.  Consecutive
 * calls pipeline: frame k+1's renders may start while frame k's last paths, gather and un-permute
 * run. */
/* Everything a render of (scene, camera, opts) needs before its first launch, done now (ABI 7): the
 * upload to the device, and with opts->gpus = N the upload to every device, the RCCL communicators
 * and the shard / staging buffers, so a timed first render (render.rs:57-62) pays none of it.
 * NRT_E_UNSUPPORTED when gpus >= 2 and librccl (ncclGather, ncclCommInitAll) is not usable: a host
 * may then render row shards per device itself (nrt_render_opts row_offset / row_stride). */
int nrt_render_prepare(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts);
/* HIP-event times (ms) of the scene's last gpus >= 1 render (waits for it): out[d] = the render
 * launch on device first+d, d < N (begin to end; consecutive frames overlap, so this can include the
 * previous frame's tail); out[N] = the gather + un-permute on the first device (from its own render's
 * end, so the slowest device's lag is in it); out[N+1] = the device time per frame since the previous
 * call that wrote it: from the first device's render start of that window's first frame to the last
 * frame's completion (gather + un-permute done), over the frames (0 with fewer than two); a call that
 * writes out[N+1] starts a new window.  *count = N + 2; at most n written. */
int nrt_render_timings(const nrt_scene* scene, float* out, size_t n, size_t* count);
/* Number of rows selected by opts for an image of `height` rows. */
uint32_t nrt_rows_selected(uint32_t height, const nrt_render_opts* opts);
/* Upload the flattened scene to `device` now (otherwise done on first render). */
int nrt_scene_upload(nrt_scene* scene, int32_t device);

int nrt_scene_stats_get(const nrt_scene* scene, nrt_scene_stats* out);
/* Canonical text dump of the scene graph (BVH, boxes, transforms, materials) in
 * hex floats; *needed = bytes incl. NUL.  Used by parity tests. */
int nrt_scene_dump(const nrt_scene* scene, char* buf, size_t cap, size_t* needed);
void nrt_scene_destroy(nrt_scene* scene);

/* Image::try_from_path -> into_rgb32f (lib/textures/image.rs:24-28): decode an image file
 * (baseline JPEG) to W*H*3 f32 in [0, 1].  Call with rgb = NULL to get the size. */
int nrt_image_load(const char* path, uint32_t* width, uint32_t* height, float* rgb, size_t cap);

/* gamma_correction + to_rgb8 (lib/image.rs:53-57; image crate Rgb32F->Rgb8). */
int nrt_image_to_rgb8(const float* rgb, size_t n_floats, float gamma, uint8_t* out);

/* Tests: first `count` next_u64 draws of `lanes` consecutive pixel streams
 * (rng 0 ChaCha8: stream = pixel index, below 2^32 as every image pixel's: stream0 + lanes > 2^32 - 1
 * is NRT_E_INVALID; rng 1 Philox4x32-10: counter (pixel, sample, pair)),
 * or with rng 2 the f32 render loop's Philox2x32-10 blocks: word k of lane l = the block
 * of (pixel stream0 + l, sample, step k), lo | hi << 32 (count <= 256, sample < 2^24). */
int nrt_debug_rng(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample, uint64_t* out);

/* Tests: the 256-entry permutation table of the Perlin source for `seed` (noise 0.9.0
 * PermutationTable::new, used by the Noise / Marble textures, lib/textures/noise.rs:85-92). */
int nrt_debug_perlin_permutation(uint32_t seed, uint8_t* out);

/* Diagnostics: one render with per-wave s_memtime stamps; out[0..4] = {loop
 * iterations, camera-ray cycles, trace cycles, shading cycles, waves} summed over
 * waves, and with n >= 8 out[5..7] = the shading cycles split into {hit record +
 * material, sample claim + Philox block, scatter / camera ray + accumulate}.  With
 * rng = Philox, camera rays are part of shading and out[1] counts the lane-iterations
 * that shaded a path instead.  Slower than nrt_render; never timed. */
int nrt_debug_phase_profile(const nrt_scene* scene, const nrt_camera* camera, const nrt_render_opts* opts,
                            uint64_t* out, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* NRT_H */
