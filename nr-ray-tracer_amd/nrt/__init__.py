"""Python binding of libnrt.so (the C ABI in include/nrt.h), mirroring the
reference's library surface for the render path:

    SceneConfig::try_load_scene + merge_with + try_build  -> Scene.load(path, CameraConfig)
    Scene::render / Camera::render (lib/scene.rs:13-18)    -> Scene.render(camera, ...)
    CameraBuilder / Camera (lib/camera.rs:30-227)          -> CameraBuilder / Camera
    Sphere/Plane/BVH/Translate/Rotate/Scale/... builders    -> Builder

The renderer is the HIP megakernel in csrc/render.hip; there is no CPU
fallback: every render call goes through libnrt.so and fails loudly (NrtError)
when the library or a GPU is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NRT_LIB: an experiment build of the same library (make OUT=... EXTRA=...); default the in-tree one
LIB_PATH = os.environ.get("NRT_LIB") or os.path.join(_HERE, "libnrt.so")

PRECISION = {"f64": 0, "f32": 1}
RNG = {"chacha8": 0, "philox": 1}
TRACE = {"auto": 0, "bvh": 1, "world-list": 2, "world-bvh": 3}  # nrt_trace (f32 kernel traversal)

NRT_OK = 0
ERRORS = {-1: "invalid argument", -2: "load error", -3: "device error", -4: "unsupported"}


class NrtError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"[{ERRORS.get(code, code)}] {message}")
        self.code = code


class _CameraConfig(C.Structure):
    _fields_ = [("set", C.c_uint32), ("reserved", C.c_uint32), ("width", C.c_uint64), ("height", C.c_uint64),
                ("aspect_ratio", C.c_double), ("background_color", C.c_double * 3), ("look_at", C.c_double * 3),
                ("look_from", C.c_double * 3), ("view_up", C.c_double * 3), ("focal_length", C.c_double),
                ("field_of_view", C.c_double), ("defocus_angle", C.c_double), ("focus_distance", C.c_double),
                ("samples_per_pixel", C.c_uint64), ("ray_max_bounces", C.c_uint64)]


class _CameraBuilder(C.Structure):
    _fields_ = [("width", C.c_uint64), ("height", C.c_uint64), ("background_color", C.c_double * 3),
                ("look_from", C.c_double * 3), ("look_at", C.c_double * 3), ("view_up", C.c_double * 3),
                ("defocus_angle", C.c_double), ("focus_dist", C.c_double), ("field_of_view", C.c_double),
                ("ray_max_bounces", C.c_uint64), ("samples_per_pixel", C.c_uint64)]


class _Camera(C.Structure):
    _fields_ = [("width", C.c_uint64), ("height", C.c_uint64), ("samples_per_pixel", C.c_uint64),
                ("ray_max_bounces", C.c_uint64), ("background_color", C.c_double * 3),
                ("look_from", C.c_double * 3), ("defocus_disk_u", C.c_double * 3),
                ("defocus_disk_v", C.c_double * 3), ("pixel_delta_u", C.c_double * 3),
                ("pixel_delta_v", C.c_double * 3), ("top_left", C.c_double * 3)]


class _RenderOpts(C.Structure):
    _fields_ = [("precision", C.c_uint32), ("rng", C.c_uint32), ("device", C.c_int32), ("row_offset", C.c_uint32),
                ("row_stride", C.c_uint32), ("trace", C.c_uint32), ("gpus", C.c_uint32), ("reserved", C.c_uint32)]


class _SceneStats(C.Structure):
    _fields_ = [("nodes", C.c_uint64), ("prims", C.c_uint64), ("instances", C.c_uint64), ("xforms", C.c_uint64),
                ("materials", C.c_uint64), ("textures", C.c_uint64), ("texels", C.c_uint64), ("trees", C.c_uint32),
                ("max_instance_depth", C.c_uint32), ("device_bytes", C.c_uint64), ("world_prims", C.c_uint64),
                ("coplanar_pairs", C.c_uint32), ("world_list_ok", C.c_uint32), ("exact_mode", C.c_uint32),
                ("texel_formats", C.c_uint32), ("texel_bytes", C.c_uint64)]


PROGRESS_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64)

# Every symbol include/nrt.h declares, with its ctypes signature.
_D3 = C.POINTER(C.c_double)
SIGNATURES = {
    "nrt_abi_version": (C.c_int, []),
    "nrt_build_id": (C.c_char_p, []),
    "nrt_jit_stats": (C.c_int, [C.POINTER(C.c_uint64), C.c_size_t]),
    "nrt_debug_jit_compile": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint64)]),
    "nrt_last_error": (C.c_char_p, []),
    "nrt_device_count": (C.c_int, []),
    "nrt_camera_builder_default": (None, [C.POINTER(_CameraBuilder)]),
    "nrt_camera_build": (C.c_int, [C.POINTER(_CameraBuilder), C.POINTER(_Camera)]),
    "nrt_camera_config_apply": (C.c_int, [C.POINTER(_CameraConfig), C.POINTER(_CameraBuilder)]),
    "nrt_scene_load": (C.c_int, [C.c_char_p, C.POINTER(_CameraConfig), C.POINTER(C.c_void_p), C.POINTER(_Camera)]),
    "nrt_scene_load_ex": (C.c_int, [C.c_char_p, C.POINTER(_CameraConfig), C.c_uint32, C.POINTER(C.c_void_p),
                                    C.POINTER(_Camera)]),
    "nrt_builder_new": (C.c_void_p, []),
    "nrt_builder_free": (None, [C.c_void_p]),
    "nrt_texture_solid": (C.c_int32, [C.c_void_p, _D3]),
    "nrt_texture_image": (C.c_int32, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)]),
    "nrt_texture_image_file": (C.c_int32, [C.c_void_p, C.c_char_p]),
    "nrt_image_load": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                 C.c_size_t]),
    "nrt_texture_checker": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_double]),
    "nrt_texture_noise": (C.c_int32, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_double, C.c_double,
                                      C.c_double]),
    "nrt_texture_marble": (C.c_int32, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_double]),
    "nrt_material_lambertian": (C.c_int32, [C.c_void_p, C.c_int32]),
    "nrt_material_metal": (C.c_int32, [C.c_void_p, C.c_double, C.c_int32]),
    "nrt_material_dielectric": (C.c_int32, [C.c_void_p, C.c_double]),
    "nrt_material_diffuse_light": (C.c_int32, [C.c_void_p, C.c_double, C.c_int32]),
    "nrt_object_sphere": (C.c_int32, [C.c_void_p, _D3, C.c_double, C.c_int32]),
    "nrt_object_sphere_moving": (C.c_int32, [C.c_void_p, _D3, _D3, C.c_double, C.c_int32]),
    "nrt_object_quad": (C.c_int32, [C.c_void_p, _D3, _D3, _D3, C.c_int32]),
    "nrt_object_triangle": (C.c_int32, [C.c_void_p, _D3, _D3, _D3, C.c_int32]),
    "nrt_object_bvh": (C.c_int32, [C.c_void_p, C.POINTER(C.c_int32), C.c_size_t]),
    "nrt_object_translate": (C.c_int32, [C.c_void_p, C.c_int32, _D3]),
    "nrt_object_rotate_x": (C.c_int32, [C.c_void_p, C.c_int32, C.c_double]),
    "nrt_object_rotate_y": (C.c_int32, [C.c_void_p, C.c_int32, C.c_double]),
    "nrt_object_rotate_z": (C.c_int32, [C.c_void_p, C.c_int32, C.c_double]),
    "nrt_object_scale": (C.c_int32, [C.c_void_p, C.c_int32, _D3]),
    "nrt_builder_finish": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "nrt_render": (C.c_int, [C.c_void_p, C.POINTER(_Camera), C.POINTER(_RenderOpts), C.POINTER(C.c_float),
                             C.c_size_t, PROGRESS_FN, C.c_void_p]),
    "nrt_render_device": (C.c_int, [C.c_void_p, C.POINTER(_Camera), C.POINTER(_RenderOpts), C.c_void_p, C.c_size_t,
                                    C.c_void_p]),
    "nrt_render_prepare": (C.c_int, [C.c_void_p, C.POINTER(_Camera), C.POINTER(_RenderOpts)]),
    "nrt_render_timings": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_size_t)]),
    "nrt_rows_selected": (C.c_uint32, [C.c_uint32, C.POINTER(_RenderOpts)]),
    "nrt_scene_upload": (C.c_int, [C.c_void_p, C.c_int32]),
    "nrt_scene_stats_get": (C.c_int, [C.c_void_p, C.POINTER(_SceneStats)]),
    "nrt_scene_dump": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nrt_scene_destroy": (None, [C.c_void_p]),
    "nrt_image_to_rgb8": (C.c_int, [C.POINTER(C.c_float), C.c_size_t, C.c_float, C.POINTER(C.c_uint8)]),
    "nrt_debug_rng": (C.c_int, [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.POINTER(C.c_uint64)]),
    "nrt_debug_perlin_permutation": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint8)]),
    "nrt_debug_phase_profile": (C.c_int, [C.c_void_p, C.POINTER(_Camera), C.POINTER(_RenderOpts),
                                          C.POINTER(C.c_uint64), C.c_size_t]),
}

_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load libnrt.so (built in-tree by __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch wheels bundle their own
        # libamdhip64.so (same soname).  Loading torch first makes libnrt bind to
        # that copy instead of pulling /opt/rocm's beside it.
        if os.environ.get("NRT_NO_TORCH") != "1":
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(LIB_PATH):
            raise NrtError(-3, f"{LIB_PATH} not built: run __graft_entry__.build() / make -C nr-ray-tracer_amd")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # an A/B build named by NRT_LIB (scripts/ab_configs.py) may predate newer entry points
            if os.environ.get("NRT_LIB") and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _err() -> str:
    return lib().nrt_last_error().decode("utf-8", "replace")


def _check(code: int) -> None:
    if code != NRT_OK:
        raise NrtError(code, _err())


def _handle(h: int) -> int:
    if h < 0:
        raise NrtError(h, _err())
    return h


def _d3(v: Sequence[float]):
    return (C.c_double * 3)(*[float(x) for x in v])


def device_count() -> int:
    return lib().nrt_device_count()


def build_id() -> str:
    """sha256 prefix of the sources the loaded libnrt.so was built from (nrt_build_id)."""
    return lib().nrt_build_id().decode()


def jit_stats() -> dict:
    """Scene-specialised kernels (nrt_jit_stats): built by hiprtc in this process, renders using one,
    builds that failed (the generic kernel rendered instead), seconds spent compiling or loading, code
    objects read from the on-disk cache, module loads left to a later render."""
    out = (C.c_uint64 * 6)()
    _check(lib().nrt_jit_stats(out, 6))
    return {"compiled": int(out[0]), "launches": int(out[1]), "failed": int(out[2]),
            "compile_s": round(int(out[3]) * 1e-9, 4), "disk_hits": int(out[4]), "load_retries": int(out[5])}


def debug_jit_compile(targs: str) -> int:
    """hiprtc-compile render_kernel<targs> from the library's embedded headers (no GPU): code bytes."""
    n = C.c_uint64(0)
    _check(lib().nrt_debug_jit_compile(targs.encode(), C.byref(n)))
    return int(n.value)


def source_hash(pkg_dir: Optional[str] = None) -> str:
    """The same hash over the sources in this tree (Makefile SRC_HASH: csrc/*.cpp, *.hpp, *.hip
    in byte-wise sorted order, then include/nrt.h)."""
    import glob
    import hashlib

    pkg = pkg_dir or os.path.dirname(_HERE)
    files = sorted(sum((glob.glob(os.path.join("csrc", ext), root_dir=pkg) for ext in ("*.cpp", "*.hpp", "*.hip")), []))
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(pkg, "..", "include", "nrt.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


@dataclass
class CameraConfig:
    """CameraConfig (app cli.rs:160-270): CLI/env overrides; angles in degrees."""
    width: Optional[int] = None
    height: Optional[int] = None
    aspect_ratio: Optional[float] = None
    background_color: Optional[Sequence[float]] = None
    look_at: Optional[Sequence[float]] = None
    look_from: Optional[Sequence[float]] = None
    view_up: Optional[Sequence[float]] = None
    focal_length: Optional[float] = None
    field_of_view: Optional[float] = None
    defocus_angle: Optional[float] = None
    focus_distance: Optional[float] = None
    samples_per_pixel: Optional[int] = None
    ray_max_bounces: Optional[int] = None

    _BITS = ("width", "height", "aspect_ratio", "background_color", "look_at", "look_from", "view_up",
             "focal_length", "field_of_view", "defocus_angle", "focus_distance", "samples_per_pixel",
             "ray_max_bounces")

    def _c(self) -> _CameraConfig:
        c = _CameraConfig()
        for bit, name in enumerate(self._BITS):
            v = getattr(self, name)
            if v is None:
                continue
            c.set |= 1 << bit
            if name in ("background_color", "look_at", "look_from", "view_up"):
                setattr(c, name, _d3(v))
            else:
                setattr(c, name, v)
        return c


@dataclass
class Camera:
    """Camera after CameraBuilder::build (lib/camera.rs:205-227)."""
    width: int
    height: int
    samples_per_pixel: int
    ray_max_bounces: int
    background_color: tuple
    look_from: tuple
    defocus_disk_u: tuple
    defocus_disk_v: tuple
    pixel_delta_u: tuple
    pixel_delta_v: tuple
    top_left: tuple

    @staticmethod
    def _from_c(c: _Camera) -> "Camera":
        t = lambda a: tuple(a[i] for i in range(3))  # noqa: E731
        return Camera(c.width, c.height, c.samples_per_pixel, c.ray_max_bounces, t(c.background_color),
                      t(c.look_from), t(c.defocus_disk_u), t(c.defocus_disk_v), t(c.pixel_delta_u),
                      t(c.pixel_delta_v), t(c.top_left))

    def _c(self) -> _Camera:
        c = _Camera()
        c.width, c.height = self.width, self.height
        c.samples_per_pixel, c.ray_max_bounces = self.samples_per_pixel, self.ray_max_bounces
        for name in ("background_color", "look_from", "defocus_disk_u", "defocus_disk_v", "pixel_delta_u",
                     "pixel_delta_v", "top_left"):
            setattr(c, name, _d3(getattr(self, name)))
        return c

    def with_samples(self, spp: int) -> "Camera":
        import dataclasses
        return dataclasses.replace(self, samples_per_pixel=spp)


@dataclass
class CameraBuilder:
    """CameraBuilder (lib/camera.rs:30-203); angles in radians."""
    width: int = 1200
    height: int = 800
    background_color: tuple = (0.0, 0.0, 0.0)
    look_from: tuple = (1.0, 1.0, 1.0)
    look_at: tuple = (0.0, 0.0, 0.0)
    view_up: tuple = (0.0, 1.0, 0.0)
    defocus_angle: float = 0.0
    focus_dist: float = 1.0
    field_of_view: float = 1.5707963267948966
    ray_max_bounces: int = 10
    samples_per_pixel: int = 10

    def _c(self) -> _CameraBuilder:
        b = _CameraBuilder()
        for k in ("width", "height", "defocus_angle", "focus_dist", "field_of_view", "ray_max_bounces",
                  "samples_per_pixel"):
            setattr(b, k, getattr(self, k))
        for k in ("background_color", "look_from", "look_at", "view_up"):
            setattr(b, k, _d3(getattr(self, k)))
        return b

    def apply(self, cfg: CameraConfig) -> "CameraBuilder":
        """CameraConfig::try_update (cli.rs:357-402)."""
        b = self._c()
        _check(lib().nrt_camera_config_apply(C.byref(cfg._c()), C.byref(b)))
        out = CameraBuilder()
        for k in ("width", "height", "defocus_angle", "focus_dist", "field_of_view", "ray_max_bounces",
                  "samples_per_pixel"):
            setattr(out, k, getattr(b, k))
        for k in ("background_color", "look_from", "look_at", "view_up"):
            setattr(out, k, tuple(getattr(b, k)[i] for i in range(3)))
        return out

    def build(self) -> Camera:
        out = _Camera()
        _check(lib().nrt_camera_build(C.byref(self._c()), C.byref(out)))
        return Camera._from_c(out)


def _opts(precision: str, rng: str, device: int, row_offset: int, row_stride: int,
          trace: str = "auto", gpus: int = 0) -> _RenderOpts:
    if precision not in PRECISION:
        raise ValueError(f"precision must be one of {list(PRECISION)}")
    if rng not in RNG:
        raise ValueError(f"rng must be one of {list(RNG)}")
    if trace not in TRACE:
        raise ValueError(f"trace must be one of {list(TRACE)}")
    o = _RenderOpts()
    o.precision, o.rng, o.device = PRECISION[precision], RNG[rng], device
    o.row_offset, o.row_stride, o.trace = row_offset, row_stride, TRACE[trace]
    o.gpus = gpus
    return o


class Scene:
    """Scene { camera, objects: BVH } (lib/scene.rs:6-19), flattened for the GPU."""

    def __init__(self, handle: int, camera: Optional[Camera] = None):
        self._h = C.c_void_p(handle)
        self.camera = camera

    @staticmethod
    def load(path: str, overrides: Optional[CameraConfig] = None, legacy_schema: bool = False) -> "Scene":
        """SceneConfig::try_load_scene + merge_with + try_build; legacy_schema also accepts the index
        schema of scenes/triangles.toml (nrt_scene_load_ex, NRT_LOAD_LEGACY_SCHEMA)."""
        h = C.c_void_p()
        cam = _Camera()
        ov = C.byref(overrides._c()) if overrides is not None else None
        if legacy_schema:
            _check(lib().nrt_scene_load_ex(os.fsencode(path), ov, 1, C.byref(h), C.byref(cam)))
        else:
            _check(lib().nrt_scene_load(os.fsencode(path), ov, C.byref(h), C.byref(cam)))
        return Scene(h.value, Camera._from_c(cam))

    def close(self) -> None:
        if self._h and self._h.value:
            lib().nrt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> dict:
        s = _SceneStats()
        _check(lib().nrt_scene_stats_get(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in _SceneStats._fields_}

    def dump(self) -> str:
        need = C.c_size_t()
        _check(lib().nrt_scene_dump(self._h, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        _check(lib().nrt_scene_dump(self._h, buf, need.value, None))
        return buf.value.decode()

    def upload(self, device: int = -1) -> None:
        _check(lib().nrt_scene_upload(self._h, device))

    def rows_selected(self, height: int, row_offset: int = 0, row_stride: int = 1) -> int:
        return lib().nrt_rows_selected(height, C.byref(_opts("f64", "chacha8", -1, row_offset, row_stride)))

    def render(self, camera: Optional[Camera] = None, precision: str = "f64", rng: str = "chacha8",
               device: int = -1, row_offset: int = 0, row_stride: int = 1,
               progress: Optional[Callable[[int], None]] = None, trace: str = "auto", gpus: int = 0) -> np.ndarray:
        """Camera::render -> Rgb32FImage as float32 array (rows, W, 3).  gpus = N >= 1: the whole frame
        over devices device .. device+N-1 (device -1: 0), one RCCL gather (nrt_render_opts.gpus)."""
        cam = camera or self.camera
        if cam is None:
            raise ValueError("no camera")
        o = _opts(precision, rng, device, row_offset, row_stride, trace, gpus)
        rows = lib().nrt_rows_selected(cam.height, C.byref(o))
        out = np.empty((rows, cam.width, 3), dtype=np.float32)
        cb = PROGRESS_FN(lambda _u, n: progress(n)) if progress else PROGRESS_FN()
        _check(lib().nrt_render(self._h, C.byref(cam._c()), C.byref(o),
                                out.ctypes.data_as(C.POINTER(C.c_float)), out.size, cb, None))
        return out

    def phase_profile(self, camera: Optional[Camera] = None, precision: str = "f32", rng: str = "philox",
                      device: int = -1, trace: str = "auto") -> dict:
        """Diagnostic render with per-wave stamps: cycle shares of camera / trace / shading."""
        cam = camera or self.camera
        o = _opts(precision, rng, device, 0, 1, trace)
        out = (C.c_uint64 * 16)()
        _check(lib().nrt_debug_phase_profile(self._h, C.byref(cam._c()), C.byref(o), out, 16))
        iters, cam_c, trace_c, shade_c, waves, rec_c, rng_c, scat_c = list(out)[:8]
        vt, vl, lt, ll, rt, rl = list(out)[8:14]
        res = {"iterations_per_wave": iters / max(waves, 1), "waves": waves}
        if rng == "philox":
            # sample-pool loop: camera rays are part of the shading step; slot 1 counts
            # lane-iterations that shaded a path (lane occupancy of the loop)
            tot = max(trace_c + shade_c, 1)
            res["lane_occupancy"] = cam_c / max(64 * iters, 1)
            res["camera_share"] = 0.0
        else:
            tot = max(cam_c + trace_c + shade_c, 1)
            res["camera_share"] = cam_c / tot
        res.update({"trace_share": trace_c / tot, "shade_share": shade_c / tot,
                    "shade_record_share": rec_c / tot, "shade_rng_share": rng_c / tot,
                    "shade_scatter_share": scat_c / tot, "cycles_per_iteration": tot / max(iters, 1)})
        if vt:  # world-BVH traversal events (wave trips and active lanes per trip)
            res.update({"visit_trips_per_wave": vt / max(waves, 1), "visit_lane_util": vl / (64.0 * vt),
                        "leaf_trips_per_wave": lt / max(waves, 1), "leaf_lane_util": ll / (64.0 * max(lt, 1)),
                        "shade_rounds_per_wave": rt / max(waves, 1), "shade_round_lane_util": rl / (64.0 * max(rt, 1)),
                        "node_visits": vl, "prim_tests": ll, "rays_shaded": rl})
        return res

    def render_device(self, out_ptr: int, out_len: int, camera: Optional[Camera] = None, precision: str = "f32",
                      rng: str = "philox", device: int = -1, row_offset: int = 0, row_stride: int = 1,
                      stream: int = 0, trace: str = "auto", gpus: int = 0) -> None:
        """Enqueue a render into device memory (e.g. a torch tensor's data_ptr) on a HIP stream; gpus = N
        >= 1: the whole frame over N devices into out_ptr on the first (nrt_render_opts.gpus)."""
        cam = camera or self.camera
        o = _opts(precision, rng, device, row_offset, row_stride, trace, gpus)
        _check(lib().nrt_render_device(self._h, C.byref(cam._c()), C.byref(o), C.c_void_p(out_ptr), out_len,
                                       C.c_void_p(stream)))


    def prepare(self, camera: Optional[Camera] = None, precision: str = "f32", rng: str = "philox",
                device: int = -1, trace: str = "auto", gpus: int = 0) -> None:
        """nrt_render_prepare: the uploads and, with gpus = N >= 1, the RCCL communicators and shard
        buffers of such a render, done now (NrtError code -4 when librccl cannot gather)."""
        cam = camera or self.camera
        o = _opts(precision, rng, device, 0, 1, trace, gpus)
        _check(lib().nrt_render_prepare(self._h, C.byref(cam._c()), C.byref(o)))

    def render_timings(self) -> dict:
        """HIP-event times of the last gpus >= 1 render (nrt_render_timings): per-device render launch ms,
        the gather + un-permute ms on the first device, and the first device's render-to-render period."""
        n = C.c_size_t(0)
        _check(lib().nrt_render_timings(self._h, None, 0, C.byref(n)))
        out = (C.c_float * n.value)()
        _check(lib().nrt_render_timings(self._h, out, n.value, None))
        vals = [float(x) for x in out]
        return {"kernel_ms": vals[:-2], "gather_ms": vals[-2], "period_ms": vals[-1]}


class Builder:
    """The library's constructors (SphereBuilder, PlaneBuilder, BVH::from, Translate::new, ...)."""

    def __init__(self):
        self._b = C.c_void_p(lib().nrt_builder_new())

    def __del__(self):
        try:
            if self._b.value:
                lib().nrt_builder_free(self._b)
        except Exception:
            pass

    def solid(self, color) -> int:
        return _handle(lib().nrt_texture_solid(self._b, _d3(color)))

    def image(self, rgb: np.ndarray) -> int:
        a = np.ascontiguousarray(rgb, dtype=np.float32)
        return _handle(lib().nrt_texture_image(self._b, a.shape[1], a.shape[0], a.ctypes.data_as(C.POINTER(C.c_float))))

    def image_file(self, path: str) -> int:
        return _handle(lib().nrt_texture_image_file(self._b, os.fsencode(path)))

    def checker(self, even: int, odd: int, scale: float = 0.5) -> int:
        return _handle(lib().nrt_texture_checker(self._b, even, odd, scale))

    def noise(self, seed: Optional[int] = None, octaves: Optional[int] = None, frequency: Optional[float] = None,
              lacunarity: Optional[float] = None, persistence: Optional[float] = None) -> int:
        """PerlinRidgedNoiseBuilder (noise.rs:30-101): None = the builder's default."""
        fields = (seed, octaves, frequency, lacunarity, persistence)
        set_ = sum(1 << k for k, v in enumerate(fields) if v is not None)
        return _handle(lib().nrt_texture_noise(self._b, set_, seed or 0, octaves or 0, frequency or 0.0,
                                               lacunarity or 0.0, persistence or 0.0))

    def marble(self, seed: Optional[int] = None, frequency: Optional[float] = None) -> int:
        """MarbleBuilder (marble.rs:24-60): None = the builder's default."""
        set_ = (1 if seed is not None else 0) | (4 if frequency is not None else 0)
        return _handle(lib().nrt_texture_marble(self._b, set_, seed or 0, frequency or 0.0))

    def lambertian(self, tex: int) -> int:
        return _handle(lib().nrt_material_lambertian(self._b, tex))

    def metal(self, fuzz: float, tex: int) -> int:
        return _handle(lib().nrt_material_metal(self._b, fuzz, tex))

    def dielectric(self, ri: float) -> int:
        return _handle(lib().nrt_material_dielectric(self._b, ri))

    def diffuse_light(self, intensity: float, tex: int) -> int:
        return _handle(lib().nrt_material_diffuse_light(self._b, intensity, tex))

    def sphere(self, center, radius: float, mat: int, speed=None) -> int:
        """SphereBuilder; `speed` = SphereBuilder::with_speed (sphere.rs:45-50): a moving sphere."""
        if speed is not None:
            return _handle(lib().nrt_object_sphere_moving(self._b, _d3(center), _d3(speed), radius, mat))
        return _handle(lib().nrt_object_sphere(self._b, _d3(center), radius, mat))

    def quad(self, p, u, v, mat: int) -> int:
        return _handle(lib().nrt_object_quad(self._b, _d3(p), _d3(u), _d3(v), mat))

    def triangle(self, p, u, v, mat: int) -> int:
        return _handle(lib().nrt_object_triangle(self._b, _d3(p), _d3(u), _d3(v), mat))

    def bvh(self, objects: Sequence[int]) -> int:
        arr = (C.c_int32 * max(len(objects), 1))(*objects)
        return _handle(lib().nrt_object_bvh(self._b, arr, len(objects)))

    def translate(self, obj: int, offset) -> int:
        return _handle(lib().nrt_object_translate(self._b, obj, _d3(offset)))

    def rotate(self, axis: str, obj: int, angle: float) -> int:
        fn = {"x": lib().nrt_object_rotate_x, "y": lib().nrt_object_rotate_y, "z": lib().nrt_object_rotate_z}[axis]
        return _handle(fn(self._b, obj, angle))

    def scale(self, obj: int, s) -> int:
        return _handle(lib().nrt_object_scale(self._b, obj, _d3(s)))

    def finish(self, bvh: int, camera: Optional[Camera] = None) -> Scene:
        h = C.c_void_p()
        _check(lib().nrt_builder_finish(self._b, bvh, C.byref(h)))
        return Scene(h.value, camera)


def image_load(path: str) -> np.ndarray:
    """Image::try_from_path(..).into_rgb32f(): (H, W, 3) float32 texels in [0, 1]."""
    w, h = C.c_uint32(), C.c_uint32()
    _check(lib().nrt_image_load(os.fsencode(path), C.byref(w), C.byref(h), None, 0))
    out = np.empty((h.value, w.value, 3), dtype=np.float32)
    _check(lib().nrt_image_load(os.fsencode(path), C.byref(w), C.byref(h),
                                out.ctypes.data_as(C.POINTER(C.c_float)), out.size))
    return out


def to_rgb8(img: np.ndarray, gamma: float = 0.5) -> np.ndarray:
    """gamma_correction + DynamicImage::to_rgb8 (lib/image.rs:53-57, render.rs:74-102)."""
    a = np.ascontiguousarray(img, dtype=np.float32)
    out = np.empty(a.shape, dtype=np.uint8)
    _check(lib().nrt_image_to_rgb8(a.ctypes.data_as(C.POINTER(C.c_float)), a.size, gamma,
                                   out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def debug_rng(rng: str, stream0: int, lanes: int, count: int, sample: int = 0) -> np.ndarray:
    """First `count` draws of `lanes` consecutive pixel streams, computed on the GPU.

    rng "philox2x32_block": the f32 render loop's Philox2x32-10 blocks instead, word k of
    lane l = block (pixel stream0 + l, `sample`, step k) as lo | hi << 32 (nrt.h)."""
    code = 2 if rng == "philox2x32_block" else RNG[rng]
    out = np.empty((lanes, count), dtype=np.uint64)
    _check(lib().nrt_debug_rng(code, stream0, lanes, count, sample, out.ctypes.data_as(C.POINTER(C.c_uint64))))
    return out


def debug_perlin_permutation(seed: int) -> np.ndarray:
    """Permutation table of the Perlin source for `seed` (Noise / Marble textures), host-side."""
    out = np.empty(256, dtype=np.uint8)
    _check(lib().nrt_debug_perlin_permutation(seed, out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out
