"""ORACLE — test infrastructure only (never imported by the product path).

Independent Python restatement of the reference's scene loading, written
against packages/ray-tracer/src/scene_config.rs:26-497 and cli.rs:157-402, that
emits the line-based "oracle tree" consumed by oracle/oracle.cpp.  It shares no
code with the product's C++ loader (nr-ray-tracer_amd/csrc/scene_config.cpp),
so comparing the two (tests/test_loader_parity.py) checks the product loader.

Tree format (one item per line, floats as float.hex()):
    CAMERA W H spp bounces bg3 look_from3 look_at3 view_up3 defocus_rad focus fov_rad
    TEX id SOLID r g b | TEX id IMAGE w h <raw f32 file> | TEX id CHECKER even odd scale
    TEX id NOISE seed octaves frequency lacunarity persistence | TEX id MARBLE seed frequency
    MAT id LAMBERTIAN tex | METAL fuzz tex | DIELECTRIC ri | DIFFUSE_LIGHT intensity tex
    OBJ id SPHERE c3 r mat [speed3] | QUAD p3 u3 v3 mat | TRIANGLE p3 u3 v3 mat
    OBJ id BVH n child... | TRANSLATE child o3 | ROTATE x|y|z child angle | SCALE child s3
    ROOT id

Number parsing: Python's json / tomli give correctly rounded floats; serde_json
1.0.145 (no float_roundtrip) agrees on every number with a <2^53 significand and
|exp10| <= 22, which covers every file in the reference's scenes/.
"""
from __future__ import annotations

import json
import math
import os
import sys
from dataclasses import dataclass, field
from typing import Any

import tomli

PI = math.pi


class LoadError(Exception):
    pass


def _f(x: float) -> str:
    return float(x).hex()


@dataclass
class CameraConfig:  # cli.rs:160-270
    width: int | None = None
    height: int | None = None
    aspect_ratio: float | None = None
    background_color: tuple | None = None
    look_at: tuple | None = None
    look_from: tuple | None = None
    view_up: tuple | None = None
    focal_length: float | None = None
    field_of_view: float | None = None
    defocus_angle: float | None = None
    focus_distance: float | None = None
    samples_per_pixel: int | None = None
    ray_max_bounces: int | None = None

    MERGE_ORDER = ("background_color", "width", "height", "aspect_ratio", "field_of_view", "focus_distance",
                   "defocus_angle", "samples_per_pixel", "ray_max_bounces", "view_up", "look_at", "look_from")

    def merge_with(self, other: "CameraConfig") -> None:  # cli.rs:316-355 (focal_length not merged)
        for k in self.MERGE_ORDER:
            v = getattr(other, k)
            if v is not None:
                setattr(self, k, v)


@dataclass
class CameraBuilder:  # camera.rs:162-203
    width: int = 1200
    height: int = 800
    background_color: tuple = (0.0, 0.0, 0.0)
    look_from: tuple = (1.0, 1.0, 1.0)
    look_at: tuple = (0.0, 0.0, 0.0)
    view_up: tuple = (0.0, 1.0, 0.0)
    defocus_angle: float = 0.0
    focus_dist: float = 1.0
    field_of_view: float = PI / 2.0
    ray_max_bounces: int = 10
    samples_per_pixel: int = 10


def _as_usize_cast(x: float) -> int:  # Rust `as usize` saturating
    if x != x or x <= 0:
        return 0
    return min(int(x), 2**64 - 1)


def try_update(cfg: CameraConfig, b: CameraBuilder) -> None:  # cli.rs:273-312, 357-402
    w, h, r = cfg.width, cfg.height, cfg.aspect_ratio
    key = (w is not None, h is not None, r is not None)
    if key == (True, True, False):
        b.width, b.height = w, h
    elif key == (True, False, True):
        b.width, b.height = w, max(_as_usize_cast(float(w) / r), 1)
    elif key == (False, True, True):
        b.width, b.height = max(_as_usize_cast(float(h) * r), 1), h
    elif key != (False, False, False):
        raise LoadError("invalid image size arguments")
    if cfg.background_color is not None:
        b.background_color = cfg.background_color
    if cfg.field_of_view is not None:
        b.field_of_view = (cfg.field_of_view * PI) / 180.0
    if cfg.focus_distance is not None:
        b.focus_dist = cfg.focus_distance
    if cfg.defocus_angle is not None:
        b.defocus_angle = (cfg.defocus_angle * PI) / 180.0
    if cfg.samples_per_pixel is not None:
        b.samples_per_pixel = cfg.samples_per_pixel
    if cfg.ray_max_bounces is not None:
        b.ray_max_bounces = cfg.ray_max_bounces
    if cfg.view_up is not None:
        b.view_up = cfg.view_up
    if cfg.look_at is not None:
        b.look_at = cfg.look_at
    if cfg.look_from is not None:
        b.look_from = cfg.look_from


def _num(v: Any, what: str) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise LoadError(f"invalid type for `{what}`: expected f64")
    return float(v)


def _usize(v: Any, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, int) or v < 0:
        raise LoadError(f"invalid type for `{what}`: expected usize")
    return v


def _u32(v: Any, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, int) or not 0 <= v <= 0xFFFFFFFF:
        raise LoadError(f"invalid type for `{what}`: expected u32")
    return v


def _vec3(v: Any, what: str) -> tuple:
    if not isinstance(v, list) or len(v) != 3:
        raise LoadError(f"invalid value for `{what}`")
    return tuple(_num(x, what) for x in v)


def camera_config(d: Any) -> CameraConfig:
    if not isinstance(d, dict):
        raise LoadError("invalid type for `camera`")
    c = CameraConfig()
    conv = {"width": _usize, "height": _usize, "aspect_ratio": _num, "background_color": _vec3, "look_at": _vec3,
            "look_from": _vec3, "view_up": _vec3, "focal_length": _num, "field_of_view": _num,
            "defocus_angle": _num, "focus_distance": _num, "samples_per_pixel": _usize, "ray_max_bounces": _usize}
    for k, fn in conv.items():
        if d.get(k) is not None:
            setattr(c, k, fn(d[k], k))
    return c


def _variant(v: Any, ctx: str) -> tuple[str, dict]:
    if not isinstance(v, dict) or len(v) != 1:
        raise LoadError(f"invalid {ctx}")
    (k, body), = v.items()
    if not isinstance(body, dict):
        raise LoadError(f"invalid {ctx} body")
    return k, body


def _pairs(v: Any, ctx: str) -> list:
    """Vec<(Box<str>, T)>; the legacy TOML table form is accepted too."""
    if v is None:
        return []
    if isinstance(v, list):
        out = []
        for e in v:
            if not (isinstance(e, list) and len(e) == 2 and isinstance(e[0], str)):
                raise LoadError(f"invalid {ctx} entry")
            out.append((e[0], e[1]))
        return out
    if isinstance(v, dict):
        return list(v.items())
    raise LoadError(f"invalid type for `{ctx}`")


class TreeWriter:
    def __init__(self, texel_dir: str):
        self.lines: list[str] = []
        self.ntex = self.nmat = self.nobj = 0
        self.texel_dir = texel_dir
        self.image_cache: dict[str, tuple[int, int, str]] = {}

    def tex(self, body: str) -> int:
        i = self.ntex
        self.ntex += 1
        self.lines.append(f"TEX {i} {body}")
        return i

    def mat(self, body: str) -> int:
        i = self.nmat
        self.nmat += 1
        self.lines.append(f"MAT {i} {body}")
        return i

    def obj(self, body: str) -> int:
        i = self.nobj
        self.nobj += 1
        self.lines.append(f"OBJ {i} {body}")
        return i

    def image(self, path: str) -> tuple[int, int, str]:
        """Image::try_from_path -> into_rgb32f: u8/255 per channel (decoded with PIL)."""
        if path not in self.image_cache:
            from PIL import Image
            import numpy as np

            if not os.path.exists(path):
                raise LoadError(f"No such file or directory (os error 2): {path}")
            im = Image.open(path).convert("RGB")
            arr = np.asarray(im, dtype=np.uint8).astype(np.float32) / np.float32(255.0)
            os.makedirs(self.texel_dir, exist_ok=True)
            raw = os.path.join(self.texel_dir, f"tex{len(self.image_cache)}.f32")
            arr.astype("<f4").tofile(raw)
            self.image_cache[path] = (im.width, im.height, os.path.abspath(raw))
        return self.image_cache[path]


class Builder:
    def __init__(self, w: TreeWriter, legacy: bool = False):
        self.w = w
        self.depth = 0
        self.legacy = legacy

    def make_texture(self, cfg: Any, textures: dict) -> int:  # scene_config.rs:52-123
        kind, b = _variant(cfg, "texture config")
        if kind == "SolidColor":
            c = _vec3(b.get("color"), "color")
            return self.w.tex("SOLID " + " ".join(_f(x) for x in c))
        if kind == "Image":
            if not isinstance(b.get("path"), str):
                raise LoadError("missing field `path`")
            wd, ht, raw = self.w.image(b["path"])
            return self.w.tex(f"IMAGE {wd} {ht} {raw}")
        if kind == "Checker":
            even = self.w.tex("SOLID " + " ".join(_f(x) for x in (1.0, 1.0, 1.0)))
            odd = self.w.tex("SOLID " + " ".join(_f(x) for x in (0.0, 0.0, 0.0)))
            if b.get("even") is not None:
                if b["even"] not in textures:
                    raise LoadError("invalid texture index")
                even = textures[b["even"]]
            if b.get("odd") is not None:
                if b["odd"] not in textures:
                    raise LoadError("invalid texture index")
                odd = textures[b["odd"]]
            scale = _num(b["scale"], "scale") if b.get("scale") is not None else 0.5
            return self.w.tex(f"CHECKER {even} {odd} {_f(scale)}")
        if kind == "Marble":  # MarbleBuilder (marble.rs:46-60); the oracle applies octaves = 7
            seed = _u32(b["seed"], "seed") if b.get("seed") is not None else 0
            freq = _num(b["frequency"], "frequency") if b.get("frequency") is not None else 1.0
            return self.w.tex(f"MARBLE {seed} {_f(freq)}")
        if kind == "Noise":  # PerlinRidgedNoiseBuilder (noise.rs:79-101): builder defaults, Fbm clamps
            seed = _u32(b["seed"], "seed") if b.get("seed") is not None else 0
            octaves = _usize(b["octaves"], "octaves") if b.get("octaves") is not None else 1
            freq = _num(b["frequency"], "frequency") if b.get("frequency") is not None else 1.0
            lac = _num(b["lacunarity"], "lacunarity") if b.get("lacunarity") is not None else math.pi * 2.0 / 3.0
            pers = _num(b["persistence"], "persistence") if b.get("persistence") is not None else 0.5
            return self.w.tex(f"NOISE {seed} {octaves} {_f(freq)} {_f(lac)} {_f(pers)}")
        raise LoadError(f"unknown variant `{kind}`")

    @staticmethod
    def _get_tex(b: dict, textures: dict, fallback: int) -> int:
        if b.get("texture") is None:
            return fallback
        t = b["texture"]
        if t not in textures:
            raise LoadError(f"invalid texture id: '{t}'")
        return textures[t]

    def make_material(self, cfg: Any, textures: dict, tex_fallback: int) -> int:  # scene_config.rs:162-198
        kind, b = _variant(cfg, "material config")
        if kind == "Dielectric":
            return self.w.mat(f"DIELECTRIC {_f(_num(b['refraction_index'], 'refraction_index'))}")
        if kind == "DiffuseLight":
            inten = _num(b["intensity"], "intensity")
            t = self._get_tex(b, textures, tex_fallback)
            return self.w.mat(f"DIFFUSE_LIGHT {_f(inten)} {t}")
        if kind == "Lambertian":
            return self.w.mat(f"LAMBERTIAN {self._get_tex(b, textures, tex_fallback)}")
        if kind == "Metal":
            fuzz = _num(b["fuzz"], "fuzz")
            return self.w.mat(f"METAL {_f(fuzz)} {self._get_tex(b, textures, tex_fallback)}")
        raise LoadError(f"unknown variant `{kind}`")

    @staticmethod
    def _get_mat(b: dict, materials: dict, fallback: int) -> int:
        if b.get("material") is None:
            return fallback
        m = b["material"]
        if m not in materials:
            raise LoadError(f"invalid material id: '{m}'")
        return materials[m]

    def make_object(self, cfg: Any, instances: dict, materials: dict, fallback: int) -> int:  # :277-381
        kind, b = _variant(cfg, "object config")
        if kind in ("Quad", "Triangle"):
            m = self._get_mat(b, materials, fallback)
            p, u, v = (_vec3(b[k], k) for k in ("point", "u", "v"))
            return self.w.obj(f"{kind.upper()} " + " ".join(_f(x) for x in (*p, *u, *v)) + f" {m}")
        if kind == "Sphere":
            m = self._get_mat(b, materials, fallback)
            c = _vec3(b["center"], "center")
            r = _num(b["radius"], "radius")
            return self.w.obj("SPHERE " + " ".join(_f(x) for x in (*c, r)) + f" {m}")
        if kind == "Group":
            m = self._get_mat(b, materials, fallback)
            kids = [self.make_object(o, instances, materials, m) for o in b["objects"]]
            return self.w.obj(f"BVH {len(kids)} " + " ".join(map(str, kids)))
        if kind == "Scene":
            m = self._get_mat(b, materials, fallback)
            self.depth += 1
            if self.depth > 64:
                raise LoadError("nested scene too deep")
            root, _ = self.build_aux(load_doc(b["path"], self.legacy), m, None)
            self.depth -= 1
            return root
        if kind == "Ref":
            if b.get("id") not in instances:
                raise LoadError("invalid object id")
            return instances[b["id"]]
        child = lambda: self.make_object(b["object"], instances, materials, fallback)  # noqa: E731
        if kind in ("RotateX", "RotateY", "RotateZ"):
            a = _num(b["angle"], "angle")
            return self.w.obj(f"ROTATE {kind[-1].lower()} {child()} {_f(a)}")
        if kind == "ScaleU":
            f = _num(b["factor"], "factor")
            s = (f * 1.0, f * 1.0, f * 1.0)
            return self.w.obj(f"SCALE {child()} " + " ".join(_f(x) for x in s))
        if kind == "ScaleV":
            s = _vec3(b["scale"], "scale")
            return self.w.obj(f"SCALE {child()} " + " ".join(_f(x) for x in s))
        if kind == "Translate":
            o = _vec3(b["offset"], "offset")
            return self.w.obj(f"TRANSLATE {child()} " + " ".join(_f(x) for x in o))
        raise LoadError(f"unknown variant `{kind}`")

    def build_aux(self, doc: Any, material_fallback: int | None, cli: CameraConfig | None):
        if not isinstance(doc, dict) or "camera" not in doc:
            raise LoadError("missing field `camera`")
        cam = camera_config(doc["camera"])
        if cli is not None:
            cam.merge_with(cli)
        textures: dict = {}
        for tid, tcfg in _pairs(doc.get("textures"), "textures"):
            textures[tid] = self.make_texture(tcfg, textures)
        if doc.get("texture_fallback") is not None:
            tex_fallback = self.make_texture(doc["texture_fallback"], textures)
        else:
            tex_fallback = self.w.tex("SOLID " + " ".join(_f(0.5 * 1.0) for _ in range(3)))
        materials: dict = {}
        for mid, mcfg in _pairs(doc.get("materials"), "materials"):
            materials[mid] = self.make_material(mcfg, textures, tex_fallback)
        # unwrap_or evaluates its argument eagerly (scene_config.rs:437-443)
        if doc.get("material_fallback") is not None:
            own = self.make_material(doc["material_fallback"], textures, tex_fallback)
        else:
            own = self.w.mat(f"LAMBERTIAN {tex_fallback}")
        fb = material_fallback if material_fallback is not None else own
        instances: dict = {}
        for iid, icfg in _pairs(doc.get("instances"), "instances"):
            instances[iid] = self.make_object(icfg, instances, materials, fb)
        objs = [self.make_object(o, instances, materials, fb) for o in (doc.get("scene") or [])]
        builder = CameraBuilder()
        try_update(cam, builder)
        root = self.w.obj(f"BVH {len(objs)} " + " ".join(map(str, objs)))
        return root, builder


_LEGACY_REFS = ("material", "texture", "even", "odd")


def _legacy_refs(v: Any) -> Any:
    """Integer texture / material references of the legacy schema -> the ids normalize_legacy gives."""
    if isinstance(v, dict):
        return {k: (str(x) if k in _LEGACY_REFS and isinstance(x, int) and not isinstance(x, bool) else _legacy_refs(x))
                for k, x in v.items()}
    if isinstance(v, list):
        return [_legacy_refs(x) for x in v]
    return v


def normalize_legacy(doc: Any) -> Any:
    """The legacy scene schema of scenes/triangles.toml:22-189: `textures` and
    `materials` are arrays of variant tables referenced by integer index and the objects
    sit in `objects`.  It maps onto the current schema with ids "0", "1", ... -- the scene
    `nr-ray-tracer create triangles` now writes with named ids (create/triangles.rs:10-86)."""
    if not isinstance(doc, dict) or "objects" not in doc or "scene" in doc:
        return doc
    out = dict(doc)
    for key in ("textures", "materials"):
        v = doc.get(key)
        if isinstance(v, list) and all(isinstance(e, dict) for e in v):
            out[key] = [[str(i), _legacy_refs(e)] for i, e in enumerate(v)]
    out["scene"] = _legacy_refs(out.pop("objects"))
    return out


def load_doc(path: str, legacy: bool = False) -> Any:  # scene_config.rs:475-492
    ext = os.path.splitext(path)[1]
    if ext not in (".json", ".toml"):
        raise LoadError("invalid scene file format!")
    if not os.path.exists(path):
        raise LoadError(f"No such file or directory (os error 2): {path}")
    with open(path, "rb") as fh:
        raw = fh.read()
    doc = json.loads(raw.decode("utf-8")) if ext == ".json" else tomli.loads(raw.decode("utf-8"))
    return normalize_legacy(doc) if legacy else doc  # the legacy schema only on request


def build_tree(path: str, overrides: CameraConfig | None, texel_dir: str,
               legacy: bool = False) -> tuple[str, CameraBuilder]:
    """SceneConfig::try_load_scene + merge_with(cli) + try_build -> tree text (legacy: also the
    index schema of scenes/triangles.toml, mapped by normalize_legacy)."""
    w = TreeWriter(texel_dir)
    root, cam = Builder(w, legacy).build_aux(load_doc(path, legacy), None, overrides)
    head = ("CAMERA {} {} {} {} ".format(cam.width, cam.height, cam.samples_per_pixel, cam.ray_max_bounces)
            + " ".join(_f(x) for x in (*cam.background_color, *cam.look_from, *cam.look_at, *cam.view_up))
            + f" {_f(cam.defocus_angle)} {_f(cam.focus_dist)} {_f(cam.field_of_view)}")
    return "\n".join([head, *w.lines, f"ROOT {root}"]) + "\n", cam


def main(argv: list[str]) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="scene file -> oracle tree (test infrastructure)")
    ap.add_argument("scene")
    ap.add_argument("out")
    ap.add_argument("-W", "--width", type=int)
    ap.add_argument("-H", "--height", type=int)
    ap.add_argument("--samples-per-pixel", type=int)
    ap.add_argument("--ray-max-bounces", type=int)
    ap.add_argument("--texel-dir", default=None)
    a = ap.parse_args(argv)
    cli = CameraConfig(width=a.width, height=a.height, samples_per_pixel=a.samples_per_pixel,
                       ray_max_bounces=a.ray_max_bounces)
    text, _ = build_tree(a.scene, cli, a.texel_dir or os.path.dirname(os.path.abspath(a.out)))
    with open(a.out, "w") as fh:
        fh.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
