#!/usr/bin/env python3
"""Generate tests/golden/scenes/utah-teapot-model.toml.

The reference's utah-teapot-scene.json instances scenes/utah-teapot-model.toml,
which the reference repository does not contain.  This script builds a teapot
triangle mesh and writes it the way the reference's `convert-stl` command
would (app/commands/create/convert_stl.rs:19-138):

  * vertices read as (x, z, -y)              (convert_stl.rs:45)
  * k = 1 / max extent, point = k (a - p_min), u = k (b - a), v = k (c - a)
  * one Group of Triangle objects, camera look_at (k l/2, k h/2, 0),
    look_from = look_at + Z, white background, fov 50, 50 bounces, spp 200,
    header line "# model bbox: l=.. h=.. w=.."

Geometry (z up, classic teapot units): body, lid and knob are surfaces of
revolution of cubic Bezier profiles; spout and handle are tubes swept along
cubic Bezier centre lines.  The extents are the classic Newell teapot's
(x -3.0 .. 3.434, |y| <= 2.0, z 0 .. 3.15: 6.434 x 3.15 x 4.0 after the swap,
1 : 0.4896 : 0.6217), which the scene's Translate(-0.5, -0.244, -0.311)
centres.  The Newell patch data itself is not used: this is a generated
stand-in, so C4 parity is oracle-vs-GPU on this model (reference parity
unpinned).  Deterministic: same file every run.
"""
import math
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "scenes",
                   "utah-teapot-model.toml")


def bez(p, t):
    a, b, c, d = p
    s = 1.0 - t
    return tuple(s * s * s * a[i] + 3 * s * s * t * b[i] + 3 * s * t * t * c[i] + t * t * t * d[i]
                 for i in range(len(a)))


def bez_d(p, t):
    a, b, c, d = p
    s = 1.0 - t
    return tuple(3 * s * s * (b[i] - a[i]) + 6 * s * t * (c[i] - b[i]) + 3 * t * t * (d[i] - c[i])
                 for i in range(len(a)))


# (r, z) profiles of the rotational parts, outer surface, top to bottom
BODY = [
    [(1.4, 2.4), (1.3375, 2.53125), (1.4375, 2.53125), (1.5, 2.4)],   # rim lip
    [(1.5, 2.4), (1.75, 1.875), (2.0, 1.35), (2.0, 0.9)],             # upper body
    [(2.0, 0.9), (2.0, 0.45), (1.5, 0.225), (1.5, 0.15)],             # lower body
    [(1.5, 0.15), (1.5, 0.075), (1.425, 0.0), (0.0, 0.0)],            # bottom
]
LID = [
    [(0.0, 3.15), (0.8, 3.15), (0.0, 2.85), (0.2, 2.7)],              # knob
    [(0.2, 2.7), (0.4, 2.55), (1.3, 2.55), (1.3, 2.4)],               # lid
]
# swept parts: centre line (x, z) and radius profile (ry, rz half-widths)
SPOUT = ([(1.7, 1.275), (2.6, 1.275), (2.3, 1.95), (2.7, 2.25)],
         [(2.7, 2.25), (2.97, 2.42), (3.2, 2.45), (3.357, 2.4)])
HANDLE = ([(-1.55, 1.99), (-2.4, 1.99), (-2.85, 1.99), (-2.85, 1.65)],
          [(-2.85, 1.65), (-2.85, 1.31), (-2.575, 0.88), (-1.95, 0.6)])


def revolve(profile_segs, n_around, n_per_seg):
    pts = []
    for seg in profile_segs:
        for j in range(n_per_seg + (1 if seg is profile_segs[-1] else 0)):
            pts.append(bez(seg, j / n_per_seg))
    tris = []
    ring = lambda r, z: [(r * math.cos(2 * math.pi * k / n_around), r * math.sin(2 * math.pi * k / n_around), z)
                         for k in range(n_around)]
    rings = [ring(r, z) for r, z in pts]
    for a in range(len(rings) - 1):
        for k in range(n_around):
            k2 = (k + 1) % n_around
            p00, p01, p10, p11 = rings[a][k], rings[a][k2], rings[a + 1][k], rings[a + 1][k2]
            tris.append((p00, p10, p11))
            tris.append((p00, p11, p01))
    return tris


def sweep(centre_segs, radius, n_around, n_per_seg):
    """Tube along a planar (x, z) centre line; radius(t in [0,1]) -> (r_side, r_plane)."""
    frames = []
    total = len(centre_segs) * n_per_seg
    idx = 0
    for seg in centre_segs:
        for j in range(n_per_seg + (1 if seg is centre_segs[-1] else 0)):
            t = j / n_per_seg
            x, z = bez(seg, t)
            dx, dz = bez_d(seg, t)
            L = math.hypot(dx, dz) or 1.0
            nx, nz = -dz / L, dx / L  # in-plane normal of the centre line
            rs, rp = radius(idx / total)
            frames.append([(x + rp * math.cos(a) * nx, rs * math.sin(a), z + rp * math.cos(a) * nz)
                           for a in (2 * math.pi * k / n_around for k in range(n_around))])
            idx += 1
    tris = []
    for a in range(len(frames) - 1):
        for k in range(n_around):
            k2 = (k + 1) % n_around
            p00, p01, p10, p11 = frames[a][k], frames[a][k2], frames[a + 1][k], frames[a + 1][k2]
            tris.append((p00, p10, p11))
            tris.append((p00, p11, p01))
    return tris


def area2(t):
    a, b, c = t
    u = [b[i] - a[i] for i in range(3)]
    v = [c[i] - a[i] for i in range(3)]
    cx = (u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0])
    return math.sqrt(sum(q * q for q in cx))


def build():
    tris = []
    tris += revolve(BODY, 48, 10)
    tris += revolve(LID, 48, 8)
    tris += sweep(SPOUT, lambda s: (0.62 - 0.40 * s, 0.62 - 0.40 * s), 24, 14)
    tris += sweep(HANDLE, lambda s: (0.30, 0.15), 16, 14)
    return [t for t in tris if area2(t) > 1e-12]


def fmt(x):
    r = repr(float(x))
    return "0.0" if r == "-0.0" else r


def write(tris, path):
    # STL (x, y, z) -> convert_stl's DVec3::new(x, z, -y)
    sw = [tuple((p[0], p[2], -p[1]) for p in t) for t in tris]
    lo = [min(p[i] for t in sw for p in t) for i in range(3)]
    hi = [max(p[i] for t in sw for p in t) for i in range(3)]
    l, h, w = hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]
    k = 1.0 / max(l, w, h)
    look_at = (k * l / 2.0, k * h / 2.0, 0.0)
    out = [f"# model bbox: l={k * l:.4f} h={k * h:.4f} w={k * w:.4f}\n",
           "# generated by scripts/make_teapot.py (stand-in for the absent reference model, SURVEY.md Q16)\n",
           "[camera]\n",
           "background_color = [1.0, 1.0, 1.0]\n",
           f"look_at = [{fmt(look_at[0])}, {fmt(look_at[1])}, {fmt(look_at[2])}]\n",
           f"look_from = [{fmt(look_at[0])}, {fmt(look_at[1])}, {fmt(look_at[2] + 1.0)}]\n",
           "field_of_view = 50.0\n", "samples_per_pixel = 200\n", "ray_max_bounces = 50\n\n",
           "[[scene]]\n\n[scene.Group]\n"]
    for a, b, c in sw:
        pt = [k * (a[i] - lo[i]) for i in range(3)]
        u = [k * (b[i] - a[i]) for i in range(3)]
        v = [k * (c[i] - a[i]) for i in range(3)]
        out.append("\n[[scene.Group.objects]]\n\n[scene.Group.objects.Triangle]\n")
        out.append("point = [" + ", ".join(fmt(q) for q in pt) + "]\n")
        out.append("u = [" + ", ".join(fmt(q) for q in u) + "]\n")
        out.append("v = [" + ", ".join(fmt(q) for q in v) + "]\n")
    with open(path, "w") as fh:
        fh.writelines(out)
    return (l, h, w), k


if __name__ == "__main__":
    tris = build()
    (l, h, w), k = write(tris, sys.argv[1] if len(sys.argv) > 1 else OUT)
    print(f"{len(tris)} triangles; extents l={l:.4f} h={h:.4f} w={w:.4f} -> 1 : {h / l:.4f} : {w / l:.4f}")
