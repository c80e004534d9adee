"""Procedural benchmark scenes (no assets ship with the reference).

``write_cornell_box`` emits the config-1/config-2 Cornell box as OBJ+MTL: five
walls, two boxes and a (non-emissive) light-fixture quad, 32 triangles. OBJ
loading creates no lights (reference WavefrontOBJLoading.cpp:305-338), so
``setup_cornell`` adds one point light the way the UI's "Create -> Point Light"
does (ImGui.cpp:322-331). The OBJ is written in right-handed coordinates; the
loader mirrors x into the renderer's left-handed world, exactly like the
reference's OBJ import.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
CORNELL_DIR = ROOT / "tests" / "golden"
CORNELL_OBJ = CORNELL_DIR / "cornell_box.obj"

# world-space (left-handed, y up, camera at (0,1,0) looking +z)
ROOM = dict(x0=-1.5, x1=1.5, y0=0.0, y1=2.0, z0=1.0, z1=4.5)
POINT_LIGHT_POSITION = (0.0, 1.6, 2.8)
POINT_LIGHT_COLOR = (2.0, 2.0, 2.0)

_MTL = """# Cornell box materials (procedural fixture)
newmtl white
Kd 0.73 0.73 0.73
Ni 1.0
newmtl red
Kd 0.65 0.05 0.05
Ni 1.0
newmtl green
Kd 0.12 0.45 0.15
Ni 1.0
newmtl box_short
Kd 0.73 0.73 0.73
Ni 1.5
Pr 0.3
newmtl box_tall
Kd 0.70 0.70 0.75
Ni 1.5
Pr 0.08
newmtl fixture
Kd 0.78 0.78 0.78
Ni 1.0
"""


def _box_faces(cx, cz, sx, sy, sz, angle):
    """Five outward faces (no bottom) of a y-rotated box standing on the floor."""
    c, s = math.cos(angle), math.sin(angle)

    def p(x, y, z):
        return (cx + c * x - s * z, y, cz + s * x + c * z)

    def n(x, y, z):
        return (c * x - s * z, y, s * x + c * z)

    hx, hz = sx / 2, sz / 2
    return [
        ([p(-hx, sy, -hz), p(hx, sy, -hz), p(hx, sy, hz), p(-hx, sy, hz)], n(0, 1, 0)),     # top
        ([p(-hx, 0, -hz), p(hx, 0, -hz), p(hx, sy, -hz), p(-hx, sy, -hz)], n(0, 0, -1)),    # front
        ([p(hx, 0, hz), p(-hx, 0, hz), p(-hx, sy, hz), p(hx, sy, hz)], n(0, 0, 1)),         # back
        ([p(-hx, 0, hz), p(-hx, 0, -hz), p(-hx, sy, -hz), p(-hx, sy, hz)], n(-1, 0, 0)),    # left
        ([p(hx, 0, -hz), p(hx, 0, hz), p(hx, sy, hz), p(hx, sy, -hz)], n(1, 0, 0)),         # right
    ]


def cornell_groups():
    r = ROOM
    x0, x1, y0, y1, z0, z1 = r["x0"], r["x1"], r["y0"], r["y1"], r["z0"], r["z1"]
    groups = [
        ("floor", "white", [([(x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1)], (0, 1, 0))]),
        ("ceiling", "white", [([(x0, y1, z1), (x1, y1, z1), (x1, y1, z0), (x0, y1, z0)], (0, -1, 0))]),
        ("back", "white", [([(x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1)], (0, 0, -1))]),
        ("left", "red", [([(x0, y0, z0), (x0, y0, z1), (x0, y1, z1), (x0, y1, z0)], (1, 0, 0))]),
        ("right", "green", [([(x1, y0, z1), (x1, y0, z0), (x1, y1, z0), (x1, y1, z1)], (-1, 0, 0))]),
        ("fixture", "fixture", [([(-0.3, y1 - 0.01, 2.7), (0.3, y1 - 0.01, 2.7), (0.3, y1 - 0.01, 3.3),
                                  (-0.3, y1 - 0.01, 3.3)], (0, -1, 0))]),
        ("short_box", "box_short", _box_faces(0.55, 2.9, 0.7, 0.7, 0.7, math.radians(17.0))),
        ("tall_box", "box_tall", _box_faces(-0.55, 3.6, 0.7, 1.4, 0.7, math.radians(-20.0))),
    ]
    return groups


def cornell_obj_text() -> str:
    lines = ["# Procedural Cornell box (right-handed OBJ; x is mirrored on import)", "mtllib cornell_box.mtl"]
    vi = vti = vni = 0
    for name, mat, quads in cornell_groups():
        lines.append(f"g {name}")
        lines.append(f"usemtl {mat}")
        for quad, normal in quads:
            base_v, base_t, base_n = vi, vti, vni
            for (x, y, z) in quad:
                lines.append(f"v {-x:.6f} {y:.6f} {z:.6f}")
                vi += 1
            for (s, t) in ((0, 0), (1, 0), (1, 1), (0, 1)):
                lines.append(f"vt {s} {t}")
                vti += 1
            nx, ny, nz = normal
            lines.append(f"vn {-nx:.6f} {ny:.6f} {nz:.6f}")
            vni += 1
            idx = [f"{base_v + k + 1}/{base_t + k + 1}/{base_n + 1}" for k in range(4)]
            # mirrored x flips handedness: emit the winding the importer swaps back
            lines.append(f"f {idx[0]} {idx[2]} {idx[1]}")
            lines.append(f"f {idx[0]} {idx[3]} {idx[2]}")
    return "\n".join(lines) + "\n"


def write_cornell_box(directory: Path | str = CORNELL_DIR) -> Path:
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    obj = d / "cornell_box.obj"
    text = cornell_obj_text()
    if not obj.exists() or obj.read_text() != text:
        obj.write_text(text)
    mtl = d / "cornell_box.mtl"
    if not mtl.exists() or mtl.read_text() != _MTL:
        mtl.write_text(_MTL)
    return obj


def setup_cornell(scene, width: int, height: int, max_bounce: int, obj_path: Path | None = None):
    """Config 1/2: Reset defaults (Scene.cpp:626-660) + OBJ + one point light."""
    path = Path(obj_path) if obj_path else CORNELL_OBJ
    if not path.exists():
        path = write_cornell_box(path.parent)
    scene.reset(width, height)
    scene.load_from_file(path)
    scene.add_point_light(POINT_LIGHT_POSITION, POINT_LIGHT_COLOR)
    scene.set_max_bounce(max_bounce)
    return scene


def env_cube(size: int = 16, seed: int = 1234) -> np.ndarray:
    """Procedural float cube map (6 x size x size x 3) for HAS_ENV_TEXTURE tests."""
    rng = np.random.default_rng(seed)
    base = rng.uniform(0.05, 1.5, size=(6, 1, 1, 3)).astype(np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, size, dtype=np.float32), np.linspace(0, 1, size, dtype=np.float32),
                         indexing="ij")
    grad = (0.5 + 0.5 * np.sin(6.0 * xx + 3.0 * yy))[None, :, :, None]
    return np.ascontiguousarray(base * grad, dtype=np.float32)
