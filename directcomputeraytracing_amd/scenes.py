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


# ---------------------------------------------------------------------------------------
# Mitsuba 3 XML scenes for configs 3-5 (coffee-like, spaceship-like, lamp-like). All
# geometry is procedural with a fixed seed; OBJ meshes are loaded through the XML path
# (one mesh per file, instanced by repeated <shape type="obj">, SceneXMLLoading.cpp).
# Coordinates are Mitsuba's (right-handed, y up); the loader converts them.

def mitsuba_matrix(translate=(0.0, 0.0, 0.0), yaw=0.0, pitch=0.0, scale=(1.0, 1.0, 1.0)) -> str:
    """Row-major 4x4 (column-vector convention) = T * Ry(yaw) * Rx(pitch) * S, degrees."""
    cy, sy = math.cos(math.radians(yaw)), math.sin(math.radians(yaw))
    cp, sp = math.cos(math.radians(pitch)), math.sin(math.radians(pitch))
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    m = np.eye(4)
    m[:3, :3] = ry @ rx @ np.diag(scale)
    m[:3, 3] = translate
    # single spaces only: the reference splits the value on ' ' and needs exactly 16 fields
    return " ".join(f"{v:.6g}" for v in m.reshape(-1))


def lathe(profile, segments: int):
    """Surface of revolution about +y. profile: [(r, y), ...]. Returns V, N, UV, F (0-based)."""
    prof = np.asarray(profile, np.float64)
    n = len(prof)
    # profile tangents -> outward 2D normals (r, y) rotated by -90 degrees
    t = np.gradient(prof, axis=0)
    t /= np.maximum(np.linalg.norm(t, axis=1, keepdims=True), 1e-12)
    n2 = np.stack([t[:, 1], -t[:, 0]], axis=1)
    phi = np.linspace(0.0, 2 * math.pi, segments, endpoint=False)
    c, s = np.cos(phi), np.sin(phi)
    V = np.stack([np.outer(prof[:, 0], c), np.repeat(prof[:, 1:2], segments, 1), np.outer(prof[:, 0], s)], -1).reshape(-1, 3)
    N = np.stack([np.outer(n2[:, 0], c), np.repeat(n2[:, 1:2], segments, 1), np.outer(n2[:, 0], s)], -1).reshape(-1, 3)
    N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-12)
    u = np.tile(np.arange(segments) / segments, n)
    v = np.repeat(np.linspace(0, 1, n), segments)
    UV = np.stack([u, v], 1)
    i = np.arange(n - 1)[:, None] * segments
    j = np.arange(segments)[None, :]
    a = (i + j).reshape(-1)
    b = (i + (j + 1) % segments).reshape(-1)
    F = np.concatenate([np.stack([a, b, a + segments], 1), np.stack([b, b + segments, a + segments], 1)])
    # drop triangles collapsed on the axis (r == 0 rings)
    area = np.linalg.norm(np.cross(V[F[:, 1]] - V[F[:, 0]], V[F[:, 2]] - V[F[:, 0]]), axis=1)
    return V, N, UV, F[area > 1e-12]


def write_obj(path: Path, V, N, UV, F) -> Path:
    """Vertices/normals/texcoords share indices (f a/a/a ...); 1-based."""
    path = Path(path)
    lines = [f"# procedural mesh, {len(F)} triangles"]
    lines += [f"v {x:.6f} {y:.6f} {z:.6f}" for x, y, z in V]
    lines += [f"vn {x:.6f} {y:.6f} {z:.6f}" for x, y, z in N]
    lines += [f"vt {x:.6f} {y:.6f}" for x, y in UV]
    F1 = np.asarray(F) + 1
    lines += [f"f {a}/{a}/{a} {b}/{b}/{b} {c}/{c}/{c}" for a, b, c in F1]
    text = "\n".join(lines) + "\n"
    if not path.exists() or path.read_text() != text:
        path.write_text(text)
    return path


def _xml(body: str) -> str:
    return '<?xml version="1.0" encoding="utf-8"?>\n<scene version="3.0.0">\n' + body + "</scene>\n"


def _sensor(kind, width, height, to_world, extra="", rfilter='<rfilter type="gaussian"><float name="stddev" value="0.5"/></rfilter>'):
    return (f'  <sensor type="{kind}">\n{extra}'
            f'    <transform name="to_world"><matrix value="{to_world}"/></transform>\n'
            f'    <film type="hdrfilm"><integer name="width" value="{width}"/><integer name="height" value="{height}"/>\n'
            f'      {rfilter}</film>\n  </sensor>\n')


def write_coffee(directory: Path | str, width: int = 1920, height: int = 1080, segments: int = 96) -> Path:
    """Config 3: roughconductor / roughplastic / roughdielectric, MIS, constant env (+ cube map
    set through the API, the HAS_ENV_TEXTURE path), path max_depth 8."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    cup = [(0.0, 0.0), (0.26, 0.0), (0.30, 0.02), (0.32, 0.2), (0.35, 0.45), (0.38, 0.68), (0.385, 0.7),
           (0.36, 0.7), (0.355, 0.66), (0.33, 0.45), (0.30, 0.2), (0.27, 0.06), (0.0, 0.06)]
    write_obj(d / "cup.obj", *lathe(_densify(cup, 40), segments))
    write_obj(d / "coffee.obj", *lathe([(0.34, 0.6), (0.17, 0.6), (0.0, 0.6)], segments))   # normal up
    saucer = [(0.0, 0.0), (0.45, 0.0), (0.6, 0.06), (0.62, 0.08), (0.6, 0.08), (0.45, 0.03), (0.0, 0.03)]
    write_obj(d / "saucer.obj", *lathe(_densify(saucer, 30), segments))
    glass = [(0.0, 0.0), (0.2, 0.0), (0.22, 0.9), (0.2, 0.9), (0.18, 0.05), (0.0, 0.05)]
    write_obj(d / "glass.obj", *lathe(_densify(glass, 30), segments))
    body = (
        '  <integrator type="path"><integer name="max_depth" value="8"/></integrator>\n'
        + _sensor("perspective", width, height, mitsuba_matrix((0.3, 1.35, -3.2), yaw=-5, pitch=18),
                  '    <float name="fov" value="38"/>\n')
        + '  <bsdf type="twosided" id="wood"><bsdf type="roughplastic"><rgb name="diffuse_reflectance" value="0.35, 0.2, 0.1"/>'
          '<float name="alpha" value="0.2"/><boolean name="nonlinear" value="true"/></bsdf></bsdf>\n'
          '  <bsdf type="diffuse" id="wall"><rgb name="reflectance" value="0.7, 0.7, 0.65"/></bsdf>\n'
          '  <bsdf type="roughplastic" id="porcelain"><rgb name="diffuse_reflectance" value="0.9, 0.9, 0.85"/>'
          '<float name="alpha" value="0.05"/><float name="int_ior" value="1.5"/></bsdf>\n'
          '  <bsdf type="plastic" id="coffee"><rgb name="diffuse_reflectance" value="0.15, 0.07, 0.03"/>'
          '<float name="int_ior" value="1.33"/></bsdf>\n'
          '  <bsdf type="roughconductor" id="gold"><rgb name="eta" value="0.143, 0.374, 1.442"/>'
          '<rgb name="k" value="3.983, 2.385, 1.603"/><float name="alpha" value="0.05"/></bsdf>\n'
          '  <bsdf type="roughdielectric" id="glass"><float name="int_ior" value="1.5"/><float name="alpha" value="0.01"/></bsdf>\n'
        f'  <shape type="rectangle" id="shape_table"><ref id="wood"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 0), pitch=-90, scale=(4, 4, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_backwall"><ref id="wall"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 1.5, 3), yaw=180, scale=(5, 3, 1))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_saucer"><string name="filename" value="saucer.obj"/><ref id="gold"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0.001, 0))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_cup"><string name="filename" value="cup.obj"/><ref id="porcelain"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0.031, 0))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_coffee"><string name="filename" value="coffee.obj"/><ref id="coffee"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0.0, 0))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_glass"><string name="filename" value="glass.obj"/><ref id="glass"/><transform name="to_world"><matrix value="{mitsuba_matrix((0.9, 0.0, 0.4))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_softbox"><emitter type="area"><rgb name="radiance" value="6, 5.6, 5"/></emitter><transform name="to_world"><matrix value="{mitsuba_matrix((-1.2, 2.6, -0.5), pitch=90, scale=(0.6, 0.6, 1))}"/></transform></shape>\n'
        '  <emitter type="constant"><rgb name="radiance" value="0.6, 0.65, 0.75"/></emitter>\n'
    )
    p = d / "coffee.xml"
    p.write_text(_xml(body))
    return p


def _densify(profile, n):
    """Resample a polyline profile to about n points (keeps corners)."""
    pts = np.asarray(profile, np.float64)
    seg = np.linalg.norm(np.diff(pts, axis=0), axis=1)
    out = [pts[0]]
    per = max(1, n // max(1, len(seg)))
    for k in range(len(seg)):
        for t in np.linspace(0, 1, per + 1)[1:]:
            out.append(pts[k] * (1 - t) + pts[k + 1] * t)
    return [tuple(p) for p in out]


def hull_mesh(nu: int, nv: int, seed: int = 1234):
    """Spaceship-like hull: an elongated ellipsoid with panelled, greebled displacement."""
    rng = np.random.default_rng(seed)
    u = np.linspace(0, 2 * math.pi, nu, endpoint=False)
    v = np.linspace(0.02, math.pi - 0.02, nv)
    U, Vv = np.meshgrid(u, v)
    panels = rng.uniform(-1, 1, size=(16, 32))
    pu = (U / (2 * math.pi) * 32).astype(int) % 32
    pv = (Vv / math.pi * 16).astype(int).clip(0, 15)
    disp = 1 + 0.04 * panels[pv, pu] + 0.03 * np.sin(7 * U) * np.sin(5 * Vv)
    x = 0.55 * np.sin(Vv) * np.cos(U) * disp
    y = 0.35 * np.sin(Vv) * np.sin(U) * disp
    z = 2.0 * np.cos(Vv) * (1 + 0.02 * panels[pv, pu])
    V = np.stack([x, y, z], -1).reshape(-1, 3)
    # normals from the grid
    P = V.reshape(nv, nu, 3)
    du = np.roll(P, -1, axis=1) - np.roll(P, 1, axis=1)
    dv = np.concatenate([P[1:2] - P[0:1], P[2:] - P[:-2], P[-1:] - P[-2:-1]], axis=0)
    N = np.cross(dv, du).reshape(-1, 3)
    N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-12)
    UV = np.stack([(U / (2 * math.pi)).reshape(-1), (Vv / math.pi).reshape(-1)], 1)
    i = np.arange(nv - 1)[:, None] * nu
    j = np.arange(nu)[None, :]
    a = (i + j).reshape(-1)
    b = (i + (j + 1) % nu).reshape(-1)
    F = np.concatenate([np.stack([a, a + nu, b], 1), np.stack([b, a + nu, b + nu], 1)])
    return V, N, UV, F


def write_spaceship(directory: Path | str, width: int = 3840, height: int = 2160, nu: int = 512, nv: int = 256,
                    ships: int = 8, seed: int = 1234, framing: str = "wide") -> Path:
    """Config 4: one procedural hull mesh (2*nu*(nv-1) triangles) instanced `ships` times
    through repeated <shape type="obj"> with the same filename; engine glows are area lights.

    framing "wide" (the configs[3] scene since round 1): ships scattered over a deep field,
    about 10 % of the camera rays hit a hull. "close": a fleet in formation filling the frame
    (broadside hulls in rows, staggered in depth) -- most camera rays hit a hull and most paths
    bounce between hulls, a two-level-BVH traversal workload rather than a sky one."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    write_obj(d / f"hull_{nu}x{nv}.obj", *hull_mesh(nu, nv, seed))
    rng = np.random.default_rng(seed)
    shapes = []
    if framing not in ("wide", "close"):
        raise ValueError(f"unknown spaceship framing {framing!r}")
    for k in range(ships):
        if framing == "close":
            col, row = k % 2, k // 2
            pos = (float(-1.45 + 2.9 * col + rng.uniform(-0.2, 0.2)), float(-1.05 + 0.7 * row + rng.uniform(-0.05, 0.05)),
                   float(3.2 + 0.9 * ((row + col) % 3) + rng.uniform(0.0, 0.3)))
            yaw = float(90.0 + rng.uniform(-12, 12))
            pitch = float(rng.uniform(-6, 6))
        else:
            pos = (float(rng.uniform(-4, 4)), float(rng.uniform(-1.5, 1.5)), float(rng.uniform(2, 14)))
            yaw = float(rng.uniform(-60, 60))
            pitch = float(rng.uniform(-15, 15))
        shapes.append(f'  <shape type="obj" id="shape_ship{k}"><string name="filename" value="hull_{nu}x{nv}.obj"/><ref id="hullmetal"/>'
                      f'<transform name="to_world"><matrix value="{mitsuba_matrix(pos, yaw=yaw, pitch=pitch)}"/></transform></shape>\n')
        # engine glow at the stern (local z = -2.02), facing backwards
        yr = math.radians(yaw)
        back = (pos[0] - 2.02 * math.sin(yr), pos[1], pos[2] - 2.02 * math.cos(yr))
        shapes.append(f'  <shape type="rectangle" id="shape_engine{k}"><emitter type="area"><rgb name="radiance" value="4, 6, 12"/></emitter>'
                      f'<transform name="to_world"><matrix value="{mitsuba_matrix(back, yaw=yaw + 180, scale=(0.15, 0.1, 1))}"/></transform></shape>\n')
    camera = mitsuba_matrix((0, 0.5, -6), pitch=3) if framing == "wide" else mitsuba_matrix((0, 0.0, -1.2), pitch=0)
    body = (
        '  <integrator type="path"><integer name="max_depth" value="8"/></integrator>\n'
        + _sensor("perspective", width, height, camera, '    <float name="fov" value="55"/>\n',
                  '<rfilter type="box"><float name="radius" value="1"/></rfilter>')
        + '  <bsdf type="roughconductor" id="hullmetal"><rgb name="eta" value="1.657, 0.880, 0.521"/>'
          '<rgb name="k" value="9.224, 6.270, 4.837"/><float name="alpha" value="0.09"/></bsdf>\n'
        + "".join(shapes)
        + '  <emitter type="constant"><rgb name="radiance" value="0.02, 0.03, 0.06"/></emitter>\n'
          '  <emitter type="directional"><vector name="direction" value="-0.4, -0.5, 0.75"/><rgb name="irradiance" value="3, 2.9, 2.7"/></emitter>\n'
    )
    p = d / (f"spaceship_{nu}x{nv}.xml" if framing == "wide" else f"spaceship_close_{nu}x{nv}.xml")
    p.write_text(_xml(body))
    return p


def write_lamp(directory: Path | str, width: int = 3840, height: int = 2160, segments: int = 96) -> Path:
    """Config 5: thinlens sensor (aperture_radius, focus_distance), rectangle area emitters
    (triangle lights), a rough dielectric shade."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    base = [(0.0, 0.0), (0.35, 0.0), (0.36, 0.04), (0.08, 0.08), (0.05, 0.3), (0.04, 1.2), (0.06, 1.25), (0.0, 1.25)]
    write_obj(d / "lamp_base.obj", *lathe(_densify(base, 40), segments))
    shade = [(0.45, 1.0), (0.22, 1.5)]                     # open truncated cone
    write_obj(d / "lamp_shade.obj", *lathe(_densify(shade, 24), segments))
    body = (
        '  <integrator type="path"><integer name="max_depth" value="8"/></integrator>\n'
        + _sensor("thinlens", width, height, mitsuba_matrix((0.2, 1.2, -3.0), yaw=-4, pitch=6),
                  '    <string name="focal_length" value="50mm"/>\n    <float name="aperture_radius" value="0.012"/>\n'
                  '    <float name="focus_distance" value="3.1"/>\n',
                  '<rfilter type="tent"><float name="radius" value="1"/></rfilter>')
        + '  <bsdf type="roughplastic" id="floor"><rgb name="diffuse_reflectance" value="0.45, 0.3, 0.2"/><float name="alpha" value="0.15"/></bsdf>\n'
          '  <bsdf type="diffuse" id="wall"><rgb name="reflectance" value="0.75, 0.72, 0.7"/></bsdf>\n'
          '  <bsdf type="roughconductor" id="brass"><rgb name="eta" value="0.444, 0.527, 1.094"/>'
          '<rgb name="k" value="3.695, 2.765, 1.829"/><float name="alpha" value="0.1"/></bsdf>\n'
          '  <bsdf type="twosided" id="shade"><bsdf type="roughdielectric"><float name="int_ior" value="1.5"/><float name="alpha" value="0.3"/></bsdf></bsdf>\n'
          '  <bsdf type="thindielectric" id="pane"><float name="int_ior" value="1.5"/></bsdf>\n'
        f'  <shape type="rectangle" id="shape_floor"><ref id="floor"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 1), pitch=-90, scale=(5, 5, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_wall"><ref id="wall"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 2, 2.5), yaw=180, scale=(5, 2, 1))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_base"><string name="filename" value="lamp_base.obj"/><ref id="brass"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 1))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_shade"><string name="filename" value="lamp_shade.obj"/><ref id="shade"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_pane"><ref id="pane"/><transform name="to_world"><matrix value="{mitsuba_matrix((-1.1, 0.6, 0.6), yaw=30, scale=(0.4, 0.6, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_bulb_a"><emitter type="area"><rgb name="radiance" value="40, 34, 26"/></emitter><transform name="to_world"><matrix value="{mitsuba_matrix((0, 1.3, 1), yaw=0, scale=(0.06, 0.1, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_bulb_b"><emitter type="area"><rgb name="radiance" value="40, 34, 26"/></emitter><transform name="to_world"><matrix value="{mitsuba_matrix((0, 1.3, 1), yaw=90, scale=(0.06, 0.1, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_ceiling"><emitter type="area"><rgb name="radiance" value="1.5, 1.6, 1.8"/></emitter><transform name="to_world"><matrix value="{mitsuba_matrix((1.5, 3.2, 1.5), pitch=90, scale=(0.8, 0.8, 1))}"/></transform></shape>\n'
    )
    p = d / "lamp.xml"
    p.write_text(_xml(body))
    return p


def _write_bytes(path: Path, data: bytes) -> Path:
    if not path.exists() or path.read_bytes() != data:
        path.write_bytes(data)
    return path


def write_anyhit(directory: Path | str, width: int = 64, height: int = 48) -> Path:
    """ALLOW_ANYHIT_SHADER / texture fixture: a cut-out leaf (``mask`` BSDF with a PGM opacity
    bitmap) on an OBJ quad, a half-transparent veil (``mask`` with a float opacity) on the
    shared rectangle mesh (material via instance override; the reference's rectangle has zero
    texcoords, Mesh.cpp:31-36), an opaque wall and a floor with a PPM albedo bitmap; an area
    light and a constant environment. Textures are binary PGM/PPM."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    n = 16
    yy, xx = np.mgrid[0:n, 0:n]
    r = np.hypot(xx - (n - 1) / 2, yy - (n - 1) / 2) / (n / 2)
    mask = np.clip(255 * (1.2 - r), 0, 255).astype(np.uint8)
    mask[::4, :] = 0                                   # slits: fully cut-out rows
    _write_bytes(d / "leaf_mask.pgm", f"P5 {n} {n} 255\n".encode() + mask.tobytes())
    m = 8
    checker = ((np.arange(m)[:, None] // 2 + np.arange(m)[None, :] // 2) % 2).astype(bool)
    rgb = np.where(checker[..., None], np.array([200, 180, 60], np.uint8), np.array([40, 90, 160], np.uint8))
    _write_bytes(d / "floor_albedo.ppm", f"P6 {m} {m} 255\n".encode() + rgb.astype(np.uint8).tobytes())
    write_obj(d / "quad.obj", [(-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1)], [(0, 1, 0)] * 4,
              [(0, 0), (1, 0), (1, 1), (0, 1)], [(0, 1, 2), (0, 2, 3)])
    body = (
        '  <integrator type="path"><integer name="max_depth" value="6"/></integrator>\n'
        + _sensor("perspective", width, height, mitsuba_matrix((0.0, 1.0, -3.5), pitch=8),
                  '    <float name="fov" value="55"/>\n')
        + '  <bsdf type="twosided" id="floor"><bsdf type="diffuse"><texture name="reflectance" type="bitmap">'
          '<string name="filename" value="floor_albedo.ppm"/></texture></bsdf></bsdf>\n'
          '  <bsdf type="mask" id="leaf"><texture name="opacity" type="bitmap"><string name="filename" value="leaf_mask.pgm"/>'
          '</texture><bsdf type="twosided"><bsdf type="diffuse"><rgb name="reflectance" value="0.2, 0.7, 0.25"/></bsdf></bsdf></bsdf>\n'
          '  <bsdf type="mask" id="veil"><float name="opacity" value="0.4"/><bsdf type="roughplastic">'
          '<rgb name="diffuse_reflectance" value="0.8, 0.3, 0.3"/><float name="alpha" value="0.1"/></bsdf></bsdf>\n'
          '  <bsdf type="diffuse" id="wall"><rgb name="reflectance" value="0.7, 0.7, 0.7"/></bsdf>\n'
        f'  <shape type="obj" id="shape_floor"><string name="filename" value="quad.obj"/><ref id="floor"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 0), scale=(3, 1, 3))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_wall"><ref id="wall"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 1.5, 2.0), yaw=180, scale=(3, 1.5, 1))}"/></transform></shape>\n'
        f'  <shape type="obj" id="shape_leaf"><string name="filename" value="quad.obj"/><ref id="leaf"/><transform name="to_world"><matrix value="{mitsuba_matrix((-0.5, 1.0, 0.0), pitch=-90, scale=(0.7, 1, 0.7))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_veil"><ref id="veil"/><transform name="to_world"><matrix value="{mitsuba_matrix((0.6, 0.9, 0.6), yaw=180, scale=(0.6, 0.6, 1))}"/></transform></shape>\n'
        f'  <shape type="rectangle" id="shape_light"><emitter type="area"><rgb name="radiance" value="7, 6.5, 6"/></emitter><transform name="to_world"><matrix value="{mitsuba_matrix((0.3, 2.4, -0.5), pitch=90, scale=(0.5, 0.5, 1))}"/></transform></shape>\n'
        '  <emitter type="constant"><rgb name="radiance" value="0.25, 0.3, 0.4"/></emitter>\n'
    )
    p = d / "anyhit.xml"
    p.write_text(_xml(body))
    return p


CONFIGS = ("cornell", "coffee", "spaceship", "lamp", "spaceship_close")


# ---- analytic scenes (tier 6: checks whose answer does not come from the renderer) ----
# Six rectangles (SceneXMLLoading.cpp:1358-1378: one shared rectangle mesh, an instance per face)
# form the cube [-1, 1]^3, each face's front (the rectangle's +z) pointing `inward` or outward.
_CUBE_FACES = [((0, 0, 1), 180, 0), ((0, 0, -1), 0, 0), ((0, 1, 0), 0, 90), ((0, -1, 0), 0, -90),
               ((1, 0, 0), -90, 0), ((-1, 0, 0), 90, 0)]   # (centre, yaw, pitch): fronts facing the centre


def _cube_shapes(inner: str, inward: bool, scale: float = 1.0) -> str:
    out = ""
    for (c, yaw, pitch) in _CUBE_FACES:
        t = tuple(scale * v for v in c)
        m = mitsuba_matrix(t, yaw=yaw + (0 if inward else 180) if pitch == 0 else yaw, pitch=pitch if inward or pitch == 0 else -pitch,
                           scale=(scale, scale, 1))
        out += f'  <shape type="rectangle">{inner}<transform name="to_world"><matrix value="{m}"/></transform></shape>\n'
    return out


def write_emissive_box(directory: Path | str, width: int = 64, height: int = 64, albedo: float = 0.5,
                       radiance: float = 1.0, max_bounce: int = 8) -> Path:
    """The camera inside a closed cube whose six faces are diffuse (albedo rho) AND emit Le towards
    the inside. Every path vertex lies on a wall, so the expected radiance of every pixel is
    Le * (1 + rho + ... + rho^B) for B bounces: emission seen directly plus, at each of the B
    vertices that continue, the next vertex's emission weighted by the albedo (cosine-sampled
    Lambertian: weight rho; light sampling + MIS: the same expectation)."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    inner = (f'<bsdf type="diffuse"><rgb name="reflectance" value="{albedo}, {albedo}, {albedo}"/></bsdf>'
             f'<emitter type="area"><rgb name="radiance" value="{radiance}, {radiance}, {radiance}"/></emitter>')
    xml = _xml(f'  <integrator type="path"><integer name="max_depth" value="{max_bounce}"/></integrator>\n'
               + _sensor("perspective", width, height, mitsuba_matrix((0.1, -0.05, 0.2), yaw=20, pitch=10),
                         extra='    <float name="fov" value="90"/>\n', rfilter='<rfilter type="box"/>')
               + _cube_shapes(inner, inward=True))
    path = d / "emissive_box.xml"
    path.write_text(xml)
    return path


def write_lit_plane(directory: Path | str, width: int = 64, height: int = 64, albedo: float = 0.6) -> Path:
    """A diffuse plane (the rectangle [-4, 4]^2 at y = 0, front +y) seen from above, no light and no
    bounce (max_depth 0): the caller adds a point light, whose direct lighting is then the whole
    image (known irradiance, tests/test_physics.py)."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    xml = _xml('  <integrator type="path"><integer name="max_depth" value="0"/></integrator>\n'
               + _sensor("perspective", width, height, mitsuba_matrix((0.0, 3.0, -1.0), pitch=55),
                         extra='    <float name="fov" value="60"/>\n', rfilter='<rfilter type="box"/>')
               + f'  <bsdf type="diffuse" id="plane"><rgb name="reflectance" value="{albedo}, {albedo}, {albedo}"/></bsdf>\n'
               + f'  <shape type="rectangle"><ref id="plane"/><transform name="to_world"><matrix value="{mitsuba_matrix((0, 0, 0), pitch=-90, scale=(4, 4, 1))}"/></transform></shape>\n')
    path = d / "lit_plane.xml"
    path.write_text(xml)
    return path


def write_furnace(directory: Path | str, width: int = 64, height: int = 64, bsdf: str | None = None,
                  radiance: float = 1.0, max_bounce: int = 8) -> Path:
    """White furnace: a closed cube, fronts outward, under a constant environment of radiance Le,
    the camera outside at a corner so the cube fills the frame. The cube is convex, so a ray leaving
    its surface sees the environment: with an energy-conserving BSDF of albedo 1 (diffuse
    reflectance 1) the expected radiance of every pixel is Le. `bsdf` replaces the material
    (e.g. a rough conductor, for the Kulla-Conty energy check)."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    inner = bsdf or '<bsdf type="diffuse"><rgb name="reflectance" value="1, 1, 1"/></bsdf>'
    xml = _xml(f'  <integrator type="path"><integer name="max_depth" value="{max_bounce}"/></integrator>\n'
               + _sensor("perspective", width, height, mitsuba_matrix((-1.35, 1.3, -1.45), yaw=42, pitch=35),
                         extra='    <float name="fov" value="30"/>\n', rfilter='<rfilter type="box"/>')
               + _cube_shapes(inner, inward=False)
               + f'  <emitter type="constant"><rgb name="radiance" value="{radiance}, {radiance}, {radiance}"/></emitter>\n')
    path = d / "furnace.xml"
    path.write_text(xml)
    return path


def setup_config(scene, name: str, scene_dir: Path | str, small: bool = False, multiscattering: bool = True) -> str:
    """BASELINE.json configs[1..4] as procedural scenes (written into `scene_dir`), loaded
    into `scene` at their resolutions; returns a workload description.

    configs[2] names "Cook-Torrance/Kulla-Conty": both reference loaders force
    SMaterial::m_Multiscattering off (SceneXMLLoading.cpp:869) and only the UI's checkbox
    turns it on (ImGui.cpp:620-626), so the coffee scene ticks it programmatically on every
    plastic / conductor / dielectric material (``multiscattering=False`` keeps the loader's
    state, for the A/B)."""
    d = Path(scene_dir)
    if name == "cornell":
        setup_cornell(scene, 1920, 1080, 8)
        return "Cornell box OBJ 1920x1080, 8 bounces, point light (configs[1])"
    if name == "coffee":
        scene.load_from_file(write_coffee(d, 1920, 1080, segments=48 if small else 96))
        scene.set_environment_light((1.0, 1.0, 1.0), env_cube(64))
        ms = scene.enable_multiscattering() if multiscattering else []
        return ("coffee-like Mitsuba XML 1920x1080, env cube + constant, max_depth 8, Kulla-Conty multiscattering "
                + (f"on ({len(ms)} materials)" if ms else "off") + " (configs[2])")
    if name in ("spaceship", "spaceship_close"):
        nu, nv = (64, 32) if small else (512, 256)
        framing = "close" if name == "spaceship_close" else "wide"
        scene.load_from_file(write_spaceship(d, 3840, 2160, nu=nu, nv=nv, ships=8, framing=framing))
        return (f"spaceship-like Mitsuba XML 3840x2160, {2 * nu * (nv - 1)} tris x 8 instances, {framing} framing"
                + (" (fleet filling the frame: a traversal workload)" if framing == "close" else "") + " (configs[3])")
    if name == "lamp":
        scene.load_from_file(write_lamp(d, 3840, 2160, segments=48 if small else 96))
        return "lamp-like Mitsuba XML 3840x2160, thin lens, triangle emitters (configs[4])"
    raise ValueError(f"unknown config {name!r} (one of {', '.join(CONFIGS)})")


def default_pool(width: int, height: int, streams: int = 2) -> int:
    """Path-pool slots for several images in flight, split over `streams` pipelines: 2^24 per
    pipeline at 1080p (8 images per batch: 2^23 measured 1-2 % slower on Cornell and 3.6 % on
    coffee, 2^25 slower again, profiles/r05_ab_pool.txt), 2^26 in all at 4K (two pipelines of
    2^25: the most 32-bit pool offsets allow one tracer is 2^26)."""
    return max(1, streams) << 24 if width * height <= (1 << 21) else 1 << 26

