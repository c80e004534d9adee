"""Seeded random scenes for the parity tests (test infrastructure, not part of the product).

Each seed writes a triangle soup that aims at the traversal's and the loaders' corner cases --
a jittered height field (shared edges, exactly flat axis-aligned patches), loose random
triangles, zero-area triangles (a repeated vertex, collinear vertices) and exact duplicates
(coincident triangles: equal hit distances, so the reference's visit order decides the hit) --
into a Mitsuba XML scene with several transformed instances of it, rectangles, random BSDFs
(every type the loader knows, an albedo bitmap on some), an area light, and optionally a constant environment and a
directional light; or into an OBJ scene (identity instances, the cache-only IDENT kernel) with a
point light, a random lens and sometimes an environment cube map. Inputs are generated here; the expected
outputs come from the oracle."""
from pathlib import Path

import numpy as np

from directcomputeraytracing_amd.scenes import _sensor, _xml, mitsuba_matrix

_BSDFS = [
    '<bsdf type="diffuse" id="{id}"><rgb name="reflectance" value="{c}"/></bsdf>',
    '<bsdf type="roughplastic" id="{id}"><rgb name="diffuse_reflectance" value="{c}"/><float name="alpha" value="{a}"/></bsdf>',
    '<bsdf type="plastic" id="{id}"><rgb name="diffuse_reflectance" value="{c}"/></bsdf>',
    '<bsdf type="roughconductor" id="{id}"><rgb name="eta" value="0.2, 0.9, 1.1"/><rgb name="k" value="3.9, 2.4, 2.2"/>'
    '<float name="alpha" value="{a}"/></bsdf>',
    '<bsdf type="conductor" id="{id}"><rgb name="eta" value="0.15, 0.4, 1.4"/><rgb name="k" value="3.6, 2.6, 2.3"/></bsdf>',
    '<bsdf type="roughdielectric" id="{id}"><float name="int_ior" value="1.5"/><float name="alpha" value="{a}"/></bsdf>',
    '<bsdf type="dielectric" id="{id}"><float name="int_ior" value="1.33"/></bsdf>',
    '<bsdf type="thindielectric" id="{id}"><float name="int_ior" value="1.5"/></bsdf>',
    '<bsdf type="twosided" id="{id}"><bsdf type="roughplastic"><rgb name="diffuse_reflectance" value="{c}"/>'
    '<float name="alpha" value="{a}"/></bsdf></bsdf>',
]


def soup(rng, n_grid=6, n_loose=12):
    """Vertices, normals, texcoords and faces of one random soup (about 2 n_grid^2 + n_loose + 6
    triangles) in [-1, 1]^2 x [0, 1]."""
    g = np.linspace(-1.0, 1.0, n_grid + 1)
    xx, zz = np.meshgrid(g, g, indexing="ij")
    yy = rng.uniform(0.0, 0.6, xx.shape)
    yy[: n_grid // 2, : n_grid // 2] = 0.25                     # an exactly flat patch
    V = [np.stack([xx.ravel(), yy.ravel(), zz.ravel()], 1)]
    F = []
    w = n_grid + 1
    for i in range(n_grid):
        for j in range(n_grid):
            a, b, c, d = i * w + j, (i + 1) * w + j, (i + 1) * w + j + 1, i * w + j + 1
            F += [(a, b, c), (a, c, d)]
    base = w * w
    loose = rng.uniform([-1, 0, -1], [1, 1, 1], (3 * n_loose, 3))
    V.append(loose)
    F += [(base + 3 * k, base + 3 * k + 1, base + 3 * k + 2) for k in range(n_loose)]
    base += 3 * n_loose
    p = rng.uniform([-1, 0, -1], [1, 1, 1], (2, 3))
    V.append(np.stack([p[0], p[1], 0.5 * (p[0] + p[1]), p[0] + 0.25 * (p[1] - p[0])]))
    F += [(base, base + 1, base + 2),          # collinear: zero area
          (base, base, base + 1),              # a repeated vertex
          (base, base + 3, base + 1)]          # collinear again, other order
    for k in rng.choice(len(F) - 3, 3, replace=False):
        F.append(F[k])                         # exact duplicates: coincident triangles
    V = np.concatenate(V).astype(np.float64)
    N = rng.normal(size=V.shape)
    N[:, 1] = np.abs(N[:, 1]) + 1.0
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    UV = rng.uniform(0.0, 1.0, (len(V), 2))
    return V, N, UV, np.asarray(F)


def _write_soup(path: Path, V, N, UV, F, groups=None, mtl=None):
    lines = ["# random soup"] + ([f"mtllib {mtl}"] if mtl else [])
    lines += [f"v {x:.6f} {y:.6f} {z:.6f}" for x, y, z in V]
    lines += [f"vn {x:.6f} {y:.6f} {z:.6f}" for x, y, z in N]
    lines += [f"vt {x:.6f} {y:.6f}" for x, y in UV]
    for gi, faces in enumerate(groups or [range(len(F))]):
        if groups:
            lines += [f"o part{gi}", f"usemtl m{gi}"]
        for k in faces:
            a, b, c = np.asarray(F[k]) + 1
            lines.append(f"f {a}/{a}/{a} {b}/{b}/{b} {c}/{c}/{c}")
    path.write_text("\n".join(lines) + "\n")
    return path


def _c(rng):
    return ", ".join(f"{v:.3f}" for v in rng.uniform(0.05, 0.95, 3))


def write_xml_scene(directory, seed: int, width: int = 48, height: int = 36, n_grid: int = 6, n_loose: int = 12,
                    n_instances: int = 0) -> Path:
    rng = np.random.default_rng(seed)
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    _write_soup(d / "soup.obj", *soup(rng, n_grid, n_loose))
    n_b = len(_BSDFS)
    picks = rng.choice(n_b, 4, replace=False)
    bsdfs = "".join("  " + _BSDFS[k].format(id=f"b{i}", c=_c(rng), a=f"{rng.uniform(0.02, 0.8):.3f}") + "\n"
                    for i, k in enumerate(picks))
    if rng.random() < 0.5:   # an albedo bitmap (binary PPM) on the last material: texture sampling in MATERIAL
        m = int(rng.integers(2, 9))
        img = rng.integers(0, 256, (m, m + 1, 3), dtype=np.uint8)
        (d / "albedo.ppm").write_bytes(f"P6 {m + 1} {m} 255\n".encode() + img.tobytes())
        kind = "diffuse" if rng.random() < 0.5 else "roughplastic"
        field = "reflectance" if kind == "diffuse" else "diffuse_reflectance"
        bsdfs += (f'  <bsdf type="{kind}" id="bt"><texture name="{field}" type="bitmap"><string name="filename" '
                  'value="albedo.ppm"/></texture></bsdf>\n')
    textured = "bt" in bsdfs
    shapes = []
    for k in range(n_instances or int(rng.integers(2, 5))):
        m = mitsuba_matrix(tuple(rng.uniform([-1.5, -0.3, -1.5], [1.5, 0.5, 1.5])), yaw=float(rng.uniform(0, 360)),
                           pitch=float(rng.choice([0.0, rng.uniform(-30, 30)])), scale=(float(rng.uniform(0.6, 1.4)),) * 3)
        if k == 0:
            m = mitsuba_matrix()                       # one identity instance beside the transformed ones
        ref = "bt" if textured and k == 1 else f"b{k % 4}"
        shapes.append(f'  <shape type="obj" id="soup{k}"><string name="filename" value="soup.obj"/><ref id="{ref}"/>'
                      f'<transform name="to_world"><matrix value="{m}"/></transform></shape>\n')
    shapes.append(f'  <shape type="rectangle" id="floor"><ref id="b{int(rng.integers(0, 4))}"/><transform name="to_world">'
                  f'<matrix value="{mitsuba_matrix((0, -0.31, 0), pitch=-90, scale=(4, 4, 1))}"/></transform></shape>\n')
    shapes.append(f'  <shape type="rectangle" id="lamp"><emitter type="area"><rgb name="radiance" value="{rng.uniform(3, 9):.2f}, '
                  f'{rng.uniform(3, 9):.2f}, {rng.uniform(3, 9):.2f}"/></emitter><transform name="to_world"><matrix value="'
                  f'{mitsuba_matrix(tuple(rng.uniform([-1, 2.0, -1], [1, 3.0, 1])), pitch=90, scale=(0.5, 0.5, 1))}"/></transform></shape>\n')
    emit = ""
    if rng.random() < 0.6:
        emit += f'  <emitter type="constant"><rgb name="radiance" value="{_c(rng)}"/></emitter>\n'
    if rng.random() < 0.5:
        emit += ('  <emitter type="directional"><vector name="direction" value="-0.3, -0.8, 0.5"/>'
                 '<rgb name="irradiance" value="2, 1.9, 1.7"/></emitter>\n')
    cam = mitsuba_matrix((float(rng.uniform(-0.5, 0.5)), 1.4, -4.2), pitch=float(rng.uniform(10, 20)), yaw=float(rng.uniform(-10, 10)))
    if rng.random() < 0.5:
        sensor = _sensor("perspective", width, height, cam, '    <float name="fov" value="50"/>\n')
    else:
        sensor = _sensor("thinlens", width, height, cam, '    <string name="focal_length" value="35mm"/>\n'
                         '    <float name="aperture_radius" value="0.05"/><float name="focus_distance" value="4"/>\n',
                         '<rfilter type="tent"><float name="radius" value="1"/></rfilter>')
    body = (f'  <integrator type="path"><integer name="max_depth" value="{int(rng.integers(3, 8))}"/></integrator>\n'
            + sensor + bsdfs + "".join(shapes) + emit)
    p = d / "random.xml"
    p.write_text(_xml(body))
    return p


def write_obj_scene(directory, seed: int) -> Path:
    """An OBJ scene (identity instances: one per `o` group) with an .mtl of three materials."""
    rng = np.random.default_rng(seed)
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    V, N, UV, F = soup(rng, n_grid=4, n_loose=6)   # (about 45 triangles: the whole scene fits the LDS cache)
    order = rng.permutation(len(F))
    groups = np.array_split(order, 3)
    mtl = "".join(f"newmtl m{k}\nKd {_c(rng).replace(',', '')}\nNs {rng.uniform(10, 200):.1f}\n\n" for k in range(3))
    (d / "random.mtl").write_text(mtl)
    return _write_soup(d / "random.obj", V, N, UV, F, groups=[list(g) for g in groups], mtl="random.mtl")


def setup_obj_scene(scene, path, seed: int, width: int = 48, height: int = 36):
    """Load an OBJ scene and randomise what the OBJ cannot say: materials (every type), a point
    light, the camera and the bounce count -- through the product's own scene API."""
    rng = np.random.default_rng(seed + 1000)
    scene.reset(width, height)
    scene.load_from_file(path)
    for i in range(scene.material_count):
        t = int(rng.integers(0, 5))
        scene.set_material(i, t, tuple(rng.uniform(0.1, 0.9, 3)), float(rng.choice([0.0, rng.uniform(0.05, 0.8)])),
                           (1.5, 1.5, 1.5) if t != 2 else (0.2, 0.9, 1.1), (3.9, 2.4, 2.2) if t == 2 else None,
                           bool(t in (1, 2, 3) and rng.random() < 0.5), bool(rng.random() < 0.5))
    scene.add_point_light(tuple(rng.uniform([-1, 1.5, -1], [1, 2.5, 1])), (6.0, 5.5, 5.0))
    if rng.random() < 0.5:
        from directcomputeraytracing_amd.scenes import env_cube
        scene.set_environment_light(tuple(rng.uniform(0.1, 0.6, 3)), env_cube(8, seed) if rng.random() < 0.5 else None)
    scene.set_camera((float(rng.uniform(-0.3, 0.3)), 1.6, -3.2), (float(rng.uniform(0.2, 0.35)), 0.0, 0.0))
    scene.set_max_bounce(int(rng.integers(2, 7)))
    # the lens (Scene.cpp:837-847, RayTracingCommon.inc.hlsl:38-86): pinhole or thin lens, disk
    # (blades <= 2) or polygonal aperture, any rotation
    scene.set_lens(camera_type=int(rng.integers(0, 2)), fov_x=float(rng.uniform(0.6, 1.4)),
                   focal_length=float(rng.uniform(0.03, 0.07)), focal_distance=float(rng.uniform(2.0, 6.0)),
                   relative_aperture=float(rng.uniform(1.4, 16.0)), blade_count=int(rng.choice([0, 1, 2, 3, 5, 6, 8])),
                   aperture_rotation=float(rng.uniform(0.0, 6.3)))
    return scene
