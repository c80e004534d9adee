"""The Mitsuba-XML translation pinned against the oracle's own restatement.

tests/test_xml_pin.py pins the parse tree (the product's XML parser against the reference's own
RapidXml). This file pins what the loaders make of that tree -- the CScene state the flattening
starts from -- against oracle/xml_scene.py, an independent restatement of
SceneXMLLoading.cpp:247-1512 (+ Scene.cpp:103-160, 626-660) that walks the tree RapidXml itself
parsed (oracle/_ref/librefxml.so) and loads OBJ shapes with the reference's own tinyobjloader +
MikkTSpace (oracle/_ref/librefobj.so). Compared field by field, floats bit for bit: the settings
(resolution, bounces, camera type and lens, film size, camera position and Euler angles), the
reconstruction filter, every material (SMaterial as the scene holds it), the mesh lights, the
punctual lights, the environment light, every instance (mesh, transform, material override), and
every loaded mesh (vertices, triangles, material ids after the default-material pass) -- on every
fixture XML, the bench's generated config scenes and corner documents. A document the reference
fails to load must fail in the product too. Skipped where the reference sources are absent (the GPU
box)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REFXML = ROOT / "oracle" / "_ref" / "librefxml.so"
REFOBJ = ROOT / "oracle" / "_ref" / "librefobj.so"
pytestmark = pytest.mark.skipif(not (REFXML.exists() and REFOBJ.exists()),
                                reason="oracle/_ref reference checkers not built (no /root/reference)")


@pytest.fixture(scope="module")
def oracle_xml(native_lib):
    sys.path.insert(0, str(ROOT))
    from oracle import xml_scene
    import test_obj_pin
    ref_xml = C.CDLL(str(REFXML))
    ref_xml.refxml_dump_tree.restype = C.c_int
    ref_xml.refxml_dump_tree.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
    ref_obj = C.CDLL(str(REFOBJ))
    ref_obj.refobj_load.argtypes = [C.c_char_p, C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]
    ref_obj.refobj_mesh_count.argtypes = [C.c_void_p]
    ref_obj.refobj_get_mesh.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint32),
                                        C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.POINTER(C.c_uint32)),
                                        C.POINTER(C.c_uint32)]
    ref_obj.refobj_material_count.argtypes = [C.c_void_p]
    ref_obj.refobj_get_material.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int32)]
    ref_obj.refobj_free.argtypes = [C.c_void_p]

    def dump(path):
        n = C.c_uint32()
        rc = ref_xml.refxml_dump_tree(str(path).encode(), None, 0, C.byref(n))
        if rc not in (0, -5):
            return None
        buf = C.create_string_buffer(n.value + 1)
        assert ref_xml.refxml_dump_tree(str(path).encode(), buf, n.value + 1, C.byref(n)) == 0
        return buf.raw[:n.value].decode("utf-8", errors="replace")

    def load_obj(path):
        r = test_obj_pin.ref_load(ref_obj, path, 0)
        if r is None:
            return None
        mesh = r["meshes"][0]
        # (SceneXMLLoading.cpp:1334-1341 leaves SMeshProcessingParams::m_MaterialIndexBase
        # uninitialised: an OBJ with usemtl materials is undefined through the XML loader)
        if (mesh["material_ids"] != 0xFFFFFFFF).any():
            raise xml_scene.Unpinned(f"{path}: usemtl materials through the XML loader")
        return mesh

    def translate(path, width, height):
        text = dump(path)
        if text is None:
            raise xml_scene.LoadFailed("RapidXml parse error")
        return xml_scene.translate(xml_scene.parse_dump(text), Path(path), width, height, load_obj)

    return xml_scene, translate


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def same(a, b):
    return np.array_equal(bits(a), bits(b))


def product_state(path, width, height):
    from directcomputeraytracing_amd import DCRTError, Scene
    s = Scene((width, height))
    try:
        s.load_from_file(path)
    except DCRTError:
        return None
    return s


def compare(s, o, what=""):
    """Product scene `s` against the oracle's state `o`, field by field."""
    st = s.settings()
    assert list(st.resolution) == o["resolution"], what
    assert st.max_bounce_count == o["max_bounce"], what
    assert st.camera_type == o["camera_type"], what
    for k in ("fov_x", "focal_length", "focal_distance", "relative_aperture", "aperture_rotation"):
        assert same(getattr(st, k), o[k]), (what, k, getattr(st, k), o[k])
    assert st.aperture_blade_count == o["blade_count"]
    assert same(list(st.film_size), o["film_size"]), (what, list(st.film_size), o["film_size"])
    if o["camera"] is not None:
        pos, euler = o["camera"]
        assert same(list(st.camera_position), pos), (what, list(st.camera_position), pos)
        assert same(list(st.camera_euler_angles), euler), (what, list(st.camera_euler_angles), euler)
    f = s.filter_params()
    of = o["filter"]
    assert f.filter == of["kind"] and same(f.radius, o["filter_radius"]), (what, f.filter, f.radius, of, o["filter_radius"])
    assert same([f.gaussian_alpha, f.mitchell_b, f.mitchell_c], [of["gaussian"], of["b"], of["c"]]), (what, "filter params")
    assert f.lanczos_tau == of["tau"]
    # environment and lights
    assert bool(st.has_environment_light) == (o["environment"] is not None), what
    if o["environment"] is not None:
        assert same(list(st.environment_color), o["environment"]), what
    ml = s.mesh_lights()
    assert len(ml) == len(o["mesh_lights"]), what
    for (inst, col), (oi, oc) in zip(ml, o["mesh_lights"]):
        assert inst == oi and same(col, oc), (what, inst, col, oi, oc)
    pl = s.punctual_lights()
    assert len(pl) == len(o["punctual"]), what
    for (pos, euler, col, directional), (opos, oeuler, ocol, odir) in zip(pl, o["punctual"]):
        assert directional == odir and same(col, ocol) and same(euler, oeuler), (what, euler, oeuler)
        if opos is not None:
            assert same(pos, opos)
    # materials
    assert s.material_count == len(o["materials"]), (what, s.material_count, len(o["materials"]))
    assert st.texture_count == o["textures"], what
    for i, om in enumerate(o["materials"]):
        m = s.material_setting(i)
        for k, v in om.items():
            if v is None or k == "name":
                continue
            got = getattr(m, k)
            got = list(got) if hasattr(got, "__len__") else got
            if isinstance(v, (bool, int)) and not isinstance(v, np.floating):
                assert int(got) == int(v), (what, i, k, got, v)
            else:
                assert same(got, v), (what, i, k, got, v)
    # instances and meshes
    meshes, instances = s.loaded_content()
    assert len(instances) == len(o["instances"]), (what, len(instances), len(o["instances"]))
    overrides = s.instance_material_overrides()
    for j, ((mesh, t), (omesh, ot, oov)) in enumerate(zip(instances, o["instances"])):
        assert mesh == omesh and same(t, ot), (what, j, t, ot)
        assert overrides[j] == oov, (what, j, overrides[j], oov)
    assert len(meshes) == len(o["meshes"]), what
    for k, (a, b) in enumerate(zip(meshes, o["meshes"])):
        assert a["vertices"].shape == b["vertices"].shape and same(a["vertices"], b["vertices"]), (what, "mesh", k)
        assert np.array_equal(a["indices"], b["indices"]) and np.array_equal(a["material_ids"], b["material_ids"]), (what, "mesh", k)


def check(oracle_xml, path, width=64, height=48):
    xml_scene, translate = oracle_xml
    try:
        o = translate(path, width, height)
    except xml_scene.LoadFailed:
        o = None
    s = product_state(path, width, height)
    assert (s is None) == (o is None), f"{path.name}: load success differs (product {s is not None})"
    if s is not None:
        compare(s, o, path.name)
    return o


def _fixture_xmls():
    return sorted(GOLDEN.rglob("*.xml"))


@pytest.mark.parametrize("path", _fixture_xmls(), ids=lambda p: str(p.relative_to(GOLDEN)))
def test_fixture_xml_translation_matches_oracle(oracle_xml, path):
    o = check(oracle_xml, path)
    assert o is not None and o["instances"]


def test_generated_scenes_translation_matches_oracle(oracle_xml, tmp_path):
    """The bench's config scenes (coffee, lamp, spaceship in both framings), the any-hit fixture
    and the physics scenes."""
    from directcomputeraytracing_amd import scenes
    files = [scenes.write_coffee(tmp_path / "c", 64, 36, segments=8), scenes.write_lamp(tmp_path / "l", 64, 36, segments=8),
             scenes.write_spaceship(tmp_path / "s", 64, 36, nu=16, nv=8, ships=3),
             scenes.write_spaceship(tmp_path / "sc", 64, 36, nu=16, nv=8, ships=3, framing="close"),
             scenes.write_anyhit(tmp_path / "a"), scenes.write_furnace(tmp_path / "f", 32, 32),
             scenes.write_emissive_box(tmp_path / "e", 32, 32), scenes.write_lit_plane(tmp_path / "p", 32, 32)]
    for f in files:
        assert check(oracle_xml, f) is not None, f


HEAD = '<?xml version="1.0"?>\n<scene version="3.0.0">\n'
SENSOR = ('<sensor type="perspective"><float name="fov" value="45"/><transform name="to_world">'
          '<matrix value="0.8 0 0.6 1 0 1 0 2 -0.6 0 0.8 3 0 0 0 1"/></transform>'
          '<film type="hdrfilm"><integer name="width" value="40"/><integer name="height" value="30"/></film></sensor>\n')
RECT = '<shape type="rectangle">{inner}<transform name="to_world"><matrix value="2 0 0 0 0 0 -1 0 0 2 0 1 0 0 0 1"/></transform></shape>\n'

CORNERS = {
    # default alpha (0.1 -> roughness sqrt(0.1)), default IORs, a non-float int_ior (ignored), conductor eta
    # and k defaults, an integer alpha (read as a float's bits), the plastic nonlinear flag
    "materials": HEAD + SENSOR
    + '<bsdf type="roughplastic" id="a"><rgb name="diffuse_reflectance" value="0.2, 0.3,0.4"/></bsdf>\n'
    + '<bsdf type="roughdielectric" id="b"><string name="int_ior" value="bk7"/><float name="ext_ior" value="1.2"/></bsdf>\n'
    + '<bsdf type="roughconductor" id="c"><float name="alpha" value="0.3"/></bsdf>\n'
    + '<bsdf type="conductor" id="d"><rgb name="eta" value="0.2, 0.9, 1.1"/><rgb name="k" value="3.9, 12, 2.2"/>'
      '<float name="ext_eta" value="1.5"/></bsdf>\n'
    + '<bsdf type="roughdiffuse" id="e"><integer name="alpha" value="1"/></bsdf>\n'
    + '<bsdf type="plastic" id="f"><boolean name="nonlinear" value="t"/><float name="int_ior" value="9"/></bsdf>\n'
    + '<bsdf type="thindielectric" id="g"/>\n<bsdf type="velvet" id="h"/>\n'
    + RECT.format(inner='<ref id="a"/>') + RECT.format(inner='<ref id="d"/>') + RECT.format(inner='<ref id="h"/>')
    + '</scene>\n',
    # nested twosided(mask(...)) and mask(twosided(...)), a texture-less bitmap opacity, a shared inline bsdf
    "nested": HEAD + SENSOR
    + '<bsdf type="twosided" id="ts"><bsdf type="mask"><float name="opacity" value="0.25"/>'
      '<bsdf type="diffuse"><rgb name="reflectance" value="0.5, 0.6, 0.7"/></bsdf></bsdf></bsdf>\n'
    + '<bsdf type="mask" id="mt"><texture type="bitmap" name="opacity"><string name="filename" value="leaf.png"/></texture>'
      '<bsdf type="twosided"><bsdf type="diffuse"><texture type="bitmap" name="reflectance" id="wood">'
      '<string name="filename" value="wood.png"/></texture></bsdf></bsdf></bsdf>\n'
    + '<bsdf type="twosided" id="empty"/>\n'
    + RECT.format(inner='<ref id="ts"/>') + RECT.format(inner='<ref id="mt"/>') + RECT.format(inner='<ref id="empty"/>')
    + '</scene>\n',
    # emitter-only shapes (the black light material), a shared rectangle with per-instance overrides,
    # an area light's default radiance, unsupported shape and emitter types, two constant emitters
    "emitters": HEAD + SENSOR
    + RECT.format(inner='<emitter type="area"><rgb name="radiance" value="4, 3, 2"/></emitter>')
    + RECT.format(inner='<bsdf type="diffuse"/><emitter type="area"/>')
    + RECT.format(inner='<emitter type="point"/>')
    + '<shape type="sphere"><bsdf type="diffuse"/></shape>\n'
    + '<emitter type="constant"><rgb name="radiance" value="0.5, 0.5, 0.5"/></emitter>\n'
    + '<emitter type="constant"><rgb name="radiance" value="9, 9, 9"/></emitter>\n'
    + '<emitter type="directional"><vector name="direction" value="0.3, -1, 0.2"/><rgb name="irradiance" value="2, 2, 1"/></emitter>\n'
    + '<emitter type="directional"/>\n<emitter type="directional"><vector name="direction" value="1, 0, 0"/></emitter>\n'
    + '<emitter type="directional"><vector name="direction" value="-1, 0, 0"/></emitter>\n'
    + '</scene>\n',
    # thin lens: focal length string, aperture radius, focus distance; 35 mm film of a 4:3 image;
    # the Mitchell filter's B <- C quirk; $defaults; integrator depth
    "thinlens": HEAD + '<default name="spp" value="16"/><default name="w" value="64"/><default name="depth" value="6"/>\n'
    + '<integrator type="path"><integer name="max_depth" value="$depth"/></integrator>\n'
    + '<sensor type="thinlens"><string name="focal_length" value="35mm"/><float name="aperture_radius" value="0.01"/>'
      '<float name="focus_distance" value="3.5"/><transform name="to_world"><matrix value="1 0 0 0 0 1 0 1 0 0 1 -4 0 0 0 1"/>'
      '</transform><film type="hdrfilm"><integer name="width" value="$w"/><integer name="height" value="48"/>'
      '<rfilter type="mitchell"><float name="B" value="0.2"/><float name="C" value="0.7"/></rfilter></film></sensor>\n'
    + RECT.format(inner='<bsdf type="diffuse"/>') + '</scene>\n',
    # pinhole with fov_axis y, a gaussian filter, fields given twice (the first one stays), duplicate
    # ids, a transform with two matrices (the last one replaces the first) and an unsupported child
    "pinhole": HEAD + '<integrator type="path"><integer name="max_depth" value="3"/><integer name="max_depth" value="9"/></integrator>\n'
    + '<sensor type="perspective"><float name="fov" value="30"/><string name="fov_axis" value="y"/>'
      '<transform name="to_world"><translate x="1"/><matrix value="1 0 0 5 0 1 0 5 0 0 1 5 0 0 0 1"/>'
      '<matrix value="0 0 1 0.5 0 1 0 1.5 -1 0 0 2 0 0 0 1"/></transform>'
      '<film type="hdrfilm"><integer name="width" value="50"/><integer name="height" value="20"/>'
      '<rfilter type="gaussian"><float name="stddev" value="0.7"/></rfilter></film></sensor>\n'
    + '<bsdf type="diffuse" id="x"><rgb name="reflectance" value="0.1, 0.1, 0.1"/></bsdf>\n'
    + '<bsdf type="diffuse" id="x"><rgb name="reflectance" value="0.9, 0.9, 0.9"/></bsdf>\n'
    + RECT.format(inner='<ref id="x"/>') + '</scene>\n',
    # lanczos and tent filters in two sensors (the last one wins), an unsupported filter
    "filters": HEAD + '<sensor type="perspective"><film type="hdrfilm"><rfilter type="lanczos"><integer name="lobes" value="2"/>'
      '</rfilter></film></sensor>\n<sensor type="orthographic"><film type="hdrfilm"><integer name="width" value="20"/>'
      '<rfilter type="tent"/></film></sensor>\n'
    + RECT.format(inner='') + '</scene>\n',
    # refs: a root texture shared by two materials (one texture index), a named ref (a field, not the
    # shape's nested bsdf: no override), an unknown id, a $default in a type attribute; boolean
    # prefixes ("" and "f" read as false, "tr" as true); an unsupported texture type
    "refs": HEAD + '<default name="mat" value="roughconductor"/>\n'
    + '<texture type="bitmap" id="tex"><string name="filename" value="albedo.png"/></texture>\n'
    + '<bsdf type="diffuse" id="m1"><ref id="tex" name="reflectance"/></bsdf>\n'
    + '<bsdf type="roughplastic" id="m2"><ref id="tex" name="diffuse_reflectance"/><boolean name="nonlinear" value=""/></bsdf>\n'
    + '<bsdf type="plastic" id="m3"><boolean name="nonlinear" value="tr"/></bsdf>\n'
    + '<bsdf type="plastic" id="m4"><boolean name="nonlinear" value="f"/></bsdf>\n'
    + '<bsdf type="$mat" id="m5"><float name="alpha" value="0.2"/><rgb name="eta" value="1.5, 1.5, 1.5"/></bsdf>\n'
    + '<bsdf type="diffuse" id="m6"><texture type="checkerboard" name="reflectance"/></bsdf>\n'
    + RECT.format(inner='<ref id="m2"/>') + RECT.format(inner='<ref id="m1" name="surface"/>')
    + RECT.format(inner='<ref id="nope"/><ref id="m5"/>') + '</scene>\n',
    # load failures: a bad matrix, an unknown $default, a bad boolean, an old version
    "fail_matrix": HEAD + '<shape type="rectangle"><transform name="to_world"><matrix value="1 0 0"/></transform></shape></scene>\n',
    "fail_default": HEAD + '<integrator type="path"><integer name="max_depth" value="$nope"/></integrator></scene>\n',
    "fail_boolean": HEAD + '<bsdf type="plastic"><boolean name="nonlinear" value="yes"/></bsdf></scene>\n',
    "fail_version": '<scene version="2.1.0"><integrator type="path"/></scene>\n',
}


def test_obj_shapes_translation_matches_oracle(oracle_xml, tmp_path):
    """OBJ shapes: one file instanced twice (one mesh), the same file as "./name" (another mesh: the
    key is the unnormalised path), a missing file (no instance), an inline bsdf on one instance
    and none on the other (the meshes' ids then take the default material)."""
    from directcomputeraytracing_amd import scenes
    V, N, UV, F = scenes.lathe([(0.0, 0.0), (0.4, 0.05), (0.5, 0.4), (0.3, 0.8), (0.0, 0.85)], 10)
    scenes.write_obj(tmp_path / "vase.obj", V, N, UV, F)
    m = scenes.mitsuba_matrix
    doc = (HEAD + SENSOR
           + f'<shape type="obj"><string name="filename" value="vase.obj"/><transform name="to_world"><matrix value="{m((0, 0, 1))}"/></transform></shape>\n'
           + f'<shape type="obj" id="second"><string name="filename" value="vase.obj"/><bsdf type="conductor"/>'
             f'<transform name="to_world"><matrix value="{m((1, 0, 1), yaw=30, scale=(1, 2, 1))}"/></transform></shape>\n'
           + '<shape type="obj"><string name="filename" value="./vase.obj"/></shape>\n'
           + '<shape type="obj"><string name="filename" value="missing.obj"/></shape>\n</scene>\n')
    p = tmp_path / "objs.xml"
    p.write_text(doc)
    o = check(oracle_xml, p)
    assert len(o["meshes"]) == 2 and len(o["instances"]) == 3 and o["instances"][1][2] == 0


@pytest.mark.parametrize("name", sorted(CORNERS))
def test_corner_document_translation_matches_oracle(oracle_xml, tmp_path, name):
    p = tmp_path / f"{name}.xml"
    p.write_text(CORNERS[name])
    o = check(oracle_xml, p)
    assert (o is None) == name.startswith("fail_")
