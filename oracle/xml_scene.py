"""TEST INFRASTRUCTURE ONLY -- never imported by the product (directcomputeraytracing_amd/).

The oracle's own restatement of the reference's Mitsuba-XML scene translation, separate from the
product's loader (csrc/host/xml_loader.cpp): from the element tree the reference's own RapidXml
parses (oracle/_ref/librefxml.so, oracle/ref_xml: RapidXml compiled unmodified from
/root/reference) to the CScene state the loaders leave behind, i.e. what dcrt_scene_get_settings,
_get_filter, _get_material_setting, _get_mesh_light, _get_punctual_light,
_get_instance_material_override, _get_instance and _get_loaded_mesh report.

Restated from (all /root/reference/Source/):
  * SceneXMLLoading.cpp:247-597  BuildValueGraph (object / transform / ref / value / default tags,
    first-insert-wins fields, `$name` defaults, atoi / atof on the raw buffer, the strncmp prefix
    matches), :178-245 the split helpers;
  * :670-717 GetOrAddTexture, :719-1004 TranslateMaterialFromBSDF (twosided / mask recursion,
    the per-type defaults, sqrt(alpha), the IOR ratios, ClampValueToValidRange :599-608),
    :1006-1018 CreateAndAddMaterial;
  * :1045-1512 LoadFromXMLFile (integrator, sensor + film + rfilter incl. the Mitchell B <- C
    quirk, the 35 mm film, focal length / fov / fov_axis / thin lens; shapes: obj / rectangle,
    the emitter-only light material, instances and overrides, area / constant / directional
    emitters, the 5000-light cap);
  * Scene.cpp:103-160 the default-material pass, :39-55 GetDefaultMaterial, :626-660 Reset,
    :913-944 SPunctualLight::SetEulerAnglesFromDirection; MathHelper.cpp:9-30
    MatrixRotationToRollPitchYall; Mesh.cpp:7-56 GenerateRectangle (texcoords value-initialised).
  * DirectXMath (not vendored; Windows SDK 10.0.26100, x64 SSE2): XMVector3Cross / Length /
    Dot / Divide, XMScalarSinCos (scalar reduction rounding half away from zero, 11/10-degree
    polynomials), XMMatrixRotationNormal's SSE product order -- restated from the published
    library, parity unpinned where no reference output exists.

Floating point is float32 throughout (numpy float32 scalars: every operation rounds like the
x64 SSE scalar code); atof is strtod's longest numeric prefix rounded to float, as the CRT.
OBJ meshes are loaded by the reference's own tinyobjloader + MikkTSpace (oracle/_ref/librefobj.so,
the XML layout, WavefrontOBJLoading.cpp:374-407).

Not restated (undefined in the reference, never compared): reading a union member the value does
not hold where the reference does no type check on a string / object / matrix (e.g. a <float>
focal_length, read through m_String) -- the restatement raises Unpinned; text directly under
<scene> (a data node the value-graph walk treats as a nested "transform" that the root loop then
dereferences as an object); the K and tiling of the emitter-only light material (left
uninitialised by SceneXMLLoading.cpp:1286-1298).
"""
from __future__ import annotations

import math
import os
import re
import struct
from pathlib import Path

import numpy as np

f32 = np.float32
INDEX_NONE = -1
INVALID_MATERIAL_ID = 0xFFFFFFFF
MAX_MATERIAL_IOR, MAX_MATERIAL_ETA, MAX_MATERIAL_K = f32(3.0), f32(7.0), f32(9.5)   # Constants.h:3-5
MAX_LIGHTS = 5000                                                                     # Scene.h:109
INTERNAL_SCATTERING_SINGLE, INTERNAL_SCATTERING_MULTIPLE = 1, 2                      # InternalScatteringMode.inc.hlsl:4-6
MAT_DIFFUSE, MAT_PLASTIC, MAT_CONDUCTOR, MAT_DIELECTRIC, MAT_THIN = 0, 1, 2, 3, 4    # Material.h:5-12
FILTER_BOX, FILTER_TRIANGLE, FILTER_GAUSSIAN, FILTER_MITCHELL, FILTER_LANCZOS = 0, 1, 2, 3, 4


class LoadFailed(Exception):
    """CScene::LoadFromXMLFile returned false (the reference logs and keeps the earlier state)."""


class Unpinned(Exception):
    """The document reaches reference behaviour that is undefined (see the module docstring)."""


# ---------------------------------------------------------------- the RapidXml element tree
class Node:
    __slots__ = ("name", "attrs", "children")

    def __init__(self, name):
        self.name, self.attrs, self.children = name, [], []

    def attr(self, name):
        """xml_node::first_attribute(name): the first attribute of exactly that name."""
        for k, v in self.attrs:
            if k == name:
                return v
        return None

    def first_node(self, name):
        for c in self.children:
            if c.name == name:
                return c
        return None


def parse_dump(text: str) -> Node:
    """refxml_dump_tree's serialisation (E<name> / A<name>=<value> / '/' lines, element nodes
    only) back into a tree rooted at the document."""
    doc = Node("")
    stack = [doc]
    for line in text.split("\n"):
        if not line:
            continue
        if line[0] == "E":
            n = Node(line[1:])
            stack[-1].children.append(n)
            stack.append(n)
        elif line[0] == "A":
            k, _, v = line[1:].partition("=")
            stack[-1].attrs.append((k, v))
        elif line == "/":
            stack.pop()
        else:
            raise ValueError(f"bad dump line {line!r}")
    return doc


# ---------------------------------------------------------------- CRT number parsing
_FLOAT_RE = re.compile(r"[+-]?(?:inf(?:inity)?|nan(?:\([0-9A-Za-z_]*\))?|0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)"
                       r"(?:[pP][+-]?[0-9]+)?|(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)", re.IGNORECASE)
_INT_RE = re.compile(r"[+-]?[0-9]+")
_C_SPACE = " \t\n\v\f\r"


def c_atof(s: str) -> np.float32:
    """(float)atof(s): strtod's longest valid prefix after leading white space, 0 when none,
    correctly rounded to double, then to float."""
    t = s.lstrip(_C_SPACE)
    m = _FLOAT_RE.match(t)
    if not m:
        return f32(0.0)
    tok = m.group(0)
    # a hex mantissa without digits after "0x" is just "0"; an exponent without digits is dropped
    low = tok.lower()
    if "x" in low:
        sign = -1.0 if tok[0] == "-" else 1.0
        body = low.lstrip("+-")[2:]
        mant, _, exp = body.partition("p")
        ip, _, fp = mant.partition(".")
        if not (ip or fp):
            return f32(0.0)
        val = float.fromhex(("0x" + (ip or "0") + "." + (fp or "0")) + ("p" + exp if exp else ""))
        return f32(sign * val)
    if "inf" in low or "nan" in low:
        v = float(low.split("(")[0])
        return f32(v)
    return f32(float(tok))


def c_atoi(s: str) -> int:
    """atoi: leading white space, sign, decimal digits (int32; overflow is undefined and not used)."""
    m = _INT_RE.match(s.lstrip(_C_SPACE))
    if not m:
        return 0
    v = int(m.group(0))
    if not -(1 << 31) <= v < (1 << 31):
        raise Unpinned(f"atoi overflow: {s!r}")
    return v


def split_by(s: str, delim: str):
    """SplitByDelimeter (SceneXMLLoading.cpp:218-235): (start offset, length) of each field; a
    field's atof reads on past its end into the rest of the string (string_view data())."""
    out, i = [], 0
    while i < len(s):
        j = s.find(delim, i)
        j = len(s) if j < 0 else j
        out.append((i, j - i))
        i = j + 1
    return out


def c_prefix(literal: str, name: str) -> bool:
    """strncmp(literal, name, len(name)) == 0 (the reference compares only len(name) chars)."""
    return literal.startswith(name)


# ---------------------------------------------------------------- the value graph
class Value:
    """SValue (SceneXMLLoading.cpp:53-158): a tagged union; `raw` keeps the union's first word
    for the readers that ignore the tag (m_Float of an integer / boolean value)."""
    __slots__ = ("type", "v", "fields", "nested")

    def __init__(self, type_, v=None):
        self.type, self.v = type_, v
        self.fields, self.nested = ({}, []) if type_ == "object" else (None, None)

    def insert_field(self, name, value):      # unordered_map::insert: the first one stays
        self.fields.setdefault(name, value)

    def field(self, name):
        return self.fields.get(name) if self.fields is not None else None

    def get(self, name, kind, default):
        """GetObjectField<T>: the field when it holds T (eVector and eRGB are one type)."""
        f = self.field(name)
        return f.v if f is not None and f.type == kind else default

    def first_nested(self, name):
        for k, v in self.nested:
            if k == name:
                return v
        return None

    def as_float(self):
        """m_Float read whatever the tag (the reference's unchecked reads)."""
        if self.type == "float":
            return self.v
        if self.type == "integer":
            return np.frombuffer(struct.pack("<i", self.v), np.float32)[0]
        if self.type == "boolean":   # SValue() zeroes the first word, m_Boolean sets its low byte
            return np.frombuffer(struct.pack("<I", 1 if self.v else 0), np.float32)[0]
        if self.type == "vector":
            return self.v[0]
        if self.type == "matrix":
            return self.v[0, 0]
        raise Unpinned(f"m_Float of a {self.type} value")

    def as_string(self):
        if self.type != "string":
            raise Unpinned(f"m_String of a {self.type} value")
        return self.v


OBJECT_TAGS = {"scene", "integrator", "sensor", "sampler", "film", "bsdf", "rfilter", "emitter", "shape", "texture"}
VALUE_TAGS = {"float", "integer", "boolean", "string", "point", "vector", "rgb"}


def _parse_matrix(s: str) -> np.ndarray:
    toks = split_by(s, " ")
    if len(toks) != 16:
        raise LoadFailed(f"matrix value {s!r}")
    m = np.zeros((4, 4), np.float32)
    for r in range(4):
        for c in range(4):
            m[c, r] = c_atof(s[toks[r * 4 + c][0]:])   # transposed: row vectors (:420-422)
    m[:, 0] = -m[:, 0]                                # right- to left-handed (:424-428)
    return m


def build_value_graph(doc: Node):
    """BuildValueGraph (SceneXMLLoading.cpp:247-597): the scene values (the first is used)."""
    defaults = {}
    objects = {}
    scenes = []

    def evaluate(s):
        if s and s[0] == "$":
            if s[1:] not in defaults:
                raise LoadFailed(f"default parameter {s!r}")
            return defaults[s[1:]]
        return s

    def register(node, value):
        ident = node.attr("id")
        if ident is not None:
            objects.setdefault(ident, (node.name, value))
            value.insert_field("id", Value("string", ident))

    def walk(nodes, parent):
        for node in nodes:
            name = node.name
            if parent is None and name not in OBJECT_TAGS and (c_prefix("transform", name) or c_prefix("ref", name)
                                                               or name in VALUE_TAGS):
                raise Unpinned(f"<{name}> beside the scene element (the reference dereferences no parent)")
            if name in OBJECT_TAGS:
                value = Value("object")
                if parent is None:
                    if scenes:
                        # (a second root object: the version split appends to the split buffer the
                        # value parsing left filled, so its field count is never 3 -- :278-291)
                        raise LoadFailed("a second scene-level object")
                    version = node.attr("version")
                    if version is None:
                        raise LoadFailed("scene version")
                    parts = split_by(version, ".")
                    if len(parts) != 3 or c_atoi(version) < 3:
                        raise LoadFailed(f"scene version {version!r}")
                    scenes.append(value)
                else:
                    fname = node.attr("name")
                    if fname is not None:
                        parent.insert_field(fname, value)
                    else:
                        parent.nested.append((name, value))
                    register(node, value)
                    t = node.attr("type")
                    if t is not None:
                        value.insert_field("type", Value("string", evaluate(t)))
                walk(node.children, value)
            elif c_prefix("transform", name):
                value = Value("matrix", np.eye(4, dtype=np.float32))
                fname = node.attr("name")
                if fname is not None:
                    parent.insert_field(fname, value)
                else:
                    parent.nested.append((name, value))
                register(node, value)
                for child in node.children:
                    if c_prefix("matrix", child.name):
                        v = child.attr("value")
                        if v is not None:
                            value.v = _parse_matrix(evaluate(v))   # (each <matrix> replaces the last)
            elif c_prefix("ref", name):
                ident = node.attr("id")
                if ident is None:
                    raise LoadFailed("ref without id")
                if ident in objects:
                    tag, value = objects[ident]
                    fname = node.attr("name")
                    if fname is not None:
                        parent.insert_field(fname, value)
                    else:
                        parent.nested.append((tag, value))
            elif name in VALUE_TAGS:
                fname = node.attr("name")
                if fname is None:
                    raise LoadFailed(f"<{name}> without name")
                raw = node.attr("value")
                if raw is None:
                    raise LoadFailed(f"<{name}> without value")
                s = evaluate(raw)
                if name == "integer":
                    value = Value("integer", c_atoi(s))
                elif name == "float":
                    value = Value("float", c_atof(s))
                elif name == "boolean":
                    if c_prefix("false", s):
                        value = Value("boolean", False)
                    elif c_prefix("true", s):
                        value = Value("boolean", True)
                    else:
                        raise LoadFailed(f"boolean {s!r}")
                elif name == "string":
                    value = Value("string", s)
                else:   # point / vector / rgb
                    toks = split_by(s, ",")
                    if len(toks) != 3:
                        raise LoadFailed(f"{name} value {s!r}")
                    value = Value("vector", tuple(c_atof(s[o:]) for o, _ in toks))
                parent.insert_field(fname, value)
            elif c_prefix("default", name):
                k, v = node.attr("name"), node.attr("value")
                if k is not None and v is not None:
                    defaults.setdefault(k, v)
            # (anything else: "Unsupported tag name", skipped with its children)

    scene = doc.first_node("scene")
    if scene is None:
        return scenes
    siblings = doc.children[doc.children.index(scene):]
    walk(siblings, None)
    return scenes


# ---------------------------------------------------------------- DirectXMath / MathHelper
_XM_PI, _XM_2PI, _XM_1DIV2PI, _XM_PIDIV2 = f32(3.141592654), f32(6.283185307), f32(0.159154943), f32(1.570796327)


def xm_scalar_sincos(value: np.float32):
    """XMScalarSinCos: quotient rounded half away from zero through int, reflection into
    [-pi/2, pi/2], 11-degree sine and 10-degree cosine polynomials."""
    value = f32(value)
    q = f32(_XM_1DIV2PI * value)
    q = f32(int(q + f32(0.5))) if value >= 0 else f32(int(q - f32(0.5)))
    y = f32(value - f32(_XM_2PI * q))
    if y > _XM_PIDIV2:
        y, sign = f32(_XM_PI - y), f32(-1.0)
    elif y < -_XM_PIDIV2:
        y, sign = f32(-_XM_PI - y), f32(-1.0)
    else:
        sign = f32(1.0)
    y2 = f32(y * y)
    s = f32(f32(-2.3889859e-08) * y2 + f32(2.7525562e-06))
    s = f32(s * y2 - f32(0.00019840874))
    s = f32(s * y2 + f32(0.0083333310))
    s = f32(s * y2 - f32(0.16666667))
    s = f32(s * y2 + f32(1.0))
    s = f32(s * y)
    c = f32(f32(-2.6051615e-07) * y2 + f32(2.4760495e-05))
    c = f32(c * y2 - f32(0.0013888378))
    c = f32(c * y2 + f32(0.041666638))
    c = f32(c * y2 - f32(0.5))
    c = f32(c * y2 + f32(1.0))
    return s, f32(sign * c)


def xm_matrix_rotation_normal(n, angle):
    """XMMatrixRotationNormal, SSE path: rows of the 3x3 rotation."""
    s, c = xm_scalar_sincos(angle)
    t = f32(f32(1.0) - c)
    x, y, z = (f32(v) for v in n)
    tyz, tzx, txy = f32(f32(t * y) * z), f32(f32(t * z) * x), f32(f32(t * x) * y)   # (C2 * N0) * N1
    r0 = (f32(f32(t * x) * x + c), f32(f32(t * y) * y + c), f32(f32(t * z) * z + c))
    r1 = (f32(f32(s * x) + tyz), f32(f32(s * y) + tzx), f32(f32(s * z) + txy))       # C0 * N + V0
    r2 = (f32(tyz - f32(s * x)), f32(tzx - f32(s * y)), f32(txy - f32(s * z)))       # V0 - C0 * N
    return np.array([[r0[0], r1[2], r2[1]],
                     [r2[2], r0[1], r1[0]],
                     [r1[1], r2[0], r0[2]]], np.float32)


_LIBM = None


def atan2f(y, x) -> np.float32:
    """The C library's atan2f (the CRT call of MathHelper.cpp; numpy's float32 arctan2 may take a
    SIMD path with other rounding). MSVC's CRT is not available: parity unpinned."""
    global _LIBM
    if _LIBM is None:
        import ctypes
        import ctypes.util
        _LIBM = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _LIBM.atan2f.restype = ctypes.c_float
        _LIBM.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    return f32(_LIBM.atan2f(float(y), float(x)))


def rotation_to_roll_pitch_yaw(m):
    """MathHelper::MatrixRotationToRollPitchYall (MathHelper.cpp:9-25) on the top-left 3x3."""
    m = np.asarray(m, np.float32)
    cy = np.sqrt(f32(f32(m[2, 2] * m[2, 2]) + f32(m[2, 0] * m[2, 0])))
    x = atan2f(f32(-m[2, 1]), cy)
    if cy > f32(16.0) * np.finfo(np.float32).eps:
        y = atan2f(m[2, 0], m[2, 2])
        z = atan2f(m[0, 1], m[1, 1])
    else:
        y = f32(0.0)
        z = atan2f(f32(-m[1, 0]), m[0, 0])
    return (f32(x), f32(y), f32(z))


def euler_from_direction(d):
    """SPunctualLight::SetEulerAnglesFromDirection (Scene.cpp:913-944)."""
    dx, dy, dz = (f32(v) for v in d)
    one, zero = f32(1.0), f32(0.0)
    # XMVector3Cross((1, 0, 0), d): (y1 z2 - z1 y2, z1 x2 - x1 z2, x1 y2 - y1 x2)
    axis = (f32(f32(zero * dz) - f32(zero * dy)), f32(f32(zero * dx) - f32(one * dz)), f32(f32(one * dy) - f32(zero * dx)))
    length = np.sqrt(f32(f32(f32(axis[0] * axis[0]) + f32(axis[2] * axis[2])) + f32(axis[1] * axis[1])))
    dot = f32(f32(f32(dx * one) + f32(dy * zero)) + f32(dz * zero))
    if length < f32(1e-7):
        return (zero, zero, zero) if dot >= 0 else (zero, f32(math.pi), zero)
    axis = tuple(f32(a / length) for a in axis)
    angle = f32(math.acos(float(dot)))
    return rotation_to_roll_pitch_yaw(xm_matrix_rotation_normal(axis, angle))


# ---------------------------------------------------------------- the translation
def _clamp(v, lo, hi):
    """ClampValueToValidRange (:599-608): std::clamp only when out of range (NaN passes)."""
    v = f32(v)
    return f32(min(max(v, lo), hi)) if (v < lo or v > hi) else v


def _material(**kw):
    m = dict(albedo=None, roughness=None, ior=None, opacity=None, k=None, tiling=None, material_type=None,
             albedo_texture_index=None, opacity_texture_index=None, internal_scattering_mode=None,
             multiscattering=None, is_two_sided=None, has_roughness_texture=None)
    m.update(kw)
    return m


def default_material():
    """GetDefaultMaterial (Scene.cpp:39-55)."""
    return _material(albedo=(f32(1), f32(0), f32(1)), roughness=f32(1), ior=(f32(1),) * 3, opacity=f32(1), k=(f32(1),) * 3,
                     tiling=(f32(1), f32(1)), material_type=MAT_DIFFUSE, albedo_texture_index=INDEX_NONE,
                     opacity_texture_index=INDEX_NONE, multiscattering=False, is_two_sided=False,
                     has_roughness_texture=False, internal_scattering_mode=INTERNAL_SCATTERING_MULTIPLE)


XML_MATERIALS = {"diffuse": "diffuse", "roughdiffuse": "roughdiffuse", "dielectric": "dielectric",
                 "thindielectric": "thindielectric", "roughdielectric": "roughdielectric", "conductor": "conductor",
                 "roughconductor": "roughconductor", "plastic": "plastic", "roughplastic": "roughplastic",
                 "twosided": "twosided", "mask": "mask"}


class _Textures:
    def __init__(self, base):
        self.base, self.index, self.count = base, {}, 0

    def get_or_add(self, value):
        """GetOrAddTexture (:670-717): bitmaps get the next index on first use (per value)."""
        t = value.get("type", "string", "")
        if not c_prefix("bitmap", t):
            return INDEX_NONE
        key = id(value)
        if key not in self.index:
            self.index[key] = self.base + len(self.index)
        return self.index[key]


def translate_material(bsdf, textures, mat, two_sided, mask):
    """TranslateMaterialFromBSDF (:719-1004) into `mat` (a dict); False when it fails."""
    tv = bsdf.field("type")
    if tv is None:
        return False
    kind = XML_MATERIALS.get(tv.v if tv.type == "string" else None, "unsupported")
    if kind in ("twosided", "mask"):
        if kind == "mask":
            opacity, tex = f32(0.5), INDEX_NONE
            ov = bsdf.field("opacity")
            if ov is not None:
                if ov.type == "float":
                    opacity = ov.v
                elif ov.type == "object":
                    tex = textures.get_or_add(ov)
            mat["opacity"] = opacity if tex == INDEX_NONE else f32(1.0)
            mat["opacity_texture_index"] = tex
        child = bsdf.first_nested("bsdf")
        if child is None:
            return False
        return translate_material(child, textures, mat, kind == "twosided" or two_sided, kind == "mask" or mask)
    target = {"diffuse": MAT_DIFFUSE, "roughdiffuse": MAT_DIFFUSE, "dielectric": MAT_DIELECTRIC, "thindielectric": MAT_THIN,
              "roughdielectric": MAT_DIELECTRIC, "conductor": MAT_CONDUCTOR, "roughconductor": MAT_CONDUCTOR,
              "plastic": MAT_PLASTIC, "roughplastic": MAT_PLASTIC}.get(kind, MAT_DIFFUSE)
    dielectric_ior = kind in ("dielectric", "thindielectric", "roughdielectric", "plastic", "roughplastic")
    conductor_ior = kind in ("conductor", "roughconductor")
    rough = kind in ("roughdiffuse", "roughdielectric", "roughconductor", "roughplastic")
    diffuse_refl = kind in ("diffuse", "roughdiffuse", "plastic", "roughplastic")
    mat.update(albedo=(f32(0),) * 3, roughness=f32(0), ior=[f32(1)] * 3, k=(f32(1),) * 3, tiling=(f32(1), f32(1)),
               material_type=target, albedo_texture_index=INDEX_NONE, multiscattering=False, is_two_sided=two_sided,
               has_roughness_texture=False, internal_scattering_mode=INTERNAL_SCATTERING_MULTIPLE)
    if not mask:
        mat.update(opacity=f32(1), opacity_texture_index=INDEX_NONE)
    if target == MAT_PLASTIC:
        nonlinear = bsdf.get("nonlinear", "boolean", False)
        mat["internal_scattering_mode"] = INTERNAL_SCATTERING_MULTIPLE if nonlinear else INTERNAL_SCATTERING_SINGLE
    if rough:
        av = bsdf.field("alpha")
        alpha = av.as_float() if av is not None else f32(0.1)
        mat["roughness"] = f32(np.sqrt(f32(alpha)))
    ior = list(mat["ior"])
    if dielectric_ior:
        iv, ev = bsdf.field("int_ior"), bsdf.field("ext_ior")
        int_ior = iv.v if iv is not None and iv.type == "float" else f32(1.49)
        ext_ior = ev.v if ev is not None and ev.type == "float" else f32(1.000277)
        ior[0] = f32(int_ior / ext_ior)
    elif conductor_ior:
        ev, xv = bsdf.field("eta"), bsdf.field("ext_eta")
        eta = ev.v if ev is not None and ev.type == "vector" else (f32(0),) * 3
        ext = xv.v if xv is not None and xv.type == "float" else f32(1.000277)
        ior = [f32(e / ext) for e in eta]
        kv = bsdf.field("k")
        mat["k"] = kv.v if kv is not None and kv.type == "vector" else (f32(1),) * 3
    if diffuse_refl:
        albedo, tex = (f32(0.5),) * 3, INDEX_NONE
        rv = bsdf.field("reflectance" if not dielectric_ior else "diffuse_reflectance")
        if rv is not None:
            if rv.type == "vector":
                albedo = rv.v
            elif rv.type == "object":
                tex = textures.get_or_add(rv)
        mat["albedo"] = albedo if tex == INDEX_NONE else (f32(1),) * 3
        mat["albedo_texture_index"] = tex
    conductor = target == MAT_CONDUCTOR
    lo, hi = (f32(0), MAX_MATERIAL_ETA) if conductor else (f32(1), MAX_MATERIAL_IOR)
    mat["ior"] = tuple(_clamp(v, lo, hi) for v in ior)
    mat["k"] = tuple(_clamp(v, f32(0), MAX_MATERIAL_K) for v in mat["k"])
    return True


def translate(doc: Node, scene_path: Path, width: int, height: int, ref_obj_load):
    """CScene::Reset(width, height) followed by LoadFromFile(scene_path) on an XML file
    (Scene.cpp:103-160, 626-660; SceneXMLLoading.cpp:1045-1512). `ref_obj_load(path)` returns
    the reference's XML-layout mesh of an OBJ file ({"vertices", "indices", "material_ids"}) or
    None when tinyobjloader fails. Returns the scene state as a dict."""
    st = dict(resolution=[width, height], max_bounce=2, film_size=(f32(0.05333), f32(0.03)), camera_type=1,
              fov_x=f32(1.221730), focal_length=f32(0.05), focal_distance=f32(2.0), relative_aperture=f32(8.0),
              blade_count=7, aperture_rotation=f32(0.0), filter=None, filter_radius=f32(1.0), camera=None,
              environment=None, punctual=[], mesh_lights=[], materials=[], meshes=[], instances=[], textures=0)
    scenes = build_value_graph(doc)
    if not scenes:
        raise LoadFailed("no scene")
    textures = _Textures(0)
    bsdf_ids = {}

    def create_material(bsdf):
        m = _material(name=None)
        if translate_material(bsdf, textures, m, False, False):
            bsdf_ids[id(bsdf)] = len(st["materials"])
            st["materials"].append(m)
            return bsdf_ids[id(bsdf)]
        return None

    obj_meshes = {}
    rectangle = None
    filt = dict(kind=FILTER_BOX, gaussian=f32(1.5), b=f32(1 / 3), c=f32(1 / 3), tau=3)   # Scene.h:132-136
    filter_set = False
    for tag, value in scenes[0].nested:
        if value.type != "object":
            if c_prefix("integrator", tag) or c_prefix("sensor", tag) or c_prefix("bsdf", tag) or c_prefix("shape", tag) \
                    or c_prefix("emitter", tag):
                raise Unpinned(f"a non-object nested value {tag!r} at the scene root")
            continue
        if c_prefix("integrator", tag):
            t = value.field("type")
            if t is None:
                raise Unpinned("integrator without type")
            if c_prefix("path", t.as_string()):
                st["max_bounce"] = value.get("max_depth", "integer", 3) & 0xFFFFFFFF
        elif c_prefix("sensor", tag):
            kind = value.get("type", "string", "")
            if c_prefix("perspective", kind):
                st["camera_type"] = 0
            elif c_prefix("thinlens", kind):
                st["camera_type"] = 1
            tw = value.field("to_world")
            pos, euler = (f32(0),) * 3, (f32(0),) * 3
            if tw is not None:
                if tw.type != "matrix":
                    raise Unpinned("to_world is not a transform")
                pos = (tw.v[3, 0], tw.v[3, 1], tw.v[3, 2])
                euler = rotation_to_roll_pitch_yaw(tw.v[:3, :3])
            st["camera"] = (pos, euler)
            film = value.first_nested("film")
            if film is not None:
                st["resolution"] = [film.get("width", "integer", 768) & 0xFFFFFFFF, film.get("height", "integer", 576) & 0xFFFFFFFF]
                rf = film.first_nested("rfilter")
                if rf is not None and rf.field("type") is not None:
                    ft = rf.field("type").as_string()
                    if c_prefix("box", ft):
                        filt["kind"], st["filter_radius"] = FILTER_BOX, rf.get("radius", "float", f32(0.5))
                    elif c_prefix("tent", ft):
                        filt["kind"], st["filter_radius"] = FILTER_TRIANGLE, rf.get("radius", "float", f32(1.0))
                    elif c_prefix("gaussian", ft):
                        filt["kind"] = FILTER_GAUSSIAN
                        filt["gaussian"] = rf.get("stddev", "float", f32(0.5))
                        st["filter_radius"] = f32(filt["gaussian"] * f32(4))
                    elif c_prefix("mitchell", ft):
                        filt["kind"] = FILTER_MITCHELL
                        filt["b"] = rf.get("B", "float", f32(1 / 3))
                        filt["b"] = rf.get("C", "float", f32(1 / 3))     # (the reference assigns C to B)
                        st["filter_radius"] = f32(2.0)
                    elif c_prefix("lanczos", ft):
                        filt["kind"] = FILTER_LANCZOS
                        filt["tau"] = rf.get("lobes", "integer", 3) & 0xFFFFFFFF
                        st["filter_radius"] = f32(filt["tau"])
                    filter_set = True   # (an unsupported type changes nothing)
            aspect = f32(f32(st["resolution"][0]) / f32(st["resolution"][1]))
            st["film_size"] = (f32(0.035), f32(f32(0.035) / max(aspect, f32(0.0001))))
            fl = value.field("focal_length")
            st["focal_length"] = f32(c_atof(fl.as_string()) * f32(0.001)) if fl is not None else f32(0.05)
            fov = f32(50.0)
            fv = value.field("fov")
            if fv is not None and fv.type == "float":
                fov = f32(min(max(fv.v, f32(0.0001)), f32(179.99)))
            st["fov_x"] = f32(fov * f32(_XM_PI / f32(180.0)))
            if st["camera_type"] == 0:
                axis = value.get("fov_axis", "string", "x")
                if c_prefix("x", axis):
                    pass
                elif c_prefix("y", axis):
                    st["fov_x"] = f32(st["fov_x"] * aspect)
            elif st["camera_type"] == 1:
                av = value.field("aperture_radius")
                st["relative_aperture"] = f32(st["focal_length"] / f32(av.as_float() * f32(2))) if av is not None else f32(8.0)
                dv = value.field("focus_distance")
                st["focal_distance"] = dv.as_float() if dv is not None else f32(2.0)
        elif c_prefix("bsdf", tag):
            create_material(value)
        elif c_prefix("shape", tag):
            tv = value.field("type")
            if tv is None:
                continue
            tw = value.field("to_world")
            if tw is not None and tw.type != "matrix":
                raise Unpinned("to_world is not a transform")
            transform = tw.v if tw is not None else np.eye(4, dtype=np.float32)
            emitter = value.first_nested("emitter")
            material = INVALID_MATERIAL_ID
            bsdf = value.first_nested("bsdf")
            if bsdf is not None:
                if id(bsdf) in bsdf_ids:
                    material = bsdf_ids[id(bsdf)]
                else:
                    mid = create_material(bsdf)
                    material = INVALID_MATERIAL_ID if mid is None else mid
            elif emitter is not None:
                material = len(st["materials"])
                st["materials"].append(_material(albedo=(f32(0),) * 3, roughness=f32(0), ior=(f32(1),) * 3, opacity=f32(1),
                                                 material_type=MAT_DIFFUSE, albedo_texture_index=INDEX_NONE,
                                                 opacity_texture_index=INDEX_NONE, multiscattering=False, is_two_sided=False,
                                                 has_roughness_texture=False,
                                                 internal_scattering_mode=INTERNAL_SCATTERING_MULTIPLE))   # K, tiling: uninitialised
            shape = tv.v if tv.type == "string" else None
            mesh_index = None
            if shape == "obj":
                fv = value.field("filename")
                if fv is not None:
                    # GetAbsoluteExternalFilename (:659-668): parent_path() / name, not normalised
                    name = fv.as_string()
                    key = name if name.startswith("/") else os.path.join(os.path.dirname(str(scene_path)), name)
                    p = Path(key)
                    if key in obj_meshes:
                        mesh_index = obj_meshes[key]
                    else:
                        mesh = ref_obj_load(p)
                        if mesh is not None:
                            mesh_index = len(st["meshes"])
                            st["meshes"].append(mesh)
                            obj_meshes[key] = mesh_index
            elif shape == "rectangle":
                if rectangle is None:
                    rectangle = len(st["meshes"])
                    st["meshes"].append(rectangle_mesh(material))
                mesh_index = rectangle
            if mesh_index is None:
                continue
            instance = len(st["instances"])
            st["instances"].append((mesh_index, transform[:, :3].copy(), material))
            light_count = len(st["mesh_lights"]) + len(st["punctual"]) + (1 if st["environment"] is not None else 0)
            if light_count >= MAX_LIGHTS:
                continue
            if emitter is not None:
                et = emitter.field("type")
                if et is not None and et.type == "string" and c_prefix("area", et.v):
                    st["mesh_lights"].append((instance, emitter.get("radiance", "vector", (f32(1),) * 3)))
        elif c_prefix("emitter", tag):
            et = value.field("type")
            if et is None or et.type != "string":
                continue
            light_count = len(st["mesh_lights"]) + len(st["punctual"]) + (1 if st["environment"] is not None else 0)
            if light_count >= MAX_LIGHTS:
                continue
            if c_prefix("constant", et.v):
                if st["environment"] is not None:
                    continue
                st["environment"] = value.get("radiance", "vector", (f32(1),) * 3)
            elif c_prefix("directional", et.v):
                euler = euler_from_direction((0.0, -1.0, 0.0))
                color = value.get("irradiance", "vector", (f32(1),) * 3)
                dv = value.field("direction")
                if dv is not None and dv.type == "vector":
                    euler = euler_from_direction(dv.v)
                st["punctual"].append((None, euler, color, True))   # (m_Position: uninitialised, unused)
    st["textures"] = len(textures.index)
    st["filter"] = filt
    st["filter_set"] = filter_set
    # Scene.cpp:124-160: every INVALID material id of the meshes this load created -> one default
    # material appended after the load's materials
    default = None
    for mesh in st["meshes"]:
        ids = np.asarray(mesh["material_ids"], np.uint32).copy()
        bad = ids == INVALID_MATERIAL_ID
        if bad.any():
            if default is None:
                default = len(st["materials"])
            ids[bad] = default
        mesh["material_ids"] = ids
    if default is not None:
        st["materials"].append(default_material())
    return st


def rectangle_mesh(material_id):
    """Mesh::GenerateRectangle (Mesh.cpp:7-56) with the identity: texcoords value-initialised."""
    v = np.zeros((4, 11), np.float32)
    v[:, 0:3] = [(1, 1, 0), (1, -1, 0), (-1, -1, 0), (-1, 1, 0)]
    v[:, 3:6] = (0, 0, 1)
    v[:, 6:9] = (1, 0, 0)
    return {"vertices": v, "indices": np.array([[0, 1, 3], [1, 2, 3]], np.uint32),
            "material_ids": np.array([material_id, material_id], np.uint32)}
