"""The Mitsuba XML parse pinned against the reference's own parser.

The reference reads scenes with its vendored RapidXml (`xml_document<>::parse<
parse_non_destructive>`, Source/SceneXMLLoading.cpp:1044-1056) and walks the element /
attribute tree (:247-581). oracle/ref_xml builds that RapidXml UNMODIFIED from /root/reference
with a harness that serialises the tree its walk reads; the product's XML loader
(csrc/host/xml_loader.cpp, its own parser) must produce the same tree for every fixture scene
and for documents made to hit the parser's corners (declaration, comments, DOCTYPE, CDATA,
text, entities left as written, single quotes, whitespace around '=', self-closing tags).
Skipped where the reference sources are absent (the GPU box)."""
import ctypes as C
from pathlib import Path

import pytest

from conftest import GOLDEN, ROOT

REFXML = ROOT / "oracle" / "_ref" / "librefxml.so"
pytestmark = pytest.mark.skipif(not REFXML.exists(), reason="oracle/_ref/librefxml.so not built (no /root/reference)")


def _dump(fn, path):
    n = C.c_uint32()
    rc = fn(str(path).encode(), None, 0, C.byref(n))
    assert rc in (0, -5), f"dump failed ({rc}) for {path}"
    buf = C.create_string_buffer(n.value + 1)
    assert fn(str(path).encode(), buf, n.value + 1, C.byref(n)) == 0
    return buf.raw[:n.value].decode("utf-8", errors="replace")


@pytest.fixture(scope="module")
def dumpers(native_lib):
    ref = C.CDLL(str(REFXML))
    ref.refxml_dump_tree.restype = C.c_int
    ref.refxml_dump_tree.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
    return native_lib.dcrt_xml_dump_tree, ref.refxml_dump_tree


CORNERS = {
    "entities.xml": '<?xml version="1.0"?>\n<scene version="3.0.0">\n'
                    '  <string name="filename" value="a&amp;b &lt;c&gt; &quot;q&quot;.obj"/>\n'
                    "  <rgb name='reflectance' value='0.1, 0.2,0.3'/>\n"
                    '  <float name = "alpha"   value  =  "0.25" />\n</scene>\n',
    "comments.xml": '<?xml version="1.0" encoding="utf-8"?>\n<!-- a comment with <tags> inside -->\n'
                    '<!DOCTYPE scene>\n<scene version="3.0.0"><!-- inner --><integrator type="path">'
                    '<integer name="max_depth" value="5"/></integrator>\n  text between elements\n'
                    '<bsdf type="diffuse" id="d"><![CDATA[ x > y ]]><rgb name="reflectance" value="1,1,1"/></bsdf>\n'
                    '<shape type="rectangle"><ref id="d"/><transform name="to_world"><matrix value="1 0 0 0 0 1 0 0 0 0 1 0 0 0 0 1"/>'
                    '</transform></shape></scene>\n',
    "nesting.xml": '<scene version="3.0.0">\n\t<default name="spp" value="16"/>\n\t<sensor type="perspective">\n'
                   '\t\t<film type="hdrfilm"><integer name="width" value="$spp"/><rfilter type="box"/></film>\n'
                   '\t</sensor>\n\t<emitter type="constant"><rgb name="radiance" value="1"/></emitter>\n</scene>',
}


def _fixture_xmls():
    return sorted(GOLDEN.rglob("*.xml"))


@pytest.mark.parametrize("path", _fixture_xmls(), ids=lambda p: p.name)
def test_fixture_xml_tree_matches_rapidxml(dumpers, path):
    prod, ref = dumpers
    a, b = _dump(prod, path), _dump(ref, path)
    assert a == b and a.count("\nE") + 1 > 3


@pytest.mark.parametrize("name", sorted(CORNERS))
def test_corner_xml_tree_matches_rapidxml(dumpers, tmp_path, name):
    prod, ref = dumpers
    p = tmp_path / name
    p.write_text(CORNERS[name])
    a, b = _dump(prod, p), _dump(ref, p)
    assert a == b, f"product:\n{a}\nrapidxml:\n{b}"
    if name == "entities.xml":
        assert "a&amp;b &lt;c&gt;" in a    # non-destructive parse: entities stay as written


def test_generated_config_scenes_match_rapidxml(dumpers, tmp_path):
    """The bench's generated config scenes (coffee, spaceship in both framings, lamp, anyhit)."""
    from directcomputeraytracing_amd import scenes
    prod, ref = dumpers
    files = [scenes.write_coffee(tmp_path, 64, 36, segments=8), scenes.write_lamp(tmp_path, 64, 36, segments=8),
             scenes.write_spaceship(tmp_path, 64, 36, nu=16, nv=8, ships=3),
             scenes.write_spaceship(tmp_path, 64, 36, nu=16, nv=8, ships=3, framing="close"),
             scenes.write_anyhit(tmp_path)]
    for f in files:
        assert _dump(prod, f) == _dump(ref, f), f.name
