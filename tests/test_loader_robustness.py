"""Malformed scene files: the loaders refuse them with an error instead of reading out of
bounds or never finishing. The cases come from a mutation fuzz of the golden OBJ / XML
fixtures (one file per child process); the reference's loaders read these out of bounds
(WavefrontOBJLoading.cpp:125-128, 231-234 index with `!= -1` only) or build a BVH over
infinite bounds, so the product's answer is an error, and valid files load as before.
"""
import random
import subprocess
import sys

import pytest

from conftest import ROOT


def _load(path):
    from directcomputeraytracing_amd import DCRTError, Scene
    s = Scene((64, 64))
    try:
        s.load_from_file(str(path))
        return None
    except DCRTError as e:
        return str(e)


_QUAD = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 1 1\nvn 0 0 1\n"


def test_obj_texcoord_index_before_the_first_is_refused(native_lib, tmp_path):
    # -9 resolves to 3 - 9 = -6: neither "no texcoord" (-1) nor an element
    p = tmp_path / "bad_vt.obj"
    p.write_text(_QUAD + "f 1/1/1 2/2/1 3/-9/1\n")
    assert _load(p) is not None
    ok = tmp_path / "ok_vt.obj"
    ok.write_text(_QUAD + "f 1/1/1 2/2/1 3/-1/1\nf 1//1 3//1 4//1\n")
    assert _load(ok) is None


@pytest.mark.parametrize("bad", ["1e39", "-1e39", "3.5e38"])   # (past FLT_MAX: inf; "inf" / "nan" text parses as 0, as in tinyobjloader)
def test_obj_non_finite_vertex_is_refused(native_lib, tmp_path, bad):
    p = tmp_path / "inf.obj"
    p.write_text(f"v 0 0 0\nv 1 0 0\nv 0 {bad} 0\nv 0 0 1\nvn 0 0 1\nf 1//1 2//1 3//1\nf 1//1 2//1 4//1\n")
    err = _load(p)
    assert err is not None and ("non-finite" in err or "failed" in err)


_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[2])
from directcomputeraytracing_amd import DCRTError, Scene
s = Scene((64, 64))
try:
    s.load_from_file(sys.argv[1])
except DCRTError:
    pass
print("survived")
"""


def test_mutated_fixtures_never_crash_or_hang(native_lib, tmp_path):
    """A short seeded mutation run over the golden OBJ / XML fixtures (each written into a copy
    of its seed's directory, so the references inside resolve): every load returns, with a
    scene or an error."""
    import shutil
    seeds = sorted((ROOT / "tests" / "golden").rglob("*.obj")) + sorted((ROOT / "tests" / "golden").rglob("*.xml"))
    seeds = [p for p in seeds if p.stat().st_size < 64 << 10]   # (small ones: the run stays quick)
    assert seeds
    rng = random.Random(5)
    tokens = [b"<", b">", b'"', b"/", b"=", b"-1", b"-99", b"1e39", b"nan", b" ", b"\n", b"0", b"99999999999", b"f 1/2/3 -4/-5/-6 7"]
    for it in range(24):
        src = rng.choice(seeds)
        data = bytearray(src.read_bytes())
        for _ in range(rng.randint(1, 6)):
            if not data:
                break
            p = rng.randrange(len(data))
            op = rng.random()
            if op < 0.35:
                data[p] = rng.randrange(256)
            elif op < 0.55:
                del data[p:p + rng.randint(1, 40)]
            elif op < 0.85:
                data[p:p] = rng.choice(tokens)
            else:
                del data[p:]
        case = tmp_path / f"case{it}"
        shutil.copytree(src.parent, case)
        path = case / f"mutated{src.suffix}"
        path.write_bytes(bytes(data))
        r = subprocess.run([sys.executable, "-c", _CHILD, str(path), str(ROOT)], capture_output=True, text=True,
                           errors="replace", timeout=120)
        shutil.rmtree(case)
        assert r.returncode == 0 and "survived" in r.stdout, f"case {it} from {src.name}: rc {r.returncode} {r.stderr[-500:]}"


def test_xml_overflowing_instance_transform_is_refused(native_lib, tmp_path):
    """A matrix entry past FLT_MAX (3E9612 in a fuzzed spaceship XML) makes the instance's
    world box infinite: refused, where the TLAS build over it did not finish."""
    import shutil
    src = ROOT / "tests" / "golden" / "xml_mix"
    for f in src.iterdir():
        shutil.copy(f, tmp_path / f.name)
    xml = (tmp_path / "scene.xml").read_text()
    import re
    ms = list(re.finditer(r'<matrix value="([^"]+)"', xml))
    assert len(ms) >= 2, "the fixture has a shape with a matrix transform"
    m = ms[1]   # (the first is the sensor's)
    vals = m.group(1).split()
    vals[3] = "3E9612"
    (tmp_path / "scene.xml").write_text(xml.replace(m.group(0), '<matrix value="' + " ".join(vals) + '"', 1))
    err = _load(tmp_path / "scene.xml")
    assert err is not None and "non-finite" in err
