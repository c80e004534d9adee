"""C-ABI argument checks: every entry point include/dcrt.h declares answers null handles, null
output pointers and out-of-range indices with a status code (DCRT_E_INVALID_ARG), never a crash --
the boundary's error behaviour ("nothing throws", dcrt.h), swept over the whole signature table
(directcomputeraytracing_amd/_abi.py SIGNATURES) in a child process so a fault shows as a failed
test instead of ending the run. The GPU case repeats the sweep with a live tracer handle."""
import subprocess
import sys

import pytest

from conftest import ROOT

_CHILD = r"""
import ctypes as C, json, sys
sys.path.insert(0, sys.argv[1])
from directcomputeraytracing_amd import _abi
lib = _abi.load_library()
mode = sys.argv[2]

def zeros(args):
    return [None if (a is _abi._P or a is C.c_char_p or hasattr(a, "contents") or a is _abi._FP) else 0 for a in args]

out = {}
handle = None
if mode in ("scene", "loaded"):
    h = _abi._P()
    assert lib.dcrt_scene_create(C.byref(h)) == 0
    if mode == "loaded":
        assert lib.dcrt_scene_load_from_file(h, sys.argv[3].encode()) == 0
    handle, prefix = h, "dcrt_scene_"
elif mode == "tracer":
    h = _abi._P()
    rc = lib.dcrt_tracer_create(None, C.byref(h))
    assert rc == 0, rc
    handle, prefix = h, ("dcrt_tracer_", "dcrt_device_math_eval")
for name, res, args in _abi.SIGNATURES:
    if res is not _abi._I or not args:
        continue
    if name in ("dcrt_scene_create", "dcrt_tracer_create", "dcrt_device_count"):
        vals = [None] * len(args)
    elif handle is not None:
        if not name.startswith(prefix):
            continue
        vals = [handle] + zeros(args[1:])
        # a nonzero count with null buffers (the case a zero count would let through)
        if name in ("dcrt_tracer_trace_rays", "dcrt_tracer_occluded", "dcrt_tracer_trace_rays_device"):
            vals[2] = 7
        if name == "dcrt_device_math_eval":
            vals[3] = 7
        if name in ("dcrt_scene_get_material_setting", "dcrt_scene_set_material", "dcrt_scene_set_material_opacity",
                    "dcrt_scene_set_material_multiscattering", "dcrt_scene_get_mesh_light", "dcrt_scene_get_punctual_light",
                    "dcrt_scene_get_instance_material_override", "dcrt_scene_get_loaded_mesh", "dcrt_scene_get_instance"):
            vals[1] = 1 << 30   # an index past every table
    else:
        vals = zeros(args)
    out[name] = getattr(lib, name)(*vals)
if mode == "tracer":
    lib.dcrt_tracer_destroy(handle)
elif handle is not None:
    lib.dcrt_scene_destroy(handle)
print(json.dumps(out))
"""


def _sweep(mode, extra=()):
    import json
    r = subprocess.run([sys.executable, "-c", _CHILD, str(ROOT), mode, *extra], capture_output=True, text=True,
                       errors="replace", timeout=300)
    assert r.returncode == 0, f"{mode}: rc {r.returncode}\n{r.stderr[-2000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_null_handles_and_pointers_are_refused(native_lib):
    """All-null / all-zero arguments: every status-returning entry point says INVALID_ARG."""
    rcs = _sweep("null")
    assert len(rcs) >= 70
    bad = {n: rc for n, rc in rcs.items() if rc != -1}
    assert not bad, bad


# arguments a null / zero value may legitimately take (optional outputs and inputs, a zero
# setting): these may succeed on an empty scene
_OPTIONAL_OK = {"dcrt_scene_set_lens", "dcrt_scene_set_max_bounce", "dcrt_scene_set_features", "dcrt_scene_get_bvh_info"}


def test_scene_calls_with_null_outputs_or_bad_indices(native_lib):
    """A live scene handle with null outputs and indices past every table: INVALID_ARG (or the
    scene's own 'no content' status), never a write through the null pointer."""
    rcs = _sweep("scene")
    assert len(rcs) >= 25
    bad = {n: rc for n, rc in rcs.items() if n not in _OPTIONAL_OK and rc not in (-1, -3)}
    assert not bad, bad
    assert all(rcs[n] == 0 for n in _OPTIONAL_OK), {n: rcs[n] for n in _OPTIONAL_OK}


def test_loaded_scene_calls_with_null_outputs_do_not_crash(native_lib):
    from directcomputeraytracing_amd import scenes
    rcs = _sweep("loaded", (str(scenes.CORNELL_OBJ),))
    assert rcs["dcrt_scene_get_flat"] == -1 and rcs["dcrt_scene_get_loaded_mesh"] == -1
    assert all(rc in (0, -1, -3) for rc in rcs.values()), rcs


@pytest.mark.gpu
def test_tracer_calls_with_null_outputs_are_refused():
    """A live tracer: null outputs / inputs (with nonzero counts) are refused before any copy or
    launch touches them."""
    rcs = _sweep("tracer")
    assert len(rcs) >= 30
    ok_with_nulls = {"dcrt_tracer_render", "dcrt_tracer_reset_image", "dcrt_tracer_set_mode", "dcrt_tracer_set_image_batch",
                     "dcrt_tracer_set_instrumentation", "dcrt_tracer_reset_stats", "dcrt_tracer_synchronize",
                     "dcrt_tracer_prepare_images", "dcrt_tracer_clear_film",
                     "dcrt_tracer_set_row_cost_probe"}   # (an int switch: no pointer to refuse)
    bad = {n: rc for n, rc in rcs.items() if n not in ok_with_nulls and rc not in (-1, -3)}
    assert not bad, bad
    # without a scene: rendering reports NO_SCENE
    assert rcs["dcrt_tracer_render"] in (-3, -1), rcs["dcrt_tracer_render"]
