#!/usr/bin/env python3
"""Diagnostic: where the cast kernel's waves spend their time (1080p Cornell, 8 images).

Needs a library built with -DDCRT_PHASE_CLOCKS (DCRT_LIB=gpu_ab/phase.so). Prints the
shader-clock cycles summed over all waves per phase of the persistent loop (hand-over +
stores + ray set-up / phase A node visits / phase B leaf work) and the loop counts.
"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    arg = sys.argv[1] if len(sys.argv) > 1 else "8"
    scene = Scene((1920, 1080))
    if arg.isdigit():   # Cornell with this max bounce
        bounces = int(arg)
        scenes.setup_cornell(scene, 1920, 1080, bounces)
    else:               # a BASELINE config scene (coffee / spaceship / lamp)
        print(scenes.setup_config(scene, arg, "/tmp/dcrt_scenes"))
        bounces = scene.frame_params(0).max_bounce_count
    tr = WavefrontPathTracer(path_pool_size=scenes.default_pool(*scene.resolution), iterations_per_render=16)
    tr.on_scene_loaded(scene)
    filt = scene.filter_params()
    tr.clear_film()
    tr.render_images(100, 2, filt)
    fn = tr._lib.dcrt_debug_phase_clocks
    fn.restype = C.c_int
    out = np.zeros(24, np.uint64)
    assert fn(tr._h, out.ctypes.data_as(C.c_void_p)) == 0
    # node visits of the same 8 images (instrumented kernel), then the clocked run
    tr.set_instrumentation(True, False)
    tr.reset_stats()
    images = 8 if arg.isdigit() else 2
    tr.render_images(0, images, filt)
    st = tr.traversal_stats()
    tr.set_instrumentation(False, False)
    assert fn(tr._h, out.ctypes.data_as(C.c_void_p)) == 0
    diag = out[16:20].copy()
    tr.reset_stats()
    tr.render_images(0, images, filt)
    assert fn(tr._h, out.ctypes.data_as(C.c_void_p)) == 0
    c = tr.counters()
    visits = st["ext_node_visits"] + st["shadow_node_visits"]
    leaves = st["ext_triangle_tests"] + st["shadow_triangle_tests"] + st["ext_blas_entries"] + st["shadow_blas_entries"]
    print(f"max bounce {bounces}: node visits {visits}, leaf events {leaves}; from the LDS cache "
          f"{100 * diag[0] / max(1, visits):.1f} %; pushes onto >= 4 / 8 / 12 entries {int(diag[1])} / {int(diag[2])} / {int(diag[3])}")
    tot = float(out[0] + out[1] + out[2])
    for i, name in enumerate(("hand-over + stores + set-up", "phase A (node visits)", "phase B (leaf work)")):
        print(f"{name:30s} {out[i] / 1e9:9.3f} Gcycles  {100 * out[i] / tot:5.1f} %")
    print(f"loop trips {int(out[3])}, phase-A checks {int(out[4])}, phase-B entries {int(out[5])}")
    rays = c["extension_rays"] + c["shadow_rays"]
    print(f"rays {rays}, per loop trip {rays / max(1, out[3]):.2f}, cycles per ray (summed over waves) {tot / rays:.1f}")
    print(f"wave-cycles per node visit: phase A {out[1] / max(1, visits):.2f}, all phases {tot / max(1, visits):.2f}; "
          f"phase B per leaf event {out[2] / max(1, leaves):.2f}")
    m = out[8:15].astype(np.float64)
    mt = m.sum()
    print(f"MATERIAL: {int(out[15])} lane-items (waves x items), wave-cycles per wave-item {mt / max(1, out[15]):.0f}")
    # (material_kernel's DCRT_MCLK sections; 1-4 inside shade_path)
    for i, name in ((0, "loads (hit, state halves) + Li update"), (1, "HitInfoToIntersection"),
                    (3, "emission + NEE (BSDF frame, light sample, eval + pdf, shadow ray)"), (4, "BSDF sample + next ray"),
                    (5, "end-of-path (pixel, debug RNG)"), (6, "queue appends (barriers + atomics)"), (2, "record / sample stores")):
        print(f"  {name:50s} {m[i] / 1e9:8.3f} Gcycles  {100 * m[i] / mt:5.1f} %")
    tr.destroy()


if __name__ == "__main__":
    main()
