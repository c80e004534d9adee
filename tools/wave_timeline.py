#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of the cast kernels (1080p Cornell; argv: log2 pool size,
images, optional .npz output for the raw stamps -- default 21 1; `24 8` is one batch of the bench's workload, one pipeline).

Needs a library built with -DDCRT_WAVE_TIMELINE (gpu_ab/timeline.so, DCRT_LIB=...).
For each iteration slot prints: waves, items, kernel span (first start .. last end),
mean wave lifetime / span (= average residency), and the end-time percentiles that
show how long the last waves keep the kernel alive.
"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    scene = Scene((1920, 1080))
    scenes.setup_cornell(scene, 1920, 1080, 8)
    pool = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    images = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tr = WavefrontPathTracer(path_pool_size=1 << pool, iterations_per_render=16)
    tr.on_scene_loaded(scene)
    filt = scene.filter_params()
    tr.clear_film()
    if images == 1:
        tr.render_images(100, 1, filt)
    tr.render_images(0, images, filt)
    tr.synchronize()
    fn = tr._lib.dcrt_debug_wave_timeline
    fn.restype = C.c_int
    stamps = np.zeros((2, 16, 8192, 2), np.uint64)
    items = np.zeros((2, 16, 8192), np.uint32)
    rc = fn(tr._h, stamps.ctypes.data_as(C.c_void_p), items.ctypes.data_as(C.c_void_p))
    assert rc == 0, rc
    if len(sys.argv) > 3:
        np.savez_compressed(sys.argv[3], stamps=stamps, items=items)
    for k, name in enumerate(("EXT", "SHADOW")):
        for it in range(16):
            st = stamps[k, it]
            valid = st[:, 1] > 0
            if not valid.any():
                continue
            s0, s1 = st[valid, 0].astype(np.int64), st[valid, 1].astype(np.int64)
            t0 = s0.min()
            span = (s1.max() - t0) / 100.0    # wall_clock64: 100 MHz -> us
            life = (s1 - s0) / 100.0
            ends = np.percentile((s1 - t0) / 100.0, [50, 90, 99, 100])
            starts = np.percentile((s0 - t0) / 100.0, [50, 99, 100])
            # per-XCD view: workgroup b runs on XCD b % 8 (4 waves per workgroup)
            wid = np.nonzero(valid)[0]
            xcd = (wid // 4) % 8
            endx = [(s1[xcd == x] - t0).mean() / 100.0 for x in range(8)]
            life_x = [((s1 - s0)[xcd == x]).mean() / 100.0 for x in range(8)]
            print("        mean end per XCD", " ".join(f"{e:6.1f}" for e in endx), "| mean life", " ".join(f"{e:6.1f}" for e in life_x))
            print(f"{name:6s} it{it:2d} waves {valid.sum():5d} items {int(items[k, it][valid].sum()):8d} span {span:7.1f}us "
                  f"residency {life.mean() / span:5.2f} start p50/p99/max {starts[0]:5.1f}/{starts[1]:5.1f}/{starts[2]:5.1f} "
                  f"end p50/p90/p99/max {ends[0]:6.1f}/{ends[1]:6.1f}/{ends[2]:6.1f}/{ends[3]:6.1f}")
    tr.destroy()


if __name__ == "__main__":
    main()
