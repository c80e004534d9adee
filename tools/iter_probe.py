#!/usr/bin/env python3
"""Diagnostic: per-iteration ray counts, traversal counts and wall time of one image.

    python tools/iter_probe.py spaceship [images]

Renders `images` images one iteration per Render() call (synchronised), printing per
iteration: extension / shadow rays started, the instrumented kernel's node visits per ray
(a second, instrumented pass over the same images) and the iteration's wall time. Run it
under `rocprofv3 --kernel-trace --stats` to split the wall time by kernel.
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def run(tr, images, instrument):
    tr.set_instrumentation(instrument, False)
    rows = []
    for img in range(images):
        tr.reset_image()
        it = 0
        while True:
            if instrument:
                tr.reset_stats()            # per-iteration maxima
            c0 = tr.counters()
            s0 = tr.traversal_stats() if instrument else None
            t0 = time.perf_counter()
            tr.render(1)
            tr.synchronize()
            dt = time.perf_counter() - t0
            c1 = tr.counters()
            row = {"image": img, "iter": it, "ms": dt * 1e3,
                   "ext": c1["extension_rays"] - c0["extension_rays"],
                   "shadow": c1["shadow_rays"] - c0["shadow_rays"]}
            if instrument:
                s1 = tr.traversal_stats()
                for k in s1:
                    row[k] = s1[k] if "max" in k else s1[k] - s0[k]
            rows.append(row)
            it += 1
            if tr.is_image_complete() or it > 64:
                break
    return rows


def main():
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    cfg = sys.argv[1] if len(sys.argv) > 1 else "spaceship"
    images = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    scene = Scene((1920, 1080))
    print(scenes.setup_config(scene, cfg, "/tmp/dcrt_scenes"), flush=True)
    tr = WavefrontPathTracer(path_pool_size=scenes.default_pool(*scene.resolution), iterations_per_render=1)
    tr.on_scene_loaded(scene)
    print({k: v for k, v in tr.info().items()}, flush=True)
    run(tr, 1, False)                     # warm-up
    plain = run(tr, images, False)
    instr = run(tr, images, True)
    keys = [k for k in instr[0] if k not in ("image", "iter", "ms", "ext", "shadow")]
    print("image iter ms ext shadow " + " ".join(keys) + " instr_ms")
    for p, q in zip(plain, instr):
        print(p["image"], p["iter"], f"{p['ms']:.3f}", p["ext"], p["shadow"], " ".join(str(q[k]) for k in keys),
              f"{q['ms']:.3f}", flush=True)


if __name__ == "__main__":
    main()
