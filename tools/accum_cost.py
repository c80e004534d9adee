#!/usr/bin/env python3
"""Round 6: how long the ordered film pass of image-interleaved pipelines takes beside their
render (one rank of N = 8, bench.py's construction, 20 steps = 160 image slices).

  python tools/accum_cost.py [--world 8] [--rank 3] [--steps 20]
"""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    from directcomputeraytracing_amd import Scene, make_pipelines, prepare_pipelines, probe_row_cost, scenes
    from directcomputeraytracing_amd.tracer import _run_threads
    s = Scene((1920, 1080))
    scenes.setup_cornell(s, 1920, 1080, 8)
    filt = s.filter_params()
    n = args.steps * args.world
    ts = make_pipelines(s, 3 << 24, streams=3, images=n, iterations=16, world=args.world, rank=args.rank,
                        row_cost=probe_row_cost(s), interleave=True, bands_per_rank=1)
    try:
        K = len(ts)
        prepare_pipelines(ts, n)
        for rep in range(3):
            for t in ts:
                t.clear_film()
            chunk = K * min(t.pool_images for t in ts)
            t_render = t_acc = 0.0
            t0 = time.perf_counter()
            for c0 in range(0, n, chunk):
                m = min(chunk, n - c0)
                a = time.perf_counter()
                _run_threads(ts, lambda s_, t: t.render_images(c0 + s_, len(range(s_, m, K)), filt, seed_stride=K,
                                                               convolve=False) if s_ < m else None)
                for t in ts:
                    t.synchronize()
                b = time.perf_counter()
                ptrs = [ts[j % K].image_sample_ptrs(j // K) for j in range(m)]
                ts[0].accumulate_images([p for p, _ in ptrs], [v for _, v in ptrs], filt)
                c = time.perf_counter()
                t_render += b - a
                t_acc += c - b
            total = time.perf_counter() - t0
            print(f"rep {rep}: {n} image slices, chunk {chunk}: render {t_render * 1e3:.2f} ms, ordered film pass "
                  f"{t_acc * 1e3:.2f} ms ({t_acc / total * 100:.1f} % of {total * 1e3:.2f} ms)", flush=True)
    finally:
        for t in ts:
            t.destroy()


if __name__ == "__main__":
    main()
