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
    ap.add_argument("--per-image-calls", action="store_true", help="one image_sample_ptrs call per image (round-6 first form)")
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
                if args.per_image_calls:
                    ptrs = [ts[j % K].image_sample_ptrs(j // K) for j in range(m)]
                    pos, val = [p for p, _ in ptrs], [v for _, v in ptrs]
                else:   # (render_images_concurrently's arithmetic)
                    W, H = ts[0].width, ts[0].height
                    base = [t.image_sample_ptrs(0) for t in ts[:min(K, m)]]
                    pos = [base[j % K][0] + (j // K) * W * H * 8 for j in range(m)]
                    val = [base[j % K][1] + (j // K) * W * H * 16 for j in range(m)]
                    assert all((pos[j], val[j]) == ts[j % K].image_sample_ptrs(j // K) for j in (0, m - 1, m // 2))
                b2 = time.perf_counter()
                ts[0].accumulate_images(pos, val, filt)
                c = time.perf_counter()
                t_render += b - a
                t_acc += c - b
                t_ptrs = b2 - b
            total = time.perf_counter() - t0
            print(f"rep {rep}: {n} image slices, chunk {chunk}: render {t_render * 1e3:.2f} ms, ordered film pass "
                  f"{t_acc * 1e3:.2f} ms ({t_acc / total * 100:.1f} % of {total * 1e3:.2f} ms; pointer lists "
                  f"{t_ptrs * 1e3:.2f} ms of it)", flush=True)
    finally:
        for t in ts:
            t.destroy()


if __name__ == "__main__":
    main()
