"""Per-iteration kernel durations in launch order from a rocprofv3 kernel trace.

  python tools/kseq.py gpurun_out/prof/trace_kernel_trace.csv [first_iteration] [count]

One row per wavefront iteration (a control_kernel launch starts one): CONTROL, MATERIAL,
cast, drain and film durations in us, and the gap from the iteration's first start to its
last end. Use a one-pipeline run (--streams 1) so the launches do not interleave.
"""
import csv
import sys


def main(path, first=0, count=40):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iters = []
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "").replace("dcrt::dev::", "").split("(")[0]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        key = ("control" if name.startswith("control_kernel") else "material" if name.startswith("material_kernel")
               else "cast" if name.startswith(("cast_kernel", "extension_kernel")) else "drain" if name.startswith("drain_kernel")
               else "film" if name.startswith("film_kernel") else None)
        if key is None:
            continue
        if key == "control":
            iters.append({"t0": t0})
        if not iters:
            continue
        it = iters[-1]
        it[key] = it.get(key, 0.0) + (t1 - t0) / 1e3
        it["t1"] = t1
    print(f"# {path}: {len(iters)} iterations")
    print(f"{'iter':>5} {'CONTROL':>9} {'MATERIAL':>9} {'cast':>9} {'drain':>8} {'film':>8} {'span':>9}")
    tot = {}
    for k, it in enumerate(iters):
        for key in ("control", "material", "cast", "drain", "film"):
            tot[key] = tot.get(key, 0.0) + it.get(key, 0.0)
        if first <= k < first + count:
            print(f"{k:5d} {it.get('control', 0):9.1f} {it.get('material', 0):9.1f} {it.get('cast', 0):9.1f} "
                  f"{it.get('drain', 0):8.1f} {it.get('film', 0):8.1f} {(it['t1'] - it['t0']) / 1e3:9.1f}")
    print("# totals (ms): " + ", ".join(f"{k} {v / 1e3:.3f}" for k, v in tot.items()))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
