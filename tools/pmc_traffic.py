"""Summarise rocprofv3 outputs of tools/profile.sh into profiles/.

* kernel stats (kernel-trace --stats) -> per-kernel call count / average duration
* PMC passes: FETCH_SIZE and WRITE_SIZE are in KiB (1 KiB = 16 x 64-B
  TCC_EA0_RDREQ, checked against the TCC_EA0_RDREQ_sum pass). Per the MI355X
  guide, gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so read bytes are
  doubled; WRITE_SIZE is taken as is. The doubling holds for the traversal's scattered
  16/32/64/128-B dependent fetches too: every L2 read request to the fabric is a 128-B
  request whatever the access width (tools/probe/fetch_calib.hip, tools/fetch_calib.py,
  profiles/r05_fetch_calibration.txt: FETCH_SIZE x 2 = TCC_EA0_RDREQ_128B x 128 B to 0.2 %). Traffic is averaged per launch over the
  same whole-image launch mix the bench's roofline leg uses.

Usage: python tools/pmc_traffic.py gpurun_out/prof profiles/r02_i20   (-> profiles/r02_i20_pmc_traffic.json)
"""
import collections
import csv
import json
import sys
from pathlib import Path


def per_kernel(path: Path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return agg


def main(src, dst_prefix):
    src, dst_prefix = Path(src), str(dst_prefix)
    out = {"kernels": {}}
    stats = src / "trace_kernel_stats.csv"
    if stats.exists():
        for r in csv.DictReader(open(stats)):
            name = r["Name"].split("(")[0].replace("void ", "")
            out["kernels"].setdefault(name, {})
            out["kernels"][name].update(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                                        total_ms=float(r["TotalDurationNs"]) / 1e6)
    counters = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE", "TCC_EA0_RDREQ_sum"):
        p = src / f"pmc_{ctr}_counter_collection.csv"
        if p.exists():
            counters[ctr] = per_kernel(p)
    for name in set().union(*[set(v) for v in counters.values()]) if counters else []:
        d = out["kernels"].setdefault(name, {})
        for ctr, agg in counters.items():
            if name in agg:
                vals = agg[name]
                d[f"{ctr}_avg"] = sum(vals) / len(vals)
        if "FETCH_SIZE_avg" in d and "WRITE_SIZE_avg" in d:
            d["hbm_read_bytes_per_launch"] = d["FETCH_SIZE_avg"] * 1024 * 2
            d["hbm_write_bytes_per_launch"] = d["WRITE_SIZE_avg"] * 1024
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_per_launch"] + d["hbm_write_bytes_per_launch"]
        if "FETCH_SIZE_avg" in d and "TCC_EA0_RDREQ_sum_avg" in d and d["TCC_EA0_RDREQ_sum_avg"]:
            d["fetch_kib_per_rdreq"] = d["FETCH_SIZE_avg"] / d["TCC_EA0_RDREQ_sum_avg"]
    # multi-counter passes (pmc_A+B+..._counter_collection.csv): per kernel and counter
    for p in sorted(src.glob("pmc_*+*_counter_collection.csv")):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (name, ctr), vals in agg.items():
            out["kernels"].setdefault(name, {})[f"{ctr}_avg"] = sum(vals) / len(vals)
    for name, d in out["kernels"].items():
        # VALU issue: a wave64 VALU instruction issues over 2 cycles on its SIMD (MI355X guide);
        # GRBM_GUI_ACTIVE of a dispatch sums the 8 XCDs' active cycles; 1024 SIMDs
        if d.get("SQ_INSTS_VALU_avg") and d.get("GRBM_GUI_ACTIVE_avg"):
            cyc = d["GRBM_GUI_ACTIVE_avg"] / 8.0
            d["valu_issue_frac"] = d["SQ_INSTS_VALU_avg"] * 2.0 / (cyc * 1024.0)
            if d.get("avg_us"):
                d["implied_clock_ghz"] = cyc / (d["avg_us"] * 1e3)
    # the timed ray-cast launch: the merged cast_kernel, else (DCRT_SPLIT_CASTS=1) the EXT kernel
    ext = next((v for k, v in out["kernels"].items() if k.startswith("dcrt::dev::cast_kernel<false")), None) or \
        next((v for k, v in out["kernels"].items() if k.startswith("dcrt::dev::extension_kernel<false")), {})
    out["ext_hbm_bytes_per_launch"] = ext.get("hbm_bytes_per_launch")
    out["ext_valu_issue_frac"] = ext.get("valu_issue_frac")
    out["ext_valu_insts_per_launch"] = ext.get("SQ_INSTS_VALU_avg")
    out["ext_implied_clock_ghz"] = ext.get("implied_clock_ghz")
    # MATERIAL's own statement (the second-heaviest kernel)
    mat = next((v for k, v in out["kernels"].items() if k.startswith("dcrt::dev::material_kernel")), {})
    out["material_hbm_bytes_per_launch"] = mat.get("hbm_bytes_per_launch")
    out["material_valu_issue_frac"] = mat.get("valu_issue_frac")
    out["material_read_bytes_per_launch"] = mat.get("hbm_read_bytes_per_launch")
    out["material_write_bytes_per_launch"] = mat.get("hbm_write_bytes_per_launch")
    # the workload the PMC passes profiled (bench.py matches its own run against it)
    log = src / "pmc_FETCH_SIZE.log"
    line = next((l for l in (log.read_text().splitlines() if log.exists() else []) if l.startswith("{")), None)
    if line:
        b = json.loads(line)
        cfg, roof = b["config"], b["roofline"]
        out["workload"] = {"config": cfg["name"], "resolution": cfg["resolution"], "images": roof["images"],
                           "path_pool": cfg["path_pool"], "world": b["n_gpus"]}
        out["bench_avg_launch_us"] = roof["avg_launch_us"]
        # Whole-pipeline HBM bytes per image. The profiled command (tools/prof_config.sh: one
        # pipeline, one repeat, no warm-up) renders the same images three times -- the timed
        # run, the roofline leg's counting pass (instrumented cast kernel) and its timing pass
        # -- so a per-iteration kernel's launches cover 3 x images, the plain cast kernel's 2 x
        # images and the instrumented cast's (a diagnostic variant, left out) 1 x images.
        # One-time scene set-up kernels (LUT integration, triangle gathers) are not per image.
        images = roof["images"]
        per_image = {}
        for name, d in out["kernels"].items():
            if not name.startswith("dcrt::dev::") or "hbm_bytes_per_launch" not in d or "calls" not in d:
                continue
            short = name.split("::")[-1]
            if short.startswith(("lut_", "build_tri_verts")) or short.startswith("cast_kernel<true"):
                continue
            legs = 2 if short.startswith(("cast_kernel", "extension_kernel", "shadow_kernel")) else 3
            per_image[short] = d["hbm_bytes_per_launch"] * d["calls"] / (legs * images)
        out["pipeline_hbm_bytes_per_image"] = sum(per_image.values())
        out["pipeline_hbm_bytes_per_image_by_kernel"] = per_image
    Path(dst_prefix + "_pmc_traffic.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps({"ext_hbm_bytes_per_launch": out["ext_hbm_bytes_per_launch"]}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
