#!/usr/bin/env python3
"""Summarise the FETCH_SIZE calibration (tools/probe/fetch_calib.hip under rocprofv3, one PMC pass
per counter group: FETCH_SIZE; TCC_EA0_RDREQ_sum; TCC_EA0_RDREQ_{32B,64B,128B}_sum;
TCC_EA0_RDREQ_DRAM{,_32B}_sum; TCC_HIT/MISS_sum) against the bytes each probe kernel requested.

Usage: python tools/fetch_calib.py gpurun_out/fc > profiles/r05_fetch_calibration.txt
"""
import collections
import csv
import sys
from pathlib import Path


def main(src):
    src = Path(src)
    agg = collections.defaultdict(dict)
    for p in sorted(src.glob("p*_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    req = {}
    for line in open(src / "plain.txt"):
        f = line.split()
        if len(f) >= 5 and f[1] == "requested_bytes":
            req[f[0].replace("chase", "chase<").replace("<", "<", 1) + (">" if f[0].startswith("chase") else "")] = (int(f[2]), int(f[4]))
    print("# FETCH_SIZE calibration on gfx950 (MI355X): tools/probe/fetch_calib.hip, 2 GiB buffer (8x the Infinity Cache)")
    print("# stream16: coalesced 16 B/lane streaming read of 1 GiB; chase<R>: 1 M lanes x 64 dependent random R-byte records")
    print("# columns: requested bytes | accesses | RDREQ 32B / 64B / 128B | FETCH_SIZE (KiB) | FETCH_SIZE x 2 KiB | RDREQ-size bytes | "
          "(FETCH_SIZE x 2) / RDREQ-size bytes | fabric bytes / requested | 128-B requests per access | L2 hit rate")
    for k in ("stream16", "chase<16>", "chase<32>", "chase<64>", "chase<128>"):
        c = agg.get(k)
        if not c or k not in req:
            continue
        rb, acc = req[k]
        r32, r64, r128 = c.get("TCC_EA0_RDREQ_32B_sum", 0), c.get("TCC_EA0_RDREQ_64B_sum", 0), c.get("TCC_EA0_RDREQ_128B_sum", 0)
        sized = 32 * r32 + 64 * r64 + 128 * r128
        fs2 = c["FETCH_SIZE"] * 2 * 1024
        hit = c.get("TCC_HIT_sum", 0) / max(1.0, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0))
        print(f"{k:10s} {rb:12d} {acc:10d} | {r32:8.0f} {r64:8.0f} {r128:10.0f} | {c['FETCH_SIZE']:12.1f} {fs2 / 1024:12.1f} | "
              f"{sized:14.0f} | {fs2 / sized:6.4f} | {sized / rb:6.2f} | {r128 / acc:5.2f} | {hit:5.3f}")
    print("# Every read the L2 sends to the fabric is a 128-B request (RDREQ_32B / _64B ~ 0, whatever the access width),")
    print("# and FETCH_SIZE = TCC_EA0_RDREQ x 64 B: FETCH_SIZE x 2 equals the fabric read bytes exactly for the")
    print("# scattered 16/32/64/128-B dependent fetches of the traversal as for streaming reads, so tools/pmc_traffic.py's")
    print("# doubling is calibrated for the cast kernels too (the spaceship / coffee traffic figures stand). A random")
    print("# 16- or 32-B fetch costs ~1.5 128-B requests (12x / 6x the requested bytes); FETCH_SIZE counts Infinity-Cache")
    print("# hits (fabric traffic, not DRAM only: TCC_EA0_RDREQ_DRAM equals TCC_EA0_RDREQ).")


if __name__ == "__main__":
    main(sys.argv[1])
