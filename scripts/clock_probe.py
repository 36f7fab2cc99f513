#!/usr/bin/env python3
"""Effective shader clock of the ping-pong MFMA GEMM with few vs all CUs busy (the power-limit
reading of profiles/r6_splitk/README.md).  Run under
``rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d DIR -- python3
scripts/clock_probe.py``; ``--summarize DIR`` then joins the counter and kernel-trace CSVs by
dispatch and prints MHz = GRBM_GUI_ACTIVE / duration per (kernel, grid) group.

Variants (70B shapes, eager, 20 launches each, cold weights rotated):
  qkv 512 rows, split-K off: 80 whole tiles on 80 CUs;
  qkv 512 rows, default: 3 K pieces per tile on 240 CUs;
  gate_up 512 rows (SwiGLU): 448 tiles, 1.75 waves on 256 CUs."""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dgi import ops
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    x = torch.randn(512, 8192, device=dev, dtype=bf)
    for name, N, epi, sk in (("qkv_whole", 10240, 0, 1), ("qkv_split", 10240, 0, 0), ("gate_up", 57344, 1, 0)):
        nbuf = max(2, int(1.2e9 // (N * 8192 * 2)))
        ws = [torch.randn(N, 8192, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for i in range(20):
            ops.mfma_gemm(x, ws[i % nbuf], epi, sched=3, streamk=sk)
        torch.cuda.synchronize()
        print(json.dumps({"variant": name, "launches": 20}), flush=True)
        del ws


def summarize(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        sys.exit(f"no counter / kernel trace CSVs under {d}")
    dur, meta = {}, {}
    for row in csv.DictReader(open(kt[0])):
        i = row["Dispatch_Id"]
        dur[i] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        meta[i] = (row["Kernel_Name"][:60], row.get("Grid_Size", row.get("Grid_Size_X", "?")))
    cnt = defaultdict(dict)
    for row in csv.DictReader(open(cc[0])):
        cnt[row["Dispatch_Id"]][row["Counter_Name"]] = float(row["Counter_Value"])
    groups = defaultdict(list)
    for i, c in cnt.items():
        if i in dur and "GRBM_GUI_ACTIVE" in c and "mfma_gemm" in meta[i][0]:
            groups[meta[i]].append((c["GRBM_GUI_ACTIVE"], dur[i]))
    out = []
    for (name, grid), v in sorted(groups.items()):
        cyc = sum(a for a, _ in v) / len(v)
        ns = sum(b for _, b in v) / len(v)
        out.append({"kernel": name, "grid": grid, "n": len(v), "avg_us": round(ns / 1e3, 2),
                    "gui_active_cycles": round(cyc), "mhz": round(cyc / ns * 1e3, 1)})
    for o in out:
        print(json.dumps(o))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    summarize(a.summarize) if a.summarize else run()
