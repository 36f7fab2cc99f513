#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--pmc`` run (counter_collection.csv) per kernel.

Derived metrics (gfx950, 256 CUs x 4 SIMDs; ROCm 7.2 ships no gfx950 derived
counters, so they are computed here):

* MFMA busy %  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
  (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy cycles over SIMDs)
* bf16 MFMA TF/s = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / kernel time
* LDS bank-conflict % = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* MFMA / LDS instructions per wave
"""
import collections
import csv
import glob
import os
import sys

SIMDS = 256 * 4


def _key(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").strip()
    for sep in ("(", "<"):
        i = n.find(sep)
        if i > 0:
            n = n[:i] + ("<..>" if sep == "<" else "")
            break
    return n[:60]


BY_GRID = "--by-grid" in sys.argv


def load(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                           recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    seen = set()
    for f in files:
        for r in csv.DictReader(open(f)):
            key = _key(r.get("Kernel_Name", "?")) + (f" grid={r.get('Grid_Size')}" if BY_GRID else "")
            disp = (f, r.get("Dispatch_Id"))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if disp not in seen and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                seen.add(disp)
                dur[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                per[key]["_dispatches"] += 1
    if not dur:  # durations from the kernel trace of the same run
        tfiles = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"),
                                                              recursive=True)
        for f in tfiles:
            if not f.endswith("kernel_trace.csv"):
                continue
            for r in csv.DictReader(open(f)):
                key = _key(r.get("Kernel_Name", "?"))
                dur[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                per[key]["_dispatches"] += 1
    return per, dur


def main(path, title=""):
    per, dur = load(path)
    print(f"# {title or path}\n")
    print("| kernel | dispatches | time ms | eff. clock GHz | MFMA busy % | bf16 MFMA TF/s | LDS bank-conflict % |"
          " MFMA inst/wave | LDS inst/wave | wait % | issue-stall % |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, c in sorted(per.items(), key=lambda kv: -dur.get(kv[0], 0)):
        t = dur.get(k, 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        busy = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * SIMDS) if gui else float("nan")
        tf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / t / 1e12 if t else float("nan")
        lds_act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = 100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds_act if lds_act else float("nan")
        waves = c.get("SQ_WAVES", 0.0)
        mi = c.get("SQ_INSTS_MFMA", c.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)) / waves if waves else float("nan")
        li = c.get("SQ_INSTS_LDS", 0.0) / waves if waves else float("nan")
        clk = gui / 8 / t / 1e9 if t else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        wait = 100.0 * c.get("SQ_WAIT_ANY", 0.0) / wc if wc else float("nan")
        stall = 100.0 * c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan")
        print(f"| `{k}` | {int(c['_dispatches'])} | {t * 1e3:.2f} | {clk:.2f} | {busy:.1f} | {tf:.1f} | {conf:.2f} |"
              f" {mi:.1f} | {li:.1f} | {wait:.1f} | {stall:.1f} |")
    print("\nRaw counter totals:\n")
    for k, c in per.items():
        vals = ", ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()) if not n.startswith("_"))
        print(f"- `{k}`: {vals}")


if __name__ == "__main__":
    sys.argv = [a for a in sys.argv if a != "--by-grid"]
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
