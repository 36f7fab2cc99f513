#!/usr/bin/env python3
"""One steady-state decode step from a rocprofv3 kernel trace: per-kernel busy
time and the idle gaps between dependent kernels (graph-replayed decode).

    python scripts/decode_trace_layer.py run_kernel_trace.csv [--steps 16]

Steps are delimited by the sampler kernel; the last ``--steps`` complete steps
are averaged.  Prints a markdown table: kernel, launches per step, busy us per
step, avg us per launch, and the step's total busy / gap / wall time.
"""
import argparse
import collections
import csv


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    i = n.find("(")
    n = n[:i] if i > 0 else n
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--delim", default="sample_kernel")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.delim in r[2]]
    if len(marks) < 3:
        print("not enough steps in the trace")
        return
    spans = list(zip(marks[:-1], marks[1:]))[-a.steps:]
    busy = collections.defaultdict(float)
    count = collections.defaultdict(int)
    tot_busy = tot_gap = tot_wall = 0.0
    for i0, i1 in spans:
        seg = rows[i0 + 1: i1 + 1]
        tot_wall += (seg[-1][1] - rows[i0][1]) / 1e3
        prev_end = rows[i0][1]
        for s, e, n in seg:
            k = short(n)
            busy[k] += (e - s) / 1e3
            count[k] += 1
            tot_busy += (e - s) / 1e3
            tot_gap += max(0, s - prev_end) / 1e3
            prev_end = max(prev_end, e)
    n = len(spans)
    print(f"# Decode step from `{a.trace}` (mean of the last {n} steps)\n")
    print(f"wall {tot_wall / n:.1f} us per step = kernel busy {tot_busy / n:.1f} us + idle gaps {tot_gap / n:.1f} us\n")
    print("| kernel | launches / step | busy us / step | avg us |")
    print("|---|---:|---:|---:|")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"| `{k}` | {count[k] / n:.1f} | {v / n:.1f} | {v / count[k]:.2f} |")


if __name__ == "__main__":
    main()
