#!/usr/bin/env python3
"""Kernel statistics table from a rocprofv3 rocpd database (ROCm 7 default output).

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [--top 30] [--match decode]

Prints a markdown table (% of kernel time, calls, avg us, kernel) plus group
totals (dgi HIP kernels / hipBLASLt GEMMs / other), the format of profiles/*.md.
"""
from __future__ import annotations

import argparse
import collections
import sqlite3


def load(db: str) -> dict:
    c = sqlite3.connect(db)
    q = ("select s.display_name, count(*), sum(d.end - d.start) from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.display_name")
    return {name: (n, ns) for name, n, ns in c.execute(q)}


def group(name: str) -> str:
    if name.startswith(("Cijk_", "Custom_Cijk")):
        return "GEMM (hipBLASLt)"
    if "anonymous namespace" in name or name.startswith(("rmsnorm", "rope_cache", "silu", "kv_", "sample")):
        return "dgi HIP kernels"
    return "other (torch)"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    st = load(a.db)
    if a.match:
        st = {k: v for k, v in st.items() if a.match in k}
    tot = sum(ns for _n, ns in st.values()) or 1
    print(f"Total kernel time: {tot / 1e6:.1f} ms over {sum(n for n, _ in st.values())} dispatches\n")
    print("| % time | calls | avg us | kernel |\n|---:|---:|---:|---|")
    for name, (n, ns) in sorted(st.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"| {100 * ns / tot:.2f} | {n} | {ns / n / 1e3:.1f} | `{name[:100]}` |")
    g = collections.Counter()
    for name, (_n, ns) in st.items():
        g[group(name)] += ns
    print("\n| group | % time |\n|---|---:|")
    for k, v in g.most_common():
        print(f"| {k} | {100 * v / tot:.1f} |")


if __name__ == "__main__":
    main()
