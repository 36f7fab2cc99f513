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


def per_step(db: str, last: int, marker: str = "sample_kernel") -> None:
    """Mean per-step table over the last ``last`` steps, a step ending at each ``marker``
    dispatch: wall (marker end to marker end), kernel busy (union of dispatch intervals,
    so overlapping kernels on two streams count once), idle gaps and the kernel split."""
    c = sqlite3.connect(db)
    q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    rows = list(c.execute(q))
    ends = [i for i, (n, _s, _e) in enumerate(rows) if marker in n]
    if len(ends) < last + 1:
        raise SystemExit(f"only {len(ends)} '{marker}' dispatches")
    sel = ends[-(last + 1):]
    per = collections.defaultdict(lambda: [0, 0])
    wall = busy = overlap = 0
    for a_, b_ in zip(sel, sel[1:]):
        seg = rows[a_ + 1: b_ + 1]
        wall += rows[b_][2] - rows[a_][2]
        cur_s, cur_e = None, None
        tot = 0
        for n, s0, e0 in seg:
            per[n][0] += 1
            per[n][1] += e0 - s0
            tot += e0 - s0
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        busy += cur_e - cur_s
        overlap += tot
    overlap -= busy
    print(f"wall {wall / last / 1e3:.1f} us per step = kernel busy {busy / last / 1e3:.1f} us + idle gaps "
          f"{(wall - busy) / last / 1e3:.1f} us (kernel time hidden under other kernels: {overlap / last / 1e3:.1f} us)\n")
    print("| kernel | launches / step | busy us / step | avg us |\n|---|---:|---:|---:|")
    for n, (k, ns) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{n[:90]}` | {k / last:.1f} | {ns / last / 1e3:.1f} | {ns / k / 1e3:.2f} |")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--match", default="")
    ap.add_argument("--steps", type=int, default=0, help="per-step table over the last N steps")
    ap.add_argument("--marker", default="sample_kernel", help="kernel that ends a step (--steps)")
    a = ap.parse_args()
    if a.steps:
        per_step(a.db, a.steps, a.marker)
        return
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
