#!/usr/bin/env python3
"""Per speculative step timeline from a rocprofv3 database: steps are the intervals between
consecutive ``tree_verify`` dispatches that follow each other within ``--max-gap-ms`` (a run of
speculative steps; plain-decode baselines and checks in the same trace are skipped).  Prints wall,
kernel busy (union of dispatch intervals) and idle per step, median over the steps.

    python scripts/spec_step_timeline.py gpurun_out/.../run_results.db"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="tree_verify")
    ap.add_argument("--max-gap-ms", type=float, default=20.0)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    ends = [i for i, (n, _s, _e) in enumerate(rows) if a.marker in n]
    walls, busys, counts = [], [], []
    per = {}
    for i0, i1 in zip(ends, ends[1:]):
        t0, t1 = rows[i0][2], rows[i1][2]
        if (t1 - t0) / 1e6 > a.max_gap_ms:
            continue
        iv = sorted((max(s, t0), min(e, t1)) for _n, s, e in rows[i0 + 1:i1 + 1] if e > t0)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        for n, s, e in rows[i0 + 1:i1 + 1]:
            k = n[:90]
            per.setdefault(k, [0, 0.0])
            per[k][0] += 1
            per[k][1] += (e - s) / 1e3
        walls.append((t1 - t0) / 1e3)
        busys.append(busy / 1e3)
        counts.append(i1 - i0)
    if not walls:
        raise SystemExit("no consecutive speculative steps found")
    w, b = statistics.median(walls), statistics.median(busys)
    print(f"{len(walls)} speculative steps: median wall {w:.1f} us = kernel busy {b:.1f} us + idle {w - b:.1f} us; "
          f"{statistics.median(counts):.0f} dispatches per step")
    ns = len(walls)
    print("\n| kernel | launches / step | us / step |\n|---|---:|---:|")
    for k, (cnt, us) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{k}` | {cnt / ns:.1f} | {us / ns:.1f} |")


if __name__ == "__main__":
    main()
