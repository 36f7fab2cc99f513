#!/usr/bin/env python3
"""Merge cold-weight qkv / o-proj timings (scripts/gemm_table_cold_proj.py) into the shipped routing
table: the pq_* / po_* raw columns of the covered grid points are replaced, everything else (the MLP
columns, the padding objective) is kept; the table records where the columns came from.

    python scripts/gemm_table_patch_cold.py dgi/tuned/gemm_table_....json cold_proj.json --source <path>"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("table")
    ap.add_argument("cold")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    with open(a.table) as f:
        t = json.load(f)
    with open(a.cold) as f:
        cold = {int(k): v for k, v in json.load(f).items()}
    n = 0
    for m, r in zip(t["grid"], t["raw"]):
        c = cold.get(m)
        if c is None:
            continue
        for k in ("pq_blas", "pq_mfma", "po_blas", "po_mfma"):
            r[k] = c[k]
        n += 1
    t["cold_proj"] = {"rows": sorted(cold), "source": a.source}
    with open(a.table, "w") as f:
        json.dump(t, f)
    print(f"patched {n} grid points")


if __name__ == "__main__":
    main()
