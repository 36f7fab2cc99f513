#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) as markdown."""
import csv
import sys


def main(path, title="", top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title or path}\n")
    print(f"Total kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches\n")
    print("| % time | calls | avg us | kernel |\n|---:|---:|---:|---|")
    groups = {}
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        n = r["Name"].replace("|", "/")
        print(f"| {float(r['TotalDurationNs']) / tot * 100:.2f} | {r['Calls']} | {float(r['AverageNs']) / 1000:.1f} | `{n[:100]}` |")
    for r in rows:
        n = r["Name"]
        k = ("GEMM (hipBLASLt)" if "Cijk" in n else "dgi HIP kernels" if any(x in n for x in (
            "rmsnorm", "rope_cache", "paged_decode", "prefill_attn", "silu_mul", "sample_kernel", "decode_reduce",
            "kv_", "tree_", "topk", "mfma_gemm", "skinny", "topkp")) else "other (torch)")
        groups[k] = groups.get(k, 0.0) + float(r["TotalDurationNs"])
    print("\n| group | % time |\n|---|---:|")
    for k, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v / tot * 100:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
