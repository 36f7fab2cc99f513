#!/usr/bin/env python3
"""Markdown table of RCCL rehearsal runs (``scripts/rehearse_rccl_bench.sh`` JSON lines).

    python scripts/summarize_rehearsal.py gpurun_out/rehearse_*_r3*.json
"""
from __future__ import annotations

import json
import os
import sys


def row(path: str) -> str:
    name = os.path.basename(path)[len("rehearse_"):-len(".json")]
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 - a failed case has no JSON line
        return f"| `{name}` | — | — | FAILED ({type(e).__name__}) | | | | |"
    e = d["extra"]
    ranks = e.get("ranks", [])
    kv_tx = sum((r.get("kv_transport") or {}).get("received", 0) for r in ranks
                if r.get("role") in ("decode_driver", "decode_stage"))
    rtts = [r["pd_scheduler"]["kv_transport"]["cts_rtt_us_p50"] for r in ranks
            if r.get("role") == "prefill" and r.get("pd_scheduler", {}).get("kv_transport", {}).get("cts_rtt_us_p50")]
    migrated = sum(r.get("migrated", 0) for r in ranks if r.get("role") == "prefill")
    rtt = f"{sorted(rtts)[len(rtts) // 2]:.0f}" if rtts else "—"
    lay = e["layout"]["describe"] if isinstance(e.get("layout"), dict) else d["config"].get("parallelism")
    return (f"| `{name}` | {d['config']['model']} | {lay} | completes | "
            f"{e.get('pair_setup_s', 0):.2f} | {migrated} | {kv_tx} | {rtt} |")


def main() -> None:
    print("| case | model | layout | result | comm set-up s | migrations | KV transfers landed | "
          "RTS->CTS round trip p50 us |")
    print("|---|---|---|---|---:|---:|---:|---:|")
    for p in sys.argv[1:]:
        print(row(p))


if __name__ == "__main__":
    main()
