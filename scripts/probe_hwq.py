#!/usr/bin/env python3
"""Which torch streams share a hardware queue on this box?

A bounded spin kernel (``torch.cuda._sleep``) runs on stream A; a tiny kernel
is then launched on stream B.  If B completes long before A's spin ends the two
streams have independent hardware queues; if B waits for A they share one
(a false dependency: the failure mode behind the round-2 RCCL rehearsal hang).

Prints one JSON line: the calibrated spin time and, per (A, B) pair, B's
completion time in ms.  Usage: python scripts/probe_hwq.py [--streams N]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=6)
    ap.add_argument("--spin-ms", type=float, default=60.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x = torch.zeros(16, device=dev)
    # calibrate the spin
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    cyc = 10_000_000
    t0 = time.perf_counter()
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    per_ms = cyc / ((time.perf_counter() - t0) * 1000)
    spin = int(per_ms * args.spin_ms)
    names = ["null"] + [f"pool{i}" for i in range(args.streams)] + ["high0", "high1"]
    streams = [torch.cuda.default_stream()] + [torch.cuda.Stream() for _ in range(args.streams)] + \
              [torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=-1)]
    res = {}
    for i, a in enumerate(streams):
        for j, b in enumerate(streams):
            if i == j:
                continue
            torch.cuda.synchronize()
            with torch.cuda.stream(a):
                torch.cuda._sleep(spin)
            t0 = time.perf_counter()
            with torch.cuda.stream(b):
                x.add_(1.0)
                ev = torch.cuda.Event()
                ev.record(b)
            ev.synchronize()
            res[f"{names[i]}->{names[j]}"] = round((time.perf_counter() - t0) * 1000, 2)
            torch.cuda.synchronize()
    shared = sorted(k for k, v in res.items() if v > 0.5 * args.spin_ms)
    print(json.dumps({"hw_queues_env": os.environ.get("GPU_MAX_HW_QUEUES"), "spin_ms": args.spin_ms,
                      "cycles_per_ms": round(per_ms), "shared_pairs": shared, "ms": res}), flush=True)


if __name__ == "__main__":
    main()
