#!/usr/bin/env python3
"""Can a CU-masked side stream run HBM-bound work beside a GEMM on the rest of the chip?

``graph_overlap_probe.py`` showed that two plain streams do not overlap a
full-chip GEMM with an HBM-bound kernel: the GEMM's workgroups hold every CU.
Here the two streams get disjoint CU masks (``hipExtStreamCreateWithCUMask``):
the GEMM keeps ``256 - side`` CUs, the stream kernel ``side`` CUs.  Timed
eagerly and as a captured fork/join graph (does the captured kernel node keep
its stream's mask?).  Prints one JSON line per mask layout."""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics

import torch


def _hip():
    return ctypes.CDLL("libamdhip64.so")


def masked_stream(cus: list, n_cus: int = 256) -> torch.cuda.ExternalStream:
    words = [0] * ((n_cus + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    rc = _hip().hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(s.value)


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=384)
    ap.add_argument("--copy-mb", type=int, default=256)
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--copies", type=int, default=2)
    ap.add_argument("--side", type=int, default=32)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.cuda.init()
    x = torch.randn(a.rows, 8192, device=dev, dtype=torch.bfloat16)
    w = torch.randn(57344, 8192, device=dev, dtype=torch.bfloat16) * 0.01
    y = torch.empty(a.rows, 57344, device=dev, dtype=torch.bfloat16)
    n = a.copy_mb * (1 << 20) // 2
    src = torch.randn(n, device=dev, dtype=torch.bfloat16)
    dst = torch.empty_like(src)
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count

    def gemm():
        for _ in range(a.gemms):
            torch.matmul(x, w.t(), out=y)

    def copy():
        for _ in range(a.copies):
            dst.copy_(src)

    base = {"n_cus": n_cus, "rows": a.rows, "side_cus": a.side, "gemm_full_ms": timed(gemm, a.reps),
            "copy_full_ms": timed(copy, a.reps)}
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in base.items()}), flush=True)
    layouts = {
        "low_bits": list(range(a.side)),
        "strided": list(range(0, n_cus, max(1, n_cus // a.side)))[: a.side],
        "high_bits": list(range(n_cus - a.side, n_cus)),
    }
    for name, side_cus in layouts.items():
        main_cus = [c for c in range(n_cus) if c not in set(side_cus)]
        sg, sc = masked_stream(main_cus, n_cus), masked_stream(side_cus, n_cus)
        cur = torch.cuda.current_stream()

        def on(stream, fn):
            def run():
                stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(stream):
                    fn()
                torch.cuda.current_stream().wait_stream(stream)
            return run

        def both():
            sg.wait_stream(torch.cuda.current_stream())
            sc.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(sc):
                copy()
            with torch.cuda.stream(sg):
                gemm()
            torch.cuda.current_stream().wait_stream(sg)
            torch.cuda.current_stream().wait_stream(sc)

        r = {"layout": name, "gemm_masked_ms": timed(on(sg, gemm), a.reps), "copy_masked_ms": timed(on(sc, copy), a.reps),
             "both_eager_ms": timed(both, a.reps)}
        both()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                both()
            torch.cuda.synchronize()
            r["both_graph_ms"] = timed(g.replay, a.reps)
            gc = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gc):
                on(sc, copy)()
            torch.cuda.synchronize()
            r["copy_masked_graph_ms"] = timed(gc.replay, a.reps)
        except Exception as e:       # capture on an external stream may be refused
            r["graph_error"] = f"{type(e).__name__}: {e}"[:200]
        del cur
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
