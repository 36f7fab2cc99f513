#!/usr/bin/env python3
"""Measure and print the MLP row-padding table (dgi.runtime.gemm_pad) for a model on this GPU."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi.models.config import get_config  # noqa: E402
from dgi.models.llama import LlamaModel  # noqa: E402
from dgi.runtime.gemm_pad import MlpPadTable  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--m-max", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    mc = get_config(a.model)
    m = LlamaModel(mc, torch.device("cuda"), torch.bfloat16, 0, 1)      # one layer is enough for the shapes
    t = MlpPadTable.measure(m.layers[0].gate_up, m.layers[0].down, m_max=a.m_max)
    rows = []
    for T in range(512, a.m_max + 1, 16):
        p = t.pad(T)
        i0 = t.grid.index(((T + 31) // 32) * 32) if ((T + 31) // 32) * 32 in t.grid else None
        t_plain = t.times[i0] if i0 is not None else None
        t_pad = t.times[t.grid.index(p)] if p in t.grid else None
        rows.append({"T": T, "padded": p, "ms_at_T": t_plain, "ms_padded": t_pad})
    res = {"model": a.model, "grid": t.grid, "ms": [round(x, 4) for x in t.times], "pad": rows}
    gain = [r["ms_at_T"] / r["ms_padded"] for r in rows if r["ms_at_T"] and r["ms_padded"]]
    print(json.dumps({"model": a.model, "points": len(t.grid), "mean_speedup": round(sum(gain) / len(gain), 4),
                      "max_speedup": round(max(gain), 3)}))
    for r in rows[::16]:
        print(json.dumps(r))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
