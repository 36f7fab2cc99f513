"""Time top-k/top-p sampling on decode-sized logits: a full-row sort + mask
(what the runner did before) vs the threshold kernel + threshold-aware sampler.

    python scripts/topkp_bench.py [B] [V]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from dgi import ops  # noqa: E402


def sort_path(logits, temps, seeds, tk, tp):
    lf = logits.float()
    s, idx = lf.sort(dim=-1, descending=True)
    V = lf.shape[-1]
    ranks = torch.arange(V, device=lf.device)[None, :]
    mask = ranks >= torch.where(tk > 0, tk, torch.full_like(tk, V))[:, None]
    pr = torch.softmax(s / temps[:, None], dim=-1)
    mask |= (pr.cumsum(-1) - pr) > tp[:, None]
    masked = torch.empty_like(lf).scatter_(-1, idx, s.masked_fill(mask, float("-inf")))
    return ops.sample(masked, temps, seeds, 0)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    ops.load_native(required=True)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 384
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 128256
    for dtype in (torch.bfloat16, torch.float32):
        logits = (torch.randn(B, V, device="cuda") * 3).to(dtype)
        temps = torch.full((B,), 0.7, device="cuda")
        seeds = torch.arange(B, device="cuda")
        tk = torch.full((B,), 50, dtype=torch.long, device="cuda")
        tp = torch.full((B,), 0.9, device="cuda")
        t_sort = timeit(lambda: sort_path(logits, temps, seeds, tk, tp))
        t_kern = timeit(lambda: ops.sample(logits, temps, seeds, 0, top_k=tk, top_p=tp))
        t_plain = timeit(lambda: ops.sample(logits, temps, seeds, 0))
        print(json.dumps({"B": B, "V": V, "dtype": str(dtype).split(".")[-1], "sort_mask_sample_ms": round(t_sort, 3),
                          "threshold_kernel_sample_ms": round(t_kern, 3), "plain_sample_ms": round(t_plain, 3),
                          "speedup": round(t_sort / t_kern, 1)}), flush=True)


if __name__ == "__main__":
    main()
