"""MALL (Infinity Cache) probe for decode-step weight prefetch.

Question: if a kernel streams a projection's weights just before the decode
GEMV that uses them, does the GEMV read them from the 256 MB MALL instead of
HBM, and how much faster is it?  Cycles over 32 distinct weight matrices
(> MALL) so nothing is warm from the previous iteration.

    python scripts/mall_probe.py            # builds scripts/mall_probe.so if missing
"""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "mall_probe.so")


def build():
    src = os.path.join(HERE, "mall_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", SO])


def main():
    build()
    if not torch.cuda.is_available():
        print("no GPU")
        return
    sys.path.insert(0, os.path.dirname(HERE))
    from dgi import ops
    lib = ctypes.CDLL(SO)
    lib.mall_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p]
    dev = torch.device("cuda")
    sink = torch.zeros(256, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    out = []
    for (N, K, name) in [(4096, 4096, "8b_o"), (6144, 4096, "8b_qkv"), (4096, 14336, "8b_down")]:
        nmat = max(8, (1 << 30) // (N * K * 2))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nmat)]
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
        nbytes = N * K * 2

        def rd(w, nt, blocks=1024):
            lib.mall_read(w.data_ptr(), nbytes, sink.data_ptr(), nt, blocks, s)

        def gemv(w):
            ops.linear(x, w, out=y)

        def timed(fn, iters=4):
            for _ in range(2):
                for i in range(nmat):
                    fn(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                for i in range(nmat):
                    fn(i)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / (iters * nmat)

        r = {"shape": name, "N": N, "K": K, "MB": round(nbytes / 1e6, 1)}
        r["gemv_us"] = timed(lambda i: gemv(ws[i]))
        for nt in (0, 1):
            tag = "nt" if nt else "ld"
            r[f"read_{tag}_us"] = timed(lambda i: rd(ws[i], nt))
            r[f"read_{tag}_x2_us"] = timed(lambda i: (rd(ws[i], nt), rd(ws[i], nt)))
            r[f"read_{tag}+gemv_us"] = timed(lambda i: (rd(ws[i], nt), gemv(ws[i])))
            r[f"gemv_after_{tag}_us"] = r[f"read_{tag}+gemv_us"] - r[f"read_{tag}_us"]
            r[f"reread_{tag}_us"] = r[f"read_{tag}_x2_us"] - r[f"read_{tag}_us"]
        r = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}
        r["read_ld_TBs"] = round(nbytes / r["read_ld_us"] / 1e6, 2)
        r["reread_ld_TBs"] = round(nbytes / max(r["reread_ld_us"], 1e-3) / 1e6, 2)
        r["gemv_TBs"] = round(nbytes / r["gemv_us"] / 1e6, 2)
        print(json.dumps(r), flush=True)
        out.append(r)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
