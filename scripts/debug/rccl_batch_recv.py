#!/usr/bin/env python3
"""Debug: one RCCL group of receives from two sources on a shared GPU (DGI_SHARED_GPU=1).
VARIANT=plain|nostream|groupsend|warm|warmgroupsend selects how the receives / sends are issued."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dgi.parallel.fabric import Fabric  # noqa: E402

v = os.environ.get("VARIANT", "plain")
f = Fabric()
r = f.rank
n = 1 << 16
print(f"rank {r} variant {v} up", flush=True)
if v.startswith("warm"):
    f.connect_pairs([(0, 1), (0, 2)])
    print(f"rank {r} pairs connected", flush=True)
if r == 0:
    bufs = [f.alloc_recv((n,), torch.float32) for _ in range(2)]
    ops_ = [dist.P2POp(dist.irecv, b, s, group=f.kv_group) for b, s in zip(bufs, (1, 2))]
    if v == "nostream":
        works = dist.batch_isend_irecv(ops_)
    else:
        with torch.cuda.stream(f.recv_stream):
            works = dist.batch_isend_irecv(ops_)
    print(f"rank 0 posted, {len(works)} work(s)", flush=True)
    f.barrier()
    t0 = time.time()
    while not all(w.is_completed() for w in works):
        if time.time() - t0 > 30:
            print("rank 0 TIMEOUT waiting", flush=True)
            os._exit(3)
        time.sleep(0.01)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    print("rank 0 got", [float(b[0]) for b in bufs], flush=True)
else:
    f.barrier()
    t = torch.full((n,), float(r), device=f.device)
    if v.endswith("groupsend"):
        ws = dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 0, group=f.kv_group)])
        for w in ws:
            w.wait()
    else:
        dist.send(t, 0, group=f.kv_group)
    torch.cuda.synchronize()
    print(f"rank {r} sent", flush=True)
f.barrier()
print(f"rank {r} done", flush=True)
