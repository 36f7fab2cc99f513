"""Named HIP streams: every long-lived stream the runtime issues work on is created
here, so a rank's stream budget can be checked against what really exists.

HIP maps a process's streams lazily onto ``GPU_MAX_HW_QUEUES`` (4) hardware
queues per priority class, round-robin; two streams that land on one queue are
serialised (``profiles/r3_hw_queue_probe.md``).  ``dgi.parallel.fabric.
Fabric.stream_budget`` lists what each role should use; ``created()`` lists what
this process actually made, and the GPU tests compare the two.

Long-lived streams (name: who; the last two are CU-masked, one hardware queue each):
  compute        the default stream (every kernel of a step)
  attn_side      decode-row attention beside prefill-row attention in a mixed
                 step (dgi.models.llama)
  kv_host_copy   pinned host KV tier spill / restore (dgi.kv.host_tier)
  recv           high priority: KV receives are posted from it (dgi.parallel.fabric)
  tbo_gemm       CU-masked (all but ``side`` CUs of every XCD): the GEMM chain of a
                 two-batch-overlap decode step (dgi.models.llama.forward_layers_tbo)
  tbo_attn       CU-masked (``side`` CUs of every XCD): that step's decode attention
Transient: graph capture warm-up (``capture``) runs only while graphs are
captured, before serving.
"""
from __future__ import annotations

from typing import Optional

import torch

_STREAMS: dict = {}      # (name, device index) -> (stream, priority)


def named_stream(name: str, device, priority: int = 0) -> "torch.cuda.Stream":
    dev = torch.device(device)
    key = (name, dev.index if dev.index is not None else torch.cuda.current_device())
    hit = _STREAMS.get(key)
    if hit is None:
        hit = (torch.cuda.Stream(device=dev, priority=priority), priority)
        _STREAMS[key] = hit
    return hit[0]


def xcd_split(n_cus: int, side_per_xcd: int, xcds: int = 8) -> tuple:
    """(main CUs, side CUs) with ``side_per_xcd`` CUs of EVERY XCD on the side.

    CU-mask bits are XCD-major on MI355X (bits 32x .. 32x+31 = XCD x): a mask of
    bits 0-31 streams at 1.3 TB/s (one XCD), 4 CUs of each of the 8 XCDs at
    4.2 TB/s, and a GEMM whose mask leaves two XCDs empty runs 1.5x slower
    (``scripts/cu_mask_probe.py``, profiles/r5_pd/)."""
    per = n_cus // xcds
    side = [x * per + j for x in range(xcds) for j in range(side_per_xcd)]
    ss = set(side)
    return [c for c in range(n_cus) if c not in ss], side


def cu_masked_stream(name: str, device, cus: list) -> "torch.cuda.ExternalStream":
    """A stream whose kernels run only on CUs ``cus`` (``hipExtStreamCreateWithCUMask``).

    The mask binds to the stream's hardware queue, so it holds for kernels
    launched on the stream; kernels captured into a hipGraph lose it (the graph
    replays on the launching stream's queue), so CU-masked work runs eagerly."""
    import ctypes
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (name, idx)
    hit = _STREAMS.get(key)
    if hit is not None:
        return hit[0]
    n = torch.cuda.get_device_properties(idx).multi_processor_count
    words = [0] * ((n + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    hs = ctypes.c_void_p()
    lib = ctypes.CDLL("libamdhip64.so")
    with torch.cuda.device(idx):
        rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(hs), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask({name}) failed: {rc}")
    st = torch.cuda.ExternalStream(hs.value, device=torch.device("cuda", idx))
    _STREAMS[key] = (st, "masked")
    return st


def created(device_index: Optional[int] = None) -> dict:
    """Streams this process created through ``named_stream``, by priority class
    (``normal`` always includes the default ``compute`` stream)."""
    out = {"normal": ["compute"], "high": [], "dedicated": []}
    for (name, idx), (_s, prio) in sorted(_STREAMS.items()):
        if device_index is not None and idx != device_index:
            continue
        out["dedicated" if prio == "masked" else "high" if prio < 0 else "normal"].append(name)
    return out


def engine_streams(engine) -> list:
    """Normal-priority streams an engine uses while serving: the default stream, the
    mixed-step attention side stream (on GPU, when ATTN_OVERLAP is on), the host KV
    tier's copy stream when the engine has one."""
    from dgi.models import llama
    names = ["compute"]
    dev = getattr(engine, "device", torch.device("cpu"))
    if dev.type == "cuda" and llama.ATTN_OVERLAP:
        names.append("attn_side")
    if getattr(engine, "host_tier", None) is not None and dev.type == "cuda":
        names.append("kv_host_copy")
    return names


def dedicated_streams(engine) -> list:
    """CU-masked streams an engine may use (two-batch-overlap decode steps).  A CU mask is a
    property of a hardware queue, so each gets a queue of its own outside the round-robin
    pool that ``engine_streams`` is budgeted against."""
    from dgi.models import llama
    dev = getattr(engine, "device", torch.device("cpu"))
    return ["tbo_gemm", "tbo_attn"] if dev.type == "cuda" and llama.TBO else []
