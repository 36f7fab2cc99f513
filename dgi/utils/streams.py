"""Named HIP streams: every long-lived stream the runtime issues work on is created
here, so a rank's stream budget can be checked against what really exists.

HIP maps a process's streams lazily onto ``GPU_MAX_HW_QUEUES`` (4) hardware
queues per priority class, round-robin; two streams that land on one queue are
serialised (``profiles/r3_hw_queue_probe.md``).  ``dgi.parallel.fabric.
Fabric.stream_budget`` lists what each role should use; ``created()`` lists what
this process actually made, and the GPU tests compare the two.

Long-lived streams (name: who):
  compute        the default stream (every kernel of a step)
  attn_side      decode-row attention beside prefill-row attention in a mixed
                 step (dgi.models.llama)
  kv_host_copy   pinned host KV tier spill / restore (dgi.kv.host_tier)
  recv           high priority: KV receives are posted from it (dgi.parallel.fabric)
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


def created(device_index: Optional[int] = None) -> dict:
    """Streams this process created through ``named_stream``, by priority class
    (``normal`` always includes the default ``compute`` stream)."""
    out = {"normal": ["compute"], "high": []}
    for (name, idx), (_s, prio) in sorted(_STREAMS.items()):
        if device_index is not None and idx != device_index:
            continue
        out["high" if prio < 0 else "normal"].append(name)
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
