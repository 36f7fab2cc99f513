"""Debug modes for bisecting GPU / multi-rank faults.

The reference has no race detection or sanitizer support at all.  Three
opt-in modes, all off by default and free when off:

* ``DGI_DEBUG_SYNC=1`` — *serialized* execution: every dgi HIP op is followed
  by a device synchronize and an error check, so an asynchronous fault is
  reported at the op that caused it (with its name and input shapes) instead
  of at some later, unrelated sync.  After every MFMA GEMM it also reads the
  split-K error word (``ops.gemm_split_timeouts``: a last piece whose bounded
  wait for the other pieces' slabs ran out) and raises on a nonzero count.
  ``enable_serialized()`` also exports
  ``HIP_LAUNCH_BLOCKING=1`` / ``AMD_SERIALIZE_KERNEL=3`` for processes spawned
  afterwards (the HIP runtime reads them at start-up).
* ``DGI_DEBUG_STREAMS=1`` — *stream-ordering checker* on the RCCL fabric:
  every send buffer's tensor version is recorded when the send is enqueued on
  the comm stream and re-checked when the send completes; an in-place write
  to a buffer whose transfer was still in flight (the compute stream reusing
  memory the comm stream is still reading) raises ``StreamOrderError``.
  Receive buffers must be ``complete()``-d before they are read.
* ``PYTHONASYNCIODEBUG=1`` — asyncio debug mode for the worker daemon, the
  batcher and the servers; CI runs the asyncio-based suites under it.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


class StreamOrderError(RuntimeError):
    pass


def sync_enabled() -> bool:
    return os.environ.get("DGI_DEBUG_SYNC", "0") == "1"


def streams_enabled() -> bool:
    return os.environ.get("DGI_DEBUG_STREAMS", "0") == "1"


def enable_serialized() -> None:
    """Turn on serialized mode for this process and the ones it starts."""
    os.environ["DGI_DEBUG_SYNC"] = "1"
    os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
    os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")


def after_op(name: str, *tensors) -> None:
    """Serialized mode: synchronize after a native op and name it on failure."""
    if not sync_enabled():
        return
    if not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        return
    try:
        torch.cuda.synchronize()
    except Exception as e:  # pragma: no cover - needs a faulting kernel
        shapes = [tuple(t.shape) for t in tensors if isinstance(t, torch.Tensor)]
        raise RuntimeError(f"dgi op {name} failed (inputs {shapes}): {e}") from e
    if name.startswith("mfma_gemm"):
        from dgi import ops
        n = ops.gemm_split_timeouts(reset=True)
        if n:  # pragma: no cover - needs a broken split-K counter
            shapes = [tuple(t.shape) for t in tensors if isinstance(t, torch.Tensor)]
            raise RuntimeError(f"dgi op {name}: {n} split-K wait(s) timed out (inputs {shapes}): wrong tiles")


class StreamOrderChecker:
    """Send-buffer reuse detector for ``Fabric`` (enabled by DGI_DEBUG_STREAMS=1)."""

    def __init__(self):
        self.sends = 0
        self.checked = 0
        self.violations: list = []

    def on_send(self, t: torch.Tensor) -> tuple:
        """Record the buffer: its version counter, or (inference-mode tensors have
        none) a snapshot of its bytes compared when the send completes."""
        self.sends += 1
        snap = t.detach().clone() if t.is_inference() else None
        ver = None if snap is not None else t._version
        return (t, ver, snap, t.data_ptr(), t.numel() * t.element_size())

    def on_complete(self, rec: tuple) -> None:
        t, ver, snap, ptr, nbytes = rec
        self.checked += 1
        changed = (t._version != ver) if snap is None else not torch.equal(t, snap)
        if changed:
            msg = (f"send buffer {ptr:#x} ({nbytes} B) was written while its transfer was in flight "
                   "on the comm stream")
            self.violations.append(msg)
            raise StreamOrderError(msg)

    def stats(self) -> dict:
        return {"sends": self.sends, "checked": self.checked, "violations": len(self.violations)}


_checker: Optional[StreamOrderChecker] = None


def stream_checker() -> Optional[StreamOrderChecker]:
    global _checker
    if not streams_enabled():
        return None
    if _checker is None:
        _checker = StreamOrderChecker()
    return _checker
