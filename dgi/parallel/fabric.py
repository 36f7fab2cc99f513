"""RCCL fabric: process groups and point-to-point channels between ranks.

One process per GPU.  On MI355X the default group is ``nccl`` (= RCCL on
ROCm) and every tensor moved between GPUs of the node goes over xGMI as an
RCCL send/recv — pipeline activations and prefill->decode KV pages alike
(SURVEY §2.9.2 C1-C4).  A second ``gloo`` group carries small control
messages that must be polled without blocking a GPU stream (P/D admission
headers, credits).  On a CPU-only box both roles fall back to gloo, which is
how the multi-process tests run.

Sends run on a dedicated comm stream so a send waiting for its peer never
stalls the compute stream; buffers stay referenced until their work
completes.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist


class Fabric:
    def __init__(self, backend: Optional[str] = None, device: Optional[torch.device] = None,
                 timeout_s: float = 1800.0):
        self.owns_pg = False
        if not dist.is_initialized():
            be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            if be == "nccl":
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
            dist.init_process_group(be, timeout=datetime.timedelta(seconds=timeout_s))
            self.owns_pg = True
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        self.on_gpu = self.backend == "nccl"
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.on_gpu else torch.device("cpu")
        self.device = device
        self.ctrl = dist.new_group(backend="gloo") if self.on_gpu else None
        self.comm_stream = torch.cuda.Stream(device=device) if self.on_gpu else None
        self._pending: list = []

    # ------------------------------------------------------------------ data (device tensors)
    def send(self, t: torch.Tensor, dst: int) -> None:
        """Ordered send on the data group; the compute stream is not blocked."""
        if self.on_gpu:
            ev = torch.cuda.current_stream().record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                w = dist.isend(t, dst)
            self._pending.append((w, t))
            self._reap()
        else:
            dist.send(t, dst)

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        """Blocking (stream-ordered on GPU) receive into ``t``."""
        w = dist.irecv(t, src)
        w.wait()
        return t

    def _reap(self) -> None:
        self._pending = [(w, t) for (w, t) in self._pending if not w.is_completed()]

    def flush(self) -> None:
        for w, _t in self._pending:
            w.wait()
        self._pending = []
        if self.on_gpu:
            torch.cuda.current_stream().wait_stream(self.comm_stream)

    # ------------------------------------------------------------------ control (host, pollable)
    def ctrl_group(self):
        return self.ctrl

    def ctrl_isend(self, arr: np.ndarray, dst: int):
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
        w = dist.isend(t, dst, group=self.ctrl)
        self._pending.append((w, t))
        return w

    def ctrl_irecv(self, size: int, src: int):
        t = torch.zeros(size, dtype=torch.int64)
        w = dist.irecv(t, src, group=self.ctrl)
        return w, t

    def barrier(self) -> None:
        dist.barrier()

    def close(self) -> None:
        self.flush()
        if self.owns_pg and dist.is_initialized():
            dist.destroy_process_group()


class CtrlChannel:
    """Pollable fixed-size int64 control messages from one peer."""

    def __init__(self, fabric: Fabric, peer: int, size: int = 32):
        self.f = fabric
        self.peer = peer
        self.size = size
        self._post()

    def _post(self):
        self.work, self.buf = self.f.ctrl_irecv(self.size, self.peer)

    def poll(self) -> Optional[np.ndarray]:
        if self.work.is_completed():
            self.work.wait()
            msg = self.buf.numpy().copy()
            self._post()
            return msg
        return None

    def wait(self) -> np.ndarray:
        self.work.wait()
        msg = self.buf.numpy().copy()
        self._post()
        return msg

    def send(self, arr) -> None:
        a = np.zeros(self.size, np.int64)
        v = np.asarray(arr, np.int64).ravel()
        a[: v.size] = v
        self.f.ctrl_isend(a, self.peer)
