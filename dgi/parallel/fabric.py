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


def shared_gpu() -> bool:
    """``DGI_SHARED_GPU=1``: several ranks share one GPU and still talk RCCL.

    RCCL refuses two ranks on one device of one host ("Duplicate GPU
    detected"); giving every rank its own ``NCCL_HOSTID`` makes each look like
    a separate host, so the data plane runs RCCL's network transport over
    loopback.  Slow, but every send/recv is a real RCCL kernel on a real
    stream with RCCL's blocking semantics (a send waits for its matching
    receive), which a gloo rehearsal cannot show: the rehearsal for the
    8-GPU layouts on a one-GPU box."""
    return os.environ.get("DGI_SHARED_GPU", "0") == "1"


def local_device_index() -> int:
    lr = int(os.environ.get("LOCAL_RANK", 0))
    if shared_gpu():
        return lr % max(1, torch.cuda.device_count())
    return lr


def prepare_rccl_env() -> None:
    """Environment RCCL must see before its first communicator (call before
    ``init_process_group('nccl')``).

    ``NCCL_RUNTIME_CONNECT=0``: every channel of a communicator connects when the
    communicator is created (``Fabric.connect_pairs`` at start-up) instead of at the
    first transfer that needs it.  A runtime connect is a blocking host handshake
    with the peer; with one host thread per rank serving several pairs (a prefill
    rank feeding three replicas, a replica fed by five prefill ranks) those
    handshakes can wait on each other in a cycle in the middle of serving."""
    os.environ.setdefault("NCCL_RUNTIME_CONNECT", "0")
    if shared_gpu():
        os.environ["NCCL_HOSTID"] = f"dgi-shared-rank{os.environ.get('RANK', '0')}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")


class Fabric:
    def __init__(self, backend: Optional[str] = None, device: Optional[torch.device] = None,
                 timeout_s: float = 1800.0):
        self.owns_pg = False
        if not dist.is_initialized():
            be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            if be == "nccl":
                prepare_rccl_env()
                torch.cuda.set_device(local_device_index())
            dist.init_process_group(be, timeout=datetime.timedelta(seconds=timeout_s))
            self.owns_pg = True
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        self.on_gpu = self.backend == "nccl"
        # "staged" mode: GPU compute with a gloo data plane (tensors bounce
        # through host memory).  Lets the multi-rank GPU code paths run when
        # the ranks share one device (rehearsals on a single-GPU box).
        self.staged = False
        if device is None:
            if self.on_gpu:
                device = torch.device("cuda", torch.cuda.current_device())
            elif torch.cuda.is_available() and os.environ.get("DGI_STAGED_GPU", "0") == "1":
                device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
                torch.cuda.set_device(device)
                self.staged = True
            else:
                device = torch.device("cpu")
        self.device = device
        # control traffic gets its own gloo group so it never queues behind (or
        # forms a dependency cycle with) data transfers on the RCCL pair channel
        self.ctrl = dist.new_group(backend="gloo")
        self.comm_stream = torch.cuda.Stream(device=device) if self.on_gpu else None
        # KV-migration receives land on their own stream so decode compute never
        # queues behind a multi-hundred-MB transfer (see ``irecv_async``)
        self.recv_stream = torch.cuda.Stream(device=device) if self.on_gpu else None
        self._pending: list = []
        # DGI_DEBUG_STREAMS=1: send buffers must not be rewritten while in flight (dgi.utils.debug)
        from dgi.utils.debug import stream_checker
        self.checker = stream_checker()
        # liveness watchdog over the rendezvous store (dgi.parallel.fault)
        self.watchdog = None
        if self.world > 1 and os.environ.get("DGI_WATCHDOG", "1") != "0":
            from dgi.parallel.fault import Watchdog
            self.watchdog = Watchdog(self.rank, self.world).start()

    # ------------------------------------------------------------------ data (device tensors)
    def send(self, t: torch.Tensor, dst: int) -> None:
        """Ordered send on the data group; the compute stream is not blocked."""
        if self.staged:
            h = t.detach().cpu()
            self._pending.append((dist.isend(h, dst), h, None))
            self._reap()
            return
        if self.on_gpu:
            ev = torch.cuda.current_stream().record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                w = dist.isend(t, dst)
            self._track(w, t)
        else:
            self._track(dist.isend(t, dst), t)

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        """Blocking (stream-ordered on GPU) receive into ``t``."""
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src)
            t.copy_(h)
            return t
        w = dist.irecv(t, src)
        w.wait()
        return t

    def irecv_async(self, t: torch.Tensor, src: int) -> "AsyncRecv":
        """Post a receive into ``t`` without ordering it before later compute.

        On RCCL the receive is enqueued with ``recv_stream`` as the issuing
        stream, so nothing on the compute stream waits for it; poll
        ``ready()`` from the host and call ``complete()`` to order follow-up
        work (e.g. a page scatter) on ``recv_stream``."""
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            return AsyncRecv(self, dist.irecv(h, src), t, host=h)
        if self.on_gpu:
            with torch.cuda.stream(self.recv_stream):
                w = dist.irecv(t, src)
            return AsyncRecv(self, w, t)
        return AsyncRecv(self, dist.irecv(t, src), t)

    def _track(self, w, t: torch.Tensor) -> None:
        rec = self.checker.on_send(t) if self.checker is not None else None
        self._pending.append((w, t, rec))
        self._reap()

    def _done(self, rec) -> None:
        if rec is not None:
            self.checker.on_complete(rec)

    def _reap(self) -> None:
        keep = []
        for w, t, rec in self._pending:
            if w.is_completed():
                self._done(rec)
            else:
                keep.append((w, t, rec))
        self._pending = keep

    def flush(self) -> None:
        for w, _t, rec in self._pending:
            w.wait()
            self._done(rec)
        self._pending = []
        if self.on_gpu:
            torch.cuda.current_stream().wait_stream(self.comm_stream)

    def connect_pairs(self, pairs: list) -> float:
        """Create every point-to-point communicator this rank will use NOW, with
        one tiny send/recv per pair, so that RCCL set-up (and any failure of
        it) happens at start-up instead of inside the first KV migration or
        pipeline hop.  ``pairs`` must be the same sorted list on every rank
        (``NodeLayout.p2p_pairs``): each rank walks its own pairs in that
        global order and the first unfinished pair always has both ends ready,
        so the walk cannot deadlock.  Returns the seconds it took."""
        import time as _time
        t0 = _time.perf_counter()
        dev = self.device if (self.on_gpu or self.staged) else torch.device("cpu")
        for a, b in pairs:
            if self.rank not in (a, b):
                continue
            peer = b if self.rank == a else a
            # big enough for every protocol / channel a KV page transfer uses
            n = int(os.environ.get("DGI_PAIR_WARMUP_ELEMS", 1 << 21)) if self.on_gpu else 1
            t = torch.full((n,), self.rank, dtype=torch.int64, device=dev)
            r = torch.empty(n, dtype=torch.int64, device=dev)
            if self.staged:
                t, r = t.cpu(), r.cpu()
            if self.rank == a:
                dist.send(t, peer)
                dist.recv(r, peer)
            else:
                dist.recv(r, peer)
                dist.send(t, peer)
            if int(r[0].item()) != peer or int(r[-1].item()) != peer:
                raise RuntimeError(f"rank {self.rank}: pair warm-up with {peer} returned {int(r.item())}")
        if self.on_gpu:
            torch.cuda.synchronize(self.device)
        self.pairs_connected = len([1 for a, b in pairs if self.rank in (a, b)])
        return _time.perf_counter() - t0

    # ------------------------------------------------------------------ control (host, pollable)
    def ctrl_group(self):
        return self.ctrl

    def ctrl_isend(self, arr: np.ndarray, dst: int):
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
        w = dist.isend(t, dst, group=self.ctrl)
        self._pending.append((w, t, None))
        return w

    def ctrl_send_tensor(self, t: torch.Tensor, dst: int) -> None:
        """Non-blocking host tensor send on the control group."""
        t = t.detach().cpu().contiguous()
        self._pending.append((dist.isend(t, dst, group=self.ctrl), t, None))

    def ctrl_recv_tensor(self, t: torch.Tensor, src: int) -> torch.Tensor:
        dist.recv(t, src, group=self.ctrl)
        return t

    def ctrl_irecv(self, size: int, src: int):
        t = torch.zeros(size, dtype=torch.int64)
        w = dist.irecv(t, src, group=self.ctrl)
        return w, t

    def barrier(self) -> None:
        """Host-side barrier on the gloo control group.  Callers synchronise their
        own device first; an RCCL barrier would add an all-reduce kernel that spins
        on every GPU until the last rank arrives (and, with ranks sharing a GPU in the
        DGI_SHARED_GPU rehearsal, starves the work the late ranks still have queued)."""
        dist.barrier(group=self.ctrl)

    def close(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        self.flush()
        if self.owns_pg and dist.is_initialized():
            dist.destroy_process_group()


class AsyncRecv:
    """Handle of one ``Fabric.irecv_async``."""

    __slots__ = ("f", "work", "t", "host", "done")

    def __init__(self, fabric: Fabric, work, t: torch.Tensor, host: Optional[torch.Tensor] = None):
        self.f, self.work, self.t, self.host, self.done = fabric, work, t, host, False

    def ready(self) -> bool:
        # gloo completes a p2p receive only inside wait(): on CPU / staged runs
        # report ready and let complete() block (rehearsals, not a hot path)
        if self.done or not self.f.on_gpu:
            return True
        return self.work.is_completed()

    def complete(self) -> None:
        """Make the data visible: afterwards work issued on ``fabric.recv_stream``
        (GPU) or the host (CPU / staged) sees the received bytes."""
        if self.done:
            return
        if self.f.on_gpu:
            with torch.cuda.stream(self.f.recv_stream):
                self.work.wait()
        else:
            self.work.wait()
            if self.host is not None:
                self.t.copy_(self.host)
        self.done = True


class CtrlChannel:
    """Pollable fixed-size int64 control messages to/from one peer.

    Carried by the c10d rendezvous store (TCPStore): a gloo ``irecv`` cannot
    be polled (its completion is only observed by ``wait``), while a store
    key can be checked without blocking.  Messages are sequence-numbered per
    direction and deleted once read.  Used for P/D admission headers,
    credits and end-of-stream markers — a few small messages per step.
    """

    def __init__(self, fabric: Fabric, peer: int, size: int = 32, tag: str = "ctrl"):
        from torch.distributed import distributed_c10d as c10d
        self.f = fabric
        self.peer = peer
        self.size = size
        self.store = c10d._get_default_store()
        self.me = fabric.rank
        self.tag = tag
        self.sseq = 0
        self.rseq = 0

    def _key(self, src: int, dst: int, seq: int) -> str:
        return f"dgi/{self.tag}/{src}->{dst}/{seq}"

    def send(self, arr) -> None:
        a = np.zeros(self.size, np.int64)
        v = np.asarray(arr, np.int64).ravel()
        a[: v.size] = v
        self.store.set(self._key(self.me, self.peer, self.sseq), a.tobytes())
        self.sseq += 1

    def send_var(self, arr) -> None:
        """Variable-length message (e.g. a prompt's token ids)."""
        self.store.set(self._key(self.me, self.peer, self.sseq), np.asarray(arr, np.int64).ravel().tobytes())
        self.sseq += 1

    def poll(self) -> Optional[np.ndarray]:
        k = self._key(self.peer, self.me, self.rseq)
        if not self.store.check([k]):
            return None
        return self._take(k)

    def wait(self) -> np.ndarray:
        k = self._key(self.peer, self.me, self.rseq)
        self.store.wait([k])
        return self._take(k)

    def _take(self, k: str) -> np.ndarray:
        v = self.store.get(k)
        self.store.delete_key(k)
        self.rseq += 1
        return np.frombuffer(v, dtype=np.int64).copy()
