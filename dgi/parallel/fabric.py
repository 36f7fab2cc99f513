"""RCCL fabric: process groups, data channels and the node-local control plane.

One process per GPU.  On MI355X the data plane is RCCL (``nccl`` backend) over
xGMI; on a CPU box (tests) everything falls back to gloo.

Data plane (device tensors)
  * ``kv`` — the world communicator, created EAGERLY (``init_process_group``
    with ``device_id``) so every point-to-point op runs on the one world
    communicator instead of a lazily created 2-rank communicator per pair
    (round 2: one extra RCCL stream per peer).  Carries prefill -> decode KV
    pages only.
  * ``pp`` — one sub-communicator per decode layer pipeline (``setup_layout``),
    carrying stage activations only.  Keeping KV and activations on separate
    communicators (= separate RCCL streams) is what makes the P/D protocol
    deadlock-free: a KV receive never queues behind an activation transfer
    and vice versa (``dgi.parallel.pd`` docstring has the argument).

Hardware queues.  HIP maps a process's streams lazily onto
``GPU_MAX_HW_QUEUES`` (4) hardware queues PER PRIORITY, round-robin; two
streams on one queue are ordered (a spinning RCCL kernel blocks the other
stream's work) — measured with ``scripts/probe_hwq.py``
(``profiles/r3_hw_queue_probe.md``).  So communication lives on HIGH-priority
streams (both RCCL communicators and the stream receives are posted from) and
compute on the default stream: at most 3 high-priority streams per rank,
never sharing a queue with each other or with compute.  ``stream_budget``
counts them and the tests assert the bound for every role.

Control plane (host, pollable): ``CtrlChannel`` — one shared-memory SPSC ring
per directed rank pair and tag (``dgi/csrc/host/shm_ring.cc``), a memcpy and a
release store per message, instead of the round-2 TCPStore round trip to rank
0 per poll.  ``DGI_CTRL=store`` selects the store transport (multi-host
debugging only).
"""
from __future__ import annotations

import atexit
import datetime
import os
import time
import uuid
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

GPU_HW_QUEUES = 4          # HIP default hardware queues per priority class per process
# CTS'd sends to several peers leave as one RCCL group (concurrent links; every receive of the
# group is already posted, so the group cannot wait on anything).  DGI_BATCH_P2P=0: one ordered
# send each on the world communicator's stream (round 3).  Shared-GPU rehearsals, 2P+6D:
# prefill RTS->CTS p50 131 ms batched vs 427 ms one by one (profiles/r4_rccl_rehearsal/)
BATCH_P2P = os.environ.get("DGI_BATCH_P2P", "1") == "1"


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
    """Environment RCCL must see before its first communicator.

    ``NCCL_RUNTIME_CONNECT=0``: every channel connects when the communicator
    is created instead of at the first transfer that needs it (a runtime
    connect is a blocking host handshake with the peer in the middle of
    serving)."""
    os.environ.setdefault("NCCL_RUNTIME_CONNECT", "0")
    # which transport each connection uses (P2P/IPC over xGMI vs a network fallback) goes into
    # the bench JSON: RCCL's INIT log, one file per rank, parsed by ``rccl_transports``
    # (DGI_RCCL_LOG=0, or a NCCL_DEBUG set by the user, leaves RCCL's logging alone)
    # (the image exports NCCL_DEBUG=VERSION, a one-line banner: that is not a user's logging choice)
    if os.environ.get("DGI_RCCL_LOG", "1") != "0" and os.environ.get("NCCL_DEBUG", "VERSION") in ("", "VERSION"):
        os.environ["NCCL_DEBUG"] = "INFO"
        os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT")
        os.environ["NCCL_DEBUG_FILE"] = rccl_log_path()
    # eager init already serialises unbatched p2p on the world communicator: that
    # is the point, so the one-time warning is noise
    os.environ.setdefault("TORCH_NCCL_SHOW_EAGER_INIT_P2P_SERIALIZATION_WARNING", "0")
    if shared_gpu():
        os.environ["NCCL_HOSTID"] = f"dgi-shared-rank{os.environ.get('RANK', '0')}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")


def rccl_log_path() -> str:
    d = os.environ.get("TMPDIR", "/tmp")
    return os.path.join(d, f"dgi_rccl_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('RANK', '0')}.log")


_VIA = None


def rccl_transports(path: Optional[str] = None) -> Optional[dict]:
    """Transport of every RCCL connection this rank set up, from its INIT log:
    ``{"by_transport": {"P2P/IPC": n, ...}, "peers": {"0->3": "P2P/IPC", ...}}``
    (None when no log was written: gloo, or logging left to the user)."""
    import re
    global _VIA
    path = path or os.environ.get("NCCL_DEBUG_FILE") or rccl_log_path()
    if not os.path.exists(path):
        return None
    if _VIA is None:
        _VIA = re.compile(r"(\d+)\[[^\]]*\]\s*->\s*(\d+)\[[^\]]*\]\s*(?:\[(?:send|receive)\]\s*)?via\s+(\S+)")
    by, peers = {}, {}
    with open(path, errors="replace") as fh:
        for line in fh:
            m = _VIA.search(line)
            if m is None:
                continue
            a, b, via = m.group(1), m.group(2), m.group(3)
            by[via] = by.get(via, 0) + 1
            peers[f"{a}->{b}"] = via
    return {"by_transport": by, "peers": peers, "log": path}


def _nccl_options():
    """RCCL communicators on high-priority streams (their own hardware queues)."""
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except Exception:  # pragma: no cover - CPU-only torch builds
        return None


# Default budget of the process group (every collective) and of control-ring waits.  Serving
# start-up waits span a peer's model load and graph capture (a cold 70B checkpoint load can
# take minutes), so the default is long; the benchmark passes its short rendezvous budget
# (DGI_INIT_S) explicitly and relies on the watchdog's phase deadlines for hangs.
LONG_WAIT_S = float(os.environ.get("DGI_PG_TIMEOUT_S", "1800"))


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> str:
    """Initialise the default process group for this process (idempotent).

    RCCL: eager init bound to this rank's GPU (``device_id``) with
    high-priority communicator streams.  Returns the backend in use."""
    if timeout_s is None:
        timeout_s = LONG_WAIT_S
    if dist.is_initialized():
        return dist.get_backend()
    be = backend or ("nccl" if torch.cuda.is_available() and os.environ.get("DGI_STAGED_GPU", "0") != "1"
                     else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    to = datetime.timedelta(seconds=timeout_s)
    if be == "nccl":
        prepare_rccl_env()
        dev = torch.device("cuda", local_device_index())
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", timeout=to, device_id=dev, pg_options=_nccl_options())
    else:
        dist.init_process_group(be, timeout=to)
    return be


_FABRICS = [0]


class Fabric:
    """Per-rank view of the node: communicators, streams and control rings."""

    def __init__(self, backend: Optional[str] = None, device: Optional[torch.device] = None,
                 timeout_s: Optional[float] = None):
        self.owns_pg = not dist.is_initialized()
        init_distributed(backend, timeout_s)
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        self.on_gpu = self.backend == "nccl"
        if self.on_gpu and getattr(dist.distributed_c10d._get_default_group(), "bound_device_id", None) is None:
            # lazily initialised RCCL: every point-to-point pair would get its own 2-rank
            # communicator and stream, and a first batched op hangs unless every rank joins it
            raise RuntimeError("dgi needs the RCCL process group initialised eagerly: call "
                               "dgi.parallel.fabric.init_distributed() (init_process_group(device_id=...))")
        # "staged" mode: GPU compute with a gloo data plane (tensors bounce
        # through host memory).  Lets the multi-rank GPU code paths run when
        # the ranks share one device without RCCL.
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
        self.kv_group = None                 # world communicator
        self.pp_groups: dict = {}           # tuple(stage ranks) -> sub-communicator
        # host barriers / object gathers: gloo, never a spinning RCCL collective
        self.ctrl = dist.new_group(backend="gloo")
        # receives are POSTED from this (empty, high-priority) stream so the RCCL
        # stream waits on nothing the compute stream has queued (a KV receive must
        # never depend on this rank's own compute: pd.py deadlock argument)
        if self.on_gpu:
            from dgi.utils.streams import named_stream
            self.recv_stream = named_stream("recv", device, priority=-1)
        else:
            self.recv_stream = None
        self._pending: list = []
        # DGI_DEBUG_STREAMS=1: send buffers must not be rewritten while in flight (dgi.utils.debug)
        from dgi.utils.debug import stream_checker
        self.checker = stream_checker()
        # control plane
        self.job = self._job_id()
        self._rings_out: dict = {}
        self._rings_in: dict = {}
        self.ctrl_kind = os.environ.get("DGI_CTRL", "shm")
        self.sent_msgs = 0
        self.ring_bytes = 0                  # shared memory of the rings this rank created
        self.pairs_connected = 0
        atexit.register(self._unlink_rings)
        # liveness watchdog over the rendezvous store (dgi.parallel.fault)
        self.watchdog = None
        if self.world > 1 and os.environ.get("DGI_WATCHDOG", "1") != "0":
            from dgi.parallel.fault import Watchdog, current_watchdog
            self.watchdog = current_watchdog() or Watchdog(self.rank, self.world).start()

    # ------------------------------------------------------------------ set-up
    def _job_id(self) -> str:
        """Name space of this fabric's shared-memory rings (same on every rank)."""
        from torch.distributed import distributed_c10d as c10d
        _FABRICS[0] += 1
        key = f"dgi/job/{_FABRICS[0]}"
        store = c10d._get_default_store()
        if self.rank == 0:
            store.set(key, uuid.uuid4().hex[:12])
        return store.get(key).decode()

    def setup_layout(self, layout, warmup: bool = True) -> float:
        """Create every communicator this node layout uses, on every rank in the
        same order (collective), and move one tensor over each pair so that RCCL
        connection set-up (and any failure of it) happens now.  Returns seconds."""
        t0 = time.perf_counter()
        groups = [tuple(g) for g in layout.pipeline_groups()]
        for g in groups:                       # every rank, same order: new_group is collective
            pg = dist.new_group(ranks=list(g), pg_options=_nccl_options() if self.on_gpu else None)
            if self.rank in g:
                self.pp_groups[g] = pg
        if warmup:
            self._warm(layout.kv_pairs(), None)
            for g in groups:
                if self.rank in g:
                    self._warm(list(zip(g, g[1:])), self.pp_groups[g])
        if self.on_gpu:
            torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    def connect_pairs(self, pairs: list) -> float:
        """Warm up the world communicator over ``pairs`` (sorted, same list on every
        rank: each rank walks its own pairs in that global order, so the walk cannot
        deadlock on one FIFO stream)."""
        t0 = time.perf_counter()
        self._warm(pairs, None)
        if self.on_gpu:
            torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    def _warm(self, pairs, group) -> None:
        dev = self.device if (self.on_gpu or self.staged) else torch.device("cpu")
        n = int(os.environ.get("DGI_PAIR_WARMUP_ELEMS", 1 << 21)) if self.on_gpu else 1
        for a, b in sorted(pairs):
            if self.rank not in (a, b):
                continue
            peer = b if self.rank == a else a
            t = torch.full((n,), self.rank, dtype=torch.int64, device=dev)
            r = torch.empty(n, dtype=torch.int64, device=dev)
            if self.staged:
                t, r = t.cpu(), r.cpu()
            if self.rank == a:
                dist.send(t, peer, group=group)
                dist.recv(r, peer, group=group)
            else:
                dist.recv(r, peer, group=group)
                dist.send(t, peer, group=group)
            if int(r[0]) != peer or int(r[-1]) != peer:
                raise RuntimeError(f"rank {self.rank}: pair warm-up with {peer} returned "
                                   f"{int(r[0])}..{int(r[-1])}")
            self.pairs_connected += 1

    def pp_group(self, ranks) -> Optional[object]:
        return self.pp_groups.get(tuple(ranks))

    def stream_budget(self, engines=()) -> dict:
        """Streams this rank issues GPU work on, per priority class.

        normal: per engine this rank serves (``dgi.utils.streams.engine_streams``)
        the compute (default) stream, the mixed-step attention side stream and the
        host KV tier's copy stream; high: the world (KV) communicator's RCCL
        stream, each pipeline sub-communicator's, and the stream receives are
        posted from.  Each class must fit in ``GPU_HW_QUEUES`` so no two streams
        share a hardware queue (``dgi.utils.streams.created`` lists what exists)."""
        from dgi.utils.streams import engine_streams
        normal = ["compute"]
        for e in engines:
            normal += [n for n in engine_streams(e) if n not in normal]
        high = ["rccl:kv", "recv"] + [f"rccl:pp{list(g)}" for g in self.pp_groups]
        return {"normal": normal, "high": high}

    # ------------------------------------------------------------------ data plane (device tensors)
    def send(self, t: torch.Tensor, dst: int, group=None) -> None:
        """Ordered send; ordered after the compute stream's queued work (the
        buffer's producer), never blocking it."""
        if self.staged:
            h = t.detach().cpu()
            self._pending.append((dist.isend(h, dst, group=group), h, None))
            self._reap()
            return
        self._track(dist.isend(t, dst, group=group), t)

    def send_many(self, items: list, group=None) -> None:
        """Several sends (``[(tensor, dst), ...]``) as ONE RCCL group: transfers to
        different peers progress concurrently over their own xGMI links."""
        if not items:
            return
        if self.staged or not self.on_gpu or len(items) == 1 or not BATCH_P2P:
            for t, d in items:
                self.send(t, d, group=group)
            return
        ops_ = [dist.P2POp(dist.isend, t, d, group=group) for t, d in items]
        works = list(dist.batch_isend_irecv(ops_) or [])
        if len(works) != len(items):        # RCCL: one coalesced work for the whole group
            works = [works[-1]] * len(items)
        for w, (t, _d) in zip(works, items):
            self._track(w, t)

    def recv(self, t: torch.Tensor, src: int, group=None) -> torch.Tensor:
        """Receive into ``t``, stream-ordered after this rank's compute and before
        anything the compute stream enqueues next (pipeline activations)."""
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src, group=group)
            t.copy_(h)
            return t
        w = dist.irecv(t, src, group=group)
        w.wait()
        return t

    def irecv_async(self, t: torch.Tensor, src: int, group=None) -> "AsyncRecv":
        """Post a receive into ``t`` that waits on NOTHING this rank has queued.

        On RCCL it is posted from ``recv_stream`` (empty, high priority), so its
        kernel starts at once on the communicator's own hardware queue; poll
        ``ready()`` from the host and call ``complete()`` to order follow-up work
        on the current stream.  ``t`` must have been allocated on
        ``recv_stream`` (``alloc_recv``)."""
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            return AsyncRecv(self, dist.irecv(h, src, group=group), t, host=h)
        if self.on_gpu:
            with torch.cuda.stream(self.recv_stream):
                w = dist.irecv(t, src, group=group)
            return AsyncRecv(self, w, t)
        return AsyncRecv(self, dist.irecv(t, src, group=group), t)

    def irecv_batch(self, items: list, group=None) -> list:
        """Post several receives (``[(tensor, src), ...]``, distinct sources) as ONE
        RCCL group from ``recv_stream``: they progress concurrently over their own
        links and none waits behind another (``dgi.parallel.kv_transfer`` deadlock
        argument).  One ``AsyncRecv`` per item."""
        if len(items) == 1:
            t, src = items[0]
            return [self.irecv_async(t, src, group=group)]
        if self.staged:
            hs = [torch.empty(t.shape, dtype=t.dtype) for t, _s in items]
            works = dist.batch_isend_irecv([dist.P2POp(dist.irecv, h, s, group=group) for h, (_t, s) in zip(hs, items)])
            return [AsyncRecv(self, w, t, host=h) for w, h, (t, _s) in zip(works, hs, items)]
        ops_ = [dist.P2POp(dist.irecv, t, s, group=group) for t, s in items]
        if self.on_gpu:
            with torch.cuda.stream(self.recv_stream):
                works = dist.batch_isend_irecv(ops_)
        else:
            works = dist.batch_isend_irecv(ops_)
        works = list(works or [])
        if len(works) != len(items):
            # RCCL coalesces the group into ONE work (torch's _coalescing_manager): every
            # receive of the batch completes with it
            assert works, "batch_isend_irecv returned no work handle"
            works = [works[-1]] * len(items)
        return [AsyncRecv(self, w, t) for w, (t, _s) in zip(works, items)]

    def alloc_recv(self, shape, dtype) -> torch.Tensor:
        """A receive buffer owned by ``recv_stream`` (caching-allocator safe for
        ``irecv_async``)."""
        if self.on_gpu:
            with torch.cuda.stream(self.recv_stream):
                return torch.empty(shape, dtype=dtype, device=self.device)
        return torch.empty(shape, dtype=dtype, device=self.device if self.staged else "cpu")

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

    def sends_in_flight(self) -> int:
        self._reap()
        return len(self._pending)

    def flush(self) -> None:
        """Host-wait for every tracked send.  Only call when each of them is known
        to have its receive posted (P/D: every send is clear-to-send gated)."""
        for w, _t, rec in self._pending:
            w.wait()
            self._done(rec)
        self._pending = []

    # ------------------------------------------------------------------ control plane
    def _ring_name(self, src: int, dst: int, tag: str) -> str:
        return f"/dgi.{self.job}.{src}.{dst}.{tag}"

    def ring_out(self, peer: int, tag: str, capacity: int):
        key = (peer, tag)
        r = self._rings_out.get(key)
        if r is None:
            from dgi.parallel.shm import create_ring, shm_free_bytes
            free = shm_free_bytes()
            if free is not None and free < capacity:
                raise RuntimeError(
                    f"rank {self.rank}: /dev/shm has {free >> 20} MiB free, the {tag} control ring to rank {peer} "
                    f"needs {capacity >> 20} MiB ({self.ring_bytes >> 20} MiB already mapped by this rank): give "
                    f"the container a larger /dev/shm (docker --shm-size, e.g. 1g for an 8-GPU node)")
            r = create_ring(self._ring_name(self.rank, peer, tag), capacity)
            self._rings_out[key] = r
            self.ring_bytes += capacity
        return r

    def ring_in(self, peer: int, tag: str, wait_s: float = 0.0):
        key = (peer, tag)
        r = self._rings_in.get(key)
        if r is None:
            from dgi.parallel.shm import open_ring
            r = open_ring(self._ring_name(peer, self.rank, tag), wait_s)
            if r is not None:
                self._rings_in[key] = r
        return r

    def _unlink_rings(self) -> None:
        from dgi.parallel.shm import unlink
        for r in list(self._rings_out.values()):
            unlink(r.name)

    def ctrl_group(self):
        return self.ctrl

    def barrier(self) -> None:
        """Host-side barrier on the gloo control group.  Callers synchronise their
        own device first; an RCCL barrier would add an all-reduce kernel that spins
        on every GPU until the last rank arrives."""
        dist.barrier(group=self.ctrl)

    def close(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        self.flush()
        self._unlink_rings()
        if self.owns_pg and dist.is_initialized():
            dist.destroy_process_group()


class AsyncRecv:
    """Handle of one ``Fabric.irecv_async``."""

    __slots__ = ("f", "work", "t", "host", "done", "t_post")

    def __init__(self, fabric: Fabric, work, t: torch.Tensor, host: Optional[torch.Tensor] = None):
        self.f, self.work, self.t, self.host, self.done = fabric, work, t, host, False
        self.t_post = time.perf_counter()

    def ready(self) -> bool:
        # gloo completes a p2p receive only inside wait(): on CPU / staged runs
        # report ready and let complete() block (the sender is clear-to-send
        # gated, so the data is on its way)
        if self.done or not self.f.on_gpu:
            return True
        return self.work.is_completed()

    def complete(self) -> None:
        """Make the data visible to work issued next on the CURRENT stream (GPU) or
        to the host (CPU / staged)."""
        if self.done:
            return
        self.work.wait()       # GPU: current stream waits on the RCCL stream's event
        if self.host is not None:
            self.t.copy_(self.host)
        if self.f.on_gpu:
            self.t.record_stream(torch.cuda.current_stream())
        self.done = True


class CtrlChannel:
    """Pollable int64 control messages to/from one peer (one direction each way).

    Shared-memory rings by default (``dgi.parallel.shm``); ``DGI_CTRL=store``
    uses the c10d store.  ``send`` pads to ``size`` words, ``send_var`` sends
    any length; ``poll`` returns the next message or None, ``wait`` blocks.
    Both ends must construct the channel (each creates its outgoing ring)."""

    RING_BYTES = 1 << 21

    def __init__(self, fabric: Fabric, peer: int, size: int = 32, tag: str = "ctrl", capacity: int = 0):
        self.f = fabric
        self.peer = peer
        self.size = size
        self.tag = tag
        self.me = fabric.rank
        self.sseq = 0
        self.rseq = 0
        self.shm = fabric.ctrl_kind == "shm"
        if self.shm:
            cap = capacity or int(os.environ.get("DGI_SHM_RING_BYTES", self.RING_BYTES))
            self._out = fabric.ring_out(peer, tag, cap)
            self._in = None
        else:
            from torch.distributed import distributed_c10d as c10d
            self.store = c10d._get_default_store()

    # ---------------------------------------------------------------- shm
    def _inbox(self, wait_s: float = 0.0):
        if self._in is None:
            self._in = self.f.ring_in(self.peer, self.tag, wait_s)
        return self._in

    def send_bytes(self, b: bytes) -> None:
        self.f.sent_msgs += 1
        if self.shm:
            self._out.send(b, 600.0)
        else:
            self.store.set(f"dgi/{self.tag}/{self.me}->{self.peer}/{self.sseq}", b)
        self.sseq += 1

    def poll_bytes(self) -> Optional[bytes]:
        if self.shm:
            r = self._inbox()
            return None if r is None else r.poll()
        k = f"dgi/{self.tag}/{self.peer}->{self.me}/{self.rseq}"
        if not self.store.check([k]):
            return None
        v = self.store.get(k)
        self.store.delete_key(k)
        self.rseq += 1
        return v

    def wait_bytes(self, timeout_s: Optional[float] = None) -> bytes:
        if timeout_s is None:
            timeout_s = LONG_WAIT_S
        if self.shm:
            r = self._inbox(timeout_s)
            if r is None:
                raise TimeoutError(f"rank {self.me}: ring {self.tag} from {self.peer} never created")
            v = r.wait(timeout_s)
            if v is None:
                raise TimeoutError(f"rank {self.me}: no {self.tag} message from {self.peer} in {timeout_s}s")
            return v
        k = f"dgi/{self.tag}/{self.peer}->{self.me}/{self.rseq}"
        self.store.wait([k], datetime.timedelta(seconds=timeout_s))
        v = self.store.get(k)
        self.store.delete_key(k)
        self.rseq += 1
        return v

    # ---------------------------------------------------------------- int64 messages
    def send(self, arr) -> None:
        a = np.zeros(self.size, np.int64)
        v = np.asarray(arr, np.int64).ravel()
        a[: v.size] = v
        self.send_bytes(a.tobytes())

    def send_var(self, arr) -> None:
        """Variable-length message (e.g. a prompt's token ids)."""
        self.send_bytes(np.ascontiguousarray(np.asarray(arr, np.int64).ravel()).tobytes())

    def poll(self) -> Optional[np.ndarray]:
        v = self.poll_bytes()
        return None if v is None else np.frombuffer(v, dtype=np.int64).copy()

    def wait(self, timeout_s: Optional[float] = None) -> np.ndarray:
        return np.frombuffer(self.wait_bytes(timeout_s), dtype=np.int64).copy()
