"""Deadlock-free KV page transfers over RCCL: ready-to-send / clear-to-send.

Round 2 enqueued a prefill rank's RCCL sends as soon as a step produced the
pages.  On RCCL a send kernel waits for its matching receive, and each rank
talked to several peers through one FIFO stream, so sends to different decode
ranks could wait on each other in a cycle (the 8-rank 5P+3D hang,
profiles/r2_rccl_rehearsal/OPEN_pd8_5p_3d_*.err; ADVICE r2 "high").  Here
every transfer is a three-message handshake on the shared-memory control
plane, and the data moves only once both ends are committed:

    prefill rank P                                    decode rank X
    gather pages (compute stream), event
    event complete  --RTS(tid, group, shape)------->  queue (FIFO over all P)
                                                      when X has NO receive in flight:
                                                        post irecv (own stream, waits on nothing)
                    <-------------------CTS(tid)---
    enqueue the send (batched with the other
    CTS'd sends of this poll: one RCCL group)
                                                      poll: landed -> scatter into the pool

Why it cannot deadlock (on the KV communicator's FIFO stream of every rank):
  (1) a decode rank has at most ONE receive posted, and posts it from an empty
      stream, so the receive kernel is running from the moment it is posted
      (communicators live on their own high-priority hardware queues,
      dgi.parallel.fabric);
  (2) a prefill rank enqueues a send only after its receiver's CTS, i.e. the
      partner of EVERY send in a prefill rank's stream is a running receive;
  (3) so the head of each prefill stream completes as soon as its own compute
      (the gather) is done, and by induction every send and receive completes.
Nothing on either side waits on the other's compute or on another transfer.
The decode side never blocks its host on a transfer it has not posted; a
prefill rank drains (``KVSender.drain``) only at phase boundaries, while every
decode rank keeps servicing its queue.

Control messages (int64, tag "kv"):
  RTS  [1, tid, key, group, ngroups, c0, c1, nblk]    (c0, c1: the receiver's local layers)
  CTS  [2, tid]
"""
from __future__ import annotations

import collections
import os
import time
from typing import Optional

import numpy as np
import torch

from dgi.parallel.fabric import CtrlChannel, Fabric

RTS, CTS = 1, 2
KV_TAG = "kv"
# DGI_KV_CHECKSUM=1 (tests): the sender hashes every gathered buffer and the receiver
# re-gathers every installed group from its pool and hashes it, so a test can require
# the landed pages to be bit-identical to what the prefill rank gathered
CHECKSUM = os.environ.get("DGI_KV_CHECKSUM") == "1"


def buf_digest(t: torch.Tensor) -> str:
    import hashlib
    return hashlib.sha1(t.detach().contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()
DIAG_S = float(os.environ.get("DGI_KV_DIAG_S", "30"))    # print protocol state every DIAG_S s of a stuck wait


def _diag(msg: str) -> None:
    import sys
    sys.stderr.write(f"[dgi kv {time.strftime('%H:%M:%S')}] {msg}\n")
    sys.stderr.flush()


class _Tx:
    __slots__ = ("tid", "dst", "buf", "event", "key", "group", "ngroups", "c0", "c1", "nblk", "t_rts", "state")

    def __init__(self, tid, dst, buf, event, key, group, ngroups, c0, c1, nblk):
        self.tid, self.dst, self.buf, self.event = tid, dst, buf, event
        self.key, self.group, self.ngroups, self.c0, self.c1, self.nblk = key, group, ngroups, c0, c1, nblk
        self.t_rts = 0.0
        self.state = 0      # 0 gathered, 1 RTS sent, 2 send enqueued


class KVSender:
    """Prefill-rank end: transfers are submitted as gathered buffers and leave
    once their receiver is clear to send."""

    def __init__(self, fabric: Fabric, targets: list):
        self.f = fabric
        self.ch = {x: CtrlChannel(fabric, x, 8, tag=KV_TAG) for x in sorted(set(targets))}
        self.next_tid = 1
        self.gathered: collections.deque = collections.deque()   # waiting for the gather event
        self.await_cts: dict = {}                                   # tid -> _Tx
        self.sent: list = []                                        # (work-tracked in fabric) tx
        self.handshake_us: list = []                                # RTS -> CTS round trips
        self.bytes_sent = 0
        self.transfers = 0
        # DGI_KV_TRACE=1: (event, tid, dst, t) for the protocol-order tests
        self.trace = [] if os.environ.get("DGI_KV_TRACE") == "1" else None
        self.digests: dict = {}         # DGI_KV_CHECKSUM: (dst, key, c0, c1) -> sha1 of the gathered group

    def submit(self, dst: int, buf: torch.Tensor, key: int, group: int, ngroups: int, c0: int, c1: int,
               nblk: int) -> None:
        if CHECKSUM:
            self.digests[(dst, key, c0, c1)] = buf_digest(buf)
        ev = None
        if buf.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.gathered.append(_Tx(self.next_tid, dst, buf, ev, key, group, ngroups, c0, c1, nblk))
        self.next_tid += 1

    def service(self) -> None:
        # RTS for every transfer whose pages are gathered (in submission order)
        while self.gathered:
            tx = self.gathered[0]
            if tx.event is not None and not tx.event.query():
                break
            self.gathered.popleft()
            tx.state = 1
            tx.t_rts = time.perf_counter()
            self.await_cts[tx.tid] = tx
            self.ch[tx.dst].send([RTS, tx.tid, tx.key, tx.group, tx.ngroups, tx.c0, tx.c1, tx.nblk])
            if self.trace is not None:
                self.trace.append(("rts", tx.tid, tx.dst, time.perf_counter()))
        # CTS'd transfers leave as one RCCL group per poll
        go = []
        for x, ch in self.ch.items():
            while True:
                m = ch.poll()
                if m is None:
                    break
                assert m[0] == CTS, m
                tx = self.await_cts.pop(int(m[1]))
                self.handshake_us.append((time.perf_counter() - tx.t_rts) * 1e6)
                tx.state = 2
                go.append(tx)
                if self.trace is not None:
                    self.trace.append(("cts", tx.tid, tx.dst, time.perf_counter()))
        if go:
            if self.trace is not None:
                self.trace += [("send", tx.tid, tx.dst, time.perf_counter()) for tx in go]
            self.f.send_many([(tx.buf, tx.dst) for tx in go], group=self.f.kv_group)
            for tx in go:
                self.bytes_sent += tx.buf.numel() * tx.buf.element_size()
                self.transfers += 1
                tx.buf = None        # the fabric keeps the tensor alive until its send completes

    def pending(self) -> int:
        """Transfers not yet handed to RCCL plus sends still in flight."""
        return len(self.gathered) + len(self.await_cts) + (self.f.sends_in_flight() if self.f.on_gpu else 0)

    def drain(self, timeout_s: float = 600.0, idle=None) -> None:
        """Service until every submitted transfer has completed (phase boundaries,
        shutdown).  Safe: every decode rank keeps servicing its queue meanwhile."""
        t0 = time.perf_counter()
        nxt = t0 + DIAG_S
        while self.gathered or self.await_cts or (self.f.on_gpu and self.f.sends_in_flight()):
            self.service()
            if idle is not None:
                idle()
            if time.perf_counter() > nxt:
                nxt += DIAG_S
                _diag(self.describe())
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"rank {self.f.rank}: KV drain: {len(self.gathered)} gathered, "
                                   f"{len(self.await_cts)} awaiting CTS from "
                                   f"{sorted({t.dst for t in self.await_cts.values()})}, "
                                   f"{self.f.sends_in_flight()} sends in flight")
            time.sleep(0.0002)
        if not self.f.on_gpu:
            self.f.flush()        # gloo: completion is only observed by wait(); every send is CTS'd

    def describe(self) -> str:
        """One line of protocol state (hang diagnostics)."""
        aw = sorted((t.tid, t.dst, round(time.perf_counter() - t.t_rts, 1)) for t in self.await_cts.values())
        return (f"KVSender rank {self.f.rank}: gathered {len(self.gathered)} "
                f"(first event done: {self.gathered[0].event.query() if self.gathered and self.gathered[0].event is not None else None}), "
                f"awaiting CTS (tid, dst, s) {aw[:8]}, sends in flight {self.f.sends_in_flight()}, "
                f"sent {self.transfers}")

    def stats(self) -> dict:
        h = sorted(self.handshake_us)
        return {"transfers": self.transfers, "bytes": self.bytes_sent,
                "cts_rtt_us_p50": round(h[len(h) // 2], 1) if h else None,
                "cts_rtt_us_p95": round(h[int(0.95 * (len(h) - 1))], 1) if h else None}


class KVReceiver:
    """Decode-rank end: one receive in flight at a time, FIFO over every source."""

    def __init__(self, fabric: Fabric, sources: list, page_shape: tuple, dtype: torch.dtype):
        self.f = fabric
        self.ch = {p: CtrlChannel(fabric, p, 8, tag=KV_TAG) for p in sorted(set(sources))}
        self.page_shape = tuple(page_shape)      # (2, nkv, bs, hd): one page of one layer
        self.dtype = dtype
        self.queue: collections.deque = collections.deque()      # (src, rts fields)
        self.cur = None                                           # (src, fields, AsyncRecv, buf)
        self.landed: dict = collections.defaultdict(list)         # (src, key) -> [(c0, c1, buf)]
        self.expected: dict = {}                                  # (src, key) -> ngroups
        self.received = 0
        self.recv_bytes = 0
        self.wait_us: list = []                                   # post -> landed per transfer
        self.trace = [] if os.environ.get("DGI_KV_TRACE") == "1" else None
        self.digests = {} if CHECKSUM else None                   # (src, key, c0, c1) -> sha1 of installed pages

    def service(self) -> int:
        """Take in RTS messages, retire the receive in flight, post the next one.
        Returns the number of transfers that landed."""
        for p, ch in self.ch.items():
            while True:
                m = ch.poll()
                if m is None:
                    break
                assert m[0] == RTS, m
                self.queue.append((p, [int(x) for x in m[1:8]]))
        n = 0
        while True:
            if self.cur is not None:
                src, fl, rec, buf = self.cur
                if not rec.ready():
                    break
                rec.complete()
                self.wait_us.append((time.perf_counter() - rec.t_post) * 1e6)
                tid, key, group, ng, c0, c1, nblk = fl
                self.landed[(src, key)].append((c0, c1, buf))
                self.expected[(src, key)] = ng
                self.received += 1
                self.recv_bytes += buf.numel() * buf.element_size()
                self.cur = None
                n += 1
                if self.trace is not None:
                    self.trace.append(("land", tid, src, time.perf_counter()))
            if not self.queue:
                break
            src, fl = self.queue.popleft()
            tid, key, group, ng, c0, c1, nblk = fl
            nkv_2 = self.page_shape
            buf = self.f.alloc_recv((c1 - c0, nkv_2[0], nblk) + nkv_2[1:], self.dtype)
            rec = self.f.irecv_async(buf, src, group=self.f.kv_group)
            self.cur = (src, fl, rec, buf)
            if self.trace is not None:
                self.trace.append(("post", tid, src, time.perf_counter()))
            self.ch[src].send([CTS, tid])
        return n

    def is_landed(self, src: int, key: int) -> bool:
        ng = self.expected.get((src, key))
        return ng is not None and len(self.landed[(src, key)]) == ng

    def take(self, src: int, key: int) -> list:
        self.expected.pop((src, key), None)
        return self.landed.pop((src, key), [])

    def wait_landed(self, src: int, key: int, timeout_s: float = 600.0, idle=None) -> list:
        t0 = time.perf_counter()
        nxt = t0 + DIAG_S
        while not self.is_landed(src, key):
            if time.perf_counter() > nxt:
                nxt += DIAG_S
                _diag(f"waiting for migration {key} from {src}: " + self.describe())
            if not self.service():
                if idle is not None:
                    idle()
                if time.perf_counter() - t0 > timeout_s:
                    raise TimeoutError(f"rank {self.f.rank}: KV of migration {key} from rank {src} "
                                       f"not landed in {timeout_s}s (queue {len(self.queue)})")
                time.sleep(0.0001)
        return self.take(src, key)

    def busy(self) -> bool:
        return self.cur is not None or bool(self.queue)

    def describe(self) -> str:
        cur = None
        if self.cur is not None:
            src, fl, rec, _buf = self.cur
            cur = (src, fl[0], round(time.perf_counter() - rec.t_post, 1), rec.work.is_completed() if self.f.on_gpu else None)
        return (f"KVReceiver rank {self.f.rank}: in flight (src, tid, s, done) {cur}, queued "
                f"{[(p, fl[0]) for p, fl in list(self.queue)[:8]]}, landed {self.received}")

    def stats(self) -> dict:
        w = sorted(self.wait_us)
        return {"received": self.received, "bytes": self.recv_bytes,
                "post_to_land_us_p50": round(w[len(w) // 2], 1) if w else None}


def scatter_groups(pool_kv: torch.Tensor, ids_t: torch.Tensor, groups: list, digests: Optional[dict] = None,
                   src: int = -1, key: int = -1) -> None:
    """Install landed layer groups [(c0, c1, buf)] into the paged pool (current stream).
    With ``digests`` (DGI_KV_CHECKSUM), each installed group is gathered back out of the
    pool and hashed under (src, key, c0, c1)."""
    from dgi import ops
    for c0, c1, buf in groups:
        ops.kv_scatter(pool_kv[c0:c1], ids_t, buf)
        if digests is not None:
            digests[(src, key, c0, c1)] = buf_digest(ops.kv_gather(pool_kv[c0:c1], ids_t))
