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
    event complete  --RTS(tid, group, shape)------->  queue (FIFO per source)
                                                      when X has NO batch in flight:
                                                        post ONE batch: the oldest queued
                                                        RTS of each source, as one RCCL
                                                        group (own stream, waits on nothing)
                    <-------------------CTS(tid)---   (one CTS per receive of the batch)
    enqueue the send (batched with the other
    CTS'd sends of this poll: one RCCL group)
                                                      poll: batch landed -> scatter into the pool

A batch holds at most one receive per source (``DGI_KV_RECV_BATCH`` caps its
size; 1 = round 3's single receive in flight), so a decode rank pulls from up
to P prefill ranks at once, each over its own xGMI link (round 3: one receive
at a time per decode rank).

Why it cannot deadlock (on the KV communicator's FIFO stream of every rank):
  (1) a decode rank has at most ONE batch posted, and posts it from an empty
      stream as one RCCL group, so every receive of the batch is running (a
      group's point-to-point operations progress independently of each other)
      from the moment it is posted (communicators live on their own
      high-priority hardware queues, dgi.parallel.fabric);
  (2) a prefill rank enqueues a send only after its receiver's CTS, i.e. the
      partner of EVERY send in a prefill rank's stream is a running receive;
  (3) so the head of each prefill stream completes as soon as its own compute
      (the gather) is done, and by induction every send and every batch
      completes.  (Two SEPARATELY posted receives on one stream would break
      (1): the second would wait behind the first while its sender's stream
      waits on it — the cycle the single group avoids.)
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
# receives per posted batch (at most one per source); 0 = one per source
RECV_BATCH = int(os.environ.get("DGI_KV_RECV_BATCH", "0"))


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
    """Decode-rank end: one batch of receives in flight (at most one per source),
    each source's transfers in FIFO order."""

    def __init__(self, fabric: Fabric, sources: list, page_shape: tuple, dtype: torch.dtype,
                 max_batch: Optional[int] = None):
        self.f = fabric
        self.ch = {p: CtrlChannel(fabric, p, 8, tag=KV_TAG) for p in sorted(set(sources))}
        self.page_shape = tuple(page_shape)      # (2, nkv, bs, hd): one page of one layer
        self.dtype = dtype
        self.queue: dict = {p: collections.deque() for p in self.ch}   # src -> RTS fields, FIFO
        mb = RECV_BATCH if max_batch is None else max_batch
        self.max_batch = max(1, mb) if mb else len(self.ch)
        self.cur: list = []                                       # the batch in flight: (src, fields, AsyncRecv, buf)
        self.batches = 0
        self.landed: dict = collections.defaultdict(list)         # (src, key) -> [(c0, c1, buf)]
        self.expected: dict = {}                                  # (src, key) -> ngroups
        self.received = 0
        self.recv_bytes = 0
        self.wait_us: list = []                                   # post -> landed per transfer
        self.batch_sizes: list = []
        self.trace = [] if os.environ.get("DGI_KV_TRACE") == "1" else None
        self.digests = {} if CHECKSUM else None                   # (src, key, c0, c1) -> sha1 of installed pages
        self._rr = 0                                              # round-robin start over sources

    def _queued(self) -> int:
        return sum(len(q) for q in self.queue.values())

    def service(self) -> int:
        """Take in RTS messages, retire the batch in flight once all of it has landed,
        post the next batch.  Returns the number of transfers that landed."""
        for p, ch in self.ch.items():
            while True:
                m = ch.poll()
                if m is None:
                    break
                assert m[0] == RTS, m
                self.queue[p].append([int(x) for x in m[1:8]])
        n = 0
        while True:
            if self.cur:
                if not all(rec.ready() for _s, _f, rec, _b in self.cur):
                    break
                for src, fl, rec, buf in self.cur:
                    rec.complete()
                    self.wait_us.append((time.perf_counter() - rec.t_post) * 1e6)
                    tid, key, group, ng, c0, c1, nblk = fl
                    self.landed[(src, key)].append((c0, c1, buf))
                    self.expected[(src, key)] = ng
                    self.received += 1
                    self.recv_bytes += buf.numel() * buf.element_size()
                    n += 1
                    if self.trace is not None:
                        self.trace.append(("land", tid, src, time.perf_counter(), self.batches))
                self.cur = []
            srcs = [p for p in self.queue if self.queue[p]]
            if not srcs:
                break
            # the oldest RTS of up to max_batch sources, rotating the start so no source waits
            k = self._rr % len(srcs)
            pick = (srcs[k:] + srcs[:k])[: self.max_batch]
            self._rr += 1
            items = []
            for src in pick:
                fl = self.queue[src].popleft()
                tid, key, group, ng, c0, c1, nblk = fl
                nkv_2 = self.page_shape
                items.append((src, fl, self.f.alloc_recv((c1 - c0, nkv_2[0], nblk) + nkv_2[1:], self.dtype)))
            recs = self.f.irecv_batch([(buf, src) for src, _fl, buf in items], group=self.f.kv_group)
            self.batches += 1
            self.batch_sizes.append(len(items))
            self.cur = [(src, fl, rec, buf) for (src, fl, buf), rec in zip(items, recs)]
            for src, fl, _buf in items:
                if self.trace is not None:
                    self.trace.append(("post", fl[0], src, time.perf_counter(), self.batches))
                self.ch[src].send([CTS, fl[0]])
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
                                       f"not landed in {timeout_s}s (queue {self._queued()})")
                time.sleep(0.0001)
        return self.take(src, key)

    def busy(self) -> bool:
        return bool(self.cur) or self._queued() > 0

    def describe(self) -> str:
        cur = [(src, fl[0], round(time.perf_counter() - rec.t_post, 1),
                rec.work.is_completed() if self.f.on_gpu else None) for src, fl, rec, _buf in self.cur]
        q = [(p, fl[0]) for p, dq in self.queue.items() for fl in list(dq)[:2]]
        return (f"KVReceiver rank {self.f.rank}: batch in flight (src, tid, s, done) {cur}, queued "
                f"{q[:8]}, landed {self.received}")

    def stats(self) -> dict:
        w = sorted(self.wait_us)
        b = self.batch_sizes
        return {"received": self.received, "bytes": self.recv_bytes,
                "post_to_land_us_p50": round(w[len(w) // 2], 1) if w else None,
                "batches": self.batches, "mean_batch": round(sum(b) / len(b), 2) if b else None,
                "max_batch": self.max_batch}


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
