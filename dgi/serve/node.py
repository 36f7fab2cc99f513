"""Node server: the in-node serving runtime behind one HTTP endpoint.

One process per GPU (launch with ``torch.distributed.run``; a single process
serves on one GPU).  The layout is the benchmark's (``dgi.parallel.plan``):

* ``single`` — one engine;
* ``pd`` / ``pdpp`` — prefill ranks + a decode GPU or decode layer pipeline.

The *router* lives on the first decode replica's driver: an HTTP front-end
(FastAPI/uvicorn thread) queues requests; the router loop places each prompt
on a prefill rank with a node-local ``PrefillDecodeScheduler`` (the
reference's P/D scheduler API, server/app/services/pd_scheduler.py) over a
control channel (the rendezvous store), steps its own decode replica, and
resolves HTTP futures as tokens arrive — its own, and those the other decode
replicas forward to it.  The first token is sampled on the prefill rank and
arrives with the migrated KV, so TTFT is measured at that arrival.  The
prefill ranks pick the decode replica of each request (pd.PrefillServer).

This replaces the reference's per-request HTTP/gRPC hops between shard
workers (worker/distributed/session.py:49-455, grpc_server.py:351-388) for
the in-node case; the worker daemon talks to it through ``NodeLLMEngine``.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m dgi.serve.node --model llama3-70b --port 8100
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import json
import os
import queue
import threading
import time
from typing import Optional

import numpy as np
import torch

from dgi.sched.request import SamplingParams

STOP_RID = -1
REQ_HDR = 8   # rid, n_tokens, max_tokens, temp_bits, top_p_bits, top_k, seed, ignore_eos


def _f2i(x: float) -> int:
    return int(np.float32(x).view(np.int32))


def _i2f(x: int) -> float:
    return float(np.int32(x).view(np.float32))


def encode_request(rid: int, prompt: list, sp: SamplingParams) -> np.ndarray:
    hdr = [rid, len(prompt), sp.max_tokens, _f2i(sp.temperature), _f2i(sp.top_p), sp.top_k,
           -1 if sp.seed is None else int(sp.seed) & 0x7FFFFFFF, int(sp.ignore_eos)]
    return np.asarray(hdr + list(prompt), np.int64)


def decode_request(msg: np.ndarray):
    rid, n, mt, tb, pb, tk, seed, ign = (int(x) for x in msg[:REQ_HDR])
    sp = SamplingParams(max_tokens=mt, temperature=_i2f(tb), top_p=_i2f(pb), top_k=tk,
                        seed=None if seed < 0 else seed, ignore_eos=bool(ign))
    return rid, [int(x) for x in msg[REQ_HDR: REQ_HDR + n]], sp


class _Pending:
    __slots__ = ("rid", "prompt", "params", "tokens", "future", "loop", "stream", "t0", "ttft", "done", "dst")

    def __init__(self, rid, prompt, params, loop, stream):
        self.rid, self.prompt, self.params = rid, prompt, params
        self.tokens: list = []
        self.future = loop.create_future()
        self.loop = loop
        self.stream: Optional[asyncio.Queue] = asyncio.Queue() if stream else None
        self.t0 = time.perf_counter()
        self.ttft: Optional[float] = None
        self.done = False
        self.dst = -1


class Router:
    """Runs on the decode driver (or the only rank): HTTP in, tokens out."""

    def __init__(self, args, fabric=None, layout=None):
        from dgi.engine import EngineConfig
        from dgi.utils.tokenizer import load_tokenizer
        from dgi.models.config import get_config
        self.args = args
        self.f = fabric
        self.layout = layout
        self.inbox: "queue.Queue[_Pending]" = queue.Queue()
        self.live: dict = {}
        self.next_rid = 1
        self.stats = collections.Counter()
        mc = get_config(args.model)
        self.tok = load_tokenizer(args.tokenizer or args.model, vocab_size=mc.vocab_size, bos=mc.bos_token_id,
                                  eos=mc.eos_token_id)
        dev = str(fabric.device) if fabric is not None else ("cuda" if torch.cuda.is_available() else "cpu")
        cfg = EngineConfig(model=args.model, device=dev, max_num_seqs=args.max_num_seqs,
                           max_num_batched_tokens=args.max_batched_tokens, max_model_len=args.max_model_len,
                           use_graphs=dev.startswith("cuda") and not args.no_graphs, seed=args.seed)
        self.drv = None
        self.chans = {}
        self.load = collections.Counter()
        if layout is None or layout.kind == "single":
            from dgi.engine import LLMEngine
            self.engine = LLMEngine(cfg)
            self.engine.warmup()
        else:
            from dgi.parallel.fabric import CtrlChannel
            from dgi.parallel.pd import MI355X_TFLOPS, DecodeDriver, pd_scheduler_module
            self.drv = DecodeDriver(cfg, fabric, layout)
            self.drv.track_arrivals = True
            self.engine = self.drv.engine
            self.chans = {p: CtrlChannel(fabric, p, 1, tag="req") for p in layout.prefill_ranks}
            # node-local P/D scheduler: prefill placement (flops / (1 + active prefill jobs))
            m = pd_scheduler_module()
            self._pdm = m
            self.pd = m.PrefillDecodeScheduler()
            for p in layout.prefill_ranks:
                self.pd.register_worker(str(p), m.WorkerCapability(str(p), m.WorkerRole.PREFILL,
                                                                   compute_flops=MI355X_TFLOPS))
        self.ready = threading.Event()

    # ------------------------------------------------------------------ request intake (HTTP thread)
    def submit(self, prompt: list, params: SamplingParams, loop, stream: bool = False) -> _Pending:
        p = _Pending(0, prompt, params, loop, stream)
        self.inbox.put(p)
        return p

    def _emit(self, p: _Pending, tok: int, finished: bool, reason: Optional[str]) -> None:
        if p.ttft is None:
            p.ttft = time.perf_counter() - p.t0
        p.tokens.append(tok)

        def deliver():
            if p.stream is not None:
                p.stream.put_nowait(("token", tok))
            if finished and not p.future.done():
                if p.stream is not None:
                    p.stream.put_nowait(("done", reason))
                p.future.set_result(reason)
        p.loop.call_soon_threadsafe(deliver)

    # ------------------------------------------------------------------ engine loop (main thread)
    def _dispatch(self) -> None:
        while True:
            try:
                p = self.inbox.get_nowait()
            except queue.Empty:
                return
            p.rid = self.next_rid
            self.next_rid += 1
            self.live[p.rid] = p
            self.stats["requests"] += 1
            if self.drv is None:
                self.engine.add_request(p.prompt, p.params, rid=p.rid)
            else:
                from dgi.parallel.pd import run_sync
                m = self._pdm
                run_sync(self.pd.submit_job(str(p.rid), len(p.prompt), p.params.max_tokens))
                for job, a in run_sync(self.pd.get_batch(m.JobPhase.PREFILL, 64)):
                    q = self.live.get(int(job.job_id))
                    if q is None:
                        continue
                    dst = int(a.worker_id)
                    self.load[dst] += 1
                    q.dst = dst
                    self.chans[dst].send_var(encode_request(q.rid, q.prompt, q.params))

    def _prefill_done(self, p: "_Pending") -> None:
        """First token arrived: the prompt's prefill job is complete."""
        if self.drv is not None and p.dst >= 0:
            from dgi.parallel.pd import run_sync
            self.load[p.dst] -= 1
            run_sync(self.pd.complete_job(str(p.rid), self._pdm.JobPhase.PREFILL,
                                          (time.perf_counter() - p.t0) * 1000.0))
            p.dst = -1

    def _finish(self, rid: int, reason: Optional[str]) -> None:
        p = self.live.pop(rid, None)
        if p is not None:
            p.done = True
            self.stats["finished"] += 1

    def step(self) -> bool:
        self._dispatch()
        worked = False
        if self.drv is not None:
            self.drv.poll()
            for r in self.drv.arrivals:            # first token, sampled on the prefill rank
                p = self.live.get(r.user)
                if p is not None:
                    self._prefill_done(p)
                    self._emit(p, r.output[0], False, None)
            self.drv.arrivals.clear()
            outs = self.drv.step(poll=False)
        else:
            outs = self.engine.step() if self.engine.has_unfinished() else []
        for o in outs:
            worked = True
            key = o.request.user if self.drv is not None else o.rid
            p = self.live.get(key)
            if p is None:
                continue
            self._emit(p, o.token, o.finished, o.finish_reason)
            if o.finished:
                self._finish(key, o.finish_reason)
        if self.drv is not None:
            for rid, tok, reason in self.drv.prefill_finished:   # done at the first token
                p = self.live.get(rid)
                if p is not None:
                    self._prefill_done(p)
                    self._emit(p, tok, True, reason)
                    self._finish(rid, reason)
            self.drv.prefill_finished.clear()
            # decoded on a prefill rank (overflow) or on another decode replica
            for rid, tok, reason in self.drv.remote_tokens:
                p = self.live.get(rid)
                if p is None:
                    continue
                worked = True
                if not p.tokens:
                    self._prefill_done(p)
                self._emit(p, tok, reason is not None, reason)
                if reason is not None:
                    self._finish(rid, reason)
            self.drv.remote_tokens.clear()
        return worked

    def serve_forever(self, stop: threading.Event) -> None:
        self.ready.set()
        while not stop.is_set():
            if not self.step() and not self.live:
                time.sleep(0.001)
        if self.drv is not None:
            for ch in self.chans.values():
                ch.send_var([STOP_RID])
            while not self.drv.all_prefill_done():
                self.drv.poll()
                time.sleep(0.002)
            self.drv.finish()


try:
    from pydantic import BaseModel

    class GenReq(BaseModel):
        prompt: Optional[str] = None
        prompt_ids: Optional[list] = None
        messages: Optional[list] = None
        max_tokens: int = 128
        temperature: float = 0.0
        top_p: float = 1.0
        top_k: int = 0
        seed: Optional[int] = None
        ignore_eos: bool = False
        stream: bool = False
except Exception:  # pragma: no cover - pydantic ships with fastapi
    GenReq = None


def build_app(router: Router, stop: threading.Event):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import StreamingResponse

    app = FastAPI(title="dgi node")
    tok = router.tok

    def ids_of(r: GenReq) -> list:
        if r.prompt_ids:
            return [int(x) for x in r.prompt_ids]
        if r.messages:
            from dgi.utils.tokenizer import chat_prompt_ids
            return chat_prompt_ids(tok, r.messages)
        if r.prompt is not None:
            return tok.encode(r.prompt)
        raise HTTPException(400, "prompt, prompt_ids or messages required")

    @app.get("/health")
    async def health():
        return {"status": "ok" if router.ready.is_set() else "starting",
                "layout": router.layout.kind if router.layout else "single"}

    @app.get("/stats")
    async def stats():
        out = {"requests": router.stats["requests"], "finished": router.stats["finished"],
               "live": len(router.live), "engine": dict(router.engine.stats),
               "scheduler": router.engine.scheduler.stats()}
        if router.drv is not None:
            out["pd_scheduler"] = router.pd.get_stats()
            out["layout"] = router.layout.describe()
        return out

    @app.post("/generate")
    async def generate(r: GenReq):
        ids = ids_of(r)
        sp = SamplingParams(max_tokens=r.max_tokens, temperature=r.temperature, top_p=r.top_p, top_k=r.top_k,
                            seed=r.seed, ignore_eos=r.ignore_eos)
        p = router.submit(ids, sp, asyncio.get_running_loop(), stream=r.stream)
        if r.stream:
            async def events():
                from dgi.utils.tokenizer import StreamDecoder
                dec = StreamDecoder(tok)        # text pieces concatenate to the full decode
                while True:
                    kind, v = await p.stream.get()
                    if kind == "token":
                        yield f"data: {json.dumps({'token_id': v, 'text': dec.add(v)})}\n\n"
                    else:
                        tail = dec.flush()
                        yield f"data: {json.dumps({'done': True, 'finish_reason': v, 'text': tail})}\n\n"
                        return
            return StreamingResponse(events(), media_type="text/event-stream")
        reason = await p.future
        return {"token_ids": p.tokens, "text": tok.decode(p.tokens), "finish_reason": reason,
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(p.tokens),
                          "total_tokens": len(ids) + len(p.tokens)},
                "ttft_ms": None if p.ttft is None else round(p.ttft * 1000, 2)}

    @app.post("/shutdown")
    async def shutdown():
        stop.set()
        return {"status": "stopping"}

    return app


def _prefill_loop(args, fabric, layout) -> None:
    from dgi.engine import EngineConfig
    from dgi.parallel.fabric import CtrlChannel
    from dgi.parallel.pd import PrefillServer
    from dgi.parallel.plan import prefill_overflow_cap
    cap = args.prefill_local_cap if args.prefill_local_cap >= 0 else prefill_overflow_cap(layout)
    cfg = EngineConfig(model=args.model, device=str(fabric.device), max_num_seqs=64 + cap,
                       max_num_batched_tokens=args.max_batched_tokens, max_model_len=args.max_model_len,
                       use_graphs=str(fabric.device).startswith("cuda") and not args.no_graphs, seed=args.seed)
    srv = PrefillServer(cfg, fabric, layout, local_cap=cap, report_tokens=True)
    inbox = CtrlChannel(fabric, layout.drivers[0], 1, tag="req")
    stopping = False
    while True:
        while True:
            m = inbox.poll()
            if m is None:
                break
            rid, prompt, sp = decode_request(m) if m[0] != STOP_RID else (STOP_RID, None, None)
            if rid == STOP_RID:
                stopping = True
                break
            srv.submit(prompt, sp, rid=rid)
        if srv.busy():
            srv.step()
        elif stopping:
            break
        else:
            time.sleep(0.001)
    srv.finish()


def _replica_loop(args, fabric, layout) -> None:
    """Driver of a decode replica other than the router's: serve migrations,
    forward every token to the router, stop once all prefill ranks are done."""
    from dgi.engine import EngineConfig
    from dgi.parallel.pd import DecodeDriver
    cfg = EngineConfig(model=args.model, device=str(fabric.device), max_num_seqs=args.max_num_seqs,
                       max_num_batched_tokens=args.max_batched_tokens, max_model_len=args.max_model_len,
                       use_graphs=str(fabric.device).startswith("cuda") and not args.no_graphs, seed=args.seed)
    drv = DecodeDriver(cfg, fabric, layout)
    drv.track_arrivals = True
    drv.forward_tokens = True
    while True:
        drv.poll()
        if drv.engine.has_unfinished() or drv.arrivals:
            drv.step(poll=False)
        elif drv.all_prefill_done():
            break
        else:
            time.sleep(0.001)
    drv.finish()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--layout", default="auto")
    ap.add_argument("--prefill-ranks", type=int, default=0)
    ap.add_argument("--decode-stages", type=int, default=0)
    ap.add_argument("--decode-replicas", type=int, default=0)
    ap.add_argument("--prefill-local-cap", type=int, default=-1,
                    help="sequences a prefill rank decodes itself when the decode side is full (-1 = auto)")
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=4096)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    fabric = layout = None
    if world > 1:
        from dgi.parallel.fabric import Fabric
        from dgi.parallel.plan import plan_node_layout
        fabric = Fabric()
        layout = plan_node_layout(world, "pdpp" if args.layout == "auto" else args.layout,
                                  args.prefill_ranks or None, decode_stages=args.decode_stages or None,
                                  decode_replicas=args.decode_replicas or None, model=args.model)
        fabric.setup_layout(layout)
        role = layout.role(fabric.rank)
        if role == "prefill":
            _prefill_loop(args, fabric, layout)
            fabric.close()
            return 0
        if role == "decode_driver" and fabric.rank != layout.drivers[0]:
            _replica_loop(args, fabric, layout)
            fabric.close()
            return 0
        if role == "decode_stage":
            from dgi.engine import EngineConfig
            from dgi.parallel.pipeline import StageWorker
            cfg = EngineConfig(model=args.model, device=str(fabric.device), max_num_seqs=args.max_num_seqs,
                               max_num_batched_tokens=args.max_batched_tokens, max_model_len=args.max_model_len,
                               use_graphs=str(fabric.device).startswith("cuda") and not args.no_graphs,
                               seed=args.seed, enable_prefix_caching=False)
            w = StageWorker(cfg, fabric, layout.group_of(fabric.rank), kv_sources=layout.prefill_ranks)
            while w.run() != "stop":
                pass
            fabric.close()
            return 0
    router = Router(args, fabric, layout)
    stop = threading.Event()
    app = build_app(router, stop)
    import uvicorn
    server = uvicorn.Server(uvicorn.Config(app, host=args.host, port=args.port, log_level="warning"))
    th = threading.Thread(target=server.run, name="http", daemon=True)
    th.start()
    try:
        router.serve_forever(stop)
    finally:
        server.should_exit = True
        th.join(10)
        if fabric is not None:
            fabric.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
