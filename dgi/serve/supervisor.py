"""Elastic node supervisor: launch the ranks, watch them, re-plan on failure,
resume in-flight requests by re-prefill.

The ranks of a node (``dgi.serve.node``, one process per GPU) fail as a
unit: an RCCL communicator cannot lose a member, and the rank watchdog
(``dgi.parallel.fault``) turns one rank's death into every rank exiting.
The supervisor stays outside that blast radius:

* it starts the ranks itself (``RANK`` / ``WORLD_SIZE`` / ``LOCAL_RANK``, a
  fresh rendezvous port per generation, ``HIP_VISIBLE_DEVICES`` restricted to
  the GPUs still trusted), so a restart is a local decision;
* it is the public HTTP endpoint — the node's ``/generate`` / ``/health`` /
  ``/stats`` / ``/shutdown`` surface — and journals every request: prompt
  ids, sampling parameters, tokens delivered so far;
* when a generation dies it blames the first rank that exited abnormally
  (the watchdog's follow-on exits, status 3, only when nothing else is
  there), stops the other ranks, drops the blamed GPU, re-plans the layout
  for the survivors (``dgi.parallel.plan`` runs inside the new ranks) and
  starts the next generation;
* every unfinished request is re-submitted as ``prompt + delivered tokens``
  with the remaining budget, so its KV is rebuilt by re-prefill from token
  history — the Petals-style recovery the reference planned
  (REFACTORING_PLAN.md:323-342) while its session code raised instead
  (worker/distributed/session.py:339-365).  A greedy request resumes on the
  same trajectory and the client sees one uninterrupted stream.

    python -m dgi.serve.supervisor --nproc 8 --port 8100 -- --model llama3-70b
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Optional

import httpx

from dgi.serve.node import GenReq

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
WATCHDOG_EXIT = 3


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def blame(codes: dict) -> Optional[int]:
    """Rank to drop, from ``{rank: exit status}`` of the ranks seen exited (in
    the order they were seen): the first abnormal status that is not the
    watchdog's follow-on abort, else the first abnormal one."""
    bad = [(r, c) for r, c in codes.items() if c not in (0, None)]
    for r, c in bad:
        if c != WATCHDOG_EXIT:
            return r
    return bad[0][0] if bad else None


class _Job:
    __slots__ = ("prompt", "params", "tokens", "done", "reason", "events", "t0", "ttft", "resumes")

    def __init__(self, prompt: list, params: dict):
        self.prompt = list(prompt)
        self.params = dict(params)
        self.tokens: list = []
        self.done = asyncio.Event()
        self.reason: Optional[str] = None
        self.events: asyncio.Queue = asyncio.Queue()
        self.t0 = time.perf_counter()
        self.ttft: Optional[float] = None
        self.resumes = 0


class NodeSupervisor:
    """Owns the node's rank processes across failures."""

    def __init__(self, node_args: list, nproc: int = 1, gpus: Optional[list] = None, max_restarts: int = 3,
                 first_env: Optional[dict] = None, env: Optional[dict] = None, startup_timeout: float = 1800.0,
                 log_dir: Optional[str] = None):
        self.node_args = list(node_args)
        self.alive = list(gpus) if gpus else list(range(nproc))
        self.pin_devices = bool(gpus)
        self.max_restarts = max_restarts
        self.first_env = dict(first_env or {})    # generation 1 only (e.g. DGI_FAULT)
        self.env = dict(env or {})
        self.startup_timeout = startup_timeout
        self.log_dir = log_dir
        self.procs: list = []
        self.gen = 0
        self.ready_gen = 0          # generation whose router answers /health (0 = none)
        self.url: Optional[str] = None
        self.restarts = 0
        self.failures: list = []
        self.resumed = 0
        self.stopping = False
        self.dead = False           # no GPU left or restart budget spent
        self._mon: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ rank processes
    def _spawn(self) -> None:
        self.gen += 1
        world = len(self.alive)
        mport, iport = _free_port(), _free_port()
        base = dict(os.environ)
        for k in self.first_env:
            base.pop(k, None)
        base.update(self.env)
        if self.gen == 1:
            base.update(self.first_env)
        base["PYTHONPATH"] = ROOT + os.pathsep + base.get("PYTHONPATH", "")
        base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.pin_devices:
            base["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in self.alive)
        procs = []
        for r in range(world):
            e = dict(base, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                     MASTER_ADDR="127.0.0.1", MASTER_PORT=str(mport))
            out = None
            if self.log_dir:
                os.makedirs(self.log_dir, exist_ok=True)
                out = open(os.path.join(self.log_dir, f"gen{self.gen}_rank{r}.log"), "w")
            # own session per rank: a failure kill reaches exactly this rank's process group
            procs.append(subprocess.Popen([sys.executable, "-m", "dgi.serve.node", *self.node_args,
                                           "--port", str(iport)], cwd=ROOT, env=e, stdout=out,
                                          stderr=subprocess.STDOUT if out else None, start_new_session=True))
            if out is not None:
                out.close()
        self.procs = procs
        self.url = f"http://127.0.0.1:{iport}"

    def _wait_ready(self) -> None:
        deadline = time.time() + self.startup_timeout
        while time.time() < deadline:
            if any(p.poll() is not None for p in self.procs):
                raise RuntimeError("a rank exited during startup")
            try:
                if httpx.get(self.url + "/health", timeout=2).json().get("status") == "ok":
                    self.ready_gen = self.gen
                    return
            except (httpx.HTTPError, ValueError):
                pass
            time.sleep(0.2)
        raise TimeoutError(f"generation {self.gen} did not become healthy")

    def _kill_all(self) -> None:
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        for p in self.procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                pass

    def _exited(self) -> dict:
        return {r: p.poll() for r, p in enumerate(self.procs) if p.poll() is not None}

    def _fail(self, codes: dict) -> None:
        """One generation is gone: blame, stop the rest, drop the blamed GPU."""
        self.ready_gen = 0
        time.sleep(0.3)          # let a failing rank's own exit status land before the others are killed
        codes = {**codes, **self._exited()}
        r = blame(codes)
        self._kill_all()
        gpu = self.alive[r] if r is not None and r < len(self.alive) else None
        self.failures.append({"generation": self.gen, "rank": r, "gpu": gpu,
                              "status": None if r is None else codes.get(r), "world": len(self.alive)})
        if r is not None:
            self.alive.pop(r)

    def _restart(self) -> None:
        while not self.stopping:
            if self.restarts >= self.max_restarts or not self.alive:
                self.dead = True
                return
            self.restarts += 1
            self._spawn()
            try:
                self._wait_ready()
                return
            except (RuntimeError, TimeoutError):
                self._fail(self._exited())

    def _monitor(self) -> None:
        while not self.stopping:
            codes = self._exited()
            if not codes:
                time.sleep(0.1)
                continue
            if self.stopping:
                return
            self._fail(codes)
            self._restart()
            if self.dead:
                return

    def start(self) -> "NodeSupervisor":
        self._spawn()
        self._wait_ready()
        self._mon = threading.Thread(target=self._monitor, name="dgi-supervisor", daemon=True)
        self._mon.start()
        return self

    def stop(self) -> None:
        self.stopping = True
        if self.url and self.ready_gen:
            try:
                httpx.post(self.url + "/shutdown", timeout=10)
            except httpx.HTTPError:
                pass
        deadline = time.time() + 120
        while time.time() < deadline and any(p.poll() is None for p in self.procs):
            time.sleep(0.2)
        self._kill_all()

    # ------------------------------------------------------------------ requests
    async def run_job(self, job: _Job) -> None:
        """Drive one request through the live generation; when the generation
        dies mid-stream, wait for the next one and resume from token history."""
        while True:
            if self.dead:
                self._finish(job, "error")
                return
            gen = self.ready_gen
            if gen == 0:
                await asyncio.sleep(0.05)
                continue
            remaining = int(job.params.get("max_tokens", 128)) - len(job.tokens)
            if remaining <= 0:
                self._finish(job, "length")
                return
            body = dict(job.params, prompt_ids=job.prompt + job.tokens, max_tokens=remaining, stream=True)
            try:
                async with httpx.AsyncClient(timeout=None) as c:
                    async with c.stream("POST", self.url + "/generate", json=body) as resp:
                        resp.raise_for_status()
                        async for line in resp.aiter_lines():
                            if not line.startswith("data: "):
                                continue
                            ev = json.loads(line[6:])
                            if ev.get("done"):
                                self._finish(job, ev.get("finish_reason"))
                                return
                            if job.ttft is None:
                                job.ttft = time.perf_counter() - job.t0
                            job.tokens.append(int(ev["token_id"]))
                            job.events.put_nowait(("token", int(ev["token_id"])))
            except (httpx.HTTPError, OSError, ValueError):
                pass
            # the stream ended without "done": the generation is failing
            job.resumes += 1
            self.resumed += 1
            t0 = time.time()
            while self.ready_gen == gen and not self.dead and time.time() - t0 < 5.0:
                await asyncio.sleep(0.05)

    @staticmethod
    def _finish(job: _Job, reason: Optional[str]) -> None:
        job.reason = reason
        job.events.put_nowait(("done", reason))
        job.done.set()


def build_app(sup: NodeSupervisor, tok, on_shutdown=None):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import StreamingResponse

    app = FastAPI(title="dgi elastic node")

    def ids_of(r) -> list:
        if r.prompt_ids:
            return [int(x) for x in r.prompt_ids]
        if r.messages:
            from dgi.utils.tokenizer import chat_prompt_ids
            return chat_prompt_ids(tok, r.messages)
        if r.prompt is not None:
            return tok.encode(r.prompt)
        raise HTTPException(400, "prompt, prompt_ids or messages required")

    def status() -> str:
        return "dead" if sup.dead else ("ok" if sup.ready_gen else "recovering")

    @app.get("/health")
    async def health():
        return {"status": status(), "generation": sup.gen, "gpus": list(sup.alive), "restarts": sup.restarts}

    @app.get("/stats")
    async def stats():
        out = {"supervisor": {"generation": sup.gen, "gpus": list(sup.alive), "restarts": sup.restarts,
                              "failures": sup.failures, "resumed_streams": sup.resumed, "status": status()}}
        if sup.ready_gen:
            try:
                async with httpx.AsyncClient(timeout=10) as c:
                    out.update((await c.get(sup.url + "/stats")).json())
            except (httpx.HTTPError, ValueError):
                pass
        return out

    @app.post("/generate")
    async def generate(r: GenReq):
        ids = ids_of(r)
        params = {"max_tokens": r.max_tokens, "temperature": r.temperature, "top_p": r.top_p, "top_k": r.top_k,
                  "seed": r.seed, "ignore_eos": r.ignore_eos}
        job = _Job(ids, params)
        asyncio.create_task(sup.run_job(job))
        if r.stream:
            async def events():
                from dgi.utils.tokenizer import StreamDecoder
                dec = StreamDecoder(tok)        # text pieces concatenate to the full decode
                while True:
                    kind, v = await job.events.get()
                    if kind == "token":
                        yield f"data: {json.dumps({'token_id': v, 'text': dec.add(v)})}\n\n"
                    else:
                        tail = dec.flush()
                        yield f"data: {json.dumps({'done': True, 'finish_reason': v, 'text': tail})}\n\n"
                        return
            return StreamingResponse(events(), media_type="text/event-stream")
        await job.done.wait()
        if job.reason == "error":
            raise HTTPException(503, "node failed and could not be restarted")
        return {"token_ids": job.tokens, "text": tok.decode(job.tokens), "finish_reason": job.reason,
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(job.tokens),
                          "total_tokens": len(ids) + len(job.tokens)},
                "ttft_ms": None if job.ttft is None else round(job.ttft * 1000, 2), "resumes": job.resumes}

    @app.post("/shutdown")
    async def shutdown():
        threading.Thread(target=sup.stop, daemon=True).start()
        if on_shutdown is not None:
            on_shutdown()
        return {"status": "stopping"}

    return app


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    node_args = []
    if "--" in argv:
        i = argv.index("--")
        argv, node_args = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description="elastic dgi node: supervised ranks, re-plan and resume on failure")
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--gpus", default="", help="comma-separated device ids (default: 0..nproc-1, not pinned)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--startup-timeout", type=float, default=1800.0)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--first-env", action="append", default=[],
                    help="KEY=VALUE set for the first generation only (fault injection)")
    a = ap.parse_args(argv)
    nargs = argparse.ArgumentParser(add_help=False)
    nargs.add_argument("--model", default="llama3-8b")
    nargs.add_argument("--tokenizer", default=None)
    na, _ = nargs.parse_known_args(node_args)
    gpus = [int(x) for x in a.gpus.split(",") if x.strip()]
    sup = NodeSupervisor(node_args, nproc=len(gpus) or a.nproc, gpus=gpus or None, max_restarts=a.max_restarts,
                         first_env=dict(kv.split("=", 1) for kv in a.first_env),
                         startup_timeout=a.startup_timeout, log_dir=a.log_dir)
    from dgi.models.config import get_config
    from dgi.utils.tokenizer import load_tokenizer
    mc = get_config(na.model)
    tok = load_tokenizer(na.tokenizer or na.model, vocab_size=mc.vocab_size, bos=mc.bos_token_id,
                         eos=mc.eos_token_id)
    sup.start()
    import uvicorn
    server = uvicorn.Server(uvicorn.Config(build_app(sup, tok, lambda: setattr(server, "should_exit", True)),
                                           host=a.host, port=a.port, log_level="warning"))
    try:
        server.run()
    finally:
        if not sup.stopping:
            sup.stop()
        else:
            deadline = time.time() + 150
            while time.time() < deadline and any(p.poll() is None for p in sup.procs):
                time.sleep(0.2)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
