"""Failure detection and fault injection for the in-node multi-rank runtime.

* **Liveness watchdog** (``Watchdog``): every rank publishes a heartbeat in the
  rendezvous store (a gloo/TCP side channel that does not share a queue with
  RCCL).  A rank that stops beating for ``DGI_WATCHDOG_S`` seconds (default
  600), or that published a failure record, makes every other rank dump its
  Python stacks and exit non-zero — a dead or wedged rank can no longer
  leave the node hanging in an RCCL wait forever (the reference had no
  data-plane failure handling at all: its ``_handle_failure`` raised).
* **Phase deadlines** (``Watchdog.phase``): a multi-rank run moves
  through named phases (rendezvous, pair warm-up, start-up probe, engine build,
  first hop, serving window, teardown), each with a time budget (``DGI_PHASE_S``,
  default 120 s; engine build ``DGI_BUILD_S`` 300 s; the serving phase is
  ``serve_budget``: 3x the expected time of the steps it runs, at least
  ``DGI_SERVE_S`` 420 s).  Every rank publishes
  its current phase in the store.  The first rank whose phase overruns prints ONE
  JSON line on stdout — ``{"status": "timeout", ...}`` with the stuck rank, its
  phase and every rank's phase — records a failure (so every other rank exits
  too) and exits with status 4: a wedged first contact with a real node ends in
  minutes with evidence, instead of a silent lease-long hang (the reference's
  ``DistributedInferenceSession._handle_failure`` raised with no state:
  worker/distributed/session.py:339-365).
* **Fault injection** (``DGI_FAULT=rank:step:kind[:arg]``, several separated by
  ``,``) at named sites of the step loops:

  ``kill``     the rank exits with status 17 at that step
  ``delay``    sleep ``arg`` ms (default 200) at that step (a site that passes
               ``idle`` keeps calling it meanwhile: slow compute, live comms)
  ``raise``    raise ``InjectedFault`` (exercises the failure record path)
  ``corrupt``  the site's ``corrupt`` hook flips bytes of the payload it owns
               (P/D: the migrated KV buffer)
  ``stall``    sleep ``arg`` s (default 3600) without servicing anything: a wedged
               rank (phase-deadline tests; site ``PHASE_SITES[name]`` stalls in
               that start-up phase)

The multi-process tests (tests/test_parallel_cpu.py) drive each kind.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Optional


class InjectedFault(RuntimeError):
    pass


class FaultPlan:
    def __init__(self, spec: Optional[str] = None):
        self.rules = []
        for part in (spec if spec is not None else os.environ.get("DGI_FAULT", "")).split(","):
            part = part.strip()
            if not part:
                continue
            f = part.split(":")
            rank, step, kind = int(f[0]), int(f[1]), f[2]
            arg = f[3] if len(f) > 3 else None
            self.rules.append((rank, step, kind, arg))
        self.fired = set()

    def __bool__(self) -> bool:
        return bool(self.rules)

    def check(self, rank: int, step: int, corrupt=None, idle=None) -> None:
        for i, (r, s, kind, arg) in enumerate(self.rules):
            if r != rank or s != step or i in self.fired:
                continue
            self.fired.add(i)
            if kind == "kill":
                sys.stderr.write(f"[dgi fault] rank {rank} killed at step {step}\n")
                sys.stderr.flush()
                os._exit(17)
            elif kind == "delay":
                end = time.perf_counter() + float(arg or 200) / 1000.0
                if idle is None:
                    time.sleep(max(0.0, end - time.perf_counter()))
                while idle is not None and time.perf_counter() < end:
                    idle()
                    time.sleep(0.0005)
            elif kind == "raise":
                raise InjectedFault(f"injected fault on rank {rank} at step {step}")
            elif kind == "corrupt" and corrupt is not None:
                corrupt()
            elif kind == "stall":
                time.sleep(float(arg or 3600))


# fault-injection step ids of the start-up phases (``DGI_FAULT=rank:<site>:stall``)
PHASE_SITES = {"pair_warmup": 300001, "probe": 300002, "engine_build": 300003, "first_hop": 300004}
DEFAULT_PHASE_S = float(os.environ.get("DGI_PHASE_S", "120"))
BUILD_S = float(os.environ.get("DGI_BUILD_S", "300"))       # model load + graph capture of one rank
SERVE_FLOOR_S = float(os.environ.get("DGI_SERVE_S", "420"))   # serving-window floor


def serve_budget(n_steps: int, step_s: float = 0.25, slack: float = 3.0) -> float:
    """Deadline of a serving phase of ``n_steps`` engine steps (ramp + warm-up + timed
    window, counted in the steps the rank itself runs): ``slack`` x the expected time at
    ``step_s`` per step, never below ``DGI_SERVE_S`` (420 s).  A long ``--steps`` run
    on a slow layout is thus not mistaken for a hang."""
    return max(SERVE_FLOOR_S, slack * max(0, int(n_steps)) * float(step_s))

_plan: Optional[FaultPlan] = None


def plan() -> FaultPlan:
    global _plan
    if _plan is None:
        _plan = FaultPlan()
    return _plan


class Watchdog:
    """Per-rank heartbeat thread over the rendezvous store."""

    def __init__(self, rank: int, world: int, store=None, interval: float = 1.0, timeout: Optional[float] = None):
        if store is None:
            from torch.distributed import distributed_c10d as c10d
            store = c10d._get_default_store()
        self.store, self.rank, self.world = store, rank, world
        self.interval = interval
        self.timeout = float(os.environ.get("DGI_WATCHDOG_S", timeout or 600))
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="dgi-watchdog", daemon=True)
        self.last_seen = {r: time.time() for r in range(world)}
        self.phase_name: Optional[str] = None
        self.phase_t0 = time.time()
        self.deadline: Optional[float] = None
        self.timeout_info: dict = {}            # extra fields of the timeout JSON line

    def start(self) -> "Watchdog":
        import atexit
        _WATCHDOG.append(self)
        self.beat()
        self._t.start()
        atexit.register(self.stop)
        return self

    def beat(self) -> None:
        self.store.set(f"dgi/hb/{self.rank}", repr(time.time()))

    def phase(self, name: str, budget_s: Optional[float] = None) -> None:
        """Enter phase ``name``: it must end (the next ``phase`` call) within ``budget_s``
        seconds (``DGI_PHASE_S`` by default; <= 0: no deadline)."""
        b = DEFAULT_PHASE_S if budget_s is None else float(budget_s)
        self.phase_name, self.phase_t0 = name, time.time()
        self.deadline = self.phase_t0 + b if b > 0 else None
        try:
            self.store.set(f"dgi/phase/{self.rank}", f"{name}@{self.phase_t0:.3f}")
        except Exception:
            pass

    def _phases(self) -> dict:
        out = {}
        now = time.time()
        for r in range(self.world):
            k = f"dgi/phase/{r}"
            try:
                if self.store.check([k]):
                    name, _, t = self.store.get(k).decode().partition("@")
                    out[str(r)] = {"phase": name, "s": round(now - float(t), 1) if t else None}
                else:
                    out[str(r)] = None
            except Exception:
                out[str(r)] = "?"
        return out

    def _timeout(self) -> None:
        """This rank overran its phase: one JSON line (first rank only), failure record, exit 4."""
        import json
        waited = time.time() - self.phase_t0
        msg = {"status": "timeout", "value": None, "n_gpus": self.world,
               "stuck": {"rank": self.rank, "phase": self.phase_name, "waited_s": round(waited, 1)},
               "phases": self._phases(), **self.timeout_info}
        first = True
        try:
            first = self.store.add("dgi/timeout_json", 1) == 1
        except Exception:
            pass
        if first:
            os.write(1, (json.dumps(msg) + "\n").encode())
        self.report_failure(f"phase {self.phase_name} timed out after {waited:.0f}s")
        sys.stderr.write(f"[dgi watchdog] rank {self.rank}: phase {self.phase_name} timed out after {waited:.0f}s\n")
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(4)

    def report_failure(self, msg: str) -> None:
        try:
            self.store.set("dgi/failed", f"rank {self.rank}: {msg}")
        except Exception:
            pass

    def stop(self) -> None:
        self._stop.set()
        try:
            self.store.set(f"dgi/hb/{self.rank}", "done")
        except Exception:
            pass

    def _abort(self, why: str) -> None:
        sys.stderr.write(f"[dgi watchdog] rank {self.rank} (phase {self.phase_name}): {why}; aborting\n")
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(3)

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            if self.deadline is not None and time.time() > self.deadline:
                self._timeout()
            try:
                self.beat()
                if self.store.check(["dgi/failed"]):
                    self._abort("peer failure: " + self.store.get("dgi/failed").decode())
                now = time.time()
                for r in range(self.world):
                    if r == self.rank:
                        continue
                    v = self.store.get(f"dgi/hb/{r}").decode() if self.store.check([f"dgi/hb/{r}"]) else None
                    if v == "done":
                        self.last_seen[r] = now
                        continue
                    if v is not None:
                        self.last_seen[r] = max(self.last_seen[r], float(v))
                    if now - self.last_seen[r] > self.timeout:
                        self._abort(f"rank {r} silent for {now - self.last_seen[r]:.0f}s")
            except Exception:
                # the store itself is gone: the job is tearing down (rank 0 left);
                # never turn a normal shutdown into a failure exit
                return


def phase(name: str, budget_s: Optional[float] = None) -> None:
    """Enter start-up / serving phase ``name`` on this rank's watchdog (no-op without
    one: single-rank runs), and fire any ``stall`` fault injected at that phase."""
    w = current_watchdog()
    if w is not None:
        w.phase(name, budget_s)
    site = PHASE_SITES.get(name)
    if site is not None and plan():
        rank = w.rank if w is not None else int(os.environ.get("RANK", "0"))
        plan().check(rank, site)


_WATCHDOG: list = []


def current_watchdog() -> Optional[Watchdog]:
    return _WATCHDOG[-1] if _WATCHDOG else None
