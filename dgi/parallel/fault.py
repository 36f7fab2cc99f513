"""Failure detection and fault injection for the in-node multi-rank runtime.

* **Liveness watchdog** (``Watchdog``): every rank publishes a heartbeat in the
  rendezvous store (a gloo/TCP side channel that does not share a queue with
  RCCL).  A rank that stops beating for ``DGI_WATCHDOG_S`` seconds (default
  600), or that published a failure record, makes every other rank dump its
  Python stacks and exit non-zero — a dead or wedged rank can no longer
  leave the node hanging in an RCCL wait forever (the reference had no
  data-plane failure handling at all: its ``_handle_failure`` raised).
* **Fault injection** (``DGI_FAULT=rank:step:kind[:arg]``, several separated by
  ``,``) at named sites of the step loops:

  ``kill``     the rank exits with status 17 at that step
  ``delay``    sleep ``arg`` ms (default 200) at that step (a site that passes
               ``idle`` keeps calling it meanwhile: slow compute, live comms)
  ``raise``    raise ``InjectedFault`` (exercises the failure record path)
  ``corrupt``  the site's ``corrupt`` hook flips bytes of the payload it owns
               (P/D: the migrated KV buffer)

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

    def start(self) -> "Watchdog":
        import atexit
        self.beat()
        self._t.start()
        atexit.register(self.stop)
        return self

    def beat(self) -> None:
        self.store.set(f"dgi/hb/{self.rank}", repr(time.time()))

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
        sys.stderr.write(f"[dgi watchdog] rank {self.rank}: {why}; aborting\n")
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(3)

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
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
