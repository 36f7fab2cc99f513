"""Wake-up for long-polling workers (``GET /api/v1/workers/{id}/next-job?wait=S``).

The reference's workers poll ``next-job`` every ``poll_interval`` seconds (2 s by default), so a job
submitted to an idle worker waits on average half an interval before anyone looks at it.  With
``wait`` the endpoint keeps the request open.  Whenever a job becomes QUEUED (created,
re-queued after a worker loss, or a P/D job entering its decode phase) ``notify()`` wakes the
waiting requests, and they try to assign again at once.

The wake-up is process-local (one asyncio event per loop).  A waiting request also re-checks the
database every ``RECHECK_S``, so a job queued by another server process is picked up no later than
the old 50 ms poll would have picked it up.  Without ``wait`` the endpoint behaves exactly as before.
"""
from __future__ import annotations

import asyncio
import threading
from typing import Optional

RECHECK_S = 0.05


class JobSignal:
    """One generation of waiters per event: ``notify`` sets the current event and drops it, and the
    next waiter makes a fresh one.  Safe to call from any thread."""

    def __init__(self) -> None:
        self._ev: Optional[asyncio.Event] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._lock = threading.Lock()
        self.notified = 0

    async def wait(self, timeout: float) -> bool:
        """Wait until the next ``notify`` or ``timeout`` seconds; True when notified."""
        loop = asyncio.get_running_loop()
        with self._lock:
            if self._ev is None or self._loop is not loop:
                self._ev, self._loop = asyncio.Event(), loop
            ev = self._ev
        try:
            await asyncio.wait_for(ev.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def notify(self) -> None:
        with self._lock:
            ev, loop = self._ev, self._loop
            self._ev = None
            self.notified += 1
        if ev is None:
            return
        try:
            running = asyncio.get_running_loop()
        except RuntimeError:
            running = None
        if running is loop or loop is None or not loop.is_running():
            ev.set()
        else:
            loop.call_soon_threadsafe(ev.set)


job_queued = JobSignal()
