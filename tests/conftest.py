"""Test configuration.

* ``gpu`` marker: needs a real MI355X (run via gpurun: ``pytest -m gpu``).
* Reference-compat tests import the server/worker packages both as packages
  and flat (``worker/`` and ``server/`` on sys.path), like the reference's
  own suite (SURVEY §4 "Import-path duality").
* A tiny built-in asyncio runner replaces pytest-asyncio (not installed).
"""
import asyncio
import inspect
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "worker"), os.path.join(ROOT, "server"), os.path.join(ROOT, "sdk", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)
# a file database: the API tests drive the app from several threads at once, and
# an in-memory SQLite database is one shared connection (not thread-safe)
import tempfile  # noqa: E402
_DB = "sqlite+aiosqlite:///" + os.path.join(tempfile.gettempdir(), f"dgi_test_{os.getpid()}.db")
if os.environ.get("PYTEST_XDIST_WORKER"):
    # xdist workers inherit the controller's DATABASE_URL: one file per worker process, or one
    # worker's table setup races another's (sqlite "no such table" under -n)
    os.environ["DATABASE_URL"] = _DB
    # each worker's torch would start one OpenMP thread per CPU: under -n 6 on 8 CPUs the
    # spin-waiting pools made single tests 100x slower (a 6 s spec test took 659 s); give each
    # worker its share (subprocesses the tests start inherit it)
    _n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1") or 1)
    _share = str(max(1, (os.cpu_count() or 1) // max(1, _n)))
    os.environ["OMP_NUM_THREADS"] = _share
    import torch  # noqa: E402
    torch.set_num_threads(int(_share))
else:
    os.environ.setdefault("DATABASE_URL", _DB)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (HIP kernels)")
    config.addinivalue_line("markers", "asyncio: run the coroutine test in an event loop")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "bench: benchmark-style test")


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    if inspect.iscoroutinefunction(pyfuncitem.obj):
        funcargs = pyfuncitem.funcargs
        names = pyfuncitem._fixtureinfo.argnames
        kwargs = {n: funcargs[n] for n in names}
        loop = asyncio.new_event_loop()
        try:
            asyncio.set_event_loop(loop)
            loop.run_until_complete(pyfuncitem.obj(**kwargs))
        finally:
            asyncio.set_event_loop(None)
            loop.close()
        return True
    return None


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
