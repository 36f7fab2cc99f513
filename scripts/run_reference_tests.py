#!/usr/bin/env python3
"""Run the reference repository's own test-suite, unmodified, against this repo.

The reference tests (Baozhi888/distributed-gpu-inference ``tests/``) import
``common``, ``worker``, ``server`` and ``sdk`` from their repository root.  This
script copies them into a scratch directory next to symlinks of THIS repo's
packages and runs pytest there, so every compatibility surface the reference
pins (engines registry, P/D scheduler, sessions, KV cache, serialization,
SDK, server services) is checked against the rebuild.  ``pytest-asyncio`` is
not installed here: a 10-line plugin runs ``async def`` tests in a fresh event
loop.  Nothing from the reference is executed except its tests.

    python scripts/run_reference_tests.py [--reference /root/reference] [-- pytest args]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = '''import asyncio, inspect
import pytest


def pytest_configure(config):
    config.addinivalue_line("markers", "asyncio: run the coroutine test in a fresh event loop")


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    if inspect.iscoroutinefunction(pyfuncitem.obj):
        args = {a: pyfuncitem.funcargs[a] for a in pyfuncitem._fixtureinfo.argnames}
        asyncio.run(pyfuncitem.obj(**args))
        return True
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("REFERENCE_DIR", "/root/reference"))
    ap.add_argument("pytest_args", nargs="*")
    a = ap.parse_args()
    src = os.path.join(a.reference, "tests")
    if not os.path.isdir(src):
        print(f"no reference tests at {src}", file=sys.stderr)
        return 2
    work = tempfile.mkdtemp(prefix="dgi-reftests-")
    try:
        shutil.copytree(src, os.path.join(work, "tests"))
        with open(os.path.join(work, "tests", "_dgi_asyncio_shim.py"), "w") as f:
            f.write(SHIM)
        for d in ("common", "worker", "server", "sdk", "proto", "dgi"):
            os.symlink(os.path.join(ROOT, d), os.path.join(work, d))
        cmd = [sys.executable, "-m", "pytest", "tests", "-q", "-p", "tests._dgi_asyncio_shim",
               "-p", "no:cacheprovider", *a.pytest_args]
        return subprocess.call(cmd, cwd=work)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    raise SystemExit(main())
