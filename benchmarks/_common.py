"""Shared helpers for the benchmark CLIs: launch bench.py (single or multi-rank) and collect its JSON line."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_bench(gpus: int, args: List[str], timeout: Optional[int] = None, env: Optional[dict] = None) -> dict:
    """Run bench.py on ``gpus`` ranks (torch.distributed.run for >1) and return its JSON result."""
    cmd = [sys.executable]
    if gpus > 1:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}", "--master-addr",
                "127.0.0.1", "--master-port", str(free_port())]
    cmd += [os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)] + args
    e = dict(os.environ)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e.update(env or {})
    out = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)
    line = next((ln for ln in reversed(out.stdout.splitlines()) if ln.startswith("{")), None)
    if out.returncode != 0 or line is None:
        raise RuntimeError(f"bench failed rc={out.returncode}\n{out.stdout[-2000:]}\n{out.stderr[-4000:]}")
    return json.loads(line)


def save(path: str, obj) -> None:
    with open(path, "w") as f:
        json.dump(obj, f, indent=2)
    print(f"saved {path}")
