"""bench.py's multi-rank P/D paths end to end on CPU (gloo, torch.distributed.run):
2 prefill + 1 decode, 2 prefill + 2 decode replicas, 1 prefill + a 2-stage decode
pipeline.  Covers the phase-boundary protocol (phase message -> prefill fence ->
drivers post every announced receive -> synchronise -> barrier) that keeps RCCL
KV sends from waiting on receives nobody will post."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n,args", [
    (3, ["--layout", "pd", "--prefill-ranks", "2", "--decode-replicas", "1"]),
    (4, ["--layout", "pd", "--prefill-ranks", "2", "--decode-replicas", "2"]),
    (3, ["--layout", "pdpp", "--prefill-ranks", "1", "--decode-stages", "2"]),
])
def test_bench_pd_layouts_on_gloo(n, args):
    env = {**os.environ, "OMP_NUM_THREADS": "1", "DGI_WATCHDOG": "0"}
    env.pop("DGI_STAGED_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(n),
           "--model", "llama-tiny", "--steps", "4", "--warmup", "1", "--ramp-steps", "2", "--concurrency", "8",
           "--output-len", "8", "--prompt-len", "32", "--max-batched-tokens", "256", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')][-1]
    d = json.loads(line)
    assert d["n_gpus"] == n and d["value"] > 0
    assert d["extra"]["layout"]["kind"] in ("pd", "pdpp")
