"""Launch the served path as separate processes for the HTTP benchmarks: the control plane
(uvicorn, SQLite) and one worker daemon with the ``llm_native`` engine on a GPU.

This is the reference's live path (SDK -> server -> worker pull loop -> engine,
reference worker/main.py:313-376), started the way an operator would start it, so the
HTTP numbers include every hop: the server's job queue, the worker's poll interval,
the result post-back and, for the SSE path, the worker's direct endpoint.

    python benchmarks/serve_stack.py worker --server-url URL --model llama3-8b --direct-port P
(the worker entry ``ServeStack`` uses; ``ServeStack`` is what ``single_worker.py --launch`` uses).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _common import free_port  # noqa: E402


def wait_http(url: str, timeout: float = 120.0, proc=None) -> None:
    import httpx
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"process for {url} exited with {proc.returncode}")
        try:
            if httpx.get(url, timeout=2).status_code == 200:
                return
        except httpx.HTTPError:
            pass
        time.sleep(0.25)
    raise TimeoutError(url)


class ServeStack:
    """Control plane + one worker daemon, each its own process; ``close`` stops both."""

    def __init__(self, model: str, out_dir: str, poll_interval: float = 0.05, engine: dict | None = None,
                 start_timeout: float = 600.0):
        os.makedirs(out_dir, exist_ok=True)
        self.dir = tempfile.mkdtemp(prefix="dgi_stack_")
        self.sport, self.dport = free_port(), free_port()
        self.server_url = f"http://127.0.0.1:{self.sport}"
        self.direct_url = f"http://127.0.0.1:{self.dport}"
        env = dict(os.environ)
        env["DATABASE_URL"] = "sqlite:///" + os.path.join(self.dir, "cp.db")
        env["HOME"] = self.dir                  # the worker's machine fingerprint / config live here
        self.logs = [open(os.path.join(out_dir, "server.log"), "w"), open(os.path.join(out_dir, "worker.log"), "w")]
        self.procs = []
        self.procs.append(subprocess.Popen(
            [sys.executable, "-m", "uvicorn", "app.main:app", "--app-dir", os.path.join(ROOT, "server"),
             "--host", "127.0.0.1", "--port", str(self.sport), "--log-level", "warning"],
            cwd=ROOT, env=env, stdout=self.logs[0], stderr=subprocess.STDOUT))
        try:
            wait_http(self.server_url + "/health", 120, self.procs[0])
            self.procs.append(subprocess.Popen(
                [sys.executable, os.path.abspath(__file__), "worker", "--server-url", self.server_url,
                 "--model", model, "--direct-port", str(self.dport), "--poll-interval", str(poll_interval),
                 "--engine", json.dumps(engine or {})],
                cwd=ROOT, env=env, stdout=self.logs[1], stderr=subprocess.STDOUT))
            wait_http(self.direct_url + "/health", start_timeout, self.procs[1])
            self._wait_registered(start_timeout)
        except BaseException:
            self.close()
            raise

    def _wait_registered(self, timeout: float) -> None:
        import httpx
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self.procs[1].poll() is not None:
                raise RuntimeError(f"worker exited with {self.procs[1].returncode}")
            try:
                r = httpx.get(self.server_url + "/api/v1/workers", timeout=5)
                if r.status_code == 200 and any(w.get("status") in ("online", "idle", "busy")
                                                for w in (r.json() or [])):
                    return
            except (httpx.HTTPError, ValueError):
                pass
            time.sleep(0.5)
        raise TimeoutError("worker did not register")

    def close(self) -> None:
        for p in reversed(self.procs):
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(60)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait(10)
        for f in self.logs:
            f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def run_worker(a) -> None:
    sys.path.insert(0, os.path.join(ROOT, "worker"))
    sys.path.insert(0, ROOT)
    from config import WorkerConfig
    from main import Worker
    eng = {"model_id": a.model, "backend": "mi355x", "max_num_seqs": 128, "max_num_batched_tokens": 8192,
           "max_model_len": 4096, "warmup": True, "seed": 0, **json.loads(a.engine or "{}")}
    cfg = WorkerConfig(name="bench-worker", region="asia-east", supported_types=["llm"], engines={"llm": eng},
                       heartbeat_interval=2, poll_interval=a.poll_interval)
    cfg.server.url = a.server_url
    cfg.direct.enabled, cfg.direct.host, cfg.direct.port = True, "127.0.0.1", a.direct_port
    cfg.direct.public_url = f"http://127.0.0.1:{a.direct_port}"
    cfg.load_control.max_concurrent_jobs = int(eng["max_num_seqs"])
    w = Worker(cfg, config_path=os.path.join(os.environ.get("HOME", "."), "worker.yaml"))
    w.start(install_signals=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("role", choices=["worker"])
    ap.add_argument("--server-url", required=True)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--direct-port", type=int, required=True)
    ap.add_argument("--poll-interval", type=float, default=0.05)
    ap.add_argument("--engine", default="{}")
    run_worker(ap.parse_args())


if __name__ == "__main__":
    main()
