"""Node server: HTTP front-end over the native engine, single process and P/D (gloo, 2 ranks)."""
import os
import socket
import subprocess
import sys
import time

import httpx
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(nproc, port, max_num_seqs=16, extra=()):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("CUDA_VISIBLE_DEVICES", None)
    args = ["-m", "dgi.serve.node", "--model", "llama-tiny", "--port", str(port), "--max-model-len", "512",
            "--max-num-seqs", str(max_num_seqs), "--max-batched-tokens", "512", *extra]
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)


def _wait(url, proc, timeout=180):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(proc.stdout.read().decode()[-3000:])
        try:
            if httpx.get(url + "/health", timeout=2).json().get("status") == "ok":
                return
        except (httpx.HTTPError, ValueError):
            pass
        time.sleep(0.3)
    raise TimeoutError("node server did not start")


def _reference(prompts, max_tokens):
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", max_num_seqs=16, max_num_batched_tokens=512,
                                 max_model_len=512, use_graphs=False))
    return [r.output for r in eng.generate(prompts, SamplingParams(max_tokens=max_tokens, temperature=0.0,
                                                                   ignore_eos=True))]


@pytest.mark.parametrize("nproc,max_num_seqs,extra", [(1, 16, ()), (2, 16, ()), (3, 2, ()),
                                                       (4, 16, ("--layout", "pd", "--prefill-ranks", "2"))])
def test_node_server_generate_matches_engine(nproc, max_num_seqs, extra):
    """(3, 2): two prefill ranks, a decode rank that holds 2 sequences — the
    rest overflow into the prefill ranks' own decode and stream back through
    the router.  (4, pd, 2 prefill): two decode replicas; the second forwards
    its tokens to the router on the first."""
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (9, 23, 40)]
    ref = _reference(prompts, 8)
    port = _port()
    proc = _start(nproc, port, max_num_seqs, extra)
    url = f"http://127.0.0.1:{port}"
    try:
        _wait(url, proc)
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(3) as ex:
            outs = list(ex.map(lambda p: httpx.post(url + "/generate", json={
                "prompt_ids": p, "max_tokens": 8, "temperature": 0.0, "ignore_eos": True}, timeout=120).json(),
                prompts))
        assert [o["token_ids"] for o in outs] == ref
        assert all(o["usage"]["completion_tokens"] == 8 and o["ttft_ms"] is not None for o in outs)
        one = httpx.post(url + "/generate", json={"prompt_ids": prompts[0], "max_tokens": 1,
                                                   "temperature": 0.0, "ignore_eos": True}, timeout=60).json()
        assert one["token_ids"] == ref[0][:1]
        with httpx.stream("POST", url + "/generate", json={"prompt_ids": prompts[1], "max_tokens": 5,
                                                           "temperature": 0.0, "ignore_eos": True, "stream": True},
                          timeout=60) as r:
            evs = [ln for ln in r.iter_lines() if ln.startswith("data: ")]
        assert len(evs) == 6 and '"done": true' in evs[-1]
        st = httpx.get(url + "/stats", timeout=10).json()
        assert st["finished"] >= 5
        httpx.post(url + "/shutdown", timeout=10)
        proc.wait(timeout=120)
        assert proc.returncode == 0, proc.stdout.read().decode()[-2000:]
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()


@pytest.mark.parametrize("elastic", [False, True])
def test_worker_node_engine_attaches_and_generates(elastic):
    """The worker's NodeLLMEngine launches a 2-rank node server (directly, or
    under the elastic supervisor) and serves inference() through it."""
    sys.path.insert(0, os.path.join(ROOT, "worker"))
    from engines import get_engine
    eng = get_engine("mi355x-node")({"model_id": "llama-tiny", "gpus": 2, "max_num_seqs": 16, "elastic": elastic,
                                      "max_num_batched_tokens": 512, "max_model_len": 512, "startup_timeout": 240})
    eng.load_model()
    try:
        out = eng.inference({"messages": [{"role": "user", "content": "hi"}], "max_tokens": 6, "temperature": 0.0})
        assert out["usage"]["completion_tokens"] == 6
        assert eng.get_status()["engine"]["finished"] >= 1
    finally:
        eng.unload_model()
