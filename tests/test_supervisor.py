"""Elastic node supervisor (dgi.serve.supervisor): blame rules, and a 3-rank P/D
node on CPU (gloo) that loses a prefill rank while serving, restarts on the two
survivors and completes every request on its greedy trajectory (re-prefill
from token history)."""
import concurrent.futures as cf
import json
import os
import socket
import subprocess
import sys
import time

import httpx
import torch

from dgi.serve.supervisor import blame

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE_ARGS = ["--model", "llama-tiny", "--max-model-len", "512", "--max-num-seqs", "16", "--max-batched-tokens", "512"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_blame_prefers_the_first_hand_failure():
    assert blame({1: 17}) == 1
    assert blame({0: 3, 2: 1}) == 2            # 3 = the watchdog's follow-on abort, not the cause
    assert blame({0: 3}) == 0
    assert blame({0: 0}) is None
    assert blame({}) is None


def test_supervisor_replans_and_resumes_after_rank_loss():
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.spec.eagle3 import greedy_gap
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("DGI_FAULT", None)
    # world 3 = prefill ranks [0, 1] + decode rank 2; rank 0 dies at its second prefill step
    cmd = [sys.executable, "-m", "dgi.serve.supervisor", "--nproc", "3", "--port", str(port), "--max-restarts", "2",
           "--startup-timeout", "240", "--first-env", "DGI_FAULT=0:1:kill", "--"] + NODE_ARGS
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{port}"
    try:
        t0 = time.time()
        while True:
            assert proc.poll() is None, proc.stdout.read().decode()[-3000:]
            try:
                if httpx.get(url + "/health", timeout=2).json().get("status") == "ok":
                    break
            except (httpx.HTTPError, ValueError):
                pass
            assert time.time() - t0 < 240, "supervisor did not start"
            time.sleep(0.3)
        g = torch.Generator().manual_seed(5)
        prompts = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (9, 23)]
        body = {"max_tokens": 24, "temperature": 0.0, "ignore_eos": True}
        streamed = []
        # A decodes long enough on the decode rank to still be streaming when the restart tears it down
        with httpx.stream("POST", url + "/generate", json=dict(body, prompt_ids=prompts[0], stream=True,
                                                                 max_tokens=360),
                          timeout=300) as r:
            lines = r.iter_lines()
            for ln in lines:                  # A is decoding (prefilled at rank 0's step 0) ...
                if ln.startswith("data: ") and "token_id" in ln:
                    streamed.append(json.loads(ln[6:])["token_id"])
                    if len(streamed) == 3:
                        break
            with cf.ThreadPoolExecutor(1) as ex:   # ... when B's prefill (rank 0, step 1) kills the rank
                fb = ex.submit(lambda: httpx.post(url + "/generate", json=dict(body, prompt_ids=prompts[1]),
                                                  timeout=300).json())
                for ln in lines:
                    if ln.startswith("data: "):
                        ev = json.loads(ln[6:])
                        if ev.get("done"):
                            assert ev["finish_reason"] == "length"
                            break
                        streamed.append(ev["token_id"])
                out_b = fb.result()
        st = httpx.get(url + "/stats", timeout=30).json()["supervisor"]
        assert st["restarts"] == 1 and st["gpus"] == [1, 2], st
        assert st["failures"][0]["rank"] == 0 and st["failures"][0]["status"] == 17
        assert st["resumed_streams"] >= 2
        eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", max_num_seqs=16, max_num_batched_tokens=512,
                                     max_model_len=512, use_graphs=False))
        outs = [streamed, out_b["token_ids"]]
        for p, o, n in zip(prompts, outs, (360, 24)):
            assert len(o) == n
            assert greedy_gap(eng, p, o) < 1e-3     # one greedy trajectory across the restart
        assert out_b["resumes"] >= 1
        # the second generation (1 prefill + 1 decode rank) keeps serving
        one = httpx.post(url + "/generate", json={"prompt_ids": prompts[0], "max_tokens": 4, "temperature": 0.0,
                                                  "ignore_eos": True}, timeout=120).json()
        assert one["token_ids"] == outs[0][:4] and one["resumes"] == 0
        httpx.post(url + "/shutdown", timeout=10)
        proc.wait(timeout=200)
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()
