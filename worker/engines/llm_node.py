"""LLM engine backed by a dgi node server (multi-GPU P/D / pipeline node).

``NativeLLMEngine`` runs one engine in the worker process (one GPU).  For a
whole MI355X node the worker starts — or attaches to — ``dgi.serve.node``
(one process per GPU under ``torch.distributed.run``, prefill ranks + decode
pipeline, KV over RCCL) and forwards requests to its HTTP endpoint, the way
the reference delegated to an external vLLM/SGLang server
(worker/engines/llm_vllm.py, llm_sglang.py).

Config keys: ``node_url`` (attach) or ``gpus`` / ``device_ids`` / ``layout`` /
``port`` (launch), plus ``model_id``, ``max_num_seqs``,
``max_num_batched_tokens``, ``max_model_len``.  ``elastic: true`` launches
the node under ``dgi.serve.supervisor`` (rank loss -> re-plan on the
surviving GPUs, in-flight requests resumed by re-prefill; ``max_restarts``).
"""
from __future__ import annotations

import json
import logging
import os
import socket
import subprocess
import sys
import time
from typing import Any, AsyncIterator, Dict, List, Optional

import httpx

from .llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine

logger = logging.getLogger(__name__)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class NodeLLMEngine(LLMBaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type = LLMBackend.NATIVE_MI355X
        self.url: Optional[str] = config.get("node_url")
        self.proc: Optional[subprocess.Popen] = None
        self.model_id = config.get("model_id", "llama3-70b")

    # ------------------------------------------------------------------ lifecycle
    def _launch(self) -> None:
        c = self.config
        ids = c.get("device_ids") or list(range(int(c.get("gpus", 1))))
        n = len(ids)
        port = int(c.get("port") or _free_port())
        args = ["-m", "dgi.serve.node", "--model", self.model_id, "--port", str(port),
                "--max-num-seqs", str(c.get("max_num_seqs", 512)),
                "--max-batched-tokens", str(c.get("max_num_batched_tokens", 4096)),
                "--max-model-len", str(c.get("max_model_len", 4096)),
                "--layout", str(c.get("layout", "auto") if c.get("layout") not in (None, "single") else "auto")]
        env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if c.get("elastic"):
            # the supervisor owns the ranks (and their device pinning) and serves the same HTTP surface
            node = list(args[2:])          # drop "-m dgi.serve.node"
            i = node.index("--port")
            del node[i:i + 2]
            cmd = [sys.executable, "-m", "dgi.serve.supervisor", "--nproc", str(n), "--port", str(port),
                   "--max-restarts", str(c.get("max_restarts", 3))]
            if c.get("device_ids"):
                cmd += ["--gpus", ",".join(str(i) for i in ids)]
            cmd += ["--"] + node
        elif n > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
        else:
            cmd = [sys.executable] + args
        if ids and not c.get("elastic"):
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(i) for i in ids)
        logger.info("launching node server: %s", " ".join(cmd))
        self.proc = subprocess.Popen(cmd, cwd=ROOT, env=env)
        self.url = f"http://127.0.0.1:{port}"

    def load_model(self) -> None:
        if not self.url:
            self._launch()
        deadline = time.time() + float(self.config.get("startup_timeout", 1800))
        while time.time() < deadline:
            if self.proc is not None and self.proc.poll() is not None:
                raise RuntimeError(f"node server exited with {self.proc.returncode}")
            try:
                if httpx.get(self.url + "/health", timeout=2).json().get("status") == "ok":
                    self.loaded = True
                    from dgi.models.config import get_config
                    from dgi.utils.tokenizer import load_tokenizer
                    mc = get_config(self.model_id)
                    self.tokenizer = load_tokenizer(self.config.get("tokenizer", self.model_id),
                                                    vocab_size=mc.vocab_size, bos=mc.bos_token_id,
                                                    eos=mc.eos_token_id)
                    return
            except (httpx.HTTPError, ValueError):
                pass
            time.sleep(0.5)
        raise TimeoutError("node server did not become healthy")

    def unload_model(self) -> None:
        if self.proc is not None:
            try:
                httpx.post(self.url + "/shutdown", timeout=10)
                self.proc.wait(timeout=120)
            except Exception:
                self.proc.kill()
            self.proc = None
        self.loaded = False

    # ------------------------------------------------------------------ generation
    def _body(self, messages, cfg: GenerationConfig, stream: bool = False) -> Dict[str, Any]:
        return {"messages": messages, "max_tokens": cfg.max_tokens, "temperature": cfg.temperature,
                "top_p": cfg.top_p, "top_k": cfg.top_k, "stream": stream}

    async def generate_async(self, messages: List[Dict[str, str]],
                             config: Optional[GenerationConfig] = None) -> GenerationResult:
        cfg = config or GenerationConfig()
        async with httpx.AsyncClient(timeout=None) as c:
            r = await c.post(self.url + "/generate", json=self._body(messages, cfg))
            r.raise_for_status()
            d = r.json()
        u = d["usage"]
        return GenerationResult(text=d["text"], prompt_tokens=u["prompt_tokens"],
                                completion_tokens=u["completion_tokens"], total_tokens=u["total_tokens"],
                                finish_reason="stop" if d.get("finish_reason") == "stop" else "length")

    async def batch_generate(self, batch_messages: List[List[Dict[str, str]]],
                             config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        import asyncio
        return list(await asyncio.gather(*[self.generate_async(m, config) for m in batch_messages]))

    async def stream_generate(self, messages: List[Dict[str, str]],
                              config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        cfg = config or GenerationConfig()
        async with httpx.AsyncClient(timeout=None) as c:
            async with c.stream("POST", self.url + "/generate", json=self._body(messages, cfg, True)) as r:
                async for line in r.aiter_lines():
                    if line.startswith("data: "):
                        ev = json.loads(line[6:])
                        if ev.get("done"):
                            return
                        yield ev["text"]

    def supports_streaming(self) -> bool:
        return True

    def supports_batch_inference(self) -> bool:
        return True

    def get_status(self) -> Dict[str, Any]:
        s = {"loaded": self.loaded, "node_url": self.url, "backend": "mi355x-node"}
        if self.loaded:
            try:
                s["engine"] = httpx.get(self.url + "/stats", timeout=5).json()
            except httpx.HTTPError as e:
                s["error"] = str(e)
        return s
