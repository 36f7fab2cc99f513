"""NativeLLMEngine — the MI355X-native ``dgi`` runtime behind the reference's
``LLMBaseEngine`` contract (registry name ``llm_native``, alias ``mi355x``).

Where the reference offloads to SGLang/vLLM (worker/engines/llm_sglang.py,
llm_vllm.py) this engine provides the same features itself: paged KV,
radix prefix cache, iteration-level continuous batching, chunked prefill,
streaming, on-device sampling and hipGraph decode.

Threading: one daemon thread owns the ``dgi.engine.LLMEngine`` and steps it
while work exists; asyncio callers submit through a thread-safe queue and
are resolved with ``loop.call_soon_threadsafe`` (no per-call threads).

Config keys accepted (SURVEY Appendix C mapping): ``model_id``, ``device``,
``mem_fraction_static``/``gpu_memory_utilization`` -> KV fraction,
``max_running_requests``/``max_num_seqs``, ``chunked_prefill_size``,
``enable_prefix_caching``, ``context_length``/``max_model_len``,
``num_blocks``, ``use_graphs``/``enforce_eager``; nested ``sglang``/``vllm``/
``native`` dicts are merged in.
"""
from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time
from typing import Any, AsyncIterator, Dict, List, Optional

import torch

from dgi.utils.tokenizer import StreamDecoder, chat_prompt_ids, load_tokenizer

from .llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine

logger = logging.getLogger(__name__)


def _merged(config: Dict[str, Any]) -> Dict[str, Any]:
    out = dict(config)
    for k in ("sglang", "vllm", "native", "mi355x"):
        if isinstance(config.get(k), dict):
            out.update(config[k])
    return out


class _Pending:
    __slots__ = ("req", "loop", "future", "stream_q", "sent", "cfg", "prompt_len", "export_key", "export_token")

    def __init__(self, loop, future, stream_q, cfg, prompt_len, export_key=None, export_token=None):
        self.req = None
        self.export_key = export_key    # cluster P/D prefill phase: export the KV at the first token
        self.export_token = export_token  # secret the decode worker presents to pull it
        self.loop = loop
        self.future = future
        self.stream_q = stream_q
        self.sent = 0
        self.cfg = cfg
        self.prompt_len = prompt_len


class NativeLLMEngine(LLMBaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type = LLMBackend.NATIVE_MI355X
        self.engine = None
        self._inbox: "queue.Queue" = queue.Queue()
        self._pending: Dict[Any, _Pending] = {}
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._wake = threading.Event()
        self.stats = {"requests": 0, "completed": 0, "errors": 0, "kv_exported": 0, "kv_imported": 0}
        # cluster P/D: sequences this worker prefilled, waiting for their decode worker's pull
        from dgi.kv.transfer import KVExportStore
        self.kv_exports = KVExportStore(int(float(_merged(config).get("kv_export_gb", 8)) * (1 << 30)))

    # ------------------------------------------------------------------ lifecycle
    def load_model(self) -> None:
        from dgi.engine import EngineConfig, LLMEngine
        from dgi.models.config import get_config

        from dgi.models.config import PRESETS
        from dgi.models.weights import resolve_checkpoint

        c = _merged(self.config)
        model_id = c.get("model_id", "llama3-8b")
        device = c.get("device", "cuda" if torch.cuda.is_available() else "cpu")
        # real weights when a local checkpoint exists (explicit model_path, a directory
        # model_id, or an offline HF cache snapshot); random init only for the built-in
        # benchmark presets or when explicitly allowed — never silently for a hub id
        ckpt = resolve_checkpoint(model_id, c.get("model_path"))
        if ckpt is None and model_id not in PRESETS and not c.get("allow_random_weights", False):
            raise FileNotFoundError(
                f"no local safetensors checkpoint for {model_id!r}: set engines.llm.model_path, or "
                "allow_random_weights: true to serve random-init weights of that architecture")
        if ckpt is None and model_id not in PRESETS:
            logger.warning("serving RANDOM-INIT weights for %s (allow_random_weights)", model_id)
        self.weights = ckpt or "random-init"
        mc = get_config(ckpt or model_id)
        frac = c.get("mem_fraction_static", c.get("gpu_memory_utilization", c.get("kv_fraction", 0.9)))
        ecfg = EngineConfig(
            model=model_id, device=device, model_path=ckpt,
            max_num_seqs=int(c.get("max_running_requests", c.get("max_num_seqs", 256))),
            max_num_batched_tokens=int(c.get("chunked_prefill_size", c.get("max_num_batched_tokens", 8192))),
            max_model_len=int(c.get("context_length", c.get("max_model_len", 8192))),
            kv_fraction=float(frac), num_blocks=c.get("num_blocks"),
            enable_prefix_caching=bool(c.get("enable_prefix_caching", True)),
            use_graphs=bool(c.get("use_graphs", not c.get("enforce_eager", False))) and device != "cpu",
            seed=int(c.get("seed", 0)), block_size=int(c.get("block_size", 16)),
            host_kv_gb=float(c.get("host_kv_gb", 0.0)),
            graph_buckets=tuple(c["graph_batch_buckets"]) if c.get("graph_batch_buckets") else None)
        spec = c.get("speculative")
        if spec:
            # EAGLE-3 tree speculation for greedy requests (dgi.spec.eagle3)
            from dgi.spec.eagle3 import SpecConfig, SpecEngine
            sc = spec if isinstance(spec, dict) else {}
            keys = ("depth", "width", "topk", "adaptive_depth", "min_accept_rate", "raise_accept_rate",
                    "auto_off", "probe_every", "min_gain")
            self.engine = SpecEngine(ecfg, SpecConfig(**{k: sc[k] for k in keys if k in sc}),
                                     model_cfg=mc)
            if sc.get("draft_path"):
                from safetensors.torch import load_file
                self.engine.draft.load(load_file(sc["draft_path"], device=str(self.engine.device)))
        else:
            self.engine = LLMEngine(ecfg, model_cfg=mc)
        self.tokenizer = load_tokenizer(c.get("tokenizer", ckpt or model_id), vocab_size=mc.vocab_size,
                                        bos=mc.bos_token_id, eos=mc.eos_token_id)
        self.device = device
        if c.get("warmup", False):
            self.engine.warmup()
            if spec and hasattr(self.engine, "warmup_spec"):
                # speculation graphs for the batch buckets this worker serves, at every depth
                sb = (spec if isinstance(spec, dict) else {}).get("graph_batches", (1, 2, 4, 8))
                self.engine.warmup_spec(tuple(sb))
        self.engine.first_token_hook = self._on_first_token
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name="dgi-engine", daemon=True)
        self._thread.start()
        self.loaded = True

    def unload_model(self) -> None:
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        self._thread = None
        self.engine = None
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        self.loaded = False

    # ------------------------------------------------------------------ engine thread
    def _loop(self) -> None:
        from dgi.sched.request import SamplingParams, Status
        eng = self.engine
        while not self._stop.is_set():
            while True:
                try:
                    prompt, p, cfg, imported = self._inbox.get_nowait()
                except queue.Empty:
                    break
                try:
                    sp = SamplingParams(max_tokens=cfg.max_tokens, temperature=cfg.temperature, top_p=cfg.top_p,
                                        top_k=cfg.top_k)
                    if imported is not None:       # decode phase of a cluster P/D job: KV pulled from its prefill worker
                        first, kv, seed = imported
                        p.req = eng.import_prefilled(prompt, first, kv, sp, seed=seed)
                        self.stats["kv_imported"] += 1
                        if p.stream_q is not None:
                            p.loop.call_soon_threadsafe(p.stream_q.put_nowait, first)
                        if p.req.status is Status.FINISHED:   # EOS / stop id / max_tokens at the first token
                            self._resolve(p, p.req)
                            continue
                    else:
                        p.req = eng.add_request(prompt, sp)
                    self._pending[p.req.rid] = p
                except Exception as e:  # prompt too long etc.
                    self._resolve_error(p, e)
            if not eng.has_unfinished():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                outs = eng.step()
            except Exception as e:  # pragma: no cover - surfaced to callers
                logger.exception("engine step failed")
                for p in list(self._pending.values()):
                    self._resolve_error(p, e)
                self._pending.clear()
                continue
            for o in outs:
                p = self._pending.get(o.rid)
                if p is None:
                    continue
                if p.stream_q is not None:
                    p.loop.call_soon_threadsafe(p.stream_q.put_nowait, o.token)
                if o.finished:
                    self._pending.pop(o.rid, None)
                    self._resolve(p, o.request)

    def _on_first_token(self, req) -> None:
        """Engine thread, first token of ``req`` sampled and its pages still held:
        a P/D prefill-phase request exports them for its decode worker.  Only the
        page gather is enqueued here (a fresh tensor, so the pages may be freed
        right after); the device-to-host copy waits on an event and the packing
        runs on the export thread, so the other sequences of the batch never wait
        for it (``KVExportStore.put_pending``)."""
        p = self._pending.get(req.rid)
        if p is None or p.export_key is None:
            return
        from dgi import ops
        from dgi.kv.transfer import pack_kv
        eng = self.engine
        mc = eng.model_cfg
        meta = {"prompt": list(req.prompt), "first_token": int(req.output[0]), "model": mc.name,
                "num_layers": mc.num_layers, "seed": int(req.seed)}
        nb = (req.num_computed + eng.pool.block_size - 1) // eng.pool.block_size
        ids = torch.tensor(req.blocks[:nb], dtype=torch.int32, device=eng.device)
        pages = ops.kv_gather(eng.pool.kv, ids)
        ev = None
        if pages.is_cuda:
            host = torch.empty(pages.shape, dtype=pages.dtype, pin_memory=True)
            host.copy_(pages, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host = pages

        def pack():
            if ev is not None:
                ev.synchronize()
            return pack_kv(host, meta)
        self.kv_exports.put_pending(p.export_key, self._export_pool().submit(pack), token=p.export_token)
        self.stats["kv_exported"] += 1

    def _export_pool(self):
        if getattr(self, "_exporter", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._exporter = ThreadPoolExecutor(max_workers=1, thread_name_prefix="kv-export")
        return self._exporter

    def _resolve(self, p: _Pending, req) -> None:
        text = self.tokenizer.decode(req.output, skip_special_tokens=True)
        res = GenerationResult(text=text, prompt_tokens=len(req.prompt), completion_tokens=len(req.output),
                               total_tokens=len(req.prompt) + len(req.output),
                               finish_reason="stop" if req.finish_reason == "stop" else "length",
                               cached_tokens=req.num_cached)
        self.stats["completed"] += 1

        def _set():
            if not p.future.done():
                p.future.set_result(res)
            if p.stream_q is not None:
                p.stream_q.put_nowait(None)
        p.loop.call_soon_threadsafe(_set)

    def _resolve_error(self, p: _Pending, e: Exception) -> None:
        self.stats["errors"] += 1

        def _set():
            if not p.future.done():
                p.future.set_exception(e)
            if p.stream_q is not None:
                p.stream_q.put_nowait(None)
        p.loop.call_soon_threadsafe(_set)

    def _submit(self, messages, cfg: GenerationConfig, stream: bool = False, export_key: Optional[str] = None,
                prompt: Optional[List[int]] = None, imported=None, export_token: Optional[str] = None) -> _Pending:
        if not self.loaded:
            raise RuntimeError("model not loaded")
        loop = asyncio.get_running_loop()
        if prompt is None:
            prompt = chat_prompt_ids(self.tokenizer, messages)
        p = _Pending(loop, loop.create_future(), asyncio.Queue() if stream else None, cfg, len(prompt), export_key,
                     export_token)
        self.stats["requests"] += 1
        self._inbox.put((prompt, p, cfg, imported))
        self._wake.set()
        return p

    # ------------------------------------------------------------------ cluster P/D (server services/pd_runtime.py)
    def prefill_export(self, params: Dict[str, Any], key: str) -> Dict[str, Any]:
        """Prefill phase: sample the first token and keep the sequence's KV pages under
        ``key`` (``kv_exports``) for the decode worker to pull (``GET /kv/{key}`` with
        the returned ``kv_token``, or straight from the store when the decode phase
        lands on this worker)."""
        from dgi.kv.transfer import new_token
        from .llm_base import generation_config_from_params, result_to_response
        cfg = generation_config_from_params({**params, "max_tokens": 1})
        token = new_token()

        async def run():
            return await self._submit(self._messages_of(params), cfg, export_key=key, export_token=token).future
        res = self._run_sync(run())
        out = result_to_response(res)
        out["kv_cache_key"] = key
        out["kv_token"] = token
        return out

    def decode_import(self, params: Dict[str, Any], blob: bytes) -> Dict[str, Any]:
        """Decode phase with the prefill worker's pages: no prompt recompute."""
        from dgi.kv.transfer import unpack_kv
        from .llm_base import generation_config_from_params, result_to_response
        kv, meta = unpack_kv(blob)
        if meta.get("model") not in (None, self.engine.model_cfg.name):
            raise ValueError(f"KV of model {meta.get('model')} offered to a {self.engine.model_cfg.name} engine")
        cfg = generation_config_from_params(params)

        seed = meta.get("seed")

        async def run():
            return await self._submit(None, cfg, prompt=list(meta["prompt"]),
                                      imported=(int(meta["first_token"]), kv, seed)).future
        return result_to_response(self._run_sync(run()))

    def _run_sync(self, coro):
        try:
            asyncio.get_running_loop()
        except RuntimeError:
            return asyncio.run(coro)
        return self._run_coroutine_in_new_thread(coro)

    # ------------------------------------------------------------------ LLMBaseEngine
    async def generate_async(self, messages: List[Dict[str, str]],
                             config: Optional[GenerationConfig] = None) -> GenerationResult:
        p = self._submit(messages, config or GenerationConfig())
        return await p.future

    async def batch_generate(self, batch_messages: List[List[Dict[str, str]]],
                             config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        cfg = config or GenerationConfig()
        ps = [self._submit(m, cfg) for m in batch_messages]
        return list(await asyncio.gather(*[p.future for p in ps]))

    async def stream_generate(self, messages: List[Dict[str, str]],
                              config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        p = self._submit(messages, config or GenerationConfig(), stream=True)
        dec = StreamDecoder(self.tokenizer)          # O(window) per token, multi-byte safe
        while True:
            t = await p.stream_q.get()
            if t is None:
                break
            piece = dec.add(t)
            if piece:
                yield piece
        tail = dec.flush()
        if tail:
            yield tail
        await p.future

    def batch_inference(self, params_list: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        try:
            asyncio.get_running_loop()
        except RuntimeError:
            return asyncio.run(self.batch_inference_async(params_list))
        return self._run_coroutine_in_new_thread(self.batch_inference_async(params_list))

    def supports_streaming(self) -> bool:
        return True

    def supports_prefix_caching(self) -> bool:
        return True

    def supports_batch_inference(self) -> bool:
        return True

    def get_status(self) -> Dict[str, Any]:
        s = super().get_status()
        s["features"] = ["paged_attention", "radix_attention", "continuous_batching", "chunked_prefill",
                         "streaming", "prefix_caching", "hipgraph_decode", "speculative_decoding"]
        if self.engine is not None:
            s["engine"] = {**self.engine.stats, **self.engine.scheduler.stats(),
                           "model": self.engine.model_cfg.name, "num_blocks": self.engine.pool.num_blocks,
                           "weights": getattr(self, "weights", "random-init")}
        s["stats"] = dict(self.stats)
        return s

    def get_cache_stats(self) -> Dict[str, Any]:
        if self.engine is None:
            return {}
        sch = self.engine.scheduler
        return {"prefix_hit_rate": sch.radix.hit_rate() if sch.radix else 0.0,
                "free_blocks": self.engine.pool.num_free, "used_blocks": self.engine.pool.num_used,
                "evictions": self.engine.pool.stats["evictions"]}


def _now() -> float:
    return time.perf_counter()
