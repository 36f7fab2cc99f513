"""Worker configuration: env > config.yaml > defaults (reference worker/config.py:12-213).

Same env keys (``GPU_SERVER_URL``, ``GPU_REGION``, ``GPU_SUPPORTED_TYPES``,
``GPU_LLM_MODEL`` …) and YAML layout.  MI355X additions: the ``llm`` engine
defaults to the native ``dgi`` backend, ``gpu.device_ids`` lists the GPUs
this worker drives and ``gpu.layout`` picks the in-node layout
(``single`` | ``pd`` | ``pdpp`` | ``pp``) for multi-GPU engines.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional

import yaml
from pydantic import BaseModel, Field

_TRUE = ("1", "true", "yes", "on")


def get_env(key: str, default: Any = None, cast: type = str) -> Any:
    raw = os.environ.get(key)
    if raw is None:
        return default
    if cast is bool:
        return raw.strip().lower() in _TRUE
    if cast is list:
        return [p.strip() for p in raw.split(",") if p.strip()]
    try:
        return cast(raw)
    except (TypeError, ValueError):
        return default


def _env(key: str, default: Any = None, cast: type = str) -> Callable[[], Any]:
    return lambda: get_env(key, default, cast)


class ServerConfig(BaseModel):
    url: str = Field(default_factory=_env("GPU_SERVER_URL", "http://localhost:8000"))
    timeout: int = Field(default_factory=_env("GPU_SERVER_TIMEOUT", 30, int))
    verify_ssl: bool = Field(default_factory=_env("GPU_SERVER_VERIFY_SSL", True, bool))


class GPUConfig(BaseModel):
    enable_cpu_offload: bool = Field(default_factory=_env("GPU_ENABLE_CPU_OFFLOAD", False, bool))
    max_memory_gb: Optional[float] = Field(default_factory=_env("GPU_MAX_MEMORY_GB", None, float))
    device_id: int = Field(default_factory=_env("GPU_DEVICE_ID", 0, int))
    device_ids: List[int] = Field(default_factory=lambda: [int(x) for x in get_env("GPU_DEVICE_IDS", [], list)])
    layout: str = Field(default_factory=_env("GPU_LAYOUT", "single"))


class DirectConfig(BaseModel):
    enabled: bool = Field(default_factory=_env("GPU_DIRECT_ENABLED", False, bool))
    host: str = Field(default_factory=_env("GPU_DIRECT_HOST", "0.0.0.0"))
    port: int = Field(default_factory=_env("GPU_DIRECT_PORT", 8080, int))
    public_url: Optional[str] = Field(default_factory=_env("GPU_DIRECT_PUBLIC_URL", None))


class LoadControlConfig(BaseModel):
    acceptance_rate: float = Field(default_factory=_env("GPU_ACCEPTANCE_RATE", 1.0, float))
    # a dgi engine batches continuously, so many jobs can be in flight at once
    max_concurrent_jobs: int = Field(default_factory=_env("GPU_MAX_CONCURRENT_JOBS", 64, int))
    max_jobs_per_hour: int = Field(default_factory=_env("GPU_MAX_JOBS_PER_HOUR", 0, int))
    working_hours_start: Optional[int] = Field(default_factory=_env("GPU_WORKING_HOURS_START", None, int))
    working_hours_end: Optional[int] = Field(default_factory=_env("GPU_WORKING_HOURS_END", None, int))


# ---------------------------------------------------------------------------
# v2.0 sections documented by the reference README (README.md:815-910) but
# never parsed there; here they are typed and feed the engines.
# ---------------------------------------------------------------------------

class BatchConfig(BaseModel):
    max_batch_size: int = 32
    max_wait_ms: float = 50.0


class NativeRuntimeConfig(BaseModel):
    """``dgi`` runtime knobs (``DGI_*`` env > yaml ``inference.native`` > defaults)."""
    block_size: int = Field(default_factory=_env("DGI_BLOCK_SIZE", 16, int))
    max_num_seqs: int = Field(default_factory=_env("DGI_MAX_NUM_SEQS", 256, int))
    max_num_batched_tokens: int = Field(default_factory=_env("DGI_MAX_BATCHED_TOKENS", 8192, int))
    graph_batch_buckets: List[int] = Field(
        default_factory=lambda: [int(x) for x in get_env("DGI_GRAPH_BATCH_BUCKETS", [], list)])
    kv_fraction: float = Field(default_factory=_env("DGI_KV_FRACTION", 0.9, float))
    # pinned host KV tier (GB): < 0 = auto (half the HBM KV pool, capped by host RAM), 0 = off
    cpu_tier_gb: float = Field(default_factory=_env("DGI_CPU_TIER_GB", -1.0, float))
    pp: int = Field(default_factory=_env("DGI_PP", 1, int))
    pd: Optional[str] = Field(default_factory=_env("DGI_PD", None))          # "P:D", e.g. "6:2"
    spec: Optional[str] = Field(default_factory=_env("DGI_SPEC", None))      # "eagle3"


class InferenceConfig(BaseModel):
    engine: Optional[str] = None        # llm | llm_native | llm_sglang | llm_vllm | llm_vllm_async
    sglang: Dict[str, Any] = Field(default_factory=dict)
    vllm: Dict[str, Any] = Field(default_factory=dict)
    batch: BatchConfig = Field(default_factory=BatchConfig)
    native: NativeRuntimeConfig = Field(default_factory=NativeRuntimeConfig)


class ModelShardSection(BaseModel):
    model_id: Optional[str] = None
    start_layer: int = 0
    end_layer: Optional[int] = None


class GrpcSection(BaseModel):
    host: str = "0.0.0.0"
    port: int = 50051


class KVCacheSection(BaseModel):
    gpu_cache_size_gb: float = 4.0
    cpu_cache_size_gb: float = 16.0
    enable_redis: bool = False
    redis_url: str = "redis://localhost:6379"


class DistributedConfig(BaseModel):
    enabled: bool = False
    role: str = "hybrid"                # prefill | decode | hybrid
    model_shard: ModelShardSection = Field(default_factory=ModelShardSection)
    grpc: GrpcSection = Field(default_factory=GrpcSection)
    kv_cache: KVCacheSection = Field(default_factory=KVCacheSection)


class SpeculativeSection(BaseModel):
    enabled: bool = False
    num_speculative_tokens: int = 5
    tree_width: int = 3
    tree_depth: int = 5
    adaptive_depth: bool = True
    min_accept_rate: float = 0.3
    draft_path: Optional[str] = None    # trained EAGLE-3 draft (safetensors)


class MetricsSection(BaseModel):
    enabled: bool = True
    port: int = 9090


class TracingSection(BaseModel):
    enabled: bool = False
    exporter: str = "otlp"              # otlp | console
    endpoint: Optional[str] = None
    sample_rate: float = 1.0


class ObservabilityConfig(BaseModel):
    metrics: MetricsSection = Field(default_factory=MetricsSection)
    tracing: TracingSection = Field(default_factory=TracingSection)


_ENGINE_ALIASES = {"llm": "native", "llm_native": "mi355x", "llm_sglang": "sglang", "llm_vllm": "vllm",
                   "llm_vllm_async": "vllm_async"}


class WorkerConfig(BaseModel):
    worker_id: Optional[str] = Field(default_factory=_env("GPU_WORKER_ID", None))
    token: Optional[str] = Field(default_factory=_env("GPU_WORKER_TOKEN", None))
    refresh_token: Optional[str] = Field(default_factory=_env("GPU_WORKER_REFRESH_TOKEN", None))
    signing_secret: Optional[str] = Field(default_factory=_env("GPU_WORKER_SIGNING_SECRET", None))
    name: Optional[str] = Field(default_factory=_env("GPU_WORKER_NAME", None))
    role: str = Field(default_factory=_env("GPU_WORKER_ROLE", "hybrid"))
    region: str = Field(default_factory=_env("GPU_REGION", "asia-east"))
    country: Optional[str] = Field(default_factory=_env("GPU_COUNTRY", None))
    city: Optional[str] = Field(default_factory=_env("GPU_CITY", None))
    timezone: Optional[str] = Field(default_factory=_env("GPU_TIMEZONE", None))
    server: ServerConfig = Field(default_factory=ServerConfig)
    gpu: GPUConfig = Field(default_factory=GPUConfig)
    direct: DirectConfig = Field(default_factory=DirectConfig)
    load_control: LoadControlConfig = Field(default_factory=LoadControlConfig)
    supported_types: List[str] = Field(default_factory=_env("GPU_SUPPORTED_TYPES", ["llm"], list))
    engines: Dict[str, Dict[str, Any]] = Field(default_factory=dict)
    heartbeat_interval: int = Field(default_factory=_env("GPU_HEARTBEAT_INTERVAL", 30, int))
    poll_interval: float = Field(default_factory=_env("GPU_POLL_INTERVAL", 2.0, float))
    # long-poll the next-job endpoint for up to this many seconds (0: plain polling every
    # poll_interval); a job then reaches an idle worker as soon as it is queued
    long_poll_s: float = Field(default_factory=_env("GPU_LONG_POLL_S", 5.0, float))
    inference: InferenceConfig = Field(default_factory=InferenceConfig)
    distributed: DistributedConfig = Field(default_factory=DistributedConfig)
    speculative: SpeculativeSection = Field(default_factory=SpeculativeSection)
    observability: ObservabilityConfig = Field(default_factory=ObservabilityConfig)

    def save(self, path: str = "config.yaml") -> None:
        with open(path, "w", encoding="utf-8") as f:
            yaml.safe_dump(self.model_dump(), f, default_flow_style=False, allow_unicode=True, sort_keys=False)

    @classmethod
    def from_env(cls) -> "WorkerConfig":
        return cls()

    def engine_config(self, engine_type: str) -> Dict[str, Any]:
        cfg = dict(DEFAULT_ENGINE_CONFIGS.get(engine_type, {}))
        cfg.update(self.engines.get(engine_type, {}))
        cfg.setdefault("enable_cpu_offload", self.gpu.enable_cpu_offload)
        if self.gpu.device_ids:
            cfg.setdefault("device_ids", list(self.gpu.device_ids))
        cfg.setdefault("layout", self.gpu.layout)
        if engine_type == "llm":
            self._apply_llm_sections(cfg)
        return cfg

    def _apply_llm_sections(self, cfg: Dict[str, Any]) -> None:
        inf = self.inference
        if inf.engine and "backend" not in self.engines.get("llm", {}):
            cfg["backend"] = _ENGINE_ALIASES.get(inf.engine, inf.engine)
        for k in ("sglang", "vllm"):
            d = getattr(inf, k)
            if d:
                cfg[k] = {**d, **cfg.get(k, {})}
        n = inf.native
        native = {"block_size": n.block_size, "max_num_seqs": n.max_num_seqs,
                  "max_num_batched_tokens": n.max_num_batched_tokens, "kv_fraction": n.kv_fraction,
                  "host_kv_gb": n.cpu_tier_gb}
        if n.graph_batch_buckets:
            native["graph_batch_buckets"] = list(n.graph_batch_buckets)
        cfg["native"] = {**native, **cfg.get("native", {})}
        if n.pd:
            cfg.setdefault("layout", "pdpp" if n.pp > 1 else "pd")
            cfg["prefill_ranks"] = int(n.pd.split(":")[0])
        elif n.pp > 1:
            cfg["layout"] = "pp"
        sp = self.speculative
        if (sp.enabled or (n.spec or "").lower() == "eagle3") and "speculative" not in cfg:
            cfg["speculative"] = {"depth": sp.tree_depth, "width": sp.tree_width,
                                  "topk": max(sp.tree_width, 1), "adaptive_depth": sp.adaptive_depth,
                                  "min_accept_rate": sp.min_accept_rate,
                                  **({"draft_path": sp.draft_path} if sp.draft_path else {})}
        d = self.distributed
        if d.enabled:
            cfg["distributed"] = d.model_dump()


def load_dotenv(path: str = ".env") -> None:
    """Populate ``os.environ`` from a .env file without overriding variables that are already set."""
    p = Path(path)
    if not p.is_file():
        return
    for line in p.read_text(encoding="utf-8").splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        k = k.strip()
        if k.startswith("export "):
            k = k[7:].strip()
        v = v.strip()
        if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
            v = v[1:-1]
        os.environ.setdefault(k, v)


_SECTIONS = {"server": ServerConfig, "gpu": GPUConfig, "direct": DirectConfig, "load_control": LoadControlConfig,
             "inference": InferenceConfig, "distributed": DistributedConfig, "speculative": SpeculativeSection,
             "observability": ObservabilityConfig}


def load_config(path: str = "config.yaml") -> WorkerConfig:
    load_dotenv()
    p = Path(path)
    data: Dict[str, Any] = {}
    if p.is_file():
        data = yaml.safe_load(p.read_text(encoding="utf-8")) or {}
    for key, model in _SECTIONS.items():
        if isinstance(data.get(key), dict):
            data[key] = model(**data[key])
    cfg = WorkerConfig(**data)
    _load_engine_configs_from_env(cfg)
    return cfg


_ENGINE_ENV = {"llm": "GPU_LLM_MODEL", "image_gen": "GPU_IMAGE_MODEL", "vision": "GPU_VISION_MODEL",
               "whisper": "GPU_WHISPER_MODEL", "embedding": "GPU_EMBEDDING_MODEL"}


def _load_engine_configs_from_env(config: WorkerConfig) -> None:
    for engine_type, key in _ENGINE_ENV.items():
        model = get_env(key)
        if model:
            config.engines.setdefault(engine_type, {})["model_id"] = model
    backend = get_env("GPU_LLM_BACKEND")
    if backend:
        config.engines.setdefault("llm", {})["backend"] = backend


DEFAULT_ENGINE_CONFIGS: Dict[str, Dict[str, Any]] = {
    "llm": {"model_id": "llama3-8b", "backend": "mi355x", "max_new_tokens": 2048, "temperature": 0.7,
            "max_num_seqs": 256, "max_num_batched_tokens": 8192},
    "image_gen": {"model_id": "stabilityai/sdxl-turbo", "default_steps": 4, "default_width": 1024,
                  "default_height": 1024},
    "vision": {"model_id": "Qwen/Qwen2-VL-7B-Instruct", "max_new_tokens": 1024},
    "whisper": {"model_id": "openai/whisper-large-v3"},
    "embedding": {"model_id": "BAAI/bge-large-zh-v1.5"},
}
