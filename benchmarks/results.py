"""Result records of the benchmark CLIs, field for field the reference's schemas.

The reference defines ``BenchmarkResult`` (benchmarks/single_worker.py:38-73),
``DistributedBenchmarkResult`` (benchmarks/distributed.py:48-87),
``PDSeparationResult`` (benchmarks/pd_separation.py:54-99) and
``SpeculativeResult`` (benchmarks/speculative.py:47-83); its runs never
produced them with measured values (three of the four were ``asyncio.sleep``
simulators).  The converters below fill them from measured dgi
runs: ``bench.py``'s JSON line (latency distributions in ``latency_ms``,
per-role / migration extras) and ``scripts/bench_spec.py``'s rows.
Fields the MI355X runtime has no counterpart for are documented per record.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Any, Dict, Optional


def _l(res: dict, kind: str, stat: str) -> float:
    v = ((res.get("latency_ms") or {}).get(kind) or {}).get(stat)
    return float(v) if v is not None else 0.0


@dataclass
class BenchmarkResult:
    backend: str
    model_id: str
    total_tokens: int
    total_time_s: float
    tokens_per_second: float
    avg_ttft_ms: float
    p50_ttft_ms: float
    p95_ttft_ms: float
    p99_ttft_ms: float
    avg_e2e_ms: float
    p50_e2e_ms: float
    p95_e2e_ms: float
    p99_e2e_ms: float
    gpu_memory_used_gb: float
    gpu_memory_total_gb: float
    gpu_utilization_pct: float
    avg_batch_size: float
    total_requests: int
    prefix_cache_hit_rate: Optional[float] = None

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


@dataclass
class DistributedBenchmarkResult:
    model_id: str
    num_workers: int
    layers_per_worker: int
    total_requests: int
    successful_requests: int
    total_tokens: int
    total_time_s: float
    tokens_per_second: float
    avg_ttft_ms: float
    p50_ttft_ms: float
    p95_ttft_ms: float
    p99_ttft_ms: float
    avg_e2e_ms: float
    p50_e2e_ms: float
    p95_e2e_ms: float
    p99_e2e_ms: float
    avg_kv_transfer_ms: float
    total_kv_bytes_transferred: int
    avg_hop_latency_ms: float
    total_hops: int
    failover_tested: bool = False
    avg_failover_time_ms: float = 0.0
    failover_success_rate: float = 0.0

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


@dataclass
class PDSeparationResult:
    mode: str
    model_id: str
    prefill_workers: int
    decode_workers: int
    total_requests: int
    successful_requests: int
    total_tokens: int
    total_time_s: float
    tokens_per_second: float
    avg_ttft_ms: float
    p50_ttft_ms: float
    p95_ttft_ms: float
    p99_ttft_ms: float
    avg_tpot_ms: float
    p50_tpot_ms: float
    p95_tpot_ms: float
    avg_e2e_ms: float
    p50_e2e_ms: float
    p95_e2e_ms: float
    avg_migration_ms: float = 0.0
    migration_count: int = 0
    migration_bytes: int = 0
    avg_prefill_queue_time_ms: float = 0.0
    avg_decode_queue_time_ms: float = 0.0
    max_prefill_queue_size: int = 0
    max_decode_queue_size: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


@dataclass
class SpeculativeResult:
    enabled: bool
    model_id: str
    tree_depth: int
    tree_width: int
    num_speculative_tokens: int
    total_requests: int
    total_tokens: int
    total_time_s: float
    avg_latency_ms: float
    p50_latency_ms: float
    p95_latency_ms: float
    p99_latency_ms: float
    avg_accept_rate: float
    avg_tokens_per_step: float
    avg_speedup: float
    avg_draft_time_ms: float
    avg_verify_time_ms: float
    draft_overhead_pct: float
    avg_effective_depth: float = 0.0

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


# ----------------------------------------------------------------------------- converters

def from_bench_single(res: dict, backend: str = "mi355x", gpu: Optional[dict] = None) -> BenchmarkResult:
    """``bench.py`` single/dp run -> BenchmarkResult.  ``gpu``: memory / utilisation
    sampled by the caller (``gpu_stats``); batch size = scheduled rows per step."""
    ex = res.get("extra", {})
    eng = ex.get("engine", {})
    steps = max(1, int(eng.get("steps", 0) or 1))
    rows = (eng.get("decode_tokens", 0) or 0) + (eng.get("prefill_tokens", 0) or 0)
    el = res["steps"] * res["ms_per_step"] / 1000.0
    g = gpu or {}
    return BenchmarkResult(
        backend=backend, model_id=res["config"]["model"], total_tokens=int(round(res["value"] * el)),
        total_time_s=round(el, 4), tokens_per_second=res["value"],
        avg_ttft_ms=_l(res, "ttft", "avg"), p50_ttft_ms=_l(res, "ttft", "p50"), p95_ttft_ms=_l(res, "ttft", "p95"),
        p99_ttft_ms=_l(res, "ttft", "p99"), avg_e2e_ms=_l(res, "e2e", "avg"), p50_e2e_ms=_l(res, "e2e", "p50"),
        p95_e2e_ms=_l(res, "e2e", "p95"), p99_e2e_ms=_l(res, "e2e", "p99"),
        gpu_memory_used_gb=float(g.get("memory_used_gb", 0.0)), gpu_memory_total_gb=float(g.get("memory_total_gb", 0.0)),
        gpu_utilization_pct=float(g.get("utilization_pct", 0.0)), avg_batch_size=round(rows / steps, 2),
        total_requests=int((res.get("latency_ms") or {}).get("requests_finished", 0)),
        prefix_cache_hit_rate=(ex.get("stats") or {}).get("prefix_hit_rate"))


def from_bench_pipeline(res: dict, num_workers: int, num_layers: int) -> DistributedBenchmarkResult:
    """``bench.py --layout pp|pdpp`` -> DistributedBenchmarkResult.  Hops are the
    pipeline's stage-to-stage transfers (RCCL p2p); KV transfer fields come from
    P/D migrations when the layout has prefill ranks."""
    ex = res.get("extra", {})
    el = res["steps"] * res["ms_per_step"] / 1000.0
    ranks = ex.get("ranks", [])
    stage_steps = sum(int(r.get("stage_steps", 0) or 0) for r in ranks)
    pre = [r for r in ranks if r.get("role") == "prefill"]
    kv_bytes = int(sum(float(r.get("sent_GB", 0.0)) * 1e9 for r in pre))
    n_fin = int((res.get("latency_ms") or {}).get("requests_finished", 0))
    return DistributedBenchmarkResult(
        model_id=res["config"]["model"], num_workers=num_workers, layers_per_worker=num_layers // max(1, num_workers),
        total_requests=n_fin, successful_requests=n_fin, total_tokens=int(round(res["value"] * el)),
        total_time_s=round(el, 4), tokens_per_second=res["value"], avg_ttft_ms=_l(res, "ttft", "avg"),
        p50_ttft_ms=_l(res, "ttft", "p50"), p95_ttft_ms=_l(res, "ttft", "p95"), p99_ttft_ms=_l(res, "ttft", "p99"),
        avg_e2e_ms=_l(res, "e2e", "avg"), p50_e2e_ms=_l(res, "e2e", "p50"), p95_e2e_ms=_l(res, "e2e", "p95"),
        p99_e2e_ms=_l(res, "e2e", "p99"), avg_kv_transfer_ms=float(ex.get("migration_ms_p50") or 0.0),
        total_kv_bytes_transferred=kv_bytes,
        avg_hop_latency_ms=round(res["ms_per_step"] / max(1, num_workers), 3), total_hops=stage_steps)


def from_bench_pd(res: dict, mode: str, prefill: int, decode: int) -> PDSeparationResult:
    ex = res.get("extra", {})
    el = res["steps"] * res["ms_per_step"] / 1000.0
    ranks = ex.get("ranks", [])
    pre = [r for r in ranks if r.get("role") == "prefill"]
    sched = [r.get("pd_scheduler") or {} for r in pre]
    n_fin = int((res.get("latency_ms") or {}).get("requests_finished", 0))
    return PDSeparationResult(
        mode=mode, model_id=res["config"]["model"], prefill_workers=prefill, decode_workers=decode,
        total_requests=n_fin, successful_requests=n_fin, total_tokens=int(round(res["value"] * el)),
        total_time_s=round(el, 4), tokens_per_second=res["value"], avg_ttft_ms=_l(res, "ttft", "avg"),
        p50_ttft_ms=_l(res, "ttft", "p50"), p95_ttft_ms=_l(res, "ttft", "p95"), p99_ttft_ms=_l(res, "ttft", "p99"),
        avg_tpot_ms=_l(res, "tpot", "avg"), p50_tpot_ms=_l(res, "tpot", "p50"), p95_tpot_ms=_l(res, "tpot", "p95"),
        avg_e2e_ms=_l(res, "e2e", "avg"), p50_e2e_ms=_l(res, "e2e", "p50"), p95_e2e_ms=_l(res, "e2e", "p95"),
        avg_migration_ms=float(ex.get("migration_ms_p50") or 0.0),
        migration_count=int(sum(int(s.get("migrations", 0)) for s in sched)),
        migration_bytes=int(sum(int(s.get("migration_bytes", 0)) for s in sched)),
        max_prefill_queue_size=int(max([s.get("prefill_queue_size", 0) for s in sched] or [0])),
        max_decode_queue_size=int(max([s.get("decode_queue_size", 0) for s in sched] or [0])))


def from_spec_row(row: dict, model: str, depth: int, width: int, enabled: bool = True,
                  output_len: int = 128) -> SpeculativeResult:
    """One ``scripts/bench_spec.py`` row (batch B) -> SpeculativeResult: latency is
    the per-request generation time of the batch (B requests decode together)."""
    B = int(row["batch"])
    tps = row["spec_tok_s"] if enabled else row["plain_tok_s"]
    toks = B * output_len
    t = toks / max(tps, 1e-9)
    lat = t * 1000.0
    steps = max(1e-9, toks / max(row.get("tokens_per_step", 1.0), 1e-9) / max(1, B))
    draft_ms = row.get("draft_s", 0.0) * 1000.0 / steps if enabled else 0.0
    verify_ms = row.get("verify_s", 0.0) * 1000.0 / steps if enabled else 0.0
    return SpeculativeResult(
        enabled=enabled, model_id=model, tree_depth=depth, tree_width=width, num_speculative_tokens=depth,
        total_requests=B, total_tokens=toks, total_time_s=round(t, 4), avg_latency_ms=round(lat, 2),
        p50_latency_ms=round(lat, 2), p95_latency_ms=round(lat, 2), p99_latency_ms=round(lat, 2),
        avg_accept_rate=round(row.get("mean_accepted", 0.0) / max(1, depth), 4) if enabled else 0.0,
        avg_tokens_per_step=row.get("tokens_per_step", 1.0) if enabled else 1.0,
        avg_speedup=row.get("speedup", 1.0) if enabled else 1.0, avg_draft_time_ms=round(draft_ms, 3),
        avg_verify_time_ms=round(verify_ms, 3),
        draft_overhead_pct=round(100.0 * draft_ms / max(1e-9, draft_ms + verify_ms), 2) if enabled else 0.0,
        avg_effective_depth=float((row.get("controller") or {}).get("current_depth", depth)) if enabled else 0.0)


def gpu_stats() -> dict:
    """Device memory of this process's GPU (utilisation needs amd-smi; 0 when absent)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return {}
        free, total = torch.cuda.mem_get_info()
        return {"memory_used_gb": round((total - free) / 2 ** 30, 2), "memory_total_gb": round(total / 2 ** 30, 2)}
    except Exception:
        return {}
