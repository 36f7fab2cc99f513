"""Benchmark CLIs report the reference's result schemas (benchmarks/results.py).

Field lists are the reference's dataclasses (benchmarks/single_worker.py:38-73,
distributed.py:48-87, pd_separation.py:54-99, speculative.py:47-83); the
converters are fed a bench.py JSON line / a bench_spec row of the shapes the
GPU runs produce (profiles/), since bench.py itself needs a GPU."""
import dataclasses
import importlib.util
import os
import sys

# loaded by path: putting benchmarks/ on sys.path would shadow worker's flat ``distributed`` package
_spec = importlib.util.spec_from_file_location(
    "bench_results", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks",
                                  "results.py"))
R = importlib.util.module_from_spec(_spec)
sys.modules["bench_results"] = R          # dataclasses resolve their module through sys.modules
_spec.loader.exec_module(R)

REF_FIELDS = {
    "BenchmarkResult": "backend model_id total_tokens total_time_s tokens_per_second avg_ttft_ms p50_ttft_ms "
                       "p95_ttft_ms p99_ttft_ms avg_e2e_ms p50_e2e_ms p95_e2e_ms p99_e2e_ms gpu_memory_used_gb "
                       "gpu_memory_total_gb gpu_utilization_pct avg_batch_size total_requests prefix_cache_hit_rate",
    "DistributedBenchmarkResult": "model_id num_workers layers_per_worker total_requests successful_requests "
                                  "total_tokens total_time_s tokens_per_second avg_ttft_ms p50_ttft_ms p95_ttft_ms "
                                  "p99_ttft_ms avg_e2e_ms p50_e2e_ms p95_e2e_ms p99_e2e_ms avg_kv_transfer_ms "
                                  "total_kv_bytes_transferred avg_hop_latency_ms total_hops failover_tested "
                                  "avg_failover_time_ms failover_success_rate",
    "PDSeparationResult": "mode model_id prefill_workers decode_workers total_requests successful_requests "
                          "total_tokens total_time_s tokens_per_second avg_ttft_ms p50_ttft_ms p95_ttft_ms "
                          "p99_ttft_ms avg_tpot_ms p50_tpot_ms p95_tpot_ms avg_e2e_ms p50_e2e_ms p95_e2e_ms "
                          "avg_migration_ms migration_count migration_bytes avg_prefill_queue_time_ms "
                          "avg_decode_queue_time_ms max_prefill_queue_size max_decode_queue_size",
    "SpeculativeResult": "enabled model_id tree_depth tree_width num_speculative_tokens total_requests total_tokens "
                         "total_time_s avg_latency_ms p50_latency_ms p95_latency_ms p99_latency_ms avg_accept_rate "
                         "avg_tokens_per_step avg_speedup avg_draft_time_ms avg_verify_time_ms draft_overhead_pct "
                         "avg_effective_depth",
}


def test_result_records_match_reference_schemas():
    for name, fields in REF_FIELDS.items():
        got = [f.name for f in dataclasses.fields(getattr(R, name))]
        assert got == fields.split(), name


LAT = {"ttft": {"avg": 220.0, "p50": 214.0, "p95": 230.0, "p99": 240.0},
       "tpot": {"avg": 110.0, "p50": 108.0, "p95": 130.0, "p99": 140.0},
       "e2e": {"avg": 14000.0, "p50": 13900.0, "p95": 15000.0, "p99": 16000.0}, "requests_finished": 120}


def test_single_and_pd_converters():
    res = {"value": 1787.6, "steps": 30, "ms_per_step": 214.8, "config": {"model": "llama3-70b"},
           "latency_ms": LAT, "extra": {"engine": {"steps": 163, "decode_tokens": 37719, "prefill_tokens": 250368},
                                        "stats": {"prefix_hit_rate": 0.0}}}
    b = R.from_bench_single(res, gpu={"memory_used_gb": 270.0, "memory_total_gb": 288.0})
    assert b.tokens_per_second == 1787.6 and b.p99_ttft_ms == 240.0 and b.p95_e2e_ms == 15000.0
    assert b.total_requests == 120 and abs(b.avg_batch_size - (37719 + 250368) / 163) < 0.01
    pd = {**res, "extra": {"migration_ms_p50": 12.5, "ranks": [
        {"role": "prefill", "pd_scheduler": {"migrations": 40, "migration_bytes": 4 << 30, "prefill_queue_size": 0,
                                             "decode_queue_size": 0}},
        {"role": "decode_driver"}]}}
    r = R.from_bench_pd(pd, "separated", 5, 3)
    assert (r.prefill_workers, r.decode_workers, r.migration_count, r.avg_migration_ms) == (5, 3, 40, 12.5)
    assert r.p50_tpot_ms == 108.0
    d = R.from_bench_pipeline({**pd, "extra": {**pd["extra"], "ranks": pd["extra"]["ranks"] +
                                               [{"role": "decode_stage", "stage_steps": 95}]}}, 8, 80)
    assert d.layers_per_worker == 10 and d.total_hops == 95


def test_spec_converter():
    row = {"batch": 4, "plain_tok_s": 914.2, "spec_tok_s": 2086.5, "speedup": 2.282, "mean_accepted": 5.0,
           "tokens_per_step": 5.952, "draft_s": 0.013, "verify_s": 0.215, "controller": {"current_depth": 5}}
    on = R.from_spec_row(row, "llama3-8b", 5, 4, True, 128)
    off = R.from_spec_row(row, "llama3-8b", 5, 4, False, 128)
    assert on.avg_accept_rate == 1.0 and on.avg_speedup == 2.282 and on.avg_effective_depth == 5.0
    assert on.total_time_s < off.total_time_s and off.avg_tokens_per_step == 1.0
