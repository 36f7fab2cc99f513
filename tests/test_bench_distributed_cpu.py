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
    assert d["tpot_p50_ms"] is not None and d["tpot_p50_ms"] > 0     # in-window inter-token times
    _check_metric_fields(d)


def test_window_tpot_counts_unfinished_requests():
    """TPOT samples come from every request with >= 2 tokens inside the window, finished or not
    (a 20-step window is shorter than one 128-token generation on the 8-GPU layouts)."""
    import types
    from dgi.parallel.bench_dist import _window_tpots
    a = types.SimpleNamespace(token_times=[0.0, 1.0, 2.0, 3.0, 4.0])       # running, 3 in window
    b = types.SimpleNamespace(token_times=[1.5, 5.0])                       # one token in window
    c = types.SimpleNamespace(token_times=[2.0, 2.5, 3.5])                  # all in window
    got = _window_tpots([a, b, c], 1.0, 3.6)
    assert got == [1.0, 0.75]


def _check_metric_fields(d):
    """metric / metric_scope / vs_baseline agree with config.parallelism."""
    sys.path.insert(0, ROOT)
    from bench import HEADLINE_METRIC
    kind = d["config"]["parallelism"].rstrip("0123456789")
    n = d["n_gpus"]
    assert d["config"]["parallelism"] == f"{kind}{n}"
    headline = n == 8 and d["config"]["model"] == "llama3-70b" and kind in ("pd", "pdpp")
    if headline:
        assert d["metric"] == HEADLINE_METRIC and d["metric_scope"].startswith("headline")
        assert d["vs_baseline"] is not None
    else:
        assert d["metric"].startswith(HEADLINE_METRIC + " [this run: ") and d["vs_baseline"] is None
        assert not d["metric_scope"].startswith("headline")
        assert f"{n}-GPU" in d["metric_scope"]
        if kind not in ("pd", "pdpp"):
            assert "not the P/D-split headline layout" in d["metric"]


def test_metric_fields_match_the_layout():
    sys.path.insert(0, ROOT)
    from bench import HEADLINE_METRIC, metric_fields
    h = metric_fields(8, "pdpp", "llama3-70b", "5P+1D[pp3]")
    assert h["headline"] and h["metric"] == HEADLINE_METRIC
    for world, kind, model in ((8, "dp", "llama3-70b"), (1, "single", "llama3-70b"), (8, "pd", "llama3-8b"),
                               (4, "pdpp", "llama3-70b")):
        m = metric_fields(world, kind, model)
        assert not m["headline"] and m["metric"] != HEADLINE_METRIC and m["metric"].startswith(HEADLINE_METRIC)
        assert (kind in ("pd", "pdpp")) == ("not the P/D-split" not in m["metric"])


def test_stalled_pair_warmup_ends_the_run_with_a_timeout_line():
    """a rank wedged in pair warm-up (``DGI_FAULT`` stall at the phase's
    site) ends the run within the phase budget: ONE JSON line with status "timeout",
    the stuck phase per rank, and a non-zero exit — not a lease-long hang."""
    import time
    env = {**os.environ, "OMP_NUM_THREADS": "1", "DGI_PHASE_S": "6", "DGI_FAULT": "1:300001:stall:120"}
    env.pop("DGI_STAGED_GPU", None)
    env.pop("DGI_WATCHDOG", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--model", "llama-tiny", "--steps", "4", "--warmup", "1", "--ramp-steps", "2", "--concurrency", "8",
           "--output-len", "8", "--prompt-len", "32", "--max-batched-tokens", "256", "--layout", "pd",
           "--prefill-ranks", "1", "--decode-replicas", "1"]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    took = time.time() - t0
    assert r.returncode != 0
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"status"' in x]
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-2000:]
    d = lines[0]
    assert d["status"] == "timeout" and d["value"] is None and d["n_gpus"] == 2
    assert d["stuck"]["phase"] == "pair_warmup"
    assert d["phases"]["1"]["phase"] == "pair_warmup"
    assert d["metric"].startswith("output tokens/sec")
    assert took < 100, took


def test_pd_separation_cli_runs_config4_as_2p_6d(tmp_path):
    """BASELINE config #4: ``benchmarks/pd_separation.py --prefill-workers 2
    --decode-workers 6`` is 2 prefill GPUs + 6 single-GPU decode replicas (8 gloo
    ranks here), reported in the reference's PDSeparationResult schema."""
    env = {**os.environ, "OMP_NUM_THREADS": "1", "DGI_WATCHDOG": "0"}
    env.pop("DGI_STAGED_GPU", None)
    out = tmp_path / "pd.json"
    cmd = [sys.executable, "benchmarks/pd_separation.py", "--model", "llama-tiny", "--prefill-workers", "2",
           "--decode-workers", "6", "--steps", "3", "--warmup", "1", "--max-tokens", "8", "--prompt-length", "32",
           "--concurrent", "8", "--output", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())["separated"]
    assert d["prefill_workers"] == 2 and d["decode_workers"] == 6 and d["tokens_per_second"] > 0
    assert "2P+6D[1+1+1+1+1+1]" in r.stdout + r.stderr or d["mode"] == "separated"


@pytest.mark.parametrize("n,args", [
    (3, ["--layout", "pdpp", "--prefill-ranks", "1", "--decode-stages", "2", "--decode-local-frac", "0.3"]),
    (3, ["--layout", "pd", "--prefill-ranks", "2", "--decode-replicas", "1", "--prefill-local-cap", "4"]),
    (2, ["--layout", "pp"]),
])
def test_bench_window_counts_exactly_the_tokens_inside_it(n, args):
    """Timestamp window (dgi.parallel.bench_dist): every rank keeps serving across
    both edges and counts the tokens it produced inside [t0, t1].  The reported
    total equals an independent recount from the requests' own token timestamps,
    the rate is that total over t1 - t0, and prefill ranks step inside it."""
    env = {**os.environ, "OMP_NUM_THREADS": "1", "DGI_WATCHDOG": "0", "DGI_BENCH_RECOUNT": "1"}
    env.pop("DGI_STAGED_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(n),
           "--model", "llama-tiny", "--steps", "20", "--warmup", "2", "--ramp-steps", "4", "--concurrency", "8",
           "--output-len", "4", "--prompt-len", "32", "--max-batched-tokens", "256", *args]
    # (20 node steps: on a loaded host a 12-step window could close before a credit-starved
    # prefill rank got its next step in)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric"')][-1])
    ranks = d["extra"]["ranks"]
    total = sum(int(o.get("tokens", 0)) for o in ranks)
    assert total > 0
    win = d["steps"] * d["ms_per_step"] / 1000.0
    assert abs(d["value"] * win - total) <= 0.02 * total + 1
    if args[1] == "pp":
        drv = [o for o in ranks if o["role"] == "decode_driver"][0]
        assert drv["micro_per_step"] >= 2
        return
    for o in ranks:
        if o["role"] in ("prefill", "decode_driver"):
            assert o["recount"] == o["tokens"], o
    pre = [o for o in ranks if o["role"] == "prefill"]
    assert sum(o["prefill_steps_in_window"] for o in pre) >= 1       # (a credit-starved rank may idle)
    drv = [o for o in ranks if o["role"] == "decode_driver"][0]
    assert drv["micro_steps_in_window"] >= d["steps"] * drv["micro_per_step"] - 1


def test_node_step_covers_one_prefill_step():
    """A P/D node step is enough decode micro-steps of the clock replica to cover one
    prefill step: from the measured times when the prefill ranks reported them, else
    from the capacity table, never less than one pipeline round."""
    sys.path.insert(0, ROOT)
    from dgi.parallel.bench_dist import node_step_micro
    from dgi.parallel.plan import CAPACITY
    cap = CAPACITY["llama3-70b"]
    assert node_step_micro(cap, 3, 3) == 6                       # 201.5 ms / 39.6 ms -> 6
    assert node_step_micro(cap, 3, 3, prefill_ms=500.0, micro_ms=40.0) == 13
    assert node_step_micro(cap, 3, 3, prefill_ms=50.0, micro_ms=40.0) == 3   # one pipeline round at least
    assert node_step_micro(None, 1, 1) == 1


def test_bench_auto_layout_plans_from_the_startup_probe():
    """--layout auto on 2 gloo ranks with the start-up probe forced on: every rank probes,
    the ranks agree on one plan from the median capacity, the run completes, and the
    JSON carries the planner's source and reason."""
    env = {**os.environ, "OMP_NUM_THREADS": "1", "DGI_WATCHDOG": "0", "DGI_PROBE": "1"}
    env.pop("DGI_STAGED_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--model", "llama-tiny", "--steps", "4", "--warmup", "1", "--ramp-steps", "2", "--concurrency", "8",
           "--output-len", "8", "--prompt-len", "32", "--max-batched-tokens", "256"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric"')][-1])
    pl = d["extra"]["planner"]
    assert pl["source"] == "probe" and pl["kind"] in ("dp", "pd", "pdpp") and pl["reason"]
    assert d["value"] > 0 and "auto:" in d["metric_scope"]


def test_dp_run_after_the_probe_enters_its_own_phases(monkeypatch):
    """``--layout auto`` resolving to dp used to leave the probe's
    120 s deadline armed over the whole DP engine build and serving window, so the
    watchdog killed a healthy 70B DP run.  ``run_single`` now enters ``engine_build``,
    then ``serve`` with a budget sized from the run's steps, then ``report``."""
    sys.path.insert(0, ROOT)
    import bench
    from dgi.parallel import fault

    seen = []

    class _WD:
        rank = 0

        def phase(self, name, budget_s=None):
            seen.append((name, budget_s))

    monkeypatch.setattr(fault, "_WATCHDOG", [_WD()])
    monkeypatch.setattr(sys, "argv", ["bench.py", "--model", "llama-tiny", "--steps", "3", "--warmup", "1",
                                      "--ramp-steps", "2", "--concurrency", "4", "--output-len", "4",
                                      "--prompt-len", "16", "--max-batched-tokens", "128", "--no-graphs"])
    res = bench.run_single(bench.parse())
    assert res["tokens"] > 0
    names = [n for n, _ in seen]
    assert names == ["engine_build", "serve", "report"], seen
    assert seen[0][1] == fault.BUILD_S
    assert seen[1][1] >= fault.SERVE_FLOOR_S
    assert fault.serve_budget(10_000, step_s=0.5) == 15_000      # scales with the steps past the floor


def test_distributed_serve_budget_scales_with_steps():
    """the P/D serving deadline grows with --steps / --warmup."""
    import types
    from dgi.parallel.bench_dist import dist_serve_budget
    from dgi.parallel.fault import SERVE_FLOOR_S
    small = types.SimpleNamespace(ramp_steps=-1, output_len=128, warmup=10, steps=20)
    big = types.SimpleNamespace(ramp_steps=-1, output_len=128, warmup=10, steps=2000)
    assert dist_serve_budget(small) >= SERVE_FLOOR_S
    assert dist_serve_budget(big) > 3 * 8 * 2000 * 0.25 - 1
