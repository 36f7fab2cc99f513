"""Multi-rank runtime on the GPU ("staged": all ranks share one MI355X, the data
plane is gloo through host memory, compute is the HIP path).

Covers the GPU-only parts the CPU suite cannot: stage hipGraph replay of
decode micro-steps (pipeline.StageGraphs), padded decode microbatches,
top-k/top-p sampling inside the last stage's graph, and P/D replicas with
kv_gather / kv_scatter migrations.  Outputs are compared with a single-process
GPU engine; bf16 GEMMs pick kernels by row count (a padded 8-row microbatch
and a 4-row step can round differently), so token agreement is required on
most positions rather than all of them.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

import test_parallel_cpu as tpc  # noqa: E402


def _agree(a, b):
    n = sum(len(x) for x in a)
    same = sum(int(x == y) for xs, ys in zip(a, b) for x, y in zip(xs, ys))
    return same / max(1, n)


@pytest.fixture
def staged(monkeypatch):
    monkeypatch.setenv("DGI_STAGED_GPU", "1")
    monkeypatch.setenv("DGI_TEST_DEVICE", "cuda")
    monkeypatch.setenv("DGI_TEST_MODEL", "llama-tiny-hd128")
    monkeypatch.setenv("DGI_WATCHDOG", "0")


@pytest.mark.parametrize("sampled", [False, True])
def test_staged_pipeline_replays_stage_graphs(staged, monkeypatch, sampled):
    if sampled:
        monkeypatch.setenv("DGI_TEST_SAMPLED", "1")
    ref = tpc._reference_outputs(model="llama-tiny-hd128")
    out = tpc._spawn("_pp_body", 2, timeout=240)
    assert out[0]["replays"] > 0 and out[1]["replays"] > 0      # both stages replayed graphs
    assert [len(x) for x in out[0]["out"]] == [len(x) for x in ref]
    assert _agree(out[0]["out"], ref) >= 0.75, (out[0]["out"], ref)


def test_staged_pd_replicas_match_local_decode(staged, monkeypatch):
    monkeypatch.setenv("DGI_TEST_PREFILL", "1")
    monkeypatch.setenv("DGI_TEST_REPLICAS", "2")
    ref = tpc._reference_outputs(model="llama-tiny-hd128")
    out = tpc._spawn("_pd_body", 3, timeout=240)
    got = tpc._merged(out, 1, 2)
    assert _agree(got, ref) >= 0.75, (got, ref)
