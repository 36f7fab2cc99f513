"""Multi-rank runtime on the GPU ("staged": all ranks share one MI355X, the data
plane is gloo through host memory, compute is the HIP path).

Covers the GPU-only parts the CPU suite cannot: stage hipGraph replay of
decode micro-steps (pipeline.StageGraphs), padded decode microbatches,
top-k/top-p sampling inside the last stage's graph, and P/D replicas with
kv_gather / kv_scatter migrations.  Every output token is checked per step, teacher forced, against the fp32 CPU
model with the same seeded weights (``_teacher_forced_ok``: the chosen token is
an argmax of the fp32 logits up to a bf16 tolerance; sampled runs: inside the
fp32 top-k).  bf16 GEMMs pick kernels by row count, so layouts may legitimately
pick a different near-tied token — each pick must still be a right one; no test
accepts partial agreement.  P/D runs also hash every migrated layer group on the
prefill rank and again after it is installed in the receiver's pool
(DGI_KV_CHECKSUM): the pages must be bit-identical.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

import test_parallel_cpu as tpc  # noqa: E402


MODEL = "llama-tiny-hd128"


def _seeded(model=MODEL):
    """The weights every rank builds (per-layer seeded init on the device, seed 0)."""
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    return LlamaModel(get_config(model), "cuda", seed=0)


def _check(outs, prompts=None, model=MODEL, sampled=False):
    """Teacher-forced per-step check of every token of ``outs`` (lists in prompt order)."""
    from test_kernels_gpu import _teacher_forced_ok, _teacher_forced_topk_ok
    prompts = prompts or tpc.PROMPTS
    assert len(outs) == len(prompts) and all(len(x) > 0 for x in outs)
    if sampled:
        n = _teacher_forced_topk_ok(model, _seeded(model), prompts, outs, k=12)
    else:
        n = _teacher_forced_ok(model, _seeded(model), prompts, outs)
    assert n == sum(len(x) for x in outs)


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
    out = tpc._spawn("_pp_body", 2, timeout=240)
    assert out[0]["replays"] > 0 and out[1]["replays"] > 0      # both stages replayed graphs
    _check(out[0]["out"], sampled=sampled)


def test_staged_pd_replicas_match_local_decode(staged, monkeypatch):
    monkeypatch.setenv("DGI_TEST_PREFILL", "1")
    monkeypatch.setenv("DGI_TEST_REPLICAS", "2")
    monkeypatch.setenv("DGI_KV_CHECKSUM", "1")
    out = tpc._spawn("_pd_body", 3, timeout=240)
    _check(tpc._merged(out, 1, 2))
    assert tpc.check_kv_digests(out) >= 2


# ---------------------------------------------------------------------------- RCCL on one GPU
# DGI_SHARED_GPU=1 (dgi.parallel.fabric.shared_gpu): every rank on device 0 with
# its own NCCL_HOSTID, so RCCL accepts the ranks and moves data over its
# network transport.  Every send/recv is a real RCCL operation with RCCL's
# blocking semantics (a send waits for its receive): the ordering bugs a gloo
# rehearsal cannot show surface here as hangs, which the timeouts turn into
# failures.

@pytest.fixture
def shared_rccl(monkeypatch):
    monkeypatch.setenv("DGI_SHARED_GPU", "1")
    monkeypatch.setenv("DGI_TEST_BACKEND", "nccl")
    monkeypatch.setenv("DGI_TEST_DEVICE", "cuda")
    monkeypatch.setenv("DGI_TEST_MODEL", "llama-tiny-hd128")
    monkeypatch.setenv("DGI_WATCHDOG", "0")
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")


@pytest.mark.parametrize("sampled", [False, True])
def test_rccl_pipeline_on_shared_gpu(shared_rccl, monkeypatch, sampled):
    if sampled:
        monkeypatch.setenv("DGI_TEST_SAMPLED", "1")
    out = tpc._spawn("_pp_body", 2, timeout=150)
    assert out[0]["replays"] > 0 and out[1]["replays"] > 0
    _check(out[0]["out"], sampled=sampled)


@pytest.mark.parametrize("replicas,world", [(2, 3), (1, 3)])
def test_rccl_pd_on_shared_gpu(shared_rccl, monkeypatch, replicas, world):
    """1 prefill rank + 2 whole-model decode replicas, and 1 prefill rank + one
    2-stage decode pipeline (pdpp): KV migration, layer streaming and stage hops
    all over RCCL."""
    monkeypatch.setenv("DGI_TEST_PREFILL", "1")
    monkeypatch.setenv("DGI_TEST_REPLICAS", str(replicas))
    monkeypatch.setenv("DGI_TEST_SAMPLED", "1")
    monkeypatch.setenv("DGI_KV_CHECKSUM", "1")
    out = tpc._spawn("_pd_body", world, timeout=150)
    drivers = [1, 2] if replicas == 2 else [1]
    _check(tpc._merged(out, *drivers), sampled=True)
    assert tpc.check_kv_digests(out) >= 2


def test_rccl_pdpp_serves_local_prompts_on_shared_gpu(shared_rccl, monkeypatch):
    """1 prefill rank + a 2-stage decode pipeline whose driver also admits prompts
    of its own (the hybrid decode of the 70B N=4 layout), over RCCL."""
    monkeypatch.setenv("DGI_TEST_PREFILL", "1")
    monkeypatch.setenv("DGI_TEST_LOCAL", "2")
    monkeypatch.setenv("DGI_KV_CHECKSUM", "1")
    out = tpc._spawn("_pd_body", 3, timeout=150)
    _check(tpc._merged(out, 1))
    assert tpc.check_kv_digests(out) >= 2


def test_rccl_tensor_parallel_on_shared_gpu(shared_rccl):
    """2-way tensor parallelism with its two all-reduces per layer on RCCL (eager
    world communicator), against a single-GPU engine with the same seeded weights."""
    out = tpc._spawn("_tp_gpu_body", 2, timeout=150)
    assert out[0]["out"] == out[1]["out"]                  # SPMD: both ranks emit the same tokens
    _check(out[0]["out"], prompts=out[0]["prompts"], model="llama-tiny-tp")


def test_rccl_two_prefill_sources_batched_receives_on_shared_gpu(shared_rccl, monkeypatch):
    """2 prefill ranks feeding one decode rank over RCCL: the decode rank posts its
    receives from both sources as one RCCL group (dgi.parallel.kv_transfer); the
    migrated pages land bit-identical and every token is right."""
    monkeypatch.setenv("DGI_TEST_PREFILL", "2")
    monkeypatch.setenv("DGI_KV_CHECKSUM", "1")
    out = tpc._spawn("_pd_body", 3, timeout=150)
    _check(tpc._merged(out, 2))
    assert tpc.check_kv_digests(out) >= 2


def test_rccl_receive_batch_completes_every_receive(shared_rccl):
    """One RCCL group of receives from two sources: RCCL coalesces it into a single work
    handle, and every receive of the batch must be reported complete with it (a batch
    that tracked only one handle lost the other transfers)."""
    out = tpc._spawn("_recv_batch_body", 3, timeout=120)
    assert out[0] == [1.0, 2.0, 1.0, 2.0]
