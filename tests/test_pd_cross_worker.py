"""Cluster P/D across workers (server/app/services/pd_runtime.py path): the prefill
worker exports the sequence's KV pages at its first token, the decode worker pulls
them over HTTP (``GET /kv/{key}`` on the prefill worker's direct server) and
decodes from the first token without recomputing the prompt (dgi/kv/transfer.py).
The reference's migrator is ``asyncio.sleep(0.05)``
(reference server/app/services/pd_scheduler.py:452-479)."""
import os
import socket
import sys
import time

import httpx
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "worker"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine():
    from engines.llm_native import NativeLLMEngine
    e = NativeLLMEngine({"model_id": "llama-tiny", "device": "cpu", "use_graphs": False, "num_blocks": 128,
                         "max_num_seqs": 8, "max_model_len": 512, "enable_prefix_caching": False})
    e.load_model()
    return e


def _daemon(wid, engine):
    from worker.main import Worker as Daemon
    d = Daemon.__new__(Daemon)
    d.worker_id = wid
    d.engines = {"llm": engine}
    d.tracer = d.metrics = None
    d._batchers = {}
    return d


def test_kv_blob_roundtrip_is_lossless():
    from dgi.kv.transfer import KVExportStore, pack_kv, unpack_kv
    kv = torch.randn(3, 2, 5, 2, 16, 64).to(torch.bfloat16)
    t, meta = unpack_kv(pack_kv(kv, {"prompt": [1, 2, 3], "first_token": 7}))
    assert torch.equal(t, kv) and meta["prompt"] == [1, 2, 3] and meta["first_token"] == 7
    st = KVExportStore(max_bytes=1000, ttl_s=60)
    st.put("a", b"x" * 600)
    st.put("b", b"y" * 600)            # over the byte cap: the oldest leaves
    assert st.take("a") is None and st.take("b") == b"y" * 600 and st.take("b") is None
    # a guarded export is only handed to the holder of its secret; a wrong guess leaves it in place
    st.put("c", b"z" * 10, token="s3cret")
    assert st.take("c") is None and st.take("c", token="guess") is None and len(st) == 1
    assert st.take("c", token="s3cret") == b"z" * 10 and st.stats["refused"] == 2
    # pending export (packed on another thread): take() waits for it
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(1) as ex:
        st.put_pending("d", ex.submit(lambda: (time.sleep(0.05), b"w" * 7)[1]), token="t")
        assert st.take("d", token="t") == b"w" * 7


def test_decode_worker_pulls_kv_instead_of_reprefilling():
    from direct_server import DirectServer
    pre_eng, dec_eng, ref_eng = _engine(), _engine(), _engine()
    try:
        params = {"prompt": "the quick brown fox jumps over the lazy dog", "max_tokens": 12, "temperature": 0.0}
        ref = ref_eng.inference(dict(params))
        pre = _daemon("pre", pre_eng)
        port = _port()
        srv = DirectServer(pre, "127.0.0.1", port)
        srv.start_background()
        pre.direct_url = f"http://127.0.0.1:{port}"
        for _ in range(100):
            try:
                httpx.get(pre.direct_url + "/health", timeout=1)
                break
            except httpx.HTTPError:
                time.sleep(0.1)
        pre.kv_loopback_ok = True          # test: decode worker on the same host
        out1 = pre.execute("llm", {**params, "pd": True}, "job-7")
        assert out1["phase"] == "prefill" and out1["kv_url"].endswith("/kv/pre:job-7") and out1["kv_token"]
        assert len(pre_eng.kv_exports) == 1
        # the export is guarded: a pull without (or with a wrong) secret gets nothing and leaves it
        assert httpx.get(out1["kv_url"], timeout=10).status_code == 404
        assert httpx.get(out1["kv_url"], headers={"X-KV-Token": "nope"}, timeout=10).status_code == 404
        assert len(pre_eng.kv_exports) == 1
        dec = _daemon("dec", dec_eng)
        # a URL that is not this job's /kv/ export is never fetched (client-chosen URL)
        assert not dec._kv_url_ok("http://169.254.169.254/latest/meta-data", "job-7")
        assert not dec._kv_url_ok(out1["kv_url"].replace("job-7", "job-8"), "job-7")
        assert dec._kv_url_ok(out1["kv_url"], "job-7")
        before = dict(dec_eng.engine.stats)
        out2 = dec.execute("llm", {**params, "pd": True, "pd_phase": "decode", "kv_source": "pre",
                                   "kv_url": out1["kv_url"], "kv_token": out1["kv_token"],
                                   "first_token": out1["first_token"]}, "job-7")
        assert out2["reprefilled"] is False and out2["kv_bytes"] > 0
        assert out2["response"] == ref["response"]
        assert dec_eng.engine.stats["prefill_tokens"] == before["prefill_tokens"]   # no prompt recompute
        assert dec_eng.stats["kv_imported"] == 1 and len(pre_eng.kv_exports) == 0
        # the key is consumed: a second pull falls back to re-prefilling, same text
        out3 = dec.execute("llm", {**params, "pd": True, "pd_phase": "decode", "kv_url": out1["kv_url"]}, "job-7")
        assert out3["reprefilled"] is True and out3["response"] == ref["response"]
        srv.stop()
    finally:
        for e in (pre_eng, dec_eng, ref_eng):
            e.unload_model()


def test_decode_on_the_prefilling_worker_uses_its_own_export():
    """The P/D scheduler may place the decode phase on the worker that prefilled
    (no migration, no kv_url): it decodes from its own export, no recompute."""
    eng, ref_eng = _engine(), _engine()
    try:
        params = {"prompt": "pack my box with five dozen liquor jugs", "max_tokens": 9, "temperature": 0.0}
        ref = ref_eng.inference(dict(params))
        w = _daemon("solo", eng)
        w.direct_url = None              # no direct server at all
        out1 = w.execute("llm", {**params, "pd": True}, "job-3")
        assert out1["kv_url"] is None and len(eng.kv_exports) == 1
        before = eng.engine.stats["prefill_tokens"]
        out2 = w.execute("llm", {**params, "pd": True, "pd_phase": "decode"}, "job-3")
        assert out2["reprefilled"] is False and out2["kv_source"] == "local"
        assert out2["response"] == ref["response"] and eng.engine.stats["prefill_tokens"] == before
    finally:
        eng.unload_model()
        ref_eng.unload_model()


def test_import_stops_at_a_first_token_that_ends_the_sequence():
    """EOS sampled by the prefill worker: the imported sequence is finished at once
    (no decoding past it); the exported seed is kept."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams, Status
    e = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", num_blocks=64, max_num_seqs=4, max_model_len=256,
                               max_num_batched_tokens=64, enable_prefix_caching=False, use_graphs=False))
    prompt = list(range(5, 25))
    src = e.add_request(prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    while e.has_unfinished():
        e.step()
    kv = torch.zeros(e.pool.kv.shape[0], 2, 2, *e.pool.kv.shape[3:], dtype=e.pool.kv.dtype)
    free0 = e.pool.num_free
    eos = e.model_cfg.eos_token_id
    r = e.import_prefilled(prompt, eos, kv, SamplingParams(max_tokens=8), seed=1234)
    assert r.status is Status.FINISHED and r.finish_reason == "stop" and r.output == [eos]
    assert e.pool.num_free == free0 and not e.has_unfinished() and r.seed == 1234
    r2 = e.import_prefilled(prompt, 7, kv, SamplingParams(max_tokens=1))        # max_tokens reached
    assert r2.status is Status.FINISHED and r2.finish_reason == "length"
    r3 = e.import_prefilled(prompt, 7, kv, SamplingParams(max_tokens=3, temperature=0.8), seed=99)
    assert r3.status is not Status.FINISHED and r3.seed == 99
    while e.has_unfinished():
        e.step()
    assert len(r3.output) == 3 and src.output
