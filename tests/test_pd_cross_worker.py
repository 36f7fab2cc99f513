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
        out1 = pre.execute("llm", {**params, "pd": True}, "job-7")
        assert out1["phase"] == "prefill" and out1["kv_url"].endswith("/kv/pre:job-7")
        assert len(pre_eng.kv_exports) == 1
        dec = _daemon("dec", dec_eng)
        before = dict(dec_eng.engine.stats)
        out2 = dec.execute("llm", {**params, "pd": True, "pd_phase": "decode", "kv_source": "pre",
                                   "kv_url": out1["kv_url"], "first_token": out1["first_token"]}, "job-7")
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
