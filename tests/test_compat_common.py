"""common/ wire types and tensor serialization.

Behavioural parity with the reference's tests/test_common_data_structures.py
and tests/test_common_serialization.py (BlockRange, WorkerInfo health,
InferenceState, KVCacheBlock ref counting, TensorSerializer / streaming
buffer round trips), plus the fixes listed in SURVEY Appendix E: prefix
hashes of ids >= 256, GQA-aware KV sizing and a lossless bf16 wire mode.
"""
import time

import numpy as np
import pytest
import torch

from common.data_structures import (BlockRange, InferenceState, KVCacheBlock, ModelShardConfig, SessionConfig,
                                    WorkerInfo, WorkerRole, WorkerState, compute_prefix_hash, estimate_kv_cache_size)
from common.serialization import StreamingTensorBuffer, TensorSerializer, deserialize_tensor, serialize_tensor


# ----------------------------------------------------------------------------- data structures

@pytest.mark.parametrize("start,end", [(0, 1), (2, 5), (40, 80)])
def test_block_range_membership_length_and_dict(start, end):
    br = BlockRange(start=start, end=end)
    assert br.length == end - start
    assert start in br and (end - 1) in br
    assert end not in br and (start - 1) not in br
    assert BlockRange.from_dict(br.to_dict()) == br


def test_enums_match_reference_values():
    assert {r.value for r in WorkerRole} == {"prefill", "decode", "hybrid"}
    assert WorkerState.ONLINE in WorkerState


def test_worker_info_utilisation_and_heartbeat_health():
    now = time.time()
    w = WorkerInfo(worker_id="w", state=WorkerState.ONLINE, gpu_memory_gb=8.0, gpu_memory_used_gb=2.0,
                   cache_tokens_available=400, cache_tokens_used=100, last_heartbeat=now)
    assert w.cache_utilization == pytest.approx(0.25)
    assert w.gpu_utilization == pytest.approx(0.25)
    assert w.is_healthy(timeout_seconds=30.0)
    w.last_heartbeat = now - 31.0
    assert not w.is_healthy(timeout_seconds=30.0)
    back = WorkerInfo.from_dict(w.to_dict())
    assert back.worker_id == "w" and back.gpu_memory_gb == 8.0


def test_inference_state_position_advances():
    s = InferenceState(session_id="s", position=5)
    t = s.updated_at
    s.update_position(new_tokens=7)
    assert s.position == 12 and s.updated_at >= t


def test_kv_block_reference_counting():
    b = KVCacheBlock(block_id="b", layer_idx=3, ref_count=1)
    assert not b.is_shared
    b.increment_ref()
    b.increment_ref()
    assert b.ref_count == 3 and b.is_shared
    assert [b.decrement_ref() for _ in range(3)] == [2, 1, 0]
    assert b.decrement_ref() == 0  # never negative


def test_session_config_defaults():
    c = SessionConfig(model_name="m")
    assert (c.max_length, c.max_retries, c.use_speculative_decoding) == (4096, 3, False)


def test_prefix_hash_distinguishes_large_token_ids():
    # the reference hashed bytes(token_ids), which raises for ids >= 256
    a = compute_prefix_hash([1, 128000, 5])
    b = compute_prefix_hash([1, 128001, 5])
    assert a != b and len(a) == 16
    assert compute_prefix_hash([1, 128000, 5]) == a


def test_kv_size_estimate_is_gqa_aware():
    mha = estimate_kv_cache_size(80, 64, 128, 512)
    gqa = estimate_kv_cache_size(80, 64, 128, 512, num_kv_heads=8)
    assert mha == 2 * 80 * 512 * 64 * 128 * 2
    assert gqa * 8 == mha


def test_model_shard_config_routes_and_completeness():
    msc = ModelShardConfig(model_id="m", total_layers=10,
                           shard_mapping={"b": BlockRange(4, 10), "a": BlockRange(0, 4)})
    assert [w for w, _ in msc.get_inference_route()] == ["a", "b"]
    assert msc.get_worker_for_layer(3) == "a" and msc.get_worker_for_layer(4) == "b"
    assert msc.get_worker_for_layer(10) is None
    assert msc.is_complete()
    msc.shard_mapping["c"] = BlockRange(8, 9)  # overlap
    assert not msc.is_complete()


# ----------------------------------------------------------------------------- serialization

@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float32, np.float16, np.uint8])
def test_numpy_roundtrip(dtype):
    a = (np.arange(24) % 7).astype(dtype).reshape(2, 3, 4)
    b, shape, ds = TensorSerializer.serialize(a, compression="none")
    r = TensorSerializer.deserialize(b, shape, ds, compression="none", device="numpy")
    assert isinstance(r, np.ndarray) and r.dtype == a.dtype and np.array_equal(r, a)


def test_base64_dict_roundtrip():
    a = np.linspace(-1, 1, 9, dtype=np.float32).reshape(3, 3)
    payload = serialize_tensor(a)
    assert set(payload) >= {"data", "shape", "dtype"}
    assert np.array_equal(deserialize_tensor(payload, device="numpy"), a)


@pytest.mark.parametrize("chunk", [1, 13, 4096])
def test_streaming_buffer_reassembles(chunk):
    a = np.arange(257, dtype=np.int64)
    raw, shape, ds = TensorSerializer.serialize(a)
    buf = StreamingTensorBuffer(chunk_size=chunk)
    hdr = buf.read_header(buf.write_header(shape=shape, dtype_str=ds))
    assert hdr["shape"] == shape and hdr["dtype"] == ds
    for c in buf.iter_chunks(raw):
        assert len(c) <= chunk
        buf.write_chunk(c)
    assert np.array_equal(buf.finalize(device="numpy"), a)


def test_streaming_finalize_without_header_raises():
    with pytest.raises(ValueError, match="Header not received"):
        StreamingTensorBuffer().finalize(device="numpy")


def test_unsupported_type_raises():
    with pytest.raises(TypeError, match="Unsupported type"):
        TensorSerializer.serialize([1, 2, 3])


@pytest.mark.parametrize("method", ["lz4", "zstd"])
def test_optional_compression_roundtrips_or_falls_back(method):
    a = np.zeros(1000, dtype=np.float32)
    b, shape, ds = TensorSerializer.serialize(a, compression=method)
    r = TensorSerializer.deserialize(b, shape, ds, compression=method, device="numpy")
    assert np.array_equal(r, a)


def test_torch_fp16_roundtrip():
    t = torch.arange(6, dtype=torch.float16).reshape(2, 3)
    r = TensorSerializer.deserialize(*TensorSerializer.serialize(t), device="cpu")
    assert r.dtype == torch.float16 and torch.equal(r, t)


def test_bf16_default_wire_is_reference_compatible():
    t = torch.tensor([[1.0, -2.5, 3.0, 0.125]], dtype=torch.bfloat16)
    b, shape, ds = TensorSerializer.serialize(t)
    assert ds == "bfloat16"
    r = TensorSerializer.deserialize(b, shape, ds, device="cpu")
    assert r.dtype == torch.bfloat16 and torch.equal(r, t)


def test_bf16_raw_mode_is_lossless_beyond_fp16_range():
    t = torch.tensor([1e30, -3e-30, 7.0], dtype=torch.bfloat16)  # not representable in fp16
    b, shape, ds = TensorSerializer.serialize(t, bf16_mode="raw")
    r = TensorSerializer.deserialize(b, shape, ds, device="cpu")
    assert r.dtype == torch.bfloat16 and torch.equal(r, t)
