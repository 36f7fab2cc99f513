"""Shared types and tensor wire format (compatible with the reference's ``common``)."""
from .data_structures import (BlockRange, InferenceRequest, InferenceResponse, InferenceState, KVCacheBlock,
                              ModelShardConfig, SessionConfig, WorkerInfo, WorkerRole, WorkerState,
                              compute_prefix_hash, estimate_kv_cache_size)
from .serialization import StreamingTensorBuffer, TensorSerializer, deserialize_tensor, serialize_tensor

__all__ = ["BlockRange", "WorkerInfo", "WorkerRole", "WorkerState", "InferenceState", "KVCacheBlock",
           "InferenceRequest", "InferenceResponse", "SessionConfig", "ModelShardConfig", "compute_prefix_hash",
           "estimate_kv_cache_size", "TensorSerializer", "serialize_tensor", "deserialize_tensor",
           "StreamingTensorBuffer"]
