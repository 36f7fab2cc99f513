"""Cross-node distributed inference (shards, KV tiers, sessions, shard servers).

In-node parallelism (RCCL pipeline, P/D migration) lives in ``dgi.parallel``.
"""
from .kv_cache import CacheBlock, CacheLocation, DistributedKVCacheManager, KVCachePool, PagedKVCache
from .model_shard import LayerInfo, ModelShard, ShardedModelLoader, get_layer_range_for_worker
from .session import DistributedInferenceSession, SessionManager, SessionState, WorkerSession

__all__ = ["CacheBlock", "CacheLocation", "DistributedKVCacheManager", "KVCachePool", "PagedKVCache", "LayerInfo",
           "ModelShard", "ShardedModelLoader", "get_layer_range_for_worker", "DistributedInferenceSession",
           "SessionManager", "SessionState", "WorkerSession", "InferenceServicer", "GRPCServer",
           "HTTPInferenceServer"]


def __getattr__(name):
    if name in ("InferenceServicer", "GRPCServer", "HTTPInferenceServer"):
        from . import grpc_server
        return getattr(grpc_server, name)
    raise AttributeError(name)
