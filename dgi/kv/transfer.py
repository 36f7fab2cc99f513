"""Cross-worker KV transfer: a prefilled sequence's pages as one binary blob.

Inside one MI355X node KV pages move over RCCL (``dgi.parallel.kv_transfer``).
Between workers of the cluster P/D path (server/app/services/pd_runtime.py —
the reference's ``KVCacheMigrator._do_migrate`` is ``asyncio.sleep(0.05)``,
reference server/app/services/pd_scheduler.py:452-479, and its gRPC
``TransferKVCache`` stores nothing a decode engine can use,
reference worker/distributed/grpc_server.py:190-235) the prefill worker keeps
the sequence's pages in an export store and the decode worker pulls them over
HTTP (``GET /kv/{key}`` on the prefill worker's direct server) and installs them
with ``LLMEngine.import_prefilled`` — it decodes from the first token without
re-running the prompt.

Wire format: ``b"DGKV"`` | u32 header length | JSON header | raw page bytes.
The header carries the tensor shape and dtype, the prompt token ids, the first
token and the model geometry the importer checks; bf16 travels as its raw 16-bit
pattern (lossless, unlike the reference serializer's fp16 round trip,
common/serialization.py).
"""
from __future__ import annotations

import collections
import json
import struct
import threading
import time
from typing import Optional

import numpy as np
import torch

MAGIC = b"DGKV"
_DT = {torch.bfloat16: ("bfloat16", torch.int16), torch.float16: ("float16", torch.int16),
       torch.float32: ("float32", torch.float32)}
_DT_BACK = {"bfloat16": (torch.bfloat16, np.int16), "float16": (torch.float16, np.int16),
            "float32": (torch.float32, np.float32)}


def pack_kv(kv: torch.Tensor, meta: dict) -> bytes:
    """[L, 2, n_pages, n_kv, page, head_dim] pages + metadata -> one blob."""
    kv = kv.detach().contiguous().cpu()
    name, view = _DT[kv.dtype]
    hdr = dict(meta, shape=list(kv.shape), dtype=name)
    h = json.dumps(hdr).encode()
    return MAGIC + struct.pack("<I", len(h)) + h + kv.view(view).numpy().tobytes()


def unpack_kv(blob: bytes) -> tuple:
    """blob -> (pages tensor on the host, metadata dict)."""
    if blob[:4] != MAGIC:
        raise ValueError("not a dgi KV blob")
    (n,) = struct.unpack("<I", blob[4:8])
    hdr = json.loads(blob[8:8 + n].decode())
    dt, npdt = _DT_BACK[hdr.pop("dtype")]
    shape = hdr.pop("shape")
    arr = np.frombuffer(blob, dtype=npdt, offset=8 + n, count=int(np.prod(shape)))
    t = torch.from_numpy(arr.copy()).view(dt).view(*shape)
    return t, hdr


def new_token() -> str:
    """Per-export secret: only the holder (the decode worker the coordinator
    placed the job on) may pull the pages."""
    import secrets
    return secrets.token_urlsafe(24)


class KVExportStore:
    """Exported sequences by key, bounded by bytes and age (oldest leave first).

    An entry may carry a secret ``token``: ``take`` then hands the blob only to a
    caller presenting the same token (constant-time compare) and leaves it in
    place otherwise.  An entry may also be *pending* (``put_pending``): the
    exporting engine packs the pages off its step thread and the store resolves
    the future on ``take``."""

    def __init__(self, max_bytes: int = 8 << 30, ttl_s: float = 600.0):
        self.max_bytes = max_bytes
        self.ttl_s = ttl_s
        # key -> (time, blob bytes | Future[bytes], token | None)
        self._d: "collections.OrderedDict[str, tuple]" = collections.OrderedDict()
        self._bytes = 0
        self._lock = threading.Lock()
        self.stats = {"exported": 0, "served": 0, "expired": 0, "bytes_served": 0, "refused": 0}

    @staticmethod
    def _size(v) -> int:
        return len(v) if isinstance(v, (bytes, bytearray)) else 0

    def put(self, key: str, blob: bytes, token: Optional[str] = None) -> None:
        self._put(key, blob, token)

    def put_pending(self, key: str, future, token: Optional[str] = None) -> None:
        """``future`` resolves to the blob (packed on a worker thread); once done
        its bytes count towards the cap."""
        self._put(key, future, token)

        def _done(f):
            with self._lock:
                v = self._d.get(key)
                if v is not None and v[1] is f and f.exception() is None:
                    self._d[key] = (v[0], f.result(), v[2])
                    self._bytes += len(f.result())
                    self._evict()
        future.add_done_callback(_done)

    def _put(self, key: str, v, token: Optional[str]) -> None:
        with self._lock:
            old = self._d.pop(key, None)
            if old is not None:
                self._bytes -= self._size(old[1])
            self._d[key] = (time.time(), v, token)
            self._bytes += self._size(v)
            self.stats["exported"] += 1
            self._evict()

    def take(self, key: str, token: Optional[str] = None, wait_s: float = 30.0,
             check_token: bool = True) -> Optional[bytes]:
        """The blob of ``key`` (removed: one decode worker consumes it), or None when
        absent, expired, or guarded by a token the caller does not present
        (``check_token=False``: the owning worker itself, decoding its own export)."""
        import hmac
        with self._lock:
            self._evict()
            v = self._d.get(key)
            if v is None:
                return None
            want = v[2]
            if check_token and want is not None and (token is None or not hmac.compare_digest(str(token), want)):
                self.stats["refused"] += 1
                return None
            del self._d[key]
            self._bytes -= self._size(v[1])
        blob = v[1]
        if not isinstance(blob, (bytes, bytearray)):
            try:
                blob = blob.result(timeout=wait_s)
            except Exception:
                return None
        with self._lock:
            self.stats["served"] += 1
            self.stats["bytes_served"] += len(blob)
        return blob

    def _evict(self) -> None:
        now = time.time()
        while self._d:
            k, (t, b, _tok) = next(iter(self._d.items()))
            if self._bytes <= self.max_bytes and now - t <= self.ttl_s:
                break
            self._d.popitem(last=False)
            self._bytes -= self._size(b)
            self.stats["expired"] += 1

    def __len__(self) -> int:
        return len(self._d)
