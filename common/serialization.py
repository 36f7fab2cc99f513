"""Tensor wire format for the cross-node / HTTP data path.

Same API and byte layout as the reference (``TensorSerializer``,
``serialize_tensor``/``deserialize_tensor`` base64 dicts,
``StreamingTensorBuffer`` header ``[ndim u32][dims u64...][dtype u8]``) so
the HTTP/gRPC shard servers interoperate.  In-node GPU transfers never use
this path: they go over RCCL (``dgi.parallel``).

Addition: ``bf16_mode="raw"`` sends bfloat16 losslessly as its 16-bit
pattern under dtype ``"bfloat16_raw"``; the default (``"fp16"``) keeps the
reference's fp16-carrier encoding for dtype ``"bfloat16"``.
"""
from __future__ import annotations

import base64
import io
import struct
from typing import Any, Dict, Optional, Tuple

import numpy as np

try:
    import torch
    HAS_TORCH = True
except ImportError:  # pragma: no cover
    torch = None
    HAS_TORCH = False

DTYPE_TO_ID = {"float16": 0, "float32": 1, "bfloat16": 2, "int8": 3, "int32": 4, "int64": 5,
               "bfloat16_raw": 6, "uint8": 7, "float64": 8, "bool": 9}
ID_TO_DTYPE = {v: k for k, v in DTYPE_TO_ID.items()}
DTYPE_TO_NUMPY = {"float16": np.float16, "float32": np.float32, "int8": np.int8, "int32": np.int32,
                  "int64": np.int64, "uint8": np.uint8, "float64": np.float64, "bool": np.bool_,
                  "bfloat16": np.float16, "bfloat16_raw": np.int16}
if HAS_TORCH:
    DTYPE_TO_TORCH = {"float16": torch.float16, "float32": torch.float32, "bfloat16": torch.bfloat16,
                      "int8": torch.int8, "int32": torch.int32, "int64": torch.int64, "uint8": torch.uint8,
                      "float64": torch.float64, "bool": torch.bool}
    TORCH_TO_DTYPE = {v: k for k, v in DTYPE_TO_TORCH.items()}


def _compress(b: bytes, method: str) -> bytes:
    if method == "lz4":
        try:
            import lz4.frame
            return lz4.frame.compress(b)
        except ImportError:
            return b
    if method == "zstd":
        try:
            import zstandard
            return zstandard.ZstdCompressor().compress(b)
        except ImportError:
            return b
    return b


def _decompress(b: bytes, method: str) -> bytes:
    if method == "lz4":
        try:
            import lz4.frame
            return lz4.frame.decompress(b)
        except ImportError:
            return b
        except RuntimeError:
            return b
    if method == "zstd":
        try:
            import zstandard
            return zstandard.ZstdDecompressor().decompress(b)
        except ImportError:
            return b
        except Exception:
            return b
    return b


class TensorSerializer:
    @staticmethod
    def serialize(data: Any, compression: str = "none", bf16_mode: str = "fp16") -> Tuple[bytes, Tuple[int, ...], str]:
        if HAS_TORCH and isinstance(data, torch.Tensor):
            t = data.detach()
            if t.dtype == torch.bfloat16:
                if bf16_mode == "raw":
                    arr = t.cpu().contiguous().view(torch.int16).numpy()
                    dtype = "bfloat16_raw"
                else:
                    arr = t.to(torch.float16).cpu().numpy()
                    dtype = "bfloat16"
            else:
                arr = t.cpu().contiguous().numpy()
                dtype = TORCH_TO_DTYPE.get(t.dtype, "float32")
        elif isinstance(data, np.ndarray):
            arr = data
            dtype = str(arr.dtype)
        else:
            raise TypeError(f"Unsupported type: {type(data)}")
        return _compress(np.ascontiguousarray(arr).tobytes(), compression), tuple(arr.shape), dtype

    @staticmethod
    def deserialize(data_bytes: bytes, shape: Tuple[int, ...], dtype_str: str, compression: str = "none",
                    device: str = "cpu") -> Any:
        raw = _decompress(data_bytes, compression)
        arr = np.frombuffer(raw, dtype=DTYPE_TO_NUMPY.get(dtype_str, np.float32)).reshape(shape)
        if not HAS_TORCH or device == "numpy":
            return arr
        t = torch.from_numpy(arr.copy())
        if dtype_str == "bfloat16":
            t = t.to(torch.bfloat16)
        elif dtype_str == "bfloat16_raw":
            t = t.view(torch.bfloat16)
        if device.startswith("cuda") and torch.cuda.is_available():
            t = t.to(device)
        return t


def serialize_tensor(data: Any, compression: str = "none", bf16_mode: str = "fp16") -> Dict[str, Any]:
    b, shape, dtype = TensorSerializer.serialize(data, compression, bf16_mode)
    return {"data": base64.b64encode(b).decode("ascii"), "shape": list(shape), "dtype": dtype,
            "compression": compression}


def deserialize_tensor(serialized: Dict[str, Any], device: str = "cpu") -> Any:
    return TensorSerializer.deserialize(base64.b64decode(serialized["data"]), tuple(serialized["shape"]),
                                        serialized["dtype"], serialized.get("compression", "none"), device)


class StreamingTensorBuffer:
    """Chunked receive of one tensor: header, then raw chunks, then ``finalize``."""

    def __init__(self, chunk_size: int = 1 << 20):
        self.chunk_size = chunk_size
        self.buffer = io.BytesIO()
        self.metadata: Optional[Dict[str, Any]] = None

    def write_header(self, shape: Tuple[int, ...], dtype_str: str) -> bytes:
        hdr = struct.pack("I", len(shape)) + b"".join(struct.pack("Q", int(d)) for d in shape)
        hdr += struct.pack("B", DTYPE_TO_ID.get(dtype_str, 0))
        self.metadata = {"shape": tuple(shape), "dtype": dtype_str}
        return hdr

    def read_header(self, header_bytes: bytes) -> Dict[str, Any]:
        (ndim,) = struct.unpack_from("I", header_bytes, 0)
        dims = struct.unpack_from(f"{ndim}Q", header_bytes, 4)
        (did,) = struct.unpack_from("B", header_bytes, 4 + 8 * ndim)
        meta = {"shape": tuple(int(d) for d in dims), "dtype": ID_TO_DTYPE.get(did, "float32")}
        if self.metadata is None:
            self.metadata = dict(meta)
        return meta

    def iter_chunks(self, data_bytes: bytes):
        for i in range(0, len(data_bytes), self.chunk_size):
            yield data_bytes[i:i + self.chunk_size]

    def write_chunk(self, chunk: bytes) -> None:
        self.buffer.write(chunk)

    def finalize(self, device: str = "cpu") -> Any:
        if self.metadata is None:
            raise ValueError("Header not received")
        return TensorSerializer.deserialize(self.buffer.getvalue(), self.metadata["shape"],
                                            self.metadata["dtype"], device=device)
