"""Engine base class (compatible with the reference's ``worker/engines/base.py``).

GPU facts come from ``torch.cuda`` (HIP on ROCm) plus ``amd-smi`` when
present; there is no NVIDIA path.
"""
from __future__ import annotations

import logging
from abc import ABC, abstractmethod
from typing import Any, Dict, Optional

import torch

logger = logging.getLogger(__name__)


def gpu_summary(index: int = 0) -> Optional[Dict[str, Any]]:
    if not torch.cuda.is_available():
        return None
    props = torch.cuda.get_device_properties(index)
    return {
        "name": torch.cuda.get_device_name(index),
        "arch": getattr(props, "gcnArchName", ""),
        "memory_used_gb": torch.cuda.memory_allocated(index) / 1024 ** 3,
        "memory_total_gb": props.total_memory / 1024 ** 3,
        "compute_units": getattr(props, "multi_processor_count", 0),
    }


class BaseEngine(ABC):
    """All engines implement load / inference / unload; status is shared."""

    def __init__(self, config: Dict[str, Any]):
        self.config = config or {}
        self.model = None
        self.device = "cuda" if torch.cuda.is_available() else "cpu"
        self.loaded = False

    @abstractmethod
    def load_model(self) -> None: ...

    @abstractmethod
    def inference(self, params: Dict[str, Any]) -> Dict[str, Any]: ...

    @abstractmethod
    def unload_model(self) -> None: ...

    def get_status(self) -> Dict[str, Any]:
        status: Dict[str, Any] = {"loaded": self.loaded, "device": self.device}
        g = gpu_summary(0)
        if g is not None:
            status["gpu"] = g
        return status

    def _get_gpu_memory(self) -> Optional[Dict[str, float]]:
        g = gpu_summary(0)
        if g is None:
            return None
        return {"used_gb": g["memory_used_gb"], "total_gb": g["memory_total_gb"]}
