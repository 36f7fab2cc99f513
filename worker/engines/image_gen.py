"""Image generation engine (diffusers on ROCm; reference worker/engines/image_gen.py:13-83).

Out of the MI355X-native scope: runs the diffusers pipeline
when the package is installed; ``load_model`` raises a clear ImportError
otherwise.  Returns base64 PNGs like the reference.
"""
from __future__ import annotations

import base64
import io
import logging
from typing import Any, Dict

import torch

from .base import BaseEngine

logger = logging.getLogger(__name__)


class ImageGenEngine(BaseEngine):
    def load_model(self) -> None:
        try:
            from diffusers import DiffusionPipeline
        except ImportError as e:
            raise ImportError(f"image_gen requires diffusers: {e}")
        model_id = self.config.get("model_id", "black-forest-labs/FLUX.1-schnell")
        self.model = DiffusionPipeline.from_pretrained(model_id, torch_dtype=torch.bfloat16)
        if self.config.get("enable_cpu_offload", True) and self.device == "cuda":
            self.model.enable_sequential_cpu_offload()
        else:
            self.model.to(self.device)
        self.loaded = True

    def inference(self, params: Dict[str, Any]) -> Dict[str, Any]:
        gen = None
        if params.get("seed") is not None:
            gen = torch.Generator(device="cpu").manual_seed(int(params["seed"]))
        width, height = int(params.get("width", 1024)), int(params.get("height", 1024))
        steps = int(params.get("steps", 4))
        out = self.model(prompt=params.get("prompt", ""), negative_prompt=params.get("negative_prompt") or None,
                         width=width, height=height, num_inference_steps=steps, generator=gen)
        img = out.images[0]
        buf = io.BytesIO()
        img.save(buf, format="PNG")
        return {"image_base64": base64.b64encode(buf.getvalue()).decode(), "width": width, "height": height,
                "steps": steps, "seed": params.get("seed")}

    def unload_model(self) -> None:
        self.model = None
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        self.loaded = False
