"""Vision-language engine (HF on ROCm; reference worker/engines/vision.py:14-139).

Tasks ``image_qa``, ``image_caption``, ``ocr``.  Loads a local HF VLM; the
image arrives base64-encoded.  Out of the MI355X-native scope.
"""
from __future__ import annotations

import base64
import io
import logging
from typing import Any, Dict

import torch

from .base import BaseEngine

logger = logging.getLogger(__name__)

_TASK_PROMPTS = {
    "image_caption": "Describe this image in detail.",
    "ocr": "Extract all text in this image.",
}


class VisionEngine(BaseEngine):
    def load_model(self) -> None:
        from transformers import AutoModelForCausalLM, AutoTokenizer
        model_id = self.config.get("model_id", "THUDM/glm-4v-9b")
        self.tokenizer = AutoTokenizer.from_pretrained(model_id, trust_remote_code=True)
        kw: Dict[str, Any] = {"torch_dtype": torch.bfloat16, "trust_remote_code": True}
        kw["device_map"] = "auto" if self.config.get("enable_cpu_offload", True) else {"": self.device}
        self.model = AutoModelForCausalLM.from_pretrained(model_id, **kw).eval()
        self.loaded = True

    @staticmethod
    def decode_image(b64: str):
        from PIL import Image
        if "," in b64 and b64.strip().startswith("data:"):
            b64 = b64.split(",", 1)[1]
        return Image.open(io.BytesIO(base64.b64decode(b64))).convert("RGB")

    def inference(self, params: Dict[str, Any]) -> Dict[str, Any]:
        task = params.get("task", "image_qa")
        question = params.get("question") or _TASK_PROMPTS.get(task, "What is in this image?")
        image = self.decode_image(params["image_base64"])
        inputs = self.tokenizer.apply_chat_template([{"role": "user", "image": image, "content": question}],
                                                    add_generation_prompt=True, tokenize=True,
                                                    return_tensors="pt", return_dict=True).to(self.model.device)
        with torch.no_grad():
            out = self.model.generate(**inputs, max_new_tokens=int(params.get("max_tokens", 1024)), do_sample=False)
        n_in = inputs["input_ids"].shape[1]
        text = self.tokenizer.decode(out[0][n_in:], skip_special_tokens=True)
        return {"response": text, "task": task,
                "usage": {"prompt_tokens": n_in, "completion_tokens": int(out.shape[1] - n_in)}}

    def unload_model(self) -> None:
        self.model = None
        self.tokenizer = None
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        self.loaded = False
