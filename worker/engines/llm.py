"""HF Transformers LLM engine (reference worker/engines/llm.py:11-97).

The portable CPU path (BASELINE config #1: OPT-125m greedy on CPU).  With no
network, a model id that is not on local disk is instantiated from its
built-in architecture with random weights (``random_init``), and the
tokenizer falls back to ``dgi.utils.tokenizer.ByteTokenizer``.
"""
from __future__ import annotations

import logging
from typing import Any, Dict

import torch

from dgi.utils.tokenizer import ByteTokenizer, chat_prompt_ids, load_tokenizer

from .base import BaseEngine

logger = logging.getLogger(__name__)

_BUILTIN_HF = {
    "facebook/opt-125m": ("OPTConfig", dict(vocab_size=50272, hidden_size=768, num_hidden_layers=12,
                                            ffn_dim=3072, num_attention_heads=12, max_position_embeddings=2048,
                                            word_embed_proj_dim=768, bos_token_id=2, eos_token_id=2,
                                            pad_token_id=1)),
    "opt-125m": None,
}


def _hf_random_model(model_id: str, seed: int = 0):
    import transformers
    key = model_id if model_id in _BUILTIN_HF and _BUILTIN_HF[model_id] else "facebook/opt-125m"
    cls_name, kw = _BUILTIN_HF[key]
    cfg = getattr(transformers, cls_name)(**kw)
    torch.manual_seed(seed)
    return transformers.AutoModelForCausalLM.from_config(cfg)


class LLMEngine(BaseEngine):
    def load_model(self) -> None:
        from transformers import AutoModelForCausalLM

        model_id = self.config.get("model_id", "facebook/opt-125m")
        dev = self.config.get("device", self.device)
        self.device = dev
        dtype = torch.bfloat16 if dev != "cpu" else torch.float32
        try:
            kw: Dict[str, Any] = {"torch_dtype": dtype, "local_files_only": True}
            if self.config.get("enable_cpu_offload", False) and dev != "cpu":
                kw["device_map"] = "auto"
            self.model = AutoModelForCausalLM.from_pretrained(model_id, **kw)
            if "device_map" not in kw:
                self.model.to(dev)
        except Exception as e:
            if not self.config.get("random_init", True):
                raise
            logger.warning("model %s not available locally (%s); using random-init weights", model_id, e)
            self.model = _hf_random_model(model_id, self.config.get("seed", 0)).to(dev).to(dtype)
        self.model.eval()
        vocab = getattr(self.model.config, "vocab_size", 32000)
        self.tokenizer = load_tokenizer(model_id, vocab_size=vocab,
                                        bos=getattr(self.model.config, "bos_token_id", 1) or 1,
                                        eos=getattr(self.model.config, "eos_token_id", 2) or 2)
        self.loaded = True

    def inference(self, params: Dict[str, Any]) -> Dict[str, Any]:
        messages = params.get("messages", [])
        max_tokens = int(params.get("max_tokens", 2048))
        temperature = float(params.get("temperature", 0.7))
        top_p = float(params.get("top_p", 0.9))
        ids = chat_prompt_ids(self.tokenizer, messages)
        input_ids = torch.tensor([ids], device=self.model.device)
        gen_kw = dict(max_new_tokens=max_tokens, do_sample=temperature > 0,
                      pad_token_id=getattr(self.tokenizer, "eos_token_id", 2))
        if temperature > 0:
            gen_kw.update(temperature=temperature, top_p=top_p)
        if params.get("ignore_eos"):
            gen_kw["min_new_tokens"] = max_tokens
        with torch.no_grad():
            out = self.model.generate(input_ids=input_ids, attention_mask=torch.ones_like(input_ids), **gen_kw)
        new = out[0][len(ids):].tolist()
        text = self.tokenizer.decode(new, skip_special_tokens=True)
        eos = getattr(self.tokenizer, "eos_token_id", None)
        reason = "stop" if (new and new[-1] == eos) else "length"
        return {"response": text, "tokens": new,
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(new), "total_tokens": len(ids) + len(new)},
                "finish_reason": reason}

    def batch_inference(self, params_list):
        return [self.inference(p) for p in params_list]

    def unload_model(self) -> None:
        self.model = None
        self.tokenizer = None
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        self.loaded = False


__all__ = ["LLMEngine", "ByteTokenizer"]
