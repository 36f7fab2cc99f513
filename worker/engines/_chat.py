"""Chat-message formatting shared by the external-server adapters."""
from __future__ import annotations

from typing import Dict, List


def format_messages(tokenizer, messages: List[Dict[str, str]]) -> str:
    """The tokenizer's chat template when it has one, else ``role: content`` lines + ``assistant:``."""
    if tokenizer is not None and hasattr(tokenizer, "apply_chat_template"):
        try:
            return tokenizer.apply_chat_template(messages, tokenize=False, add_generation_prompt=True)
        except Exception:
            pass
    lines = [f"{m.get('role', 'user')}: {m.get('content', '')}" for m in messages]
    return "\n".join(lines + ["assistant:"])
