"""Tokenizer loading without network access.

``load_tokenizer(model_id)`` returns a local HF tokenizer when the files are
on disk, otherwise a deterministic byte-level tokenizer (ids = byte + offset)
that round-trips any UTF-8 text — enough for the serving plumbing and for
synthetic-prompt benchmarks with random-init weights.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


class ByteTokenizer:
    """UTF-8 bytes -> ids ``offset + byte``; specials below ``offset``."""

    def __init__(self, vocab_size: int = 32000, bos_token_id: int = 1, eos_token_id: int = 2, offset: int = 3):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.pad_token_id = eos_token_id
        self.offset = offset

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [self.offset + b for b in text.encode("utf-8")]
        return ([self.bos_token_id] if add_bos else []) + ids

    # ids above the byte range (a random-init model samples them almost always) decode to one
    # U+25A1 each instead of nothing: every generated token is visible text, so a stream's
    # first chunk arrives with the first token and SSE TTFT measures what it says.  (Not U+FFFD:
    # that marks an incomplete UTF-8 sequence, which a StreamDecoder holds back.)
    UNKNOWN = "\u25a1".encode("utf-8")

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        off, unk = self.offset, self.UNKNOWN
        if skip_special_tokens:
            # one bytes object per id from a table (no per-id branches): ~4x faster on long outputs
            table = self._table
            return b"".join(table[i - off] if 0 <= i - off < 256 else (unk if i >= off else b"")
                            for i in map(int, ids)).decode("utf-8", errors="replace")
        out = bytearray()
        for i in ids:
            i = int(i)
            b = i - off
            if 0 <= b < 256:
                out.append(b)
            elif b >= 256:
                out.extend(unk)
            else:
                out.extend(f"<{i}>".encode())
        return out.decode("utf-8", errors="replace")

    _table = [bytes([b]) for b in range(256)]

    def apply_chat_template(self, messages: List[Dict[str, str]], tokenize: bool = False,
                            add_generation_prompt: bool = True):
        parts = [f"<|{m.get('role', 'user')}|>\n{m.get('content', '')}\n" for m in messages]
        if add_generation_prompt:
            parts.append("<|assistant|>\n")
        text = "".join(parts)
        return self.encode(text) if tokenize else text

    def __call__(self, text, return_tensors=None):
        import torch
        ids = self.encode(text)
        if return_tensors == "pt":
            class _Enc(dict):
                def to(self, dev):
                    return _Enc({k: v.to(dev) for k, v in self.items()})

                def __getattr__(self, k):
                    return self[k]
            t = torch.tensor([ids])
            return _Enc(input_ids=t, attention_mask=torch.ones_like(t))
        return {"input_ids": ids}


class StreamDecoder:
    """Incremental detokenization of one generated sequence: ``add(token_id)`` returns the text
    the token completes ("" while it only starts a multi-byte character).

    Decoding every token alone loses what depends on its neighbours (SentencePiece word-boundary
    spaces, UTF-8 characters split over byte tokens), and re-decoding the whole output each token
    costs O(n) per token.  This decodes a short window instead: the tokens since the last
    emitted prefix, against the text that prefix already produced (the prefix / read offset
    scheme of streaming LLM servers).  A trailing U+FFFD is an incomplete UTF-8 sequence and is
    held back until the next token completes it.  The emitted pieces concatenate to the full
    decode."""

    def __init__(self, tokenizer, skip_special_tokens: bool = True):
        self.tok = tokenizer
        self.skip = skip_special_tokens
        self.ids: List[int] = []
        self.prefix = 0          # start of the decode window
        self.read = 0            # tokens whose text is already emitted

    def _decode(self, ids) -> str:
        return self.tok.decode(ids, skip_special_tokens=self.skip)

    def add(self, token_id: int) -> str:
        self.ids.append(int(token_id))
        prefix_text = self._decode(self.ids[self.prefix:self.read])
        text = self._decode(self.ids[self.prefix:])
        if len(text) > len(prefix_text) and not text.endswith("\ufffd"):
            self.prefix, self.read = self.read, len(self.ids)
            return text[len(prefix_text):]
        return ""

    def flush(self) -> str:
        """Text still held back at the end of the sequence (an incomplete character)."""
        prefix_text = self._decode(self.ids[self.prefix:self.read])
        text = self._decode(self.ids[self.prefix:])
        self.prefix = self.read = len(self.ids)
        return text[len(prefix_text):] if len(text) > len(prefix_text) else ""


def load_tokenizer(model_id: Optional[str], vocab_size: int = 32000, bos: int = 1, eos: int = 2):
    if model_id and os.path.isdir(model_id):
        try:
            from transformers import AutoTokenizer
            return AutoTokenizer.from_pretrained(model_id, local_files_only=True)
        except Exception:
            pass
    if model_id:
        try:
            from transformers import AutoTokenizer
            return AutoTokenizer.from_pretrained(model_id, local_files_only=True)
        except Exception:
            pass
    return ByteTokenizer(vocab_size=vocab_size, bos_token_id=bos, eos_token_id=eos)


def chat_prompt_ids(tokenizer, messages: List[Dict[str, str]]) -> List[int]:
    try:
        text = tokenizer.apply_chat_template(messages, tokenize=False, add_generation_prompt=True)
    except Exception:
        text = "\n".join(f"{m.get('role', 'user')}: {m.get('content', '')}" for m in messages) + "\nassistant:"
    if isinstance(tokenizer, ByteTokenizer):
        return tokenizer.encode(text)
    return list(tokenizer(text)["input_ids"])
