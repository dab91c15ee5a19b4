"""Tokenizers.

The GPU box has no network, so checkpoints' tokenizers are only available when a
local model directory is given.  :func:`load_tokenizer` uses the HF
``tokenizers``/``transformers`` fast tokenizer from a local path when present,
otherwise a deterministic :class:`HashTokenizer` that maps words to stable ids
(synthetic prompts, random-init weights: the workloads' shapes, not their text,
set the cost).
"""
from __future__ import annotations

import os
import re
import zlib
from typing import List, Optional, Sequence

import torch

_WORDS = ("the a of and to in is it that on for with as was at by an be this from or are his her they we you "
          "image photo light warrior chief astronaut horse mars city river cat dog portrait detailed sky night "
          "blue red green gold old young sunset forest mountain ocean robot castle dragon flower garden").split()


class HashTokenizer:
    """Deterministic offline tokenizer: word -> crc32 bucket in [n_special, vocab)."""

    def __init__(self, vocab_size: int, bos_id: Optional[int] = None, eos_id: Optional[int] = None, pad_id: int = 0,
                 model_max_length: int = 77, n_special: int = 256, specials: Optional[dict] = None):
        self.vocab_size = vocab_size
        self.bos_token_id, self.eos_token_id, self.pad_token_id = bos_id, eos_id, pad_id
        self.model_max_length = model_max_length
        self.n_special = min(n_special, vocab_size // 4)
        # literal special-token strings (e.g. "<|image|>") -> fixed ids, matched before word splitting
        self.specials = dict(specials or {})
        self._special_re = (re.compile("(" + "|".join(re.escape(s) for s in sorted(self.specials, key=len,
                                                                                    reverse=True)) + ")")
                            if self.specials else None)
        fixed = {i for i in (bos_id, eos_id, pad_id) if i is not None}
        self._hi = vocab_size
        while self._hi - 1 in fixed:
            self._hi -= 1

    def _tok(self, w: str) -> int:
        span = max(1, self._hi - self.n_special)
        return self.n_special + zlib.crc32(w.encode()) % span

    def _words(self, text: str) -> List[int]:
        return [self._tok(w) for w in re.findall(r"\w+|[^\w\s]", text.lower())]

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        if self._special_re is None:
            ids = self._words(text)
        else:
            ids = []
            for part in self._special_re.split(text):
                ids += [self.specials[part]] if part in self.specials else self._words(part)
        if add_special_tokens:
            if self.bos_token_id is not None and not (ids and ids[0] == self.bos_token_id):
                ids = [self.bos_token_id] + ids
            if self.eos_token_id is not None:
                ids = ids + [self.eos_token_id]
        return ids

    def __call__(self, texts: Sequence[str] | str, max_length: Optional[int] = None, padding: str = "max_length",
                 truncation: bool = True, return_tensors: str = "pt"):
        if isinstance(texts, str):
            texts = [texts]
        L = max_length or self.model_max_length
        rows = []
        for t in texts:
            ids = self.encode(t)
            if truncation and len(ids) > L:
                ids = ids[: L - 1] + ([self.eos_token_id] if self.eos_token_id is not None else [ids[L - 1]])
            rows.append(ids)
        if padding == "max_length":
            width = L
        else:
            width = max(len(r) for r in rows)
        ids = torch.full((len(rows), width), self.pad_token_id, dtype=torch.long)
        mask = torch.zeros((len(rows), width), dtype=torch.long)
        for i, r in enumerate(rows):
            ids[i, : len(r)] = torch.tensor(r)
            mask[i, : len(r)] = 1
        return {"input_ids": ids, "attention_mask": mask}

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out = []
        for i in (ids.tolist() if hasattr(ids, "tolist") else ids):
            if skip_special_tokens and i in (self.bos_token_id, self.eos_token_id, self.pad_token_id):
                continue
            out.append(_WORDS[i % len(_WORDS)])
        return " ".join(out)

    def apply_chat_template(self, messages, add_generation_prompt=True, tokenize=False):
        text = "\n".join(f"{m['role']}: {m['content'] if isinstance(m['content'], str) else ''}" for m in messages)
        return text + ("\nassistant:" if add_generation_prompt else "")


def load_tokenizer(path: Optional[str], *, vocab_size: int, bos_id=None, eos_id=None, pad_id=0,
                   model_max_length: int = 77, subfolder: Optional[str] = None, specials: Optional[dict] = None):
    """HF fast tokenizer from a local directory if available, else HashTokenizer."""
    if path:
        d = os.path.join(path, subfolder) if subfolder else path
        if os.path.isdir(d) and any(os.path.exists(os.path.join(d, f)) for f in
                                    ("tokenizer.json", "vocab.json", "tokenizer.model", "spiece.model", "vocab.txt")):
            try:
                from transformers import AutoTokenizer
                tok = AutoTokenizer.from_pretrained(d, local_files_only=True)
                return tok
            except Exception:  # pragma: no cover - depends on local files
                pass
    return HashTokenizer(vocab_size, bos_id, eos_id, pad_id, model_max_length, specials=specials)
