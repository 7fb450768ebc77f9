"""Query/document embedders replacing ``OpenAIEmbeddings.embed_query`` (``tools/qdrant_tool.py:137``).

* :class:`HashEmbedder` -- deterministic signed feature hashing of word unigrams/bigrams on
  the host; lexically meaningful, used by the CPU plumbing config and tests.
* :class:`BgeEmbedder` -- bge-base-en architecture (12-layer BERT, d=768, CLS pooling,
  L2-normalised) running on the GPU through ``models.bert`` (K14: HIP LayerNorm/GELU/attention
  kernels + hipBLASLt GEMMs).
"""
from __future__ import annotations

import hashlib
import re
from typing import List, Sequence

import numpy as np

_WORD = re.compile(r"[a-z0-9]+")


def _h(tok: str) -> int:
    return int.from_bytes(hashlib.blake2b(tok.encode(), digest_size=8).digest(), "little")


class HashEmbedder:
    def __init__(self, dim: int = 768):
        self.dim = dim

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        out = np.zeros((len(texts), self.dim), np.float32)
        for i, t in enumerate(texts):
            words = _WORD.findall(t.lower())
            feats = words + [a + "_" + b for a, b in zip(words, words[1:])]
            for f in feats:
                h = _h(f)
                out[i, h % self.dim] += 1.0 if (h >> 63) & 1 else -1.0
            n = np.linalg.norm(out[i])
            if n > 0:
                out[i] /= n
            else:
                out[i, 0] = 1.0
        return out

    def embed_query(self, text: str) -> List[float]:
        return self.embed([text])[0].tolist()


class BgeEmbedder:
    """On-device bge-base-en encoder.  Random-init unless ``weights`` (an HF safetensors file or
    directory) is given; real WordPiece ids when ``vocab`` (``vocab.txt`` / ``tokenizer.json``)
    is given -- real weights need the real vocabulary, hashed ids would make them meaningless."""

    def __init__(self, model_name: str = "bge-base-en", device: str = "cuda", weights: str = None,
                 max_len: int = 64, seed: int = 0, vocab: str = None):
        from ..models.bert import BertEncoder
        from ..models.configs import get_model_config
        from ..engine.tokenizer import load_wordpiece
        self.cfg = get_model_config(model_name)
        self.dim = self.cfg.hidden_size
        self.tokenizer = load_wordpiece(vocab, self.cfg.vocab_size)
        self.model = BertEncoder.build(self.cfg, device=device, weights=weights, seed=seed)
        self.max_len = min(max_len, self.cfg.max_position)

    def tokenize(self, texts: Sequence[str], max_len: int = None) -> List[List[int]]:
        # truncation keeps [SEP] (the encoder was trained on [CLS] ... [SEP])
        return self.tokenizer.encode_batch(list(texts), max_len or self.max_len)

    def embed(self, texts: Sequence[str], max_len: int = None):
        return self.model.encode(self.tokenize(texts, max_len))

    def embed_query(self, text: str) -> List[float]:
        return self.embed([text])[0].float().cpu().tolist()
