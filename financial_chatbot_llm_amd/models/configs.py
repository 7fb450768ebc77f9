"""Model architecture registry (SURVEY §2.B shapes).

Public shapes of the north-star models plus tiny variants for CPU/GPU tests.  ``from_hf`` maps
a HuggingFace ``config.json`` onto :class:`ModelConfig` so real checkpoints can be served.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str                       # "llama" | "mixtral" | "bert"
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    max_position: int = 8192
    rope_theta: float = 500000.0
    rope_scaling: Optional[Dict] = None
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    num_experts: int = 0
    top_k_experts: int = 0
    type_vocab_size: int = 0        # bert
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)
    pad_token_id: int = 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, F, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * F * (self.num_experts or 1) + (H * self.num_experts if self.num_experts else 0)
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H


_LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                   "original_max_position_embeddings": 8192}

REGISTRY: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama3-8b", "llama", 128256, 4096, 32, 32, 8, 128, 14336),
    "llama3.1-8b": ModelConfig("llama3.1-8b", "llama", 128256, 4096, 32, 32, 8, 128, 14336, max_position=131072,
                               rope_scaling=_LLAMA3_SCALING),
    "llama3-70b": ModelConfig("llama3-70b", "llama", 128256, 8192, 80, 64, 8, 128, 28672),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32000, 4096, 32, 32, 8, 128, 14336, max_position=32768,
                                rope_theta=1e6, num_experts=8, top_k_experts=2, bos_token_id=1, eos_token_ids=(2,)),
    "bge-base-en": ModelConfig("bge-base-en", "bert", 30522, 768, 12, 12, 12, 64, 3072, max_position=512,
                               norm_eps=1e-12, type_vocab_size=2, bos_token_id=101, eos_token_ids=(102,)),
    # tiny variants for tests / smoke (same code paths, GQA and MoE preserved)
    "llama-tiny": ModelConfig("llama-tiny", "llama", 128256, 256, 2, 8, 2, 128, 512),
    "llama-tiny-tp": ModelConfig("llama-tiny-tp", "llama", 4096, 256, 2, 8, 4, 64, 384, max_position=2048),
    "mixtral-tiny": ModelConfig("mixtral-tiny", "mixtral", 32000, 256, 2, 8, 2, 128, 384, max_position=4096,
                                rope_theta=1e6, num_experts=4, top_k_experts=2, bos_token_id=1, eos_token_ids=(2,)),
    "bert-tiny": ModelConfig("bert-tiny", "bert", 30522, 128, 2, 2, 2, 64, 512, max_position=512,
                             norm_eps=1e-12, type_vocab_size=2, bos_token_id=101, eos_token_ids=(102,)),
}


def get_model_config(name: str) -> ModelConfig:
    if name in REGISTRY:
        return REGISTRY[name]
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        return from_hf(os.path.join(name, "config.json"))
    raise KeyError(f"unknown model {name!r}; known: {sorted(REGISTRY)}")


def from_hf(path: str, name: Optional[str] = None) -> ModelConfig:
    with open(path) as fh:
        c = json.load(fh)
    mt = c.get("model_type", "llama")
    if mt == "bert":
        return ModelConfig(name or "hf-bert", "bert", c["vocab_size"], c["hidden_size"], c["num_hidden_layers"],
                           c["num_attention_heads"], c["num_attention_heads"],
                           c["hidden_size"] // c["num_attention_heads"], c["intermediate_size"],
                           max_position=c.get("max_position_embeddings", 512),
                           norm_eps=c.get("layer_norm_eps", 1e-12), type_vocab_size=c.get("type_vocab_size", 2),
                           bos_token_id=101, eos_token_ids=(102,))
    eos = c.get("eos_token_id", 2)
    eos = tuple(eos) if isinstance(eos, list) else (eos,)
    heads = c["num_attention_heads"]
    return ModelConfig(
        name or f"hf-{mt}", "mixtral" if mt == "mixtral" else "llama", c["vocab_size"], c["hidden_size"],
        c["num_hidden_layers"], heads, c.get("num_key_value_heads", heads),
        c.get("head_dim") or c["hidden_size"] // heads, c["intermediate_size"],
        max_position=c.get("max_position_embeddings", 8192), rope_theta=c.get("rope_theta", 10000.0),
        rope_scaling=c.get("rope_scaling"), norm_eps=c.get("rms_norm_eps", 1e-5),
        tie_embeddings=c.get("tie_word_embeddings", False), num_experts=c.get("num_local_experts", 0),
        top_k_experts=c.get("num_experts_per_tok", 0), bos_token_id=c.get("bos_token_id", 1), eos_token_ids=eos)
