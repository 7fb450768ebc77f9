"""Checkpoint loading: HuggingFace safetensors -> internal fused/sharded layout.

Only safe loaders are used (``safetensors.safe_open``; never pickle).  Names handled:

* Llama: ``q/k/v_proj`` -> fused ``qkv``; ``gate/up_proj`` -> fused ``gate_up``.
* Mixtral: ``block_sparse_moe.experts.{e}.w1/w3/w2`` (original checkpoints) or
  ``mlp.experts.gate_up_proj/down_proj`` (transformers>=5 fused) -> ``w13`` [E, 2F, H], ``w2``.
* BERT/bge: ``embeddings.*``, ``encoder.layer.{i}.*`` -> fused ``qkv`` (+bias).
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, Iterable

import torch

_L = re.compile(r"^model\.layers\.(\d+)\.(.+)$")


def hf_decoder_to_internal(sd: Dict[str, torch.Tensor], num_layers: int, num_experts: int = 0) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {}
    layers: Dict[int, Dict[str, torch.Tensor]] = {i: {} for i in range(num_layers)}
    for k, v in sd.items():
        if k == "model.embed_tokens.weight":
            out["embed"] = v
        elif k == "model.norm.weight":
            out["final_norm"] = v
        elif k == "lm_head.weight":
            out["lm_head"] = v
        else:
            m = _L.match(k)
            if m:
                layers[int(m.group(1))][m.group(2)] = v
    for i, d in layers.items():
        p = f"layers.{i}."
        out[p + "in_norm"] = d["input_layernorm.weight"]
        out[p + "post_norm"] = d["post_attention_layernorm.weight"]
        out[p + "qkv"] = torch.cat([d["self_attn.q_proj.weight"], d["self_attn.k_proj.weight"],
                                    d["self_attn.v_proj.weight"]], 0)
        out[p + "o"] = d["self_attn.o_proj.weight"]
        if num_experts:
            if "mlp.experts.gate_up_proj" in d:
                out[p + "w13"] = d["mlp.experts.gate_up_proj"]
                out[p + "w2"] = d["mlp.experts.down_proj"]
                out[p + "router"] = d["mlp.gate.weight"]
            else:
                pre = "block_sparse_moe."
                out[p + "router"] = d[pre + "gate.weight"]
                out[p + "w13"] = torch.stack([torch.cat([d[f"{pre}experts.{e}.w1.weight"],
                                                         d[f"{pre}experts.{e}.w3.weight"]], 0)
                                              for e in range(num_experts)])
                out[p + "w2"] = torch.stack([d[f"{pre}experts.{e}.w2.weight"] for e in range(num_experts)])
        else:
            out[p + "gate_up"] = torch.cat([d["mlp.gate_proj.weight"], d["mlp.up_proj.weight"]], 0)
            out[p + "down"] = d["mlp.down_proj.weight"]
    return out


def hf_bert_to_internal(sd: Dict[str, torch.Tensor], num_layers: int) -> Dict[str, torch.Tensor]:
    sd = {k[len("bert."):] if k.startswith("bert.") else k: v for k, v in sd.items()}
    out = {
        "word_emb": sd["embeddings.word_embeddings.weight"],
        "pos_emb": sd["embeddings.position_embeddings.weight"],
        "type_emb": sd["embeddings.token_type_embeddings.weight"],
        "emb_ln_g": sd["embeddings.LayerNorm.weight"], "emb_ln_b": sd["embeddings.LayerNorm.bias"],
    }
    for i in range(num_layers):
        s, p = f"encoder.layer.{i}.", f"layers.{i}."
        a = s + "attention."
        out[p + "qkv"] = torch.cat([sd[a + "self.query.weight"], sd[a + "self.key.weight"], sd[a + "self.value.weight"]])
        out[p + "qkv_b"] = torch.cat([sd[a + "self.query.bias"], sd[a + "self.key.bias"], sd[a + "self.value.bias"]])
        out[p + "o"], out[p + "o_b"] = sd[a + "output.dense.weight"], sd[a + "output.dense.bias"]
        out[p + "ln1_g"], out[p + "ln1_b"] = sd[a + "output.LayerNorm.weight"], sd[a + "output.LayerNorm.bias"]
        out[p + "fc1"], out[p + "fc1_b"] = sd[s + "intermediate.dense.weight"], sd[s + "intermediate.dense.bias"]
        out[p + "fc2"], out[p + "fc2_b"] = sd[s + "output.dense.weight"], sd[s + "output.dense.bias"]
        out[p + "ln2_g"], out[p + "ln2_b"] = sd[s + "output.LayerNorm.weight"], sd[s + "output.LayerNorm.bias"]
    return out


def read_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors import safe_open
    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    if not files:
        raise FileNotFoundError(f"no .safetensors under {path}")
    sd: Dict[str, torch.Tensor] = {}
    for f in files:
        with safe_open(f, framework="pt") as fh:
            for k in fh.keys():
                sd[k] = fh.get_tensor(k)
    return sd


def load_decoder_weights(model, path: str) -> None:
    sd = read_safetensors(path)
    full = hf_decoder_to_internal(sd, model.cfg.num_layers, model.cfg.num_experts)
    if model.cfg.tie_embeddings:
        full.pop("lm_head", None)
    model.load_state(full)
    if getattr(model, "fp8", False):
        model.quantize_experts()
