"""Decoder-level check of the prefill GEMM paths (ops/gemm.py PREFILL_POLICY) at the REAL
Llama-3-8B layer shapes (2 layers): the measured policy (tile kernels with the fused QKV+RoPE,
SiLU, split-K slab and in-place residual epilogues, hipBLASLt where measured faster), every tile
kernel forced (``PENNY_PREFILL_GEMM=force``: O / down add the residual stream in their epilogue),
and hipBLASLt everywhere (``=0``) must give the same final hidden states up to bf16 rounding."""
import dataclasses

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from financial_chatbot_llm_amd.models.configs import get_model_config
    from financial_chatbot_llm_amd.models.llama import LlamaModel
    cfg = dataclasses.replace(get_model_config("llama3-8b"), name="llama3-8b-2l", num_layers=2)
    return LlamaModel(cfg, device="cuda").init_random(seed=3, std=0.02)


def _hidden(m, T):
    from financial_chatbot_llm_amd.models.common import AttentionMetadata, KVCache
    from financial_chatbot_llm_amd.ops.attention import KV_BS
    nb = (T + KV_BS - 1) // KV_BS
    kv = KVCache(m.cfg.num_layers, nb + 1, m.hkv, m.D, device="cuda")
    bt = torch.arange(1, nb + 1, dtype=torch.int32, device="cuda")[None]
    p = torch.arange(T, dtype=torch.int32, device="cuda")
    slots = ((1 + p // KV_BS) * KV_BS + p % KV_BS).to(torch.int32)
    meta = AttentionMetadata(slots=slots, num_prefill_tokens=T,
                             cu_q=torch.tensor([0, T], dtype=torch.int32, device="cuda"),
                             ctx_lens_p=torch.tensor([T], dtype=torch.int32, device="cuda"), block_tables_p=bt,
                             max_q_len=T)
    ids = ((p * 37 + 11) % 120000 + 100).to(torch.int32)
    with torch.no_grad():
        return m.forward(ids, p, meta, kv).float()


@pytest.mark.parametrize("T", [1536, 4096])
def test_prefill_gemm_paths_agree_on_llama3_8b_layers(T, monkeypatch):
    m = _model()
    out = {}
    for mode in ("0", "1", "force"):
        monkeypatch.setenv("PENNY_PREFILL_GEMM", mode)
        out[mode] = _hidden(m, T)
    ref = out["0"]
    scale = ref.abs().max().item()
    for mode in ("1", "force"):
        err = (out[mode] - ref).abs()
        cos = torch.nn.functional.cosine_similarity(out[mode], ref, dim=-1)
        assert err.max().item() < 0.05 * scale, (mode, err.max().item(), scale)
        assert cos.min().item() > 0.999, (mode, cos.min().item())
