"""Parity of the decoder/encoder implementations against HuggingFace transformers (CPU, fp32).

transformers is installed in the image, so these pin numerics against the library the real
checkpoints come from: our forward (paged KV, fused QKV/gate-up, torch-reference ops) must
reproduce HF logits, and engine greedy generation must reproduce ``model.generate``.
"""
import dataclasses

import pytest
import torch

transformers = pytest.importorskip("transformers")

from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
from financial_chatbot_llm_amd.models.common import AttentionMetadata, KVCache
from financial_chatbot_llm_amd.models.configs import ModelConfig, get_model_config
from financial_chatbot_llm_amd.models.llama import LlamaModel
from financial_chatbot_llm_amd.models.mixtral import MixtralModel
from financial_chatbot_llm_amd.models.weights import hf_decoder_to_internal
from financial_chatbot_llm_amd.ops.attention import KV_BS


def _hf_llama(moe=False, seed=0):
    torch.manual_seed(seed)
    kw = dict(vocab_size=512, hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, head_dim=32, max_position_embeddings=512, rms_norm_eps=1e-5,
              rope_theta=500000.0, tie_word_embeddings=False)
    if moe:
        cfg = transformers.MixtralConfig(num_local_experts=4, num_experts_per_tok=2, **kw)
        m = transformers.MixtralForCausalLM(cfg)
    else:
        cfg = transformers.LlamaConfig(**kw)
        m = transformers.LlamaForCausalLM(cfg)
    with torch.no_grad():  # HF inits norms to 1 and small weights; perturb norms to catch mix-ups
        for n, p in m.named_parameters():
            if "norm" in n:
                p.add_(torch.randn_like(p) * 0.1)
    return m.float().eval()


def _ours(hf, moe=False):
    c = hf.config
    mc = ModelConfig("hf-tiny", "mixtral" if moe else "llama", c.vocab_size, c.hidden_size, c.num_hidden_layers,
                     c.num_attention_heads, c.num_key_value_heads, c.head_dim, c.intermediate_size,
                     max_position=c.max_position_embeddings, rope_theta=500000.0, norm_eps=c.rms_norm_eps,
                     num_experts=4 if moe else 0, top_k_experts=2 if moe else 0, eos_token_ids=(1,))
    cls = MixtralModel if moe else LlamaModel
    m = cls(mc, device="cpu", tp_rank=0, tp_size=1, dtype=torch.float32)
    m.load_state(hf_decoder_to_internal(hf.state_dict(), mc.num_layers, mc.num_experts))
    return m


def _prefill_logits(m, ids):
    T = len(ids)
    nb = (T + KV_BS - 1) // KV_BS
    kv = KVCache(m.cfg.num_layers, nb + 1, m.hkv, m.D, dtype=torch.float32, device="cpu")
    bt = torch.arange(1, nb + 1, dtype=torch.int32)[None]
    slots = torch.tensor([int(bt[0, p // KV_BS]) * KV_BS + p % KV_BS for p in range(T)], dtype=torch.int32)
    meta = AttentionMetadata(slots=slots, num_prefill_tokens=T, cu_q=torch.tensor([0, T], dtype=torch.int32),
                             ctx_lens_p=torch.tensor([T], dtype=torch.int32), block_tables_p=bt, max_q_len=T)
    h = m.forward(torch.tensor(ids, dtype=torch.int32), torch.arange(T, dtype=torch.int32), meta, kv)
    return m.logits(h)


@pytest.mark.parametrize("moe", [False, True])
def test_logits_match_hf(moe):
    hf = _hf_llama(moe)
    ours = _ours(hf, moe)
    ids = torch.randint(0, 512, (1, 150), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(ids).logits[0]
    got = _prefill_logits(ours, ids[0].tolist())
    assert torch.allclose(got, ref, atol=2e-4, rtol=1e-3), (got - ref).abs().max()


@pytest.mark.parametrize("moe", [False, True])
def test_engine_greedy_matches_hf_generate(moe):
    hf = _hf_llama(moe, seed=3)
    ours = _ours(hf, moe)
    prompt = torch.randint(2, 512, (1, 70), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = hf.generate(prompt, max_new_tokens=12, do_sample=False, eos_token_id=None, pad_token_id=0)[0, 70:].tolist()
    ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=512,
                        max_num_batched_tokens=32, use_cuda_graph=False)  # 32-token chunks: chunked prefill
    from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
    eng = LLMEngine(ecfg, model=ours, tokenizer=SyntheticLlamaTokenizer(512))
    out = eng.generate([prompt[0].tolist()], SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True))[0]
    assert out == ref


def test_prefix_cache_hit_same_output():
    hf = _hf_llama(False, seed=4)
    ours = _ours(hf)
    from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
    ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=512,
                        max_num_batched_tokens=512, use_cuda_graph=False)
    eng = LLMEngine(ecfg, model=ours, tokenizer=SyntheticLlamaTokenizer(512))
    p = torch.randint(2, 512, (200,), generator=torch.Generator().manual_seed(5)).tolist()
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    a = eng.generate([p], sp)[0]
    assert eng.bm.hits == 0
    b = eng.generate([p], sp)[0]
    assert eng.bm.hits == 3 and a == b       # 3 full 64-token blocks served from the cache
    c = eng.generate([p + a + [5, 6, 7]], sp)[0]  # next "turn" extends the previous prompt
    assert eng.bm.hits >= 6


def test_bert_cls_matches_hf():
    from financial_chatbot_llm_amd.models.bert import BertEncoder
    from financial_chatbot_llm_amd.models.weights import hf_bert_to_internal
    torch.manual_seed(0)
    hc = transformers.BertConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                 intermediate_size=128, max_position_embeddings=128, layer_norm_eps=1e-12)
    hf = transformers.BertModel(hc, add_pooling_layer=False).float().eval()
    mc = ModelConfig("bert-t", "bert", 300, 64, 2, 2, 2, 32, 128, max_position=128, norm_eps=1e-12, type_vocab_size=2)
    ours = BertEncoder(mc, device="cpu", dtype=torch.float32).load_state(hf_bert_to_internal(hf.state_dict(), 2))
    seqs = [[101, 5, 9, 77, 102], [101] + list(range(10, 90)) + [102]]
    got = ours.encode(seqs)
    for i, s in enumerate(seqs):
        with torch.no_grad():
            ref = hf(torch.tensor([s])).last_hidden_state[0, 0]
        assert torch.allclose(got[i], torch.nn.functional.normalize(ref, dim=-1), atol=1e-4)


def test_mixtral_fp8_expert_path_cpu():
    """fp8 e4m3 experts (tiled + per-row scales), eager bucketed path: close to the bf16 experts."""
    cfg = get_model_config("mixtral-tiny")
    m = MixtralModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=3, std=0.05)
    ids = list(range(20, 90))
    ref = _prefill_logits(m, ids)
    m.quantize_experts()
    assert "layers.0.w13_t" in m.w and "layers.0.w13" not in m.w
    got = _prefill_logits(m, ids)
    # random tiny model: many near-tied logits, so bound the mean error (~3 %) and a loose argmax agreement
    assert (got - ref).abs().mean() < 0.05 * ref.abs().mean()
    assert (got.argmax(-1) == ref.argmax(-1)).float().mean() > 0.7
