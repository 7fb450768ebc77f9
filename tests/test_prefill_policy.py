"""Host-side logic of the prefill GEMM policy (ops/gemm.py) and its fused-residual path, on CPU."""
import torch

from financial_chatbot_llm_amd import ops
from financial_chatbot_llm_amd.ops import gemm


def test_policy_table_choices(monkeypatch):
    monkeypatch.delenv("PENNY_PREFILL_GEMM", raising=False)
    # O: the 128 x 128 tile's slabs at small steps, 256 x 256 split-K slabs, then the residual
    # epilogue, where the caller can take them, else the library
    assert gemm.prefill_choice(4096, 4096, 4096, None, True, fused_residual=True) == "R"
    assert gemm.prefill_choice(4096, 4096, 4096, None, True, fused_residual=False) == "lib"
    assert gemm.prefill_choice(2048, 4096, 4096, None, True, fused_residual=True) == "S2"
    assert gemm.prefill_choice(1536, 4096, 4096, None, True, fused_residual=True) == "S2"
    assert gemm.prefill_choice(512, 4096, 4096, None, True, fused_residual=True) == "M2"
    assert gemm.prefill_choice(320, 4096, 4096, None, True, fused_residual=True) == "M4"
    # down: 128 x 128 slabs to 512 rows, 256 x 256 slabs only when the consumer reads slabs
    assert gemm.prefill_choice(384, 4096, 14336, None, slabs=True) == "M4"
    assert gemm.prefill_choice(1024, 4096, 14336, None, slabs=True) == "S4"
    assert gemm.prefill_choice(1024, 4096, 14336, None, slabs=False) == "lib"
    assert gemm.prefill_choice(1280, 4096, 14336, None, slabs=True) == "hip"
    # gate|up + SiLU on the tile kernel at every prefill size
    assert gemm.prefill_choice(512, 28672, 4096, "silu") == "hip"
    assert gemm.prefill_choice(257, 28672, 4096, "silu") == "hip"
    # 70B TP=8 shards (r6): the 128 x 128 tile kernel at small steps, the 256 x 256 one above; no
    # SURVEY-named shard takes hipBLASLt at any prefill size
    assert gemm.prefill_choice(384, 8192, 1024, None) == "M1"
    assert gemm.prefill_choice(4096, 8192, 1024, None) == "hip"
    assert gemm.prefill_choice(384, 1280, 8192, None, slabs=True) == "M8"
    assert gemm.prefill_choice(2048, 1280, 8192, None, slabs=True) == "S4"
    assert gemm.prefill_choice(384, 7168, 8192, "silu") == "M4"
    assert gemm.prefill_choice(2048, 7168, 8192, "silu") == "hip"
    assert gemm.prefill_choice(384, 8192, 3584, None) == "M2"
    assert gemm.prefill_choice(3072, 8192, 3584, None) == "hip"
    shards = [(1280, 8192, None, True), (8192, 1024, None, False), (7168, 8192, "silu", False),
              (8192, 3584, None, False), (10240, 8192, None, True)]
    for n, k, epi, slabs in shards:
        for m in (257, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 8192):
            assert gemm.prefill_choice(m, n, k, epi, slabs=slabs) != "lib", (n, k, m)
    # force: every tile path, the residual epilogue where offered
    monkeypatch.setenv("PENNY_PREFILL_GEMM", "force")
    assert gemm.prefill_choice(512, 4096, 4096, None, True, fused_residual=True) == "R"
    assert gemm.prefill_choice(512, 4096, 4096, None, False) == "hip"
    monkeypatch.setenv("PENNY_PREFILL_GEMM", "0")
    assert gemm.prefill_choice(4096, 4096, 4096, None, True, fused_residual=True) == "lib"


def test_residual_sum_norm_equals_add_then_norm():
    """GEMM adding the residual in place + plain RMSNorm == GEMM -> add&RMSNorm (CPU reference path)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(300, 128, generator=g).bfloat16()
    w = (torch.randn(256, 128, generator=g) * 0.05).bfloat16()
    nw = torch.rand(256, generator=g).bfloat16() + 0.5
    r1 = torch.randn(300, 256, generator=g).bfloat16()
    r2 = r1.clone()
    y = gemm.prefill_gemm(x, w)
    h_ref = ops.rms_norm(y, nw, 1e-5, residual=r1)                 # r1 <- y + r1
    rs = gemm.ResidualSum(gemm.prefill_gemm(x, w, "residual", residual=r2, out=r2))
    h = ops.rms_norm(rs, nw, 1e-5, residual=r2)
    assert rs.t is r2
    assert torch.allclose(r2.float(), r1.float(), atol=2e-2)
    assert torch.allclose(h.float(), h_ref.float(), atol=3e-2)


def test_fused_lm_head_gating(monkeypatch):
    """The fused LM head + sampler is taken on the device only, for a vocabulary that tiles by 256:
    the tile kernel from FUSED_LM_HEAD_MIN_M rows, the weight-streaming kernel below (off with
    PENNY_LM_STREAM=0); PENNY_FUSED_LM_HEAD=0 / force override."""
    from financial_chatbot_llm_amd.ops import sampling
    w = torch.zeros(512, 128, dtype=torch.bfloat16)
    h = torch.zeros(200, 128, dtype=torch.bfloat16)
    monkeypatch.delenv("PENNY_FUSED_LM_HEAD", raising=False)
    assert not sampling.fused_lm_head_ok(h, w)                 # CPU tensors: no native kernel
    monkeypatch.setattr(sampling.N, "use_native", lambda t: True)
    assert sampling.fused_lm_head_ok(h, w)
    assert sampling.fused_lm_head_ok(h[:sampling.FUSED_LM_HEAD_MIN_M - 1], w)     # streaming kernel
    assert sampling.stream_cfg(1) == (4, True) and sampling.stream_cfg(127)[0] == 8
    monkeypatch.setenv("PENNY_LM_STREAM", "0")
    assert not sampling.fused_lm_head_ok(h[:sampling.FUSED_LM_HEAD_MIN_M - 1], w)
    monkeypatch.delenv("PENNY_LM_STREAM")
    assert not sampling.fused_lm_head_ok(h, torch.zeros(500, 128, dtype=torch.bfloat16))   # V % 256
    monkeypatch.setenv("PENNY_FUSED_LM_HEAD", "force")
    assert sampling.fused_lm_head_ok(h[:1], w)
    monkeypatch.setenv("PENNY_FUSED_LM_HEAD", "0")
    assert not sampling.fused_lm_head_ok(h, w)


def test_context_parallel_prefix_length():
    """CP prefills all but the prompt's last token, rounded down to whole zig-zag chunk pairs."""
    from financial_chatbot_llm_amd.engine.context_prefill import cp_prefix_len
    assert cp_prefix_len(301, 2) == 300
    assert cp_prefix_len(300, 2) == 296
    assert cp_prefix_len(100_001, 8) == 100_000
    assert cp_prefix_len(5, 4) == 0
