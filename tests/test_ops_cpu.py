"""CPU checks of the op reference paths (the oracles for the HIP kernels) and the paged layout."""
import math

import torch

from financial_chatbot_llm_amd import ops
from financial_chatbot_llm_amd.ops.attention import KV_BS, gather_kv_ref, kv_index_tables, write_kv_ref


def test_kv_tiles_are_fragment_native_permutations():
    for D in (64, 128):
        ki, vi = kv_index_tables(D)
        assert sorted(ki.flatten().tolist()) == list(range(KV_BS * D))
        assert sorted(vi.flatten().tolist()) == list(range(KV_BS * D))
        # a K row's 8 consecutive dims are one contiguous 16-byte piece
        assert all(int(ki[k, 8 * c + 7] - ki[k, 8 * c]) == 7 for k in range(KV_BS) for c in range(D // 8))
        # V fragment of (dim tile 0, key step 0, lane 16g+row) = keys {4g..4g+3, 16+4g..16+4g+3} of that dim
        for g in range(4):
            for row in (0, 5):
                base = (g * 16 + row) * 8
                keys = sorted(k for k in range(32) if base <= int(vi[k, row]) < base + 8)
                assert keys == [4 * g + j for j in range(4)] + [16 + 4 * g + j for j in range(4)]


def test_paged_roundtrip():
    Hkv, D, nb = 2, 64, 5
    kc = torch.zeros(nb, Hkv, KV_BS * D)
    vc = torch.zeros(nb, Hkv, KV_BS * D)
    L = 150
    blocks = torch.tensor([3, 0, 4], dtype=torch.int32)
    slots = torch.tensor([int(blocks[i // KV_BS]) * KV_BS + i % KV_BS for i in range(L)], dtype=torch.int32)
    k, v = torch.randn(L, Hkv, D), torch.randn(L, Hkv, D)
    write_kv_ref(k, v, slots, kc, vc)
    k2, v2 = gather_kv_ref(kc, vc, blocks, L)
    assert torch.equal(k, k2) and torch.equal(v, v2)


def test_prefill_ref_chunked_equals_full():
    torch.manual_seed(0)
    Hq, Hkv, D, L = 4, 2, 32, 90
    kc = torch.zeros(4, Hkv, KV_BS * D)
    vc = torch.zeros(4, Hkv, KV_BS * D)
    blocks = torch.tensor([[2, 1]], dtype=torch.int32)
    slots = torch.tensor([int(blocks[0, i // KV_BS]) * KV_BS + i % KV_BS for i in range(L)], dtype=torch.int32)
    write_kv_ref(torch.randn(L, Hkv, D), torch.randn(L, Hkv, D), slots, kc, vc)
    q = torch.randn(L, Hq, D)
    s = 1 / math.sqrt(D)
    full = ops.prefill(q, torch.tensor([0, L], dtype=torch.int32), torch.tensor([L], dtype=torch.int32), blocks,
                       kc, vc, s)
    # second chunk only (prefix-cache hit of 60 tokens)
    tail = ops.prefill(q[60:], torch.tensor([0, L - 60], dtype=torch.int32), torch.tensor([L], dtype=torch.int32),
                       blocks, kc, vc, s)
    assert torch.allclose(full[60:], tail, atol=1e-5)
    dec = ops.decode(q[-1:], torch.tensor([L], dtype=torch.int32), blocks, kc, vc, s)
    assert torch.allclose(full[-1:], dec, atol=1e-5)


def test_rope_matches_complex_rotation():
    D, T = 64, 3
    cs = ops.rope_cos_sin(D, 16, 10000.0)
    Hq, Hkv = 1, 1
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D)
    pos = torch.tensor([0, 1, 5], dtype=torch.int32)
    kc = torch.zeros(1, Hkv, KV_BS * D)
    vc = torch.zeros(1, Hkv, KV_BS * D)
    q = ops.rope_kv_write(qkv, pos, cs, torch.tensor([0, 1, 2], dtype=torch.int32), kc, vc, Hq, Hkv, D)
    x = qkv[:, :D]
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2).double() / D))
    for t in range(T):
        c = torch.complex(x[t, : D // 2].double(), x[t, D // 2:].double()) * torch.exp(1j * pos[t].double() * inv)
        assert torch.allclose(q[t, 0], torch.cat([c.real, c.imag]).float(), atol=1e-5)


def test_llama3_rope_scaling_changes_low_freqs_only():
    a = ops.attention.rope_inv_freq(128, 500000.0)
    b = ops.attention.rope_inv_freq(128, 500000.0, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                    "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    assert torch.allclose(a[:10], b[:10]) and (b[-5:] < a[-5:]).all()


def test_sampler_ref_greedy_and_topk_mask():
    lg = torch.randn(3, 50)
    ids = ops.sample(lg, torch.zeros(3), torch.zeros(3, dtype=torch.int64))
    assert ids.tolist() == lg.argmax(-1).tolist()
    m = ops.apply_top_k_top_p(lg, torch.tensor([2, 0, 0]), torch.tensor([1.0, 1.0, 1e-6]))
    assert torch.isfinite(m[0]).sum() == 2 and torch.isfinite(m[1]).sum() == 50 and torch.isfinite(m[2]).sum() == 1


def test_filtered_topk_ref():
    corpus = torch.nn.functional.normalize(torch.randn(100, 16), dim=-1)
    users = torch.arange(100, dtype=torch.int32) % 4
    dates = torch.arange(100, dtype=torch.int64)
    q = corpus[[8, 9]].clone()
    ids, sc, cnt = ops.filtered_topk(corpus, users, dates, q, torch.tensor([0, 1], dtype=torch.int32),
                                     torch.tensor([0, 50], dtype=torch.int64), torch.tensor([3, 100]), 100)
    assert ids[0, 0] == 8 and cnt[0] == 3
    assert cnt[1] == 12 and (ids[1, :12] >= 50).all() and (ids[1, :12] % 4 == 1).all()


def test_splitk_slabs_cpu_reference_and_consumers():
    """CPU path of the split-K op: slabs sum to x @ w.T, and the slab-aware consumers
    (rms_norm, rope_kv_write) equal the same ops on the reduced activation."""
    from financial_chatbot_llm_amd import ops
    from financial_chatbot_llm_amd.ops.gemm import Slabs, splitk_partials, tile_weight, untile_weight
    g = torch.Generator().manual_seed(0)
    w = torch.randn(128, 256, generator=g).to(torch.bfloat16)
    assert torch.equal(untile_weight(tile_weight(w)), w)
    x = torch.randn(9, 256, generator=g).to(torch.bfloat16)
    P = splitk_partials(x, tile_weight(w), 128, 4, 4)
    assert P.shape == (4, 9, 128)
    assert torch.allclose(P.sum(0), x.float() @ w.float().t(), atol=1e-4)
    nw = torch.ones(128, dtype=torch.bfloat16)
    r1 = torch.randn(9, 128, generator=g).to(torch.bfloat16)
    r2 = r1.clone()
    assert torch.equal(ops.rms_norm(Slabs(P), nw, 1e-5, residual=r1), ops.rms_norm(Slabs(P).materialize(), nw, 1e-5,
                                                                                   residual=r2))
    assert torch.equal(r1, r2)


def test_gateup_splitk_cpu_reference():
    """CPU path of the split-K gate|up op: the SiLU*up of the summed slabs (interleave16 layout)."""
    from financial_chatbot_llm_amd.ops import gemm
    from financial_chatbot_llm_amd.ops.activation import silu_mul
    g = torch.Generator().manual_seed(1)
    gate, up = torch.randn(64, 256, generator=g).to(torch.bfloat16), torch.randn(64, 256, generator=g).to(torch.bfloat16)
    wi = gemm.interleave16(gate, up)
    x = torch.randn(5, 256, generator=g).to(torch.bfloat16)
    y = gemm.gateup_splitk(x, wi, 128, 4, 2, rowmajor=True)
    ref = silu_mul((x.float() @ wi.float().t()).to(torch.bfloat16), interleave16=True)
    assert y.shape == (5, 64)
    assert torch.allclose(y.float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_decode_gemm_dispatch_tables(monkeypatch):
    """Which decode kernel a projection shape gets, and whether it keeps a tiled weight copy."""
    from financial_chatbot_llm_amd.ops import gemm
    # Llama-3-8B: measured split-K / fused gate|up configs, tiled copies
    assert gemm.splitk_config(128, 6144, 4096) == (4, 6)
    assert gemm.splitk_config(300, 6144, 4096) is None              # prefill size: the tile kernels
    assert gemm.gateup_config(128, 28672, 4096) == 8 and gemm.gateup_config(200, 28672, 4096) == 8
    assert gemm.gateup_config(300, 28672, 4096) is None
    # 70B gate|up: split-K + reduce-SiLU (TP=8 shard tiled, TP=1 row-major at M <= 16 only)
    assert gemm.gateup_splitk_config(64, 7168, 8192) == (2, 4, False)
    assert gemm.gateup_splitk_config(200, 7168, 8192) == (4, 8, False)
    assert gemm.gateup_splitk_config(1, 57344, 8192) == (8, 2, True)
    assert gemm.gateup_splitk_config(32, 57344, 8192) is None
    # the 70B TP=1 gate|up keeps only its tiled copy (TILED_ONLY), else no tiled copy at all (75 GB)
    assert gemm.uses_tiled_weight(7168, 8192)
    assert gemm.uses_tiled_weight(57344, 8192) == gemm.tiled_only(57344, 8192)
    assert gemm.uses_tiled_weight(6144, 4096) and gemm.uses_tiled_weight(28672, 4096)
    # Llama-3-70B TP=1 (r5 re-measure): split-K on the row-major stream at every decode M, no copies
    assert gemm.splitk_config(32, 8192, 8192) == (8, 2) and gemm.splitk_config(128, 8192, 8192) == (8, 8)
    assert gemm.splitk_config(128, 8192, 28672) == (4, 8) and gemm.splitk_config(4, 8192, 28672) == (8, 2)
    assert gemm.splitk_config(16, 10240, 8192) == (8, 2) and gemm.splitk_config(200, 10240, 8192) == (2, 8)
    assert not any(gemm.uses_tiled_weight(*s) for s in ((8192, 28672), (8192, 8192), (10240, 8192)))
    # Llama-3-70B TP=8 row-parallel shards: bf16 output for the all-reduce (no K split, then slabs)
    assert gemm.bf16_config(1, 8192, 1024) == (1, 4, True) and gemm.bf16_config(200, 8192, 1024) == (1, 2, True)
    assert gemm.bf16_config(64, 8192, 3584) == (1, 2, True) and gemm.bf16_config(128, 8192, 3584) == (4, 8, True)
    assert gemm.bf16_config(300, 8192, 3584) is None and gemm.bf16_config(8, 4096, 4096) is None
    # unmeasured shapes stay on the library without copies unless forced
    assert gemm.splitk_config(64, 1536, 256) is None and not gemm.uses_tiled_weight(1536, 256)
    monkeypatch.setenv("PENNY_SPLITK", "force")
    assert gemm.splitk_config(64, 1536, 256) is not None and gemm.uses_tiled_weight(1536, 256)


def test_rowmajor_and_tiled_decode_gemm_agree_on_cpu():
    """The CPU fallbacks of the split-K / gate|up kernels accept either weight form."""
    from financial_chatbot_llm_amd.ops import gemm
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 256, generator=g).to(torch.bfloat16)
    w = torch.randn(64, 256, generator=g).to(torch.bfloat16)
    P1 = gemm.splitk_partials(x, gemm.tile_weight(w), 64, 2, 2)
    P2 = gemm.splitk_partials(x, w, 64, 2, 2, rowmajor=True)
    assert torch.allclose(P1, P2)
    wi = gemm.interleave16(w[:32], w[32:])
    y1 = gemm.gateup_silu(x, gemm.tile_weight(wi), 64, 4)
    y2 = gemm.gateup_silu(x, wi, 64, 4, rowmajor=True)
    assert torch.equal(y1, y2)


def test_kernel_lib_override_path(monkeypatch):
    """PENNY_KERNEL_LIB points the loader at another build of the kernel library (A/B runs)."""
    from financial_chatbot_llm_amd.ops import _native
    monkeypatch.delenv("PENNY_KERNEL_LIB", raising=False)
    assert _native.lib_path().endswith("libpenny_kernels.so")
    monkeypatch.setenv("PENNY_KERNEL_DEBUG", "1")
    assert _native.lib_path().endswith("libpenny_kernels_debug.so")
    monkeypatch.setenv("PENNY_KERNEL_LIB", "/tmp/other/libpenny_kernels_ab.so")
    assert _native.lib_path() == "/tmp/other/libpenny_kernels_ab.so"


def test_prefill_work_list_lpt_order():
    """One entry per real (sequence, 256-row tile); tiles walking the most KV blocks first; None
    when every chunk fits the 4-wave kernel's 128 rows."""
    import numpy as np
    from financial_chatbot_llm_amd.ops.attention import prefill_work_list
    cu = np.array([0, 200, 220, 420], np.int32)          # q lens 200, 20, 200
    ctx = np.array([4800, 100, 1000], np.int32)
    w = prefill_work_list(cu, ctx, 4)                      # TQ = 64 tokens per tile
    assert w.shape == (4 + 1 + 4, 2)
    assert w[0][0] == 0 and w[0][1] in (2, 3)             # a last tile of the long-context sequence
    blocks = [((min(c, c - n + min((t + 1) * 64, n)) + 63) // 64) for s, t in w.tolist()
              for n, c in [((cu[s + 1] - cu[s]), ctx[s])]]
    assert blocks == sorted(blocks, reverse=True)
    assert prefill_work_list(np.array([0, 30, 60], np.int32), np.array([100, 200], np.int32), 4) is None


def test_mx_block_grouping_round_trip_and_fake_quant_bounds():
    """The MX hand-off's CPU model (ops.moe): mx_blocks / mx_unblocks are inverse permutations that
    group 16-element chunks {0,2}, {4,6}, {1,3}, {5,7} of each 128-wide K-tile (the measured
    block-scaled MFMA grouping), and the fake quantiser's blocks use power-of-two scales with every
    scaled element inside e4m3's range, error <= half an e4m3 step of the block's scale."""
    from financial_chatbot_llm_amd.ops import moe
    g = torch.Generator().manual_seed(0)
    x = torch.randn((5, 256), generator=g) * torch.logspace(-3, 3, 256)
    b = moe.mx_blocks(x)
    assert b.shape == (5, 2, 4, 32)
    assert torch.equal(moe.mx_unblocks(b), x)
    assert torch.equal(b[0, 0, 0, :16], x[0, 0:16]) and torch.equal(b[0, 0, 0, 16:], x[0, 32:48])
    assert torch.equal(b[0, 0, 2, :16], x[0, 16:32]) and torch.equal(b[0, 1, 1, 16:], x[0, 128 + 96:128 + 112])
    q = moe._fake_quant_mx(x)
    amax = b.abs().amax(-1)
    X = torch.ceil(torch.log2(amax / moe.FP8_MAX))
    assert (amax / torch.exp2(X) <= moe.FP8_MAX).all()
    err = (moe.mx_blocks(q) - b).abs()
    # e4m3 has 3 mantissa bits: relative rounding <= 2^-4 of the element, or a subnormal step
    assert (err <= b.abs() * 2 ** -4 + torch.exp2(X - 9)[..., None] + 1e-30).all()


def test_mark_shared_blocks_and_cpu_decode():
    """Leading blocks shared with another row at the same position are marked -id - 1 (only inside the
    rows' contexts); the torch decode path reads marked tables like unmarked ones."""
    import numpy as np
    from financial_chatbot_llm_amd.ops.attention import mark_shared_blocks
    bt = np.array([[5, 6, 7, 8], [5, 6, 9, 0], [5, 10, 11, 12], [13, 14, 15, 16]], np.int32)
    m = mark_shared_blocks(bt.copy(), np.array([256, 190, 256, 256]))
    assert m.tolist() == [[-6, -7, 7, 8], [-6, -7, 9, 0], [-6, 10, 11, 12], [13, 14, 15, 16]]
    assert mark_shared_blocks(bt[:1].copy(), np.array([256])).tolist() == bt[:1].tolist()
    g = torch.Generator().manual_seed(0)
    Hq, Hkv, D = 4, 2, 64
    kc = torch.randn(17, Hkv, 64 * D, generator=g).bfloat16()
    vc = torch.randn(17, Hkv, 64 * D, generator=g).bfloat16()
    q = torch.randn(4, Hq, D, generator=g).bfloat16()
    ctx = torch.tensor([256, 190, 256, 256], dtype=torch.int32)
    a = ops.decode(q, ctx, torch.from_numpy(bt), kc, vc, 0.125)
    b = ops.decode(q, ctx, torch.from_numpy(m), kc, vc, 0.125)
    assert torch.equal(a, b)


def test_mark_shared_blocks_native_matches_numpy():
    """The runtime's C++ marking and the numpy form agree on prefix-closed tables (disjoint groups of
    rows sharing a leading run, contexts of any length)."""
    import numpy as np
    from financial_chatbot_llm_amd.ops import attention as A
    if A._runtime() is None:
        import pytest
        pytest.skip("native runtime not built")
    rng = np.random.default_rng(1)
    for _ in range(100):
        B, W = int(rng.integers(2, 160)), int(rng.integers(1, 100))
        bt = rng.permutation(B * W + 1000)[:B * W].reshape(B, W).astype(np.int32)
        rows = rng.permutation(B)
        i = 0
        while i < B - 1:
            n = int(rng.integers(2, 9))
            grp = rows[i:i + n]
            L = int(rng.integers(1, W + 1))
            bt[grp, :L] = bt[grp[0], :L]
            i += n
        ctx = rng.integers(0, W * 64 + 1, B).astype(np.int32)
        native = A.mark_shared_blocks(bt.copy(), ctx)
        orig = A._runtime
        try:
            A._runtime = lambda: None
            ref = A.mark_shared_blocks(bt.copy(), ctx)
        finally:
            A._runtime = orig
        assert np.array_equal(native, ref)


def test_paired_stage_table(monkeypatch):
    """W-layout flags of the decode GEMMs: bit 0 row-major, bit 1 paired stages -- per the PAIRED table
    up to its row limit, always / never under PAIR_MODE 1 / 0."""
    from financial_chatbot_llm_amd.ops import gemm
    monkeypatch.setattr(gemm, "PAIR_MODE", "table")
    assert gemm._wrow(False, 64, 4096, 4096) == 2 and gemm._wrow(True, 64, 4096, 4096) == 3
    assert gemm._wrow(False, 129, 4096, 4096) == 0 and gemm._wrow(True, 200, 4096, 4096) == 1
    assert gemm._wrow(True, 16, 57344, 8192) == 3 and gemm._wrow(True, 17, 57344, 8192) == 1
    assert gemm._wrow(False, 8, 1000, 1000) == 0            # unmeasured shape
    monkeypatch.setattr(gemm, "PAIR_MODE", "1")
    assert gemm._wrow(False, 256, 1000, 1000) == 2
    monkeypatch.setattr(gemm, "PAIR_MODE", "0")
    assert gemm._wrow(True, 8, 4096, 4096) == 1
