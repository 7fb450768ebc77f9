"""Shape fuzzing of the attention / norm kernels against the fp32 torch references (SURVEY §4:
"hypothesis for shape fuzzing").  Bounded example counts keep the GPU run to seconds."""
import math

import pytest
import torch

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from financial_chatbot_llm_amd import ops  # noqa: E402
from test_kernels_gpu import DEV, _paged_setup, close, rnd  # noqa: E402

pytestmark = pytest.mark.gpu
FUZZ = settings(max_examples=12, deadline=None, derandomize=True)


@FUZZ
@given(G=st.sampled_from([1, 2, 4, 8]), Hkv=st.sampled_from([1, 2, 8]), D=st.sampled_from([64, 128]),
       lens=st.lists(st.tuples(st.integers(1, 300), st.integers(0, 400)), min_size=1, max_size=4),
       causal=st.booleans())
def test_prefill_fuzz(G, Hkv, D, lens, causal):
    g = torch.Generator().manual_seed(len(lens) * 131 + G)
    Hq = G * Hkv
    qlens = [a for a, _ in lens]
    ctx = [a + b for a, b in lens]                       # prefix-cache hits of b tokens
    tables, kc, vc = _paged_setup(ctx, Hkv, D, gen=g)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32)
    q = rnd(int(cu[-1]), Hq, D, gen=g)
    ctx_t = torch.tensor(ctx, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.prefill(q.to(DEV), cu.to(DEV), ctx_t.to(DEV), tables.to(DEV), kc.to(DEV), vc.to(DEV), scale, causal,
                      max_q_len=max(qlens))
    close(out, ops.prefill(q, cu, ctx_t, tables, kc, vc, scale, causal), atol=2e-2)


@FUZZ
@given(G=st.sampled_from([1, 4, 8, 16]), Hkv=st.sampled_from([1, 8]),
       ctxs=st.lists(st.integers(1, 3000), min_size=1, max_size=40))
def test_decode_fuzz(G, Hkv, ctxs):
    g = torch.Generator().manual_seed(sum(ctxs) % 9973)
    D, Hq = 128, G * Hkv
    tables, kc, vc = _paged_setup(ctxs, Hkv, D, gen=g)
    q = rnd(len(ctxs), Hq, D, gen=g)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32)
    ws = ops.DecodeWorkspace.create(len(ctxs), Hq, D, 4096, DEV)
    out = ops.decode(q.to(DEV), ctx_t.to(DEV), tables.to(DEV), kc.to(DEV), vc.to(DEV), 0.088, workspace=ws)
    close(out, ops.decode(q, ctx_t, tables, kc, vc, 0.088), atol=2e-2)


@FUZZ
@given(T=st.integers(1, 700), H=st.sampled_from([512, 768, 1024, 2048, 4096, 8192]), res=st.booleans())
def test_rmsnorm_fuzz(T, H, res):
    torch.manual_seed(T * 7 + H)
    x, r, w = rnd(T, H), rnd(T, H), rnd(H, scale=0.1) + 1
    if res:
        r_dev = r.to(DEV)
        y = ops.rms_norm(x.to(DEV), w.to(DEV), 1e-5, residual=r_dev)
        ref_r = r.float() + x.float()
        close(r_dev, ref_r.to(torch.bfloat16), atol=2e-2)
        ref = ops.rms_norm(x, w, 1e-5, residual=r.clone())
    else:
        y = ops.rms_norm(x.to(DEV), w.to(DEV), 1e-5)
        ref = ops.rms_norm(x, w, 1e-5)
    close(y, ref, atol=3e-2)
