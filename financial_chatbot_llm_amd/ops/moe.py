"""K13 MoE helpers: router top-k softmax, token bucketing by expert, fp8-e4m3 (OCP) weights.

gfx950 uses the OCP ``e4m3fn`` encoding (not MI300's ``fnuz``), which is torch.float8_e4m3fn.
"""
from __future__ import annotations

import os
from typing import Tuple

import torch

FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


def topk_softmax(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """HF Mixtral routing: softmax over all experts (f32), top-k, renormalise."""
    p = torch.softmax(logits.float(), dim=-1)
    w, i = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, i.to(torch.int32)


# prefill-size fp8 MoE steps run moe_prefill_fp8_tiles (PENNY_MOE_PREFILL_TILES=0: the per-expert
# hipBLASLt fp8 loop with one host read of the bucket sizes per layer)
PREFILL_TILES = os.environ.get("PENNY_MOE_PREFILL_TILES", "1") != "0"
# fp8 tile GEMMs: the balanced fragment-read schedule (default); PENNY_MOE_TILE_SCHED=plain takes
# the plain 12/4/8/0 one (A/B reference; the kernel takes it as epi + 16)
TILE_SCHED = 16 if os.environ.get("PENNY_MOE_TILE_SCHED", "balanced") == "plain" else 0
# prefill tiles: the SiLU intermediate handed from GEMM1 to GEMM2 as MX fp8 (e4m3 + one E8M0 scale per
# 32 columns, written by GEMM1's epilogue) instead of bf16 + a per-row quantisation pass
MX_HANDOFF = os.environ.get("PENNY_MOE_MX", "1") == "1"
# expert-parallel receives of at least this many rows run moe_grouped_fp8_tiles
EP_TILE_MIN_ROWS = int(os.environ.get("PENNY_EP_TILE_MIN_ROWS", "512"))


def route(topi: torch.Tensor, topw: torch.Tensor, num_experts: int):
    """Bucket (token, expert) pairs by expert.

    Returns ``order`` (permutation of the flattened pairs), ``offsets`` [E+1] (bucket bounds),
    ``tok_idx`` (token of each sorted pair) and ``tok_w`` (its routing weight)."""
    T, k = topi.shape
    flat_e = topi.reshape(-1).long()
    order = torch.argsort(flat_e, stable=True)
    counts = torch.bincount(flat_e, minlength=num_experts)
    offsets = torch.zeros(num_experts + 1, dtype=torch.long, device=topi.device)
    offsets[1:] = counts.cumsum(0)
    tok_idx = (order // k)
    tok_w = topw.reshape(-1)[order].float()
    return order, offsets, tok_idx, tok_w


def route_device(topi: torch.Tensor, topw: torch.Tensor, num_experts: int):
    """:func:`route` without a host round trip (prefill buckets of any size): expert offsets as an
    int32 DEVICE tensor for the grouped kernels, plus the sorted token index, routing weight and
    the inverse map pair -> sorted position.  No ``bincount`` (it syncs to size its output)."""
    T, k = topi.shape
    flat_e = topi.reshape(-1).long()
    order = torch.argsort(flat_e, stable=True)
    counts = torch.zeros(num_experts, dtype=torch.int32, device=topi.device)
    counts.scatter_add_(0, flat_e, torch.ones_like(flat_e, dtype=torch.int32))
    offsets = torch.zeros(num_experts + 1, dtype=torch.int32, device=topi.device)
    offsets[1:] = counts.cumsum(0)
    tok_idx = (order // k).to(torch.int32)
    tok_w = topw.reshape(-1)[order].float().contiguous()
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel(), device=order.device, dtype=order.dtype)
    return offsets, tok_idx, tok_w, inv.to(torch.int32)


# prefill routing + hidden-row quantisation in two HIP launches (penny_moe_route_quant);
# PENNY_MOE_FUSED_ROUTE=0: torch top-k + route_device + quant_rows
FUSED_ROUTE = os.environ.get("PENNY_MOE_FUSED_ROUTE", "1") != "0"


def route_quant_device(h: torch.Tensor, router_logits: torch.Tensor, top_k: int, num_experts: int):
    """Route the T tokens and quantise their hidden rows on the device: -> (xq [T, H] e4m3 bytes,
    xs [T] f32 row scales, offsets [E+1] i32, tok_idx [T*k] i32, tok_w [T*k] f32, inv [T*k] i32),
    the outputs of :func:`topk_softmax` + :func:`route_device` + ``quant_rows`` (bucket order
    inside an expert may differ; every row is computed independently)."""
    from . import _native as N
    T, H = h.shape
    dev = h.device
    P = T * top_k
    lg = router_logits if router_logits.dtype == torch.bfloat16 else router_logits.to(torch.bfloat16)
    lg = lg.contiguous()
    xq = torch.empty((T, H), dtype=torch.uint8, device=dev)
    xs = torch.empty(T, dtype=torch.float32, device=dev)
    scratch = torch.empty(2 * P, dtype=torch.int32, device=dev)
    tok_idx = torch.empty(P, dtype=torch.int32, device=dev)
    tok_w = torch.empty(P, dtype=torch.float32, device=dev)
    offsets = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
    inv = torch.empty(P, dtype=torch.int32, device=dev)
    N.call("penny_moe_route_quant", N.ptr(h), h.stride(0), N.ptr(lg), T, H, num_experts, top_k, N.ptr(xq), N.ptr(xs),
           N.ptr(scratch), N.ptr(scratch[P:]), N.ptr(tok_idx), N.ptr(tok_w), N.ptr(offsets), N.ptr(inv), N.stream())
    return xq, xs, offsets, tok_idx, tok_w, inv


def _route_and_quant(h, router_logits, top_k, E):
    """Fused device routing + quantisation, or the unfused torch chain (PENNY_MOE_FUSED_ROUTE=0)."""
    from . import _native as N
    if FUSED_ROUTE and h.stride(1) == 1 and h.stride(0) % 8 == 0:
        return route_quant_device(h, router_logits, top_k, E)
    T, H = h.shape
    topw, topi = topk_softmax(router_logits, top_k)
    offsets, tok_idx, tok_w, inv = route_device(topi, topw, E)
    xq = torch.empty((T, H), dtype=torch.uint8, device=h.device)
    xs = torch.empty(T, dtype=torch.float32, device=h.device)
    N.call("penny_quant_rows_fp8", N.ptr(h), h.stride(0), T, H, N.ptr(xq), N.ptr(xs), N.stream())
    return xq, xs, offsets, tok_idx, tok_w, inv


def moe_prefill_fp8(h: torch.Tensor, router_logits: torch.Tensor, w13t: torch.Tensor, s13: torch.Tensor,
                    w2t: torch.Tensor, s2: torch.Tensor, top_k: int) -> torch.Tensor:
    """Prefill-size fp8 MoE entirely on the device, no host sync: torch top-k routing +
    :func:`route_device`, then the decode pipeline's grouped fp8 x fp8 MFMA GEMMs over the expert
    buckets (gathered token rows, fused SiLU / routing-weight epilogues) and the combine."""
    from . import _native as N
    T, H = h.shape
    E, F2 = s13.shape
    F_ = F2 // 2
    P = T * top_k
    xq, xs, offsets, tok_idx, tok_w, inv = _route_and_quant(h, router_logits, top_k, E)
    st = N.stream()
    a = torch.empty((P, F_), dtype=torch.bfloat16, device=h.device)
    ntf13, ntf2 = MOE_NTF
    N.call("penny_moe_gemm_fp8", N.ptr(xq), N.ptr(xs), N.ptr(tok_idx), N.ptr(offsets), N.ptr(w13t), N.ptr(s13), None,
           N.ptr(a), E, F2, H, 1, ntf13, st)
    aq = torch.empty((P, F_), dtype=torch.uint8, device=h.device)
    as_ = torch.empty(P, dtype=torch.float32, device=h.device)
    N.call("penny_quant_rows_fp8", N.ptr(a), F_, P, F_, N.ptr(aq), N.ptr(as_), st)
    y2 = torch.empty((P, H), dtype=torch.bfloat16, device=h.device)
    N.call("penny_moe_gemm_fp8", N.ptr(aq), N.ptr(as_), None, N.ptr(offsets), N.ptr(w2t), N.ptr(s2), N.ptr(tok_w),
           N.ptr(y2), E, H, F_, 2, ntf2, st)
    out = torch.empty_like(h)
    N.call("penny_moe_combine", N.ptr(y2), N.ptr(inv), T, top_k, H, N.ptr(out), st)
    return out


def moe_prefill_fp8_tiles(h: torch.Tensor, router_logits: torch.Tensor, w13q: torch.Tensor, s13: torch.Tensor,
                          w2q: torch.Tensor, s2: torch.Tensor, top_k: int) -> torch.Tensor:
    """Prefill-size fp8 MoE on the 256x256 tile kernel (gemm_prefill.hip, block-scaled
    v_mfma_scale_f32_16x16x128_f8f6f4 at unit scales = 2x the bf16 MFMA rate), no host sync:
    device routing (:func:`route_device`), per-row fp8 activations, grouped GEMM1 over the expert
    buckets gathering the routed token rows with the SiLU(gate)*up epilogue, per-row fp8 of the
    intermediate, grouped GEMM2 with the routing weight in its epilogue, atomics-free combine.
    ``w13q`` / ``w2q`` are the row-major e4m3 experts [E, N, K] (W13 16-row gate|up interleave)."""
    from . import _native as N
    T, H = h.shape
    E, F2 = s13.shape
    F_ = F2 // 2
    P = T * top_k
    xq, xs, offsets, tok_idx, tok_w, inv = _route_and_quant(h, router_logits, top_k, E)
    st = N.stream()
    if MX_HANDOFF and F_ % 128 == 0:
        # GEMM1 writes the intermediate as e4m3 + E8M0 block scales, GEMM2 consumes them in its
        # block-scaled MFMAs: no bf16 intermediate, no per-row quantisation pass
        nkt = F_ // 128
        mxs = torch.empty((((P + 255) // 256 + E) * nkt * 256,), dtype=torch.int32, device=h.device)
        aq = torch.empty((P, F_), dtype=torch.uint8, device=h.device)
        N.call("penny_moe_gemm_prefill_fp8_mx", N.ptr(xq), H, N.ptr(tok_idx), N.ptr(xs), N.ptr(offsets),
               N.ptr(w13q), N.ptr(s13), None, N.ptr(aq), F_, P, E, F2, H, 10, N.ptr(mxs), nkt, st)
        y2 = torch.empty((P, H), dtype=torch.bfloat16, device=h.device)
        N.call("penny_moe_gemm_prefill_fp8_mx", N.ptr(aq), F_, None, None, N.ptr(offsets), N.ptr(w2q), N.ptr(s2),
               N.ptr(tok_w), N.ptr(y2), H, P, E, H, F_, 11, N.ptr(mxs), nkt, st)
        out = torch.empty_like(h)
        N.call("penny_moe_combine", N.ptr(y2), N.ptr(inv), T, top_k, H, N.ptr(out), st)
        return out
    a = torch.empty((P, F_), dtype=torch.bfloat16, device=h.device)
    N.call("penny_moe_gemm_prefill_fp8", N.ptr(xq), H, N.ptr(tok_idx), N.ptr(xs), N.ptr(offsets), N.ptr(w13q),
           N.ptr(s13), None, N.ptr(a), F_, P, E, F2, H, 7 + TILE_SCHED, st)
    aq = torch.empty((P, F_), dtype=torch.uint8, device=h.device)
    as_ = torch.empty(P, dtype=torch.float32, device=h.device)
    N.call("penny_quant_rows_fp8", N.ptr(a), F_, P, F_, N.ptr(aq), N.ptr(as_), st)
    y2 = torch.empty((P, H), dtype=torch.bfloat16, device=h.device)
    N.call("penny_moe_gemm_prefill_fp8", N.ptr(aq), F_, None, N.ptr(as_), N.ptr(offsets), N.ptr(w2q), N.ptr(s2),
           N.ptr(tok_w), N.ptr(y2), H, P, E, H, F_, 8 + TILE_SCHED, st)
    out = torch.empty_like(h)
    N.call("penny_moe_combine", N.ptr(y2), N.ptr(inv), T, top_k, H, N.ptr(out), st)
    return out


def moe_grouped_fp8(x: torch.Tensor, expert_ids: torch.Tensor, w13t: torch.Tensor, s13: torch.Tensor,
                    w2t: torch.Tensor, s2: torch.Tensor) -> torch.Tensor:
    """y[i] = expert_{ids[i]}(x[i]) for every row (ids -1 = padding -> 0), one grouped fp8
    pipeline over the (local) expert bank, no host sync (expert-parallel receive side)."""
    from . import _native as N
    M, H = x.shape
    E, F2 = s13.shape
    F_ = F2 // 2
    ids = expert_ids.long()
    key = torch.where(ids >= 0, ids, torch.full_like(ids, E))
    order = torch.argsort(key, stable=True)
    counts = torch.zeros(E + 1, dtype=torch.int32, device=x.device)
    counts.scatter_add_(0, key, torch.ones_like(key, dtype=torch.int32))
    offsets = torch.zeros(E + 1, dtype=torch.int32, device=x.device)
    offsets[1:] = counts[:E].cumsum(0)
    rows = order.to(torch.int32)
    st = N.stream()
    xq = torch.empty((M, H), dtype=torch.uint8, device=x.device)
    xs = torch.empty(M, dtype=torch.float32, device=x.device)
    N.call("penny_quant_rows_fp8", N.ptr(x), x.stride(0), M, H, N.ptr(xq), N.ptr(xs), st)
    a = torch.zeros((M, F_), dtype=torch.bfloat16, device=x.device)
    ntf13, ntf2 = MOE_NTF
    N.call("penny_moe_gemm_fp8", N.ptr(xq), N.ptr(xs), N.ptr(rows), N.ptr(offsets), N.ptr(w13t), N.ptr(s13), None,
           N.ptr(a), E, F2, H, 1, ntf13, st)
    aq = torch.empty((M, F_), dtype=torch.uint8, device=x.device)
    as_ = torch.empty(M, dtype=torch.float32, device=x.device)
    N.call("penny_quant_rows_fp8", N.ptr(a), F_, M, F_, N.ptr(aq), N.ptr(as_), st)
    ones = torch.ones(M, dtype=torch.float32, device=x.device)
    y2 = torch.zeros((M, H), dtype=torch.bfloat16, device=x.device)
    N.call("penny_moe_gemm_fp8", N.ptr(aq), N.ptr(as_), None, N.ptr(offsets), N.ptr(w2t), N.ptr(s2), N.ptr(ones),
           N.ptr(y2), E, H, F_, 2, ntf2, st)
    y = torch.empty_like(y2)
    y.index_copy_(0, order, y2)
    return torch.where((ids >= 0)[:, None], y, torch.zeros_like(y))


def moe_grouped_fp8_tiles(x: torch.Tensor, expert_ids: torch.Tensor, w13q: torch.Tensor, s13: torch.Tensor,
                          w2q: torch.Tensor, s2: torch.Tensor) -> torch.Tensor:
    """:func:`moe_grouped_fp8` for prefill-size receives (expert-parallel receive side): the same
    per-row result on the 256x256 fp8 tile kernel (gemm_prefill.hip) instead of the decode-shaped
    grouped kernel -- rows sorted by expert on the device, GEMM1 gathers them through the sort
    order, GEMM2 runs at unit routing weights (the home rank applies the real ones), padding rows
    (id -1) sort last, outside every expert bucket, and come back as zeros.  No host sync.
    ``w13q`` / ``w2q``: row-major e4m3 [E_local, N, K]."""
    from . import _native as N
    M, H = x.shape
    E, F2 = s13.shape
    F_ = F2 // 2
    ids = expert_ids.long()
    key = torch.where(ids >= 0, ids, torch.full_like(ids, E))
    order = torch.argsort(key, stable=True)
    counts = torch.zeros(E + 1, dtype=torch.int32, device=x.device)
    counts.scatter_add_(0, key, torch.ones_like(key, dtype=torch.int32))
    offsets = torch.zeros(E + 1, dtype=torch.int32, device=x.device)
    offsets[1:] = counts[:E].cumsum(0)
    rows = order.to(torch.int32)
    st = N.stream()
    xq = torch.empty((M, H), dtype=torch.uint8, device=x.device)
    xs = torch.empty(M, dtype=torch.float32, device=x.device)
    N.call("penny_quant_rows_fp8", N.ptr(x), x.stride(0), M, H, N.ptr(xq), N.ptr(xs), st)
    a = torch.zeros((M, F_), dtype=torch.bfloat16, device=x.device)
    N.call("penny_moe_gemm_prefill_fp8", N.ptr(xq), H, N.ptr(rows), N.ptr(xs), N.ptr(offsets), N.ptr(w13q),
           N.ptr(s13), None, N.ptr(a), F_, M, E, F2, H, 7 + TILE_SCHED, st)
    aq = torch.empty((M, F_), dtype=torch.uint8, device=x.device)
    as_ = torch.empty(M, dtype=torch.float32, device=x.device)
    N.call("penny_quant_rows_fp8", N.ptr(a), F_, M, F_, N.ptr(aq), N.ptr(as_), st)
    ones = torch.ones(M, dtype=torch.float32, device=x.device)
    y2 = torch.zeros((M, H), dtype=torch.bfloat16, device=x.device)
    N.call("penny_moe_gemm_prefill_fp8", N.ptr(aq), F_, None, N.ptr(as_), N.ptr(offsets), N.ptr(w2q), N.ptr(s2),
           N.ptr(ones), N.ptr(y2), H, M, E, H, F_, 8 + TILE_SCHED, st)
    y = torch.empty_like(y2)
    y.index_copy_(0, order, y2)
    return y


def quant_rows_fp8(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-row e4m3 quantisation on the device (HIP ``penny_quant_rows_fp8``, the decode
    pipeline's activation quantiser): x [M, K] bf16 -> (fp8 [M, K], f32 scale [M])."""
    from . import _native as N
    M, K = x.shape
    if not N.use_native(x):
        q, s = quantize_fp8_rowwise(x)
        return q, s.float()
    q = torch.empty((M, K), dtype=torch.uint8, device=x.device)
    s = torch.empty(M, dtype=torch.float32, device=x.device)
    N.call("penny_quant_rows_fp8", N.ptr(x), x.stride(0), M, K, N.ptr(q), N.ptr(s), N.stream())
    return q.view(FP8), s


def silu_quant_rows_fp8(gu: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """silu(gate) * up of a 16-interleaved gate|up GEMM output [M, 2F], quantised per row to e4m3 in
    the same pass (HIP ``penny_silu_quant_rows_fp8``): -> (fp8 [M, F], f32 scale [M])."""
    from . import _native as N
    from .activation import silu_mul
    M, F2 = gu.shape
    if not N.use_native(gu):
        return quant_rows_fp8(silu_mul(gu, interleave16=True))
    q = torch.empty((M, F2 // 2), dtype=torch.uint8, device=gu.device)
    s = torch.empty(M, dtype=torch.float32, device=gu.device)
    src = gu.contiguous()                      # alive across the launch
    N.call("penny_silu_quant_rows_fp8", N.ptr(src), M, F2 // 2, N.ptr(q), N.ptr(s), N.stream())
    return q.view(FP8), s


def combine_weighted(ys: torch.Tensor, order: torch.Tensor, tok_w: torch.Tensor, T: int, k: int) -> torch.Tensor:
    """out[t] = sum_j w * ys[pos(t, j)] for expert-sorted rows ``ys`` [T*k, H] (``order``/``tok_w``
    from :func:`route`): a gather per token with f32 accumulation (HIP ``penny_moe_combine_weighted``)
    instead of float copies + a scaled ``index_add_`` over the sorted rows."""
    from . import _native as N
    H = ys.shape[1]
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel(), device=order.device, dtype=order.dtype)
    if not N.use_native(ys):
        w = ys.float() * tok_w[:, None].float()
        return w[inv].view(T, k, H).sum(1).to(ys.dtype)
    inv32 = inv.to(torch.int32)
    w32 = tok_w.float().contiguous()
    out = torch.empty((T, H), dtype=ys.dtype, device=ys.device)
    N.call("penny_moe_combine_weighted", N.ptr(ys), N.ptr(inv32), N.ptr(w32), T, k, H, N.ptr(out), N.stream())
    return out


def quantize_fp8_rowwise(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """w [..., out, in] -> (fp8 e4m3fn, f32 scale [..., out]) with w ~= q * scale[..., None]."""
    amax = w.float().abs().amax(dim=-1).clamp_min(1e-12)
    scale = amax / FP8_MAX
    q = (w.float() / scale[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, scale


def dequant_fp8(q: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    return (q.float() * scale[..., None]).to(dtype)


# ----------------------------------------------------------------------------------------------
# fp8 expert bank in MFMA-fragment tiles + the HIP decode pipeline (csrc/kernels/moe.hip)
# ----------------------------------------------------------------------------------------------
def tile_fp8_weight(q: torch.Tensor) -> torch.Tensor:
    """fp8 [E, N, K] -> uint8 [E, N/16, K/64, 64, 16]: fragment pair (row group, 2 k-steps) is
    1 KiB contiguous; lane 16g+r holds row r, k = 64p + 16g + 8s + j at byte 8s + j -- 16
    CONTIGUOUS k of the row, so the activation operand of the same lane is one 16-byte load too
    (the MFMA's k slots are a permutation of the physical k, applied to both operands)."""
    E, N_, K = q.shape
    assert N_ % 16 == 0 and K % 64 == 0
    u = q.view(torch.uint8).view(E, N_ // 16, 16, K // 64, 4, 2, 8)      # e rg r kp g s j
    return u.permute(0, 1, 3, 4, 2, 5, 6).reshape(E, N_ // 16, K // 64, 64, 16).contiguous()


def untile_fp8_weight(t: torch.Tensor) -> torch.Tensor:
    E, RG, KP, _, _ = t.shape
    u = t.view(E, RG, KP, 4, 16, 2, 8).permute(0, 1, 4, 2, 3, 5, 6)       # e rg r kp g s j
    return u.reshape(E, RG * 16, KP * 64).contiguous().view(FP8)


def _fake_quant_rows(x: torch.Tensor) -> torch.Tensor:
    """Round-trip rows through dynamic per-row fp8 e4m3 (what ``penny_quant_rows_fp8`` does)."""
    q, s = quantize_fp8_rowwise(x)
    return q.float() * s[..., None]


# the 16-column chunks of a 128-column K-tile that one E8M0 scale of the block-scaled MFMA covers,
# with the tile kernel's fp8 fragment layout (lane group g: chunks 2g, 2g + 1): measured on the
# GPU (tests/test_kernels_gpu.py test_mfma_scale_operand_map_dump) -- scale k-block b of a chunk
MX_CHUNK_BLOCK = (0, 2, 0, 2, 1, 3, 1, 3)


def mx_blocks(x: torch.Tensor) -> torch.Tensor:
    """[R, C] -> [R, C / 128, 4 k-blocks, 32] in the MFMA's scale-block grouping (MX_CHUNK_BLOCK)."""
    R, C = x.shape
    ch = x.reshape(R, C // 128, 8, 16)
    order = [c for b in range(4) for c in range(8) if MX_CHUNK_BLOCK[c] == b]
    return ch[:, :, order].reshape(R, C // 128, 4, 32)


def mx_unblocks(b: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`mx_blocks`."""
    R, T = b.shape[0], b.shape[1]
    order = [c for k in range(4) for c in range(8) if MX_CHUNK_BLOCK[c] == k]
    inv = [order.index(c) for c in range(8)]
    return b.reshape(R, T, 8, 16)[:, :, inv].reshape(R, T * 128)


def _fake_quant_mx(x: torch.Tensor) -> torch.Tensor:
    """Round-trip rows through MX fp8 as the hand-off does: per scale block (32 columns grouped as
    the block-scaled MFMA groups them, :func:`mx_blocks`) an E8M0 scale 2^X with
    X = ceil(log2(amax / 448)), e4m3 of value / 2^X (the GEMM1 epilogue of the MX hand-off)."""
    b = mx_blocks(x.float())
    amax = b.abs().amax(-1, keepdim=True)
    X = torch.where(amax > 0, torch.ceil(torch.log2(amax / FP8_MAX)), torch.full_like(amax, -127.0)).clamp(-127, 126)
    sc = torch.exp2(X)
    return mx_unblocks((b / sc).to(FP8).float() * sc)


def moe_fp8_reference(h, router_w, w13q, s13, w2q, s2, top_k, quant_act=False):
    """fp32 reference of the fp8 MoE MLP (weights dequantised).  ``quant_act`` additionally rounds
    both GEMM inputs through dynamic per-row fp8, matching the HIP pipeline's arithmetic;
    ``quant_act="mx"`` rounds the intermediate through MX fp8 (the tiles' MX hand-off) instead."""
    topw, topi = topk_softmax(h.float() @ router_w.float().t(), top_k)
    out = torch.zeros(h.shape, dtype=torch.float32, device=h.device)
    from .activation import silu_mul
    for e in range(w13q.shape[0]):
        sel = (topi == e)
        rows = sel.any(-1).nonzero().flatten()
        if rows.numel() == 0:
            continue
        w13 = w13q[e].float() * s13[e][:, None]
        w2 = w2q[e].float() * s2[e][:, None]
        x = h[rows].float()
        if quant_act:
            x = _fake_quant_rows(x)
        a = silu_mul((x @ w13.t()).to(torch.bfloat16), interleave16=True).float()
        if quant_act == "mx":
            a = _fake_quant_mx(a)
        elif quant_act:
            a = _fake_quant_rows(a)
        y = a @ w2.t()
        wt = (topw * sel).sum(-1)[rows]
        out[rows] += y * wt[:, None]
    return out.to(h.dtype)


# 16-row weight groups per workgroup for the (W13, W2) grouped fp8 GEMMs (PENNY_MOE_NTF="a,b"):
# 4,4 measured 6-16 % faster than 2,2 at T = 64-256 decode tokens (profiles/r1_moe_ntf.jsonl)
MOE_NTF = tuple(int(v) for v in os.environ.get("PENNY_MOE_NTF", "4,4").split(","))


class MoEWorkspace:
    """Device buffers for one decode-sized MoE step (reused across layers; graph-capturable)."""

    def __init__(self, max_tokens: int, top_k: int, num_experts: int, H: int, F: int, device):
        P = max_tokens * top_k
        self.max_tokens = max_tokens
        i32 = dict(dtype=torch.int32, device=device)
        self.sorted_tok = torch.zeros(P, **i32)
        self.sorted_w = torch.zeros(P, dtype=torch.float32, device=device)
        self.offsets = torch.zeros(num_experts + 1, **i32)
        self.inv = torch.zeros(P, **i32)
        self.xq = torch.zeros((max_tokens, H), dtype=torch.uint8, device=device)
        self.xs = torch.zeros(max_tokens, dtype=torch.float32, device=device)
        self.a = torch.zeros((P, F), dtype=torch.bfloat16, device=device)
        self.aq = torch.zeros((P, F), dtype=torch.uint8, device=device)
        self.as_ = torch.zeros(P, dtype=torch.float32, device=device)
        self.y2 = torch.zeros((P, H), dtype=torch.bfloat16, device=device)


def moe_decode_fp8(h: torch.Tensor, router_logits: torch.Tensor, w13t: torch.Tensor, s13: torch.Tensor,
                   w2t: torch.Tensor, s2: torch.Tensor, top_k: int, ws: "MoEWorkspace") -> torch.Tensor:
    """HIP fp8 MoE for decode-sized batches: route -> quant -> grouped GEMM(SiLU) -> quant ->
    grouped GEMM(x routing weight) -> combine.  Returns [T, H] bf16 (TP partial sum)."""
    from . import _native as N
    T, H = h.shape
    E, F2 = s13.shape
    F_ = F2 // 2
    P = T * top_k
    st = N.stream()
    N.call("penny_moe_route", N.ptr(router_logits), T, E, top_k, N.ptr(ws.sorted_tok), N.ptr(ws.sorted_w),
           N.ptr(ws.offsets), N.ptr(ws.inv), st)
    N.call("penny_quant_rows_fp8", N.ptr(h), h.stride(0), T, H, N.ptr(ws.xq), N.ptr(ws.xs), st)
    ntf13, ntf2 = MOE_NTF
    N.call("penny_moe_gemm_fp8", N.ptr(ws.xq), N.ptr(ws.xs), N.ptr(ws.sorted_tok), N.ptr(ws.offsets), N.ptr(w13t),
           N.ptr(s13), None, N.ptr(ws.a), E, F2, H, 1, ntf13, st)
    N.call("penny_quant_rows_fp8", N.ptr(ws.a), F_, P, F_, N.ptr(ws.aq), N.ptr(ws.as_), st)
    N.call("penny_moe_gemm_fp8", N.ptr(ws.aq), N.ptr(ws.as_), None, N.ptr(ws.offsets), N.ptr(w2t), N.ptr(s2),
           N.ptr(ws.sorted_w), N.ptr(ws.y2), E, H, F_, 2, ntf2, st)
    out = torch.empty_like(h)
    N.call("penny_moe_combine", N.ptr(ws.y2), N.ptr(ws.inv), T, top_k, H, N.ptr(out), st)
    return out
