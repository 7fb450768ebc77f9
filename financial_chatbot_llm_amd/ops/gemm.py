"""Projection GEMMs: hand-written MFMA kernels -- weight-streaming ones for decode, the 256x256 tile
kernel (gemm_prefill.hip) with fused epilogues for prefill -- and hipBLASLt where it measured faster.

``linear(x, w, epilogue=..., wt=..., slabs=...)`` is the single entry point the models use.  For a
decode-size M on the GPU, in order:

* ``slabs=True`` and a ``SPLITK`` entry -> ``penny_splitk_gemm``: split-K f32 slabs left unreduced
  for the consumer (RMSNorm / RoPE-KV-write sum them in their own row pass);
* ``epilogue="silu"`` and a ``GATEUP`` entry -> ``penny_gateup_silu_gemm``: the interleaved
  gate|up GEMM with SiLU(gate)*up fused into its epilogue;
* a ``TUNING`` entry -> ``penny_skinny_gemm`` (M <= 16-32, fused SiLU / residual epilogues).

These kernels stream either the fragment-tiled copy ``wt`` (``tile_weight``; made at load only
for shapes with an entry, see ``uses_tiled_weight``) or the row-major weight itself.  Prefill-size
M (> 256 rows) follows ``PREFILL_POLICY``: the tile kernel with the SiLU / residual epilogue or
split-K slabs, or hipBLASLt via ``torch.nn.functional.linear`` plus the matching HIP epilogue
kernel (``silu_mul(interleave16=True)``) or a fused add.  Every table entry was measured on MI355X
with ``bench/kernels.py`` (profiles named next to each table).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple, Union

import torch
import torch.nn.functional as F

from . import _native as N
from .activation import silu_mul

EPI = {None: 0, "silu": 1, "residual": 2}
MAX_SKINNY_M = 64
# (N, K) -> (ntf, nw): 16*ntf weight rows per workgroup, nw waves splitting K.  Measured on MI355X
# (profiles/r1_skinny_gemm.jsonl): the hand-written kernel beats hipBLASLt by 1.3-1.6x on the
# small-N projections (QKV, O) at M <= 16 and ties at M = 64; hipBLASLt already streams the wide
# gate|up / LM-head weights at ~6 TB/s, so those stay on the library.
TUNING: Dict[Tuple[int, int], Tuple[int, int]] = {(6144, 4096): (2, 4), (4096, 4096): (1, 4)}
SKINNY_MAX_M: Dict[Tuple[int, int], int] = {(6144, 4096): 16, (4096, 4096): 32}


def _config(N_: int, K: int, epilogue: Optional[str]) -> Tuple[int, int]:
    if (N_, K) in TUNING:
        return TUNING[(N_, K)]
    ntf = 2
    wgs = N_ // (16 * ntf)
    nw = 8 if wgs < 512 else 4
    if K % (nw * 128):
        nw = 4 if K % 512 == 0 else 1
    return ntf, nw


def tile_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> MFMA-fragment-tiled [N/16, K/32, 64, 8] copy for the decode GEMM: fragment
    (row group, k-step) is 1 KiB contiguous and a row group's k-steps are consecutive."""
    N_, K = w.shape
    assert N_ % 16 == 0 and K % 32 == 0
    return w.view(N_ // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N_ // 16, K // 32, 64, 8).contiguous()


def skinny_ok(x: torch.Tensor, w: torch.Tensor, epilogue: Optional[str] = None,
              wt: Optional[torch.Tensor] = None) -> bool:
    M, K = x.shape
    N_ = w.shape[0]
    if wt is None or not N.use_native(x) or M > MAX_SKINNY_M or os.environ.get("PENNY_SKINNY", "1") == "0":
        return False
    if M > SKINNY_MAX_M.get((N_, K), MAX_SKINNY_M if (N_, K) in TUNING else 0):
        return False
    ntf, nw = _config(N_, K, epilogue)
    return N_ % (16 * ntf) == 0 and K % (nw * 128) == 0 and x.stride(1) == 1 and w.is_contiguous()


def linear(x: torch.Tensor, w: torch.Tensor, epilogue: Optional[str] = None,
           residual: Optional[torch.Tensor] = None, wt: Optional[torch.Tensor] = None,
           slabs: bool = False, fuse_residual: Optional[torch.Tensor] = None) -> Union[torch.Tensor, "Slabs",
                                                                                     "ResidualSum"]:
    """y = x @ w.T with an optional fused epilogue ("silu": w is gate|up 16-interleaved).

    ``wt`` is the fragment-tiled copy of ``w`` (``tile_weight``); when given, decode-sized
    batches run the hand-written MFMA kernels on it.  ``slabs=True`` lets the caller receive the
    split-K GEMM's unreduced :class:`Slabs` (the consumer -- ``ops.rms_norm`` /
    ``ops.rope_kv_write`` -- sums them in its own pass).  ``fuse_residual`` (the residual stream the
    consumer's add + RMSNorm would add this output to) lets a prefill-size GEMM add it in its
    epilogue, in place, returning :class:`ResidualSum` (the norm then only normalises)."""
    M, K = x.shape
    N_ = w.shape[0]
    if M > 256 and prefill_ok(x, w) and epilogue in (None, "silu", "residual"):
        fr = fuse_residual is not None and epilogue is None and residual is None
        c = prefill_choice(M, N_, K, epilogue, slabs and residual is None, fused_residual=fr)
        if c.startswith("K"):
            return splitk_bf16(x, w, N_, int(c[1:]))
        if c == "R":
            prefill_gemm(x, w, "residual", residual=fuse_residual, out=fuse_residual)
            return ResidualSum(fuse_residual)
        if c == "hip":
            return prefill_gemm(x, w, epilogue, residual=residual)
        if c.startswith("S"):
            return Slabs(prefill_gemm(x, w, "slabs", int(c[1:])))
        if c.startswith("M"):
            return mid_linear(x, w, int(c[1:]), epilogue, slabs and residual is None, residual)
    # the decode kernels stream either the fragment-tiled copy or (DECODE_WEIGHTS == "rowmajor",
    # or no copy was made) the row-major weight itself
    src = wt if wt is not None else (w if w.is_contiguous() else None)
    rowmajor = wt is None
    if slabs and src is not None and epilogue is None and residual is None:
        cfg = splitk_config(M, N_, K) if N.use_native(x) and x.stride(1) == 1 and x.stride(0) % 8 == 0 else None
        if cfg is not None:
            return Slabs(splitk_partials(x, src, N_, *cfg, rowmajor=rowmajor))
    if not slabs and epilogue is None and residual is None and N.use_native(x) and x.stride(1) == 1 \
            and x.stride(0) % 8 == 0:
        cfg = bf16_config(M, N_, K)
        if cfg is not None:
            # row-parallel TP shard (O / down): bf16 straight into the all-reduce -- one launch with
            # no K split, or split-K slabs + the reduce where the shard is too narrow for that
            S, nf, rm = cfg
            rm = rm or wt is None
            ww = w if rm else wt
            if S == 1:
                return splitk_bf16(x, ww, N_, nf, rowmajor=rm)
            return splitk_reduce(splitk_partials(x, ww, N_, S, nf, rowmajor=rm))
    if epilogue == "silu" and src is not None and residual is None:
        ok = N.use_native(x) and x.stride(1) == 1 and x.stride(0) % 8 == 0
        nf = gateup_config(M, N_, K) if ok else None
        if nf is not None:
            return gateup_silu(x, src, N_, nf, rowmajor=rowmajor)
        cfg = gateup_splitk_config(M, N_, K) if ok else None
        if cfg is not None and (cfg[2] or not rowmajor):
            S, nf, rm = cfg
            return gateup_splitk(x, w if rm else src, N_, S, nf, rowmajor=rm)
    if skinny_ok(x, w, epilogue, wt):
        ntf, nw = _config(N_, K, epilogue)
        out_n = N_ // 2 if epilogue == "silu" else N_
        y = torch.empty((M, out_n), dtype=x.dtype, device=x.device)
        N.call("penny_skinny_gemm", N.ptr(x), x.stride(0), N.ptr(wt), K, N.ptr(y), out_n, N.ptr(residual),
               residual.stride(0) if residual is not None else 0, M, N_, EPI[epilogue], ntf, nw, N.stream())
        return y
    y = F.linear(x, w)
    if epilogue == "silu":
        return silu_mul(y, interleave16=True)
    if epilogue == "residual":
        return (y.float() + residual.float()).to(y.dtype) if not N.use_native(y) else y.add_(residual)
    return y


def interleave16(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[F, H] gate and up -> [2F, H] with rows alternating in 16-row groups (skinny SiLU layout)."""
    Fr, H = gate.shape
    return torch.stack([gate.view(Fr // 16, 16, H), up.view(Fr // 16, 16, H)], dim=1).reshape(2 * Fr, H)


# ----------------------------------------------------------------------------------------------
# Curated hipBLASLt/rocBLAS solution table for the decode buckets (bench/tune_gemm.py)
# ----------------------------------------------------------------------------------------------
TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")
_LOADED_TUNING: Optional[str] = None


def tuning_file(model: str, tp: int = 1) -> str:
    suffix = "" if tp == 1 else f"_tp{tp}"
    return os.path.join(TUNING_DIR, f"gemm_{model}{suffix}_mi355x.csv")


def load_gemm_tuning(model: str, tp: int = 1) -> Optional[str]:
    """Enable PyTorch TunableOp READ-ONLY with the curated per-shape solutions for ``model``
    (shapes not in the table, e.g. prefill M, keep the default heuristic).  Never tunes online,
    so hipGraph capture and serving latency are unaffected.  Returns the file used, if any."""
    global _LOADED_TUNING
    path = tuning_file(model, tp)
    if os.environ.get("PENNY_GEMM_TUNING", "1") != "1" or not os.path.exists(path) or not torch.cuda.is_available():
        return None
    if _LOADED_TUNING == path:
        return path
    tun = torch.cuda.tunable
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    if not tun.read_file(path):
        return None
    tun.enable(True)
    _LOADED_TUNING = path
    return path


# ----------------------------------------------------------------------------------------------
# Mid-batch decode GEMM (32 < M <= 256): split-K f32 slabs, reduced by the consumer
# ----------------------------------------------------------------------------------------------
# (N, K) -> [(max M, S, nf), ...] for the split-K kernel, measured on MI355X against hipBLASLt with
# the weights streamed from HBM (bench/kernels.py --only splitk, profiles/r1_splitk_v3.jsonl),
# choosing by GEMM time + the consumer's extra slab read (S*M*N*4 B at ~5 TB/s).  Llama-3-8B:
# QKV 1.4-1.9x, O 1.5-2.2x, down 1.4-2.8x faster than the library at M = 16..192.  Every chosen
# config launches exactly 256 workgroups (one per CU): QKV 64 tiles x S=4, O 64 x 4, down 32 x 8
# (profiles/r1_splitk_v4_qkv.jsonl: the 96-row QKV tile beats 128 rows x 192 workgroups by 10 %).
SPLITK: Dict[Tuple[int, int], List[Tuple[int, int, int]]] = {
    (6144, 4096): [(256, 4, 6)],                             # QKV: 96-row tiles -> 256 workgroups
    # O (r5: S4 nf4 also ahead at M = 256, 23.4 vs 24.4 us; with paired stages S4 nf2 is 2-8 % ahead of
    # S4 nf4 to 32 rows, profiles/r5_decode_gemm_paired_stages_ab.jsonl)
    (4096, 4096): [(32, 4, 2), (256, 4, 4)],
    (4096, 14336): [(16, 8, 8), (32, 4, 4), (256, 8, 8)],    # down
    # Llama-3-70B (TP=1), streamed row-major (profiles/r1_splitk_70b.jsonl): down 1.2-1.9x hipBLASLt
    # at M = 32..256; O 1.1-1.5x from M = 96 (S = 0: the library is as fast below that)
    # r5 re-measure at HEAD (profiles/r5_shard_shapes.jsonl, row-major W): down 1.2-2.1x, O 1.2-1.5x,
    # QKV 1.1-1.2x at M = 1..256 (QKV: S = 2 above 32 rows keeps the RoPE pass's slab read small)
    (8192, 28672): [(8, 8, 2), (256, 4, 8)],
    (8192, 8192): [(32, 8, 2), (128, 8, 8), (256, 4, 8)],
    (10240, 8192): [(32, 8, 2), (256, 2, 8)],
    # Llama-3-70B TP=8 per-rank QKV shard (column-parallel: the RoPE/KV-write pass consumes the
    # slabs, no all-reduce in between): 1.4-2.9x hipBLASLt at M = 1..256 (r5_shard_shapes.jsonl)
    (1280, 8192): [(256, 8, 4)],
}
# shapes whose row-major stream measured within a few % of the tiled copy: never tiled (70B: 61 GB
# saved at TP=1, where HBM is the KV pool's)
TILE_FREE = {(8192, 28672), (8192, 8192), (1280, 8192), (10240, 8192)}


# (N, K) -> [(max M, S, nf, rowmajor), ...]: decode-size projections whose caller wants a bf16 output
# (no slabs: the row-parallel TP shards of O / down, whose output goes straight into the
# all-reduce): S = 1 -> the split-K kernel without a K split and the SK_BF16 epilogue
# (penny_splitk_gemm_bf16), S > 1 -> split-K slabs + penny_splitk_reduce.  Measured against hipBLASLt
# with W streamed from HBM (bench/kernels.py shard_shapes, profiles/r5_shard_shapes*.jsonl):
# Llama-3-70B TP=8 O 1.5-2.0x, down 1.1-1.6x at M = 1..256.
DECODE_BF16: Dict[Tuple[int, int], List[Tuple[int, int, int, bool]]] = {
    (8192, 1024): [(32, 1, 4, True), (256, 1, 2, True)],                                        # 70B TP=8 O
    (8192, 3584): [(64, 1, 2, True), (96, 2, 4, True), (128, 4, 8, True), (256, 2, 4, True)],   # 70B TP=8 down
}


def bf16_config(M: int, N_: int, K: int) -> Optional[Tuple[int, int, bool]]:
    """(S, nf, rowmajor) for the bf16-output decode GEMM at this shape, or None (``PENNY_SPLITK=0``
    disables; ``PENNY_SPLITK=force`` takes it for any shape the kernel accepts)."""
    mode = os.environ.get("PENNY_SPLITK", "1")
    if mode == "0" or M > 256 or K % 64:
        return None
    for max_m, S, nf, rm in DECODE_BF16.get((N_, K), ()):
        if M <= max_m:
            return (S, nf, rm) if nf > 0 and K % (64 * S) == 0 else None
    if mode == "force":
        for nf in (2, 4):
            if N_ % (16 * nf) == 0:
                return 1, nf, True
    return None


def splitk_bf16(x: torch.Tensor, w: torch.Tensor, N_: int, nf: int, rowmajor: bool = True,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 y = x @ w.T on the decode split-K kernel without a K split (``w`` row-major [N, K], or
    ``tile_weight``'s copy with ``rowmajor=False``)."""
    M, K = x.shape
    if not N.use_native(x):
        return F.linear(x.float(), (w if rowmajor else untile_weight(w)).float()).to(x.dtype)
    y = out if out is not None else torch.empty((M, N_), dtype=x.dtype, device=x.device)
    N.call("penny_splitk_gemm_bf16", N.ptr(x), x.stride(0), N.ptr(w), K, N.ptr(y), y.stride(0), M, N_, nf,
           _wrow(rowmajor, M, N_, K), N.stream())
    return y


# "tiled": the decode kernels stream a fragment-tiled copy of each measured projection (made once
# at load, ``tile_weight``; 3-10 % faster for gate|up); "rowmajor": they always stream the
# row-major weights directly (no extra HBM).  Shapes without a tiled copy use row-major anyway.
DECODE_WEIGHTS = os.environ.get("PENNY_DECODE_WEIGHTS", "tiled")
# Decode streams whose BK=64 stages are issued (and waited for) in pairs (gemm_splitk.hip BKM = 2:
# half the ring iterations and barriers per K slice) -- (N, K) -> up to how many rows.  Measured per
# table config, paired vs single, interleaved (bench/kernels.py rm_pair,
# profiles/r5_decode_gemm_paired_stages_ab.jsonl; bit-identical outputs): at M <= 128 Llama-3-8B QKV
# +4-6 %, O +5-12 %, down +2-4 %, gate|up +3-6 %; Llama-3-70B TP=8 shards QKV +5-13 %, O +3-17 %,
# down +10-25 %, gate|up +2-5 %; 70B TP=1 +1-6 %.  From 192 rows the MFMA work per stage hides the
# barrier and the two forms tie.  PENNY_PAIR_STAGES=0 / 1: never / always (A/B).
PAIRED: Dict[Tuple[int, int], int] = {
    (6144, 4096): 128, (4096, 4096): 128, (4096, 14336): 128, (28672, 4096): 128,        # Llama-3-8B
    (1280, 8192): 128, (8192, 1024): 128, (8192, 3584): 128, (7168, 8192): 128,          # 70B TP=8 shards
    (10240, 8192): 128, (8192, 8192): 128, (8192, 28672): 128, (57344, 8192): 16,        # 70B TP=1
}
PAIR_MODE = os.environ.get("PENNY_PAIR_STAGES", "table")


def _wrow(rowmajor: bool, M: int = 0, N_: int = 0, K: int = 0) -> int:
    """The kernels' W-layout argument: bit 0 row-major (else fragment-tiled), bit 1 paired stages."""
    pair = PAIR_MODE == "1" or (PAIR_MODE == "table" and M <= PAIRED.get((N_, K), 0))
    return int(bool(rowmajor)) | (2 if pair else 0)


# Shapes that keep ONLY the fragment-tiled copy (no row-major weight): every path runs on it -- the
# prefill tile kernel's tiled form (penny_gemm_prefill_wt, bit-equal and at speed parity,
# profiles/r5_tile_gemm_fragment_tiled_w.jsonl) and the decode kernels.  Llama-3-70B TP=1 gate|up: its
# row-major decode stream lost to hipBLASLt from 17 rows (4.3 TB/s), the tiled fused kernel wins
# (168-198 vs 184-205 us at M = 16-128, profiles/r5_gateup_shapes.jsonl), and a second copy would cost
# 75 GB of KV pool.  Config 4 short run (6/2) A/B on one box: 3.25 vs 3.28 turns/s, p50 TTFT 4.38 vs
# 4.63 s (neutral; profiles/r5_bench_llama70b_tp1_toolsteps3_6x2_tiled_only_gateup.json) -- and no
# hipBLASLt on the 70B gate|up.  PENNY_TILED_ONLY=0: row-major as before.
TILED_ONLY = {(57344, 8192)} if os.environ.get("PENNY_TILED_ONLY", "1") != "0" else set()
# decode configs on the tiled-only gate|up: [(max M, S, nf)], S = 1 -> the fused kernel
TILED_ONLY_GATEUP: Dict[Tuple[int, int], List[Tuple[int, int, int]]] = {
    (57344, 8192): [(1, 8, 2), (8, 2, 2), (256, 1, 8)],      # guS8nf2 155 us, guS2nf2 165, gu_nf8 168-320
}


def tiled_only(N_: int, K: int) -> bool:
    return (N_, K) in TILED_ONLY


def linear_tiled(x: torch.Tensor, wt: torch.Tensor, N_: int, epilogue: Optional[str] = None) -> torch.Tensor:
    """``linear`` for a weight kept only as its fragment-tiled copy (``TILED_ONLY``): the prefill tile
    kernel's tiled form above 256 rows, the decode kernels below (gate|up + SiLU only)."""
    M, K = x.shape
    if epilogue != "silu":
        raise ValueError("tiled-only weights: gate|up with the SiLU epilogue only")
    if not N.use_native(x) or x.stride(1) != 1 or x.stride(0) % 8:
        return linear(x, untile_weight(wt).contiguous(), epilogue=epilogue)
    if M > 256:
        return prefill_gemm_tiled(x, wt, N_, "silu")
    for max_m, S, nf in TILED_ONLY_GATEUP.get((N_, K), [(256, 1, 8)]):
        if M <= max_m:
            return gateup_silu(x, wt, N_, nf) if S == 1 else gateup_splitk(x, wt, N_, S, nf)
    return gateup_silu(x, wt, N_, 8)


def uses_tiled_weight(N_: int, K: int) -> bool:
    """Does any decode kernel stream a fragment-tiled copy of an [N, K] weight?  Only shapes with a
    measured entry (``TUNING`` skinny, ``SPLITK``, ``GATEUP``) do; everything else stays on
    hipBLASLt and a tiled copy would only take HBM from the KV pool (Llama-3-70B at TP=1: 62 GB)."""
    if (N_, K) in TUNING or (N_, K) in TILED_ONLY:   # the skinny kernel reads tiled weights only
        return True
    if DECODE_WEIGHTS == "rowmajor" or (N_, K) in TILE_FREE:
        return False
    if os.environ.get("PENNY_SPLITK", "1") == "force":
        return True
    return (N_, K) in SPLITK or (N_, K) in GATEUP or any(not e[4] for e in GATEUP_SPLITK.get((N_, K), ()))


def splitk_config(M: int, N_: int, K: int) -> Optional[Tuple[int, int]]:
    """(S, nf) for a split-K launch of this shape, or None.  ``PENNY_SPLITK=0`` disables the
    path; ``PENNY_SPLITK=force`` takes it for any shape the kernel accepts (tests)."""
    mode = os.environ.get("PENNY_SPLITK", "1")
    if mode == "0" or M > 256:
        return None
    for max_m, S, nf in SPLITK.get((N_, K), ()):
        if M <= max_m:
            return (S, nf) if S > 0 else None
    if mode == "force":
        nf = 4 if N_ % 64 == 0 else 2
        for S in (4, 2, 1):
            if K % (64 * S) == 0 and N_ % (16 * nf) == 0:
                return S, nf
    return None


# (N, K) of the interleave16 gate|up weight -> [(min M, max M, nf), ...] for the fused
# gate|up + SiLU*up MFMA kernel (penny_gateup_silu_gemm; no split-K), measured against hipBLASLt
# (curated solutions) + silu_mul with W streamed from HBM (bench/kernels.py --only gateup,
# profiles/r1_gateup_v1.jsonl): 1.4x at M <= 16, 1.22-1.35x at M = 32..96, 1.14x at M = 128; at
# M >= 192 the 3-deep ring of the 256-token tile is MFMA/LDS-latency bound and the library wins.
GATEUP: Dict[Tuple[int, int], List[Tuple[int, int, int]]] = {
    # r5 re-measure (profiles/r5_gateup_shapes.jsonl): 1.5x at M <= 16, 1.2-1.3x at 32-128, and also
    # ahead above 160 rows (1.15x at 192, 1.02x at 256)
    # (r5 paired stages: one row is the split-K form's, GATEUP_SPLITK)
    (28672, 4096): [(2, 256, 8)],
}


def gateup_config(M: int, N_: int, K: int) -> Optional[int]:
    """nf for the fused gate|up kernel at this shape, or None (``PENNY_GATEUP=0`` disables;
    ``PENNY_GATEUP=force`` takes it for any shape the kernel accepts)."""
    mode = os.environ.get("PENNY_GATEUP", "1")
    if mode == "0" or M > 256 or K % 64:
        return None
    for lo, hi, nf in GATEUP.get((N_, K), ()):
        if lo <= M <= hi:
            return nf
    if mode == "force":
        return 8 if N_ % 128 == 0 else (4 if N_ % 64 == 0 else None)
    return None


def gateup_silu(x: torch.Tensor, wt: torch.Tensor, N_: int, nf: int,
                out: Optional[torch.Tensor] = None, rowmajor: bool = False) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) from the interleave16 gate|up weight: its fragment-tiled copy
    ``wt`` or (``rowmajor``) the [N, K] weight itself."""
    M, K = x.shape
    if not N.use_native(x):
        return silu_mul(F.linear(x, wt if rowmajor else untile_weight(wt)), interleave16=True)
    y = out if out is not None else torch.empty((M, N_ // 2), dtype=x.dtype, device=x.device)
    N.call("penny_gateup_silu_gemm", N.ptr(x), x.stride(0), N.ptr(wt), K, N.ptr(y), y.stride(0), M, N_, nf,
           _wrow(rowmajor, M, N_, K), N.stream())
    return y


# (N, K) of the interleave16 gate|up weight -> [(min M, max M, S, nf, rowmajor), ...]: split-K slabs +
# the reduce-SiLU pass (penny_splitk_reduce_silu) where the fused kernel's column tiles alone underfill
# the chip or its weights stream row-major (Llama-3-70B: TP=8 shard, TP=1 without a tiled copy).
# Filled from bench/kernels.py --only shard_shapes (guS* rows).
GATEUP_SPLITK: Dict[Tuple[int, int], List[Tuple[int, int, int, int, bool]]] = {
    # Llama-3-70B TP=8 gate|up shard (interleave16 of 2 x 3584 rows), fragment-tiled: 1.26-1.48x
    # hipBLASLt + silu_mul at every M = 1..256 (the fused kernel: 112 column tiles, 0.96-1.10x)
    (7168, 8192): [(1, 64, 2, 4, False), (65, 256, 4, 8, False)],
    # Llama-3-70B TP=1, row-major (no tiled copy: 75 GB): 1.23x at M = 1, 1.08x at 8, 1.04x at 16;
    # hipBLASLt from 32 rows
    (57344, 8192): [(1, 1, 8, 2, True), (2, 16, 4, 2, True)],
    # Llama-3-8B at one row: S4 nf2 + reduce-SiLU with paired stages 44.4 us vs the fused kernel's 50.3
    # (r5_decode_gemm_paired_stages_ab.jsonl)
    (28672, 4096): [(1, 1, 4, 2, False)],
}


def gateup_splitk_config(M: int, N_: int, K: int) -> Optional[Tuple[int, int, bool]]:
    """(S, nf, rowmajor) for the split-K gate|up path at this shape, or None."""
    if os.environ.get("PENNY_GATEUP", "1") == "0" or M > 256:
        return None
    for lo, hi, S, nf, rm in GATEUP_SPLITK.get((N_, K), ()):
        if lo <= M <= hi and K % (64 * S) == 0 and N_ % (32 * nf) == 0:
            return S, nf, rm
    return None


def gateup_splitk(x: torch.Tensor, w: torch.Tensor, N_: int, S: int, nf: int, rowmajor: bool = False,
                  slabs: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) as split-K f32 slabs of the interleave16 gate|up weight (``w`` its
    fragment-tiled copy, or the [N, K] weight with ``rowmajor``) + one reduce-SiLU pass -- the same
    roundings as the fused kernel (gate / up rounded to bf16, SiLU in bf16, product rounded)."""
    M, K = x.shape
    P = splitk_partials(x, w, N_, S, nf, out=slabs, rowmajor=rowmajor)
    if not N.use_native(x):
        g = P.sum(0).to(torch.bfloat16)
        return silu_mul(g, interleave16=True)
    y = out if out is not None else torch.empty((M, N_ // 2), dtype=x.dtype, device=x.device)
    N.call("penny_splitk_reduce_silu", N.ptr(P), S, M, N_, N.ptr(y), y.stride(0), N.stream())
    return y


class ResidualSum:
    """A row-parallel projection whose residual add already happened: the tile kernel's residual
    epilogue wrote ``x @ w.T + residual`` over the residual stream in place.  ``ops.rms_norm``
    given it (with that same residual) only normalises -- one HBM pass less than GEMM -> bf16 ->
    add&norm, and no [M, N] projection output."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        self.t = t

    @property
    def shape(self):
        return self.t.shape


class Slabs:
    """A split-K GEMM output left unreduced: f32 partial sums ``P`` [S, M, N].  Consumers that
    read the activation anyway (``ops.rms_norm``, ``ops.rope_kv_write``) sum the slabs inside
    their own row pass; anything else calls :meth:`materialize`."""

    __slots__ = ("P",)

    def __init__(self, P: torch.Tensor):
        self.P = P

    @property
    def shape(self) -> Tuple[int, int]:
        return (self.P.shape[1], self.P.shape[2])

    def materialize(self) -> torch.Tensor:
        return splitk_reduce(self.P)


def splitk_partials(x: torch.Tensor, wt: torch.Tensor, N_: int, S: int, nf: int,
                    out: Optional[torch.Tensor] = None, rowmajor: bool = False) -> torch.Tensor:
    """P[s] = x @ w[:, slice s].T as f32 slabs [S, M, N] (``wt`` = ``tile_weight(w)``, or ``w``
    itself with ``rowmajor``)."""
    M, K = x.shape
    if not N.use_native(x):
        w = (wt if rowmajor else untile_weight(wt)).float()
        xs = x.float().view(M, S, K // S).transpose(0, 1)
        return torch.einsum("smk,snk->smn", xs, w.view(N_, S, K // S).transpose(0, 1))
    P = out if out is not None else torch.empty((S, M, N_), dtype=torch.float32, device=x.device)
    N.call("penny_splitk_gemm", N.ptr(x), x.stride(0), N.ptr(wt), K, N.ptr(P), M, N_, S, nf,
           _wrow(rowmajor, M, N_, K), N.stream())
    return P


def splitk_reduce(P: torch.Tensor, residual: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y = bf16(sum_s P[s]) (+ residual)."""
    S, M, N_ = P.shape
    if not N.use_native(P):
        y = P.sum(0).to(torch.bfloat16)
        return y if residual is None else (y.float() + residual.float()).to(torch.bfloat16)
    y = out if out is not None else torch.empty((M, N_), dtype=torch.bfloat16, device=P.device)
    N.call("penny_splitk_reduce", N.ptr(P), S, M, N_, N.ptr(y), y.stride(0), N.ptr(residual),
           residual.stride(0) if residual is not None else 0, N.stream())
    return y


# ----------------------------------------------------------------------------------------------
# Prefill GEMM (M > 256 token rows): 256x256-tile MFMA kernel with fused epilogues
# ----------------------------------------------------------------------------------------------
PREFILL_EPI = {None: 0, "silu": 1, "slabs": 2, "residual": 3, "bias": 5, "bias_gelu": 6}


# Which path each Llama-3-8B projection takes at a prefill step of M rows (M > 256), measured with
# its consumer on MI355X, interleaved A/B (bench/kernels.py prefill_policy), with the tile kernel's
# wave-quantisation tail (profiles/r3_prefill_policy_v5_tail.jsonl; before the tail:
# r3_prefill_policy_v3_widestores.jsonl, the residual epilogue: r3_prefill_policy_v4_residual.jsonl):
# (N, K) -> [(max M, choice), ...], first match wins.
#   "lib"  hipBLASLt (+ the separate epilogue pass)       "hip"  tile kernel, fused epilogue
#   "S<n>" tile kernel split-K into n f32 slabs (only where the consumer reads slabs)
#   "fused" (QKV only) tile kernel with RoPE + paged-KV-write epilogue (prefill_qkv_rope)
#   "R"    tile kernel adding the residual stream in place (ResidualSum; the consumer's RMSNorm
#          then skips the add): O from M = 2816 is 3-5 % faster than hipBLASLt + add&norm; only
#          where the caller passes fuse_residual
#   "K<nf>" the decode kernel's bf16-output form (row-major W, nf row groups per workgroup) with
#          256-row token chunks side by side -- narrow row-parallel TP shards at small prefill steps
#   "M<S>" the 128 x 128 tile kernel (gemm_mid.hip) with S K-slices: S = 1 its fused epilogue (bf16 /
#          SiLU), S > 1 f32 slabs for a slab-reading consumer, else slabs + penny_splitk_reduce{,_silu}
# QKV (r4): the fused RoPE + paged-KV-write tile kernel at every M > 256 as well (hipBLASLt was
# 7-15 us per layer faster at 257-1280 rows; at the driver config the bench is unchanged, 32.2
# turns/s, profiles/r4_bench128_20x5_all_prefill_gemms_tile_kernel.json).
# O (r4): every M > 256 on the tile kernel -- split-K slabs to 2048 rows, the residual epilogue
# above.  Between 257 and 3072 rows hipBLASLt is 2-7 us per layer faster (5-8 %, 256x256 tiles
# underfill the CUs: profiles/r4_gemm_stream_k_tail_rejected.jsonl "r3 kernel" rows), ~0.2 ms
# per prefill step of ~35 ms; the slab / in-place epilogues keep the O output out of a separate
# add pass, and the projection on the framework's own MFMA kernel at every prefill size.
# r6: no projection of the SURVEY-named models takes hipBLASLt at prefill any more.  Shapes without
# an entry use ``_default_choice``.
PREFILL_POLICY: Dict[Tuple[int, int], List[Tuple[int, str]]] = {
    (6144, 4096): [(1 << 30, "fused")],                                                   # QKV
    # r6: the 8B O / down at small steps (decide-only and short respond steps) on the 128 x 128 tile's
    # slabs (bench/kernels.py --only mid_8b, profiles/r6_mid_8b_prefill.jsonl, GEMM + the consumer's
    # slab read at ~5 TB/s): O 26.5-27.1 vs 36.1-36.6 us at 320-384 rows (M4), 29.9-44.2 vs 38.6-50.5 at
    # 512-1024 (M2); down 58.6-66.3 vs 78.6-80.8 us at 320-512 rows (M4).  QKV keeps the fused
    # RoPE / KV-write tile (mid2 slabs + the separate RoPE pass: within a few us of it)
    (4096, 4096): [(384, "M4"), (1024, "M2"), (2048, "S2"), (1 << 30, "R")],             # O
    (28672, 4096): [(1 << 30, "hip")],                                                    # gate|up + SiLU
    (4096, 14336): [(512, "M4"), (1024, "S4"), (1280, "hip"), (2048, "S2"), (1 << 30, "R")],   # down
    # Llama-3-70B TP=1 (r5, r6): each projection WITH its consumer (RoPE/KV write, add&RMSNorm, SiLU),
    # interleaved, M = 384..4096 (bench/kernels.py --only prefill_policy_70b,
    # profiles/r5_prefill_policy_70b_tp1_with_consumers.jsonl; QKV small steps on the 128 x 128 tile,
    # profiles/r6_mid_shards.jsonl: mid2 64.6 vs hipBLASLt 67.5 us at 384 rows).  O with the residual
    # epilogue is 2-5 % behind the library at 1.5-4k rows, down S2 / S4 7 % at 768 / 1536 rows, QKV
    # fused ~5 % at 1024 rows (134.6 us library + the RoPE pass vs 146.7 fused)
    (10240, 8192): [(384, "M2"), (768, "S2"), (1 << 30, "fused")],                       # QKV
    (8192, 8192): [(512, "S4"), (1024, "S2"), (1 << 30, "R")],                           # O
    (57344, 8192): [(1 << 30, "hip")],          # gate|up (kept fragment-tiled only: linear_tiled)
    (8192, 28672): [(512, "S4"), (768, "S2"), (1024, "hip"), (1536, "S4"), (1 << 30, "R")],   # down
    # Llama-3-70B TP=8 per-rank shards (r6, profiles/r6_mid_shards.jsonl, bench/kernels.py --only
    # mid_shards: every hand-written form interleaved against hipBLASLt per M = 384..4096): the 128 x 128
    # tile where the 256 x 256 one underfills the CUs, the 256 x 256 one from ~1.5k rows.
    #   QKV   1.13-1.67x hipBLASLt to 3072 rows, 0.98x at 4096
    #   O     1.21-1.59x to 1024 rows, 0.94-1.07x above
    #   gate|up 0.97x at 384-512, 0.90-0.99x at 768-1024, 1.02-1.09x at 1536-3072, 0.96x at 4096
    #   down  0.82x at 384, 0.93x at 512-768, 0.99-1.02x at 1024-2048, 0.89x at 3072, 0.97x at 4096
    # (the library's lead at the smallest down / gate|up steps is its smaller-tile kernel set; those
    # steps are a few % of a config-4 prefill step's GEMM time -- the framework's kernels run them)
    (1280, 8192): [(1024, "M8"), (1536, "M4"), (3072, "S4"), (1 << 30, "S2")],           # QKV shard
    (8192, 1024): [(1536, "M1"), (1 << 30, "hip")],                                      # O shard
    (7168, 8192): [(384, "M4"), (512, "M2"), (1 << 30, "hip")],                          # gate|up shard
    (8192, 3584): [(384, "M2"), (1024, "M1"), (1 << 30, "hip")],                         # down shard
}


def _default_choice(M: int, N_: int, K: int, epilogue: Optional[str]) -> str:
    """Unmeasured shapes: the tile kernel once its 256x256 tiles cover the 256 CUs (one tile
    alone runs ~80 us at K = 4096, so fewer tiles lose to the library's smaller ones)."""
    tiles = -(-M // 256) * (N_ // 256)
    # a fused activation also saves the library path's separate pass over the [M, N] output
    return "hip" if tiles >= 224 or (epilogue in ("silu", "bias_gelu") and tiles >= 112) else "lib"


def prefill_choice(M: int, N_: int, K: int, epilogue: Optional[str] = None, slabs: bool = False,
                   fused_residual: bool = False) -> str:
    if os.environ.get("PENNY_PREFILL_GEMM", "1") == "0":
        return "lib"
    force = os.environ.get("PENNY_PREFILL_GEMM") == "force"
    rows = PREFILL_POLICY.get((N_, K))
    choice = None
    if rows is not None and not force:
        for max_m, c in rows:
            if M <= max_m:
                choice = c
                break
    if choice is None:
        choice = "hip" if force else _default_choice(M, N_, K, epilogue)
    if force and fused_residual and epilogue is None:
        choice = "R"
    if choice.startswith("S") and not (slabs and epilogue is None and K % (64 * int(choice[1:])) == 0):
        choice = "hip" if force else "lib"
    if choice == "R" and not fused_residual:
        choice = "hip" if force else "lib"
    if choice == "fused":           # only the QKV entry point (qkv_rope_choice) fuses RoPE
        choice = "hip"
    if choice.startswith("K") and epilogue is not None:
        choice = "lib"
    if choice.startswith("M") and (N_ % 128 or K % (64 * int(choice[1:])) or
                                   (epilogue == "residual" and int(choice[1:]) > 1)):
        choice = "lib"
    return choice


# ----------------------------------------------------------------------------------------------
# 128 x 128 tile kernel (gemm_mid.hip): the narrow TP shards and small prefill steps, where the
# 256 x 256 tile leaves most CUs idle.  PREFILL_POLICY choice "M<S>": S = 1 fused epilogue, S > 1
# split-K slabs (the consumer's reduce, or penny_splitk_reduce{,_silu} for bf16 / SiLU outputs).
# ----------------------------------------------------------------------------------------------
MID_EPI = {None: 0, "silu": 1, "slabs": 2, "residual": 3}


def mid_variant(v: int = -1) -> int:
    """Select the mid kernel's staging variant (gemm_mid.hip: 0 = BK 64 x 2 stages, 1 = BK 64 x 3
    counted stages, 2 = BK 32 x 3 counted stages) and return the previous one; -1 only reads it.
    ``PENNY_MID_VARIANT`` sets the initial value.  In-process A/B runs and tests."""
    return int(N.load().penny_gemm_mid_variant(int(v)))


def mid_gemm(x: torch.Tensor, w: torch.Tensor, epilogue: Optional[str] = None, S: int = 1,
             residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x @ w.T on the 128 x 128 tile kernel: bf16 [M, N]; "silu" -> silu(gate)*up bf16 [M, N/2] of the
    interleave16 gate|up weight; "slabs" -> f32 split-K partials [S, M, N]; "residual" -> bf16 + R."""
    M, K = x.shape
    N_ = w.shape[0]
    if not N.use_native(x):
        return prefill_gemm(x, w, epilogue, S, residual=residual, out=out)
    if epilogue == "slabs":
        y = out if out is not None else torch.empty((S, M, N_), dtype=torch.float32, device=x.device)
        ldy = N_
    else:
        S = 1
        cols = N_ // 2 if epilogue == "silu" else N_
        y = out if out is not None else torch.empty((M, cols), dtype=x.dtype, device=x.device)
        ldy = y.stride(0)
    N.call("penny_gemm_mid", N.ptr(x), x.stride(0), N.ptr(w), K, N.ptr(y), ldy, N.ptr(residual),
           residual.stride(0) if residual is not None else 0, M, N_, S, MID_EPI[epilogue], N.stream())
    return y


def mid_linear(x: torch.Tensor, w: torch.Tensor, S: int, epilogue: Optional[str] = None, slabs: bool = False,
               residual: Optional[torch.Tensor] = None) -> Union[torch.Tensor, "Slabs"]:
    """``linear`` on the 128 x 128 tile kernel with S K-slices: the fused epilogue at S = 1; at S > 1
    the slabs themselves where the consumer reduces them (``slabs``), else the reduce pass with the
    bf16 / SiLU output."""
    if S == 1:
        return mid_gemm(x, w, epilogue, residual=residual)
    P = mid_gemm(x, w, "slabs", S)
    if epilogue == "silu":
        M, N_ = x.shape[0], w.shape[0]
        if not N.use_native(x):
            return silu_mul(P.sum(0).to(x.dtype), interleave16=True)
        y = torch.empty((M, N_ // 2), dtype=x.dtype, device=x.device)
        N.call("penny_splitk_reduce_silu", N.ptr(P), S, M, N_, N.ptr(y), y.stride(0), N.stream())
        return y
    if slabs and residual is None:
        return Slabs(P)
    return splitk_reduce(P, residual=residual)


def qkv_rope_fused(x: torch.Tensor, w: torch.Tensor, D: int) -> bool:
    """Does this prefill step run the fused QKV + RoPE + KV-write tile kernel?"""
    M, K = x.shape
    N_ = w.shape[0]
    if D != 128 or M <= 256 or not prefill_ok(x, w):
        return False
    mode = os.environ.get("PENNY_PREFILL_GEMM", "1")
    if mode == "0":
        return False
    if mode == "force":
        return True
    rows = PREFILL_POLICY.get((N_, K))
    if rows is None:
        return _default_choice(M, N_, K, None) == "hip"
    return next(c for max_m, c in rows if M <= max_m) == "fused"


def prefill_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    M, K = x.shape
    N_ = w.shape[0]
    return (N.use_native(x) and os.environ.get("PENNY_PREFILL_GEMM", "1") != "0" and N_ % 256 == 0
            and K % 64 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous())


def prefill_gemm(x: torch.Tensor, w: torch.Tensor, epilogue: Optional[str] = None, S: int = 1,
                 residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x @ w.T on the hand-written 256x256 MFMA tile kernel (``gemm_prefill.hip``).

    ``epilogue``: None -> bf16 [M, N]; "silu" -> silu(gate)*up bf16 [M, N/2] from the
    interleave16 gate|up weight; "slabs" -> f32 split-K partials [S, M, N]; "residual" -> bf16
    x @ w.T + residual; "bias" / "bias_gelu" -> bf16(x @ w.T + bias) [-> exact GELU].  The torch
    path (CPU) computes the same math in f32."""
    M, K = x.shape
    N_ = w.shape[0]
    if not N.use_native(x):
        if epilogue == "slabs":
            xs = x.float().view(M, S, K // S).transpose(0, 1)
            return torch.einsum("smk,snk->smn", xs, w.float().view(N_, S, K // S).transpose(0, 1))
        y = F.linear(x.float(), w.float(), bias.float() if bias is not None else None).to(x.dtype)
        if epilogue == "bias_gelu":
            y = F.gelu(y.float()).to(x.dtype)
        elif epilogue == "silu":
            y = silu_mul(y, interleave16=True)
        elif epilogue == "residual":
            y = (y.float() + residual.float()).to(x.dtype)
        return out.copy_(y) if out is not None else y
    if epilogue == "slabs":
        y = out if out is not None else torch.empty((S, M, N_), dtype=torch.float32, device=x.device)
        ldy = N_
    else:
        S = 1
        cols = N_ // 2 if epilogue == "silu" else N_
        y = out if out is not None else torch.empty((M, cols), dtype=x.dtype, device=x.device)
        ldy = y.stride(0)
    R = bias if epilogue in ("bias", "bias_gelu") else residual
    N.call("penny_gemm_prefill", N.ptr(x), x.stride(0), N.ptr(w), K, N.ptr(y), ldy, N.ptr(R),
           residual.stride(0) if residual is not None else 0, M, N_, S, PREFILL_EPI[epilogue],
           *tail_workspace(x.device), N.stream())
    return y


def prefill_gemm_tiled(x: torch.Tensor, wt: torch.Tensor, N_: int, epilogue: Optional[str] = None, S: int = 1,
                       residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``prefill_gemm`` on the fragment-tiled weight (``tile_weight``'s copy, the layout the decode
    kernels stream) instead of the row-major one: same MFMA sequence, bit-equal output.  Epilogues
    None / "silu" / "slabs" / "residual"."""
    M, K = x.shape
    if not N.use_native(x):
        return prefill_gemm(x, untile_weight(wt), epilogue, S, residual=residual, out=out)
    if epilogue == "slabs":
        y = out if out is not None else torch.empty((S, M, N_), dtype=torch.float32, device=x.device)
        ldy = N_
    else:
        S = 1
        cols = N_ // 2 if epilogue == "silu" else N_
        y = out if out is not None else torch.empty((M, cols), dtype=x.dtype, device=x.device)
        ldy = y.stride(0)
    N.call("penny_gemm_prefill_wt", N.ptr(x), x.stride(0), N.ptr(wt), K, N.ptr(y), ldy, N.ptr(residual),
           residual.stride(0) if residual is not None else 0, M, N_, S, PREFILL_EPI[epilogue],
           *tail_workspace(x.device), N.stream())
    return y


# Wave-quantisation tail of the tile kernel (gemm_prefill.hip TailArgs): one workspace per
# (device, stream) -- f32 partial tiles of at most one round of tail workgroups (64 MB) and
# self-resetting ticket counters.  PENNY_GEMM_TAIL=0 launches whole tiles only (A/B).
_TAIL_WS: Dict[Tuple[int, int], Tuple[torch.Tensor, torch.Tensor, int]] = {}


def tail_workspace(dev: torch.device) -> Tuple:
    if os.environ.get("PENNY_GEMM_TAIL", "1") == "0":
        return (None, 0, None, 0, 0)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), torch.cuda.current_stream(dev).cuda_stream)
    ent = _TAIL_WS.get(key)
    if ent is None:
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        part = torch.empty((cus * 256 * 256,), dtype=torch.float32, device=dev)
        cnt = torch.zeros((cus,), dtype=torch.int32, device=dev)
        ent = _TAIL_WS[key] = (part, cnt, cus)
    part, cnt, cus = ent
    return (N.ptr(part), part.numel(), N.ptr(cnt), cnt.numel(), cus)


# bge query batches up to this many tokens run every projection on the tile kernel: the encoder is
# launch-bound there (~2 ms for 12 layers) and the fused bias / bias+GELU epilogues save launches and
# passes -- 1.72 vs 2.15 ms for 1 query, 2.12 vs 2.24 ms for 24, 2.18 vs 2.26 ms for 64 (1.5k tokens)
# against hipBLASLt + the GELU pass; at 4k tokens the per-shape policy decides
# (profiles/r3_bge_query_tile_vs_hipblaslt.jsonl)
BGE_TILE_MAX_M = 2048


def linear_bias(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, gelu: bool = False) -> torch.Tensor:
    """Encoder projection bf16(x @ w.T + b) [-> exact GELU] on the tile kernel with the bias (+GELU)
    epilogue: always for query-size batches (<= BGE_TILE_MAX_M tokens), by the measured per-shape
    policy for bulk ingest; hipBLASLt's bias GEMM + the HIP GELU pass otherwise
    (``PENNY_PREFILL_GEMM=0``: always the library)."""
    M, K = x.shape
    N_ = w.shape[0]
    mode = os.environ.get("PENNY_PREFILL_GEMM", "1")
    if mode != "0" and prefill_ok(x, w) and (M <= BGE_TILE_MAX_M or mode == "force" or
                                            prefill_choice(M, N_, K, "bias_gelu" if gelu else "bias") == "hip"):
        return prefill_gemm(x, w, "bias_gelu" if gelu else "bias", bias=b)
    y = F.linear(x, w, b)
    if gelu:
        from .activation import gelu_
        return gelu_(y)
    return y


def prefill_qkv_rope(x: torch.Tensor, w: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                     slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, Hq: int,
                     Hkv: int, qscale: float = 1.0) -> torch.Tensor:
    """Fused QKV projection + RoPE + paged KV write (head dim 128) on the prefill tile kernel:
    returns the rotated q [M, Hq, 128] -- times ``qscale`` before its one bf16 rounding (the
    attention's prescaled-q form) -- while k / v land in the caches (slots < 0 are skipped)."""
    from .attention import rope_kv_write
    M, K = x.shape
    if not N.use_native(x):
        if qscale == 1.0:
            return rope_kv_write(F.linear(x.float(), w.float()).to(x.dtype), positions, cos_sin, slots, k_cache,
                                 v_cache, Hq, Hkv, 128)
        from .attention import _rope_ref
        qkv = F.linear(x.float(), w.float()).to(x.dtype)
        rope_kv_write(qkv, positions, cos_sin, slots, k_cache, v_cache, Hq, Hkv, 128)
        qr = _rope_ref(qkv[:, :Hq * 128].float().view(M, Hq, 128), positions, cos_sin)   # f32
        return (qr * qscale).to(x.dtype)
    q = torch.empty((M, Hq, 128), dtype=x.dtype, device=x.device)
    N.call("penny_gemm_prefill_qkv_rope", N.ptr(x), x.stride(0), N.ptr(w), K, M, N.ptr(positions), N.ptr(cos_sin),
           N.ptr(slots), N.ptr(q), N.ptr(k_cache), N.ptr(v_cache), Hq, Hkv, float(qscale), *tail_workspace(x.device),
           N.stream())
    return q


def untile_weight(wt: torch.Tensor) -> torch.Tensor:
    """Inverse of ``tile_weight``: [N/16, K/32, 64, 8] -> [N, K]."""
    G, KS = wt.shape[0], wt.shape[1]
    return wt.view(G, KS, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(G * 16, KS * 32)
