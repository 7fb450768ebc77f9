"""ctypes binding of ``libpenny_kernels.so`` (the gfx950 HIP kernel library).

The library is loaded AFTER ``import torch`` so its ``libamdhip64.so.7`` dependency resolves
to the HIP runtime torch already mapped (one runtime, one device context, torch's streams are
valid handles).  Every launcher takes the current torch stream, so calls are ordered with
torch's own kernels and are captured by ``torch.cuda.graph`` (hipGraph) like any other launch.

Policy: on a GPU tensor a missing or failing library is an ERROR (ops never fall back silently
on the device -- the round-end check records which native code actually ran).  CPU tensors take
the fp32 PyTorch reference path in each op module (CI / numerics oracle).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_LOCK = threading.Lock()
_LIB: Optional[ctypes.CDLL] = None
_ERR: Optional[str] = None

c_int, c_long, c_float, c_void_p = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_void_p
P = c_void_p

_SIGS = {
    "penny_rmsnorm": [P, P, P, P, c_int, c_int, c_float, c_int, P],
    "penny_rmsnorm_slabs": [P, c_int, P, P, P, c_int, c_int, c_float, c_int, P],
    "penny_layernorm": [P, P, P, P, P, c_int, c_int, c_float, c_int, P],
    "penny_silu_mul": [P, P, c_int, c_int, c_int, P],
    "penny_skinny_gemm": [P, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "penny_splitk_gemm": [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_splitk_reduce": [P, c_int, c_int, c_int, P, c_int, P, c_int, P],
    "penny_splitk_gemm_bf16": [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_lm_head_stream_sample": [P, c_int, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P, c_int, c_int,
                                    c_int, P],
    "penny_lm_sample_final": [P, P, c_int, c_int, P, P, P],
    "penny_gateup_silu_gemm": [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_gemm_prefill": [P, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int,
                           P, c_long, P, c_int, c_int, P],
    "penny_gemm_prefill_wt": [P, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int,
                              P, c_long, P, c_int, c_int, P],
    "penny_gemm_prefill_qkv_rope": [P, c_int, P, c_int, c_int, P, P, P, P, P, P, c_int, c_int,
                                    c_float, P, c_long, P, c_int, c_int, P],
    "penny_gemm_mid_variant": [c_int],
    "penny_gemm_mid": [P, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_gemm_prefill_ablate": [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, P],
    "penny_moe_gemm_prefill_fp8": [P, c_int, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "penny_probe_mfma_scale": [P, P, P, P, P, c_int, P],
    "penny_moe_gemm_prefill_fp8_mx": [P, c_int, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P,
                                      c_int, P],
    "penny_gelu": [P, c_long, P],
    "penny_embedding": [P, P, P, c_int, c_int, c_int, c_int, P],
    "penny_rope_qk": [P, P, P, P, c_int, c_int, c_int, c_int, P],
    "penny_rope_kv_write": [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_rope_kv_write_slabs": [P, c_int, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_attention_prefill": [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, P, P,
                                c_int, P],
    "penny_attention_prefill_variant": [c_int],
    "penny_gemm_prefill_set_group": [c_int],
    "penny_attention_prefill_lean": [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_int, P, P, c_int, P,
                                     c_int, P, P, P],
    "penny_splitk_reduce_silu": [P, c_int, c_int, c_int, P, c_int, P],
    "penny_attention_decode": [P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_float, c_int, P, c_int, c_int, P],
    "penny_sample": [P, c_int, c_long, P, P, P, P, P, P, c_int, c_int, P],
    "penny_lm_head_sample": [P, c_int, P, c_int, c_int, c_int, P, P, P, P, P],
    "penny_lm_head_sample_shard": [P, c_int, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P],
    "penny_sample_shard": [P, c_int, c_long, P, P, P, P, c_int, c_int, c_int, P],
    "penny_topk_topp_threshold": [P, c_int, c_long, P, P, P, P, c_int, c_int, P],
    "penny_moe_route": [P, c_int, c_int, c_int, P, P, P, P, P],
    "penny_moe_route_quant": [P, c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P],
    "penny_quant_rows_fp8": [P, c_int, c_int, c_int, P, P, P],
    "penny_silu_quant_rows_fp8": [P, c_int, c_int, P, P, P],
    "penny_moe_gemm_fp8": [P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "penny_moe_combine": [P, P, c_int, c_int, c_int, P, P],
    "penny_moe_combine_weighted": [P, P, P, c_int, c_int, c_int, P, P],
    "penny_filtered_topk": [P, P, P, c_long, c_int, P, P, P, P, c_int, c_int, P, P, P, c_int, P, P, P, P],
}


def lib_path() -> str:
    """The production kernel library, or its bounds-checked debug build with PENNY_KERNEL_DEBUG=1.
    ``PENNY_KERNEL_LIB`` names another build of the same library (whole-library A/B runs)."""
    if os.environ.get("PENNY_KERNEL_LIB"):
        return os.environ["PENNY_KERNEL_LIB"]
    from .._build import kernel_lib
    return kernel_lib(os.environ.get("PENNY_KERNEL_DEBUG") == "1")


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = lib_path()
        if not os.path.exists(path) and build_if_missing:
            from .._build import build_kernels
            build_kernels(debug=os.environ.get("PENNY_KERNEL_DEBUG") == "1")
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            _ERR = str(e)
            raise RuntimeError(f"penny kernel library unavailable: {e}") from e
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        _LIB = lib
        return lib


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:  # noqa: BLE001
        return False


_FORCE_TORCH_OPS = os.environ.get("PENNY_FORCE_TORCH_OPS") == "1"   # read once: checked on every op


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def stream() -> int:
    """The current HIP stream of the current device, raw (two C calls: ``torch.cuda.current_stream``
    costs ~7 us of Python per call, and every kernel launch asks); the public API where this torch
    build lacks the private entry points."""
    if _RAW_STREAM is not None and _CUR_DEVICE is not None:
        return _RAW_STREAM(_CUR_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")


def use_native(t: torch.Tensor) -> bool:
    """True -> run the HIP kernel.  CPU tensors use the torch reference path."""
    return t.device.type == "cuda" and not _FORCE_TORCH_OPS
