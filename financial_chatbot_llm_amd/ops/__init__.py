"""Op layer: Python entry points for the gfx950 HIP kernels (``csrc/kernels``).

Each op dispatches on the tensor's device: CUDA(HIP) tensors run the native kernel (and fail
loudly if the library is missing), CPU tensors run an fp32 PyTorch reference that is also the
oracle in the numerics tests.
"""
from .activation import gelu_, silu_mul
from .attention import (KV_BS, DecodeWorkspace, decode, default_scale, prefill, rope_cos_sin, rope_kv_write,
                        write_kv_ref)
from .embedding import embedding
from .norm import layer_norm, rms_norm
from .retrieval import filtered_topk
from .sampling import (apply_top_k_top_p, fused_lm_head_ok, lm_head_sample, lm_head_sample_shard, lm_head_stream_sample,
                       pick_pairs, sample,
                       sample_shard)

__all__ = ["gelu_", "silu_mul", "KV_BS", "DecodeWorkspace", "decode", "default_scale", "prefill", "rope_cos_sin",
           "rope_kv_write", "write_kv_ref", "embedding", "layer_norm", "rms_norm", "filtered_topk",
           "apply_top_k_top_p", "sample"]
