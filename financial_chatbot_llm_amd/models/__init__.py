"""Model families: Llama-3 (8B/70B), Mixtral-8x7B MoE, BERT/bge encoder."""
from __future__ import annotations

from .configs import REGISTRY, ModelConfig, get_model_config


def build_model(engine_cfg, device, seed: int = 0):
    """Instantiate the decoder named by ``engine_cfg.model`` on ``device`` (random-init unless
    ``engine_cfg.weights`` points at a safetensors checkpoint directory)."""
    from .llama import LlamaModel
    from .mixtral import MixtralModel
    cfg = get_model_config(engine_cfg.model)
    if cfg.arch == "mixtral":
        model = MixtralModel(cfg, device=device, fp8=getattr(engine_cfg, "dtype", "bf16") == "fp8",
                             moe_parallel=getattr(engine_cfg, "moe_parallel", "tp"))
    elif cfg.arch == "llama":
        shard = int(getattr(engine_cfg, "shard_of_tp", 0) or 0)
        # estimate mode: rank 0's shard of a TP=shard group, alone on this device (collectives are
        # identity while the process group is TP=1)
        model = LlamaModel(cfg, device=device, tp_rank=0, tp_size=shard) if shard > 1 else LlamaModel(cfg, device=device)
    else:
        raise ValueError(f"{cfg.name} is not a decoder")
    model.sequence_parallel = bool(getattr(engine_cfg, "sequence_parallel", False))
    if engine_cfg.weights:
        from .weights import load_decoder_weights
        load_decoder_weights(model, engine_cfg.weights)
        if cfg.arch == "mixtral" and model.fp8:
            model.quantize_experts()          # checkpoint experts (bf16) -> tiled fp8 + row scales
    else:
        model.init_random(seed=engine_cfg.seed if hasattr(engine_cfg, "seed") else seed)
    return model


__all__ = ["REGISTRY", "ModelConfig", "get_model_config", "build_model"]
