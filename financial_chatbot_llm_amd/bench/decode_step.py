"""Decode-step anatomy: replay the hipGraph decode step of a batch of B running sequences.

    python -m financial_chatbot_llm_amd.bench.decode_step --batch 128 --ctx 1500 --steps 200

Prefills B synthetic prompts of ``--ctx`` tokens (sharing ``--shared`` leading tokens, like the
agent's system prompt), then times ``--steps`` pure decode steps (graph replays through the real
engine: scheduler, block manager, overlap scheduling).  Under ``rocprofv3 --kernel-trace --stats``
the per-kernel table is dominated by the decode step's kernels (``--steps`` >> prefill launches).
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=1500)
    ap.add_argument("--shared", type=int, default=800)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args(argv)
    from ..config import EngineConfig
    from ..engine import LLMEngine, SamplingParams
    cfg = EngineConfig(model=a.model, device="cuda", max_num_seqs=max(a.batch, 1), max_model_len=8192,
                       graph_batch_sizes=(a.batch,))
    eng = LLMEngine(cfg)
    eng.warmup()
    shared = list(range(1000, 1000 + a.shared))
    sp = SamplingParams(temperature=0.7, max_tokens=a.steps + 8, ignore_eos=True, seed=1)
    seqs = [eng.add_request(f"d{i}", shared + [(7 * i + j) % 30000 + 2000 for j in range(a.ctx - a.shared)], sp)
            for i in range(a.batch)]
    while any(s.num_computed < len(s.prompt_ids) for s in seqs):     # prefill everything
        eng.step()
    for _ in range(4):
        eng.step()
    torch.cuda.synchronize()
    g0 = eng.runner.stats["graph_steps"]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"model": a.model, "batch": a.batch, "ctx": a.ctx, "shared": a.shared, "steps": a.steps,
                      "graph_steps": eng.runner.stats["graph_steps"] - g0,
                      "ms_per_step": round(1e3 * dt / a.steps, 3),
                      "tokens_per_s": round(a.batch * a.steps / dt, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
