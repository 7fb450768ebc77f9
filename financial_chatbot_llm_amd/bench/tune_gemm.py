"""Curate a per-shape GEMM solution table for the decode buckets (PyTorch TunableOp, offline).

TunableOp benchmarks every hipBLASLt / rocBLAS solution for a GEMM shape.  Its own timing uses
cold rotating buffers, which misranks some decode shapes, so this script re-times each candidate
the way the engine runs it (hot, back-to-back) and keeps a tuned entry only where it beats the
default heuristic by ``--min-gain``; everything else is written as ``Default``.  The engine loads
the resulting CSV read-only at start-up (``ops/gemm.py: load_gemm_tuning``), so graph capture and
serving never tune.

    python -m financial_chatbot_llm_amd.bench.tune_gemm --model llama3-8b \\
        --out financial_chatbot_llm_amd/tuning/gemm_llama3-8b_mi355x.csv
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics
import tempfile
from typing import Dict, List, Tuple

import torch


def _time(fn, iters: int = 30, rounds: int = 5) -> float:
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / iters)
    return statistics.median(res)


def projection_shapes(model: str, tp: int = 1) -> Dict[str, Tuple[int, int]]:
    from ..models.configs import get_model_config
    c = get_model_config(model)
    H, F_ = c.hidden_size, c.intermediate_size
    shapes = {"qkv": ((c.q_size + 2 * c.kv_size) // tp, H), "o": (H, c.q_size // tp),
              "lm_head": (c.vocab_size // tp, H)}
    if c.arch == "llama":
        shapes.update({"gate_up": (2 * F_ // tp, H), "down": (H, F_ // tp)})
    return shapes


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ms", default="1,2,4,8,16,24,32,48,64,96,128,192,256")
    ap.add_argument("--min-gain", type=float, default=0.05)
    ap.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    tun = torch.cuda.tunable
    shapes = projection_shapes(args.model, args.tp)
    Ms = [int(m) for m in args.ms.split(",")]
    W = {k: torch.randn(v, device=dev).to(torch.bfloat16) for k, v in shapes.items()}
    X = {(M, k): torch.randn((M, v[1]), device=dev).to(torch.bfloat16) for M in Ms for k, v in shapes.items()}
    lin = torch.nn.functional.linear
    base = {key: _time(lambda key=key: lin(X[key], W[key[1]])) for key in X}

    raw = os.path.join(tempfile.mkdtemp(), "tunableop_raw.csv")
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(raw, False)
    tun.set_max_tuning_duration(60)
    for key in X:
        lin(X[key], W[key[1]])
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    tuned = {key: _time(lambda key=key: lin(X[key], W[key[1]])) for key in X}
    results = tun.get_results()      # ((op_sig, params_sig, solution, ms), ...)
    validators = tun.get_validators()
    tun.enable(False)

    # params_sig "tn_{N}_{M}_{K}_ld_..." -> keep the tuned solution only where it measured faster
    keep: List[Tuple[str, str, str, float]] = []
    report = []
    for op_sig, params, sol, ms in results:
        parts = params.split("_")
        N_, M, K = int(parts[1]), int(parts[2]), int(parts[3])
        name = next((k for k, v in shapes.items() if v == (N_, K)), None)
        if name is None or (M, name) not in base:
            continue
        b, t = base[(M, name)], tuned[(M, name)]
        win = sol != "Default" and t < b * (1 - args.min_gain)
        keep.append((op_sig, params, sol if win else "Default", ms))
        report.append({"name": name, "M": M, "default_us": round(b, 1), "tuned_us": round(t, 1),
                       "solution": sol, "kept": win})
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w", newline="") as fh:
        w = csv.writer(fh, lineterminator="\n")     # TunableOp's reader does not strip "\r"
        for k, v in validators:
            w.writerow(["Validator", k, v])
        for row in keep:
            w.writerow(list(row))
    for r in report:
        print(json.dumps(r), flush=True)
    kept = [r for r in report if r["kept"]]
    saved = sum(r["default_us"] - r["tuned_us"] for r in kept)
    print(json.dumps({"kept": len(kept), "of": len(report), "saved_us_sum": round(saved, 1), "out": args.out}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
