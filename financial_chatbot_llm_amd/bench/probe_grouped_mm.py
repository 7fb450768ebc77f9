"""Probe: does this torch build run device-offset grouped GEMMs (bf16 ``torch._grouped_mm`` /
fp8 ``torch._scaled_grouped_mm``) on the GPU, and how fast at Mixtral expert shapes?

    python -m financial_chatbot_llm_amd.bench.probe_grouped_mm
"""
from __future__ import annotations

import json
import time

import torch


def _time(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main() -> int:
    dev = "cuda"
    E, H, F2 = 8, 4096, 2 * 14336
    for T in (2048, 8192):
        P = 2 * T
        counts = torch.full((E,), P // E, dtype=torch.int32)
        offs = torch.cumsum(counts, 0).to(torch.int32).to(dev)
        x = torch.randn(P, H, device=dev, dtype=torch.bfloat16)
        w = torch.randn(E, H, F2, device=dev, dtype=torch.bfloat16) * 0.02
        res = {"T": T, "rows": P}
        try:
            y = torch._grouped_mm(x, w, offs=offs)
            t = _time(lambda: torch._grouped_mm(x, w, offs=offs))
            ref = x[: P // E].float() @ w[0].float()
            res["bf16_grouped_mm_ms"] = round(t * 1e3, 3)
            res["bf16_tflops"] = round(2 * P * H * F2 / t / 1e12, 1)
            res["bf16_err"] = float((y[: P // E].float() - ref).abs().max() / ref.abs().max())
        except Exception as e:  # noqa: BLE001
            res["bf16_grouped_mm"] = f"unsupported: {type(e).__name__}: {str(e)[:200]}"
        try:
            xq = x.to(torch.float8_e4m3fn)
            wq = w.to(torch.float8_e4m3fn).transpose(-2, -1).contiguous().transpose(-2, -1)
            sa = torch.ones(P, device=dev, dtype=torch.float32)
            sb = torch.ones(E, F2, device=dev, dtype=torch.float32)
            y = torch._scaled_grouped_mm(xq, wq, sa, sb, offs=offs, out_dtype=torch.bfloat16)
            t = _time(lambda: torch._scaled_grouped_mm(xq, wq, sa, sb, offs=offs, out_dtype=torch.bfloat16))
            res["fp8_scaled_grouped_mm_ms"] = round(t * 1e3, 3)
            res["fp8_tflops"] = round(2 * P * H * F2 / t / 1e12, 1)
        except Exception as e:  # noqa: BLE001
            res["fp8_scaled_grouped_mm"] = f"unsupported: {type(e).__name__}: {str(e)[:200]}"
        # per-expert loop baseline (what the prefill path does today)
        ws = [w[e].t().contiguous() for e in range(E)]
        t = _time(lambda: [torch.nn.functional.linear(x[e * (P // E):(e + 1) * (P // E)], ws[e]) for e in range(E)])
        res["bf16_loop_ms"] = round(t * 1e3, 3)
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
