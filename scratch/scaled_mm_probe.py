"""Probe: hipBLASLt fp8 GEMM (torch._scaled_mm, rowwise scales) vs bf16 F.linear at Mixtral
prefill expert shapes on gfx950."""
import json
import torch
import torch.nn.functional as F

dev = "cuda"
def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters

for (M, N, K) in [(768, 28672, 4096), (768, 4096, 14336), (1536, 28672, 4096), (384, 28672, 4096)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    base = timeit(lambda: F.linear(x, w))
    row = {"M": M, "N": N, "K": K, "bf16_us": round(base, 1), "bf16_TF": round(2 * M * N * K / base / 1e6, 1)}
    try:
        xs = x.float().abs().amax(1, keepdim=True) / 448.0
        ws = w.float().abs().amax(1, keepdim=True) / 448.0
        xq = (x.float() / xs).to(torch.float8_e4m3fn)
        wq = (w.float() / ws).to(torch.float8_e4m3fn)
        f = lambda: torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws.t(), out_dtype=torch.bfloat16)
        y = f()
        err = (y.float() - x.float() @ w.float().t()).abs().max().item()
        us = timeit(f)
        row.update({"fp8_rowwise_us": round(us, 1), "fp8_TF": round(2 * M * N * K / us / 1e6, 1), "max_abs_err": err})
    except Exception as e:  # noqa: BLE001
        row["fp8_error"] = f"{type(e).__name__}: {str(e)[:200]}"
    print(json.dumps(row), flush=True)
