"""Probe: hipBLASLt split-K via strided-batched bmm (zero-copy K-chunk views) on decode shapes."""
import json, statistics
import torch
dev = torch.device("cuda")

def timeit(fn, iters=20, rounds=5):
    fn(); torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters): fn()
        b.record(); b.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / iters)
    return statistics.median(res)

shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096)}
for M in (32, 64, 128, 256):
    for name, (N, K) in shapes.items():
        w = torch.randn((N, K), device=dev).to(torch.bfloat16)
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        ref = torch.nn.functional.linear(x, w).float()
        row = {"M": M, "name": name, "linear_us": round(timeit(lambda: torch.nn.functional.linear(x, w)), 1)}
        for S in (2, 4, 8):
            if K % S: continue
            xs = x.view(M, S, K // S).transpose(0, 1)          # [S, M, K/S]
            ws = w.view(N, S, K // S).permute(1, 2, 0)         # [S, K/S, N]
            f32 = lambda: torch.bmm(xs, ws, out_dtype=torch.float32).sum(0).to(torch.bfloat16)
            err = (f32().float() - ref).abs().max().item()
            row[f"S{S}_f32_us"] = round(timeit(f32), 1)
            row[f"S{S}_err"] = round(err, 3)
        print(json.dumps(row), flush=True)
