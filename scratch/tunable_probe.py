"""Probe: hipBLASLt default vs TunableOp-selected kernels on Llama-3-8B decode GEMM shapes."""
import json, os, statistics, sys, time
import torch
torch.cuda.set_device(0)
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

shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336), "lm_head": (128256, 4096)}
Ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32, 64, 128, 256]
W = {k: torch.randn(v, device=dev).to(torch.bfloat16) for k, v in shapes.items()}
X = {M: {k: torch.randn((M, v[1]), device=dev).to(torch.bfloat16) for k, v in shapes.items()} for M in Ms}
base = {}
for M in Ms:
    for k in shapes:
        base[(M, k)] = timeit(lambda: torch.nn.functional.linear(X[M][k], W[k]))
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_filename("gpurun_out/tunableop_results.csv")
torch.cuda.tunable.set_max_tuning_duration(100)
t0 = time.time()
for M in Ms:
    for k in shapes:
        torch.nn.functional.linear(X[M][k], W[k])
torch.cuda.synchronize()
print("tuning took", round(time.time() - t0, 1), "s", flush=True)
torch.cuda.tunable.tuning_enable(False)
for M in Ms:
    for k, (N, K) in shapes.items():
        t = timeit(lambda: torch.nn.functional.linear(X[M][k], W[k]))
        byts = (N * K + M * K + M * N) * 2
        print(json.dumps({"M": M, "name": k, "default_us": round(base[(M, k)], 1), "tuned_us": round(t, 1),
                          "default_GBps": round(byts / base[(M, k)] / 1e3), "tuned_GBps": round(byts / t / 1e3)}), flush=True)
torch.cuda.tunable.write_file()
