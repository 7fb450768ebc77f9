import sys; sys.path.insert(0, ".")
import os

import torch, time
from financial_chatbot_llm_amd.ops import gemm
t = torch.cuda.tunable
p = gemm.tuning_file("llama3-8b")
q = "/tmp/strip.csv"
lines = []
for l in open(p):
    if l.startswith("Validator,ROCBLAS"):
        continue
    parts = l.rstrip("\n").split(",")
    if len(parts) == 4 and parts[2].startswith("Gemm_Rocblas"):
        parts[2] = "Default"
    lines.append(",".join(parts) + "\n")
open(q, "w").write("".join(lines))
t.enable(True); t.tuning_enable(False)
print("read", t.read_file(p), "n", len(t.get_results()), t.get_validators())
x = torch.randn(128, 14336, device="cuda").to(torch.bfloat16); w = torch.randn(4096, 14336, device="cuda").to(torch.bfloat16)
for _ in range(3): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); t0=time.perf_counter()
for _ in range(50): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); print("down M128 us", (time.perf_counter()-t0)/50*1e6)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    y = torch.nn.functional.linear(x, w)
g.replay(); torch.cuda.synchronize(); print("graph ok", float((y.float() - torch.nn.functional.linear(x, w).float()).abs().max()))
