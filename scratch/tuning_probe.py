import sys; sys.path.insert(0, ".")
import torch, os
from financial_chatbot_llm_amd.ops import gemm
t = torch.cuda.tunable
p = gemm.tuning_file("llama3-8b")
print("exists", os.path.exists(p), p)
print("read(before enable)", t.read_file(p))
t.enable(True)
print("read(after enable)", t.read_file(p))
print("n results", len(t.get_results()))
print("validators", t.get_validators())
t.tuning_enable(False)
x = torch.randn(128, 14336, device="cuda").to(torch.bfloat16); w = torch.randn(4096, 14336, device="cuda").to(torch.bfloat16)
import time
for _ in range(3): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); t0=time.perf_counter()
for _ in range(50): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); print("down M128 us", (time.perf_counter()-t0)/50*1e6)
t.enable(False)
torch.cuda.synchronize(); t0=time.perf_counter()
for _ in range(50): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); print("default down M128 us", (time.perf_counter()-t0)/50*1e6)
