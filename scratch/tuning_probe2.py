import sys; sys.path.insert(0, ".")
import torch, os, time
from financial_chatbot_llm_amd.ops import gemm
t = torch.cuda.tunable
p = gemm.tuning_file("llama3-8b")
mode = sys.argv[1]
if mode == "warm":
    a = torch.randn(64, 64, device="cuda").to(torch.bfloat16); torch.nn.functional.linear(a, a); torch.cuda.synchronize()
    t.enable(True)
    print("warm read", t.read_file(p))
elif mode == "strip":
    q = "/tmp/strip.csv"
    open(q, "w").write("".join(l for l in open(p) if not l.startswith("Validator,ROCBLAS")))
    t.enable(True)
    print("strip read", t.read_file(q))
elif mode == "enable_first":
    t.enable(True); t.tuning_enable(False)
    a = torch.randn(64, 64, device="cuda").to(torch.bfloat16); torch.nn.functional.linear(a, a); torch.cuda.synchronize()
    print("enable+gemm read", t.read_file(p))
print("n results", len(t.get_results()))
t.tuning_enable(False)
x = torch.randn(128, 14336, device="cuda").to(torch.bfloat16); w = torch.randn(4096, 14336, device="cuda").to(torch.bfloat16)
for _ in range(3): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); t0=time.perf_counter()
for _ in range(50): torch.nn.functional.linear(x, w)
torch.cuda.synchronize(); print(mode, "down M128 us", (time.perf_counter()-t0)/50*1e6)
