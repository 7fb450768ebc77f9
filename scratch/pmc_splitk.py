"""PMC probe: one split-K config (qkv M=128 S=4 nf=6 by default) in a loop over rotating weights."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from financial_chatbot_llm_amd.ops import gemm  # noqa: E402

N, K, M, S, nf = (int(v) for v in (sys.argv[1:] + ["6144", "4096", "128", "4", "6"][len(sys.argv) - 1:])[:5])
copies = max(2, (768 << 20) // (N * K * 2))
wts = [gemm.tile_weight(torch.randn((N, K), device="cuda").to(torch.bfloat16)) for _ in range(copies)]
x = torch.randn((M, K), device="cuda").to(torch.bfloat16)
P = torch.empty((S, M, N), dtype=torch.float32, device="cuda")
for i in range(200):
    gemm.splitk_partials(x, wts[i % copies], N, S, nf, out=P)
torch.cuda.synchronize()
print("done")
