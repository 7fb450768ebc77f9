"""Probe: decode attention time vs partition size pb (fixed max_ctx 8192 => grid.y = 128/pb)."""
import json, sys
import torch
sys.path.insert(0, ".")
from financial_chatbot_llm_amd import ops
from financial_chatbot_llm_amd.bench.kernels import _paged, timeit
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
Hq, Hkv, D = 32, 8, 128
for B, ctx, shared in [(128, 2304, 1984), (128, 1536, 768), (128, 2048, 0), (64, 2048, 1024), (16, 2048, 1024), (4, 4096, 0), (128, 6000, 0)]:
    tables, kc, vc, total = _paged(B, ctx, shared, Hkv, D, dev, g)
    q = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
    lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    # variable lengths too
    lens_var = torch.randint(max(shared + 65, ctx // 2), ctx + 1, (B,), generator=g, device=dev, dtype=torch.int32)
    o = torch.empty_like(q)
    row = {"B": B, "ctx": ctx, "shared": shared}
    for pb in (4, 8, 16, 32):
        ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev, pb=pb)
        row[f"pb{pb}_us"] = round(timeit(lambda: ops.decode(q, lens, tables, kc, vc, 0.088, workspace=ws, out=o)), 1)
        row[f"pb{pb}_var_us"] = round(timeit(lambda: ops.decode(q, lens_var, tables, kc, vc, 0.088, workspace=ws, out=o)), 1)
    print(json.dumps(row), flush=True)
