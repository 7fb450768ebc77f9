"""A fixed decode-attention workload for rocprofv3 counter runs of the lean kernel's cache policy:
``PENNY_DECODE_LEAN_FLAGS=0`` (default policy) vs ``=1`` (non-temporal loads for the blocks only one
row reads, shared blocks marked by the host as in the engine).  One process per policy, so each
kernel template's counters stand alone:

    rocprofv3 --pmc FETCH_SIZE -d out -o run -- python3 -m financial_chatbot_llm_amd.bench.lean_nt_pmc --b 128

The batch matches bench/kernels.py decode_lean (ctx 1.5-6.5k, a 1k shared prefix at B = 64 / 128).
"""
from __future__ import annotations

import argparse
import json

import numpy as np
import torch

from .. import ops
from ..ops import attention as A

KV_BS = A.KV_BS


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=128)
    ap.add_argument("--shared", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    B, Hq, Hkv, D = args.b, 32, 8, 128
    rng = torch.Generator().manual_seed(B + 1500)
    ctxs = torch.randint(1500, 6500, (B,), generator=rng).tolist()
    nsh = args.shared // KV_BS
    W = max((c + KV_BS - 1) // KV_BS for c in ctxs)
    tables = torch.zeros((B, W), dtype=torch.int32)
    nxt = nsh
    for b, c in enumerate(ctxs):
        nb = (c + KV_BS - 1) // KV_BS
        tables[b, :nsh] = torch.arange(nsh, dtype=torch.int32)
        tables[b, nsh:nb] = torch.arange(nxt, nxt + nb - nsh, dtype=torch.int32)
        nxt += nb - nsh
    g = torch.Generator(device=dev).manual_seed(3)
    kc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
    vc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
    if A.LEAN_FLAGS & 1:
        tables = torch.from_numpy(A.mark_shared_blocks(tables.numpy().copy(), np.asarray(ctxs)))
    q = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
    lens = torch.tensor(ctxs, dtype=torch.int32, device=dev)
    ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev)
    o = torch.empty_like(q)
    bt = tables.to(dev)
    for _ in range(args.iters):
        ops.decode(q, lens, bt, kc, vc, 0.088, workspace=ws, out=o)
    torch.cuda.synchronize()
    uniq = (sum(ctxs) - (B - 1) * args.shared) * Hkv * D * 2 * 2
    print(json.dumps({"B": B, "flags": A.LEAN_FLAGS, "unique_kv_bytes": uniq, "iters": args.iters}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
