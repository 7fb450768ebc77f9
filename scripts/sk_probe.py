"""Stream-K tail probe: the tile GEMM at the O / down projection shapes, 30 calls each, for a
rocprofv3 kernel trace (per-dispatch durations) -- run once per kernel library."""
import sys

import torch

from financial_chatbot_llm_amd.ops import gemm


def main() -> int:
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N_, K in ((512, 4096, 4096), (2048, 4096, 4096), (2560, 4096, 4096), (2304, 4096, 14336)):
        x = (torch.randn((M, K), generator=g, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn((N_, K), generator=g, device=dev) * 0.05).to(torch.bfloat16)
        for _ in range(30):
            gemm.prefill_gemm(x, w, None)
        torch.cuda.synchronize()
        print(M, N_, K, "done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
