"""Effective shader clock of the tile GEMM vs how many CUs it occupies: the O-projection shape
(N = K = 4096) at M = 512 .. 4096 (32 .. 256 tiles of 256x256), 20 calls each, whole tiles only
(PENNY_GEMM_TAIL=0).  Run under `rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace`:
GRBM_GUI_ACTIVE / kernel duration = average GPU clock while the kernel runs."""
import os
import sys

os.environ["PENNY_GEMM_TAIL"] = "0"
import torch  # noqa: E402

from financial_chatbot_llm_amd.ops import gemm  # noqa: E402


def main() -> int:
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn((4096, 4096), generator=g, device=dev) * 0.05).to(torch.bfloat16)
    for M in (512, 1024, 2048, 3072, 4096):
        x = (torch.randn((M, 4096), generator=g, device=dev) * 0.5).to(torch.bfloat16)
        for _ in range(20):
            gemm.prefill_gemm(x, w, None)
        torch.cuda.synchronize()
        print(M, "done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
