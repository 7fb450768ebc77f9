"""Static checks of hand-scheduled kernel code in the generated gfx950 assembly.

(r5: the weight-in-VGPR decode GEMM this file first checked was removed -- measured at parity with
the LDS-ring kernel, profiles/r4_decode_vw_vs_ldsring_rejected.jsonl.)  Its notes on why such
checks exist:

Its W fragments are loaded by inline-asm ``global_load_dwordx4`` that hipcc's waitcnt pass does
not track (the kernel's own counted ``s_waitcnt vmcnt`` covers them).  That is only sound if, in
the generated code, no instruction other than an MFMA operand read touches a W destination
register between its load and its consuming MFMA (or the final ``vmcnt(0)``): a register copy,
an AGPR spill or a reuse by the epilogue would read or clobber a value still in flight.  This
test compiles the file for gfx950 and walks every instantiation's assembly in program order.
Also checked: no compiler-inserted ``vmcnt(0)`` inside the main loop (which would serialise the
ring), and no scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

GEMM_SRC = os.path.join(os.path.dirname(__file__), "..", "financial_chatbot_llm_amd", "csrc", "kernels",
                        "gemm_prefill.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.timeout(300)
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_tile_gemm_mfmas_stay_in_their_phases(tmp_path):
    """gemm_prefill.hip's ping-pong needs each phase's MFMAs between its two barriers (16 bf16 or
    8 fp8 block-scaled MFMAs per phase): hipcc once sank every fp8 MFMA of a K-tile into the last
    phase (1 + 31), which serialised the partner waves and made the balanced schedule spill."""
    asm = tmp_path / "gp.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    GEMM_SRC, "-o", str(asm)], check=True, capture_output=True)
    s = asm.read_text()
    names = re.findall(r"^(_ZN12_GLOBAL__N_119gemm_prefill_kernel\w+):", s, re.M)
    assert any("Lb1E" in n for n in names) and any("Lb0E" in n for n in names)
    for name in names:
        i = s.index(name + ":")
        body = [ln.strip() for ln in s[i:s.index(".Lfunc_end", i)].splitlines()]
        fp8 = bool(re.search(r"gemm_prefill_kernelILi\d+ELi\d+ELi\d+ELb1E", name))
        counts, m = [], 0
        for ln in body:
            if ln.startswith("s_barrier"):
                counts.append(m)
                m = 0
            elif ln.startswith("v_mfma"):
                m += 1
        per_phase = 8 if fp8 else 16
        assert set(counts) <= {0, per_phase}, (name, counts[:30])
        assert counts.count(per_phase) >= 4, (name, counts[:30])
        diagnostic = re.search(r"gemm_prefill_kernelILi\d+ELi[123]E", name)   # ablation builds
        if not diagnostic and "ILi9E" not in name:
            # no spill traffic inside the K loop (first to last MFMA); a dword folded around the
            # prologue's tile / stream-K segment arithmetic is harmless
            mf = [k for k, ln in enumerate(body) if ln.startswith("v_mfma")]
            assert not any(ln.startswith("scratch_") for ln in body[mf[0]:mf[-1] + 1]), name
