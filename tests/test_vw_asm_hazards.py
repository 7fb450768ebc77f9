"""Static check of the weight-in-VGPR decode GEMM (gemm_splitk.hip splitk_vw_kernel).

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

SRC = os.path.join(os.path.dirname(__file__), "..", "financial_chatbot_llm_amd", "csrc", "kernels", "gemm_splitk.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _regs(txt):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", txt):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


@pytest.mark.timeout(300)
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_vw_kernel_untracked_loads_are_never_read_early(tmp_path):
    asm = tmp_path / "gsk.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    SRC, "-o", str(asm)], check=True, capture_output=True)
    s = asm.read_text()
    names = re.findall(r"^(_ZN12_GLOBAL__N_116splitk_vw_kernel\w+):", s, re.M)
    assert len(names) >= 12
    for name in names:
        i = s.index(name + ":")
        body = [ln.strip() for ln in s[i:s.index(".Lfunc_end", i)].splitlines()]
        pending, bad, loop_waits, in_loop = {}, [], [], False
        for k, ln in enumerate(body):
            if "Loop Header" in ln:
                in_loop = True
            if not ln or ln.startswith((";", ".")):
                continue
            op, rest = ln.split()[0], ln[len(ln.split()[0]):]
            if op == "s_waitcnt":
                if in_loop and "vmcnt(0)" in ln and "ASMSTART" not in body[k - 1]:
                    loop_waits.append(k)
                if "vmcnt(0)" in ln:
                    pending.clear()
                continue
            m = re.match(r"global_load_dwordx4 v\[(\d+):(\d+)\], v\[\d+:\d+\], off$", ln)
            if m:
                for r in range(int(m.group(1)), int(m.group(2)) + 1):
                    pending[r] = k
                continue
            if op.startswith("v_mfma"):
                parts = [p.strip() for p in rest.split(",")]
                for r in _regs(parts[1]) | _regs(parts[2]):
                    pending.pop(r, None)
                continue
            if op.startswith("s_cbranch") and "Loop" not in ln:
                pass
            if _regs(rest) & set(pending):
                bad.append((k, ln))
        assert not bad, (name, bad[:5])
        # the compiler may only drain vmcnt after the loop (the kernel's own final wait)
        assert len(loop_waits) == 0, (name, loop_waits[:5])


GEMM_SRC = os.path.join(os.path.dirname(SRC), "gemm_prefill.hip")


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
