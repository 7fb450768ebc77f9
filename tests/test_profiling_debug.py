"""Aux subsystems: the engine-step profiler hook and the bounds-checked
debug build of the kernel library."""
import json
import os
import subprocess
import sys

import pytest
import torch

from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
from financial_chatbot_llm_amd.utils.profiling import StepProfiler, marker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_step_profiler_writes_chrome_trace(tmp_path, monkeypatch):
    monkeypatch.setenv("PENNY_TORCH_PROFILE", str(tmp_path))
    monkeypatch.setenv("PENNY_TORCH_PROFILE_STEPS", "1:4")
    eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", num_kv_blocks=32, max_model_len=512,
                                 max_num_seqs=4, use_cuda_graph=False))
    assert eng.profiler.enabled and (eng.profiler.start, eng.profiler.stop) == (1, 4)
    eng.generate([list(range(5, 40))], SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    path = tmp_path / "engine_rank0.json"
    assert path.exists() and eng.profiler.trace_path == str(path)
    events = json.loads(path.read_text())["traceEvents"]
    assert any("aten::" in str(e.get("name", "")) for e in events)


def test_profiler_off_by_default_and_marker_noop(monkeypatch):
    monkeypatch.delenv("PENNY_TORCH_PROFILE", raising=False)
    p = StepProfiler()
    assert not p.enabled
    p.on_step()
    assert p.finish() is None
    with marker("noop"):        # no GPU / markers off: a plain context
        pass
    with pytest.raises(ValueError):
        StepProfiler(out_dir="x", window="5:5")


def test_debug_kernel_library_builds_with_device_asserts():
    """The debug library compiles every kernel with PENNY_DASSERT live and exports the same
    launcher API as the production library."""
    from financial_chatbot_llm_amd import _build
    dbg = _build.build_kernels(jobs=min(8, os.cpu_count() or 1), debug=True)
    prod = _build.build_kernels(jobs=min(8, os.cpu_count() or 1))
    assert dbg.endswith("libpenny_kernels_debug.so") and os.path.exists(dbg)

    def exports(lib):
        out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
        return {l.split()[-1] for l in out.splitlines() if " T penny_" in l}

    assert exports(dbg) == exports(prod) and "penny_splitk_gemm" in exports(dbg)
    # the assert's message string is only in the debug code objects
    blob = open(dbg, "rb").read()
    assert b"device assert failed" in blob and b"device assert failed" not in open(prod, "rb").read()


@pytest.mark.gpu
def test_debug_kernel_library_runs_engine_on_gpu():
    """PENNY_KERNEL_DEBUG=1 loads the bounds-checked library (no assert fires on valid inputs)
    and greedy generation matches the production library."""
    code = (
        "import os, torch\n"
        "from financial_chatbot_llm_amd.config import EngineConfig\n"
        "from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams\n"
        "e = LLMEngine(EngineConfig(model='llama-tiny', device='cuda', num_kv_blocks=64, max_model_len=1024,"
        " max_num_seqs=4, graph_batch_sizes=(1, 2, 4)))\n"
        "out = e.generate([list(range(9, 90)), list(range(300, 333))],"
        " SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))\n"
        "maps = open(f'/proc/{os.getpid()}/maps').read()\n"
        "print('DBG' if 'libpenny_kernels_debug.so' in maps else 'PROD', out)\n")
    res = {}
    for mode in ("1", "0"):
        env = dict(os.environ, PENNY_KERNEL_DEBUG=mode, PYTHONPATH=ROOT)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[mode] = r.stdout.strip().splitlines()[-1]
    assert res["1"].startswith("DBG") and res["0"].startswith("PROD")
    assert res["1"][3:] == res["0"][4:]
