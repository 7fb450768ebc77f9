"""The torchrun serving launcher: a TP=2 group (gloo, CPU) serves one Kafka turn end to end."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_launch_tp2_smoke():
    from test_tp_gloo import _free_port
    env = dict(os.environ, LOG_LEVEL="WARNING", PENNY_MAX_RESPONSE_TOKENS="8")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
           "financial_chatbot_llm_amd.serving.launch", "--tp", "2", "--model", "llama-tiny-tp", "--smoke",
           "--device", "cpu", "--max-model-len", "2048"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "smoke turn complete: type=complete error=False" in r.stdout


@pytest.mark.timeout(600)
def test_launch_cp2_smoke_prefills_context_parallel():
    """--cp 2: one context-parallel replica (gloo, CPU); with PENNY_CP_MIN_TOKENS low the smoke
    turn's prompts are prefilled by both ranks, the leader decodes and streams the reply."""
    from test_tp_gloo import _free_port
    env = dict(os.environ, LOG_LEVEL="INFO", PENNY_MAX_RESPONSE_TOKENS="8", PENNY_CP_MIN_TOKENS="128")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
           "financial_chatbot_llm_amd.serving.launch", "--cp", "2", "--model", "llama-tiny", "--smoke",
           "--device", "cpu", "--max-model-len", "2048"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "smoke turn complete: type=complete error=False" in r.stdout
    assert "context-parallel prefill of" in r.stdout + r.stderr
