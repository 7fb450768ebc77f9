"""Prefill-token accounting of the RAG workload without a GPU (VERDICT r1 "account for every
prefill token").

Drives the REAL agent + prompt assembly + tokenizer + worker + Mongo/Kafka fakes of
``bench/workload.py``, but replaces the engine by :class:`AuditEngine`, which runs the engine's
own block manager (prefix caching, 64-token blocks) and generates random token ids for the
respond stream (what random-init weights sample).  For every LLM call it records the prompt
length and how many prompt tokens the prefix cache served, so the per-turn computed-token count
can be compared with the structural minimum:

* ``minimum``: an infinite-capacity cache (every block ever computed stays resident).
* ``pool=N``: the same replay with an N-block pool and the engine's eviction policy.

    python -m financial_chatbot_llm_amd.bench.prefix_audit --convs 128 --turns 25 --pool 12000
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import statistics
from dataclasses import dataclass
from typing import Dict, List, Optional

from ..engine.block_manager import make_block_manager
from ..engine.sequence import SamplingParams, Sequence
from ..engine.tokenizer import SyntheticLlamaTokenizer
from ..retrieval.store import Hit, synthetic_payload


@dataclass
class _Out:
    request_id: str
    new_token_ids: List[int]
    finished: bool
    finish_reason: Optional[str]
    seq: Sequence


class AuditEngine:
    """Engine stand-in: prefix-cache bookkeeping only (no model).  Each request is admitted,
    'computed' and finished atomically, which is what a GPU step sequence does to the block
    manager when requests do not overlap in time; overlap is modelled by ``hold`` (requests keep
    their blocks until ``hold`` later requests finished)."""

    def __init__(self, num_blocks: int, seed: int = 0, hold: int = 0, policy: str = "lru", hints: bool = True):
        self.tokenizer = SyntheticLlamaTokenizer()
        self.bm = make_block_manager(num_blocks, 64, True, prefer_native=False)
        if hasattr(self.bm, "set_policy"):
            self.bm.set_policy(policy)
        self.rng = random.Random(seed)
        self.calls: List[Dict] = []
        self.hold = hold
        self.hints = hints          # honour the agent's ephemeral_kv retention hint
        self._held: List[Sequence] = []

    def _run(self, prompt_ids, params: SamplingParams, purpose: str, conv: str = "") -> Sequence:
        seq = Sequence(f"a{len(self.calls)}", list(prompt_ids), params)
        cached = self.bm.match_prefix(seq)
        if not self.bm.grow(seq, seq.num_tokens):
            self._release_all()
            if not self.bm.grow(seq, seq.num_tokens):
                raise MemoryError("pool too small for one prompt")
        seq.num_computed = seq.num_tokens
        self.bm.commit(seq)
        n = params.max_tokens
        forced = params.forced_output
        for k in range(n):
            if forced is not None and k < len(forced):
                tok = forced[k]
            else:
                tok = self.rng.randrange(0, 128256)
            seq.output_ids.append(tok)
            if forced is not None and k + 1 >= len(forced) and not params.ignore_eos:
                break
        seq.num_computed = seq.num_tokens - 1
        self.bm.grow(seq, seq.num_tokens)
        self.bm.commit(seq)
        self.calls.append({"purpose": purpose, "prompt": len(prompt_ids), "cached": cached,
                           "computed": len(prompt_ids) - cached, "out": len(seq.output_ids)})
        self._held.append(seq)
        while len(self._held) > self.hold:
            done = self._held.pop(0)
            self.bm.free(done, evict_first=self.hints and done.params.ephemeral_kv)
        return seq

    def _release_all(self):
        while self._held:
            done = self._held.pop(0)
            self.bm.free(done, evict_first=self.hints and done.params.ephemeral_kv)

    async def generate_all(self, prompt_ids, params):
        seq = self._run(prompt_ids, params, "decide")
        return _Out(seq.request_id, seq.output_ids[-1:], True, "stop", seq)

    async def generate(self, prompt_ids, params, request_id=None):
        seq = self._run(prompt_ids, params, "respond")
        for i, t in enumerate(seq.output_ids):
            yield _Out(seq.request_id, [t], i == len(seq.output_ids) - 1, None, seq)


class _FakeRetrieval:
    """Returns ``limit`` synthetic transactions of the user (same text format as the bench)."""

    def __init__(self, seed: int = 0):
        self.rng = random.Random(seed)

    async def search(self, query, user_id, date_gte, limit):
        base = self.rng.randrange(1 << 30)
        return [Hit(base + i, 1.0 - i * 1e-3, synthetic_payload(base + i, user_id, 1_700_000_000 + i * 3600))
                for i in range(min(limit, 10000))]

    def search_sync(self, query, user_id, date_gte, limit):
        return asyncio.get_event_loop().run_until_complete(self.search(query, user_id, date_gte, limit))


async def _replay(convs: int, turns: int, num_blocks: int, respond_tokens: int, hold: int, policy: str,
                  warmup: int, hints: bool = True, tool_steps: int = 1):
    from ..engine.backend import EngineLLM
    from .workload import RagWorkload, decide_script

    eng = AuditEngine(num_blocks, hold=hold, policy=policy, hints=hints)
    llm = EngineLLM(eng, max_model_len=8192, decide_script=decide_script, respond_ignore_eos=True,
                    respond_tokens=respond_tokens)
    wl = RagWorkload(llm, _FakeRetrieval(), convs, 10_000, respond_tokens, max_tool_steps=tool_steps)
    wl.kafka.setup_consumer()
    consumer = asyncio.create_task(wl.worker.consume_messages())
    per_turn: List[Dict] = []
    for t in range(turns):
        c0 = len(eng.calls)
        await wl.run_wave()
        calls = eng.calls[c0:]
        per_turn.append({
            "turn": t, "calls": len(calls),
            "prompt": sum(c["prompt"] for c in calls) / convs,
            "computed": sum(c["computed"] for c in calls) / convs,
            "decide_computed": sum(c["computed"] for c in calls if c["purpose"] == "decide") / convs,
            "respond_computed": sum(c["computed"] for c in calls if c["purpose"] == "respond") / convs,
            "decide_prompt": sum(c["prompt"] for c in calls if c["purpose"] == "decide") / convs,
            "respond_prompt": sum(c["prompt"] for c in calls if c["purpose"] == "respond") / convs,
        })
    wl.worker.stop()
    await consumer
    timed = per_turn[warmup:]
    summary = {k: round(statistics.mean(p[k] for p in timed), 1)
               for k in ("prompt", "computed", "decide_computed", "respond_computed", "decide_prompt",
                         "respond_prompt")}
    return summary, per_turn


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--convs", type=int, default=32)
    ap.add_argument("--turns", type=int, default=25)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--respond-tokens", type=int, default=128)
    ap.add_argument("--pool", type=int, default=0, help="KV blocks (0 = infinite: structural minimum)")
    ap.add_argument("--hold", type=int, default=0, help="requests in flight (blocks pinned)")
    ap.add_argument("--policy", default="lru")
    ap.add_argument("--no-hints", action="store_true", help="ignore the agent's ephemeral_kv hint (plain LRU)")
    ap.add_argument("--tool-steps", type=int, default=1, help="agent tool-call rounds per turn (config 4: 3)")
    ap.add_argument("--per-turn", action="store_true")
    a = ap.parse_args(argv)
    pool = a.pool or 10_000_000
    summary, per_turn = asyncio.run(_replay(a.convs, a.turns, pool, a.respond_tokens, a.hold, a.policy, a.warmup,
                                        not a.no_hints, a.tool_steps))
    print(json.dumps({"convs": a.convs, "turns": a.turns, "warmup": a.warmup, "pool_blocks": a.pool or "inf",
                      "policy": a.policy, "hold": a.hold, "hints": not a.no_hints, "tool_steps": a.tool_steps,
                      "per_turn_timed_mean": summary}))
    if a.per_turn:
        for p in per_turn:
            print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in p.items()}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
