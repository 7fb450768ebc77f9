"""Request / sequence state for the continuous-batching engine."""
from __future__ import annotations

import contextvars
import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence as Seq


# Start of the user turn a request belongs to (time.perf_counter), set by the serving layer for
# everything the turn awaits (serving.worker): the scheduler orders prefill work by it, so a
# turn's respond prefill -- already a decide call deep into its TTFT -- is not queued behind the
# decide prefills of turns that arrived after it.
TURN_START: contextvars.ContextVar = contextvars.ContextVar("penny_turn_start", default=None)


@dataclass
class SamplingParams:
    temperature: float = 0.5            # reference: llm_agent.py:37,44
    top_k: int = 0                      # 0 = disabled
    top_p: float = 1.0
    max_tokens: int = 256
    ignore_eos: bool = False            # benchmarks force fixed decode lengths
    stop_token_ids: Seq[int] = ()
    seed: Optional[int] = None
    forced_output: Optional[List[int]] = None   # teacher-forced continuation (scripted tool calls)
    # jump-forward decoding (agent.grammar): forced_jump[k] -- output token k is forced by the
    # output grammar given tokens[:k], so it is appended with its predecessor instead of being
    # sampled; grammar -- the same oracle for sampled outputs (``forced(text) -> (str, ends)``)
    forced_jump: Optional[List[bool]] = None
    grammar: Optional[object] = None
    # KV retention hint: the prompt's uncached part will not recur (e.g. the respond prompt around
    # a one-off retrieval context), so its blocks are recycled before any other cached block
    ephemeral_kv: bool = False
    # prompt-lookup speculative decoding (engine.speculative): up to this many draft tokens copied
    # from the prompt are verified per step (0 = off)
    prompt_lookup: int = 0
    priority_ts: Optional[float] = None   # scheduling time (TURN_START); None: the request's arrival


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


_ids = itertools.count()


PENDING = -1   # placeholder token id (never fed to the model: gathered on the device instead)


class Sequence:
    def __init__(self, request_id: str, prompt_ids: List[int], params: SamplingParams, arrival: Optional[float] = None):
        self.seq_id = next(_ids)
        self.request_id = request_id
        self.prompt_ids = list(prompt_ids)
        self.output_ids: List[int] = []
        self.params = params
        self.status = SeqStatus.WAITING
        self.block_table: List[int] = []
        self.num_computed = 0          # tokens whose KV is in the cache
        self.num_cached_prompt = 0     # prefix-cache hit (tokens)
        self.num_prefilled = 0         # tokens run through prefill chunks (recomputes included)
        self.arrival = time.perf_counter() if arrival is None else arrival
        self.first_token_time: Optional[float] = None
        self.admit_time: Optional[float] = None   # first admitted into a step (scheduler clock)
        self.finish_reason: Optional[str] = None
        self.seed = params.seed if params.seed is not None else (hash((request_id, self.seq_id)) & 0x7FFFFFFF)
        self.num_preemptions = 0
        # overlap scheduling (LLMEngine, async_scheduling): while step N runs, the sequence carries
        # a placeholder for N's sampled token (output_ids[-1] == PENDING); pending_src is its row in
        # N's sampled vector, gathered on the device by step N+1.  awaiting: N's token certainly
        # ends the sequence (length / forced end), so it sits out N+1.
        self.pending_src = -1
        self.awaiting = False
        self.jump_queue: List[int] = []    # grammar-forced tokens staged for the next launch
        self.last_run: List[int] = []      # tokens appended at launch (emitted on resolve)
        self.jump_tail: List[int] = []     # final run of an awaiting sequence
        # prompt-lookup speculation: spec_rows -- sampled positions at the tail of the next chunk
        # (draft + 1; 0 = an ordinary row); spec_reject -- draft tokens already known to be rejected
        # at launch (teacher-forced output) and dropped once the chunk is launched
        self.spec_rows = 0
        self.spec_reject = 0
        self.spec_lookup = None
        self.spec_proposed = 0
        self.spec_accepted = 0

    def drop_draft(self) -> None:
        """Forget a prompt-lookup draft that was appended but never launched (preemption)."""
        m = self.spec_rows - 1
        if m > 0:
            accepted = m - self.spec_reject
            del self.output_ids[len(self.output_ids) - m:]
            if self.last_run and accepted:
                self.last_run = self.last_run[:len(self.last_run) - accepted]
        self.spec_rows = 0
        self.spec_reject = 0

    @property
    def priority_time(self) -> float:
        return self.arrival if self.params.priority_ts is None else self.params.priority_ts

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    def __len__(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def num_tokens(self) -> int:
        return len(self)

    @property
    def in_prefill(self) -> bool:
        return self.num_computed < self.num_tokens - 1 or (self.num_computed == 0)

    @property
    def remaining_prefill(self) -> int:
        return self.num_tokens - self.num_computed

    @property
    def finished(self) -> bool:
        return self.status == SeqStatus.FINISHED

    def step_seed(self) -> int:
        """Per-token seed: depends only on the request and the position (batch-invariant)."""
        return self.step_seed_at(len(self.output_ids))

    def step_seed_at(self, k: int) -> int:
        """Seed of the sample that becomes output token k."""
        return (self.seed * 0x9E3779B1 + k * 0x85EBCA77 + 1) & 0x7FFFFFFFFFFFFFFF
