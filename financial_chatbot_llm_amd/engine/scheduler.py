"""Continuous-batching scheduler with chunked prefill, prefix caching and preemption.

Every step builds ONE flat batch: a decode token for every running sequence that has finished
its prompt, plus prefill chunks (new or continuing prompts) filling the rest of the token
budget.  The reference processes one chat turn per worker process at a time (``main.py:138``);
here every in-flight turn of every conversation shares each forward pass.

Memory: a sequence holds KV blocks for exactly its computed tokens (+ the step's new tokens).
When the pool runs dry the youngest running sequence is preempted (blocks freed, re-queued at
the front, recomputed later -- its full blocks usually come back from the prefix cache).

Admission order (TTFT): preempted sequences first, then SHORT-OUTPUT requests -- the agent's
decide call (``max_tokens <= short_output_tokens``: a tool call or "No tool call") gates the whole
turn's TTFT and its prompt is mostly prefix-cached, so it should not queue behind long respond
prefills -- then everything else, each class FCFS.  Aging keeps it starvation-free: a request
that has waited ``aging_s`` joins the first class.  Within a class the key is the request's
``priority_time``: the start of the user turn it serves when the serving layer provides one
(``sequence.TURN_START``), so the respond prefill of an older turn goes before the decide
prefills of newer turns -- the oldest TTFT clock first.

Step-time bound (``StepCostModel``, off unless ``step_time_target_ms`` > 0): every token of a
decide call costs one engine step, so its latency is (tokens) x (step time) -- and a mixed step
carrying a full prefill chunk takes ~3.5x a decode-only one.  While a short-output sequence is
DECODING, the step's prefill tokens are capped so that the modelled step time stays under the
target; prefill still gets at least ``min_prefill_tokens`` per step (never starved), and the cap
lifts as soon as no decide call is decoding.
"""
from __future__ import annotations

import os
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Tuple

from ..utils.logging import get_logger
from .sequence import Sequence, SeqStatus

logger = get_logger(__name__)


@dataclass
class ScheduledBatch:
    prefill: List[Tuple[Sequence, int, int]] = field(default_factory=list)  # (seq, start, n_tokens)
    decode: List[Sequence] = field(default_factory=list)
    preempted: List[Sequence] = field(default_factory=list)

    @property
    def num_prefill_tokens(self) -> int:
        return sum(n for _, _, n in self.prefill)

    @property
    def num_tokens(self) -> int:
        return self.num_prefill_tokens + len(self.decode)

    def empty(self) -> bool:
        return not self.prefill and not self.decode


@dataclass
class StepCostModel:
    """Modelled device time of one step (ms) = base + per_row * decode rows + per_token * prefill
    tokens (defaults: Llama-3-8B on MI355X at the driver config -- decode-only steps of ~128 rows
    ~12 ms, mixed steps ~44 ms at ~2.4k prefill tokens, profiles/r2_bench128_20x5_step_gpu_timing.txt)."""
    target_ms: float = 0.0
    base_ms: float = 3.0
    per_row_ms: float = 0.07
    per_token_ms: float = 0.013
    min_prefill_tokens: int = 256

    def prefill_cap(self, decode_rows: int) -> int:
        room = self.target_ms - self.base_ms - self.per_row_ms * decode_rows
        return max(self.min_prefill_tokens, int(room / self.per_token_ms))


# step-row quantisation may cut any chunk (not only the last one) to reach a multiple of the quantum;
# PENNY_QUANTISE_ANY=0 restores the last-chunk-only form.  Driver bench A/B, two runs each on one box:
# 33.23 / 33.58 vs 33.26 / 33.45 turns/s (neutral; profiles/r5_bench128_20x5_quantise_any*_run*.json)
QUANTISE_ANY = os.environ.get("PENNY_QUANTISE_ANY", "1") != "0"


class Scheduler:
    def __init__(self, block_manager, max_num_seqs: int = 256, max_num_batched_tokens: int = 8192,
                 max_model_len: int = 8192, decode_first: bool = True, short_output_tokens: int = 160,
                 aging_s: float = 1.0, clock=time.perf_counter, token_quantum: int = 0,
                 cost_model: "StepCostModel" = None, burst_tokens: int = 0, burst_age_s: float = 0.5,
                 sjf_tokens: int = 0, sjf_step_cap: int = 0, short_reserve_tokens: int = 0,
                 short_first: bool = False):
        self.bm = block_manager
        self.max_num_seqs = max_num_seqs
        self.max_num_batched_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: Deque[Sequence] = deque()
        self.running: List[Sequence] = []
        self.num_preemptions = 0
        self.short_output_tokens = short_output_tokens
        self.aging_s = aging_s
        self.clock = clock
        self.token_quantum = token_quantum
        self.cost = cost_model if cost_model is not None else StepCostModel()
        self.num_capped_steps = 0
        # burst drain (TTFT tail): when the oldest pending prefill's turn has waited burst_age_s, the
        # step takes up to burst_tokens prefill tokens instead of max_num_batched_tokens (0 = off)
        self.burst_tokens = burst_tokens
        self.burst_age_s = burst_age_s
        self.num_burst_steps = 0
        # short-job-first admission (TTFT tail): a waiting request whose uncached prompt is at most
        # sjf_tokens is admitted ahead of the continuing chunks of long prefills (0 = off)
        self.sjf_tokens = sjf_tokens
        self.sjf_step_cap = sjf_step_cap      # at most this many tokens of a step go to 2a (0: budget)
        self.num_sjf_admits = 0
        # per-step reservation for the short-output class (TTFT tail): while decide-class prompts
        # wait, the continuing prefills of long prompts may take at most budget - reserve tokens of
        # a step, so a burst of long respond prefills delays a decide call by at most one step
        # instead of by the whole burst; the long prefills keep >= budget - reserve per step
        # (starvation-free) and the reserve is only held while short prompts actually wait
        self.short_reserve_tokens = short_reserve_tokens
        self.num_reserved_steps = 0
        # short_first: aged long-output prompts keep priority over fresh long ones but no longer
        # over short-output (decide-class) prompts, which are bounded in size (admission classes
        # 0 preempted, 1 short, 2 aged long, 3 rest; off: short and aged share class 1)
        # The reservation is only meaningful with short_first: otherwise aged long-output prompts
        # share class 1 with the short ones and, sorted by arrival, could spend the reserved tokens
        #  -- so a reserve turns short_first on.
        self.short_first = short_first or short_reserve_tokens > 0
        if short_reserve_tokens > 0 and not short_first:
            logger.warning(f"short_reserve_tokens={short_reserve_tokens} turns sched_short_first on (the reserve "
                           "needs short-output prompts in their own admission class)")
        # TTFT-tail anatomy: steps that ended with a short-output prompt still waiting, by what
        # stopped admission ("budget" / "grow" / "seqs" / "pending") and where those steps'
        # tokens went (decode rows, speculative chunks, continuing prefills, admitted prompts)
        self.short_wait: Dict[str, int] = {k: 0 for k in (
            "steps", "budget", "grow", "seqs", "pending", "tok_decode", "tok_spec", "tok_cont",
            "tok_admit_short", "tok_admit_long", "waiting_short", "waiting_short_tokens")}

    def _priority(self, seq: Sequence, now: float):
        if seq.num_preemptions:
            cls = 0
        elif seq.params.max_tokens <= self.short_output_tokens:
            cls = 1
        elif now - seq.arrival >= self.aging_s:
            cls = 2 if self.short_first else 1
        else:
            cls = 3
        return (cls, seq.priority_time)

    def add(self, seq: Sequence) -> None:
        if seq.num_tokens >= self.max_model_len:
            raise ValueError(f"prompt of {seq.num_tokens} tokens exceeds max_model_len {self.max_model_len}")
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def abort(self, seq: Sequence) -> None:
        if seq in self.running:
            self.running.remove(seq)
            self.bm.free(seq)
        elif seq in self.waiting:
            self.waiting.remove(seq)
            if seq.block_table:
                self.bm.free(seq)
        seq.status = SeqStatus.FINISHED

    def _preempt(self, seq: Sequence, batch: ScheduledBatch) -> None:
        if seq.spec_rows and not seq.awaiting:
            seq.drop_draft()                # not launched: recomputed later without it
        self.running.remove(seq)
        self.bm.free(seq)
        seq.num_computed = 0
        seq.status = SeqStatus.WAITING
        seq.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(seq)
        batch.preempted.append(seq)

    def _burst(self) -> bool:
        if self.burst_tokens <= self.max_num_batched_tokens:
            return False
        now = self.clock()
        oldest = min((s.priority_time for s in self.waiting), default=None)
        cont = [s.priority_time for s in self.running if s.remaining_prefill > 1 and not s.spec_rows]
        if cont:
            oldest = min(cont) if oldest is None else min(oldest, min(cont))
        return oldest is not None and now - oldest >= self.burst_age_s

    def schedule(self) -> ScheduledBatch:
        batch = ScheduledBatch()
        budget = self.max_num_batched_tokens
        if self._burst():
            budget = self.burst_tokens
            self.num_burst_steps += 1
        # 1) decodes (oldest first); preempt youngest when blocks run out
        decodes = [s for s in self.running if s.remaining_prefill == 1 and not s.awaiting]
        for seq in sorted(decodes, key=lambda s: s.arrival):
            if seq not in self.running:
                continue
            while not self.bm.can_grow(seq, seq.num_tokens):
                victim = max(self.running, key=lambda s: s.arrival)
                self._preempt(victim, batch)
                if victim is seq:
                    break
            if seq not in self.running:
                continue
            self.bm.grow(seq, seq.num_tokens)
            batch.decode.append(seq)
            budget -= 1
        tok_spec = 0
        # 1b) speculative chunks (last token + prompt-lookup draft, engine.speculative): decode-class
        # rows, scheduled whole -- every draft position must be sampled in the same step
        for seq in sorted((s for s in self.running if s.spec_rows and not s.awaiting
                           and s.remaining_prefill >= s.spec_rows), key=lambda s: s.arrival):
            n = seq.remaining_prefill
            if n > max(budget, 0) or not self.bm.grow(seq, seq.num_tokens):
                # no room for the chunk: forget the draft, so the sequence is an ordinary row
                # again (a 1-token decode, or the rest of a forced run) and next step's decode
                # pass -- which preempts when the pool is dry -- schedules it
                seq.drop_draft()
                continue
            batch.prefill.append((seq, seq.num_computed, n))
            budget -= n
            tok_spec += n
        # step-time bound: a decide call is decoding -> keep this step short (its next token waits
        # for it); the cap never drops below min_prefill_tokens, so prefill always progresses
        if self.cost.target_ms > 0 and any(s.params.max_tokens <= self.short_output_tokens for s in batch.decode):
            cap = self.cost.prefill_cap(len(batch.decode))
            if cap < budget:
                budget = cap
                self.num_capped_steps += 1
        # 2a) short-job-first: short uncached prompts (an agent decide call: ~200 new tokens behind a
        # cached few-shot prefix) go before the continuing chunks of long prefills
        if self.sjf_tokens > 0 and self.waiting and budget > 0:
            budget = self._admit_short(batch, budget)
        # reservation: short-output prompts waiting for admission hold back up to
        # short_reserve_tokens of this step from the continuing long prefills (pass 2); pass 3
        # admits them first (class order) with whatever is left plus the reserve
        reserve = 0
        if self.short_reserve_tokens > 0 and self.waiting and budget > 0:
            need = sum(q.remaining_prefill for q in self.waiting
                       if q.params.max_tokens <= self.short_output_tokens and q.pending_src < 0 and not q.awaiting)
            reserve = min(self.short_reserve_tokens, need, budget)
            if reserve > 0:
                self.num_reserved_steps += 1
        budget -= reserve
        # 2) continuing prefills (not the sequences 2a just admitted: their computed count moves only
        # when this step resolves)
        taken = {id(q) for q, _, _ in batch.prefill}
        tok_cont = 0
        for seq in sorted((s for s in self.running if s.remaining_prefill > 1 and not s.awaiting
                           and not s.spec_rows and id(s) not in taken), key=lambda s: s.priority_time):
            if budget <= 0:
                break
            n = min(seq.remaining_prefill, budget)
            if not self.bm.grow(seq, seq.num_computed + n):
                continue
            batch.prefill.append((seq, seq.num_computed, n))
            seq.num_prefilled += n
            budget -= n
            tok_cont += n
        budget += reserve
        # 3) admit waiting sequences, by priority class (preempted, short-output/aged, rest)
        if len(self.waiting) > 1:
            now = self.clock()
            self.waiting = deque(sorted(self.waiting, key=lambda q: self._priority(q, now)))
        stop, tok_admit = "", [0, 0]
        while True:
            if not self.waiting:
                break
            if budget <= 0:
                stop = "budget"
                break
            if len(self.running) >= self.max_num_seqs:
                stop = "seqs"
                break
            seq = self.waiting[0]
            if seq.pending_src >= 0 or seq.awaiting:
                stop = "pending"
                break   # preempted with an in-flight token: re-admit once it is known
            if not seq.block_table:
                self.bm.match_prefix(seq)
            n = min(seq.remaining_prefill, budget)
            if not self.bm.grow(seq, seq.num_computed + n):
                if seq.block_table and not self.running:
                    raise MemoryError("KV pool too small for a single prompt")
                stop = "grow"
                break
            self.waiting.popleft()
            tok_admit[seq.params.max_tokens > self.short_output_tokens] += n
            if seq.admit_time is None:
                seq.admit_time = self.clock()
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            batch.prefill.append((seq, seq.num_computed, n))
            seq.num_prefilled += n
            budget -= n
        short = [q for q in self.waiting if q.params.max_tokens <= self.short_output_tokens]
        if short:
            sw = self.short_wait
            sw["steps"] += 1
            sw[stop] += 1
            sw["tok_decode"] += len(batch.decode)
            sw["tok_spec"] += tok_spec
            sw["tok_cont"] += tok_cont
            sw["tok_admit_short"] += tok_admit[0]
            sw["tok_admit_long"] += tok_admit[1]
            sw["waiting_short"] += len(short)
            sw["waiting_short_tokens"] += sum(q.remaining_prefill for q in short)
        self._quantise(batch)
        return batch

    def _admit_short(self, batch: ScheduledBatch, budget: int) -> int:
        now = self.clock()
        cap = self.sjf_step_cap if self.sjf_step_cap > 0 else budget
        for seq in sorted(self.waiting, key=lambda q: self._priority(q, now)):
            if budget <= 0 or len(self.running) >= self.max_num_seqs:
                break
            if seq.pending_src >= 0 or seq.awaiting or seq.num_preemptions:
                continue
            if not seq.block_table:
                self.bm.match_prefix(seq)
            n = seq.remaining_prefill
            if n > self.sjf_tokens or n > budget or n > cap:
                continue
            if not self.bm.grow(seq, seq.num_computed + n):
                break
            self.waiting.remove(seq)
            if seq.admit_time is None:
                seq.admit_time = now
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            batch.prefill.append((seq, seq.num_computed, n))
            seq.num_prefilled += n
            budget -= n
            cap -= n
            self.num_sjf_admits += 1
        return budget

    def _quantise(self, batch: ScheduledBatch) -> None:
        """Round the step's row count DOWN to a multiple of ``token_quantum`` by shortening prefill
        chunks (those tokens run next step; nothing is padded).  The prefill GEMMs' M is the step's row
        count: the tile kernel's last 256-row tile runs whole however few rows it holds, and
        hipBLASLt's speed swings with M between neighbouring values (1139 vs 1417 TF/s at M = 2816 /
        2560 on the default heuristic; profiles/r2_gemm_prefill_tunableop_sweep.jsonl).  The cut comes
        from chunks that do not finish their prompt first, long-output ones before short-output ones,
        the most recently added first; speculative chunks are never cut, and a step that cannot reach
        a multiple stays as it is."""
        q = self.token_quantum
        if q <= 0 or not batch.prefill:
            return
        total = batch.num_tokens
        r = total % q
        if total <= q or r == 0:
            return

        def rank(i: int):
            seq, start, n = batch.prefill[i]
            final = start + n >= seq.num_tokens
            short = seq.params.max_tokens <= self.short_output_tokens
            return (final, short, -i)
        order = [i for i in sorted(range(len(batch.prefill)), key=rank)
                 if not batch.prefill[i][0].spec_rows and batch.prefill[i][2] > 1]
        if not QUANTISE_ANY:        # r2 form (A/B): the last chunk only
            order = [len(batch.prefill) - 1] if (len(batch.prefill) - 1) in order else []
        # one chunk that can take the whole cut, else the cut spread over several
        one = next((i for i in order if batch.prefill[i][2] > r), None)
        cuts, left = ({one: r}, 0) if one is not None else ({}, r)
        for i in order if one is None else ():
            c = min(left, batch.prefill[i][2] - 1)
            cuts[i] = c
            left -= c
            if left == 0:
                break
        if left:
            return
        for i, c in cuts.items():
            seq, start, n = batch.prefill[i]
            batch.prefill[i] = (seq, start, n - c)
            seq.num_prefilled -= c

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        if seq in self.running:
            self.running.remove(seq)
        elif seq in self.waiting:          # preempted while its last token was in flight
            self.waiting.remove(seq)
        self.bm.free(seq, evict_first=seq.params.ephemeral_kv)
