"""Synchronous engine core: model + paged KV pool + scheduler + runner, stepped by the caller.

One :class:`LLMEngine` serves one TP group (a DP replica).  On TP>1 only the group leader runs
the scheduler; each step it broadcasts the packed :class:`StepInputs` (C4, one flat buffer over
a gloo twin of the TP group) and every rank runs the identical forward (``follower_loop`` on the
other ranks).  Decode-size TP all-reduces take the custom one-shot xGMI kernel by default
(``EngineConfig.custom_all_reduce``), RCCL the rest.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence as Seq, Tuple

import torch

from ..config import EngineConfig
from ..models import build_model
from ..models.common import KVCache
from ..ops.attention import KV_BS
from ..parallel import comm
from ..parallel.dist import state as pstate
from ..utils.logging import get_logger
from ..utils.metrics import METRICS
from ..utils.profiling import StepProfiler, marker
from .block_manager import make_block_manager
from .model_runner import CollectiveTimeout, ModelRunner, StepInputs, build_step_inputs, sample_rows
from .scheduler import Scheduler, StepCostModel
from .sequence import PENDING, SamplingParams, Sequence, SeqStatus
from .speculative import PromptLookup, accept_draft
from .tokenizer import BaseTokenizer, load_tokenizer

logger = get_logger(__name__)
MAX_DRAFT = 16          # draft tokens per speculative chunk (ModelRunner sizes its sampler rows for it)


@dataclass
class StepOutput:
    request_id: str
    new_token_ids: List[int]
    finished: bool
    finish_reason: Optional[str]
    seq: Sequence


def plan_kv_blocks(cfg: EngineConfig, model, device) -> int:
    if cfg.num_kv_blocks:
        return cfg.num_kv_blocks
    per_block = KVCache.bytes_per_block(model.cfg.num_layers, model.hkv, model.D)
    if device.type != "cuda":
        return max(64, (cfg.max_num_seqs * cfg.max_model_len // KV_BS) // 8)
    free, _ = torch.cuda.mem_get_info(device)
    reserve = 6 << 30  # activations, hipBLASLt workspaces, graph pools
    n = int(max(free - reserve, 0) * cfg.kv_mem_fraction) // per_block
    return max(n, 16)


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model=None, tokenizer: Optional[BaseTokenizer] = None):
        self.cfg = cfg
        device = torch.device(cfg.device if (cfg.device != "cuda" or torch.cuda.is_available()) else "cpu")
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        t0 = time.perf_counter()
        self.model = model if model is not None else build_model(cfg, device)
        if device.type == "cuda":
            from ..ops.gemm import load_gemm_tuning
            self.gemm_tuning = load_gemm_tuning(cfg.model, cfg.tp_size)
        self.tokenizer = tokenizer or load_tokenizer(cfg.tokenizer, self.model.cfg.vocab_size)
        self.eos_ids = set(self.tokenizer.eos_ids)
        nblocks = plan_kv_blocks(cfg, self.model, device)
        self.kv = KVCache(self.model.cfg.num_layers, nblocks, self.model.hkv, self.model.D,
                          dtype=getattr(self.model, "dtype", torch.bfloat16), device=device)
        self.bm = make_block_manager(nblocks, KV_BS, cfg.enable_prefix_caching)
        base, per_row, per_tok = cfg.step_cost_ms
        self.scheduler = Scheduler(self.bm, cfg.max_num_seqs, cfg.max_num_batched_tokens, cfg.max_model_len,
                                   token_quantum=cfg.step_token_quantum if device.type == "cuda" else 0,
                                   aging_s=cfg.sched_aging_s,
                                   cost_model=StepCostModel(cfg.step_time_target_ms, base, per_row, per_tok),
                                   burst_tokens=getattr(cfg, "sched_burst_tokens", 0),
                                   burst_age_s=getattr(cfg, "sched_burst_age_s", 0.5),
                                   sjf_tokens=getattr(cfg, "sched_sjf_tokens", 0),
                                   sjf_step_cap=getattr(cfg, "sched_sjf_step_cap", 0),
                                   short_reserve_tokens=getattr(cfg, "sched_short_reserve_tokens", 0),
                                   short_first=getattr(cfg, "sched_short_first", False))
        self.runner = ModelRunner(self.model, self.kv, cfg.max_model_len, max_decode_batch=cfg.max_num_seqs,
                                  use_graphs=cfg.use_cuda_graph, graph_sizes=cfg.graph_batch_sizes)
        self.requests: Dict[str, Sequence] = {}
        self.timing = {"prepare_s": 0.0, "execute_s": 0.0, "post_s": 0.0}   # host-side step anatomy
        self.spec_stats = {"proposed": 0, "accepted": 0}   # prompt-lookup draft tokens
        self.async_scheduling = bool(getattr(cfg, "async_scheduling", True))
        self._inflight = None      # (batch, samplers, PendingStep) of the step on the GPU
        self.ps = pstate()
        if self.ps.tp_size > 1 and device.type == "cuda" and getattr(cfg, "custom_all_reduce", True):
            try:   # collective over the TP group: every rank constructs its engine together
                comm.enable_custom_all_reduce()
                if getattr(cfg, "tp_dual_decode", False):
                    comm.enable_second_channel()     # the second decode micro-batch chain's AR
            except Exception as e:  # noqa: BLE001 - no IPC on this host: RCCL carries everything
                logger.warning(f"custom all-reduce unavailable ({e}); using RCCL for every TP all-reduce")
                comm.AR_STATUS.update(custom=False, self_test=f"unavailable: {e}")
            # every rank must hold the same custom instances before the self-test's collectives (an
            # enable that raised on some ranks only would send the group down different collective
            # sequences): agree on presence bits first, all ranks, raised or not
            comm.agree_custom_all_reduce(want_second=bool(getattr(cfg, "tp_dual_decode", False)))
            # first contact: the custom kernels must reproduce the exact sum on THIS node before any
            # token depends on them; any rank's failure sends every rank to RCCL
            if comm.custom_all_reduce() is not None and getattr(cfg, "custom_ar_self_test", True):
                comm.verify_custom_all_reduce()
        if self.ps.tp_size > 1 and getattr(cfg, "step_ring", True):
            comm.enable_step_channel()      # collective too; None -> gloo C4
        self.profiler = StepProfiler(rank=self.ps.rank)
        # context parallelism: long prompts prefilled by the whole CP replica (engine/context_prefill.py)
        self.cp = None
        if getattr(cfg, "cp_size", 1) > 1 and self.ps.cp_size > 1:
            from .context_prefill import ContextParallelPrefill
            self.cp = ContextParallelPrefill(self)
        logger.info(f"engine ready: model={self.model.cfg.name} tp={self.model.tp_size} kv_blocks={nblocks} "
                    f"({nblocks * KV_BS} tokens) weights={self.model.num_bytes() / 2**30:.1f} GiB "
                    f"init={time.perf_counter() - t0:.1f}s")

    # ------------------------------------------------------------------------------------
    def add_request(self, request_id: str, prompt_ids: Seq[int], params: SamplingParams) -> Sequence:
        if not prompt_ids:
            raise ValueError("empty prompt")
        max_prompt = self.cfg.max_model_len - 1
        seq = Sequence(request_id, list(prompt_ids)[-max_prompt:], params)
        self.requests[request_id] = seq
        if self.cp is not None and self.cp.wants(seq):
            self.cp.queue.append(seq)          # prefilled context-parallel before the next step
        else:
            self.scheduler.add(seq)
        return seq

    def abort(self, request_id: str) -> None:
        seq = self.requests.pop(request_id, None)
        if seq is not None and not seq.finished:
            self.scheduler.abort(seq)
            seq.finish_reason = "abort"

    def has_work(self) -> bool:
        return self.scheduler.has_work() or self._inflight is not None or bool(self.cp and self.cp.busy())

    def warmup(self) -> None:
        """Capture decode graphs (all TP ranks must call this together)."""
        if self.runner.use_graphs:
            self.runner.capture_graphs()

    def step(self) -> List[StepOutput]:
        """One engine iteration.  Overlap mode (``async_scheduling``): schedule + launch step N+1
        while step N is still on the GPU, then collect N -- the host's scheduling, input packing
        and token bookkeeping hide behind the device instead of idling it between steps."""
        self.profiler.on_step()
        if self.cp is not None and self.cp.busy():
            with marker("engine.cp_prefill"):
                self.cp.run_pending()      # one layer slice of a long prompt; the step follows
        with marker("engine.step"):
            try:
                return self._step_overlap() if self.async_scheduling else self._step_sync()
            except CollectiveTimeout as e:
                self._collective_failed(e)
                raise

    def _collective_failed(self, e: BaseException) -> None:
        """A step's TP all-reduce failed on the device (custom xGMI kernel: a peer missed the bounded
        wait; the kernels wrote NaN and set the error flag -- allreduce.hip).  Every request on the
        engine saw stale hidden states, so all are failed (the caller re-raises: AsyncEngine turns it
        into the reference's error event per waiting turn, main.py:112-122), and the whole TP group
        switches to RCCL at this step boundary: the leader sends the fallback control message over
        C4 before any further step, followers apply it in order (``follower_loop``)."""
        logger.error(f"TP collective failed ({e}); failing {len(self.requests)} request(s), falling back to RCCL")
        METRICS.inc("custom_ar_runtime_failures")
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)      # the in-flight step (its sums are NaN) drains
        self._inflight = None
        for seq in list(self.requests.values()):
            if not seq.finished:
                self.scheduler.abort(seq)
                seq.finish_reason = "error"
        self.requests.clear()
        if self.ps.tp_size > 1 and self.ps.is_tp_leader:
            comm.broadcast_step(StepInputs.control(StepInputs.CTRL_RCCL_FALLBACK))
        comm.fallback_to_rccl(str(e))
        self.runner.drop_graphs()

    # -- overlap (one-step lookahead) ------------------------------------------------------------
    def _samplers(self, batch) -> List[Sequence]:
        """Rows of a batch that sample a token, in sampled-vector order (a speculative chunk's
        sequence repeats once per verified position)."""
        rows: List[Sequence] = []
        for seq, start, n in batch.prefill:
            if start + n == seq.num_tokens:
                rows.extend([seq] * sample_rows(seq, n))
        return rows + list(batch.decode)

    @staticmethod
    def _group(samplers: List[Sequence], sampled: Optional[List[int]] = None):
        """(seq, first row, its sampled ids) per sequence of a sampler list."""
        out = []
        i = 0
        while i < len(samplers):
            j = i + 1
            while j < len(samplers) and samplers[j] is samplers[i]:
                j += 1
            out.append((samplers[i], i, sampled[i:j] if sampled is not None else None))
            i = j
        return out

    def _ends_after(self, seq: Sequence, tok: Optional[int], run: int = 1) -> bool:
        """Will the token(s) about to be appended certainly finish ``seq``?  ``tok``: the known
        last token of the run (None: sampled), ``run``: tokens appended at once (jump-forward)."""
        k = len(seq.output_ids) + run
        p = seq.params
        if k >= p.max_tokens or seq.num_tokens + run >= self.cfg.max_model_len:
            return True
        if p.forced_output is not None and k >= len(p.forced_output) and not p.ignore_eos:
            return True
        return tok is not None and not p.ignore_eos and (tok in self.eos_ids or tok in p.stop_token_ids)

    def _known_run(self, seq: Sequence) -> List[int]:
        """Tokens known at launch time for the sampler row of ``seq``: a teacher-forced token
        plus the grammar-forced tokens that follow it (jump-forward), or the grammar-forced run
        staged by the previous resolve.  Empty: the token must be sampled."""
        p = seq.params
        k = len(seq.output_ids)
        room = max(p.max_tokens - k, 1)   # never append past max_tokens
        if seq.jump_queue:
            run, seq.jump_queue = seq.jump_queue, []
            return run[:room]
        forced = p.forced_output
        if forced is None or k >= len(forced):
            return []
        run = [forced[k]]
        jump = p.forced_jump
        if jump is not None:
            j = k + 1
            while j < len(forced) and j < len(jump) and jump[j]:
                run.append(forced[j])
                j += 1
        return run[:room]

    def _stage_grammar(self, seq: Sequence) -> None:
        """After a SAMPLED token: stage the output grammar's forced continuation (if any).

        The forced text is tokenized TOGETHER with the output so far: BPE merges across the
        boundary (Llama-3: around '{"' or '": "') would otherwise give token ids the model would
        never have produced itself.  Only the tokens past the current output are appended, and
        only if the output is a token-prefix of that joint encoding; otherwise this token jumps
        nothing and the model continues sampling."""
        g = seq.params.grammar
        if g is None or seq.params.forced_output is not None:
            return
        text = self.tokenizer.decode(seq.output_ids)
        forced, ends = g.forced(text)
        run: List[int] = []
        if forced:
            joint = self.tokenizer.encode(text + forced, allow_special=False)
            n = len(seq.output_ids)
            if joint[:n] != list(seq.output_ids) or len(joint) <= n:
                seq.jump_queue = []
                return
            run = joint[n:]
        if ends and self.eos_ids:
            run.append(self.tokenizer.special.get("<|eot_id|>", next(iter(self.eos_ids))))
        seq.jump_queue = run

    # -- prompt-lookup speculation (engine.speculative) -------------------------------------------
    def _propose(self, seq: Sequence, after: Seq[int] = (), min_ngram: int = 0) -> List[int]:
        """Draft tokens to follow output + ``after``, capped so the chunk never reaches max_tokens,
        max_model_len or the teacher-forced output's last token; cut before any stop token (the
        model's own stop token then arrives as the bonus sample and ends the sequence as usual)."""
        p = seq.params
        if p.prompt_lookup <= 0 or seq.finished:
            return []
        k = len(seq.output_ids) + len(after)
        room = min(p.prompt_lookup, MAX_DRAFT, p.max_tokens - k - 1, self.cfg.max_model_len - seq.num_tokens - len(after) - 2)
        if p.forced_output is not None:
            room = min(room, len(p.forced_output) - k - 1)
        if room <= 0:
            return []
        if seq.spec_lookup is None:
            # recency 256: a 1-gram in the latest user turn beats a 2-gram in the few-shot
            # examples far above it (decide drafts: 47 -> 44 steps over the 5 spend questions)
            seq.spec_lookup = PromptLookup(seq.prompt_ids, recency=256)
        draft = seq.spec_lookup.propose(list(seq.output_ids) + list(after), room, min_ngram)
        if not p.ignore_eos:
            stops = self.eos_ids | set(p.stop_token_ids)
            for i, t in enumerate(draft):
                if t in stops:
                    draft = draft[:i]
                    break
        if draft and p.grammar is not None and p.forced_output is None:
            draft = self._grammar_cut(seq, list(after), draft)
        return draft

    def _grammar_cut(self, seq: Sequence, after: List[int], draft: List[int]) -> List[int]:
        """Longest draft prefix d[:k] such that the output grammar forces nothing after any of
        d[:1] .. d[:k]: one-token-per-step decoding would jump forward (override the sample) at
        the first such position, so the chunk's samples there -- an accepted draft token's
        successor or the bonus -- are not what it would emit.  With the cut, every sampled
        position of the chunk is one where the grammar is free, and ``_stage_grammar`` after the
        bonus resumes exactly as without speculation."""
        g = seq.params.grammar
        base = [t for t in seq.output_ids if t != PENDING] + after
        for k in range(len(draft)):
            forced, ends = g.forced(self.tokenizer.decode(base + draft[:k + 1]))
            if forced or ends:
                return draft[:k]
        return draft

    def _model_tokens(self, seq: Sequence, base: int, toks: Seq[int], m: int) -> List[int]:
        """The model's tokens at output positions base .. base+m-1: the teacher-forced ones, or
        the samples of the verified rows."""
        forced = seq.params.forced_output
        if forced is not None:
            return list(forced[base:base + m])
        return [int(t) for t in toks[:m]]

    def _verify(self, seq: Sequence, toks: Seq[int]) -> Tuple[List[int], int]:
        """Resolve a speculative chunk of ``seq`` (its draft is the output tail): drop the rejected
        draft tokens and clamp ``num_computed`` to the valid prefix.  Returns (accepted draft,
        bonus sample: the model's token after the accepted prefix)."""
        m = seq.spec_rows - 1
        base = len(seq.output_ids) - m
        draft = seq.output_ids[base:]
        j = accept_draft(draft, self._model_tokens(seq, base, toks, m))
        del seq.output_ids[base + j:]
        seq.spec_rows = 0
        seq.spec_proposed += m
        seq.spec_accepted += j
        self.spec_stats["proposed"] += m
        self.spec_stats["accepted"] += j
        seq.num_computed = min(seq.num_computed, seq.num_tokens)
        return draft[:j], int(toks[j])

    def _sit_out(self, seq: Sequence) -> bool:
        """Overlap mode, sampled output: skip the next step so the NEXT token is known at the
        following launch and a draft can ride with it -- only inside a copy span (the last 2+
        tokens occur earlier in the prompt), where a draft will likely be accepted."""
        if seq.params.prompt_lookup <= 0 or PENDING in seq.output_ids[-3:]:
            return False
        return bool(self._propose(seq, min_ngram=2))

    def _advance(self, batch, samplers: List[Sequence]) -> None:
        """Host view of an in-flight step as if it had completed: KV written (num_computed), full
        blocks committed, one placeholder token per sampler (device-gathered by the next step)
        -- or the known run of tokens (teacher-forced / grammar-forced), appended at once; a
        run longer than one token is computed as a prefill chunk by the next step.  A known run
        also carries a prompt-lookup draft: teacher-forced drafts are verified right here (the
        model's tokens are known), so only the accepted part is kept after the chunk launches."""
        for seq, start, n in batch.prefill:
            if not seq.finished:
                seq.num_computed = min(start + n, seq.num_tokens)
        for seq in batch.decode:
            if not seq.finished:
                seq.num_computed = seq.num_tokens
        for seq, i, _ in self._group(samplers):
            if seq.finished:
                continue
            if seq.spec_rows > 1:              # sampled draft in flight: verified on resolve
                # no commit here: num_computed counts the unverified draft, and a full block
                # holding draft positions must not enter the prefix cache under the draft's token
                # ids (a rejection rewrites that KV); _resolve commits after _verify
                seq.awaiting = True
                seq.jump_tail = []
                continue
            run = self._known_run(seq)
            tok = run[-1] if run else None
            if self._ends_after(seq, tok, max(len(run), 1)):
                seq.awaiting = True            # sits out the next step; resolved by _resolve
                seq.jump_tail = run
            elif run:
                # a draft rides with a teacher-forced run only: sampled runs (grammar jumps) leave
                # the model's tokens unknown at launch
                draft = self._propose(seq, run) if seq.params.forced_output is not None else []
                j = accept_draft(draft, self._model_tokens(seq, len(seq.output_ids) + len(run), (), len(draft)))
                seq.output_ids.extend(run + draft)
                seq.pending_src = -1
                seq.last_run = run + draft[:j]
                seq.spec_rows = len(draft) + 1 if draft else 0
                seq.spec_reject = len(draft) - j
                if draft:
                    seq.spec_proposed += len(draft)
                    seq.spec_accepted += j
                    self.spec_stats["proposed"] += len(draft)
                    self.spec_stats["accepted"] += j
            elif self._sit_out(seq):
                seq.awaiting = True
                seq.jump_tail = []
            else:
                seq.output_ids.append(PENDING)
                seq.pending_src = i
            self.bm.commit(seq)
        for seq, start, n in batch.prefill:
            if not seq.finished and start + n < seq.num_tokens:
                self.bm.commit(seq)

    def _finish_reason(self, seq: Sequence, tok: int) -> Optional[str]:
        forced = seq.params.forced_output
        if len(seq.output_ids) >= seq.params.max_tokens:
            return "length"
        if forced is not None and len(seq.output_ids) >= len(forced) and not seq.params.ignore_eos:
            return "stop"
        if not seq.params.ignore_eos and (tok in self.eos_ids or tok in seq.params.stop_token_ids):
            return "stop"
        if seq.num_tokens >= self.cfg.max_model_len:
            return "length"
        return None

    def _resolve(self, samplers: List[Sequence], sampled: List[int]) -> List[StepOutput]:
        now = time.perf_counter()
        outs: List[StepOutput] = []
        for seq, _, toks in self._group(samplers, sampled):
            tok = toks[-1]
            if seq.finished:                   # aborted (or finished) while in flight
                continue
            was_sampled = False
            sat_out = False                    # not in the step launched just now: may draft
            if seq.awaiting:
                seq.awaiting = False
                sat_out = True
                if seq.spec_rows > 1:          # sampled draft: keep the accepted prefix + bonus
                    acc, bonus = self._verify(seq, toks)
                    self.bm.commit(seq)        # verified positions only (num_computed clamped)
                    seq.output_ids.append(bonus)
                    new = acc + [bonus]
                    was_sampled = True
                elif seq.jump_tail:
                    new = seq.jump_tail
                    seq.jump_tail = []
                    seq.output_ids.extend(new)
                else:
                    new = [int(tok)]
                    seq.output_ids.extend(new)
                    was_sampled = seq.params.forced_output is None
            elif seq.pending_src >= 0:
                new = [int(tok)]
                seq.output_ids[-1] = new[0]
                seq.pending_src = -1
                was_sampled = True
            else:                              # known run, appended at launch time
                new = seq.last_run or [seq.output_ids[-1]]
                seq.last_run = []
            tok = new[-1]
            if seq.first_token_time is None:
                seq.first_token_time = now
            reason = self._finish_reason(seq, tok)
            if reason is not None:
                # its speculative row in the step now in flight writes into blocks freed here; any
                # reuse is by a LATER step, ordered after it on the stream
                self.scheduler.finish(seq, reason)
                self.requests.pop(seq.request_id, None)
            elif was_sampled:
                self._stage_grammar(seq)    # used by the next launch (overrides its sample)
                if sat_out and not seq.jump_queue and seq.status == SeqStatus.RUNNING:
                    draft = self._propose(seq)
                    if draft:                  # rides with the just-known token next step
                        seq.output_ids.extend(draft)
                        seq.spec_rows = len(draft) + 1
            outs.append(StepOutput(seq.request_id, new, reason is not None, reason, seq))
        return outs

    def _step_overlap(self) -> List[StepOutput]:
        t0 = time.perf_counter()
        prev = self._inflight
        if prev is not None:
            with marker("engine.advance"):
                self._advance(prev[0], prev[1])
        with marker("engine.schedule"):
            batch = self.scheduler.schedule()
        launched = None
        t1 = t0
        if not batch.empty():
            with marker("engine.inputs"):
                si = build_step_inputs(batch)
            if self.ps.tp_size > 1:
                tb = time.perf_counter()
                comm.broadcast_step(si)
                self.timing["c4_s"] = self.timing.get("c4_s", 0.0) + time.perf_counter() - tb
            t1 = time.perf_counter()
            launched = (batch, self._samplers(batch), self.runner.launch(si))
            # teacher-forced drafts were verified at _advance: drop the rejected tail now that the
            # chunk (all of it, as a real verification computes) is on its way
            for seq, _, _ in batch.prefill:
                if seq.spec_reject:
                    del seq.output_ids[len(seq.output_ids) - seq.spec_reject:]
                    seq.spec_reject = 0
                    seq.spec_rows = 0
                elif seq.spec_rows and seq.params.forced_output is not None:
                    seq.spec_rows = 0
        t2 = time.perf_counter()
        outs: List[StepOutput] = []
        if prev is not None:
            with marker("engine.wait"):
                res = prev[2].result()
            with marker("engine.resolve"):
                outs = self._resolve(prev[1], res)
        self._inflight = launched
        t3 = time.perf_counter()
        tm = self.timing
        tm["prepare_s"] += t1 - t0
        tm["execute_s"] += t2 - t1
        tm["post_s"] += t3 - t2
        return outs

    # -- synchronous ------------------------------------------------------------------------------
    def _step_sync(self) -> List[StepOutput]:
        t0 = time.perf_counter()
        batch = self.scheduler.schedule()
        if batch.empty():
            return []
        si = build_step_inputs(batch)
        if self.ps.tp_size > 1:
            comm.broadcast_step(si)
        t1 = time.perf_counter()
        sampled = self.runner.execute(si)
        now = time.perf_counter()
        tm = self.timing
        tm["prepare_s"] += t1 - t0
        tm["execute_s"] += now - t1
        outs: List[StepOutput] = []
        samplers = self._samplers(batch)   # before num_computed moves (sampled-vector order)
        for seq, start, n in batch.prefill:
            seq.num_computed = start + n
        for seq in batch.decode:
            seq.num_computed = seq.num_tokens
        for seq, _, toks in self._group(samplers, sampled):
            acc: List[int] = []
            tok = toks[-1]
            if seq.spec_rows > 1:
                acc, tok = self._verify(seq, toks)
            known = self._known_run(seq)
            run = known or [int(tok)]
            seq.output_ids.extend(run)
            if seq.first_token_time is None:
                seq.first_token_time = now
            reason = self._finish_reason(seq, run[-1])
            if reason is None and not known:
                self._stage_grammar(seq)        # nothing in flight: append the forced run now
                if seq.jump_queue:
                    extra, seq.jump_queue = seq.jump_queue, []
                    extra = extra[:max(seq.params.max_tokens - len(seq.output_ids), 0)]
                    seq.output_ids.extend(extra)
                    run = run + extra
                    reason = self._finish_reason(seq, run[-1])
            self.bm.commit(seq)
            if reason is not None:
                self.scheduler.finish(seq, reason)
                self.requests.pop(seq.request_id, None)
            else:
                draft = self._propose(seq)
                if draft:
                    seq.output_ids.extend(draft)
                    seq.spec_rows = len(draft) + 1
            outs.append(StepOutput(seq.request_id, acc + run, reason is not None, reason, seq))
        for seq, start, n in batch.prefill:
            if start + n < seq.num_tokens:
                self.bm.commit(seq)
        tm["post_s"] += time.perf_counter() - now
        return outs

    def follower_loop(self) -> None:
        """Non-leader TP ranks: replay the leader's steps until it broadcasts None -- with the
        leader's own one-step-in-flight pipeline: step N+1 is launched before step N is collected,
        so the follower's host (C4 receive, input staging) works while its GPU runs, and it never
        adds a device sync between the leader's launches."""
        prev = None
        t = self.timing
        steps = 0

        def collect(p) -> None:
            # a follower's own collective failure is the leader's to act on: the device-side poison
            # (allreduce.hip) fails the leader's collectives too, and it answers with the fallback
            # control message; until then this rank keeps replaying in lockstep
            try:
                p.result()
            except CollectiveTimeout as e:
                logger.error(f"tp follower rank {self.ps.rank}: {e}; waiting for the leader's fallback")

        while True:
            t0 = time.perf_counter()
            si = comm.broadcast_step(None)
            t1 = time.perf_counter()
            t["recv_s"] = t.get("recv_s", 0.0) + t1 - t0
            if si is None:
                break
            if si.control_code == StepInputs.CTRL_RCCL_FALLBACK:
                if prev is not None:
                    collect(prev)
                    prev = None
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                comm.fallback_to_rccl("leader: TP collective failed")
                self.runner.drop_graphs()
                continue
            cur = self.runner.launch(si)
            t2 = time.perf_counter()
            t["execute_s"] += t2 - t1
            if prev is not None:
                collect(prev)
            t["post_s"] += time.perf_counter() - t2
            prev = cur
            steps += 1
        if prev is not None:
            collect(prev)
        # the C4 anatomy of this follower: time blocked receiving the leader's steps, launching them,
        # and waiting for its own previous step's results (its GPU time not hidden by the receive)
        logger.info(f"tp follower rank {self.ps.rank}: {steps} steps, recv {t.get('recv_s', 0.0):.2f}s, "
                    f"launch {t['execute_s']:.2f}s, wait {t['post_s']:.2f}s")

    def stop_followers(self) -> None:
        if self.ps.tp_size > 1 and self.ps.is_tp_leader:
            comm.broadcast_step(None)
        if self.cp is not None:
            self.cp.stop()

    def cp_follower_loop(self) -> None:
        """Context-parallel follower ranks: join the leader's long-prompt prefills until it stops."""
        if self.cp is None:
            raise RuntimeError("cp_follower_loop needs cp_size > 1 and init_cp_groups")
        self.cp.follower_loop()

    # -- convenience --------------------------------------------------------------------
    def generate(self, prompts: Seq[Seq[int]], params: SamplingParams) -> List[List[int]]:
        seqs = [self.add_request(f"gen-{i}-{id(p)}", p, params) for i, p in enumerate(prompts)]
        while any(not s.finished for s in seqs):
            self.step()
        return [s.output_ids for s in seqs]

    def stats(self) -> Dict[str, float]:
        return {"running": len(self.scheduler.running), "waiting": len(self.scheduler.waiting),
                "kv_usage": self.bm.usage(), "prefix_hit_rate": self.bm.hit_rate(),
                "kv_blocks": self.bm.num_blocks, "kv_evictions": int(getattr(self.bm, "evictions", 0)),
                "preemptions": self.scheduler.num_preemptions,
                "time_capped_steps": self.scheduler.num_capped_steps,
                "burst_steps": self.scheduler.num_burst_steps,
                "sjf_admits": self.scheduler.num_sjf_admits,
                "short_reserved_steps": self.scheduler.num_reserved_steps,
                "short_wait": dict(self.scheduler.short_wait),
                "spec_draft_tokens": self.spec_stats["proposed"], "spec_accepted_tokens": self.spec_stats["accepted"],
                "steps": self.runner.stats["steps"], "graph_steps": self.runner.stats["graph_steps"],
                "tokens": self.runner.stats["tokens"], **{k: round(v, 3) for k, v in self.timing.items()},
                "gemm_tuning": float(bool(getattr(self, "gemm_tuning", None))),
                "prefill_steps": self.runner.stats["prefill_steps"],
                "prefill_step_tokens": self.runner.stats["prefill_step_tokens"],
                **(self.cp.stats if self.cp is not None else {}),
                "prefill_step_tokens_mean": round(self.runner.stats["prefill_step_tokens"]
                                                  / max(1, self.runner.stats["prefill_steps"]), 1),
                # share of the prefill steps' GEMM rows that are 256-row tile padding
                "prefill_tile_pad_frac": round(self.runner.stats["prefill_tile_pad_rows"]
                                               / max(1, self.runner.stats["prefill_step_tokens"]
                                                     + self.runner.stats["prefill_tile_pad_rows"]), 4),
                "prefill_m_hist": dict(zip(("le256", "le512", "le1k", "le2k", "le3k", "le4k", "gt4k"),
                                           self.runner.stats["prefill_m_hist"])),
                # device time per step (PENNY_STEP_GPU_TIMING=1): compare with step_p50_ms (host cadence)
                "gpu_graph_ms_mean": round(1e3 * self.runner.stats["gpu_graph_s"]
                                           / max(1, self.runner.stats["graph_steps"]), 3),
                "gpu_eager_ms_mean": round(1e3 * self.runner.stats["gpu_eager_s"]
                                           / max(1, self.runner.stats["steps"] - self.runner.stats["graph_steps"]), 3),
                "gpu_step_s": round(self.runner.stats["gpu_graph_s"] + self.runner.stats["gpu_eager_s"], 3),
                "gpu_idle_between_steps_s": round(self.runner.stats["gpu_idle_s"], 3),
                "gpu_idle_gaps": self.runner.stats["gpu_idle_gaps"], **self._memory_stats()}

    def _memory_stats(self) -> Dict[str, float]:
        """HBM in use on the device (all allocators) and the caching allocator's peak: the
        headroom ``kv_mem_fraction`` leaves is checked against these, not assumed."""
        if self.device.type != "cuda":
            return {}
        free, total = torch.cuda.mem_get_info(self.device)
        g = float(1 << 30)
        return {"hbm_used_gib": round((total - free) / g, 1), "hbm_total_gib": round(total / g, 1),
                "torch_peak_reserved_gib": round(torch.cuda.max_memory_reserved(self.device) / g, 1),
                "kv_pool_gib": round(self.bm.num_blocks * KVCache.bytes_per_block(
                    self.model.cfg.num_layers, self.model.hkv, self.model.D) / g, 1)}
