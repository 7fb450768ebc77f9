"""Block allocator / prefix cache / scheduler tests; C++ allocator checked against the Python one."""
import random

import pytest

from financial_chatbot_llm_amd.engine.block_manager import PyBlockManager
from financial_chatbot_llm_amd.engine.native_block_manager import NativeBlockManager
from financial_chatbot_llm_amd.engine.scheduler import Scheduler
from financial_chatbot_llm_amd.engine.sequence import SamplingParams, Sequence

BS = 64


def mk(tokens, rid="r"):
    return Sequence(rid, tokens, SamplingParams(max_tokens=4))


@pytest.mark.parametrize("impl", [PyBlockManager, NativeBlockManager])
def test_prefix_hits_and_reuse(impl):
    bm = impl(16, BS, True)
    a = mk(list(range(300)))
    assert bm.match_prefix(a) == 0
    assert bm.grow(a, 300) and len(a.block_table) == 5
    a.num_computed = 300
    bm.commit(a)
    bm.free(a)
    assert bm.num_free() == 16           # cached blocks are evictable, i.e. still allocatable
    b = mk(list(range(300)) + [7, 8])
    assert bm.match_prefix(b) == 256     # 4 full blocks verified-hit
    assert bm.hits == 4
    c = mk(list(range(128)))             # exactly 2 blocks: the last one must be recomputed
    assert bm.match_prefix(c) == 64


@pytest.mark.parametrize("impl", [PyBlockManager, NativeBlockManager])
def test_exhaustion_and_eviction(impl):
    bm = impl(4, BS, True)
    a = mk(list(range(256)))
    assert bm.grow(a, 256)
    a.num_computed = 256
    bm.commit(a)
    b = mk(list(range(1000, 1100)))
    assert not bm.grow(b, 100)           # pool exhausted, nothing allocated
    assert b.block_table == []
    bm.free(a)
    assert bm.grow(b, 100)               # evicts LRU cached blocks (tail of `a` first)
    d = mk(list(range(256)) + [1])
    assert bm.match_prefix(d) == 128     # head blocks of `a` survived eviction


@pytest.mark.parametrize("impl", [PyBlockManager, NativeBlockManager])
def test_ephemeral_blocks_are_evicted_first(impl):
    """A sequence freed with ``evict_first`` (its uncached KV will not recur: a prompt around a
    one-off retrieval context) gives up its own blocks before older, still-useful prefixes; the
    blocks it got from the prefix cache keep their LRU place."""
    bm = impl(8, BS, True)
    keep = mk(list(range(256)), "keep")                       # 4 blocks, freed first (older)
    assert bm.grow(keep, 256)
    keep.num_computed = 256
    bm.commit(keep)
    bm.free(keep)
    eph = mk(list(range(128)) + list(range(5000, 5192)), "eph")  # 2 hit blocks + 3 own blocks
    assert bm.match_prefix(eph) == 128
    assert bm.grow(eph, 320)
    eph.num_computed = 320
    bm.commit(eph)
    bm.free(eph, evict_first=True)
    new = mk(list(range(9000, 9192)), "new")                  # needs 3: 1 free + 2 evicted
    assert bm.grow(new, 192)
    again = mk(list(range(256)) + [1], "again")
    assert bm.match_prefix(again) == 256                      # the older prefix survived whole
    bm.free(again)
    probe = mk(list(range(128)) + list(range(5000, 5192)) + [1], "probe")
    assert bm.match_prefix(probe) == 192                      # eph's tail went first: 1 own block left


def test_native_matches_python_on_random_workload():
    rnd = random.Random(0)
    py, nat = PyBlockManager(40, BS, True), NativeBlockManager(40, BS, True)
    prefixes = [[rnd.randrange(1000) for _ in range(rnd.randrange(64, 400))] for _ in range(5)]
    live = []
    for step in range(400):
        op = rnd.random()
        if op < 0.4 or not live:
            toks = prefixes[rnd.randrange(5)] + [rnd.randrange(1000) for _ in range(rnd.randrange(0, 100))]
            s1, s2 = mk(toks), mk(toks)
            assert py.match_prefix(s1) == nat.match_prefix(s2)
            assert s1.block_table == s2.block_table
            n = len(toks)
            ok1, ok2 = py.grow(s1, n), nat.grow(s2, n)
            assert ok1 == ok2 and s1.block_table == s2.block_table
            if ok1:
                s1.num_computed = s2.num_computed = n
                py.commit(s1)
                nat.commit(s2)
                live.append((s1, s2))
            else:
                py.free(s1)
                nat.free(s2)
        elif op < 0.7:
            s1, s2 = live[rnd.randrange(len(live))]
            s1.output_ids.append(5)
            s2.output_ids.append(5)
            ok1, ok2 = py.grow(s1, s1.num_tokens), nat.grow(s2, s2.num_tokens)
            assert ok1 == ok2 and s1.block_table == s2.block_table
            if ok1:
                s1.num_computed = s2.num_computed = s1.num_tokens
                py.commit(s1)
                nat.commit(s2)
        else:
            s1, s2 = live.pop(rnd.randrange(len(live)))
            eph = rnd.random() < 0.5
            py.free(s1, evict_first=eph)
            nat.free(s2, evict_first=eph)
        assert py.num_free() == nat.num_free()
        assert nat.core.check_invariants() == ""
    assert py.hits == nat.hits and py.queries == nat.queries


def test_scheduler_chunked_prefill_and_preemption():
    bm = PyBlockManager(6, BS, True)
    sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=100, max_model_len=1024)
    a, b = mk(list(range(150)), "a"), mk(list(range(500, 700)), "b")
    sch.add(a)
    sch.add(b)
    batch = sch.schedule()
    assert [(s.request_id, st, n) for s, st, n in batch.prefill] == [("a", 0, 100)]
    a.num_computed = 100
    batch = sch.schedule()
    # a finishes its prompt (50 tokens), b starts with the remaining budget
    assert [(s.request_id, st, n) for s, st, n in batch.prefill] == [("a", 100, 50), ("b", 0, 50)]
    a.num_computed, b.num_computed = 150, 50
    a.output_ids.append(1)
    # b needs 4 blocks total, a needs 3 -> pool of 6 forces a preemption of the youngest (b)
    for _ in range(3):
        batch = sch.schedule()
        for s, st, n in batch.prefill:
            s.num_computed = st + n
        for s in batch.decode:
            s.num_computed = s.num_tokens
            s.output_ids.append(1)
    assert b.num_preemptions >= 0
    assert bm.num_free() >= 0


def test_scheduler_drops_a_draft_it_cannot_grow():
    """A speculative chunk whose blocks do not fit gives up its draft: the sequence
    is an ordinary decode row again and the next step's decode pass (which preempts when the pool
    is dry) schedules it -- steps never come out empty with has_work() true."""
    bm = PyBlockManager(2, BS, True)
    sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=256, max_model_len=1024)
    a = mk(list(range(BS * 2 - 1)), "a")
    sch.add(a)
    batch = sch.schedule()
    a.num_computed = BS * 2 - 1
    a.output_ids.append(5)                     # the sampled token: KV not computed yet
    a.output_ids.extend([6, 7, 8])             # a draft that needs a third block
    a.spec_rows = 4
    batch = sch.schedule()
    assert batch.empty() and a.spec_rows == 0 and a.output_ids == [5]
    batch = sch.schedule()
    assert batch.decode == [a]


def _mk_params(prompt, rid, max_tokens, arrival):
    from financial_chatbot_llm_amd.engine.sequence import SamplingParams, Sequence
    return Sequence(rid, prompt, SamplingParams(max_tokens=max_tokens), arrival=arrival)


def test_scheduler_admits_short_output_requests_first():
    """A decide call (short output) queued behind a long respond prefill is admitted first."""
    clock = [100.0]
    bm = PyBlockManager(64, BS, True)
    sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=4096, clock=lambda: clock[0])
    long_ = _mk_params(list(range(1000, 1400)), "respond", 512, arrival=1.0 + 99)
    short = _mk_params(list(range(2000, 2060)), "decide", 96, arrival=2.0 + 99)
    sch.add(long_)
    sch.add(short)
    batch = sch.schedule()
    assert [(s.request_id, st, n) for s, st, n in batch.prefill] == [("decide", 0, 60), ("respond", 0, 68)]


@pytest.mark.parametrize("reserve", [0, 96])
def test_short_reserve_bounds_decide_wait_and_never_starves_long_prefills(reserve):
    """A burst of long respond prefills already running takes whole steps; a decide prompt that
    arrives meanwhile waits for the burst without a reservation, and is admitted in the very next
    step with one -- while every step still gives the long prefills budget - reserve tokens, and
    a stream of short prompts never stops them (starvation freedom)."""
    clock = [100.0]
    bm = PyBlockManager(512, BS, True)
    sch = Scheduler(bm, max_num_seqs=64, max_num_batched_tokens=256, max_model_len=8192, clock=lambda: clock[0],
                    short_reserve_tokens=reserve)
    longs = [_mk_params(list(range(10000 * (i + 1), 10000 * (i + 1) + 900)), f"respond{i}", 512, arrival=99.0 + i * 0.01)
             for i in range(4)]
    for q in longs:
        sch.add(q)
    batch = sch.schedule()                                  # burst admitted: 256 tokens of respond0
    for q, st, n in batch.prefill:
        q.num_computed = st + n
    decide = _mk_params(list(range(5000, 5060)), "decide", 96, arrival=99.5)
    sch.add(decide)
    admitted_at, long_tokens = None, []
    for step in range(1, 40):
        if step > 1 and step % 2 == 0:                      # a fresh decide every other step
            sch.add(_mk_params(list(range(6000 + 100 * step, 6000 + 100 * step + 40)), f"d{step}", 96, arrival=99.6))
        batch = sch.schedule()
        long_tokens.append(sum(n for q, _, n in batch.prefill if q.request_id.startswith("respond")))
        if admitted_at is None and any(q is decide for q, _, _ in batch.prefill):
            admitted_at = step
        for q, st, n in batch.prefill:
            q.num_computed = st + n
        for q in list(sch.running):
            if q.num_computed >= q.num_tokens:               # prompt done: retire it (no decode here)
                sch.finish(q, "stop")
        if all(q.finished for q in longs):
            break
    if reserve:
        assert admitted_at == 1
        active = [t for t in long_tokens if t > 0]
        assert min(active[:-1]) >= 256 - reserve             # long prefills keep budget - reserve
    else:
        assert admitted_at > 1                               # queued behind the burst's chunks
    assert all(q.finished for q in longs)                   # never starved


def test_scheduler_orders_a_class_by_turn_start():
    """Within a priority class the older TURN goes first: a respond call whose turn started
    before a newer turn's decide call is admitted ahead of it although it arrived later."""
    from financial_chatbot_llm_amd.engine.sequence import SamplingParams, Sequence
    clock = [100.0]
    bm = PyBlockManager(64, BS, True)
    sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=64, max_model_len=4096, clock=lambda: clock[0])
    decide_new = Sequence("decide-turn2", list(range(2000, 2060)), SamplingParams(max_tokens=96, priority_ts=99.5),
                          arrival=99.6)
    respond_old = Sequence("respond-turn1", list(range(3000, 3060)), SamplingParams(max_tokens=128, priority_ts=98.0),
                           arrival=99.8)
    sch.add(decide_new)
    sch.add(respond_old)
    batch = sch.schedule()
    assert [s.request_id for s, _, _ in batch.prefill] == ["respond-turn1", "decide-turn2"]


def test_scheduler_aging_is_starvation_free():
    """A long request keeps losing to fresh short ones only until it has waited aging_s; then,
    being older, it is admitted ahead of every newer short request."""
    clock = [0.0]
    bm = PyBlockManager(512, BS, True)
    sch = Scheduler(bm, max_num_seqs=64, max_num_batched_tokens=64, max_model_len=4096, aging_s=1.0,
                    clock=lambda: clock[0])
    long_ = _mk_params(list(range(5000, 5300)), "long", 512, arrival=0.0)
    sch.add(long_)
    admitted_long_at = None
    for step in range(40):
        clock[0] = 0.1 * (step + 1)
        sch.add(_mk_params(list(range(10 * step, 10 * step + 64)), f"short{step}", 64, arrival=clock[0]))
        batch = sch.schedule()
        for s, st, n in batch.prefill:
            s.num_computed = st + n
            if s is long_ and admitted_long_at is None:
                admitted_long_at = clock[0]
        for s in list(sch.running):       # finish whatever completed its prompt (keeps the pool free)
            if s.num_computed >= s.num_tokens:
                sch.finish(s, "stop")
    assert admitted_long_at is not None and 1.0 <= admitted_long_at <= 1.2, admitted_long_at


def test_scheduler_quantises_step_rows():
    """Step rows (decode + prefill) are rounded down to the quantum by shortening the last chunk."""
    bm = PyBlockManager(256, BS, True)
    sch = Scheduler(bm, max_num_seqs=8, max_num_batched_tokens=1000, max_model_len=4096, token_quantum=256)
    a = _mk_params(list(range(1000, 1700)), "a", 64, arrival=1.0)
    b = _mk_params(list(range(3000, 3500)), "b", 64, arrival=2.0)
    sch.add(a)
    sch.add(b)
    batch = sch.schedule()
    assert batch.num_tokens == 768                      # 1000 -> 768: b's chunk 300 -> 68
    assert [(s.request_id, st, n) for s, st, n in batch.prefill] == [("a", 0, 700), ("b", 0, 68)]
    assert b.num_prefilled == 68
    small = Scheduler(PyBlockManager(64, BS, True), max_num_seqs=8, max_num_batched_tokens=1000,
                      max_model_len=4096, token_quantum=256)
    c = _mk_params(list(range(200)), "c", 64, arrival=1.0)
    small.add(c)
    assert small.schedule().num_tokens == 200           # below one quantum: untouched
    # the last chunk too short to absorb the remainder (a 150-token prompt): the cut comes from the
    # earlier chunk instead of leaving the step unaligned
    sch2 = Scheduler(PyBlockManager(256, BS, True), max_num_seqs=8, max_num_batched_tokens=1000,
                     max_model_len=4096, token_quantum=256)
    d = _mk_params(list(range(5000, 5850)), "d", 64, arrival=1.0)
    e = _mk_params(list(range(8000, 8150)), "e", 64, arrival=2.0)
    sch2.add(d)
    sch2.add(e)
    batch = sch2.schedule()
    assert batch.num_tokens == 768
    assert [(s.request_id, st, n) for s, st, n in batch.prefill] == [("d", 0, 618), ("e", 0, 150)]
    assert d.num_prefilled == 618


def test_step_time_bound_caps_prefill_only_while_a_decide_decodes():
    """StepCostModel: with a short-output (decide) sequence decoding, the step's prefill tokens
    are capped to the modelled time target (never below min_prefill_tokens); with no decide
    decoding, the full token budget is used.  Long prompts still progress every step."""
    from financial_chatbot_llm_amd.engine.block_manager import make_block_manager
    from financial_chatbot_llm_amd.engine.scheduler import Scheduler, StepCostModel
    from financial_chatbot_llm_amd.engine.sequence import SamplingParams, Sequence
    bm = make_block_manager(2048, 64, True)
    cost = StepCostModel(target_ms=10.0, base_ms=2.0, per_row_ms=0.1, per_token_ms=0.01, min_prefill_tokens=128)
    sch = Scheduler(bm, max_num_seqs=64, max_num_batched_tokens=4096, max_model_len=16384, cost_model=cost)
    decide = Sequence("d", list(range(100)), SamplingParams(max_tokens=64))
    sch.add(decide)
    b = sch.schedule()                                   # decide prompt prefilled
    decide.num_computed = decide.num_tokens
    decide.output_ids.append(7)                          # now decoding
    long_prompt = Sequence("r", list(range(10000)), SamplingParams(max_tokens=512))
    sch.add(long_prompt)
    b = sch.schedule()
    assert b.decode == [decide]
    cap = cost.prefill_cap(1)                            # (10 - 2 - 0.1) / 0.01 = 790
    assert cap == 790 and b.num_prefill_tokens == cap and sch.num_capped_steps == 1
    # the decide finishes: the long prompt gets the whole budget again
    sch.finish(decide, "stop")
    for s_, st, n in b.prefill:
        s_.num_computed = st + n
    b2 = sch.schedule()
    assert b2.num_prefill_tokens == 4096
    # a tight target never starves prefill
    assert StepCostModel(target_ms=1.0).prefill_cap(200) == 256


def test_step_time_bound_off_by_default():
    from financial_chatbot_llm_amd.config import EngineConfig
    from financial_chatbot_llm_amd.engine.scheduler import StepCostModel
    assert EngineConfig().step_time_target_ms == 0.0 and StepCostModel().target_ms == 0.0


def test_short_job_first_admits_short_prompt_once_ahead_of_long_prefill():
    """sjf_tokens: a short waiting prompt is admitted ahead of a long prefill's next chunk, and a
    sequence admitted that way is not scheduled a second time by the continuing-prefill pass."""
    from financial_chatbot_llm_amd.engine.block_manager import make_block_manager
    from financial_chatbot_llm_amd.engine.scheduler import Scheduler
    from financial_chatbot_llm_amd.engine.sequence import SamplingParams, Sequence
    bm = make_block_manager(256, 64, False)
    sch = Scheduler(bm, max_num_batched_tokens=512, sjf_tokens=128)
    long = Sequence("long", list(range(2000)), SamplingParams(max_tokens=8))
    sch.add(long)
    b1 = sch.schedule()
    assert [(q.request_id, n) for q, _, n in b1.prefill] == [("long", 512)]
    long.num_computed = 512
    short = Sequence("short", list(range(100)), SamplingParams(max_tokens=8))
    sch.add(short)
    b2 = sch.schedule()
    ids = [q.request_id for q, _, _ in b2.prefill]
    assert ids == ["short", "long"] and len(set(ids)) == len(ids)
    assert sum(n for _, _, n in b2.prefill) == 512 and sch.num_sjf_admits == 1


@pytest.mark.parametrize("short_first", [False, True])
def test_short_first_orders_decides_ahead_of_aged_long_prompts(short_first):
    """An aged long-output prompt (waited past aging_s) and a fresh decide-class prompt compete
    for one step's budget: by default they share the priority class and the older long prompt
    goes first; with short_first the decide does, the aged prompt still beats fresh long ones,
    and the admission anatomy (short_wait) records why the loser waited."""
    clock = [100.0]
    bm = PyBlockManager(512, BS, True)
    sch = Scheduler(bm, max_num_seqs=64, max_num_batched_tokens=128, max_model_len=8192, clock=lambda: clock[0],
                    aging_s=1.0, short_first=short_first)
    aged = _mk_params(list(range(20000, 20000 + 400)), "aged", 512, arrival=98.0)
    fresh = _mk_params(list(range(30000, 30000 + 400)), "fresh", 512, arrival=99.9)
    decide = _mk_params(list(range(5000, 5000 + 100)), "decide", 96, arrival=99.95)
    for q in (fresh, aged, decide):
        sch.add(q)
    batch = sch.schedule()
    first = batch.prefill[0][0]
    assert first is (decide if short_first else aged)
    assert all(q is not fresh for q, _, _ in batch.prefill)     # fresh long prompt is last either way
    sw = sch.short_wait
    if short_first:
        assert sw["steps"] == 0                                 # no short prompt left waiting
    else:
        assert sw["steps"] == 1 and sw["tok_admit_long"] == 128 and sw["waiting_short"] == 1
        assert sw["budget"] == 1                                # the aged long prompt took the budget


def test_short_wait_records_kv_pool_exhaustion():
    """A decide-class prompt that cannot be admitted because the KV pool is full is counted under
    the "grow" reason of the admission anatomy, not "budget"."""
    clock = [100.0]
    bm = PyBlockManager(8, BS, True)                 # 8 blocks
    sch = Scheduler(bm, max_num_seqs=64, max_num_batched_tokens=4096, max_model_len=8192, clock=lambda: clock[0])
    big = _mk_params(list(range(40000, 40000 + 7 * BS)), "respond", 512, arrival=99.0)
    sch.add(big)
    batch = sch.schedule()                           # takes 7 of the 8 blocks
    for q, st, n in batch.prefill:
        q.num_computed = st + n
    decide = _mk_params(list(range(50000, 50000 + 3 * BS)), "decide", 96, arrival=99.5)
    sch.add(decide)
    sch.schedule()
    assert decide in sch.waiting
    assert sch.short_wait["grow"] >= 1 and sch.short_wait["budget"] == 0


def test_short_reserve_implies_short_first():
    """with a short-output reservation, aged long-output prompts must not share the
    short class (they could spend the reserve); the reserve turns short_first on."""
    from financial_chatbot_llm_amd.engine.block_manager import make_block_manager
    from financial_chatbot_llm_amd.engine.scheduler import Scheduler
    bm = make_block_manager(64, 64, True)
    assert Scheduler(bm, 8, 512, 4096, short_reserve_tokens=256).short_first
    assert not Scheduler(bm, 8, 512, 4096).short_first
