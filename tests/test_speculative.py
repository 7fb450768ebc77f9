"""Prompt-lookup speculative decoding (engine.speculative, LLMEngine).

* the n-gram draft source finds the most recent earlier occurrence of the output's tail;
* teacher-forced decide outputs (the benchmark's scripted tool calls, whose arguments copy the
  user's words) come out identical with fewer engine steps, in both step modes;
* sampled outputs (greedy and seeded temperature sampling) are identical with and without
  speculation -- drafts are verified against the model's own samples at the same seeds -- and
  drafts do get accepted (a random tiny model falls into repetition loops it can copy from);
* a draft never runs past max_tokens and never carries a stop token.
"""
import pytest

from financial_chatbot_llm_amd.agent import scripted_decision
from financial_chatbot_llm_amd.agent.grammar import ToolCallGrammar, jump_mask
from financial_chatbot_llm_amd.agent.toolcall import format_tool_call
from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
from financial_chatbot_llm_amd.engine.speculative import PromptLookup, accept_draft
from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
from financial_chatbot_llm_amd.tools import make_retrieval_tool

BASE = dict(model="llama-tiny", device="cpu", max_model_len=1024, max_num_batched_tokens=256,
            use_cuda_graph=False, max_num_seqs=8, num_kv_blocks=96)
TOK = SyntheticLlamaTokenizer()
EOT = TOK.special["<|eot_id|>"]
RET = make_retrieval_tool(None)


def test_prompt_lookup_most_recent_longest_match():
    pl = PromptLookup([5, 6, 7, 8, 1, 2, 5, 6, 9, 9, 4])
    assert pl.propose([5, 6], 3) == [9, 9, 4]          # 2-gram (5, 6): most recent occurrence
    assert pl.propose([7], 2) == [8, 1]
    assert pl.propose([3], 4) == []
    assert pl.propose([2, 5, 6], 2, min_ngram=2) == [9, 9]
    assert pl.propose([1, 3], 2, min_ngram=2) == []     # no 2-gram match
    assert accept_draft([1, 2, 3], [1, 2, 4]) == 2 and accept_draft([], [1]) == 0
    # recency: the 1-gram (6,) 300 tokens after the 2-gram (5, 6) wins at recency 256, not at 0
    ids = [5, 6, 1] + [0] * 300 + [6, 2]
    assert PromptLookup(ids).propose([5, 6], 1) == [1]
    assert PromptLookup(ids, recency=256).propose([5, 6], 1) == [2]


def _run(params_list, prompts, mode, **cfg):
    eng = LLMEngine(EngineConfig(async_scheduling=mode, seed=0, **{**BASE, **cfg}))
    seqs = [eng.add_request(f"r{i}", p, sp) for i, (p, sp) in enumerate(zip(prompts, params_list))]
    while any(not s.finished for s in seqs) or eng.has_work():
        eng.step()
    return seqs, eng


@pytest.mark.parametrize("mode", [True, False])
def test_forced_decide_identical_with_fewer_steps(mode):
    g = ToolCallGrammar([RET])
    qs = ["What did I spend on groceries last month?", "Show me my recent transactions at Amazon.",
          "How should I invest for retirement?"]
    forced, prompts = [], []
    for i, q in enumerate(qs):
        call = scripted_decision(q)
        f = TOK.encode(format_tool_call(call) if call else "No tool call", allow_special=False) + [EOT]
        forced.append(f)
        prompts.append(list(range(300 + 7 * i, 340 + 7 * i)) + TOK.encode(" user: " + q, allow_special=False))

    def params(lookup):
        return [SamplingParams(temperature=0.5, max_tokens=96, forced_output=f, forced_jump=jump_mask(f, TOK.decode, g, EOT),
                               grammar=g, prompt_lookup=lookup) for f in forced]
    a, ea = _run(params(0), prompts, mode)
    b, eb = _run(params(8), prompts, mode)
    for sa, sb, f in zip(a, b, forced):
        assert sa.output_ids == f and sb.output_ids == f
        assert sa.finish_reason == sb.finish_reason == "stop"
    assert eb.spec_stats["accepted"] >= 6
    assert eb.runner.stats["steps"] < ea.runner.stats["steps"]


@pytest.mark.parametrize("mode", [True, False])
@pytest.mark.parametrize("temperature", [0.0, 0.8])
def test_sampled_outputs_identical_with_speculation(mode, temperature):
    prompts = [[400 + (i * 13) % 50 for i in range(60)] + [900 + i for i in range(20)],
               [700 + (i * 7) % 30 for i in range(90)]]

    def params(lookup):
        return [SamplingParams(temperature=temperature, max_tokens=48, ignore_eos=True, seed=11 + i,
                               prompt_lookup=lookup) for i in range(len(prompts))]
    a, _ = _run(params(0), prompts, mode)
    b, eb = _run(params(8), prompts, mode)
    for sa, sb in zip(a, b):
        assert sa.output_ids == sb.output_ids
        assert len(sb.output_ids) == 48
    if temperature == 0.0:
        assert eb.spec_stats["accepted"] > 0            # greedy loops get copied


class _EveryFifthChar:
    """Output grammar stub that forces " the" whenever the output text's length is a multiple of
    5: jump-forward fires often on a random model's text, inside drafted spans too."""
    def __init__(self):
        self.forcing = 0

    def forced(self, text):
        if text and len(text) % 5 == 0:
            self.forcing += 1
            return " the", False
        return "", False


@pytest.mark.parametrize("mode", [True, False])
@pytest.mark.parametrize("temperature", [0.0, 0.8])
def test_sampled_outputs_identical_with_speculation_under_grammar(mode, temperature):
    """Jump-forward inside a draft: the draft is cut before the first position where the grammar
    forces, so speculation emits exactly the one-token-per-step output."""
    prompts = [[400 + (i * 13) % 50 for i in range(60)] + [900 + i for i in range(20)],
               [700 + (i * 7) % 30 for i in range(90)]]

    def run(lookup):
        g = _EveryFifthChar()
        ps = [SamplingParams(temperature=temperature, max_tokens=40, ignore_eos=True, seed=5 + i, grammar=g,
                             prompt_lookup=lookup) for i in range(len(prompts))]
        seqs, eng = _run(ps, prompts, mode)
        return [s.output_ids for s in seqs], eng, g
    a, _, ga = run(0)
    b, eb, gb = run(8)
    assert a == b
    assert ga.forcing > 0 and gb.forcing > 0


def test_rejected_sampled_draft_never_enters_prefix_cache():
    """A sampled draft crossing a 64-token block boundary is rejected: the block holding draft
    positions must not be registered under the draft's token ids, since the bonus token then
    rewrites that KV.  A second request whose prompt carries the rejected draft must
    miss the prefix cache and compute what the uncached engine computes."""
    from financial_chatbot_llm_amd.ops.attention import KV_BS
    prompt = [500 + (i * 3) % 40 for i in range(KV_BS - 3)]
    bad = [7, 8, 9, 10, 11, 12]      # positions 63..68: d0 lands in block 0, the rest in block 1

    def engine(caching):
        return LLMEngine(EngineConfig(async_scheduling=True, seed=0, **{**BASE, "enable_prefix_caching": caching}))

    eng = engine(True)
    used = {"n": 0}

    def propose(seq, after=(), min_ngram=0):     # inject the draft once, after output token 2
        k = len(seq.output_ids) + len(after)
        if used["n"] == 0 and k in (1, 2):
            used["n"] = k == 2
            return list(bad)
        return []
    eng._propose = propose
    seq = eng.add_request("a", prompt, SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True, prompt_lookup=8))
    while eng.has_work():
        eng.step()
    assert used["n"] and eng.spec_stats["proposed"] == len(bad)
    assert seq.output_ids[2] != bad[0]            # rejected at its first token (bonus differs)
    p2 = prompt + seq.output_ids[:2] + bad + [42, 43, 44]
    outs = []
    for e in (eng, engine(False)):
        s = e.add_request("b", p2, SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
        while e.has_work():
            e.step()
        outs.append((s.num_cached_prompt, s.output_ids))
    assert outs[0][0] == 0, "block 0 was cached under the rejected draft"
    assert outs[0][1] == outs[1][1]


def test_draft_respects_max_tokens_and_stops():
    eng = LLMEngine(EngineConfig(async_scheduling=False, seed=0, **BASE))
    seq = eng.add_request("r", [9, 1, 2, 3, EOT, 7, 4, 5, 6, 7, 8, 9, 10], SamplingParams(max_tokens=6, prompt_lookup=8))
    seq.output_ids = [1, 2]
    assert eng._propose(seq) == [3]                       # cut before the stop token
    seq.output_ids = [4]
    assert eng._propose(seq) == [5, 6, 7, 8]              # k=1 -> room = 6 - 1 - 1 = 4
