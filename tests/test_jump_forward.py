"""Jump-forward decoding of grammar-forced decide tokens (agent.grammar, LLMEngine runs).

* the tool-call grammar forces exactly the JSON skeleton / unambiguous parts;
* teacher-forced (scripted) outputs come out identical with fewer engine steps;
* sampled outputs: the grammar's forced run is appended and computed as one chunk, and the
  tokens sampled after the chunk equal what a plain prefill of the same tokens predicts;
* both engine step modes (overlap and synchronous).
"""
import pytest

from financial_chatbot_llm_amd.agent import scripted_decision
from financial_chatbot_llm_amd.agent.grammar import ToolCallGrammar, jump_mask
from financial_chatbot_llm_amd.agent.toolcall import format_tool_call, parse_tool_calls
from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
from financial_chatbot_llm_amd.tools import make_plot_tool, make_retrieval_tool

BASE = dict(model="llama-tiny", device="cpu", max_model_len=1024, max_num_batched_tokens=256,
            use_cuda_graph=False, max_num_seqs=8, num_kv_blocks=96)
TOK = SyntheticLlamaTokenizer()
EOT = TOK.special["<|eot_id|>"]
RET = make_retrieval_tool(None)


def test_grammar_forces_skeleton_only():
    g = ToolCallGrammar([RET])
    assert g.forced("") == ("", False)                                   # tool or not: free
    assert g.forced("{") == ('"name": "', False)
    assert g.forced('{"name": "') == ('retrieve_transactions", "parameters": {', False)
    assert g.forced('{"name": "retrieve_transactions", "parameters": {') == ("", False)   # key or '}'
    assert g.forced('{"name": "retrieve_transactions", "parameters": {"sea') == ('rch_query": "', False)
    assert g.forced('{"name": "retrieve_transactions", "parameters": {"search_query": "gro') == ("", False)
    assert g.forced('{"name": "retrieve_transactions", "parameters": {"num_transactions": 2') == ("", False)
    assert g.forced('{"name": "retrieve_transactions", "parameters": {"num_transactions": 20,') == (' "', False)
    assert g.forced('{"name": "retrieve_transactions", "parameters": {"num_transactions": 20}') == ("}", True)
    assert g.forced("No") == (" tool call", True)
    assert g.forced("Hello") == ("", False)                             # outside the grammar
    two = ToolCallGrammar([RET, make_plot_tool()])
    assert two.forced('{"name": "') == ("", False)                       # two tools: name is a choice
    assert two.forced('{"name": "c') == ('reate_financial_plot", "parameters": {', False)


def test_jump_mask_marks_forced_tokens_of_a_real_call():
    text = format_tool_call(scripted_decision("What did I spend on groceries last month?", always_limit=True))
    ids = TOK.encode(text, allow_special=False) + [EOT]
    m = jump_mask(ids, TOK.decode, ToolCallGrammar([RET]), EOT)
    assert not m[0] and m[-1]                      # first token sampled, final EOT forced
    free = [TOK.decode([t]) for t, f in zip(ids, m) if not f]
    assert "What" in free and "20" in free and "30" in free               # values stay free
    assert 0.4 < sum(m) / len(m) < 0.75
    assert parse_tool_calls(TOK.decode(ids), [RET])[0].args["num_transactions"] == 20


def test_scripted_decide_follows_the_reference_few_shot():
    """tool_prompt.txt:15-23: a topical query carries num_transactions 20; a time-window query
    carries time_period_days and no num_transactions (limit -> 10000, qdrant_tool.py:145)."""
    topical = scripted_decision("What did I spend on groceries?")
    assert topical.args == {"search_query": "What did I spend on groceries", "num_transactions": 20}
    window = scripted_decision("How much did I spend two days ago?")
    assert window.args["time_period_days"] == 2 and "num_transactions" not in window.args
    assert scripted_decision("How should I invest for retirement?") is None
    legacy = scripted_decision("How much did I spend last week?", always_limit=True)
    assert legacy.args["num_transactions"] == 20 and legacy.args["time_period_days"] == 7


def _run(params_list, prompts, mode):
    eng = LLMEngine(EngineConfig(async_scheduling=mode, seed=0, **BASE))
    seqs = [eng.add_request(f"r{i}", p, sp) for i, (p, sp) in enumerate(zip(prompts, params_list))]
    while any(not s.finished for s in seqs) or eng.has_work():
        eng.step()
    return seqs, eng.runner.stats["steps"]


@pytest.mark.parametrize("mode", [True, False])
def test_scripted_outputs_identical_with_fewer_steps(mode):
    g = ToolCallGrammar([RET])
    calls = [format_tool_call(scripted_decision(q)) for q in
             ("What did I spend on groceries last month?", "Show me my recent transactions at Amazon.")]
    forced = [TOK.encode(c, allow_special=False) + [EOT] for c in calls] + [TOK.encode("No tool call", allow_special=False) + [EOT]]
    prompts = [list(range(300 + 11 * i, 360 + 11 * i)) for i in range(3)]
    plain = [SamplingParams(temperature=0.5, max_tokens=96, forced_output=f) for f in forced]
    jumped = [SamplingParams(temperature=0.5, max_tokens=96, forced_output=f,
                             forced_jump=jump_mask(f, TOK.decode, g, EOT), grammar=g) for f in forced]
    a, steps_a = _run(plain, prompts, mode)
    b, steps_b = _run(jumped, prompts, mode)
    for sa, sb, f in zip(a, b, forced):
        assert sa.output_ids == f and sb.output_ids == f
        assert sa.finish_reason == sb.finish_reason == "stop"
    free = max(sum(not x for x in jump_mask(f, TOK.decode, g, EOT)) for f in forced)
    assert steps_b < steps_a and steps_b <= free + 3


class _SuffixGrammar:
    """After the first sampled token the answer must continue with ' tool call' and end."""

    def forced(self, text):
        if text and not text.endswith(" tool call"):
            return " tool call", True
        return "", False


@pytest.mark.parametrize("mode", [True, False])
def test_sampled_output_gets_forced_run_appended(mode):
    prompt = list(range(500, 570))
    sp = SamplingParams(temperature=0.0, max_tokens=16, grammar=_SuffixGrammar())
    (seq,), steps = _run([sp], [prompt], mode)
    run = TOK.encode(" tool call", allow_special=False)
    assert seq.output_ids[1:] == run + [EOT] and seq.finish_reason == "stop"
    assert steps <= 3


@pytest.mark.parametrize("mode", [True, False])
def test_tokens_after_a_jump_chunk_match_plain_prefill(mode):
    """Greedy tokens sampled after a jump chunk == greedy continuation of a prompt that already
    contains those tokens (the chunk's KV/positions are right)."""
    run = TOK.encode(" the budget plan for", allow_special=False)

    class G:
        def __init__(self):
            self.fired = False

        def forced(self, text):
            if not self.fired and text:
                self.fired = True
                return " the budget plan for", False
            return "", False
    prompt = list(range(600, 690))
    sp = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True, grammar=G())
    (seq,), _ = _run([sp], [prompt], mode)
    out = seq.output_ids
    assert out[1:1 + len(run)] == run
    ref_prompt = prompt + out[:1 + len(run)]
    (ref,), _ = _run([SamplingParams(temperature=0.0, max_tokens=12 - 1 - len(run), ignore_eos=True)], [ref_prompt], mode)
    assert out[1 + len(run):] == ref.output_ids


def test_jump_run_tokenized_jointly_with_the_output(tmp_path):
    """With a real byte-level BPE (merges across '{"', '": "'), the staged jump run is exactly the
    tail of the JOINT encoding of output + forced text, and a non-canonical output (its tokens
    are not a prefix of that encoding) jumps nothing (advisor finding on _stage_grammar)."""
    from types import SimpleNamespace

    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
    from financial_chatbot_llm_amd.engine.tokenizer import HFTokenizer
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    corpus = ['{"name": "retrieve_transactions", "parameters": {"search_query": "groceries", "num_transactions": 20}}']
    tk.train_from_iterator(corpus * 300, trainers.BpeTrainer(vocab_size=420, special_tokens=["<|eot_id|>"],
                                                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    path = tmp_path / "tokenizer.json"
    tk.save(str(path))
    tok = HFTokenizer(str(path))
    eng = SimpleNamespace(tokenizer=tok, eos_ids=set(tok.eos_ids))
    g = ToolCallGrammar([RET])
    text = '{"'
    out = tok.encode(text, allow_special=False)
    seq = SimpleNamespace(params=SimpleNamespace(grammar=g, forced_output=None), output_ids=list(out), jump_queue=[])
    LLMEngine._stage_grammar(eng, seq)
    forced, _ = g.forced(text)
    assert forced and seq.jump_queue
    assert list(out) + seq.jump_queue == tok.encode(text + forced, allow_special=False)
    # non-canonical: '{' sampled alone where the joint encoding merges '{"' -> no jump
    brace = tok.encode("{", allow_special=False)
    joint = tok.encode("{" + g.forced("{")[0], allow_special=False)
    if joint[:len(brace)] != brace:
        seq2 = SimpleNamespace(params=seq.params, output_ids=list(brace), jump_queue=[1, 2])
        LLMEngine._stage_grammar(eng, seq2)
        assert seq2.jump_queue == []
