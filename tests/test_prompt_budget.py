"""Token-budget policy, memoised chat encoding and streaming detokenisation."""
import asyncio
import time

import pytest

from financial_chatbot_llm_amd.engine.chat_template import ChatEncoder, clamp_transactions, encode_chat, render
from financial_chatbot_llm_amd.engine.tokenizer import HFTokenizer, IncrementalDetokenizer, SyntheticLlamaTokenizer
from financial_chatbot_llm_amd.retrieval.store import synthetic_payload
from financial_chatbot_llm_amd.wire import AIMessage, ChatMessage, HumanMessage

TOK = SyntheticLlamaTokenizer()


def _history(turns):
    out = []
    for t in range(turns):
        out.append(HumanMessage(f"Question number {t}: how much did I spend on groceries last month?"))
        out.append(AIMessage(f"Answer {t}: " + "you spent a reasonable amount on food and dining " * 12))
    return out


def _msgs(turns, system="The current date is 2026-10-15.\nYou are Penny.\nMy name is Ada."):
    hist = _history(turns)
    return [ChatMessage("system", system), *hist, HumanMessage("What about rent?")]


def test_piecewise_encoding_equals_whole_render():
    msgs = _msgs(6)
    enc = ChatEncoder(TOK)
    assert enc.encode(msgs) == TOK.encode(render(msgs))
    assert enc.encode(msgs) == TOK.encode(render(msgs))          # memoised path, same ids


def test_history_cut_is_quantised_and_prefix_stable():
    enc = ChatEncoder(TOK, history_quantum=8)
    prev_cut, changes, prompts = None, 0, []
    for turns in range(10, 40):
        ids = enc.encode(_msgs(turns), max_prompt_tokens=4096)
        assert len(ids) <= 4096
        prompts.append(ids)
        cut = enc.last.dropped_messages
        assert cut % 8 == 0
        if prev_cut is not None and cut != prev_cut:
            changes += 1
        prev_cut = cut
    # history grows by 2 messages/turn: the cut moves at most once every 4 turns
    assert 0 < changes <= 30 // 4 + 1
    # between moves the previous prompt (minus its generation header) is a prefix of the next
    tail = len(enc.encode([HumanMessage("What about rent?")])) - 1        # final user turn + gen header
    stable = sum(prompts[i + 1][:len(prompts[i]) - tail] == prompts[i][:-tail] for i in range(len(prompts) - 1))
    assert stable >= 29 - changes


def test_system_and_query_kept_and_generation_header_never_cut():
    huge = "The current date is 2026-10-15.\nPenny.\nRetrieved Transaction Data:\n" + "\n".join(
        synthetic_payload(i, "u", 1_700_000_000 + i)["page_content"] for i in range(3000))
    msgs = _msgs(50, system=huge)
    enc = ChatEncoder(TOK)
    ids = enc.encode(msgs, max_prompt_tokens=8000)
    assert len(ids) <= 8000
    gen = list(enc.ids("<|start_header_id|>assistant<|end_header_id|>\n\n"))
    assert ids[-len(gen):] == gen
    text = TOK.decode(ids, skip_special=False)
    assert text.startswith("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\nThe current date is")
    assert "What about rent?<|eot_id|>" in text
    assert enc.last.dropped_messages == 100 and enc.last.trimmed_system > 0


def test_no_budget_pressure_keeps_everything():
    msgs = _msgs(5)
    assert encode_chat(TOK, msgs, max_prompt_tokens=8191) == TOK.encode(render(msgs))
    assert encode_chat(TOK, msgs, history_token_budget=10) != TOK.encode(render(msgs))


def test_ten_thousand_hits_and_long_history_stay_fast():
    """num_transactions=None -> 10,000 hits; a 50-turn history; the event loop is not blocked >50 ms."""
    hits = [synthetic_payload(i, "u", 1_700_000_000 + i)["page_content"] for i in range(10_000)]
    enc = ChatEncoder(TOK)
    history = _history(50)
    enc.encode([ChatMessage("system", "warm"), *history, HumanMessage("q")])    # history seen last turn
    t0 = time.perf_counter()
    kept = clamp_transactions(hits, 3000, enc.count)
    system = "The current date is 2026-10-15.\n\nPenny\nMy name is Ada.\n\nRetrieved Transaction Data:\n" + "\n".join(kept)
    ids = enc.encode([ChatMessage("system", system), *history, HumanMessage("q")], max_prompt_tokens=8191 - 513)
    dt = time.perf_counter() - t0
    assert len(ids) <= 8191 - 513 and 0 < len(kept) < len(hits)
    assert sum(enc.count(t) + 1 for t in kept) <= 3000
    assert dt < 0.05, f"encode blocked the loop for {dt * 1e3:.1f} ms"


def _tiny_bpe(tmp_path, metaspace=False):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE(unk_token=None if not metaspace else "<unk>"))
    if metaspace:
        tk.pre_tokenizer = pre_tokenizers.Metaspace()
        tk.decoder = decoders.Metaspace()
        tr = trainers.BpeTrainer(vocab_size=200, special_tokens=["<unk>", "<|eot_id|>"])
    else:
        tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
        tk.decoder = decoders.ByteLevel()
        tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|begin_of_text|>", "<|eot_id|>"],
                                 initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["hello world this is a test of the budget"] * 10, tr)
    path = tmp_path / "tokenizer.json"
    tk.save(str(path))
    return HFTokenizer(str(path))


@pytest.mark.parametrize("metaspace", [False, True])
def test_hf_incremental_detokenizer_streams_exact_text(tmp_path, metaspace):
    tok = _tiny_bpe(tmp_path, metaspace)
    text = "hello world this is a test" if metaspace else "héllo 😀 world 日本 test"
    ids = tok.encode(text)
    detok = IncrementalDetokenizer(tok)
    pieces = [detok.push([i]) for i in ids] + [detok.flush()]
    assert "".join(pieces) == tok.decode(ids)
    assert not any("�" in p for p in pieces)
