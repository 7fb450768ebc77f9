"""Prompt-lookup speculative decoding (draft-model-free).

The agent's decide call mostly COPIES from its prompt: the tool call's ``search_query`` repeats
the user's question (``/root/reference/tool_prompt.txt:15-23`` few-shot, ``llm_agent.py:87-93``),
and a plot call repeats column names of the retrieved rows.  Every copied token would otherwise
cost one full engine step on the TTFT-critical path.

Proposal: the most recent earlier occurrence of the sequence's last n tokens (n = 3, 2, 1) in
prompt + output; the tokens that followed it are the draft (up to ``k``).  Longer n-grams win
unless a shorter one occurs more than ``recency`` tokens later (the user's latest message sits at
the end of the prompt, the few-shot examples thousands of tokens above it).  Verification: the
draft is appended after the next token and computed as ONE chunk whose last ``len(draft) + 1``
positions are all sampled; draft token i is accepted while it equals the token the model sampled
at the position before it, and the first mismatch's sample is the bonus token.  The output is
exactly what one-token-per-step decoding would produce with the same per-position seeds
(``Sequence.step_seed_at``); rejected draft positions leave stale KV beyond ``num_computed`` that
the next chunk overwrites.
"""
from __future__ import annotations

from typing import List, Sequence as Seq

import numpy as np


class PromptLookup:
    """n-gram draft source over one sequence's prompt + output.  The prompt is indexed once as a
    numpy array; each proposal is a vectorised match of the last token plus a check of the n-1
    tokens before it (~20 us on a 7k-token prompt)."""

    def __init__(self, prompt_ids: Seq[int], max_ngram: int = 3, min_ngram: int = 1, recency: int = 0):
        self.prompt = np.asarray(prompt_ids, dtype=np.int64)
        self.max_ngram = max_ngram
        self.min_ngram = min_ngram
        self.recency = recency

    def propose(self, output_ids: Seq[int], k: int, min_ngram: int = 0) -> List[int]:
        if k <= 0:
            return []
        ids = np.concatenate([self.prompt, np.asarray(output_ids, dtype=np.int64)]) if output_ids else self.prompt
        L = len(ids)
        best_e, best_n = -1, 0
        for n in range(min(self.max_ngram, L - 1), max(min_ngram, self.min_ngram) - 1, -1):
            pat = ids[L - n:]
            # candidate ends: earlier positions e (< L - 1) with ids[e] == last token
            ends = np.flatnonzero(ids[:L - 1] == pat[-1])
            ends = ends[ends >= n - 1]
            for back in range(1, n):
                if not len(ends):
                    break
                ends = ends[ids[ends - back] == pat[-1 - back]]
            if len(ends) and ends[-1] + 1 < L - 1:
                e = int(ends[-1])              # most recent occurrence of this n-gram
                if not self.recency:
                    best_e, best_n = e, n
                    break
                # recency: a shorter n-gram wins if it occurs later by more than `recency` tokens
                if best_e < 0 or e > best_e + self.recency:
                    best_e, best_n = e, n
        if best_e < 0:
            return []
        return ids[best_e + 1:best_e + 1 + k].tolist()


def accept_draft(draft: Seq[int], model_tokens: Seq[int]) -> int:
    """Number of leading draft tokens equal to the model's own tokens at those positions
    (``model_tokens[i]`` is the model's token where ``draft[i]`` sits)."""
    j = 0
    for d, t in zip(draft, model_tokens):
        if d != t:
            break
        j += 1
    return j
