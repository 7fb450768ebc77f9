"""Deterministic-continuation oracle for the decide step's output language (jump-forward decoding).

The decide call (reference ``llm_agent.py:87-93``, tool bound at ``:38``) answers either with the
literal ``No tool call`` (``tool_prompt.txt:1-13``) or with one function call in the canonical
Llama-3.1 JSON layout ``{"name": NAME, "parameters": {KEY: VALUE, ...}}`` (``json.dumps``
separators, keys from the bound tools' JSON schemas).  Under that grammar many characters are
FORCED -- after ``{`` the text ``"name": "`` is the only legal continuation, with one bound tool
the name is forced too, a key is forced once its prefix is unambiguous, ``", "parameters": {``
follows every name, ``}`` closes the call and the answer must end there.

:meth:`ToolCallGrammar.forced` returns that forced continuation for an output prefix.  The
engine appends the forced tokens without sampling and computes them as one prefill chunk in the
next step (jump-forward decoding, as grammar-constrained servers do): the KV of every output
token is still computed by the model, but a run of forced tokens costs one forward pass instead
of one per token.  Free choices (tool vs. no tool, which key, every value character) are still
decoded one token per step.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence, Tuple

NO_CALL = "No tool call"
_OPEN = '{"name": "'
_MID = '", "parameters": {'


def _string_only(schema: Dict) -> bool:
    if schema.get("type") == "string":
        return True
    return False


class ToolCallGrammar:
    def __init__(self, tools: Sequence):
        self.props: Dict[str, Dict[str, Dict]] = {}
        for t in tools:
            schema = t.parameters_schema() if hasattr(t, "parameters_schema") else t
            name = t.name if hasattr(t, "name") else schema["name"]
            self.props[name] = dict(schema.get("properties", {}))

    # ------------------------------------------------------------------------------------
    def forced(self, text: str) -> Tuple[str, bool]:
        """(forced continuation of ``text``, must-end-after-it).  ``("", False)``: the next
        character is a free choice (or ``text`` is outside the grammar -- never force then)."""
        if not text:
            return "", False
        if text[0] != "{":
            if NO_CALL.startswith(text):
                return NO_CALL[len(text):], True
            return "", False
        if len(text) < len(_OPEN):
            return (_OPEN[len(text):], False) if _OPEN.startswith(text) else ("", False)
        rest = text[len(_OPEN):]
        # --- tool name -------------------------------------------------------------------
        q = rest.find('"')
        if q < 0:
            cands = [n for n in self.props if n.startswith(rest)]
            if len(cands) == 1:
                return cands[0][len(rest):] + _MID, False
            return "", False
        name, rest = rest[:q], rest[q:]
        if name not in self.props:
            return "", False
        if len(rest) < len(_MID):
            return (_MID[len(rest):], False) if _MID.startswith(rest) else ("", False)
        return self._params(self.props[name], rest[len(_MID):])

    def _params(self, props: Dict[str, Dict], s: str) -> Tuple[str, bool]:
        used: List[str] = []
        i, n = 0, len(s)
        first = True
        while True:
            if i == n:
                return "", False                      # '"' (a key) or '}' -- a choice
            c = s[i]
            if c == "}":
                tail = s[i + 1:]
                return ("}"[len(tail):], True) if "}".startswith(tail) else ("", False)
            if c == ",":
                if first:
                    return "", False
                if i + 1 == n:
                    return ' "', False
                if s[i + 1:i + 3] != ' "'[: len(s[i + 1:i + 3])]:
                    return "", False
                if i + 3 > n:
                    return ' "'[n - i - 1:], False
                i += 3
            elif c == '"' and first:
                i += 1
            else:
                return "", False
            first = False
            # --- key -----------------------------------------------------------------------
            q = s.find('"', i)
            avail = [k for k in props if k not in used]
            if q < 0:
                part = s[i:]
                cands = [k for k in avail if k.startswith(part)]
                if len(cands) == 1:
                    k = cands[0]
                    return k[len(part):] + '": ' + ('"' if _string_only(props[k]) else ""), False
                return "", False
            key = s[i:q]
            if key not in avail:
                return "", False
            used.append(key)
            sep = '": ' + ('"' if _string_only(props[key]) else "")
            got = s[q:q + len(sep)]
            if len(got) < len(sep):
                return (sep[len(got):], False) if sep.startswith(got) else ("", False)
            if got != sep:
                return "", False
            i = q + len(sep)
            # --- value (free text; skip it) -------------------------------------------------
            if _string_only(props[key]):
                j = i
                while j < n and s[j] != '"':
                    j += 2 if s[j] == "\\" else 1
                if j >= n:
                    return "", False                  # inside the string
                i = j + 1
            else:
                try:
                    _, end = json.JSONDecoder().raw_decode(s, i)
                except json.JSONDecodeError:
                    return "", False                  # inside a number / null / literal
                if end >= n:
                    return "", False                  # the value may still grow ("2" -> "20")
                i = end


def jump_mask(tokens: Sequence[int], decode, grammar: ToolCallGrammar, eos: Optional[int]) -> List[bool]:
    """``mask[k]``: output token k is forced by the grammar given tokens[:k] (k=0 never is).

    ``decode(ids) -> str``.  Token k is forced when its text is a non-empty prefix of the forced
    continuation, or when it is ``eos`` and the grammar requires the answer to end there."""
    mask = [False] * len(tokens)
    text = ""
    for k, tok in enumerate(tokens):
        if k > 0:
            forced, ends = grammar.forced(text)
            if eos is not None and tok == eos:
                mask[k] = ends and forced == ""
            else:
                piece = decode([tok])
                mask[k] = bool(piece) and bool(forced) and forced.startswith(piece)
        if eos is None or tok != eos:
            text += decode([tok])
    return mask
