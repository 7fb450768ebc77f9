"""Tokenizers for the local models (no network: real vocab files are optional).

* :class:`HFTokenizer` -- wraps a ``tokenizer.json`` (``tokenizers`` library) when one is
  provided (``PENNY_TOKENIZER``), e.g. the real Llama-3 BPE.
* :class:`SyntheticLlamaTokenizer` -- offline stand-in with Llama-3's id layout: 256 byte
  tokens, a word-level vocabulary up to id 127999 (every pre-token of the bundled prompts and
  tool schemas plus deterministic pseudo-words, so prompts tokenize at a realistic ~1 token per
  word), and the Llama-3 special tokens at 128000+.  It is a bijection id <-> bytes, so any id
  a random-weight model samples decodes to text, and encode/decode round-trips.
* :class:`SyntheticWordPiece` -- hashed word-piece ids in BERT's 30522 vocab for the bge encoder.
* :class:`IncrementalDetokenizer` -- emits only complete UTF-8 text for streaming.
"""
from __future__ import annotations

import hashlib
import os
from functools import lru_cache
from typing import Dict, Iterable, List, Optional, Sequence

import regex as re

# Llama-3 style pre-tokenizer (tiktoken cl100k-like)
PRETOKEN = re.compile(
    r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")

LLAMA3_SPECIAL = {
    "<|begin_of_text|>": 128000,
    "<|end_of_text|>": 128001,
    "<|reserved_special_token_0|>": 128002,
    "<|reserved_special_token_1|>": 128003,
    "<|finetune_right_pad_id|>": 128004,
    "<|reserved_special_token_2|>": 128005,
    "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007,
    "<|eom_id|>": 128008,
    "<|eot_id|>": 128009,
    "<|python_tag|>": 128010,
}

_SYLL = ["ka", "lo", "mi", "ne", "ru", "sa", "ti", "vo", "ze", "pa", "qu", "ra", "be", "do", "fi", "gu",
         "ha", "jo", "ke", "li", "mo", "nu", "pe", "ri", "so", "ta", "ve", "wi", "xa", "yo", "zu", "an",
         "el", "in", "on", "un", "ar", "er", "ir", "or"]


class BaseTokenizer:
    bos_id: int
    eos_ids: Sequence[int]
    vocab_size: int
    special: Dict[str, int]

    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> List[int]:
        raise NotImplementedError

    def decode_bytes(self, ids: Iterable[int]) -> bytes:
        raise NotImplementedError

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        ids = [i for i in ids if not (skip_special and i in self._special_ids)]
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    @property
    def _special_ids(self) -> set:
        return set(self.special.values())

    def token_id(self, s: str) -> int:
        return self.special[s]


@lru_cache(maxsize=1)
def _seed_words() -> List[str]:
    """Pre-tokens from the bundled prompts and schemas: common text tokenizes to words."""
    from ..prompts import load_prompt
    texts = [load_prompt("penny_persona.prompt"), load_prompt("retrieval_decision.prompt")]
    extra = ("The current date is My name is I make dollars a month I want to save Here is a list of my "
             "current account balances recurring monthly expenses Name Amount Description Retrieved Transaction "
             "Data Date Merchant Category Groceries Gas Entertainment Dining Transportation Shopping Utilities "
             "Rent Health Fitness Travel Insurance Transfer Checking Savings Credit Card USD system user "
             "assistant ipython Environment function name parameters description type object properties string "
             "integer null default minimum maximum anyOf retrieve_transactions search_query num_transactions "
             "time_period_days user_id What did spend on How much should invest for retirement grocery store "
             "purchases all recent transactions week last days ago Thanks Based your data plan")
    texts.append(extra)
    seen, out = set(), []
    for t in texts:
        for m in PRETOKEN.findall(t):
            for w in (m, m.strip(), " " + m.strip()):
                if w and w not in seen and len(w.encode()) > 1:
                    seen.add(w)
                    out.append(w)
    return out


class SyntheticLlamaTokenizer(BaseTokenizer):
    WORD_LO = 256

    def __init__(self, vocab_size: int = 128256):
        # Llama-3 puts its 256 special tokens at the top of the vocab (128000..128255); smaller
        # vocabs (Mixtral's 32000) get the same special strings at vocab_size - 256.
        self.vocab_size = vocab_size
        base = vocab_size - 256
        self.special = {k: base + (v - 128000) for k, v in LLAMA3_SPECIAL.items()}
        for j in range(256 - 11):
            self.special[f"<|reserved_special_token_{3 + j}|>"] = base + 11 + j
        self.WORD_HI = base
        self.bos_id = self.special["<|begin_of_text|>"]
        self.eos_ids = (self.special["<|eot_id|>"], self.special["<|end_of_text|>"])
        self._id_to_bytes: List[bytes] = [bytes([i]) for i in range(256)]
        self._word_to_id: Dict[str, int] = {}
        hi = self.WORD_HI
        words = _seed_words()
        n_syl = len(_SYLL)
        k = 0
        for i in range(self.WORD_LO, hi):
            if k < len(words):
                w = words[k]
                k += 1
            else:
                j, parts = i, []
                while True:
                    parts.append(_SYLL[j % n_syl])
                    j //= n_syl
                    if j == 0:
                        break
                w = " " + "".join(parts)
                while w in self._word_to_id:
                    w = w + "x"
            self._word_to_id[w] = i
            self._id_to_bytes.append(w.encode("utf-8"))
        self._special_by_id = {v: k for k, v in self.special.items()}
        specials = sorted(self.special, key=len, reverse=True)
        self._special_re = re.compile("(" + "|".join(re.escape(s) for s in specials) + ")") if specials else None

    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> List[int]:
        ids: List[int] = [self.bos_id] if add_bos else []
        pieces = self._special_re.split(text) if (allow_special and self._special_re) else [text]
        for piece in pieces:
            if not piece:
                continue
            sid = self.special.get(piece) if allow_special else None
            if sid is not None:
                ids.append(sid)
                continue
            for m in PRETOKEN.findall(piece):
                wid = self._word_to_id.get(m)
                if wid is not None:
                    ids.append(wid)
                    continue
                stripped = m.lstrip(" ")
                if m != stripped and self._word_to_id.get(stripped) is not None and m.startswith(" "):
                    ids.extend(m[: len(m) - len(stripped)].encode())
                    ids.append(self._word_to_id[stripped])
                    continue
                ids.extend(m.encode("utf-8"))
        return ids

    def decode_bytes(self, ids: Iterable[int]) -> bytes:
        out = bytearray()
        for i in ids:
            i = int(i)
            if i < len(self._id_to_bytes):
                out += self._id_to_bytes[i]
            elif i in self._special_by_id:
                out += self._special_by_id[i].encode()
        return bytes(out)


class HFTokenizer(BaseTokenizer):
    def __init__(self, path: str):
        from tokenizers import Tokenizer
        self.tk = Tokenizer.from_file(path)
        self.vocab_size = self.tk.get_vocab_size(with_added_tokens=True)
        vocab = self.tk.get_vocab(with_added_tokens=True)
        self.special = {t: i for t, i in vocab.items() if t.startswith("<|") and t.endswith("|>")}
        self.bos_id = self.special.get("<|begin_of_text|>", vocab.get("<s>", 1))
        eos = [self.special.get("<|eot_id|>"), self.special.get("<|end_of_text|>"), vocab.get("</s>")]
        self.eos_ids = tuple(i for i in eos if i is not None)

    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> List[int]:
        ids = self.tk.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] + ids) if add_bos else ids

    def decode_bytes(self, ids: Iterable[int]) -> bytes:
        return self.tk.decode(list(ids), skip_special_tokens=False).encode("utf-8")

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        return self.tk.decode(list(ids), skip_special_tokens=skip_special)


class SyntheticWordPiece:
    """BERT-vocab ids by hashing lower-cased words (no vocab file offline)."""

    CLS, SEP, PAD, UNK = 101, 102, 0, 100
    _WORD = re.compile(r"\p{L}+|\p{N}+|[^\s\p{L}\p{N}]")

    def __init__(self, vocab_size: int = 30522):
        self.vocab_size = vocab_size

    def _wid(self, w: str) -> int:
        h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=4).digest(), "little")
        return 1000 + h % (self.vocab_size - 1000)

    def encode(self, text: str, max_len: int = 512) -> List[int]:
        ids = [self._wid(w) for w in self._WORD.findall(text.lower())][: max_len - 2]
        return [self.CLS] + ids + [self.SEP]

    def encode_batch(self, texts: Sequence[str], max_len: int = 512) -> List[List[int]]:
        return [self.encode(t, max_len) for t in texts]


class WordPieceTokenizer:
    """Real BERT WordPiece (``tokenizers``, Rust) from a ``vocab.txt`` or a ``tokenizer.json`` --
    what bge-base-en ships.  ``[CLS] pieces [SEP]``, truncated to ``max_len`` WITH the ``[SEP]``
    kept (BERT's truncation); ``encode_batch`` tokenises in parallel outside the GIL."""

    def __init__(self, path: str, lowercase: bool = True):
        from tokenizers import Tokenizer
        if path.endswith(".json"):
            self.tk = Tokenizer.from_file(path)
        else:
            from tokenizers import BertWordPieceTokenizer
            self.tk = BertWordPieceTokenizer(path, lowercase=lowercase)
        vocab = self.tk.get_vocab()
        self.vocab_size = self.tk.get_vocab_size()
        self.CLS, self.SEP = vocab.get("[CLS]", 101), vocab.get("[SEP]", 102)
        self.PAD, self.UNK = vocab.get("[PAD]", 0), vocab.get("[UNK]", 100)
        self._max = None

    def _truncate(self, max_len: int) -> None:
        if self._max != max_len:
            self.tk.enable_truncation(max_len)
            self._max = max_len

    def encode(self, text: str, max_len: int = 512) -> List[int]:
        self._truncate(max_len)
        return self.tk.encode(text).ids

    def encode_batch(self, texts: Sequence[str], max_len: int = 512) -> List[List[int]]:
        self._truncate(max_len)
        return [e.ids for e in self.tk.encode_batch(list(texts))]


def load_wordpiece(path: Optional[str] = None, vocab_size: int = 30522):
    """Real WordPiece when a vocab/tokenizer file is given (``PENNY_EMBED_VOCAB``), else hashed ids."""
    path = path or os.environ.get("PENNY_EMBED_VOCAB")
    if path and os.path.exists(path):
        return WordPieceTokenizer(path)
    return SyntheticWordPiece(vocab_size)


class IncrementalDetokenizer:
    """Turns a growing list of token ids into text deltas without splitting characters.

    Byte-level vocabularies (the synthetic one): buffer bytes, emit the longest valid UTF-8
    prefix.  ``tokenizers`` vocabularies (:class:`HFTokenizer`): decoding a token on its own is
    wrong twice over -- a character split across byte-level BPE tokens decodes to U+FFFD, and a
    Metaspace/SentencePiece decoder drops a lone token's leading space.  So keep every id and
    decode a sliding window ``ids[prefix:]`` against ``ids[prefix:read]`` (the window already
    emitted); emit the new suffix only once it does not end in an incomplete character."""

    def __init__(self, tokenizer: BaseTokenizer, skip_special: bool = True):
        self.tk = tokenizer
        self.skip = tokenizer._special_ids if skip_special else set()
        self.pending = b""
        self.ids: List[int] = []
        self.prefix = 0          # window start: context tokens re-decoded for spacing
        self.read = 0            # tokens whose text has been emitted

    def _push_hf(self, ids: Iterable[int]) -> str:
        self.ids.extend(i for i in ids if i not in self.skip)
        done = self.tk.decode(self.ids[self.prefix:self.read], skip_special=True)
        full = self.tk.decode(self.ids[self.prefix:], skip_special=True)
        if len(full) > len(done) and not full.endswith("\ufffd"):
            self.prefix, self.read = self.read, len(self.ids)
            return full[len(done):]
        return ""

    def push(self, ids: Iterable[int]) -> str:
        if isinstance(self.tk, HFTokenizer):
            return self._push_hf(ids)
        self.pending += self.tk.decode_bytes(i for i in ids if i not in self.skip)
        # emit the longest valid UTF-8 prefix
        for cut in range(len(self.pending), max(len(self.pending) - 4, -1), -1):
            try:
                text = self.pending[:cut].decode("utf-8")
            except UnicodeDecodeError:
                continue
            self.pending = self.pending[cut:]
            return text
        text = self.pending.decode("utf-8", errors="replace")
        self.pending = b""
        return text

    def flush(self) -> str:
        if isinstance(self.tk, HFTokenizer):
            done = self.tk.decode(self.ids[self.prefix:self.read], skip_special=True)
            full = self.tk.decode(self.ids[self.prefix:], skip_special=True)
            self.prefix = self.read = len(self.ids)
            return full[len(done):]
        text = self.pending.decode("utf-8", errors="replace")
        self.pending = b""
        return text


def load_tokenizer(path: Optional[str] = None, vocab_size: int = 128256) -> BaseTokenizer:
    path = path or os.environ.get("PENNY_TOKENIZER")
    if path and os.path.exists(path):
        return HFTokenizer(path)
    return SyntheticLlamaTokenizer(vocab_size)
