"""Typed configuration for the MI355X-native Penny serving stack.

Wire-level names (env vars, Kafka topics, Mongo collections) are kept identical to the
reference so a deployment can switch without touching its environment:

* Kafka: ``KAFKA_SERVER``/``KAFKA_USERNAME``/``KAFKA_PASSWORD`` -> SASL_SSL+PLAIN when both
  credentials are set, PLAINTEXT otherwise (reference ``config.py:8-23``); topics
  ``user_message``/``ai_response`` and group ``message_consumer`` (``config.py:26-28``).
* Mongo: ``MONGODB_URI``, collections ``contexts``/``messages`` (``config.py:31-33``).
* Model keys kept for compatibility (``config.py:36-47``) although every model now runs
  locally on the GPU; ``QDRANT_COLLECTION_NAME`` names the on-device corpus.

Engine knobs (model, TP degree, KV block size, graph buckets, retrieval corpus, ...) are
new; each has a ``PENNY_*`` env override.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .utils.env import load_dotenv

load_dotenv()

# --------------------------------------------------------------------------------------
# Wire-compatible constants (reference config.py:26-47)
# --------------------------------------------------------------------------------------
USER_MESSAGE_TOPIC = "user_message"
AI_RESPONSE_TOPIC = "ai_response"
GROUP_ID = "message_consumer"
MONGO_DATABASE_NAME = "conversations"
CONTEXT_COLLECTION_NAME = "contexts"
MESSAGE_COLLECTION_NAME = "messages"
QDRANT_COLLECTION_NAME = "transactions"

# Reference operating parameters
MESSAGE_TIMEOUT_S = 100.0          # main.py:138
IDLE_SLEEP_S = 0.01                # main.py:156
LOOP_ERROR_BACKOFF_S = 1.0         # main.py:157-159
KAFKA_POLL_TIMEOUT_S = 0.1         # kafka_client.py:47
KAFKA_SESSION_TIMEOUT_MS = "45000"  # kafka_client.py:15
DEFAULT_TEMPERATURE = 0.5          # llm_agent.py:37,44
RETRIEVAL_DEFAULT_LIMIT = 10000    # tools/qdrant_tool.py:145
RETRIEVAL_HNSW_EF = 128            # tools/qdrant_tool.py:99 (we search exactly; kept for API parity)
MAX_TRANSACTION_TOKENS = 3000      # token-budget clamp of stuffed transactions (new)


def _env(name: str, default: str = "") -> str:
    return os.getenv(name, default)


def _env_int(name: str, default: int) -> int:
    v = os.getenv(name)
    return int(v) if v not in (None, "") else default


def _env_float(name: str, default: float) -> float:
    v = os.getenv(name)
    return float(v) if v not in (None, "") else default


def _env_bool(name: str, default: bool) -> bool:
    v = os.getenv(name)
    if v in (None, ""):
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def build_kafka_config() -> Dict[str, str]:
    """librdkafka config dict with the reference's SASL/PLAINTEXT switch (config.py:8-23)."""
    cfg: Dict[str, str] = {"bootstrap.servers": _env("KAFKA_SERVER", "")}
    user, pw = _env("KAFKA_USERNAME", ""), _env("KAFKA_PASSWORD", "")
    if user and pw:
        cfg.update({
            "security.protocol": "SASL_SSL",
            "sasl.mechanisms": "PLAIN",
            "sasl.username": user,
            "sasl.password": pw,
        })
    else:
        cfg["security.protocol"] = "PLAINTEXT"
    return cfg


KAFKA_CONFIG = build_kafka_config()
MONGODB_URI = _env("MONGODB_URI", "")
OPENAI_KEY = _env("OPENAI_API_KEY", "")
OPENAI_MODEL_NAME = _env("OPENAI_MODEL_NAME", "")
OPENAI_EMBEDDINGS_MODEL_NAME = _env("OPENAI_EMBEDDINGS_MODEL_NAME", "")
GEMINI_KEY = _env("GEMINI_API_KEY", "")
GEMINI_MODEL_NAME = _env("GEMINI_MODEL", "")
QDRANT_URL = _env("QDRANT_URL", "")
QDRANT_API_KEY = _env("QDRANT_API_KEY", "")


# --------------------------------------------------------------------------------------
# Engine configuration (new)
# --------------------------------------------------------------------------------------
@dataclass
class EngineConfig:
    """Knobs for one inference-engine replica (one TP group)."""

    model: str = "llama3-8b"                # registry key in models.configs
    dtype: str = "bf16"
    moe_parallel: str = "tp"                # Mixtral under TP: "tp" (FFN-sharded experts) | "ep" (all-to-all)
    sequence_parallel: bool = False         # TP prefills >= 1024 rows: reduce-scatter/all-gather (Megatron SP)
    async_scheduling: bool = True           # overlap host scheduling of step N+1 with GPU step N
    custom_all_reduce: bool = True          # TP decode all-reduces on the one-shot xGMI P2P kernel
    custom_ar_self_test: bool = True        # init-time check of the custom kernels vs the exact sum
    step_ring: bool = True                  # C4 step broadcast over the node-local shm ring (else gloo)
    tp_dual_decode: bool = False            # TP graph decode as two micro-batch chains on two streams (opt-in until an 8-GPU A/B exists)
    weights: Optional[str] = None           # safetensors dir; None -> random init
    tokenizer: Optional[str] = None         # tokenizer.json; None -> built-in synthetic vocab
    tp_size: int = 1
    # estimate mode (bench.py --tp-shard-estimate N): build only the rank-0 shard of a TP=N group on
    # this one device, its collectives identity -- the per-rank compute of a TP step, measured
    shard_of_tp: int = 0
    # context parallelism (SURVEY §5.7 stretch): cp_size ranks, each with the full weights, form one
    # replica; its leader serves, and a prompt with >= cp_min_tokens uncomputed tokens is prefilled
    # by all of them at once (zig-zag shards, ring attention over xGMI), its K/V gathered into the
    # leader's paged pool (engine/context_prefill.py)
    cp_size: int = 1
    cp_min_tokens: int = 16384
    cp_layers_per_step: int = 4             # CP prefill layers run per engine step (decode in between)
    kv_block_size: int = 64                 # tokens per KV block (one MFMA KV tile)
    # of (free HBM after weights - 6 GiB); 0.92 leaves ~20 GiB of the 288 GiB unused at the end of
    # the 20/5 bench (engine stats hbm_used_gib: 8B 264.5, Mixtral fp8 267.9; 0.95 measured no
    # faster: profiles/r2_bench_kv_fraction.txt)
    kv_mem_fraction: float = 0.92
    num_kv_blocks: Optional[int] = None     # explicit override (tests)
    max_num_seqs: int = 256                 # running-batch cap
    max_num_batched_tokens: int = 4096      # per-step token budget (chunked prefill; measured best: profiles/r1_sweep_max_batched_tokens.txt)
    max_model_len: int = 8192
    step_token_quantum: int = 256           # step rows rounded down to a multiple (prefill GEMM M)
    sched_aging_s: float = 1.0              # a waiting long-output request joins the priority class after this
    # step-time bound (TTFT): while a short-output request (the agent's decide call) is decoding,
    # cap each step's prefill tokens so the step's modelled device time stays under this (ms;
    # 0 = off).  Cost model: base + per decode row + per prefill token (engine/scheduler.py)
    step_time_target_ms: float = 0.0
    step_cost_ms: tuple = (3.0, 0.07, 0.013)
    # burst drain: steps take up to this many prefill tokens while the oldest pending prefill's turn
    # has waited >= sched_burst_age_s (0 = off)
    sched_burst_tokens: int = 0
    sched_burst_age_s: float = 0.5
    # short-job-first admission: waiting prompts with <= this many uncached tokens are admitted before
    # the continuing chunks of long prefills (0 = off)
    sched_sjf_tokens: int = 0
    sched_sjf_step_cap: int = 0             # tokens per step the short-first pass may take (0: all)
    # per-step reservation for waiting short-output (decide) prompts against continuing long
    # prefills (engine/scheduler.py; 0 = off)
    sched_short_reserve_tokens: int = 0
    # admission order: short-output (decide) prompts ahead of aged long-output ones (scheduler.py)
    sched_short_first: bool = False
    enable_prefix_caching: bool = True
    # (a shared-prefix "cascade" decode attention was built in r1 and removed in r5: the lean
    # split-K decode grid already reads a shared prefix ~once from L2/MALL, and the extra launch +
    # partials only paid at very high sharing, profiles/r1_decode_cascade.jsonl)
    use_cuda_graph: bool = True             # hipGraph capture of decode steps
    graph_batch_sizes: Tuple[int, ...] = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 256)
    seed: int = 0
    device: str = "cuda"
    step_timeout_s: float = 60.0            # GPU-step watchdog

    @classmethod
    def from_env(cls, **overrides) -> "EngineConfig":
        c = cls(
            model=_env("PENNY_MODEL", cls.model),
            dtype=_env("PENNY_DTYPE", cls.dtype),
            weights=os.getenv("PENNY_WEIGHTS") or None,
            tokenizer=os.getenv("PENNY_TOKENIZER") or None,
            tp_size=_env_int("PENNY_TP", cls.tp_size),
            cp_size=_env_int("PENNY_CP", cls.cp_size),
            cp_min_tokens=_env_int("PENNY_CP_MIN_TOKENS", cls.cp_min_tokens),
            kv_block_size=_env_int("PENNY_KV_BLOCK", cls.kv_block_size),
            kv_mem_fraction=_env_float("PENNY_KV_FRACTION", cls.kv_mem_fraction),
            max_num_seqs=_env_int("PENNY_MAX_SEQS", cls.max_num_seqs),
            max_num_batched_tokens=_env_int("PENNY_MAX_BATCHED_TOKENS", cls.max_num_batched_tokens),
            max_model_len=_env_int("PENNY_MAX_MODEL_LEN", cls.max_model_len),
            step_token_quantum=_env_int("PENNY_STEP_TOKEN_QUANTUM", cls.step_token_quantum),
            sched_aging_s=_env_float("PENNY_SCHED_AGING_S", cls.sched_aging_s),
            step_time_target_ms=_env_float("PENNY_STEP_TIME_TARGET_MS", cls.step_time_target_ms),
            sched_burst_tokens=_env_int("PENNY_BURST_TOKENS", cls.sched_burst_tokens),
            sched_burst_age_s=_env_float("PENNY_BURST_AGE_S", cls.sched_burst_age_s),
            sched_sjf_tokens=_env_int("PENNY_SJF_TOKENS", cls.sched_sjf_tokens),
            sched_sjf_step_cap=_env_int("PENNY_SJF_STEP_CAP", cls.sched_sjf_step_cap),
            sched_short_reserve_tokens=_env_int("PENNY_SHORT_RESERVE", cls.sched_short_reserve_tokens),
            sched_short_first=bool(_env_int("PENNY_SHORT_FIRST", int(cls.sched_short_first))),
            enable_prefix_caching=_env_bool("PENNY_PREFIX_CACHE", True),
            moe_parallel=_env("PENNY_MOE_PARALLEL", cls.moe_parallel),
            sequence_parallel=_env_bool("PENNY_SEQUENCE_PARALLEL", False),
            async_scheduling=_env_bool("PENNY_ASYNC_SCHEDULING", True),
            custom_all_reduce=_env_bool("PENNY_CUSTOM_AR", True),
            step_ring=_env_bool("PENNY_STEP_RING", True),
            custom_ar_self_test=_env_bool("PENNY_AR_SELF_TEST", True),
            tp_dual_decode=_env_bool("PENNY_TP_DUAL_DECODE", False),
            use_cuda_graph=_env_bool("PENNY_HIPGRAPH", True),
            device=_env("PENNY_DEVICE", cls.device),
        )
        return dataclasses.replace(c, **overrides)


@dataclass
class RetrievalConfig:
    embed_model: str = "bge-base-en"
    corpus_size: int = 1_000_000
    num_users: int = 10_000
    max_limit_tokens: int = MAX_TRANSACTION_TOKENS   # clamp of stuffed transactions
    weights: Optional[str] = None           # bge safetensors dir (None: random init)
    vocab: Optional[str] = None             # BERT vocab.txt / tokenizer.json (None: hashed word ids)
    corpus_path: Optional[str] = None       # JSONL/Parquet transactions or a store snapshot to load
    device: str = "cuda"

    @classmethod
    def from_env(cls, **overrides) -> "RetrievalConfig":
        c = cls(
            embed_model=_env("PENNY_EMBED_MODEL", cls.embed_model),
            corpus_size=_env_int("PENNY_CORPUS_SIZE", cls.corpus_size),
            num_users=_env_int("PENNY_CORPUS_USERS", cls.num_users),
            max_limit_tokens=_env_int("PENNY_MAX_TRANSACTION_TOKENS", cls.max_limit_tokens),
            weights=os.getenv("PENNY_EMBED_WEIGHTS") or None,
            vocab=os.getenv("PENNY_EMBED_VOCAB") or None,
            corpus_path=os.getenv("PENNY_CORPUS_PATH") or None,
            device=_env("PENNY_DEVICE", cls.device),
        )
        return dataclasses.replace(c, **overrides)


@dataclass
class ServingConfig:
    host: str = "0.0.0.0"
    port: int = 8000
    max_concurrent_turns: int = 256         # replaces the reference's 1-turn-per-worker
    message_timeout_s: float = MESSAGE_TIMEOUT_S
    temperature: float = DEFAULT_TEMPERATURE
    max_response_tokens: int = 512
    max_decide_tokens: int = 96
    # history beyond this many tokens is cut oldest-first in prefix-stable steps;
    # None: only what max_model_len forces (the reference re-sends the whole history)
    history_token_budget: Optional[int] = None
    backend: str = "engine"                 # "engine" | "stub"
    tools: bool = True                      # False: legacy single-chain chat, no decide step (A9)
    # POST /v1/transactions is only served when an operator token is configured, and every call
    # must present it (Authorization: Bearer <token>); unset = the write path does not exist
    ingest_token: Optional[str] = None

    @classmethod
    def from_env(cls, **overrides) -> "ServingConfig":
        c = cls(
            port=_env_int("PORT", cls.port),
            max_concurrent_turns=_env_int("PENNY_MAX_CONCURRENT_TURNS", cls.max_concurrent_turns),
            max_response_tokens=_env_int("PENNY_MAX_RESPONSE_TOKENS", cls.max_response_tokens),
            max_decide_tokens=_env_int("PENNY_MAX_DECIDE_TOKENS", cls.max_decide_tokens),
            history_token_budget=(_env_int("PENNY_HISTORY_TOKEN_BUDGET", 0) or None),
            backend=_env("PENNY_BACKEND", cls.backend),
            tools=_env_bool("PENNY_TOOLS", True),
            ingest_token=_env("PENNY_INGEST_TOKEN", "") or None,
        )
        return dataclasses.replace(c, **overrides)


from .utils.logging import get_logger  # noqa: E402  (re-export, reference config.py:49)

logger = get_logger(__name__)

__all__ = [
    "USER_MESSAGE_TOPIC", "AI_RESPONSE_TOPIC", "GROUP_ID", "MONGO_DATABASE_NAME",
    "CONTEXT_COLLECTION_NAME", "MESSAGE_COLLECTION_NAME", "QDRANT_COLLECTION_NAME",
    "KAFKA_CONFIG", "MONGODB_URI", "EngineConfig", "RetrievalConfig", "ServingConfig",
    "build_kafka_config", "get_logger",
]
