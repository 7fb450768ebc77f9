"""Local inference engine: tokenizer, chat template, paged KV + prefix cache, continuous
batching scheduler, model runner with hipGraph decode, async front-end."""
from .llm_engine import LLMEngine, StepOutput
from .sequence import SamplingParams, Sequence

__all__ = ["LLMEngine", "StepOutput", "SamplingParams", "Sequence"]
