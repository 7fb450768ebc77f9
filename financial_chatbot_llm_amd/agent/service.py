"""Legacy single-chain chat service (reference ``llm_service.py:8-33``; BASELINE config 2).

The reference builds ``prompt | gemini`` over ``[system "{system_prompt}\\n{context}",
*history, user "{input}"]`` at temperature 0.5 and returns the chain's chunk stream -- no tool
binding, no decide call, no date line (the caller passes ``SYSTEM_PROMPT`` verbatim,
``main.py:15-16``).  It is instantiated but never called upstream (``main.py:21``); here it is
live as the ``tools=False`` serving mode (``PENNY_TOOLS=0``) and ``bench.py --no-tools``.

:meth:`stream_with_status` yields the agent's event vocabulary (``status`` / ``response_chunk`` /
``complete``), so :class:`~..serving.worker.ChatWorker` drives either object unchanged.
"""
from __future__ import annotations

from typing import Any, AsyncGenerator, AsyncIterator, Dict, Optional, Sequence

from .. import config
from ..prompts import system_prompt as _load_system_prompt
from ..utils.logging import get_logger
from ..wire import ChatMessage, build_messages
from .llm import LLMBackend

logger = get_logger(__name__)


class LLMService:
    def __init__(self, llm: LLMBackend, system_prompt: Optional[str] = None,
                 temperature: float = config.DEFAULT_TEMPERATURE, max_response_tokens: int = 512):
        self.llm = llm
        self.system_prompt = system_prompt if system_prompt is not None else _load_system_prompt()
        self.temperature = temperature
        self.max_response_tokens = max_response_tokens

    def messages(self, message: str, context: str, chat_history: Sequence[ChatMessage],
                 system_prompt: Optional[str] = None):
        return build_messages(self.system_prompt if system_prompt is None else system_prompt,
                              context, chat_history, message)

    async def process_message(self, message: str, context: str, chat_history: Sequence[ChatMessage],
                              system_prompt: Optional[str] = None) -> AsyncIterator[str]:
        """Chunk stream of one reply (``llm_service.py:21-30``; async here, sync upstream)."""
        try:
            return self.llm.astream(self.messages(message, context, chat_history, system_prompt),
                                    temperature=self.temperature, max_tokens=self.max_response_tokens,
                                    purpose="respond")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error streaming LLM response: {e}")
            raise

    async def stream_with_status(self, user_query: str, user_id: str, user_context: str = "",
                                 chat_history: Sequence[ChatMessage] = ()) -> AsyncGenerator[Dict[str, Any], None]:
        yield {"type": "status", "message": "Generating response..."}
        stream = await self.process_message(user_query, user_context, chat_history)
        async for piece in stream:
            if piece:
                yield {"type": "response_chunk", "content": piece}
        yield {"type": "complete", "message": "Query processing completed"}

    async def query(self, user_query: str, user_id: str, user_context: str = "",
                    chat_history: Sequence[ChatMessage] = ()) -> Dict[str, Any]:
        parts = []
        async for upd in self.stream_with_status(user_query, user_id, user_context, chat_history):
            if upd["type"] == "response_chunk":
                parts.append(upd["content"])
        return {"response": "".join(parts), "retrieved_transactions_count": 0, "state": None}
