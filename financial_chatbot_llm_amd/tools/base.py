"""Minimal tool abstraction replacing LangChain's ``@tool`` (reference ``tools/*.py``).

A :class:`Tool` has a name, a description (the docstring the LLM sees), a pydantic argument
model whose JSON schema becomes the function declaration, and a callable.  ``invoke(dict)``
validates the arguments the way LangChain's ``args_schema`` does, then calls the function.
"""
from __future__ import annotations

import inspect
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable, Dict, Optional, Type

from pydantic import BaseModel


@dataclass
class ToolCall:
    name: str
    args: Dict[str, Any]
    id: str = ""

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "args": dict(self.args), "id": self.id}


@dataclass
class Tool:
    name: str
    description: str
    args_schema: Type[BaseModel]
    func: Callable[..., Any]
    coroutine: Optional[Callable[..., Awaitable[Any]]] = None

    def parameters_schema(self) -> Dict[str, Any]:
        schema = self.args_schema.model_json_schema()
        schema.pop("title", None)
        for p in schema.get("properties", {}).values():
            p.pop("title", None)
        return schema

    def function_declaration(self) -> Dict[str, Any]:
        """OpenAI/Llama-3.1 style ``{"type":"function","function":{...}}`` declaration."""
        return {"type": "function", "function": {
            "name": self.name, "description": self.description,
            "parameters": self.parameters_schema()}}

    def validate(self, args: Dict[str, Any]) -> Dict[str, Any]:
        model = self.args_schema.model_validate(args or {})
        return model.model_dump()

    def invoke(self, args: Dict[str, Any]) -> Any:
        return self.func(**self.validate(args))

    async def ainvoke(self, args: Dict[str, Any]) -> Any:
        kwargs = self.validate(args)
        if self.coroutine is not None:
            return await self.coroutine(**kwargs)
        res = self.func(**kwargs)
        if inspect.isawaitable(res):
            res = await res
        return res
