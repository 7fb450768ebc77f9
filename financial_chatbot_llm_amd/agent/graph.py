"""A small async state machine standing in for LangGraph's ``StateGraph`` (``llm_agent.py:57-79``).

Nodes are async callables ``state -> state``; edges are static or conditional (router
returns a label mapped to the next node).  ``compile()`` validates the wiring and returns a
runnable with ``ainvoke(state)``.  No checkpointer, exactly like the reference.
"""
from __future__ import annotations

import inspect
from typing import Any, Awaitable, Callable, Dict, Optional

END = "__end__"


class StateGraph:
    def __init__(self):
        self.nodes: Dict[str, Callable[[Any], Any]] = {}
        self.edges: Dict[str, str] = {}
        self.cond: Dict[str, tuple] = {}
        self.entry: Optional[str] = None

    def add_node(self, name: str, fn: Callable[[Any], Any]) -> None:
        if name in self.nodes or name == END:
            raise ValueError(f"duplicate node {name}")
        self.nodes[name] = fn

    def set_entry_point(self, name: str) -> None:
        self.entry = name

    def add_edge(self, src: str, dst: str) -> None:
        self.edges[src] = dst

    def add_conditional_edges(self, src: str, router: Callable[[Any], str], mapping: Dict[str, str]) -> None:
        self.cond[src] = (router, dict(mapping))

    def compile(self) -> "CompiledGraph":
        if self.entry not in self.nodes:
            raise ValueError("entry point not set")
        for s, d in self.edges.items():
            if s not in self.nodes or (d != END and d not in self.nodes):
                raise ValueError(f"bad edge {s}->{d}")
        for s, (_, m) in self.cond.items():
            for d in m.values():
                if d != END and d not in self.nodes:
                    raise ValueError(f"bad conditional edge {s}->{d}")
        return CompiledGraph(self)


class CompiledGraph:
    def __init__(self, g: StateGraph, max_steps: int = 64):
        self.g, self.max_steps = g, max_steps

    async def ainvoke(self, state: Any, trace: Optional[list] = None) -> Any:
        node = self.g.entry
        for _ in range(self.max_steps):
            if node == END:
                return state
            if trace is not None:
                trace.append(node)
            res = self.g.nodes[node](state)
            if inspect.isawaitable(res):
                res = await res
            state = res if res is not None else state
            if node in self.g.cond:
                router, mapping = self.g.cond[node]
                node = mapping[router(state)]
            else:
                node = self.g.edges.get(node, END)
        raise RuntimeError("graph did not terminate")
