"""Tool-calling agent: decide -> (retrieve) -> respond (reference llm_agent.py)."""
from .agent import AgentState, LLMAgent, initial_state
from .graph import END, StateGraph
from .llm import LLMBackend, LLMResult, StubLLM, scripted_decision
from .service import LLMService
from .toolcall import format_tool_call, parse_tool_calls, render_tools_block

__all__ = ["AgentState", "LLMAgent", "initial_state", "END", "StateGraph", "LLMBackend", "LLMResult", "LLMService",
           "StubLLM", "scripted_decision", "format_tool_call", "parse_tool_calls", "render_tools_block"]
