"""Agent tools: transaction retrieval (on-device RAG) and financial plotting."""
from .base import Tool, ToolCall
from .plot import PlotConfig, create_financial_plot, make_plot_tool
from .retrieval import RetrievalIntent, make_retrieval_tool

__all__ = ["Tool", "ToolCall", "PlotConfig", "create_financial_plot", "make_plot_tool",
           "RetrievalIntent", "make_retrieval_tool"]
