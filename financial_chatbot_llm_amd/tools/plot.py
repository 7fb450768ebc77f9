"""``create_financial_plot`` tool (reference ``tools/plot_tool.py:9-78``).

Dormant in the reference (never bound); live here for the multi-step agent config.  Same
contract: a JSON string of transactions + a :class:`PlotConfig`; chart kinds line (optional
per-group lines), bar (optional group-by sum), pie (optional group-by sum, ``%1.1f%%``),
scatter, histogram (30 bins) on a 10x6 figure; returns ``data:image/png;base64,...`` or
``"Error creating plot: ..."``.
"""
from __future__ import annotations

import base64
import io
import json
import threading
from typing import Any, Dict, Literal, Optional, Union

from pydantic import BaseModel, Field

from .base import Tool

_MPL_LOCK = threading.Lock()  # pyplot's global state is not thread-safe


class PlotConfig(BaseModel):
    plot_type: Literal["line", "bar", "pie", "scatter", "histogram"] = Field(description="Type of plot to create")
    x_axis: str = Field(description="Column for x-axis")
    y_axis: Optional[str] = Field(default=None, description="Column for y-axis")
    title: str = Field(description="Plot title")
    group_by: Optional[str] = Field(default=None, description="Column to group by")


class PlotArgs(BaseModel):
    transactions_json: str = Field(description="JSON string of transaction data")
    plot_config: PlotConfig = Field(description="Configuration for the plot including type, axes, and grouping")


PLOT_TOOL_DESCRIPTION = (
    "Create visualizations of financial data.\n\nArgs:\n    transactions_json: JSON string of transaction data\n"
    "    plot_config: Configuration for the plot including type, axes, and grouping\n\n"
    "Returns:\n    Base64 encoded plot image"
)


def _draw(df, cfg: PlotConfig, plt) -> None:
    kind, x, y, g = cfg.plot_type, cfg.x_axis, cfg.y_axis, cfg.group_by
    if kind == "line":
        if g:
            for key, part in df.groupby(g, sort=False):
                plt.plot(part[x], part[y], label=key)
            plt.legend()
        else:
            plt.plot(df[x], df[y])
    elif kind == "bar":
        if g and y:
            df.groupby(g)[y].sum().plot(kind="bar")
        else:
            df.plot(kind="bar", x=x, y=y)
    elif kind == "pie":
        if g and y:
            sums = df.groupby(g)[y].sum()
            plt.pie(sums, labels=[str(i) for i in sums.index], autopct="%1.1f%%")
        else:
            plt.pie(df[y], labels=df[x].astype(str).tolist(), autopct="%1.1f%%")
    elif kind == "scatter":
        plt.scatter(df[x], df[y])
    elif kind == "histogram":
        plt.hist(df[x], bins=30)


def create_financial_plot(transactions_json: str, plot_config: Union[PlotConfig, Dict[str, Any]]) -> str:
    try:
        import matplotlib
        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt
        import pandas as pd

        cfg = plot_config if isinstance(plot_config, PlotConfig) else PlotConfig.model_validate(plot_config)
        df = pd.read_json(io.StringIO(transactions_json))
        with _MPL_LOCK:
            plt.figure(figsize=(10, 6))
            try:
                _draw(df, cfg, plt)
                plt.title(cfg.title)
                plt.tight_layout()
                buf = io.BytesIO()
                plt.savefig(buf, format="png")
            finally:
                plt.close()
        return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode("utf-8")
    except Exception as e:  # noqa: BLE001 - reference returns the error string
        return f"Error creating plot: {e}"


def _invoke(transactions_json: str, plot_config: Dict[str, Any]) -> str:
    if isinstance(transactions_json, (list, dict)):
        transactions_json = json.dumps(transactions_json)
    return create_financial_plot(transactions_json, plot_config)


async def _ainvoke(transactions_json: str, plot_config: Dict[str, Any]) -> str:
    # matplotlib rendering takes tens of ms of CPU: off the serving event loop
    import asyncio
    return await asyncio.to_thread(_invoke, transactions_json, plot_config)


def make_plot_tool() -> Tool:
    return Tool(name="create_financial_plot", description=PLOT_TOOL_DESCRIPTION,
                args_schema=PlotArgs, func=_invoke, coroutine=_ainvoke)
