"""Summarise a ``rocprofv3 --kernel-trace --stats`` run into a markdown table for ``profiles/``.

    python -m financial_chatbot_llm_amd.bench.profsum gpurun_out/prof/run_kernel_stats.csv \\   # or run_results.db
        --title "bench.py default" --top 30 > profiles/r1_bench128_kernel_stats.md

Kernels are also bucketed into coarse classes (GEMM / attention / norm+elementwise / sampling /
retrieval / copies) so the per-step budget is visible at a glance.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

CLASSES = [
    ("attention-decode", r"decode_kernel|decode_reduce"),
    ("attention-prefill", r"prefill_kernel"),
    ("gemm-skinny (HIP)", r"skinny"),
    ("moe (HIP)", r"moe_|quant_rows"),
    ("gemm (hipBLASLt)", r"^Cijk|^Custom_Cijk|gemm"),
    ("norm/rope/act (HIP)", r"rmsnorm|layernorm|rope_kv|silu_mul|gelu|embedding"),
    ("sampling (HIP)", r"sample"),
    ("retrieval (HIP)", r"score_kernel|select_kernel|filter_compact|topk"),
    ("torch elementwise/copy", r"at::native|elementwise|copy|Fill|reduce"),
]


def classify(name: str) -> str:
    for cls, pat in CLASSES:
        if re.search(pat, name):
            return cls
    return "other"


def summarise(path: str, title: str, top: int) -> str:
    rows = []
    if path.endswith(".db"):   # rocpd sqlite (rocprofv3's default output format)
        import sqlite3
        con = sqlite3.connect(path)
        for n, c, ns in con.execute("select name, count(*), sum(duration) from kernels group by name"):
            rows.append((n, int(c), float(ns) / 1e6))
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6))
    total = sum(r[2] for r in rows) or 1.0
    calls = sum(r[1] for r in rows)
    out = [f"# rocprofv3 --kernel-trace --stats: {title}", "",
           f"Total GPU kernel time {total:.1f} ms over {calls} dispatches.", "",
           "| class | total ms | % |", "|---|---:|---:|"]
    by = defaultdict(float)
    for n, _, ms in rows:
        by[classify(n)] += ms
    for cls, ms in sorted(by.items(), key=lambda kv: -kv[1]):
        out.append(f"| {cls} | {ms:.1f} | {100 * ms / total:.1f} |")
    out += ["", "| total ms | % | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for n, c, ms in sorted(rows, key=lambda r: -r[2])[:top]:
        out.append(f"| {ms:.1f} | {100 * ms / total:.1f} | {c} | {1e3 * ms / max(c, 1):.1f} | `{n[:90]}` |")
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv)
    print(summarise(a.csv, a.title, a.top), end="")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
