"""Summarise a ``rocprofv3 --kernel-trace --stats`` run into a markdown table for ``profiles/``.

    python -m financial_chatbot_llm_amd.bench.profsum gpurun_out/prof/run_kernel_stats.csv \\   # or run_results.db
        --title "bench.py default" --top 30 > profiles/r1_bench128_kernel_stats.md

Kernels are also bucketed into coarse classes (GEMM / attention / norm+elementwise / sampling /
retrieval / copies) so the per-step budget is visible at a glance.
"""
from __future__ import annotations

import argparse
import bisect
import csv
import re
from collections import defaultdict

CLASSES = [
    ("gemm-prefill tile (HIP)", r"gemm_prefill_kernel|gemm_mid_kernel"),
    ("attention-decode", r"decode_kernel|decode_reduce|decode_lean"),
    ("attention-prefill", r"prefill_kernel|prefill2_kernel|prefill3_kernel|prefill_merge"),
    ("gemm-skinny (HIP)", r"skinny"),
    ("gemm-splitk (HIP)", r"splitk"),
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


def utilisation(trace_csv: str) -> str:
    """GPU busy time (union of kernel intervals) over the traced span -- what the host leaves idle."""
    iv = []
    with open(trace_csv) as fh:
        for r in csv.DictReader(fh):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    busy, (cs, ce) = 0, iv[0]
    for s_, e_ in iv[1:]:
        if s_ > ce:
            busy += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    busy += ce - cs
    span = iv[-1][1] - iv[0][0]
    return f"GPU busy {busy / 1e9:.2f} s of a {span / 1e9:.2f} s traced span ({100 * busy / span:.1f} %).\n"


def gaps(trace_csv: str, top: int = 12) -> str:
    """Where the idle time of the traced span sits: every gap of the kernel-interval union, binned by
    length, and attributed to the (kernel class before -> kernel class after) transition.  Short gaps
    (< 5 us) are kernel boundaries; long ones are the host not having launched the next kernel yet
    (launch-bound stretches, step turnarounds)."""
    iv = []
    with open(trace_csv) as fh:
        for r in csv.DictReader(fh):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    iv.sort()
    bins = [(2e3, "< 2 us"), (5e3, "2-5 us"), (20e3, "5-20 us"), (100e3, "20-100 us"), (1e6, "0.1-1 ms"),
            (float("inf"), "> 1 ms")]
    by_bin = defaultdict(lambda: [0, 0.0])
    by_pair = defaultdict(lambda: [0, 0.0])
    ce, cname = iv[0][1], iv[0][2]
    for s_, e_, n in iv[1:]:
        if s_ > ce:
            g = s_ - ce
            lab = next(lbl for lim, lbl in bins if g < lim)
            by_bin[lab][0] += 1
            by_bin[lab][1] += g
            k = (classify(cname), classify(n))
            by_pair[k][0] += 1
            by_pair[k][1] += g
        if e_ >= ce:
            ce, cname = e_, n
    out = ["| idle gap | count | total s |", "|---|---:|---:|"]
    for _, lbl in bins:
        c, t = by_bin.get(lbl, (0, 0.0))
        out.append(f"| {lbl} | {c} | {t / 1e9:.3f} |")
    out += ["", "| previous kernel -> next kernel | gaps | total s | mean us |", "|---|---:|---:|---:|"]
    for (a, b), (c, t) in sorted(by_pair.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"| {a} -> {b} | {c} | {t / 1e9:.3f} | {t / max(c, 1) / 1e3:.1f} |")
    return "\n".join(out) + "\n"


def _ranges(marker_csv: str):
    """roctx ranges of a rocprofv3 --marker-trace CSV: {thread: sorted [(start, end, name)]}."""
    by_t = defaultdict(list)
    with open(marker_csv) as fh:
        for r in csv.DictReader(fh):
            s_, e_ = int(r.get("Start_Timestamp") or 0), int(r.get("End_Timestamp") or 0)
            name = r.get("Function") or r.get("Operation") or r.get("Name") or "?"
            if e_ > s_:
                by_t[r.get("Thread_Id", "0")].append((s_, e_, name))
    for v in by_t.values():
        v.sort()
    return by_t


def _innermost(rs, starts, maxdur, t):
    """Shortest range of one thread's sorted ranges containing time t (None: outside all)."""
    i = bisect.bisect_right(starts, t) - 1
    best = None
    while i >= 0 and starts[i] >= t - maxdur:
        s_, e_, n = rs[i]
        if e_ >= t and (best is None or e_ - s_ < best[1] - best[0]):
            best = (s_, e_, n)
        i -= 1
    return best


def gaps_by_marker(trace_csv: str, marker_csv: str, min_us: float = 100.0, top: int = 16) -> str:
    """Attribute every GPU idle gap >= min_us to what the host threads were doing at its midpoint:
    the innermost roctx range (PENNY_MARKERS=1) of the engine thread (the one issuing
    ``engine.step``) and of any other thread active then (serving loop, retrieval)."""
    iv = []
    with open(trace_csv) as fh:
        for r in csv.DictReader(fh):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    gaps = []
    ce = iv[0][1]
    for s_, e_ in iv[1:]:
        if s_ - ce >= min_us * 1e3:
            gaps.append((ce, s_))
        ce = max(ce, e_)
    by_t = _ranges(marker_csv)
    eng = next((t for t, rs in by_t.items() if any(n.startswith("engine.step") for _, _, n in rs)), None)
    idx = {t: ([x[0] for x in rs], max(e_ - s_ for s_, e_, _ in rs)) for t, rs in by_t.items()}
    norm = lambda n: re.sub(r"\[\d+\]", "[n]", n)  # noqa: E731
    eng_tab = defaultdict(lambda: [0, 0.0])
    oth_tab = defaultdict(lambda: [0, 0.0])
    for gs, ge in gaps:
        mid = (gs + ge) // 2
        d = ge - gs
        lab = "(engine thread outside every range)"
        if eng is not None:
            hit = _innermost(by_t[eng], idx[eng][0], idx[eng][1], mid)
            if hit is not None:
                lab = norm(hit[2])
        eng_tab[lab][0] += 1
        eng_tab[lab][1] += d
        others = sorted({norm(h[2]) for t, rs in by_t.items() if t != eng
                         for h in [_innermost(rs, idx[t][0], idx[t][1], mid)] if h is not None})
        k = (lab, ", ".join(others) or "-")
        oth_tab[k][0] += 1
        oth_tab[k][1] += d
    tot = sum(ge - gs for gs, ge in gaps)
    out = [f"GPU idle gaps >= {min_us:.0f} us: {len(gaps)}, {tot / 1e9:.3f} s", "",
           "| engine thread in | gaps | total s | mean us |", "|---|---:|---:|---:|"]
    for k, (c, t) in sorted(eng_tab.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"| {k} | {c} | {t / 1e9:.3f} | {t / max(c, 1) / 1e3:.1f} |")
    out += ["", "| engine thread in | other threads in | gaps | total s |", "|---|---|---:|---:|"]
    for (a, b), (c, t) in sorted(oth_tab.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"| {a} | {b} | {c} | {t / 1e9:.3f} |")
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--trace", default="", help="kernel_trace.csv: also report GPU busy fraction")
    ap.add_argument("--markers", default="", help="marker_api_trace.csv (with --trace): idle gaps by host range")
    a = ap.parse_args(argv)
    text = summarise(a.csv, a.title, a.top)
    if a.trace:
        head, rest = text.split("\n\n", 1)
        extra = gaps_by_marker(a.trace, a.markers) + "\n" if a.markers else ""
        text = head + "\n\n" + utilisation(a.trace) + "\n" + gaps(a.trace) + "\n" + extra + rest
    print(text, end="")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
