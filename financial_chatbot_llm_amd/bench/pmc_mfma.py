"""Per-kernel MFMA utilisation from a rocprofv3 ``--pmc`` counter CSV.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), summed over a
kernel's dispatches (GRBM_GUI_ACTIVE is the sum over the 8 XCDs: MI355X_MICROARCH.md 'DVFS give-back');
VALU / MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA; clock = GRBM_GUI_ACTIVE / 8 / wall.  Usage:

    python -m financial_chatbot_llm_amd.bench.pmc_mfma counters.csv [--match prefill2] [--md]
"""
from __future__ import annotations

import argparse
import collections
import csv
import re
from typing import Dict


def short(name: str) -> str:
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([\w:]+)(<[^()]*>)?", name)
    base = m.group(1) if m else name[:60]
    return base + (m.group(2) if m and m.group(2) else "")


def summarise(path: str, match: str = "") -> Dict[str, Dict[str, float]]:
    acc: Dict[str, Dict[str, float]] = collections.defaultdict(lambda: collections.defaultdict(float))
    disp: Dict[str, set] = collections.defaultdict(set)
    wall: Dict[str, Dict[str, float]] = collections.defaultdict(dict)
    with open(path, newline="") as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if match and match not in name:
                continue
            k = short(name)
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
            wall[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, c in acc.items():
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        simd_cycles = gui / 8 * 1024
        w = sum(wall[k].values())
        out[k] = {
            "dispatches": len(disp[k]),
            "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles if simd_cycles else 0.0,
            "valu_per_mfma": c.get("SQ_INSTS_VALU", 0.0) / max(c.get("SQ_INSTS_MFMA", 0.0), 1.0),
            "clock_ghz": gui / 8 / w / 1e9 if w else 0.0,
            "lds_bank_conflict_ratio": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                                        if c.get("SQ_LDS_IDX_ACTIVE") else None),
            **{kk: v for kk, v in c.items()},
        }
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="")
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args(argv)
    res = summarise(a.csv, a.match)
    rows = sorted(res.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0.0))
    if a.md:
        print("| kernel | dispatches | MFMA busy | VALU / MFMA | clock GHz |")
        print("|---|---:|---:|---:|---:|")
        for k, v in rows:
            print(f"| `{k[:90]}` | {v['dispatches']} | {100 * v['mfma_busy']:.1f} % | {v['valu_per_mfma']:.2f} | "
                  f"{v['clock_ghz']:.2f} |")
    else:
        for k, v in rows:
            print(k[:100], {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
