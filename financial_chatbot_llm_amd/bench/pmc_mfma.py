"""Per-kernel MFMA utilisation from a rocprofv3 ``--pmc`` counter CSV.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), summed over a
kernel's dispatches (GRBM_GUI_ACTIVE is the sum over the 8 XCDs: MI355X_MICROARCH.md 'DVFS give-back');
SQ_INSTS_VALU counts the MFMAs too (a GEMM whose loop holds ~0.3 non-MFMA VALU per MFMA reads 1.35),
so both SQ_INSTS_VALU / SQ_INSTS_MFMA ("valu_per_mfma", the r4 tables' figure) and
(SQ_INSTS_VALU - SQ_INSTS_MFMA) / SQ_INSTS_MFMA ("other_valu_per_mfma") are reported; wave-cycle
shares: SQ_WAIT_ANY (waitcnt / barrier), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY, of
SQ_WAVE_CYCLES; clock = GRBM_GUI_ACTIVE / 8 / wall.  Usage:

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
            "other_valu_per_mfma": ((c["SQ_INSTS_VALU"] - c["SQ_INSTS_MFMA"]) / c["SQ_INSTS_MFMA"]
                                    if c.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in c else None),
            **{f"share_{k[3:].lower()}": c[k] / c["SQ_WAVE_CYCLES"]
               for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")
               if k in c and c.get("SQ_WAVE_CYCLES")},
            "lds_util": (c["SQ_LDS_IDX_ACTIVE"] / (gui / 8 * 256) if c.get("SQ_LDS_IDX_ACTIVE") and gui else None),
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
        print("| kernel | dispatches | MFMA busy | VALU (incl. MFMA) / MFMA | other VALU / MFMA | clock GHz |")
        print("|---|---:|---:|---:|---:|---:|")
        for k, v in rows:
            ov = v["other_valu_per_mfma"]
            print(f"| `{k[:90]}` | {v['dispatches']} | {100 * v['mfma_busy']:.1f} % | {v['valu_per_mfma']:.2f} | "
                  f"{'-' if ov is None else f'{ov:.2f}'} | {v['clock_ghz']:.2f} |")
    else:
        for k, v in rows:
            print(k[:100], {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
