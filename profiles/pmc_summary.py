#!/usr/bin/env python3
"""Per-kernel pipe utilisation from the SQ counter passes of collect_pmc.sh.

Reads the counter_collection.csv of each pass (p1: wave-cycle breakdown and
MFMA busy cycles; p2: instruction mix and LDS bank conflicts; p3: more mix)
and prints / writes, per kernel (mean over its dispatches):

  mfma_busy     SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs):
                the fraction of the kernel's wall cycles the matrix pipes of
                the whole chip were busy (MI355X_MICROARCH.md: MFMA busy counts
                cycles, GRBM_GUI_ACTIVE is summed over the 8 XCDs);
  valu_per_mfma SQ_INSTS_VALU / SQ_INSTS_MFMA (wave instructions);
  lds_conflict  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (cycles lost per LDS
                instruction-cycle);
  wait_frac     SQ_WAIT_ANY / SQ_WAVE_CYCLES, valu_frac SQ_ACTIVE_INST_VALU /
                SQ_WAVE_CYCLES, lds_frac SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
                (all quad-cycle counters: the ratios are unit-free).

usage: python3 profiles/pmc_summary.py <pmc_dir> [out.json]
       (pmc_dir holds p1/, p2/, p3/ from profiles/collect_pmc.sh)
"""

import csv
import json
import os
import sys
from collections import defaultdict

from pmc_traffic import short_name

SIMDS = 256 * 4
XCDS = 8


def load(path):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
    per_disp = defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            key = (row["Dispatch_Id"], short_name(row["Kernel_Name"]))
            per_disp[key][row["Counter_Name"]] = per_disp[key].get(row["Counter_Name"], 0.0) + float(
                row["Counter_Value"])
    for (_, k), cs in per_disp.items():
        for c, v in cs.items():
            vals[k][c].append(v)
    return vals


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    merged = defaultdict(dict)
    for p in ("p1", "p2", "p3"):
        path = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for k, cs in load(path).items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
    rows = {}
    for k, c in merged.items():
        if k.startswith("__amd") or "elementwise" in k or "at::" in k:
            continue
        r = {}
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * g / XCDS), 4)
        if c.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"], 2)
        if c.get("SQ_ACTIVE_INST_LDS"):
            r["lds_conflict"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_ACTIVE_INST_LDS"], 4)
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for name, cnt in (("wait_frac", "SQ_WAIT_ANY"), ("valu_frac", "SQ_ACTIVE_INST_VALU"),
                              ("lds_frac", "SQ_ACTIVE_INST_LDS"), ("vmem_frac", "SQ_ACTIVE_INST_VMEM")):
                if cnt in c:
                    r[name] = round(c[cnt] / w, 4)
        r["counters"] = {n: round(v, 1) for n, v in sorted(c.items())}
        rows[k] = r
    order = sorted(rows, key=lambda k: -rows[k]["counters"].get("GRBM_GUI_ACTIVE", 0.0))
    for k in order:
        r = rows[k]
        print(f"{k[:48]:48s} mfma_busy={r.get('mfma_busy', '-')!s:7s} valu/mfma={r.get('valu_per_mfma', '-')!s:7s} "
              f"wait={r.get('wait_frac', '-')!s:7s} valu={r.get('valu_frac', '-')!s:7s} "
              f"lds={r.get('lds_frac', '-')!s:7s} ldsconf={r.get('lds_conflict', '-')}")
    if out:
        with open(out, "w") as f:
            json.dump({"source": f"rocprofv3 --kernel-trace --pmc passes p1/p2/p3 of profiles/collect_pmc.sh in {d}",
                       "kernels": {k: rows[k] for k in order}}, f, indent=1)


if __name__ == "__main__":
    main()
