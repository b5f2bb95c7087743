#!/usr/bin/env python3
"""HBM traffic per launch, by kernel, from rocprofv3 PMC passes.

Reads the counter_collection.csv of a FETCH_SIZE pass and of a WRITE_SIZE pass
(they cannot share one pass: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2, of 4)
and writes profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM / rocprofv3 section):
  - FETCH_SIZE and WRITE_SIZE are in KiB;
  - on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide coalesced
    streaming read (TCC_EA0_RDREQ x 64 B for 128-B requests): doubled here;
  - WRITE_SIZE is exact for 16-B-per-lane streaming stores: taken as is.
Infinity-Cache hits are counted by these counters, so re-reads served on-die
still show up as traffic.

usage: python3 profiles/pmc_traffic.py <fetch_pass.csv> <write_pass.csv> [source-label] [out.json]
"""

import csv
import json
import os
import sys
from collections import defaultdict


def short_name(kname: str) -> str:
    """rocprofv3 kernel name -> the name the library's launch records use."""
    n = kname.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("mmf::(anonymous namespace)::", "")
    # drop the trailing "(arg types)"
    depth = 0
    for i in range(len(n) - 1, -1, -1):
        if n[i] == ")":
            depth += 1
        elif n[i] == "(":
            depth -= 1
            if depth == 0:
                return n[:i]
    return n


def per_kernel(path: str, counter: str) -> dict:
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                vals[short_name(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return vals


def main() -> None:
    fetch_csv, write_csv = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else f"{fetch_csv} + {write_csv}"
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        rd = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wr = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {
            "dispatches": max(len(f), len(w)),
            "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": (rd or 0.0) + (wr or 0.0) if (rd is not None and wr is not None) else None,
        }
    dst = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump({"source": label,
                   "method": "FETCH_SIZE*2 (gfx950) + WRITE_SIZE, KiB->B, mean over dispatches",
                   "kernels": out}, fh, indent=1, sort_keys=True)
    print(f"wrote {dst}: {len(out)} kernels")


if __name__ == "__main__":
    main()
