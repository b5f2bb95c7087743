#!/usr/bin/env python3
"""GPU timeline of a host-bound step from a rocprofv3 --kernel-trace csv: per step (a step starts at
each launch of `--first` kernel), the span from its first kernel's start to the next step's, the
kernels' busy time inside it, and the idle gaps before each kernel -- whether the GPU waits for the
host (gaps) or the host for the GPU (no gaps).
usage: python scripts/kernel_timeline.py <kernel_trace.csv> --first l1_pair_fwd [--skip 20] [--out f.json]"""

import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", required=True)
    ap.add_argument("--skip", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if args.first in r[2]]
    steps = []
    for a, b in zip(starts[args.skip:], starts[args.skip + 1:]):
        ks = rows[a:b]
        span = rows[b][0] - ks[0][0]
        busy = sum(e - s for s, e, _ in ks)
        gaps = [(ks[i][0] - ks[i - 1][1], ks[i][2][:48]) for i in range(1, len(ks))] + [(rows[b][0] - ks[-1][1], "->next")]
        steps.append((span, busy, gaps))
    if not steps:
        raise SystemExit("no complete steps found")
    res = {"steps": len(steps), "kernels_per_step": len(steps[0][2]),
           "span_us_median": statistics.median(s[0] for s in steps) / 1e3,
           "busy_us_median": statistics.median(s[1] for s in steps) / 1e3}
    per_gap = {}
    for _, _, gaps in steps:
        for i, (g, name) in enumerate(gaps):
            per_gap.setdefault((i, name), []).append(g)
    res["gap_before_us_median"] = [(name, round(statistics.median(v) / 1e3, 2)) for (i, name), v in sorted(per_gap.items())]
    txt = json.dumps(res, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
