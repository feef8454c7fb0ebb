#!/usr/bin/env python3
"""Per-step stage split of a bench.py run from a rocprofv3 kernel trace.

    python tools/step_breakdown.py RUN_kernel_trace.csv [--anchor NAME] [--last N] [--with NAME] [--json]

A step is the span from one launch of the anchor kernel (default: the query
preprocess, the first launch of every search) to the next one. For the last N
complete steps the tool reports, per kernel name, the mean duration and count
per step, the idle time between consecutive kernels on the device (the gaps),
and the step span; so "outside the main pass" = span - main pass is read off
directly. Kernels of the CPU-side setup (generate,
quantize) fall outside the steps and are ignored. --with NAME keeps only the
steps that launch a kernel whose short name contains NAME, --without NAME
drops those that do (bench.py's run
holds the main line's steps, then the secondary line's and the bf16_pass
line's: `--with true>` picks the int8 pass's, `mfma<768,0,2304,2,false,false>`
the bf16 pass's).
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    """vsk::mfma_topk_kernel<768, 0, 2304, 2, false, true>(...) -> mfma<768,0,2304,2,false,true>."""
    n = name.strip('"')
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "").replace("vsk::", "").replace("(anonymous namespace)::", "")
    n = n.replace("_kernel", "").replace("mfma_topk", "mfma").replace(" ", "")
    return n


def load(path):
    rows = []
    with open(path) as f:
        rd = csv.DictReader(f)
        for r in rd:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="query_prep")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--with", dest="with_", default=None)
    ap.add_argument("--without", default=None)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace)
    starts = [i for i, r in enumerate(rows) if r[2].startswith(a.anchor)]
    if len(starts) < 3:
        sys.exit(f"fewer than 3 anchors ({a.anchor}) in the trace")
    # steps: [starts[j], starts[j+1]); keep the last N complete ones
    spans = list(zip(starts[:-1], starts[1:]))
    if a.with_:
        spans = [(i0, i1) for i0, i1 in spans if any(a.with_ in r[2] for r in rows[i0:i1])]
    if a.without:
        spans = [(i0, i1) for i0, i1 in spans if not any(a.without in r[2] for r in rows[i0:i1])]
    spans = spans[-a.last:]
    if not spans:
        sys.exit("no complete step matches")
    per = defaultdict(lambda: [0.0, 0])
    gaps, span_ns = 0.0, 0.0
    for i0, i1 in spans:
        seg = rows[i0:i1]
        for j, (s, e, n) in enumerate(seg):
            per[n][0] += e - s
            per[n][1] += 1
            if j:
                gaps += max(0, s - seg[j - 1][1])
        span_ns += rows[i1][0] - rows[i0][0]
    ns = len(spans)
    out = {"steps": ns, "span_us": round(span_ns / ns / 1e3, 2),
           "idle_gaps_us": round(gaps / ns / 1e3, 2),
           "kernels": {n: {"us": round(v[0] / ns / 1e3, 2), "per_step": round(v[1] / ns, 2)}
                       for n, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    if a.json:
        print(json.dumps(out))
        return
    print(f"{ns} steps, span {out['span_us']} us/step, idle between kernels {out['idle_gaps_us']} us")
    for n, v in out["kernels"].items():
        print(f"  {v['us']:9.2f} us  x{v['per_step']:<5} {n}")


if __name__ == "__main__":
    main()
