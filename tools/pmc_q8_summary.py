"""Summarise tools/pmc_q8.sh's counter passes: per arm, each counter's mean per
dispatch of mfma_topk_kernel, and the wave-cycle split the guide defines
(MI355X_MICROARCH.md, rocprofv3 PMC slots: WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES, disjoint; SQ_* cycle counters in quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES in cycles).

    python tools/pmc_q8_summary.py [gpurun_out] > profiles/r05_pmc_q8.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    arms = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "pmcq8_*_p*", "**", "*counter_collection.csv"),
                                 recursive=True)):
        arm = os.path.relpath(path, root).split(os.sep)[0][len("pmcq8_"):].rsplit("_p", 1)[0]
        rows = [r for r in csv.DictReader(open(path)) if "mfma_topk_kernel" in r["Kernel_Name"]]
        # the arm's kernel: the most dispatched one (the setup's sample pass is another)
        n = defaultdict(set)
        for r in rows:
            n[r["Kernel_Name"]].add(r["Dispatch_Id"])
        kern = max(n, key=lambda x: len(n[x]))
        per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
        for r in rows:
            if r["Kernel_Name"] == kern:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in per.values():
            for ctr, v in d.items():
                arms[arm][ctr].append(v)
    out = {}
    for arm, ctrs in arms.items():
        m = {c: sum(v) / len(v) for c, v in ctrs.items()}
        o = {"dispatches": max(len(v) for v in ctrs.values()), "mean": m}
        if "FETCH_SIZE" in m:
            o["fetch_bytes"] = m["FETCH_SIZE"] * 1024  # FETCH_SIZE counts KiB
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # MFMA busy per SIMD-cycle: busy cycles over 1024 SIMDs x the
            # per-XCD GUI cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
            o["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            o["split_of_wave_cycles"] = {c: m[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                 "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")
                                         if c in m}
        if "GRBM_GUI_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
            o["sq_busy_of_gui"] = m["SQ_BUSY_CYCLES"] / m["GRBM_GUI_ACTIVE"]
        out[arm] = o
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
