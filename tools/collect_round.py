#!/usr/bin/env python3
"""Copies a measure_round.sh batch from gpurun_out/ into profiles/ (tracked):
the bench lines, the rocprofv3 kernel stats and the main-pass per-launch
trace named with the benched binary's build id, C1 and the concurrency
trials; prints the bench's kernel_ms beside the trace's post-warmup mean.

    python tools/collect_round.py TAG
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def main_pass(bench):
    """The kernel name of the bench's dominant pass: the int8 prefilter pass
    when the line says so (r04), else the bf16 pass."""
    i8 = "i8" in str(bench.get("dtype", ""))
    return f"mfma_topk_kernel<768, 0, 2304, 2, false, {'true' if i8 else 'false'}>"


def pmc_mfma(tag, bid, kname):
    """MFMA utilisation and clock of the C3 main pass from the counter pass:
    busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
    clock = GRBM_GUI_ACTIVE / 8 / wall (MI355X_MICROARCH.md 'DVFS give-back')."""
    f = os.path.join(G, f"{tag}_pmc_mfma_c3", "run_counter_collection.csv")
    if not os.path.exists(f):
        return
    per = {}
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        d = per.setdefault(r["Dispatch_Id"], {"wall_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = list(per.values())
    # (r05) launches that stood down (the gated fallback behind a verified
    # speculative batch: its grid exits at once) are not the pass
    top = max((x["wall_ns"] for x in rows), default=0)
    rows = [x for x in rows if x["wall_ns"] > 0.25 * top][3:]  # past the clock-settling first ones
    if not rows:
        return
    def avg(k):
        return sum(x[k] for x in rows) / len(rows)
    wall = avg("wall_ns") / 1e9
    cyc = avg("GRBM_GUI_ACTIVE") / 8
    busy = avg("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024)
    # the busy counter counts an i8 16x16x64 like a bf16 16x16x32 (same cycles)
    rec = {"kernel": kname + " (C3 main pass)", "build_id": bid,
           "launches": len(rows), "wall_ms": round(wall * 1e3, 4),
           "clock_ghz": round(cyc / wall / 1e9, 3), "mfma_busy_frac": round(busy, 4),
           "mfma_busy_x_clock_over_peak_clock": round(busy * cyc / wall / 2.4e9, 4),
           "sq_busy_cycles": avg("SQ_BUSY_CYCLES"), "sq_wave_cycles": avg("SQ_WAVE_CYCLES"),
           "note": "profiled passes run below the un-profiled clock (MI355X_MICROARCH.md give-back 2)"}
    json.dump(rec, open(os.path.join(P, f"{tag}_c3_{bid}_pmc_mfma.json"), "w"), indent=1)
    print(json.dumps(rec))


def main():
    tag = sys.argv[1]
    b = json.load(open(os.path.join(G, f"{tag}_bench_c3.json")))
    bid = b["config"]["build_id"]
    shutil.copy(os.path.join(G, f"{tag}_bench_c3.json"), os.path.join(P, f"{tag}_c3_{bid}_bench.json"))
    shutil.copy(os.path.join(G, f"{tag}_prof_c3.json"),
                os.path.join(P, f"{tag}_c3_{bid}_bench_under_rocprof.json"))
    d = os.path.join(G, f"{tag}_prof_c3")
    shutil.copy(os.path.join(d, "run_kernel_stats.csv"), os.path.join(P, f"{tag}_c3_{bid}_kernel_stats.csv"))
    kname = main_pass(b)
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))
            if kname in r["Kernel_Name"]]
    with open(os.path.join(P, f"{tag}_c3_{bid}_main_pass_trace.csv"), "w") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Duration_ns"])
        for r in rows:
            w.writerow([r["Kernel_Name"], r["Start_Timestamp"], r["End_Timestamp"],
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    # (r05) without the gated launches that stood down (a few us each)
    nstand = sum(1 for x in dur if x <= 0.25 * max(dur))
    dur = [x for x in dur if x > 0.25 * max(dur)]
    pr = json.load(open(os.path.join(G, f"{tag}_prof_c3.json")))
    print(f"build {bid}: bench kernel_ms {b['roofline']['kernel_ms']} (frac {b['roofline']['frac']}); "
          f"under rocprof {pr['roofline']['kernel_ms']}; trace mean after 10 launches "
          f"{statistics.mean(dur[10:]):.4f} ms over {len(dur) - 10} ({nstand} stood down)")
    pmc_mfma(tag, bid, kname)
    fetch = []
    for cfg in ("c3", "c3b1", "c3_s125"):
        f = os.path.join(G, f"{tag}_pmc_fetch_{cfg}", "run_counter_collection.csv")
        if os.path.exists(f):
            dst = os.path.join(P, f"{tag}_{cfg}_{bid}_pmc_fetch.csv")
            shutil.copy(f, dst)
            if cfg == "c3_s125":  # (r05) the int8 pass at the N = 8 share
                key = "c3_i8@1250000"
            elif cfg == "c3":
                key = cfg + ("_i8" if "true" in kname else "")
            else:  # (r05) B = 1 runs the int8 copy's scan when the collection keeps one
                key = cfg + ("_i8" if "gemv_q8_scan" in open(f).read() else "")
            fetch.append(f"{key}={dst}")
    if fetch:
        import subprocess
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"),
                        f"{tag} build {bid}", *fetch], check=True)
    # (r06) tools/r06_close2.sh's records too, when present
    for src, dst in ((f"{tag}_c1_http.jsonl", f"{tag}_c1_http_both_backends.jsonl"),
                     (f"{tag}_rt_floor.json", f"{tag}_c1_rt_floor.json"),
                     (f"{tag}_concurrency_overlap.json", f"{tag}_concurrency_overlap.json"),
                     (f"{tag}_shares.jsonl", f"{tag}_c3_shares_{bid[:8]}.jsonl"),
                     (f"{tag}_specab_10m_0.jsonl", f"{tag}_specab_10m_0.jsonl"),
                     (f"{tag}_specab_10m_1.jsonl", f"{tag}_specab_10m_1.jsonl"),
                     (f"{tag}_specab_s125_0.jsonl", f"{tag}_specab_s125_0.jsonl"),
                     (f"{tag}_specab_s125_1.jsonl", f"{tag}_specab_s125_1.jsonl"),
                     (f"{tag}_s125_exchange.json", f"{tag}_s125_exchange_bench.json"),
                     (f"{tag}_c4share.json", f"{tag}_c4share_bench.json"),
                     (f"{tag}_c5_loadgen.jsonl", f"{tag}_c5_loadgen_both.jsonl"),
                     (f"{tag}_pipe_s125.json", f"{tag}_share_pipe_s125.json"),
                     (f"{tag}_pipe_10m.json", f"{tag}_share_pipe_10m.json")):
        if os.path.exists(os.path.join(G, src)):
            shutil.copy(os.path.join(G, src), os.path.join(P, dst))
    for fn in sorted(os.listdir(G)):
        if fn.startswith(f"{tag}_bench_") and fn.endswith(".json") and fn != f"{tag}_bench_c3.json":
            shutil.copy(os.path.join(G, fn), os.path.join(P, fn.replace("_bench_", "_") + ""))


if __name__ == "__main__":
    main()
