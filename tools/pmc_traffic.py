"""Builds profiles/pmc_traffic.json from rocprofv3 --pmc FETCH_SIZE runs of bench.py.

    python tools/pmc_traffic.py TAG c3=gpurun_out/pmc_c3/run_counter_collection.csv \
        c3b1=... c2=... c3_i8@1250000=...   (cfg@ROWS: a run with --rows ROWS)

HBM bytes per launch = FETCH_SIZE (KB) x 1024 x 2 (the gfx950 correction,
MI355X_MICROARCH.md HBM/rocprofv3 section), averaged over the scan kernel's
launches (the MFMA main pass for batched configs, the GEMV scan for B = 1).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (r04) batched bf16 configs run the int8 prefilter pass by default: "_i8"
# entries are that pass (the bf16 pass's launch behind it stands down at once
# and must not enter the average), the plain ones the bf16 pass
SCAN = {"c3": "mfma_topk_kernel<768, 0, 2304, 2, false, false>",
        "c3_i8": "mfma_topk_kernel<768, 0, 2304, 2, false, true>",
        "c5b256_i8": "mfma_topk_kernel<1024, 0, 256, 1, false, true>",
        "c3b1": "gemv_topk_kernel<768, true, 1",
        # (r05) one query on the int8 copy: its scan kernel
        "c3b1_i8": "gemv_q8_scan_kernel<768, 1>", "c2_i8": "gemv_q8_scan_kernel<768, 1>",
        "c2": "gemv_topk_kernel<768, false, 1", "c4": "mfma_topk_kernel<768, 0,",
        "c4b1": "gemv_topk_kernel<768, true, 2", "c5b256": "mfma_topk_kernel<1024, 0,"}


# each config's corpus rows (bench.py CONFIGS) for entries measured at N = 1
DEFAULT_ROWS = {"c3": 10_000_000, "c3b1": 10_000_000, "c2": 1_000_000, "c2b256": 1_000_000,
                "c3f32": 10_000_000, "c3f32b1": 10_000_000, "c5b256": 5_000_000,
                "c4": 100_000_000, "c4b1": 100_000_000}


def main():
    tag, specs = sys.argv[1], sys.argv[2:]
    # entries for configs not re-measured this time are kept
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(p)) if os.path.exists(p) else {}
    out["_doc"] = ("HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE (KB, x1024, x2 gfx950 "
                   "correction: MI355X_MICROARCH.md HBM section), averaged over the scan launches "
                   "of `python bench.py --config <cfg> --steps 5 --warmup 2`; each entry names "
                   "its build")
    for spec in specs:
        key, path = spec.split("=", 1)
        cfg, _, rows = key.partition("@")
        vals, name = [], None
        for r in csv.DictReader(open(path)):
            if SCAN[cfg] in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                vals.append(float(r["Counter_Value"]))
                name = r["Kernel_Name"].split("(")[0].replace("void vsk::", "")
        if not vals:
            raise SystemExit(f"no FETCH_SIZE rows for {SCAN[cfg]} in {path}")
        # (r05) launches that stood down (the gated fallback behind a verified
        # speculative batch) fetch next to nothing: not the pass
        vals = [v for v in vals if v > 0.25 * max(vals)]
        kb = sum(vals) / len(vals)
        # rows one launch scanned: bench.py reports the entry only for a run
        # whose rows_per_gpu equals it (an N > 1 share is a different launch)
        n = int(rows) if rows else DEFAULT_ROWS[cfg.replace("_i8", "")]
        out[key] = {"kernel": name, "launches": len(vals), "fetch_size_kb_avg": round(kb, 1),
                    "hbm_bytes_per_launch": int(kb * 1024 * 2), "rows": n, "build": tag}
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
