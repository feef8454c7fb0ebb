"""Summarise rocprofv3 --pmc CSVs per kernel symbol (debug aid, not product)."""
import csv, collections, re, sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(dict)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        nm = r["Kernel_Name"]
        m = re.search(r"mfma_topk_kernel<(\d+), (\d+), (\d+)(?:, (\d+))?(?:, (?:true|false))?>", nm)
        nm = f"mfma<{m.group(2)},{m.group(3)},{m.group(4)}>" if m else nm[:30]
        rows[nm][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[nm][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for nm, c in rows.items():
    d = list(durs[nm].values()); ms = sorted(d)[len(d) // 2]
    out = {k: sum(v) / len(v) for k, v in c.items()}
    g = out.get("GRBM_GUI_ACTIVE", 0) / 8
    line = f"{nm:22s} ms {ms:6.3f} clk {g / ms / 1e6 if ms else 0:5.2f}GHz cyc/XCD {g/1e6:6.2f}M"
    wc = out.get("SQ_WAVE_CYCLES")
    for k in sorted(out):
        if k == "GRBM_GUI_ACTIVE": continue
        v = out[k]
        line += f" {k.replace('SQ_','')}={v/1e6:.1f}M"
    print(line)
