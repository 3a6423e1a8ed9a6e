"""Summarise rocprofv3 PMC csv files of one profile directory per kernel (mean per launch)."""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1]
res = collections.defaultdict(dict)
for f in glob.glob(f"{d}/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "egnn_layer" in n:
            key = "layer" + ("<SEGNO>" if "Li1E" in n or "<1," in n else "")
        elif "tconv" in n:
            key = "tconv_first" if ("<true>" in n or "<true," in n) else "tconv"
        else:
            continue
        res[key].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
stats = {}
for row in csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")):
    stats[row["Name"]] = float(row["AverageNs"])
for k, dd in res.items():
    out = {c: statistics.mean(v) for c, v in dd.items()}
    ns = [v for n, v in stats.items() if ("egnn_layer" in n if k.startswith("layer") else ("tconv" in n and ((("<true>" in n) or ("<true," in n)) == (k == "tconv_first"))))]
    ns = ns[0] if ns else None
    line = f"{k}: avg {ns/1e3 if ns else 0:.1f} us"
    if "GRBM_GUI_ACTIVE" in out and ns:
        line += f" | clock {out['GRBM_GUI_ACTIVE'] / 8 / ns:.2f} GHz"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in out and "GRBM_GUI_ACTIVE" in out:
        line += f" | MFMA busy {out['SQ_VALU_MFMA_BUSY_CYCLES'] / (out['GRBM_GUI_ACTIVE'] / 8 * 1024):.1%}"
    if "SQ_WAVE_CYCLES" in out:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in out:
                line += f" | {c} {out[c] / out['SQ_WAVE_CYCLES']:.1%}"
    for c in ("SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA"):
        if c in out and "SQ_WAVE_CYCLES" in out:
            line += f" | {c} {out[c] / out['SQ_WAVE_CYCLES']:.1%}"
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES"):
        if c in out:
            line += f" | {c} {out[c]:.3g}"
    print(line)
    if "-v" in sys.argv:
        wc = out.get("SQ_WAVE_CYCLES")
        for c in sorted(out):
            print(f"    {c:32s} {out[c]:14.4g}" + (f"  ({out[c] / wc:.1%} of wave cycles)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""))
