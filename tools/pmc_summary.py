"""Summarise rocprofv3 PMC csv files of one profile directory per kernel (mean per launch).

Clock (round 6 correction): rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs, and the busy
window it counts includes the dispatch's launch and drain, so GRBM_GUI_ACTIVE / 8 / kernel time reads
HIGH on dispatches shorter than about 0.3 ms (MI355X_MICROARCH.md, DVFS give-back): rounds 1-5 printed
3.4-3.5 GHz for the 18 us TimeConv launch, above the 2.4 GHz maximum. The effective clock is printed
only for dispatches >= 0.3 ms; otherwise the GRBM window at the 2.4 GHz maximum clock (a lower bound
of the window's length) is printed beside the kernel time, and cycle figures use the 2.4 GHz maximum
(an upper bound of the cycles the kernel had)."""
import collections
import csv
import glob
import statistics
import sys

MAX_GHZ = 2.4       # MI355X maximum engine clock (MI355X_MICROARCH.md)
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
    clk = MAX_GHZ
    if "GRBM_GUI_ACTIVE" in out and ns:
        per_xcd = out["GRBM_GUI_ACTIVE"] / 8
        if ns >= 3e5:
            clk = min(per_xcd / ns, MAX_GHZ)
            line += f" | clock {clk:.2f} GHz"
        else:
            line += f" | GRBM window {per_xcd / MAX_GHZ / 1e3:.1f} us at {MAX_GHZ} GHz (dispatch < 0.3 ms: no clock derived)"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in out and ns:
        # kernel cycles at clk x 1024 SIMDs (clk = the 2.4 GHz maximum for short dispatches: a lower bound)
        line += f" | MFMA busy {out['SQ_VALU_MFMA_BUSY_CYCLES'] / (ns * clk * 1024):.1%}"
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
