"""Per-kernel HBM traffic per launch of one workload from a `tools/gpu.sh profile` output directory.

Usage: python3 tools/pmc_traffic.py WORKLOAD gpurun_out/prof_TAG_<workload> [--merge profiles/pmc_traffic.json]
(WORKLOAD = the key bench.py's pmc_traffic() looks up: C2, C3, C4, C4@B=4096, C5, segno_train, f1)

FETCH_SIZE / WRITE_SIZE are in KB per dispatch. On gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM / rocprofv3 section), so
hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import collections
import csv
import glob
import json
import re
import statistics
import sys


def kernel_key(name):
    if "egnn_layer_kernel" in name:
        m = re.search(r"egnn_layer_kernel<(\d+)", name)
        variant = "SEGNO" if (m and m.group(1) == "1") or "ILi1E" in name else "EGNO"
        return f"egnn_layer_kernel<{variant}>"
    if "tconv_kernel" in name:
        return "tconv_kernel<first>" if ("<true>" in name or "<true," in name or "ILb1E" in name) else "tconv_kernel"
    if "edge_bwd_kernel" in name:   # edge_bwd_kernel<NE, PASS>
        m = re.search(r"edge_bwd_kernel<\d+,\s*(\d+)>", name) or re.search(r"edge_bwd_kernelILi\d+ELi(\d+)E", name)
        return f"edge_bwd_kernel<pass {m.group(1)}>" if m else "edge_bwd_kernel"
    if "tconv_bwd_kernel" in name:
        return "tconv_bwd_kernel"
    for k in ("temb_kernel", "embed_kernel", "node_bwd_kernel", "node_wgrad_kernel"):
        if k in name:
            return k
    return None


def main(workload, d, merge=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/pmc_*/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if k:
                per[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, c, _), v in per.items():
            vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        row = {c: statistics.mean(v) for c, v in cs.items()}
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes_per_launch"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
            row["correction"] = "(2*FETCH_SIZE + WRITE_SIZE) KB -> bytes; FETCH doubled per MI355X_MICROARCH.md HBM section"
        out[k] = row
    if merge:
        try:
            allw = json.load(open(merge))
        except FileNotFoundError:
            allw = {}
        allw[workload] = out
        with open(merge, "w") as f:
            json.dump(allw, f, indent=1, sort_keys=True)
            f.write("\n")
    json.dump({workload: out}, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    a = sys.argv[1:]
    m = None
    if "--merge" in a:
        i = a.index("--merge")
        m = a[i + 1]
        a = a[:i] + a[i + 2:]
    main(a[0], a[1], m)
