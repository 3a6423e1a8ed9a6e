"""Per-kernel HBM traffic per launch from a tools/gpu_profile.sh output directory.

Usage: python3 tools/pmc_traffic.py gpurun_out/prof_TAG > profiles/pmc_traffic.json

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
    for k in ("temb_kernel", "embed_kernel", "node_bwd_kernel", "node_post_kernel"):
        if k in name:
            return k
    return None


def main(d):
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
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
