"""Per-kernel register / instruction summary of a device assembly file (tools/isa.sh output).

python tools/isa_stats.py a.s [b.s] [--kernel substr]"""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z[^:\s]+):", line)
        if m and not line.startswith("."):
            cur, body = m.group(1), []
            out[cur] = {"body": body}
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
            cur = None
            continue
        body.append(line)
    meta = {}
    for k in out:
        meta[k] = out[k]
    txt = open(path).read()
    for k in out:
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
            m = re.search(r"\.name:\s+" + re.escape(k) + r".*?\n", txt)
        ins = [ln.split()[0] for ln in out[k]["body"] if ln.startswith("\t") and not ln.startswith("\t.") and ln.split()]
        out[k]["n"] = len(ins)
        out[k]["mfma"] = sum(1 for i in ins if i.startswith("v_mfma"))
        out[k]["trans"] = sum(1 for i in ins if i in ("v_exp_f32", "v_rcp_f32"))
        out[k]["pk"] = sum(1 for i in ins if i.startswith("v_pk_"))
        out[k]["acc"] = sum(1 for i in ins if i.startswith("v_accvgpr"))
        out[k]["scratch"] = sum(1 for i in ins if i.startswith("scratch_") or i.startswith("buffer_store_dword") and "off," in i)
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?", txt):
        pass
    res = {}
    for blk in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", txt, re.S):
        name, b = blk.group(1), blk.group(2)
        g = lambda f: int(re.search(r"\." + f + r" (\d+)", b).group(1)) if re.search(r"\." + f + r" (\d+)", b) else -1  # noqa: E731
        res[name] = dict(next_free_vgpr=g("amdhsa_next_free_vgpr"), accum_offset=g("amdhsa_accum_offset"),
                         sgpr=g("amdhsa_next_free_sgpr"), scratch=g("amdhsa_private_segment_fixed_size"),
                         lds=g("amdhsa_group_segment_fixed_size"))
    for k in out:
        out[k].update(res.get(k, {}))
        for f in ("num_vgpr", "num_agpr", "private_seg_size"):
            m = re.search(r"\.set " + re.escape(k) + r"\." + f + r", (\d+)", txt)
            out[k][f] = int(m.group(1)) if m else -1
    return out


def main():
    files = [a for a in sys.argv[1:] if not a.startswith("--")]
    sub = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "egnn_layer"
    ks = [kernels(f) for f in files if f != sub]
    names = sorted(k for k in ks[0] if sub in k)
    for n in names:
        for f, K in zip(files, ks):
            d = K.get(n)
            if d is None:
                continue
            print(f"{n[:70]:70s} {f[-12:]:>12s} instr {d['n']:6d} mfma {d['mfma']:5d} trans {d['trans']:5d} pk {d['pk']:5d} "
                  f"accv {d['acc']:5d} vgpr {d['num_vgpr']} agpr {d['num_agpr']} scratch {d['private_seg_size']}")


if __name__ == "__main__":
    main()


def loops(path, kname):
    """(label, n_instr, n_mfma, n_accvgpr, n_pk, n_trans) of every backward-branch loop in kernel kname."""
    body = kernels(path)[kname]["body"]
    lab = {}
    res = []
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            lab[m.group(1)] = i
        m = re.match(r"^\ts_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(1) in lab:
            seg = [x.split()[0] for x in body[lab[m.group(1)]:i + 1] if x.startswith("\t") and not x.startswith("\t.")]
            res.append((m.group(1), len(seg), sum(x.startswith("v_mfma") for x in seg),
                        sum(x.startswith("v_accvgpr") for x in seg), sum(x.startswith("v_pk_") for x in seg),
                        sum(x.startswith(("v_exp", "v_rcp")) for x in seg)))
    return res


def loop_hist(path, kname, label, nth=-1):
    """instruction histogram of the loop headed by `label` (the nth backward branch to it)"""
    import collections
    body = kernels(path)[kname]["body"]
    start = next(i for i, ln in enumerate(body) if ln.startswith(label + ":"))
    ends = [i for i, ln in enumerate(body) if re.match(r"^\ts_(?:cbranch_\w+|branch)\s+" + re.escape(label) + r"\b", ln)]
    seg = [x.split()[0] for x in body[start:ends[nth] + 1] if x.startswith("\t") and not x.startswith("\t.")]
    return collections.Counter(seg)


def blocks(path, kname, label, nth=-1):
    """basic blocks (label, instruction list) of the loop headed by `label`"""
    body = kernels(path)[kname]["body"]
    start = next(i for i, ln in enumerate(body) if ln.startswith(label + ":"))
    ends = [i for i, ln in enumerate(body) if re.match(r"^\ts_(?:cbranch_\w+|branch)\s+" + re.escape(label) + r"\b", ln)]
    out, cur, name = [], [], label
    for ln in body[start:ends[nth] + 1]:
        m = re.match(r"^(\.LBB\S+):|^; %(bb\.\d+):", ln)
        if m:
            if cur:
                out.append((name, cur))
            name, cur = m.group(1) or m.group(2), []
            continue
        if ln.startswith("\t") and not ln.startswith("\t.") and not ln.startswith("\t;"):
            cur.append(ln.split()[0])
    if cur:
        out.append((name, cur))
    return out
