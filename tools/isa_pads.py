"""Static check of the wait-state padding around the inline-asm MFMA blocks.

The edge backward's weight-gradient MFMAs are inline asm with AGPR accumulators ("+a": amfma32_block,
amfma16_block, amfma4_block in csrc/nonode_train.hip). LLVM's hazard recognizer does not look inside
asm, so each block pads its own wait states. This tool disassembles the device code of a BUILT
libnonode.so (its .hip_fatbin bundles) and checks, for every MFMA that writes an AGPR in the kernels
that use those blocks (the edge backward's pass A, edge_bwd_kernel<NE, 0>: in the VGPR-form unit the
compiler emits no AGPR-destination MFMA of its own there, so every one is an asm block's), that
  - no instruction reads or writes one of its result registers within 11 wait states (except an MFMA
    taking the whole result as its accumulator C, the chain the hardware interlocks), and
  - no VALU instruction wrote one of its source registers within 2 wait states before it.
(Pass B's AGPR-destination MFMAs are the compiler's own, padded by its recognizer, and not checked.)
Round 4's first version (one asm statement per MFMA; the compiler put v_accvgpr_mov copies of the
results right after) fails the first rule.

    python3 tools/isa_pads.py [path/to/libnonode.so]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
READ_AFTER = 11    # XDL result -> any other read (the 8-pass 16x16 MFMAs need fewer; pads give 12)
WRITE_BEFORE = 2   # VALU / load write -> MFMA source read

_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(operand):
    out = set()
    for m in _REG.finditer(operand):
        if m.group(1):
            out |= {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def parse(line):
    """(mnemonic, [operand strings]) of one disassembly line, or None."""
    s = line.split("//")[0].strip()
    if not s or s.endswith(":") or s.startswith("<") or s.startswith("."):
        return None
    parts = s.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def wait_states(ins):
    m, ops = ins
    if m == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 1


def writes(ins):
    m, ops = ins
    if not ops:
        return set()
    if m.startswith(("v_", "ds_read", "ds_load", "global_load", "buffer_load", "flat_load", "scratch_load")):
        return regs(ops[0])
    return set()


def reads(ins):
    m, ops = ins
    if m.startswith(("v_", "ds_", "global_", "buffer_", "flat_", "scratch_")):
        rest = ops[1:] if writes(ins) else ops
        out = set()
        for o in rest:
            out |= regs(o)
        return out
    return set()


def is_agpr_mfma(ins):
    return ins[0].startswith("v_mfma") and ins[1] and ins[1][0].startswith("a")


def functions(asm):
    """{function name: [instructions]} of an llvm-objdump disassembly."""
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        if cur is not None:
            ins = parse(line)
            if ins:
                cur.append(ins)
    return out


def check_function(ins):
    """(number of AGPR MFMAs, [violations]) of one function's instruction list."""
    bad, n = [], 0
    for i, x in enumerate(ins):
        if not is_agpr_mfma(x):
            continue
        n += 1
        dst = regs(x[1][0])
        srcs = set().union(*(regs(o) for o in x[1][1:]))
        # results: later readers
        ws, j = 0, i + 1
        while j < len(ins) and ws < READ_AFTER:
            y = ins[j]
            if y[0].startswith("v_mfma"):
                ydst, ysrc_ab, ysrc_c = regs(y[1][0]), regs(y[1][1]) | regs(y[1][2]), regs(y[1][3])
                if dst & ysrc_ab or (dst & ysrc_c and ysrc_c != dst):
                    bad.append(f"#{j} {y[0]} reads {x[0]} #{i}'s result after {ws} wait states")
            elif dst & reads(y) or dst & writes(y):
                bad.append(f"#{j} {y[0]} touches {x[0]} #{i}'s result after {ws} wait states")
            ws += wait_states(y)
            j += 1
        # sources: earlier writers (the previous MFMA of the chain is interlocked)
        ws, j = 0, i - 1
        while j >= 0 and ws < WRITE_BEFORE:
            y = ins[j]
            if y[0].startswith("v_") and not y[0].startswith("v_mfma") and srcs & writes(y):
                bad.append(f"#{i} {x[0]} reads registers #{j} {y[0]} wrote {ws} wait states before")
            ws += wait_states(y)
            j -= 1
    return n, bad


def device_asm(lib_path, bundles=(0, 1)):
    """Disassembly of the given offload bundles (build units, in link order) of a built library."""
    with tempfile.TemporaryDirectory() as tmp:
        fb = os.path.join(tmp, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib_path, os.devnull],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)] + [len(data)]
        text = []
        for b in bundles:
            part = os.path.join(tmp, f"b{b}.bin")
            open(part, "wb").write(data[starts[b]:starts[b + 1]])
            co = os.path.join(tmp, f"b{b}.o")
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                            f"--input={part}", f"--output={co}"], check=True, capture_output=True)
            text.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                       capture_output=True, text=True).stdout)
        return "\n".join(text)


ASM_KERNELS = re.compile(r"edge_bwd_kernelILi\dELi0EE")   # edge_bwd_kernel<NE, 0>: pass A


def check_library(lib_path):
    """{function: (AGPR MFMA count, violations)} for every kernel that uses the asm MFMA blocks."""
    out = {}
    for name, ins in functions(device_asm(lib_path)).items():
        if ASM_KERNELS.search(name):
            out[name] = check_function(ins)
    return out


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "no-node-comparison_amd", "libnonode.so")
    res = check_library(lib)
    nbad = 0
    for name, (n, bad) in sorted(res.items()):
        print(f"{n:6d} AGPR MFMAs, {len(bad)} violations  {name[:90]}")
        for b in bad[:5]:
            print("      ", b)
        nbad += len(bad)
    sys.exit(1 if nbad else 0)
