"""Instruction mix of a kernel's loops from a hipcc --save-temps .s file.

usage: python scripts/isa_loops.py FILE.s SYMBOL_SUBSTRING
Prints, per loop (a backward branch to an earlier label), its body's instruction count by
class: fp64 VALU (v_*_f64), other VALU, DPP moves, LDS, VMEM loads/stores, SMEM, SALU."""
import re
import sys


def classify(op, line):
    if op.startswith("v_"):
        if "dpp" in line or "row_" in line or "quad_perm" in line:
            return "v_dpp"
        if op.endswith("_f64") or "_f64_" in op:
            return "v_f64"
        if op.startswith("v_mfma"):
            return "mfma"
        return "v_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
        return "vmem_st"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, sym):
    text = open(path).read().split("\n")
    start = None
    for i, l in enumerate(text):
        if l.startswith(sym) or (sym in l and l.rstrip().endswith(":") and l.startswith("_Z")):
            start = i
            break
    if start is None:
        sys.exit("symbol not found")
    end = start + 1
    while end < len(text) and not text[end].startswith(".Lfunc_end"):
        end += 1
    body = text[start:end]
    labels = {}
    insts = []  # (index, label_before, op, line)
    for l in body:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        insts.append((op, t))
    print(f"{sym}: {len(insts)} instructions")
    tot = {}
    for op, t in insts:
        c = classify(op, t)
        tot[c] = tot.get(c, 0) + 1
    print("  whole kernel:", tot)
    for k, (op, t) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                a = labels[tgt]
                cnt = {}
                for op2, t2 in insts[a:k + 1]:
                    c = classify(op2, t2)
                    cnt[c] = cnt.get(c, 0) + 1
                print(f"  loop {tgt} [{a}, {k}] {k - a + 1} insts:", dict(sorted(cnt.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
