#!/usr/bin/env python3
"""Static check for the packed-fp32 co-residency fault: for every packed VALU
instruction (v_pk_*) of a kernel's assembly, the instruction that last wrote each of its VGPR-pair
sources, classified as a vector memory load (global/buffer/flat), an LDS read, or a VALU
instruction.  The fault needs packed ops that read pairs straight from global_load returns
(deform.hip features_to_lds under SLP); the compositors' packed operands come from LDS.
Usage: tools/pk_sources.py file.s [kernel-substring ...]   (hipcc --cuda-device-only -S output)"""
import collections
import re
import sys


def regs(op):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", op):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(lines):
    name, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            body.append(ln.strip())
            if ln.strip().startswith("s_endpgm"):
                yield name, body
                name, body = None, []


def classify(body):
    last = {}
    stats = collections.Counter()
    for ins in body:
        if not ins or ins.startswith((".", ";")) or ins.endswith(":"):
            if ins.endswith(":"):
                last = {}          # a label: writers before it are not known on every path
            continue
        parts = ins.split(None, 1)
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if mn.startswith("v_pk_") and ops:
            for o in ops[1:]:
                if "[" in o and o.startswith("v["):
                    w = {last.get(r, "unknown") for r in regs(o)}
                    stats["pair from " + "/".join(sorted(w))] += 1
        if mn.startswith(("global_store", "buffer_store", "ds_write", "global_atomic", "s_", "flat_store")):
            continue
        if ops:
            kind = ("vmem_load" if mn.startswith(("global_load", "buffer_load", "flat_load")) else
                    "lds_read" if mn.startswith("ds_read") else "valu")
            for r in regs(ops[0]):
                last[r] = kind
    return stats


def main():
    lines = open(sys.argv[1]).read().splitlines()
    want = sys.argv[2:]
    for name, body in kernels(lines):
        if want and not any(w in name for w in want):
            continue
        st = classify(body)
        if st:
            print(name[:90], dict(sorted(st.items())))


if __name__ == "__main__":
    main()
