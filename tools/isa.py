#!/usr/bin/env python3
"""Disassembly of one kernel of the built library, with the instruction mix of each loop (dev tool):

    python tools/isa.py KERNEL_SUBSTRING [--lib path.so] [--dump out.s]
Loops come from backward branches; per loop: MFMA, other VALU, SALU, LDS, VMEM, s_waitcnt, s_nop,
s_barrier counts.  Nested loops are reported separately (an outer loop's counts include them).
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_isa_hazards as th  # noqa: E402


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    for pre, c in (("v_", "valu"), ("ds_", "lds"), ("buffer_", "vmem"), ("global_", "vmem"),
                   ("scratch_", "scratch"), ("s_waitcnt", "wait"), ("s_nop", "nop"),
                   ("s_barrier", "barrier"), ("s_", "salu")):
        if op.startswith(pre):
            return c
    return "other"


def kernels(lib):
    blob = open(lib, "rb").read()
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for n, co in enumerate(th._code_objects(blob)):
            p = os.path.join(tmp, f"co{n}.elf")
            open(p, "wb").write(co)
            txt = subprocess.run([th.OBJDUMP, "-d", "--mcpu=gfx950", p], capture_output=True, text=True,
                                 check=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = out.setdefault(m.group(1), [])
                    continue
                m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
                if cur is not None and m:
                    cur.append((int(m.group(2), 16), m.group(1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--lib", default=os.path.join(ROOT, "xhy-flash-attention_amd", "libflash_attn_mi355x.so"))
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    ks = kernels(a.lib)
    names = [n for n in ks if a.kernel in n]
    if not names:
        sys.exit(f"no kernel matching {a.kernel}")
    name = min(names, key=len)
    ins = ks[name]
    idx = {addr: i for i, (addr, _) in enumerate(ins)}
    if a.dump:
        with open(a.dump, "w") as f:
            f.write("\n".join(f"{i:5d} {addr:6x}  {s}" for i, (addr, s) in enumerate(ins)))
    print(name, len(ins), "instructions:", dict(collections.Counter(classify(s.split()[0]) for _, s in ins)))
    for i, (addr, s) in enumerate(ins):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(-?\d+)", s)
        if not m:
            continue
        off = int(m.group(2))
        off = off - 65536 if off >= 32768 else off
        if off >= 0:
            continue
        tgt = addr + 4 + 4 * off
        j = idx.get(tgt)
        if j is None:
            continue
        c = collections.Counter(classify(x.split()[0]) for _, x in ins[j:i + 1])
        print(f"loop [{j}..{i}] ({i - j + 1} instr): " + " ".join(f"{k} {v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
