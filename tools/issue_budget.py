#!/usr/bin/env python3
"""Issue budget of one block of a generated assembly kernel (dev tool).

    python tools/issue_budget.py GEN.py KERNEL START_LABEL END_LABEL [--env K=V ...]

Counts the instructions between two labels of a kernel in the generator's output by class and prices
each with the one-wave-per-SIMD issue costs of MI355X_MICROARCH.md ("Per-instruction cycle constants":
a VALU op 4 cycles, a transcendental 8, an MFMA holds the SIMD's issue for 8 of its 32, v_cvt_pk 4-5,
an LDS-DMA piece 60 among bare MFMAs (25-185 by context); SALU, LDS reads, waits and branches take one
4-cycle issue slot each; s_nop n takes n + 1 slots).  The out-of-line refit blocks a guard branch
jumps to are not counted (they run rarely).  Prints the table and the ratio of the issue total to the
block's matrix-pipe time (32 cycles per v_mfma_f32_32x32x16)."""
import argparse
import collections
import os
import re
import subprocess
import sys

COST = {"mfma": 8, "trans": 8, "cvt_pk": 4.5, "valu": 4, "lds_read": 4, "lds_write": 4, "lds_dma": 60,
        "vmem": 4, "salu": 4, "wait": 4, "nop": 4, "branch": 4, "barrier": 4, "other": 4}
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def classify(text):
    op = text.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_cvt_pk"):
        return "cvt_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read"):
        return "lds_read"
    if op.startswith("ds_write"):
        return "lds_write"
    if op.startswith("buffer_load") and text.rstrip().endswith("lds"):
        return "lds_dma"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op == "s_nop":
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def block(text, kernel, start, end):
    lines = text.split("\n")
    i0 = lines.index(f"{kernel}:")
    out, on = [], False
    for ln in lines[i0 + 1:]:
        s = ln.strip()
        if s.startswith(f".L{kernel}_fend"):
            break
        if s.endswith(":"):
            name = s[:-1]
            if name.startswith(f".L{kernel}_{start}"):
                on = True
                continue
            if on and name.startswith(f".L{kernel}_{end}"):
                break
            continue
        if on and s and not s.startswith((";", ".")):
            out.append(s)
    return out


def budget(insts):
    n = collections.Counter()
    cyc = collections.Counter()
    for t in insts:
        c = classify(t)
        n[c] += 1
        w = COST[c]
        if c == "nop":
            w = 4 * (int(t.split()[1]) + 1)
        cyc[c] += w
    return n, cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("gen")
    ap.add_argument("kernel")
    ap.add_argument("start")
    ap.add_argument("end")
    ap.add_argument("--env", nargs="*", default=[])
    a = ap.parse_args()
    env = dict(os.environ, **dict(kv.split("=", 1) for kv in a.env))
    text = subprocess.run([sys.executable, a.gen], check=True, capture_output=True, text=True, env=env).stdout
    ins = block(text, a.kernel, a.start, a.end)
    n, cyc = budget(ins)
    mf = n["mfma"] * 32
    tot = sum(cyc.values())
    print(f"{a.kernel} [{a.start} .. {a.end}): {len(ins)} instructions, {n['mfma']} MFMAs = {mf} matrix-pipe cycles")
    print(f"{'class':>10} {'count':>6} {'issue cyc':>10} {'per MFMA gap':>13}")
    for c in sorted(cyc, key=lambda k: -cyc[k]):
        print(f"{c:>10} {n[c]:6d} {cyc[c]:10.0f} {cyc[c] / max(n['mfma'], 1):13.1f}")
    print(f"{'total':>10} {len(ins):6d} {tot:10.0f} {tot / max(n['mfma'], 1):13.1f}   "
          f"issue / pipe = {tot / max(mf, 1):.2f}  (non-MFMA issue {tot - cyc['mfma']:.0f} vs gaps "
          f"{n['mfma'] * 24} at 24 cycles each)")


if __name__ == "__main__":
    main()
