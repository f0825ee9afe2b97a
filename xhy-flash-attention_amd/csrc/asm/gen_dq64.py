#!/usr/bin/env python3
"""Generates fa_dq64_asm.s: the gfx950 dQ kernel for head dim 64 (round 6), gen_dq.py's d = 128
kernel instantiated at d = 64 (one wave per SIMD, all 512 registers).

    python3 gen_dq64.py > fa_dq64_asm.s

Same algorithm, kernel arguments (DqAsmArgs), fused preprocessing, Q fold, work order and step
structure as gen_dq.py (the reference's compute_dq_dk_dv_1colblock dQ half,
csrc/flash_attn/src/flash_bwd_kernel.h:897-1008, head-dim-64 instance
flash_bwd_launch_template.h:194-235).  What changes at d = 64:

  * a phase has 24 MFMAs (S^T 8, dP^T 8, dQ^T 8: 4 k-steps and 2 d-tiles for each of the wave's two
    32-row q-blocks) beside the same per-subtile softmax VALU as at d = 128;
  * a K (or V) subtile of 32 keys is 4 KiB: the two 64-byte panels of gen_dq.py's LDS layout; each wave
    DMAs one 1-KiB piece of K and one of V per subtile (panel w & 1, rows 16 (w >> 1)), so the ring's
    9 slots take 72 KiB and a step issues 4 pieces a wave (VMCNT_STEP 4);
  * registers keep gen_dq.py's map (dQ^T a[64 j + 16 dt], Q a[128 + 32 j + 4 ks], dO a[192 + ...]);
    the A-fragment ring moves into the AGPRs that leaves free (a[32:63], a[96:127]), and its VGPRs
    v[160:223] hold per-row chain starts (gen_dq.py CHAIN_S / CHAIN_D): S^T starts from -LSE log2 e / c and dP^T
    from -D, so the softmax VALU per score is exp (+ one multiply unless c = 1: the _c1 kernels, the
    folded backward) and dS = P dP' -- 64 fewer VALU ops a phase than gen_dq.py's v_fma + v_sub.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_dq as G  # noqa: E402

D = G.D = 64
G.KS = D // 16                      # 4 k-steps of S^T / dP^T
G.NP = D // 32                      # 2 d-tiles of dQ^T
G.KT = G.SUB * D * 2                # 4 KiB: one K (or V) subtile
G.SLOT = 2 * G.KT
G.RING = G.NS * G.SLOT              # 72 KiB
G.LDS_BYTES = G.RING
G.PIECES = 2
G.VMCNT_STEP = 2 * G.PIECES
G.CHAIN_S = G.CHAIN_D = True
G.RING_SLOTS = 16
G.RING_FILE = "a"
assert G.RING % 4096 == 0


def main():
    kernels = [G.K(bf, ca, u) for u in (False, True) for bf in (True, False) for ca in (True, False)]
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 5", "\t.text"]
    for k in kernels:
        out.append(k.render())
        out.append(k.descriptor())
    out.append("\t.amdgpu_metadata\n---\namdhsa.kernels:")
    for k in kernels:
        out.append(k.metadata().rstrip("\n"))
    out.append("amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata")
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
