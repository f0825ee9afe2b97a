#!/usr/bin/env python3
"""Generates fa_fwdnf_asm.s: gen_fwd.py's forward kernels without the Q fold (round 6), for the calls
that score from the exact Q (attn_folds_q false: FLASH_ATTN_MI355X_NO_QFOLD=1, or fp16 with
|scale log2 e| > 1).

    python3 gen_fwdnf.py > fa_fwdnf_asm.s

The same kernels as gen_fwd.py generated with its FA_GEN_FOLD=0 path: Q stays as given, every
tile's S chain starts from zero and the softmax takes P = exp2(c S - c m) with one v_fma_f32 per
score (c = scale log2 e in fp32), as the reference's scale_apply_exp2 (softmax.h:66-85).  Kernel
names fa_fwdnf_asm_d{128,64}_{bf16,f16}_{causal,full}.
"""
import os
import sys

os.environ["FA_GEN_FOLD"] = "0"
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fwd as G  # noqa: E402

G.NAME = "fa_fwdnf_asm"

if __name__ == "__main__":
    G.main()
