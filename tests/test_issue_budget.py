"""tools/issue_budget.py (the static issue-cycle table of a generated kernel's block)
on the shipped generators: the steady steps hold the MFMA counts their designs state, and the d = 64
chain starts (gen_dq64.py CHAIN_S / CHAIN_D) remove the per-score v_fma / v_sub from dQ's step."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
ASM = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm")

import issue_budget as ib  # noqa: E402


def _block(gen, kernel, start, end):
    text = subprocess.run([sys.executable, os.path.join(ASM, gen)], check=True, capture_output=True, text=True).stdout
    return ib.block(text, kernel, start, end)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("gen,kernel,start,end,mfmas", [
    ("gen_fwd.py", "fa_fwd_asm_d128_bf16_causal", "fast0", "sel0", 128),     # two 64-key steps, 2 q-blocks
    ("gen_fwd.py", "fa_fwd_asm_d64_bf16_causal", "fast0", "sel0", 64),
    ("gen_bwd.py", "fa_bwd_dkdv_asm_d128_bf16_causal_c1", "step_R", "tail", 64),
    ("gen_dq.py", "fa_bwd_dq_asm_d128_bf16_causal", "step_R", "tail", 96),
    ("gen_dq64.py", "fa_bwd_dq_asm_d64_bf16_causal_c1", "step_R", "tail", 48),
])
def test_step_mfma_counts(gen, kernel, start, end, mfmas):
    n, cyc = ib.budget(_block(gen, kernel, start, end))
    assert n["mfma"] == mfmas
    assert sum(cyc.values()) > cyc["mfma"]


@pytest.mark.timeout(300)
def test_d64_dq_chain_starts_remove_the_score_fma_and_sub():
    ops = [x.split()[0] for x in _block("gen_dq64.py", "fa_bwd_dq_asm_d64_bf16_causal_c1", "step_R", "tail")]
    assert "v_fma_f32" not in ops and "v_sub_f32_e32" not in ops
    assert ops.count("v_exp_f32_e32") == 64 and ops.count("v_mul_f32_e32") == 64   # P = exp2(S'), dS = P dP'
    ops128 = [x.split()[0] for x in _block("gen_dq.py", "fa_bwd_dq_asm_d128_bf16_causal", "step_R", "tail")]
    assert ops128.count("v_fma_f32") == 64 and "v_sub_f32_e32" not in ops128   # d = 128: CHAIN_D only
