"""CPU checks of the decode-burst dev switches (FA_GEN_DECBURST / FA_GDQ_DECBURST / FA_GBW_DECBURST).

Off (the shipped build): each kernel waits for its kernargs, then loads the work order (fa_params.h
ItemDecode) and waits again.  On: the ItemDecode loads join the kernarg burst, so the kernel's first
`s_waitcnt lgkmcnt(0)` already covers them ("One scalar round trip less").
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm")
SWITCH = {"fwd": "FA_GEN_DECBURST", "dq": "FA_GDQ_DECBURST", "bwd": "FA_GBW_DECBURST"}
# the ItemDecode dword offset in each kernel's kernargs (gen_*.py DEC_OFF)
DEC_OFF = {"fwd": 184, "dq": 184, "bwd": 224}


def first_kernel(kind, on):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("FA_GEN_", "FA_GDQ_", "FA_GBW_"))}
    if on:
        env[SWITCH[kind]] = "1"
    text = subprocess.run([sys.executable, os.path.join(ASM, f"gen_{kind}.py")], env=env, check=True,
                          capture_output=True, text=True).stdout
    body = text.split(".text", 1)[-1]
    lines = [ln.strip() for ln in body.splitlines()]
    start = next(i for i, ln in enumerate(lines) if ln.endswith(":") and not ln.startswith("."))
    end = next(i for i in range(start + 1, len(lines)) if lines[i] == "s_endpgm")
    return lines[start:end]


@pytest.mark.parametrize("kind", ["fwd", "dq", "bwd"])
def test_decode_loads_join_the_kernarg_burst_only_when_switched_on(kind):
    dec = f"s[0:1], {DEC_OFF[kind]}"
    for on in (False, True):
        ins = first_kernel(kind, on)
        # the kernarg burst starts with the load of dwords 0..15 (the kernels may wait for other scalar
        # loads before it, e.g. the dQ kernel's item index)
        burst = next(i for i, ln in enumerate(ins) if ln.startswith("s_load_dwordx16") and ln.endswith("s[0:1], 0x0"))
        wait = next(i for i in range(burst, len(ins)) if ins[i].startswith("s_waitcnt") and "lgkmcnt(0)" in ins[i])
        first_dec = next(i for i in range(burst, len(ins)) if ins[i].startswith("s_load_dwordx8") and ins[i].endswith(dec))
        assert (first_dec < wait) == on, (kind, on, first_dec, wait)
