"""Varlen calls with sequences that have query rows but no keys, or keys but no query rows
(cu_seqlens_q != cu_seqlens_k with zero-length entries).  Rows without keys get O = 0 and
LSE = +inf, the reference epilogue's values for an empty softmax (row sum 0,
flash_fwd_kernel.h:509-518), and their backward adds nothing.  (The reference itself starts such a
sequence's key loop at block -1, flash_fwd_kernel.h:300-303, and reads the rows before it: its
result there is undefined.)  Every other sequence is held to the 2x rule
(tests/test_flash_attn.py:774-783).  At head dims 64 / 128 the rows without keys take the assembly
forward's item start for an item with no K/V tiles (gen_fwd.py item_start): through the persistent
device-built list and, with FLASH_ATTN_MI355X_FWD_PERSIST=0, one workgroup per item."""
import random

import pytest
import torch

from knobs import FWD_PERSIST, knob
from oracle.attention_ref import attention_ref, check_within_bound

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _ref(q, k, v, g, causal):
    out = {}
    for upcast, key in ((True, "ref"), (False, "pt")):
        qr, kr, vr = (x.detach().clone().requires_grad_() for x in (q, k, v))
        o, _ = attention_ref(qr, kr, vr, causal=causal, upcast=upcast, reorder_ops=not upcast)
        out[key] = (o,) + tuple(torch.autograd.grad(o, (qr, kr, vr), g))
    return out


@pytest.mark.parametrize("persist", [1, 0])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128, 96])
def test_varlen_sequences_without_keys(d, causal, dtype, persist):
    _check([300, 5, 0, 257, 64, 700], [0, 130, 90, 0, 64, 333], 4, 2, d, causal, dtype, persist, 7)


# seeded random cu_seqlens_q != cu_seqlens_k (zero-length entries on either side), GQA, head dims of
# the assembly (64, 128) and HIP (96) paths
@pytest.mark.parametrize("seed", range(48))
def test_varlen_random_q_k_lengths(seed):
    r = random.Random(5000 + seed)
    n = r.randint(1, 5)
    pick = lambda: r.choice([0, 1, r.randint(2, 130), r.randint(131, 700)])  # noqa: E731
    lens_q, lens_k = [pick() for _ in range(n)], [pick() for _ in range(n)]
    if sum(lens_q) == 0:
        lens_q[0] = 33
    if sum(lens_k) == 0:
        lens_k[-1] = 41
    hk = r.choice([1, 2])
    # max_seqlen_q / _k above the longest sequence, as a caller may pass (the grid covers more blocks)
    slack = (r.choice([0, 0, 37, 300]), r.choice([0, 0, 64, 129]))
    _check(lens_q, lens_k, hk * r.choice([1, 2, 3]), hk, r.choice([64, 128, 128, 96]), r.random() < 0.5,
           r.choice([torch.bfloat16, torch.float16]), 1, seed, slack)


def _check(lens_q, lens_k, h, hk, d, causal, dtype, persist, seed, slack=(0, 0)):
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(seed)
    cu_q = torch.tensor([0] + lens_q, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    cu_k = torch.tensor([0] + lens_k, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    q = torch.randn(sum(lens_q), h, d, device=DEV, dtype=dtype, requires_grad=True)
    k, v = (torch.randn(sum(lens_k), hk, d, device=DEV, dtype=dtype, requires_grad=True) for _ in range(2))
    with knob(FWD_PERSIST, persist):
        out, lse, _ = flash_attn_varlen_func(q, k, v, cu_q, cu_k, max(lens_q) + slack[0], max(lens_k) + slack[1],
                                             causal=causal,
                                             return_attn_probs=True)
        g = torch.randn_like(out)
        dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
    torch.cuda.synchronize()
    for name, t in (("out", out), ("lse", lse), ("dq", dq), ("dk", dk), ("dv", dv)):
        assert not torch.isnan(t).any(), f"{name} has NaN"
    for i, (lq, lk) in enumerate(zip(lens_q, lens_k)):
        qa, qe, ka, ke = int(cu_q[i]), int(cu_q[i + 1]), int(cu_k[i]), int(cu_k[i + 1])
        if lq and not lk:
            # no keys: O = 0, LSE = +inf, no gradient
            assert (out[qa:qe] == 0).all() and (dq[qa:qe] == 0).all(), f"sequence {i}: rows without keys"
            assert torch.isinf(lse[i, :, :lq]).all() and (lse[i, :, :lq] > 0).all(), f"sequence {i}: lse"
            continue
        if lk and not lq:
            assert (dk[ka:ke] == 0).all() and (dv[ka:ke] == 0).all(), f"sequence {i}: keys without rows"
            continue
        if not lq:
            continue
        sl = lambda t, a, e: t.detach()[a:e].unsqueeze(0)  # noqa: E731
        r = _ref(sl(q, qa, qe), sl(k, ka, ke), sl(v, ka, ke), sl(g, qa, qe), causal)
        for j, (name, got) in enumerate((("out", out[qa:qe]), ("dq", dq[qa:qe]), ("dk", dk[ka:ke]),
                                         ("dv", dv[ka:ke]))):
            ok, err, bound = check_within_bound(got.float(), r["ref"][j][0].float(), r["pt"][j][0].float(),
                                                floor=1e-4)
            assert ok, f"sequence {i} ({lq} rows, {lk} keys): {name} max|err| {err:.3e} > bound {bound:.3e}"
        live = lse[i, :, :lq].detach()
        assert torch.isfinite(live).all(), f"sequence {i}: lse not finite"


# fixed-length calls with no keys (k / v of seqlen 0) or no query rows: refused with a RuntimeError.
# The reference does not define them either: seqlen_q = 0 launches an empty grid (grid.x = 0,
# flash_fwd_launch_template.h:21-61, a launch error) and seqlen_k = 0 starts its key loop at block -1
# (flash_fwd_kernel.h:300-303), reading before K.  Empty tensors reach the C ABI as null pointers,
# which it rejects (fa_capi.cpp fwd_impl).
@pytest.mark.parametrize("sq,sk", [(37, 0), (0, 50), (0, 0)])
@pytest.mark.parametrize("d", [64, 128, 96])
def test_fixed_length_without_keys_or_rows_is_refused(sq, sk, d):
    from flash_attn import flash_attn_func

    q = torch.randn(2, sq, 4, d, device=DEV, dtype=torch.bfloat16)
    k, v = (torch.randn(2, sk, 2, d, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    with pytest.raises(RuntimeError):
        flash_attn_func(q, k, v, causal=True)
    torch.cuda.synchronize()
