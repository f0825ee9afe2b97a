"""Pins the oracle (oracle/attention_ref.py) to the reference's own outputs (tests/golden/).

CPU only.  Every golden case was produced by running the reference's ``attention_ref`` /
``bert_padding`` (see tests/golden/make_golden.py); here the repo's restatements must reproduce
them: the torch restatement bit-for-bit (same ops on the same CPU), the float64 numpy kernel
restatement within the reference's own error bound, and the varlen builders exactly.
"""
import math

import numpy as np
import pytest
import torch

from golden_io import Golden, golden_names
from oracle.attention_ref import (attention_lse_ref, attention_ref, check_within_bound,
                                  flash_bwd_np, flash_fwd_np, generate_qkv)

NAMES = golden_names()
DENSE = [n for n in NAMES if not n.startswith("varlen")]
VARLEN = [n for n in NAMES if n.startswith("varlen")]


def test_golden_present():
    assert len(DENSE) >= 8 and len(VARLEN) >= 2


def _grad_inputs(g):
    return [g.t(x).clone().requires_grad_() for x in ("q", "k", "v")]


@pytest.mark.parametrize("name", NAMES)
def test_attention_ref_matches_reference(name):
    g = Golden(name)
    q, k, v = _grad_inputs(g)
    dout = g.t("dout")
    qm = km = None
    if g.kind == "varlen":
        qm = km = torch.from_numpy(g.z["mask"])
    out_ref, _ = attention_ref(q, k, v, qm, km, causal=g.causal)
    out_pt, _ = attention_ref(q, k, v, qm, km, causal=g.causal, upcast=False, reorder_ops=True)
    assert torch.equal(out_ref, g.t("out_ref"))
    assert torch.equal(out_pt, g.t("out_pt"))
    grads_ref = torch.autograd.grad(out_ref, (q, k, v), dout)
    grads_pt = torch.autograd.grad(out_pt, (q, k, v), dout)
    for got, key in zip(grads_ref, ("dq_ref", "dk_ref", "dv_ref")):
        assert torch.equal(got, g.t(key)), key
    for got, key in zip(grads_pt, ("dq_pt", "dk_pt", "dv_pt")):
        assert torch.equal(got, g.t(key)), key


@pytest.mark.parametrize("name", DENSE)
def test_lse_ref(name):
    g = Golden(name)
    lse = attention_lse_ref(g.t("q"), g.t("k"), causal=g.causal)
    torch.testing.assert_close(lse, g.t("lse_ref"), rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("name", DENSE)
def test_numpy_kernel_restatement(name):
    """float64 restatement of the kernel algebra is inside the reference's 2x bound everywhere."""
    g = Golden(name)
    q, k, v, dout = (g.t(x).double().numpy() for x in ("q", "k", "v", "dout"))
    out_ref, out_pt = g.t("out_ref"), g.t("out_pt")
    floor = 1e-5 if g.dtype == torch.float32 else 0.0
    for bi in range(g.b):
        o, lse = flash_fwd_np(q[bi], k[bi], v[bi], causal=g.causal)
        ok, err, bound = check_within_bound(torch.from_numpy(o).to(g.dtype), out_ref[bi], out_pt[bi], floor=floor)
        assert ok, (err, bound)
        np.testing.assert_allclose(lse, g.t("lse_ref")[bi].double().numpy(), rtol=1e-6, atol=1e-5)
        dq, dk, dv = flash_bwd_np(q[bi], k[bi], v[bi], o, dout[bi], lse, causal=g.causal)
        for got, key in zip((dq, dk, dv), ("dq", "dk", "dv")):
            ok, err, bound = check_within_bound(torch.from_numpy(got).to(g.dtype), g.t(key + "_ref")[bi],
                                                g.t(key + "_pt")[bi], floor=floor)
            assert ok, (key, err, bound)


def test_c1_exact_float64():
    """C1 (fp32, d=64) has a zero-width 2x bound (power-of-two scale): pin to fp64 at atol 1e-5."""
    g = Golden("c1_fp32_b2_s128_h4_d64")
    q, k, v = (g.t(x).double().numpy() for x in ("q", "k", "v"))
    for bi in range(g.b):
        o, _ = flash_fwd_np(q[bi], k[bi], v[bi], causal=False)
        np.testing.assert_allclose(o, g.t("out_ref")[bi].double().numpy(), atol=1e-5, rtol=0)
    # and against torch SDPA on CPU (the reference's "PyTorch SDPA path on the host CPU")
    qt, kt, vt = (g.t(x).transpose(1, 2) for x in ("q", "k", "v"))
    sdpa = torch.nn.functional.scaled_dot_product_attention(qt, kt, vt).transpose(1, 2)
    torch.testing.assert_close(sdpa, g.t("out_ref"), atol=1e-5, rtol=0)


@pytest.mark.parametrize("name", VARLEN)
def test_varlen_builders(name):
    from flash_attn.bert_padding import pad_input, unpad_input

    g = Golden(name)
    mask = torch.from_numpy(g.z["mask"])
    q = g.t("q")
    q_unpad, indices, cu_seqlens, max_seqlen = unpad_input(q, mask)
    assert torch.equal(cu_seqlens, torch.from_numpy(g.z["cu_seqlens"]))
    assert torch.equal(indices, torch.from_numpy(g.z["indices"]))
    assert max_seqlen == int(g.z["max_seqlen"])
    assert cu_seqlens.dtype == torch.int32
    back = pad_input(q_unpad, indices, g.b, g.sq)
    assert torch.equal(back, q.masked_fill(~mask[:, :, None, None], 0))
    # generate_qkv packs the same tokens
    qkv_unpad, cu2, ms2, _, out_pad_fn, _ = generate_qkv(q, g.t("k"), g.t("v"), mask, mask, qkvpacked=True)
    assert torch.equal(cu2, cu_seqlens) and ms2 == max_seqlen
    assert torch.equal(qkv_unpad[:, 0].detach(), q_unpad)


def test_bert_padding_gradients():
    from flash_attn.bert_padding import index_first_axis, pad_input

    torch.manual_seed(0)
    x = torch.randn(10, 3, requires_grad=True)
    idx = torch.tensor([7, 2, 5])
    y = index_first_axis(x, idx)
    y.sum().backward()
    expect = torch.zeros(10, 3)
    expect[idx] = 1
    assert torch.equal(x.grad, expect)
    t = torch.randn(3, 4, requires_grad=True)
    p = pad_input(t, idx, 2, 5)
    assert p.shape == (2, 5, 4)
    (p * 2).sum().backward()
    assert torch.equal(t.grad, torch.full((3, 4), 2.0))


def test_empty_row_lse_is_inf():
    """A row with no admissible key has LSE = +inf and O = 0 (flash_fwd_kernel.h:509-518)."""
    q = np.random.RandomState(0).randn(4, 1, 8)
    k = np.random.RandomState(1).randn(0, 1, 8)
    v = np.random.RandomState(2).randn(0, 1, 8)
    o, lse = flash_fwd_np(q, k, v)
    assert np.all(o == 0) and np.all(np.isinf(lse))
    assert math.isinf(float(attention_lse_ref(torch.zeros(1, 2, 1, 8), torch.zeros(1, 0, 1, 8)).max()))
