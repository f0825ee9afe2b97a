"""GPU parity tests of the MI355X FlashAttention-2 path against the oracle (run on a gfx950 box).

Structure follows the reference's tests/test_flash_attn.py: the HIP result must satisfy the
reference's acceptance rule ``max|x - ref| <= 2 * max|x_pt - ref|`` for out, dq, dk and dv, where
``ref`` is the oracle's fp32 attention and ``pt`` the same math in the input dtype with reordered
ops (the reference's own estimate of PyTorch's numerical error).  The oracle's torch
restatement runs on the kernel's device (as the reference's tests do); shapes are reduced in batch/heads (not in the seqlen / head-dim grid) so it finishes in
seconds.  Headline-size runs are checked through sampled rows against a float64 restatement.
"""
import math

import numpy as np
import pytest
import torch

from golden_io import Golden, golden_names
from oracle.attention_ref import (attention_lse_pt, attention_lse_ref, attention_ref, check_lse_within_bound,
                                  check_within_bound,
                                  generate_qkv, generate_random_padding_mask)

pytestmark = pytest.mark.gpu

DEV = "cuda"
DTYPES = [torch.float16, torch.bfloat16]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401  (fails loudly if the library is missing)


# The oracle's torch restatement runs on the same device as the kernel under test, exactly as the
# reference's own tests run attention_ref on cuda (tests/test_flash_attn.py:575-578): fp32 ``ref``
# and the low-precision ``pt`` estimate then share the device BLAS, and the suite finishes in
# minutes instead of hours of host matmuls.
REF_DEV = DEV


def _cpu_leaf(*xs):
    return [x.detach().to(REF_DEV).clone().requires_grad_() for x in xs]


def _assert_bound(name, got, ref, pt, factor=2.0, floor=0.0):
    ok, err, bound = check_within_bound(got.detach().to(ref.device), ref, pt.to(ref.device), factor=factor, floor=floor)
    assert ok, f"{name}: max|err| {err:.3e} > bound {bound:.3e}"


def _assert_lse(lse, ref, pt, atol=1e-3, rtol=1e-4):
    """softmax_lse under the 2x rule (oracle check_lse_within_bound): the forward holds Q as
    bf16/f16(scale log2(e) Q), one rounding of the kind the PyTorch path's k / sqrt(d) makes"""
    ok, err, pt_err = check_lse_within_bound(lse, ref, pt, atol=atol, rtol=rtol)
    assert ok, f"lse: max|err| {err:.3e} > max(2 x pt error {pt_err:.3e}, {atol} + {rtol} |ref|)"


def _ref_and_pt(q, k, v, qm=None, km=None, causal=False):
    out_ref, _ = attention_ref(q, k, v, qm, km, causal=causal)
    out_pt, _ = attention_ref(q, k, v, qm, km, causal=causal, upcast=False, reorder_ops=True)
    return out_ref, out_pt


# ------------------------------------------------------------------------------------------------
# golden vectors produced by the reference itself
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", [n for n in golden_names() if not n.startswith("c1_")])
def test_golden_parity(name):
    from flash_attn import flash_attn_func, flash_attn_varlen_qkvpacked_func
    from flash_attn.bert_padding import pad_input, unpad_input

    g = Golden(name)
    q, k, v = (g.t(x).to(DEV).requires_grad_() for x in ("q", "k", "v"))
    dout = g.t("dout").to(DEV)
    if g.kind == "dense":
        out, lse, _ = flash_attn_func(q, k, v, causal=g.causal, return_attn_probs=True)
        _assert_lse(lse, g.t("lse_ref"), attention_lse_pt(g.t("q"), g.t("k"), causal=g.causal))
        grads = torch.autograd.grad(out, (q, k, v), dout)
    else:
        mask = torch.from_numpy(g.z["mask"]).to(DEV)
        qkv_unpad = torch.stack([unpad_input(x, mask)[0] for x in (q, k, v)], dim=1).detach().requires_grad_()
        _, indices, cu, max_s = unpad_input(q, mask)
        out_unpad = flash_attn_varlen_qkvpacked_func(qkv_unpad, cu, max_s, causal=g.causal)
        out = pad_input(out_unpad, indices, g.b, g.sq)
        dqkv_unpad, = torch.autograd.grad(out_unpad, qkv_unpad, unpad_input(dout, mask)[0])
        dqkv = pad_input(dqkv_unpad, indices, g.b, g.sq)
        grads = dqkv.unbind(2)
    _assert_bound("out", out, g.t("out_ref"), g.t("out_pt"))
    for got, key in zip(grads, ("dq", "dk", "dv")):
        _assert_bound(key, got, g.t(key + "_ref"), g.t(key + "_pt"))


def test_fp32_rejected_like_reference():
    from flash_attn import flash_attn_func

    q = torch.randn(1, 16, 2, 64, device=DEV)
    with pytest.raises(RuntimeError, match="fp16 and bf16"):
        flash_attn_func(q, q, q)


# ------------------------------------------------------------------------------------------------
# test_flash_attn_output (reference :517-639) on a reduced batch / head count
# ------------------------------------------------------------------------------------------------
SEQ_PAIRS = [(113, 203), (128, 217), (113, 211), (108, 256), (256, 512), (512, 256),
             (1024, 1024), (1023, 1024), (1024, 1023)]


# (mha_type, kvpacked): the kvpacked layout is covered on GQA only (no skip-only combinations)
LAYOUTS = [("mha", False), ("mqa", False), ("gqa", False), ("gqa", True)]
LAYOUT_IDS = ["mha", "mqa", "gqa", "gqa-kvpacked"]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("mha_type,kvpacked", LAYOUTS, ids=LAYOUT_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 40, 59, 64, 80, 96, 111, 128, 160, 192, 224, 256])
@pytest.mark.parametrize("seqlen_q,seqlen_k", SEQ_PAIRS)
def test_flash_attn_output(seqlen_q, seqlen_k, d, causal, mha_type, kvpacked, dtype):
    from flash_attn import flash_attn_func, flash_attn_kvpacked_func

    torch.manual_seed(0)
    batch_size, nheads = 2, 6
    nheads_k = nheads if mha_type == "mha" else (1 if mha_type == "mqa" else 3)
    q = torch.randn(batch_size, seqlen_q, nheads, d, device=DEV, dtype=dtype, requires_grad=True)
    if kvpacked:
        kv = torch.randn(batch_size, seqlen_k, 2, nheads_k, d, device=DEV, dtype=dtype, requires_grad=True)
        out = flash_attn_kvpacked_func(q, kv, causal=causal)
        k, v = kv[:, :, 0], kv[:, :, 1]
    else:
        k = torch.randn(batch_size, seqlen_k, nheads_k, d, device=DEV, dtype=dtype, requires_grad=True)
        v = torch.randn(batch_size, seqlen_k, nheads_k, d, device=DEV, dtype=dtype, requires_grad=True)
        out = flash_attn_func(q, k, v, causal=causal)
    g = torch.randn_like(out)
    if kvpacked:
        dq, dkv = torch.autograd.grad(out, (q, kv), g)
        dk, dv = dkv.unbind(2)
    else:
        dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)

    qc, kc, vc = _cpu_leaf(q, k, v)
    out_ref, out_pt = _ref_and_pt(qc, kc, vc, causal=causal)
    _assert_bound("out", out, out_ref, out_pt)
    gc = g.to(REF_DEV)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), gc)
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), gc)
    for name, got, r, p in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        _assert_bound(name, got, r, p)


# ------------------------------------------------------------------------------------------------
# qkvpacked + varlen (reference :333-514, :642-783)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 64, 80, 128, 192, 256])
@pytest.mark.parametrize("seqlen", [97, 128, 200, 257, 384, 1025])
def test_flash_attn_qkvpacked(seqlen, d, causal, dtype):
    from flash_attn import flash_attn_qkvpacked_func

    torch.manual_seed(0)
    qkv = torch.randn(3, seqlen, 3, 5, d, device=DEV, dtype=dtype, requires_grad=True)
    out, lse, s_dmask = flash_attn_qkvpacked_func(qkv, 0.0, return_attn_probs=True, causal=causal)
    assert s_dmask is None
    g = torch.randn_like(out)
    dqkv, = torch.autograd.grad(out, qkv, g)
    qkvc = qkv.detach().to(REF_DEV).clone().requires_grad_()
    out_ref, _ = attention_ref(qkvc[:, :, 0], qkvc[:, :, 1], qkvc[:, :, 2], causal=causal)
    out_pt, _ = attention_ref(qkvc[:, :, 0], qkvc[:, :, 1], qkvc[:, :, 2], causal=causal,
                              upcast=False, reorder_ops=True)
    _assert_bound("out", out, out_ref, out_pt)
    qd, kd = qkv.detach()[:, :, 0], qkv.detach()[:, :, 1]
    _assert_lse(lse, attention_lse_ref(qd, kd, causal=causal), attention_lse_pt(qd, kd, causal=causal))
    dref, = torch.autograd.grad(out_ref, qkvc, g.to(REF_DEV))
    dpt, = torch.autograd.grad(out_pt, qkvc, g.to(REF_DEV))
    _assert_bound("dqkv", dqkv, dref, dpt)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("mha_type,kvpacked", LAYOUTS, ids=LAYOUT_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 64, 96, 128, 160, 256])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(113, 203), (128, 217), (256, 512), (512, 256), (1023, 1024)])
def test_flash_attn_varlen_output(seqlen_q, seqlen_k, d, causal, mha_type, kvpacked, dtype):
    from flash_attn import flash_attn_varlen_func, flash_attn_varlen_kvpacked_func

    torch.manual_seed(0)
    batch_size, nheads = 4, 6
    nheads_k = nheads if mha_type == "mha" else (1 if mha_type == "mqa" else 3)
    q = torch.randn(batch_size, seqlen_q, nheads, d, device=DEV, dtype=dtype)
    k = torch.randn(batch_size, seqlen_k, nheads_k, d, device=DEV, dtype=dtype)
    v = torch.randn(batch_size, seqlen_k, nheads_k, d, device=DEV, dtype=dtype)
    qm = generate_random_padding_mask(seqlen_q, batch_size, DEV, mode="random")
    km = generate_random_padding_mask(seqlen_k, batch_size, DEV, mode="random")
    if kvpacked:
        (q_unpad, kv_unpad, cu_q, cu_k, max_q, max_k, q, kv, out_pad_fn, dq_pad_fn,
         dkv_pad_fn) = generate_qkv(q, k, v, qm, km, kvpacked=True)
        out_unpad = flash_attn_varlen_kvpacked_func(q_unpad, kv_unpad, cu_q, cu_k, max_q, max_k, causal=causal)
    else:
        (q_unpad, k_unpad, v_unpad, cu_q, cu_k, max_q, max_k, q, k, v, out_pad_fn, dq_pad_fn,
         dk_pad_fn) = generate_qkv(q, k, v, qm, km)
        out_unpad = flash_attn_varlen_func(q_unpad, k_unpad, v_unpad, cu_q, cu_k, max_q, max_k, causal=causal)
    out = out_pad_fn(out_unpad)
    g = torch.randn_like(out)
    if kvpacked:
        dq_unpad, dkv_unpad = torch.autograd.grad(out_unpad, (q_unpad, kv_unpad), g[qm])
        dk, dv = dkv_pad_fn(dkv_unpad).unbind(2)
        k, v = kv[:, :, 0], kv[:, :, 1]
    else:
        dq_unpad, dk_unpad, dv_unpad = torch.autograd.grad(out_unpad, (q_unpad, k_unpad, v_unpad), g[qm])
        dk, dv = dk_pad_fn(dk_unpad), dk_pad_fn(dv_unpad)
    dq = dq_pad_fn(dq_unpad)

    qc, kc, vc = _cpu_leaf(q, k, v)
    qmc, kmc = qm.to(REF_DEV), km.to(REF_DEV)
    out_ref, out_pt = _ref_and_pt(qc, kc, vc, qmc, kmc, causal=causal)
    _assert_bound("out", out, out_ref, out_pt)
    gc = g.to(REF_DEV).masked_fill(~qmc[:, :, None, None], 0)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), gc)
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), gc)
    for name, got, r, p in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        _assert_bound(name, got, r, p)


# ------------------------------------------------------------------------------------------------
# determinism (reference test_flash_attn_race_condition :786-832)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 64, 96, 128, 256])
def test_flash_attn_race_condition(d, causal, dtype):
    from flash_attn import flash_attn_qkvpacked_func

    torch.manual_seed(0)
    qkv = torch.randn(60, 128, 3, 4, d, device=DEV, dtype=dtype, requires_grad=True)
    out0, lse0, _ = flash_attn_qkvpacked_func(qkv, 0.0, return_attn_probs=True, causal=causal)
    g = torch.randn_like(out0)
    dqkv0, = torch.autograd.grad(out0, qkv, g)
    dq_atol = 2 * ((dqkv0[:, :, 0] + 0.3 - 0.3) - dqkv0[:, :, 0]).abs().max().item()
    for _ in range(25):
        out, lse, _ = flash_attn_qkvpacked_func(qkv, 0.0, return_attn_probs=True, causal=causal)
        assert torch.equal(out, out0)
        assert torch.equal(lse, lse0)
        dqkv, = torch.autograd.grad(out, qkv, g)
        assert torch.allclose(dqkv[:, :, 0], dqkv0[:, :, 0], atol=dq_atol)
        assert torch.equal(dqkv[:, :, 1], dqkv0[:, :, 1])
        assert torch.equal(dqkv[:, :, 2], dqkv0[:, :, 2])


# ------------------------------------------------------------------------------------------------
# edge cases (reference :835-959)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [16, 32, 64])
@pytest.mark.parametrize("seqlen", [1, 2, 5, 17, 128])
def test_flash_attn_bwd_overflow(seqlen, d, causal):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    dtype = torch.float16
    q = (torch.randn(2, seqlen, 5, d, dtype=dtype, device=DEV) * 5).requires_grad_()
    k, v = [(torch.randn(2, seqlen, 5, d, dtype=dtype, device=DEV) * 3).requires_grad_() for _ in range(2)]
    out = flash_attn_func(q, k, v, causal=causal)
    g = torch.randn_like(out)
    out.backward(g)
    qc, kc, vc = _cpu_leaf(q, k, v)
    out_ref, out_pt = _ref_and_pt(qc, kc, vc, causal=causal)
    _assert_bound("out", out, out_ref, out_pt)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), g.to(REF_DEV))
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), g.to(REF_DEV))
    for name, got, r, p in zip(("dq", "dk", "dv"), (q.grad, k.grad, v.grad), gr, gp):
        _assert_bound(name, got, r, p, factor=5.0, floor=1e-3)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("seqlen", [97, 128, 200, 256])
def test_flash_attn_bwd_transpose(seqlen, d, causal, dtype):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    q, k, v = [torch.randn(5, seqlen, 2, d, dtype=dtype, device=DEV, requires_grad=True) for _ in range(3)]
    out = flash_attn_func(q, k, v, causal=causal).transpose(0, 1)
    g = torch.randn(seqlen, 10, 2, d, dtype=dtype, device=DEV)[:, ::2]   # non-contiguous dout
    out.backward(g)
    qc, kc, vc = _cpu_leaf(q, k, v)
    out_ref, out_pt = _ref_and_pt(qc, kc, vc, causal=causal)
    gc = g.to(REF_DEV).transpose(0, 1)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), gc)
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), gc)
    _assert_bound("out", out.transpose(0, 1), out_ref, out_pt)
    for name, got, r, p in zip(("dq", "dk", "dv"), (q.grad, k.grad, v.grad), gr, gp):
        _assert_bound(name, got, r, p)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [16, 32, 64])
def test_flash_attn_bwd_varlen_overflow(d, causal):
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(0)
    dtype = torch.float16
    cu_q = torch.tensor([0, 76, 110, 256], device=DEV, dtype=torch.int32)
    cu_k = torch.tensor([0, 1, 2, 3], device=DEV, dtype=torch.int32)
    q = (torch.randn(256, 5, d, dtype=dtype, device=DEV) * 3).requires_grad_()
    k, v = [(torch.randn(3, 5, d, dtype=dtype, device=DEV) * 3).requires_grad_() for _ in range(2)]
    out = flash_attn_varlen_func(q, k, v, cu_q, cu_k, 256, 3, causal=causal)
    out.backward(torch.randn_like(out))
    assert not q.grad.isnan().any()
    assert not k.grad.isnan().any()
    assert not v.grad.isnan().any()


# ------------------------------------------------------------------------------------------------
# C-ABI level: Paddle-style call with expanded GQA gradients and raw pointers
# ------------------------------------------------------------------------------------------------
def test_capi_expanded_gqa_matches_fused_reduction():
    import flash_attn_2_cuda as m
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, s, h, hk, d = 2, 300, 8, 2, 128
    q = torch.randn(b, s, h, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(b, s, hk, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(b, s, hk, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out, lse, _ = flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
    g = torch.randn_like(out)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)

    sq_r = (s + 127) // 128 * 128
    dq2 = torch.empty_like(q)
    dk_exp = torch.empty(b, s, h, d, device=DEV, dtype=q.dtype)
    dv_exp = torch.empty_like(dk_exp)
    softmax_d = torch.empty(b, h, sq_r, device=DEV)
    dq_accum = torch.empty(b, h, sq_r, 128, device=DEV)
    P = m._ptr
    st = lambda t: (t.stride(1), t.stride(2), t.stride(0))  # noqa: E731 (row, head, batch)
    (qr, qh, qb), (kr, kh, kb), (vr, vh, vb), (orr, oh, ob) = st(q), st(k), st(v), st(out)
    (dqr, dqh, dqb), (dkr, dkh, dkb), (dvr, dvh, dvb), (dor, doh, dob) = st(dq2), st(dk_exp), st(dv_exp), st(g)
    ok = m._lib.flash_attn_bwd(P(g), P(q), P(k), P(v), P(out), P(softmax_d), P(lse), None, P(dq2),
                               P(dk_exp), P(dv_exp), P(dq_accum), b, s, s, sq_r, sq_r, h, hk, d, 128,
                               0.0, d ** -0.5, 1.0, True, True, 1, m._stream(q), 0, 0,
                               None, None, None, None, None, None, None, None,
                               qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob,
                               dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, dqb, dkb, dvb, dob)
    assert ok, m._lib.flash_attn_error()
    torch.cuda.synchronize()
    assert torch.allclose(dq2.float(), dq.float(), atol=2e-2)
    dk_sum = dk_exp.float().reshape(b, s, hk, h // hk, d).sum(3)
    dv_sum = dv_exp.float().reshape(b, s, hk, h // hk, d).sum(3)
    torch.testing.assert_close(dk_sum, dk.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(dv_sum, dv.float(), atol=3e-2, rtol=2e-2)


def test_return_softmax_requires_dropout_and_mask_needs_dims():
    """Reference mha_fwd: return_softmax only with p_dropout > 0 (flash_api.cpp:276-279); a dense
    Paddle mask without its mask_dims is rejected loudly (mask parity: tests/test_mask_gpu.py)."""
    import flash_attn_2_cuda as m

    q = torch.randn(1, 64, 2, 64, device=DEV, dtype=torch.float16)
    with pytest.raises(RuntimeError, match="return_softmax"):
        m.fwd(q, q, q, None, 0.0, 0.125, False, True, None)
    lse = torch.empty(1, 2, 64, device=DEV)
    out = torch.empty_like(q)
    st = (q.stride(1), q.stride(1), q.stride(1), q.stride(2), q.stride(2), q.stride(2), out.stride(1),
          out.stride(2), q.stride(0), q.stride(0), q.stride(0), out.stride(0))
    ok = m._lib.flash_attn_fwd(m._ptr(q), m._ptr(q), m._ptr(q), None, m._ptr(out), None, m._ptr(lse),
                               1, 64, 64, 128, 128, 2, 2, 64, 64, 0.0, 0.125, 1.0, False, False, False,
                               m._stream(q), 0, 0, m._ptr(lse), None, None, None, None, None, None,
                               None, *st)
    assert not ok and b"mask_dims" in m._lib.flash_attn_error()


# ------------------------------------------------------------------------------------------------
# headline sizes: sampled rows / keys against a float64 restatement (size-independent check)
# ------------------------------------------------------------------------------------------------
def _rows_fp64(q, k, v, dout, b, h, rows, keys, causal, scale):
    """float64 O, LSE, dQ for the given query rows and dK, dV for the given keys of (b, h)."""
    hk_idx = h // (q.shape[2] // k.shape[2])
    Q = q[b, :, h].double().cpu().numpy()
    K = k[b, :, hk_idx].double().cpu().numpy()
    V = v[b, :, hk_idx].double().cpu().numpy()
    dO = dout[b, :, h].double().cpu().numpy()
    sq, sk = Q.shape[0], K.shape[0]

    def row_probs(i):
        s = (K @ Q[i]) * scale
        if causal:
            s[i + 1:] = -np.inf
        m = s.max()
        e = np.exp(s - m)
        return e / e.sum(), m + np.log(e.sum())

    O_all = np.zeros((sq, Q.shape[1]))
    lse_all = np.zeros(sq)
    # D = rowsum(dO * O) needs O for every query that touches the sampled keys: compute all rows
    S = (Q @ K.T) * scale
    if causal:
        S = np.where(np.triu(np.ones((sq, sk), dtype=bool), 1), -np.inf, S)
    M = S.max(1, keepdims=True)
    E = np.exp(S - M)
    L = E.sum(1, keepdims=True)
    Pm = E / L
    O_all = Pm @ V
    lse_all = (M + np.log(L))[:, 0]
    Dsum = (dO * O_all).sum(1)
    dP = dO @ V.T
    dS = Pm * (dP - Dsum[:, None])
    res = dict(O=O_all[rows], lse=lse_all[rows], dQ=scale * (dS[rows] @ K))
    res["dK"] = scale * (dS[:, keys].T @ Q)
    res["dV"] = Pm[:, keys].T @ dO
    return res


@pytest.mark.parametrize("cfg", [
    dict(b=4, s=8192, h=16, hk=16, d=128, dtype=torch.bfloat16, causal=True),    # C3 headline
    dict(b=4, s=2048, h=16, hk=16, d=64, dtype=torch.bfloat16, causal=True),     # C2
    dict(b=1, s=8192, h=32, hk=8, d=128, dtype=torch.float16, causal=True),      # C5-class GQA
])
def test_headline_sizes_sampled(cfg):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, s, h, hk, d, dtype, causal = (cfg[x] for x in ("b", "s", "h", "hk", "d", "dtype", "causal"))
    q = torch.randn(b, s, h, d, device=DEV, dtype=dtype, requires_grad=True)
    k = torch.randn(b, s, hk, d, device=DEV, dtype=dtype, requires_grad=True)
    v = torch.randn(b, s, hk, d, device=DEV, dtype=dtype, requires_grad=True)
    out, lse, _ = flash_attn_func(q, k, v, causal=causal, return_attn_probs=True)
    g = torch.randn_like(out)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
    assert torch.isfinite(out).all() and torch.isfinite(dq).all()
    assert torch.isfinite(dk).all() and torch.isfinite(dv).all()
    rng = np.random.RandomState(0)
    # tolerances: |x| is O(1) for out; 16-bit storage rounding (2^-8 bf16 / 2^-11 fp16 relative)
    # plus fp32 accumulation error -- stated explicitly instead of the 2x-pt rule, which needs a
    # full-size low-precision reference.
    tol = 2.0 ** -6 if dtype == torch.bfloat16 else 2.0 ** -8
    scale = d ** -0.5
    for (bi, hi) in [(0, 0), (b - 1, h - 1)]:
        rows = np.sort(rng.choice(s, 24, replace=False))
        keys = np.sort(rng.choice(s, 24, replace=False))
        ref = _rows_fp64(q.detach(), k.detach(), v.detach(), g, bi, hi, rows, keys, causal, scale)
        o = out.detach()[bi, rows, hi].double().cpu().numpy()
        np.testing.assert_allclose(o, ref["O"], atol=tol * max(1.0, np.abs(ref["O"]).max()), rtol=0)
        # LSE of the PyTorch-precision path for these rows: bf16/f16 scores q (k / sqrt(d))
        rr = torch.as_tensor(rows, device=q.device)
        sp = (q.detach()[bi, rr, hi] @ (k.detach()[bi, :, hi // (h // hk)] / d ** 0.5).T).float()
        if causal:
            sp = sp.masked_fill(torch.arange(s, device=q.device)[None, :] > rr[:, None], float("-inf"))
        _assert_lse(lse.detach()[bi, hi, rows], torch.from_numpy(ref["lse"]), torch.logsumexp(sp, -1), atol=2e-3)
        gq = dq[bi, rows, hi].double().cpu().numpy()
        np.testing.assert_allclose(gq, ref["dQ"], atol=tol * max(1.0, np.abs(ref["dQ"]).max()), rtol=0)
        if hk == h:
            gk = dk[bi, keys, hi].double().cpu().numpy()
            gv = dv[bi, keys, hi].double().cpu().numpy()
            np.testing.assert_allclose(gk, ref["dK"], atol=tol * max(1.0, np.abs(ref["dK"]).max()), rtol=0)
            np.testing.assert_allclose(gv, ref["dV"], atol=tol * max(1.0, np.abs(ref["dV"]).max()), rtol=0)


# ------------------------------------------------------------------------------------------------
# deferred-max rescale (fa_fwd.hip kFwdRescaleThr): inputs that FORCE the rare branches
# (cdna_hip_programming.md §5.4 rule 26) -- a key that jumps a row's max far past the threshold
# at a late tile, and keys that raise the max gradually (each step below the threshold, so P grows
# towards 2^8 before a rescale) -- checked with the reference's 2x rule on out and grads.
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("mode", ["jump", "ramp"])
def test_fwd_deferred_max_forced(mode, causal, dtype):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, s, h, d = 2, 1024, 2, 128
    q = torch.randn(b, s, h, d, device=DEV, dtype=torch.float32)
    k = torch.randn(b, s, h, d, device=DEV, dtype=torch.float32)
    v = torch.randn(b, s, h, d, device=DEV, dtype=torch.float32)
    qn = q / q.norm(dim=-1, keepdim=True)
    rows = [700, 901, 1023, 777]
    for i in rows:
        if mode == "jump":
            # one key at a late tile with score ~ +24 (natural log) above the rest for row i
            j = i - 3
            k[:, j] = qn[:, i] * (24.0 * d ** 0.5)
        else:
            # keys 64 apart whose scores for row i rise by ~2 per tile: many sub-threshold steps
            for t, j in enumerate(range(i % 64, i + 1, 64)):
                k[:, j] = qn[:, i] * ((2.0 * t) * d ** 0.5 / 1.0)
    q, k, v = (x.to(dtype).requires_grad_() for x in (q, k, v))
    out = flash_attn_func(q, k, v, causal=causal)
    g = torch.randn_like(out)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
    assert torch.isfinite(out).all() and torch.isfinite(dq).all()
    qc, kc, vc = _cpu_leaf(q, k, v)
    out_ref, out_pt = _ref_and_pt(qc, kc, vc, causal=causal)
    _assert_bound("out", out, out_ref, out_pt)
    gc = g.to(REF_DEV)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), gc)
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), gc)
    for name, got, r, p in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        _assert_bound(name, got, r, p)


# ------------------------------------------------------------------------------------------------
# XCD-grouped work order (fa_common.h xcd_order_grouped): launches whose K/V stream exceeds the
# 256 MiB Infinity Cache run a head-grouped order; the result must be bitwise the head-fastest one
# (the NO_XCD_GROUP switch, tests/knobs.py, forces that order).
# ------------------------------------------------------------------------------------------------
def test_xcd_grouped_order_is_bitwise_head_fastest():
    from flash_attn import flash_attn_func
    from knobs import NO_XCD_GROUP, knob

    torch.manual_seed(0)
    # K + V = 402 MB > 256 MiB: grouped order for the forward and dQ kernels
    q = torch.randn(3, 16384, 32, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(3, 16384, 16, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(3, 16384, 16, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn_like(q)
    res = {}
    for flag in ("0", "1"):
        with knob(NO_XCD_GROUP, int(flag)):
            out, lse, _ = flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
            dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
            torch.cuda.synchronize()
        res[flag] = (out, lse, dq, dk, dv)
    for name, a, b in zip(("out", "lse", "dq", "dk", "dv"), res["0"], res["1"]):
        assert torch.isfinite(a.float()).all(), name
        assert torch.equal(a, b), name
