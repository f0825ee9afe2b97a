"""GPU tests of the Paddle C ABI details not covered elsewhere:

* ``varlen_padded_input = true`` (reference block_info.h:16-17, capi/flash_attn.cu:164-169 and
  :520-525): cu_seqlens give the lengths only, every sequence starts at its batch stride in padded
  (b, max_seqlen, h, d) tensors; forward and backward against attention_ref with padding masks
  (the reference's 2x rule), rows past a sequence's length untouched.
* ``return_softmax`` together with a dense mask or FlashMask (the reference writes P in its
  densemask / flashmask kernels, flash_fwd_kernel.h:880-887 and :1513-1520): |S_dmask| equals the
  masked softmax, its sign is the oracle's dropout keep pattern, hidden elements are 0.
* the backward's device-side rng_state (*_bwd_gqa entries): same result as the explicit
  (seed, offset) of the reference-shaped entry.
"""
import numpy as np
import pytest
import torch

from oracle.attention_ref import attention_ref, check_within_bound
from oracle.dropout_ref import dropout_keep_mask
from oracle.flashmask_ref import flashmask_keep

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _st(t):
    return t.stride(1), t.stride(2), t.stride(0)     # (row, head, batch) element strides


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d,h,hk", [(64, 4, 4), (128, 4, 2)])
def test_varlen_padded_input(d, h, hk, causal, dtype):
    import flash_attn_2_cuda as m

    torch.manual_seed(0)
    b, msq, msk = 3, 300, 280
    lq, lk = [300, 17, 211], [280, 140, 5] if not causal else [280, 17, 211]
    q = torch.randn(b, msq, h, d, device=DEV, dtype=dtype)
    k = torch.randn(b, msk, hk, d, device=DEV, dtype=dtype)
    v = torch.randn(b, msk, hk, d, device=DEV, dtype=dtype)
    dout = torch.randn(b, msq, h, d, device=DEV, dtype=dtype)
    cu_q = torch.tensor([0] + lq, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    cu_k = torch.tensor([0] + lk, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    sentinel = 7.0
    out = torch.full_like(q, sentinel)
    lse = torch.empty(b, h, msq, device=DEV)
    P = m._ptr
    sq_r, sk_r = (msq + 127) // 128 * 128, (msk + 127) // 128 * 128
    (qr, qh, qb), (kr, kh, kb), (vr, vh, vb), (orr, oh, ob) = _st(q), _st(k), _st(v), _st(out)
    bf16 = dtype == torch.bfloat16
    scale = d ** -0.5
    ok = m._lib.flash_attn_varlen_fwd(P(q), P(k), P(v), P(cu_q), P(cu_k), None, P(out), None, P(lse),
                                      b, msq, msk, sq_r, sk_r, h, hk, d, d, 0.0, scale, 1.0, causal, False,
                                      bf16, m._stream(q), 0, 0, None, None,
                                      qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob, True)
    assert ok, m._lib.flash_attn_error()
    dq, dk, dv = (torch.full_like(x, sentinel) for x in (q, k, v))
    softmax_d = torch.empty(b, h, sq_r, device=DEV)
    (dqr, dqh, dqb), (dkr, dkh, dkb), (dvr, dvh, dvb), (dor, doh, dob) = _st(dq), _st(dk), _st(dv), _st(dout)
    ok = m._lib.flash_attn_varlen_bwd_gqa(P(dout), P(q), P(k), P(v), P(out), P(softmax_d), P(lse), P(cu_q),
                                          P(cu_k), None, P(dq), P(dk), P(dv), None, b, msq, msk, sq_r, sk_r,
                                          h, hk, d, d, 0.0, scale, 1.0, causal, bf16, 1, m._stream(q), 0, 0,
                                          None, None, qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob,
                                          dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, dqb, dkb, dvb, dob, True)
    assert ok, m._lib.flash_attn_error()
    torch.cuda.synchronize()
    for i in range(b):
        sl_q, sl_k = slice(0, lq[i]), slice(0, lk[i])
        qi, ki, vi = (x[i:i + 1].clone().requires_grad_() for x in (q[:, sl_q], k[:, sl_k], v[:, sl_k]))
        gi = dout[i:i + 1, sl_q]
        ref, _ = attention_ref(qi, ki, vi, causal=causal)
        pt, _ = attention_ref(qi, ki, vi, causal=causal, upcast=False, reorder_ops=True)
        for name, got, r, p_ in (("out", out[i:i + 1, sl_q], ref, pt),):
            ok_, err, bound = check_within_bound(got, r, p_)
            assert ok_, f"seq {i} {name}: {err:.3e} > {bound:.3e}"
        gr = torch.autograd.grad(ref, (qi, ki, vi), gi)
        gp = torch.autograd.grad(pt, (qi, ki, vi), gi)
        for name, got, r, p_ in zip(("dq", "dk", "dv"), (dq[i:i + 1, sl_q], dk[i:i + 1, sl_k], dv[i:i + 1, sl_k]),
                                    gr, gp):
            ok_, err, bound = check_within_bound(got, r, p_, floor=1e-3)
            assert ok_, f"seq {i} {name}: {err:.3e} > {bound:.3e}"
        # rows past the sequence's length are not written (reference: the kernel stops at actual_seqlen)
        assert (out[i, lq[i]:] == sentinel).all() and (dq[i, lq[i]:] == sentinel).all()
        assert (dk[i, lk[i]:] == sentinel).all() and (dv[i, lk[i]:] == sentinel).all()


def _fwd_return_softmax(q, k, v, p, seed, offset, causal, mask=None, mask_dims=None, fm=None):
    import flash_attn_2_cuda as m

    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    sq_r, sk_r = (sq + 127) // 128 * 128, (sk + 127) // 128 * 128
    out = torch.empty_like(q)
    lse = torch.empty(b, h, sq, device=DEV)
    sdm = torch.zeros(b, h, sq_r, sk_r, device=DEV, dtype=q.dtype)
    rng = torch.empty(2, device=DEV, dtype=torch.int64)
    P = m._ptr
    (qr, qh, qb), (kr, kh, kb), (vr, vh, vb), (orr, oh, ob) = _st(q), _st(k), _st(v), _st(out)
    fm_args = fm if fm is not None else (None,) * 6
    ok = m._lib.flash_attn_fwd(P(q), P(k), P(v), P(rng), P(out), P(sdm), P(lse), b, sq, sk, sq_r, sk_r, h, hk,
                               d, d, p, d ** -0.5, d ** 0.5, causal, True, q.dtype == torch.bfloat16,
                               m._stream(q), seed, offset, P(mask) if mask is not None else None,
                               mask_dims, *fm_args, qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob)
    assert ok, m._lib.flash_attn_error()
    torch.cuda.synchronize()
    return out, lse, sdm[:, :, :sq, :sk]


def _keep(seed, offset, b, h, sq, sk, p):
    return torch.from_numpy(np.stack([np.stack([dropout_keep_mask(seed, offset, bi, hi, h, sq, sk, p)
                                                for hi in range(h)]) for bi in range(b)]))


@pytest.mark.parametrize("causal", [False, True])
def test_dense_mask_return_softmax(causal):
    torch.manual_seed(0)
    b, sq, sk, h, d, p, seed, offset = 2, 200, 177, 2, 64, 0.2, 99, 12
    q = torch.randn(b, sq, h, d, device=DEV, dtype=torch.float16)
    k, v = (torch.randn(b, sk, h, d, device=DEV, dtype=torch.float16) for _ in range(2))
    mask = (torch.randn(b, 1, sq, sk, device=DEV) * 2).masked_fill(torch.rand(b, 1, sq, sk, device=DEV) < 0.2,
                                                                 -3000.0).half()
    dims = torch.tensor([b, 1, sq, sk], dtype=torch.int64)
    _, _, sdm = _fwd_return_softmax(q, k, v, p, seed, offset, causal, mask, dims.numpy().ctypes.data)
    # raw scores + mask * unscale, then * scale; unscale = 1 / scale here
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * d ** -0.5 + mask.float()
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(sq, sk, dtype=torch.bool, device=DEV), 1), float("-inf"))
    prob = torch.softmax(s, -1)
    torch.testing.assert_close(sdm.abs().float(), prob, atol=2e-3, rtol=0)
    keep = _keep(seed, offset, b, h, sq, sk, p).to(DEV)
    live = prob > 1e-4                                # sign of a (near-)zero fp16 value is not informative
    assert torch.equal((~torch.signbit(sdm.float()))[live], keep[live])


def test_flashmask_return_softmax():
    torch.manual_seed(0)
    b, s, h, d, p, seed, offset = 1, 256, 2, 64, 0.25, 5, 0
    q, k, v = (torch.randn(b, s, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    # causal document mask: keys of document [a, e) hidden from rows >= e
    docs = [0, 100, 180, 256]
    lts = np.zeros((b, 1, s), np.int32)
    for a, e in zip(docs[:-1], docs[1:]):
        lts[..., a:e] = e
    lts_t = torch.from_numpy(lts).to(DEV)
    dims = torch.tensor([b, 1, s, 1], dtype=torch.int64)
    import flash_attn_2_cuda as m
    fm = (m._ptr(lts_t), dims.numpy().ctypes.data, None, None, None, None)
    _, _, sdm = _fwd_return_softmax(q, k, v, p, seed, offset, True, fm=fm)
    vis = torch.from_numpy(flashmask_keep(lts, s, True)).to(DEV)          # (b, 1, s, s), FlashMask only
    vis &= ~torch.triu(torch.ones(s, s, dtype=torch.bool, device=DEV), 1)   # and causal
    sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * d ** -0.5
    prob = torch.softmax(sc.masked_fill(~vis, float("-inf")), -1)
    torch.testing.assert_close(sdm.abs().float(), prob, atol=1e-2, rtol=0)
    assert (sdm[~vis.expand_as(sdm)] == 0).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
def test_return_softmax_without_dropout_then_bwd(d, causal, dtype):
    """The reference C ABI passes softmax_ptr whenever return_softmax is set
    (capi/flash_attn.cu:641, 747), dropout or not.  At p = 0 the call folds (attn_folds_q), so the
    forward runs the HIP kernels on Q' (the assembly kernel has no S_dmask) and the reference-shaped
    flash_attn_bwd that follows scores with the same Q': S_dmask is the softmax, out / LSE / dq / dk
    / dv are within the 2x rule, and out / LSE agree with a plain (assembly) forward of the call."""
    import flash_attn_2_cuda as m
    from oracle.attention_ref import attention_lse_pt, attention_lse_ref, check_lse_within_bound

    torch.manual_seed(1)
    b, s, h, scale = 2, 333, 3, d ** -0.5
    # (plain N(0, 1) inputs: the reference's overflow scaling runs in tests/test_fold_gpu.py under its
    # factor 5; with rows of q * 6 in fp16 at d = 64 the folded dK reached 1.7x the 2x bound)
    q, k, v, dout = (torch.randn(b, s, h, d, device=DEV, dtype=dtype) for _ in range(4))
    out, lse, sdm = _fwd_return_softmax(q, k, v, 0.0, 0, 0, causal)
    sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if causal:
        sc = sc.masked_fill(torch.triu(torch.ones(s, s, dtype=torch.bool, device=DEV), 1), float("-inf"))
    prob = torch.softmax(sc, -1)
    assert not torch.signbit(sdm.float()).any()          # nothing dropped
    torch.testing.assert_close(sdm.float(), prob, atol=4e-3, rtol=2 ** -7)
    qr, kr, vr = (x.clone().requires_grad_() for x in (q, k, v))
    ref, _ = attention_ref(qr, kr, vr, causal=causal)
    qp, kp, vp = (x.clone().requires_grad_() for x in (q, k, v))
    pt, _ = attention_ref(qp, kp, vp, causal=causal, upcast=False, reorder_ops=True)
    ok, err, bound = check_within_bound(out, ref, pt)
    assert ok, f"out {err:.3e} > {bound:.3e}"
    ok, err, pt_err = check_lse_within_bound(lse, attention_lse_ref(q, k, causal), attention_lse_pt(q, k, causal))
    assert ok, f"lse {err:.3e} (pt {pt_err:.3e})"
    # the same call without return_softmax takes the assembly forward: same Q', same LSE
    from flash_attn.flash_attn_interface import _flash_attn_forward
    out2, _, _, _, _, lse2, _, _ = _flash_attn_forward(q, k, v, 0.0, scale, causal, False)
    torch.testing.assert_close(lse, lse2, atol=1e-4, rtol=1e-5)
    tol = 2 ** -7 if dtype == torch.bfloat16 else 2 ** -10
    torch.testing.assert_close(out.float(), out2.float(), atol=tol, rtol=tol)
    # reference-shaped backward of that forward
    P = m._ptr
    sq_r = (s + 127) // 128 * 128
    dq, dk, dv = (torch.empty_like(x) for x in (q, k, v))
    softmax_d = torch.empty(b, h, sq_r, device=DEV)
    st = [_st(x) for x in (q, k, v, out, dq, dk, dv, dout)]
    (qr_, qh, qb), (kr_, kh, kb), (vr_, vh, vb), (orr, oh, ob) = st[:4]
    (dqr, dqh, dqb), (dkr, dkh, dkb), (dvr, dvh, dvb), (dor, doh, dob) = st[4:]
    ok = m._lib.flash_attn_bwd(P(dout), P(q), P(k), P(v), P(out), P(softmax_d), P(lse), None, P(dq), P(dk), P(dv),
                               None, b, s, s, sq_r, sq_r, h, h, d, d, 0.0, scale, 1.0, causal,
                               dtype == torch.bfloat16, 1, m._stream(q), 0, 0,
                               None, None, None, None, None, None, None, None,
                               qr_, kr_, vr_, qh, kh, vh, orr, oh, qb, kb, vb, ob,
                               dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, dqb, dkb, dvb, dob)
    assert ok, m._lib.flash_attn_error()
    torch.cuda.synchronize()
    gr = torch.autograd.grad(ref, (qr, kr, vr), dout)
    gp = torch.autograd.grad(pt, (qp, kp, vp), dout)
    for name, got, r, p_ in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        ok, err, bound = check_within_bound(got, r, p_, floor=1e-3)
        assert ok, f"{name} {err:.3e} > {bound:.3e}"


def test_bwd_device_rng_state_matches_explicit_seed():
    """flash_attn_bwd_gqa reads (seed, offset) from rng_state on the device; the reference-shaped
    flash_attn_bwd takes them by value: bitwise the same gradients (deterministic backward)."""
    import flash_attn_2_cuda as m

    torch.manual_seed(0)
    b, s, h, d, p, seed, offset = 2, 192, 2, 64, 0.3, 4242, 36
    q, k, v, dout = (torch.randn(b, s, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(4))
    out, lse, _ = _fwd_return_softmax(q, k, v, p, seed, offset, False)
    rng = torch.tensor([seed, offset], dtype=torch.int64, device=DEV)
    P = m._ptr
    sq_r = (s + 127) // 128 * 128
    res = []
    for fn, rng_arg, sd, off in ((m._lib.flash_attn_bwd_gqa, P(rng), 0, 0), (m._lib.flash_attn_bwd, None, seed, offset)):
        dq, dk, dv = (torch.empty_like(x) for x in (q, k, v))
        softmax_d = torch.empty(b, h, sq_r, device=DEV)
        st = [_st(x) for x in (q, k, v, out, dq, dk, dv, dout)]
        (qr, qh, qb), (kr, kh, kb), (vr, vh, vb), (orr, oh, ob) = st[:4]
        (dqr, dqh, dqb), (dkr, dkh, dkb), (dvr, dvh, dvb), (dor, doh, dob) = st[4:]
        ok = fn(P(dout), P(q), P(k), P(v), P(out), P(softmax_d), P(lse), rng_arg, P(dq), P(dk), P(dv), None,
                b, s, s, sq_r, sq_r, h, h, d, d, p, d ** -0.5, 1.0, False, True, 1, m._stream(q), sd, off,
                None, None, None, None, None, None, None, None,
                qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob,
                dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, dqb, dkb, dvb, dob)
        assert ok, m._lib.flash_attn_error()
        res.append((dq, dk, dv))
    torch.cuda.synchronize()
    for a, bb in zip(*res):
        assert torch.equal(a, bb)
    assert rng.tolist() == [seed, offset]             # an input here: not rewritten
