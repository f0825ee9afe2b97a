"""ORACLE -- test infrastructure only (never imported by the product path).

CPU restatement of the reference's numerical oracle for the FlashAttention-2 hot path, used by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` as the
CHECKER.  Nothing under ``xhy-flash-attention_amd/`` imports this module.

Contents
  * ``attention_ref``          -- restates ``attention_ref`` of the reference tests
                                  (tests/test_flash_attn.py:111-159): fp32 einsum attention
                                  (``upcast``), GQA by repeating kv heads (:135-136), key / query
                                  padding masks, top-left causal ``triu(ones, 1)`` (:144-146),
                                  ``reorder_ops`` (scale k instead of q) for the PyTorch-error bound.
  * ``attention_lse_ref``      -- logsumexp of the scaled, masked scores (the ``softmax_lse``
                                  output, flash_fwd_kernel.h:509-518: +inf for an empty row).
  * ``attention_lse_pt`` / ``check_lse_within_bound`` -- the LSE of the PyTorch-precision path and
                                  the 2x rule applied to ``softmax_lse``.
  * ``flash_fwd_np`` / ``flash_bwd_np`` -- float64 numpy restatement of the kernel algebra:
        O = softmax(s QK^T) V, LSE = max*s + ln(sum)                (flash_fwd_kernel.h:509-518)
        P = exp(s QK^T - LSE)                                        (flash_bwd_kernel.h:847)
        D = rowsum(dO o O)                                           (flash_bwd_kernel.h:181-182)
        dS = P o (dO V^T - D)                                        (flash_bwd_kernel.h:897-906)
        dV = P^T dO, dK = s dS^T Q, dQ = s dS K                      (flash_bwd_kernel.h:1046-1051)
    GQA gradients are summed over each query-head group (flash_api.cpp:682-686).
  * ``generate_random_padding_mask`` / ``generate_qkv`` -- the varlen fixture builders of the
    reference tests (tests/test_flash_attn.py:26-108), on top of this repo's bert_padding.
  * ``check_within_bound``     -- the acceptance rule max|x - ref| <= 2 * max|x_pt - ref|
                                  (tests/test_flash_attn.py:420-427, 630-639, 774-783).

Pinning: tests/test_oracle.py checks every function here against the golden vectors in
tests/golden/, which tests/golden/make_golden.py produced by running the reference's own
``attention_ref`` and ``bert_padding`` (imported from /root/reference) on seeded inputs.
"""
from __future__ import annotations

import math

import numpy as np
import torch

__all__ = [
    "attention_ref", "attention_lse_ref", "attention_lse_pt", "check_lse_within_bound", "flash_fwd_np", "flash_bwd_np",
    "generate_random_padding_mask", "generate_qkv", "check_within_bound", "max_abs_diff",
]


def _repeat_kv(x: torch.Tensor, groups: int) -> torch.Tensor:
    """(b, s, hk, d) -> (b, s, hk*groups, d), kv head j serving query heads j*groups .. +groups-1."""
    if groups == 1:
        return x
    b, s, hk, d = x.shape
    return x.unsqueeze(3).expand(b, s, hk, groups, d).reshape(b, s, hk * groups, d)


def attention_ref(q, k, v, query_padding_mask=None, key_padding_mask=None, dropout_p=0.0,
                  dropout_mask=None, causal=False, upcast=True, reorder_ops=False):
    """q (b, sq, h, d), k/v (b, sk, hk, d) -> (out (b, sq, h, d), attention (b, h, sq, sk)),
    both cast back to q's dtype (reference tests/test_flash_attn.py:111-159)."""
    dtype_og = q.dtype
    if upcast:
        q, k, v = q.float(), k.float(), v.float()
    seqlen_q, seqlen_k = q.shape[1], k.shape[1]
    groups = q.shape[2] // k.shape[2]
    k = _repeat_kv(k, groups)
    v = _repeat_kv(v, groups)
    d = q.shape[-1]
    if not reorder_ops:
        scores = torch.einsum("bthd,bshd->bhts", q / math.sqrt(d), k)
    else:
        scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask[:, None, None, :], float("-inf"))
    if causal:
        upper = torch.triu(torch.ones(seqlen_q, seqlen_k, dtype=torch.bool, device=q.device), 1)
        scores.masked_fill_(upper, float("-inf"))
    attention = torch.softmax(scores, dim=-1)
    dropout_scaling = 1.0 / (1 - dropout_p)
    attention_drop = attention.masked_fill(~dropout_mask, 0.0) if dropout_mask is not None else attention
    output = torch.einsum("bhts,bshd->bthd", attention_drop, v * dropout_scaling)
    if query_padding_mask is not None:
        output.masked_fill_(~query_padding_mask[:, :, None, None], 0.0)
        attention = attention.masked_fill(~query_padding_mask[:, None, :, None], 0.0)
    return output.to(dtype=dtype_og), attention.to(dtype=dtype_og)


def attention_lse_ref(q, k, causal=False, softmax_scale=None, key_padding_mask=None):
    """softmax_lse (b, h, sq) float32 of scale * QK^T with the kernel's masks; +inf if a row has no key."""
    q, k = q.double(), k.double()
    groups = q.shape[2] // k.shape[2]
    k = _repeat_kv(k, groups)
    scale = q.shape[-1] ** -0.5 if softmax_scale is None else softmax_scale
    scores = torch.einsum("bthd,bshd->bhts", q, k) * scale
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask[:, None, None, :], float("-inf"))
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        scores.masked_fill_(torch.triu(torch.ones(sq, sk, dtype=torch.bool, device=q.device), 1), float("-inf"))
    lse = torch.logsumexp(scores, dim=-1)
    lse = torch.where(torch.isneginf(lse), torch.full_like(lse, float("inf")), lse)
    return lse.float()


def attention_lse_pt(q, k, causal=False, key_padding_mask=None):
    """The softmax_lse implied by the reference's PyTorch-precision path (``attention_ref`` with
    upcast=False, reorder_ops=True: scores = einsum(q, k / sqrt(d)) in the input dtype,
    tests/test_flash_attn.py:137-141), its logsumexp taken in fp32: the LSE side of the 2x rule."""
    groups = q.shape[2] // k.shape[2]
    k = _repeat_kv(k, groups)
    scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(q.shape[-1])).float()
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask[:, None, None, :], float("-inf"))
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        scores.masked_fill_(torch.triu(torch.ones(sq, sk, dtype=torch.bool, device=q.device), 1), float("-inf"))
    lse = torch.logsumexp(scores, dim=-1)
    return torch.where(torch.isneginf(lse), torch.full_like(lse, float("inf")), lse)


def fold_lse_bound(q, k, causal=False, softmax_scale=None):
    """Per row (b, h, sq): the a-priori LSE error of scoring from Q' = round(scale log2 e Q) in Q's
    dtype (the assembly kernels' fold, DESIGN.md deviation 8) -- u max_j sum_d |scale q_d k_jd| over
    the row's visible keys, u the dtype's unit roundoff (bf16 2^-8, fp16 2^-11): the LSE is a smooth
    max of the scores, each off by at most that -- and the row's visible key count."""
    u = 2.0 ** -8 if q.dtype == torch.bfloat16 else 2.0 ** -11
    qd, kd = q.double(), _repeat_kv(k.double(), q.shape[2] // k.shape[2])
    scale = q.shape[-1] ** -0.5 if softmax_scale is None else softmax_scale
    s_abs = torch.einsum("bthd,bshd->bhts", qd.abs(), kd.abs()) * scale
    sq, sk = q.shape[1], k.shape[1]
    vis = torch.ones(sq, sk, dtype=torch.bool, device=q.device)
    if causal:
        vis = ~torch.triu(vis, 1)
    s_abs = s_abs.masked_fill(~vis, 0.0)
    return u * s_abs.amax(dim=-1), vis.sum(dim=-1).expand(q.shape[0], q.shape[2], sq)


def check_lse_within_bound(lse, ref, pt, atol=1e-3, rtol=1e-4, factor=2.0):
    """softmax_lse acceptance: rows without a key must read +inf; elsewhere
    |lse - ref| <= max(factor * max|pt - ref|, atol + rtol |ref|) -- the 2x rule of the outputs
    (check_within_bound), never stricter than the plain atol / rtol check it replaces.
    Returns (ok, max err, pt error)."""
    lse, ref, pt = (x.detach().double().cpu() for x in (lse, ref, pt))
    dead = torch.isinf(ref)
    if dead.any() and not (torch.isinf(lse[dead]) & (lse[dead] > 0)).all():
        return False, float("inf"), 0.0
    live = ~dead
    err = (lse[live] - ref[live]).abs()
    pt_err = float((pt[live] - ref[live]).abs().max()) if live.any() else 0.0
    bound = torch.clamp(atol + rtol * ref[live].abs(), min=factor * pt_err)
    ok = bool((err <= bound).all()) if live.any() else True
    return ok, float(err.max()) if live.any() else 0.0, pt_err


# ------------------------------------------------------------------------------------------------
# float64 numpy restatement of the kernel algebra (one sequence; arrays (s, h, d))
# ------------------------------------------------------------------------------------------------
def _mask_np(sq, sk, causal):
    if not causal:
        return np.zeros((sq, sk), dtype=bool)
    return np.triu(np.ones((sq, sk), dtype=bool), 1)   # key > query masked (top-left aligned)


def flash_fwd_np(q, k, v, scale=None, causal=False):
    """q (sq, h, d), k/v (sk, hk, d) -> out (sq, h, d) f64, lse (h, sq) f64 (+inf for empty rows)."""
    q, k, v = (np.asarray(x, dtype=np.float64) for x in (q, k, v))
    sq, h, d = q.shape
    sk, hk, _ = k.shape
    g = h // hk
    scale = d ** -0.5 if scale is None else scale
    masked = _mask_np(sq, sk, causal)
    out = np.zeros((sq, h, d))
    lse = np.full((h, sq), np.inf)
    for hi in range(h):
        s = q[:, hi, :] @ k[:, hi // g, :].T                       # raw scores
        s = np.where(masked, -np.inf, s)
        m = s.max(axis=1, initial=-np.inf)
        ok = np.isfinite(m)
        e = np.where(ok[:, None], np.exp((s - np.where(ok, m, 0)[:, None]) * scale), 0.0)
        l = e.sum(axis=1)
        good = l > 0
        out[good, hi, :] = (e[good] @ v[:, hi // g, :]) / l[good, None]
        lse[hi, good] = m[good] * scale + np.log(l[good])
    return out, lse


def flash_bwd_np(q, k, v, out, dout, lse, scale=None, causal=False):
    """Recompute backward: returns dq (sq,h,d), dk/dv (sk,hk,d) f64, GQA groups summed."""
    q, k, v, out, dout = (np.asarray(x, dtype=np.float64) for x in (q, k, v, out, dout))
    lse = np.asarray(lse, dtype=np.float64)
    sq, h, d = q.shape
    sk, hk, _ = k.shape
    g = h // hk
    scale = d ** -0.5 if scale is None else scale
    masked = _mask_np(sq, sk, causal)
    dq = np.zeros_like(q)
    dk = np.zeros_like(k)
    dv = np.zeros_like(v)
    for hi in range(h):
        kh, vh = k[:, hi // g, :], v[:, hi // g, :]
        s = q[:, hi, :] @ kh.T
        lrow = lse[hi][:, None]
        p = np.where(masked | ~np.isfinite(lrow), 0.0, np.exp(s * scale - np.where(np.isfinite(lrow), lrow, 0)))
        dsum = (dout[:, hi, :] * out[:, hi, :]).sum(axis=1, keepdims=True)
        dp = dout[:, hi, :] @ vh.T
        ds = p * (dp - dsum)
        dv[:, hi // g, :] += p.T @ dout[:, hi, :]
        dk[:, hi // g, :] += scale * (ds.T @ q[:, hi, :])
        dq[:, hi, :] = scale * (ds @ kh)
    return dq, dk, dv


# ------------------------------------------------------------------------------------------------
# varlen fixture builders (reference tests/test_flash_attn.py:26-108)
# ------------------------------------------------------------------------------------------------
def generate_random_padding_mask(max_seqlen, batch_size, device="cpu", mode="random"):
    assert mode in ("full", "random", "third")
    if mode == "full":
        lengths = torch.full((batch_size, 1), max_seqlen, device=device, dtype=torch.int32)
    elif mode == "random":
        lengths = torch.randint(max(1, max_seqlen - 20), max_seqlen, (batch_size, 1), device=device)
    else:
        lengths = torch.randint(max_seqlen // 3, max_seqlen, (batch_size, 1), device=device)
    return torch.arange(max_seqlen, device=device)[None, :].expand(batch_size, max_seqlen) < lengths


def generate_qkv(q, k, v, query_padding_mask=None, key_padding_mask=None, kvpacked=False,
                 qkvpacked=False):
    """Same return tuples as the reference helper; uses this repo's bert_padding."""
    from flash_attn.bert_padding import pad_input, unpad_input

    assert not (kvpacked and qkvpacked)
    b, sq, h, d = q.shape
    _, sk, hk, _ = k.shape
    if query_padding_mask is not None:
        q_unpad, indices_q, cu_seqlens_q, max_seqlen_q = unpad_input(q, query_padding_mask)
        output_pad_fn = lambda o: pad_input(o, indices_q, b, sq)  # noqa: E731
    else:
        q_unpad = q.reshape(b * sq, h, d)
        cu_seqlens_q = torch.arange(0, (b + 1) * sq, step=sq, dtype=torch.int32, device=q.device)
        max_seqlen_q = sq
        output_pad_fn = lambda o: o.reshape(b, sq, *o.shape[1:])  # noqa: E731
    if key_padding_mask is not None:
        k_unpad, indices_k, cu_seqlens_k, max_seqlen_k = unpad_input(k, key_padding_mask)
        v_unpad, _, _, _ = unpad_input(v, key_padding_mask)
    else:
        k_unpad = k.reshape(b * sk, hk, d)
        v_unpad = v.reshape(b * sk, hk, d)
        cu_seqlens_k = torch.arange(0, (b + 1) * sk, step=sk, dtype=torch.int32, device=k.device)
        max_seqlen_k = sk
        indices_k = None

    if qkvpacked:
        assert nheads_equal(h, hk)
        qkv_unpad = torch.stack([q_unpad, k_unpad, v_unpad], dim=1)
        qkv = torch.stack([q, k, v], dim=2)
        if query_padding_mask is not None:
            dqkv_pad_fn = lambda x: pad_input(x, indices_q, b, sq)  # noqa: E731
        else:
            dqkv_pad_fn = lambda x: x.reshape(b, sq, *x.shape[1:])  # noqa: E731
        return (qkv_unpad.detach().requires_grad_(), cu_seqlens_q, max_seqlen_q,
                qkv.detach().requires_grad_(), output_pad_fn, dqkv_pad_fn)
    if kvpacked:
        kv_unpad = torch.stack([k_unpad, v_unpad], dim=1)
        kv = torch.stack([k, v], dim=2)
        if key_padding_mask is not None:
            dkv_pad_fn = lambda x: pad_input(x, indices_k, b, sk)  # noqa: E731
        else:
            dkv_pad_fn = lambda x: x.reshape(b, sk, *x.shape[1:])  # noqa: E731
        return (q_unpad.detach().requires_grad_(), kv_unpad.detach().requires_grad_(),
                cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                q.detach().requires_grad_(), kv.detach().requires_grad_(),
                output_pad_fn, output_pad_fn, dkv_pad_fn)
    if key_padding_mask is not None:
        dk_pad_fn = lambda x: pad_input(x, indices_k, b, sk)  # noqa: E731
    else:
        dk_pad_fn = lambda x: x.reshape(b, sk, *x.shape[1:])  # noqa: E731
    return (q_unpad.detach().requires_grad_(), k_unpad.detach().requires_grad_(),
            v_unpad.detach().requires_grad_(), cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
            max_seqlen_k, q.detach().requires_grad_(), k.detach().requires_grad_(),
            v.detach().requires_grad_(), output_pad_fn, output_pad_fn, dk_pad_fn)


def nheads_equal(h, hk):
    return h == hk


# ------------------------------------------------------------------------------------------------
# acceptance rule
# ------------------------------------------------------------------------------------------------
def max_abs_diff(a, b) -> float:
    return (a.float() - b.float()).abs().max().item() if a.numel() else 0.0


def check_within_bound(x, ref, pt, factor=2.0, floor=0.0):
    """max|x - ref| <= factor * max|pt - ref| + floor.  Returns (ok, err, bound)."""
    err = max_abs_diff(x, ref)
    bound = factor * max_abs_diff(pt, ref) + floor
    return err <= bound, err, bound
