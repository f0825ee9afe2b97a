"""Public FlashAttention-2 API and its autograd wiring (MI355X build).

Drop-in for the reference's ``flash_attn/flash_attn_interface.py``: the six public functions
(reference ``:282-492``) and six ``torch.autograd.Function`` classes (``:88-279``) keep their
names, positional order, defaults, return tuples, saved tensors and backward gradient tuples.
Underneath, ``flash_attn_2_cuda`` is this build's ctypes binding of ``libflash_attn_mi355x.so``.

Behavioural notes shared with the reference:
  * ``softmax_scale=None`` means ``headdim ** -0.5``;
  * ``return_attn_probs`` returns ``(out, softmax_lse, S_dmask)`` and ``S_dmask`` is only produced
    when ``dropout_p > 0`` (``_flash_attn_forward`` passes ``return_softmax and dropout_p > 0``);
  * the head dim is padded to a multiple of 8 inside the extension and gradients are sliced back;
  * MQA / GQA: ``nheads % nheads_k == 0``; query head ``i`` reads kv head ``i // (nheads/nheads_k)``.
"""
import torch

import flash_attn_2_cuda as flash_attn_cuda

__all__ = [
    "flash_attn_func", "flash_attn_kvpacked_func", "flash_attn_qkvpacked_func",
    "flash_attn_varlen_func", "flash_attn_varlen_kvpacked_func",
    "flash_attn_varlen_qkvpacked_func", "_get_block_size",
]


def _get_block_size(device, head_dim, is_dropout, is_causal):
    """(block_m, block_n) of this build's forward tiles (reference ``:8-36`` reports the CUDA ones)."""
    assert head_dim <= 256
    return flash_attn_cuda.block_size(head_dim, False)


def _last_dim_contiguous(*xs):
    return [x if x.stride(-1) == 1 else x.contiguous() for x in xs]


def _flash_attn_forward(q, k, v, dropout_p, softmax_scale, causal, return_softmax):
    q, k, v = _last_dim_contiguous(q, k, v)
    return tuple(flash_attn_cuda.fwd(q, k, v, None, dropout_p, softmax_scale, causal,
                                     return_softmax, None))


def _flash_attn_varlen_forward(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                               dropout_p, softmax_scale, causal, return_softmax):
    q, k, v = _last_dim_contiguous(q, k, v)
    return tuple(flash_attn_cuda.varlen_fwd(q, k, v, None, cu_seqlens_q, cu_seqlens_k,
                                            max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale,
                                            False, causal, return_softmax, None))


def _flash_attn_backward(dout, q, k, v, out, softmax_lse, dq, dk, dv, dropout_p, softmax_scale,
                         causal, rng_state=None):
    dout, q, k, v, out = _last_dim_contiguous(dout, q, k, v, out)
    dq, dk, dv, softmax_d = flash_attn_cuda.bwd(dout, q, k, v, out, softmax_lse, dq, dk, dv,
                                                dropout_p, softmax_scale, causal, None, rng_state)
    return dq, dk, dv, softmax_d


def _flash_attn_varlen_backward(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q,
                                cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale,
                                causal, rng_state=None):
    dout, q, k, v, out = _last_dim_contiguous(dout, q, k, v, out)
    dq, dk, dv, softmax_d = flash_attn_cuda.varlen_bwd(
        dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
        max_seqlen_k, dropout_p, softmax_scale, False, causal, None, rng_state)
    return dq, dk, dv, softmax_d


def _default_scale(softmax_scale, x):
    return x.shape[-1] ** (-0.5) if softmax_scale is None else softmax_scale


def _result(out, softmax_lse, S_dmask, return_softmax):
    return (out, softmax_lse, S_dmask) if return_softmax else out


def _stash(ctx, dropout_p, softmax_scale, causal, **extra):
    ctx.dropout_p = dropout_p
    ctx.softmax_scale = softmax_scale
    ctx.causal = causal
    for key, val in extra.items():
        setattr(ctx, key, val)


class FlashAttnQKVPackedFunc(torch.autograd.Function):
    """qkv: (batch, seqlen, 3, nheads, headdim)   (reference :88-114)."""

    @staticmethod
    def forward(ctx, qkv, dropout_p, softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, qkv)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_forward(
            qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], dropout_p, softmax_scale, causal=causal,
            return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, rng_state = ctx.saved_tensors
        dqkv = torch.empty(q.shape[:-2] + (3,) + q.shape[-2:], dtype=q.dtype, device=q.device)
        _flash_attn_backward(dout, q, k, v, out, softmax_lse, dqkv[:, :, 0], dqkv[:, :, 1],
                             dqkv[:, :, 2], ctx.dropout_p, ctx.softmax_scale, ctx.causal,
                             rng_state=rng_state)
        return dqkv[..., :dout.shape[-1]], None, None, None, None


class FlashAttnVarlenQKVPackedFunc(torch.autograd.Function):
    """qkv: (total, 3, nheads, headdim) with cu_seqlens (batch+1,) int32   (reference :117-145)."""

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, max_seqlen, dropout_p, softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, qkv)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_varlen_forward(
            qkv[:, 0], qkv[:, 1], qkv[:, 2], cu_seqlens, cu_seqlens, max_seqlen, max_seqlen,
            dropout_p, softmax_scale, causal=causal,
            return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, cu_seqlens, rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal, max_seqlen=max_seqlen)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, cu_seqlens, rng_state = ctx.saved_tensors
        dqkv = torch.empty(q.shape[:-2] + (3,) + q.shape[-2:], dtype=q.dtype, device=q.device)
        _flash_attn_varlen_backward(dout, q, k, v, out, softmax_lse, dqkv[:, 0], dqkv[:, 1],
                                    dqkv[:, 2], cu_seqlens, cu_seqlens, ctx.max_seqlen,
                                    ctx.max_seqlen, ctx.dropout_p, ctx.softmax_scale, ctx.causal,
                                    rng_state=rng_state)
        return dqkv[..., :dout.shape[-1]], None, None, None, None, None, None


class FlashAttnKVPackedFunc(torch.autograd.Function):
    """q: (batch, seqlen_q, nheads, d), kv: (batch, seqlen_k, 2, nheads_k, d)   (reference :148-177)."""

    @staticmethod
    def forward(ctx, q, kv, dropout_p, softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, q)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_forward(
            q, kv[:, :, 0], kv[:, :, 1], dropout_p, softmax_scale, causal=causal,
            return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, rng_state = ctx.saved_tensors
        dq = torch.empty_like(q)
        dkv = torch.empty(k.shape[:-2] + (2,) + k.shape[-2:], dtype=k.dtype, device=k.device)
        _flash_attn_backward(dout, q, k, v, out, softmax_lse, dq, dkv[:, :, 0], dkv[:, :, 1],
                             ctx.dropout_p, ctx.softmax_scale, ctx.causal, rng_state=rng_state)
        d = dout.shape[-1]
        return dq[..., :d], dkv[..., :d], None, None, None, None


class FlashAttnVarlenKVPackedFunc(torch.autograd.Function):
    """q: (total_q, nheads, d), kv: (total_k, 2, nheads_k, d)   (reference :180-213)."""

    @staticmethod
    def forward(ctx, q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, q)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_varlen_forward(
            q, kv[:, 0], kv[:, 1], cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
            dropout_p, softmax_scale, causal=causal,
            return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, cu_seqlens_q, cu_seqlens_k,
                              rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal, max_seqlen_q=max_seqlen_q,
               max_seqlen_k=max_seqlen_k)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, cu_seqlens_q, cu_seqlens_k, rng_state = ctx.saved_tensors
        dq = torch.empty_like(q)
        dkv = torch.empty(k.shape[:-2] + (2,) + k.shape[-2:], dtype=k.dtype, device=k.device)
        _flash_attn_varlen_backward(dout, q, k, v, out, softmax_lse, dq, dkv[:, 0], dkv[:, 1],
                                    cu_seqlens_q, cu_seqlens_k, ctx.max_seqlen_q,
                                    ctx.max_seqlen_k, ctx.dropout_p, ctx.softmax_scale,
                                    ctx.causal, rng_state=rng_state)
        d = dout.shape[-1]
        return dq[..., :d], dkv[..., :d], None, None, None, None, None, None, None, None


class FlashAttnFunc(torch.autograd.Function):
    """q: (batch, seqlen_q, nheads, d), k/v: (batch, seqlen_k, nheads_k, d)   (reference :216-244)."""

    @staticmethod
    def forward(ctx, q, k, v, dropout_p, softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, q)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_forward(
            q, k, v, dropout_p, softmax_scale, causal=causal,
            return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, rng_state = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _flash_attn_backward(dout, q, k, v, out, softmax_lse, dq, dk, dv, ctx.dropout_p,
                             ctx.softmax_scale, ctx.causal, rng_state=rng_state)
        # slice the padded head dim back to the caller's (dout's) head dim; the reference slices by
        # the saved *padded* q here (:240-243), which breaks head dims that are not multiples of 8
        d = dout.shape[-1]
        return dq[..., :d], dk[..., :d], dv[..., :d], None, None, None, None, None, None, None, None


class FlashAttnVarlenFunc(torch.autograd.Function):
    """q: (total_q, nheads, d), k/v: (total_k, nheads_k, d)   (reference :247-279)."""

    @staticmethod
    def forward(ctx, q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                softmax_scale, causal, return_softmax):
        softmax_scale = _default_scale(softmax_scale, q)
        out, q, k, v, out_padded, softmax_lse, S_dmask, rng_state = _flash_attn_varlen_forward(
            q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
            softmax_scale, causal=causal, return_softmax=return_softmax and dropout_p > 0)
        ctx.save_for_backward(q, k, v, out_padded, softmax_lse, cu_seqlens_q, cu_seqlens_k,
                              rng_state)
        _stash(ctx, dropout_p, softmax_scale, causal, max_seqlen_q=max_seqlen_q,
               max_seqlen_k=max_seqlen_k)
        return _result(out, softmax_lse, S_dmask, return_softmax)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, cu_seqlens_q, cu_seqlens_k, rng_state = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _flash_attn_varlen_backward(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q,
                                    cu_seqlens_k, ctx.max_seqlen_q, ctx.max_seqlen_k,
                                    ctx.dropout_p, ctx.softmax_scale, ctx.causal,
                                    rng_state=rng_state)
        # slice the padded head dim back to the caller's (dout's) head dim; the reference slices by
        # the saved *padded* q here (:240-243), which breaks head dims that are not multiples of 8
        d = dout.shape[-1]
        return dq[..., :d], dk[..., :d], dv[..., :d], None, None, None, None, None, None, None, None


# ------------------------------------------------------------------------------------------------
# public functions (reference :282-492)
# ------------------------------------------------------------------------------------------------
def flash_attn_qkvpacked_func(qkv, dropout_p=0.0, softmax_scale=None, causal=False,
                              return_attn_probs=False):
    """qkv: (batch_size, seqlen, 3, nheads, headdim) -> out (batch_size, seqlen, nheads, headdim).

    With ``return_attn_probs``: ``(out, softmax_lse (batch, nheads, seqlen), S_dmask)``.
    ``dropout_p`` must be 0.0 during evaluation."""
    return FlashAttnQKVPackedFunc.apply(qkv, dropout_p, softmax_scale, causal, return_attn_probs)


def flash_attn_kvpacked_func(q, kv, dropout_p=0.0, softmax_scale=None, causal=False,
                             return_attn_probs=False):
    """q: (batch, seqlen_q, nheads, d), kv: (batch, seqlen_k, 2, nheads_k, d); MQA/GQA when
    nheads_k < nheads (nheads % nheads_k == 0)."""
    return FlashAttnKVPackedFunc.apply(q, kv, dropout_p, softmax_scale, causal, return_attn_probs)


def flash_attn_func(q, k, v, dropout_p=0.0, softmax_scale=None, causal=False,
                    return_attn_probs=False):
    """q: (batch, seqlen_q, nheads, d), k/v: (batch, seqlen_k, nheads_k, d) -> out like q.

    Causal masking is top-left aligned (query i attends keys j <= i).  MQA/GQA when
    nheads_k < nheads: query head h uses kv head h // (nheads // nheads_k)."""
    return FlashAttnFunc.apply(q, k, v, dropout_p, softmax_scale, causal, return_attn_probs)


def flash_attn_varlen_qkvpacked_func(qkv, cu_seqlens, max_seqlen, dropout_p=0.0,
                                     softmax_scale=None, causal=False, return_attn_probs=False):
    """qkv: (total, 3, nheads, d), cu_seqlens: (batch+1,) int32 -> out (total, nheads, d).
    softmax_lse is (batch, nheads, max_seqlen)."""
    return FlashAttnVarlenQKVPackedFunc.apply(qkv, cu_seqlens, max_seqlen, dropout_p,
                                              softmax_scale, causal, return_attn_probs)


def flash_attn_varlen_kvpacked_func(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                                    dropout_p=0.0, softmax_scale=None, causal=False,
                                    return_attn_probs=False):
    """q: (total_q, nheads, d), kv: (total_k, 2, nheads_k, d) with per-side cu_seqlens."""
    return FlashAttnVarlenKVPackedFunc.apply(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                                             max_seqlen_k, dropout_p, softmax_scale, causal,
                                             return_attn_probs)


def flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                           dropout_p=0.0, softmax_scale=None, causal=False,
                           return_attn_probs=False):
    """q: (total_q, nheads, d), k/v: (total_k, nheads_k, d) with per-side cu_seqlens."""
    return FlashAttnVarlenFunc.apply(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                                     max_seqlen_k, dropout_p, softmax_scale, causal,
                                     return_attn_probs)
