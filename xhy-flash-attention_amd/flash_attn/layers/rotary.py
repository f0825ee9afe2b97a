"""Rotary position embedding (reference flash_attn/layers/rotary.py:1-337), MI355X build.

Same public names, signatures and in-place semantics as the reference: ``apply_rotary_emb_func``
(out of place or in place), ``apply_rotary_emb_qkv_`` and ``apply_rotary_emb_kv_`` (in place on
packed tensors, GPT-NeoX halves or GPT-J interleaved pairs, optional separate cos/sin for k as
XPos uses), and the ``RotaryEmbedding`` module with its cos/sin cache.  The reference's extension
op ``rotary_emb.apply_rotary`` is replaced by the HIP kernel behind ``flash_attn_rotary_apply``
(csrc/fa_rotary.hip) -- there is no eager-PyTorch path; ``apply_rotary_emb_torch`` is the
reference's plain-torch formula, kept for tests as the reference keeps it.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch
from einops import rearrange, repeat

import flash_attn_2_cuda as _ext

_lib = _ext._lib
_P, _I, _I64, _B = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_bool
_lib.flash_attn_rotary_apply.argtypes = [_P] * 4 + [_I] * 4 + [_I64] * 7 + [_B] * 3 + [_P]
_lib.flash_attn_rotary_apply.restype = ctypes.c_bool


def _apply_rotary(x: torch.Tensor, out: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                  interleaved: bool, conj: bool):
    """out[..., :rd] = rotary(x[..., :rd]) on (b, s, h, d) views (out may be x); cos/sin (s, rd/2)."""
    _ext._check(x.is_cuda and out.is_cuda and cos.is_cuda and sin.is_cuda,
                "rotary: tensors must be on the GPU")
    _ext._check(x.dtype in (torch.float16, torch.bfloat16), "rotary: only fp16 and bf16 are supported")
    _ext._check(x.dtype == out.dtype == cos.dtype == sin.dtype, "rotary: x, out, cos, sin must share a dtype")
    b, s, h, d = x.shape
    _ext._check(out.shape == x.shape, "rotary: out must have the shape of x")
    rd = cos.shape[-1] * 2
    _ext._check(rd <= d and cos.shape == sin.shape and cos.shape[0] >= s, "rotary: bad cos/sin shape")
    _ext._check(x.stride(-1) == 1 and out.stride(-1) == 1, "rotary: last dim must be contiguous")
    if cos.stride(-1) != 1 or sin.stride(-1) != 1 or cos.stride(0) != sin.stride(0):
        cos, sin = cos.contiguous(), sin.contiguous()
    ok = _lib.flash_attn_rotary_apply(
        _ext._ptr(x), _ext._ptr(out), _ext._ptr(cos), _ext._ptr(sin), b, s, h, rd,
        x.stride(0), x.stride(1), x.stride(2), out.stride(0), out.stride(1), out.stride(2),
        cos.stride(0), bool(interleaved), bool(conj), x.dtype == torch.bfloat16, _ext._stream(x))
    if not ok:
        _ext._raise_lib_error("flash_attn_rotary_apply")


def rotate_half(x, interleaved=False):
    if not interleaved:
        x1, x2 = x.chunk(2, dim=-1)
        return torch.cat((-x2, x1), dim=-1)
    x1, x2 = x[..., ::2], x[..., 1::2]
    return rearrange(torch.stack((-x2, x1), dim=-1), "... d two -> ... (d two)", two=2)


def apply_rotary_emb_torch(x, cos, sin, interleaved=False):
    """x: (batch, seqlen, nheads, headdim); cos, sin: (seqlen, rotary_dim / 2) (reference :22-32).

    With interleaved=True the reference repeats cos/sin as (2 d), which does not match its own
    CUDA op (pair i of columns 2i, 2i+1 uses cos[i]); here they are repeated as (d 2), so this
    formula agrees with the kernel in both layouts."""
    ro_dim = cos.shape[-1] * 2
    assert ro_dim <= x.shape[-1]
    pattern = "s d -> s 1 (d 2)" if interleaved else "s d -> s 1 (2 d)"
    cos = repeat(cos, pattern)
    sin = repeat(sin, pattern)
    return torch.cat([x[..., :ro_dim] * cos + rotate_half(x[..., :ro_dim], interleaved) * sin,
                      x[..., ro_dim:]], dim=-1)


class ApplyRotaryEmb(torch.autograd.Function):
    """reference rotary.py:35-92"""

    @staticmethod
    def forward(ctx, x, cos, sin, interleaved=False, inplace=False):
        _, seqlen, _, headdim = x.shape
        rotary_dim = cos.shape[1] * 2
        assert rotary_dim <= headdim and seqlen <= cos.shape[0]
        assert sin.shape == cos.shape
        out = x if inplace else torch.empty_like(x)
        _apply_rotary(x, out, cos[:seqlen], sin[:seqlen], interleaved, False)
        if not inplace and rotary_dim < headdim:
            out[..., rotary_dim:].copy_(x[..., rotary_dim:])
        ctx.save_for_backward(cos, sin)
        ctx.interleaved = interleaved
        ctx.inplace = inplace
        return out

    @staticmethod
    def backward(ctx, do):
        cos, sin = ctx.saved_tensors
        seqlen, headdim = do.shape[1], do.shape[-1]
        rotary_dim = cos.shape[-1] * 2
        if ctx.inplace:
            do = do if do.stride(-1) == 1 else do.contiguous()
            dx = do
        else:
            do = do if do.stride(-1) == 1 else do.contiguous()
            dx = torch.empty_like(do)
        _apply_rotary(do, dx, cos[:seqlen], sin[:seqlen], ctx.interleaved, True)
        if not ctx.inplace and rotary_dim < headdim:
            dx[..., rotary_dim:].copy_(do[..., rotary_dim:])
        return dx, None, None, None, None


apply_rotary_emb_func = ApplyRotaryEmb.apply


class ApplyRotaryEmbQKV_(torch.autograd.Function):
    """reference rotary.py:98-148: in place on q (index 0) and k (index 1) of (b, s, 3, h, d)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, cos_k=None, sin_k=None, interleaved=False):
        _, seqlen, three, _, headdim = qkv.shape
        assert three == 3
        rotary_dim = cos.shape[1] * 2
        assert rotary_dim <= headdim and seqlen <= cos.shape[0]
        cos_k = cos if cos_k is None else cos_k
        sin_k = sin if sin_k is None else sin_k
        assert sin.shape == cos_k.shape == sin_k.shape == cos.shape
        q, k = qkv[:, :, 0], qkv[:, :, 1]
        _apply_rotary(q, q, cos[:seqlen], sin[:seqlen], interleaved, False)
        _apply_rotary(k, k, cos_k[:seqlen], sin_k[:seqlen], interleaved, False)
        ctx.save_for_backward(cos, sin, cos_k, sin_k)
        ctx.interleaved = interleaved
        return qkv

    @staticmethod
    def backward(ctx, dqkv):
        cos, sin, cos_k, sin_k = ctx.saved_tensors
        seqlen = dqkv.shape[1]
        dqkv = dqkv if dqkv.stride(-1) == 1 else dqkv.contiguous()
        dq, dk = dqkv[:, :, 0], dqkv[:, :, 1]
        _apply_rotary(dq, dq, cos[:seqlen], sin[:seqlen], ctx.interleaved, True)
        _apply_rotary(dk, dk, cos_k[:seqlen], sin_k[:seqlen], ctx.interleaved, True)
        return dqkv, None, None, None, None, None


apply_rotary_emb_qkv_ = ApplyRotaryEmbQKV_.apply


class ApplyRotaryEmbKV_(torch.autograd.Function):
    """reference rotary.py:154-193: in place on k (index 0) of (b, s, 2, h, d)."""

    @staticmethod
    def forward(ctx, kv, cos, sin, interleaved=False):
        _, seqlen, two, _, headdim = kv.shape
        assert two == 2
        rotary_dim = cos.shape[1] * 2
        assert rotary_dim <= headdim and seqlen <= cos.shape[0]
        k = kv[:, :, 0]
        _apply_rotary(k, k, cos[:seqlen], sin[:seqlen], interleaved, False)
        ctx.save_for_backward(cos, sin)
        ctx.interleaved = interleaved
        return kv

    @staticmethod
    def backward(ctx, dkv):
        cos, sin = ctx.saved_tensors
        seqlen = dkv.shape[1]
        dkv = dkv if dkv.stride(-1) == 1 else dkv.contiguous()
        dk = dkv[:, :, 0]
        _apply_rotary(dk, dk, cos[:seqlen], sin[:seqlen], ctx.interleaved, True)
        return dkv, None, None, None


apply_rotary_emb_kv_ = ApplyRotaryEmbKV_.apply


class RotaryEmbedding(torch.nn.Module):
    """RoFormer rotary embedding with the optional XPos scaling (reference rotary.py:199-337):
    same constructor, cos/sin cache policy and forward(qkv, kv=None, seqlen_offset=0)."""

    def __init__(self, dim: int, base=10000.0, interleaved=False, scale_base=None,
                 pos_idx_in_fp32=True, device=None):
        super().__init__()
        self.dim = dim
        self.base = float(base)
        self.pos_idx_in_fp32 = pos_idx_in_fp32
        self.register_buffer("inv_freq", self._compute_inv_freq(device), persistent=False)
        self.interleaved = interleaved
        self.scale_base = scale_base
        scale = ((torch.arange(0, dim, 2, device=device, dtype=torch.float32) + 0.4 * dim) / (1.4 * dim)
                 if scale_base is not None else None)
        self.register_buffer("scale", scale, persistent=False)
        self._seq_len_cached = 0
        self._cos_cached = None
        self._sin_cached = None
        self._cos_k_cached = None
        self._sin_k_cached = None

    def _compute_inv_freq(self, device=None):
        return 1.0 / (self.base ** (torch.arange(0, self.dim, 2, device=device, dtype=torch.float32)
                                    / self.dim))

    def _update_cos_sin_cache(self, seqlen, device=None, dtype=None):
        if (seqlen > self._seq_len_cached or self._cos_cached.device != device
                or self._cos_cached.dtype != dtype
                or (self.training and self._cos_cached.is_inference())):
            self._seq_len_cached = seqlen
            if self.pos_idx_in_fp32:
                t = torch.arange(seqlen, device=device, dtype=torch.float32)
                inv_freq = (self._compute_inv_freq(device=device) if self.inv_freq.dtype != torch.float32
                            else self.inv_freq)
            else:
                t = torch.arange(seqlen, device=device, dtype=self.inv_freq.dtype)
                inv_freq = self.inv_freq
            freqs = torch.outer(t, inv_freq)
            if self.scale is None:
                self._cos_cached = torch.cos(freqs).to(dtype)
                self._sin_cached = torch.sin(freqs).to(dtype)
            else:
                power = ((torch.arange(seqlen, dtype=self.scale.dtype, device=self.scale.device)
                          - seqlen // 2) / self.scale_base)
                scale = self.scale.to(device=power.device) ** rearrange(power, "s -> s 1")
                self._cos_cached = (torch.cos(freqs) * scale).to(dtype)
                self._sin_cached = (torch.sin(freqs) * scale).to(dtype)
                self._cos_k_cached = (torch.cos(freqs) / scale).to(dtype)
                self._sin_k_cached = (torch.sin(freqs) / scale).to(dtype)

    def forward(self, qkv: torch.Tensor, kv: Optional[torch.Tensor] = None,
                seqlen_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        seqlen = qkv.shape[1]
        self._update_cos_sin_cache(seqlen + seqlen_offset, device=qkv.device, dtype=qkv.dtype)
        cos, sin = self._cos_cached[seqlen_offset:], self._sin_cached[seqlen_offset:]
        if kv is None:
            if self.scale is None:
                return apply_rotary_emb_qkv_(qkv, cos, sin, None, None, self.interleaved)
            return apply_rotary_emb_qkv_(qkv, cos, sin, self._cos_k_cached[seqlen_offset:],
                                         self._sin_k_cached[seqlen_offset:], self.interleaved)
        q = apply_rotary_emb_func(qkv, cos, sin, self.interleaved, True)
        if self.scale is None:
            kv = apply_rotary_emb_kv_(kv, cos, sin, self.interleaved)
        else:
            kv = apply_rotary_emb_kv_(kv, self._cos_k_cached[seqlen_offset:],
                                      self._sin_k_cached[seqlen_offset:], self.interleaved)
        return q, kv
