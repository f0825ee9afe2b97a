"""MI355X replacement for the reference's ``flash_attn_2_cuda`` extension module.

The reference builds ``flash_attn_2_cuda`` from ``csrc/flash_attn/flash_api.cpp`` (module name
``setup.py:162``; ops ``flash_api.cpp:914-920``).  This module exports the same four ops with the
same argument lists, return lists, allocation/ownership rules and error behaviour (RuntimeError
on a failed check), but every kernel launch goes through the C ABI of
``libflash_attn_mi355x.so`` (declared in ``include/flash_attn.h``): the torch tensors are only
used for device memory, strides and the current HIP stream.

There is no CPU or eager-PyTorch fallback: CPU tensors are rejected exactly as the reference
rejects them, and a missing library raises ImportError at import time.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

__all__ = ["fwd", "varlen_fwd", "bwd", "varlen_bwd", "block_size", "LIBRARY_PATH"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBRARY_PATH = os.environ.get("FLASH_ATTN_MI355X_LIB", os.path.join(_HERE, "libflash_attn_mi355x.so"))

if not os.path.exists(LIBRARY_PATH):
    raise ImportError(
        f"flash_attn_2_cuda: {LIBRARY_PATH} is missing; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C xhy-flash-attention_amd/csrc`)")

_lib = ctypes.CDLL(LIBRARY_PATH)

_P, _I, _F, _B, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool, ctypes.c_uint64

# argument kinds, in declaration order (include/flash_attn.h)
_FWD = ([_P] * 7 + [_I] * 9 + [_F] * 3 + [_B] * 3 + [_P, _U64, _U64] + [_P] * 8 + [_I] * 12)
_VARLEN_FWD = ([_P] * 9 + [_I] * 9 + [_F] * 3 + [_B] * 3 + [_P, _U64, _U64, _P, _P]
               + [_I] * 12 + [_B])
_BWD = ([_P] * 12 + [_I] * 9 + [_F] * 3 + [_B] * 2 + [_I, _P, _U64, _U64] + [_P] * 8 + [_I] * 24)
_VARLEN_BWD = ([_P] * 14 + [_I] * 9 + [_F] * 3 + [_B] * 2 + [_I, _P, _U64, _U64, _P, _P]
               + [_I] * 24 + [_B])

for _name, _sig in (("flash_attn_fwd", _FWD), ("flash_attn_varlen_fwd", _VARLEN_FWD),
                    ("flash_attn_bwd", _BWD), ("flash_attn_bwd_gqa", _BWD),
                    ("flash_attn_varlen_bwd", _VARLEN_BWD),
                    ("flash_attn_varlen_bwd_gqa", _VARLEN_BWD)):
    _fn = getattr(_lib, _name)
    _fn.argtypes = _sig
    _fn.restype = ctypes.c_bool
_lib.flash_attn_error.argtypes = []
_lib.flash_attn_error.restype = ctypes.c_char_p
_lib.flash_attn_block_size.argtypes = [_I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)]
_lib.flash_attn_block_size.restype = None

_INT_MAX = 2 ** 31 - 1


def block_size(head_dim: int, is_backward: bool = False):
    """(block_m, block_n) tiles of this build's launchers (feeds ``_get_block_size``)."""
    m, n = _I(), _I()
    _lib.flash_attn_block_size(int(head_dim), int(bool(is_backward)), ctypes.byref(m), ctypes.byref(n))
    return m.value, n.value


def _check(cond: bool, msg: str):
    if not cond:
        raise RuntimeError(msg)


def _raise_lib_error(op: str):
    err = _lib.flash_attn_error()
    raise RuntimeError(f"{op}: " + (err.decode() if err else "unknown error"))


def _round_multiple(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _device_guard(dev: torch.device):
    """the launch runs with `dev` current (the C ABI launches on the current device, as the
    reference's CUDAGuard arranges); no guard when it already is (host overhead per call)"""
    if dev.index is None or dev.index == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(dev)


_GFX950 = {}   # device index -> is gfx950 (device properties are fixed for the process)


def _is_gfx950(dev: torch.device) -> bool:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    ok = _GFX950.get(idx)
    if ok is None:
        ok = getattr(torch.cuda.get_device_properties(idx), "gcnArchName", "").startswith("gfx950")
        _GFX950[idx] = ok
    return ok


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _strides(t: torch.Tensor, nd_row: int):
    """(batch, row, head) element strides; batch stride 0 for 3-D (varlen) tensors."""
    st = t.stride()
    batch = st[0] if t.dim() == 4 else 0
    row, head = st[-3], st[-2]
    for s in (batch, row, head):
        _check(abs(s) <= _INT_MAX, "stride does not fit the C ABI's int")
    return batch, row, head


def _aligned(t: torch.Tensor) -> bool:
    """16-byte vector access requirement of the kernels (8 x 16-bit elements)."""
    if t.data_ptr() % 16 != 0:
        return False
    return all(s % 8 == 0 for s in t.stride()[:-1])


def _vec_ok(t: torch.Tensor) -> torch.Tensor:
    return t if _aligned(t) else t.contiguous()


def _check_inputs(q, k, v, name="FlashAttention"):
    _check(q.is_cuda and k.is_cuda and v.is_cuda, "Input tensor must be on CUDA device")
    _check(_is_gfx950(q.device),
           "FlashAttention MI355X build only supports gfx950 (MI355X) GPUs")
    _check(q.dtype in (torch.float16, torch.bfloat16),
           "FlashAttention only support fp16 and bf16 data type")
    _check(k.dtype == q.dtype, "query and key must have the same dtype")
    _check(v.dtype == q.dtype, "query and value must have the same dtype")
    _check(q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1,
           "Input tensor must have contiguous last dimension")


def _pad8(x: torch.Tensor, d_og: int):
    if d_og % 8 == 0:
        return x
    return torch.nn.functional.pad(x, (0, 8 - d_og % 8))


def _seed_offset(p_dropout, gen, device, counter_offset):
    """Philox (seed, offset) for one dropout call, as the reference takes them from the CUDA
    generator: gen->philox_cuda_state(batch * nheads * 32) (flash_api.cpp:297-312), i.e. the current
    offset, then the generator's offset advanced by the increment rounded up to a multiple of 4.
    Without dropout nothing is drawn and (0, 0) is recorded."""
    if not p_dropout > 0.0:
        return 0, 0
    if gen is None:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        gen = torch.cuda.default_generators[idx]
    seed = gen.initial_seed()
    offset = gen.get_offset()
    gen.set_offset(offset + (counter_offset + 3) // 4 * 4)
    return int(seed) & (2 ** 64 - 1), int(offset)


def _bwd_rng(p_dropout, rng_state, gen, device, counter_offset):
    """(rng_state pointer, seed, offset) for the backward.  With the forward's rng_state the kernels
    read (seed, offset) from it on the device (the *_bwd_gqa entries; reference mha_bwd
    flash_api.cpp:669-670 and flash_bwd_kernel.h:783-784): no host round trip, capturable.  Without
    one, dropout draws from the generator as the reference does (flash_api.cpp:671-677)."""
    if not p_dropout > 0.0 or rng_state is not None:
        return _ptr(rng_state), 0, 0
    seed, offset = _seed_offset(p_dropout, gen, device, counter_offset)
    return None, seed, offset


# --------------------------------------------------------------------------------------------------
# fwd  (reference mha_fwd, flash_api.cpp:186-324)
# --------------------------------------------------------------------------------------------------
def fwd(q, k, v, out_, p_dropout, softmax_scale, is_causal, return_softmax, gen_):
    _check_inputs(q, k, v)
    _check(q.dim() == 4, "q must have shape (batch, seqlen_q, num_heads, head_size)")
    batch_size, seqlen_q, num_heads, head_size_og = q.shape
    seqlen_k, num_heads_k = k.shape[1], k.shape[2]
    _check(batch_size > 0, "batch size must be postive")
    _check(head_size_og <= 256, "FlashAttention forward only supports head dimension at most 256")
    _check(num_heads % num_heads_k == 0,
           "Number of heads in key/value must divide number of heads in query")
    _check(tuple(k.shape) == (batch_size, seqlen_k, num_heads_k, head_size_og),
           "k must have shape (batch_size, seqlen_k, num_heads_k, head_size_og)")
    _check(tuple(v.shape) == (batch_size, seqlen_k, num_heads_k, head_size_og),
           "v must have shape (batch_size, seqlen_k, num_heads_k, head_size_og)")
    if return_softmax:
        _check(p_dropout > 0.0, "return_softmax is only supported when p_dropout > 0.0")

    q_padded, k_padded, v_padded = (_pad8(x, head_size_og) for x in (q, k, v))
    qk, kk, vk = (_vec_ok(x) for x in (q_padded, k_padded, v_padded))

    if out_ is not None:
        out = out_
        _check(out.dtype == q.dtype, "Output must have the same dtype as inputs")
        _check(out.is_cuda, "Output tensor must be on CUDA device")
        _check(out.stride(-1) == 1, "Output tensor must have contiguous last dimension")
        _check(tuple(out.shape) == (batch_size, seqlen_q, num_heads, head_size_og),
               "out must have shape (batch_size, seqlen_q, num_heads, head_size_og)")
        if head_size_og % 8 != 0 or not _aligned(out):
            out = torch.empty_like(q_padded)
    else:
        out = torch.empty_like(q_padded)

    head_size = _round_multiple(head_size_og, 8)
    head_size_rounded = _round_multiple(head_size, 32)
    seqlen_q_rounded = _round_multiple(seqlen_q, 128)
    seqlen_k_rounded = _round_multiple(seqlen_k, 128)

    with _device_guard(q.device):
        softmax_lse = torch.empty((batch_size, num_heads, seqlen_q), dtype=torch.float32, device=q.device)
        p = None
        if return_softmax:   # S_dmask (b, h, sq_r, sk_r), dropped elements negated
            p = torch.empty((batch_size, num_heads, seqlen_q_rounded, seqlen_k_rounded), dtype=q.dtype,
                            device=q.device)
        rng_state = torch.empty((2,), dtype=torch.int64, device=q.device)
        seed, offset = _seed_offset(p_dropout, gen_, q.device, batch_size * num_heads * 32)
        qb, qr, qh = _strides(qk, 4)
        kb, kr, kh = _strides(kk, 4)
        vb, vr, vh = _strides(vk, 4)
        ob, orr, oh = _strides(out, 4)
        ok = _lib.flash_attn_fwd(
            _ptr(qk), _ptr(kk), _ptr(vk), _ptr(rng_state), _ptr(out), _ptr(p), _ptr(softmax_lse),
            batch_size, seqlen_q, seqlen_k, seqlen_q_rounded, seqlen_k_rounded,
            num_heads, num_heads_k, head_size, head_size_rounded,
            float(p_dropout), float(softmax_scale), 1.0, bool(is_causal), bool(return_softmax),
            q.dtype == torch.bfloat16, _stream(q), seed, offset,
            None, None, None, None, None, None, None, None,
            qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob)
        if not ok:
            _raise_lib_error("flash_attn_fwd")

    out_padded = out
    if head_size_og % 8 != 0:
        out = out[..., :head_size_og]
        if out_ is not None:
            out_.copy_(out)
    elif out_ is not None and out is not out_:
        out_.copy_(out)
        out = out_
    return [out, q_padded, k_padded, v_padded, out_padded, softmax_lse, p, rng_state]


# --------------------------------------------------------------------------------------------------
# varlen_fwd  (reference mha_varlen_fwd, flash_api.cpp:326-483)
# --------------------------------------------------------------------------------------------------
def varlen_fwd(q, k, v, out_, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, p_dropout,
               softmax_scale, zero_tensors, is_causal, return_softmax, gen_):
    _check_inputs(q, k, v)
    _check(cu_seqlens_q.dtype == torch.int32, "cu_seqlens_q must have dtype int32")
    _check(cu_seqlens_k.dtype == torch.int32, "cu_seqlens_k must have dtype int32")
    _check(cu_seqlens_q.is_cuda and cu_seqlens_k.is_cuda, "cu_seqlens must be on CUDA device")
    _check(cu_seqlens_q.is_contiguous() and cu_seqlens_k.is_contiguous(), "cu_seqlens must be contiguous")
    _check(q.dim() == 3, "q must have shape (total_q, num_heads, head_size)")
    batch_size = cu_seqlens_q.numel() - 1
    total_q, num_heads, head_size_og = q.shape
    total_k, num_heads_k = k.shape[0], k.shape[1]
    _check(batch_size > 0, "batch size must be positive")
    _check(head_size_og <= 256, "FlashAttention forward only supports head dimension at most 256")
    _check(num_heads % num_heads_k == 0,
           "Number of heads in key/value must divide number of heads in query")
    _check(tuple(k.shape) == (total_k, num_heads_k, head_size_og), "k must have shape (total_k, num_heads_k, head_size_og)")
    _check(tuple(v.shape) == (total_k, num_heads_k, head_size_og), "v must have shape (total_k, num_heads_k, head_size_og)")
    _check(cu_seqlens_k.numel() == batch_size + 1, "cu_seqlens_k must have shape (batch_size + 1)")
    if return_softmax:
        _check(p_dropout > 0.0, "return_softmax is only supported when p_dropout > 0.0")

    q_padded, k_padded, v_padded = (_pad8(x, head_size_og) for x in (q, k, v))
    qk, kk, vk = (_vec_ok(x) for x in (q_padded, k_padded, v_padded))
    if out_ is not None:
        out = out_
        _check(out.dtype == q.dtype, "Output must have the same dtype as inputs")
        _check(out.stride(-1) == 1, "Output tensor must have contiguous last dimension")
        _check(tuple(out.shape) == (total_q, num_heads, head_size_og),
               "out must have shape (total_q, num_heads, head_size_og)")
        if head_size_og % 8 != 0 or not _aligned(out):
            out = torch.empty_like(q_padded)
    else:
        out = torch.empty_like(q_padded)

    head_size = _round_multiple(head_size_og, 8)
    head_size_rounded = _round_multiple(head_size, 32)
    seqlen_q_rounded = _round_multiple(max_seqlen_q, 128)
    seqlen_k_rounded = _round_multiple(max_seqlen_k, 128)

    with _device_guard(q.device):
        softmax_lse = torch.empty((batch_size, num_heads, max_seqlen_q), dtype=torch.float32, device=q.device)
        if zero_tensors:
            out.zero_()
            softmax_lse.fill_(float("-inf"))
        p = None
        if return_softmax:   # S_dmask (b, h, sq_r, sk_r), dropped elements negated
            p = torch.empty((batch_size, num_heads, seqlen_q_rounded, seqlen_k_rounded), dtype=q.dtype,
                            device=q.device)
        rng_state = torch.empty((2,), dtype=torch.int64, device=q.device)
        seed, offset = _seed_offset(p_dropout, gen_, q.device, batch_size * num_heads * 32)
        _, qr, qh = _strides(qk, 3)
        _, kr, kh = _strides(kk, 3)
        _, vr, vh = _strides(vk, 3)
        _, orr, oh = _strides(out, 3)
        ok = _lib.flash_attn_varlen_fwd(
            _ptr(qk), _ptr(kk), _ptr(vk), _ptr(cu_seqlens_q), _ptr(cu_seqlens_k), _ptr(rng_state),
            _ptr(out), _ptr(p), _ptr(softmax_lse), batch_size, int(max_seqlen_q), int(max_seqlen_k),
            seqlen_q_rounded, seqlen_k_rounded, num_heads, num_heads_k, head_size,
            head_size_rounded, float(p_dropout), float(softmax_scale), 1.0, bool(is_causal),
            bool(return_softmax), q.dtype == torch.bfloat16, _stream(q), seed, offset, None, None,
            qr, kr, vr, qh, kh, vh, orr, oh, 0, 0, 0, 0, False)
        if not ok:
            _raise_lib_error("flash_attn_varlen_fwd")

    out_padded = out
    if head_size_og % 8 != 0:
        out = out[..., :head_size_og]
        if out_ is not None:
            out_.copy_(out)
    elif out_ is not None and out is not out_:
        out_.copy_(out)
        out = out_
    return [out, q_padded, k_padded, v_padded, out_padded, softmax_lse, p, rng_state]


# --------------------------------------------------------------------------------------------------
# bwd  (reference mha_bwd, flash_api.cpp:493-694)
# --------------------------------------------------------------------------------------------------
def _grad_buffer(given, like):
    """Caller-provided dq/dk/dv are written in place (reference :581-601); unaligned or padded
    destinations go through a temporary that is copied back."""
    if given is None:
        return torch.empty_like(like), None
    if given.shape[-1] == like.shape[-1] and _aligned(given):
        return given, None
    return torch.empty(like.shape, dtype=like.dtype, device=like.device), given


def _finish_grad(buf, given, head_size_og):
    if given is None:
        return buf[..., :head_size_og] if buf.shape[-1] != head_size_og else buf
    given.copy_(buf[..., :given.shape[-1]])
    return given


def bwd(dout, q, k, v, out, softmax_lse, dq_, dk_, dv_, p_dropout, softmax_scale, is_causal,
        gen_, rng_state):
    _check_inputs(q, k, v)
    _check(out.dtype == q.dtype and dout.dtype == q.dtype, "out and dout must have the same dtype as q")
    _check(q.dim() == 4, "q must have shape (batch, seqlen_q, num_heads, head_size)")
    batch_size, seqlen_q, num_heads, head_size = q.shape
    head_size_og = dout.shape[3]
    seqlen_k, num_heads_k = k.shape[1], k.shape[2]
    _check(batch_size > 0, "batch size must be positive")
    _check(head_size % 8 == 0, "head_size should be a multiple of 8")
    _check(head_size <= 256, "FlashAttention backward only supports head dimension at most 256")
    _check(num_heads % num_heads_k == 0,
           "Number of heads in key/value must divide number of heads in query")
    _check(out.stride(-1) == 1 and dout.stride(-1) == 1, "out/dout must have contiguous last dimension")

    head_size_rounded = _round_multiple(head_size, 32)
    seqlen_q_rounded = _round_multiple(seqlen_q, 128)
    seqlen_k_rounded = _round_multiple(seqlen_k, 128)

    dout_padded = _pad8(dout, head_size_og)
    qk, kk, vk, ok_, dok = (_vec_ok(x) for x in (q, k, v, out, dout_padded))
    dq, dq_given = _grad_buffer(dq_, q)
    dk, dk_given = _grad_buffer(dk_, k)
    dv, dv_given = _grad_buffer(dv_, v)

    with _device_guard(q.device):
        softmax_d = torch.empty((batch_size, num_heads, seqlen_q_rounded), dtype=torch.float32, device=q.device)
        # scratch for the kernels' -LSE/scale rows (the reference allocates (b, h, sq_r, d_r) here for
        # its fp32 atomic dQ accumulator; the MI355X backward needs only (b, h, sq_r))
        dq_accum = torch.empty((batch_size, num_heads, seqlen_q_rounded), dtype=torch.float32, device=q.device)
        # the *_gqa entry: dk/dv with num_heads_k heads (== the reference's result after its
        # sum_out), rng_state read on the device
        rng_p, seed, offset = _bwd_rng(p_dropout, rng_state, gen_, q.device, batch_size * num_heads * 32)
        st = [_strides(x, 4) for x in (qk, kk, vk, ok_, dq, dk, dv, dok)]
        (qb, qr, qh), (kb, kr, kh), (vb, vr, vh), (ob, orr, oh) = st[:4]
        (dqb, dqr, dqh), (dkb, dkr, dkh), (dvb, dvr, dvh), (dob, dor, doh) = st[4:]
        ok = _lib.flash_attn_bwd_gqa(
                _ptr(dok), _ptr(qk), _ptr(kk), _ptr(vk), _ptr(ok_), _ptr(softmax_d),
                _ptr(softmax_lse), rng_p, _ptr(dq), _ptr(dk), _ptr(dv), _ptr(dq_accum),
                batch_size, seqlen_q, seqlen_k, seqlen_q_rounded, seqlen_k_rounded,
                num_heads, num_heads_k, head_size, head_size_rounded,
                float(p_dropout), float(softmax_scale), 1.0, bool(is_causal),
                q.dtype == torch.bfloat16, 0, _stream(q), seed, offset,
                None, None, None, None, None, None, None, None,
                qr, kr, vr, qh, kh, vh, orr, oh, qb, kb, vb, ob,
                dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, dqb, dkb, dvb, dob)
        if not ok:
            _raise_lib_error("flash_attn_bwd")

    dq = _finish_grad(dq, dq_given, head_size_og)
    dk = _finish_grad(dk, dk_given, head_size_og)
    dv = _finish_grad(dv, dv_given, head_size_og)
    return [dq, dk, dv, softmax_d]


# --------------------------------------------------------------------------------------------------
# varlen_bwd  (reference mha_varlen_bwd, flash_api.cpp:696-912)
# --------------------------------------------------------------------------------------------------
def varlen_bwd(dout, q, k, v, out, softmax_lse, dq_, dk_, dv_, cu_seqlens_q, cu_seqlens_k,
               max_seqlen_q, max_seqlen_k, p_dropout, softmax_scale, zero_tensors, is_causal,
               gen_, rng_state):
    _check_inputs(q, k, v)
    _check(out.dtype == q.dtype and dout.dtype == q.dtype, "out and dout must have the same dtype as q")
    _check(cu_seqlens_q.dtype == torch.int32 and cu_seqlens_k.dtype == torch.int32,
           "cu_seqlens_q/k must have dtype int32")
    _check(q.dim() == 3, "q must have shape (total_q, num_heads, head_size)")
    batch_size = cu_seqlens_q.numel() - 1
    total_q, num_heads, head_size = q.shape
    head_size_og = dout.shape[2]
    total_k, num_heads_k = k.shape[0], k.shape[1]
    _check(batch_size > 0, "batch size must be positive")
    _check(head_size % 8 == 0, "head_size should be a multiple of 8")
    _check(head_size <= 256, "FlashAttention backward only supports head dimension at most 256")
    _check(num_heads % num_heads_k == 0,
           "Number of heads in key/value must divide number of heads in query")

    head_size_rounded = _round_multiple(head_size, 32)
    seqlen_q_rounded = _round_multiple(max_seqlen_q, 128)
    seqlen_k_rounded = _round_multiple(max_seqlen_k, 128)

    dout_padded = _pad8(dout, head_size_og)
    qk, kk, vk, ok_, dok = (_vec_ok(x) for x in (q, k, v, out, dout_padded))
    dq, dq_given = _grad_buffer(dq_, q)
    dk, dk_given = _grad_buffer(dk_, k)
    dv, dv_given = _grad_buffer(dv_, v)

    with _device_guard(q.device):
        softmax_d = torch.empty((batch_size, num_heads, seqlen_q_rounded), dtype=torch.float32, device=q.device)
        # scratch for the kernels' -LSE/scale rows (the reference allocates (b, h, sq_r, d_r) here for
        # its fp32 atomic dQ accumulator; the MI355X backward needs only (b, h, sq_r))
        dq_accum = torch.empty((batch_size, num_heads, seqlen_q_rounded), dtype=torch.float32, device=q.device)
        if zero_tensors:
            dq.zero_(); dk.zero_(); dv.zero_(); softmax_d.zero_()
        rng_p, seed, offset = _bwd_rng(p_dropout, rng_state, gen_, q.device, batch_size * num_heads * 32)
        st = [_strides(x, 3) for x in (qk, kk, vk, ok_, dq, dk, dv, dok)]
        (_, qr, qh), (_, kr, kh), (_, vr, vh), (_, orr, oh) = st[:4]
        (_, dqr, dqh), (_, dkr, dkh), (_, dvr, dvh), (_, dor, doh) = st[4:]
        ok = _lib.flash_attn_varlen_bwd_gqa(
                _ptr(dok), _ptr(qk), _ptr(kk), _ptr(vk), _ptr(ok_), _ptr(softmax_d),
                _ptr(softmax_lse), _ptr(cu_seqlens_q), _ptr(cu_seqlens_k), rng_p,
                _ptr(dq), _ptr(dk), _ptr(dv), _ptr(dq_accum), batch_size, int(max_seqlen_q),
                int(max_seqlen_k), seqlen_q_rounded, seqlen_k_rounded, num_heads, num_heads_k,
                head_size, head_size_rounded, float(p_dropout), float(softmax_scale), 1.0,
                bool(is_causal), q.dtype == torch.bfloat16, 0, _stream(q),
                seed, offset, None, None,
                qr, kr, vr, qh, kh, vh, orr, oh, 0, 0, 0, 0,
                dqr, dkr, dvr, dqh, dkh, dvh, dor, doh, 0, 0, 0, 0, False)
        if not ok:
            _raise_lib_error("flash_attn_varlen_bwd")

    dq = _finish_grad(dq, dq_given, head_size_og)
    dk = _finish_grad(dk, dk_given, head_size_og)
    dv = _finish_grad(dv, dv_given, head_size_og)
    return [dq, dk, dv, softmax_d]
