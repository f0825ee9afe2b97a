"""Attention modules over the MI355X kernels (the reference's callers).

Drop-in for the attention-core classes of the reference's ``flash_attn/modules/mha.py``:

  * ``FlashSelfAttention``  (reference ``:35-84``)   -- packed qkv, fixed-length or varlen;
  * ``FlashCrossAttention`` (reference ``:87-142``)  -- q plus packed kv, fixed-length or varlen;
  * ``MHA``                 (reference ``:343-561``) -- the projection wrapper, restricted to what
    sits on this path: fused Wqkv (or Wq + Wkv for cross attention), MQA / GQA through
    ``num_heads_kv``, rotary embedding (``flash_attn.layers.rotary``, HIP kernel), causal /
    dropout / softmax_scale, and the output projection.  The reference's tensor-parallel linears,
    fused dense and KV-cache inference are out of scope (SURVEY.md §8 marks the callers' own
    subsystems outside the hot path); asking for them raises.

Same constructor arguments, forward signatures, shape conventions and dropout semantics
(``self.drop.p`` while training, 0 in eval) as the reference.  Everything runs through
``flash_attn.flash_attn_interface`` -- there is no PyTorch fallback attention here.
"""
import torch
import torch.nn as nn

from flash_attn.flash_attn_interface import (flash_attn_kvpacked_func, flash_attn_qkvpacked_func,
                                             flash_attn_varlen_kvpacked_func,
                                             flash_attn_varlen_qkvpacked_func)

__all__ = ["FlashSelfAttention", "FlashCrossAttention", "MHA"]


class FlashSelfAttention(nn.Module):
    """Scaled dot-product attention with softmax over packed qkv (reference mha.py:35-84).

    softmax_scale: temperature (default 1/sqrt(headdim)); attention_dropout: dropout rate.
    """

    def __init__(self, causal=False, softmax_scale=None, attention_dropout=0.0):
        super().__init__()
        self.causal = causal
        self.softmax_scale = softmax_scale
        self.drop = nn.Dropout(attention_dropout)

    def forward(self, qkv, causal=None, cu_seqlens=None, max_seqlen=None):
        """qkv: (B, S, 3, H, D), or (total, 3, H, D) with cu_seqlens (B+1,) int32 and max_seqlen.
        Returns (B, S, H, D), or (total, H, D) for varlen."""
        assert qkv.dtype in (torch.float16, torch.bfloat16)
        assert qkv.is_cuda
        causal = self.causal if causal is None else causal
        dropout_p = self.drop.p if self.training else 0.0
        if cu_seqlens is not None:
            assert cu_seqlens.dtype == torch.int32
            assert max_seqlen is not None and isinstance(max_seqlen, int)
            return flash_attn_varlen_qkvpacked_func(qkv, cu_seqlens, max_seqlen, dropout_p,
                                                    softmax_scale=self.softmax_scale, causal=causal)
        return flash_attn_qkvpacked_func(qkv, dropout_p, softmax_scale=self.softmax_scale, causal=causal)


class FlashCrossAttention(nn.Module):
    """Scaled dot-product attention of q against packed kv (reference mha.py:87-142)."""

    def __init__(self, causal=False, softmax_scale=None, attention_dropout=0.0):
        super().__init__()
        self.causal = causal
        self.softmax_scale = softmax_scale
        self.drop = nn.Dropout(attention_dropout)

    def forward(self, q, kv, causal=None, cu_seqlens=None, max_seqlen=None, cu_seqlens_k=None,
                max_seqlen_k=None):
        """q: (B, Sq, H, D), kv: (B, Sk, 2, H_k, D); varlen: q (total_q, H, D), kv (total_k, 2, H_k, D)
        with cu_seqlens / cu_seqlens_k (B+1,) int32 and max_seqlen / max_seqlen_k."""
        assert q.dtype in (torch.float16, torch.bfloat16)
        assert q.is_cuda and kv.is_cuda
        causal = self.causal if causal is None else causal
        dropout_p = self.drop.p if self.training else 0.0
        if cu_seqlens is not None:
            assert cu_seqlens.dtype == torch.int32
            assert max_seqlen is not None and isinstance(max_seqlen, int)
            assert cu_seqlens_k is not None and cu_seqlens_k.dtype == torch.int32
            assert max_seqlen_k is not None and isinstance(max_seqlen_k, int)
            return flash_attn_varlen_kvpacked_func(q, kv, cu_seqlens, cu_seqlens_k, max_seqlen,
                                                   max_seqlen_k, dropout_p,
                                                   softmax_scale=self.softmax_scale, causal=causal)
        batch_size = q.shape[0]
        assert kv.shape[0] == batch_size and kv.shape[4] == q.shape[3]
        return flash_attn_kvpacked_func(q, kv, dropout_p, softmax_scale=self.softmax_scale,
                                        causal=causal)


class MHA(nn.Module):
    """Multi-head attention block: Wqkv -> FlashSelfAttention / FlashCrossAttention -> out_proj.

    Constructor arguments follow the reference (mha.py:347-448, forward :449-561); rotary_emb_dim > 0
    applies flash_attn.layers.rotary.RotaryEmbedding (HIP kernel) to q and k as the reference does.
    The ones that select subsystems outside this build (fused_bias_fc, dwconv, return_residual,
    process_group, use_flash_attn=False) are accepted only at their neutral value.
    """

    def __init__(self, embed_dim, num_heads, num_heads_kv=None, cross_attn=False, qkv_proj_bias=True,
                 out_proj_bias=True, dropout=0.0, softmax_scale=None, causal=False, layer_idx=None,
                 dwconv=False, rotary_emb_dim=0, rotary_emb_base=10000.0, rotary_emb_scale_base=None,
                 rotary_emb_interleaved=False, fused_bias_fc=False, use_flash_attn=True,
                 return_residual=False, checkpointing=False, device=None, dtype=None):
        super().__init__()
        for name, val, neutral in (("dwconv", dwconv, False),
                                   ("fused_bias_fc", fused_bias_fc, False),
                                   ("use_flash_attn", use_flash_attn, True),
                                   ("return_residual", return_residual, False)):
            if val != neutral:
                raise NotImplementedError(f"MHA({name}={val!r}) is outside the MI355X attention build")
        factory = {"device": device, "dtype": dtype}
        self.embed_dim = embed_dim
        self.cross_attn = cross_attn
        self.causal = causal
        self.layer_idx = layer_idx
        self.checkpointing = checkpointing
        self.num_heads = num_heads
        self.num_heads_kv = num_heads_kv if num_heads_kv is not None else num_heads
        assert self.num_heads % self.num_heads_kv == 0, "num_heads must be divisible by num_heads_kv"
        assert self.embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        self.head_dim = self.embed_dim // num_heads
        self.rotary_emb_dim = rotary_emb_dim
        if rotary_emb_dim > 0:   # reference mha.py:379-384
            assert not cross_attn, "MHA with rotary embedding does not support cross-attention yet"
            from flash_attn.layers.rotary import RotaryEmbedding
            self.rotary_emb = RotaryEmbedding(rotary_emb_dim, base=rotary_emb_base,
                                              scale_base=rotary_emb_scale_base,
                                              interleaved=rotary_emb_interleaved, device=device)
        qkv_dim = self.head_dim * (self.num_heads + 2 * self.num_heads_kv)
        kv_dim = 2 * self.head_dim * self.num_heads_kv
        if not self.cross_attn:
            self.Wqkv = nn.Linear(embed_dim, qkv_dim, bias=qkv_proj_bias, **factory)
        else:
            self.Wq = nn.Linear(embed_dim, embed_dim, bias=qkv_proj_bias, **factory)
            self.Wkv = nn.Linear(embed_dim, kv_dim, bias=qkv_proj_bias, **factory)
        self.inner_attn = FlashSelfAttention(causal=causal, softmax_scale=softmax_scale,
                                             attention_dropout=dropout)
        self.inner_cross_attn = FlashCrossAttention(causal=causal, softmax_scale=softmax_scale,
                                                    attention_dropout=dropout)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=out_proj_bias, **factory)

    def forward(self, x, x_kv=None, key_padding_mask=None, cu_seqlens=None, max_seqlen=None,
                mixer_subset=None, inference_params=None, **kwargs):
        """x: (B, S, E), or (total, E) with cu_seqlens / max_seqlen (varlen, self-attention only).
        x_kv: (B, Sk, E) for cross attention.  key_padding_mask is the reference's padded-batch
        convenience: it unpads, runs varlen attention and pads back."""
        if inference_params is not None or mixer_subset is not None:
            raise NotImplementedError("MHA inference cache / mixer_subset is outside the MI355X build")
        if key_padding_mask is not None:
            assert cu_seqlens is None and not self.cross_attn
            from flash_attn.bert_padding import pad_input, unpad_input
            b, s = x.shape[:2]
            x_unpad, indices, cu, max_s = unpad_input(x, key_padding_mask)
            out = self.forward(x_unpad, cu_seqlens=cu, max_seqlen=max_s)
            return pad_input(out, indices, b, s)
        h, hk, d = self.num_heads, self.num_heads_kv, self.head_dim
        if self.rotary_emb_dim > 0 and cu_seqlens is not None:
            raise NotImplementedError("MHA: rotary embedding with varlen / key_padding_mask input")
        if not self.cross_attn:
            qkv = self.Wqkv(x)
            lead = qkv.shape[:-1]
            if hk == h:
                qkv = qkv.view(*lead, 3, h, d)
                if self.rotary_emb_dim > 0:   # reference mha.py:499-500
                    qkv = self.rotary_emb(qkv)
                context = self.inner_attn(qkv, cu_seqlens=cu_seqlens, max_seqlen=max_seqlen)
            else:
                q = qkv[..., : h * d].reshape(*lead, h, d)
                kv = qkv[..., h * d:].reshape(*lead, 2, hk, d)
                if self.rotary_emb_dim > 0:   # reference mha.py:544-545
                    q, kv = self.rotary_emb(q, kv)
                if cu_seqlens is not None:
                    context = self.inner_cross_attn(q, kv, cu_seqlens=cu_seqlens, max_seqlen=max_seqlen,
                                                    cu_seqlens_k=cu_seqlens, max_seqlen_k=max_seqlen)
                else:
                    context = self.inner_cross_attn(q, kv)
        else:
            assert cu_seqlens is None, "varlen cross attention: call FlashCrossAttention directly"
            x_kv = x if x_kv is None else x_kv
            q = self.Wq(x).reshape(*x.shape[:-1], h, d)
            kv = self.Wkv(x_kv).reshape(*x_kv.shape[:-1], 2, hk, d)
            context = self.inner_cross_attn(q, kv)
        return self.out_proj(context.reshape(*context.shape[:-2], h * d))

