"""Padding helpers that build the varlen (cu_seqlens) inputs of the FlashAttention API.

Same public functions and semantics as the reference's ``flash_attn/bert_padding.py``
(``index_first_axis``, ``index_put_first_axis``, ``unpad_input :97-117``, ``pad_input :120-132``):
``cu_seqlens`` is int32 ``(batch + 1,)`` with a leading 0, ``max_seqlen`` a Python int, and the
gather / scatter along the token axis are differentiable (gather <-> scatter adjoints).
"""
import torch

__all__ = ["index_first_axis", "index_put_first_axis", "unpad_input", "pad_input"]


class _GatherRows(torch.autograd.Function):
    """out[i] = x[indices[i]] over the first axis; backward scatters the rows back."""

    @staticmethod
    def forward(ctx, x, indices):
        ctx.save_for_backward(indices)
        ctx.first_dim = x.shape[0]
        return x.reshape(x.shape[0], -1)[indices].reshape((indices.numel(),) + x.shape[1:])

    @staticmethod
    def backward(ctx, grad):
        (indices,) = ctx.saved_tensors
        out = grad.new_zeros((ctx.first_dim,) + grad.shape[1:])
        out.index_copy_(0, indices, grad)
        return out, None


class _ScatterRows(torch.autograd.Function):
    """out = zeros(first_dim, ...); out[indices] = x; backward gathers the rows."""

    @staticmethod
    def forward(ctx, x, indices, first_dim):
        ctx.save_for_backward(indices)
        out = x.new_zeros((first_dim,) + x.shape[1:])
        out.index_copy_(0, indices, x)
        return out

    @staticmethod
    def backward(ctx, grad):
        (indices,) = ctx.saved_tensors
        return grad.index_select(0, indices), None, None


index_first_axis = _GatherRows.apply
index_put_first_axis = _ScatterRows.apply


def unpad_input(hidden_states, attention_mask):
    """hidden_states (batch, seqlen, ...), attention_mask (batch, seqlen) bool/int (1 = valid)
    -> (tokens (total_nnz, ...), indices (total_nnz,), cu_seqlens (batch+1,) int32, max_seqlen)."""
    seqlens = attention_mask.sum(dim=-1, dtype=torch.int32)
    indices = torch.nonzero(attention_mask.flatten(), as_tuple=False).flatten()
    max_seqlen = int(seqlens.max().item())
    cu_seqlens = torch.zeros(seqlens.numel() + 1, dtype=torch.int32, device=seqlens.device)
    cu_seqlens[1:] = torch.cumsum(seqlens, dim=0, dtype=torch.int32)
    flat = hidden_states.reshape((-1,) + hidden_states.shape[2:])
    return index_first_axis(flat, indices), indices, cu_seqlens, max_seqlen


def pad_input(hidden_states, indices, batch, seqlen):
    """tokens (total_nnz, ...) + indices -> (batch, seqlen, ...) with zeros at padded positions."""
    out = index_put_first_axis(hidden_states, indices, batch * seqlen)
    return out.reshape((batch, seqlen) + hidden_states.shape[1:])
