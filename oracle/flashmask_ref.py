"""ORACLE -- test infrastructure only (never imported by the product path).

CPU restatement of the reference's FlashMask column-range mask, as a boolean
"keep" matrix that the tests turn into an attention reference.

FlashMask gives, per (batch, mask head, key column k), int32 row bounds:
  LTStart = flashmask_downstart, LTEnd = flashmask_downend, UTStart = flashmask_upstart,
  UTEnd = flashmask_upend  (C ABI csrc/capi/flash_attn.h:38-43).
The reference removes (row, k), comparing as uint32 (csrc/flash_attn/src/softmax.h):
  causal, LTEnd absent   apply_sparse_mask_causal          :180-211   k > row  or  row >= LTStart
  causal, LTEnd given    apply_sparse_mask_causal_withend  :213-247   k > row  or  LTStart <= row < LTEnd
  non-causal, UTStart    apply_sparse_mask pairwise        :249-296   LTStart <= row < LTEnd  or
                         (called twice, flash_fwd_kernel.h:1360-1382)  UTStart <= row < UTEnd
  non-causal, no UTStart apply_sparse_mask non-pairwise    (fwd :1384-1394)   row >= LTStart  or  row < UTEnd
and keys >= seqlen_k always.  The mask head of attention head h is h / (h_q / mask_heads)
(flash_fwd_kernel.h:1109).  The reference takes this path iff downstart is given
(capi/flash_attn.cu:540).  Its tile-skip scan (mask.h:4-126, the maxmin scratch) only skips tiles
that this rule removes entirely, so it does not change results and is not restated.

Parity: the reference's own tests hold no FlashMask fixtures (FlashMask is exercised from Paddle),
so this restatement is checked against the per-element loop form below and hand-derived known
answers (tests/test_flashmask_oracle.py) -- parity unpinned against reference outputs.
"""
from __future__ import annotations

import numpy as np


def _u32(x):
    return np.asarray(x, dtype=np.int64).astype(np.uint32)


def flashmask_keep(lts, sq, causal, lte=None, uts=None, ute=None):
    """keep[b, hm, q, k] (bool) for bounds of shape (b, hm, sk); numpy, vectorised."""
    lts = _u32(lts)
    b, hm, sk = lts.shape
    row = np.arange(sq, dtype=np.uint32)[None, None, :, None]
    col = np.arange(sk, dtype=np.uint32)[None, None, None, :]
    L = lts[:, :, None, :]
    if causal:
        masked = col > row
        lt = row >= L
        if lte is not None:
            lt &= row < _u32(lte)[:, :, None, :]
        masked = masked | lt
    else:
        U = _u32(ute)[:, :, None, :]
        if uts is not None:
            masked = ((row >= L) & (row < _u32(lte)[:, :, None, :])) | \
                     ((row >= _u32(uts)[:, :, None, :]) & (row < U))
        else:
            masked = (row >= L) | (row < U)
    return ~masked


def flashmask_keep_loops(lts, sq, causal, lte=None, uts=None, ute=None):
    """The same, element by element in the reference's branch order (small cases only)."""
    lts = np.asarray(lts)
    b, hm, sk = lts.shape
    keep = np.ones((b, hm, sq, sk), dtype=bool)
    u = lambda x: int(x) & 0xFFFFFFFF  # noqa: E731  (uint32 compare)
    for bi in range(b):
        for hi in range(hm):
            for k in range(sk):
                s0 = u(lts[bi, hi, k])
                for r in range(sq):
                    if causal:
                        if k >= min(sk, r + 1):
                            m = True
                        elif lte is not None:
                            m = s0 <= r < u(lte[bi, hi, k])
                        else:
                            m = r >= s0
                    elif uts is not None:
                        m = (s0 <= r < u(lte[bi, hi, k])) or (u(uts[bi, hi, k]) <= r < u(ute[bi, hi, k]))
                    else:
                        m = r >= s0 or r < u(ute[bi, hi, k])
                    keep[bi, hi, r, k] = not m
    return keep


def document_lts(doc_lens, sq):
    """LTStart of a causal document mask: key k may be seen by rows up to the end of its document."""
    ends = np.cumsum(doc_lens)
    assert ends[-1] == sq
    out = np.empty(sq, dtype=np.int32)
    start = 0
    for e in ends:
        out[start:e] = e
        start = e
    return out
