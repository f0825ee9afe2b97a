"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

What it executes from the reference (read-only, nothing copied into this repo):
  * ``attention_ref`` and ``generate_random_padding_mask`` of /root/reference/tests/test_flash_attn.py
    (lines 26-35 and 111-159).  The test module's top level needs CUDA and the compiled
    ``flash_attn_2_cuda``, so only those two function definitions are extracted from its AST and
    executed with torch / math / einops in scope.
  * /root/reference/flash_attn/bert_padding.py (unpad_input / pad_input), loaded by file path.

Each case stores seeded inputs and the reference's outputs (in the case dtype, exactly as the
reference returns them): out_ref / out_pt (attention_ref with
upcast=True, and upcast=False + reorder_ops=True: the "PyTorch error" baseline of the 2x rule),
lse_ref (logsumexp of the scaled masked scores, float64), and dq/dk/dv for both (autograd).
16-bit tensors are stored as their raw uint16 bits; dtype recorded per case.
"""
import ast
import importlib.util
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F
from einops import rearrange, repeat

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_reference_functions():
    path = os.path.join(REF, "tests", "test_flash_attn.py")
    tree = ast.parse(open(path).read(), filename=path)
    wanted = {"attention_ref", "generate_random_padding_mask"}
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in wanted]
    assert {n.name for n in body} == wanted
    ns = {"torch": torch, "math": math, "F": F, "rearrange": rearrange, "repeat": repeat}
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    spec = importlib.util.spec_from_file_location("ref_bert_padding", os.path.join(REF, "flash_attn", "bert_padding.py"))
    bp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bp)
    return ns["attention_ref"], ns["generate_random_padding_mask"], bp


def to_store(t):
    t = t.detach().cpu()
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def lse_of(q, k, causal, key_padding_mask=None, query_padding_mask=None):
    q, k = q.double(), k.double()
    g = q.shape[2] // k.shape[2]
    k = repeat(k, "b s h d -> b s (h g) d", g=g)
    s = torch.einsum("bthd,bshd->bhts", q, k) / math.sqrt(q.shape[-1])
    if key_padding_mask is not None:
        s.masked_fill_(rearrange(~key_padding_mask, "b s -> b 1 1 s"), float("-inf"))
    if causal:
        s.masked_fill_(torch.triu(torch.ones(s.shape[-2], s.shape[-1], dtype=torch.bool), 1), float("-inf"))
    return torch.logsumexp(s, -1).float()


def dense_case(attention_ref, name, b, sq, sk, h, hk, d, dtype, causal, qscale=1.0, kvscale=1.0):
    torch.manual_seed(0)
    q = (torch.randn(b, sq, h, d, dtype=dtype) * qscale).requires_grad_()
    k = (torch.randn(b, sk, hk, d, dtype=dtype) * kvscale).requires_grad_()
    v = (torch.randn(b, sk, hk, d, dtype=dtype) * kvscale).requires_grad_()
    g = torch.randn(b, sq, h, d, dtype=dtype)
    out_ref, _ = attention_ref(q, k, v, causal=causal)
    out_pt, _ = attention_ref(q, k, v, causal=causal, upcast=False, reorder_ops=True)
    dq_ref, dk_ref, dv_ref = torch.autograd.grad(out_ref, (q, k, v), g)
    dq_pt, dk_pt, dv_pt = torch.autograd.grad(out_pt, (q, k, v), g)
    rec = dict(kind="dense", dtype=str(dtype).split(".")[-1], causal=causal,
               shape=np.array([b, sq, sk, h, hk, d]),
               q=to_store(q), k=to_store(k), v=to_store(v), dout=to_store(g),
               out_ref=to_store(out_ref), out_pt=to_store(out_pt),
               lse_ref=to_store(lse_of(q, k, causal)),
               dq_ref=to_store(dq_ref), dk_ref=to_store(dk_ref), dv_ref=to_store(dv_ref),
               dq_pt=to_store(dq_pt), dk_pt=to_store(dk_pt), dv_pt=to_store(dv_pt))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(name, "eps_out", (out_pt.float() - out_ref.float()).abs().max().item())


def varlen_case(attention_ref, gen_mask, bp, name, b, s, h, d, dtype, causal):
    torch.manual_seed(0)
    qkv = torch.randn(b, s, 3, h, d, dtype=dtype)
    mask = gen_mask(s, b, "cpu", mode="random")
    q, k, v = [x.detach().clone().requires_grad_() for x in qkv.unbind(2)]
    _, indices, cu_seqlens, max_seqlen = bp.unpad_input(q, mask)
    g = torch.randn(b, s, h, d, dtype=dtype)
    g = g.masked_fill(~mask[:, :, None, None], 0.0)
    out_ref, _ = attention_ref(q, k, v, mask, mask, causal=causal)
    out_pt, _ = attention_ref(q, k, v, mask, mask, causal=causal, upcast=False, reorder_ops=True)
    dq_ref, dk_ref, dv_ref = torch.autograd.grad(out_ref, (q, k, v), g)
    dq_pt, dk_pt, dv_pt = torch.autograd.grad(out_pt, (q, k, v), g)
    rec = dict(kind="varlen", dtype=str(dtype).split(".")[-1], causal=causal,
               shape=np.array([b, s, s, h, h, d]), mask=mask.numpy(),
               indices=indices.numpy(), cu_seqlens=cu_seqlens.numpy(), max_seqlen=np.array(max_seqlen),
               q=to_store(q), k=to_store(k), v=to_store(v), dout=to_store(g),
               out_ref=to_store(out_ref), out_pt=to_store(out_pt),
               lse_ref=to_store(lse_of(q, k, causal, mask)),
               dq_ref=to_store(dq_ref), dk_ref=to_store(dk_ref), dv_ref=to_store(dv_ref),
               dq_pt=to_store(dq_pt), dk_pt=to_store(dk_pt), dv_pt=to_store(dv_pt))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(name, "cu_seqlens", cu_seqlens.tolist(), "eps_out", (out_pt.float() - out_ref.float()).abs().max().item())


def main():
    attention_ref, gen_mask, bp = load_reference_functions()
    # C1 exactly (fp32, the CPU plumbing config)
    dense_case(attention_ref, "c1_fp32_b2_s128_h4_d64", 2, 128, 128, 4, 4, 64, torch.float32, False)
    # C2-class: bf16 hdim64 causal, odd seqlen
    dense_case(attention_ref, "bf16_s97_h3_d64_causal", 2, 97, 97, 3, 3, 64, torch.bfloat16, True)
    # C3-class: bf16 hdim128 causal / non-causal
    dense_case(attention_ref, "bf16_s257_h2_d128_causal", 1, 257, 257, 2, 2, 128, torch.bfloat16, True)
    dense_case(attention_ref, "bf16_s200_h2_d128", 1, 200, 200, 2, 2, 128, torch.bfloat16, False)
    # C5-class: fp16 GQA causal with seqlen_q != seqlen_k (both directions)
    dense_case(attention_ref, "fp16_gqa_sq113_sk203_h6_hk2_d128_causal", 1, 113, 203, 6, 2, 128, torch.float16, True)
    dense_case(attention_ref, "fp16_gqa_sq211_sk113_h4_hk1_d64_causal", 1, 211, 113, 4, 1, 64, torch.float16, True)
    # head dim not a multiple of 32 (and one not a multiple of 8: padded by the extension)
    dense_case(attention_ref, "fp16_s64_h2_d40", 2, 64, 64, 2, 2, 40, torch.float16, False)
    dense_case(attention_ref, "bf16_s80_h2_d59_causal", 1, 80, 80, 2, 2, 59, torch.bfloat16, True)
    # overflow regime of test_flash_attn_bwd_overflow (q*5, k/v*3, short seqlen)
    dense_case(attention_ref, "fp16_overflow_s17_h5_d32_causal", 2, 17, 17, 5, 5, 32, torch.float16, True, 5.0, 3.0)
    # C4-class: varlen qkvpacked, random key padding
    varlen_case(attention_ref, gen_mask, bp, "varlen_bf16_b3_s150_h2_d128_causal", 3, 150, 2, 128, torch.bfloat16, True)
    varlen_case(attention_ref, gen_mask, bp, "varlen_fp16_b4_s70_h2_d64", 4, 70, 2, 64, torch.float16, False)


if __name__ == "__main__":
    sys.exit(main())
