"""GPU tests of attention dropout against the oracle's restatement of the reference's
Philox stream (oracle/dropout_ref.py).

* The keep/drop pattern the kernels use -- read from the sign of the returned S_dmask -- must equal
  the oracle's mask for the same (seed, offset) bit for bit, for every (batch, head) and element.
* Output and gradients follow the reference's test (tests/test_flash_attn.py:517-639 with
  dropout_p = 0.17): attention_ref with that dropout mask, the 2x-of-PyTorch-error bound.
"""
import numpy as np
import pytest
import torch

from oracle.attention_ref import attention_ref, check_within_bound, generate_qkv, generate_random_padding_mask
from oracle.dropout_ref import dropout_keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _gen_state():
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    return gen.initial_seed(), gen.get_offset()


def _oracle_mask(seed, offset, b, h, sq, sk, p):
    return torch.from_numpy(np.stack([np.stack([dropout_keep_mask(seed, offset, bi, hi, h, sq, sk, p)
                                                for hi in range(h)]) for bi in range(b)]))


def _valid(sq, sk, causal):
    v = torch.ones(sq, sk, dtype=torch.bool)
    if causal:
        v = ~torch.triu(v, 1)
    return v


def _bound(name, got, ref, pt, factor=2.0, floor=0.0):
    ok, err, bound = check_within_bound(got.detach().float(), ref.float(), pt.float(), factor=factor, floor=floor)
    assert ok, f"{name}: max|err| {err:.3e} > bound {bound:.3e}"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("sq,sk", [(113, 203), (256, 256), (512, 384)])
def test_dropout_mask_is_the_reference_stream(sq, sk, d, causal, dtype):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, h, p = 2, 3, 0.17
    q, k, v = (torch.randn(b, s, h, d, device=DEV, dtype=dtype) for s in (sq, sk, sk))
    seed, offset = _gen_state()
    out, lse, s_dmask = flash_attn_func(q, k, v, p, causal=causal, return_attn_probs=True)
    # the generator advanced by b * h * 32 (rounded to 4), as the reference's philox_cuda_state
    assert _gen_state()[1] == offset + (b * h * 32 + 3) // 4 * 4
    keep = _oracle_mask(seed, offset, b, h, sq, sk, p)
    sd = s_dmask[:, :, :sq, :sk].cpu()
    got_keep = ~torch.signbit(sd.float())
    valid = _valid(sq, sk, causal).expand_as(keep)
    mism = (got_keep != keep) & valid
    assert not mism.any(), f"{int(mism.sum())} of {int(valid.sum())} elements differ from the oracle stream"
    # |S_dmask| = softmax probabilities, zero where masked
    _, attn = attention_ref(q, k, v, causal=causal)
    torch.testing.assert_close(sd.abs().float(), attn.cpu().float().masked_fill(~valid, 0.0),
                               atol=2e-2 if dtype == torch.bfloat16 else 4e-3, rtol=0)
    # the measured keep rate is the reference's (floor(keep * 255) + 1) / 256
    rate = keep[valid].float().mean().item()
    assert abs(rate - (int(np.floor((1 - np.float32(p)) * 255.0)) + 1) / 256) < 0.02


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("mha_type", ["mha", "gqa"])
@pytest.mark.parametrize("d", [32, 64, 128, 192])
@pytest.mark.parametrize("sq,sk", [(113, 203), (128, 217), (256, 512), (512, 256), (1023, 1024)])
def test_dropout_output_and_grads(sq, sk, d, mha_type, causal, dtype):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, h, p = 2, 6, 0.17
    hk = h if mha_type == "mha" else 3
    q = torch.randn(b, sq, h, d, device=DEV, dtype=dtype, requires_grad=True)
    k = torch.randn(b, sk, hk, d, device=DEV, dtype=dtype, requires_grad=True)
    v = torch.randn(b, sk, hk, d, device=DEV, dtype=dtype, requires_grad=True)
    seed, offset = _gen_state()
    out, lse, s_dmask = flash_attn_func(q, k, v, p, causal=causal, return_attn_probs=True)
    keep = _oracle_mask(seed, offset, b, h, sq, sk, p).to(DEV)
    g = torch.randn_like(out)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)

    qc, kc, vc = (x.detach().clone().requires_grad_() for x in (q, k, v))
    out_ref, _ = attention_ref(qc, kc, vc, dropout_p=p, dropout_mask=keep, causal=causal)
    out_pt, _ = attention_ref(qc, kc, vc, dropout_p=p, dropout_mask=keep, causal=causal,
                              upcast=False, reorder_ops=True)
    _bound("out", out, out_ref, out_pt)
    gr = torch.autograd.grad(out_ref, (qc, kc, vc), g)
    gp = torch.autograd.grad(out_pt, (qc, kc, vc), g)
    for name, got, r, pt in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        _bound(name, got, r, pt)


@pytest.mark.parametrize("causal", [False, True])
def test_dropout_varlen(causal):
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(0)
    b, s, h, d, p, dtype = 4, 257, 4, 64, 0.2, torch.bfloat16
    q, k, v = (torch.randn(b, s, h, d, device=DEV, dtype=dtype) for _ in range(3))
    qm = generate_random_padding_mask(s, b, DEV, mode="random")
    (q_unpad, k_unpad, v_unpad, cu_q, cu_k, max_q, max_k, q, k, v, out_pad_fn, dq_pad_fn,
     dk_pad_fn) = generate_qkv(q, k, v, qm, qm)
    seed, offset = _gen_state()
    out_unpad, lse, s_dmask = flash_attn_varlen_func(q_unpad, k_unpad, v_unpad, cu_q, cu_k, max_q, max_k,
                                                     p, causal=causal, return_attn_probs=True)
    # per-sequence masks: rows / cols relative to each sequence, offset by (batch, head)
    lens = (cu_q[1:] - cu_q[:-1]).tolist()
    keep = torch.zeros(b, h, s, s, dtype=torch.bool)
    for bi, L in enumerate(lens):
        for hi in range(h):
            keep[bi, hi, :L, :L] = torch.from_numpy(dropout_keep_mask(seed, offset, bi, hi, h, L, L, p))
        sd = s_dmask[bi, :, :L, :L].cpu()
        valid = _valid(L, L, causal)
        got = ~torch.signbit(sd.float())
        assert not ((got != keep[bi, :, :L, :L]) & valid).any()
    out = out_pad_fn(out_unpad)
    qc, kc, vc = (x.detach().float() for x in (q, k, v))
    out_ref, _ = attention_ref(qc, kc, vc, qm, qm, dropout_p=p, dropout_mask=keep.to(DEV), causal=causal)
    out_pt, _ = attention_ref(q.detach(), k.detach(), v.detach(), qm, qm, dropout_p=p,
                              dropout_mask=keep.to(DEV), causal=causal, upcast=False, reorder_ops=True)
    _bound("out", out, out_ref, out_pt)


def test_dropout_reproducible_and_fresh():
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 300, 4, 64, device=DEV, dtype=torch.float16) for _ in range(3))
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    off = gen.get_offset()
    o1 = flash_attn_func(q, k, v, 0.3)
    gen.set_offset(off)
    o2 = flash_attn_func(q, k, v, 0.3)
    o3 = flash_attn_func(q, k, v, 0.3)   # next offset: a new mask
    assert torch.equal(o1, o2)
    assert not torch.equal(o1, o3)
