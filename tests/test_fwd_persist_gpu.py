"""The persistent assembly forward (knob 5, fa_fwd_asm.cpp) against its one-workgroup-per-item
launch: every item is computed by the same instruction sequence whichever workgroup runs it and
whether its tiles were prefetched by a predecessor (warm) or not (cold), so out and LSE must agree
bit for bit.  Shapes with more items than CUs (persistent grid), head dims 128 / 64, causal or
not, GQA, ragged lengths (cold successors), varlen (device-built work list)."""
import pytest
import torch

from knobs import FWD_PERSIST, knob

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _both(fn):
    with knob(FWD_PERSIST, 1):
        a = fn()
    with knob(FWD_PERSIST, 0):
        b = fn()
    return a, b


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("b,s,sk,h,hk", [(4, 2048, 2048, 32, 8), (3, 1000, 1000, 40, 40), (2, 700, 130, 64, 16)])
def test_persistent_forward_bitwise(b, s, sk, h, hk, dtype, causal, d):
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    q = torch.randn(b, s, h, d, device=DEV, dtype=dtype)
    k = torch.randn(b, sk, hk, d, device=DEV, dtype=dtype)
    v = torch.randn(b, sk, hk, d, device=DEV, dtype=dtype)
    (o1, l1, _), (o0, l0, _) = _both(lambda: flash_attn_func(q, k, v, causal=causal, return_attn_probs=True))
    assert torch.equal(o1, o0)
    assert torch.equal(l1, l0)


@pytest.mark.parametrize("d", [128, 64])
def test_persistent_forward_varlen_bitwise(d):
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(0)
    lens = [1, 300, 4100, 0, 2048, 777, 64, 3000, 1500, 255, 256, 257] * 3
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total, h = sum(lens), 16
    q, k, v = (torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    (o1, l1, _), (o0, l0, _) = _both(lambda: flash_attn_varlen_func(
        q, k, v, cu, cu, max(lens), max(lens), causal=True, return_attn_probs=True))
    assert torch.equal(o1, o0)
    for i, n in enumerate(lens):     # LSE rows past a sequence's length are not written
        assert torch.equal(l1[i, :, :n], l0[i, :, :n])


@pytest.mark.parametrize("nseq", [3000, 5000])
def test_persistent_forward_many_sequences(nseq):
    """thousands of short sequences: the device-built list (3000; its shared memory holds 2 ints per
    sequence) and, past the builder's limit (5000), the host table with one workgroup per item"""
    from flash_attn import flash_attn_varlen_func

    g = torch.Generator().manual_seed(nseq)
    lens = torch.randint(1, 300, (nseq,), generator=g).tolist()
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total, h, d = sum(lens), 2, 64
    torch.manual_seed(0)
    q, k, v = (torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    (o1, l1, _), (o0, l0, _) = _both(lambda: flash_attn_varlen_func(
        q, k, v, cu, cu, max(lens), max(lens), causal=True, return_attn_probs=True))
    assert torch.equal(o1, o0)
    n = torch.tensor(lens, device=DEV)
    valid = torch.arange(l1.shape[-1], device=DEV)[None, None, :] < n[:, None, None]
    assert torch.equal(l1[valid.expand_as(l1)], l0[valid.expand_as(l0)])
