"""GPU parity of calc_reduced_attn_scores (reference
csrc/flash_attn/src/calc_reduced_attn_scores_kernel.h:119-307, C ABI csrc/capi/flash_attn.cu:1107-1201):
reduced[b][h][k] = sum_q exp(scale q.k - LSE[q]) and, with return_softmax, the probabilities.
The oracle is the same formula in float64 on the kernel's inputs (LSE from the oracle as well, so the
kernel is checked in isolation); fp32 accumulation over up to 1000 queries -> rtol 2e-3."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _bind():
    import flash_attn_2_cuda as m

    f = m._lib.calc_reduced_attn_scores
    P, I, F, B = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool
    f.argtypes = [P] * 5 + [I] * 6 + [F, B, B, I, P] + [I] * 9
    f.restype = B
    return m, f


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("d,sq,sk,h,hk", [(64, 300, 257, 4, 4), (128, 1000, 130, 4, 2), (256, 97, 300, 2, 1),
                                          (40, 64, 64, 3, 3)])
@pytest.mark.parametrize("return_softmax", [False, True])
def test_reduced_attn_scores(return_softmax, d, sq, sk, h, hk, dtype):
    m, f = _bind()
    torch.manual_seed(0)
    b = 2
    q = torch.randn(b, sq, h, d, device=DEV, dtype=dtype)
    k = torch.randn(b, sk, hk, d, device=DEV, dtype=dtype)
    scale = d ** -0.5
    s64 = torch.einsum("bqhd,bkhd->bhqk", q.double(), k.double().repeat_interleave(h // hk, dim=2)) * scale
    lse = torch.logsumexp(s64, dim=-1).float()                       # (b, h, sq)
    p64 = torch.exp(s64 - lse.double()[..., None])
    reduced = torch.full((b, h, sk), float("nan"), device=DEV)       # written, not accumulated
    probs = torch.empty(b, h, sq, sk, device=DEV) if return_softmax else None
    P = m._ptr
    ok = f(P(q), P(k), P(lse), P(reduced), P(probs), b, sq, sk, h, hk, d, scale, return_softmax,
           dtype == torch.bfloat16, 1, m._stream(q),
           q.stride(1), k.stride(1), q.stride(1), q.stride(2), k.stride(2), q.stride(2),
           q.stride(0), k.stride(0), q.stride(0))
    assert ok, m._lib.flash_attn_error()
    torch.cuda.synchronize()
    torch.testing.assert_close(reduced.double(), p64.sum(2), rtol=2e-3, atol=1e-5)
    if return_softmax:
        torch.testing.assert_close(probs.double(), p64, rtol=2e-3, atol=1e-5)
