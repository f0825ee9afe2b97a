"""The fused backward preprocessing (knob 8, FLASH_ATTN_MI355X_FUSE_PRE): the assembly dQ kernel
computes D = rowsum(dO o O) itself and writes softmax_d and the dK/dV kernel's [-LSE / scale | -D]
scratch (bwd_pre_kernel's outputs, fa_bwd.hip), then dK/dV runs.  Against the unfused launch
(bwd_pre_kernel -> dK/dV -> dQ): D is the same sum in another order (v_dot2 pairs, fp32), so
softmax_d agrees to fp32 rounding and the gradients to a bf16/fp16 ulp or two."""
import pytest
import torch

from knobs import FUSE_PRE, knob

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _close(a, b, name, tol):
    a, b = a.float(), b.float()
    scale = max(b.abs().max().item(), 1e-6)
    err = (a - b).abs().max().item() / scale
    assert err <= tol, f"{name}: max|diff| / max|ref| = {err:.3e} > {tol}"


def _check(fused, plain, n_rows=None):
    for name, x1, x0, tol in zip(("dq", "dk", "dv"), fused[:3], plain[:3], (1e-2, 1e-2, 1e-2)):
        _close(x1, x0, name, tol)
    d1, d0 = fused[3], plain[3]
    if n_rows is not None:     # varlen: rows past a sequence's length are not written
        d1, d0 = d1[..., :n_rows], d0[..., :n_rows]
    _close(d1, d0, "softmax_d", 1e-5)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
# (4, 4096, 4096, 32, 32): 512 dQ items, twice the CUs, so the persistent dQ loop (knob 6, on by
# default) reloads its fused-D state per item within one workgroup
@pytest.mark.parametrize("b,s,sk,h,hk", [(2, 1024, 1024, 16, 16), (3, 1000, 700, 8, 2), (1, 33, 300, 4, 4),
                                         (2, 4100, 4100, 4, 1), (4, 4096, 4096, 32, 32)])
def test_fused_pre_matches_bwd_pre(b, s, sk, h, hk, dtype, causal):
    from flash_attn.flash_attn_interface import _flash_attn_backward, _flash_attn_forward

    torch.manual_seed(0)
    q = torch.randn(b, s, h, 128, device=DEV, dtype=dtype)
    k = torch.randn(b, sk, hk, 128, device=DEV, dtype=dtype)
    v = torch.randn(b, sk, hk, 128, device=DEV, dtype=dtype)
    do = torch.randn_like(q)
    scale = 128 ** -0.5
    r = _flash_attn_forward(q, k, v, 0.0, scale, causal, False)
    out, lse = r[0], r[5]

    def run():
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        return _flash_attn_backward(do, q, k, v, out, lse, dq, dk, dv, 0.0, scale, causal)

    with knob(FUSE_PRE, 1):
        fused = run()
    with knob(FUSE_PRE, 0):
        plain = run()
    _check(fused, plain, n_rows=s)


@pytest.mark.parametrize("causal", [True, False])
def test_fused_pre_varlen(causal):
    from flash_attn.flash_attn_interface import _flash_attn_varlen_backward, _flash_attn_varlen_forward

    torch.manual_seed(1)
    lens = [1, 300, 4100, 0, 2048, 777, 64, 3000, 255, 256, 257]
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total, h, d = sum(lens), 8, 128
    q, k, v, do = (torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(4))
    scale = d ** -0.5
    mx = max(lens)
    r = _flash_attn_varlen_forward(q, k, v, cu, cu, mx, mx, 0.0, scale, causal, False)
    out, lse = r[0], r[5]

    def run():
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        return _flash_attn_varlen_backward(do, q, k, v, out, lse, dq, dk, dv, cu, cu, mx, mx, 0.0, scale, causal)

    with knob(FUSE_PRE, 1):
        fused = run()
    with knob(FUSE_PRE, 0):
        plain = run()
    for name, x1, x0 in zip(("dq", "dk", "dv"), fused[:3], plain[:3]):
        _close(x1, x0, name, 1e-2)
    for i, n in enumerate(lens):
        if n:
            _close(fused[3][i, :, :n], plain[3][i, :, :n], f"softmax_d[{i}]", 1e-5)
