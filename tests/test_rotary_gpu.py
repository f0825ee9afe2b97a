"""GPU tests of the rotary embedding kernel (reference flash_attn/layers/rotary.py,
csrc/rotary/rotary_cuda.cu:9-45) against the reference's plain-torch formula in fp32
(``apply_rotary_emb_torch``, rotary.py:22-32): the kernel computes in fp32 and rounds once, so it
must match the fp32 formula rounded to the input dtype within one unit of that dtype; gradients
(the conj path) against torch autograd of the same formula."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _ulp(dtype):
    return 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10


def _cos_sin(seqlen, rd, dtype, offset=0):
    inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, device=DEV, dtype=torch.float32) / rd))
    f = torch.outer(torch.arange(seqlen + offset, device=DEV, dtype=torch.float32), inv)
    return torch.cos(f).to(dtype), torch.sin(f).to(dtype)


def _close(got, want, dtype):
    # one rounding of a value of magnitude |want|: |err| <= ulp * max(1, |want|)
    err = (got.float() - want.float()).abs()
    tol = _ulp(dtype) * torch.clamp(want.float().abs(), min=1.0)
    assert (err <= tol).all(), float((err - tol).max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("interleaved", [False, True])
@pytest.mark.parametrize("rd,d", [(64, 64), (32, 128), (128, 128), (16, 80)])
@pytest.mark.parametrize("inplace", [False, True])
def test_apply_rotary_emb_func(rd, d, interleaved, inplace, dtype):
    from flash_attn.layers.rotary import apply_rotary_emb_func, apply_rotary_emb_torch

    torch.manual_seed(0)
    b, s, h = 2, 217, 3
    x = torch.randn(b, s, h, d, device=DEV, dtype=dtype)
    cos, sin = _cos_sin(s + 5, rd, dtype)       # the cache may be longer than the sequence
    xr = x.detach().clone().float().requires_grad_()
    ref = apply_rotary_emb_torch(xr, cos[:s].float(), sin[:s].float(), interleaved)
    xi = x.clone().requires_grad_() if not inplace else x.clone()
    if inplace:
        out = apply_rotary_emb_func(xi, cos, sin, interleaved, True)
        assert out.data_ptr() == xi.data_ptr()
    else:
        out = apply_rotary_emb_func(xi, cos, sin, interleaved, False)
    _close(out, ref, dtype)
    assert torch.equal(out[..., rd:], x[..., rd:])
    if not inplace:
        g = torch.randn_like(out)
        (gx,) = torch.autograd.grad(out, xi, g)
        (gr,) = torch.autograd.grad(ref, xr, g.float())
        _close(gx, gr, dtype)


@pytest.mark.parametrize("interleaved", [False, True])
@pytest.mark.parametrize("xpos", [False, True])
def test_rotary_embedding_module_qkv_and_kv(interleaved, xpos):
    from flash_attn.layers.rotary import RotaryEmbedding, apply_rotary_emb_torch

    torch.manual_seed(0)
    dtype = torch.bfloat16
    b, s, h, d, rd = 2, 130, 4, 64, 32
    emb = RotaryEmbedding(rd, interleaved=interleaved, scale_base=512 if xpos else None, device=DEV)
    qkv = torch.randn(b, s, 3, h, d, device=DEV, dtype=dtype)
    out = emb(qkv.clone(), seqlen_offset=3)
    cos, sin = emb._cos_cached[3:3 + s].float(), emb._sin_cached[3:3 + s].float()
    ck = emb._cos_k_cached[3:3 + s].float() if xpos else cos
    sk = emb._sin_k_cached[3:3 + s].float() if xpos else sin
    _close(out[:, :, 0], apply_rotary_emb_torch(qkv[:, :, 0].float(), cos, sin, interleaved), dtype)
    _close(out[:, :, 1], apply_rotary_emb_torch(qkv[:, :, 1].float(), ck, sk, interleaved), dtype)
    assert torch.equal(out[:, :, 2], qkv[:, :, 2])
    # q + packed kv form (the MQA / GQA path of MHA)
    q = torch.randn(b, s, h, d, device=DEV, dtype=dtype)
    kv = torch.randn(b, s, 2, 2, d, device=DEV, dtype=dtype)
    q2, kv2 = emb(q.clone(), kv.clone())
    cos, sin = emb._cos_cached[:s].float(), emb._sin_cached[:s].float()
    ck = emb._cos_k_cached[:s].float() if xpos else cos
    sk = emb._sin_k_cached[:s].float() if xpos else sin
    _close(q2, apply_rotary_emb_torch(q.float(), cos, sin, interleaved), dtype)
    _close(kv2[:, :, 0], apply_rotary_emb_torch(kv[:, :, 0].float(), ck, sk, interleaved), dtype)
    assert torch.equal(kv2[:, :, 1], kv[:, :, 1])


@pytest.mark.parametrize("num_heads_kv", [8, 2])
def test_mha_with_rotary_trains(num_heads_kv):
    from flash_attn.layers.rotary import apply_rotary_emb_torch
    from flash_attn.modules.mha import MHA
    from oracle.attention_ref import attention_ref, check_within_bound

    torch.manual_seed(0)
    E, H, S = 512, 8, 190
    mha = MHA(E, H, num_heads_kv=num_heads_kv, causal=True, rotary_emb_dim=32, device=DEV,
              dtype=torch.bfloat16)
    x = torch.randn(2, S, E, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = mha(x)
    y.float().pow(2).mean().backward()
    assert torch.isfinite(x.grad).all() and torch.isfinite(mha.Wqkv.weight.grad).all()
    with torch.no_grad():
        d = E // H
        qkv = mha.Wqkv(x)
        q = qkv[..., : H * d].reshape(2, S, H, d)
        kv = qkv[..., H * d:].reshape(2, S, 2, num_heads_kv, d)
        cos, sin = mha.rotary_emb._cos_cached[:S].float(), mha.rotary_emb._sin_cached[:S].float()
        q2, kv2 = mha.rotary_emb(q.clone(), kv.clone())
        _close(q2, apply_rotary_emb_torch(q.float(), cos, sin), torch.bfloat16)
        _close(kv2[:, :, 0], apply_rotary_emb_torch(kv[:, :, 0].float(), cos, sin), torch.bfloat16)
        ref, _ = attention_ref(q2, kv2[:, :, 0], kv2[:, :, 1], causal=True)
        pt, _ = attention_ref(q2, kv2[:, :, 0], kv2[:, :, 1], causal=True, upcast=False, reorder_ops=True)
        core = mha.inner_cross_attn(q2, kv2)
        ok, err, bound = check_within_bound(core, ref, pt)
        assert ok, (err, bound)
        assert torch.equal(y, mha.out_proj(core.reshape(2, S, E)))
