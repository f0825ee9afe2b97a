"""GPU tests of the attention modules (reference flash_attn/modules/mha.py:35-142):
FlashSelfAttention / FlashCrossAttention must be exactly the functional calls they wrap, and MHA's
attention core must meet the reference's 2x rule against the oracle on its own projections."""
import pytest
import torch

from oracle.attention_ref import attention_ref, check_within_bound

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


@pytest.mark.parametrize("causal", [False, True])
def test_flash_self_attention_is_the_functional_call(causal):
    from flash_attn import flash_attn_qkvpacked_func, flash_attn_varlen_qkvpacked_func
    from flash_attn.modules.mha import FlashSelfAttention

    torch.manual_seed(0)
    qkv = torch.randn(2, 300, 3, 4, 64, device=DEV, dtype=torch.bfloat16)
    m = FlashSelfAttention(causal=causal, attention_dropout=0.3).eval()
    assert torch.equal(m(qkv), flash_attn_qkvpacked_func(qkv, 0.0, causal=causal))
    cu = torch.tensor([0, 100, 300], device=DEV, dtype=torch.int32)
    flat = qkv.reshape(600, 3, 4, 64)[:300]
    assert torch.equal(m(flat, cu_seqlens=cu, max_seqlen=200),
                       flash_attn_varlen_qkvpacked_func(flat, cu, 200, 0.0, causal=causal))


@pytest.mark.parametrize("causal", [False, True])
def test_flash_cross_attention_matches_oracle(causal):
    from flash_attn.modules.mha import FlashCrossAttention

    torch.manual_seed(0)
    q = torch.randn(2, 200, 6, 128, device=DEV, dtype=torch.float16)
    kv = torch.randn(2, 333, 2, 3, 128, device=DEV, dtype=torch.float16)
    out = FlashCrossAttention(causal=causal)(q, kv)
    ref, _ = attention_ref(q, kv[:, :, 0], kv[:, :, 1], causal=causal)
    pt, _ = attention_ref(q, kv[:, :, 0], kv[:, :, 1], causal=causal, upcast=False, reorder_ops=True)
    ok, err, bound = check_within_bound(out, ref, pt)
    assert ok, (err, bound)


@pytest.mark.parametrize("num_heads_kv", [8, 2])
@pytest.mark.parametrize("causal", [False, True])
def test_mha_attention_core_and_grads(num_heads_kv, causal):
    from flash_attn.modules.mha import MHA

    torch.manual_seed(0)
    E, H = 512, 8
    mha = MHA(E, H, num_heads_kv=num_heads_kv, causal=causal, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2, 257, E, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = mha(x)
    y.float().pow(2).mean().backward()
    assert torch.isfinite(x.grad).all() and torch.isfinite(mha.Wqkv.weight.grad).all()
    # the attention core against the oracle, on the module's own projections
    with torch.no_grad():
        d = E // H
        qkv = mha.Wqkv(x)
        q = qkv[..., : H * d].reshape(2, 257, H, d)
        kv = qkv[..., H * d:].reshape(2, 257, 2, num_heads_kv, d)
        ref, _ = attention_ref(q, kv[:, :, 0], kv[:, :, 1], causal=causal)
        pt, _ = attention_ref(q, kv[:, :, 0], kv[:, :, 1], causal=causal, upcast=False, reorder_ops=True)
        ctx = mha.inner_cross_attn(q, kv) if num_heads_kv != H else mha.inner_attn(qkv.view(2, 257, 3, H, d))
        ok, err, bound = check_within_bound(ctx, ref, pt)
        assert ok, (err, bound)
        assert torch.equal(y, mha.out_proj(ctx.reshape(2, 257, E)))


def test_mha_key_padding_mask_is_varlen():
    from flash_attn.modules.mha import MHA

    torch.manual_seed(0)
    mha = MHA(256, 4, causal=True, device=DEV, dtype=torch.float16).eval()
    x = torch.randn(3, 96, 256, device=DEV, dtype=torch.float16)
    mask = torch.arange(96, device=DEV)[None, :] < torch.tensor([96, 50, 7], device=DEV)[:, None]
    y = mha(x, key_padding_mask=mask)
    for i, n in enumerate((96, 50, 7)):
        yi = mha(x[i:i + 1, :n])
        torch.testing.assert_close(y[i:i + 1, :n], yi, atol=2e-3, rtol=0)
        assert (y[i, n:] == 0).all()
