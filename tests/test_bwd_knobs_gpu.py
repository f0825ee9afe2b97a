"""The backward's launch switches against the oracle: the fused preprocessing
(knob 8: D = rowsum(dO o O) and the dK/dV chain starts computed inside the assembly dQ kernel,
reference compute_dot_do_o, flash_bwd_kernel.h:112-188) and the persistent item loops (knob 6) each
run under the reference's 2x rule (tests/test_flash_attn.py:630-639) in both settings, so the fused
D path keeps oracle coverage whatever the defaults are.  A C3-class fixed-length case and a varlen
case with ragged sequences; d = 128 and 64 (the assembly backward's domain: gen_bwd / gen_dq and,
since round 6, gen_bwd64 / gen_dq64)."""
import pytest
import torch

from knobs import BWD_PERSIST, FUSE_PRE, VARLEN_ROUNDS, knob
from oracle.attention_ref import attention_ref, check_within_bound

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _bound(name, got, ref, pt):
    ok, err, bound = check_within_bound(got.float(), ref.float(), pt.float())
    assert ok, f"{name}: max|err| {err:.3e} > bound {bound:.3e}"


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("persist", [0, 1])
@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("causal", [True, False])
def test_fixed_length_2x_rule(fuse, persist, causal, d):
    """C3-class (bf16, 2 x 2048 x 16 heads: 256 dK/dV items at d 128, more than the CUs, so the
    persistent loops run several rounds)"""
    from flash_attn import flash_attn_func

    torch.manual_seed(0)
    b, s, h = 2, 2048, 16
    q, k, v = (torch.randn(b, s, h, d, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    out = flash_attn_func(q, k, v, causal=causal)
    g = torch.randn_like(out)
    with knob(FUSE_PRE, fuse), knob(BWD_PERSIST, persist):
        dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
    qr, kr, vr = (x.detach().clone().requires_grad_() for x in (q, k, v))
    ref, _ = attention_ref(qr, kr, vr, causal=causal)
    gr = torch.autograd.grad(ref, (qr, kr, vr), g)
    qp, kp, vp = (x.detach().clone().requires_grad_() for x in (q, k, v))
    pt, _ = attention_ref(qp, kp, vp, causal=causal, upcast=False, reorder_ops=True)
    gp = torch.autograd.grad(pt, (qp, kp, vp), g)
    _bound("out", out, ref, pt)
    for name, got, r, p in zip(("dq", "dk", "dv"), (dq, dk, dv), gr, gp):
        _bound(name, got, r, p)


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("causal", [True, False])
def test_varlen_2x_rule(fuse, causal, d):
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(1)
    lens = [1, 300, 1500, 0, 777, 64, 255, 256, 257]
    h = 4
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total = sum(lens)
    q, k, v = (torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    out = flash_attn_varlen_func(q, k, v, cu, cu, max(lens), max(lens), causal=causal)
    g = torch.randn_like(out)
    with knob(FUSE_PRE, fuse):
        dq, dk, dv = torch.autograd.grad(out, (q, k, v), g)
    # the reference's varlen test applies the rule to the whole packed tensors (test_flash_attn.py:774-783)
    refs = {x: torch.zeros(total, h, d, device=DEV) for x in ("out", "dq", "dk", "dv")}
    pts = {x: torch.zeros(total, h, d, device=DEV) for x in ("out", "dq", "dk", "dv")}
    for i, n in enumerate(lens):
        if n == 0:
            continue
        a, e = int(cu[i]), int(cu[i + 1])
        qs, ks, vs = (x.detach()[a:e].unsqueeze(0) for x in (q, k, v))
        gs = g[a:e].unsqueeze(0)
        for upcast, dst in ((True, refs), (False, pts)):
            qr, kr, vr = (x.clone().requires_grad_() for x in (qs, ks, vs))
            o, _ = attention_ref(qr, kr, vr, causal=causal, upcast=upcast, reorder_ops=not upcast)
            gr = torch.autograd.grad(o, (qr, kr, vr), gs)
            for name, t in zip(("out", "dq", "dk", "dv"), (o,) + tuple(gr)):
                dst[name][a:e] = t[0].float()
    for name, got in (("out", out), ("dq", dq), ("dk", dk), ("dv", dv)):
        _bound(name, got, refs[name], pts[name])


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("hk", [4, 1])
def test_varlen_rounds_bitwise(causal, hk):
    """knob 9 (items per dK/dV workgroup on varlen launches, snake-paired rounds) and knob 6 = 2 (the
    persistent loop over the device-built work list): the same per-item arithmetic in any work
    order, so dK / dV are bitwise those of one workgroup per item -- for items without keys (an
    empty sequence, blocks past a sequence's end) and GQA reduced in the kernel as well"""
    from flash_attn import flash_attn_varlen_func

    torch.manual_seed(2)
    lens = [700, 0, 130, 2100, 64, 1025, 9]
    h, d = 4, 128
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total = sum(lens)
    q = torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k, v = (torch.randn(total, hk, d, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(2))
    out = flash_attn_varlen_func(q, k, v, cu, cu, max(lens), max(lens), causal=causal)
    g = torch.randn_like(out)
    res = {}
    for rounds, persist in ((1, 1), (2, 1), (3, 1), (1, 2)):
        with knob(VARLEN_ROUNDS, rounds), knob(BWD_PERSIST, persist):
            res[(rounds, persist)] = torch.autograd.grad(out, (q, k, v), g, retain_graph=True)
    base = res[(1, 1)]
    for key, grads in res.items():
        for name, x, y in zip(("dq", "dk", "dv"), grads, base):
            assert torch.equal(x, y), (key, name, (x.float() - y.float()).abs().max().item())


@pytest.mark.parametrize("case", [
    dict(b=2, s=2048, h=16, hk=16, causal=True, dt=torch.bfloat16),        # persistent, several rounds
    dict(b=1, s=1000, h=8, hk=2, causal=False, dt=torch.float16),          # GQA reduced, ragged
    dict(b=3, s=77, h=4, hk=1, causal=True, dt=torch.bfloat16),            # one subtile pair, MQA
    dict(b=1, s=4096 + 33, h=4, hk=4, causal=True, dt=torch.float16),      # long, ragged tail
    dict(lens=[1, 300, 0, 1023, 64], h=8, hk=4, causal=True, dt=torch.bfloat16),   # varlen
], ids=["c3class", "gqa_full", "mqa_short", "long_ragged", "varlen"])
def test_two_waves_per_simd_bitwise(case):
    """knob 10: the dK/dV kernel with two waves per SIMD (gen_bwd2.py: 8 waves specialised by role, P
    crossing between them in LDS) against the one-wave kernel (gen_bwd.py): the same MFMA chains in
    the same order, so dQ / dK / dV are bitwise equal; and under the 2x rule against the oracle."""
    from flash_attn import flash_attn_func, flash_attn_varlen_func
    from knobs import BWD_2W

    torch.manual_seed(7)
    dt, h, hk, causal = case["dt"], case["h"], case["hk"], case["causal"]
    d = 128
    if "lens" in case:
        lens = case["lens"]
        cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
        tot, mx = sum(lens), max(lens)
        q = torch.randn(tot, h, d, device=DEV, dtype=dt, requires_grad=True)
        k, v = (torch.randn(tot, hk, d, device=DEV, dtype=dt, requires_grad=True) for _ in range(2))
        out = flash_attn_varlen_func(q, k, v, cu, cu, mx, mx, causal=causal)
    else:
        b, s = case["b"], case["s"]
        q = torch.randn(b, s, h, d, device=DEV, dtype=dt, requires_grad=True)
        k, v = (torch.randn(b, s, hk, d, device=DEV, dtype=dt, requires_grad=True) for _ in range(2))
        out = flash_attn_func(q, k, v, causal=causal)
    g = torch.randn_like(out)
    res = []
    for two in (0, 1):
        with knob(BWD_2W, two):
            res.append(torch.autograd.grad(out, (q, k, v), g, retain_graph=True))
    for name, a, bb in zip(("dq", "dk", "dv"), *res):
        assert torch.equal(a, bb), name
    if "lens" in case:
        return
    qr, kr, vr = (x.detach().clone().requires_grad_() for x in (q, k, v))
    ref, _ = attention_ref(qr, kr, vr, causal=causal)
    gr = torch.autograd.grad(ref, (qr, kr, vr), g)
    qp, kp, vp = (x.detach().clone().requires_grad_() for x in (q, k, v))
    pt, _ = attention_ref(qp, kp, vp, causal=causal, upcast=False, reorder_ops=True)
    gp = torch.autograd.grad(pt, (qp, kp, vp), g)
    for name, got, r, p in zip(("dq", "dk", "dv"), res[1], gr, gp):
        ok, err, bound = check_within_bound(got.float(), r.float(), p.float(), floor=1e-4)
        assert ok, f"{name}: max|err| {err:.3e} > bound {bound:.3e}"


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("causal", [True, False])
def test_forward_varlen_rounds_bitwise(causal, d):
    """knob 11 (items per workgroup of the assembly forward on varlen calls, snake-paired rounds over
    the decoded order): the same per-item arithmetic in any work order, so out and LSE are bitwise
    those of one workgroup per item -- empty sequences and blocks past a sequence's end included"""
    import flash_attn_2_cuda as m
    from knobs import FWD_VARLEN_ROUNDS

    torch.manual_seed(3)
    lens = [700, 0, 130, 2100, 64, 1025, 9, 3000, 1]
    h = 8
    cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(DEV)
    total = sum(lens)
    q, k, v = (torch.randn(total, h, d, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    res = {}
    for rounds in (1, 2, 3):
        with knob(FWD_VARLEN_ROUNDS, rounds):
            r = m.varlen_fwd(q, k, v, None, cu, cu, max(lens), max(lens), 0.0, d ** -0.5, False, causal, False, None)
        res[rounds] = (r[0].clone(), r[5].clone())
    for rounds, (o, lse) in res.items():
        assert torch.equal(o, res[1][0]), rounds
        for i, n in enumerate(lens):     # (LSE rows past a sequence's length are not written)
            assert torch.equal(lse[i, :, :n], res[1][1][i, :, :n]), (rounds, i)
