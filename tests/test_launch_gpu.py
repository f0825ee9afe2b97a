"""GPU tests of the launch path itself: graph capture and bounded device memory.

The assembly kernels compute their work order from the workgroup index (fa_params.h ItemDecode), so
a launch makes no host->device copy and caches nothing per shape (the reference's launch path makes
no copies either, flash_bwd_launch_template.h:49-88).  Checked here:
  * a C3-shaped forward + backward (4 x 8192 x 16 x 128 bf16, causal) captured under
    torch.cuda.graph replays bitwise equal to eager launches, also after new inputs are copied in;
  * a varlen forward + backward (device-built work list, stream-ordered scratch) captured likewise;
  * 20 varlen training steps whose max_seqlen and batch count change every step leave the device
    memory in use after the second pass over the shapes equal to that after the first (no cache grows).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flash_attn_2_cuda  # noqa: F401


def _fwd_bwd(m, q, k, v, do, causal=True):
    scale = q.shape[-1] ** -0.5
    res = m.fwd(q, k, v, None, 0.0, scale, causal, False, None)
    dq, dk, dv = m.bwd(do, q, k, v, res[0], res[5], None, None, None, 0.0, scale, causal, None, res[7])[:3]
    return res[0], res[5], dq, dk, dv


def test_graph_capture_c3_fwd_bwd_bitwise():
    import flash_attn_2_cuda as m

    torch.manual_seed(0)
    b, s, h, d = 4, 8192, 16, 128
    q, k, v, do = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    eager = [x.clone() for x in _fwd_bwd(m, q, k, v, do)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):       # warm-up on a side stream, as torch.cuda.graph wants
        _fwd_bwd(m, q, k, v, do)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = _fwd_bwd(m, q, k, v, do)
    g.replay()
    torch.cuda.synchronize()
    for name, a, e in zip(("out", "lse", "dq", "dk", "dv"), outs, eager):
        assert torch.equal(a, e), name
    # new inputs into the captured buffers
    for x in (q, k, v, do):
        x.copy_(torch.randn_like(x))
    eager2 = [x.clone() for x in _fwd_bwd(m, q, k, v, do)]
    g.replay()
    torch.cuda.synchronize()
    for name, a, e in zip(("out", "lse", "dq", "dk", "dv"), outs, eager2):
        assert torch.equal(a, e), name + " (second inputs)"


def _varlen_step(m, qkv, cu, maxlen, do):
    q, k, v = qkv.unbind(1)
    scale = q.shape[-1] ** -0.5
    res = m.varlen_fwd(q, k, v, None, cu, cu, maxlen, maxlen, 0.0, scale, False, True, False, None)
    grads = m.varlen_bwd(do, q, k, v, res[0], res[5], None, None, None, cu, cu, maxlen, maxlen, 0.0, scale,
                         False, True, None, res[7])[:3]
    return [res[0], res[5]] + list(grads)


def _cu(lens):
    return torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")


def test_graph_capture_varlen_fwd_bwd_bitwise():
    import flash_attn_2_cuda as m

    torch.manual_seed(1)
    lens = [700, 1500, 33, 2048, 512]
    cu = _cu(lens)
    total, h, d = sum(lens), 8, 128
    qkv = torch.randn(total, 3, h, d, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(total, h, d, device="cuda", dtype=torch.bfloat16)
    eager = [x.clone() for x in _varlen_step(m, qkv, cu, max(lens), do)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        _varlen_step(m, qkv, cu, max(lens), do)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = _varlen_step(m, qkv, cu, max(lens), do)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    # softmax_lse is (b, h, max_seqlen): rows past a sequence's length are never written (the
    # reference allocates it with torch::empty as well), so only the written rows are compared
    valid = torch.zeros(len(lens), 1, max(lens), dtype=torch.bool, device="cuda")
    for i, n in enumerate(lens):
        valid[i, :, :n] = True
    for name, a, e in zip(("out", "lse", "dq", "dk", "dv"), outs, eager):
        if name == "lse":
            a, e = a.masked_select(valid), e.masked_select(valid)
        assert torch.equal(a, e), name


def test_varlen_shapes_do_not_grow_device_memory():
    """20 steps, max_seqlen and batch count changing every step (10 shapes, twice): the device
    memory in use after the second pass equals that after the first"""
    import flash_attn_2_cuda as m

    g = torch.Generator().manual_seed(2)
    shapes = []
    for i in range(10):
        nb = 2 + i % 5
        lens = torch.randint(64, 1500 + 300 * i, (nb,), generator=g).tolist()
        shapes.append(lens)
    h, d = 8, 128

    def one_pass():
        for lens in shapes:
            total = sum(lens)
            qkv = torch.randn(total, 3, h, d, device="cuda", dtype=torch.bfloat16)
            do = torch.randn(total, h, d, device="cuda", dtype=torch.bfloat16)
            outs = _varlen_step(m, qkv, _cu(lens), max(lens), do)
            assert all(torch.isfinite(x.float()).all() for i, x in enumerate(outs) if i != 1)   # (lse: unwritten tail)
            del outs, qkv, do
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        free, total_mem = torch.cuda.mem_get_info()
        return total_mem - free

    used1 = one_pass()
    used2 = one_pass()
    assert used2 <= used1, (used1, used2)
