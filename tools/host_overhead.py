import sys, time, cProfile, pstats, io
sys.path.insert(0, "xhy-flash-attention_amd")
import torch
from flash_attn import flash_attn_func
q = torch.randn(1, 128, 4, 64, device="cuda", dtype=torch.bfloat16)
k = torch.randn_like(q); v = torch.randn_like(q)
with torch.no_grad():
    for _ in range(50): flash_attn_func(q, k, v, causal=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2000): flash_attn_func(q, k, v, causal=True)
    torch.cuda.synchronize()
    print(f"no_grad fwd: {(time.perf_counter() - t) / 2000 * 1e6:.1f} us per call")
    pr = cProfile.Profile(); pr.enable()
    for _ in range(2000): flash_attn_func(q, k, v, causal=True)
    pr.disable()
    s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18); print(s.getvalue()[:4000])
