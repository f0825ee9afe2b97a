import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "xhy-flash-attention_amd")]
from flash_attn import flash_attn_func
torch.manual_seed(0)
for (s, d, causal) in [(64, 64, False), (128, 128, False), (300, 128, False), (300, 128, True)]:
    q, k, v = (torch.randn(1, s, 1, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    out, lse, _ = flash_attn_func(q, k, v, causal=causal, return_attn_probs=True)
    S = (q[0, :, 0].float() @ k[0, :, 0].float().T) * d ** -0.5
    if causal:
        S = S.masked_fill(torch.triu(torch.ones(s, s, dtype=torch.bool, device="cuda"), 1), float("-inf"))
    ref_lse = torch.logsumexp(S, -1)
    ref = torch.softmax(S, -1) @ v[0, :, 0].float()
    e = (out[0, :, 0].float() - ref).abs().max(-1).values
    el = (lse[0, 0] - ref_lse).abs()
    bad = (e > 0.05).nonzero().flatten().tolist()
    print(s, d, causal, "max out err", e.max().item(), "max lse err", el.max().item(), "bad rows", bad[:20], len(bad))
    print("  lse got", lse[0, 0, :6].tolist(), "ref", ref_lse[:6].tolist())
