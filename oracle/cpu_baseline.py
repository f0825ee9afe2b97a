"""ORACLE -- test / measurement infrastructure only (imported by bench.py's cpu_baseline leg).

The reference's own CPU-capable path for this workload is PyTorch's
``torch.nn.functional.scaled_dot_product_attention`` on the host CPU (``north_star``; SURVEY
§8(d) "CPU baseline"), which tests/test_oracle.py pins against the reference's ``attention_ref``
(tests/test_flash_attn.py:111-159).  This module times it on a bounded sample of a GPU workload.
"""
import os
import time

import torch

__all__ = ["sdpa_fwd_bwd_tflops", "cpu_model_name"]


def cpu_model_name() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def sdpa_fwd_bwd_tflops(batch, seqlen, nheads, headdim, causal, dtype, threads, repeats=3,
                        flops_fn=None, fwd_only=False):
    """Times fwd+bwd (or the forward alone) of CPU SDPA (1 warm-up + `repeats`), returns
    (tflops, seconds_per_rep)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        q, k, v = (torch.randn(batch, nheads, seqlen, headdim, generator=g).to(dtype).requires_grad_()
                   for _ in range(3))
        dout = torch.randn(batch, nheads, seqlen, headdim, generator=g).to(dtype)

        def step():
            if fwd_only:
                with torch.no_grad():
                    torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)
                return
            out = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)
            torch.autograd.grad(out, (q, k, v), dout)

        step()
        t0 = time.perf_counter()
        for _ in range(repeats):
            step()
        dt = (time.perf_counter() - t0) / repeats
    finally:
        torch.set_num_threads(prev)
    flops = flops_fn(batch) if flops_fn else 0.0
    return flops / dt / 1e12, dt


if __name__ == "__main__":
    n = min(16, os.cpu_count() or 1)
    print(sdpa_fwd_bwd_tflops(1, 2048, 4, 128, True, torch.bfloat16, n,
                              flops_fn=lambda b: 3.5 * 4 * b * 2048 ** 2 * 4 * 128 / 2))
