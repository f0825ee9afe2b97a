#!/usr/bin/env python3
"""Headline benchmark: attention TFLOPS (fwd, fwd+bwd) at seqlen 8k, hdim 128, causal.

One "step" = one forward + backward of ``flash_attn_func`` on the C3 workload
(batch 4 x seqlen 8192 x 16 heads x hdim 128, bf16, causal; BASELINE.json configs[2]) with the
inputs already resident in HBM.  FLOPs follow the reference's convention
(benchmarks/benchmark_flash_attention.py:27-30): F_fwd = 4 b s^2 h d / 2 (causal),
F_bwd = 2.5 F_fwd, F_fwd+bwd = 3.5 F_fwd.  Other workloads (``--workload``): c2 (forward only,
configs[1]), c4 (varlen qkvpacked, total 65536 tokens, configs[3]), c5 (fp16 GQA 32k, configs[4]).

Multi-GPU: one process per GPU.  Under ``torch.distributed.run`` the ranks come from the
environment; ``python bench.py --gpus N`` with no WORLD_SIZE starts the N rank processes itself
(children, before any GPU call in the parent) and exits with their status.  Every rank runs the
same per-GPU batch (weak scaling, batch-sharded, no collective on the data path); a barrier +
synchronize bracket the timed region on every rank and the MAX elapsed time over ranks is reduced
with one all-reduce after the region.  ``value`` = total FLOPs of all ranks / that max time.

Also reported: live per-kernel device time from HIP events recorded on the launch stream by the
library (``flash_attn_timing_*``, over the timed steps only), the roofline of the dominant kernel
against the 2516.6 TF dense bf16 MFMA peak, rocprof PMC figures (MFMA utilisation, HBM bytes) from
the committed profile of the same command (profiles/pmc.json), and the reference's CPU path (torch
SDPA) timed on this host on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "xhy-flash-attention_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "attention TFLOPS/GPU (fwd, fwd+bwd) at seqlen 8k hdim 128 causal"
PEAK_TFLOPS = 2516.6          # 256 CU x 4 SIMD x 1024 bf16/f16 MFMA FLOP/clk x 2.4 GHz (dense)
PEAK_HBM_GBPS = 8000.0        # HBM3E spec (MI355X_MICROARCH.md)
H100_FWD_BWD_TFLOPS = 308.0   # FA2 fwd+bwd, causal, hdim128, s=8k, H100 SXM5
KERNELS = {0: "fwd_kernel", 1: "bwd_pre_kernel", 2: "bwd_dkdv_kernel", 3: "bwd_dq_kernel",
           4: "bwd_dkdv_dq_window", 5: "bwd_qfold_kernel"}   # 4: from the dK/dV launch to the end of dQ (they overlap, two streams)
# algorithmic flops of each kernel in units of F_fwd (the atomic-free backward recomputes S and dP
# in both kernels: dK/dV = S, dP, dV, dK GEMMs; dQ = S, dP, dQ GEMMs)
KERNEL_FLOP_FACTOR = {"fwd_kernel": 1.0, "bwd_dkdv_kernel": 2.0, "bwd_dq_kernel": 1.5}

WORKLOADS = {
    # name: (batch per GPU, seqlen, nheads, nheads_k, headdim, dtype, causal, kind)
    "c2": (4, 2048, 16, 16, 64, "bf16", True, "fwd"),          # configs[1]: forward only
    "c3": (4, 8192, 16, 16, 128, "bf16", True, "fwd_bwd"),     # configs[2]: headline
    "c4": (None, 65536, 32, 32, 128, "bf16", True, "varlen"),  # configs[3]: total tokens
    "c5": (8, 32768, 32, 8, 128, "fp16", True, "fwd_bwd"),     # configs[4]: 8 per GPU
    # dev shapes (not BASELINE configs): head dim 64 at the C3 length, causal and not
    "d64": (4, 8192, 32, 32, 64, "bf16", True, "fwd_bwd"),
    "d64nc": (4, 8192, 32, 32, 64, "bf16", False, "fwd_bwd"),
}


def flops_fwd(b, s, h, d, causal):
    return 4.0 * b * s * s * h * d / (2.0 if causal else 1.0)


def c4_seqlens(total=65536, lo=512, hi=4096, seed=0):
    """SURVEY.md 8(d) C4 recipe: torch.manual_seed(0); draw s_i ~ U{lo..hi} until the sum reaches
    `total`, then clip the last length so that the sum is exactly `total`."""
    import torch

    g = torch.Generator().manual_seed(seed)
    lens, acc = [], 0
    while acc < total:
        s = int(torch.randint(lo, hi + 1, (1,), generator=g).item())
        s = min(s, total - acc)
        lens.append(s)
        acc += s
    return lens


def varlen_flops_fwd(lens, h, d, causal):
    return sum(4.0 * s * s * h * d / (2.0 if causal else 1.0) for s in lens)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ramp-s", type=float, default=0.5,
                    help="untimed seconds of headline steps before either leg (clock / allocator ramp)")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="dropout_p of every call (dev lines: the dropout training path; 0 = the BASELINE configs)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: the affinity set, capped by OMP_NUM_THREADS)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc.json"),
                    help="JSON with rocprof PMC figures per workload and kernel (profiles/pmc.py)")
    ap.add_argument("--rank-timeout", type=float, default=None,
                    help="--gpus N launcher: seconds before every rank is terminated and the launcher exits "
                         "non-zero (default 900 + 5 s per warm-up / timed step)")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness only (gloo, CPU sleep as the step): tests the launcher and timing")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------
# launcher: --gpus N without an external torch.distributed.run
# ------------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, timeout=None):
    """Start n child processes of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
    (the parent has made no GPU call), wait for all, return the worst exit status.  A rank that
    fails ends the others (they would wait at the barrier forever)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0 = time.time()
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad or (timeout and time.time() - t0 > timeout):
                rc = bad[0].returncode if bad else 124
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for p in procs:
        code = p.returncode
        if code != 0:
            rc = rc or (code if code > 0 else 128 - code)
    return rc


# ------------------------------------------------------------------------------------------------
# harness (shared with tests/test_bench_dist.py)
# ------------------------------------------------------------------------------------------------
def dist_init(dry_run=False):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if dry_run:
            dist.init_process_group(backend="gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
        rank = dist.get_rank()
    elif not dry_run:
        torch.cuda.set_device(0)
    return rank, local, world


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world, device=None):
    """MAX of a per-rank float over the job (one all-reduce outside the timed region)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    if device is None:
        device = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(step, steps, warmup, world, sync=None, on_start=None, on_stop=None, step_ms=None):
    """W untimed steps, then EXACTLY `steps` steps bracketed by barrier + synchronize on every
    rank; returns the MAX elapsed seconds over ranks.  on_start / on_stop run right inside the
    bracket (the kernel timer: its windows then cover the timed steps only).  `step_ms` (a list)
    receives this rank's per-step device times from events recorded between the steps on the
    current stream (median and min next to the mean)."""
    if sync is None:
        import torch
        sync = torch.cuda.synchronize
    for _ in range(warmup):
        step()
    barrier(world)
    sync()
    ev = None
    if step_ms is not None:
        import torch
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    if on_start:
        on_start()
    t0 = time.perf_counter()
    for i in range(steps):
        if ev is not None:
            ev[i].record()
        step()
    if ev is not None:
        ev[steps].record()
    sync()
    t1 = time.perf_counter()
    if on_stop:
        on_stop()
    if ev is not None:
        step_ms.extend(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
    barrier(world)
    return max_over_ranks(t1 - t0, world)


def ramp(step, seconds, sync=None):
    """Untimed steps for about `seconds` of wall time before the measured legs (the ranks share no
    collective inside a step, and timed() opens with a barrier, so per-rank counts may differ)."""
    if seconds <= 0:
        return 0
    if sync is None:
        import torch
        sync = torch.cuda.synchronize
    # the first step (code-object loading, allocator growth) is outside the measured stretch
    step()
    sync()
    t0 = time.perf_counter()
    n = 1
    while time.perf_counter() - t0 < seconds:
        step()
        n += 1
        if n % 8 == 0:
            sync()
    sync()
    return n


def aggregate_tflops(flops_per_rank_step, steps, world, max_seconds):
    """Whole-job throughput: every rank ran `steps` steps of `flops_per_rank_step` (weak scaling),
    divided by the slowest rank's time."""
    return world * flops_per_rank_step * steps / max_seconds / 1e12


class KernelTimer:
    """Reads the library's HIP-event per-kernel timings (recorded on the launch stream)."""

    def __init__(self):
        import flash_attn_2_cuda as m
        self.lib = m._lib
        self.lib.flash_attn_timing_enable.argtypes = [ctypes.c_int]
        self.lib.flash_attn_timing_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(ctypes.c_long)]
        self.result = {}

    def start(self):
        self.lib.flash_attn_timing_enable(1)

    def stop(self):
        out = {}
        for kid, name in KERNELS.items():
            ms, n = ctypes.c_double(), ctypes.c_long()
            self.lib.flash_attn_timing_read(kid, ctypes.byref(ms), ctypes.byref(n))
            if n.value:
                out[name] = {"total_ms": ms.value, "launches": n.value, "avg_ms": ms.value / n.value}
        self.lib.flash_attn_timing_enable(0)
        self.result = out
        return out


def cpu_threads(requested=0):
    """Threads for the CPU baseline: the process's CPU affinity set, capped by OMP_NUM_THREADS when
    the job was given a CPU share that way (the GPU pool sets it to the box's share)."""
    if requested > 0:
        return requested
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def lib_sha(path):
    """sha256[:16] of a library file (the build a PMC profile describes, profiles/pmc_run.sh)"""
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def load_pmc(path, workload, lib=None):
    """(per-kernel PMC figures, source note) of the workload -- (None, note) when the profile was
    taken on another build than `lib` (the library this run loaded): counters of kernels that no
    longer ship must not be reported next to the timed ones"""
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return None, None
    figs, src = data.get("workloads", {}).get(workload), data.get("source", {}).get(workload)
    want = data.get("lib_sha", {}).get(workload)
    have = lib_sha(lib) if lib else None
    if figs is not None and lib is not None and (want is None or want != have):
        return None, (f"omitted: the PMC profile ({src}) is of library {want}, this run loaded {have}"
                      " -- re-run profiles/pmc_run.sh on this build")
    return figs, src


# ------------------------------------------------------------------------------------------------
# workloads
# ------------------------------------------------------------------------------------------------
def make_workload(name, dev, rank, dropout_p=0.0):
    """-> (fwd_only, fwd_bwd, f_fwd, config dict, dtype name, sdpa sample for the CPU baseline)."""
    import torch

    from flash_attn import flash_attn_func, flash_attn_varlen_qkvpacked_func

    b, s, h, hk, d, dt_name, causal, kind = WORKLOADS[name]
    dtype = torch.bfloat16 if dt_name == "bf16" else torch.float16
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    if kind == "varlen":
        lens = c4_seqlens(total=s)
        cu = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(dev)
        max_s = max(lens)
        qkv = torch.randn(s, 3, h, d, device=dev, dtype=dtype, generator=g).requires_grad_()
        dout = torch.randn(s, h, d, device=dev, dtype=dtype, generator=g)

        def fwd_only():
            with torch.no_grad():
                flash_attn_varlen_qkvpacked_func(qkv, cu, max_s, dropout_p, causal=causal)

        def fwd_bwd():
            out = flash_attn_varlen_qkvpacked_func(qkv, cu, max_s, dropout_p, causal=causal)
            torch.autograd.grad(out, (qkv,), dout)

        f_fwd = varlen_flops_fwd(lens, h, d, causal)
        cfg = {"workload": "flash_attn_varlen_qkvpacked_func fwd+bwd (c4)", "total_tokens": s,
               "batch": len(lens), "max_seqlen": max_s, "seqlens": "U{512..4096}, seed 0 (SURVEY 8(d))",
               "nheads": h, "headdim": d, "causal": causal}
        if dropout_p > 0:
            cfg["dropout_p"] = dropout_p
        sample = ("varlen", lens[:2], h, d)
        return fwd_only, fwd_bwd, f_fwd, cfg, dt_name, sample
    q = torch.randn(b, s, h, d, device=dev, dtype=dtype, generator=g).requires_grad_()
    k = torch.randn(b, s, hk, d, device=dev, dtype=dtype, generator=g).requires_grad_()
    v = torch.randn(b, s, hk, d, device=dev, dtype=dtype, generator=g).requires_grad_()
    dout = torch.randn(b, s, h, d, device=dev, dtype=dtype, generator=g)

    def fwd_only():
        with torch.no_grad():
            flash_attn_func(q, k, v, dropout_p, causal=causal)

    def fwd_bwd():
        out = flash_attn_func(q, k, v, dropout_p, causal=causal)
        torch.autograd.grad(out, (q, k, v), dout)

    f_fwd = flops_fwd(b, s, h, d, causal)
    label = "forward only" if kind == "fwd" else "fwd+bwd"
    cfg = {"workload": f"flash_attn_func {label} ({name})", "batch_per_gpu": b, "seq_len": s,
           "nheads": h, "nheads_k": hk, "headdim": d, "causal": causal}
    if dropout_p > 0:
        cfg["dropout_p"] = dropout_p
    # CPU sample: one batch element; the 32k context is cut to 8k keys/queries (bounded time)
    sample = ("dense", 1, min(s, 8192), h, d)
    return fwd_only, fwd_bwd, f_fwd, cfg, dt_name, sample


def cpu_baseline(sample, causal, dtype, threads, fwd_only):
    from oracle.cpu_baseline import cpu_model_name, sdpa_fwd_bwd_tflops

    if sample[0] == "varlen":
        _, lens, h, d = sample
        tot_f, tot_t = 0.0, 0.0
        for s in lens:
            f = (1.0 if fwd_only else 3.5) * flops_fwd(1, s, h, d, causal)
            tf, sec = sdpa_fwd_bwd_tflops(1, s, h, d, causal, dtype, threads, repeats=2,
                                          flops_fn=lambda bb, f=f: f, fwd_only=fwd_only)
            tot_f += f
            tot_t += sec
        desc = f"sequences of length {lens} of the c4 draw"
        return tot_f / tot_t / 1e12, tot_t, desc
    _, b, s, h, d = sample
    f = (1.0 if fwd_only else 3.5) * flops_fwd(b, s, h, d, causal)
    tf, sec = sdpa_fwd_bwd_tflops(b, s, h, d, causal, dtype, threads, repeats=2, flops_fn=lambda bb: f,
                                  fwd_only=fwd_only)
    return tf, sec, f"batch {b}, seqlen {s}, {h} heads, d {d}"


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        # launcher: no torch / GPU call has happened in this process
        # a rank that hangs (e.g. in RCCL init) must not hang the launcher: bounded wait, then every
        # child is terminated and the launcher exits non-zero (124)
        limit = args.rank_timeout if args.rank_timeout is not None else 900.0 + 5.0 * (args.steps + args.warmup)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], timeout=limit))

    import torch

    rank, local, world = dist_init(args.dry_run)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} ranks")

    if args.dry_run:
        hang = os.environ.get("FA_BENCH_DRYRUN_HANG_RANK")   # test hook: this rank never reaches the barrier
        if hang is not None and int(hang) == rank:
            time.sleep(3600)
        t = timed(lambda: time.sleep(0.005), args.steps, args.warmup, world, sync=lambda: None)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "steps": args.steps,
                              "ms_per_step": round(t / args.steps * 1e3, 4)}), flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    dev = torch.device("cuda", local)
    fwd_only, fwd_bwd, f_fwd, cfg, dt_name, sample = make_workload(args.workload, dev, rank, args.dropout)
    kind = WORKLOADS[args.workload][7]
    causal = WORKLOADS[args.workload][6]
    f_step = f_fwd if kind == "fwd" else 3.5 * f_fwd
    headline_step = fwd_only if kind == "fwd" else fwd_bwd

    timer = KernelTimer()
    # Ramp: the first ~50 ms of GPU work run 10-30 % slower (rocprofv3 trace of this command,
    # profiles/r02/c3_kernel_stats_r02h.csv: fwd_kernel 1.37 -> 1.04 ms over its first 25 launches),
    # so both legs start after a fixed, untimed stretch of headline steps.
    ramp(headline_step, args.ramp_s)
    # forward-only leg (the north_star's >= 50%-of-peak target is quoted on the forward)
    t_fwd = timed(fwd_only, args.steps, args.warmup, world)
    # headline leg, with live per-kernel event timing over the timed steps only
    step_ms = []
    t_step = timed(headline_step, args.steps, args.warmup, world, on_start=timer.start, on_stop=timer.stop,
                   step_ms=step_ms)
    kt = timer.result
    if kind == "fwd":
        # forward-only workloads (c2): the headline step IS the forward-only leg's step, timed without
        # the per-launch event instrumentation, which at 50 us per step outweighs the launch itself
        # (the instrumented leg above only supplies the kernel windows)
        t_step = t_fwd
    ms_per_step = t_step / args.steps * 1e3
    # disjoint intervals inside the timed region: the forward, bwd_pre and the dK/dV + dQ window (dK/dV
    # and dQ run concurrently on two streams, so their own windows overlap and are not summed)
    if "bwd_dkdv_dq_window" in kt:
        disjoint = [n for n in kt if n not in ("bwd_dkdv_kernel", "bwd_dq_kernel")]
    else:
        disjoint = list(kt)
    windows_per_step = sum(kt[n]["total_ms"] for n in disjoint) / args.steps
    assert windows_per_step <= ms_per_step * 1.01 + 0.01, (windows_per_step, ms_per_step)

    value = aggregate_tflops(f_step, args.steps, world, t_step)
    fwd_tflops = aggregate_tflops(f_fwd, args.steps, world, t_fwd)

    import flash_attn_2_cuda as fa_ext
    pmc, pmc_src = load_pmc(args.pmc, args.workload, fa_ext.LIBRARY_PATH)
    kernels = {}
    for n, x in kt.items():
        e = {"avg_ms": round(x["avg_ms"], 4), "launches": x["launches"]}
        if n in KERNEL_FLOP_FACTOR:
            e["tflops"] = round(KERNEL_FLOP_FACTOR[n] * f_fwd / (x["avg_ms"] / 1e3) / 1e12, 1)
        p = (pmc or {}).get(n)
        if p:
            e["hbm_bytes"] = p["hbm_bytes"]
            e["hbm_gbps"] = round(p["hbm_bytes"] / (x["avg_ms"] / 1e3) / 1e9, 1)
            if "mfma_util" in p:
                e["mfma_util"] = p["mfma_util"]
        kernels[n] = e

    # roofline of the dominant kernel (largest device time in the headline leg)
    dom = max((n for n in kt if n in KERNEL_FLOP_FACTOR), key=lambda n: kt[n]["total_ms"], default=None)
    roofline = None
    if dom in KERNEL_FLOP_FACTOR:
        alg = KERNEL_FLOP_FACTOR[dom] * f_fwd
        achieved = alg / (kt[dom]["avg_ms"] / 1e3) / 1e12
        traffic = ((pmc or {}).get(dom) or {}).get("hbm_bytes")
        roofline = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / PEAK_TFLOPS, 4), "traffic": traffic,
                    "alg_flops_per_launch": alg, "avg_launch_ms": round(kt[dom]["avg_ms"], 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.dropout == 0:
        from oracle.cpu_baseline import cpu_model_name
        threads = cpu_threads(args.cpu_threads)
        dtype = torch.bfloat16 if dt_name == "bf16" else torch.float16
        tf, sec, desc = cpu_baseline(sample, causal, dtype, threads, kind == "fwd")
        cpu = {"value": round(tf, 4), "unit": "TFLOPS", "cores": threads, "kind": "port",
               "sample": f"torch SDPA {'fwd' if kind == 'fwd' else 'fwd+bwd'} on CPU ({cpu_model_name()}, "
                         f"{threads} threads = affinity set capped by OMP_NUM_THREADS), {desc} of the "
                         f"{args.workload} workload ({dt_name}, causal={causal}), {sec:.2f} s per rep, "
                         f"1 warm-up + 2 reps"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "TFLOPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "value_estimator": ("wall clock of the forward-only leg: K back-to-back steps without per-step events, "
                                "between barrier + synchronize" if kind == "fwd" else
                                "wall clock of K steps between barrier + synchronize (events between steps)"),
            "ms_per_step_median": round(statistics.median(step_ms), 4) if step_ms else None,
            "ms_per_step_min": round(min(step_ms), 4) if step_ms else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / world / H100_FWD_BWD_TFLOPS, 4) if args.workload == "c3" else None,
            "dtype": dt_name,
            "data": "synthetic N(0,1) Q/K/V/dO, resident in HBM",
            "config": dict(cfg, global_batch=(cfg.get("batch_per_gpu") or cfg.get("batch")) * world,
                           parallelism=f"batch-sharded x{world}, no collectives on the hot path"),
            "fwd_tflops": round(fwd_tflops, 2),
            "fwd_ms": round(t_fwd / args.steps * 1e3, 4),
            "fwd_frac_of_peak": round(fwd_tflops / world / PEAK_TFLOPS, 4),
            "tflops_per_gpu": round(value / world, 2),
            "baseline_note": "vs_baseline = per-GPU fwd+bwd TFLOPS / 308 (FA2 on H100 SXM5, causal hdim128 s8k, "
                             "BASELINE.md); c3 only",
            "kernels": kernels,
            "kernel_windows_ms_per_step": round(windows_per_step, 4),
            "lib_sha": lib_sha(fa_ext.LIBRARY_PATH),
            "pmc_source": pmc_src,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
