"""Multi-process (gloo, world_size 2) checks of the N>1 path on CPU.

bench.py's multi-GPU mode is weak scaling with the batch sharded across ranks and no collective on
the data path: every rank runs its own batch slice, a barrier + synchronize
bracket the timed region, and one all-reduce(MAX) of the elapsed time follows it.  These tests run
that harness code (``bench.timed`` / ``max_over_ranks`` / ``aggregate_tflops``) under gloo, and
check with the CPU oracle that per-rank batch shards reproduce the whole-batch attention exactly
(the unit of work -- one (batch element, kv-head group) -- has no cross-unit dependency).
"""
import os
import socket
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle.attention_ref import attention_ref

        # 1. harness: rank r sleeps (r+1)*10 ms per step; the reported time is the slowest rank's
        steps = 3
        t = bench.timed(lambda: time.sleep(0.01 * (rank + 1)), steps, 1, world, sync=lambda: None)
        # 2. batch-sharded attention: rank r computes its slice of a seeded global batch
        g = torch.Generator().manual_seed(0)
        B, S, H, HK, D = 4, 37, 4, 2, 16
        q = torch.randn(B, S, H, D, generator=g)
        k = torch.randn(B, S, HK, D, generator=g)
        v = torch.randn(B, S, HK, D, generator=g)
        per = B // world
        sl = slice(rank * per, (rank + 1) * per)
        out_shard, _ = attention_ref(q[sl], k[sl], v[sl], causal=True)
        gathered = [torch.empty_like(out_shard) for _ in range(world)]
        dist.all_gather(gathered, out_shard.contiguous())
        out_full, _ = attention_ref(q, k, v, causal=True)
        torch.save({"t": t, "sharded": torch.cat(gathered), "full": out_full},
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_harness_and_batch_sharding(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # every rank reports the same (max) elapsed time, at least the slowest rank's 3 x 20 ms
    assert res[0]["t"] == res[1]["t"]
    assert res[0]["t"] >= 3 * 0.02 * 0.95
    # sharding the batch across ranks reproduces the whole-batch result bit for bit
    for r in res:
        assert torch.equal(r["sharded"], r["full"])


def test_aggregate_tflops_is_whole_job():
    sys.path.insert(0, ROOT)
    import bench

    f = bench.flops_fwd(4, 8192, 16, 128, True) * 3.5
    one = bench.aggregate_tflops(f, 10, 1, 0.055)
    eight = bench.aggregate_tflops(f, 10, 8, 0.055)
    assert eight == pytest.approx(8 * one)
    assert bench.flops_fwd(4, 8192, 16, 128, True) == pytest.approx(1.0995e12, rel=1e-4)


def test_ramp_runs_untimed_steps_for_its_duration():
    sys.path.insert(0, ROOT)
    import time

    import bench

    calls, syncs = [], []
    t0 = time.perf_counter()
    n = bench.ramp(lambda: (calls.append(1), time.sleep(0.002)), 0.05, sync=lambda: syncs.append(1))
    assert n == len(calls) > 0 and time.perf_counter() - t0 >= 0.05
    assert syncs   # drained at least once (the last sync)
    assert bench.ramp(lambda: calls.append(1), 0.0, sync=lambda: None) == 0


@pytest.mark.timeout(300)
def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` without torch.distributed.run starts the two rank processes itself and
    reports n_gpus from the initialised process group (gloo, harness-only dry run)."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--no-cpu-baseline", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["steps"] == 3


@pytest.mark.timeout(240)
def test_bench_launcher_times_out_a_hung_rank():
    """A rank that never reaches the barrier (FA_BENCH_DRYRUN_HANG_RANK) does not hang the launcher:
    after --rank-timeout every child is terminated and bench.py exits non-zero (124) within it."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FA_BENCH_DRYRUN_HANG_RANK"] = "1"
    limit = 40.0
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--no-cpu-baseline", "--steps", "3", "--warmup", "1", "--rank-timeout", str(limit)],
                       capture_output=True, text=True, env=env, timeout=200)
    elapsed = time.time() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert elapsed < limit + 35, elapsed   # terminate + join of the children after the limit


@pytest.mark.timeout(120)
def test_bench_world_mismatch_is_an_error():
    """A process group whose size differs from --gpus is refused (no silent 1-GPU timing)."""
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=100)
    assert r.returncode != 0 and "--gpus 2" in r.stderr


def test_c4_seqlens_recipe():
    sys.path.insert(0, ROOT)
    import bench

    lens = bench.c4_seqlens()
    assert sum(lens) == 65536
    assert all(512 <= s <= 4096 for s in lens[:-1]) and 1 <= lens[-1] <= 4096
    assert lens == bench.c4_seqlens()          # seeded, reproducible
    assert 20 <= len(lens) <= 40
