#!/usr/bin/env python3
"""Register / LDS dump comparison of the assembly forward between the GPU and the CPU emulator
(dev tool).  A library variant generated with FA_GEN_DUMP=POINT makes workgroup 0 store every
register of each wave (and the LDS) at POINT to the buffer passed as the `seed` kernarg, then end.

    python tools/asm_dump.py inputs                  # writes tools/dump_in.npz (small causal case)
    python tools/asm_dump.py gpu POINT LIB           # on the GPU box: gpurun_out/dump_POINT.npy
    python tools/asm_dump.py cpu POINT               # emulator, compares with gpurun_out/dump_POINT.npy
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
IN = os.path.join(ROOT, "tools", "dump_in.npz")
SLOTS = 640
DUMP_WORDS = 4 * SLOTS * 64 + 163840 // 4
B, SQ, SK, H, HK, D = 1, 64, 64, 1, 1, 128
CAUSAL = True


def inputs():
    rng = np.random.default_rng(0)
    from asm_emu import f32_to_bf16
    q, k, v = (f32_to_bf16(rng.standard_normal(s).astype(np.float32)).astype(np.uint16)
               for s in ((B, SQ, H, D), (B, SK, HK, D), (B, SK, HK, D)))
    np.savez(IN, q=q, k=k, v=v)


def gpu(point, lib):
    os.environ["FLASH_ATTN_MI355X_LIB"] = lib
    os.environ["FLASH_ATTN_MI355X_FWD_ASM"] = "1"
    sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
    import torch
    import flash_attn_2_cuda as m
    z = np.load(IN)
    q, k, v = (torch.from_numpy(z[n].view(np.int16)).cuda().view(torch.bfloat16) for n in ("q", "k", "v"))
    out = torch.zeros_like(q)
    lse = torch.zeros(B, H, SQ, dtype=torch.float32, device="cuda")
    rng = torch.zeros(2, dtype=torch.int64, device="cuda")
    dump = torch.zeros(DUMP_WORDS, dtype=torch.int32, device="cuda")
    ptr = lambda t: t.data_ptr()  # noqa: E731
    ok = m._lib.flash_attn_fwd(ptr(q), ptr(k), ptr(v), ptr(rng), ptr(out), None, ptr(lse),
                               B, SQ, SK, SQ, SK, H, HK, D, D, 0.0, D ** -0.5, 1.0, CAUSAL, False, True,
                               torch.cuda.current_stream().cuda_stream, ptr(dump), 0,
                               None, None, None, None, None, None, None, None,
                               H * D, HK * D, HK * D, D, D, D, H * D, D, SQ * H * D, SK * HK * D, SK * HK * D, SQ * H * D)
    torch.cuda.synchronize()
    print("ok", ok, m._lib.flash_attn_error())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"dump_{point}.npy"), dump.cpu().numpy())
    np.save(os.path.join(ROOT, "gpurun_out", f"dumpout_{point}.npy"), out.float().cpu().numpy())


def cpu(point):
    from asm_emu import Emu, Heap
    from emu_fwd import fwd_item_decode, pack_args
    env = dict(os.environ, FA_GEN_DUMP=point)
    text = subprocess.run([sys.executable, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_fwd.py")],
                          check=True, capture_output=True, text=True, env=env).stdout
    z = np.load(IN)
    heap = Heap(64 << 20)
    aq, ak, av = heap.put(z["q"]), heap.put(z["k"]), heap.put(z["v"])
    ao = heap.alloc(B * SQ * H * D * 2)
    alse = heap.alloc(B * H * SQ * 4)
    arng = heap.alloc(16)
    adump = heap.alloc(DUMP_WORDS * 4)
    kw = dict(q=aq, k=ak, v=av, o=ao, lse=alse, sched=0, cuq=0, cuk=0, rng=arng, seed=adump, off=0,
              q_batch=SQ * H * D * 2, k_batch=SK * HK * D * 2, v_batch=SK * HK * D * 2, o_batch=SQ * H * D * 2,
              q_row=H * D * 2, kv_row=HK * D * 2, o_row=H * D * 2, q_head=D * 2, k_head=D * 2, v_head=D * 2,
              o_head=D * 2, sq=SQ, sk=SK, lse_pitch=SQ, h=H, c=float(np.float32(D ** -0.5 * 1.4426950408889634)), flags=0,
              n_items=1, grid=1, dec=fwd_item_decode(B * H, H, H // HK, (SQ + 255) // 256))
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    emu = Emu(text, f"fa_fwd_asm_d128_bf16_{'causal' if CAUSAL else 'full'}", heap)
    emu.run_wg(0, akarg)
    mine = heap.get(adump, DUMP_WORDS * 4).view(np.int32).copy()
    gpu_d = np.load(os.path.join(ROOT, "gpurun_out", f"dump_{point}.npy"))
    regs_c = mine[:4 * SLOTS * 64].reshape(4, SLOTS, 64)
    regs_g = gpu_d[:4 * SLOTS * 64].reshape(4, SLOTS, 64)
    names = [f"v{i}" for i in range(256)] + [f"a{i}" for i in range(256)] + [f"s{i}" for i in range(128)]
    for w in range(4):
        diff = [i for i in range(SLOTS) if i not in (254, 255) and not (i >= 512 + 100)
                and not np.array_equal(regs_c[w, i], regs_g[w, i])]
        print(f"wave {w}: {len(diff)} registers differ: " + " ".join(names[i] for i in diff[:60]))
        for i in diff[:6]:
            print(f"   {names[i]}: cpu {regs_c[w, i][:6]} gpu {regs_g[w, i][:6]}")
    lc = mine[4 * SLOTS * 64:]
    lg = gpu_d[4 * SLOTS * 64:]
    bad = np.nonzero(lc != lg)[0]
    print(f"LDS: {bad.size} of {lc.size} dwords differ" + (f", first at byte {4 * bad[0]}" if bad.size else ""))
    if bad.size:
        for blk in sorted(set((4 * bad) // 1024))[:20]:
            n = np.sum((4 * bad) // 1024 == blk)
            print(f"   1-KiB block {blk} (slot {blk // 16}, byte {blk * 1024}): {n} dwords differ")


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "inputs":
        inputs()
    elif cmd == "gpu":
        gpu(sys.argv[2], sys.argv[3])
    else:
        cpu(sys.argv[2])
