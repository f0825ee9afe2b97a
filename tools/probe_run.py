#!/usr/bin/env python3
"""Build / run the semantic probe kernel (tools/probe_gen.py) and compare with the emulator (dev tool).

    python tools/probe_run.py build        # tools/probe.co (assembled here, CPU)
    python tools/probe_run.py gpu          # on the GPU box: gpurun_out/probe_out.npy
    python tools/probe_run.py cpu          # emulator + comparison with gpurun_out/probe_out.npy
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
CO = os.path.join(ROOT, "tools", "probe.co")
IN_BYTES = 65536


def inputs():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(IN_BYTES // 2).astype(np.float32)
    from asm_emu import f32_to_bf16
    return f32_to_bf16(x).astype(np.uint16)


def build():
    s = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_gen.py")], check=True,
                       capture_output=True, text=True).stdout
    open("/tmp/probe.s", "w").write(s)
    ll = "/opt/rocm/lib/llvm/bin"
    subprocess.run([f"{ll}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    "/tmp/probe.s", "-o", "/tmp/probe.o"], check=True)
    subprocess.run([f"{ll}/ld.lld", "-shared", "/tmp/probe.o", "-o", CO], check=True)


def gpu():
    import torch
    from probe_gen import OUT_ROWS
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    data = open(CO, "rb").read()
    buf = ctypes.create_string_buffer(data, len(data))
    assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"fa_probe") == 0
    inp = torch.from_numpy(inputs().view(np.int16)).cuda()
    out = torch.zeros(OUT_ROWS * 64, dtype=torch.int32, device="cuda")
    args = (ctypes.c_uint64 * 2)(inp.data_ptr(), out.data_ptr())
    size = ctypes.c_size_t(16)
    cfg = (ctypes.c_void_p * 5)(ctypes.c_void_p(1), ctypes.cast(args, ctypes.c_void_p), ctypes.c_void_p(2),
                                ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), ctypes.c_void_p(3))
    hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 6 + [ctypes.c_uint, ctypes.c_void_p,
                                                                                      ctypes.c_void_p, ctypes.c_void_p]
    r = hip.hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, None, None, cfg)
    assert r == 0, r
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "probe_out.npy"), out.cpu().numpy())
    print("probe ok")


def cpu():
    from asm_emu import Emu, Heap
    from probe_gen import OUT_ROWS
    text = open("/tmp/probe.s").read()
    heap = Heap(1 << 20)
    ain = heap.put(inputs())
    aout = heap.alloc(OUT_ROWS * 256)
    akarg = heap.put(np.array([ain, aout], dtype=np.uint64))
    emu = Emu(text, "fa_probe", heap)
    emu.run_wg(0, akarg, nwaves=1)
    mine = heap.get(aout, OUT_ROWS * 256).view(np.int32).reshape(OUT_ROWS, 64)
    g = np.load(os.path.join(ROOT, "gpurun_out", "probe_out.npy")).reshape(OUT_ROWS, 64)
    for r in range(OUT_ROWS):
        if not np.array_equal(mine[r], g[r]):
            print(f"row {r}: cpu {mine[r][:8].tolist()} ... gpu {g[r][:8].tolist()}")
            bad = np.nonzero(mine[r] != g[r])[0]
            print(f"        lanes differing: {bad.tolist()[:32]}")
    print("compared", OUT_ROWS, "rows")


if __name__ == "__main__":
    {"build": build, "gpu": gpu, "cpu": cpu}[sys.argv[1]]()
