#!/usr/bin/env python3
"""rocprofv3 PMC passes (profiles/pmc_run.sh) -> per-kernel figures in profiles/pmc.json, which
bench.py reports next to its live kernel times.

Per kernel, averaged over its dispatches in the profiled bench command:
  * hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 -- kilobyte counters at the L2's memory
    side; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads (16 B per lane,
    buffer_load ... lds included), MI355X_MICROARCH.md "HBM" (Infinity-Cache hits are counted);
  * mfma_util = SQ_INSTS_MFMA * 32 / (1024 * GRBM_GUI_ACTIVE / 8): matrix-pipe busy fraction (one
    v_mfma_f32_32x32x16 holds a SIMD's matrix pipe for 32 cycles; 1024 SIMDs; GRBM_GUI_ACTIVE is
    summed over the 8 XCDs);
  * mfma_flops = SQ_INSTS_MFMA * 32768 (executed, vs the algorithmic count in bench.py);
  * valu_per_mfma, lds_per_mfma, wait_inst_frac (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES), wait_any_frac,
    lds_bank_conflict_frac (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE);
  * clock_ghz = GRBM_GUI_ACTIVE / 8 / profiled duration (DVFS under the profiler);
  * lib_sha: sha256[:16] of the libflash_attn_mi355x.so the passes ran (pmc_run.sh lib_sha.txt).
    python3 profiles/pmc.py gpurun_out/pmc_c3 c3 [source-note]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
OURS = ("fwd_kernel", "bwd_pre_kernel", "bwd_dkdv_kernel", "bwd_dq_kernel", "splitkv_combine_kernel")


def short(name):
    if name.startswith(("fa_fwd_asm_", "fa_fwdnf_asm_")):   # the assembly forward (gen_fwd.py / gen_fwdnf.py) is the fwd_kernel slot
        return "fwd_kernel"
    if name.startswith(("fa_bwd_dkdv_asm_", "fa_bwd2_dkdv_asm_")):   # the assembly dK/dV kernels (gen_bwd*.py)
        return "bwd_dkdv_kernel"
    if name.startswith("fa_bwd_dq_asm_"):     # the assembly dQ kernel (gen_dq.py)
        return "bwd_dq_kernel"
    return name.split("(")[0].split("::")[-1].split("<")[0].strip()


def collect(root):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k not in OURS:
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}, \
        {k: sum(v) / len(v) for k, v in dur.items() if v}


def derive(c, dur_s):
    out = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["hbm_bytes"] = round(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024)
    mf = c.get("SQ_INSTS_MFMA")
    gr = c.get("GRBM_GUI_ACTIVE")
    if mf and gr:
        out["mfma_util"] = round(mf * 32 / (1024 * gr / 8), 4)
        out["mfma_flops"] = mf * 32768
        if c.get("SQ_INSTS_VALU"):
            out["valu_per_mfma"] = round(c["SQ_INSTS_VALU"] / mf, 2)
        if c.get("SQ_INSTS_LDS"):
            out["lds_per_mfma"] = round(c["SQ_INSTS_LDS"] / mf, 2)
    if c.get("SQ_WAVE_CYCLES"):
        for key, name in (("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_WAIT_ANY", "wait_any_frac"),
                          ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
            if key in c:
                out[name] = round(c[key] / c["SQ_WAVE_CYCLES"], 4)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    if gr and dur_s:
        out["clock_ghz"] = round(gr / 8 / dur_s / 1e9, 3)
        out["profiled_ms"] = round(dur_s * 1e3, 4)
    out["counters"] = {k: round(v, 1) for k, v in sorted(c.items())}
    return out


def main(root, workload, note=None):
    counters, dur = collect(root)
    path = os.path.join(HERE, "pmc.json")
    data = {"workloads": {}, "source": {}}
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    data["workloads"][workload] = {k: derive(c, dur.get(k)) for k, c in sorted(counters.items())}
    data["source"][workload] = note or f"rocprofv3 --pmc passes of profiles/pmc_run.sh ({root})"
    # the library the passes profiled (pmc_run.sh lib_sha.txt): bench.py drops these figures for
    # any other build
    sha = None
    if os.path.exists(os.path.join(root, "lib_sha.txt")):
        with open(os.path.join(root, "lib_sha.txt")) as f:
            sha = f.read().strip() or None
    data.setdefault("lib_sha", {})[workload] = sha
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(json.dumps(data["workloads"][workload], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc",
         sys.argv[2] if len(sys.argv) > 2 else "c3",
         sys.argv[3] if len(sys.argv) > 3 else None)
