#!/usr/bin/env python3
"""One line per bench log: value, ms/step, the roofline kernel and fraction, PMC traffic, CPU baseline.

    python tools/bench_summary.py gpurun_out/r06/bench_*.log
"""
import json
import sys


def main(paths):
    for p in paths:
        try:
            line = next(x for x in open(p) if x.startswith('{"metric"'))
        except (OSError, StopIteration):
            print(f"{p}: no bench line")
            continue
        d = json.loads(line)
        r = d.get("roofline") or {}
        c = d.get("cpu_baseline") or {}
        k = d.get("kernels") or {}
        ks = " ".join(f"{n}={v['avg_ms']:.4f}" for n, v in k.items() if isinstance(v, dict) and "avg_ms" in v)
        print(f"{p}: {d['value']} {d['unit']} | {d['ms_per_step']} ms/step | {r.get('kernel')} frac {r.get('frac')} "
              f"traffic {r.get('traffic')} | cpu {c.get('value')} {c.get('unit', '')} | {ks}")


if __name__ == "__main__":
    main(sys.argv[1:])
