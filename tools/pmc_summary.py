#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs written by tools/pmc_ab.sh: per variant and kernel, the
mean of every counter over dispatches (dev tool)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    for vdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(vdir):
            continue
        acc = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(vdir, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    short = name.split("(")[0].split("::")[-1].split("<")[0]
                    if not short or ("kernel" not in short and not short.startswith("fa_")):
                        continue
                    acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
        print(f"== {os.path.basename(vdir)}")
        for k, cs in sorted(acc.items()):
            items = ", ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
            print(f"  {k}: {items}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
