#!/usr/bin/env python3
"""Writes a C++ source that embeds a binary file as `extern "C" const unsigned char NAME[]` and
`extern "C" const unsigned long NAME_size` (the assembly forward's code object, fa_fwd_asm.cpp).

    python3 embed.py FILE NAME > out.cpp
"""
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    data = open(path, "rb").read()
    out = [f"// generated from {path.split('/')[-1]} by asm/embed.py -- do not edit",
           f'extern "C" const unsigned long {name}_size = {len(data)}ul;',
           f'extern "C" __attribute__((aligned(4096))) const unsigned char {name}[{len(data)}] = {{']
    for i in range(0, len(data), 24):
        out.append("  " + ",".join(str(b) for b in data[i:i + 24]) + ",")
    out.append("};")
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
