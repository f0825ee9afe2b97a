"""Loader for the golden vectors in tests/golden/ (made by tests/golden/make_golden.py)."""
import glob
import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_DT = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}


def golden_names():
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


class Golden:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.z = z
        self.kind = str(z["kind"])
        self.dtype = _DT[str(z["dtype"])]
        self.causal = bool(z["causal"])
        self.b, self.sq, self.sk, self.h, self.hk, self.d = (int(x) for x in z["shape"])

    def t(self, key):
        a = self.z[key]
        if a.dtype == np.uint16:
            return torch.from_numpy(a.view(np.int16).copy()).view(self.dtype)
        return torch.from_numpy(a.copy())

    def has(self, key):
        return key in self.z.files
