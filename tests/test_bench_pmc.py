"""bench.py reports rocprof PMC figures only for the build they were measured on (VERDICT r04
item 2): profiles/pmc.json records the sha256 of the profiled library per workload, and load_pmc
returns the figures only when the library this run loaded has that hash (CPU test)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _write(tmp_path, sha):
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"build A")
    pmc = tmp_path / "pmc.json"
    pmc.write_text(json.dumps({"workloads": {"c3": {"fwd_kernel": {"hbm_bytes": 1, "mfma_util": 0.5}}},
                               "source": {"c3": "test passes"},
                               "lib_sha": {"c3": sha if sha != "same" else bench.lib_sha(str(lib))}}))
    return str(lib), str(pmc)


def test_pmc_of_this_build_is_reported(tmp_path):
    lib, pmc = _write(tmp_path, "same")
    figs, src = bench.load_pmc(pmc, "c3", lib)
    assert figs["fwd_kernel"]["hbm_bytes"] == 1 and src == "test passes"


def test_pmc_of_another_build_is_omitted(tmp_path):
    lib, pmc = _write(tmp_path, "0123456789abcdef")
    figs, src = bench.load_pmc(pmc, "c3", lib)
    assert figs is None and "omitted" in src


def test_pmc_without_a_build_hash_is_omitted(tmp_path):
    lib, pmc = _write(tmp_path, None)
    figs, src = bench.load_pmc(pmc, "c3", lib)
    assert figs is None and "omitted" in src
