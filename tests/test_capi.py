"""CPU checks of the drop-in boundary: the C-ABI library and the Python mirror's host logic.

No kernel is launched here (no GPU in the build container): the library must load, export every
entry point include/flash_attn.h declares, and reject calls through its error channel; the
Python layer must reject what the reference rejects, with the reference's messages.
"""
import ctypes
import os
import re

import pytest
import torch

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "flash_attn.h")
LIB = os.path.join(PKG, "libflash_attn_mi355x.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:bool|void|const char \*)\s*\*?\s*(\w+)\s*\(", text, flags=re.M)))


def test_header_declares_reference_entry_points():
    names = declared_functions()
    for ref_name in ("flash_attn_fwd", "flash_attn_varlen_fwd", "flash_attn_bwd",
                     "flash_attn_varlen_bwd", "flash_attn_set_error", "flash_attn_error"):
        assert ref_name in names


def test_set_error_round_trip():
    """flash_attn_set_error / flash_attn_error (reference capi/flash_attn.h:313-315): the message is
    copied into the thread-local slot; NULL or empty gives "unknown error"."""
    lib = ctypes.CDLL(LIB)
    lib.flash_attn_set_error.argtypes = [ctypes.c_char_p]
    lib.flash_attn_error.restype = ctypes.c_char_p
    lib.flash_attn_set_error(b"caller message")
    assert lib.flash_attn_error() == b"caller message"
    lib.flash_attn_set_error(None)
    assert lib.flash_attn_error() == b"unknown error"


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build() must produce the library"
    lib = ctypes.CDLL(LIB)
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_library_is_gfx950_only():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_error_channel_without_device():
    import flash_attn_2_cuda as m

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    ok = m._lib.flash_attn_fwd(*([None] * 7 + [1, 8, 8, 128, 128, 1, 1, 64, 64] + [0.0, 0.125, 1.0]
                                 + [False, False, True] + [None, 0, 0] + [None] * 8 + [0] * 12))
    assert ok is False
    assert m._lib.flash_attn_error()  # non-empty message


def test_python_mirror_rejects_cpu_tensors():
    from flash_attn import flash_attn_func, flash_attn_qkvpacked_func, flash_attn_varlen_func

    q = torch.randn(1, 8, 2, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="CUDA device"):
        flash_attn_func(q, q, q)
    with pytest.raises(RuntimeError, match="CUDA device"):
        flash_attn_qkvpacked_func(torch.randn(1, 8, 3, 2, 64, dtype=torch.bfloat16))
    cu = torch.tensor([0, 8], dtype=torch.int32)
    with pytest.raises(RuntimeError, match="CUDA device"):
        flash_attn_varlen_func(q[0], q[0], q[0], cu, cu, 8, 8)


def test_block_size_reporting():
    from flash_attn.flash_attn_interface import _get_block_size

    bm, bn = _get_block_size("cpu", 128, False, True)
    assert bm > 0 and bn > 0 and bm % 32 == 0 and bn % 32 == 0


def test_interface_signatures_match_reference():
    """Names, positional order and defaults of the public API (reference :282-492)."""
    import inspect

    import flash_attn

    expect = {
        "flash_attn_qkvpacked_func": ["qkv", "dropout_p", "softmax_scale", "causal", "return_attn_probs"],
        "flash_attn_kvpacked_func": ["q", "kv", "dropout_p", "softmax_scale", "causal", "return_attn_probs"],
        "flash_attn_func": ["q", "k", "v", "dropout_p", "softmax_scale", "causal", "return_attn_probs"],
        "flash_attn_varlen_qkvpacked_func": ["qkv", "cu_seqlens", "max_seqlen", "dropout_p",
                                             "softmax_scale", "causal", "return_attn_probs"],
        "flash_attn_varlen_kvpacked_func": ["q", "kv", "cu_seqlens_q", "cu_seqlens_k", "max_seqlen_q",
                                            "max_seqlen_k", "dropout_p", "softmax_scale", "causal",
                                            "return_attn_probs"],
        "flash_attn_varlen_func": ["q", "k", "v", "cu_seqlens_q", "cu_seqlens_k", "max_seqlen_q",
                                   "max_seqlen_k", "dropout_p", "softmax_scale", "causal",
                                   "return_attn_probs"],
    }
    assert flash_attn.__version__ == "2.0.8"
    for name, params in expect.items():
        sig = inspect.signature(getattr(flash_attn, name))
        assert list(sig.parameters) == params, name
        assert sig.parameters["dropout_p"].default == 0.0
        assert sig.parameters["softmax_scale"].default is None
        assert sig.parameters["causal"].default is False
        assert sig.parameters["return_attn_probs"].default is False


def test_product_path_does_not_import_oracle():
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle", src, flags=re.M), f
                assert "attention_ref" not in src, f


def test_mha_module_surface_on_cpu():
    """The modules construct without a GPU and refuse the reference options outside this build."""
    from flash_attn.modules.mha import MHA, FlashCrossAttention, FlashSelfAttention

    FlashSelfAttention(causal=True, attention_dropout=0.1)
    FlashCrossAttention()
    m = MHA(128, 4, num_heads_kv=2)
    assert m.Wqkv.out_features == 32 * (4 + 2 * 2)
    with pytest.raises(NotImplementedError, match="fused_bias_fc"):
        MHA(128, 4, fused_bias_fc=True)
    r = MHA(128, 4, rotary_emb_dim=16, rotary_emb_interleaved=True)
    assert r.rotary_emb.dim == 16 and r.rotary_emb.interleaved
    with pytest.raises(AssertionError):
        MHA(128, 4, cross_attn=True, rotary_emb_dim=16)
    with pytest.raises(AssertionError):
        FlashSelfAttention()(torch.randn(1, 8, 3, 2, 64))
