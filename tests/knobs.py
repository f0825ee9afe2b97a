"""Launcher switches of the library (include/flash_attn.h flash_attn_set_knob), for the GPU tests
that compare a launch path with its alternative (the library reads them from the environment once;
a test sets and restores them through the C entry point instead)."""
import contextlib
import ctypes

NO_SPLITKV, NO_XCD_GROUP, XCD_GROUP_MIN_MIB, BWD_ASM, DQ_ASM, FWD_PERSIST, BWD_PERSIST, ASM_XCD_GROUP_MIN_MIB, FUSE_PRE, \
    VARLEN_ROUNDS, BWD_2W, FWD_VARLEN_ROUNDS = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11


def _lib():
    import flash_attn_2_cuda as m
    lib = m._lib
    lib.flash_attn_set_knob.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.flash_attn_get_knob.argtypes = [ctypes.c_int]
    lib.flash_attn_get_knob.restype = ctypes.c_int
    return lib


@contextlib.contextmanager
def knob(kid, value):
    lib = _lib()
    old = lib.flash_attn_get_knob(kid)
    lib.flash_attn_set_knob(kid, value)
    try:
        yield
    finally:
        lib.flash_attn_set_knob(kid, old)


def no_splitkv():
    return knob(NO_SPLITKV, 1)


@contextlib.contextmanager
def hip_forward():
    """every forward through fwd_kernel (fa_fwd.hip) instead of the assembly kernels: a comparison
    that needs the HIP kernel's arithmetic (fp32 scores; the assembly forward holds Q as
    bf16/f16(scale log2(e) Q)) on both sides"""
    import flash_attn_2_cuda as m
    m._lib.flash_attn_fwd_use_asm(0)
    try:
        yield
    finally:
        m._lib.flash_attn_fwd_use_asm(1)
