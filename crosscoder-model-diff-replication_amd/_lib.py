"""ctypes binding of libcrosscoder_hip.so (the C ABI declared in include/crosscoder_hip.h).

The library is built in-tree (`make -C crosscoder-model-diff-replication_amd/csrc`, or
`__graft_entry__.build()`) and loaded from this package directory.  There is no fallback:
if the library is missing every compute entry point raises.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcrosscoder_hip.so")
# test-only build of the same kernels that also exports the launch-form setters (csrc/Makefile)
DEBUG_LIB_PATH = os.path.join(_HERE, "libcrosscoder_hip_dbg.so")
DEFAULT_PP_MASK = 7  # the ping-pong layouts both libraries default to (csrc/gemm.hip: g_pp_mask)
DEBUG_SETTERS = ("cc_debug_set_pp_mask", "cc_debug_set_pp_fast", "cc_debug_set_dec_one_launch",
                 "cc_debug_set_wave_sync", "cc_debug_set_epi_store", "cc_debug_set_q4")

CC_BF16 = 1
CC_F32 = 2
CC_LAYOUT_KC = 0
CC_LAYOUT_MN = 1

_p = ctypes.c_void_p


class LossTailJob(ctypes.Structure):
    """cc_loss_tail_job (include/crosscoder_hip.h)"""
    _fields_ = [("colsum_acts", ctypes.c_void_p), ("tn", ctypes.c_void_p), ("h", ctypes.c_int64),
                ("l1_part", ctypes.c_void_p), ("row_part", ctypes.c_void_p), ("ncb", ctypes.c_int64),
                ("l0_part", ctypes.c_void_p), ("n_l0", ctypes.c_int64), ("ev", ctypes.c_void_p),
                ("ev_a", ctypes.c_void_p), ("ev_b", ctypes.c_void_p), ("scalars", ctypes.c_void_p),
                ("l1l0_out", ctypes.c_void_p), ("host_out", ctypes.c_void_p), ("seq", ctypes.c_uint32),
                ("B", ctypes.c_int64), ("n", ctypes.c_int64), ("counter", ctypes.c_void_p)]


class ColsumJob(ctypes.Structure):
    """cc_colsum_job (include/crosscoder_hip.h)"""
    _fields_ = [("part", ctypes.c_void_p), ("rows", ctypes.c_int64), ("cols", ctypes.c_int64), ("ld", ctypes.c_int64),
                ("scale", ctypes.c_float), ("out", ctypes.c_void_p)]
_i64 = ctypes.c_int64
_i = ctypes.c_int
_f = ctypes.c_float
_d = ctypes.c_double

# name -> (restype, argtypes); must list every symbol of include/crosscoder_hip.h
SIGNATURES = {
    "cc_version": (_i, []),
    "cc_strerror": (ctypes.c_char_p, [_i]),
    "cc_col_part_rows": (_i64, [_i64]),
    "cc_wave_parts": (_i64, [_i64, _i64]),
    "cc_wgrad_parts": (_i64, [_i64, _i64, _i]),
    "cc_prep_part_rows": (_i64, [_i64]),
    "cc_loss_part_rows": (_i64, [_i64]),
    "cc_loss_col_blocks": (_i64, [_i64]),
    "cc_loss_scalars_len": (_i64, [_i64]),
    "cc_gemm_f32out": (_i, [_p, _i, _i64, _p, _i, _i64, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_prep_input": (_i, [_p, _i, _p, _i, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_prep_input_t": (_i, [_p, _i, _p, _i, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_reduce_rows": (_i, [_p, _i64, _i64, _i64, _f, _p, _p, _i, _p, _p, _p, _p]),
    "cc_reduce_parts": (_i64, [_i64]),
    "cc_dec_norms": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_encode_fwd": (_i, [_p, _p, _p, _p, _p, _i, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_decode_fwd": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_decode_ws_floats": (_i64, [_i64, _i64, _i64, _i]),
    "cc_decode_fwd_ws": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_decode_partial": (_i, [_p, _p, _p, _p, _i64, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _p, _i64, _i64, _i64,
                               _i64, _i, _p]),
    "cc_decode_fwd_ws_t": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_loss_fwd_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _f, _i64, _i64, _i64, _i, _p]),
    "cc_loss_fwd_bwd_rows": (_i, [_p, _p, _p, _p, _p, _p, _p, _f, _i64, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_loss_fwd_bwd_rows_t": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _f, _i64, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_loss_finalize": (_i, [_p, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "cc_loss_finalize_mapped": (_i, [_p, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _i64, _i64,
                                     _i64, _p]),
    "cc_segment_sums": (_i, [_p, ctypes.POINTER(_i64), _i, _i, _p, _p]),
    "cc_dacts_bwd": (_i, [_p, _p, _p, _p, _f, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_wgrad_dec": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_wgrad_enc": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_wgrad_both_t": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_wgrad_tile_sums": (_i64, [_i64, _i64]),
    "cc_wgrad_both_clip_t": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p,
                                  _p, _p, _i64, _p, _p, _p, ctypes.POINTER(_i64), _i, _f, _i, _p, _p, _p, _p, _p, _i, _p]),
    "cc_wgrad_both_sums_t": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p,
                                  _p, _p, _i64, _p, _p, _p, ctypes.POINTER(_i64), _i, _i, _p, _p, _p, _p, _p, _i, _p]),
    "cc_wgrad_both": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_clip_finalize": (_i, [_p, ctypes.POINTER(_i64), _i, _f, _i, _p, _p]),
    "cc_grad_tail": (_i, [_p, _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _i, _p, ctypes.POINTER(_i64), _i, _f, _i, _p,
                          _p, _p]),
    "cc_grad_tail_sums": (_i, [_p, _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _i, _p, ctypes.POINTER(_i64), _i, _i, _p,
                               _p, _p]),
    "cc_loss_tail": (_i, [_p, _p, _i64, _p, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _i64, _i64,
                          _i64, _p, _p]),
    "cc_loss_finalize_nb": (_i, [_p, _i64, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _i64, _i64,
                                 _i64, _p]),
    "cc_decode_loss_ncb": (_i64, [_i64, _i64, _i64, _i64, _i]),
    "cc_decode_loss_t": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i, _p]),
    "cc_decode_loss": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _p,
                            _i64, _i64, _i64, _i64, _i, _p]),
    "cc_transposed_ok": (_i, [_i64, _i64, _i64, _i]),
    "cc_encode_fwd_t": (_i, [_p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_mask_bits_words": (_i64, [_i64, _i64]),
    "cc_dacts_bwd_t": (_i, [_p, _p, _p, _p, _f, _p, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_transpose_b16": (_i, [_p, _i64, _i64, _i64, _p, _i64, _p]),
    "cc_dec_norms_part_floats": (_i64, [_i64, _i64, _i64]),
    "cc_transpose_dec_norms": (_i, [_p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p]),
    "cc_dec_norms_finalize": (_i, [_p, _i64, _i64, _i64, _p, _p, _p, _p]),
    "cc_adam_dec_transposed": (_i, [_p, _p, _p, _p, _i64, _i64, _p, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, _i64, _i64, _p, _p, _i, _p]),
    "cc_gather_rows": (_i, [_p, _i64, _p, _p, _i64, _i64, _p]),
    "cc_fold_scaling": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "cc_decoder_stats": (_i, [_p, _i64, _i64, _i64, _i, _p, _p, _p, _p]),
    "cc_adam_step": (_i, [_p, _p, _p, _p, _i64, _p, _d, _d, _d, _d, _i64, _i64, _i, _p]),
    "cc_adam_step_clip": (_i, [_p, _p, _p, _p, _i64, _p, _i, _f, _i, _p, _d, _d, _d, _d, _i64, _i64, _i, _p]),
    "cc_adam_dec_norms": (_i, [_p, _p, _p, _p, _i64, _p, _p, _i, _f, _i, _d, _d, _d, _d, _i64, _i64, _p, _i64, _i64, _i,
                               _p, _p]),
    "cc_adam_capped_blocks": (_i64, [_i64, _i64]),
}

_lib = None
_debug = None


class HipLibraryMissing(RuntimeError):
    pass


def _open(path):
    if not os.path.exists(path):
        raise HipLibraryMissing(
            f"{path} not found: build it with `make -C {os.path.dirname(path)}/csrc` "
            "(crosscoder_amd has no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load(path=None):
    """Load (once) and type the in-tree library; raises HipLibraryMissing if it is not built.  (A tool
    may pass the path of an experiment build on the FIRST call; the product never does.)"""
    global _lib
    if _lib is not None:
        return _lib
    _lib = _open(path or LIB_PATH)
    return _lib


def load_debug():
    """The test-only debug build (same kernels + cc_debug_set_* launch-form setters)."""
    global _debug
    if _debug is None:
        lib = _open(DEBUG_LIB_PATH)
        for name in DEBUG_SETTERS:
            fn = getattr(lib, name)
            fn.restype = None
            fn.argtypes = [ctypes.c_int]
        lib.cc_debug_spin.restype = _i
        lib.cc_debug_spin.argtypes = [_i64, _i64, _i64, _p]
        lib.cc_debug_set_stamps.restype = None
        lib.cc_debug_set_stamps.argtypes = [_p]
        lib.cc_debug_spin_ev.restype = _i
        lib.cc_debug_spin_ev.argtypes = [_i64, _i64, _p, _p]
        lib.cc_debug_get_q4.restype = _i
        lib.cc_debug_get_q4.argtypes = []
        lib.q4_default = lib.cc_debug_get_q4()  # (the build's CC_Q4_MASK: the product library's fixed form)
        _debug = lib
    return _debug


@contextlib.contextmanager
def debug_library():
    """Route every ops.* call through the debug build for the duration (tests comparing launch forms);
    its setters are reset to the product defaults on exit."""
    global _lib
    prev = load()
    dbg = load_debug()
    _lib = dbg
    try:
        yield dbg
    finally:
        dbg.cc_debug_set_pp_mask(DEFAULT_PP_MASK)
        dbg.cc_debug_set_pp_fast(1)
        dbg.cc_debug_set_dec_one_launch(1)
        dbg.cc_debug_set_wave_sync(0)
        dbg.cc_debug_set_epi_store(1)
        dbg.cc_debug_set_q4(dbg.q4_default)
        _lib = prev


def check(rc):
    if rc != 0:
        msg = load().cc_strerror(rc)
        raise RuntimeError(f"crosscoder_hip error {rc}: {msg.decode() if msg else '?'}")
