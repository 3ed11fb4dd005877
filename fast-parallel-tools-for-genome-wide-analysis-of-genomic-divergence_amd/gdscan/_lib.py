"""ctypes binding of lib/libgdscan.so (the C ABI in include/gdscan.h).

The library is the product: there is no Python or CPU fallback.  If it is
missing or cannot be loaded this module raises at import time.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent.parent
LIB_DIR = PKG_DIR / "lib"
LIB_PATH = Path(os.environ.get("GDSCAN_LIB", LIB_DIR / "libgdscan.so"))  # override: A/B builds

GD_OK = 0
GD_ERR_ARG = -1
GD_ERR_HIP = -2
GD_ERR_UNSORTED = -4
GD_ERR_BOUNDS = -5
GD_ERR_SIZE = -6
GD_ERR_NOPACK = -7
GD_DEFAULT_SEED = 20261015
GD_WINDOWS_THREADED = 0
GD_WINDOWS_SERIAL = 1
GD_NSTAGES = 4
GD_SELECT_GE = 0
GD_SELECT_LE = 1
GD_FET_REFERENCE = 0
GD_FET_EXACT = 1

# every symbol include/gdscan.h declares
EXPORTS = (
    "gd_fet_threadcompute", "gd_fet_compute", "gd_fet_scan_host", "gd_fet_scan_host_ex",
    "gd_set_fet_mode", "gd_get_fet_mode", "gd_fet_scan_device_ex", "gd_fet_scan_host_batch_ex",
    "gd_css_threadcompute", "gd_css_compute", "gd_css_scan_host", "gd_css_scan_host_ex", "gd_css_coords_host",
    "gd_ctx_create", "gd_ctx_destroy", "gd_window_count",
    "gd_fet_scan_device", "gd_css_scan_device", "gd_css_scan_device_ex", "gd_fet_scan_host_batch",
    "gd_css_scan_host_batch", "gd_css_scan_host_batch_ex",
    "gd_set_seed", "gd_get_seed", "gd_last_error", "gd_last_status", "gd_device_count",
    "gd_last_stage_ms", "gd_synth_device",
    "gd_gtrack_read", "gd_gtrack_free", "gd_gtrack_nseq", "gd_gtrack_seqid", "gd_gtrack_len", "gd_gtrack_copy",
    "gd_ptrack_read", "gd_ptrack_free", "gd_ptrack_nseq", "gd_ptrack_seqid", "gd_ptrack_shape", "gd_ptrack_copy",
    "gd_write_tabular", "gd_format_py2_float",
    "gd_tabular_read", "gd_tabular_free", "gd_tabular_rows", "gd_tabular_nseq", "gd_tabular_seqid",
    "gd_tabular_copy",
    "gd_fet_region_limit", "gd_css_fdr_threshold", "gd_css_top_limit", "gd_merge_regions",
    "gd_pack_shape", "gd_pack_chrom", "gd_pack_chrom_mt", "gd_pack_chrom_device", "gd_fet_scan_packed_device",
    "gd_css_scan_packed_device", "gd_fet_scan_packed_host", "gd_css_scan_packed_host",
)


class GdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gdscan error {code}: {msg}")
        self.code = code


class Chrom(C.Structure):
    _fields_ = [
        ("a_off", C.c_int64), ("b_off", C.c_int64),
        ("alen", C.c_int32), ("blen", C.c_int32),
        ("regend", C.c_int32), ("w_first", C.c_int32),
        ("w_out", C.c_int64), ("seed", C.c_uint64),
        ("w_count", C.c_int32), ("pad_", C.c_int32),
    ]


class PChrom(C.Structure):
    """gd_pchrom (include/gdscan.h): one chromosome of a packed batch."""
    _fields_ = [
        ("row_off", C.c_int64), ("a_word", C.c_int64), ("b_word", C.c_int64),
        ("nrows", C.c_int32), ("asize", C.c_int32), ("bsize", C.c_int32), ("regend", C.c_int32),
        ("w_out", C.c_int64), ("seed", C.c_uint64),
    ]


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` "
            "(or __graft_entry__.build()); there is no fallback implementation")
    lib = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0))
    dp, ip, vp = C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_void_p
    i32 = C.c_int
    fet_ref = [dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, C.c_double, dp, dp]
    css_ref = [dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, dp, dp]
    lib.gd_fet_threadcompute.argtypes = fet_ref
    lib.gd_fet_compute.argtypes = fet_ref
    lib.gd_fet_scan_host.argtypes = [dp, dp, ip, ip, i32, i32, i32, i32, i32, C.c_double, C.c_uint64, i32, dp, dp]
    lib.gd_fet_scan_host_ex.argtypes = [dp, dp, ip, ip, i32, i32, i32, i32, i32, C.c_double, i32, C.c_uint64, i32,
                                        dp, dp]
    lib.gd_set_fet_mode.argtypes = [i32]
    lib.gd_get_fet_mode.argtypes = []
    lib.gd_css_threadcompute.argtypes = css_ref
    lib.gd_css_compute.argtypes = css_ref
    lib.gd_css_scan_host.argtypes = [dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, i32, C.c_uint64, i32, dp, dp]
    lib.gd_css_scan_host_ex.argtypes = [dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, i32, i32, i32, C.c_uint64, i32,
                                        dp, dp]
    lib.gd_css_coords_host.argtypes = [dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, i32, i32, C.c_uint64, i32, dp,
                                       dp, dp]
    lib.gd_css_coords_host.restype = C.c_int
    lib.gd_ctx_create.argtypes = [i32]
    lib.gd_ctx_create.restype = vp
    lib.gd_ctx_destroy.argtypes = [vp]
    lib.gd_ctx_destroy.restype = None
    lib.gd_window_count.argtypes = [i32, i32, i32, i32]
    lib.gd_fet_scan_device.argtypes = [vp, C.POINTER(Chrom), i32, vp, vp, vp, vp, i32, i32, C.c_double, i32,
                                       vp, vp, vp]
    lib.gd_fet_scan_device_ex.argtypes = [vp, C.POINTER(Chrom), i32, vp, vp, vp, vp, i32, i32, C.c_double, i32, i32,
                                          vp, vp, vp]
    lib.gd_css_scan_device.argtypes = [vp, C.POINTER(Chrom), i32, vp, vp, vp, vp, i32, i32, i32, i32, i32,
                                       vp, vp, vp]
    lib.gd_css_scan_device_ex.argtypes = [vp, C.POINTER(Chrom), i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32,
                                          i32, vp, vp, vp]
    lib.gd_set_seed.argtypes = [C.c_uint64]
    lib.gd_set_seed.restype = None
    lib.gd_get_seed.restype = C.c_uint64
    lib.gd_last_error.restype = C.c_char_p
    lib.gd_last_stage_ms.argtypes = [C.POINTER(C.c_float), i32]
    lib.gd_synth_device.argtypes = [i32, i32, i32, i32, C.c_uint64, vp, vp, vp, vp, vp, vp]
    lib.gd_fet_scan_host_batch.argtypes = [C.POINTER(Chrom), i32, dp, dp, ip, ip, i32, i32, C.c_double, i32, dp, dp]
    lib.gd_fet_scan_host_batch_ex.argtypes = [C.POINTER(Chrom), i32, dp, dp, ip, ip, i32, i32, C.c_double, i32, i32,
                                              dp, dp]
    lib.gd_css_scan_host_batch.argtypes = [C.POINTER(Chrom), i32, dp, dp, ip, ip, i32, i32, i32, i32, i32, dp, dp]
    lib.gd_css_scan_host_batch_ex.argtypes = [C.POINTER(Chrom), i32, dp, dp, ip, ip, i32, i32, i32, i32, i32, i32, i32,
                                              dp, dp]
    lib.gd_css_scan_host_batch_ex.restype = C.c_int
    lib.gd_fet_scan_host_batch.restype = C.c_int
    lib.gd_css_scan_host_batch.restype = C.c_int
    lib.gd_gtrack_read.argtypes = [C.c_char_p]
    lib.gd_gtrack_read.restype = vp
    lib.gd_gtrack_free.argtypes = [vp]
    lib.gd_gtrack_free.restype = None
    lib.gd_gtrack_nseq.argtypes = [vp]
    lib.gd_gtrack_seqid.argtypes = [vp, i32]
    lib.gd_gtrack_seqid.restype = C.c_char_p
    lib.gd_gtrack_len.argtypes = [vp, i32]
    lib.gd_gtrack_len.restype = C.c_int64
    lib.gd_gtrack_copy.argtypes = [vp, i32, vp, vp]
    lib.gd_ptrack_read.argtypes = [C.c_char_p]
    lib.gd_ptrack_read.restype = vp
    lib.gd_ptrack_free.argtypes = [vp]
    lib.gd_ptrack_free.restype = None
    lib.gd_ptrack_nseq.argtypes = [vp]
    lib.gd_ptrack_seqid.argtypes = [vp, i32]
    lib.gd_ptrack_seqid.restype = C.c_char_p
    lib.gd_ptrack_shape.argtypes = [vp, i32, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    lib.gd_ptrack_copy.argtypes = [vp, i32, vp, vp]
    lib.gd_write_tabular.argtypes = [C.c_char_p, i32, C.c_char_p, C.c_char_p, i32, C.c_int64, vp, vp]
    lib.gd_format_py2_float.argtypes = [C.c_double, C.c_char_p, i32]
    i64, pi64 = C.c_int64, C.POINTER(C.c_int64)
    lib.gd_tabular_read.argtypes = [C.c_char_p]
    lib.gd_tabular_read.restype = vp
    lib.gd_tabular_free.argtypes = [vp]
    lib.gd_tabular_free.restype = None
    lib.gd_tabular_rows.argtypes = [vp]
    lib.gd_tabular_rows.restype = i64
    lib.gd_tabular_nseq.argtypes = [vp]
    lib.gd_tabular_seqid.argtypes = [vp, i32]
    lib.gd_tabular_seqid.restype = C.c_char_p
    lib.gd_tabular_copy.argtypes = [vp, vp, vp, vp, vp]
    lib.gd_fet_region_limit.argtypes = [vp, vp, vp, i64, C.c_double, C.c_double, dp, vp]
    lib.gd_css_fdr_threshold.argtypes = [vp, vp, i64, C.c_double, dp, pi64, vp]
    lib.gd_css_top_limit.argtypes = [vp, vp, i64, i64, dp, vp]
    lib.gd_merge_regions.argtypes = [vp, vp, vp, vp, i64, i32, C.c_double, i64, vp, i32, vp, vp, pi64, pi64, vp]
    for fn in ("gd_tabular_nseq", "gd_tabular_copy", "gd_fet_region_limit", "gd_css_fdr_threshold",
               "gd_css_top_limit", "gd_merge_regions"):
        getattr(lib, fn).restype = C.c_int
    lib.gd_pack_shape.argtypes = [ip, ip, i32, i32, ip, ip, ip]
    lib.gd_pack_chrom.argtypes = [dp, dp, ip, ip, i32, i32, i32, vp, vp, vp]
    lib.gd_pack_chrom_mt.argtypes = [dp, dp, ip, ip, i32, i32, i32, vp, vp, vp]
    lib.gd_pack_chrom_device.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp]
    lib.gd_fet_scan_packed_device.argtypes = [vp, C.POINTER(PChrom), i32, vp, vp, vp, i32, i32, C.c_double, i32, i32,
                                              vp, vp, vp]
    lib.gd_css_scan_packed_device.argtypes = [vp, C.POINTER(PChrom), i32, vp, vp, vp, i32, i32, i32, i32, i32, i32,
                                              vp, vp, vp]
    lib.gd_fet_scan_packed_host.argtypes = [C.POINTER(PChrom), i32, vp, vp, vp, i32, i32, C.c_double, i32, i32, dp,
                                            dp]
    lib.gd_css_scan_packed_host.argtypes = [C.POINTER(PChrom), i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, dp, dp]
    for fn in ("gd_pack_shape", "gd_pack_chrom", "gd_pack_chrom_mt", "gd_pack_chrom_device", "gd_fet_scan_packed_device",
               "gd_css_scan_packed_device", "gd_fet_scan_packed_host", "gd_css_scan_packed_host"):
        getattr(lib, fn).restype = C.c_int
    for fn in ("gd_gtrack_nseq", "gd_gtrack_copy", "gd_write_tabular", "gd_format_py2_float", "gd_ptrack_nseq",
               "gd_ptrack_shape", "gd_ptrack_copy"):
        getattr(lib, fn).restype = C.c_int
    for fn in ("gd_fet_threadcompute", "gd_fet_compute", "gd_fet_scan_host", "gd_css_threadcompute",
               "gd_css_compute", "gd_css_scan_host", "gd_css_scan_host_ex", "gd_fet_scan_device",
               "gd_css_scan_device", "gd_css_scan_device_ex", "gd_fet_scan_host_ex", "gd_fet_scan_device_ex",
               "gd_fet_scan_host_batch_ex", "gd_set_fet_mode", "gd_get_fet_mode",
               "gd_synth_device", "gd_device_count", "gd_window_count", "gd_last_stage_ms"):
        getattr(lib, fn).restype = C.c_int
    return lib


lib = _load()


def check(code: int) -> None:
    if code != GD_OK:
        raise GdError(code, lib.gd_last_error().decode(errors="replace"))


def last_stage_ms():
    buf = (C.c_float * GD_NSTAGES)()
    lib.gd_last_stage_ms(buf, GD_NSTAGES)
    return list(buf)
