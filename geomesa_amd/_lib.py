"""Loader for the in-tree HIP library (geomesa_amd/lib/libgeomesa_hip.so).

The product path is the HIP library only: there is no CPU fallback.  If the library is missing or
no GPU is visible, every compute entry point raises GeomesaHipUnavailable.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GEOMESA_HIP_LIB selects another in-tree build of the same library (variant builds for profiling)
LIB_PATH = os.environ.get("GEOMESA_HIP_LIB", os.path.join(HERE, "lib", "libgeomesa_hip.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "geomesa_hip.h")

GM_OK = 0
GM_E_INVALID = -1
GM_E_HIP = -2
GM_E_CAPACITY = -3
GM_E_ELEMENT = -4
GM_E_INDEX = -5

GM_ST_OK = 0
GM_ST_OUT_OF_BOUNDS = 1
GM_ST_BAD_TIME = 2
GM_ST_UNORDERED = 3
GM_ST_NULL_GEOM = 4

GM_PARAM_JOIN_CHUNK = 1
GM_PARAM_INDEX_BUILD = 2
GM_PARAM_RANGES_CHUNK = 3
GM_PARAM_SORT_MODE = 4
GM_PARAM_SORT_LAST = 5
GM_PARAM_INDEX_COARSE = 6
GM_PARAM_INDEX_CORE_RETIRED = 7
GM_PARAM_HIST_GRID = 8
GM_PARAM_RELATE_ROWS64 = 9

GM_JOIN_AUTO = 0
GM_JOIN_DIRECT = 1
GM_SPATIAL_NONE, GM_SPATIAL_INTERSECTS, GM_SPATIAL_CONTAINS = 0, 1, 2


class GeomesaHipUnavailable(RuntimeError):
    """The HIP library or a GPU is not available (no silent fallback exists)."""


class GeomesaHipError(RuntimeError):
    pass


class BatchStatus(ctypes.Structure):
    _fields_ = [("n_errors", ctypes.c_int64), ("first_index", ctypes.c_int64),
                ("first_code", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Range(ctypes.Structure):
    _fields_ = [("lower", ctypes.c_int64), ("upper", ctypes.c_int64),
                ("contained", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class KeyRange(ctypes.Structure):
    _fields_ = [("z_lo", ctypes.c_int64), ("z_hi", ctypes.c_int64), ("bin_lo", ctypes.c_int16),
                ("bin_hi", ctypes.c_int16), ("shard", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class ScanFilter(ctypes.Structure):
    """gm_scan_filter: the row filter (Z3Filter or Z2Filter bytes) and the full filter (envelopes x boxes,
    dtg during) of gm_table_scan."""
    _fields_ = [("z3filter", ctypes.c_void_p), ("z3filter_len", ctypes.c_size_t),
                ("z2filter", ctypes.c_void_p), ("z2filter_len", ctypes.c_size_t),
                ("xmin", ctypes.c_void_p), ("ymin", ctypes.c_void_p), ("xmax", ctypes.c_void_p),
                ("ymax", ctypes.c_void_p), ("boxes", ctypes.c_void_p), ("n_boxes", ctypes.c_int32),
                ("during", ctypes.c_int32), ("t_ms", ctypes.c_void_p), ("t_lo", ctypes.c_int64),
                ("t_hi", ctypes.c_int64)]


# numpy view of gm_key_range rows (24 B, the KeyRange layout)
KEY_RANGE_DTYPE = np.dtype([("z_lo", "<i8"), ("z_hi", "<i8"), ("bin_lo", "<i2"), ("bin_hi", "<i2"), ("shard", "u1"),
                            ("reserved", "u1", (3,))])


class PolySetC(ctypes.Structure):
    _fields_ = [("n_polys", ctypes.c_int32),
                ("poly_part_off", ctypes.c_void_p), ("part_ring_off", ctypes.c_void_p),
                ("ring_vert_off", ctypes.c_void_p), ("vx", ctypes.c_void_p), ("vy", ctypes.c_void_p)]


GM_PIP_INDEX_ARRAYS = 8
GM_PIP_LAYOUT_VERSION = 1


class PipIndexLayout(ctypes.Structure):
    _fields_ = [("version", ctypes.c_int32), ("dims", ctypes.c_int32 * 4), ("reserved", ctypes.c_int32),
                ("grid", ctypes.c_double * 6), ("stats", ctypes.c_int64 * 9),
                ("bytes", ctypes.c_int64 * GM_PIP_INDEX_ARRAYS)]


vp = ctypes.c_void_p
i64 = ctypes.c_int64
i32 = ctypes.c_int32
cint = ctypes.c_int
d = ctypes.c_double
sz = ctypes.c_size_t

# every symbol include/geomesa_hip.h declares, with its ctypes signature
SIGNATURES = {
    "gm_abi_version": (cint, []),
    "gm_ctx_create": (cint, [cint, vp, vp]),
    "gm_ctx_create_owned": (cint, [cint, vp]),
    "gm_ctx_destroy": (cint, [vp]),
    "gm_ctx_sync": (cint, [vp]),
    "gm_ctx_stream": (vp, [vp]),
    "gm_last_error": (ctypes.c_char_p, []),
    "gm_ctx_set_param": (cint, [vp, cint, i64]),
    "gm_ctx_get_param": (cint, [vp, cint, vp]),
    "gm_device_alloc": (cint, [vp, sz, vp]),
    "gm_device_free": (cint, [vp, vp]),
    "gm_copy_to_device": (cint, [vp, vp, vp, sz]),
    "gm_copy_to_host": (cint, [vp, vp, vp, sz]),
    "gm_device_copy": (cint, [vp, vp, vp, sz]),
    "gm_timer_start": (cint, [vp]),
    "gm_timer_stop": (cint, [vp, vp]),
    "gm_z3_index": (cint, [vp, vp, vp, vp, i64, cint, cint, cint, vp, vp, vp]),
    "gm_z3_index_key": (cint, [vp, vp, vp, vp, i64, cint, cint, vp, vp, vp, vp]),
    "gm_z3_invert": (cint, [vp, vp, i64, cint, cint, vp, vp, vp]),
    "gm_z2_index": (cint, [vp, vp, vp, i64, cint, cint, vp, vp, vp]),
    "gm_z2_invert": (cint, [vp, vp, i64, cint, vp, vp]),
    "gm_binned_time": (cint, [vp, vp, i64, cint, vp, vp, vp, vp]),
    "gm_xz2_index": (cint, [vp, vp, vp, vp, vp, i64, cint, cint, vp, vp, vp]),
    "gm_xz3_index": (cint, [vp, vp, vp, vp, vp, vp, vp, i64, cint, cint, cint, vp, vp, vp]),
    "gm_xz3_index_key": (cint, [vp, vp, vp, vp, vp, vp, i64, cint, cint, cint, vp, vp, vp, vp]),
    "gm_z3_ranges": (cint, [vp, i64, vp, vp, vp, vp, cint, cint, cint, cint, cint, vp, vp, i64, vp, vp]),
    "gm_z2_ranges": (cint, [vp, i64, vp, vp, cint, cint, cint, cint, vp, vp, i64, vp, vp]),
    "gm_zranges": (cint, [vp, cint, i64, vp, vp, cint, cint, cint, vp, vp, i64, vp, vp]),
    "gm_xz2_ranges": (cint, [vp, i64, vp, vp, cint, cint, vp, vp, i64, vp, vp]),
    "gm_xz3_ranges": (cint, [vp, i64, vp, vp, cint, cint, cint, vp, vp, i64, vp, vp]),
    "gm_z3filter_scan": (cint, [vp, vp, sz, vp, cint, vp, vp, i64, vp, vp, i64, vp]),
    "gm_z2filter_scan": (cint, [vp, vp, sz, vp, i64, vp, vp, i64, vp]),
    "gm_z3filter_scan_rows": (cint, [vp, vp, sz, vp, vp, cint, i64, vp, vp, i64, vp, vp]),
    "gm_z2filter_scan_rows": (cint, [vp, vp, sz, vp, vp, cint, i64, vp, vp, i64, vp, vp]),
    "gm_strict_scan": (cint, [vp, vp, vp, vp, i64, vp, cint, i64, i64, vp, vp, i64, vp]),
    "gm_query_scan": (cint, [vp, vp, vp, vp, i64, vp, cint, i64, i64, vp, cint, vp, vp, i64, vp]),
    "gm_pip_index_create": (cint, [vp, vp, vp]),
    "gm_pip_index_create_ex": (cint, [vp, vp, cint, vp]),
    "gm_pip_index_destroy": (cint, [vp]),
    "gm_pip_index_stats": (cint, [vp, vp]),
    "gm_pip_join_census": (cint, [vp, vp, vp, vp, i64, vp]),
    "gm_pip_index_export": (cint, [vp, vp]),
    "gm_pip_index_copy_array": (cint, [vp, vp, cint, vp]),
    "gm_pip_index_import": (cint, [vp, vp, vp, vp]),
    "gm_pip_join": (cint, [vp, vp, vp, vp, i64, i64, vp, vp, i64, vp]),
    "gm_pip_join_ex": (cint, [vp, vp, vp, vp, i64, i64, vp, vp, i64, vp, cint]),
    "gm_pip_join_pred": (cint, [vp, vp, vp, vp, i64, i64, vp, vp, i64, vp, cint, cint]),
    "gm_z3_key_bytes": (cint, [vp, vp, vp, vp, i64, vp]),
    "gm_sort_keys": (cint, [vp, vp, vp, vp, i64, vp, vp, vp, vp]),
    "gm_key_range_scan": (cint, [vp, vp, vp, vp, i64, vp, i64, vp, sz, vp, vp, i64, vp, vp]),
    "gm_table_scan": (cint, [vp, vp, vp, vp, i64, vp, i64, vp, vp, vp, i64, vp, vp]),
    "gm_z2_key_bytes": (cint, [vp, vp, vp, i64, vp]),
    "gm_key_sample": (cint, [vp, vp, vp, vp, i64, i32, vp, vp]),
    "gm_key_partition": (cint, [vp, vp, vp, vp, i64, vp, vp, i32, vp, i64, vp, vp, vp, vp, vp, vp]),
    "gm_z3_index_key_arrow": (cint, [vp, vp, vp, i64, cint, cint, vp, vp, vp, vp]),
    "gm_z2_index_key_arrow": (cint, [vp, vp, i64, cint, vp, vp, vp]),
    "gm_xz2_index_key_arrow": (cint, [vp, vp, i64, cint, cint, vp, vp, vp]),
    "gm_xz3_index_key_arrow": (cint, [vp, vp, vp, i64, cint, cint, cint, vp, vp, vp, vp]),
    "gm_arrow_points_to_columns": (cint, [vp, vp, i64, vp, vp]),
    "gm_pip_join_arrow": (cint, [vp, vp, vp, i64, i64, vp, vp, i64, vp, cint, cint]),
    "gm_pip_index_create_arrow": (cint, [vp, vp, i32, cint, vp]),
    "gm_pip_relate": (cint, [vp, vp, vp, vp, vp, i64, vp]),
    "gm_legacy_z3_index": (cint, [vp, vp, vp, vp, i64, cint, cint, cint, vp, vp, vp]),
    "gm_legacy_z3_invert": (cint, [vp, vp, i64, cint, cint, vp, vp, vp]),
    "gm_legacy_z2_index": (cint, [vp, vp, vp, i64, cint, vp, vp, vp]),
    "gm_legacy_z2_invert": (cint, [vp, vp, i64, vp, vp]),
    "gm_z3_histogram": (cint, [vp, vp, vp, vp, i64, cint, cint, cint, cint, cint, vp, vp, vp]),
    "gm_gen_points": (cint, [vp, ctypes.c_uint64, i64, i64, d, d, d, d, i64, i64, vp, vp, vp]),
}

_lib = None


def load():
    """Load the HIP library (torch is imported first so one HIP runtime serves both)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- binds libamdhip64.so.7 before our library resolves it
    if not os.path.exists(LIB_PATH):
        raise GeomesaHipUnavailable(
            "libgeomesa_hip.so not built (%s); run `python -m geomesa_amd.build`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    variant = "GEOMESA_HIP_LIB" in os.environ   # an older / experimental build for A/B timing
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def last_error():
    return load().gm_last_error().decode(errors="replace")


def check(rc, what):
    if rc == GM_OK:
        return
    raise GeomesaHipError("%s failed: rc=%d (%s)" % (what, rc, last_error()))


class Context:
    """One gm_ctx bound to a device and a HIP stream (torch's current stream by default)."""

    def __init__(self, device=0, stream=None):
        import torch
        lib = load()
        if not torch.cuda.is_available():
            raise GeomesaHipUnavailable("no GPU visible: the geomesa_amd product path needs a MI355X")
        torch.cuda.set_device(device)
        if stream is None:
            stream = torch.cuda.current_stream(device).cuda_stream
        self.device = device
        self._h = ctypes.c_void_p()
        check(lib.gm_ctx_create(device, ctypes.c_void_p(stream), ctypes.byref(self._h)), "gm_ctx_create")
        self.lib = lib

    @property
    def handle(self):
        return self._h

    def set_param(self, param, value):
        check(self.lib.gm_ctx_set_param(self._h, int(param), int(value)), "gm_ctx_set_param")

    def get_param(self, param):
        v = ctypes.c_int64()
        check(self.lib.gm_ctx_get_param(self._h, int(param), ctypes.byref(v)), "gm_ctx_get_param")
        return v.value

    def sync(self):
        check(self.lib.gm_ctx_sync(self._h), "gm_ctx_sync")

    def close(self):
        if self._h:
            self.lib.gm_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts = {}


def context(device=None):
    """Per-(device, stream) cached context."""
    import torch
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    if not torch.cuda.is_available():
        load()
        raise GeomesaHipUnavailable("no GPU visible: the geomesa_amd product path needs a MI355X")
    stream = torch.cuda.current_stream(device).cuda_stream
    key = (device, stream)
    if key not in _contexts:
        _contexts[key] = Context(device, stream)
    return _contexts[key]


def ptr(t):
    """Device pointer of a torch tensor (None passes through)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
