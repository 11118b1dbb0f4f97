"""ctypes binding of libdmx.so (include/dmx.h).  The library is built in-tree by
depthmapx_amd.build (hipcc, gfx950); importing this module never falls back to anything else:
if the shared object is missing or a call fails, a DmxError is raised."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DMX_LIB: another in-tree build of the same library (A/B kernel experiments, scripts/gpu_mk_ab.sh)
LIB_PATH = os.environ.get("DMX_LIB") or os.path.join(_HERE, "_lib", "libdmx.so")

DMX_OK = 0
STATUS_NAMES = {-1: "DMX_ERR_ARG", -2: "DMX_ERR_HIP", -3: "DMX_ERR_CAPACITY", -4: "DMX_ERR_STATE",
                -5: "DMX_ERR_UNSUPPORTED", -6: "DMX_ERR_OUTSIDE", -7: "DMX_ERR_CANCELLED"}
# int32_t (*dmx_progress_fn)(void* user, int32_t phase, int64_t done, int64_t total)
PROGRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64)

# every symbol include/dmx.h declares, with (restype, argtypes)
_vp, _i64, _i32, _dbl, _cs = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_char_p
SIGNATURES = {
    "dmx_abi_version": (_i32, []),
    "dmx_last_error": (ctypes.c_char_p, []),
    "dmx_ctx_create": (_i32, [_i32, _vp]),
    "dmx_ctx_free": (_i32, [_vp]),
    "dmx_ctx_last_timing": (_i32, [_vp, _vp, _vp]),
    "dmx_ctx_last_stats": (_i32, [_vp, _vp, _i32]),
    "dmx_pointmap_create": (_i32, [_vp, _dbl, _vp, _i64, _vp]),
    "dmx_pointmap_free": (_i32, [_vp]),
    "dmx_pointmap_fill": (_i32, [_vp, _dbl, _dbl, _vp]),
    "dmx_pointmap_fill_device": (_i32, [_vp, _vp, _dbl, _dbl, _vp]),
    "dmx_pointmap_make_points": (_i32, [_vp, _dbl, _dbl, _i32, _vp]),
    "dmx_graph_special_nodes": (_i32, [_vp, _vp, _vp]),
    "dmx_pointmap_make_points_device": (_i32, [_vp, _vp, _dbl, _dbl, _i32, _vp]),
    "dmx_ctx_last_fill": (_i32, [_vp, _vp, _vp, _vp]),
    "dmx_pointmap_info": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "dmx_pointmap_state": (_i32, [_vp, _vp]),
    "dmx_pointmap_cell_lines": (_i32, [_vp, _vp, _vp, _vp]),
    "dmx_makegraph": (_i32, [_vp, _vp, _dbl, _i32, _i64, _i64, _vp]),
    "dmx_makegraph_balance": (_i32, [_vp, _vp, _dbl, _i32, _i32, _i64, _vp]),
    "dmx_graph_free": (_i32, [_vp]),
    "dmx_graph_info": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dmx_graph_copy": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dmx_graph_copy_range": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _vp, _vp]),
    "dmx_graph_blob_size": (_i32, [_vp, _vp]),
    "dmx_graph_blob_write_device": (_i32, [_vp, _vp, _i64]),
    "dmx_graph_assemble_device": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp]),
    "dmx_vga_global": (_i32, [_vp, _vp, _dbl, _i32, _i64, _i64, _vp, _vp]),
    "dmx_vga_global_device": (_i32, [_vp, _vp, _dbl, _i32, _i64, _i64, _vp]),
    "dmx_metric_stepdepth": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    "dmx_visual_stepdepth": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    "dmx_vga_global_device_list": (_i32, [_vp, _vp, _dbl, _i32, _vp, _i64, _vp]),
    "dmx_graph_set_prep_shard": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "dmx_vga_local": (_i32, [_vp, _vp, _i32, _i64, _i64, _vp]),
    "dmx_vga_metric": (_i32, [_vp, _vp, _dbl, _i32, _i64, _i64, _vp]),
    "dmx_vga_angular": (_i32, [_vp, _vp, _dbl, _i32, _i64, _i64, _vp]),
    "dmx_angular_stepdepth": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    "dmx_release_cached_memory": (_i32, []),
    "dmx_ctx_set_progress": (_i32, [_vp, PROGRESS_FN, _vp, _dbl]),
    "dmx_ctx_cancel": (_i32, [_vp]),
    "dmx_ctx_last_stepdepth": (_i32, [_vp, _vp, _vp, _vp]),
    "dmx_ctx_last_stepdepth_detail": (_i32, [_vp, _vp]),
    "dmx_ctx_last_phase_cycles": (_i32, [_vp, _vp]),
    "dmx_ctx_last_mk_reruns": (_i32, [_vp, _vp, ctypes.c_int64, _vp]),
    "dmx_chunk_write": (_i32, [_vp, _i64, _vp, _vp, _i64, _vp, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "dmx_pointmap_set_state": (_i32, [_vp, _vp]),
    "dmx_chunk_parse": (_i32, [_vp, _i64, _vp]),
    "dmx_chunk_free": (_i32, [_vp]),
    "dmx_chunk_info": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dmx_chunk_column": (_i32, [_vp, _i32, _vp, _i32, _vp, _vp]),
    "dmx_chunk_arrays": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dmx_chunk_load": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dmx_graph_from_runs": (_i32, [_vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp]),
    "dmx_graph_set_merges": (_i32, [_vp, _vp, _i64]),
    "dmx_graph_set_drawing": (_i32, [_vp, _vp, _i64]),
    "dmx_pointmap_set_merges": (_i32, [_vp, _vp, _i64]),
    "dmx_chunk_merges": (_i32, [_vp, _vp, _vp]),
    "dmx_chunk_flags": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dmx_chunk_set_column": (_i32, [_vp, _cs, _vp, _vp, _i32, _i32]),
    "dmx_chunk_set_displayed": (_i32, [_vp, _i32]),
    "dmx_chunk_set_name": (_i32, [_vp, _cs]),
    "dmx_chunk_select_cells": (_i32, [_vp, _vp, _i64]),
    "dmx_chunk_unmake": (_i32, [_vp, _i32]),
    "dmx_chunk_serialize": (_i32, [_vp, _vp, _i64, _vp]),
    "dmx_graphfile_read": (_i32, [_cs, _vp]),
    "dmx_graphfile_free": (_i32, [_vp]),
    "dmx_graphfile_write": (_i32, [_vp, _cs]),
    "dmx_graphfile_info": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dmx_graphfile_lines": (_i32, [_vp, _vp]),
    "dmx_graphfile_set_view": (_i32, [_vp, _i32, _i32]),
    "dmx_graphfile_pointmap": (_i32, [_vp, _i32, _vp, _vp]),
    "dmx_graphfile_put_pointmap": (_i32, [_vp, _i32, _vp, _i64]),
    "dmx_graphfile_new_pointmap_name": (_i32, [_vp, _vp, _i32]),
    "dmx_view_vga_top": (_i32, [_i32]),
}


# dmx_allreduce_fn (include/dmx.h): sum `count` elements of dtype DMX_I32 (0) / DMX_I64 (1) in place
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p)


class DmxError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("%s (%d): %s" % (STATUS_NAMES.get(status, "?"), status, message))
        self.status = status


_lib = None


def _share_hip_runtime_with_torch():
    # torch bundles its own libamdhip64.so.7 / libhsa-runtime64; two HIP runtimes in one process
    # cannot both own the GPU.  Loading torch first makes libdmx.so bind to the same runtime
    # (same SONAME), so device pointers, streams and RCCL from torch interoperate with it.
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        _share_hip_runtime_with_torch()
        if not os.path.exists(LIB_PATH):
            raise DmxError(-2, "native library %s is missing: run depthmapx_amd.build.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("DMX_LIB") and not hasattr(L, name):
                continue   # an older A/B build (timing probes) may lack entry points added since
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status):
    if status != DMX_OK:
        raise DmxError(status, lib().dmx_last_error().decode(errors="replace"))
    return status


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)
