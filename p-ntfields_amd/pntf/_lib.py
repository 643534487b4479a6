"""ctypes binding of libpntf.so (C ABI declared in include/pntf.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc, gfx950) and loaded from
this directory.  There is no fallback: if the library is missing every compute entry point
raises, so a GPU run can never silently take a CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpntf.so")

GRAD_EXACT = 0
GRAD_BACKGRAD_COMPAT = 1

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_size = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/pntf.h exactly
SIGNATURES = {
    "pntf_abi_version": (ctypes.c_int, []),
    "pntf_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "pntf_last_error": (ctypes.c_char_p, []),
    "pntf_packed_floats": (_size, []),
    "pntf_pack_weights": (ctypes.c_int, [ctypes.POINTER(_c_void_p), ctypes.c_int, _c_void_p,
                                         _c_void_p]),
    "pntf_net_create": (_c_void_p, [ctypes.POINTER(_c_void_p), ctypes.c_int, _c_void_p]),
    "pntf_net_update": (ctypes.c_int, [_c_void_p, ctypes.POINTER(_c_void_p), ctypes.c_int,
                                       _c_void_p]),
    "pntf_net_packed": (_c_void_p, [_c_void_p]),
    "pntf_net_destroy": (None, [_c_void_p]),
    "pntf_workspace_bytes": (_size, [_i64]),
    "pntf_field_schedule_for": (ctypes.c_int, [_i64, ctypes.c_int]),
    "pntf_set_field_schedule": (ctypes.c_int, [ctypes.c_int]),
    "pntf_build_info": (ctypes.c_char_p, []),
    "pntf_field_ex": (ctypes.c_int, [ctypes.c_int, _c_void_p, ctypes.c_int, _c_void_p, _i64,
                                     _c_void_p, _c_void_p, _i32, ctypes.c_int, _c_void_p,
                                     _c_void_p, _c_void_p, _size, ctypes.c_int, _c_void_p]),
    "pntf_tau": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p, _c_void_p,
                                _i32, _c_void_p, _c_void_p]),
    "pntf_tau_grad": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                     _c_void_p, _i32, ctypes.c_int, _c_void_p, _c_void_p,
                                     _c_void_p, _size, _c_void_p]),
    "pntf_path_velocity": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                          _c_void_p, _i32, ctypes.c_int, _c_void_p, _c_void_p,
                                          _c_void_p, _size, _c_void_p]),
    "pntf_speed": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                  _c_void_p, _i32, _c_void_p, _c_void_p, _size, _c_void_p]),
    "pntf_travel_time": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                        _c_void_p, _i32, _c_void_p, _c_void_p]),
    "pntf_plan": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                 _c_void_p, _i32, ctypes.c_int, _f32, _f32, _i32, _c_void_p,
                                 _c_void_p, _c_void_p, _size, _c_void_p]),
    "pntf_plan_ex": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _i64, _c_void_p,
                                    _c_void_p, _i32, ctypes.c_int, _f32, _f32, _i32, _c_void_p,
                                    _c_void_p, _c_void_p, _size, ctypes.c_int, _c_void_p]),
    "pntf_eikonal_residual": (ctypes.c_int, [_c_void_p, ctypes.c_int, _c_void_p, _c_void_p,
                                             _i64, _c_void_p, _c_void_p, _i32, _f32,
                                             _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                             _c_void_p, _size, _c_void_p]),
    "pntf_sum": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    # training step (pntf_train.hip)
    "pntf_tt_partial_floats": (_size, []),
    "pntf_tt_last_error": (ctypes.c_char_p, []),
    "pntf_tt_fourier": (ctypes.c_int, [ctypes.c_int, _c_void_p, _i64, _c_void_p, _c_void_p, _i32,
                                       _c_void_p, _c_void_p]),
    "pntf_tt_act_fwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _c_void_p,
                                       _c_void_p, _c_void_p, _i64, ctypes.c_int, ctypes.c_int,
                                       _c_void_p]),
    "pntf_tt_act_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _c_void_p, _i64,
                                       ctypes.c_int, ctypes.c_int, _c_void_p, ctypes.c_int,
                                       _c_void_p, _c_void_p]),
    "pntf_tt_merge_fwd": (ctypes.c_int, [ctypes.c_int, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "pntf_tt_merge_bwd": (ctypes.c_int, [ctypes.c_int, _c_void_p, _c_void_p, _i64, _c_void_p,
                                         _c_void_p]),
    "pntf_tt_fourier_value": (ctypes.c_int, [ctypes.c_int, _c_void_p, _i64, _c_void_p, _c_void_p,
                                             _i32, _c_void_p, _c_void_p]),
    "pntf_tt_merge_value_fwd": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "pntf_tt_merge_value_bwd": (ctypes.c_int, [_c_void_p, _c_void_p, _i64, _c_void_p,
                                               _c_void_p]),
    "pntf_tt_head_tau": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _c_void_p]),
    "pntf_tt_head_loss": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _c_void_p,
                                         _c_void_p, _c_void_p, _c_void_p, _i64, _f32, _f32,
                                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                         _c_void_p]),
    # general VJP tape (out_laplace / out_grad / out_backgrad / Model.gradient backward)
    "pntf_tt_fourier_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_void_p,
                                          _i64, _c_void_p, _c_void_p, _i32, _c_void_p,
                                          _c_void_p]),
    "pntf_tt_fourier_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_void_p,
                                           _c_void_p, _i64, _c_void_p, _c_void_p, _i32,
                                           _c_void_p, _c_void_p]),
    "pntf_tt_merge_fwd_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _i64,
                                            _c_void_p, _c_void_p]),
    "pntf_tt_merge_bwd_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _c_void_p,
                                            _i64, _c_void_p, _c_void_p]),
    "pntf_tt_head_vjp": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _c_void_p,
                                        _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p]),
    "pntf_tt_gemm_work_floats": (ctypes.c_size_t, [_i64, _i64, _i64]),
    "pntf_tt_gemm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _c_void_p, _i64,
                                    _c_void_p, _i64, _c_void_p, _i64, _f32, _c_void_p,
                                    ctypes.c_size_t, _c_void_p]),
    "pntf_tt_gemm_last_error": (ctypes.c_char_p, []),
    "pntf_tt_set_panel_mode": (ctypes.c_int, [ctypes.c_int]),
    "pntf_tt_set_wgrad_mode": (ctypes.c_int, [ctypes.c_int]),
    "pntf_tt_set_bwd_mode": (ctypes.c_int, [ctypes.c_int]),
    "pntf_tt_linear_act": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _i64, ctypes.c_int,
                                          _c_void_p, ctypes.c_int, _c_void_p, _c_void_p, _c_void_p,
                                          _c_void_p, ctypes.c_int, ctypes.c_int, _c_void_p,
                                          ctypes.c_size_t, _c_void_p]),
    "pntf_tt_linear_bwd_work_floats": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "pntf_tt_linear_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_void_p, _i64, ctypes.c_int,
                                          _c_void_p, ctypes.c_int, _c_void_p, _c_void_p,
                                          _c_void_p, _c_void_p, _c_void_p, ctypes.c_size_t,
                                          _c_void_p]),
    "pntf_adamw": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f32, _f32,
                                  _f32, _f32, _f32, _i64, _c_void_p]),
    "pntf_adamw_multi": (ctypes.c_int, [ctypes.c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _c_void_p, _f32, _f32, _f32, _f32, _f32, _i64,
                                        _c_void_p]),
    # speed-sample generator (pntf_mesh.hip)
    "pntf_point_mesh_distance": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p,
                                                ctypes.c_int, _c_void_p]),
    "pntf_mesh_chunks": (ctypes.c_int, [_i64, _i64]),
    "pntf_mesh_last_error": (ctypes.c_char_p, []),
}

_lib = None


class PntfError(RuntimeError):
    pass


def load():
    """Load libpntf.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PntfError(
            "libpntf.so not found at %s — build it with `python -c 'import __graft_entry__ as g;"
            " g.build()'` (hipcc --offload-arch=gfx950)" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pntf_abi_version() != 1:
        raise PntfError("libpntf ABI version mismatch")
    _lib = lib
    return lib


def build_info():
    """{unit: code hash} baked into the loaded libpntf.so (include/pntf.h pntf_build_info)."""
    raw = load().pntf_build_info().decode()
    return dict(kv.split("=", 1) for kv in raw.split(";") if "=" in kv)


def check(status, what):
    if status != 0:
        lib = load()
        if what.startswith(("pntf_tt_", "pntf_adamw")):
            err = lib.pntf_tt_last_error()
        elif what.startswith("pntf_point_mesh"):
            err = lib.pntf_mesh_last_error()
        else:
            err = lib.pntf_last_error()
        err = err.decode()
        raise PntfError("%s failed: %s (%s)" % (
            what, lib.pntf_status_string(status).decode(), err))
