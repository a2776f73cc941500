"""Loader for the in-tree engine library (assistedmanipulation_amd/lib/libmppi_amd.so).

There is no fallback: if the library is missing the import fails with the build command.
The library is loaded before anything imports torch so that its ROCm runtime (/opt/rocm,
RUNPATH) is the one both share (same sonames, first loaded wins).
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPPI_AMD_LIB") or os.path.join(HERE, "lib", "libmppi_amd.so")   # override: kernel A/B builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "mppi_amd.h")

_dp = C.POINTER(C.c_double)
_h = C.c_void_p
_i64p = C.POINTER(C.c_int64)

# name -> (restype, argtypes); every function include/mppi_amd.h declares
PROTOTYPES = {
    "mppi_abi_version": (C.c_int, []),
    "mppi_build_info": (C.c_char_p, []),
    "mppi_default_frankaridgeback": (None, [C.POINTER(abi.mppi_frankaridgeback_desc)]),
    "mppi_default_assisted_manipulation": (None, [C.POINTER(abi.mppi_assisted_manipulation_desc)]),
    "mppi_default_track_point": (None, [C.POINTER(abi.mppi_track_point_desc)]),
    "mppi_create": (C.c_int, [C.POINTER(abi.mppi_config), C.POINTER(abi.mppi_dynamics_desc),
                              C.POINTER(abi.mppi_cost_desc), C.c_int, C.POINTER(_h)]),
    "mppi_destroy": (None, [_h]),
    "mppi_last_error": (C.c_char_p, [_h]),
    "mppi_shard_range": (C.c_int, [C.c_int64, C.c_int, C.c_int, _i64p, _i64p]),
    "mppi_comm_unique_id": (C.c_int, [C.c_char_p]),
    "mppi_comm_init": (C.c_int, [_h, C.c_int, C.c_int, C.c_char_p]),
    "mppi_comm_info": (C.c_int, [_h, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_int]),
    "mppi_set_shard": (C.c_int, [_h, C.c_int, C.c_int]),
    "mppi_set_noise_source": (C.c_int, [_h, C.c_int, C.c_uint64]),
    "mppi_inject_noise": (C.c_int, [_h, _dp, C.c_int64]),
    "mppi_noise_draws": (C.c_int, [_h, C.c_double, _i64p]),
    "mppi_set_index_semantics": (C.c_int, [_h, C.c_int]),
    "mppi_set_forecast": (C.c_int, [_h, _dp]),
    "mppi_forecast_attach": (C.c_int, [_h, C.POINTER(abi.mppi_forecast_config)]),
    "mppi_forecast_observe": (C.c_int, [_h, _dp, C.c_double]),
    "mppi_forecast_observe_time": (C.c_int, [_h, C.c_double]),
    "mppi_forecast_get": (C.c_int, [_h, C.c_double, _dp]),
    "mppi_step_constants": (C.c_int, [_h, _dp]),
    "mppi_update": (C.c_int, [_h, _dp, C.c_double]),
    "mppi_set_graph": (C.c_int, [_h, C.c_int]),
    "mppi_debug_inject": (C.c_int, [_h, C.c_int, C.c_int]),
    "mppi_debug_folded_cost": (C.c_int, [_h, C.POINTER(C.c_double)]),
    "mppi_graph_updates": (C.c_int, [_h, _i64p]),
    "mppi_update_phase1": (C.c_int, [_h, _dp, C.c_double]),
    "mppi_update_phase2": (C.c_int, [_h]),
    "mppi_update_phase3": (C.c_int, [_h]),
    "mppi_device_costs": (C.c_void_p, [_h]),
    "mppi_device_gradient": (C.c_void_p, [_h]),
    "mppi_stream": (C.c_void_p, [_h]),
    "mppi_synchronize": (C.c_int, [_h]),
    "mppi_get": (C.c_int, [_h, C.c_double, _dp]),
    "mppi_costs": (C.c_int, [_h, _dp]),
    "mppi_weights": (C.c_int, [_h, _dp]),
    "mppi_gradient": (C.c_int, [_h, _dp]),
    "mppi_optimal_control": (C.c_int, [_h, _dp]),
    "mppi_optimal_cost": (C.c_int, [_h, _dp]),
    "mppi_argmin": (C.c_int, [_h, _i64p]),
    "mppi_optimal_terms": (C.c_int, [_h, _dp]),
    "mppi_update_duration": (C.c_int, [_h, _dp]),
    "mppi_update_last": (C.c_int, [_h, _dp]),
    "mppi_device_costs_count": (C.c_int64, [_h]),
    "mppi_noise": (C.c_int, [_h, _dp]),
    "mppi_dims": (C.c_int, [_h, _i64p, _i64p, _i64p, _i64p]),
    "mppi_update_info": (C.c_int, [_h, _i64p, C.c_int]),
    "mppi_smoothing_windows": (C.c_int, [_h, _dp, _dp, _i64p]),
    "mppi_kernel_times": (C.c_int, [_h, C.POINTER(C.c_float)]),
    "mppi_kernel_times_nowait": (C.c_int, [_h, C.POINTER(C.c_float)]),
    "mppi_kernel_times_detail": (C.c_int, [_h, C.POINTER(C.c_float), C.c_int]),
    "mppi_set_timing": (C.c_int, [_h, C.c_int]),
    "mppi_rollout_kernel_times": (C.c_int, [_h, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]),
    "mppi_forecast_table": (C.c_int, [_h, C.c_double, C.c_double, C.c_int64, _dp]),
    "mppi_dynamics_create": (C.c_int, [C.POINTER(abi.mppi_dynamics_desc), _dp, C.c_int, C.POINTER(_h)]),
    "mppi_dynamics_destroy": (None, [_h]),
    "mppi_dynamics_set_state": (C.c_int, [_h, _dp, C.c_double]),
    "mppi_dynamics_step": (C.c_int, [_h, _dp, C.c_double, _dp]),
    "mppi_dynamics_get_state": (C.c_int, [_h, _dp]),
    "mppi_dynamics_end_effector": (C.c_int, [_h, _dp]),
    "mppi_dynamics_query": (C.c_int, [_h, _dp]),
    "mppi_dynamics_forecast": (C.c_int, [_h, _dp, C.c_double, C.c_double, C.c_int64, _dp, _dp]),
    "mppi_cost_evaluate": (C.c_int, [C.POINTER(abi.mppi_cost_desc), _h, _dp, _dp, _dp, _dp]),
}

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "assistedmanipulation_amd: engine library %s is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
            "assistedmanipulation_amd/csrc`" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    # a library chosen by MPPI_AMD_LIB (an older build under an A/B run) may lack later entry points:
    # those stay unbound and fail when called; the in-tree library must export every one
    ab = "MPPI_AMD_LIB" in os.environ
    for name, (res, args) in PROTOTYPES.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            if not ab:
                raise
            continue
        f.restype = res
        f.argtypes = args
    _lib = L
    return L
