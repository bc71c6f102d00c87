"""ctypes binding of libreporter_match.so (include/reporter_match.h).

There is no CPU fallback: if the shared library is missing or cannot be
loaded this module raises, so a product path can never silently route around
the HIP engine.
"""
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("REPORTER_MATCH_LIB") or os.path.join(_HERE, "libreporter_match.so")

_lock = threading.Lock()
_lib = None


class RmOptions(C.Structure):
    _fields_ = [("mode", C.c_int32), ("sigma_z", C.c_float), ("beta", C.c_float), ("search_radius", C.c_float),
                ("gps_accuracy", C.c_float), ("breakage_distance", C.c_float), ("interpolation_distance", C.c_float),
                ("max_route_distance_factor", C.c_float), ("max_route_time_factor", C.c_float),
                ("turn_penalty_factor", C.c_float)]


class RmWorldParams(C.Structure):
    _fields_ = [("rows", C.c_uint32), ("cols", C.c_uint32), ("block_m", C.c_double), ("seed", C.c_uint64),
                ("center_lat", C.c_double), ("center_lon", C.c_double), ("jitter", C.c_double),
                ("arterial_every", C.c_uint32), ("highway_every", C.c_uint32), ("segment_max_m", C.c_double),
                ("internal_m", C.c_double), ("service_frac", C.c_double), ("oneway_frac", C.c_double),
                ("curve_frac", C.c_double), ("cell_m", C.c_double)]


class RmCityParams(C.Structure):
    _fields_ = [("rows", C.c_uint32), ("cols", C.c_uint32), ("block_m", C.c_double), ("seed", C.c_uint64),
                ("center_lat", C.c_double), ("center_lon", C.c_double), ("jitter", C.c_double),
                ("primary_every", C.c_uint32), ("secondary_every", C.c_uint32), ("boulevard_every", C.c_uint32),
                ("diagonal_every", C.c_uint32), ("roundabout_frac", C.c_double), ("drop_frac", C.c_double),
                ("oneway_frac", C.c_double), ("spur_frac", C.c_double), ("service_frac", C.c_double),
                ("footway_frac", C.c_double), ("osmlr_local_frac", C.c_double), ("way_max_m", C.c_double),
                ("trunk", C.c_uint32)]


class RmTraceParams(C.Structure):
    _fields_ = [("n_traces", C.c_uint32), ("n_points", C.c_uint32), ("rate_s", C.c_double),
                ("noise_m", C.c_double), ("seed", C.c_uint64), ("mode", C.c_int32), ("start_epoch", C.c_int64),
                ("threads", C.c_uint32)]


class RmBatchDesc(C.Structure):
    _fields_ = [("n_traces", C.c_uint32), ("trace_off", C.c_void_p), ("lon", C.c_void_p), ("lat", C.c_void_p),
                ("time", C.c_void_p), ("accuracy", C.c_void_p), ("n_opts", C.c_uint32),
                ("opts", C.c_void_p), ("trace_opt", C.c_void_p)]


class RmRunParams(C.Structure):
    _fields_ = [("threshold_sec", C.c_double), ("report_mask", C.c_uint32), ("transition_mask", C.c_uint32),
                ("hist_dev", C.c_void_p), ("do_report", C.c_int32), ("zero_hist", C.c_int32),
                ("dur_dev", C.c_void_p)]


class RmPointsDesc(C.Structure):
    _fields_ = [("n_points", C.c_uint64), ("uuid", C.c_void_p), ("time", C.c_void_p), ("lon", C.c_void_p),
                ("lat", C.c_void_p), ("accuracy", C.c_void_p), ("inactivity_sec", C.c_double),
                ("n_uuids", C.c_uint32), ("n_opts", C.c_uint32), ("opts", C.c_void_p), ("uuid_opt", C.c_void_p)]


class RmReportDesc(C.Structure):
    _fields_ = [("n_traces", C.c_uint32), ("seg_off", C.c_void_p), ("segs", C.c_void_p),
                ("trace_end_time", C.c_void_p), ("threshold_sec", C.c_void_p), ("report_mask", C.c_void_p),
                ("transition_mask", C.c_void_p)]


class RmTileParams(C.Structure):
    _fields_ = [("quantisation", C.c_uint32), ("privacy", C.c_uint32), ("source", C.c_char_p), ("mode", C.c_char_p)]


P = C.c_void_p
U32P = C.POINTER(C.c_uint32)

# (name, restype, argtypes) — every symbol declared in include/reporter_match.h
PROTOTYPES = [
    ("rm_last_error", C.c_char_p, []),
    ("rm_abi_version", C.c_int, []),
    ("rm_set_device", C.c_int, [C.c_int]),
    ("rm_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("rm_configure", C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
    ("rm_matcher_create", P, []),
    ("rm_matcher_destroy", None, [P]),
    ("rm_match", C.c_int, [P, C.c_char_p, C.POINTER(P)]),
    ("rm_match_batch", C.c_int, [P, C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(P)]),
    ("rm_match_batch_packed", C.c_int, [P, C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(P), C.POINTER(C.c_uint64)]),
    ("rm_free", None, [P]),
    ("rm_matcher_timing", C.c_int, [P, P]),
    ("rm_coalesce_stats", C.c_int, [C.POINTER(C.c_uint64)]),
    ("rm_coalesce_timing", C.c_int, [C.POINTER(C.c_double)]),
    ("rm_default_options", None, [C.POINTER(RmOptions)]),
    ("rm_default_world_params", None, [C.POINTER(RmWorldParams)]),
    ("rm_world_build", C.c_int, [C.POINTER(RmWorldParams), C.c_char_p]),
    ("rm_graph_info", C.c_int, [C.c_char_p, C.POINTER(C.c_uint64)]),
    ("rm_graph_export_osm", C.c_int, [C.c_char_p, C.c_char_p]),
    ("rm_graph_export_pbf", C.c_int, [C.c_char_p, C.c_char_p]),
    ("rm_graph_import_osm", C.c_int, [C.c_char_p, C.c_char_p, C.c_double]),
    ("rm_default_city_params", None, [C.POINTER(RmCityParams)]),
    ("rm_osm_city_write", C.c_int, [C.POINTER(RmCityParams), C.c_char_p, C.c_int]),
    ("rm_default_trace_params", None, [C.POINTER(RmTraceParams)]),
    ("rm_traces_generate", C.c_int, [C.c_char_p, C.POINTER(RmTraceParams), P, P, P, P, P, P]),
    ("rm_traces_generate_ids", C.c_int, [C.c_char_p, C.POINTER(RmTraceParams), P, P, P, P, P, P, P]),
    ("rm_engine_create", P, [C.c_char_p, C.c_int]),
    ("rm_engine_destroy", None, [P]),
    ("rm_engine_n_segments", C.c_uint32, [P]),
    ("rm_engine_segment_ids", C.c_int, [P, P]),
    ("rm_engine_set_ball_radius", C.c_int, [P, C.c_double]),
    ("rm_engine_ball_stats", C.c_int, [P, C.c_int, P]),
    ("rm_engine_grid_split", C.c_int, [P, P]),
    ("rm_engine_grid_alt", C.c_int, [P, P, P]),
    ("rm_engine_turn_rows", C.c_int, [P, P, P]),
    ("rm_engine_ball_lookup", C.c_int, [P, C.c_int, C.c_uint64, P, P, P, P]),
    ("rm_runner_route_tiers", C.c_int, [P, P]),
    ("rm_balls_lookup", C.c_int, [C.c_char_p, C.c_int, C.c_double, C.c_uint64, P, P, P, P]),
    ("rm_graph_auto_ball_radius", C.c_int, [C.c_char_p, P]),
    ("rm_graph_fit_ball_radius", C.c_int, [C.c_char_p, C.c_int, C.c_double, C.c_double, P]),
    ("rm_graph_ball_sample", C.c_int, [C.c_char_p, C.c_int, C.c_double, P]),
    ("rm_graph_grid_split", C.c_int, [C.c_char_p, P]),
    ("rm_runner_create", P, [P]),
    ("rm_runner_destroy", None, [P]),
    ("rm_default_run_params", None, [C.POINTER(RmRunParams)]),
    ("rm_runner_run", C.c_int, [P, C.POINTER(RmBatchDesc), C.POINTER(RmRunParams)]),
    ("rm_runner_rerun", C.c_int, [P, C.POINTER(RmRunParams)]),
    ("rm_runners_rerun", C.c_int, [P, C.c_uint32, C.POINTER(RmRunParams)]),
    ("rm_runner_sizes", C.c_int, [P, C.POINTER(C.c_uint64)]),
    ("rm_runner_get_states", C.c_int, [P, P, P]),
    ("rm_runner_get_candidates", C.c_int, [P, P, P, P, P]),
    ("rm_runner_get_routes", C.c_int, [P, P, P, P]),
    ("rm_runner_get_route_terms", C.c_int, [P, P, P]),
    ("rm_runner_get_viterbi", C.c_int, [P, P, P]),
    ("rm_runner_get_paths", C.c_int, [P, P, P, P, P]),
    ("rm_runner_get_segments", C.c_int, [P, P, P]),
    ("rm_runner_get_reports", C.c_int, [P, P, P, P]),
    ("rm_runner_set_timing", C.c_int, [P, C.c_int]),
    ("rm_runner_set_timing_mask", C.c_int, [P, C.c_uint32]),
    ("rm_runner_set_isolation", C.c_int, [P, C.c_int]),
    ("rm_runner_trace_errors", C.c_int, [P, P]),
    ("rm_runner_set_locality", C.c_int, [P, C.c_int]),
    ("rm_runner_locality_used", C.c_int, [P, C.POINTER(C.c_int)]),
    ("rm_report_segments", C.c_int, [C.POINTER(RmReportDesc), P, P, P]),
    ("rm_runner_kernel_times", C.c_int, [P, P, P, C.c_int]),
    ("rm_runner_reset_times", C.c_int, [P]),
    ("rm_kernel_name", C.c_char_p, [C.c_int]),
    ("rm_num_kernels", C.c_int, []),
    ("rm_runner_run_points", C.c_int, [P, C.POINTER(RmPointsDesc), C.POINTER(RmRunParams)]),
    ("rm_runner_get_trace_uuid", C.c_int, [P, P]),
    ("rm_runner_get_batch", C.c_int, [P, P, P, P, P, P]),
    ("rm_default_tile_params", None, [C.POINTER(RmTileParams)]),
    ("rm_runner_tiles", C.c_int, [P, C.POINTER(RmTileParams), P, C.POINTER(P), C.POINTER(C.c_size_t)]),
    ("rm_comm_unique_id", C.c_int, [P]),
    ("rm_comm_init", P, [C.c_int, C.c_int, P, C.c_int]),
    ("rm_comm_destroy", None, [P]),
    ("rm_comm_allreduce", C.c_int, [P, P, C.c_size_t, C.c_int, C.c_int]),
    ("rm_comm_reduce_scatter", C.c_int, [P, P, C.c_size_t, C.c_int, C.c_int]),
    ("rm_comm_allreduce_host_f64", C.c_int, [P, C.POINTER(C.c_double), C.c_int]),
    ("rm_comm_barrier", C.c_int, [P]),
    ("rm_comm_init_host", P, [C.c_int, C.c_int, P, P, C.c_int]),
    ("rm_tile_file_owner", C.c_int, [C.c_uint64, C.c_uint32, C.c_int]),
    ("rm_device_alloc", C.c_int, [C.c_size_t, C.POINTER(P)]),
    ("rm_device_free", C.c_int, [P]),
    ("rm_device_memset", C.c_int, [P, C.c_int, C.c_size_t]),
    ("rm_device_download", C.c_int, [P, P, C.c_size_t]),
    ("rm_device_upload", C.c_int, [P, P, C.c_size_t]),
    ("rm_device_synchronize", C.c_int, []),
]


def lib():
    """Load (once) and return the shared library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError("libreporter_match.so not built at %s (run python -m reporter_amd.build)" % LIB_PATH)
            h = C.CDLL(LIB_PATH)
            for name, res, args in PROTOTYPES:
                f = getattr(h, name)
                f.restype = res
                f.argtypes = args
            _lib = h
    return _lib


class RmError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise RmError(lib().rm_last_error().decode("utf-8", "replace"))
    return rc


def last_error():
    return lib().rm_last_error().decode("utf-8", "replace")
