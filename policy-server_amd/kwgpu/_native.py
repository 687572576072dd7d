"""ctypes declarations of include/kwgpu.h (libkwgpu.so) and of libkwsynth.so.

The product library is loaded from the package directory (built in-tree by
``__graft_entry__.build()``); a missing library raises immediately — there is no Python or CPU
fallback for the hot path.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# KWGPU_LIB selects another in-tree build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("KWGPU_LIB") or os.path.join(PKG_DIR, "libkwgpu.so")
SYNTH_PATH = os.path.join(PKG_DIR, "libkwsynth.so")

# status codes (kwgpu.h)
KW_OK = 0
KW_E_INVALID_ID = 1
KW_E_INIT = 2
KW_E_NOT_FOUND = 3
KW_E_BOOTSTRAP = 4
KW_E_ENGINE = 5
KW_E_GROUP_REHYDRATE = 6
KW_E_ARG = 16
KW_E_PAYLOAD = 17
KW_E_DEVICE = 18
KW_E_NOSPACE = 19

KW_MODE_PROTECT = 0
KW_MODE_MONITOR = 1
KW_ORIGIN_VALIDATE = 0
KW_ORIGIN_AUDIT = 1
KW_DOC_ADMISSION_REVIEW = 0
KW_DOC_RAW_REVIEW = 1

KW_V_ALLOWED = 0x1
KW_V_MUTATED = 0x2
KW_F_ALLOWED = 0x4
KW_F_STATUS_SHIFT = 3
KW_F_STATUS_MASK = 0x18
KW_BYPASS = 0x20
KW_F_PATCH = 0x40
KW_FST_NONE, KW_FST_VANILLA, KW_FST_MUTATION_REFUSED, KW_FST_INIT_ERROR = 0, 1, 2, 3
KW_ARG_WIDE = 0xFFFF

REASONS = {
    0: "NONE", 1: "PRIVILEGED", 2: "NAMESPACE", 3: "REG_NOT_ALLOWED", 4: "REG_REJECTED",
    5: "TAG_REJECTED", 6: "IMG_NOT_ALLOWED", 7: "IMG_REJECTED", 8: "CAP_NOT_ALLOWED",
    9: "APPARMOR", 10: "LABEL_DENIED", 11: "LABEL_CONSTRAINT", 12: "LABEL_MANDATORY",
    13: "GROUP", 14: "GROUP_EXPR", 15: "INIT_ERROR",
}


class KwStrcol(C.Structure):
    _fields_ = [("off", C.POINTER(C.c_uint32)), ("bytes", C.POINTER(C.c_uint8)), ("n", C.c_uint64)]


class KwSoa(C.Structure):
    _fields_ = [
        ("n_requests", C.c_uint64),
        ("req_flags", C.POINTER(C.c_uint8)),
        ("ctr_off", C.POINTER(C.c_uint32)),
        ("lbl_off", C.POINTER(C.c_uint32)),
        ("uid", KwStrcol), ("ns", KwStrcol), ("op", KwStrcol), ("kind", KwStrcol),
        ("ctr_flags", C.POINTER(C.c_uint8)),
        ("capadd_off", C.POINTER(C.c_uint32)),
        ("capdrop_off", C.POINTER(C.c_uint32)),
        ("ctr_name", KwStrcol), ("ctr_image", KwStrcol), ("ctr_apparmor", KwStrcol),
        ("cap_add", KwStrcol), ("cap_drop", KwStrcol),
        ("lbl_key", KwStrcol), ("lbl_val", KwStrcol),
    ]


class KwEnvOptions(C.Structure):
    _fields_ = [("continue_on_errors", C.c_int), ("always_accept_namespace", C.c_char_p), ("device", C.c_int)]


class KwTiming(C.Structure):
    _fields_ = [("classify_ms", C.c_double), ("evaluate_ms", C.c_double), ("total_ms", C.c_double),
                ("classify_bytes", C.c_double), ("evaluate_bytes", C.c_double)]


EXPORTS = [
    "kw_env_build", "kw_env_build_yaml", "kw_yaml_to_json", "kw_env_serialize", "kw_env_deserialize", "kw_env_destroy", "kw_env_lookup",
    "kw_env_policy_count", "kw_env_policy_id", "kw_env_is_group", "kw_env_get_policy_mode",
    "kw_env_get_policy_allowed_to_mutate",
    "kw_env_should_always_accept_requests_made_inside_of_namespace",
    "kw_env_policy_initialization_error", "kw_env_validate_settings", "kw_pattern_match", "kw_pattern_match_many", "kw_env_pattern_count",
    "kw_env_pattern", "kw_env_classify", "kw_batch_wide_arg", "kw_batch_group_causes", "kw_debug_plan", "kw_debug_reorder",
    "kw_batch_from_json", "kw_batch_from_soa", "kw_batch_view", "kw_batch_to_device", "kw_batch_to_device_async",
    "kw_stream_create", "kw_stream_destroy", "kw_validate_host", "kw_batch_pin_host", "kw_host_alloc", "kw_host_free",
    "kw_batch_destroy", "kw_debug_host_walk", "kw_validate_batch", "kw_validate_rows", "kw_batch_verdicts",
    "kw_validate_timed", "kw_format_response", "kw_format_response_doc", "kw_env_group_members", "kw_evaluate",
    "kw_service_constraints", "kw_metrics_create", "kw_metrics_destroy", "kw_metrics_record", "kw_metrics_render",
    "kw_metrics_reset", "kw_version",
]

_lib = None
_synth = None


def lib():
    """The product library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    # One HIP runtime per process. The torch wheel bundles its own libamdhip64 (soname
    # libamdhip64.so.7, needed by torch as "libamdhip64.so"): loaded first, it also serves this
    # library's libamdhip64.so.7; loaded after /opt/rocm's, it is a second runtime that then finds
    # no GPU ("No HIP GPUs are available" on the caller's first torch stream). So torch goes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u32, u64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_uint32, C.c_uint64
    cp, ip = C.c_char_p, C.c_int
    sig = {
        "kw_env_build": (ip, [cp, sz, C.POINTER(KwEnvOptions), C.POINTER(vp), cp, sz]),
        "kw_env_build_yaml": (ip, [cp, sz, C.POINTER(KwEnvOptions), C.POINTER(vp), cp, sz]),
        "kw_yaml_to_json": (ip, [cp, sz, cp, sz, C.POINTER(sz)]),
        "kw_env_serialize": (ip, [vp, vp, sz, C.POINTER(sz)]),
        "kw_env_deserialize": (ip, [vp, sz, ip, C.POINTER(vp), cp, sz]),
        "kw_env_destroy": (None, [vp]),
        "kw_env_lookup": (ip, [vp, cp, sz, C.POINTER(i32)]),
        "kw_env_policy_count": (ip, [vp]),
        "kw_env_policy_id": (ip, [vp, i32, cp, sz]),
        "kw_env_is_group": (ip, [vp, i32]),
        "kw_env_get_policy_mode": (ip, [vp, i32, C.POINTER(ip)]),
        "kw_env_get_policy_allowed_to_mutate": (ip, [vp, i32, C.POINTER(ip)]),
        "kw_env_should_always_accept_requests_made_inside_of_namespace": (ip, [vp, cp, sz]),
        "kw_env_policy_initialization_error": (ip, [vp, i32, cp, sz]),
        "kw_env_validate_settings": (ip, [vp, i32, cp, sz]),
        "kw_pattern_match": (ip, [ip, cp, cp, sz]),
        "kw_pattern_match_many": (ip, [ip, cp, C.POINTER(cp), C.POINTER(sz), sz, C.POINTER(C.c_int32)]),
        "kw_env_pattern_count": (ip, [vp, ip]),
        "kw_env_pattern": (ip, [vp, ip, ip, C.POINTER(ip), cp, sz]),
        "kw_env_classify": (ip, [vp, ip, cp, sz, cp, sz, C.POINTER(u32), ip]),
        "kw_batch_wide_arg": (ip, [vp, u64, i32, C.POINTER(u64)]),
        "kw_batch_group_causes": (ip, [vp, u64, i32, C.c_uint32, C.POINTER(u64), C.c_size_t, C.POINTER(C.c_size_t)]),
        "kw_debug_plan": (ip, [vp, vp, C.POINTER(i32), u32, ip, C.POINTER(u32), ip]),
        "kw_debug_reorder": (ip, [vp, C.POINTER(u64), sz, C.POINTER(u64), C.POINTER(vp)]),
        "kw_batch_from_json": (ip, [C.POINTER(cp), C.POINTER(sz), sz, ip, C.POINTER(vp), C.POINTER(C.c_int64), cp, sz]),
        "kw_batch_from_soa": (ip, [C.POINTER(KwSoa), C.POINTER(vp)]),
        "kw_batch_view": (ip, [vp, C.POINTER(KwSoa)]),
        "kw_batch_to_device": (ip, [vp, ip]),
        "kw_batch_to_device_async": (ip, [vp, ip, vp]),
        "kw_stream_create": (ip, [ip, C.POINTER(vp)]),
        "kw_stream_destroy": (None, [vp]),
        "kw_batch_destroy": (None, [vp]),
        "kw_validate_batch": (ip, [vp, vp, C.POINTER(i32), u32, ip, vp]),
        "kw_validate_rows": (ip, [vp, vp, C.POINTER(i32), ip, vp]),
        "kw_batch_verdicts": (ip, [vp, C.POINTER(u32), sz]),
        "kw_validate_host": (ip, [vp, vp, C.POINTER(i32), u32, ip, ip, C.POINTER(u32), sz, u32]),
        "kw_batch_pin_host": (ip, [vp, ip]),
        "kw_host_alloc": (ip, [ip, sz, C.POINTER(vp)]),
        "kw_host_free": (None, [vp]),
        "kw_debug_host_walk": (ip, [vp, vp, C.POINTER(i32), u32, ip, C.POINTER(u32)]),
        "kw_validate_timed": (ip, [vp, vp, C.POINTER(i32), u32, ip, ip, ip, C.POINTER(KwTiming)]),
        "kw_format_response": (ip, [vp, vp, u64, i32, u32, C.POINTER(u32), cp, sz, C.POINTER(sz)]),
        "kw_format_response_doc": (ip, [vp, vp, u64, i32, u32, C.POINTER(u32), cp, sz, ip, cp, sz, C.POINTER(sz)]),
        "kw_env_group_members": (ip, [vp, i32, C.POINTER(i32), ip]),
        "kw_evaluate": (ip, [vp, cp, cp, sz, ip, ip, cp, sz, C.POINTER(sz)]),
        "kw_service_constraints": (ip, [u32, ip, ip, C.POINTER(u32)]),
        "kw_metrics_create": (vp, []),
        "kw_metrics_destroy": (None, [vp]),
        "kw_metrics_record": (ip, [vp, vp, vp, C.POINTER(u64), C.POINTER(i32), C.POINTER(u32), C.POINTER(u64), sz, ip]),
        "kw_metrics_render": (ip, [vp, cp, sz, C.POINTER(sz)]),
        "kw_metrics_reset": (None, [vp]),
        "kw_version": (cp, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def synth():
    """libkwsynth.so (bench / test workload generator)."""
    global _synth
    if _synth is not None:
        return _synth
    if not os.path.exists(SYNTH_PATH):
        raise ImportError(f"{SYNTH_PATH} is missing: run __graft_entry__.build()")
    S = C.CDLL(SYNTH_PATH)
    S.kws_generate.restype = C.c_void_p
    S.kws_generate.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64]
    S.kws_free.restype = None
    S.kws_free.argtypes = [C.c_void_p]
    S.kws_view.restype = C.c_int
    S.kws_view.argtypes = [C.c_void_p, C.POINTER(KwSoa)]
    S.kws_json.restype = C.c_int
    S.kws_json.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
    S.kws_shard_bounds.restype = C.c_int
    S.kws_shard_bounds.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_uint64)]
    S.kws_row_containers.restype = C.c_int
    S.kws_row_containers.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
    _synth = S
    return S
