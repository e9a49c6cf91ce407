"""ctypes binding of libmahout_cms.so (include/mahout_cms.h).

The product path has exactly one implementation: the gfx950 HIP library.  If
the in-tree shared object is missing this module raises -- there is no CPU
fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("MAHOUT_CMS_LIB") or os.path.join(HERE, "libmahout_cms.so")  # override: experiments

# status codes (include/mahout_cms.h)
CMS_ABI_VERSION = 2  # include/mahout_cms.h CMS_ABI_VERSION: the layout of the structs below
CMS_OK = 0
CMS_E_PARAM = 1
CMS_E_SHAPE = 2
CMS_E_NO_SUCH_ID = 3
CMS_E_STATE = 4
CMS_E_VALUE = 5
CMS_E_OVERFLOW = 6
CMS_E_HIP = 7
CMS_E_RCCL = 8
CMS_E_OOM = 9
CMS_E_SKETCH = 10

CMS_COUNTER_U32 = 0
CMS_COUNTER_F64 = 1
CMS_FORMAT_ITEM_SIMILARITY_JOB = 1
CMS_FORMAT_SPARK_ITEMSIMILARITY = 2
CMS_UNWEIGHTED = 0
CMS_WEIGHTED = 1
CMS_FLAG_COLLECTIVE_SINGLE_RANK = 0x1

# Every symbol the header declares (checked by tests/test_abi.py).
EXPORTS = [
    "cms_params_init", "cms_shape_from_delta_epsilon", "cms_create", "cms_destroy", "cms_last_error",
    "cms_abi_version", "cms_set_owner_ids", "cms_hash_params", "cms_hash_keys", "cms_ingest",
    "cms_ingest_device_rows", "cms_ingest_csr", "cms_ingest_csr_device", "cms_reset", "cms_release_scratch",
    "cms_comm_unique_id",
    "cms_comm_init", "cms_shard_of_key", "cms_finalize", "cms_synchronize", "cms_wait_stream", "cms_release_to_stream", "cms_similarity", "cms_similarities",
    "cms_point_query", "cms_estimate_preferences", "cms_most_similar", "cms_top_k_rows", "cms_top_k_all", "cms_top_k_all_partial", "cms_top_k_merge", "cms_write_similar_items", "cms_format_java_double", "cms_read_counters", "cms_get_stats",
    "cms_set_timing", "cms_get_timing", "cms_reset_timing",
    "cms_create_per_owner", "cms_configure_owner_shapes", "cms_set_owner_delta_epsilon", "cms_get_owner_shapes",
    "cms_read_owner_sketch", "cms_finalize_with", "cms_write_similarities", "cms_write_similarities_threshold",
    "cms_comm_init_transport", "cms_read_counters_device", "cms_owner_forms", "cms_estimate_preferences_batch", "cms_top_k_refresh", "cms_refresh_stats", "cms_refresh_classes",
    "cms_top_k_all_device", "cms_top_k_refresh_device", "cms_set_hash_params", "cms_recommend_batch",
]


class CmsParams(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("depth", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("counter_type", ctypes.c_int32),
        ("seed", ctypes.c_int64),
        ("num_owners", ctypes.c_int64),
        ("weighting", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("frac_bits", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


class CmsStats(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("pairs_ingested", ctypes.c_int64),
        ("num_owners", ctypes.c_int64),
        ("depth", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("exact_norms", ctypes.c_int32),
        ("world", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("table_bytes", ctypes.c_int64),
        ("multi_limb_owners", ctypes.c_int64),
        ("topk_redo", ctypes.c_int64),
        ("deep_limb_owners", ctypes.c_int64),
        ("fp4_owners", ctypes.c_int64),
        ("merge_words", ctypes.c_int64),
        ("hot_rows", ctypes.c_int64),
        ("stored_bytes", ctypes.c_int64),
        ("u8_rows", ctypes.c_int64),
        ("nibble_rows", ctypes.c_int64),
        ("crumb_rows", ctypes.c_int64),
        ("bit_rows", ctypes.c_int64),
        ("collective_calls", ctypes.c_int64),
        ("comm_kind", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("list_rows", ctypes.c_int64),
        ("po_wide_pairs", ctypes.c_int64),
        ("po_wide_exact", ctypes.c_int64),
    ]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_int = ctypes.c_int
_dbl = ctypes.c_double

# int (*cms_allreduce_fn)(void* d_buf, int64_t count, void* user)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
# int (*cms_allgather_fn)(const void* d_send, void* d_recv, int64_t bytes, void* user)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)

_SIGS = {
    "cms_params_init": (_int, [ctypes.POINTER(CmsParams)]),
    "cms_shape_from_delta_epsilon": (_int, [_dbl, _dbl, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "cms_create": (_int, [ctypes.POINTER(CmsParams), ctypes.POINTER(_vp)]),
    "cms_destroy": (None, [_vp]),
    "cms_last_error": (ctypes.c_char_p, []),
    "cms_abi_version": (_int, []),
    "cms_set_owner_ids": (_int, [_vp, _vp, _i64]),
    "cms_hash_params": (_int, [_vp, _vp, _vp]),
    "cms_hash_keys": (_int, [_vp, _vp, _i64, _vp]),
    "cms_ingest": (_int, [_vp, _vp, _vp, _vp, _i64]),
    "cms_ingest_device_rows": (_int, [_vp, _vp, _vp, _vp, _i64]),
    "cms_ingest_csr": (_int, [_vp, _vp, _vp, _vp]),
    "cms_ingest_csr_device": (_int, [_vp, _vp, _vp, _vp]),
    "cms_reset": (_int, [_vp]),
    "cms_release_scratch": (_int, [_vp]),
    "cms_comm_unique_id": (_int, [_vp]),
    "cms_comm_init": (_int, [_vp, _vp, _i32, _i32]),
    "cms_shard_of_key": (_i32, [_i64, _i32]),
    "cms_finalize": (_int, [_vp]),
    "cms_synchronize": (_int, [_vp]),
    "cms_wait_stream": (_int, [_vp, _vp]),
    "cms_release_to_stream": (_int, [_vp, _vp]),
    "cms_similarity": (_int, [_vp, _i64, _i64, ctypes.POINTER(_dbl)]),
    "cms_similarities": (_int, [_vp, _i64, _vp, _i64, _vp]),
    "cms_point_query": (_int, [_vp, _i64, _i64, ctypes.POINTER(_dbl)]),
    "cms_most_similar": (_int, [_vp, _i64, _i32, _vp, _vp, ctypes.POINTER(_i32)]),
    "cms_top_k_rows": (_int, [_vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    "cms_estimate_preferences": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i32, ctypes.c_float, ctypes.c_float, _vp]),
    "cms_write_similar_items": (_int, [_vp, ctypes.c_char_p, _i32, _i32]),
    "cms_format_java_double": (_int, [ctypes.c_double, ctypes.c_char_p, _i32]),
    "cms_top_k_all_partial": (_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "cms_top_k_merge": (_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cms_top_k_all": (_int, [_vp, _i32, _vp, _vp, _vp]),
    "cms_top_k_refresh": (_int, [_vp, _i32, _vp, _vp, _vp]),
    "cms_top_k_all_device": (_int, [_vp, _i32, _vp, _vp, _vp]),
    "cms_set_hash_params": (_int, [_vp, _vp, _vp, _i32]),
    "cms_top_k_refresh_device": (_int, [_vp, _i32, _vp, _vp, _vp]),
    "cms_refresh_stats": (_int, [_vp, _vp, _vp, _vp]),
    "cms_refresh_classes": (_int, [_vp, _vp]),
    "cms_read_counters": (_int, [_vp, _i64, _i64, _vp]),
    "cms_get_stats": (_int, [_vp, ctypes.POINTER(CmsStats)]),
    "cms_set_timing": (_int, [_vp, _i32]),
    "cms_get_timing": (_int, [_vp, ctypes.c_char_p, ctypes.POINTER(_dbl), ctypes.POINTER(_i64)]),
    "cms_reset_timing": (_int, [_vp]),
    "cms_create_per_owner": (_int, [ctypes.POINTER(CmsParams), ctypes.POINTER(_vp)]),
    "cms_finalize_with": (_int, [_vp, _vp, _vp]),
    "cms_comm_init_transport": (_int, [_vp, _i32, _i32, _vp, _vp, _vp]),
    "cms_read_counters_device": (_int, [_vp, _i64, _i64, _vp]),
    "cms_owner_forms": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "cms_estimate_preferences_batch": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _int, ctypes.c_float, ctypes.c_float,
                                              _vp]),
    "cms_recommend_batch": (_int, [_vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _i32, _int, ctypes.c_float,
                                   ctypes.c_float, _vp, _vp, _vp]),
    "cms_write_similarities": (_int, [_vp, ctypes.c_char_p, _i32, _i32]),
    "cms_write_similarities_threshold": (_int, [_vp, ctypes.c_char_p, _i32, _i32, ctypes.c_double]),
    "cms_configure_owner_shapes": (_int, [_vp, _dbl, _i64]),
    "cms_set_owner_delta_epsilon": (_int, [_vp, _vp, _vp]),
    "cms_get_owner_shapes": (_int, [_vp, _vp, _vp, _vp, _vp]),
    "cms_read_owner_sketch": (_int, [_vp, _i64, _vp, _i64, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
}

_lib = None


def load():
    """Load the in-tree gfx950 library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(SO_PATH):
        raise RuntimeError(
            f"{SO_PATH} is missing: build it with `python -m mahout_amd.build_lib` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    # torch (device-memory/stream plumbing for callers) ships its own
    # libamdhip64/librccl with the same SONAMEs; loading it first makes this
    # library bind to that one runtime instead of a second copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(SO_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the ctypes structs above mirror one header layout: a stale library (or
    # stale bindings) must fail here, not read cms_stats with the wrong shape
    got = lib.cms_abi_version()
    if got != CMS_ABI_VERSION:
        raise RuntimeError(f"{SO_PATH} has ABI version {got}, these bindings need {CMS_ABI_VERSION}: rebuild it "
                           "with `python -m mahout_amd.build_lib`")
    _lib = lib
    return lib


class CmsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(rc):
    if rc != CMS_OK:
        msg = load().cms_last_error()
        raise CmsError(rc, msg.decode() if msg else "")
    return rc
