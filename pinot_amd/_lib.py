"""ctypes binding of libpinotgpu.so (the C ABI in include/pinotgpu.h).

This is the same binding a Java maintainer writes with JNI/Panama; here it serves the
Python host layer, the tests and bench.py.  The product path has no CPU fallback: if the HIP library is
missing or fails to load, every entry point raises.
"""
import ctypes
import os

from .build import LIB_PATH

c_int = ctypes.c_int
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_f64p = ctypes.POINTER(ctypes.c_double)
c_voidp = ctypes.c_void_p
c_char_pp = ctypes.POINTER(ctypes.c_char_p)

PGPU_OK = 0
PGPU_ERR_INVALID_ARGUMENT = -1
PGPU_ERR_BAD_QUERY = -2
PGPU_ERR_UNSUPPORTED = -3
PGPU_ERR_DEVICE = -4
PGPU_ERR_OUT_OF_MEMORY = -5
PGPU_ERR_NOT_FOUND = -6
PGPU_ERR_TIMEOUT = -7
PGPU_ERR_CANCELLED = -8

INT, LONG, FLOAT, DOUBLE, STRING = 0, 1, 2, 3, 4
TYPE_NAMES = {"INT": INT, "LONG": LONG, "FLOAT": FLOAT, "DOUBLE": DOUBLE, "STRING": STRING}
FWD_FIXED_BIT, FWD_SORTED_PAIRS, FWD_RAW_FIXED = 0, 1, 2
PRED_EQ, PRED_NOT_EQ, PRED_IN, PRED_NOT_IN, PRED_RANGE = 0, 1, 2, 3, 4
OP_PRED, OP_AND, OP_OR, OP_NOT = 0, 1, 2, 3
LEAF_KIND_NAMES = ("none", "all", "range", "set", "docrange", "bitmap", "raw_range", "raw_in", "bitdir")
GROUP_PATH_NAMES = ("lds", "global", "hash", "partitioned", "hash_partitioned")  # enum pgpu_group_path
AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG = 0, 1, 2, 3, 4
SLOT_COUNT, SLOT_SUM_I64, SLOT_SUM_F64, SLOT_MIN_KEY, SLOT_MAX_KEY = 0, 1, 2, 3, 4
GEN_UNIFORM, GEN_ZIPF, GEN_TABLE = 0, 1, 2
COMM_RCCL, COMM_HOST = 0, 1
COMM_ID_BYTES = 128
COMBINE_LOCAL, COMBINE_ALL_REDUCE, COMBINE_REDUCE_SCATTER, COMBINE_HASH, COMBINE_ROWS = 0, 1, 2, 3, 4
COMBINE_NAMES = {COMBINE_LOCAL: "local", COMBINE_ALL_REDUCE: "all_reduce", COMBINE_REDUCE_SCATTER: "reduce_scatter",
                 COMBINE_HASH: "hash", COMBINE_ROWS: "rows"}


class ColumnBuffers(ctypes.Structure):
    _fields_ = [("cardinality", c_i32), ("bits_per_element", c_i32), ("entry_width", c_i32),
                ("padding_byte", c_i32), ("fwd_format", c_i32), ("reserved", c_i32),
                ("dict", c_voidp), ("dict_len", c_i64), ("fwd", c_voidp), ("fwd_len", c_i64)]


class SegmentDesc(ctypes.Structure):
    _fields_ = [("num_docs", c_i32), ("num_columns", c_i32), ("columns", ctypes.POINTER(ColumnBuffers))]


class PredicateC(ctypes.Structure):
    _fields_ = [("type", c_i32), ("column", c_i32), ("num_values", c_i32), ("lower_inclusive", c_i32),
                ("values", c_char_pp), ("upper_inclusive", c_i32), ("reserved", c_i32)]


# pgpu_leaf_type: Pinot's leaf operator of a predicate in one segment (pgpu_filter_entries_scanned)
OPT_NO_STAR_TREE = 1
OPT_SQL_GROUP_BY = 2
OPT_NO_PLAN_CACHE = 4
OPT_TIMING = 8
LEAF_EMPTY, LEAF_MATCH_ALL, LEAF_SCAN, LEAF_SORTED, LEAF_BITMAP, LEAF_RANGE_INDEX = 0, 1, 2, 3, 4, 5


ORDER_GROUP_BY, ORDER_AGGREGATION = 0, 1


class OrderByC(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("index", ctypes.c_int32), ("ascending", ctypes.c_int32)]


class SqlTrimC(ctypes.Structure):
    _fields_ = [("num_order_by", ctypes.c_int32), ("order_by", ctypes.POINTER(OrderByC)), ("limit", ctypes.c_int32),
                ("min_server_group_trim_size", ctypes.c_int32), ("group_trim_threshold", ctypes.c_int32),
                ("num_select", ctypes.c_int32), ("select", ctypes.POINTER(OrderByC))]


class FilterOpC(ctypes.Structure):
    _fields_ = [("op", c_i32), ("arg", c_i32)]


class AggC(ctypes.Structure):
    _fields_ = [("fn", c_i32), ("column", c_i32)]


class QueryC(ctypes.Structure):
    _fields_ = [("num_predicates", c_i32), ("num_filter_ops", c_i32), ("predicates", ctypes.POINTER(PredicateC)),
                ("filter", ctypes.POINTER(FilterOpC)), ("num_group_by", c_i32), ("num_aggs", c_i32),
                ("group_by", c_i32p), ("aggs", ctypes.POINTER(AggC)), ("num_groups_limit", c_i32),
                ("options", c_i32), ("end_time_ms", c_i64)]


class GenColumnC(ctypes.Structure):
    _fields_ = [("kind", c_i32), ("column_index", c_i32), ("lo", c_i64), ("hi", c_i64), ("n", c_i32),
                ("reserved", c_i32), ("cdf", c_f64p), ("ids", c_i64p), ("table", c_f64p)]


class StarTreeDescC(ctypes.Structure):
    _fields_ = [("num_dims", c_i32), ("num_metrics", c_i32), ("num_nodes", c_i32), ("num_docs", c_i32),
                ("dim_columns", c_i32p), ("nodes", c_u8p), ("dim_fwd", ctypes.POINTER(c_u8p)),
                ("dim_fwd_len", c_i64p), ("metrics", ctypes.POINTER(AggC)),
                ("metric_f64", ctypes.POINTER(c_f64p)), ("metric_i64", ctypes.POINTER(c_i64p))]


class ConfigC(ctypes.Structure):
    """pgpu_config (include/pinotgpu.h): a table's executor settings."""
    _fields_ = [("struct_size", ctypes.c_int32), ("plan_cache", ctypes.c_int32),
                ("partitioned_group_by", ctypes.c_int32), ("hash_partitions", ctypes.c_int32),
                ("hash_partition_bits", ctypes.c_int32), ("hash_partition_lds_kb", ctypes.c_int32),
                ("lds_table_kb", ctypes.c_int32), ("plan_chunk_segments", ctypes.c_int32),
                ("stream_chunks", ctypes.c_int32), ("compact_results", ctypes.c_int32),
                ("star_tree_workgroups", ctypes.c_int32), ("dense_selectivity", ctypes.c_double),
                ("slot_weight_step", ctypes.c_double)]


CONFIG_FIELDS = [f for f, _ in ConfigC._fields_ if f != "struct_size"]


class PinotGpuError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("pgpu error %d: %s" % (code, message))
        self.code = code
        self.message = message


class BadQueryRequestException(PinotGpuError):
    """PGPU_ERR_BAD_QUERY: mirrors org.apache.pinot.spi.exception.BadQueryRequestException."""


class UnsupportedQueryError(PinotGpuError):
    """PGPU_ERR_UNSUPPORTED: the query shape is outside the GPU path."""


class QueryCancelledError(PinotGpuError):
    """PGPU_ERR_CANCELLED: pgpu_plan_cancel abandoned the query (BaseOperator's EarlyTerminationException after the
    combine cancels its futures, BaseOperator.java:37-39 / BaseCombineOperator.java:124-130)."""


class QueryTimeoutError(PinotGpuError):
    """PGPU_ERR_TIMEOUT: the query's end time passed (the combine's TimeoutException; Pinot reports
    QueryException.EXECUTION_TIMEOUT_ERROR_CODE 250 for aggregation-only and QUERY_EXECUTION_ERROR_CODE 200 for
    group-by, BaseCombineOperator.java:193-203 / GroupByCombineOperator.java:193-203)."""


_PROTOS = {
    "pgpu_abi_version": (c_int, []),
    "pgpu_init": (c_int, [c_int]),
    "pgpu_shutdown": (c_int, []),
    "pgpu_last_error": (c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "pgpu_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "pgpu_table_create": (c_int, [c_int, c_int, c_char_pp, c_i32p, ctypes.POINTER(c_voidp)]),
    "pgpu_config_default": (c_int, [ctypes.POINTER(ConfigC)]),
    "pgpu_table_set_config": (c_int, [c_voidp, ctypes.POINTER(ConfigC)]),
    "pgpu_table_get_config": (c_int, [c_voidp, ctypes.POINTER(ConfigC)]),
    "pgpu_table_destroy": (c_int, [c_voidp]),
    "pgpu_pin_segment": (c_int, [c_voidp, ctypes.POINTER(SegmentDesc), c_i64p]),
    "pgpu_unpin_segment": (c_int, [c_voidp, c_i64]),
    "pgpu_table_num_segments": (c_int, [c_voidp, c_i32p]),
    "pgpu_table_device_bytes": (c_i64, [c_voidp]),
    "pgpu_table_add_dictionary_values": (c_int, [c_voidp, c_int, c_i64, c_i64p, c_f64p, c_u8p, c_i64p]),
    "pgpu_table_dictionary_size": (c_int, [c_voidp, c_int, c_i64p]),
    "pgpu_table_dictionary_i64": (c_int, [c_voidp, c_int, c_i64p]),
    "pgpu_table_dictionary_f64": (c_int, [c_voidp, c_int, c_f64p]),
    "pgpu_table_dictionary_str": (c_int, [c_voidp, c_int, c_u8p, c_i64, c_i64p]),
    "pgpu_read_dict_ids": (c_int, [c_voidp, c_i64, c_int, c_i32p, c_i32, c_i32p]),
    "pgpu_unpack_fixed_bit_device": (c_int, [c_voidp, c_i64, c_i32, c_i64, c_i64, c_voidp, c_voidp]),
    "pgpu_plan_create": (c_int, [c_voidp, c_i64p, c_i32, ctypes.POINTER(QueryC), ctypes.POINTER(c_voidp)]),
    "pgpu_plan_destroy": (c_int, [c_voidp]),
    "pgpu_plan_create_execute": (c_int, [c_voidp, c_i64p, c_i32, ctypes.POINTER(QueryC), c_voidp, c_voidp,
                                         ctypes.POINTER(c_voidp)]),
    "pgpu_plan_layout": (c_int, [c_voidp, c_i32p, c_i64p, c_i32p]),
    "pgpu_plan_leaf_kinds": (c_int, [c_voidp, c_i64p]),
    "pgpu_plan_group_path": (c_int, [c_voidp, c_i32p]),
    "pgpu_plan_cancel": (c_int, [c_voidp]),
    "pgpu_plan_execute": (c_int, [c_voidp, c_voidp, c_voidp]),
    "pgpu_plan_finalize": (c_int, [c_voidp, c_voidp, c_voidp, ctypes.POINTER(c_voidp)]),
    "pgpu_plan_finalize_range": (c_int, [c_voidp, c_voidp, c_voidp, c_i64, c_i64, ctypes.POINTER(c_voidp)]),
    "pgpu_plan_exchange_counts": (c_int, [c_voidp, c_voidp, c_i32, c_i64p]),
    "pgpu_plan_exchange_export": (c_int, [c_voidp, c_voidp, c_i32, c_i32p, c_voidp, c_i64]),
    "pgpu_plan_exchange_merge": (c_int, [c_voidp, c_voidp, c_i32p, c_voidp, c_i64]),
    "pgpu_execute_groupby": (c_int, [c_voidp, c_i64p, c_i32, ctypes.POINTER(QueryC), c_voidp,
                                     ctypes.POINTER(c_voidp)]),
    "pgpu_plan_timing": (c_int, [c_voidp, c_f64p]),
    "pgpu_plan_star_work": (c_int, [c_voidp, c_i64p]),
    "pgpu_plan_star_metric_bytes": (c_int, [c_voidp, c_i64p]),
    "pgpu_plan_scanned_segments": (c_int, [c_voidp, c_u8p]),
    "pgpu_attach_startree": (c_int, [c_voidp, c_i64, ctypes.POINTER(StarTreeDescC)]),
    "pgpu_attach_inverted_index": (c_int, [c_voidp, c_i64, c_i32, c_voidp, c_i64]),
    "pgpu_inverted_index_check": (c_int, [c_voidp, c_i64, c_i32, c_i32, c_voidp]),
    "pgpu_build_inverted_index": (c_int, [c_voidp, c_i64, c_i32, c_i32, c_i32, c_voidp, c_i64, c_i64p]),
    "pgpu_raw_forward_index_values": (c_int, [c_voidp, c_i64, c_i32, c_i32, c_i64p, c_f64p]),
    "pgpu_startree_build": (c_int, [ctypes.POINTER(SegmentDesc), c_i32p, c_i32p, c_i32, c_i32p, c_i32,
                                    ctypes.POINTER(AggC), c_i32, c_i32, ctypes.POINTER(c_voidp)]),
    "pgpu_startree_load": (c_int, [c_voidp, c_i64, ctypes.c_char_p, c_i64, c_i32, c_i32, c_i32, c_char_pp, c_i32p,
                                   ctypes.POINTER(c_voidp)]),
    "pgpu_startree_get_desc": (c_int, [c_voidp, ctypes.POINTER(StarTreeDescC)]),
    "pgpu_startree_num_raw_records": (c_int, [c_voidp, c_i32p]),
    "pgpu_startree_destroy": (c_int, [c_voidp]),
    "pgpu_result_num_groups": (c_int, [c_voidp, c_i64p]),
    "pgpu_result_key_dictionary": (c_int, [c_voidp, c_int, c_u64p, c_i64p]),
    "pgpu_result_key_dictionary_i64": (c_int, [c_voidp, c_int, c_i64p]),
    "pgpu_result_key_dictionary_f64": (c_int, [c_voidp, c_int, c_f64p]),
    "pgpu_result_key_dictionary_str": (c_int, [c_voidp, c_int, c_u8p, c_i64, c_i64p]),
    "pgpu_result_group_ids": (c_int, [c_voidp, c_i32p]),
    "pgpu_result_group_ids_column": (c_int, [c_voidp, c_int, c_i32p]),
    "pgpu_result_group_ids_view": (c_int, [c_voidp, c_int, ctypes.POINTER(c_voidp)]),
    "pgpu_result_words_view": (c_int, [c_voidp, c_int, ctypes.POINTER(c_voidp), c_i32p]),
    "pgpu_result_values": (c_int, [c_voidp, c_int, c_f64p]),
    "pgpu_result_avg_counts": (c_int, [c_voidp, c_int, c_i64p]),
    "pgpu_result_values_i64": (c_int, [c_voidp, c_int, c_i64p]),
    "pgpu_result_stats": (c_int, [c_voidp, c_i64p]),
    "pgpu_result_groups_limit_reached": (c_int, [c_voidp, ctypes.POINTER(ctypes.c_int32)]),
    "pgpu_result_slot_kinds": (c_int, [c_voidp, c_i32p, c_i32p]),
    "pgpu_result_exchange_rows": (c_int, [c_voidp, c_i32, c_i32p, c_i64p, c_i64p]),
    "pgpu_result_merge_rows": (c_int, [c_voidp, c_i64p, c_i64, c_i32p, ctypes.POINTER(c_voidp)]),
    "pgpu_result_destroy": (c_int, [c_voidp]),
    "pgpu_comm_unique_id": (c_int, [c_i32, c_voidp]),
    "pgpu_comm_create": (c_int, [c_i32, c_voidp, c_i32, c_i32, c_i32, ctypes.POINTER(c_voidp)]),
    "pgpu_comm_destroy": (c_int, [c_voidp]),
    "pgpu_comm_rank": (c_int, [c_voidp, c_i32p, c_i32p]),
    "pgpu_comm_allgather": (c_int, [c_voidp, c_voidp, c_i64, c_voidp]),
    "pgpu_comm_set_timeout": (c_int, [c_voidp, c_i64]),
    "pgpu_comm_abort": (c_int, [c_voidp]),
    "pgpu_comm_status": (c_int, [c_voidp, c_i32p]),
    "pgpu_attach_range_index": (c_int, [c_voidp, c_i64, c_i32, c_voidp, c_i64]),
    "pgpu_range_index_check": (c_int, [c_voidp, c_i64, c_i32, c_i32, c_i32p, c_i32p, c_i64p]),
    "pgpu_range_index_partial_entries": (c_int, [c_voidp, c_i64, c_i32, c_i32, c_i32, c_i32, c_i64p]),
    "pgpu_comm_recreate": (c_int, [c_voidp, c_voidp]),
    "pgpu_plan_combine_mode": (c_int, [c_voidp, c_voidp, c_i64, c_i32p, c_i32p]),
    "pgpu_plan_combine": (c_int, [c_voidp, c_voidp, c_voidp, c_voidp, c_i32, c_i32p, c_voidp, c_i64p, c_i64p]),
    "pgpu_result_combine_rows": (c_int, [c_voidp, c_voidp, ctypes.POINTER(c_voidp)]),
    "pgpu_free_result": (c_int, [c_voidp]),
    "pgpu_filter_bitmap": (c_int, [c_voidp, c_i64, ctypes.POINTER(QueryC), c_u64p]),
    "pgpu_result_trim_sql": (c_int, [c_voidp, ctypes.POINTER(SqlTrimC), ctypes.POINTER(c_voidp)]),
    "pgpu_result_trim_pql": (c_int, [c_voidp, c_i32, c_i32, c_i64p, c_i64, c_i64p]),
    "pgpu_result_datatable": (c_int, [c_voidp, c_voidp, c_voidp, c_i64, c_i64p]),
    "pgpu_broker_reduce_sql": (c_int, [ctypes.POINTER(c_voidp), c_i64p, c_i32, ctypes.POINTER(SqlTrimC), c_voidp,
                                       c_i64, c_i64p]),
    "pgpu_filter_entries_scanned": (c_int, [ctypes.POINTER(FilterOpC), c_i32, c_i32p, ctypes.POINTER(c_voidp), c_i32,
                                            c_i32, c_i64p]),
    "pgpu_generate_segment": (c_int, [c_voidp, ctypes.POINTER(GenColumnC), c_i32, c_i64, c_i32, c_i64p]),
    "pgpu_segment_column_info": (c_int, [c_voidp, c_i64, c_int, c_i32p, c_i32p, c_i64p, c_i64p]),
    "pgpu_segment_column_bytes": (c_int, [c_voidp, c_i64, c_int, c_u8p, c_u8p]),
}

_lib = None


def exported_symbols():
    return sorted(_PROTOS)


def load(path=None):
    """Loads libpinotgpu.so (dlopen only: no GPU call is made)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("PGPU_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise ImportError("libpinotgpu.so is not built (%s); run `python -m pinot_amd.build` "
                          "or __graft_entry__.build()" % p)
    try:
        # One HIP runtime per process: when PyTorch is present its bundled libamdhip64.so.7 must be the one the
        # dynamic linker resolves for this library too (loading the system copy first breaks torch.cuda).
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    # an A/B build of an earlier tree (PGPU_LIB, scripts/ab_lib.sh) may lack entry points added since; the
    # in-tree library must export every one
    ab = os.path.abspath(p) != os.path.abspath(LIB_PATH)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name, None)
        if fn is None and ab:
            continue
        if fn is None:
            raise ImportError("libpinotgpu.so does not export %s (rebuild it)" % name)
        fn.restype = res
        fn.argtypes = args
    if lib.pgpu_abi_version() != 3:
        raise ImportError("libpinotgpu.so ABI mismatch")
    if path is None:
        _lib = lib
    return lib


def last_error():
    lib = load()
    buf = ctypes.create_string_buffer(2048)
    lib.pgpu_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(code):
    if code == PGPU_OK:
        return
    msg = last_error()
    if code == PGPU_ERR_BAD_QUERY:
        raise BadQueryRequestException(code, msg)
    if code == PGPU_ERR_UNSUPPORTED:
        raise UnsupportedQueryError(code, msg)
    if code == PGPU_ERR_CANCELLED:
        raise QueryCancelledError(code, msg)
    if code == PGPU_ERR_TIMEOUT:
        raise QueryTimeoutError(code, msg)
    raise PinotGpuError(code, msg)


def ptr(arr, ctype):
    """Pointer to a numpy array's data (keeps no reference: the caller holds the array)."""
    return arr.ctypes.data_as(ctypes.POINTER(ctype))
