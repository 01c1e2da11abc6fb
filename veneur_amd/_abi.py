"""ctypes binding of include/veneur_amd.h and include/veneur_amd_synth.h.

The shared library is built in-tree (veneur_amd/libveneur_amd.so, `make -C veneur_amd`
or __graft_entry__.build()).  There is no fallback: if the HIP library is missing the
import fails.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# VN_LIB selects a variant built from the same sources (tools only: the profiling build)
LIB_PATH = os.path.join(HERE, os.environ.get("VN_LIB", "libveneur_amd.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "veneur_amd: %s is missing -- build the HIP engine first (make -C veneur_amd, or "
        "python -c 'import __graft_entry__; __graft_entry__.build()')" % LIB_PATH)



def _share_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm wheels bundle their own libamdhip64 and
    libhsa-runtime64 under the same sonames as /opt/rocm's.  Whichever copy loads first wins
    the soname; if the engine loads /opt/rocm's first, torch later loads its bundled copy as a
    second runtime, whose KFD open fails ("No HIP GPUs are available").  When torch is
    installed (dist.py uses it for RCCL), bind the engine to torch's runtime by loading that
    copy first -- without importing torch.  A Go host has no torch and links
    /opt/rocm's runtime as usual."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


_share_torch_hip_runtime()
lib = C.CDLL(LIB_PATH)

VN_OK, VN_EINVAL, VN_EHIP, VN_ENOMEM, VN_EDECODE = 0, -1, -2, -3, -4
VN_DT_U8, VN_DT_U32, VN_DT_U64, VN_DT_I64, VN_DT_F64 = 0, 1, 2, 3, 4
VN_OP_SUM, VN_OP_MAX, VN_OP_MIN = 0, 1, 2
VN_COMM_ID_BYTES = 128
VN_COUNTER, VN_GAUGE, VN_HISTO, VN_SET = 0, 1, 2, 3
VN_MAX_PERCENTILES = 16
VN_HISTO_STATS = 8
HLL_M = 16384

u8p, u32p, u64p, i64p, f32p, f64p = (C.POINTER(t) for t in (C.c_uint8, C.c_uint32, C.c_uint64, C.c_int64,
                                                             C.c_float, C.c_double))


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("capacity", C.c_uint32 * 4), ("compression", C.c_double),
                ("n_percentiles", C.c_uint32), ("percentiles", C.c_double * VN_MAX_PERCENTILES),
                ("max_batch_records", C.c_uint64), ("max_batch_member_bytes", C.c_uint64),
                ("histo_exact_threshold", C.c_uint32),
                ("histo_hot_prefix", C.c_uint32), ("histo_piece_growth", C.c_uint32),
                ("split_max_records", C.c_uint64), ("split_compression", C.c_double),
                ("replay_reserved_cus", C.c_uint32), ("max_batch_class_records", C.c_uint64 * 4)]


class SplitBatch(C.Structure):
    _fields_ = [("n_histo", C.c_uint64), ("histo_key", C.c_void_p), ("histo_value", C.c_void_p),
                ("histo_rate", C.c_void_p), ("n_set", C.c_uint64), ("set_key", C.c_void_p),
                ("set_member_off", C.c_void_p), ("set_member_bytes", C.c_void_p), ("set_hash", C.c_void_p)]


class Batch(C.Structure):
    _fields_ = [("n_counter", C.c_uint64), ("counter_slot", C.c_void_p), ("counter_value", C.c_void_p),
                ("counter_rate", C.c_void_p),
                ("n_gauge", C.c_uint64), ("gauge_slot", C.c_void_p), ("gauge_value", C.c_void_p),
                ("n_histo", C.c_uint64), ("histo_slot", C.c_void_p), ("histo_value", C.c_void_p),
                ("histo_rate", C.c_void_p),
                ("n_set", C.c_uint64), ("set_slot", C.c_void_p), ("set_member_off", C.c_void_p),
                ("set_member_bytes", C.c_void_p), ("set_hash", C.c_void_p)]


class BatchCounts(C.Structure):
    _fields_ = [("n_counter", C.c_uint64), ("n_gauge", C.c_uint64), ("n_histo", C.c_uint64),
                ("n_set", C.c_uint64), ("n_set_member_bytes", C.c_uint64)]


class Stage(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("member_bytes_capacity", C.c_uint64),
                ("counter_slot", u32p), ("counter_value", f64p), ("counter_rate", f32p),
                ("gauge_slot", u32p), ("gauge_value", f64p),
                ("histo_slot", u32p), ("histo_value", f64p), ("histo_rate", f32p),
                ("set_slot", u32p), ("set_member_off", u32p), ("set_member_bytes", u8p)]


class FlushResult(C.Structure):
    _fields_ = [("n_counter", C.c_uint64), ("counter_slot", u32p), ("counter_value", i64p),
                ("n_gauge", C.c_uint64), ("gauge_slot", u32p), ("gauge_value", f64p),
                ("n_histo", C.c_uint64), ("histo_slot", u32p), ("histo_stats", f64p),
                ("histo_quantiles", f64p), ("n_percentiles", C.c_uint32),
                ("n_set", C.c_uint64), ("set_slot", u32p), ("set_estimate", u64p), ("set_sparse", u8p),
                ("samples_processed", C.c_uint64), ("samples_imported", C.c_uint64),
                ("warn_flags", C.c_uint64)]


VN_WARN_SPLIT_TOUCHED = 16


class SetState(C.Structure):
    _fields_ = [("touched", C.c_uint8), ("sparse", C.c_uint8), ("b", C.c_uint8), ("pad", C.c_uint8),
                ("nz", C.c_uint32), ("list_count", C.c_uint32), ("list_bytes", C.c_uint32),
                ("list_last", C.c_uint32), ("tmp_count", C.c_uint32)]


class Export(C.Structure):
    _fields_ = [("n", C.c_uint64), ("off", u64p), ("bytes", u8p), ("dev_off", C.c_void_p), ("dev_bytes", C.c_void_p)]


class Timing(C.Structure):
    _fields_ = [("ms_ingest_counter", C.c_float), ("ms_ingest_gauge", C.c_float), ("ms_ingest_histo", C.c_float),
                ("ms_ingest_set", C.c_float), ("ms_flush", C.c_float), ("ms_sort_histo", C.c_float),
                ("ms_sort_set", C.c_float), ("sort_passes_histo", C.c_uint64), ("sort_passes_set", C.c_uint64),
                ("ms_radix_scatter_total", C.c_float), ("radix_scatter_launches", C.c_uint64),
                ("radix_scatter_bytes", C.c_uint64), ("ms_histo_replay", C.c_float),
                ("histo_replay_launches", C.c_uint64), ("histo_replay_bytes", C.c_uint64),
                ("ms_set_segments", C.c_float), ("set_segment_launches", C.c_uint64),
                ("set_segment_bytes", C.c_uint64), ("ms_flush_host", C.c_float), ("ms_split_host", C.c_float),
                ("ms_main_ready", C.c_float), ("ms_split_ready", C.c_float),
                ("ms_split_histo_ready", C.c_float), ("ms_split_set_prefix_ready", C.c_float),
                ("ms_part_scatter", C.c_float), ("part_scatter_launches", C.c_uint64),
                ("part_scatter_bytes", C.c_uint64), ("ms_import_decode", C.c_float),
                ("ms_import_drain", C.c_float)]


class SynthConfig(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_keys", C.c_uint32), ("zipf_s", C.c_double), ("mix", C.c_double * 4),
                ("n_samples", C.c_uint64), ("shard", C.c_uint32), ("n_shards", C.c_uint32),
                ("member_universe", C.c_uint64), ("rate_half", C.c_double), ("rate_tenth", C.c_double),
                ("histo_mu", C.c_double), ("histo_sigma", C.c_double), ("threads", C.c_int)]


class SynthOut(C.Structure):
    _fields_ = [("n_slots", C.c_uint32 * 4), ("n", C.c_uint64 * 4),
                ("c_slot", u32p), ("c_val", f64p), ("c_rate", f32p),
                ("g_slot", u32p), ("g_val", f64p),
                ("h_slot", u32p), ("h_val", f64p), ("h_rate", f32p),
                ("s_slot", u32p), ("s_off", u32p), ("s_bytes", u8p), ("s_nbytes", C.c_uint64),
                ("key_of_slot", u32p * 4), ("digest_of_slot", u32p * 4)]


class SynthDevConfig(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_keys", C.c_uint32), ("zipf_s", C.c_double), ("mix", C.c_double * 4),
                ("n_samples", C.c_uint64), ("rank", C.c_uint32), ("nranks", C.c_uint32),
                ("member_universe", C.c_uint64), ("rate_half", C.c_double), ("rate_tenth", C.c_double),
                ("histo_mu", C.c_double), ("histo_sigma", C.c_double), ("device", C.c_int),
                ("n_split", C.c_uint32 * 4), ("split_key", u32p * 4)]


class SynthDevOut(C.Structure):
    _fields_ = [("n_slots", C.c_uint32 * 4), ("split_slot0", C.c_uint32 * 4), ("key_of_slot", u32p * 4),
                ("digest_of_slot", u32p * 4), ("batch", Batch), ("split", SplitBatch),
                ("n_member_bytes", C.c_uint64), ("n_split_member_bytes", C.c_uint64),
                ("counter_sum", C.c_int64), ("histo_weight", C.c_double)]


class SynthHostsConfig(C.Structure):  # vn_synth_hosts_config
    _fields_ = [("seed", C.c_uint64), ("host0", C.c_uint32), ("n_hosts", C.c_uint32), ("n_histo_keys", C.c_uint32),
                ("n_set_keys", C.c_uint32), ("device", C.c_int)]


class SynthHostsOut(C.Structure):  # vn_synth_hosts_out
    _fields_ = [("n_histo", C.c_uint64), ("n_set", C.c_uint64), ("h_slot", C.c_void_p), ("h_val", C.c_void_p),
                ("h_rate", C.c_void_p), ("s_slot", C.c_void_p), ("s_hash", C.c_void_p)]


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


vp = C.c_void_p
_sig("vn_abi_version", C.c_int)
_sig("vn_struct_size", C.c_size_t, C.c_int)
_sig("vn_build_flags", C.c_int)
ABI_VERSION = 6
_sig("vn_engine_create", C.c_int, C.POINTER(Config), C.POINTER(vp))
_sig("vn_engine_destroy", None, vp)
_sig("vn_last_error", C.c_char_p, vp)
_sig("vn_stage_acquire", C.c_int, vp, C.POINTER(Stage))
_sig("vn_submit", C.c_int, vp, C.POINTER(BatchCounts))
_sig("vn_ingest_host", C.c_int, vp, C.POINTER(Batch))
_sig("vn_ingest", C.c_int, vp, C.POINTER(Batch))
_sig("vn_import_counters", C.c_int, vp, u32p, i64p, C.c_uint64)
_sig("vn_import_gauges", C.c_int, vp, u32p, f64p, C.c_uint64)
_sig("vn_import_histos", C.c_int, vp, u32p, u64p, u8p, C.c_uint64)
_sig("vn_import_sets", C.c_int, vp, u32p, u64p, u8p, C.c_uint64)
_sig("vn_import_histos_device", C.c_int, vp, vp, vp, vp, C.c_uint64)
_sig("vn_import_sets_device", C.c_int, vp, vp, vp, vp, C.c_uint64)
_sig("vn_histo_query", C.c_int, vp, C.c_int, u32p, f64p, C.c_uint64, f64p)
_sig("vn_export_histos", C.c_int, vp, u32p, C.c_uint64, C.POINTER(Export))
_sig("vn_export_sets", C.c_int, vp, u32p, C.c_uint64, C.POINTER(Export))
_sig("vn_flush", C.c_int, vp, C.POINTER(FlushResult))
_sig("vn_flush_masked", C.c_int, vp, u8p, u8p, C.POINTER(FlushResult))
_sig("vn_sync", C.c_int, vp)
_sig("vn_read_histo", C.c_int, vp, C.c_uint32, f64p, f64p, C.c_uint32, u32p, f64p)
_sig("vn_read_set", C.c_int, vp, C.c_uint32, C.POINTER(SetState), u32p, C.c_uint32, u32p, C.c_uint32, u8p)
_sig("vn_metro64", C.c_int, C.c_int, u8p, u32p, C.c_uint64, C.c_uint64, u64p)


class ParsedLine(C.Structure):  # vn_parsed_line
    _fields_ = [("line_off", C.c_uint64), ("name_off", C.c_uint64), ("value_off", C.c_uint64),
                ("tags_off", C.c_uint64), ("value", C.c_double), ("line_len", C.c_uint32),
                ("name_len", C.c_uint32), ("value_len", C.c_uint32), ("tags_len", C.c_uint32),
                ("n_tags", C.c_uint32), ("digest", C.c_uint32), ("rate", C.c_float), ("status", C.c_int32),
                ("type", C.c_uint8), ("scope", C.c_uint8), ("has_tags", C.c_uint8), ("pad", C.c_uint8)]


_sig("vn_parse_dogstatsd", C.c_int64, C.c_char_p, C.c_uint64, C.POINTER(ParsedLine), C.c_uint64, C.c_char_p,
     C.c_uint64)
_sig("vn_parser_create", C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(vp))
_sig("vn_parser_destroy", None, vp)
_sig("vn_parser_last_error", C.c_char_p, vp)
_sig("vn_parse_dogstatsd_device", C.c_int, vp, vp, C.c_uint64, vp, C.c_uint64, vp, C.c_uint64, u64p)
_sig("vn_go_parse_float", C.c_int, C.c_char_p, C.c_uint64, C.c_int, f64p)
_sig("vn_diag_index_estimate", C.c_int, C.c_int, C.c_double, f64p, C.c_uint64, u64p, f64p)


class IntakeStats(C.Structure):  # vn_intake_stats
    _fields_ = [("lines", C.c_uint64), ("processed", C.c_uint64), ("parse_errors", C.c_uint64),
                ("dropped", C.c_uint64), ("new_keys", C.c_uint64)]


class IntakeInfo(C.Structure):  # vn_intake_info
    _fields_ = [("n_keys", C.c_uint64), ("arena_bytes", C.c_uint64), ("next_slot", C.c_uint32 * 4)]


class Keys(C.Structure):  # vn_keys
    _fields_ = [("n_keys", C.c_uint64), ("map", u8p), ("slot", u32p), ("n_tags", u32p), ("name_off", u64p),
                ("name_len", u32p), ("tags_len", u32p), ("arena", u8p)]


class DDConfig(C.Structure):  # vn_dd_config
    _fields_ = [("interval", C.c_double), ("timestamp", C.c_int64), ("is_local", C.c_int32),
                ("aggregates", C.c_uint32), ("n_percentiles", C.c_uint32),
                ("percentiles", C.c_double * VN_MAX_PERCENTILES), ("engine_percentiles", f64p),
                ("hostname", C.c_char_p), ("sink_tags", C.c_char_p), ("n_sink_tags", C.c_uint32),
                ("flush_max_per_body", C.c_uint32)]


class DDPayload(C.Structure):  # vn_dd_payload
    _fields_ = [("n_intermetrics", C.c_uint64), ("n_metrics", C.c_uint64), ("n_bodies", C.c_uint32),
                ("body_off", u64p), ("body_status", C.POINTER(C.c_int32)), ("bytes", u8p)]


_sig("vn_sink_create", C.c_int, C.POINTER(vp))
_sig("vn_sink_destroy", None, vp)
_sig("vn_sink_last_error", C.c_char_p, vp)
_sig("vn_datadog_flush", C.c_int, vp, C.POINTER(FlushResult), C.POINTER(Keys), C.POINTER(DDConfig),
     C.POINTER(DDPayload))
_sig("vn_intake_create", C.c_int, vp, C.c_uint64, C.c_uint64, C.POINTER(vp))
_sig("vn_intake_destroy", None, vp)
_sig("vn_intake_last_error", C.c_char_p, vp)
_sig("vn_intake_process", C.c_int, vp, vp, C.c_uint64, C.POINTER(IntakeStats))
_sig("vn_intake_upsert", C.c_int, vp, C.c_uint64, u8p, u32p, u32p, u32p, u32p, u32p, u32p, u8p, C.c_uint64, u32p)
_sig("vn_intake_keys_info", C.c_int, vp, C.POINTER(IntakeInfo))
_sig("vn_intake_read_keys", C.c_int, vp, u8p, u32p, u32p, u64p, u32p, u32p, u8p)
_sig("vn_intake_reset", C.c_int, vp)
_sig("vn_comm_unique_id", C.c_int, u8p)
_sig("vn_comm_init", C.c_int, u8p, C.c_int, C.c_int, C.c_int, C.POINTER(vp))
_sig("vn_comm_init_local", C.c_int, C.c_int, C.c_int, C.POINTER(vp))
_sig("vn_comm_destroy", None, vp)
_sig("vn_comm_last_error", C.c_char_p, vp)
_sig("vn_comm_rank", C.c_int, vp)
_sig("vn_comm_nranks", C.c_int, vp)
_sig("vn_comm_allreduce", C.c_int, vp, vp, vp, C.c_uint64, C.c_int, C.c_int)
_sig("vn_engine_set_comm", C.c_int, vp, vp)
_sig("vn_split_keys", C.c_int, vp, C.c_int, u32p, u32p, C.c_uint32)
_sig("vn_ingest_split", C.c_int, vp, C.POINTER(SplitBatch))
_sig("vn_split_close", C.c_int, vp)
_sig("vn_split_combine", C.c_int, vp)
_sig("vn_hot_detect", C.c_int, vp, C.c_uint32)
_sig("vn_hot_keys", C.c_int, vp, C.c_int, C.c_uint64, C.c_uint32, u32p, C.POINTER(C.c_uint64), u32p)
_sig("vn_device_alloc", C.c_int, C.c_int, C.c_uint64, C.POINTER(vp))
_sig("vn_device_free", C.c_int, vp)
_sig("vn_copy_to_device", C.c_int, C.c_int, vp, vp, C.c_uint64)
_sig("vn_device_copy", C.c_int, C.c_int, vp, vp, C.c_uint64)
_sig("vn_copy_to_host", C.c_int, C.c_int, vp, vp, C.c_uint64)
_sig("vn_device_count", C.c_int, C.POINTER(C.c_int))
_sig("vn_device_synchronize", C.c_int, C.c_int)
_sig("vn_timing_enable", C.c_int, vp, C.c_int)
_sig("vn_get_timing", C.c_int, vp, C.POINTER(Timing))
_sig("vn_import_counts", C.c_int, vp, C.POINTER(C.c_uint64), C.c_int)
_sig("vn_synth_generate", C.c_int, C.POINTER(SynthConfig), C.POINTER(SynthOut))
_sig("vn_synth_free", None, C.POINTER(SynthOut))
_sig("vn_synth_device", C.c_int, C.POINTER(SynthDevConfig), C.POINTER(SynthDevOut))
_sig("vn_synth_device_free", None, C.POINTER(SynthDevOut))
_sig("vn_synth_key_counts", C.c_int, C.POINTER(SynthDevConfig), C.c_uint64, u32p)
_sig("vn_synth_hosts_device", C.c_int, C.POINTER(SynthHostsConfig), C.POINTER(SynthHostsOut))
_sig("vn_synth_hosts_free", None, C.POINTER(SynthHostsOut))

# every symbol include/*.h declares (checked by tests/test_abi.py on CPU)
EXPORTED = [
    "vn_abi_version", "vn_build_flags", "vn_struct_size", "vn_engine_create", "vn_engine_destroy", "vn_last_error", "vn_stage_acquire", "vn_submit",
    "vn_ingest_host", "vn_ingest", "vn_import_counters", "vn_import_gauges", "vn_import_histos", "vn_import_sets", "vn_import_histos_device", "vn_import_sets_device", "vn_histo_query", "vn_export_histos", "vn_export_sets", "vn_flush", "vn_flush_masked", "vn_sync",
    "vn_read_histo", "vn_read_set", "vn_metro64", "vn_parse_dogstatsd", "vn_parser_create", "vn_parser_destroy",
    "vn_parser_last_error", "vn_parse_dogstatsd_device", "vn_go_parse_float", "vn_diag_index_estimate", "vn_intake_create", "vn_intake_destroy",
    "vn_intake_last_error", "vn_intake_process", "vn_intake_upsert", "vn_intake_keys_info", "vn_intake_read_keys",
    "vn_intake_reset", "vn_sink_create", "vn_sink_destroy", "vn_sink_last_error", "vn_datadog_flush", "vn_device_alloc", "vn_device_free", "vn_copy_to_device",
    "vn_device_copy", "vn_device_count", "vn_device_synchronize", "vn_timing_enable", "vn_get_timing", "vn_synth_generate", "vn_synth_free",
    "vn_synth_device", "vn_synth_device_free", "vn_synth_key_counts", "vn_synth_hosts_device",
    "vn_synth_hosts_free",
    "vn_copy_to_host", "vn_comm_unique_id", "vn_comm_init", "vn_comm_init_local", "vn_comm_destroy", "vn_comm_last_error", "vn_comm_rank",
    "vn_comm_nranks", "vn_comm_allreduce", "vn_engine_set_comm", "vn_split_keys", "vn_ingest_split", "vn_split_close", "vn_split_combine",
    "vn_hot_detect", "vn_hot_keys", "vn_import_counts",
]


def _check_abi():
    """The library must match this binding: ABI version and every struct the two share."""
    v = lib.vn_abi_version()
    if v != ABI_VERSION:
        raise ImportError("libveneur_amd.so ABI %d, binding expects %d" % (v, ABI_VERSION))
    for which, st in ((0, Config), (1, Batch), (2, FlushResult), (3, Timing), (4, SplitBatch), (5, Stage)):
        n = lib.vn_struct_size(which)
        if n != C.sizeof(st):
            raise ImportError("libveneur_amd.so struct %s is %d bytes, binding has %d" % (st.__name__, n,
                                                                                          C.sizeof(st)))


_check_abi()
# the t-digest fast mode (histo_exact_threshold > 0) is a variant build only (include/veneur_amd.h)
FAST_MODE = bool(lib.vn_build_flags() & 1)
