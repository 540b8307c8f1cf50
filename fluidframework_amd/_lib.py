"""ctypes binding of the engine's C ABI (include/mtb.h) -> fluidframework_amd/libmtb.so.

The shared library is built in-tree by `python -m fluidframework_amd.build` (hipcc, gfx950).  There is
no CPU fallback: if the library is missing this module raises, and without a GPU every replay call
returns MTB_E_NODEV.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MTB_LIB") or os.path.join(HERE, "libmtb.so")  # MTB_LIB: alternate build (tuning)

MTB_OP_INSERT, MTB_OP_REMOVE, MTB_OP_ANNOTATE, MTB_OP_NOOP, MTB_OP_ACK = 0, 1, 2, 3, 4
MTB_F_LAST, MTB_F_MARKER, MTB_F_REWRITE, MTB_F_SEGOBJ = 0x01, 0x02, 0x04, 0x08

ERRORS = {0: "MTB_OK", -1: "MTB_E_ARG", -2: "MTB_E_NODEV", -3: "MTB_E_HIP", -4: "MTB_E_ASSERT",
          -5: "MTB_E_INSERT", -6: "MTB_E_UNSUPPORTED", -7: "MTB_E_CAPACITY", -8: "MTB_E_PARSE"}

# every entry point declared in include/mtb.h
EXPORTS = ["mtb_batch_create", "mtb_batch_destroy", "mtb_last_error", "mtb_free", "mtb_build_id", "mtb_doc_init",
           "mtb_doc_load_v1", "mtb_docs_load_v1", "mtb_matrix_init", "mtb_matrix_apply_msg_json",
           "mtb_matrix_intern_value", "mtb_matrix_summarize", "mtb_matrix_get_cell", "mtb_matrix_load",
           "mtb_apply_msg_json", "mtb_append_ops", "mtb_add_client", "mtb_intern_props", "mtb_replay",
           "mtb_get_text", "mtb_get_length", "mtb_get_seq", "mtb_dump_segments", "mtb_doc_checksum",
           "mtb_summarize_v1", "mtb_blob_list_free", "mtb_summarize_legacy", "mtb_rewind", "mtb_replay_resident", "mtb_replay_resident_ex", "mtb_refresh_digests",
           "mtb_export_pending", "mtb_props_json", "mtb_client_long_id", "mtb_map_range", "mtb_debug_blocks", "mtb_doc_digests",
           "mtb_summarize_v1_many", "mtb_blob_list_fnv", "mtb_local_op_json", "mtb_regenerate_pending_op",
           "mtb_get_launch_info", "mtb_detached_op_json", "mtb_maintenance"]


class MtbLaunchInfo(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_uint32), ("wave_slots", ctypes.c_uint32), ("chunks", ctypes.c_uint32),
                ("queues", ctypes.c_uint32), ("aborted", ctypes.c_uint32), ("passes", ctypes.c_uint32),
                ("handover_bad", ctypes.c_uint32), ("cap_retries", ctypes.c_uint32)]


KERNEL_NAMES = {0: None, 1: "mtb_replay_kernel", 3: "mtb_replay_few_kernel",
                4: "mtb_live_kernel", 5: "mtb_markers_kernel", 6: "mtb_matrix_kernel", 7: "mtb_replay_pass_kernel",
                8: "mtb_replay_tick_kernel"}


class MtbOptions(ctypes.Structure):
    _fields_ = [("new_length_calc", ctypes.c_int32), ("chunk_size", ctypes.c_int32),
                ("threads_per_doc", ctypes.c_int32), ("flags", ctypes.c_int32)]


class MtbStats(ctypes.Structure):
    _fields_ = [("ops_applied", ctypes.c_uint64), ("docs", ctypes.c_uint64), ("segments_final", ctypes.c_uint64),
                ("text_units_final", ctypes.c_uint64), ("bytes_alg", ctypes.c_uint64), ("checksum", ctypes.c_uint64),
                ("errors", ctypes.c_uint64), ("kernel_ms", ctypes.c_double)]


class MtbBlob(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("content", ctypes.c_void_p), ("content_len", ctypes.c_size_t)]


class MtbBlobList(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint32), ("blobs", ctypes.POINTER(MtbBlob)),
                ("summary_json", ctypes.c_void_p), ("summary_json_len", ctypes.c_size_t)]


_LIB = None


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build the HIP engine with `python -m fluidframework_amd.build`")
    # PyTorch-ROCm bundles its own libamdhip64.so.7.  Load it first so this process has exactly one HIP
    # runtime (the engine's DT_NEEDED soname then resolves to the already-loaded copy); loading the
    # system runtime first makes torch report "No HIP GPUs are available".
    # MTB_NO_TORCH=1 keeps torch out of the process (e.g. under rocprofv3 --pmc, whose tool library
    # binds to the system HSA runtime).
    if os.environ.get("MTB_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
    L.mtb_batch_create.argtypes = [ctypes.POINTER(MtbOptions), u32, u32, ctypes.POINTER(vp)]
    L.mtb_batch_destroy.argtypes = [vp]
    L.mtb_last_error.restype = ctypes.c_char_p
    L.mtb_last_error.argtypes = [vp]
    L.mtb_free.argtypes = [vp]
    L.mtb_build_id.restype = ctypes.c_char_p
    L.mtb_build_id.argtypes = []
    L.mtb_doc_init.argtypes = [vp, u32, vp, sz, ctypes.c_char_p, u32, u32]
    L.mtb_doc_load_v1.argtypes = [vp, u32, ctypes.POINTER(MtbBlob), u32, ctypes.c_char_p]
    L.mtb_docs_load_v1.argtypes = [vp, u32, ctypes.POINTER(u32), ctypes.POINTER(ctypes.POINTER(MtbBlob)),
                                   ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_char_p), u32]
    L.mtb_matrix_init.argtypes = [vp, u32, ctypes.c_char_p, u32, u32]
    L.mtb_matrix_apply_msg_json.argtypes = [vp, u32, ctypes.c_char_p, sz]
    L.mtb_matrix_load.argtypes = [vp, u32, vp, u32, ctypes.c_char_p]
    L.mtb_matrix_intern_value.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(u32)]
    L.mtb_matrix_get_cell.argtypes = [vp, u32, u32, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.mtb_apply_msg_json.argtypes = [vp, u32, ctypes.c_char_p, sz]
    L.mtb_local_op_json.argtypes = [vp, u32, ctypes.c_char_p, sz]
    L.mtb_detached_op_json.argtypes = [vp, u32, ctypes.c_char_p, sz]
    L.mtb_maintenance.argtypes = [vp, u32, u32]
    L.mtb_regenerate_pending_op.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(sz)]
    L.mtb_append_ops.argtypes = [vp, u32, vp, u32, vp, sz]
    L.mtb_add_client.argtypes = [vp, u32, ctypes.c_char_p]
    L.mtb_intern_props.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(u32)]
    L.mtb_replay.argtypes = [vp, ctypes.POINTER(MtbStats)]
    L.mtb_get_text.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz)]
    L.mtb_get_length.argtypes = [vp, u32, ctypes.POINTER(u32)]
    L.mtb_get_seq.argtypes = [vp, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.mtb_dump_segments.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.mtb_doc_checksum.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_uint64)]
    L.mtb_doc_digests.argtypes = [vp, u32, u32, ctypes.POINTER(ctypes.c_uint64)]
    L.mtb_get_launch_info.argtypes = [vp, ctypes.POINTER(MtbLaunchInfo)]
    L.mtb_summarize_v1.argtypes = [vp, u32, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MtbBlobList)]
    L.mtb_summarize_legacy.argtypes = [vp, u32, ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, sz,
                                       ctypes.POINTER(MtbBlobList)]
    L.mtb_blob_list_free.argtypes = [ctypes.POINTER(MtbBlobList)]
    L.mtb_blob_list_fnv.argtypes = [ctypes.POINTER(MtbBlobList), ctypes.POINTER(ctypes.c_uint64)]
    L.mtb_summarize_v1_many.argtypes = [vp, u32, ctypes.POINTER(u32), ctypes.c_int64, ctypes.c_int64, u32,
                                        ctypes.POINTER(MtbBlobList)]
    L.mtb_matrix_summarize.argtypes = [vp, u32, ctypes.POINTER(MtbBlobList)]
    L.mtb_rewind.argtypes = [vp]
    L.mtb_map_range.argtypes = [vp, u32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, u32,
                                ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.mtb_debug_blocks.argtypes = [vp, u32, ctypes.c_int64, ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.mtb_replay_resident.argtypes = [vp, ctypes.POINTER(MtbStats)]
    L.mtb_replay_resident_ex.argtypes = [vp, ctypes.POINTER(MtbStats), u32]
    L.mtb_refresh_digests.argtypes = [vp, ctypes.POINTER(MtbStats)]
    L.mtb_export_pending.argtypes = [vp, u32, vp, u32, ctypes.POINTER(u32), vp, sz, ctypes.POINTER(sz)]
    L.mtb_props_json.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.mtb_client_long_id.argtypes = [vp, u32, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    _LIB = L
    return L
