"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU restatement).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the parity checker.
The product engine (fluidframework_amd) never imports this module.
"""
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, cp, i, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t
        L.orc_create.restype = vp
        L.orc_create.argtypes = [i, i, i]
        L.orc_destroy.argtypes = [vp]
        L.orc_last_error.restype = cp
        L.orc_last_error.argtypes = [vp]
        L.orc_free.argtypes = [vp]
        L.orc_insert_text_local.argtypes = [vp, i, cp, cp]
        L.orc_insert_marker_local.argtypes = [vp, i, i, cp]
        L.orc_annotate_local.argtypes = [vp, i, i, cp]
        L.orc_remove_local.argtypes = [vp, i, i]
        L.orc_start_collab.argtypes = [vp, cp, i, i]
        L.orc_apply_msg_json.argtypes = [vp, cp, sz]
        L.orc_apply_records.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.POINTER(cp), ctypes.c_uint32]
        L.orc_add_client.argtypes = [vp, cp]
        L.orc_update_seq.argtypes = [vp, i, i]
        L.orc_get_text.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_get_length.argtypes = [vp]
        L.orc_get_remote_length.argtypes = [vp, i, i]
        L.orc_pos_from_relative.argtypes = [vp, cp, i, i]
        L.orc_current_seq.argtypes = [vp]
        L.orc_min_seq.argtypes = [vp]
        L.orc_num_clients.argtypes = [vp]
        L.orc_client_long_id.restype = cp
        L.orc_client_long_id.argtypes = [vp, i]
        L.orc_ops_applied.restype = ctypes.c_uint64
        L.orc_ops_applied.argtypes = [vp]
        L.orc_segs_touched.restype = ctypes.c_uint64
        L.orc_segs_touched.argtypes = [vp]
        L.orc_stale_updates.restype = ctypes.c_uint64
        L.orc_stale_updates.argtypes = [vp]
        L.orc_stale_deficits.restype = ctypes.c_uint64
        L.orc_stale_deficits.argtypes = [vp]
        L.orc_summarize_v1.argtypes = [vp, i, i, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_dump_segments.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_checksum.restype = ctypes.c_uint64
        L.orc_checksum.argtypes = [vp]
        L.orc_digest.restype = ctypes.c_uint64
        L.orc_digest.argtypes = [vp]
        L.orc_zamboni.argtypes = [vp]
        L.orc_pack_parent_root.argtypes = [vp]
        L.orc_load_v1.argtypes = [vp, cp, sz, cp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_enable_catch_up.argtypes = [vp]
        L.orc_summarize_legacy.argtypes = [vp, i, i, cp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_matrix_create.restype = vp
        L.orc_matrix_create.argtypes = [i, i]
        L.orc_matrix_destroy.argtypes = [vp]
        L.orc_matrix_vector.restype = vp
        L.orc_matrix_vector.argtypes = [vp, i]
        L.orc_matrix_last_error.restype = cp
        L.orc_matrix_last_error.argtypes = [vp]
        L.orc_matrix_start_collab.argtypes = [vp, cp, i, i]
        L.orc_matrix_apply_msg_json.argtypes = [vp, cp, sz]
        L.orc_matrix_load.argtypes = [vp, cp, sz, cp]
        L.orc_matrix_summarize.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.orc_matrix_get_cell.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(sz)]
        L.orc_matrix_get_cell_by_handle.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(sz)]
        u32 = ctypes.c_uint32
        pp = ctypes.POINTER(vp)
        L.orc_local_insert.argtypes = [vp, i, cp, pp, ctypes.POINTER(sz)]
        L.orc_local_remove.argtypes = [vp, i, i, pp, ctypes.POINTER(sz)]
        L.orc_local_annotate.argtypes = [vp, i, i, cp, pp, ctypes.POINTER(sz)]
        L.orc_pending_groups.argtypes = [vp]
        L.orc_regenerate.argtypes = [vp, cp, pp, ctypes.POINTER(sz)]
        L.orc_local_op_json.argtypes = [vp, cp, pp, ctypes.POINTER(sz)]
        L.orc_map_range.argtypes = [vp, i, i, i, cp, ctypes.c_uint, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.orc_debug_blocks.argtypes = [vp, i, cp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.orc_sa2d_create.restype = vp
        L.orc_sa2d_destroy.argtypes = [vp]
        L.orc_sa2d_set.argtypes = [vp, u32, u32, cp]
        L.orc_sa2d_get.argtypes = [vp, u32, u32, ctypes.c_char_p, sz]
        L.orc_sa2d_clear_rows.argtypes = [vp, u32, u32]
        L.orc_sa2d_clear_cols.argtypes = [vp, u32, u32]
        L.orc_sa2d_snapshot.restype = vp
        L.orc_sa2d_snapshot.argtypes = [vp, ctypes.POINTER(sz)]
        _LIB = L
    return _LIB


class OracleSparseArray2D:
    """SparseArray2D (matrix/src/sparsearray2d.ts) of the oracle; values are JSON texts (None = undefined)."""

    def __init__(self):
        self._L = lib()
        self._h = self._L.orc_sa2d_create()
        self._buf = ctypes.create_string_buffer(4096)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_sa2d_destroy(self._h)
            self._h = None

    def set_cell(self, r, c, value_json):
        self._L.orc_sa2d_set(self._h, r, c, None if value_json is None else value_json.encode())

    def get_cell(self, r, c):
        n = self._L.orc_sa2d_get(self._h, r, c, self._buf, len(self._buf))
        return None if n < 0 else self._buf.value.decode()

    def clear_rows(self, start, count):
        self._L.orc_sa2d_clear_rows(self._h, start, count)

    def clear_cols(self, start, count):
        self._L.orc_sa2d_clear_cols(self._h, start, count)

    def snapshot(self):
        n = ctypes.c_size_t()
        p = self._L.orc_sa2d_snapshot(self._h, ctypes.byref(n))
        try:
            return ctypes.string_at(p, n.value).decode()
        finally:
            self._L.orc_free(p)


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class OracleDoc:
    """One observer merge-tree client (Client/TestClient restated in C++)."""

    def __init__(self, new_length_calc=False, chunk_size=0, verify=False):
        self._L = lib()
        self._h = self._L.orc_create(int(new_length_calc), int(chunk_size), int(verify))

    def close(self):
        if self._h:
            self._L.orc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            raise OracleError(rc, self._L.orc_last_error(self._h).decode("utf-8", "replace"))

    # --- detached local edits -------------------------------------------------------------
    def insert_text_local(self, pos, text, props=None):
        self._chk(self._L.orc_insert_text_local(self._h, pos, text.encode("utf-8", "surrogatepass"),
                                                None if props is None else json.dumps(props).encode()))

    def insert_marker_local(self, pos, ref_type, props=None):
        self._chk(self._L.orc_insert_marker_local(self._h, pos, ref_type,
                                                  None if props is None else json.dumps(props).encode()))

    def annotate_local(self, start, end, props):
        self._chk(self._L.orc_annotate_local(self._h, start, end, json.dumps(props).encode()))

    def remove_local(self, start, end):
        self._chk(self._L.orc_remove_local(self._h, start, end))

    # --- collaboration ---------------------------------------------------------------------
    def start_collab(self, long_id, min_seq=0, cur_seq=0):
        self._chk(self._L.orc_start_collab(self._h, long_id.encode(), min_seq, cur_seq))

    def apply_msg(self, msg):
        s = msg if isinstance(msg, (bytes, bytearray)) else json.dumps(msg).encode()
        self._chk(self._L.orc_apply_msg_json(self._h, s, len(s)))

    def apply_records(self, ops_bytes, n, text_u16, props_json):
        arr = (ctypes.c_char_p * max(1, len(props_json)))(*[p.encode() if p is not None else None for p in props_json])
        tbuf = ctypes.create_string_buffer(bytes(text_u16), max(2, len(text_u16)))
        obuf = ctypes.create_string_buffer(bytes(ops_bytes), max(1, len(ops_bytes)))
        self._chk(self._L.orc_apply_records(self._h, obuf, n, tbuf, arr, len(props_json)))

    def add_client(self, long_id):
        self._chk(self._L.orc_add_client(self._h, long_id.encode()))

    def update_seq(self, min_seq, seq):
        self._chk(self._L.orc_update_seq(self._h, min_seq, seq))

    # --- read-out --------------------------------------------------------------------------
    def get_text(self):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_get_text(self._h, ctypes.byref(p), ctypes.byref(n)))
        try:
            raw = ctypes.string_at(p, n.value * 2)
        finally:
            self._L.orc_free(p)
        return raw.decode("utf-16-le", "surrogatepass")

    # --- a live client's local ops (client.ts:196-247): return the op contents to submit ------
    def _op(self, fn, *args):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(fn(self._h, *args, ctypes.byref(p), ctypes.byref(n)))
        try:
            raw = ctypes.string_at(p, n.value).decode("utf-8")
        finally:
            self._L.orc_free(p)
        return json.loads(raw) if raw else None

    def insert_local_op(self, pos, seg):
        return self._op(self._L.orc_local_insert, pos, json.dumps(seg).encode())

    def remove_local_op(self, start, end):
        return self._op(self._L.orc_local_remove, start, end)

    def annotate_local_op(self, start, end, props):
        return self._op(self._L.orc_local_annotate, start, end, json.dumps(props).encode())

    def local_op_json(self, op):
        """A live client's local op given as the IMergeTreeOp it sends (absolute or marker-relative positions)."""
        return self._op(self._L.orc_local_op_json, json.dumps(op).encode())

    def regenerate_pending_op(self, op):
        """Client.regeneratePendingOp (client.ts:917-960) for the op at the head of the pending queue."""
        return self._op(self._L.orc_regenerate, json.dumps(op).encode())

    def pending_groups(self):
        return self._L.orc_pending_groups(self._h)

    def map_range(self, start=0, end=-1, ref_seq=-1, long_client_id=None, limit=0):
        """mapRange over [start, end) in the (ref_seq, client) view: [{"pos","start","end","segment"}...]."""
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_map_range(self._h, start, end, ref_seq,
                                        None if long_client_id is None else long_client_id.encode(), limit,
                                        ctypes.byref(p), ctypes.byref(n)))
        try:
            return json.loads(ctypes.string_at(p, n.value).decode("utf-8"))
        finally:
            self._L.orc_free(p)

    def debug_blocks(self, ref_seq=-1, long_client_id=None):
        """Debug view: per block (tree order) its path, each block child's [partial length, leaf sum] in the
        (ref_seq, client) view, minLength and the main / client partial-length sets ([seq, len, seglen])."""
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_debug_blocks(self._h, ref_seq, None if long_client_id is None else long_client_id.encode(),
                                           ctypes.byref(p), ctypes.byref(n)))
        try:
            return [json.loads(x) for x in ctypes.string_at(p, n.value).decode("utf-8").splitlines()]
        finally:
            self._L.orc_free(p)

    def get_length(self):
        return self._L.orc_get_length(self._h)

    def pos_from_relative(self, rel, ref_seq, client):
        """posFromRelativePos (mergeTree.ts:1371) of an IRelativePosition dict in the (ref_seq, client) view."""
        return self._L.orc_pos_from_relative(self._h, json.dumps(rel).encode(), ref_seq, client)

    def remote_length(self, ref_seq, client):
        return self._L.orc_get_remote_length(self._h, ref_seq, client)

    @property
    def current_seq(self):
        return self._L.orc_current_seq(self._h)

    @property
    def min_seq(self):
        return self._L.orc_min_seq(self._h)

    def client_ids(self):
        return [self._L.orc_client_long_id(self._h, i).decode() for i in range(self._L.orc_num_clients(self._h))]

    def ops_applied(self):
        return self._L.orc_ops_applied(self._h)

    def segs_touched(self):
        return self._L.orc_segs_touched(self._h)

    def stale_updates(self):
        """Partial-length updates below the root that met newer entries (stale cumulative lengths)."""
        return self._L.orc_stale_updates(self._h)

    def stale_deficits(self):
        """Of those, the updates that actually left later entries short: an existing entry at the update's seq got
        its seglen replaced while entries after it kept cumulative lengths built on the old one (addSeq,
        partialLengths.ts:543-577)."""
        return self._L.orc_stale_deficits(self._h)

    def summarize_v1(self, msn=-1, seq=-1):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_summarize_v1(self._h, msn, seq, ctypes.byref(p), ctypes.byref(n)))
        try:
            raw = ctypes.string_at(p, n.value)
        finally:
            self._L.orc_free(p)
        return json.loads(raw.decode("utf-8"))

    def enable_catch_up(self):
        """Track catch-up messages like a SharedString without the V1 snapshot option (sequence.ts:697-748)."""
        self._L.orc_enable_catch_up(self._h)

    def summarize_legacy(self, msn=-1, seq=-1, catchup=None):
        """SnapshotLegacy summary (snapshotlegacy.ts): {"blobs": [[path, content]...], "summary": {...}}."""
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        cu = json.dumps(catchup, separators=(",", ":")).encode() if catchup else None
        self._chk(self._L.orc_summarize_legacy(self._h, msn, seq, cu, ctypes.byref(p), ctypes.byref(n)))
        try:
            raw = ctypes.string_at(p, n.value)
        finally:
            self._L.orc_free(p)
        return json.loads(raw.decode("utf-8"))

    def dump_segments(self):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_dump_segments(self._h, ctypes.byref(p), ctypes.byref(n)))
        try:
            raw = ctypes.string_at(p, n.value)
        finally:
            self._L.orc_free(p)
        return raw.decode("utf-8")

    def checksum(self):
        return self._L.orc_checksum(self._h)

    def zamboni(self):
        """zamboniSegments(mergeTree) called directly (mergeTree.zamboni.spec.ts)."""
        self._chk(self._L.orc_zamboni(self._h))

    def pack_parent_root(self):
        """packParent(mergeTree.root) called directly (mergeTree.zamboni.spec.ts)."""
        self._chk(self._L.orc_pack_parent_root(self._h))

    def digest(self):
        """State digest v1 (DESIGN.md "State digest"), as the engine's mtb_doc_digests computes it."""
        return self._L.orc_digest(self._h)

    def load_v1(self, blobs, observer_id):
        """Client.load of a SnapshotV1 or SnapshotLegacy summary given as [(path, content), ...]
        (snapshotLoader.ts:41; legacy chunks through toLatestVersion, snapshotChunks.ts:151-175).  Returns the
        summary's catch-up messages (snapshotLoader.ts:60-86; [] when it has none)."""
        raw = json.dumps([list(b) for b in blobs]).encode()
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.orc_load_v1(self._h, raw, len(raw), observer_id.encode(), ctypes.byref(p), ctypes.byref(n)))
        try:
            return json.loads(ctypes.string_at(p, n.value).decode("utf-8"))
        finally:
            self._L.orc_free(p)

    load = load_v1

    def apply_catch_up(self, msgs):
        """SharedSegmentSequence.loadCore's catch-up loop (sequence.ts:576-600): each message must lie above the
        collab window (else "Invalid catchup operations in snapshot"), then it is applied."""
        for m in msgs:
            if (m["minimumSequenceNumber"] < self.min_seq or m["referenceSequenceNumber"] < self.min_seq or
                    m["sequenceNumber"] <= self.min_seq or m["sequenceNumber"] <= self.current_seq):
                raise OracleError(-1, "Invalid catchup operations in snapshot")
            self.apply_msg(m)


def msg_from_compact(m):
    """Expand a compact fixture row [clientId, seq, refSeq, msn, contents] to an ISequencedDocumentMessage."""
    cid, seq, ref, msn, contents = m
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


class _VectorView(OracleDoc):
    """One PermutationVector of an OracleMatrix (borrowed handle: never destroyed on its own)."""

    def __init__(self, L, h):
        self._L = L
        self._h = h

    def close(self):
        self._h = None


class OracleMatrix:
    """SharedMatrix observer (matrix.ts:636-697) over two PermutationVectors: rows (0) and cols (1)."""

    def __init__(self, new_length_calc=False, chunk_size=0):
        self._L = lib()
        self._h = self._L.orc_matrix_create(int(new_length_calc), int(chunk_size))
        self.rows = _VectorView(self._L, self._L.orc_matrix_vector(self._h, 0))
        self.cols = _VectorView(self._L, self._L.orc_matrix_vector(self._h, 1))

    def close(self):
        if self._h:
            self._L.orc_matrix_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            raise OracleError(rc, self._L.orc_matrix_last_error(self._h).decode())

    def start_collab(self, long_id, min_seq=0, cur_seq=0):
        self._chk(self._L.orc_matrix_start_collab(self._h, long_id.encode(), min_seq, cur_seq))

    def apply_msg(self, msg):
        raw = msg if isinstance(msg, (bytes, bytearray)) else json.dumps(msg).encode()
        self._chk(self._L.orc_matrix_apply_msg_json(self._h, raw, len(raw)))

    def _take(self, fn, *args):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(fn(self._h, *args, ctypes.byref(p), ctypes.byref(n)))
        try:
            return ctypes.string_at(p, n.value).decode("utf-8")
        finally:
            self._L.orc_free(p)

    def load(self, blobs, observer="snapshot"):
        """SharedMatrix.loadCore (matrix.ts:611-634) from [(path, content)...] as summarize() gives them."""
        raw = json.dumps([list(b) for b in blobs]).encode()
        self._chk(self._L.orc_matrix_load(self._h, raw, len(raw), observer.encode()))

    def summarize(self):
        """SharedMatrix summary (matrix.ts:449-463): {"blobs": [[path, content]...], "summary": {...}}."""
        return json.loads(self._take(self._L.orc_matrix_summarize))

    def get_cell(self, row, col):
        """JSON text of SharedMatrix.getCell(row, col) in the observer's view, or None when undefined."""
        return self._take(self._L.orc_matrix_get_cell, row, col) or None

    def cell_by_handle(self, row_handle, col_handle):
        """JSON text of cells.getCell(rowHandle, colHandle), or None when undefined."""
        s = self._take(self._L.orc_matrix_get_cell_by_handle, row_handle, col_handle)
        return s or None
