"""Python mirror of the reference merge-tree `Client` / `TestClient` surface over the MI355X engine.

Reference interface (packages/dds/merge-tree/src/client.ts:98): `startOrUpdateCollaboration` (:1133),
`applyMsg` (:858), `getLength` (:1129), `getCurrentSeq` (:1122), `summarize` (:966); TestClient adds
`getText` (test/testClient.ts:185) and `insertTextLocal` (detached initial content).

Batched semantics: each `Client` is one document slot of a `MergeTreeBatch`.
`applyMsg` only validates and packs the message; `flush()` -- or any read (`getText`, `getLength`,
`summarize`) -- replays every pending op of every document of the batch on the GPU.  Per-op "delta"
events are not emitted.  Only the observer (remote-op) path is supported; local ops after
collaboration starts raise.
"""
import ctypes
import json

from . import _lib


class MergeTreeError(RuntimeError):
    """Error raised by the engine; `code` is the MTB_E_* value, `message` carries the reference's
    assert code / error text where one exists (e.g. "0x038 ...", "MergeTree insert failed")."""

    def __init__(self, code, message):
        super().__init__(message)
        self.code = code
        self.name = _lib.ERRORS.get(code, str(code))


class UsageError(MergeTreeError):
    """container-utils UsageError equivalent (mergeTree.ts:1671 "MergeTree insert failed")."""


def _check(L, h, rc):
    if rc != 0:
        msg = L.mtb_last_error(h).decode("utf-8", "replace")
        if rc == -5:
            raise UsageError(rc, msg)
        raise MergeTreeError(rc, msg)


def catch_up_ops(blobs):
    """SnapshotLoader.loadBodyAndCatchupOps (snapshotLoader.ts:60-86): the one blob beyond the summary's ordered
    chunks holds the catch-up messages ([] when there is none).  A legacy header (no "version") lists "header",
    and "body" when chunkLengthChars < totalLengthChars (buildHeaderMetadataForLegacyChunk,
    snapshotChunks.ts:178-199)."""
    paths = [p for p, _ in blobs]
    hdr = json.loads(dict(blobs)["header"])
    if hdr.get("version") is None and "headerMetadata" not in hdr:
        ids = ["header"] + (["body"] if hdr.get("chunkLengthChars", 0) < hdr.get("totalLengthChars", 0) else [])
    else:
        ids = [c["id"] for c in hdr["headerMetadata"]["orderedChunkMetadata"]]
    if len(paths) == len(ids) + 1:
        rest = [c for p, c in blobs if p not in ids]
        if len(rest) != 1:
            raise MergeTreeError(-4, "0x060 There should be only one blob with catch up ops")
        c = rest[0]
        return json.loads(c if isinstance(c, str) else bytes(c).decode("utf-8"))
    if len(paths) != len(ids):
        raise MergeTreeError(-1, "Unexpected blobs in snapshot")
    return []


def _loaded_window(blobs):
    """The collab window Client.load starts (snapshotLoader.ts:150-165): minSeq = the header's
    minSequenceNumber ?? sequenceNumber, currentSeq = sequenceNumber (a legacy header: chunkMinSequenceNumber /
    chunkSequenceNumber, snapshotChunks.ts:178-199)."""
    hdr = json.loads(dict(blobs)["header"])
    md = hdr.get("headerMetadata")
    if md is not None:
        seq, mn = md.get("sequenceNumber", 0), md.get("minSequenceNumber")
    else:
        seq, mn = hdr.get("chunkSequenceNumber", 0), hdr.get("chunkMinSequenceNumber")
    return {"minSeq": seq if mn is None else mn, "currentSeq": seq}


class MergeTreeBatch:
    """A batch of independent merge-tree documents replayed together on one MI355X, or spread over several
    (`devices`: documents by hash, each device replaying its share at the same time)."""

    def __init__(self, ndocs, new_length_calc=False, chunk_size=0, device=0, catch_up=False, _flags=0, devices=None):
        """catch_up: keep SharedSegmentSequence's catch-up messages (legacy summaries, MTB_BATCH_CATCHUP)."""
        self._L = _lib.lib()
        opts = _lib.MtbOptions(int(bool(new_length_calc)), int(chunk_size), 64, int(_flags) | (2 if catch_up else 0))
        h = ctypes.c_void_p()
        mask = sum(1 << d for d in devices) if devices else 1 << device
        rc = self._L.mtb_batch_create(ctypes.byref(opts), ndocs, mask, ctypes.byref(h))
        if rc != 0:
            raise MergeTreeError(rc, "mtb_batch_create failed")
        self._h = h
        self.ndocs = ndocs
        self._dirty = False
        self._clients = [Client(self, i) for i in range(ndocs)]
        self.last_stats = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def close(self):
        if getattr(self, "_h", None):
            self._L.mtb_batch_destroy(self._h)
            self._h = None

    def _chk(self, rc):
        _check(self._L, self._h, rc)

    def client(self, i):
        return self._clients[i]

    __getitem__ = client

    def intern_props(self, props):
        """Intern a props object (dict, or its JSON text) and return its id."""
        if isinstance(props, str):
            s = props.encode()
        elif isinstance(props, (bytes, bytearray)):
            s = bytes(props)
        else:
            s = json.dumps(props).encode()
        out = ctypes.c_uint32()
        self._chk(self._L.mtb_intern_props(self._h, s, len(s), ctypes.byref(out)))
        return out.value

    def append_records(self, doc, ops_bytes, n, payload_u16_bytes):
        ob = ctypes.create_string_buffer(bytes(ops_bytes), max(1, len(ops_bytes)))
        pb = ctypes.create_string_buffer(bytes(payload_u16_bytes), max(2, len(payload_u16_bytes)))
        self._chk(self._L.mtb_append_ops(self._h, doc, ob, n, pb, len(payload_u16_bytes) // 2))
        self._dirty = True

    def add_client(self, doc, long_id):
        self._chk(self._L.mtb_add_client(self._h, doc, long_id.encode()))

    def init_doc(self, doc, initial_text, observer_long_id, min_seq=0, cur_seq=0):
        raw = initial_text.encode("utf-16-le", "surrogatepass")
        buf = ctypes.create_string_buffer(raw, max(2, len(raw)))
        self._chk(self._L.mtb_doc_init(self._h, doc, buf, len(raw) // 2, observer_long_id.encode(), min_seq, cur_seq))
        self._dirty = True  # reads flush first: the document reaches the device with the next replay

    @staticmethod
    def _blob_array(blobs):
        pairs = [(p.encode(), c.encode("utf-8") if isinstance(c, str) else bytes(c)) for p, c in blobs]
        arr = (_lib.MtbBlob * max(1, len(pairs)))()
        keep = []
        for i, (p, c) in enumerate(pairs):
            buf = ctypes.create_string_buffer(c, max(1, len(c)))
            keep.append(buf)
            arr[i].path = p
            arr[i].content = ctypes.cast(buf, ctypes.c_void_p)
            arr[i].content_len = len(c)
        return arr, len(pairs), keep

    def load_v1(self, doc, blobs, observer_long_id="snapshot"):
        """Client.load of a SnapshotV1 summary given as [(path, content), ...] (snapshotLoader.ts:41)."""
        arr, n, _keep = self._blob_array(blobs)
        self._chk(self._L.mtb_doc_load_v1(self._h, doc, arr, n, observer_long_id.encode()))
        self._dirty = True

    def load_v1_many(self, docs, summaries, observer_long_ids, threads=16):
        """load_v1 for many documents, parsed on `threads` host threads (mtb_docs_load_v1)."""
        n = len(docs)
        arrs, keep = [], []
        for blobs in summaries:
            arr = (_lib.MtbBlob * max(1, len(blobs)))()
            for i, (p, c) in enumerate(blobs):
                pb = p.encode()
                cb = c.encode("utf-8") if isinstance(c, str) else bytes(c)
                buf = ctypes.create_string_buffer(cb, max(1, len(cb)))
                keep += [pb, buf]
                arr[i].path = pb
                arr[i].content = ctypes.cast(buf, ctypes.c_void_p)
                arr[i].content_len = len(cb)
            arrs.append(arr)
        ptrs = (ctypes.POINTER(_lib.MtbBlob) * max(1, n))(*[ctypes.cast(a, ctypes.POINTER(_lib.MtbBlob)) for a in arrs])
        counts = (ctypes.c_uint32 * max(1, n))(*[len(x) for x in summaries])
        ids = (ctypes.c_uint32 * max(1, n))(*docs)
        obs = (ctypes.c_char_p * max(1, n))(*[o.encode() for o in observer_long_ids])
        self._chk(self._L.mtb_docs_load_v1(self._h, n, ids, ptrs, counts, obs, threads))
        self._dirty = True

    def replay(self):
        """Replay every pending op of every document (blocking).  Returns the stats dict."""
        st = _lib.MtbStats()
        rc = self._L.mtb_replay(self._h, ctypes.byref(st))
        if rc not in (-1, -2, -3):  # the records were replayed (a document error is reported once, sticky)
            self._dirty = False
        self._chk(rc)
        self.last_stats = {f: getattr(st, f) for f, _ in _lib.MtbStats._fields_}
        return self.last_stats

    flush = replay

    def rewind(self):
        """Restore every document to its state before its first replay (records stay in HBM)."""
        self._chk(self._L.mtb_rewind(self._h))

    def replay_resident(self, digests=True):
        """Replay the HBM-resident records again (after rewind); returns the stats dict.  digests=False skips the
        state-digest pass (checksum / segments_final / text_units_final stay 0 until refresh_digests)."""
        st = _lib.MtbStats()
        self._chk(self._L.mtb_replay_resident_ex(self._h, ctypes.byref(st), 0 if digests else 1))
        self.last_stats = {f: getattr(st, f) for f, _ in _lib.MtbStats._fields_}
        return self.last_stats

    def refresh_digests(self):
        """The state digest of every document on its current state (mtb_refresh_digests): the stats dict's
        checksum, segments_final, text_units_final and the write-back term of bytes_alg."""
        st = _lib.MtbStats()
        self._chk(self._L.mtb_refresh_digests(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in _lib.MtbStats._fields_}

    def _ensure_flushed(self):
        if self._dirty:
            self.replay()

    # --- host-side inspection (no GPU) --------------------------------------------------------
    def export_pending(self, doc):
        """(records bytes, n, payload u16 bytes) packed for `doc` and not yet replayed."""
        n, pl = ctypes.c_uint32(), ctypes.c_size_t()
        self._chk(self._L.mtb_export_pending(self._h, doc, None, 0, ctypes.byref(n), None, 0, ctypes.byref(pl)))
        ob = ctypes.create_string_buffer(max(1, n.value * 32))
        pb = ctypes.create_string_buffer(max(2, pl.value * 2))
        self._chk(self._L.mtb_export_pending(self._h, doc, ob, n.value, ctypes.byref(n), pb, pl.value, ctypes.byref(pl)))
        return ob.raw[: n.value * 32], n.value, pb.raw[: pl.value * 2]

    def props_json(self, pid):
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_props_json(self._h, pid, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self._L.mtb_props_json(self._h, pid, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    def client_long_id(self, doc, short_id):
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_client_long_id(self._h, doc, short_id, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self._L.mtb_client_long_id(self._h, doc, short_id, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    # --- per-document read-outs ---------------------------------------------------------------
    def text(self, doc):
        self._ensure_flushed()
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_get_text(self._h, doc, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(2, n.value * 2))
        self._chk(self._L.mtb_get_text(self._h, doc, buf, n.value, ctypes.byref(n)))
        return buf.raw[: n.value * 2].decode("utf-16-le", "surrogatepass")

    def length(self, doc):
        self._ensure_flushed()
        out = ctypes.c_uint32()
        self._chk(self._L.mtb_get_length(self._h, doc, ctypes.byref(out)))
        return out.value

    def seq(self, doc):
        cur, mn = ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self._L.mtb_get_seq(self._h, doc, ctypes.byref(cur), ctypes.byref(mn)))
        return cur.value, mn.value

    def dump_segments(self, doc):
        self._ensure_flushed()
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._chk(self._L.mtb_dump_segments(self._h, doc, ctypes.byref(p), ctypes.byref(n)))
        try:
            return ctypes.string_at(p, n.value).decode("utf-8")
        finally:
            self._L.mtb_free(p)

    def checksum(self, doc):
        self._ensure_flushed()
        out = ctypes.c_uint64()
        self._chk(self._L.mtb_doc_checksum(self._h, doc, ctypes.byref(out)))
        return out.value

    def digests(self, first=0, n=None):
        """State digests v1 of documents [first, first + n) computed on the GPU by the last replay
        (DESIGN.md "State digest"; the oracle's Doc::digest computes the same values)."""
        self._ensure_flushed()
        n = self.ndocs - first if n is None else n
        arr = (ctypes.c_uint64 * max(1, n))()
        self._chk(self._L.mtb_doc_digests(self._h, first, n, arr))
        return list(arr[:n])

    def launch_info(self):
        """What the last replay launched: {"kernel": name, "wave_slots", "chunks", "queues", "aborted", "passes",
        "handover_bad", "cap_retries"}."""
        li = _lib.MtbLaunchInfo()
        self._chk(self._L.mtb_get_launch_info(self._h, ctypes.byref(li)))
        return {"kernel": _lib.KERNEL_NAMES.get(li.kernel), "wave_slots": li.wave_slots, "chunks": li.chunks,
                "queues": li.queues, "aborted": bool(li.aborted), "passes": li.passes,
                "handover_bad": li.handover_bad, "cap_retries": li.cap_retries}

    def map_range(self, doc, start=0, end=-1, ref_seq=-1, long_client_id=None, limit=0):
        """mapRange / nodeMap (mergeTree.ts:2456, 2531) over [start, end) in the (ref_seq, client) view
        (defaults: currentSeq, the observer = the local view): [{"pos", "start", "end", "segment"}...]."""
        self._ensure_flushed()
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_map_range(self._h, doc, start, end, ref_seq,
                                        None if long_client_id is None else long_client_id.encode(), limit,
                                        ctypes.byref(p), ctypes.byref(n)))
        try:
            return json.loads(ctypes.string_at(p, n.value).decode("utf-8"))
        finally:
            self._L.mtb_free(p)

    def debug_blocks(self, doc, ref_seq=-1, long_client_id=None):
        """Diagnostic: per block (tree order) its path, each child block's [length the engine walks, leaf sum] in
        the (ref_seq, client) view and the document's phantom / deficit entries for it (mtb_debug_blocks)."""
        self._ensure_flushed()
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_debug_blocks(self._h, doc, ref_seq, None if long_client_id is None else long_client_id.encode(),
                                           ctypes.byref(p), ctypes.byref(n)))
        try:
            return [json.loads(x) for x in ctypes.string_at(p, n.value).decode("utf-8").splitlines()]
        finally:
            self._L.mtb_free(p)

    def summarize_legacy(self, doc, msn=-1, seq=-1, catchup=None):
        """SnapshotLegacy summary (snapshotlegacy.ts): (blobs, ISummaryTreeWithStats); `catchup` is the list of
        messages above the MSN (SharedSegmentSequence.messagesSinceMSNChange)."""
        self._ensure_flushed()
        lst = _lib.MtbBlobList()
        cu = json.dumps(catchup, separators=(",", ":")).encode() if catchup else None
        self._chk(self._L.mtb_summarize_legacy(self._h, doc, msn, seq, cu, len(cu) if cu else 0, ctypes.byref(lst)))
        return _blob_list(self._L, lst)

    def summarize_v1(self, doc, msn=-1, seq=-1):
        """SnapshotV1 summary: returns (blobs [(path, content)], ISummaryTreeWithStats dict)."""
        self._ensure_flushed()
        lst = _lib.MtbBlobList()
        self._chk(self._L.mtb_summarize_v1(self._h, doc, msn, seq, ctypes.byref(lst)))
        try:
            blobs = [(lst.blobs[i].path.decode(), ctypes.string_at(lst.blobs[i].content, lst.blobs[i].content_len).decode("utf-8"))
                     for i in range(lst.count)]
            summary = json.loads(ctypes.string_at(lst.summary_json, lst.summary_json_len).decode("utf-8"))
        finally:
            self._L.mtb_blob_list_free(ctypes.byref(lst))
        return blobs, summary


    def summarize_v1_many(self, docs, msn=-1, seq=-1, threads=16, fingerprints=False):
        """mtb_summarize_v1_many: the SnapshotV1 summaries of many documents (one replay, one bulk download,
        host threads).  Returns [(blobs, summary)] per document, or with fingerprints=True the FNV-1a 64 of
        each blob list (mtb_blob_list_fnv) without copying the summaries out."""
        self._ensure_flushed()
        n = len(docs)
        lists = (_lib.MtbBlobList * max(1, n))()
        ids = (ctypes.c_uint32 * max(1, n))(*docs)
        import time
        t0 = time.perf_counter()
        self._chk(self._L.mtb_summarize_v1_many(self._h, n, ids, msn, seq, threads, lists))
        self.last_summary_seconds = time.perf_counter() - t0  # the summaries themselves (no copies, no hashing)
        out = []
        for k in range(n):
            if fingerprints:
                h = ctypes.c_uint64()
                self._L.mtb_blob_list_fnv(ctypes.byref(lists[k]), ctypes.byref(h))
                self._L.mtb_blob_list_free(ctypes.byref(lists[k]))
                out.append(h.value)
            else:
                out.append(_blob_list(self._L, lists[k]))
        return out


def _blob_list(L, lst):
    try:
        blobs = [(lst.blobs[i].path.decode(), ctypes.string_at(lst.blobs[i].content, lst.blobs[i].content_len).decode("utf-8"))
                 for i in range(lst.count)]
        summary = json.loads(ctypes.string_at(lst.summary_json, lst.summary_json_len).decode("utf-8"))
    finally:
        L.mtb_blob_list_free(ctypes.byref(lst))
    return blobs, summary


class Client:
    """One document slot with the reference Client/TestClient call shapes."""

    def __init__(self, batch, doc):
        self._b = batch
        self._doc = doc
        self._detached = []  # edits made before collaboration (IMergeTreeOps)
        self.longClientId = None

    # local edits: detached before collaboration (client.replay.spec.ts:27, createClientsAtInitialState
    # testClientLogger.ts:51-78), afterwards a live client's pending ops (client.ts:196, see insertSegmentLocal)
    def insertTextLocal(self, pos, text, props=None):
        seg = text if props is None else {"text": text, "props": props}
        if self.longClientId is not None:
            return self.insertSegmentLocal(pos, seg)
        return self._detach({"pos1": pos, "seg": seg, "type": 0})

    def _detach(self, op):
        if self.longClientId is not None:
            return None
        self._detached.append(op)
        return op

    def startOrUpdateCollaboration(self, longClientId, minSeq=0, currentSeq=0):
        if self.longClientId is not None:
            raise MergeTreeError(-6, "unsupported: re-keying the observer id")
        ops = self._detached
        # one detached text insert into the empty document is the document's initial segment; any other
        # detached edits are replayed as such (seq 0, LocalClientId) before the first message
        first = ops[0] if ops and ops[0]["type"] == 0 and ops[0]["pos1"] == 0 and isinstance(ops[0]["seg"], str) else None
        self._b.init_doc(self._doc, first["seg"] if first else "", longClientId, minSeq, currentSeq)
        for op in ops[1:] if first else ops:
            s = json.dumps(op).encode()
            self._b._chk(self._b._L.mtb_detached_op_json(self._b._h, self._doc, s, len(s)))
        self._detached = []
        self.longClientId = longClientId

    def zamboniSegments(self):
        """zamboniSegments(mergeTree) (zamboni.ts:19-60) as the reference's unit tests call it; applied at the
        next replay."""
        self._b._chk(self._b._L.mtb_maintenance(self._b._h, self._doc, 0))
        self._b._dirty = True

    def packParentRoot(self):
        """packParent(mergeTree.root, mergeTree) (zamboni.ts:63-120) as mergeTree.zamboni.spec.ts calls it."""
        self._b._chk(self._b._L.mtb_maintenance(self._b._h, self._doc, 1))
        self._b._dirty = True

    def load(self, storage, clientId=None):
        """Client.load (client.ts:1007) from a SnapshotV1 or SnapshotLegacy summary.  `storage` maps blob path
        -> content (a dict, or [(path, content), ...]); `clientId` is the runtime's client id (the reference
        falls back to "snapshot", snapshotLoader.ts:154).  The body is appended by the next replay.  Returns
        {"catchupOps": [...]}: the summary's catch-up messages (snapshotLoader.ts:60-86), which
        SharedSegmentSequence applies next (load_sequence)."""
        if self.longClientId is not None or self._detached:
            raise MergeTreeError(-1, "document already initialised")
        blobs = list(storage.items()) if isinstance(storage, dict) else list(storage)
        longId = clientId if clientId is not None else "snapshot"
        self._b.load_v1(self._doc, blobs, longId)
        self.longClientId = longId
        return {"catchupOps": catch_up_ops(blobs), "collabWindow": _loaded_window(blobs)}

    def loadSequence(self, storage, clientId=None):
        """SharedSegmentSequence.loadCore (sequence.ts:568-610): Client.load, then every catch-up message
        checked against the collab window (above minSeq and currentSeq, else "Invalid catchup operations in
        snapshot") and applied.  Returns the catch-up messages."""
        r = self.load(storage, clientId)
        msgs = r["catchupOps"]
        if msgs:
            # the window follows each applied message as getCollabWindow() does in the reference (computed
            # here, not read back: the batch need not replay before the other documents' loads):
            # updateSeqNumbers sets currentSeq, and setMinSeq moves minSeq up to the message's MSN
            cw = r["collabWindow"]
            cur, msn = cw["currentSeq"], cw["minSeq"]
            for m in msgs:
                if (m["minimumSequenceNumber"] < msn or m["referenceSequenceNumber"] < msn or
                        m["sequenceNumber"] <= msn or m["sequenceNumber"] <= cur):
                    raise MergeTreeError(-1, "Invalid catchup operations in snapshot: " + json.dumps(
                        {"op": {"seq": m["sequenceNumber"], "minSeq": m["minimumSequenceNumber"],
                                "refSeq": m["referenceSequenceNumber"]},
                         "collabWindow": {"seq": cur, "minSeq": msn}}))
                self.applyMsg(m)
                cur = m["sequenceNumber"]
                msn = max(msn, m["minimumSequenceNumber"])
        return msgs

    def applyMsg(self, msg, local=False):
        """client.ts:858-887.  A message from this client's own id (`local`) acks its oldest pending op."""
        s = msg if isinstance(msg, (bytes, bytearray)) else (msg.encode() if isinstance(msg, str) else json.dumps(msg).encode())
        self._b._chk(self._b._L.mtb_apply_msg_json(self._b._h, self._doc, s, len(s)))
        self._b._dirty = True

    # ---- a live client's own ops (client.ts:196-247): applied at the next replay, acked by applyMsg
    def applyLocalOp(self, op):
        """Queue the IMergeTreeOp `op` (dict or JSON) as this client's local op; returns it."""
        s = op if isinstance(op, (bytes, bytearray)) else (op.encode() if isinstance(op, str) else json.dumps(op).encode())
        self._b._chk(self._b._L.mtb_local_op_json(self._b._h, self._doc, s, len(s)))
        self._b._dirty = True
        return op

    def insertSegmentLocal(self, pos, seg):
        """insertSegmentLocal (client.ts:196): `seg` is an IJSONSegment (text, {"text", "props"} or
        {"marker": {...}, "props"}); returns the IMergeTreeInsertMsg to send."""
        return self.applyLocalOp({"pos1": pos, "seg": seg, "type": 0})

    def removeRangeLocal(self, start, end):
        """removeRangeLocal (client.ts:230): returns the IMergeTreeRemoveMsg to send (before collaboration a
        detached remove: the segments stay as tombstones with removedSeq UniversalSequenceNumber)."""
        op = {"pos1": start, "pos2": end, "type": 1}
        return self._detach(op) if self.longClientId is None else self.applyLocalOp(op)

    def regeneratePendingOp(self, resetOp, segmentGroup=None):
        """Client.regeneratePendingOp (client.ts:917-960) after a reconnect: `resetOp` is the oldest pending op
        as it was submitted (its segment groups are the oldest pending ones); returns the op to resubmit."""
        s = resetOp if isinstance(resetOp, (bytes, bytearray)) else (
            resetOp.encode() if isinstance(resetOp, str) else json.dumps(resetOp).encode())
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        L = self._b._L
        self._b._chk(L.mtb_regenerate_pending_op(self._b._h, self._doc, s, len(s), ctypes.byref(p), ctypes.byref(n)))
        self._b._dirty = False
        try:
            return json.loads(ctypes.string_at(p, n.value).decode("utf-8"))
        finally:
            L.mtb_free(p)

    def annotateMarker(self, markerId, props, combiningOp=None):
        """Client.annotateMarker (client.ts:190-197, createAnnotateMarkerOp opBuilder.ts:25-43) for the marker
        carrying `markerId`: a local annotate with marker-relative positions; returns the op to send."""
        op = {"props": props, "relativePos1": {"id": markerId, "before": True}, "relativePos2": {"id": markerId},
              "type": 2}
        return self.applyLocalOp(op if combiningOp is None else {"combiningOp": combiningOp, **op})

    def annotateMarkerNotifyConsensus(self, markerId, props):
        """Client.annotateMarkerNotifyConsensus (client.ts:155-181): a local consensus annotate of the marker carrying
        `markerId` -- each key gets {value: undefined, seq: -1} until the op's ack completes it with the ack's seq
        (updateConsensusProperty, client.ts:1050-1058); returns the op to send.  (The reference's consensus callback,
        an application notification at a later minimum sequence number, is not part of the replayed state.)"""
        op = {"combiningOp": {"name": "consensus"}, "props": props, "relativePos1": {"id": markerId, "before": True},
              "relativePos2": {"id": markerId}, "type": 2}
        self.applyLocalOp(dict(op, notifyConsensus=True))
        return op

    def annotateRangeLocal(self, start, end, props, combiningOp=None):
        """annotateRangeLocal (client.ts:206): the keys stay pending on the annotated segments until the
        op's ack (a "rewrite" combiningOp: pendingRewriteCount; other combiningOps are rejected by the
        engine); returns the IMergeTreeAnnotateMsg to send."""
        op = {"pos1": start, "pos2": end, "props": props, "type": 2}
        op = op if combiningOp is None else {"combiningOp": combiningOp, **op}
        return self._detach(op) if self.longClientId is None else self.applyLocalOp(op)

    def getText(self, start=None, end=None):
        """TestClient.getText (testClient.ts:185): the local view's text, or of [start, end) in positions that
        count markers (MergeTreeTextHelper.getText's mapRange + gatherText; markers add no text)."""
        if start is None and end is None:
            return self._b.text(self._doc)
        out = []
        for h in self._b.map_range(self._doc, start or 0, -1 if end is None else end):
            seg = h["segment"]
            if seg.get("type") != "TextSegment":
                continue
            t = seg["text"]
            s0 = max(0, h["start"])
            out.append(t[s0:] if h["end"] >= len(t) else t[s0:h["end"]])
        return "".join(out)

    # ---- TestClient helpers (test/testClient.ts:224-327): sequenced messages of other clients
    def makeOpMessage(self, op, seq=-1, refSeq=None, longClientId=None, minSeqNumber=0):
        """TestClient.makeOpMessage (testClient.ts:303-327)."""
        if op is None:
            raise MergeTreeError(-1, "op cannot be undefined")
        return {"clientId": longClientId if longClientId is not None else (self.longClientId or ""),
                "clientSequenceNumber": 1, "contents": op, "minimumSequenceNumber": minSeqNumber,
                "referenceSequenceNumber": self.getCurrentSeq() if refSeq is None else refSeq,
                "sequenceNumber": seq, "term": 1, "traces": [], "type": "op"}

    def insertTextRemote(self, pos, text, props, seq, refSeq, longClientId):
        seg = {"text": text, "props": props} if props else text
        self.applyMsg(self.makeOpMessage({"pos1": pos, "seg": seg, "type": 0}, seq, refSeq, longClientId))

    def removeRangeRemote(self, start, end, seq, refSeq, longClientId):
        self.applyMsg(self.makeOpMessage({"pos1": start, "pos2": end, "type": 1}, seq, refSeq, longClientId))

    def annotateRangeRemote(self, start, end, props, seq, refSeq, longClientId):
        self.applyMsg(self.makeOpMessage({"pos1": start, "pos2": end, "props": props, "type": 2}, seq, refSeq,
                                         longClientId))

    def insertMarkerRemote(self, pos, markerDef, props, seq, refSeq, longClientId):
        """markerDef {refType?} (default ReferenceType.Tile = 1, testClient.ts:281)."""
        seg = {"marker": {"refType": (markerDef or {}).get("refType", 1)}}
        if props:
            seg["props"] = props
        self.applyMsg(self.makeOpMessage({"pos1": pos, "seg": seg, "type": 0}, seq, refSeq, longClientId))

    def insertMarkerLocal(self, pos, behaviors, props=None):
        """A live client's marker insert (testClient.ts:270-276); returns the op to send."""
        seg = {"marker": {"refType": behaviors}}
        if props:
            seg["props"] = props
        if self.longClientId is None:
            return self._detach({"pos1": pos, "seg": seg, "type": 0})
        return self.insertSegmentLocal(pos, seg)

    def getContainingSegment(self, pos, sequenceArgs=None):
        """client.ts:1065: {"segment": dict | None, "offset": int | None} in the local view, or in the
        view of sequenceArgs = {"referenceSequenceNumber", "clientId"} (a remote message's perspective)."""
        ref, cid = (-1, None) if sequenceArgs is None else (sequenceArgs["referenceSequenceNumber"], sequenceArgs["clientId"])
        hit = self._b.map_range(self._doc, pos, pos + 1, ref, cid, limit=1)
        return {"segment": hit[0]["segment"], "offset": hit[0]["start"]} if hit else {"segment": None, "offset": None}

    def getPropertiesAtPosition(self, pos):
        """client.ts:1101: the properties of the segment at pos (local view), or None."""
        seg = self.getContainingSegment(pos)["segment"]
        return None if seg is None else seg.get("properties")

    def walkSegments(self, handler, start=None, end=None, accum=None):
        """client.ts:286 (mapRange in the local view): handler(segment, pos, refSeq, clientId, start, end,
        accum) per visited segment; returning False stops the walk.  splitRange is not supported."""
        cur = self.getCurrentSeq()
        for e in self._b.map_range(self._doc, start or 0, -1 if end is None else end):
            if handler(e["segment"], e["pos"], cur, 0, e["start"], e["end"], accum) is False:
                break

    def getClientId(self):
        """client.ts:1126: the observer's short id."""
        return 0

    def getLongClientId(self, shortClientId):
        return self._b.client_long_id(self._doc, shortClientId)

    def getLength(self):
        return self._b.length(self._doc)

    def getCurrentSeq(self):
        self._b._ensure_flushed()
        return self._b.seq(self._doc)[0]

    def getCollabWindow(self):
        self._b._ensure_flushed()
        cur, mn = self._b.seq(self._doc)
        return {"clientId": 0, "collaborating": True, "minSeq": mn, "currentSeq": cur}

    def summarize(self, minimumSequenceNumber=None, lastSequenceNumber=None):
        """Client.summarize with newMergeTreeSnapshotFormat=true -> ISummaryTreeWithStats (dict)."""
        msn = -1 if minimumSequenceNumber is None else minimumSequenceNumber
        seq = -1 if lastSequenceNumber is None else lastSequenceNumber
        return self._b.summarize_v1(self._doc, msn, seq)[1]


MTB_BATCH_MATRIX = 1


TestClient = Client  # testClient.ts:54: the same slot with the TestClient helpers above


class MatrixBatch(MergeTreeBatch):
    """A batch of SharedMatrix observers (matrix.ts): matrix m is the PermutationVector documents 2m (rows)
    and 2m+1 (cols).  Vector ops and setCell handle allocation replay on the GPU; the kernel's cell events
    (setCell handles, recycled handles) are replayed on the host into each matrix's SparseArray2D."""

    def __init__(self, nmatrices, new_length_calc=False, chunk_size=0, device=0):
        super().__init__(2 * nmatrices, new_length_calc=new_length_calc, chunk_size=chunk_size, device=device,
                         _flags=MTB_BATCH_MATRIX)
        self.nmatrices = nmatrices
        self._matrices = [SharedMatrix(self, m) for m in range(nmatrices)]

    def matrix(self, m):
        return self._matrices[m]

    __getitem__ = matrix

    def init_matrix(self, m, observer_long_id, min_seq=0, cur_seq=0):
        self._chk(self._L.mtb_matrix_init(self._h, m, observer_long_id.encode(), min_seq, cur_seq))
        self._dirty = True

    def load_matrix(self, m, blobs, observer_long_id="snapshot"):
        """SharedMatrix.loadCore (matrix.ts:611) from [(path, content), ...] as matrix_summarize gives them."""
        arr, n, _keep = self._blob_array(blobs)
        self._chk(self._L.mtb_matrix_load(self._h, m, arr, n, observer_long_id.encode()))
        self._dirty = True

    def intern_value(self, value_json):
        """Id of a setCell value (JSON text) for SETCELL records packed by the caller (0 = undefined)."""
        raw = value_json.encode()
        out = ctypes.c_uint32()
        self._chk(self._L.mtb_matrix_intern_value(self._h, raw, len(raw), ctypes.byref(out)))
        return out.value

    def matrix_summarize(self, m):
        """SharedMatrix.summarizeCore (matrix.ts:449): (blobs [(path, content)], ISummaryTreeWithStats)."""
        self._ensure_flushed()
        lst = _lib.MtbBlobList()
        self._chk(self._L.mtb_matrix_summarize(self._h, m, ctypes.byref(lst)))
        return _blob_list(self._L, lst)

    def matrix_summary_fnv(self, m):
        """FNV-1a 64 of matrix m's SharedMatrix summary blobs (mtb_blob_list_fnv over the blob paths and
        contents; the ISummaryTreeWithStats JSON left out) without copying them out (parity checks at scale)."""
        self._ensure_flushed()
        lst = _lib.MtbBlobList()
        self._chk(self._L.mtb_matrix_summarize(self._h, m, ctypes.byref(lst)))
        h = ctypes.c_uint64()
        js = lst.summary_json
        try:
            lst.summary_json = None
            self._chk(self._L.mtb_blob_list_fnv(ctypes.byref(lst), ctypes.byref(h)))
        finally:
            lst.summary_json = js
            self._L.mtb_blob_list_free(ctypes.byref(lst))
        return h.value

    def get_cell(self, m, row, col):
        """SharedMatrix.getCell (matrix.ts:173): the value's JSON text, or None when undefined."""
        self._ensure_flushed()
        buf = ctypes.create_string_buffer(1 << 16)
        n = ctypes.c_size_t()
        self._chk(self._L.mtb_matrix_get_cell(self._h, m, row, col, buf, len(buf), ctypes.byref(n)))
        if n.value >= len(buf):
            buf = ctypes.create_string_buffer(n.value + 1)
            self._chk(self._L.mtb_matrix_get_cell(self._h, m, row, col, buf, len(buf), ctypes.byref(n)))
        return buf.value.decode("utf-8") if n.value else None

    def apply_matrix_msg(self, m, msg):
        s = msg if isinstance(msg, (bytes, bytearray)) else (msg.encode() if isinstance(msg, str) else json.dumps(msg).encode())
        self._chk(self._L.mtb_matrix_apply_msg_json(self._h, m, s, len(s)))
        self._dirty = True


class SharedMatrix:
    """SharedMatrix observer slot: startOrUpdateCollaboration / applyMsg (processCore, matrix.ts:636) and
    the two PermutationVector summaries (permutationvector.ts:310)."""

    def __init__(self, batch, m):
        self._b = batch
        self._m = m

    def startOrUpdateCollaboration(self, longClientId, minSeq=0, currentSeq=0):
        self._b.init_matrix(self._m, longClientId, minSeq, currentSeq)

    def applyMsg(self, msg):
        self._b.apply_matrix_msg(self._m, msg)

    def load(self, storage, clientId=None):
        """SharedMatrix.loadCore (matrix.ts:611-634): `storage` maps blob path -> content (dict or pairs)."""
        blobs = list(storage.items()) if isinstance(storage, dict) else list(storage)
        self._b.load_matrix(self._m, blobs, clientId if clientId is not None else "snapshot")

    @property
    def rows_doc(self):
        return 2 * self._m

    @property
    def cols_doc(self):
        return 2 * self._m + 1

    def summarize(self):
        """SharedMatrix.summarizeCore (matrix.ts:449-463): (blobs, ISummaryTreeWithStats) with the rows / cols
        PermutationVector summaries and the cells blob."""
        return self._b.matrix_summarize(self._m)

    def getCell(self, row, col):
        """matrix.ts:173: the cell's value (parsed JSON), or None when undefined."""
        v = self._b.get_cell(self._m, row, col)
        return None if v is None else json.loads(v)
