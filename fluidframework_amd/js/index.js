"use strict";
/*
 * @fluid-mi355x/merge-tree-batch — drop-in for the observer (remote-op) path of the reference
 * merge-tree `Client` (packages/dds/merge-tree/src/client.ts:98) and its test harness `TestClient`
 * (packages/dds/merge-tree/src/test/testClient.ts:54), backed by the MI355X replay engine.
 *
 * Each Client is one document slot of a MergeTreeBatch.  applyMsg(msg) validates and packs the
 * ISequencedDocumentMessage (no GPU work); flush() -- or any read (getText, getLength, summarize,
 * getCurrentSeq) -- replays every pending op of every document of the batch in one GPU launch.
 * Per-op "delta"/"maintenance" events are not emitted in batched mode.  Local edits are accepted
 * only before startOrUpdateCollaboration (detached initial content, client.replay.spec.ts:27).
 *
 * Errors keep the reference's messages: a failed insert throws an Error named "UsageError" with
 * message "MergeTree insert failed" (mergeTree.ts:1671); out-of-order sequence numbers throw with
 * the reference assert code ("0x038 ...", client.ts:880).  There is no CPU fallback: without a GPU,
 * flush() throws with code -2 (MTB_E_NODEV).
 */
const path = require("path");

const native = require(path.join(__dirname, "mtb_napi.node"));

const ERR_UNSUPPORTED = -6;

function unsupported(what) {
  const e = new Error(`unsupported: ${what}`);
  e.code = ERR_UNSUPPORTED;
  e.name = "MergeTreeBatchError";
  return e;
}

const MTB_BATCH_MATRIX = 1;
const MTB_BATCH_CATCHUP = 2;

class MergeTreeBatch {
  /**
   * @param {number} ndocs documents in the batch
   * @param {object} [options] IMergeTreeOptions subset: mergeTreeUseNewLengthCalculations
   *   (mergeTree.ts:413), mergeTreeSnapshotChunkSize (snapshotV1.ts:37); plus `device` (GPU index)
   */
  /**
   * options: mergeTreeUseNewLengthCalculations, mergeTreeSnapshotChunkSize, device, and
   * newMergeTreeSnapshotFormat (IMergeTreeOptions, mergeTree.ts:413): without it summaries use
   * SnapshotLegacy and the batch keeps SharedSegmentSequence's catch-up messages (sequence.ts:697-748).
   */
  constructor(ndocs, options = {}, _rawDocs = undefined, _flags = 0) {
    const n = _rawDocs === undefined ? ndocs : _rawDocs;
    this.ndocs = n;
    this.v1 = options.newMergeTreeSnapshotFormat !== false;
    const catchUp = !this.v1 && !(_flags & MTB_BATCH_MATRIX) ? MTB_BATCH_CATCHUP : 0;
    // options.devices: GPU indices to spread the documents over (one engine and stream per device)
    const mask = Array.isArray(options.devices) ? options.devices.reduce((m, d) => m | (1 << d), 0) >>> 0 : 0;
    this.handle = native.create(n, options.mergeTreeUseNewLengthCalculations ? 1 : 0,
      options.mergeTreeSnapshotChunkSize || 0, options.device || 0, _flags | catchUp, mask);
    this.dirty = false;
    this.busy = false;
    this.lastStats = undefined;
    this.clients = [];
    // every slot is a TestClient (a Client plus the testClient.ts message helpers)
    for (let i = 0; i < ndocs; i++) this.clients.push(new TestClient(this, i));
  }

  client(i) { return this.clients[i]; }

  /** Per-document state digests (16-digit hex) of documents [first, first + n), computed on the GPU. */
  digests(first = 0, n = this.ndocs - first) {
    this.ensureFlushed();
    return native.digests(this.handle, first, n);
  }

  /**
   * SnapshotV1 summaries of many documents at once (one bulk download, `threads` host threads):
   * [{blobs: [[path, content], ...], summary}] in the order of `docs`; msn / seq < 0: the current window.
   */
  summarizeV1Many(docs, msn = -1, seq = -1, threads = 0) {
    this.ensureFlushed();
    return native.summarizeV1Many(this.handle, docs, msn, seq, threads);
  }

  checkIdle() {
    if (this.busy) throw new Error("MergeTreeBatch: an asynchronous flush is in progress");
  }

  /** Replay every pending op of every document (blocking).  Returns the replay statistics. */
  flush() {
    this.checkIdle();
    try {
      this.lastStats = native.replay(this.handle);
    } catch (e) {
      // a document's failure is thrown once (the reference throws from that applyMsg); the other
      // documents' records were replayed
      if (![-1, -2, -3].includes(e.code)) this.dirty = false;  // not MTB_E_ARG / NODEV / HIP
      throw e;
    }
    this.dirty = false;
    return this.lastStats;
  }

  /** flush() on the libuv thread pool; the batch must not be touched until the promise settles. */
  flushAsync() {
    this.checkIdle();
    this.busy = true;
    return native.replayAsync(this.handle).then((st) => {
      this.busy = false;
      this.dirty = false;
      this.lastStats = st;
      return st;
    }, (e) => {
      this.busy = false;
      throw e;
    });
  }

  ensureFlushed() {
    this.checkIdle();
    if (this.dirty) this.flush();
  }

  internProps(props) {
    this.checkIdle();
    return native.internProps(this.handle, typeof props === "string" ? props : JSON.stringify(props));
  }

  /** Pre-packed records (32-byte mtb_op each, include/mtb.h) and their UTF-16 payload. */
  appendOps(doc, records, payload) {
    this.checkIdle();
    native.appendOps(this.handle, doc, records, payload);
    this.dirty = true;
  }

  addClient(doc, longId) {
    this.checkIdle();
    native.addClient(this.handle, doc, longId);
  }

  /** Canonical segment dump (parity read-out; one JSON line per segment). */
  dumpSegments(doc) {
    this.ensureFlushed();
    return native.dumpSegments(this.handle, doc);
  }

  checksum(doc) {
    this.ensureFlushed();
    return native.checksum(this.handle, doc);
  }

  /** SnapshotV1 blobs [[path, content], ...] and the ISummaryTreeWithStats object. */
  summarizeV1(doc, msn = -1, seq = -1) {
    this.ensureFlushed();
    const r = native.summarizeV1(this.handle, doc, msn, seq);
    return { blobs: r.blobs, summary: JSON.parse(r.summary) };
  }

  /** SnapshotLegacy blobs (header / body / catchupOps) and the ISummaryTreeWithStats object. */
  summarizeLegacy(doc, msn = -1, seq = -1, catchUpMsgs = undefined) {
    this.ensureFlushed();
    const r = native.summarizeLegacy(this.handle, doc, msn, seq,
      catchUpMsgs === undefined ? null : JSON.stringify(catchUpMsgs));
    return { blobs: r.blobs, summary: JSON.parse(r.summary) };
  }

  /** Benchmark utilities: restore every document to its pre-replay state / replay resident records. */
  rewind() {
    this.checkIdle();
    native.rewind(this.handle);
  }

  replayResident() {
    this.checkIdle();
    return native.replayResident(this.handle);
  }
}

/** One document slot with the reference Client / TestClient call shapes (observer path). */
class Client {
  constructor(batch, doc) {
    this.batch = batch;
    this.doc = doc;
    this.detached = [];  // edits before collaboration (IMergeTreeOps)
    this.longClientId = undefined;
  }

  // ---- detached content (before collaboration) ------------------------------------------------
  /**
   * TestClient.insertTextLocal (testClient.ts:195): detached text before startOrUpdateCollaboration; while
   * collaborating, a live client's local insert (insertSegmentLocal) whose op is returned.
   */
  insertTextLocal(pos, text, props) {
    const seg = props === undefined ? text : { text, props };
    if (this.longClientId !== undefined) return this.insertSegmentLocal(pos, seg);
    return this.detach({ pos1: pos, seg, type: 0 });
  }

  /** An edit before collaboration (createClientsAtInitialState, testClientLogger.ts:51-78): kept until
   * startOrUpdateCollaboration, then applied at seq 0 by LocalClientId (segments and tombstones). */
  detach(op) {
    this.detached.push(op);
    return op;
  }

  /** zamboniSegments(mergeTree) (zamboni.ts:19-60), as the reference's unit tests call it. */
  zamboniSegments() {
    this.batch.checkIdle();
    native.maintenance(this.batch.handle, this.doc, 0);
    this.batch.dirty = true;
  }

  /** packParent(mergeTree.root, mergeTree) (zamboni.ts:63-120), as mergeTree.zamboni.spec.ts calls it. */
  packParentRoot() {
    this.batch.checkIdle();
    native.maintenance(this.batch.handle, this.doc, 1);
    this.batch.dirty = true;
  }

  // ---- a live client's own ops (client.ts:196-247): applied at the next flush in this client's view,
  // acked when its sequenced message comes back through applyMsg
  /** Queue an IMergeTreeOp (insert / remove, or a group of them) as this client's local op; returns it. */
  applyLocalOp(op) {
    this.batch.checkIdle();
    native.localOp(this.batch.handle, this.doc, typeof op === "string" ? op : JSON.stringify(op));
    this.batch.dirty = true;
    return op;
  }

  /** Client.insertSegmentLocal (client.ts:196): `seg` is an IJSONSegment; returns the insert op to send. */
  insertSegmentLocal(pos, seg) {
    return this.applyLocalOp({ pos1: pos, seg, type: 0 });
  }

  /** Client.removeRangeLocal (client.ts:230): returns the remove op to send. */
  removeRangeLocal(start, end) {
    const op = { pos1: start, pos2: end, type: 1 };
    return this.longClientId === undefined ? this.detach(op) : this.applyLocalOp(op);
  }

  /** Client.regeneratePendingOp (client.ts:917-960): the op to resubmit after a reconnect for the oldest
   * pending op `resetOp` (the batch is flushed first). */
  regeneratePendingOp(resetOp, segmentGroup) {
    this.batch.checkIdle();
    const out = native.regeneratePendingOp(this.batch.handle, this.doc, typeof resetOp === "string" ? resetOp : JSON.stringify(resetOp));
    this.batch.dirty = false;
    return JSON.parse(out);
  }

  /** Client.annotateMarker (client.ts:190) for the marker carrying `markerId`: returns the op to send. */
  annotateMarker(markerId, props, combiningOp) {
    // createAnnotateMarkerOp (opBuilder.ts:25-43); a combiningOp other than "rewrite" is rejected by the engine
    const op = { props, relativePos1: { id: markerId, before: true }, relativePos2: { id: markerId }, type: 2 };
    return this.applyLocalOp(combiningOp === undefined ? op : { combiningOp, ...op });
  }

  /** Client.annotateMarkerNotifyConsensus (client.ts:155-181): each key of `props` is {value: undefined, seq: -1}
   * on the marker until the op's ack completes it with the ack's seq (updateConsensusProperty, :1050-1058);
   * returns the op to send. */
  annotateMarkerNotifyConsensus(markerId, props) {
    const op = { combiningOp: { name: "consensus" }, props, relativePos1: { id: markerId, before: true },
      relativePos2: { id: markerId }, type: 2 };
    this.applyLocalOp({ ...op, notifyConsensus: true });
    return op;
  }

  /** Client.annotateRangeLocal (client.ts:206): the keys stay pending until the op's ack; returns the op. */
  annotateRangeLocal(start, end, props, combiningOp) {
    // createAnnotateRangeOp (opBuilder.ts:52-65): a local "rewrite" is pending (pendingRewriteCount) until its ack
    const op0 = { pos1: start, pos2: end, props, type: 2 };
    const op = combiningOp === undefined ? op0 : { combiningOp, ...op0 };
    return this.longClientId === undefined ? this.detach(op) : this.applyLocalOp(op);
  }

  /** Client.startOrUpdateCollaboration (client.ts:1133).  One detached text insert into the empty document
   * is its initial segment; other detached edits are applied (seq 0, LocalClientId) before the first message. */
  startOrUpdateCollaboration(longClientId, minSeq = 0, currentSeq = 0) {
    if (this.longClientId !== undefined) throw unsupported("re-keying the observer id");
    const ops = this.detached;
    const first = ops.length && ops[0].type === 0 && ops[0].pos1 === 0 && typeof ops[0].seg === "string" ? ops[0] : undefined;
    native.docInit(this.batch.handle, this.doc, first ? first.seg : "", longClientId, minSeq, currentSeq);
    for (const op of first ? ops.slice(1) : ops) native.detachedOp(this.batch.handle, this.doc, JSON.stringify(op));
    this.detached = [];
    this.longClientId = longClientId;
  }

  /**
   * Client.load (client.ts:1007) of a SnapshotV1 summary through SnapshotLoader (snapshotLoader.ts:41):
   * `storage.readBlob(path)` gives the blob contents (string, Uint8Array or ArrayBuffer);
   * `runtime.clientId` becomes the observer id ("snapshot" when absent, snapshotLoader.ts:154).  The
   * header is rebuilt at once; the body chunks are appended by the next flush.  Catch-up ops do not
   * exist in the V1 format, so `catchupOpsP` resolves to [].
   */
  async load(runtime, storage) {
    if (this.longClientId !== undefined || this.detached.length) throw new Error("document already initialised");
    const text = (x) => (typeof x === "string" ? x : Buffer.from(x instanceof ArrayBuffer ? new Uint8Array(x) : x).toString("utf8"));
    const header = text(await storage.readBlob("header"));
    const blobs = [["header", header]];
    const h = JSON.parse(header);
    // toLatestVersion (snapshotChunks.ts:151-199): a legacy header (no "version") lists "body" when
    // chunkLengthChars < totalLengthChars
    const md = h.headerMetadata;
    const ids = md && Array.isArray(md.orderedChunkMetadata) ? md.orderedChunkMetadata.map((c) => c.id)
      : ["header"].concat(h.version === undefined && h.chunkLengthChars < h.totalLengthChars ? ["body"] : []);
    for (const id of ids.slice(1)) blobs.push([id, text(await storage.readBlob(id))]);
    const longId = runtime && runtime.clientId !== undefined ? runtime.clientId : "snapshot";
    native.loadV1(this.batch.handle, this.doc, blobs, longId);
    this.longClientId = longId;
    this.batch.dirty = true;
    // the window startOrUpdateCollaboration opened (snapshotLoader.ts:150-165)
    const seq = md ? md.sequenceNumber : h.chunkSequenceNumber;
    const mn = md ? md.minSequenceNumber : h.chunkMinSequenceNumber;
    this.loadedWindow = { minSeq: mn === undefined ? seq : mn, currentSeq: seq };
    // loadBodyAndCatchupOps (snapshotLoader.ts:60-86): the one blob beyond the ordered chunks
    let catchup = [];
    if (typeof storage.list === "function") {
      const all = await storage.list("");
      if (all.length === ids.length + 1) {
        const rest = all.filter((p) => !ids.includes(p));
        if (rest.length !== 1) throw new Error("0x060 There should be only one blob with catch up ops");
        catchup = JSON.parse(text(await storage.readBlob(rest[0])));
      } else if (all.length !== ids.length) {
        throw new Error("Unexpected blobs in snapshot");
      }
    }
    return { catchupOpsP: Promise.resolve(catchup) };
  }

  /**
   * SharedSegmentSequence.loadCore (sequence.ts:568-610): Client.load, then each catch-up message checked
   * against the collab window and applied.  Resolves to the catch-up messages.
   */
  async loadSequence(runtime, storage) {
    const { catchupOpsP } = await this.load(runtime, storage);
    const msgs = await catchupOpsP;
    if (msgs.length) {
      // the window follows each applied message as getCollabWindow() does in the reference (computed, not
      // read back, so the batch's other loads need no flush): currentSeq = seq, minSeq up to the MSN
      const cw = this.loadedWindow;
      let cur = cw.currentSeq;
      let msn = cw.minSeq;
      for (const m of msgs) {
        if (m.minimumSequenceNumber < msn || m.referenceSequenceNumber < msn ||
            m.sequenceNumber <= msn || m.sequenceNumber <= cur) {
          throw new Error(`Invalid catchup operations in snapshot: ${JSON.stringify({
            op: { seq: m.sequenceNumber, minSeq: m.minimumSequenceNumber, refSeq: m.referenceSequenceNumber },
            collabWindow: { seq: cur, minSeq: msn } })}`);
        }
        this.applyMsg(m);
        cur = m.sequenceNumber;
        msn = Math.max(msn, m.minimumSequenceNumber);
      }
    }
    return msgs;
  }

  // ---- op application ---------------------------------------------------------------------------
  /** Client.applyMsg (client.ts:858): `msg` is an ISequencedDocumentMessage (object or JSON text). */
  applyMsg(msg, local = false) {
    this.batch.checkIdle();  // (a message with this client's own id acks its oldest pending op)
    native.applyMsg(this.batch.handle, this.doc, typeof msg === "string" ? msg : JSON.stringify(msg));
    this.batch.dirty = true;
  }

  /** Client.updateSeqNumbers is folded into applyMsg (client.ts:874); summarize takes (msn, seq). */

  // ---- reads (flush first) ----------------------------------------------------------------------
  /** TestClient.getText (testClient.ts:185). */
  getText(start, end) {
    this.batch.ensureFlushed();
    if (start === undefined && end === undefined) return native.getText(this.batch.handle, this.doc);
    // a range: MergeTreeTextHelper.getText's mapRange + gatherText over [start, end) in the local view
    // (positions count markers; markers add no text)
    const hits = JSON.parse(native.mapRange(this.batch.handle, this.doc, start || 0, end === undefined ? -1 : end, -1, null, 0));
    let t = "";
    for (const h of hits) {
      if (h.segment.type !== "TextSegment") continue;
      const seg = h.segment.text;
      const s0 = h.start < 0 ? 0 : h.start;
      t += h.end >= seg.length ? seg.substring(s0) : seg.substring(s0, h.end);
    }
    return t;
  }

  /** Client.getLength (client.ts:1129). */
  getLength() {
    this.batch.ensureFlushed();
    return native.getLength(this.batch.handle, this.doc);
  }

  /** Client.getCurrentSeq (client.ts:1122). */
  getCurrentSeq() {
    this.batch.ensureFlushed();
    return native.getSeq(this.batch.handle, this.doc)[0];
  }

  /** Client.getCollabWindow (client.ts:348), observer view. */
  getCollabWindow() {
    this.batch.ensureFlushed();
    const [currentSeq, minSeq] = native.getSeq(this.batch.handle, this.doc);
    return { clientId: 0, collaborating: true, minSeq, currentSeq };
  }

  /**
   * Client.getContainingSegment (client.ts:1065, mergeTree.ts:787-813): {segment, offset} in the local
   * view, or in the view of `sequenceArgs` = {referenceSequenceNumber, clientId} (a remote message's).
   * Segments are plain objects {type, text | refType | start, cachedLength, seq, clientId,
   * removedSeq?, removedClientIds?, properties?} with short client ids.
   */
  getContainingSegment(pos, sequenceArgs) {
    this.batch.ensureFlushed();
    const ref = sequenceArgs ? sequenceArgs.referenceSequenceNumber : -1;
    const id = sequenceArgs ? sequenceArgs.clientId : null;
    const hit = JSON.parse(native.mapRange(this.batch.handle, this.doc, pos, pos + 1, ref, id, 1));
    return hit.length ? { segment: hit[0].segment, offset: hit[0].start } : { segment: undefined, offset: undefined };
  }

  /** Client.getPropertiesAtPosition (client.ts:1101). */
  getPropertiesAtPosition(pos) {
    const { segment } = this.getContainingSegment(pos);
    return segment ? segment.properties : undefined;
  }

  /**
   * Client.walkSegments (client.ts:286): mapRange in the local view; handler(segment, pos, refSeq,
   * clientId, start, end, accum) returning false stops the walk.  splitRange is not supported.
   */
  walkSegments(handler, start, end, accum, splitRange = false) {
    if (splitRange) throw unsupported("walkSegments with splitRange on the observer engine");
    this.batch.ensureFlushed();
    const cur = this.getCurrentSeq();
    const hits = JSON.parse(native.mapRange(this.batch.handle, this.doc, start || 0, end === undefined ? -1 : end, -1, null, 0));
    for (const h of hits) if (handler(h.segment, h.pos, cur, 0, h.start, h.end, accum) === false) break;
  }

  /** Client.getClientId (client.ts:1126): the observer's short id. */
  getClientId() { return 0; }

  /** Client.getLongClientId (client.ts:682). */
  getLongClientId(shortClientId) { return native.clientLongId(this.batch.handle, this.doc, shortClientId); }

  /**
   * Client.summarize (client.ts:966) with newMergeTreeSnapshotFormat: the SnapshotV1 summary tree.
   * `runtime.deltaManager.{minimumSequenceNumber,lastSequenceNumber}` (client.ts:979) are passed
   * through when given.
   */
  summarize(runtime, handle, serializer, catchUpMsgs) {
    const dm = runtime && runtime.deltaManager;
    const msn = dm && dm.minimumSequenceNumber !== undefined ? dm.minimumSequenceNumber : -1;
    const seq = dm && dm.lastSequenceNumber !== undefined ? dm.lastSequenceNumber : -1;
    if (this.batch.v1) return this.batch.summarizeV1(this.doc, msn, seq).summary;
    // SnapshotLegacy (client.ts:999-1003); catchUpMsgs default to the messages the batch tracked
    return this.batch.summarizeLegacy(this.doc, msn, seq, catchUpMsgs).summary;
  }
}

/**
 * A batch of SharedMatrix observers (matrix.ts): matrix m is the PermutationVector documents 2m (rows)
 * and 2m+1 (cols).  Row/col ops and setCell handle allocation replay on the GPU (one workgroup per
 * matrix); the kernel's cell events are replayed on the host into each matrix's SparseArray2D.
 */
class MatrixBatch extends MergeTreeBatch {
  constructor(nmatrices, options = {}) {
    super(0, options, 2 * nmatrices, MTB_BATCH_MATRIX);
    this.matrices = [];
    for (let m = 0; m < nmatrices; m++) this.matrices.push(new SharedMatrix(this, m));
  }

  matrix(m) { return this.matrices[m]; }
}

/** SharedMatrix observer slot: processCore (matrix.ts:636) and the PermutationVector summaries. */
class SharedMatrix {
  constructor(batch, m) {
    this.batch = batch;
    this.m = m;
  }

  startOrUpdateCollaboration(longClientId, minSeq = 0, currentSeq = 0) {
    native.matrixInit(this.batch.handle, this.m, longClientId, minSeq, currentSeq);
  }

  applyMsg(msg) {
    this.batch.checkIdle();
    native.matrixApplyMsg(this.batch.handle, this.m, typeof msg === "string" ? msg : JSON.stringify(msg));
    this.batch.dirty = true;
  }

  /**
   * SharedMatrix.loadCore (matrix.ts:611-634) into a fresh slot: `storage.readBlob(path)` gives the blobs
   * summarize() wrote ("rows/handleTable", "rows/segments/header" and its body chunks, "cols/...",
   * "cells"); `runtime.clientId` becomes the observer id ("snapshot" when absent).
   */
  async load(runtime, storage) {
    const text = (x) => (typeof x === "string" ? x : Buffer.from(x instanceof ArrayBuffer ? new Uint8Array(x) : x).toString("utf8"));
    const blobs = [];
    for (const v of ["rows", "cols"]) {
      blobs.push([`${v}/handleTable`, text(await storage.readBlob(`${v}/handleTable`))]);
      const header = text(await storage.readBlob(`${v}/segments/header`));
      blobs.push([`${v}/segments/header`, header]);
      const md = JSON.parse(header).headerMetadata;
      const ids = md && Array.isArray(md.orderedChunkMetadata) ? md.orderedChunkMetadata.slice(1).map((c) => c.id) : [];
      for (const id of ids) blobs.push([`${v}/segments/${id}`, text(await storage.readBlob(`${v}/segments/${id}`))]);
    }
    blobs.push(["cells", text(await storage.readBlob("cells"))]);
    native.matrixLoad(this.batch.handle, this.m, blobs, runtime && runtime.clientId !== undefined ? runtime.clientId : "snapshot");
    this.batch.dirty = true;
  }

  /** SharedMatrix.summarizeCore (matrix.ts:449-463): rows / cols PermutationVector summaries + cells blob. */
  summarize() {
    this.batch.ensureFlushed();
    const r = native.matrixSummarize(this.batch.handle, this.m);
    return { blobs: r.blobs, summary: JSON.parse(r.summary) };
  }

  /** SharedMatrix.getCell(row, col) (matrix.ts:173-189) in the observer's view. */
  getCell(row, col) {
    this.batch.ensureFlushed();
    const v = native.matrixGetCell(this.batch.handle, this.m, row, col);
    return v === undefined ? undefined : JSON.parse(v);
  }

  get rowCount() { this.batch.ensureFlushed(); return native.getLength(this.batch.handle, 2 * this.m); }

  get colCount() { this.batch.ensureFlushed(); return native.getLength(this.batch.handle, 2 * this.m + 1); }

  /** PermutationVector.summarize (permutationvector.ts:310) of rows and cols. */
  summarizeVectors() {
    return { rows: this.batch.summarizeV1(2 * this.m), cols: this.batch.summarizeV1(2 * this.m + 1) };
  }
}

/** TestClient (testClient.ts:54): the same slot plus the helpers that make other clients' sequenced messages. */
class TestClient extends Client {
  /** TestClient.makeOpMessage (testClient.ts:303-327). */
  makeOpMessage(op, seq = -1, refSeq = this.getCurrentSeq(), longClientId, minSeqNumber = 0) {
    if (op === undefined) throw new Error("op cannot be undefined");
    return {
      clientId: longClientId !== undefined ? longClientId : this.longClientId !== undefined ? this.longClientId : "",
      clientSequenceNumber: 1, contents: op, metadata: undefined,
      minimumSequenceNumber: minSeqNumber, referenceSequenceNumber: refSeq, sequenceNumber: seq,
      timestamp: Date.now(), term: 1, traces: [], type: "op",
    };
  }
  insertTextRemote(pos, text, props, seq, refSeq, longClientId) {
    const seg = props ? { text, props } : text;
    this.applyMsg(this.makeOpMessage({ pos1: pos, seg, type: 0 }, seq, refSeq, longClientId));
  }
  removeRangeRemote(start, end, seq, refSeq, longClientId) {
    this.applyMsg(this.makeOpMessage({ pos1: start, pos2: end, type: 1 }, seq, refSeq, longClientId));
  }
  annotateRangeRemote(start, end, props, seq, refSeq, longClientId) {
    this.applyMsg(this.makeOpMessage({ pos1: start, pos2: end, props, type: 2 }, seq, refSeq, longClientId));
  }
  insertMarkerRemote(pos, markerDef, props, seq, refSeq, longClientId) {
    const seg = { marker: { refType: markerDef && markerDef.refType !== undefined ? markerDef.refType : 1 } };
    if (props) seg.props = props;
    this.applyMsg(this.makeOpMessage({ pos1: pos, seg, type: 0 }, seq, refSeq, longClientId));
  }
  insertMarkerLocal(pos, behaviors, props) {
    const seg = { marker: { refType: behaviors } };
    if (props) seg.props = props;
    return this.insertSegmentLocal(pos, seg);
  }
}

module.exports = { MergeTreeBatch, MatrixBatch, SharedMatrix, Client, TestClient, native };
