/*
 * mtb.h — C ABI of the MI355X merge-tree batch replay engine ("mtb" = merge-tree batch).
 *
 * One batch holds many independent documents (SharedString / PermutationVector merge-trees).
 * Each document is an *observer* merge-tree client: it receives the sequenced op stream of every
 * other client and applies it exactly as the reference `Client.applyMsg` would
 * (packages/dds/merge-tree/src/client.ts:858-887), then produces the same text
 * (MergeTreeTextHelper.ts:20) and SnapshotV1 summary (client.ts:966-1005, snapshotV1.ts:122-312).
 *
 * Interfaces replaced (reference file:line -> entry point here):
 *   Client ctor / startOrUpdateCollaboration   client.ts:107, :1133      -> mtb_batch_create, mtb_doc_init
 *   Client.load (SnapshotV1 summary)           client.ts:1007            -> mtb_doc_load_v1
 *   Client.applyMsg(ISequencedDocumentMessage) client.ts:858              -> mtb_apply_msg_json (JSON) or
 *                                                                           mtb_append_ops (pre-packed records)
 *   (replay of the appended ops; synchronous in the reference)            -> mtb_replay
 *   TestClient.getText / MergeTreeTextHelper   testClient.ts:185          -> mtb_get_text
 *   Client.getLength / getCurrentSeq           client.ts:1129, :1122      -> mtb_get_length, mtb_get_seq
 *   Client.summarize (SnapshotV1 branch)       client.ts:966-998          -> mtb_summarize_v1
 *   (segment-level parity read-out)            mergeTreeNodeWalk.ts:170   -> mtb_dump_segments
 *
 * All calls return 0 on success or a negative MTB_E_* code; mtb_last_error() gives the message,
 * which carries the reference assert code / error text where one exists (e.g. "0x038",
 * "MergeTree insert failed").  A batch handle is not thread-safe; distinct handles are independent.
 */
#ifndef MTB_H
#define MTB_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- op record (32 bytes). One record per merge-tree delta op; GROUP members are flattened into
 * consecutive records sharing seq/ref_seq/msn; the last record of a message carries MTB_F_LAST. */
enum {
  MTB_OP_INSERT = 0,   /* ops.ts:58 INSERT   pos1 = pos, pos2 = text length (UTF-16 units) */
  MTB_OP_REMOVE = 1,   /* ops.ts:59 REMOVE   [pos1, pos2) */
  MTB_OP_ANNOTATE = 2, /* ops.ts:60 ANNOTATE [pos1, pos2), props = op-props id */
  MTB_OP_NOOP = 3,     /* non-"op" message, or a member with no merge-tree effect */
  MTB_OP_ACK = 4,      /* op authored by the observer itself (client.ts:866 ack path): zamboni only */
  MTB_OP_SETCELL = 6   /* SharedMatrix setCell (matrix.ts:668-676), in both vectors' records: pos1 = the
                          row (rows vector) or col (cols vector), pos2 = the observer's short id; no
                          updateSeqNumbers.  Only in matrix batches. */
};
enum {
  MTB_F_LAST = 0x01,    /* run updateSeqNumbers(msn, seq) after this record (client.ts:874) */
  MTB_F_MARKER = 0x02,  /* insert: Marker segment, pos2 = refType (0xFFFFFFFF = undefined) */
  /* Bits 0x02-0x40 mean different things per record type (and the engine's internal records reuse 0x10 /
   * 0x20): test a flag only after testing the record's type. */
  MTB_F_COMB = 0x0C,    /* annotate: the combiningOp kind, a 2-bit field (compare masked: (flags & MTB_F_COMB)) */
  MTB_F_REWRITE = 0x04, /*   {name:"rewrite"} (segmentPropertiesManager.ts:107-123) */
  MTB_F_INCR = 0x08,    /*   {name:"incr"}: every key of props becomes combine(op, previous, undefined)
                             (properties.ts:24-69): NaN for numeric / boolean / absent previous values, a string
                             gets "undefined" appended (records carry no defaultValue / minValue: the JSON
                             path, mtb_apply_msg_json, takes them from the op) */
  MTB_F_CONSENSUS = 0x0C, /* {name:"consensus"}: combine(op, previous, undefined, seq) (properties.ts:46-62) for
                             a sequenced op: an absent key gets {value: undefined, seq}, a present one stays */
  MTB_F_SEGOBJ = 0x08,  /* insert: seg given as {text, props?} object (props id may be 0) */
  MTB_F_PERMSEG = 0x40, /* insert (matrix batches): PermutationSegment [length, start], pos2 = length */
  MTB_F_DELTA = 0x80    /* record the op's delta ranges (catch-up rewriting, MTB_BATCH_CATCHUP) */
};
typedef struct mtb_op {
  uint8_t type;
  uint8_t flags;
  uint16_t client;   /* short client id (first-seen order, 0 = the observer) */
  uint32_t seq;      /* sequenceNumber */
  uint32_t ref_seq;  /* referenceSequenceNumber */
  uint32_t msn;      /* minimumSequenceNumber */
  uint32_t pos1;
  uint32_t pos2;
  uint32_t payload;  /* insert: offset (UTF-16 units) of the text in the payload passed with it;
                        annotate: set by the host (assert 0x5ad's markerId test, mergeTree.ts:1912-1918) */
  uint32_t props;    /* insert/annotate: props id from mtb_intern_props (0 = none) */
} mtb_op;

typedef struct mtb_options {
  int32_t new_length_calc; /* IMergeTreeOptions.mergeTreeUseNewLengthCalculations (mergeTree.ts:413) */
  int32_t chunk_size;      /* IMergeTreeOptions.mergeTreeSnapshotChunkSize, 0 -> 10000 */
  int32_t threads_per_doc; /* reserved (64) */
  int32_t flags;           /* MTB_BATCH_MATRIX: a batch of SharedMatrix observers (mtb_matrix_*) */
} mtb_options;

#define MTB_BATCH_MATRIX 1 /* mtb_options.flags: documents 2m / 2m+1 are matrix m's rows / cols PermutationVectors */
#define MTB_BATCH_CATCHUP 2 /* mtb_options.flags: keep SharedSegmentSequence.messagesSinceMSNChange per document
                               (sequence.ts:697-748), lagging messages rewritten from their deltas, for
                               mtb_summarize_legacy's catch-up blob */

typedef struct mtb_stats {
  uint64_t ops_applied;     /* delta ops applied (each GROUP member counts once) */
  uint64_t docs;            /* documents replayed */
  uint64_t segments_final;  /* segments in the documents' trees after replay (tombstones included) */
  uint64_t text_units_final;/* observer-view length (Client.getLength) summed over documents */
  uint64_t bytes_alg;       /* algorithmic bytes */
  uint64_t checksum;        /* sum mod 2^64 of the per-document state digests (mtb_doc_digests); a
                               SUM so that shards reduce with one all-reduce */
  uint64_t errors;          /* documents whose replay stopped on an error */
  double kernel_ms;         /* device time of the replay kernel(s) (HIP events) */
} mtb_stats;

typedef struct mtb_blob {
  const char* path;      /* "header", "body_0", ... */
  const char* content;   /* UTF-8 blob contents (SummaryTreeBuilder.addBlob content) */
  size_t content_len;
} mtb_blob;
typedef struct mtb_blob_list {
  uint32_t count;
  mtb_blob* blobs;
  const char* summary_json; /* the ISummaryTreeWithStats object, JSON-serialized */
  size_t summary_json_len;
} mtb_blob_list;

typedef struct mtb_batch mtb_batch;

enum {
  MTB_OK = 0,
  MTB_E_ARG = -1,         /* bad argument */
  MTB_E_NODEV = -2,       /* no usable GPU / HIP runtime (the engine never falls back to CPU) */
  MTB_E_HIP = -3,         /* HIP runtime error */
  MTB_E_ASSERT = -4,      /* reference assert (message holds the 0xNNN code) */
  MTB_E_INSERT = -5,      /* UsageError("MergeTree insert failed") mergeTree.ts:1671 */
  MTB_E_UNSUPPORTED = -6, /* input outside the engine's supported subset */
  MTB_E_CAPACITY = -7,    /* a per-document arena overflowed */
  MTB_E_PARSE = -8,       /* malformed JSON message */
  MTB_E_INTERNAL = -9     /* an engine invariant failed (e.g. a document did not run all of its records) */
};

/* What the last mtb_replay / mtb_replay_resident launched (diagnostics; no reference counterpart: the
 * reference applies each message synchronously in Client.applyMsg, client.ts:858). */
enum {
  MTB_KERNEL_NONE = 0,
  MTB_KERNEL_REPLAY = 1,   /* one wave per document */
  MTB_KERNEL_SCHED = 2,    /* (retired in round 4: ticket-scheduled persistent waves, see MTB_KERNEL_TICKS) */
  MTB_KERNEL_FEW = 3,      /* one wave per document, large LDS heap (few documents) */
  MTB_KERNEL_LIVE = 4,     /* live clients (local ops, acks, reconnect) */
  MTB_KERNEL_MARKERS = 5,  /* marker ids / relative positions */
  MTB_KERNEL_MATRIX = 6,   /* SharedMatrix vector pairs */
  MTB_KERNEL_PASSES = 7,   /* more documents than resident waves: launches of equal chunks ("passes") */
  MTB_KERNEL_TICKS = 8     /* more documents than resident waves: one ticket (document chunk) per workgroup */
};
typedef struct mtb_launch_info {
  uint32_t kernel;      /* MTB_KERNEL_* */
  uint32_t wave_slots;  /* resident replay waves of the device (CUs x 16) */
  uint32_t chunks;      /* MTB_KERNEL_TICKS: tickets per document; MTB_KERNEL_PASSES: chunks per document */
  uint32_t queues;      /* MTB_KERNEL_TICKS: ticket queues (one per XCD) */
  uint32_t aborted;     /* MTB_KERNEL_TICKS: a ticket wait hit its bound and the finish kernel ran the rest */
  uint32_t passes;      /* MTB_KERNEL_PASSES: kernel launches of the replay */
  uint32_t handover_bad; /* MTB_KERNEL_TICKS: tickets that found their document's state not the one the previous
                            chunk left (never expected; such documents are finished by a fresh launch) */
  uint32_t cap_retries;  /* relaunches of the last mtb_replay's capacity retry (documents whose first replay outgrew
                            their slices, laid out again larger and replayed from their pristine state) */
} mtb_launch_info;

/* device_mask: the HIP devices the batch spreads over (bit k = device k; 0 = device 0).  With several,
 * documents are assigned by hash(document index) mod the device count (SharedMatrix batches: whole
 * matrices), each device holds its own HBM pools and stream, and mtb_replay / mtb_rewind /
 * mtb_replay_resident run every device at once (one host thread each), merging the statistics.  Props
 * objects passed to mtb_intern_props get the same id on every device; a props object first met inside a
 * message is interned by that document's device only (its id in mtb_export_pending records is that
 * device's). */
int mtb_batch_create(const mtb_options* opts, uint32_t ndocs, uint32_t device_mask, mtb_batch** out);
void mtb_batch_destroy(mtb_batch* b);
const char* mtb_last_error(mtb_batch* b);
void mtb_free(void* p);
/* The SHA-256 of the sources, headers and compile flags this library was built from (build.py embeds it;
 * a library whose hash differs from the tree's is rebuilt).  Not a reference interface. */
const char* mtb_build_id(void);

/* Initial detached content (inserted locally before collaboration, like client.replay.spec.ts:27)
 * and startOrUpdateCollaboration(observer_long_id, min_seq, cur_seq) (client.ts:1133). */
int mtb_doc_init(mtb_batch* b, uint32_t doc, const uint16_t* initial_text, size_t n_units,
                 const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq);

/* Client.load of a SnapshotV1 summary (client.ts:1007 -> SnapshotLoader, snapshotLoader.ts:41-257): the
 * blobs are the summary's [path, content] pairs (as mtb_summarize_v1 returns them; "header" plus the
 * chunks orderedChunkMetadata names).  The header segments are reloaded into a tree
 * (reloadFromSegments, mergeTree.ts:678), collaboration starts as startOrUpdateCollaboration(
 * observer_long_id, minSequenceNumber, sequenceNumber) (the reference passes runtime.clientId ??
 * "snapshot"), and the body chunks are appended on the GPU by the next replay, ahead of any op applied
 * after this call.  Instead of mtb_doc_init.  A removed body segment inserted by a collaborating client
 * is rejected with MTB_E_UNSUPPORTED. */
int mtb_doc_load_v1(mtb_batch* b, uint32_t doc, const mtb_blob* blobs, uint32_t nblobs,
                    const char* observer_long_id);
/* mtb_doc_load_v1 for n documents at once, the blobs parsed and the headers rebuilt on `threads` host
 * threads (no reference counterpart: the reference loads one channel at a time).  Documents whose load
 * fails are left fresh; the first failure's error is returned. */
int mtb_docs_load_v1(mtb_batch* b, uint32_t n, const uint32_t* docs, const mtb_blob* const* blobs,
                     const uint32_t* nblobs, const char* const* observer_long_ids, uint32_t threads);

/* Client.applyMsg(msg) with msg = JSON.stringify(ISequencedDocumentMessage).  Validates, interns the
 * long client id and props, packs records and appends them to the document (no GPU work). */
int mtb_apply_msg_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len);
/* A live client's own op: Client.insertSegmentLocal / removeRangeLocal / annotateRangeLocal (client.ts:196-247)
 * with the IMergeTreeOp it sends as JSON ({"type":0,"pos1","seg"}, {"type":1,"pos1","pos2"} or
 * {"type":2,"pos1","pos2","props"}; a group of them).
 * The document's observer id (mtb_doc_init) is the client; the op is applied at the next replay in its own
 * view with UnassignedSequenceNumber, after getValidOpRange's bounds check (a failure is reported by that
 * replay).  Its sequenced message, passed to mtb_apply_msg_json, is the ack (ackPendingSegment,
 * client.ts:641-662).  A local annotate's keys stay pending on its segments until its ack (remote annotates
 * leave them alone, segmentPropertiesManager.ts:60-157; a local rewrite annotate counts as a pending rewrite).
 * Marker-relative positions resolve in the client's own view.  Matrix and catch-up batches are
 * MTB_E_UNSUPPORTED (a live client's own ops are not tracked as catch-up messages).  A consensus annotate is
 * accepted as Client.annotateMarkerNotifyConsensus makes it (client.ts:155-181: createAnnotateMarkerOp's op,
 * flagged with the member "notifyConsensus": true, which is not part of the op sent): its values are
 * {value: undefined, seq: -1} until its ack completes them with the ack's seq (client.ts:1050-1058). */
int mtb_local_op_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len);
/* A detached edit before collaboration (TestClient.insertTextLocal / removeRangeLocal / annotateRangeLocal
 * while the collab window is not collaborating, client.ts:196-247 with getLocalSequenceNumber() =
 * UniversalSequenceNumber and clientId = LocalClientId; createClientsAtInitialState, testClientLogger.ts:51-78):
 * the op (JSON IMergeTreeOp) is applied at the next replay with seq 0, refSeq 0 and LocalClientId, no LRU entry
 * and no zamboni -- the segments and tombstones a detached client builds.  Only after mtb_doc_init(min_seq 0,
 * cur_seq 0) and before the document's first message or local op. */
int mtb_detached_op_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len);
/* The merge tree's maintenance functions that the reference's own unit tests call directly
 * (mergeTree.zamboni.spec.ts: zamboni.ts exports): kind 0 = zamboniSegments(mergeTree) (zamboni.ts:19-60),
 * kind 1 = packParent(root, mergeTree) (zamboni.ts:63-120; the root's children must be blocks, else
 * MTB_E_INTERNAL at replay).  Queued as an internal record, applied at the next replay. */
int mtb_maintenance(mtb_batch* b, uint32_t doc, uint32_t kind);
/* Client.regeneratePendingOp (client.ts:917-960) after a reconnect: `op_json` is the live client's oldest
 * pending op (as submitted; a GROUP names one pending op per member).  Replays the batch, then on the GPU
 * normalizes the segment order around pending segments (normalizeSegmentsOnRebase, mergeTree.ts:2357-2390)
 * when currentSeq moved, pops the op's segment groups and computes each segment's position in the local view
 * at the group's localSeq (findReconnectionPosition); *out = the op(s) to resubmit (JSON, a GROUP when
 * several; free with mtb_free), whose new segment groups are queued for their acks. */
int mtb_regenerate_pending_op(mtb_batch* b, uint32_t doc, const char* op_json, size_t len, char** out, size_t* out_len);
/* Pre-packed path: append records whose `payload` offsets index `payload` (UTF-16 units). */
int mtb_append_ops(mtb_batch* b, uint32_t doc, const mtb_op* ops, uint32_t n,
                   const uint16_t* payload, size_t payload_len);
/* Register the long client id for the next short id of `doc` (used with mtb_append_ops). */
int mtb_add_client(mtb_batch* b, uint32_t doc, const char* long_id);
/* Intern a props object (JSON text); id 0 is reserved for "none". */
int mtb_intern_props(mtb_batch* b, const char* json_utf8, size_t len, uint32_t* id_out);

/* ---- SharedMatrix (MTB_BATCH_MATRIX batches; matrix.ts, permutationvector.ts) ----
 * Matrix m owns documents 2m (rows) and 2m+1 (cols), each a PermutationVector observer: remote
 * insert/remove of rows/cols are merge-tree ops on that vector; a remote setCell adjusts (row, col)
 * into the observer's view (adjustPosition, permutationvector.ts:209) and allocates storage handles
 * (getAllocatedHandle, :183) on the GPU; the kernel logs each setCell's handles and each zamboni handle
 * recycling, which the host replays into the matrix's SparseArray2D (matrix.ts:96, :684, :721-733).
 * mtb_summarize_v1 and mtb_dump_segments on a vector document give PermutationVector.summarize (:310):
 * blobs "segments/header", "segments/body_i", "handleTable". */
int mtb_matrix_init(mtb_batch* b, uint32_t matrix, const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq);
int mtb_matrix_apply_msg_json(mtb_batch* b, uint32_t matrix, const char* json_utf8, size_t len);
/* Intern a setCell value (JSON text) for records packed by the caller (mtb_append_ops): the SETCELL
 * record's `props` field carries the id (0 = undefined). */
int mtb_matrix_intern_value(mtb_batch* b, const char* json_utf8, size_t len, uint32_t* id_out);
/* SharedMatrix.loadCore (matrix.ts:611-634) of a matrix slot that is still fresh (instead of
 * mtb_matrix_init): blobs as mtb_matrix_summarize writes them ("rows/handleTable", "rows/segments/header",
 * "cols/...", "cells"); the observer id becomes both vectors' client id.  PermutationVector summaries
 * with body chunks and summaries holding pending local cell writes are MTB_E_UNSUPPORTED. */
int mtb_matrix_load(mtb_batch* b, uint32_t matrix, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id);
/* SharedMatrix.summarizeCore (matrix.ts:449-463): blobs "rows/segments/header", ..., "rows/handleTable",
 * "cols/...", "cells" (JSON [cells.snapshot(), pending.snapshot()]) and the ISummaryTreeWithStats. */
int mtb_matrix_summarize(mtb_batch* b, uint32_t matrix, mtb_blob_list* out);
/* SharedMatrix.getCell(row, col) (matrix.ts:173-189) in the observer's view: the value's JSON text, or
 * *len_out = 0 when the cell is undefined or a position has no handle. */
int mtb_matrix_get_cell(mtb_batch* b, uint32_t matrix, uint32_t row, uint32_t col, char* buf, size_t cap,
                        size_t* len_out);

/* Replay every pending op of every document on the GPU(s).  Blocking. */
int mtb_replay(mtb_batch* b, mtb_stats* out);

int mtb_get_text(mtb_batch* b, uint32_t doc, uint16_t* buf, size_t cap, size_t* len_out);
int mtb_get_length(mtb_batch* b, uint32_t doc, uint32_t* len_out);
int mtb_get_seq(mtb_batch* b, uint32_t doc, uint32_t* cur_seq, uint32_t* min_seq);
/* Canonical segment dump (JSON lines, engine-allocated; free with mtb_free). */
int mtb_dump_segments(mtb_batch* b, uint32_t doc, char** out, size_t* out_len);
/* Per-document state checksum (FNV-1a 64 over the canonical dump). */
int mtb_doc_checksum(mtb_batch* b, uint32_t doc, uint64_t* out);
/* State digests v1 (DESIGN.md "State digest": the canonical dump's content folded into 64 bits on the
 * GPU by every replay) of documents [first, first + n), from the last replay; 0 for a failed document. */
int mtb_doc_digests(mtb_batch* b, uint32_t first, uint32_t n, uint64_t* out);

/* The kernel the last replay launched (first device of a multi-device batch; `aborted` of any). */
int mtb_get_launch_info(mtb_batch* b, mtb_launch_info* out);
/* MergeTree.mapRange / nodeMap (mergeTree.ts:2456-2474, 2531-2582) over [start, end) (end < 0: to the end)
 * in the view of (ref_seq, long_client_id) (ref_seq < 0: currentSeq; long_client_id NULL: the observer,
 * i.e. the local view).  Serves Client.walkSegments (client.ts:286), getContainingSegment (:1065) and
 * getPropertiesAtPosition (:1101).  *out = JSON array of {"pos", "start", "end", "segment": {"type",
 * "text" | "refType" | "start", "cachedLength", "seq", "clientId", "removedSeq"?, "removedClientIds"?,
 * "properties"?}} (short client ids), at most `limit` entries (0 = all); free with mtb_free. */
int mtb_map_range(mtb_batch* b, uint32_t doc, int64_t start, int64_t end, int64_t ref_seq,
                  const char* long_client_id, uint32_t limit, char** out, size_t* out_len);
/* Diagnostic (no reference counterpart): the partial lengths the engine walks in the (ref_seq, long_client_id)
 * view.  *out = one JSON line per block in tree order: {"path": [child indices from the root], "kids": [null for
 * a segment | [length in the view, leaf sum in the view]], "table": [[kind, t or removedSeq, length, client],
 * ...]} -- the length is the leaf sum plus the block's phantom surplus less its partial-length deficits
 * (DESIGN.md section 7), "table" the document's entries for that block.  Free with mtb_free. */
int mtb_debug_blocks(mtb_batch* b, uint32_t doc, int64_t ref_seq, const char* long_client_id, char** out,
                     size_t* out_len);
/* Client.summarize with newMergeTreeSnapshotFormat: if `msn`/`seq` >= 0 first runs
 * updateSeqNumbers(msn, seq) (client.ts:979).  long_client_ids may be NULL (use registered ids). */
int mtb_summarize_v1(mtb_batch* b, uint32_t doc, int64_t msn, int64_t seq,
                     mtb_blob_list* out);
void mtb_blob_list_free(mtb_blob_list* l);
/* mtb_summarize_v1 for n documents at once (out[k] for docs[k]; free each with mtb_blob_list_free): one
 * replay for the optional updateSeqNumbers(msn, seq), one bulk download of the documents' slices and the
 * summaries serialized on `threads` host threads.  No reference counterpart (the reference summarizes
 * one channel at a time); each blob list equals what mtb_summarize_v1 returns for that document.  The
 * batch keeps the extraction's staging (host and device, sized by the largest call) until it is destroyed. */
int mtb_summarize_v1_many(mtb_batch* b, uint32_t n, const uint32_t* docs, int64_t msn, int64_t seq, uint32_t threads,
                          mtb_blob_list* out);
/* FNV-1a 64 over a blob list (each blob's path, 0, content, 0; then the summary JSON): a compact
 * fingerprint for comparing many summaries with a checker without copying them out. */
int mtb_blob_list_fnv(const mtb_blob_list* l, uint64_t* out);
/* Client.summarize without newMergeTreeSnapshotFormat (client.ts:999-1003, snapshotlegacy.ts:122-259):
 * "header" / "body" chunks of the segments at the MSN, plus a "catchupOps" blob holding
 * `catchup_json` (a JSON array of the messages above the MSN that the caller keeps, as
 * SharedSegmentSequence.messagesSinceMSNChange does, sequence.ts:680-748) when it is non-empty. */
int mtb_summarize_legacy(mtb_batch* b, uint32_t doc, int64_t msn, int64_t seq, const char* catchup_json,
                         size_t catchup_len, mtb_blob_list* out);

/* ---- benchmark / re-replay utilities (no reference counterpart) ----
 * mtb_rewind restores every document to its state before its first replay while keeping the op
 * records resident in HBM; mtb_replay_resident then replays them again without host traffic. */
int mtb_rewind(mtb_batch* b);
int mtb_replay_resident(mtb_batch* b, mtb_stats* out);
/* mtb_replay_resident without the state-digest pass (flags MTB_REPLAY_NO_DIGEST): the statistics' checksum,
 * segments_final and text_units_final stay 0 and the write-back term of bytes_alg is left out, until
 * mtb_refresh_digests computes them (and the per-document digests) on the replayed state.  For timing the
 * replay alone; the digests are verification, not part of Client.applyMsg. */
#define MTB_REPLAY_NO_DIGEST 1u
int mtb_replay_resident_ex(mtb_batch* b, mtb_stats* out, uint32_t flags);
/* The state digest of every document on the current state (mtb_digest_kernel): fills out->checksum,
 * segments_final, text_units_final and bytes_alg (its write-back term only: 24 B per final segment record +
 * 2 B per final text unit); mtb_doc_digests reads the per-document values afterwards. */
int mtb_refresh_digests(mtb_batch* b, mtb_stats* out);

/* ---- host-side inspection (tests): the records/payload packed for `doc` and not yet replayed, the
 * JSON of an interned props id, and the long id of a short client id (Client.getLongClientId,
 * client.ts:682).  None of these touch the GPU. */
int mtb_export_pending(mtb_batch* b, uint32_t doc, mtb_op* ops, uint32_t cap, uint32_t* n_out,
                       uint16_t* payload, size_t pcap, size_t* plen_out);
int mtb_props_json(mtb_batch* b, uint32_t id, char* buf, size_t cap, size_t* len_out);
int mtb_client_long_id(mtb_batch* b, uint32_t doc, uint32_t short_id, char* buf, size_t cap, size_t* len_out);

#ifdef __cplusplus
}
#endif
#endif
