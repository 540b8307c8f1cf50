// Device-side data layout of the MI355X merge-tree batch replay engine.
//
// Every document owns disjoint slices of a few batch-wide pools in HBM (structure of arrays per
// node type, array of structures per node so one wave-instruction fetches a whole record):
//   segs   : u32          parent block of each segment (the LRU heap refers to segments)
//   blks   : FBlk (320 B) tree nodes with their children's hot fields inline
//                         (reference: MergeBlock mergeTreeNodes.ts:332 + BaseSegment :367)
//   lists  : WEnt (16 B)  per-block slot-tagged window lists (replace PartialSequenceLengths,
//                         partialLengths.ts:239)
//   text   : u16          per-document UTF-16 text arena (insert payloads + zamboni appends)
//   heap   : Lru  (8 B)   zamboni LRU heap         (reference: Heap<LRUSegment>, collections/heap.ts)
//   aux    : u32          property sets and overlapping-remove client lists
//   freel  : u32          free-block stack
// A DocState header (448 B) holds each document's slice bases, bump pointers and collab window.
#pragma once
#include <stdint.h>

#define MTB_NONE 0xFFFFFFFFu
#define MTB_LEAF 0x80000000u
#define MTB_MAXCH 8          // MaxNodesInBlock (mergeTreeNodes.ts:330)
#define MTB_MAXDEPTH 24
#define MTB_UNDEF (-1)
#define MTB_MARKER 0x80000000u  // Seg.text flag: marker, low bits = refType + 1 (0 = undefined)
#define MTB_GPROPS 0x80000000u  // props handle flag: batch-global table (else per-doc aux arena)
#define MTB_NAN_CV 0x80000000u  // Tables::nan_val flag: consensus values (no-match values besides NaN) exist
#define MTB_INCR_TAB 0x80000000u  // an incr annotate's op-props value: pool offset of its result table
                                  // [absent result, n, (string value, result) * n] (Interner::incr_props)
#define MTB_PNAN 0x40000000u    // props handle flag of a per-doc set holding NaN (an incr annotate): such a set
                                // matches no set, itself included (matchProperties: NaN !== NaN)
#define MTB_NOKEY ((int32_t)0x80000000)
#define MTB_DELTA_OLD 0x80000000u  // catch-up delta entry tag: a rewrite annotate's property set before the op
// Window lists are allocated in power-of-two capacities (8 << class) from the document's list slice;
// released lists go to a per-class free stack whose heads live in the slice's first 16 words.
#define MTB_LCLASSES 16
#define MTB_LIST_RESERVED 4  // WEnt entries (16 words) reserved for the heads
// A window list keeps its entries in non-decreasing seq order, so the entries above a view's refSeq are
// its tail.  The list capacity word (a power of two) carries this flag when the order is not known (lists
// built by a summary load's body appends, or a rebuild whose seq window exceeds the sort's buckets):
// such a list is scanned whole.
#define MTB_LUNSORTED 0x80000000u
#define MTB_SORT_BUCKETS 1024  // rebuild's counting sort: seq - minSeq - 1 in [0, 1024)

// Internal record type (never accepted from mtb_append_ops): one body segment of a SnapshotV1 load,
// appended by insertSegments(root length, [segs], UniversalSeq, client, seq) (snapshotLoader.ts:187-220).
//   client = inserting client (NonCollabClient = 0xFFFE), seq = its seq, ref_seq = removedSeq (0xFFFFFFFF =
//   none), msn = removedClientIds[0] (0xFFFF = none), pos1 = aux offset of further removers, pos2 = text
//   length (marker: refType as for inserts), payload = text offset, props = props id.
#define MTB_OP_LOADSEG 5
#define MTB_F_LDFIRST 0x10  // first segment of an insertSegments batch: ensureIntervalBoundary at the root length
#define MTB_F_LDLAST 0x20   // last segment of the batch: zamboniSegments
// Local ops of a live client (the document's own client, short id 0; client.ts:196-247): insert / remove
// records carrying MTB_F_LOCAL are applied at (currentSeq, own id) with UnassignedSequenceNumber; an
// MTB_OP_ACK record (the client's own sequenced op) has pos2 = the acked op's type.
#define MTB_F_LOCAL 0x10
// Client.regeneratePendingOp (client.ts:917-960) of the head pending op with pos1 member ops (MODE_LIVE):
// normalizeSegmentsOnRebase when currentSeq moved, then per member group the regenerated ops' entries
// [record, op type | group index << 8, segment, position] in the document's delta slice.
#define MTB_OP_REGEN 7
// The merge tree's maintenance calls made directly by the reference's unit tests (mtb_maintenance, MODE_LIVE):
// pos1 = 0 zamboniSegments(mergeTree) (zamboni.ts:19-60), 1 packParent(root, mergeTree) (zamboni.ts:63-120).
#define MTB_OP_MAINT 8
// LocalClientId (-1): the client of a detached client's segments and removals (mtb_detached_op_json)
#define MTB_LOCAL_CLIENT 0xFFFFu
// A pending (unacked) local insert / remove stores MTB_PEND + localSeq in the segment's F_SEQ / F_RSEQ:
// larger than every sequence number, so every remote perspective sees it as "not yet" and breakTie orders
// it after sequenced segments (UnassignedSequenceNumber -> Number.MAX_SAFE_INTEGER - 1, mergeTree.ts:1719).
#define MTB_PEND 0x40000000
// Pending segment groups (pendingSegments, mergeTree.ts:532; one SegmentGroup per local op that touched
// segments): a FIFO directory (MTB_PEND_GROUPS entries, doubling when full) of [localSeq, member list offset, count, capacity,
// op type, op props id, 0, 0] in the aux arena; member lists (segment ids, group order) grow by doubling.
// A segment's pending property keys (PropertiesManager.pendingKeyUpdateCount, segmentPropertiesManager.ts)
// are the keys of the pending ANNOTATE groups holding it.
#define MTB_PEND_GROUPS 256      // initial directory entries
#define MTB_PEND_MAX (1u << 20)  // unacked local ops per document
#define MTB_PEND_ENT 8  // words per directory entry
// Marker-relative positions (IRelativePosition, ops.ts:77-92; posFromRelativePos mergeTree.ts:1371-1395):
// an insert / remove / annotate record with MTB_F_RELPOS has pos1 and/or pos2 = MTB_RELPOS | the
// text-arena offset of a 6-unit descriptor [ordinal lo, ordinal hi, before, 0, offset lo, offset hi]
// (ordinal: the marker's per-document id ordinal).  A marker insert / LOADSEG record carries its id's
// ordinal + 1 in `payload` (0: no id).  Internal (never accepted from mtb_append_ops).
#define MTB_F_RELPOS 0x20
#define MTB_RELPOS 0x80000000u
// PermutationVector documents (matrix/src/permutationvector.ts): segments carry a storage-handle start
// in the F_TEXT field instead of a text offset; their handle table lives in the (otherwise unused) text
// arena as u32 words [length, handles[0], handles[1], ...] (handletable.ts: handles[0] = free-list head).
#define MTB_HANDLE_UNALLOC 0x80000000u  // Handle.unallocated (-0x80000000)

// ---- device records -------------------------------------------------------------------------
// A tree node ("fat block", 320 B).  Besides its children's ids it holds the hot fields of every
// child, so one coalesced 320-byte fetch gives everything a walk needs at that level:
//   segment child : raw length, seq, removedSeq, client | rc0 << 16, overlap-remover list, props, text
//   block child   : the child's cachedLength (observer view) and the child's window-list metadata
// A block's window list holds the remote-length corrections of its BLOCK children, each entry tagged
// with the child's slot, so a block whose children are segments has no list at all; the list metadata
// of a block lives in its parent's slot (the root's in its own header), which lets a walk issue the
// fetch of a block and of its list together.
#define F_ID 0
#define F_LEN 1     // segment: cachedLength (UTF-16 units, markers 1) | block: cachedLength (observer)
#define F_SEQ 2     // segment: seq                                     | block: list offset
#define F_RSEQ 3    // segment: removedSeq (-1 = not removed)           | block: list count
#define F_CLI 4     // segment: client & 0xFFFF | removedClientIds[0] << 16 | block: list capacity
#define F_RCX 5     // segment: aux offset of [n, c1..cn] overlapping removers | block: seq of the last entry
#define F_PROPS 6   // segment: property-set handle (0 = none)         | block: key of the last entry
#define F_TEXT 7    // segment: text arena offset or MTB_MARKER | (refType + 1) | block: 0
struct FBlk {
  uint32_t f[8][MTB_MAXCH];  // [field][slot]
  uint32_t count;            // childCount
  uint32_t parent;           // MTB_NONE for the root
  uint32_t index;            // index in parent
  int32_t scour;             // needsScour: -1 undefined, 0 false, 1 true
  int32_t len;               // cachedLength (observer view, mergeTree.ts:2392 blockUpdate)
  uint32_t loff, lcnt, lcap; // root only: its window-list metadata
  int32_t lseq, lck;
  uint32_t pad[6];
};
static_assert(sizeof(FBlk) == 320, "FBlk is fetched as 80 dwords");
#define FB_HDR 64            // dword index of `count`

// ---- host-side views (read-out; rebuilt from the device records by download_doc) ---------------
struct Seg {          // reference: BaseSegment (mergeTreeNodes.ts:367)
  int32_t len;        // cachedLength (UTF-16 units; markers 1)
  int32_t seq;        // insert seq (0 = universal)
  int32_t rseq;       // removedSeq, -1 = not removed
  uint32_t props;     // property-set handle, 0 = undefined
  uint32_t text;      // text arena offset, or MTB_MARKER | (refType + 1)
  uint32_t parent;    // block id, MTB_NONE when unlinked
  uint32_t rcx;       // aux offset of [n, c1..cn] overlapping removers (0 = none)
  int16_t client;     // inserting short client id (-1 = LocalClientId)
  int16_t rc0;        // first remover (removedClientIds[0])
};

struct Blk {          // reference: MergeBlock (mergeTreeNodes.ts:332)
  uint32_t child[MTB_MAXCH];  // MTB_LEAF | seg id, or block id
  uint32_t parent;
  int32_t len;
  uint8_t count;
  uint8_t index;
  int8_t scour;
};

// Window-list entry of block B, for B's child in slot `slot`.  For a query (R, C):
//   length(child) = child cachedLength - sum(w(e) for e in B's list, e.slot == slot, e.seq > R)
// with w = delta if (kind == MAIN && client != C) or (kind == OVERLAP && client == C), else 0.
struct WEnt {
  int32_t seq;
  int32_t ck;         // client & 0xFFFF | kind << 16 | slot << 20
  int32_t delta;
  int32_t pad;
};
#define WK_MAIN 0
#define WK_OVERLAP 1
#define WE_KEY(client, kind, slot) (((client) & 0xFFFF) | ((kind) << 16) | ((slot) << 20))

struct Lru {
  uint32_t seg;
  int32_t maxSeq;
};

struct DocState {     // 448 bytes
  // slice bases (elements) and capacities
  uint64_t op_base;
  uint64_t seg_base, blk_base, list_base, text_base, heap_base, aux_base, free_base;
  uint32_t n_ops;
  uint32_t seg_cap, blk_cap, list_cap, text_cap, heap_cap, aux_cap;
  // bump pointers / counts
  uint32_t seg_used, blk_used, free_top, list_used, text_used, heap_cnt, aux_used;
  // collab window
  int32_t min_seq, cur_seq;
  uint32_t root;
  uint32_t op_next;
  int32_t new_mode;
  int32_t err;
  uint32_t err_op;
  uint64_t ops_applied;
  uint64_t n_mod;       // segment records created or modified (SURVEY 8(d) n_mod)
  uint64_t text_bytes;  // UTF-16 payload bytes of applied inserts
  uint64_t prof[7];     // MTB_PROFILE builds: s_memtime cycles per replay phase (see mtb_replay.hip)
  uint32_t flags;       // DSF_* (host-computed document properties)
  uint32_t cnt[5];      // MTB_PROFILE builds: event counters
  // catch-up deltas (MTB_F_DELTA records): u32 entries [record, segment -> local position, length, props]
  uint64_t delta_base;
  uint32_t delta_cap, delta_used;  // entries
  uint64_t prof2[4];    // MTB_PROFILE builds: more phases (prof[7 + i])
  uint32_t cnt2[4];     // MTB_PROFILE builds: more event counters (cnt[5 + i])
  // live client (local ops): collabWindow.localSeq and the pending segment-group FIFO
  int32_t local_seq;
  uint32_t pend_dir;    // aux offset of the group directory (0: none yet)
  uint32_t pend_head;   // directory index of the oldest pending group
  uint32_t pend_n;      // pending groups
  // idToSegment (mergeTree.ts:549) for marker-relative positions: marker ordinal (host-assigned per
  // document, first-seen order of marker ids) -> segment id, MTB_NONE = not mapped
  uint32_t mk_map;      // aux offset of the map (0: none yet)
  uint32_t mk_n;        // entries allocated
  uint32_t mk_cap;      // host: marker ordinals known for the document (the map grows to this)
  uint32_t pend_ann;    // pending groups of local annotates
  int32_t last_norm;    // Client.lastNormalizationRefSeq (client.ts:909): currentSeq of the last normalization
  uint32_t orphans;     // aux offset of [n, cap, (props id, segment)*]: pending keys whose annotate group a
                        // reconnect dropped without a new op (they stay pending, as the reference's counts do)
  uint32_t pend_cap;    // directory entries (a power of two, 0: none yet; doubles when full)
  uint32_t mk_all;      // aux offset of [n, cap, (segment, ordinal)*]: every marker inserted with an id (0: none)
  uint32_t pad3[4];
  // phantom partial lengths and partial-length deficits of a loaded summary's collaborator-inserted body segments
  // (DSF_PHANTOM): aux offset of [n, cap, 8-word entry * cap], entry kinds PH_* below (mtb_replay.hip)
  uint32_t ph;
  uint32_t pad4[15];
};
static_assert(sizeof(DocState) == 448, "DocState is read as 112 dwords (two vector loads, mtb_rewind_kernel)");

// Batch-global interned tables (read-only on the device).
struct Tables {
  const uint32_t* pool;      // u32 pool: op-props lists [n, (key, val)*n] (val MTB_NONE = null/delete)
                             //           and property sets [n, (key, val)*n]
  const uint32_t* pidx;      // props id i -> pidx[2i] = op-props list offset, pidx[2i+1] = property set offset
  const uint32_t* val_class; // matchProperties equivalence class of each value id
  const uint8_t* val_falsy;  // JS falsiness of each value id
  const uint32_t* key_rank;  // array-index keys: numeric value; other keys: MTB_NONE
  uint32_t* delta;           // catch-up delta pool (per-document slices at DocState.delta_base, 4 words/entry)
  uint32_t class_trivial;    // every matchProperties class holds one value id: classes compare as value ids
  uint32_t mk_key;           // key id of "markerId" (MTB_NONE: no property set names it)
  uint32_t nan_val;          // value id of NaN (incr annotates; MTB_NONE: none packed), | MTB_NAN_CV when consensus
                             // values exist; val_falsy bit 1 marks
                             // the values that incr turns into NaN (numbers, booleans, NaN); bit 2 objects whose
                             // seq is -1 (a consensus annotate completes them in place); bit 3 values a set holding
                             // one of which matches no set (NaN, consensus values: MTB_PNAN handles)
  // matchProperties of keys whose values are no equivalence (mtb_host.cpp Interner): key_irr[k] = 1 + offset
  // of [n, n x n bits] in irr (0: regular key, compare val_class); bit (i * n + j) = matchProperties(v_i, v_j)
  // for the key's values of local index i (first argument) and j (val_local)
  const uint32_t* key_irr;
  const uint32_t* val_local;
  const uint32_t* irr;
  uint32_t irr_any;          // irregular keys exist: matchProperties is neither symmetric nor reflexive there
};

// device error codes (DocState.err)
#define DERR_INSERT 1      // "MergeTree insert failed" (mergeTree.ts:1671)
#define DERR_CAP_SEG 2
#define DERR_CAP_BLK 3
#define DERR_CAP_LIST 4
#define DERR_CAP_TEXT 5
#define DERR_CAP_HEAP 6
#define DERR_CAP_AUX 7
#define DERR_ASSERT_SEQ 8  // 0x038
#define DERR_ASSERT_MSN 9  // 0x039 / 0x04e / 0x04f
#define DERR_DEPTH 10
#define DERR_SHAPE 11      // a block mixing segment and block children (never produced by the reference)
#define DERR_CAP_DELTA 13  // catch-up delta / matrix cell-event slice exhausted
#define MTB_CELL_SET 1     // matrix cell event: this vector's handle for a setCell record
#define MTB_CELL_CLEAR 2   // matrix cell event: handles [start, start + count) recycled by zamboni
#define DERR_HANDLE 12     // handle allocation did not isolate one position (never produced by the reference)
#define DERR_HOST 14       // host-side post-processing of the document's replay failed (HostDoc::hostErr)
#define DERR_RANGE 15      // a local op outside the local view (getValidOpRange, client.ts:527-592)
#define DERR_CAP_PEND 16   // more than MTB_PEND_MAX unacked local ops
#define DERR_ACK_INSERT 17 // 0x045 "On insert, seq number already assigned!"
#define DERR_ACK_REMOVE 18 // 0x046 "On remove ack, missing removal info!"
#define DERR_LOCAL 19      // a local op the engine does not support (a local rewrite annotate)
#define DERR_RELPOS 20     // a relative position whose marker is not mapped, or resolves below 0
#define DERR_REGEN 21      // regeneratePendingOp without the pending group(s) it names (0x033 / 0x035)
#define DERR_SCHED 22      // a document without an error did not run all of its records (engine invariant)
#define DERR_ASSERT_MKID 23  // 0x5ad "Cannot change the markerId of an existing marker" (mergeTree.ts:1912-1918)
#define DERR_STALE 25        // a summary body insert whose incremental partial-length update leaves stale cumulative
                             // lengths (partialLengths.ts:543-577) in a document without a deficit table (engine
                             // invariant: the host gives every load with collaborating body segments one)
#define DERR_INCR 24         // an incr annotate over a value its op's result table lacks (engine invariant)
#define DERR_CONSENSUS 26    // a consensus annotate over an object value whose seq is -1 (completed in place, shared
                             // with split clones)
#define DERR_CONS_NULL 27    // a consensus annotate with a null defaultValue over a segment lacking the key: the
                             // reference throws reading the null's seq (properties.ts:56-57), so does the engine
// ticket scheduler words (mtb_replay_tick_kernel): queue q's ticket counter at MTB_SCHED_TICK * q (one
// 128-byte line each, q < 8), the abort flag, then per-document progress from MTB_SCHED_HDR
#define MTB_SCHED_TICK 32
#define MTB_SCHED_ABORT 256
#define MTB_SCHED_SPINS 260  // mtb_replay_tick_kernel: the wait bound (spins), written by the host
#define MTB_SCHED_BAD 264    // hand-over invariant violations (tick_check): count, then the first's document, chunk,
                             // expected op_next, seen op_next
#define MTB_SCHED_HDR 288

#define DSF_NEWLINE 1      // the document's text arena may contain a newline (TextSegment.canAppend, textSegment.ts:71)
#define DSF_PERM 2         // a PermutationVector (SharedMatrix rows or cols)
#define MTB_GRP_REWRITE 0x80000000u  // pending ANNOTATE group / orphan props word: the local op was a rewrite
#define DSF_OBS_SHIFT 16  // flags >> 16: the reference's short id of the engine's client 0 (a loaded summary's
                          // observer; mtb_host.cpp HostDoc::obsRef), mapped back by the digest
// DocState.ph table entry kinds (word 6): a phantom insert, a main-set deficit (refSeq >= t), a client-set
// deficit (client c, refSeq < t), a main-set deficit copied down into minLength (always)
#define PH_PHANTOM 0u
#define PH_DEF_MAIN 1u
#define PH_DEF_CLI 2u
#define PH_DEF_MIN 3u
#define PH_NOSEQ 0x7FFFFFFF
#define DSF_PHANTOM 8      // a loaded summary left phantom partial lengths (DocState.ph; mtb_replay.hip)
#define DSF_MKDUP 4        // a marker id is carried by two markers: blockUpdate re-maps ids (mergeTree.ts:296-306)
#define DSF_VARIANT 32     // the document replays on the marker variant (marker ids, phantom tables, irregular keys);
                           // the observer kernels skip it and the marker kernel replays only such documents
