// ORACLE / TEST INFRASTRUCTURE ONLY — CPU restatement of the reference merge-tree observer path.
//
// Parity pinning: tests/test_oracle_fixtures.py replays the reference's 30 committed conflict-farm
// logs (packages/dds/merge-tree/src/test/results/*.json, 61,200 ops, text after every group) and
// byte-compares the 6 committed SnapshotV1 summaries
// (packages/dds/sequence/src/test/snapshots/v1/*.json).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this code; the product engine never links it.
//
// Every function cites the reference file:line whose behaviour it restates
// (MT = packages/dds/merge-tree/src).
#pragma once
#include <cstdint>
#include <array>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "ojson.hpp"

namespace orc {

constexpr int MaxNodesInBlock = 8;         // MT/mergeTreeNodes.ts:330
constexpr int UniversalSeq = 0;            // MT/constants.ts:11
constexpr int UnassignedSeq = -1;          // MT/constants.ts:12
constexpr int TreeMaintenanceSeq = -2;     // MT/constants.ts:13
constexpr int LocalClientId = -1;          // MT/constants.ts:14
constexpr int NonCollabClient = -2;        // MT/constants.ts:15
constexpr int TextSegmentGranularity = 256;// MT/textSegment.ts:20
constexpr int ZamboniSegmentsMax = 2;      // MT/zamboni.ts:14
constexpr int UNDEF_LEN = -1;              // `undefined` result of nodeLength

// ICombiningOp of an annotate (ops.ts): none, "rewrite" (segmentPropertiesManager.ts:109-123) or "incr"
// (properties.ts:24-69: each key becomes combine(op, previousValue, undefined, seq), the previous value or
// defaultValue plus undefined -- NaN for numbers, booleans, null and undefined; a string gets "undefined"
// appended; then minValue when truthy and larger) or "consensus" for sequenced ops (properties.ts:46-62,
// combine_consensus).  Other names are not restated.
struct Comb {
  enum Kind { None, Rewrite, Incr, Consensus } kind = None;
  JVal defaultValue;  // Undef when absent
  JVal minValue;
};
Comb parse_comb(const JVal* comb);  // (throws OracleError unsupported for other names)

struct Block;

struct Node {
  bool leaf;
  Block* parent = nullptr;
  int index = 0;
  int cachedLength = 0;
  explicit Node(bool l) : leaf(l) {}
};

constexpr int HandleUnallocated = INT32_MIN;  // Handle.unallocated (matrix/src/handletable.ts:11)

struct Seg : Node {
  bool isMarker = false;
  bool perm = false;               // PermutationSegment (matrix/src/permutationvector.ts:41)
  int start = HandleUnallocated;   // PermutationSegment._start
  int refType = -1;                // -1 = undefined
  u16str text;                     // TextSegment text (markers: empty)
  int seq = UniversalSeq;          // BaseSegment.seq default (mergeTreeNodes.ts:368)
  int clientId = LocalClientId;    // BaseSegment.clientId default
  bool removed = false;
  int removedSeq = 0;
  std::vector<int> removedClientIds;
  std::optional<JObj> props;       // properties (undefined when nullopt)
  bool hasPropManager = false;     // propertyManager !== undefined
  // local (unacked) state of a live client (mergeTreeNodes.ts:367-440): localSeq / localRemovedSeq
  // (kNoLocalSeq = undefined), the queue of pending segment groups, PropertiesManager.pendingKeyUpdateCount
  int localSeq = INT32_MIN;
  int localRemovedSeq = INT32_MIN;
  std::vector<struct SegGroup*> groups;  // a queue (front = oldest); a vector allocates nothing when empty
  std::map<u16str, int> pendingKeys;
  int pendingRewrite = 0;          // PropertiesManager.pendingRewriteCount (segmentPropertiesManager.ts:26)
  Seg() : Node(true) {}
};

// SegmentGroup (mergeTreeNodes.ts:292-300): the segments of one local op awaiting its ack
struct SegGroup {
  std::vector<Seg*> segments;
  int localSeq = INT32_MIN;
  int refSeq = 0;
};

// PartialSequenceLength entry (MT/partialLengths.ts:105-140)
struct PSL {
  int seq = 0, len = 0, seglen = 0, clientId = 0;
  std::shared_ptr<std::map<int, int>> overlap;  // overlapRemoveClients: clientId -> seglen
};

// PartialSequenceLengthsSet (MT/partialLengths.ts:19-95 over SortedSet MT/sortedSet.ts)
struct PSLSet {
  std::vector<PSL> items;
  std::pair<bool, size_t> find(int seq) const;
  PSL* latestLeq(int seq);
  PSL* firstGte(int seq);
  void addOrUpdate(PSL item);
  int copyDown(int minSeq);
};

struct CollabWindow {  // MT/mergeTreeNodes.ts:656-673
  int clientId = LocalClientId;
  bool collaborating = false;
  int minSeq = 0;
  int currentSeq = 0;
  int localSeq = 0;
};

// PartialSequenceLengths (MT/partialLengths.ts:239-850), remote-perspective part only.
struct PartialLengths {
  int minSeq = 0;
  int minLength = 0;
  int segmentCount = 0;
  PSLSet partialLengths;
  // clientSeqNumbers[clientId] (partialLengths.ts:585), indexed by clientId + 2 (ids >= NonCollabClient)
  std::vector<PSLSet> clientSeqNumbers;
  PSLSet& cli(int clientId) {
    size_t k = (size_t)(clientId + 2);
    if (k >= clientSeqNumbers.size()) clientSeqNumbers.resize(k + 1);
    return clientSeqNumbers[k];
  }
  int getPartialLength(int refSeq, int clientId);
  void zamboni(const CollabWindow& w);
  // Shadow of the engine's deficit model (test infrastructure, checked when MTO_DEFCHECK is set; DESIGN.md §7
  // "Deficits"): kind 1 = main-set entries from t on short by d, 2 = client c's set from t on, 3 = in minLength;
  // hmin = minLength without the kind-3 shortfalls.
  struct Def { int kind, t, d, c; };
  std::vector<Def> defs;
  int hmin = 0;
  void checkDefs(const char* where) const;
  void addClientSeqNumber(int clientId, int seq, int seglen);
  void addClientSeqNumberFromPartial(const PSL& p);
};

struct Block : Node {
  int id = 0;  // creation order (diagnostics)
  int childCount = 0;
  std::vector<Node*> children;
  int needsScour = -1;  // -1 undefined, 0 false, 1 true  (IMergeBlock.needsScour)
  std::unique_ptr<PartialLengths> partial;
  Block() : Node(false), children(MaxNodesInBlock, nullptr) {}
  void assignChild(Node* c, int i) {
    c->parent = this;
    c->index = i;
    if ((int)children.size() <= i) children.resize(i + 1, nullptr);
    children[i] = c;
  }
};

struct Options {
  bool newLengthCalc = false;  // mergeTreeUseNewLengthCalculations
  int chunkSize = 10000;       // SnapshotV1.chunkSize (snapshotV1.ts:37)
  bool verify = false;         // cross-check partial lengths against a leaf sum (test-only)
};

struct OracleError : std::runtime_error {
  int code;
  OracleError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct Counters {
  uint64_t ops = 0, segsTouched = 0, maxHeap = 0, maxDepth = 0;
  // PartialSequenceLengths.update below the root met an entry newer than its seq (a summary body's insert):
  // addSeq leaves the later entries' cumulative lengths stale (the engine refuses such loads)
  uint64_t staleUpdates = 0;
  uint64_t staleDeficits = 0;  // updates that left entries after their seq short (addSeq over an existing entry)
};

class MergeTree {
 public:
  explicit MergeTree(const Options& o);
  Options options;
  CollabWindow window;
  Block* root;
  Counters counters;

  // segment / block pools (pointers stay valid for the tree's lifetime)
  std::deque<Seg> segPool;
  std::deque<Block> blockPool;
  Seg* newSeg() { segPool.emplace_back(); return &segPool.back(); }
  Block* makeBlock(int childCount);

  // LRU heap (MT/collections/heap.ts) of {segment, maxSeq}; index 0 is the {maxSeq:-2} sentinel.
  struct LRU { Seg* seg; int maxSeq; };
  std::vector<LRU> heap;
  bool heapValid = false;
  void heapAdd(LRU x);
  LRU heapGet();

  int localNetLength(const Seg* s) const;
  int nodeLength(Node* n, int refSeq, int clientId);
  int blockLength(Block* b, int refSeq, int clientId);
  int getLength(int refSeq, int clientId) { return blockLength(root, refSeq, clientId); }
  int length() const { return root->cachedLength; }

  void startCollaboration(int localClientId, int minSeq, int currentSeq);
  void setMinSeq(int minSeq);
  void insertSegments(int pos, Seg* seg, int refSeq, int clientId, int seq);
  // insertSegments with several segments (mergeTree.ts:1397-1427 over blockInsert :1594-1685)
  void insertSegmentsBatch(int pos, const std::vector<Seg*>& segs, int refSeq, int clientId, int seq);
  // reloadFromSegments (mergeTree.ts:678-721): bottom-up B-tree, MaxNodesInBlock - 1 children per block
  void reloadFromSegments(const std::vector<Seg*>& segs);
  void markRangeRemoved(int start, int end, int refSeq, int clientId, int seq);
  void annotateRange(int start, int end, const JObj& props, const Comb& comb, int refSeq, int clientId, int seq);
  // pendingSegments (mergeTree.ts:532) and ackPendingSegment (:1283-1322) for one acked delta op
  // (type INSERT 0 / REMOVE 1 / ANNOTATE 2, its props for ANNOTATE)
  std::deque<std::unique_ptr<SegGroup>> groupPool;
  std::deque<SegGroup*> pendingSegments;
  void ackPendingSegment(int opType, const JObj* props, int seq, bool rewrite = false);
  void zamboniSegments();
  // mergeTreeDeltaCallback (INSERT 0 / REMOVE 1 / ANNOTATE 2 with the annotate's props), fired after the
  // op is applied and before its zamboni, only for non-empty delta segment lists
  std::function<void(int, const std::vector<Seg*>&, const std::vector<std::vector<u16str>>*)> onDelta;  // annotates: each segment's propertyDeltas keys
  // MergeTreeMaintenanceType.UNLINK observer (zamboni.ts:139-148)
  std::function<void(Seg*)> onUnlink;
  // getContainingSegment (mergeTree.ts:787-813) and getPosition (:1240) for PermutationVector
  Seg* containingSegment(int pos, int refSeq, int clientId, int* offset);
  int localPosition(Seg* s);
  // getPosition (mergeTree.ts:768-785) in any (refSeq, clientId) view; 0 for an unlinked node
  int getPosition(Node* n, int refSeq, int clientId);
  // idToSegment (mergeTree.ts:549): marker id -> marker.  Filled by insertSegments for every inserted
  // marker with an id (:1658-1663) and by every blockUpdate for its live child markers (:2392 ->
  // addNodeReferences :296-306, last child wins); never pruned.  Keys: markerIdKey of the JSON value.
  std::map<std::string, Seg*> idToSegment;
  static std::optional<std::string> markerIdKey(const JVal* v);
  static std::optional<std::string> markerId(const Seg* s);  // Marker.getId (mergeTreeNodes.ts:612-617)
  // posFromRelativePos (mergeTree.ts:1371-1395): -1 when the id names no marker
  int posFromRelativePos(const JVal& rel, int refSeq, int clientId);
  // ---- reconnect (client.ts:690-800, 917-960; mergeTree.ts:2234-2390)
  // localNetLength(segment, refSeq, localSeq) with a localSeq (mergeTree.ts:613-665)
  int localNetLengthAt(const Seg* s, int refSeq, int localSeq) const;
  // findReconnectionPosition (client.ts:690-706): getPosition(segment, currentSeq, clientId, localSeq), the
  // local view without the pending ops after localSeq, as the sum over the leaves before the segment
  int reconnectPosition(Seg* s, int localSeq);
  // normalizeSegmentsOnRebase (mergeTree.ts:2357-2390) / normalizeAdjacentSegments (:2234-2336)
  void normalizeSegmentsOnRebase();
  void normalizeAdjacentSegments(std::vector<Seg*>& run);
  void boundary(int pos, int refSeq, int clientId) { ensureIntervalBoundary(pos, refSeq, clientId); }
  // mapRange(action, refSeq, clientId) over the whole tree (mergeTree.ts mapRange -> nodeMap)
  void mapAll(int refSeq, int clientId, const std::function<void(Seg*)>& f);
  // mapRange (mergeTree.ts:2456-2474) over [start, end) (end < 0: the whole (refSeq, clientId) length)
  void mapRange(int refSeq, int clientId, int start, int end, const std::function<bool(Seg*, int, int, int)>& f);

  // packParent(root) as the reference's zamboni tests call it directly (mergeTree.zamboni.spec.ts)
  void packParentRoot() { packParent(root); }

  // text / walks
  u16str getText();
  template <class F> void walkAllSegments(F&& f);

  // structure maintenance (public for the snapshot code)
  void nodeUpdateLengthNewStructure(Block* b, bool recur = false);
  int bruteLength(Node* n, int refSeq, int clientId);

 private:
  struct Changes { Seg* replaceCurrent = nullptr; Node* next = nullptr; };
  struct InsertCtx { bool insertMode = false; Seg* candidate = nullptr; };
  Block* const UNFINISHED = reinterpret_cast<Block*>(1);

  bool breakTie(int pos, Node* n, int seq);
  Block* insertingWalk(Block* b, int pos, int refSeq, int clientId, int seq, InsertCtx& ctx);
  Changes leafAction(InsertCtx& ctx, Seg* s, int pos);
  Seg* splitAt(Seg* s, int pos);
  void ensureIntervalBoundary(int pos, int refSeq, int clientId);
  void blockInsert(int pos, int refSeq, int clientId, int seq, Seg* seg, int localSeq = INT32_MIN,
                   SegGroup** group = nullptr);
  bool continuePredicate(Block* b);
  Block* split(Block* b);
  void updateRoot(Block* splitNode);
  void blockUpdate(Block* b);
  void blockUpdateLength(Block* b, int seq, int clientId);
  void blockUpdatePathLengths(Block* b, int seq, int clientId, bool newStructure);
  void addToLRUSet(Seg* s, int seq);
  SegGroup* addToPendingList(Seg* s, SegGroup* g, int localSeq);  // mergeTree.ts:1324-1357
  void scourNode(Block* node, std::vector<Node*>& hold);
  void packParent(Block* parent);
  template <class Leaf, class Post>
  void nodeMap(int refSeq, int clientId, Leaf&& leaf, Post&& post, int start, int end);

  // PartialSequenceLengths construction (partialLengths.ts:256-577, 636-686)
  std::unique_ptr<PartialLengths> combine(Block* b, bool recur);
  std::unique_ptr<PartialLengths> fromLeaves(Block* b);
  void plInsertSegment(PartialLengths& pl, Seg* s, bool removal);
  void plUpdate(PartialLengths& pl, Block* node, int seq, int clientId);
};

// -------------------------------------------------------------- client-level document
class Doc {
 public:
  explicit Doc(const Options& o) : mt(o) {}
  MergeTree mt;
  std::vector<std::string> longIds;         // shortClientIdMap (client.ts:104)
  std::map<std::string, int> longToShort;   // clientNameToIds
  std::optional<std::string> longClientId;  // the observer's own long id

  int getOrAddShortClientId(const std::string& id);
  std::string getLongClientId(int shortId) const;
  void startOrUpdateCollaboration(const std::string& id, int minSeq, int curSeq);
  void updateSeqNumbers(int min, int seq);

  // a live client's local ops while collaborating (client.ts:196-247 insertSegmentLocal /
  // removeRangeLocal / annotateRangeLocal): applied at (currentSeq, own id, UnassignedSequenceNumber)
  // and returned as the IMergeTreeOp JSON to submit; acked by applyMsg of the sequenced message
  std::string insertLocalOp(int pos, const JVal& segSpec);
  std::string removeLocalOp(int start, int end);
  std::string annotateLocalOp(int start, int end, const JObj& props, const JVal* combiningOp = nullptr,
                              bool notifyConsensus = false);
  // Client.pendingConsensus (client.ts:155-181, 1050-1058): marker id -> the marker annotateMarkerNotifyConsensus
  // annotated; the ack of a consensus annotate naming it completes the marker's values at the ack's seq
  std::map<std::string, Seg*> pendingConsensus;
  // a live client's local op given as the IMergeTreeOp JSON it sends (pos1 / pos2 or marker-relative
  // relativePos1 / relativePos2, resolved in the local view by getValidOpRange, client.ts:527-547); returns
  // the op to send (the input itself when it names relative positions, as Client.annotateMarker does)
  std::string localOpJson(const JVal& op);
  // Client.regeneratePendingOp (client.ts:917-960) for the op at the head of the pending queue (one segment
  // group per member op): the op(s) to resubmit after a reconnect, as JSON
  std::string regeneratePendingOp(const JVal& op);
  int lastNormalizationRefSeq = 0;
  // local, non-collaborating edits (detached documents; used for the V1 snapshot fixtures)
  void insertTextLocal(int pos, const u16str& text, const std::optional<JObj>& props);
  void insertMarkerLocal(int pos, int refType, const std::optional<JObj>& props);
  void annotateRangeLocal(int start, int end, const JObj& props);
  void removeRangeLocal(int start, int end);

  // Client.applyMsg with a parsed ISequencedDocumentMessage
  void applyMsg(const JVal& msg);
  void applyMsgCore(const JVal& msg);
  // remote delta op (already decoded)
  void applyRemoteDelta(const JVal& op, int clientShort, int refSeq, int seq);
  // binary record path (include/mtb.h mtb_op)
  struct Record {
    uint8_t type, flags;
    uint16_t client;
    uint32_t seq, refSeq, msn, pos1, pos2, payload, props;
  };
  void applyRecord(const Record& r, const uint16_t* text, const std::vector<std::string>& propsJson);
  void applyRecordParsed(const Record& r, const uint16_t* text, const std::vector<std::optional<JVal>>& props);

  // Client.load of a SnapshotV1 summary (snapshotLoader.ts:41-257): header -> reloadFromSegments ->
  // startOrUpdateCollaboration(observer, minSeq, seq) -> body chunks appended through insertSegments.
  void loadV1(const std::vector<std::pair<std::string, std::string>>& blobs, const std::string& observerId);
  // the catch-up messages blob of a (legacy) summary's blob list, "[]" when there is none (snapshotLoader.ts:60-86)
  static std::string catchUpOps(const std::vector<std::pair<std::string, std::string>>& blobs);
  // SnapshotV1 (snapshotV1.ts:46-312) -> (blob path, content) list + ISummaryTreeWithStats JSON
  std::vector<std::pair<std::string, std::string>> summarizeV1(std::string* summaryJson);
  // SnapshotLegacy (snapshotlegacy.ts:122-259): header / body chunks at the MSN, plus the catch-up
  // messages blob when `catchUpJson` is a non-empty JSON array
  std::vector<std::pair<std::string, std::string>> summarizeLegacy(const std::string& catchUpJson, std::string* summaryJson);
  // canonical segment dump used for engine parity (one JSON object per line)
  std::string dumpSegments();
  // state digest v1 (DESIGN.md "State digest"): the dump's content folded into 64 bits
  uint64_t digest();

  // ---- SharedSegmentSequence catch-up messages (sequence.ts:680-748) for SnapshotLegacy summaries
  bool catchUp = false;
  std::vector<JVal> messagesSinceMSNChange;
  void processMinSequenceNumberChanged(int minSeq);
  std::string catchUpJson(int minSeq);

  // ---- PermutationVector (matrix/src/permutationvector.ts) when `perm` is set
  bool perm = false;
  std::vector<int64_t> handles{1};  // HandleTable.handles (handletable.ts:22): [0] = head of the free list
  int allocateHandle();              // handletable.ts:36-41
  void freeHandle(int h);            // handletable.ts:55-58
  // adjustPosition (permutationvector.ts:209-226): the op's position in the local view, or -1
  int adjustPosition(int pos, int refSeq, const std::string& longClientId);
  // getAllocatedHandle (permutationvector.ts:183-207)
  int getAllocatedHandle(int pos);
  std::string handleTableJson() const;
  void enablePermutation();
  // PermutationVector.handlesRecycledCallback (permutationvector.ts:418-441): handles about to be freed
  std::function<void(int start, int count)> onHandlesRecycled;
};

// SparseArray2D (matrix/src/sparsearray2d.ts): cells keyed by Morton-interleaved (row, col) handles in a
// root array indexed by the high 16 bits of both and four 256-entry levels for the low bits.  Values are
// kept as their JSON text (nullopt = undefined).
struct SparseArray2D {
  using Leaf = std::array<std::optional<std::string>, 256>;
  template <class C> using Lvl = std::array<std::unique_ptr<C>, 256>;
  using L3 = Leaf;
  using L2 = Lvl<L3>;
  using L1 = Lvl<L2>;
  using L0 = Lvl<L1>;
  std::map<uint32_t, std::unique_ptr<L0>> root;  // sparse JS array `root`
  uint64_t rootLength = 1;                       // `[undefined]`: length 1
  void setCell(uint32_t row, uint32_t col, std::optional<std::string> value);
  const std::optional<std::string>* getCell(uint32_t row, uint32_t col) const;
  void clearRows(uint32_t rowStart, uint32_t rowCount);
  void clearCols(uint32_t colStart, uint32_t colCount);
  std::string snapshotJson() const;  // JSON.stringify(snapshot())
  static SparseArray2D load(const JVal& data);  // SparseArray2D.load (nullToUndefined over the arrays)
};

// SharedMatrix observer over two PermutationVectors (matrix/src/matrix.ts:636-697); the cell store
// (SparseArray2D) is not restated.
struct MatrixDoc {
  Doc& rows;
  Doc& cols;
  MatrixDoc(Doc& r, Doc& c) : rows(r), cols(c) {
    rows.enablePermutation();
    cols.enablePermutation();
    // onRowHandlesRecycled / onColHandlesRecycled (matrix.ts:721-733)
    rows.onHandlesRecycled = [this](int h, int n) { cells.clearRows((uint32_t)h, (uint32_t)n); };
    cols.onHandlesRecycled = [this](int h, int n) { cells.clearCols((uint32_t)h, (uint32_t)n); };
  }
  void startOrUpdateCollaboration(const std::string& id, int minSeq, int curSeq) {
    rows.startOrUpdateCollaboration(id, minSeq, curSeq);
    cols.startOrUpdateCollaboration(id, minSeq, curSeq);
  }
  void applyMsg(const JVal& msg);
  uint64_t cellsSet = 0, cellsDropped = 0;
  SparseArray2D cells;  // matrix.ts:96 (the observer's `pending` array stays empty)
  // SharedMatrix.summarizeCore (matrix.ts:449-463): {rows, cols: PermutationVector.summarize, cells}
  std::vector<std::pair<std::string, std::string>> summarize(std::string* summaryJson);
  // SharedMatrix.loadCore (matrix.ts:611-634): rows / cols PermutationVector.load (handle table, then
  // the SnapshotV1 segments, permutationvector.ts:327-345) and the cells blob
  void load(const std::vector<std::pair<std::string, std::string>>& blobs, const std::string& observerId);
};

uint64_t fnv1a64(const std::string& s);
JObj propsFromSpec(const JVal* spec);

}  // namespace orc
