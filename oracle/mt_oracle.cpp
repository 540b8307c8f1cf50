// ORACLE / TEST INFRASTRUCTURE ONLY — see mt_oracle.hpp for the contract.
// Clean-room C++ restatement of the merge-tree remote-op (observer) path.  MT = packages/dds/merge-tree/src.
#include "mt_oracle.hpp"

#include <algorithm>
#include <cassert>
#include <functional>
#include <unordered_map>

namespace orc {

static constexpr int64_t MAX_SAFE = 9007199254740991LL;

[[noreturn]] static void fail_assert(const char* code, const char* what) {
  throw OracleError(-4, std::string(code) + " " + what);
}
[[noreturn]] static void fail_unsupported(const std::string& what) {
  throw OracleError(-6, "unsupported: " + what);
}

// =====================================================================================
// PartialSequenceLengthsSet  (MT/partialLengths.ts:19-95, MT/sortedSet.ts:45-71)
// =====================================================================================
std::pair<bool, size_t> PSLSet::find(int seq) const {
  // SortedSet.findItemPosition -> lower_bound semantics
  size_t lo = 0, hi = items.size();
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (items[mid].seq < seq) lo = mid + 1;
    else hi = mid;
  }
  bool exists = lo < items.size() && items[lo].seq == seq;
  return {exists, lo};
}
PSL* PSLSet::latestLeq(int seq) {
  auto [exists, idx] = find(seq);
  long i = exists ? (long)idx : (long)idx - 1;
  return i >= 0 ? &items[i] : nullptr;
}
PSL* PSLSet::firstGte(int seq) {
  auto [exists, idx] = find(seq);
  (void)exists;
  return idx < items.size() ? &items[idx] : nullptr;
}
static void combineOverlapClients(PSL& a, const PSL& b) {  // partialLengths.ts:1009-1027
  if (a.overlap) {
    if (b.overlap)
      for (auto& kv : *b.overlap) (*a.overlap)[kv.first] += kv.second;
  } else if (b.overlap) {
    a.overlap = std::make_shared<std::map<int, int>>(*b.overlap);
  }
}
void PSLSet::addOrUpdate(PSL item) {  // partialLengths.ts:24-47
  PSL* prev = latestLeq(item.seq);
  if (!prev || prev->seq != item.seq) item.len = (prev ? prev->len : 0) + item.seglen;
  for (long i = (long)items.size() - 1; i >= 0; i--) {
    if (items[i].seq <= item.seq) break;
    items[i].len += item.seglen;
  }
  auto [exists, idx] = find(item.seq);
  if (exists) {
    PSL& cur = items[idx];
    cur.seglen += item.seglen;
    cur.len += item.seglen;
    combineOverlapClients(cur, item);
  } else {
    items.insert(items.begin() + idx, std::move(item));
  }
}
int PSLSet::copyDown(int minSeq) {  // partialLengths.ts:76-94
  auto [exists, idx] = find(minSeq);
  long mindex = exists ? (long)idx : (long)idx - 1;
  int minLength = 0;
  if (mindex >= 0) {
    minLength = items[mindex].len;
    size_t remaining = items.size() - mindex - 1;
    for (size_t i = 0; i < remaining; i++) {
      items[i] = items[i + mindex + 1];
      items[i].len -= minLength;
    }
    items.resize(remaining);
  }
  return minLength;
}

// =====================================================================================
// PartialSequenceLengths queries (partialLengths.ts:698-735, 809-819, 822-849)
// =====================================================================================
int PartialLengths::getPartialLength(int refSeq, int clientId) {
  int pLen = minLength;
  PSL* l = partialLengths.latestLeq(refSeq);
  pLen += l ? l->len : 0;
  const size_t k = (size_t)(clientId + 2);
  if (k < clientSeqNumbers.size() && !clientSeqNumbers[k].items.empty()) {
    PSLSet& cs = clientSeqNumbers[k];
    PSL& cliLatest = cs.items.back();
    if (cliLatest.seq > refSeq) {
      pLen += cliLatest.len;
      PSL* preceding = cs.latestLeq(refSeq);
      if (preceding) pLen -= preceding->len;
    }
  }
  return pLen;
}
static bool defcheck() {
  static const bool on = getenv("MTO_DEFCHECK") != nullptr;
  return on;
}
void PartialLengths::zamboni(const CollabWindow& w) {
  if (defcheck()) {
    // copyDown: the main-set deficits that began at or below the copied entry move into minLength; a client
    // set's are dropped with its minLength
    PSL* m = partialLengths.latestLeq(w.minSeq);
    if (m) {
      int h = 0;
      for (auto& e : partialLengths.items) {
        h += e.seglen;
        if (&e == m) break;
      }
      hmin += h;
      for (auto& d : defs)
        if (d.kind == 1 && d.t <= m->seq) d.kind = 3;
    }
    for (size_t k = 0; k < clientSeqNumbers.size(); k++) {
      PSL* mc = clientSeqNumbers[k].latestLeq(w.minSeq);
      if (!mc) continue;
      const int c = (int)k - 2, tm = mc->seq;
      defs.erase(std::remove_if(defs.begin(), defs.end(), [&](const Def& d) { return d.kind == 2 && d.c == c && d.t <= tm; }),
                 defs.end());
    }
  }
  minLength += partialLengths.copyDown(w.minSeq);
  minSeq = w.minSeq;
  for (auto& cs : clientSeqNumbers) cs.copyDown(w.minSeq);
  if (defcheck()) checkDefs("zamboni");
}
void PartialLengths::checkDefs(const char* where) const {
  auto check = [&](const PSLSet& st, int kind, int c) {
    int h = 0;
    for (auto& e : st.items) {
      h += e.seglen;
      int want = 0;
      for (auto& d : defs)
        if (d.kind == kind && (kind == 1 || d.c == c) && d.t <= e.seq) want += d.d;
      if (h - e.len != want)
        throw OracleError(-9, std::string("deficit model: ") + where + ": set " + (kind == 1 ? "main" : "client " + std::to_string(c)) +
                                  " entry " + std::to_string(e.seq) + " short by " + std::to_string(h - e.len) +
                                  ", model " + std::to_string(want));
    }
  };
  check(partialLengths, 1, 0);
  for (size_t k = 0; k < clientSeqNumbers.size(); k++) check(clientSeqNumbers[k], 2, (int)k - 2);
  int m = 0;
  for (auto& d : defs)
    if (d.kind == 3) m += d.d;
  if (hmin - minLength != m)
    throw OracleError(-9, std::string("deficit model: ") + where + ": minLength short by " + std::to_string(hmin - minLength) +
                              ", model " + std::to_string(m));
}
void PartialLengths::addClientSeqNumber(int clientId, int seq, int seglen) {
  PSL p;
  p.seq = seq;
  p.len = 0;
  p.seglen = seglen;
  cli(clientId).addOrUpdate(p);
}
void PartialLengths::addClientSeqNumberFromPartial(const PSL& p) {
  addClientSeqNumber(p.clientId, p.seq, p.seglen);
  if (p.overlap)
    for (auto& kv : *p.overlap)
      if (p.clientId != kv.first) addClientSeqNumber(kv.first, p.seq, kv.second);
}

// Returns the amount by which the entries after `seq` are left short: an existing entry at `seq` gets its seglen
// replaced (not added to) while the later entries' cumulative len keep the old one (0 when nothing follows).
static int addSeq(PSLSet& set, int seq, int seqSeglen, int clientId) {  // partialLengths.ts:543-577
  PSL* seqPartial = nullptr;
  PSL* penult = nullptr;
  PSL* p = set.latestLeq(seq);
  if (p) {
    if (p->seq == seq) {
      seqPartial = p;
      PSL* q = set.latestLeq(seq - 1);
      if (q) penult = q;
    } else {
      penult = p;
    }
  }
  int len = penult ? penult->len + seqSeglen : seqSeglen;
  if (!seqPartial) {
    PSL n;
    n.clientId = clientId;
    n.len = len;
    n.seglen = seqSeglen;
    n.seq = seq;
    set.addOrUpdate(n);
    return 0;
  }
  const int deficit = set.items.back().seq > seq ? seqSeglen - seqPartial->seglen : 0;
  seqPartial->seglen = seqSeglen;
  seqPartial->len = len;
  return deficit;
}

// =====================================================================================
// MergeTree
// =====================================================================================
MergeTree::MergeTree(const Options& o) : options(o) {
  root = makeBlock(0);
  heap.push_back({nullptr, -2});  // LRUSegmentComparer.min (mergeTree.ts:112)
}

Block* MergeTree::makeBlock(int childCount) {
  blockPool.emplace_back();
  Block* b = &blockPool.back();
  b->id = (int)blockPool.size() - 1;
  b->childCount = childCount;
  return b;
}

// Heap (MT/collections/heap.ts:11-66) with compare = a.maxSeq - b.maxSeq
void MergeTree::heapAdd(LRU x) {
  heap.push_back(x);
  if (heap.size() - 1 > counters.maxHeap) counters.maxHeap = heap.size() - 1;
  size_t k = heap.size() - 1;
  while (k > 1 && heap[k >> 1].maxSeq - heap[k].maxSeq > 0) {
    std::swap(heap[k >> 1], heap[k]);
    k >>= 1;
  }
}
MergeTree::LRU MergeTree::heapGet() {
  LRU x = heap[1];
  size_t count = heap.size() - 1;
  heap[1] = heap[count];
  heap.pop_back();
  count = heap.size() - 1;
  size_t k = 1;
  while ((k << 1) <= count) {
    size_t j = k << 1;
    if (j < count && heap[j].maxSeq - heap[j + 1].maxSeq > 0) j++;
    if (heap[k].maxSeq - heap[j].maxSeq <= 0) break;
    std::swap(heap[k], heap[j]);
    k = j;
  }
  return x;
}

// localNetLength (mergeTree.ts:613-634), localSeq === undefined branch
int MergeTree::localNetLength(const Seg* s) const {
  if (s->removed) {
    if (!options.newLengthCalc) {
      int64_t norm = s->removedSeq == UnassignedSeq ? MAX_SAFE : s->removedSeq;
      if (norm > window.minSeq) return 0;
      return UNDEF_LEN;
    }
    return 0;
  }
  return s->cachedLength;
}

int MergeTree::bruteLength(Node* n, int refSeq, int clientId) {
  if (n->leaf) {
    int l = nodeLength(n, refSeq, clientId);
    return l == UNDEF_LEN ? 0 : l;
  }
  Block* b = static_cast<Block*>(n);
  int sum = 0;
  for (int i = 0; i < b->childCount; i++) sum += bruteLength(b->children[i], refSeq, clientId);
  return sum;
}

// nodeLength (mergeTree.ts:916-1004); returns UNDEF_LEN for `undefined`
int MergeTree::nodeLength(Node* node, int refSeq, int clientId) {
  if (!window.collaborating || window.clientId == clientId) {
    if (node->leaf) return localNetLength(static_cast<Seg*>(node));
    return node->cachedLength;
  }
  if (!node->leaf) {
    Block* b = static_cast<Block*>(node);
    int v = b->partial->getPartialLength(refSeq, clientId);
    if (options.verify) {
      int brute = 0;
      for (int i = 0; i < b->childCount; i++) brute += bruteLength(b->children[i], refSeq, clientId);
      if (brute != v)
        throw OracleError(-4, "verify: partial length " + std::to_string(v) + " != leaf sum " + std::to_string(brute));
    }
    return v;
  }
  Seg* seg = static_cast<Seg*>(node);
  if (options.newLengthCalc) {
    int64_t seq = seg->seq == UnassignedSeq ? MAX_SAFE - 1 : seg->seq;
    if (seg->removed) {
      int64_t rs = seg->removedSeq == UnassignedSeq ? MAX_SAFE : seg->removedSeq;
      if (rs <= window.minSeq) return UNDEF_LEN;
      if (rs <= refSeq ||
          std::find(seg->removedClientIds.begin(), seg->removedClientIds.end(), clientId) != seg->removedClientIds.end())
        return 0;
    }
    return (seq <= refSeq || seg->clientId == clientId) ? seg->cachedLength : 0;
  }
  if (seg->removed && seg->removedSeq != UnassignedSeq && seg->removedSeq <= refSeq) return UNDEF_LEN;
  if (seg->clientId == clientId || (seg->seq != UnassignedSeq && seg->seq <= refSeq)) {
    if (seg->removed) {
      return std::find(seg->removedClientIds.begin(), seg->removedClientIds.end(), clientId) != seg->removedClientIds.end()
                 ? 0
                 : seg->cachedLength;
    }
    return seg->cachedLength;
  }
  if (seg->removed && seg->removedSeq != UnassignedSeq) return UNDEF_LEN;
  return 0;
}

int MergeTree::blockLength(Block* b, int refSeq, int clientId) {  // mergeTree.ts:884-888
  return window.collaborating && clientId != window.clientId ? b->partial->getPartialLength(refSeq, clientId)
                                                              : b->cachedLength;
}

// startCollaboration (mergeTree.ts:731-739)
void MergeTree::startCollaboration(int localClientId, int minSeq, int currentSeq) {
  window.clientId = localClientId;
  window.minSeq = minSeq;
  window.collaborating = true;
  window.currentSeq = currentSeq;
  heap.clear();
  heap.push_back({nullptr, -2});
  heapValid = true;
  nodeUpdateLengthNewStructure(root, true);
}

// addToLRUSet (mergeTree.ts:741-751)
void MergeTree::addToLRUSet(Seg* s, int seq) {
  if (s->parent->needsScour != 1 && seq > window.currentSeq) {
    s->parent->needsScour = 1;
    heapAdd({s, seq});
  }
}

// setMinSeq (mergeTree.ts:1025-1044)
void MergeTree::setMinSeq(int minSeq) {
  if (!(minSeq <= window.currentSeq)) fail_assert("0x04e", "Trying to set minSeq above currentSeq of collab window!");
  if (!(window.minSeq <= minSeq)) fail_assert("0x04f", "minSeq of collab window > target minSeq!");
  if (minSeq > window.minSeq) {
    window.minSeq = minSeq;
    zamboniSegments();
  }
}

// breakTie (mergeTree.ts:1719-1738)
bool MergeTree::breakTie(int pos, Node* node, int seq) {
  if (node->leaf) {
    if (pos == 0) {
      int64_t newSeq = seq == UnassignedSeq ? MAX_SAFE : seq;
      Seg* s = static_cast<Seg*>(node);
      int64_t segSeq = s->seq == UnassignedSeq ? MAX_SAFE - 1 : s->seq;
      return newSeq > segSeq;
    }
    return false;
  }
  return true;
}

// BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTreeNodes.ts:481-523, textSegment.ts:106-114)
Seg* MergeTree::splitAt(Seg* s, int pos) {
  if (pos <= 0 || s->isMarker) return nullptr;  // Marker.createSplitSegmentAt -> undefined
  Seg* r = newSeg();
  if (s->perm) {  // PermutationSegment.createSplitSegmentAt (permutationvector.ts:126-140)
    r->perm = true;
    r->start = s->start == HandleUnallocated ? HandleUnallocated : s->start + pos;
    r->cachedLength = s->cachedLength - pos;
    s->cachedLength = pos;
  } else {
    r->text = s->text.substr(pos);
    s->text.resize(pos);
    s->cachedLength = (int)s->text.size();
    r->cachedLength = (int)r->text.size();
  }
  if (s->hasPropManager && s->props) {  // copyPropertiesTo
    r->hasPropManager = true;
    r->props = *s->props;
  }
  r->parent = s->parent;
  r->removed = s->removed;
  r->removedClientIds = s->removedClientIds;
  r->removedSeq = s->removedSeq;
  r->seq = s->seq;
  r->clientId = s->clientId;
  r->localSeq = s->localSeq;
  r->localRemovedSeq = s->localRemovedSeq;
  for (SegGroup* g : s->groups) {  // segmentGroups.copyTo (mergeTreeNodes.ts:239-245)
    g->segments.push_back(r);
    r->groups.push_back(g);
  }
  if (s->hasPropManager && s->props) {  // PropertiesManager.copyTo
    r->pendingKeys = s->pendingKeys;
    r->pendingRewrite = s->pendingRewrite;
  }
  counters.segsTouched += 2;  // split: left half modified + right half created
  return r;
}

MergeTree::Changes MergeTree::leafAction(InsertCtx& ctx, Seg* segment, int pos) {
  Changes c;
  if (ctx.insertMode) {  // blockInsert.onLeaf (mergeTree.ts:1644-1654)
    if (segment) {
      c.replaceCurrent = ctx.candidate;
      c.next = segment;
    } else {
      c.next = ctx.candidate;
    }
  } else {  // splitLeafSegment (mergeTree.ts:1686-1704)
    if (!(pos > 0 && segment)) return c;
    Seg* next = splitAt(segment, pos);
    c.next = next;
  }
  return c;
}

// blockInsert.continueFrom: forwardExcursion(block) looking at the first following segment
// (mergeTree.ts:1611-1615, mergeTreeNodeWalk.ts:121-138)
bool MergeTree::continuePredicate(Block* node) {
  // find first leaf after `node` in tree order
  Node* cur = node;
  while (cur->parent) {
    Block* p = cur->parent;
    for (int i = cur->index + 1; i < p->childCount; i++) {
      Node* c = p->children[i];
      while (c && !c->leaf) {
        Block* cb = static_cast<Block*>(c);
        c = cb->childCount > 0 ? cb->children[0] : nullptr;
        if (!c) break;
      }
      if (c && c->leaf) return static_cast<Seg*>(c)->seq == UnassignedSeq;
    }
    cur = p;
  }
  return false;
}

// insertingWalk (mergeTree.ts:1740-1856)
Block* MergeTree::insertingWalk(Block* block, int pos, int refSeq, int clientId, int seq, InsertCtx& ctx) {
  int _pos = pos;
  int childIndex;
  Node* newNode = nullptr;
  Block* fromSplit = nullptr;
  for (childIndex = 0; childIndex < block->childCount; childIndex++) {
    Node* child = block->children[childIndex];
    int len = nodeLength(child, refSeq, clientId);
    if (len == UNDEF_LEN) continue;
    if (len < 0) fail_assert("0x4bc", "Length should not be negative");
    if (_pos < len || (_pos == len && breakTie(_pos, child, seq))) {
      if (!child->leaf) {
        Block* splitNode = insertingWalk(static_cast<Block*>(child), _pos, refSeq, clientId, seq, ctx);
        if (splitNode == nullptr) {
          blockUpdateLength(block, seq, clientId);
          return nullptr;
        } else if (splitNode == UNFINISHED) {
          _pos -= len;
          continue;
        } else {
          newNode = splitNode;
          fromSplit = splitNode;
          childIndex++;
        }
      } else {
        Seg* segment = static_cast<Seg*>(child);
        Changes ch = leafAction(ctx, segment, _pos);
        if (ch.replaceCurrent) block->assignChild(ch.replaceCurrent, childIndex);
        if (ch.next) {
          newNode = ch.next;
          childIndex++;
        } else {
          return nullptr;
        }
      }
      break;
    } else {
      _pos -= len;
    }
  }
  if (!newNode) {
    if (_pos == 0) {
      if (seq != UnassignedSeq && ctx.insertMode && continuePredicate(block)) {
        return UNFINISHED;
      } else {
        Changes ch = leafAction(ctx, nullptr, _pos);
        newNode = ch.next;
      }
    }
  }
  if (newNode) {
    if ((int)block->children.size() <= block->childCount) block->children.resize(block->childCount + 1, nullptr);
    for (int i = block->childCount; i > childIndex; i--) {
      block->children[i] = block->children[i - 1];
      block->children[i]->index = i;
    }
    block->assignChild(newNode, childIndex);
    block->childCount++;
    (void)fromSplit;  // ordinals are not modelled (local references only)
    if (block->childCount < MaxNodesInBlock) {
      blockUpdateLength(block, seq, clientId);
      return nullptr;
    }
    return split(block);
  }
  return nullptr;
}

// split (mergeTree.ts:1858-1871)
Block* MergeTree::split(Block* node) {
  const int half = MaxNodesInBlock / 2;
  Block* nb = makeBlock(half);
  node->childCount = half;
  for (int i = 0; i < half; i++) {
    nb->assignChild(node->children[half + i], i);
    node->children[half + i] = nullptr;
  }
  nodeUpdateLengthNewStructure(node);
  nodeUpdateLengthNewStructure(nb);
  return nb;
}

// updateRoot (mergeTree.ts:1268-1277)
void MergeTree::updateRoot(Block* splitNode) {
  if (splitNode) {
    Block* nr = makeBlock(2);
    nr->assignChild(root, 0);
    nr->assignChild(splitNode, 1);
    root = nr;
    nodeUpdateLengthNewStructure(root);
  }
}

// ensureIntervalBoundary (mergeTree.ts:1706-1716)
void MergeTree::ensureIntervalBoundary(int pos, int refSeq, int clientId) {
  InsertCtx ctx;
  ctx.insertMode = false;
  Block* sn = insertingWalk(root, pos, refSeq, clientId, TreeMaintenanceSeq, ctx);
  updateRoot(sn);
}

// blockInsert (mergeTree.ts:1594-1685), single segment
void MergeTree::blockInsert(int pos, int refSeq, int clientId, int seq, Seg* seg, int localSeq, SegGroup** group) {
  if (seg->cachedLength > 0) {
    if (auto id = markerId(seg)) idToSegment[*id] = seg;  // mapIdToSegment (mergeTree.ts:1658-1663)
    seg->seq = seq;
    seg->localSeq = localSeq;
    seg->clientId = clientId;
    InsertCtx ctx;
    ctx.insertMode = true;
    ctx.candidate = seg;
    Block* sn = insertingWalk(root, pos, refSeq, clientId, seq, ctx);
    if (seg->parent == nullptr) throw OracleError(-5, "MergeTree insert failed");
    updateRoot(sn);
    // saveIfLocal (mergeTree.ts:1617-1637)
    if (window.collaborating) {
      if (seg->seq == UnassignedSeq && clientId == window.clientId) {
        SegGroup* g = addToPendingList(seg, group ? *group : nullptr, localSeq);
        if (group) *group = g;
      } else if (seg->seq > window.minSeq) {
        addToLRUSet(seg, seg->seq);
      }
    }
    counters.segsTouched += 1;
  }
}

// insertSegments (mergeTree.ts:1397-1427)
void MergeTree::insertSegments(int pos, Seg* seg, int refSeq, int clientId, int seq) {
  ensureIntervalBoundary(pos, refSeq, clientId);
  const int localSeq = seq == UnassignedSeq ? ++window.localSeq : INT32_MIN;  // mergeTree.ts:1407-1408
  SegGroup* group = nullptr;
  blockInsert(pos, refSeq, clientId, seq, seg, localSeq, &group);
  if (onDelta && seg->parent && seg->cachedLength > 0) onDelta(0, {seg}, nullptr);
  if (window.collaborating && seq != UnassignedSeq) zamboniSegments();
}

// insertSegments with a batch of segments (mergeTree.ts:1397-1427): one ensureIntervalBoundary, each
// segment placed by blockInsert at an advancing position (insertPos += cachedLength, :1664-1684), one
// zamboni at the end.
void MergeTree::insertSegmentsBatch(int pos, const std::vector<Seg*>& segs, int refSeq, int clientId, int seq) {
  ensureIntervalBoundary(pos, refSeq, clientId);
  int insertPos = pos;
  for (Seg* sg : segs) {
    if (sg->cachedLength > 0) {
      blockInsert(insertPos, refSeq, clientId, seq, sg);
      insertPos += sg->cachedLength;
    }
  }
  if (window.collaborating && seq != UnassignedSeq) zamboniSegments();
}

// reloadFromSegments (mergeTree.ts:678-721)
void MergeTree::reloadFromSegments(const std::vector<Seg*>& segs) {
  if (window.collaborating) fail_assert("0x049", "Trying to reload from segments while collaborating!");
  const int maxChildren = MaxNodesInBlock - 1;
  if (segs.empty()) {
    root = makeBlock(0);
    return;
  }
  std::vector<Node*> nodes(segs.begin(), segs.end());
  while (true) {
    const size_t blockCount = (nodes.size() + maxChildren - 1) / maxChildren;
    std::vector<Node*> blocks;
    size_t ni = 0;
    for (size_t bi = 0; bi < blockCount; bi++) {
      Block* b = makeBlock(0);
      for (int ci = 0; ci < maxChildren && ni < nodes.size(); ci++, ni++) b->assignChild(nodes[ni], b->childCount++);
      blockUpdate(b);
      blocks.push_back(b);
    }
    if (blocks.size() == 1) {
      root = static_cast<Block*>(blocks[0]);
      return;
    }
    nodes = blocks;
  }
}

// blockUpdate (mergeTree.ts:2392-2417): cachedLength = sum(nodeTotalLength ?? 0); addNodeReferences
// (:296-306) maps every child marker with an id whose localNetLength is positive
void MergeTree::blockUpdate(Block* b) {
  int len = 0;
  for (int i = 0; i < b->childCount; i++) {
    Node* c = b->children[i];
    int l = c->leaf ? localNetLength(static_cast<Seg*>(c)) : c->cachedLength;
    len += l == UNDEF_LEN ? 0 : l;
    if (c->leaf && l > 0 && static_cast<Seg*>(c)->isMarker) {
      if (auto id = markerId(static_cast<Seg*>(c))) idToSegment[*id] = static_cast<Seg*>(c);
    }
  }
  b->cachedLength = len;
}

// Map keys of marker ids: JS Map identity (SameValueZero) of the primitive values a JSON id can be;
// object ids never equal a parsed relativePos id, so they are never looked up (and not kept).
std::optional<std::string> MergeTree::markerIdKey(const JVal* v) {
  if (js_falsy(v)) return std::nullopt;  // `if (relativePos.id)` / `if (this.properties[reservedMarkerIdKey])`
  switch (v->t) {
    case JVal::Str: return "s" + u16_to_utf8(v->str);
    case JVal::Num: return "n" + json_stringify(*v);
    case JVal::True: return std::string("t");
    default: return std::nullopt;
  }
}
std::optional<std::string> MergeTree::markerId(const Seg* s) {
  if (!s->isMarker || !s->props) return std::nullopt;
  return markerIdKey(obj_get(*s->props, u"markerId"));
}

// getPosition (mergeTree.ts:768-785)
int MergeTree::getPosition(Node* node, int refSeq, int clientId) {
  int total = 0;
  for (Block* parent = node->parent; parent; node = parent, parent = parent->parent)
    for (int i = 0; i < parent->childCount && parent->children[i] != node; i++) {
      int l = nodeLength(parent->children[i], refSeq, clientId);
      total += l == UNDEF_LEN ? 0 : l;
    }
  return total;
}

// posFromRelativePos (mergeTree.ts:1371-1395)
int MergeTree::posFromRelativePos(const JVal& rel, int refSeq, int clientId) {
  if (rel.t != JVal::Obj) return -1;
  auto key = markerIdKey(obj_get(rel.obj, u"id"));
  if (!key) return -1;
  auto it = idToSegment.find(*key);
  if (it == idToSegment.end()) return -1;
  Seg* marker = it->second;
  int pos = getPosition(marker, refSeq, clientId);
  const JVal* before = obj_get(rel.obj, u"before");
  const JVal* offset = obj_get(rel.obj, u"offset");
  if (offset && offset->t != JVal::Undef && offset->t != JVal::Null &&
      (offset->t != JVal::Num || offset->num != (double)(int)offset->num))
    fail_unsupported("non-integer relative position offset");
  const int off = offset && offset->t == JVal::Num ? (int)offset->num : 0;
  if (js_falsy(before)) pos += marker->cachedLength + off;
  else pos -= off;
  return pos;
}

// nodeUpdateLengthNewStructure (mergeTree.ts:2188-2194)
void MergeTree::nodeUpdateLengthNewStructure(Block* b, bool recur) {
  blockUpdate(b);
  if (window.collaborating) b->partial = combine(b, recur);
}

// blockUpdateLength (mergeTree.ts:2436-2454)
// addToPendingList (mergeTree.ts:1324-1357): one group per local op, enqueued on each of its segments
SegGroup* MergeTree::addToPendingList(Seg* s, SegGroup* g, int localSeq) {
  if (!g) {
    groupPool.emplace_back(new SegGroup());
    g = groupPool.back().get();
    g->localSeq = localSeq;
    g->refSeq = window.currentSeq;
    pendingSegments.push_back(g);
  }
  g->segments.push_back(s);
  s->groups.push_back(g);
  return g;
}

// ackPendingSegment (mergeTree.ts:1283-1322) with BaseSegment.ack (mergeTreeNodes.ts:439-480)
void MergeTree::ackPendingSegment(int opType, const JObj* props, int seq, bool rewrite) {
  SegGroup* g = nullptr;
  if (!pendingSegments.empty()) {
    g = pendingSegments.front();
    pendingSegments.pop_front();
  }
  std::vector<Block*> nodesToUpdate;
  bool overwrite = false;
  if (g) {
    for (Seg* s : g->segments) {
      if (s->groups.empty() || s->groups.front() != g) fail_assert("0x043", "On ack, unexpected segmentGroup!");
      s->groups.erase(s->groups.begin());
      bool overlapping = false;
      switch (opType) {
        case 2:  // PropertiesManager.ackPendingProperties (segmentPropertiesManager.ts:31-58)
          if (!s->hasPropManager) fail_assert("0x044", "On annotate ack, missing segment property manager!");
          if (rewrite) s->pendingRewrite--;  // decrementPendingCounts (segmentPropertiesManager.ts:36-58)
          if (props)
            for (auto& kv : *props) {
              if (rewrite && kv.second.t == JVal::Null) continue;
              auto it = s->pendingKeys.find(kv.first);
              if (it == s->pendingKeys.end()) continue;
              if (it->second <= 0) fail_assert("0x05c", "Trying to update more annotate props than do exist!");
              if (--it->second == 0) s->pendingKeys.erase(it);
            }
          break;
        case 0:
          if (s->seq != UnassignedSeq) fail_assert("0x045", "On insert, seq number already assigned!");
          s->seq = seq;
          s->localSeq = INT32_MIN;
          break;
        case 1:
          if (!s->removed) fail_assert("0x046", "On remove ack, missing removal info!");
          s->localRemovedSeq = INT32_MIN;
          if (s->removedSeq == UnassignedSeq) s->removedSeq = seq;
          else overlapping = true;
          break;
        default:
          throw OracleError(-8, "unrecognized operation type in ack");
      }
      overwrite = overlapping || overwrite;
      addToLRUSet(s, seq);
      if (std::find(nodesToUpdate.begin(), nodesToUpdate.end(), s->parent) == nodesToUpdate.end())
        nodesToUpdate.push_back(s->parent);
    }
    for (Block* b : nodesToUpdate) blockUpdatePathLengths(b, seq, window.clientId, overwrite);
  }
  zamboniSegments();
}

void MergeTree::blockUpdateLength(Block* b, int seq, int clientId) {
  blockUpdate(b);
  if (window.collaborating && seq != UnassignedSeq && seq != TreeMaintenanceSeq) {
    if (b->partial && clientId != NonCollabClient) plUpdate(*b->partial, b, seq, clientId);
    else b->partial = combine(b, false);
  }
}

// blockUpdatePathLengths (mergeTree.ts:2419-2434)
void MergeTree::blockUpdatePathLengths(Block* b, int seq, int clientId, bool newStructure) {
  while (b) {
    if (newStructure) nodeUpdateLengthNewStructure(b);
    else blockUpdateLength(b, seq, clientId);
    b = b->parent;
  }
}

// ---------------------------------------------------------------- partial lengths construction
void MergeTree::plInsertSegment(PartialLengths& pl, Seg* s, bool removal) {  // partialLengths.ts:444-541
  // an unacked insert / removal goes to unsequencedRecords, which only local-perspective queries with a
  // localSeq need (computeLocalPartials); the observer-side restatement does not keep them
  if ((!removal && s->seq == UnassignedSeq) || (removal && s->removedSeq == UnassignedSeq)) return;
  int seq = s->seq;
  int segLen = s->cachedLength;
  int clientId = s->clientId;
  const std::vector<int>* overlap = nullptr;
  if (removal) {
    seq = s->removedSeq;
    segLen = -segLen;
    clientId = s->removedClientIds[0];
    if (s->removedClientIds.size() > 1) overlap = &s->removedClientIds;
  }
  PSL* firstGte = pl.partialLengths.firstGte(seq);
  if (firstGte && firstGte->seq == seq) {
    firstGte->seglen += segLen;
    if (overlap) {  // accumulateRemoveClientOverlap (partialLengths.ts:405-425)
      if (firstGte->overlap) {
        for (int c : *overlap) (*firstGte->overlap)[c] += segLen;
      } else {
        firstGte->overlap = std::make_shared<std::map<int, int>>();
        for (int c : *overlap) (*firstGte->overlap)[c] = segLen;
      }
    }
  } else {
    PSL e;
    e.seq = seq;
    e.clientId = clientId;
    e.len = 0;
    e.seglen = segLen;
    if (overlap) {
      e.overlap = std::make_shared<std::map<int, int>>();
      for (int c : *overlap) (*e.overlap)[c] = segLen;  // getOverlapClients: put overwrites
    }
    pl.partialLengths.addOrUpdate(e);
  }
}

std::unique_ptr<PartialLengths> MergeTree::fromLeaves(Block* b) {  // partialLengths.ts:344-403
  auto pl = std::make_unique<PartialLengths>();
  pl->minSeq = window.minSeq;
  pl->segmentCount = b->childCount;
  auto seqLTE = [&](int seq) { return seq != UnassignedSeq && seq <= window.minSeq; };
  for (int i = 0; i < b->childCount; i++) {
    Node* c = b->children[i];
    if (!c->leaf) continue;
    Seg* s = static_cast<Seg*>(c);
    if (seqLTE(s->seq)) pl->minLength += s->cachedLength;
    else plInsertSegment(*pl, s, false);
    if (s->removed && seqLTE(s->removedSeq)) pl->minLength -= s->cachedLength;
    else if (s->removed) plInsertSegment(*pl, s, true);
  }
  int prevLen = 0;
  for (auto& p : pl->partialLengths.items) {
    p.len = prevLen + p.seglen;
    prevLen = p.len;
    pl->addClientSeqNumberFromPartial(p);
  }
  pl->hmin = pl->minLength;
  return pl;
}

std::unique_ptr<PartialLengths> MergeTree::combine(Block* b, bool recur) {  // partialLengths.ts:256-338
  auto leafPL = fromLeaves(b);
  bool hasInternal = false;
  std::vector<PartialLengths*> childPartials;
  for (int i = 0; i < b->childCount; i++) {
    Node* c = b->children[i];
    if (!c->leaf) {
      hasInternal = true;
      Block* cb = static_cast<Block*>(c);
      if (recur) cb->partial = combine(cb, true);
      childPartials.push_back(cb->partial.get());
    }
  }
  std::unique_ptr<PartialLengths> combined;
  if (hasInternal) {
    combined = std::make_unique<PartialLengths>();
    combined->minSeq = window.minSeq;
    if (!leafPL->partialLengths.items.empty()) childPartials.push_back(leafPL.get());
    std::vector<const std::vector<PSL>*> lists;
    for (auto* cp : childPartials) {
      combined->segmentCount += cp->segmentCount;
      combined->minLength += cp->minLength;
      lists.push_back(&cp->partialLengths.items);
      if (defcheck()) {  // (only the children's minLength shortfalls survive the rebuild)
        combined->hmin += cp->hmin;
        for (auto& d : cp->defs)
          if (d.kind == 3) combined->defs.push_back(d);
      }
    }
    // mergePartialLengths + mergeSortedListsBySeq (partialLengths.ts:1013-1060)
    std::vector<size_t> next(lists.size(), 0);
    while (true) {
      long best = -1;
      for (size_t i = 0; i < lists.size(); i++) {
        if (next[i] < lists[i]->size()) {
          if (best < 0 || (*lists[i])[next[i]].seq < (*lists[best])[next[best]].seq) best = (long)i;
        }
      }
      if (best < 0) break;
      PSL item = (*lists[best])[next[best]++];
      if (item.overlap) item.overlap = std::make_shared<std::map<int, int>>(*item.overlap);
      combined->partialLengths.addOrUpdate(item);
    }
    for (auto& p : combined->partialLengths.items) combined->addClientSeqNumberFromPartial(p);
  } else {
    combined = std::move(leafPL);
  }
  combined->zamboni(window);
  if (defcheck()) combined->checkDefs("combine");
  return combined;
}

void MergeTree::plUpdate(PartialLengths& pl, Block* node, int seq, int clientId) {  // partialLengths.ts:636-686
  if (node != root && !pl.partialLengths.items.empty() && pl.partialLengths.items.back().seq > seq) counters.staleUpdates++;
  int seqSeglen = 0;
  int segCount = 0;
  for (int i = 0; i < node->childCount; i++) {
    Node* c = node->children[i];
    if (!c->leaf) {
      Block* cb = static_cast<Block*>(c);
      PSL* leq = cb->partial->partialLengths.latestLeq(seq);
      if (leq && leq->seq == seq) seqSeglen += leq->seglen;
      segCount += cb->partial->segmentCount;
    } else {
      Seg* s = static_cast<Seg*>(c);
      if (s->seq == seq) {
        if (!(s->removed && s->removedSeq == seq)) seqSeglen += s->cachedLength;
      } else if (s->removed && s->removedSeq == seq) {
        seqSeglen -= s->cachedLength;
      }
      segCount++;
    }
  }
  pl.segmentCount = segCount;
  if (defcheck()) {
    // addSeq over an entry at seq: the deficits that began there begin at the next entry; the later entries are
    // short by the seglen change
    auto model = [&](PSLSet& st, int kind, int c) {
      auto [exists, idx] = st.find(seq);
      if (!exists) return;
      const int t1 = idx + 1 < st.items.size() ? st.items[idx + 1].seq : INT32_MAX;
      for (auto& d : pl.defs)
        if (d.kind == kind && (kind == 1 || d.c == c) && d.t == seq) d.t = t1;
      pl.defs.erase(std::remove_if(pl.defs.begin(), pl.defs.end(), [](const PartialLengths::Def& d) { return d.t == INT32_MAX; }),
                    pl.defs.end());
      const int dd = seqSeglen - st.items[idx].seglen;
      if (t1 != INT32_MAX && dd) pl.defs.push_back({kind, t1, dd, c});
      if (getenv("MTO_DEFTRACE"))
        fprintf(stderr, "update block %d seq %d client %d kind %d: t1 %d d %d (defs %zu)\n", node->id, seq, clientId, kind,
                t1 == INT32_MAX ? -1 : t1, dd, pl.defs.size());
    };
    model(pl.partialLengths, 1, 0);
    model(pl.cli(clientId), 2, clientId);
  }
  const int d1 = addSeq(pl.partialLengths, seq, seqSeglen, clientId);
  const int d2 = addSeq(pl.cli(clientId), seq, seqSeglen, 0);
  if (node != root && (d1 || d2)) counters.staleDeficits++;
  if (defcheck()) pl.checkDefs("update");
  pl.zamboni(window);
}

// ---------------------------------------------------------------- nodeMap / depthFirstNodeWalk
// nodeMap (mergeTree.ts:2531-2582) over depthFirstNodeWalk (mergeTreeNodeWalk.ts:35-115)
template <class Leaf, class Post>
void MergeTree::nodeMap(int refSeq, int clientId, Leaf&& leaf, Post&& post, int start, int end) {
  int endPos = end;
  if (endPos == start) return;
  int pos = 0;
  enum { CONTINUE = 0, EXIT = 1, SKIP = 2 };
  auto down = [&](Node* node) -> int {
    if (endPos <= pos) return EXIT;
    int len = nodeLength(node, refSeq, clientId);
    if (len == UNDEF_LEN || len == 0) return SKIP;
    int nextPos = pos + len;
    if (start >= nextPos) {
      pos = nextPos;
      return SKIP;
    }
    if (node->leaf) {
      if (!leaf(static_cast<Seg*>(node), pos, start - pos, endPos - pos)) return EXIT;
      pos = nextPos;
    }
    return CONTINUE;
  };
  Block* block = root;
  int childCount = block->childCount;
  Node* startNode = block->childCount > 0 ? block->children[0] : nullptr;
  while (true) {
    int blockResult = CONTINUE;
    while (startNode && !startNode->leaf) {
      block = static_cast<Block*>(startNode);
      childCount = block->childCount;
      blockResult = down(block);
      startNode = blockResult == CONTINUE ? (childCount > 0 ? block->children[0] : nullptr) : nullptr;
    }
    bool exitFlag = blockResult == EXIT;
    if (startNode) {
      for (int i = startNode->index; i != -1 && i != childCount; i++) {
        if (down(block->children[i]) == EXIT) {
          exitFlag = true;
          break;
        }
      }
    }
    int nextIndex = -1;
    do {
      if (blockResult == CONTINUE) post(block);
      else blockResult = CONTINUE;
      if (block->parent == nullptr) return;
      startNode = block;
      block = block->parent;
      childCount = block->childCount;
      nextIndex = startNode->index + 1;
    } while (exitFlag || nextIndex == -1 || nextIndex == childCount);
    startNode = block->children[nextIndex];
  }
}

// markRangeRemoved (mergeTree.ts:1960-2052), remote (sequenced) ops only
void MergeTree::markRangeRemoved(int start, int end, int refSeq, int clientId, int seq) {
  bool overwrite = false;
  ensureIntervalBoundary(start, refSeq, clientId);
  ensureIntervalBoundary(end, refSeq, clientId);
  std::vector<Seg*> removed;  // removedSegments (mergeTree.ts:1973): fresh removals only
  const int localSeq = seq == UnassignedSeq ? ++window.localSeq : INT32_MIN;  // mergeTree.ts:1973-1974
  SegGroup* group = nullptr;
  auto markRemoved = [&](Seg* s, int, int, int) -> bool {
    if (!s->removed) removed.push_back(s);
    if (s->removed) {
      overwrite = true;
      if (s->removedSeq == UnassignedSeq) {
        // removed locally, but someone else removed it first: they go to the head (mergeTree.ts:1980-1988)
        s->removedClientIds.insert(s->removedClientIds.begin(), clientId);
        s->removedSeq = seq;
      } else {
        s->removedClientIds.push_back(clientId);
      }
    } else {
      s->removed = true;
      s->removedClientIds = {clientId};
      s->removedSeq = seq;
      s->localRemovedSeq = localSeq;
    }
    counters.segsTouched += 1;
    if (window.collaborating) {
      if (s->removedSeq == UnassignedSeq && clientId == window.clientId) group = addToPendingList(s, group, localSeq);
      else addToLRUSet(s, seq);
    }
    return true;
  };
  auto post = [&](Block* b) {
    if (overwrite) nodeUpdateLengthNewStructure(b);
    else blockUpdateLength(b, seq, clientId);
  };
  nodeMap(refSeq, clientId, markRemoved, post, start, end);
  if (onDelta && !removed.empty()) onDelta(1, removed, nullptr);
  if (window.collaborating && seq != UnassignedSeq) zamboniSegments();
}

// PropertiesManager.addProperties (segmentPropertiesManager.ts:60-157) combined with
// BaseSegment.addProperties: a local op (seq Unassigned) while collaborating counts its keys as pending;
// a sequenced remote op leaves the keys with pending local updates alone (shouldModifyKey), and leaves a
// segment with a pending local rewrite (pendingRewriteCount > 0) alone altogether (:75-82).
Comb parse_comb(const JVal* comb) {
  Comb c;
  if (!comb || comb->t != JVal::Obj) return c;
  const JVal* name = obj_get(comb->obj, u"name");
  if (name && name->t == JVal::Str && name->str == u"rewrite") {
    c.kind = Comb::Rewrite;
  } else if (name && name->t == JVal::Str && name->str == u"incr") {
    c.kind = Comb::Incr;
    if (const JVal* d = obj_get(comb->obj, u"defaultValue")) c.defaultValue = *d;
    if (const JVal* m = obj_get(comb->obj, u"minValue")) c.minValue = *m;
  } else if (name && name->t == JVal::Str && name->str == u"consensus") {
    c.kind = Comb::Consensus;
    if (const JVal* d = obj_get(comb->obj, u"defaultValue")) c.defaultValue = *d;
  } else {
    fail_unsupported("combiningOp other than rewrite / incr / consensus");
  }
  return c;
}
// combine(combiningOp, previousValue, undefined, seq) for "consensus" (properties.ts:46-62), sequenced ops:
// no previous value and no defaultValue gives a fresh {value: undefined, seq} (JSON {"seq":seq}); an object
// whose seq is -1 gets seq (in place: the op's defaultValue object is shared by the op's segments alone, so a
// copy equals it; a previous value may be shared with other segments by split clones -- not restated); any
// other value stays.  A null defaultValue makes the reference throw reading its seq.
// `complete`: the ack of this client's own annotateMarkerNotifyConsensus (client.ts:1050-1058), whose marker's
// value object (its own, made by the local op) is completed in place -- not a shared object
static JVal combine_consensus(const Comb& c, const JVal* prev, int seq, bool complete = false) {
  const bool fromPrev = prev && prev->t != JVal::Undef;
  JVal cur = fromPrev ? *prev : c.defaultValue;
  if (cur.t == JVal::Undef) {
    JVal cv;
    cv.t = JVal::Obj;
    obj_set(cv.obj, u"value", JVal::undef());
    obj_set(cv.obj, u"seq", JVal::number(seq));
    return cv;
  }
  if (cur.t == JVal::Null)  // (cv.seq of null: the reference's own failure, as an assert is)
    throw OracleError(-4, "TypeError: Cannot read properties of null (reading 'seq') (properties.ts:56-57: a "
                          "consensus annotate with a null defaultValue over a segment lacking the key)");
  const JVal* cs = cur.t == JVal::Obj ? obj_get(cur.obj, u"seq") : nullptr;
  if (cs && cs->t == JVal::Num && cs->num == -1) {
    if (seq == UnassignedSeq) return cur;  // (a local op sets seq -1 to -1)
    if (fromPrev && !complete)
      fail_unsupported("consensus over a property value object whose seq is -1 (mutates a shared object)");
    obj_set(cur.obj, u"seq", JVal::number(seq));
  }
  return cur;
}
// String(v) of a JSON value (ECMA-262 ToString; objects through Object.prototype.toString, arrays through
// Array.prototype.join(","), whose undefined / null elements become "")
static u16str js_to_string(const JVal& v) {
  switch (v.t) {
    case JVal::Undef: return u"undefined";
    case JVal::Null: return u"null";
    case JVal::False: return u"false";
    case JVal::True: return u"true";
    case JVal::Num: {
      if (std::isnan(v.num)) return u"NaN";
      if (std::isinf(v.num)) return v.num < 0 ? u"-Infinity" : u"Infinity";
      const std::string n = js_number_to_string(v.num);
      return u16str(n.begin(), n.end());
    }
    case JVal::Str: return v.str;
    case JVal::Obj: return u"[object Object]";
    case JVal::Arr: {
      u16str o;
      for (size_t i = 0; i < v.arr.size(); i++) {
        if (i) o += u",";
        if (v.arr[i].t != JVal::Undef && v.arr[i].t != JVal::Null) o += js_to_string(v.arr[i]);
      }
      return o;
    }
  }
  return u"";
}
// combine(combiningOp, previousValue, undefined, seq) for "incr" (properties.ts:24-69)
static JVal combine_incr(const Comb& c, const JVal* prev) {
  JVal cur = prev ? *prev : JVal::undef();
  if (cur.t == JVal::Undef) cur = c.defaultValue;
  switch (cur.t) {  // _currentValue += undefined
    case JVal::Str: cur.str += u"undefined"; break;
    case JVal::Undef:
    case JVal::Null:
    case JVal::False:
    case JVal::True:
    case JVal::Num: cur = JVal::number(std::nan("")); break;
    default: {  // an object or array: ToPrimitive is its string form, then string concatenation
      JVal r;
      r.t = JVal::Str;
      r.str = js_to_string(cur) + u"undefined";
      cur = std::move(r);
    }
  }
  if (!js_falsy(&c.minValue)) {  // if (_currentValue < minValue) _currentValue = minValue
    // NaN < x is false; "...undefined" < a number or boolean compares NaN; against a string, object or array
    // minValue (ToPrimitive: its string form) two strings compare by UTF-16 code units
    const bool strMin = c.minValue.t == JVal::Str || c.minValue.t == JVal::Obj || c.minValue.t == JVal::Arr;
    if (cur.t == JVal::Str && strMin && cur.str < js_to_string(c.minValue)) cur = c.minValue;
  }
  return cur;
}
// deltaKeys (when given) receives the keys of the returned propertyDeltas, in their insertion order
static void applyProps(Seg* s, const JObj& newProps, const Comb& comb, int seq = UniversalSeq, bool collaborating = false,
                       std::vector<u16str>* deltaKeys = nullptr, bool complete = false) {
  s->hasPropManager = true;
  if (!s->props) s->props = JObj();
  if (collaborating && s->pendingRewrite > 0 && seq != UnassignedSeq && seq != UniversalSeq) return;
  auto addDelta = [&](const u16str& k) {
    if (deltaKeys && std::find(deltaKeys->begin(), deltaKeys->end(), k) == deltaKeys->end()) deltaKeys->push_back(k);
  };
  JObj& old = *s->props;
  const bool rewrite = comb.kind == Comb::Rewrite, combining = comb.kind == Comb::Incr || comb.kind == Comb::Consensus;
  auto shouldModify = [&](const u16str& k) {
    return seq == UnassignedSeq || seq == UniversalSeq || s->pendingKeys.find(k) == s->pendingKeys.end() || combining;
  };
  if (rewrite) {
    if (collaborating && seq == UnassignedSeq) s->pendingRewrite++;
    std::vector<u16str> keys;
    for (auto& kv : old) keys.push_back(kv.first);
    for (auto& k : keys) {
      const JVal* nv = obj_get(newProps, k);
      if (js_falsy(nv) && shouldModify(k)) {
        addDelta(k);
        obj_del(old, k);
      }
    }
  }
  for (auto& kv : newProps) {
    if (collaborating) {
      if (seq == UnassignedSeq) {
        if (rewrite && kv.second.t == JVal::Null) continue;  // (a rewrite's null keys are not counted)
        s->pendingKeys[kv.first]++;
      } else if (!shouldModify(kv.first)) {
        continue;
      }
    }
    addDelta(kv.first);
    if (comb.kind == Comb::Consensus) obj_set(old, kv.first, combine_consensus(comb, obj_get(old, kv.first), seq, complete));
    else if (combining) obj_set(old, kv.first, combine_incr(comb, obj_get(old, kv.first)));
    else if (kv.second.t == JVal::Null) obj_del(old, kv.first);
    else obj_set(old, kv.first, kv.second);
  }
}

// annotateRange (mergeTree.ts:1895-1958)
void MergeTree::annotateRange(int start, int end, const JObj& props, const Comb& comb, int refSeq, int clientId, int seq) {
  ensureIntervalBoundary(start, refSeq, clientId);
  ensureIntervalBoundary(end, refSeq, clientId);
  std::vector<Seg*> annotated;
  const int localSeq = seq == UnassignedSeq ? ++window.localSeq : INT32_MIN;  // mergeTree.ts:1909-1910
  SegGroup* group = nullptr;
  // assert 0x5ad (mergeTree.ts:1912-1918): an annotate naming markerId must carry the marker's own id
  // (JS ===: primitives by value; an object or array value is a fresh object, never equal)
  const JVal* opId = obj_get(props, u"markerId");
  auto same_id = [](const JVal* a, const JVal* b) {
    const JVal::T ta = a ? a->t : JVal::Undef, tb = b ? b->t : JVal::Undef;
    if (ta != tb || ta == JVal::Obj || ta == JVal::Arr) return false;
    if (ta == JVal::Num) return a->num == b->num;
    if (ta == JVal::Str) return a->str == b->str;
    return true;
  };
  std::vector<std::vector<u16str>> deltaKeys;  // each annotated segment's propertyDeltas keys
  auto annotate = [&](Seg* s, int, int, int) -> bool {
    if (opId && s->isMarker && !same_id(opId, s->props ? obj_get(*s->props, u"markerId") : nullptr))
      fail_assert("0x5ad", "Cannot change the markerId of an existing marker");
    annotated.push_back(s);
    if (onDelta) deltaKeys.emplace_back();
    applyProps(s, props, comb, seq, window.collaborating, onDelta ? &deltaKeys.back() : nullptr);
    counters.segsTouched += 1;
    if (window.collaborating) {
      if (seq == UnassignedSeq) group = addToPendingList(s, group, localSeq);
      else addToLRUSet(s, seq);
    }
    return true;
  };
  auto post = [&](Block*) {};
  nodeMap(refSeq, clientId, annotate, post, start, end);
  if (onDelta && !annotated.empty()) {
    onDelta(2, annotated, &deltaKeys);
  }
  if (window.collaborating && seq != UnassignedSeq) zamboniSegments();
}

// ---------------------------------------------------------------- zamboni (MT/zamboni.ts)
static bool canAppend(const Seg* a, const Seg* b) {  // TextSegment.canAppend (textSegment.ts:71-78)
  if (a->perm)  // PermutationSegment.canAppend (permutationvector.ts:117-123): contiguous handles
    return a->start == HandleUnallocated ? b->start == HandleUnallocated : b->start == a->start + a->cachedLength;
  if (a->isMarker || b->isMarker) return false;
  if (!a->text.empty() && a->text.back() == u'\n') return false;
  return a->cachedLength <= TextSegmentGranularity || b->cachedLength <= TextSegmentGranularity;
}
// matchProperties(a.properties, b.properties) (properties.ts:71-96) on two property maps
static bool matchSegProps(const Seg* a, const Seg* b) {
  const JObj* pa = a->props ? &*a->props : nullptr;
  const JObj* pb = b->props ? &*b->props : nullptr;
  const size_t na = pa ? pa->size() : 0, nb = pb ? pb->size() : 0;
  if (na != nb) return false;
  for (size_t i = 0; i < na; i++) {
    const JVal* bv = obj_get(*pb, (*pa)[i].first);
    if (!bv || bv->t == JVal::Undef) return false;
    const JVal* av = &(*pa)[i].second;
    if (bv->t == JVal::Obj || bv->t == JVal::Arr || bv->t == JVal::Null) {
      if (!match_properties(av, bv)) return false;
    } else if (!js_strict_equal(bv, av)) {
      return false;
    }
  }
  return true;
}

void MergeTree::scourNode(Block* node, std::vector<Node*>& hold) {  // zamboni.ts:122-193
  Seg* prev = nullptr;
  for (int k = 0; k < node->childCount; k++) {
    Node* c = node->children[k];
    if (c->leaf) {
      Seg* s = static_cast<Seg*>(c);
      if (!s->groups.empty()) {  // a segment with pending local ops stays as it is
        hold.push_back(s);
        prev = nullptr;
      } else if (s->removed) {
        if (s->removedSeq > window.minSeq) {
          hold.push_back(s);
        } else {
          if (onUnlink) onUnlink(s);  // MergeTreeMaintenanceType.UNLINK
          s->parent = nullptr;        // unlink
        }
        prev = nullptr;
      } else {
        if (s->seq <= window.minSeq) {
          int ln = localNetLength(s);
          bool ok = prev && canAppend(prev, s) && matchSegProps(prev, s) && (ln == UNDEF_LEN ? 0 : ln) > 0;
          if (ok) {
            prev->text += s->text;  // TextSegment.append
            prev->cachedLength += s->cachedLength;
            s->parent = nullptr;
          } else {
            hold.push_back(s);
            prev = (ln == UNDEF_LEN ? 0 : ln) > 0 ? s : nullptr;
          }
        } else {
          hold.push_back(s);
          prev = nullptr;
        }
      }
    } else {
      hold.push_back(c);
      prev = nullptr;
    }
  }
}

void MergeTree::packParent(Block* parent) {  // zamboni.ts:63-120
  std::vector<Node*> hold;
  for (int i = 0; i < parent->childCount; i++) {
    Block* cb = static_cast<Block*>(parent->children[i]);
    scourNode(cb, hold);
    cb->parent = nullptr;
  }
  if (!hold.empty()) {
    int total = (int)hold.size();
    int half = MaxNodesInBlock / 2;
    int childCount = std::min(MaxNodesInBlock - 1, total / half);
    if (childCount < 1) childCount = 1;
    int base = total / childCount;
    int rem = total % childCount;
    std::vector<Block*> packed;
    int packedCount = 0;
    for (int ni = 0; ni < childCount; ni++) {
      int n = base;
      if (rem > 0) { n++; rem--; }
      Block* pb = makeBlock(n);
      if ((int)pb->children.size() < n) pb->children.resize(n, nullptr);
      for (int j = 0; j < n; j++) pb->assignChild(hold[packedCount++], j);
      pb->parent = parent;
      packed.push_back(pb);
      nodeUpdateLengthNewStructure(pb);
    }
    parent->children.assign(std::max(MaxNodesInBlock, childCount), nullptr);
    for (int j = 0; j < childCount; j++) parent->assignChild(packed[j], j);
    parent->childCount = childCount;
  } else {
    parent->children.assign(MaxNodesInBlock, nullptr);
    parent->childCount = 0;
  }
  if (parent->childCount < MaxNodesInBlock / 2 && parent->parent) {
    packParent(parent->parent);
  } else {
    blockUpdatePathLengths(parent, UnassignedSeq, -1, true);
  }
}

void MergeTree::zamboniSegments() {  // zamboni.ts:19-60
  if (!window.collaborating) return;
  for (int i = 0; i < ZamboniSegmentsMax; i++) {
    if (heap.size() <= 1) break;
    LRU top = heap[1];
    if (top.maxSeq > window.minSeq) break;
    top = heapGet();
    Seg* s = top.seg;
    if (s->parent && s->parent->needsScour != 0) {
      Block* block = s->parent;
      std::vector<Node*> copy;
      scourNode(block, copy);
      block->needsScour = 0;
      int newCount = (int)copy.size();
      if (newCount < block->childCount) {
        block->childCount = newCount;
        block->children.assign(std::max(MaxNodesInBlock, newCount), nullptr);
        for (int j = 0; j < newCount; j++) block->assignChild(copy[j], j);
        if (block->childCount < MaxNodesInBlock / 2 && block->parent) {
          packParent(block->parent);
        } else {
          blockUpdatePathLengths(block, UnassignedSeq, -1, true);
        }
      }
    }
  }
}

template <class F>
void MergeTree::walkAllSegments(F&& f) {
  std::function<void(Block*)> rec = [&](Block* b) {
    for (int i = 0; i < b->childCount; i++) {
      Node* c = b->children[i];
      if (c->leaf) f(static_cast<Seg*>(c));
      else rec(static_cast<Block*>(c));
    }
  };
  rec(root);
}

// getText (MergeTreeTextHelper.ts:20-81) at (currentSeq, local client): visible text segments
u16str MergeTree::getText() {
  u16str out;
  walkAllSegments([&](Seg* s) {
    int l = nodeLength(s, window.currentSeq, window.clientId);
    if (l != UNDEF_LEN && l > 0 && !s->isMarker) out += s->text;
  });
  return out;
}

// =====================================================================================
// Doc (Client)
// =====================================================================================
int Doc::getOrAddShortClientId(const std::string& id) {  // client.ts:673-688
  auto it = longToShort.find(id);
  if (it != longToShort.end()) return it->second;
  int s = (int)longIds.size();
  longToShort[id] = s;
  longIds.push_back(id);
  return s;
}
std::string Doc::getLongClientId(int s) const {
  return s >= 0 ? longIds.at(s) : std::string("original");
}

void Doc::startOrUpdateCollaboration(const std::string& id, int minSeq, int curSeq) {  // client.ts:1133-1146
  if (!longClientId) {
    longClientId = id;
    int s = getOrAddShortClientId(id);
    mt.startCollaboration(s, minSeq, curSeq);
  } else {
    int old = longToShort.at(*longClientId);
    longClientId = id;
    longToShort[id] = old;
    longIds[old] = id;
  }
}

void Doc::updateSeqNumbers(int min, int seq) {  // client.ts:877-887
  if (!(mt.window.currentSeq <= seq)) fail_assert("0x038", "Incoming op sequence# < local collabWindow's currentSequence#");
  mt.window.currentSeq = seq;
  if (!(min <= seq)) fail_assert("0x039", "Incoming op sequence# < minSequence#");
  mt.setMinSeq(min);
}

// Props of a segment spec: TextSegment.make(text, props) -> addProperties (textSegment.ts:35-40)
JObj propsFromSpec(const JVal* spec) {
  JObj o;
  if (!spec || spec->t != JVal::Obj) return o;
  for (auto& kv : spec->obj)
    if (kv.second.t != JVal::Null) obj_set(o, kv.first, kv.second);
  return o;
}

static Seg* makeSegFromSpec(MergeTree& mt, const JVal& spec) {  // testClient.ts:38-50 specToSegment
  if (spec.t == JVal::Arr) {  // PermutationSegment.fromJSONObject([length, start]) (permutationvector.ts:45-48)
    if (spec.arr.size() < 2 || spec.arr[0].t != JVal::Num) throw OracleError(-8, "bad PermutationSegment spec");
    Seg* s = mt.newSeg();
    s->perm = true;
    s->cachedLength = (int)spec.arr[0].num;
    s->start = spec.arr[1].t == JVal::Num ? (int)spec.arr[1].num : HandleUnallocated;
    return s;
  }
  if (spec.t == JVal::Str) {
    Seg* s = mt.newSeg();
    s->text = spec.str;
    s->cachedLength = (int)s->text.size();
    return s;
  }
  if (spec.t == JVal::Obj) {
    const JVal* text = obj_get(spec.obj, u"text");
    const JVal* props = obj_get(spec.obj, u"props");
    if (text) {
      if (text->t != JVal::Str) fail_unsupported("non-string text segment");
      Seg* s = mt.newSeg();
      s->text = text->str;
      s->cachedLength = (int)s->text.size();
      if (props && !js_falsy(props)) {
        s->hasPropManager = true;
        s->props = propsFromSpec(props);
      }
      return s;
    }
    const JVal* marker = obj_get(spec.obj, u"marker");
    if (marker) {
      Seg* s = mt.newSeg();
      s->isMarker = true;
      s->cachedLength = 1;
      const JVal* rt = marker->t == JVal::Obj ? obj_get(marker->obj, u"refType") : nullptr;
      s->refType = (rt && rt->t == JVal::Num) ? (int)rt->num : -1;
      if (props && !js_falsy(props)) {
        s->hasPropManager = true;
        s->props = propsFromSpec(props);
      }
      return s;
    }
  }
  throw OracleError(-8, "Unrecognized IJSONSegment type");
}

// getValidOpRange (client.ts:527-547): `pos1` / `pos2` if present, else posFromRelativePos of
// `relativePos1` / `relativePos2` in the op's (refSeq, clientId) view
static int getPos(MergeTree& mt, const JVal& op, const char16_t* key, const char16_t* relKey, int refSeq, int client) {
  const JVal* p = obj_get(op.obj, key);
  if (p && p->t == JVal::Num) return (int)p->num;
  const JVal* rel = obj_get(op.obj, relKey);
  if (rel && !js_falsy(rel)) {
    const int pos = mt.posFromRelativePos(*rel, refSeq, client);
    if (pos < 0) fail_unsupported("relative position names no marker of the document");
    return pos;
  }
  fail_unsupported("missing position");
}

// applyRemoteOp (client.ts:802-829) for one decoded delta op
void Doc::applyRemoteDelta(const JVal& op, int client, int refSeq, int seq) {
  const JVal* type = obj_get(op.obj, u"type");
  int t = type && type->t == JVal::Num ? (int)type->num : -1;
  mt.counters.ops += (t >= 0 && t <= 2) ? 1 : 0;
  switch (t) {
    case 0: {  // applyInsertOp (client.ts:489-524)
      int pos = getPos(mt, op, u"pos1", u"relativePos1", refSeq, client);
      const JVal* spec = obj_get(op.obj, u"seg");
      if (js_falsy(spec)) return;
      Seg* s = makeSegFromSpec(mt, *spec);
      if (perm != s->perm) fail_unsupported(perm ? "non-permutation segment in a PermutationVector" : "PermutationSegment in a SharedString");
      // PermutationVector.onDelta (permutationvector.ts:346-357): a remote insert's handle allocation is
      // dropped; the reset happens before insertSegments' zamboni, so inserting unallocated is the same
      if (s->perm) s->start = HandleUnallocated;
      mt.insertSegments(pos, s, refSeq, client, seq);
      break;
    }
    case 1: {  // applyRemoveRangeOp (client.ts:430-455)
      int a = getPos(mt, op, u"pos1", u"relativePos1", refSeq, client);
      int b = getPos(mt, op, u"pos2", u"relativePos2", refSeq, client);
      mt.markRangeRemoved(a, b, refSeq, client, seq);
      break;
    }
    case 2: {  // applyAnnotateRangeOp (client.ts:457-487)
      int a = getPos(mt, op, u"pos1", u"relativePos1", refSeq, client);
      int b = getPos(mt, op, u"pos2", u"relativePos2", refSeq, client);
      const JVal* props = obj_get(op.obj, u"props");
      const Comb comb = parse_comb(obj_get(op.obj, u"combiningOp"));
      JObj p;
      if (props && props->t == JVal::Obj) p = props->obj;
      mt.annotateRange(a, b, p, comb, refSeq, client, seq);
      break;
    }
    case 3: {  // GROUP (client.ts:816-824)
      const JVal* ops = obj_get(op.obj, u"ops");
      if (ops && ops->t == JVal::Arr)
        for (auto& m : ops->arr) applyRemoteDelta(m, client, refSeq, seq);
      break;
    }
    default:
      break;
  }
}

// applyMsg (client.ts:858-875)
static JVal jop(std::initializer_list<std::pair<const char16_t*, JVal>> kv) {
  JVal o;
  o.t = JVal::Obj;
  for (auto& p : kv) o.obj.push_back({p.first, p.second});
  return o;
}
static JVal segJson(const Seg* s);

void Doc::processMinSequenceNumberChanged(int minSeq) {  // sequence.ts:737-748
  size_t i = 0;
  for (; i < messagesSinceMSNChange.size(); i++) {
    const JVal* sq = obj_get(messagesSinceMSNChange[i].obj, u"sequenceNumber");
    if (sq && sq->num > minSeq) break;
  }
  if (i) messagesSinceMSNChange.erase(messagesSinceMSNChange.begin(), messagesSinceMSNChange.begin() + (long)i);
}
std::string Doc::catchUpJson(int minSeq) {  // SharedSegmentSequence.summarizeCore (sequence.ts:676-692)
  processMinSequenceNumberChanged(minSeq);
  JVal arr;
  arr.t = JVal::Arr;
  for (JVal& m : messagesSinceMSNChange) {
    obj_set(m.obj, u"minimumSequenceNumber", JVal::number(minSeq));
    arr.arr.push_back(m);
  }
  return json_stringify(arr);
}

void Doc::applyMsg(const JVal& msg) {
  if (catchUp && msg.t == JVal::Obj) {
    // processMergeTreeMsg (sequence.ts:697-733): a message that did not see everything before it is
    // stored rewritten from its deltas (createOpsFromDelta, sequence.ts:120-172) at refSeq = seq - 1
    const JVal* type = obj_get(msg.obj, u"type");
    const JVal* sq = obj_get(msg.obj, u"sequenceNumber");
    const JVal* rs = obj_get(msg.obj, u"referenceSequenceNumber");
    const JVal* ms = obj_get(msg.obj, u"minimumSequenceNumber");
    if (type && type->t == JVal::Str && type->str == u"op" && sq && rs && ms) {
      const int seqN = (int)sq->num;
      const bool transform = (int)rs->num != seqN - 1;
      std::vector<JVal> ops;
      if (transform)
        mt.onDelta = [&](int op, const std::vector<Seg*>& segs, const std::vector<std::vector<u16str>>* keys) {
          std::vector<JVal> evOps;  // per event
          std::vector<std::pair<int, Seg*>> ranges;
          for (Seg* s : segs) ranges.push_back({mt.localPosition(s), s});
          for (size_t ri = 0; ri < ranges.size(); ri++) {
            const int position = ranges[ri].first;
            Seg* s = ranges[ri].second;
            if (op == 2) {  // props[key] = segment.properties?.[key] ?? null over the segment's delta keys
              JVal pv;
              pv.t = JVal::Obj;
              for (auto& k : (*keys)[ri]) {
                const JVal* cur = s->props ? obj_get(*s->props, k) : nullptr;
                pv.obj.push_back({k, cur && cur->t != JVal::Undef ? *cur : JVal::null()});
              }
              JVal* last = evOps.empty() ? nullptr : &evOps.back();
              const JVal* lp2 = last ? obj_get(last->obj, u"pos2") : nullptr;
              const JVal* lpr = last ? obj_get(last->obj, u"props") : nullptr;
              if (lp2 && lp2->t == JVal::Num && (int)lp2->num == position && match_properties(lpr, &pv)) {
                obj_set(last->obj, u"pos2", JVal::number(lp2->num + s->cachedLength));
              } else {
                evOps.push_back(jop({{u"pos1", JVal::number(position)}, {u"pos2", JVal::number(position + s->cachedLength)},
                                     {u"props", pv}, {u"type", JVal::number(2)}}));
              }
            } else if (op == 0) {
              evOps.push_back(jop({{u"pos1", JVal::number(position)}, {u"seg", segJson(s)}, {u"type", JVal::number(0)}}));
            } else {
              JVal* last = evOps.empty() ? nullptr : &evOps.back();
              const JVal* lp1 = last ? obj_get(last->obj, u"pos1") : nullptr;
              const JVal* lp2 = last ? obj_get(last->obj, u"pos2") : nullptr;
              if (lp1 && lp1->t == JVal::Num && (int)lp1->num == position) {
                obj_set(last->obj, u"pos2", JVal::number(lp2->num + s->cachedLength));
              } else {
                evOps.push_back(jop({{u"pos1", JVal::number(position)}, {u"pos2", JVal::number(position + s->cachedLength)},
                                     {u"type", JVal::number(1)}}));
              }
            }
          }
          for (auto& o : evOps) ops.push_back(std::move(o));
        };
      struct Reset {
        MergeTree& t;
        ~Reset() { t.onDelta = nullptr; }
      } reset{mt};
      applyMsgCore(msg);
      JVal stash = msg;
      if (transform) {
        obj_set(stash.obj, u"referenceSequenceNumber", JVal::number(seqN - 1));
        if (ops.size() == 1) {
          obj_set(stash.obj, u"contents", ops[0]);
        } else {
          JVal arr;
          arr.t = JVal::Arr;
          arr.arr = std::move(ops);
          obj_set(stash.obj, u"contents", jop({{u"ops", arr}, {u"type", JVal::number(3)}}));
        }
      }
      messagesSinceMSNChange.push_back(std::move(stash));
      if (messagesSinceMSNChange.size() > 20) {  // "Do GC every once in a while"
        const JVal* s20 = obj_get(messagesSinceMSNChange[20].obj, u"sequenceNumber");
        if (s20 && s20->num < ms->num) processMinSequenceNumberChanged((int)ms->num);
      }
      return;
    }
  }
  applyMsgCore(msg);
}

void Doc::applyMsgCore(const JVal& msg) {
  if (msg.t != JVal::Obj) throw OracleError(-8, "message is not an object");
  const JVal* cid = obj_get(msg.obj, u"clientId");
  if (!cid || cid->t != JVal::Str) fail_unsupported("message without string clientId");
  std::string longId = u16_to_utf8(cid->str);
  int client = getOrAddShortClientId(longId);
  auto num = [&](const char16_t* k) {
    const JVal* v = obj_get(msg.obj, k);
    if (!v || v->t != JVal::Num) throw OracleError(-8, "missing numeric field");
    return (int)v->num;
  };
  int seq = num(u"sequenceNumber");
  int refSeq = num(u"referenceSequenceNumber");
  int msn = num(u"minimumSequenceNumber");
  const JVal* type = obj_get(msg.obj, u"type");
  if (type && type->t == JVal::Str && type->str == u"op") {
    const JVal* contents = obj_get(msg.obj, u"contents");
    if (!contents || contents->t != JVal::Obj) throw OracleError(-8, "op without contents");
    if (longClientId && longId == *longClientId) {
      // Client.ackPendingSegment (client.ts:641-662): one MergeTree.ackPendingSegment per member op
      auto ackOne = [&](const JVal& op) {
        const JVal* t = obj_get(op.obj, u"type");
        const JVal* pr = obj_get(op.obj, u"props");
        const JVal* comb = obj_get(op.obj, u"combiningOp");
        const JVal* cname = comb && comb->t == JVal::Obj ? obj_get(comb->obj, u"name") : nullptr;
        const bool rw = cname && cname->t == JVal::Str && cname->str == u"rewrite";
        mt.ackPendingSegment(t && t->t == JVal::Num ? (int)t->num : -1, pr && pr->t == JVal::Obj ? &pr->obj : nullptr, seq, rw);
        // updateConsensusProperty (client.ts:1050-1058): the registered marker's values at the ack's seq
        if (t && t->t == JVal::Num && (int)t->num == 2 && cname && cname->t == JVal::Str && cname->str == u"consensus") {
          const JVal* r1 = obj_get(op.obj, u"relativePos1");
          auto key = r1 && r1->t == JVal::Obj ? MergeTree::markerIdKey(obj_get(r1->obj, u"id")) : std::nullopt;
          auto it = key ? pendingConsensus.find(*key) : pendingConsensus.end();
          if (it == pendingConsensus.end())
            fail_unsupported("consensus ack without annotateMarkerNotifyConsensus (the reference throws later)");
          applyProps(it->second, pr && pr->t == JVal::Obj ? pr->obj : JObj(), parse_comb(comb), seq, true, nullptr, true);
        }
      };
      const JVal* t = obj_get(contents->obj, u"type");
      if (t && t->t == JVal::Num && (int)t->num == 3) {
        const JVal* ops = obj_get(contents->obj, u"ops");
        if (ops && ops->t == JVal::Arr)
          for (auto& m : ops->arr) ackOne(m);
      } else {
        ackOne(*contents);
      }
    } else {
      applyRemoteDelta(*contents, client, refSeq, seq);
    }
  }
  updateSeqNumbers(msn, seq);
}

void Doc::applyRecord(const Record& r, const uint16_t* text, const std::vector<std::string>& propsJson) {
  std::vector<std::optional<JVal>> parsed(propsJson.size());
  if (r.props) {
    if (r.props >= propsJson.size()) throw OracleError(-1, "bad props id");
    parsed[r.props] = json_parse(propsJson[r.props]);
  }
  applyRecordParsed(r, text, parsed);
}

void Doc::applyRecordParsed(const Record& r, const uint16_t* text, const std::vector<std::optional<JVal>>& props) {
  auto propsOf = [&](uint32_t id) -> const JVal* {
    if (id == 0) return nullptr;
    if (id >= props.size() || !props[id]) throw OracleError(-1, "bad props id");
    return &*props[id];
  };
  switch (r.type) {
    case 0: {
      mt.counters.ops++;
      Seg* s = mt.newSeg();
      if (r.flags & 0x40) {  // PermutationSegment (inserted unallocated, permutationvector.ts:346-357)
        s->perm = true;
        s->cachedLength = (int)r.pos2;
      } else if (r.flags & 0x02) {
        s->isMarker = true;
        s->cachedLength = 1;
        s->refType = r.pos2 == 0xFFFFFFFFu ? -1 : (int)r.pos2;
      } else {
        s->text.assign(reinterpret_cast<const char16_t*>(text + r.payload), r.pos2);
        s->cachedLength = (int)r.pos2;
      }
      const JVal* p = propsOf(r.props);
      if (p && !js_falsy(p)) {
        s->hasPropManager = true;
        s->props = propsFromSpec(p);
      }
      mt.insertSegments((int)r.pos1, s, (int)r.refSeq, r.client, (int)r.seq);
      break;
    }
    case 1:
      mt.counters.ops++;
      mt.markRangeRemoved((int)r.pos1, (int)r.pos2, (int)r.refSeq, r.client, (int)r.seq);
      break;
    case 2: {
      mt.counters.ops++;
      const JVal* p = propsOf(r.props);
      static const JObj empty;
      const JObj& o = (p && p->t == JVal::Obj) ? p->obj : empty;
      Comb comb;  // MTB_F_COMB 0x0C of annotate records: 0x04 rewrite, 0x08 incr, 0x0C consensus
      const int ck = (r.flags >> 2) & 3;
      comb.kind = ck == 1 ? Comb::Rewrite : ck == 2 ? Comb::Incr : ck == 3 ? Comb::Consensus : Comb::None;
      mt.annotateRange((int)r.pos1, (int)r.pos2, o, comb, (int)r.refSeq, r.client, (int)r.seq);
      break;
    }
    case 4:
      mt.zamboniSegments();
      break;
    default:
      break;
  }
  if (r.flags & 0x01) updateSeqNumbers((int)r.msn, (int)r.seq);
}

// ---------------------------------------------------------------- a live client's local ops
// insertSegmentLocal / removeRangeLocal / annotateRangeLocal (client.ts:196-247) through applyInsertOp /
// applyRemoveRangeOp / applyAnnotateRangeOp with the local client's (currentSeq, clientId) and
// UnassignedSequenceNumber; getValidOpRange (client.ts:527-592) bounds-checks the local positions.
static void validLocalRange(int start, int end, int len, bool insert) {
  // start outside [0, length] (or at the length for a remove / annotate), or end <= start for a range;
  // an end past the length is not checked (nodeMap stops at the tree's end)
  if (start < 0 || start > len || (start == len && !insert) || (!insert && end <= start))
    throw OracleError(-1, "RangeOutOfBounds");
}
std::string Doc::insertLocalOp(int pos, const JVal& segSpec) {
  if (!mt.window.collaborating) throw OracleError(-1, "not collaborating");
  validLocalRange(pos, pos, mt.length(), true);
  Seg* s = makeSegFromSpec(mt, segSpec);
  if (s->cachedLength <= 0) return "";
  mt.insertSegments(pos, s, mt.window.currentSeq, mt.window.clientId, UnassignedSeq);
  JVal op;
  op.t = JVal::Obj;
  op.obj.push_back({u"pos1", JVal::number(pos)});
  op.obj.push_back({u"seg", segSpec});
  op.obj.push_back({u"type", JVal::number(0)});
  return json_stringify(op);
}
std::string Doc::removeLocalOp(int start, int end) {
  if (!mt.window.collaborating) throw OracleError(-1, "not collaborating");
  validLocalRange(start, end, mt.length(), false);
  mt.markRangeRemoved(start, end, mt.window.currentSeq, mt.window.clientId, UnassignedSeq);
  return "{\"pos1\":" + std::to_string(start) + ",\"pos2\":" + std::to_string(end) + ",\"type\":1}";
}
std::string Doc::annotateLocalOp(int start, int end, const JObj& props, const JVal* combiningOp, bool notifyConsensus) {
  if (!mt.window.collaborating) throw OracleError(-1, "not collaborating");
  const Comb comb = parse_comb(combiningOp);  // annotateRangeLocal(start, end, props, combiningOp)
  // A local consensus value is {value: undefined, seq: -1}, completed in place at the ack -- through
  // Client.pendingConsensus, which only annotateMarkerNotifyConsensus fills (client.ts:155-181).  Any other local
  // consensus annotate leaves a minimum-sequence-number listener that dereferences the missing entry (the reference
  // throws at a later update): not restated.
  if (comb.kind == Comb::Consensus && !notifyConsensus)
    fail_unsupported("local consensus annotate other than annotateMarkerNotifyConsensus (the reference throws at a "
                     "later minimum sequence number update)");
  validLocalRange(start, end, mt.length(), false);
  mt.annotateRange(start, end, props, comb, mt.window.currentSeq, mt.window.clientId, UnassignedSeq);
  JVal pv;
  pv.t = JVal::Obj;
  pv.obj = props;
  return std::string(combiningOp ? "{\"combiningOp\":" + json_stringify(*combiningOp) + "," : "{") + "\"pos1\":" +
         std::to_string(start) + ",\"pos2\":" + std::to_string(end) + ",\"props\":" + json_stringify(pv) + ",\"type\":2}";
}

std::string Doc::localOpJson(const JVal& op) {
  if (op.t != JVal::Obj) throw OracleError(-8, "op is not an object");
  const JVal* t = obj_get(op.obj, u"type");
  const int type = t && t->t == JVal::Num ? (int)t->num : -1;
  const int refSeq = mt.window.currentSeq, client = mt.window.clientId;
  auto pos = [&](const char16_t* k, const char16_t* rk, bool opt) -> int {
    const JVal* p = obj_get(op.obj, k);
    if (p && p->t == JVal::Num) return (int)p->num;
    const JVal* r = obj_get(op.obj, rk);
    if (r && !js_falsy(r)) return mt.posFromRelativePos(*r, refSeq, client);  // -1 fails the range check
    if (opt) return INT32_MIN;
    throw OracleError(-1, "RangeOutOfBounds");
  };
  const bool rel = obj_get(op.obj, u"relativePos1") || obj_get(op.obj, u"relativePos2");
  std::string out;
  if (type == 0) {
    const JVal* seg = obj_get(op.obj, u"seg");
    if (!seg) throw OracleError(-8, "insert without seg");
    out = insertLocalOp(pos(u"pos1", u"relativePos1", false), *seg);
  } else if (type == 1) {
    out = removeLocalOp(pos(u"pos1", u"relativePos1", false), pos(u"pos2", u"relativePos2", false));
  } else if (type == 2) {
    const JVal* pr = obj_get(op.obj, u"props");
    const JVal* comb = obj_get(op.obj, u"combiningOp");
    // annotateMarkerNotifyConsensus (client.ts:155-181): the op createAnnotateMarkerOp makes, flagged by the
    // caller with "notifyConsensus": true (not part of the op sent)
    const JVal* nc = obj_get(op.obj, u"notifyConsensus");
    const bool notify = nc && nc->t == JVal::True;
    Seg* marker = nullptr;
    if (notify) {
      const JVal* r1 = obj_get(op.obj, u"relativePos1");
      auto key = r1 && r1->t == JVal::Obj ? MergeTree::markerIdKey(obj_get(r1->obj, u"id")) : std::nullopt;
      auto it = key ? mt.idToSegment.find(*key) : mt.idToSegment.end();
      if (it == mt.idToSegment.end()) throw OracleError(-1, "annotateMarkerNotifyConsensus: marker without id");
      marker = it->second;
      pendingConsensus[*key] = marker;
    }
    out = annotateLocalOp(pos(u"pos1", u"relativePos1", false), pos(u"pos2", u"relativePos2", false),
                          pr && pr->t == JVal::Obj ? pr->obj : JObj(), comb && comb->t != JVal::Undef ? comb : nullptr,
                          notify);
    if (notify) {
      JVal sent = op;
      obj_del(sent.obj, u"notifyConsensus");
      return json_stringify(sent);
    }
  } else {
    throw OracleError(-8, "unsupported local op type");
  }
  return rel ? json_stringify(op) : out;
}

// ---------------------------------------------------------------- reconnect
// localNetLength with a localSeq (mergeTree.ts:636-664): the local view as it was right after local op
// `localSeq` (later local ops and remote ops above refSeq hidden)
int MergeTree::localNetLengthAt(const Seg* s, int refSeq, int localSeq) const {
  const bool lremoved = s->localRemovedSeq != INT32_MIN && s->localRemovedSeq <= localSeq;
  if (s->seq != UnassignedSeq) {
    if (s->seq > refSeq || (s->removed && s->removedSeq != UnassignedSeq && s->removedSeq <= refSeq) || lremoved) return 0;
    return s->cachedLength;
  }
  if (s->localSeq == INT32_MIN) fail_assert("0x39a", "unacked segment with undefined localSeq");
  if (s->localSeq > localSeq || lremoved) return 0;
  return s->cachedLength;
}
// findReconnectionPosition (client.ts:690-706) -> getPosition(segment, currentSeq, clientId, localSeq)
// (mergeTree.ts:768-785): block lengths come from the local partials (computeLocalPartials), which sum
// the leaves' localNetLength(leaf, refSeq, localSeq)
int MergeTree::reconnectPosition(Seg* s, int localSeq) {
  if (localSeq > window.localSeq) fail_assert("0x032", "localSeq greater than collab window");
  const int refSeq = window.currentSeq;
  std::function<int(Node*)> len = [&](Node* n) -> int {
    if (n->leaf) return localNetLengthAt(static_cast<Seg*>(n), refSeq, localSeq);
    Block* b = static_cast<Block*>(n);
    int t = 0;
    for (int i = 0; i < b->childCount; i++) t += len(b->children[i]);
    return t;
  };
  int total = 0;
  Node* node = s;
  for (Block* parent = s->parent; parent; node = parent, parent = parent->parent)
    for (int i = 0; i < parent->childCount && parent->children[i] != node; i++) total += len(parent->children[i]);
  return total;
}
static bool isRemovedAndAcked(const Seg* s) { return s->removed && s->removedSeq != UnassignedSeq; }
// normalizeAdjacentSegments (mergeTree.ts:2234-2336): in a run of removed / unacked segments, remotely
// removed (acked) segments slide after the last locally affected one, and each locally removed one slides
// forward past later unacked inserts made after its removal; the run's slots keep their places
void MergeTree::normalizeAdjacentSegments(std::vector<Seg*>& run) {
  struct Slot { Block* parent; int index; };
  std::vector<Slot> order;
  for (Seg* s : run) order.push_back({s->parent, s->index});
  std::vector<Seg*> list(run);  // the affected-segments List, as an array
  int last = (int)list.size() - 1;
  while (last >= 0 && isRemovedAndAcked(list[last])) last--;
  if (last < 0) return;
  Seg* lastLocal = list[last];
  auto indexOf = [&](Seg* x) { return (int)(std::find(list.begin(), list.end(), x) - list.begin()); };
  Seg* toSlide = lastLocal;
  Seg* nearer = last > 0 ? list[last - 1] : nullptr;
  while (toSlide) {
    if (isRemovedAndAcked(toSlide)) {
      list.erase(list.begin() + indexOf(toSlide));
      list.insert(list.begin() + indexOf(lastLocal) + 1, toSlide);
    } else if (toSlide->removed) {
      if (toSlide->localRemovedSeq == INT32_MIN)
        fail_assert("0x54d", "Removed segment that hasnt had its removal acked should be locally removed");
      int cur = indexOf(toSlide);
      int scan = cur + 1;
      while (scan < (int)list.size() && !isRemovedAndAcked(list[scan]) && list[scan]->localSeq != INT32_MIN &&
             list[scan]->localSeq > toSlide->localRemovedSeq) {
        cur = scan;
        scan++;
      }
      if (list[cur] != toSlide) {
        Seg* after = list[cur];
        list.erase(list.begin() + indexOf(toSlide));
        list.insert(list.begin() + indexOf(after) + 1, toSlide);
      }
    }
    toSlide = nearer;
    if (nearer) {
      const int ni = indexOf(nearer);
      nearer = ni > 0 ? list[ni - 1] : nullptr;
    }
  }
  for (size_t i = 0; i < list.size(); i++) order[i].parent->assignChild(list[i], order[i].index);
  // ancestors of the moved segments, deepest first (nodeUpdateLengthNewStructure)
  std::vector<std::pair<int, Block*>> blocks;
  for (Seg* sg : list)
    for (Block* b = sg->parent; b; b = b->parent) {
      int depth = 0;
      for (Block* x = b->parent; x; x = x->parent) depth++;
      bool seen = false;
      for (auto& e : blocks) seen |= e.second == b;
      if (!seen) blocks.push_back({depth, b});
    }
  std::stable_sort(blocks.begin(), blocks.end(), [](auto& a, auto& b) { return a.first > b.first; });
  for (auto& e : blocks) nodeUpdateLengthNewStructure(e.second, false);
}
// normalizeSegmentsOnRebase (mergeTree.ts:2357-2390)
void MergeTree::normalizeSegmentsOnRebase() {
  std::vector<Seg*> run;
  bool hasLocal = false, hasRemoteRemoved = false;
  std::vector<std::vector<Seg*>> todo;
  auto flush = [&] {
    if (hasLocal && hasRemoteRemoved && run.size() > 1) todo.push_back(run);
    run.clear();
    hasLocal = hasRemoteRemoved = false;
  };
  walkAllSegments([&](Seg* s) {
    if (s->removed || s->seq == UnassignedSeq) {
      if (isRemovedAndAcked(s)) hasRemoteRemoved = true;
      if (s->seq == UnassignedSeq) hasLocal = true;
      run.push_back(s);
    } else {
      flush();
    }
  });
  flush();
  // (the runs are disjoint and normalizing one moves only its own segments among its own slots)
  for (auto& r : todo) normalizeAdjacentSegments(r);
}

// Client.regeneratePendingOp (client.ts:917-960) with resetPendingDeltaToOps (:708-800)
std::string Doc::regeneratePendingOp(const JVal& op) {
  if (!mt.window.collaborating) throw OracleError(-1, "not collaborating");
  const int rebaseTo = mt.window.currentSeq;
  if (rebaseTo != lastNormalizationRefSeq) {
    mt.normalizeSegmentsOnRebase();
    lastNormalizationRefSeq = rebaseTo;
  }
  std::vector<const JVal*> members;
  const JVal* type = obj_get(op.obj, u"type");
  if (type && type->t == JVal::Num && (int)type->num == 3) {
    const JVal* ops = obj_get(op.obj, u"ops");
    if (ops && ops->t == JVal::Arr)
      for (auto& m : ops->arr) members.push_back(&m);
  } else {
    members.push_back(&op);
  }
  std::vector<JVal> opList;
  for (const JVal* resetOp : members) {
    if (mt.pendingSegments.empty()) fail_assert("0x033", "Segment group undefined");
    SegGroup* group = mt.pendingSegments.front();
    mt.pendingSegments.pop_front();
    // the group's segments in tree order (ordinal)
    std::unordered_map<const Seg*, size_t> ord;
    mt.walkAllSegments([&](Seg* s) { ord.emplace(s, ord.size()); });
    std::vector<Seg*> segs = group->segments;
    std::stable_sort(segs.begin(), segs.end(), [&](Seg* a, Seg* b) { return ord.at(a) < ord.at(b); });
    const JVal* rt = obj_get(resetOp->obj, u"type");
    const int t = rt && rt->t == JVal::Num ? (int)rt->num : -1;
    for (Seg* s : segs) {
      if (s->groups.empty() || s->groups.front() != group) fail_assert("0x035", "Segment group not at head of segment pending queue");
      s->groups.erase(s->groups.begin());
      const int pos = mt.reconnectPosition(s, group->localSeq);
      JVal newOp;
      bool have = false;
      if (t == 2) {
        if (!s->removed || (s->localRemovedSeq != INT32_MIN && s->removedSeq == UnassignedSeq)) {
          // createAnnotateRangeOp(start, end, props, combiningOp) (opBuilder.ts:52-65)
          const JVal* comb = obj_get(resetOp->obj, u"combiningOp");
          newOp = jop({{u"pos1", JVal::number(pos)}, {u"pos2", JVal::number(pos + s->cachedLength)}});
          if (comb && comb->t != JVal::Undef) newOp.obj.insert(newOp.obj.begin(), {u"combiningOp", *comb});
          const JVal* pr = obj_get(resetOp->obj, u"props");
          if (pr) newOp.obj.push_back({u"props", *pr});
          newOp.obj.push_back({u"type", JVal::number(2)});
          have = true;
        }
      } else if (t == 0) {
        if (s->seq != UnassignedSeq) fail_assert("0x037", "Segment already has assigned sequence number");
        JVal segj = segJson(s);
        const JVal* rseg = obj_get(resetOp->obj, u"seg");
        const JVal* rprops = rseg && rseg->t == JVal::Obj ? obj_get(rseg->obj, u"props") : nullptr;
        if (rprops && rprops->t != JVal::Undef) {  // segment.clone() with properties = resetOp.seg.props
          Seg c = *s;
          c.groups.clear();
          c.props = rprops->t == JVal::Obj ? std::optional<JObj>(rprops->obj) : std::nullopt;
          segj = segJson(&c);
        }
        newOp = jop({{u"pos1", JVal::number(pos)}, {u"seg", segj}, {u"type", JVal::number(0)}});
        have = true;
      } else if (t == 1) {
        if (s->localRemovedSeq != INT32_MIN && s->removedSeq == UnassignedSeq) {
          newOp = jop({{u"pos1", JVal::number(pos)}, {u"pos2", JVal::number(pos + s->cachedLength)}, {u"type", JVal::number(1)}});
          have = true;
        }
      } else {
        throw OracleError(-8, "Invalid op type");
      }
      if (have) {
        mt.groupPool.push_back(std::make_unique<SegGroup>());
        SegGroup* g = mt.groupPool.back().get();
        g->localSeq = group->localSeq;
        g->refSeq = mt.window.currentSeq;
        g->segments.push_back(s);
        s->groups.push_back(g);
        mt.pendingSegments.push_back(g);
        opList.push_back(std::move(newOp));
      }
    }
  }
  if (opList.size() == 1) return json_stringify(opList[0]);
  JVal arr;
  arr.t = JVal::Arr;
  arr.arr = std::move(opList);
  return json_stringify(jop({{u"ops", arr}, {u"type", JVal::number(3)}}));
}

// ---------------------------------------------------------------- local (detached) edits
void Doc::insertTextLocal(int pos, const u16str& text, const std::optional<JObj>& props) {
  Seg* s = mt.newSeg();
  s->text = text;
  s->cachedLength = (int)text.size();
  if (props) { s->hasPropManager = true; s->props = *props; }
  int seq = mt.window.collaborating ? UnassignedSeq : UniversalSeq;
  if (mt.window.collaborating) fail_unsupported("local edits while collaborating");
  mt.insertSegments(pos, s, mt.window.currentSeq, mt.window.clientId, seq);
}
void Doc::insertMarkerLocal(int pos, int refType, const std::optional<JObj>& props) {
  if (mt.window.collaborating) fail_unsupported("local edits while collaborating");
  Seg* s = mt.newSeg();
  s->isMarker = true;
  s->refType = refType;
  s->cachedLength = 1;
  if (props) { s->hasPropManager = true; s->props = *props; }
  mt.insertSegments(pos, s, mt.window.currentSeq, mt.window.clientId, UniversalSeq);
}
void Doc::annotateRangeLocal(int start, int end, const JObj& props) {
  if (mt.window.collaborating) fail_unsupported("local edits while collaborating");
  mt.annotateRange(start, end, props, Comb(), mt.window.currentSeq, mt.window.clientId, UniversalSeq);
}
void Doc::removeRangeLocal(int start, int end) {
  if (mt.window.collaborating) fail_unsupported("local edits while collaborating");
  mt.markRangeRemoved(start, end, mt.window.currentSeq, mt.window.clientId, UniversalSeq);
}

// ---------------------------------------------------------------- SnapshotV1 (snapshotV1.ts)
static JVal segJson(const Seg* s) {  // TextSegment.toJSONObject / Marker.toJSONObject
  if (s->perm) {  // PermutationSegment.toJSONObject: [length, start]
    JVal a;
    a.t = JVal::Arr;
    a.arr.push_back(JVal::number(s->cachedLength));
    a.arr.push_back(JVal::number(s->start));
    return a;
  }
  if (s->isMarker) {
    JVal o;
    o.t = JVal::Obj;
    JVal m;
    m.t = JVal::Obj;
    if (s->refType >= 0) obj_set(m.obj, u"refType", JVal::number(s->refType));
    o.obj.push_back({u"marker", m});
    if (s->props) {
      JVal p; p.t = JVal::Obj; p.obj = *s->props;
      o.obj.push_back({u"props", p});
    }
    return o;
  }
  if (s->props) {
    JVal o;
    o.t = JVal::Obj;
    o.obj.push_back({u"text", JVal::string(s->text)});
    JVal p; p.t = JVal::Obj; p.obj = *s->props;
    o.obj.push_back({u"props", p});
    return o;
  }
  return JVal::string(s->text);
}

static int64_t utf8ByteLength(const std::string& utf8) {  // summaryUtils.ts:56-71 on the JS string
  u16str s = utf8_to_u16(utf8);
  int64_t n = (int64_t)s.size();
  for (long i = (long)s.size() - 1; i >= 0; i--) {
    uint32_t code = s[i];
    if (code > 0x7f && code <= 0x7ff) n++;
    else if (code > 0x7ff && code <= 0xffff) n += 2;
    if (code >= 0xdc00 && code <= 0xdfff) i--;
  }
  return n;
}

std::vector<std::pair<std::string, std::string>> Doc::summarizeV1(std::string* summaryJson) {
  MergeTree& t = mt;
  const int minSeq = t.window.minSeq;
  const int curSeq = t.window.currentSeq;
  std::vector<JVal> segments;
  std::vector<int> lengths;
  auto normalize = [](Seg* s) {
    if (s->props && s->props->empty()) {  // snapshotV1.ts:199-206 (mutates the live segment)
      s->props.reset();
      s->hasPropManager = false;
    }
  };
  // prev: either a live segment or a coalesced clone (owned here)
  std::optional<Seg> prevClone;
  Seg* prev = nullptr;
  auto pushSeg = [&](Seg* s) {
    if (!s) return;
    normalize(s);
    segments.push_back(segJson(s));
    lengths.push_back(s->cachedLength);
  };
  t.walkAllSegments([&](Seg* s) {  // extractSync (snapshotV1.ts:180-312)
    if (s->seq == UnassignedSeq || (s->removed && s->removedSeq <= minSeq)) return;
    if (s->seq <= minSeq && (!s->removed || s->removedSeq == UnassignedSeq)) {
      if (!prev) {
        prev = s;
      } else if (canAppend(prev, s) && matchSegProps(prev, s)) {
        Seg c = *prev;  // prev.clone(); prev.append(segment.clone())
        if (c.props) c.hasPropManager = true;
        c.text += s->text;
        c.cachedLength += s->cachedLength;
        c.parent = nullptr;
        prevClone = std::move(c);
        prev = &*prevClone;
      } else {
        pushSeg(prev);
        prev = s;
      }
    } else {
      pushSeg(prev);
      prev = nullptr;
      normalize(s);
      JVal raw;
      raw.t = JVal::Obj;
      raw.obj.push_back({u"json", segJson(s)});
      if (s->seq > minSeq) {
        raw.obj.push_back({u"seq", JVal::number(s->seq)});
        raw.obj.push_back({u"client", JVal::string(utf8_to_u16(getLongClientId(s->clientId)))});
      }
      if (s->removed) {
        if (s->removedSeq == UnassignedSeq || s->removedSeq <= minSeq) fail_assert("0x065", "invalid removed seq");
        raw.obj.push_back({u"removedSeq", JVal::number(s->removedSeq)});
        raw.obj.push_back({u"removedClient", JVal::string(utf8_to_u16(getLongClientId(s->removedClientIds[0])))});
        JVal ids;
        ids.t = JVal::Arr;
        for (int c : s->removedClientIds) ids.arr.push_back(JVal::string(utf8_to_u16(getLongClientId(c))));
        raw.obj.push_back({u"removedClientIds", ids});
      }
      segments.push_back(raw);
      lengths.push_back(s->cachedLength);
    }
  });
  pushSeg(prev);

  // emit (snapshotV1.ts:122-178)
  struct Chunk { int segmentCount = 0, length = 0, startIndex = 0; };
  std::vector<Chunk> chunks;
  int totalSegmentCount = 0, totalLength = 0;
  do {
    Chunk c;
    c.startIndex = totalSegmentCount;
    while (c.length < t.options.chunkSize && c.startIndex + c.segmentCount < (int)segments.size()) {
      c.length += lengths[c.startIndex + c.segmentCount];
      c.segmentCount++;
    }
    chunks.push_back(c);
    totalSegmentCount += c.segmentCount;
    totalLength += c.length;
  } while (totalSegmentCount < (int)segments.size());

  auto chunkJson = [&](const Chunk& c, bool header) {
    JVal o;
    o.t = JVal::Obj;
    o.obj.push_back({u"version", JVal::string(u"1")});
    o.obj.push_back({u"segmentCount", JVal::number(c.segmentCount)});
    o.obj.push_back({u"length", JVal::number(c.length)});
    JVal segs;
    segs.t = JVal::Arr;
    for (int i = 0; i < c.segmentCount; i++) segs.arr.push_back(segments[c.startIndex + i]);
    o.obj.push_back({u"segments", segs});
    o.obj.push_back({u"startIndex", JVal::number(c.startIndex)});
    if (header) {
      JVal h;
      h.t = JVal::Obj;
      h.obj.push_back({u"minSequenceNumber", JVal::number(minSeq)});
      h.obj.push_back({u"sequenceNumber", JVal::number(curSeq)});
      JVal ids;
      ids.t = JVal::Arr;
      for (size_t i = 0; i < chunks.size(); i++) {
        JVal id;
        id.t = JVal::Obj;
        std::string name = i == 0 ? "header" : "body_" + std::to_string(i - 1);
        id.obj.push_back({u"id", JVal::string(utf8_to_u16(name))});
        ids.arr.push_back(id);
      }
      h.obj.push_back({u"orderedChunkMetadata", ids});
      h.obj.push_back({u"totalLength", JVal::number(totalLength)});
      h.obj.push_back({u"totalSegmentCount", JVal::number(totalSegmentCount)});
      o.obj.push_back({u"headerMetadata", h});
    }
    return json_stringify(o);
  };
  std::vector<std::pair<std::string, std::string>> blobs;
  blobs.push_back({"header", chunkJson(chunks[0], true)});
  for (size_t i = 1; i < chunks.size(); i++) blobs.push_back({"body_" + std::to_string(i - 1), chunkJson(chunks[i], false)});
  if (perm) {
    // PermutationVector.summarize (permutationvector.ts:310-325): {segments: <SnapshotV1>, handleTable}
    std::string inner;
    std::vector<std::pair<std::string, std::string>> segBlobs = blobs;
    std::string ht = handleTableJson();
    if (summaryJson) {
      JVal tree;
      tree.t = JVal::Obj;
      int64_t total = 0;
      for (auto& b : segBlobs) {
        JVal blob;
        blob.t = JVal::Obj;
        blob.obj.push_back({u"type", JVal::number(2)});
        blob.obj.push_back({u"content", JVal::string(utf8_to_u16(b.second))});
        obj_set(tree.obj, utf8_to_u16(b.first), blob);
        total += utf8ByteLength(b.second);
      }
      JVal segs;
      segs.t = JVal::Obj;
      segs.obj.push_back({u"type", JVal::number(1)});
      segs.obj.push_back({u"tree", tree});
      JVal htb;
      htb.t = JVal::Obj;
      htb.obj.push_back({u"type", JVal::number(2)});
      htb.obj.push_back({u"content", JVal::string(utf8_to_u16(ht))});
      JVal outer;
      outer.t = JVal::Obj;
      outer.obj.push_back({u"segments", segs});
      outer.obj.push_back({u"handleTable", htb});
      JVal summary;
      summary.t = JVal::Obj;
      summary.obj.push_back({u"type", JVal::number(1)});
      summary.obj.push_back({u"tree", outer});
      JVal stats;
      stats.t = JVal::Obj;
      stats.obj.push_back({u"treeNodeCount", JVal::number(2)});
      stats.obj.push_back({u"blobNodeCount", JVal::number((double)segBlobs.size() + 1)});
      stats.obj.push_back({u"handleNodeCount", JVal::number(0)});
      stats.obj.push_back({u"totalBlobSize", JVal::number((double)(total + utf8ByteLength(ht)))});
      stats.obj.push_back({u"unreferencedBlobSize", JVal::number(0)});
      JVal all;
      all.t = JVal::Obj;
      all.obj.push_back({u"summary", summary});
      all.obj.push_back({u"stats", stats});
      *summaryJson = json_stringify(all);
    }
    for (auto& b : blobs) b.first = "segments/" + b.first;
    blobs.push_back({"handleTable", ht});
    return blobs;
  }
  if (summaryJson) {
    // ISummaryTreeWithStats (summaryUtils.ts:138-198)
    JVal tree;
    tree.t = JVal::Obj;
    int64_t total = 0;
    for (auto& b : blobs) {
      JVal blob;
      blob.t = JVal::Obj;
      blob.obj.push_back({u"type", JVal::number(2)});
      blob.obj.push_back({u"content", JVal::string(utf8_to_u16(b.second))});
      obj_set(tree.obj, utf8_to_u16(b.first), blob);
      total += utf8ByteLength(b.second);
    }
    JVal summary;
    summary.t = JVal::Obj;
    summary.obj.push_back({u"type", JVal::number(1)});
    summary.obj.push_back({u"tree", tree});
    JVal stats;
    stats.t = JVal::Obj;
    stats.obj.push_back({u"treeNodeCount", JVal::number(1)});
    stats.obj.push_back({u"blobNodeCount", JVal::number((double)blobs.size())});
    stats.obj.push_back({u"handleNodeCount", JVal::number(0)});
    stats.obj.push_back({u"totalBlobSize", JVal::number((double)total)});
    stats.obj.push_back({u"unreferencedBlobSize", JVal::number(0)});
    JVal all;
    all.t = JVal::Obj;
    all.obj.push_back({u"summary", summary});
    all.obj.push_back({u"stats", stats});
    *summaryJson = json_stringify(all);
  }
  return blobs;
}

// Canonical segment dump: header line then one JSON array per segment, in tree order:
// [path, kind, text|refType, seq, client, removedSeq(-1 none), [removedClientIds], props|null]
std::string Doc::dumpSegments() {
  std::string out;
  {
    JVal h;
    h.t = JVal::Obj;
    h.obj.push_back({u"minSeq", JVal::number(mt.window.minSeq)});
    h.obj.push_back({u"currentSeq", JVal::number(mt.window.currentSeq)});
    h.obj.push_back({u"length", JVal::number(mt.length())});
    if (perm) h.obj.push_back({u"handles", json_parse(handleTableJson())});
    out += json_stringify(h);
    out.push_back('\n');
  }
  std::vector<int> path;
  std::function<void(Block*)> rec = [&](Block* b) {
    for (int i = 0; i < b->childCount; i++) {
      path.push_back(i);
      Node* c = b->children[i];
      if (c->leaf) {
        Seg* s = static_cast<Seg*>(c);
        JVal row;
        row.t = JVal::Arr;
        JVal p;
        p.t = JVal::Arr;
        for (int x : path) p.arr.push_back(JVal::number(x));
        row.arr.push_back(p);
        if (s->perm) {
          row.arr.push_back(JVal::string(u"P"));
          row.arr.push_back(segJson(s));
        } else if (s->isMarker) {
          row.arr.push_back(JVal::string(u"M"));
          row.arr.push_back(s->refType >= 0 ? JVal::number(s->refType) : JVal::null());
        } else {
          row.arr.push_back(JVal::string(u"T"));
          row.arr.push_back(JVal::string(s->text));
        }
        // PermutationVectors name clients by long id (setCell interning order is lazy, matrix.ts:669-672)
        auto cl = [&](int c) { return perm ? JVal::string(utf8_to_u16(getLongClientId(c))) : JVal::number(c); };
        row.arr.push_back(JVal::number(s->seq));
        row.arr.push_back(cl(s->clientId));
        row.arr.push_back(JVal::number(s->removed ? s->removedSeq : -1));
        JVal rc;
        rc.t = JVal::Arr;
        if (s->removed)
          for (int c2 : s->removedClientIds) rc.arr.push_back(cl(c2));
        row.arr.push_back(rc);
        if (s->props && !s->props->empty()) {  // {} and undefined are interchangeable (snapshotV1.ts:199)
          JVal pr;
          pr.t = JVal::Obj;
          pr.obj = *s->props;
          row.arr.push_back(pr);
        } else {
          row.arr.push_back(JVal::null());
        }
        out += json_stringify(row);
        out.push_back('\n');
      } else {
        rec(static_cast<Block*>(c));
      }
      path.pop_back();
    }
  };
  rec(mt.root);
  return out;
}

// State digest v1 (DESIGN.md "State digest"): the canonical dump's content (tree paths, segment text /
// marker / handle span, seq, client, removal info, properties) folded into 64 bits with a definition
// that a GPU wave can evaluate over its own layout.  Checker-side restatement of the same definition.
namespace {
inline uint64_t dg_fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
inline uint64_t dg_mix(uint64_t h, uint64_t x) { return dg_fmix(h ^ (x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2))); }
}  // namespace

uint64_t Doc::digest() {
  uint64_t S = 0, nsegs = 0;
  std::vector<int> path;
  std::function<void(Block*)> rec = [&](Block* b) {
    for (int i = 0; i < b->childCount; i++) {
      path.push_back(i);
      Node* c = b->children[i];
      if (!c->leaf) {
        rec(static_cast<Block*>(c));
        path.pop_back();
        continue;
      }
      const Seg* s = static_cast<const Seg*>(c);
      uint64_t P = 0;
      for (size_t l = 0; l < path.size() && l < 16; l++) P += (uint64_t)(path[l] + 1) << (4 * l);
      uint64_t K, T = 0;
      int len;
      if (s->perm) {
        K = 2;
        len = s->cachedLength;
        T = dg_fmix(((uint64_t)(uint32_t)s->start << 32) | (uint32_t)len);
      } else if (s->isMarker) {
        K = 1;
        len = 1;
        T = dg_fmix(0x4D00000000ull | (uint32_t)(s->refType + 1));
      } else {
        K = 0;
        len = (int)s->text.size();
        for (size_t j = 0; j < s->text.size(); j++) T += dg_fmix((((uint64_t)j << 16) | (uint16_t)s->text[j]) + 0x632BE59BD9B4E019ull);
      }
      uint64_t Rc = 0;
      if (s->removed)
        for (size_t q = 0; q < s->removedClientIds.size(); q++) Rc += dg_mix(q + 1, (uint32_t)(int32_t)s->removedClientIds[q]);
      uint64_t Ph = 0;
      if (s->props) {
        uint64_t q = 0;
        for (auto& kv : *s->props) {
          if (kv.second.t == JVal::Undef) continue;  // JSON.stringify omits it
          Ph += dg_mix(dg_mix(q + 1, fnv1a64(u16_to_utf8(kv.first))), fnv1a64(json_stringify(kv.second)));
          q++;
        }
      }
      uint64_t h = 0;
      h = dg_mix(h, P);
      h = dg_mix(h, K);
      h = dg_mix(h, T);
      h = dg_mix(h, (uint32_t)len);
      h = dg_mix(h, (uint32_t)s->seq);
      h = dg_mix(h, (uint32_t)s->clientId);
      h = dg_mix(h, (uint32_t)(s->removed ? s->removedSeq : -1));
      h = dg_mix(h, Rc);
      h = dg_mix(h, Ph);
      nsegs++;
      S += dg_fmix(h + nsegs * 0xD6E8FEB86659FD93ull);
      path.pop_back();
    }
  };
  rec(mt.root);
  uint64_t D = 0x4D544231ull;  // "MTB1"
  D = dg_mix(D, (uint32_t)mt.window.minSeq);
  D = dg_mix(D, (uint32_t)mt.window.currentSeq);
  D = dg_mix(D, (uint32_t)mt.length());
  D = dg_mix(D, nsegs);
  return dg_mix(D, S);
}

// Client.load -> SnapshotLoader (snapshotLoader.ts:41-257) for SnapshotV1 chunks.
// toLatestVersion (snapshotChunks.ts:151-175): a legacy chunk (no "version", SnapshotLegacy's MergeTreeChunkLegacy)
// becomes the V1 shape the loader reads -- segments = segmentTexts, segmentCount = chunkSegmentCount, length =
// chunkLengthChars -- and a legacy header gets buildHeaderMetadataForLegacyChunk's metadata (:178-199): its own
// headerMetadata if present, else [header] + [body] when chunkLengthChars < totalLengthChars, minSequenceNumber
// = chunkMinSequenceNumber (absent in SnapshotLegacy's output), sequenceNumber = chunkSequenceNumber.
static JVal to_latest_version(const std::string& path, const JVal& chunk) {
  if (chunk.t != JVal::Obj) throw OracleError(-8, "chunk is not an object");
  const JVal* ver = obj_get(chunk.obj, u"version");
  if (ver && ver->t == JVal::Str && ver->str == u"1") return chunk;
  if (ver && ver->t != JVal::Undef) throw OracleError(-8, "Unsupported chunk path: " + path);
  JVal v;
  v.t = JVal::Obj;
  auto put = [&](const char16_t* k, const JVal* x) {
    if (x) v.obj.push_back({k, *x});
  };
  v.obj.push_back({u"version", JVal::string(u"1")});
  put(u"length", obj_get(chunk.obj, u"chunkLengthChars"));
  put(u"segmentCount", obj_get(chunk.obj, u"chunkSegmentCount"));
  if (path == "header") {
    if (const JVal* hm = obj_get(chunk.obj, u"headerMetadata")) {
      put(u"headerMetadata", hm);
    } else {
      JVal md;
      md.t = JVal::Obj;
      JVal ids;
      ids.t = JVal::Arr;
      JVal h;
      h.t = JVal::Obj;
      h.obj.push_back({u"id", JVal::string(u"header")});
      ids.arr.push_back(h);
      const JVal* cl = obj_get(chunk.obj, u"chunkLengthChars");
      const JVal* tl = obj_get(chunk.obj, u"totalLengthChars");
      if (cl && tl && cl->t == JVal::Num && tl->t == JVal::Num && cl->num < tl->num) {
        JVal bd;
        bd.t = JVal::Obj;
        bd.obj.push_back({u"id", JVal::string(u"body")});
        ids.arr.push_back(bd);
      }
      md.obj.push_back({u"orderedChunkMetadata", ids});
      if (const JVal* m = obj_get(chunk.obj, u"chunkMinSequenceNumber")) md.obj.push_back({u"minSequenceNumber", *m});
      if (const JVal* q = obj_get(chunk.obj, u"chunkSequenceNumber")) md.obj.push_back({u"sequenceNumber", *q});
      if (tl) md.obj.push_back({u"totalLength", *tl});
      if (const JVal* ts = obj_get(chunk.obj, u"totalSegmentCount")) md.obj.push_back({u"totalSegmentCount", *ts});
      v.obj.push_back({u"headerMetadata", md});
    }
  }
  put(u"segments", obj_get(chunk.obj, u"segmentTexts"));
  put(u"startIndex", obj_get(chunk.obj, u"chunkStartSegmentIndex"));
  return v;
}

std::string Doc::catchUpOps(const std::vector<std::pair<std::string, std::string>>& blobs) {
  // SnapshotLoader.loadBodyAndCatchupOps (snapshotLoader.ts:60-86): one blob beyond the ordered chunks holds
  // the catch-up messages (any name: mergeTree options.catchUpBlobName ?? "catchupOps")
  const JVal header = to_latest_version("header", json_parse(blobs.empty() ? std::string("{}") : [&]() {
    for (auto& b : blobs)
      if (b.first == "header") return b.second;
    throw OracleError(-1, "missing blob header");
  }()));
  const JVal* md = obj_get(header.obj, u"headerMetadata");
  const JVal* ocm = md ? obj_get(md->obj, u"orderedChunkMetadata") : nullptr;
  const size_t n = ocm && ocm->t == JVal::Arr ? ocm->arr.size() : 1;
  if (blobs.size() == n + 1) {
    std::vector<std::string> rest;
    for (auto& b : blobs) {
      bool listed = false;
      for (size_t i = 0; i < n && ocm; i++) {
        const JVal* id = obj_get(ocm->arr[i].obj, u"id");
        if (id && id->t == JVal::Str && u16_to_utf8(id->str) == b.first) listed = true;
      }
      if (!listed) rest.push_back(b.second);
    }
    if (rest.size() != 1) throw OracleError(-4, "0x060 There should be only one blob with catch up ops");
    return rest[0];
  }
  if (blobs.size() != n) throw OracleError(-8, "Unexpected blobs in snapshot");
  return "[]";
}

void Doc::loadV1(const std::vector<std::pair<std::string, std::string>>& blobs, const std::string& observerId) {
  auto findBlob = [&](const std::string& id) -> const std::string& {
    for (auto& b : blobs)
      if (b.first == id) return b.second;
    throw OracleError(-1, "missing blob " + id);
  };
  auto num = [](const JVal* v, int dflt) { return v && v->t == JVal::Num ? (int)v->num : dflt; };
  // specToSegment (snapshotLoader.ts:94-131)
  auto specToSegment = [&](const JVal& spec) -> Seg* {
    const bool mergeInfo = spec.t == JVal::Obj && obj_get(spec.obj, u"json") != nullptr;  // hasMergeInfo
    if (!mergeInfo) {
      Seg* s = makeSegFromSpec(mt, spec);
      s->seq = UniversalSeq;
      s->clientId = NonCollabClient;
      return s;
    }
    Seg* s = makeSegFromSpec(mt, *obj_get(spec.obj, u"json"));
    const JVal* client = obj_get(spec.obj, u"client");
    s->clientId = client && client->t == JVal::Str ? getOrAddShortClientId(u16_to_utf8(client->str)) : NonCollabClient;
    const JVal* seq = obj_get(spec.obj, u"seq");
    s->seq = seq && seq->t == JVal::Num ? (int)seq->num : UniversalSeq;
    const JVal* rseq = obj_get(spec.obj, u"removedSeq");
    if (rseq && rseq->t == JVal::Num) {
      s->removed = true;
      s->removedSeq = (int)rseq->num;
    }
    const JVal* rc = obj_get(spec.obj, u"removedClient");
    if (rc && rc->t == JVal::Str) s->removedClientIds = {getOrAddShortClientId(u16_to_utf8(rc->str))};
    const JVal* rcs = obj_get(spec.obj, u"removedClientIds");
    if (rcs && rcs->t == JVal::Arr) {
      s->removedClientIds.clear();
      for (auto& c : rcs->arr) s->removedClientIds.push_back(getOrAddShortClientId(u16_to_utf8(c.str)));
    }
    return s;
  };
  // loadHeader (snapshotLoader.ts:133-167)
  const JVal header = to_latest_version("header", json_parse(findBlob("header")));
  const JVal* hsegs = obj_get(header.obj, u"segments");
  const JVal* md = obj_get(header.obj, u"headerMetadata");
  if (!hsegs || hsegs->t != JVal::Arr || !md || md->t != JVal::Obj) throw OracleError(-8, "header metadata not available");
  std::vector<Seg*> segs;
  for (auto& sp : hsegs->arr) segs.push_back(specToSegment(sp));
  mt.reloadFromSegments(segs);
  const int seqNum = num(obj_get(md->obj, u"sequenceNumber"), 0);
  const int minSeqNum = num(obj_get(md->obj, u"minSequenceNumber"), seqNum);
  startOrUpdateCollaboration(observerId, minSeqNum, seqNum);
  // loadBody (snapshotLoader.ts:169-248)
  const JVal* ocm = obj_get(md->obj, u"orderedChunkMetadata");
  std::vector<Seg*> body;
  // (chunk1.segmentCount === headerMetadata.totalSegmentCount: nothing more to load, snapshotLoader.ts:180)
  const bool complete = num(obj_get(header.obj, u"segmentCount"), -1) == num(obj_get(md->obj, u"totalSegmentCount"), -2);
  if (ocm && ocm->t == JVal::Arr && !complete) {
    for (size_t ci = 1; ci < ocm->arr.size(); ci++) {
      const JVal* id = obj_get(ocm->arr[ci].obj, u"id");
      const std::string path = u16_to_utf8(id->str);
      const JVal chunk = to_latest_version(path, json_parse(findBlob(path)));
      const JVal* cs = obj_get(chunk.obj, u"segments");
      if (cs && cs->t == JVal::Arr)
        for (auto& sp : cs->arr) body.push_back(specToSegment(sp));
    }
  }
  std::vector<Seg*> batch;
  auto append = [&](const std::vector<Seg*>& v, int cli, int seq) {
    mt.insertSegmentsBatch(mt.root->cachedLength, v, UniversalSeq, cli, seq);
  };
  auto flushBatch = [&] {
    if (!batch.empty()) append(batch, NonCollabClient, UniversalSeq);
    batch.clear();
  };
  for (Seg* sg : body) {
    if (sg->clientId == NonCollabClient && sg->seq == UniversalSeq) {
      batch.push_back(sg);
    } else {
      flushBatch();
      append({sg}, sg->clientId, sg->seq);
    }
  }
  flushBatch();
}

// ---------------------------------------------------------------- PermutationVector / SharedMatrix
// getContainingSegment (mergeTree.ts:787-813): the first leaf of nodeMap over [pos, pos + 1)
Seg* MergeTree::containingSegment(int pos, int refSeq, int clientId, int* offset) {
  Seg* found = nullptr;
  int off = 0;
  nodeMap(
      refSeq, clientId,
      [&](Seg* s, int, int start, int) {
        found = s;
        off = start;
        return false;
      },
      [](Block*) {}, pos, pos + 1);
  if (offset) *offset = off;
  return found;
}
void MergeTree::mapRange(int refSeq, int clientId, int start, int end, const std::function<bool(Seg*, int, int, int)>& f) {
  if (end < 0) {
    const int l = blockLength(root, refSeq, clientId);
    end = l == UNDEF_LEN ? 0 : l;
  }
  nodeMap(refSeq, clientId, [&](Seg* s, int pos, int st, int en) { return f(s, pos, st, en); }, [](Block*) {}, start, end);
}
void MergeTree::mapAll(int refSeq, int clientId, const std::function<void(Seg*)>& f) {
  const int end = blockLength(root, refSeq, clientId);
  nodeMap(
      refSeq, clientId,
      [&](Seg* s, int, int, int) {
        f(s);
        return true;
      },
      [](Block*) {}, 0, end == UNDEF_LEN ? 0 : end);
}
// getPosition (mergeTree.ts:1240-1262) in the local view: lengths of everything before the node
int MergeTree::localPosition(Seg* s) {
  int total = 0;
  Node* node = s;
  for (Block* parent = s->parent; parent; node = parent, parent = parent->parent)
    for (int i = 0; i < parent->childCount && parent->children[i] != node; i++) {
      int l = nodeLength(parent->children[i], window.currentSeq, window.clientId);
      total += l == UNDEF_LEN ? 0 : l;
    }
  return total;
}

void Doc::enablePermutation() {
  perm = true;
  // onMaintenance (permutationvector.ts:418-441): handles of unlinked segments back to the free list
  mt.onUnlink = [this](Seg* s) {
    if (s->perm && s->start >= 1) {
      if (onHandlesRecycled) onHandlesRecycled(s->start, s->cachedLength);  // clear, then free
      for (int i = 0; i < s->cachedLength; i++) freeHandle(s->start + i);
    }
  };
}
int Doc::allocateHandle() {
  const int64_t free = handles[0];
  const int64_t next = free < (int64_t)handles.size() ? handles[free] : free + 1;  // `?? free + 1`
  handles[0] = next;
  if (free == (int64_t)handles.size()) handles.push_back(0);
  else handles[free] = 0;
  return (int)free;
}
void Doc::freeHandle(int h) {
  handles[h] = handles[0];
  handles[0] = h;
}
int Doc::adjustPosition(int pos, int refSeq, const std::string& longClientId) {
  const int client = getOrAddShortClientId(longClientId);  // getClientSequenceArgsForMessage
  int offset = 0;
  Seg* s = mt.containingSegment(pos, refSeq, client, &offset);
  if (!s || s->removed) return -1;
  return mt.localPosition(s) + offset;
}
int Doc::getAllocatedHandle(int pos) {
  int offset = 0;
  Seg* s = mt.containingSegment(pos, mt.window.currentSeq, mt.window.clientId, &offset);
  if (!s) throw OracleError(-4, "0x027 Trying to get handle of out-of-bounds position!");
  if (s->start >= 1) return s->start + offset;  // getMaybeHandle: start + offset (handlecache.ts:79)
  // walkSegments(pos, pos + 1, splitRange = true) in the local view
  mt.boundary(pos, mt.window.currentSeq, mt.window.clientId);
  mt.boundary(pos + 1, mt.window.currentSeq, mt.window.clientId);
  Seg* t = mt.containingSegment(pos, mt.window.currentSeq, mt.window.clientId, &offset);
  if (!t || t->cachedLength != 1 || offset != 0) throw OracleError(-4, "handle allocation did not isolate one position");
  const int h = allocateHandle();
  if (t->start != HandleUnallocated) throw OracleError(-4, "0x024 Start of PermutationSegment already allocated!");
  t->start = h;
  mt.counters.segsTouched += 1;
  return h;
}
std::string Doc::handleTableJson() const {
  std::string o = "[";
  for (size_t i = 0; i < handles.size(); i++) {
    if (i) o += ",";
    o += std::to_string(handles[i]);
  }
  return o + "]";
}

// SharedMatrix.processCore (matrix.ts:636-697): vector ops go to their PermutationVector's applyMsg;
// a remote setCell adjusts (row, col) into the local view and allocates both handles when both survive.
void MatrixDoc::applyMsg(const JVal& msg) {
  if (msg.t != JVal::Obj) throw OracleError(-8, "message is not an object");
  const JVal* type = obj_get(msg.obj, u"type");
  const JVal* contents = obj_get(msg.obj, u"contents");
  if (!type || type->t != JVal::Str || type->str != u"op" || !contents || contents->t != JVal::Obj) return;
  const JVal* target = obj_get(contents->obj, u"target");
  if (target && target->t == JVal::Str && target->str == u"rows") return rows.applyMsg(msg);
  if (target && target->t == JVal::Str && target->str == u"cols") return cols.applyMsg(msg);
  const JVal* t = obj_get(contents->obj, u"type");
  if (!t || t->t != JVal::Num || (int)t->num != 2) throw OracleError(-4, "0x021 SharedMatrix message contents have unexpected type!");
  const JVal* cid = obj_get(msg.obj, u"clientId");
  if (!cid || cid->t != JVal::Str) fail_unsupported("message without string clientId");
  const std::string longId = u16_to_utf8(cid->str);
  if (rows.longClientId && longId == *rows.longClientId) return;  // ack of a local set
  const JVal* ref = obj_get(msg.obj, u"referenceSequenceNumber");
  const JVal* r = obj_get(contents->obj, u"row");
  const JVal* c = obj_get(contents->obj, u"col");
  if (!ref || ref->t != JVal::Num || !r || r->t != JVal::Num || !c || c->t != JVal::Num)
    throw OracleError(-8, "bad setCell message");
  const int refSeq = (int)ref->num;
  const int ar = rows.adjustPosition((int)r->num, refSeq, longId);
  if (ar < 0) {
    cellsDropped++;
    return;
  }
  const int ac = cols.adjustPosition((int)c->num, refSeq, longId);
  if (ac < 0) {
    cellsDropped++;
    return;
  }
  const int rh = rows.getAllocatedHandle(ar);
  const int ch = cols.getAllocatedHandle(ac);
  // no pending local write for an observer (matrix.ts:682): cells.setCell(rowHandle, colHandle, value)
  const JVal* v = obj_get(contents->obj, u"value");
  std::optional<std::string> val;
  if (v && !v->isUndef()) val = json_stringify(*v);
  cells.setCell((uint32_t)rh, (uint32_t)ch, std::move(val));
  cellsSet++;
}

// ---------------------------------------------------------------- SparseArray2D (sparsearray2d.ts)
namespace {
uint32_t interlace8(uint32_t i) {  // x8ToInterlacedX16 (sparsearray2d.ts:8-14)
  uint32_t j = i;
  j = (j | (j << 4)) & 0x0f0f;
  j = (j | (j << 2)) & 0x3333;
  j = (j | (j << 1)) & 0x5555;
  return j;
}
uint32_t interlaceBitsX16(uint32_t x) { return (interlace8((x >> 8) & 0xff) << 16) | interlace8(x & 0xff); }
uint32_t r0ToMorton16(uint32_t row) { return interlaceBitsX16(row) << 1; }
uint32_t c0ToMorton16(uint32_t col) { return interlaceBitsX16(col); }
uint32_t morton2x16(uint32_t row, uint32_t col) { return r0ToMorton16(row) | c0ToMorton16(col); }
inline uint32_t byte0(uint32_t x) { return x >> 24; }
inline uint32_t byte1(uint32_t x) { return (x >> 16) & 0xff; }
inline uint32_t byte2(uint32_t x) { return (x >> 8) & 0xff; }
inline uint32_t byte3(uint32_t x) { return x & 0xff; }
template <class C>
C& getLevel(std::unique_ptr<C>& slot) {  // getLevel (:226-231): new Array(256).fill(undefined)
  if (!slot) slot.reset(new C());
  return *slot;
}
// the 16 keys of a 16x16 tile on one row (forEachKeyInRow :110-114) / col (forEachKeyInCol :116-120)
template <class F> void keysInRow(uint32_t rowBits, F&& f) { for (uint32_t c = 0; c < 16; c++) f(rowBits | c0ToMorton16(c)); }
template <class F> void keysInCol(uint32_t colBits, F&& f) { for (uint32_t r = 0; r < 16; r++) f(r0ToMorton16(r) | colBits); }
}  // namespace

void SparseArray2D::setCell(uint32_t row, uint32_t col, std::optional<std::string> value) {  // :93-103
  const uint32_t keyHi = morton2x16(row >> 16, col >> 16);
  const uint32_t keyLo = morton2x16(row & 0xffff, col & 0xffff);
  if (keyHi >= rootLength) rootLength = (uint64_t)keyHi + 1;  // the JS array grows with holes
  L0& l0 = getLevel(root[keyHi]);
  L1& l1 = getLevel(l0[byte0(keyLo)]);
  L2& l2 = getLevel(l1[byte1(keyLo)]);
  L3& l3 = getLevel(l2[byte2(keyLo)]);
  l3[byte3(keyLo)] = std::move(value);
}
const std::optional<std::string>* SparseArray2D::getCell(uint32_t row, uint32_t col) const {  // :68-88
  const uint32_t keyHi = morton2x16(row >> 16, col >> 16);
  auto it = root.find(keyHi);
  if (it == root.end() || !it->second) return nullptr;
  const uint32_t keyLo = morton2x16(row & 0xffff, col & 0xffff);
  const auto& l1 = (*it->second)[byte0(keyLo)];
  if (!l1) return nullptr;
  const auto& l2 = (*l1)[byte1(keyLo)];
  if (!l2) return nullptr;
  const auto& l3 = (*l2)[byte2(keyLo)];
  if (!l3) return nullptr;
  return &(*l3)[byte3(keyLo)];
}
void SparseArray2D::clearRows(uint32_t rowStart, uint32_t rowCount) {  // :150-174
  for (uint64_t row = rowStart; row < (uint64_t)rowStart + rowCount; row++) {
    const uint32_t rowHi = r0ToMorton16((uint32_t)(row >> 16));
    const uint32_t rowLo = r0ToMorton16((uint32_t)row & 0xffff);
    // the reference scans colHi 0..0xffff; only existing root entries matter
    for (auto& [keyHi, lvl0] : root) {
      if (!lvl0 || ((keyHi & 0xAAAAAAAAu) != rowHi)) continue;
      L0& l0 = *lvl0;
      keysInRow(byte0(rowLo), [&](uint32_t k1) {
        if (!l0[k1]) return;
        L1& l1 = *l0[k1];
        keysInRow(byte1(rowLo), [&](uint32_t k2) {
          if (!l1[k2]) return;
          L2& l2 = *l1[k2];
          keysInRow(byte2(rowLo), [&](uint32_t k3) {
            if (!l2[k3]) return;
            L3& l3 = *l2[k3];
            keysInRow(byte3(rowLo), [&](uint32_t k4) { l3[k4].reset(); });
          });
        });
      });
    }
  }
}
void SparseArray2D::clearCols(uint32_t colStart, uint32_t colCount) {  // :198-224
  for (uint64_t col = colStart; col < (uint64_t)colStart + colCount; col++) {
    const uint32_t colHi = c0ToMorton16((uint32_t)(col >> 16));
    const uint32_t colLo = c0ToMorton16((uint32_t)col & 0xffff);
    for (auto& [keyHi, lvl0] : root) {
      if (!lvl0 || ((keyHi & 0x55555555u) != colHi)) continue;
      L0& l0 = *lvl0;
      keysInCol(byte0(colLo), [&](uint32_t k1) {
        if (!l0[k1]) return;
        L1& l1 = *l0[k1];
        keysInCol(byte1(colLo), [&](uint32_t k2) {
          if (!l1[k2]) return;
          L2& l2 = *l1[k2];
          keysInCol(byte2(colLo), [&](uint32_t k3) {
            if (!l2[k3]) return;
            L3& l3 = *l2[k3];
            keysInCol(byte3(colLo), [&](uint32_t k4) { l3[k4].reset(); });
          });
        });
      });
    }
  }
}
std::string SparseArray2D::snapshotJson() const {  // JSON.stringify(root): holes and undefined -> null
  std::string o = "[";
  auto lvl = [&](auto& self, const auto& arr, auto leafTag) -> void {
    (void)leafTag;
    o += '[';
    for (size_t i = 0; i < 256; i++) {
      if (i) o += ',';
      using E = std::decay_t<decltype(arr[i])>;
      if constexpr (std::is_same_v<E, std::optional<std::string>>) {
        o += arr[i] ? *arr[i] : std::string("null");
      } else {
        if (arr[i]) self(self, *arr[i], 0);
        else o += "null";
      }
    }
    o += ']';
  };
  for (uint64_t k = 0; k < rootLength; k++) {
    if (k) o += ',';
    auto it = root.find((uint32_t)k);
    if (it != root.end() && it->second) lvl(lvl, *it->second, 0);
    else o += "null";
  }
  return o + "]";
}

SparseArray2D SparseArray2D::load(const JVal& data) {
  SparseArray2D a;
  if (data.t != JVal::Arr) throw OracleError(-8, "cells snapshot is not an array");
  a.rootLength = data.arr.size();
  auto level = [](auto& self, const JVal& v, auto& out) -> void {
    using C = std::decay_t<decltype(out)>;
    if (v.t != JVal::Arr) throw OracleError(-8, "cells level is not an array");
    for (size_t i = 0; i < v.arr.size() && i < 256; i++) {
      const JVal& e = v.arr[i];
      if constexpr (std::is_same_v<C, Leaf>) {
        if (e.t != JVal::Null && !e.isUndef()) out[i] = json_stringify(e);
      } else {
        if (e.t == JVal::Null || e.isUndef()) continue;
        using Child = typename std::decay_t<decltype(*out[i])>;
        out[i].reset(new Child());
        self(self, e, *out[i]);
      }
    }
  };
  for (size_t k = 0; k < data.arr.size(); k++) {
    const JVal& e = data.arr[k];
    if (e.t == JVal::Null || e.isUndef()) continue;
    auto& l0 = a.root[(uint32_t)k];
    l0.reset(new L0());
    level(level, e, *l0);
  }
  return a;
}

void MatrixDoc::load(const std::vector<std::pair<std::string, std::string>>& blobs, const std::string& observerId) {
  auto findBlob = [&](const std::string& id) -> const std::string& {
    for (auto& b : blobs)
      if (b.first == id) return b.second;
    throw OracleError(-1, "missing blob " + id);
  };
  for (int v = 0; v < 2; v++) {
    Doc& d = v ? cols : rows;
    const std::string pre = v ? "cols/" : "rows/";
    const JVal ht = json_parse(findBlob(pre + "handleTable"));  // HandleTable.load (handletable.ts:88-90)
    if (ht.t != JVal::Arr || ht.arr.empty()) throw OracleError(-8, "bad handleTable blob");
    d.handles.clear();
    for (auto& h : ht.arr) d.handles.push_back(h.t == JVal::Num ? (int64_t)h.num : 0);
    std::vector<std::pair<std::string, std::string>> seg;
    for (auto& b : blobs)
      if (b.first.rfind(pre + "segments/", 0) == 0) seg.push_back({b.first.substr(pre.size() + 9), b.second});
    d.loadV1(seg, observerId);
  }
  const JVal cd = json_parse(findBlob("cells"));  // [cells.snapshot(), pending.snapshot()]
  if (cd.t != JVal::Arr || cd.arr.size() < 2) throw OracleError(-8, "bad cells blob");
  cells = SparseArray2D::load(cd.arr[0]);
  const SparseArray2D pend = SparseArray2D::load(cd.arr[1]);
  if (pend.snapshotJson() != "[null]") throw OracleError(-6, "unsupported: pending local cell writes in a summary");
}

std::vector<std::pair<std::string, std::string>> MatrixDoc::summarize(std::string* summaryJson) {
  std::string rj, cj;
  auto rb = rows.summarizeV1(&rj);
  auto cb = cols.summarizeV1(&cj);
  const std::string cellsBlob = "[" + cells.snapshotJson() + ",[null]]";  // [cells.snapshot(), pending.snapshot()]
  std::vector<std::pair<std::string, std::string>> blobs;
  for (auto& x : rb) blobs.push_back({"rows/" + x.first, x.second});
  for (auto& x : cb) blobs.push_back({"cols/" + x.first, x.second});
  blobs.push_back({"cells", cellsBlob});
  if (summaryJson) {
    // SummaryTreeBuilder (summaryUtils.ts:138-198): addWithStats merges the vectors' stats, addBlob counts cells
    const JVal r = json_parse(rj.data(), rj.size()), c = json_parse(cj.data(), cj.size());
    auto stat = [](const JVal& v, const char16_t* k) { return (uint64_t)obj_get(obj_get(v.obj, u"stats")->obj, k)->num; };
    std::string cq;
    json_stringify_to(cq, JVal::string(utf8_to_u16(cellsBlob.data(), cellsBlob.size())));
    uint64_t bytes = stat(r, u"totalBlobSize") + stat(c, u"totalBlobSize") + cellsBlob.size();  // UTF-8 bytes (getBlobSize)
    *summaryJson = "{\"summary\":{\"type\":1,\"tree\":{\"rows\":" + json_stringify(*obj_get(r.obj, u"summary")) +
                   ",\"cols\":" + json_stringify(*obj_get(c.obj, u"summary")) + ",\"cells\":{\"type\":2,\"content\":" + cq +
                   "}}},\"stats\":{\"treeNodeCount\":" + std::to_string(1 + stat(r, u"treeNodeCount") + stat(c, u"treeNodeCount")) +
                   ",\"blobNodeCount\":" + std::to_string(1 + stat(r, u"blobNodeCount") + stat(c, u"blobNodeCount")) +
                   ",\"handleNodeCount\":0,\"totalBlobSize\":" + std::to_string(bytes) + ",\"unreferencedBlobSize\":0}}";
  }
  return blobs;
}

// ---------------------------------------------------------------- SnapshotLegacy (snapshotlegacy.ts)
std::vector<std::pair<std::string, std::string>> Doc::summarizeLegacy(const std::string& catchUpJson, std::string* summaryJson) {
  MergeTree& t = mt;
  const int seq = t.window.minSeq;  // extractSync (snapshotlegacy.ts:205-259): everything at the MSN
  const int headerLen = t.getLength(seq, NonCollabClient);
  std::vector<Seg> segs;  // coalesced copies (prev.clone().append(segment.clone()))
  Seg* prevLive = nullptr;
  std::optional<Seg> prevClone;
  auto flushPrev = [&] {
    if (prevClone) segs.push_back(*prevClone);
    else if (prevLive) segs.push_back(*prevLive);
    prevClone.reset();
    prevLive = nullptr;
  };
  t.mapAll(seq, NonCollabClient, [&](Seg* s) {
    if (s->seq != UnassignedSeq && s->seq <= seq && (!s->removed || s->removedSeq == UnassignedSeq || s->removedSeq > seq)) {
      Seg* prev = prevClone ? &*prevClone : prevLive;
      if (prev && canAppend(prev, s) && matchSegProps(prev, s)) {
        Seg c = *prev;
        if (c.props) c.hasPropManager = true;
        c.text += s->text;
        c.cachedLength += s->cachedLength;
        prevClone = std::move(c);
        prevLive = nullptr;
      } else {
        flushPrev();
        prevLive = s;
      }
    }
  });
  flushPrev();
  int totalLength = 0;
  for (Seg& s : segs) {
    totalLength += s.cachedLength;
    if (s.props && s.props->empty()) {  // properties {} -> undefined (mutates the live segment in the reference)
      s.props.reset();
      s.hasPropManager = false;
    }
  }
  // live segments normalized the same way
  t.walkAllSegments([&](Seg* s) {
    if (s->seq != UnassignedSeq && s->seq <= seq && s->props && s->props->empty()) {
      s->props.reset();
      s->hasPropManager = false;
    }
  });
  const int segmentsTotalLength = headerLen != totalLength ? totalLength : headerLen;  // SegmentsTotalLengthMismatch
  const int chunkSize = t.options.chunkSize;
  struct Chunk { int start = 0, count = 0, length = 0; };
  auto take = [&](int approx, int start) {  // getSeqLengthSegs (snapshotlegacy.ts:66-117)
    Chunk c;
    c.start = start;
    while (c.length < approx && start + c.count < (int)segs.size()) c.length += segs[start + c.count++].cachedLength;
    return c;
  };
  const int total = (int)segs.size();
  auto chunkJson = [&](const Chunk& c, bool header) {
    JVal o;
    o.t = JVal::Obj;
    o.obj.push_back({u"chunkStartSegmentIndex", JVal::number(c.start)});
    o.obj.push_back({u"chunkSegmentCount", JVal::number(c.count)});
    o.obj.push_back({u"chunkLengthChars", JVal::number(c.length)});
    o.obj.push_back({u"totalLengthChars", JVal::number(segmentsTotalLength)});
    o.obj.push_back({u"totalSegmentCount", JVal::number(total)});
    o.obj.push_back({u"chunkSequenceNumber", JVal::number(seq)});
    JVal texts;
    texts.t = JVal::Arr;
    for (int i = 0; i < c.count; i++) texts.arr.push_back(segJson(&segs[c.start + i]));
    o.obj.push_back({u"segmentTexts", texts});
    if (header) {  // buildHeaderMetadataForLegacyChunk (snapshotChunks.ts:178-200); minSequenceNumber undefined
      JVal h;
      h.t = JVal::Obj;
      JVal ids;
      ids.t = JVal::Arr;
      ids.arr.push_back(json_parse(std::string("{\"id\":\"header\"}")));
      if (c.length < segmentsTotalLength) ids.arr.push_back(json_parse(std::string("{\"id\":\"body\"}")));
      h.obj.push_back({u"orderedChunkMetadata", ids});
      h.obj.push_back({u"sequenceNumber", JVal::number(seq)});
      h.obj.push_back({u"totalLength", JVal::number(segmentsTotalLength)});
      h.obj.push_back({u"totalSegmentCount", JVal::number(total)});
      o.obj.push_back({u"headerMetadata", h});
    }
    return json_stringify(o);
  };
  // emit (snapshotlegacy.ts:122-203)
  std::vector<std::pair<std::string, std::string>> blobs;
  const Chunk c1 = take(chunkSize, 0);
  blobs.push_back({"header", chunkJson(c1, true)});
  int length = c1.length, count = c1.count;
  if (c1.count < total) {
    const Chunk c2 = take(segmentsTotalLength, c1.count);
    blobs.push_back({"body", chunkJson(c2, false)});
    length += c2.length;
    count += c2.count;
  }
  if (length != segmentsTotalLength) fail_assert("0x05d", "emit: mismatch in segmentsTotalLength");
  if (count != total) fail_assert("0x05e", "emit: mismatch in totalSegmentCount");
  std::string tracked;
  if (catchUpJson.empty() && catchUp) tracked = this->catchUpJson(seq);
  const std::string& cuText = catchUpJson.empty() ? tracked : catchUpJson;
  if (!cuText.empty()) {
    JVal cu = json_parse(cuText);
    if (cu.t == JVal::Arr && !cu.arr.empty()) blobs.push_back({"catchupOps", json_stringify(cu)});
  }
  if (summaryJson) {
    JVal tree;
    tree.t = JVal::Obj;
    int64_t bytes = 0;
    for (auto& b : blobs) {
      JVal blob;
      blob.t = JVal::Obj;
      blob.obj.push_back({u"type", JVal::number(2)});
      blob.obj.push_back({u"content", JVal::string(utf8_to_u16(b.second))});
      obj_set(tree.obj, utf8_to_u16(b.first), blob);
      bytes += utf8ByteLength(b.second);
    }
    JVal summary;
    summary.t = JVal::Obj;
    summary.obj.push_back({u"type", JVal::number(1)});
    summary.obj.push_back({u"tree", tree});
    JVal stats;
    stats.t = JVal::Obj;
    stats.obj.push_back({u"treeNodeCount", JVal::number(1)});
    stats.obj.push_back({u"blobNodeCount", JVal::number((double)blobs.size())});
    stats.obj.push_back({u"handleNodeCount", JVal::number(0)});
    stats.obj.push_back({u"totalBlobSize", JVal::number((double)bytes)});
    stats.obj.push_back({u"unreferencedBlobSize", JVal::number(0)});
    JVal all;
    all.t = JVal::Obj;
    all.obj.push_back({u"summary", summary});
    all.obj.push_back({u"stats", stats});
    *summaryJson = json_stringify(all);
  }
  return blobs;
}

uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

}  // namespace orc
