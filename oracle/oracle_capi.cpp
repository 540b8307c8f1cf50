#include <functional>
// ORACLE / TEST INFRASTRUCTURE ONLY.  C entry points over the CPU restatement, loaded by tests/
// through ctypes (tests/oracle.py) and by bench.py's cpu_baseline leg.  Never linked by the product.
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mt_oracle.hpp"

using namespace orc;

struct orc_doc {
  Doc doc;
  std::string err;
  explicit orc_doc(const Options& o) : doc(o) {}
};

static char* dupstr(const std::string& s, size_t* len) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  if (len) *len = s.size();
  return p;
}

template <class F>
static int guard(orc_doc* d, F&& f) {
  try {
    f();
    return 0;
  } catch (const OracleError& e) {
    d->err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    d->err = e.what();
    return -8;
  }
}

static std::optional<JObj> parseProps(const char* json) {
  if (!json) return std::nullopt;
  JVal v = json_parse(json, strlen(json));
  if (v.t != JVal::Obj) return std::nullopt;
  return propsFromSpec(&v);
}

struct orc_matrix {
  orc_doc rows, cols;
  MatrixDoc m;
  std::string err;
  explicit orc_matrix(const Options& o) : rows(o), cols(o), m(rows.doc, cols.doc) {}
};

extern "C" {

// SharedMatrix observer: two PermutationVector documents (rows = 0, cols = 1) reachable as orc_doc
orc_matrix* orc_matrix_create(int new_length_calc, int chunk_size) {
  Options o;
  o.newLengthCalc = new_length_calc != 0;
  if (chunk_size > 0) o.chunkSize = chunk_size;
  return new orc_matrix(o);
}
void orc_matrix_destroy(orc_matrix* m) { delete m; }
orc_doc* orc_matrix_vector(orc_matrix* m, int which) { return which ? &m->cols : &m->rows; }
const char* orc_matrix_last_error(orc_matrix* m) { return m->err.c_str(); }
int orc_matrix_start_collab(orc_matrix* m, const char* long_id, int min_seq, int cur_seq) {
  return guard(&m->rows, [&] { m->m.startOrUpdateCollaboration(long_id, min_seq, cur_seq); });
}
int orc_matrix_apply_msg_json(orc_matrix* m, const char* json, size_t len) {
  int rc = guard(&m->rows, [&] { m->m.applyMsg(json_parse(json, len)); });
  if (rc) m->err = m->rows.err;
  return rc;
}

// Client.walkSegments / getContainingSegment / getPropertiesAtPosition through mapRange (same JSON as the
// engine's mtb_map_range): [{"pos","start","end","segment":{...}}...]
// Debug view (test infrastructure): one JSON line per block in tree order -- its path, the partial length of each
// child in the (ref_seq, long_id) view next to the child's leaf sum in that view, and the block's main and
// client partial-length sets ([seq, len, seglen]).
int orc_debug_blocks(orc_doc* d, int ref_seq, const char* long_id, char** out, size_t* len) {
  return guard(d, [&] {
    Doc& doc = d->doc;
    MergeTree& t = doc.mt;
    const int R = ref_seq < 0 ? t.window.currentSeq : ref_seq;
    int C = t.window.clientId;
    if (long_id) {
      auto it = doc.longToShort.find(long_id);
      C = it == doc.longToShort.end() ? -3 : it->second;
    }
    std::string o;
    std::function<int(Node*)> leafsum = [&](Node* n) -> int {
      if (n->leaf) {
        const int l = t.nodeLength(n, R, C);
        return l > 0 ? l : 0;
      }
      Block* b = static_cast<Block*>(n);
      int s = 0;
      for (int i = 0; i < b->childCount; i++) s += leafsum(b->children[i]);
      return s;
    };
    auto set_json = [](const PSLSet& st) {
      std::string j = "[";
      for (size_t i = 0; i < st.items.size(); i++) {
        if (i) j += ",";
        j += "[" + std::to_string(st.items[i].seq) + "," + std::to_string(st.items[i].len) + "," +
             std::to_string(st.items[i].seglen) + "]";
      }
      return j + "]";
    };
    std::function<void(Block*, std::string)> visit = [&](Block* b, std::string path) {
      o += "{\"path\":[" + path + "],\"kids\":[";
      for (int i = 0; i < b->childCount; i++) {
        Node* c = b->children[i];
        if (i) o += ",";
        if (c->leaf) o += "null";
        else o += "[" + std::to_string(t.nodeLength(c, R, C)) + "," + std::to_string(leafsum(c)) + "]";
      }
      o += "]";
      if (b->partial) {
        PartialLengths& pl = *b->partial;
        o += ",\"minLength\":" + std::to_string(pl.minLength) + ",\"main\":" + set_json(pl.partialLengths);
        const size_t k = (size_t)(C + 2);
        o += ",\"cli\":" + (k < pl.clientSeqNumbers.size() ? set_json(pl.clientSeqNumbers[k]) : std::string("[]"));
        o += ",\"id\":" + std::to_string(b->id) + ",\"defs\":[";  // (the MTO_DEFCHECK shadow model)
        for (size_t q = 0; q < pl.defs.size(); q++)
          o += std::string(q ? "," : "") + "[" + std::to_string(pl.defs[q].kind) + "," + std::to_string(pl.defs[q].t) + "," +
               std::to_string(pl.defs[q].d) + "," + std::to_string(pl.defs[q].c) + "]";
        o += "]";
      }
      o += "}\n";
      for (int i = 0; i < b->childCount; i++)
        if (!b->children[i]->leaf)
          visit(static_cast<Block*>(b->children[i]), path + (path.empty() ? "" : ",") + std::to_string(i));
    };
    visit(t.root, "");
    *out = dupstr(o, len);
  });
}

int orc_map_range(orc_doc* d, int start, int end, int ref_seq, const char* long_id, unsigned limit, char** out, size_t* len) {
  return guard(d, [&] {
    Doc& doc = d->doc;
    MergeTree& t = doc.mt;
    const int R = ref_seq < 0 ? t.window.currentSeq : ref_seq;
    int C = t.window.clientId;
    if (long_id) {
      auto it = doc.longToShort.find(long_id);
      C = it == doc.longToShort.end() ? -3 : it->second;
    }
    std::string o = "[";
    unsigned n = 0;
    t.mapRange(R, C, start, end, [&](Seg* s, int pos, int st, int en) {
      if (n) o += ',';
      o += "{\"pos\":" + std::to_string(pos) + ",\"start\":" + std::to_string(st) + ",\"end\":" + std::to_string(en) +
           ",\"segment\":{\"type\":";
      if (s->perm) {
        o += "\"PermutationSegment\",\"start\":" + std::to_string(s->start);
      } else if (s->isMarker) {
        o += "\"Marker\",\"refType\":" + (s->refType < 0 ? std::string("null") : std::to_string(s->refType));
      } else {
        o += "\"TextSegment\",\"text\":";
        json_stringify_to(o, JVal::string(s->text));
      }
      o += ",\"cachedLength\":" + std::to_string(s->cachedLength) + ",\"seq\":" + std::to_string(s->seq) +
           ",\"clientId\":" + std::to_string(s->clientId);
      if (s->removed) {
        o += ",\"removedSeq\":" + std::to_string(s->removedSeq) + ",\"removedClientIds\":[";
        for (size_t q = 0; q < s->removedClientIds.size(); q++) o += (q ? "," : "") + std::to_string(s->removedClientIds[q]);
        o += "]";
      }
      if (s->props && !s->props->empty()) {
        JVal pv;
        pv.t = JVal::Obj;
        pv.obj = *s->props;
        o += ",\"properties\":" + json_stringify(pv);
      }
      o += "}}";
      return ++n != limit;
    });
    o += "]";
    *out = dupstr(o, len);
  });
}

// SharedMatrix.summarizeCore (matrix.ts:449-463): {"blobs": [[path, content]...], "summary": ISummaryTreeWithStats}
int orc_matrix_summarize(orc_matrix* m, char** out, size_t* len) {
  int rc = guard(&m->rows, [&] {
    std::string summary;
    auto blobs = m->m.summarize(&summary);
    JVal arr;
    arr.t = JVal::Arr;
    for (auto& b : blobs) {
      JVal pair;
      pair.t = JVal::Arr;
      pair.arr.push_back(JVal::string(utf8_to_u16(b.first)));
      pair.arr.push_back(JVal::string(utf8_to_u16(b.second)));
      arr.arr.push_back(pair);
    }
    std::string s = "{\"blobs\":" + json_stringify(arr) + ",\"summary\":" + summary + "}";
    *out = dupstr(s, len);
  });
  if (rc) m->err = m->rows.err;
  return rc;
}
// SharedMatrix.loadCore (matrix.ts:611-634): blobs = JSON [[path, content]...]
int orc_matrix_load(orc_matrix* m, const char* blobs_json, size_t len, const char* observer) {
  int rc = guard(&m->rows, [&] {
    const JVal a = json_parse(blobs_json, len);
    std::vector<std::pair<std::string, std::string>> blobs;
    for (auto& p : a.arr) blobs.push_back({u16_to_utf8(p.arr[0].str), u16_to_utf8(p.arr[1].str)});
    m->m.load(blobs, observer ? observer : "snapshot");
  });
  if (rc) m->err = m->rows.err;
  return rc;
}
// cells.getCell(rowHandle, colHandle) (sparsearray2d.ts:68-88): JSON text, "" when undefined
int orc_matrix_get_cell_by_handle(orc_matrix* m, uint32_t rh, uint32_t ch, char** out, size_t* len) {
  const std::optional<std::string>* v = m->m.cells.getCell(rh, ch);
  *out = dupstr(v && *v ? **v : std::string(), len);
  return 0;
}

// SharedMatrix.getCell(row, col) (matrix.ts:173-189): local positions -> handles -> cells; "" = undefined
int orc_matrix_get_cell(orc_matrix* m, uint32_t row, uint32_t col, char** out, size_t* len) {
  int rc = guard(&m->rows, [&] {
    auto handleAt = [](Doc& d, int pos) {
      int off = 0;
      Seg* s = d.mt.containingSegment(pos, d.mt.window.currentSeq, d.mt.window.clientId, &off);
      if (!s) throw OracleError(-1, "0x027 position out of range");
      return s->start >= 1 ? s->start + off : HandleUnallocated;
    };
    const int rh = handleAt(m->rows.doc, (int)row);
    const int ch = handleAt(m->cols.doc, (int)col);
    std::string v;
    if (rh != HandleUnallocated && ch != HandleUnallocated) {
      const std::optional<std::string>* c = m->m.cells.getCell((uint32_t)rh, (uint32_t)ch);
      if (c && *c) v = **c;
    }
    *out = dupstr(v, len);
  });
  if (rc) m->err = m->rows.err;
  return rc;
}

// SparseArray2D on its own (sparsearray2d.spec.ts cases)
SparseArray2D* orc_sa2d_create() { return new SparseArray2D(); }
void orc_sa2d_destroy(SparseArray2D* a) { delete a; }
void orc_sa2d_set(SparseArray2D* a, uint32_t r, uint32_t c, const char* json) {
  a->setCell(r, c, json ? std::optional<std::string>(json) : std::nullopt);
}
int orc_sa2d_get(SparseArray2D* a, uint32_t r, uint32_t c, char* buf, size_t cap) {  // -1 undefined, else length
  const std::optional<std::string>* v = a->getCell(r, c);
  if (!v || !*v) return -1;
  snprintf(buf, cap, "%s", (*v)->c_str());
  return (int)(*v)->size();
}
void orc_sa2d_clear_rows(SparseArray2D* a, uint32_t s, uint32_t n) { a->clearRows(s, n); }
void orc_sa2d_clear_cols(SparseArray2D* a, uint32_t s, uint32_t n) { a->clearCols(s, n); }
char* orc_sa2d_snapshot(SparseArray2D* a, size_t* len) { return dupstr(a->snapshotJson(), len); }

orc_doc* orc_create(int new_length_calc, int chunk_size, int verify) {
  Options o;
  o.newLengthCalc = new_length_calc != 0;
  if (chunk_size > 0) o.chunkSize = chunk_size;
  o.verify = verify != 0;
  return new orc_doc(o);
}
void orc_destroy(orc_doc* d) { delete d; }
const char* orc_last_error(orc_doc* d) { return d->err.c_str(); }
void orc_free(void* p) { free(p); }

int orc_insert_text_local(orc_doc* d, int pos, const char* utf8, const char* props_json) {
  return guard(d, [&] { d->doc.insertTextLocal(pos, utf8_to_u16(utf8, strlen(utf8)), parseProps(props_json)); });
}
int orc_insert_marker_local(orc_doc* d, int pos, int ref_type, const char* props_json) {
  return guard(d, [&] { d->doc.insertMarkerLocal(pos, ref_type, parseProps(props_json)); });
}
int orc_annotate_local(orc_doc* d, int start, int end, const char* props_json) {
  return guard(d, [&] {
    JVal v = json_parse(props_json, strlen(props_json));
    d->doc.annotateRangeLocal(start, end, v.t == JVal::Obj ? v.obj : JObj());
  });
}
int orc_remove_local(orc_doc* d, int start, int end) {
  return guard(d, [&] { d->doc.removeRangeLocal(start, end); });
}
// a live client's local ops (client.ts:196-247): the op JSON to submit ("" when nothing was inserted)
int orc_local_insert(orc_doc* d, int pos, const char* seg_json, char** out, size_t* len) {
  return guard(d, [&] { *out = dupstr(d->doc.insertLocalOp(pos, json_parse(seg_json, strlen(seg_json))), len); });
}
int orc_local_remove(orc_doc* d, int start, int end, char** out, size_t* len) {
  return guard(d, [&] { *out = dupstr(d->doc.removeLocalOp(start, end), len); });
}
int orc_local_annotate(orc_doc* d, int start, int end, const char* props_json, char** out, size_t* len) {
  return guard(d, [&] {
    JVal v = json_parse(props_json, strlen(props_json));
    *out = dupstr(d->doc.annotateLocalOp(start, end, v.t == JVal::Obj ? v.obj : JObj()), len);
  });
}
int orc_pending_groups(orc_doc* d) { return (int)d->doc.mt.pendingSegments.size(); }
int orc_local_op_json(orc_doc* d, const char* op_json, char** out, size_t* len) {
  return guard(d, [&] { *out = dupstr(d->doc.localOpJson(json_parse(op_json, strlen(op_json))), len); });
}
// Client.regeneratePendingOp (client.ts:917-960) for the op at the head of the pending queue
int orc_regenerate(orc_doc* d, const char* op_json, char** out, size_t* len) {
  return guard(d, [&] { *out = dupstr(d->doc.regeneratePendingOp(json_parse(op_json, strlen(op_json))), len); });
}
int orc_start_collab(orc_doc* d, const char* long_id, int min_seq, int cur_seq) {
  return guard(d, [&] { d->doc.startOrUpdateCollaboration(long_id, min_seq, cur_seq); });
}
int orc_apply_msg_json(orc_doc* d, const char* json, size_t len) {
  return guard(d, [&] { d->doc.applyMsg(json_parse(json, len)); });
}
// Binary records (include/mtb.h layout). props_json: array of n_props NUL-terminated JSON strings.
int orc_apply_records(orc_doc* d, const void* ops, uint32_t n, const uint16_t* text, const char* const* props_json,
                      uint32_t n_props) {
  return guard(d, [&] {
    std::vector<std::string> props(n_props);
    for (uint32_t i = 0; i < n_props; i++) props[i] = props_json[i] ? props_json[i] : "";
    const Doc::Record* r = static_cast<const Doc::Record*>(ops);
    for (uint32_t i = 0; i < n; i++) d->doc.applyRecord(r[i], text, props);
  });
}
int orc_add_client(orc_doc* d, const char* long_id) {
  return guard(d, [&] { d->doc.getOrAddShortClientId(long_id); });
}
int orc_update_seq(orc_doc* d, int min_seq, int seq) {
  return guard(d, [&] { d->doc.updateSeqNumbers(min_seq, seq); });
}
// UTF-16 text (engine-allocated)
int orc_get_text(orc_doc* d, uint16_t** out, size_t* n_units) {
  return guard(d, [&] {
    u16str t = d->doc.mt.getText();
    uint16_t* p = (uint16_t*)malloc((t.size() + 1) * 2);
    memcpy(p, t.data(), t.size() * 2);
    *out = p;
    *n_units = t.size();
  });
}
int orc_get_length(orc_doc* d) { return d->doc.mt.length(); }
// posFromRelativePos (mergeTree.ts:1371-1395) of a JSON IRelativePosition in the (ref_seq, client) view;
// -1 when the id names no marker, INT32_MIN on a malformed argument
int orc_pos_from_relative(orc_doc* d, const char* rel_json, int ref_seq, int client) {
  int pos = INT32_MIN;
  guard(d, [&] { pos = d->doc.mt.posFromRelativePos(json_parse(rel_json, strlen(rel_json)), ref_seq, client); });
  return pos;
}
int orc_get_remote_length(orc_doc* d, int ref_seq, int client) { return d->doc.mt.getLength(ref_seq, client); }
int orc_current_seq(orc_doc* d) { return d->doc.mt.window.currentSeq; }
int orc_min_seq(orc_doc* d) { return d->doc.mt.window.minSeq; }
int orc_num_clients(orc_doc* d) { return (int)d->doc.longIds.size(); }
const char* orc_client_long_id(orc_doc* d, int i) { return d->doc.longIds.at(i).c_str(); }
uint64_t orc_ops_applied(orc_doc* d) { return d->doc.mt.counters.ops; }
uint64_t orc_segs_touched(orc_doc* d) { return d->doc.mt.counters.segsTouched; }
uint64_t orc_stale_updates(orc_doc* d) { return d->doc.mt.counters.staleUpdates; }
uint64_t orc_stale_deficits(orc_doc* d) { return d->doc.mt.counters.staleDeficits; }

// Summary: returns a JSON object {"blobs":[[path, content],...], "summary": <ISummaryTreeWithStats>}
int orc_summarize_v1(orc_doc* d, int msn, int seq, char** out, size_t* len) {
  return guard(d, [&] {
    if (msn >= 0 && seq >= 0) d->doc.updateSeqNumbers(msn, seq);
    std::string summary;
    auto blobs = d->doc.summarizeV1(&summary);
    JVal arr;
    arr.t = JVal::Arr;
    for (auto& b : blobs) {
      JVal pair;
      pair.t = JVal::Arr;
      pair.arr.push_back(JVal::string(utf8_to_u16(b.first)));
      pair.arr.push_back(JVal::string(utf8_to_u16(b.second)));
      arr.arr.push_back(pair);
    }
    std::string s = "{\"blobs\":" + json_stringify(arr) + ",\"summary\":" + summary + "}";
    *out = dupstr(s, len);
  });
}
// Client.summarize without newMergeTreeSnapshotFormat (client.ts:999-1003): SnapshotLegacy
int orc_summarize_legacy(orc_doc* d, int msn, int seq, const char* catchup_json, char** out, size_t* len) {
  return guard(d, [&] {
    if (msn >= 0 && seq >= 0) d->doc.updateSeqNumbers(msn, seq);
    std::string summary;
    auto blobs = d->doc.summarizeLegacy(catchup_json ? catchup_json : "", &summary);
    JVal arr;
    arr.t = JVal::Arr;
    for (auto& b : blobs) {
      JVal pair;
      pair.t = JVal::Arr;
      pair.arr.push_back(JVal::string(utf8_to_u16(b.first)));
      pair.arr.push_back(JVal::string(utf8_to_u16(b.second)));
      arr.arr.push_back(pair);
    }
    std::string s = "{\"blobs\":" + json_stringify(arr) + ",\"summary\":" + summary + "}";
    *out = dupstr(s, len);
  });
}
// SharedSegmentSequence without newMergeTreeSnapshotFormat keeps messagesSinceMSNChange (sequence.ts:697)
void orc_enable_catch_up(orc_doc* d) { d->doc.catchUp = true; }
int orc_dump_segments(orc_doc* d, char** out, size_t* len) {
  return guard(d, [&] { *out = dupstr(d->doc.dumpSegments(), len); });
}
uint64_t orc_checksum(orc_doc* d) { return fnv1a64(d->doc.dumpSegments()); }
uint64_t orc_digest(orc_doc* d) { return d->doc.digest(); }
// direct zamboniSegments / packParent(root) calls (the reference's zamboni tests, mergeTree.zamboni.spec.ts)
int orc_zamboni(orc_doc* d) {
  return guard(d, [&] { d->doc.mt.zamboniSegments(); });
}
int orc_pack_parent_root(orc_doc* d) {
  return guard(d, [&] { d->doc.mt.packParentRoot(); });
}
// Client.load of a SnapshotV1 or SnapshotLegacy summary: blobs_json = [[path, content], ...] (as
// orc_summarize_v1 / orc_summarize_legacy return); *out = the catch-up messages blob ("[]" when none)
int orc_load_v1(orc_doc* d, const char* blobs_json, size_t len, const char* observer_id, char** out, size_t* out_len) {
  return guard(d, [&] {
    JVal v = json_parse(blobs_json, len);
    std::vector<std::pair<std::string, std::string>> blobs;
    for (auto& p : v.arr) blobs.push_back({u16_to_utf8(p.arr[0].str), u16_to_utf8(p.arr[1].str)});
    d->doc.loadV1(blobs, observer_id);
    *out = dupstr(Doc::catchUpOps(blobs), out_len);
  });
}

}  // extern "C"
