// ORACLE / TEST INFRASTRUCTURE ONLY — deterministic synthetic op-log generator.
//
// Every op is generated in its author's (refSeq, client) perspective and is therefore valid by
// construction: the generator drives the CPU oracle as the observer and asks it for
// getLength(refSeq, client) (mergeTree.ts:757) before picking positions, exactly like the
// reference farms pick positions in the author's local view (mergeTreeOperationRunner.ts:71-82,
// 253-300).  The records it emits use the engine's mtb_op layout (include/mtb.h); every record is
// applied to the oracle through Doc::applyRecord as it is generated, so the oracle's final state
// (checksum, text, counters) is the expected result of replaying the emitted log.
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "mt_oracle.hpp"

using namespace orc;

namespace {

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0; }      // U{0..n-1}
  uint32_t range(uint32_t a, uint32_t b) { return a + below(b - a + 1); }     // U{a..b}
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

}  // namespace

extern "C" {

// Configuration (mirrors bench/test parameters; all fields are plain ints for ctypes).
struct loggen_cfg {
  uint64_t seed;          // config seed (SURVEY: hash(configId, docId) -> per-doc seed)
  int32_t n_clients;      // K writers (short ids 1..K in first-seen order; 0 is the observer)
  int32_t n_ops;          // messages per document
  int32_t lag;            // L: refSeq lag bound
  int32_t initial_len;    // initial detached text length (UTF-16 units)
  int32_t pct_insert;     // op mix (percent); remainder of 100 after insert/remove = annotate
  int32_t pct_remove;
  int32_t pct_group;      // percent of messages that are GROUP{insert, annotate-inserted-range}
  int32_t new_length_calc;
  int32_t min_length;     // insert whenever the author's view is shorter than this
  int32_t annotate_keys;  // number of distinct annotate keys (>=1); key 0 is "client"
  int32_t pct_set;        // matrix logs: percent of messages that are setCell
  int32_t max_count;      // matrix logs: rows/cols per insert/remove (1..max_count)
};

// Per-matrix output (SharedMatrix logs): the records of each PermutationVector (0 rows, 1 cols), with
// setCell records present in both.  Free with loggen_matrix_free.
struct loggen_matrix {
  void* ops[2];
  uint32_t n_ops[2];
  uint32_t n_msgs;
  uint32_t n_sets;
  uint16_t client_writer[2][256];  // per vector: short id -> writer index (0 = observer)
  uint32_t n_short[2];
  uint64_t checksum[2];            // oracle's final canonical dump checksums
  int32_t error;
  uint64_t digest[2];              // oracle's final state digests v1 of the two vectors (Doc::digest)
  uint64_t summary_fnv;            // FNV-1a 64 of SharedMatrix.summarizeCore's blobs (each blob's path, 0, content,
                                   // 0): mtb_blob_list_fnv without the ISummaryTreeWithStats JSON (whose stats the
                                   // GPU tests compare as parsed objects)
};

// Per-document output.  All arrays are malloc'd; free with loggen_free.
struct loggen_doc {
  void* ops;              // mtb_op records (32 B each)
  uint32_t n_ops;         // records (GROUP members flattened)
  uint32_t n_msgs;        // messages
  uint16_t* text;         // payload arena (UTF-16); initial text at [0, initial_len)
  uint32_t n_text;
  uint32_t initial_len;
  uint16_t client_writer[256];  // short id -> writer index (0 = observer)
  uint32_t n_short;       // short ids assigned (observer included)
  uint64_t checksum;      // oracle's final state checksum (FNV-1a over canonical dump)
  uint64_t ops_applied;   // delta ops applied
  uint64_t segs_touched;  // n_mod counter
  uint32_t final_len;
  uint32_t final_segments;
  int32_t error;
  uint64_t digest;        // oracle's final state digest v1 (Doc::digest, DESIGN.md "State digest")
  uint64_t summary_fnv;   // FNV-1a 64 of the final SnapshotV1 summary (each blob's path, 0, content, 0; then
                          // the ISummaryTreeWithStats JSON), the engine's mtb_blob_list_fnv definition
};

}  // extern "C"

// Props table shared by every generated log: id -> JSON text.
static std::vector<std::string> props_table(int nclients, int nkeys) {
  std::vector<std::string> t;
  t.push_back("");                 // 0: none
  t.push_back("{\"bold\":true}");  // 1
  t.push_back("{\"bold\":null}");  // 2
  for (int w = 0; w <= nclients; w++) {   // 3 + w: {"client": tag}
    char buf[64];
    if (w < 26) snprintf(buf, sizeof buf, "{\"client\":\"%c\"}", 'A' + w);
    else snprintf(buf, sizeof buf, "{\"client\":\"%c%d\"}", 'A' + (w % 26), w / 26);  // unique beyond 26 writers
    t.push_back(buf);
  }
  for (int k = 1; k < nkeys; k++)        // extra keys for annotate-heavy configs
    for (int v = 0; v < 4; v++) {
      char buf[64];
      snprintf(buf, sizeof buf, "{\"k%d\":%d}", k, v);
      t.push_back(buf);
    }
  return t;
}

static std::vector<std::optional<JVal>> parse_table(const std::vector<std::string>& t) {
  std::vector<std::optional<JVal>> p(t.size());
  for (size_t i = 1; i < t.size(); i++) p[i] = json_parse(t[i]);
  return p;
}

static int gen_one(const loggen_cfg& cfg, uint32_t docIndex, loggen_doc* out) {
  memset(out, 0, sizeof *out);
  const int K = cfg.n_clients;
  if (K < 1 || K > 250) return -1;
  std::vector<std::optional<JVal>> props = parse_table(props_table(K, std::max(1, cfg.annotate_keys)));
  SplitMix64 rng(cfg.seed * 0x9E3779B97F4A7C15ull ^ (0xD1B54A32D192ED03ull * (docIndex + 1)));
  SplitMix64 seeder(rng.next());
  rng = SplitMix64(seeder.next());

  Options o;
  o.newLengthCalc = cfg.new_length_calc != 0;
  Doc doc(o);
  std::vector<uint16_t> text;
  std::vector<Doc::Record> recs;
  // initial text
  for (int i = 0; i < cfg.initial_len; i++) text.push_back((uint16_t)('a' + rng.below(26)));
  try {
    if (cfg.initial_len > 0)
      doc.insertTextLocal(0, u16str(reinterpret_cast<const char16_t*>(text.data()), text.size()), std::nullopt);
    doc.startOrUpdateCollaboration("obs", 0, 0);
    doc.mt.counters = Counters{};  // count the sequenced ops only (the detached initial insert is not one)
    out->client_writer[0] = 0;
    std::vector<int> shortOf(K + 1, -1);
    std::vector<uint32_t> refSeq(K + 1, 0);
    uint32_t cur = 0;
    int nshort = 1;
    for (int m = 0; m < cfg.n_ops; m++) {
      int w = (int)rng.range(1, K);
      uint32_t lagv = rng.below((uint32_t)cfg.lag + 1);
      uint32_t cand = cur > lagv ? cur - lagv : 0;
      if (cand > refSeq[w]) refSeq[w] = cand;
      if (shortOf[w] < 0) {
        shortOf[w] = nshort;
        out->client_writer[nshort] = (uint16_t)w;
        nshort++;
        doc.getOrAddShortClientId("c" + std::to_string(w));
      }
      const uint16_t c = (uint16_t)shortOf[w];
      const uint32_t r = refSeq[w];
      const uint32_t seq = cur + 1;
      uint32_t msn = UINT32_MAX;
      for (int k = 1; k <= K; k++) msn = std::min(msn, refSeq[k]);
      int len = doc.mt.getLength((int)r, c);
      uint32_t roll = rng.below(100);
      int type;
      if (len < std::max(1, cfg.min_length) || roll < (uint32_t)cfg.pct_insert) type = 0;
      else if (roll < (uint32_t)(cfg.pct_insert + cfg.pct_remove)) type = 1;
      else type = 2;
      bool group = type == 0 && rng.below(100) < (uint32_t)cfg.pct_group;
      auto base = [&](uint8_t t, uint8_t flags) {
        Doc::Record rec{};
        rec.type = t;
        rec.flags = flags;
        rec.client = c;
        rec.seq = seq;
        rec.refSeq = r;
        rec.msn = msn;
        return rec;
      };
      auto pickProps = [&]() -> uint32_t {
        uint32_t x = rng.below(10);
        if (cfg.annotate_keys > 1 && rng.below(2) == 0) {
          uint32_t k = rng.range(1, (uint32_t)cfg.annotate_keys - 1);
          return 3 + (uint32_t)(K + 1) + (k - 1) * 4 + rng.below(4);
        }
        if (x < 6) return 3 + (uint32_t)w;   // {"client": tag}
        if (x < 9) return 1;                 // {"bold": true}
        return 2;                            // {"bold": null}
      };
      if (type == 0) {
        uint32_t pos = rng.below((uint32_t)len + 1);
        uint32_t off = (uint32_t)text.size();
        uint32_t n;
        if (rng.below(2) == 0) {
          n = rng.range(1, 3);
          for (uint32_t i = 0; i < n; i++) text.push_back((uint16_t)('A' + (w % 26)));
        } else {
          n = rng.range(1, 8);
          for (uint32_t i = 0; i < n; i++) text.push_back((uint16_t)(' ' + rng.below(95)));
        }
        Doc::Record ins = base(0, group ? 0 : 0x01);
        ins.pos1 = pos;
        ins.pos2 = n;
        ins.payload = off;
        recs.push_back(ins);
        doc.applyRecordParsed(ins, text.data(), props);
        if (group) {
          Doc::Record an = base(2, 0x01);
          an.pos1 = pos;
          an.pos2 = pos + n;
          an.props = pickProps();
          recs.push_back(an);
          doc.applyRecordParsed(an, text.data(), props);
        }
      } else {
        uint32_t start = rng.below((uint32_t)len);
        double u = rng.unit();
        uint32_t span = 1 + (uint32_t)std::floor(-std::log(1.0 - u) * 2.0);
        uint32_t end = std::min<uint32_t>((uint32_t)len, start + span);
        Doc::Record rec = base((uint8_t)type, 0x01);
        rec.pos1 = start;
        rec.pos2 = end;
        if (type == 2) rec.props = pickProps();
        recs.push_back(rec);
        doc.applyRecordParsed(rec, text.data(), props);
      }
      cur = seq;
      out->n_msgs++;
    }
    out->n_short = (uint32_t)nshort;
  } catch (const OracleError& e) {
    fprintf(stderr, "loggen doc %u: %s\n", docIndex, e.what());
    out->error = e.code;
    return e.code;
  }
  out->n_ops = (uint32_t)recs.size();
  out->ops = malloc(recs.size() * sizeof(Doc::Record) + 1);
  memcpy(out->ops, recs.data(), recs.size() * sizeof(Doc::Record));
  out->n_text = (uint32_t)text.size();
  out->text = (uint16_t*)malloc(text.size() * 2 + 2);
  memcpy(out->text, text.data(), text.size() * 2);
  out->initial_len = (uint32_t)cfg.initial_len;
  std::string dump = doc.dumpSegments();
  out->checksum = fnv1a64(dump);
  out->digest = doc.digest();
  {
    std::string summary;
    const auto blobs = doc.summarizeV1(&summary);
    uint64_t h = 1469598103934665603ull;
    auto add = [&](const std::string& x, bool zero) {
      for (unsigned char c : x) {
        h ^= c;
        h *= 1099511628211ull;
      }
      if (zero) h *= 1099511628211ull;  // (FNV-1a of a 0 byte: xor 0, multiply)
    };
    for (auto& bl : blobs) {
      add(bl.first, true);
      add(bl.second, true);
    }
    add(summary, false);
    out->summary_fnv = h;
  }
  out->ops_applied = doc.mt.counters.ops;
  out->segs_touched = doc.mt.counters.segsTouched;
  out->final_len = (uint32_t)doc.mt.length();
  uint32_t segs = 0;
  for (char ch : dump) segs += ch == '\n';
  out->final_segments = segs - 1;
  return 0;
}

extern "C" {

static_assert(sizeof(Doc::Record) == 32, "record layout must match mtb_op");

int loggen_generate(const loggen_cfg* cfg, uint32_t doc_index, loggen_doc* out) {
  return gen_one(*cfg, doc_index, out);
}

// Generate docs [doc_begin, doc_end) with `threads` worker threads into out[0..n).
int loggen_generate_batch(const loggen_cfg* cfg, uint32_t doc_begin, uint32_t doc_end, int threads, loggen_doc* out) {
  uint32_t n = doc_end - doc_begin;
  if (threads < 1) threads = 1;
  std::vector<std::thread> ts;
  std::vector<int> rcs(threads, 0);
  for (int t = 0; t < threads; t++) {
    ts.emplace_back([&, t] {
      for (uint32_t i = t; i < n; i += threads) {
        int rc = gen_one(*cfg, doc_begin + i, &out[i]);
        if (rc) rcs[t] = rc;
      }
    });
  }
  for (auto& th : ts) th.join();
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

// ---- SharedMatrix logs: row/col inserts and removes of 1..max_count and setCell,
// every op valid in its author's view; the generator's oracle is a MatrixDoc observer fed the messages.
static JVal jobj(std::initializer_list<std::pair<const char16_t*, JVal>> kv) {
  JVal o;
  o.t = JVal::Obj;
  for (auto& p : kv) o.obj.push_back({p.first, p.second});
  return o;
}
static int gen_matrix_one(const loggen_cfg& cfg, uint32_t index, loggen_matrix* out) {
  memset(out, 0, sizeof *out);
  const int K = cfg.n_clients;
  if (K < 1 || K > 250) return -1;
  SplitMix64 rng(cfg.seed * 0x9E3779B97F4A7C15ull ^ (0xA24BAED4963EE407ull * (index + 1)));
  SplitMix64 seeder(rng.next());
  rng = SplitMix64(seeder.next());
  Options o;
  o.newLengthCalc = cfg.new_length_calc != 0;
  Doc rowsDoc(o), colsDoc(o);
  MatrixDoc mat(rowsDoc, colsDoc);
  std::vector<Doc::Record> recs[2];
  try {
    mat.startOrUpdateCollaboration("obs", 0, 0);
    std::vector<int> vshort[2] = {std::vector<int>(K + 1, -1), std::vector<int>(K + 1, -1)};
    for (int v = 0; v < 2; v++) {
      vshort[v][0] = 0;
      out->client_writer[v][0] = 0;
      out->n_short[v] = 1;
    }
    auto shortIn = [&](int v, int w) {
      if (vshort[v][w] < 0) {
        vshort[v][w] = (int)out->n_short[v];
        out->client_writer[v][out->n_short[v]++] = (uint16_t)w;
      }
      return (uint16_t)vshort[v][w];
    };
    std::vector<uint32_t> refSeq(K + 1, 0);
    uint32_t cur = 0;
    const int maxc = std::max(1, cfg.max_count);
    for (int m = 0; m < cfg.n_ops; m++) {
      const int w = (int)rng.range(1, K);
      const std::string name = "c" + std::to_string(w);
      const uint32_t lagv = rng.below((uint32_t)cfg.lag + 1);
      const uint32_t cand = cur > lagv ? cur - lagv : 0;
      if (cand > refSeq[w]) refSeq[w] = cand;
      const uint32_t r = refSeq[w], seq = cur + 1;
      uint32_t msn = UINT32_MAX;
      for (int k = 1; k <= K; k++) msn = std::min(msn, refSeq[k]);
      // (the records' short ids follow the documents' own interning order, so state digests agree)
      shortIn(0, w);
      shortIn(1, w);
      const int rl = rowsDoc.mt.getLength((int)r, rowsDoc.getOrAddShortClientId(name));
      const int cl = colsDoc.mt.getLength((int)r, colsDoc.getOrAddShortClientId(name));
      JVal contents;
      Doc::Record rec{};
      rec.seq = seq;
      rec.refSeq = r;
      rec.msn = msn;
      if ((int)rng.below(100) < cfg.pct_set && rl > 0 && cl > 0) {
        const uint32_t row = rng.below((uint32_t)rl), col = rng.below((uint32_t)cl);
        contents = jobj({{u"type", JVal::number(2)}, {u"row", JVal::number(row)}, {u"col", JVal::number(col)},
                         {u"value", JVal::number(m)}});
        rec.type = 6;  // MTB_OP_SETCELL, no updateSeqNumbers
        rec.props = (uint32_t)m + 1;  // the value's id when the engine interns "0", "1", ... first (matrix_value_ids)
        for (int v = 0; v < 2; v++) {
          Doc::Record x = rec;
          x.client = shortIn(v, w);
          x.pos1 = v ? col : row;
          x.pos2 = 0;  // the observer's short id
          recs[v].push_back(x);
        }
        out->n_sets++;
      } else {
        const int v = (int)rng.below(2);
        const int ln = v ? cl : rl;
        const char16_t* target = v ? u"cols" : u"rows";
        if (ln == 0 || rng.below(100) < 60) {
          const uint32_t pos = rng.below((uint32_t)ln + 1), cnt = rng.range(1, (uint32_t)maxc);
          JVal seg;
          seg.t = JVal::Arr;
          seg.arr.push_back(JVal::number(cnt));
          seg.arr.push_back(JVal::number(HandleUnallocated));
          contents = jobj({{u"type", JVal::number(0)}, {u"pos1", JVal::number(pos)}, {u"seg", seg},
                           {u"target", JVal::string(target)}});
          rec.type = 0;
          rec.flags = 0x01 | 0x40;  // MTB_F_LAST | MTB_F_PERMSEG
          rec.pos1 = pos;
          rec.pos2 = cnt;
        } else {
          const uint32_t p1 = rng.below((uint32_t)ln);
          const uint32_t p2 = std::min<uint32_t>((uint32_t)ln, p1 + rng.range(1, (uint32_t)maxc));
          contents = jobj({{u"type", JVal::number(1)}, {u"pos1", JVal::number(p1)}, {u"pos2", JVal::number(p2)},
                           {u"target", JVal::string(target)}});
          rec.type = 1;
          rec.flags = 0x01;
          rec.pos1 = p1;
          rec.pos2 = p2;
        }
        rec.client = shortIn(v, w);
        recs[v].push_back(rec);
      }
      JVal msg = jobj({{u"clientId", JVal::string(utf8_to_u16(name))}, {u"sequenceNumber", JVal::number(seq)},
                       {u"referenceSequenceNumber", JVal::number(r)}, {u"minimumSequenceNumber", JVal::number(msn)},
                       {u"type", JVal::string(u"op")}, {u"contents", contents}});
      mat.applyMsg(msg);
      cur = seq;
      out->n_msgs++;
    }
  } catch (const OracleError& e) {
    fprintf(stderr, "loggen matrix %u: %s\n", index, e.what());
    out->error = e.code;
    return e.code;
  }
  for (int v = 0; v < 2; v++) {
    out->n_ops[v] = (uint32_t)recs[v].size();
    out->ops[v] = malloc(recs[v].size() * sizeof(Doc::Record) + 1);
    memcpy(out->ops[v], recs[v].data(), recs[v].size() * sizeof(Doc::Record));
  }
  out->checksum[0] = fnv1a64(rowsDoc.dumpSegments());
  out->checksum[1] = fnv1a64(colsDoc.dumpSegments());
  out->digest[0] = rowsDoc.digest();
  out->digest[1] = colsDoc.digest();
  {
    std::string summary;
    uint64_t h = 1469598103934665603ull;
    auto add = [&](const std::string& x) {
      for (unsigned char c : x) {
        h ^= c;
        h *= 1099511628211ull;
      }
      h *= 1099511628211ull;  // (a 0 byte)
    };
    for (auto& bl : mat.summarize(&summary)) {
      add(bl.first);
      add(bl.second);
    }
    out->summary_fnv = h;
  }
  return 0;
}

int loggen_matrix_generate_batch(const loggen_cfg* cfg, uint32_t begin, uint32_t end, int threads, loggen_matrix* out) {
  const uint32_t n = end - begin;
  if (threads < 1) threads = 1;
  std::vector<std::thread> ts;
  std::vector<int> rcs(threads, 0);
  for (int t = 0; t < threads; t++)
    ts.emplace_back([&, t] {
      for (uint32_t i = t; i < n; i += threads) {
        const int rc = gen_matrix_one(*cfg, begin + i, &out[i]);
        if (rc) rcs[t] = rc;
      }
    });
  for (auto& th : ts) th.join();
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

void loggen_matrix_free(loggen_matrix* m) {
  for (int v = 0; v < 2; v++) {
    free(m->ops[v]);
    m->ops[v] = nullptr;
  }
}

// CPU baseline for matrix logs: the oracle replays each vector's records; setCell records of the two
// streams pair up in order (adjust rows, adjust cols, allocate both when both survive).
static void matrix_cpu_one(const loggen_cfg& cfg, const loggen_matrix& m, uint64_t ck[2]) {
  Options o;
  o.newLengthCalc = cfg.new_length_calc != 0;
  Doc rows(o), cols(o);
  MatrixDoc mat(rows, cols);
  mat.startOrUpdateCollaboration("obs", 0, 0);
  Doc* vec[2] = {&rows, &cols};
  for (int v = 0; v < 2; v++)
    for (uint32_t s = 1; s < m.n_short[v]; s++) vec[v]->getOrAddShortClientId("c" + std::to_string(m.client_writer[v][s]));
  const Doc::Record* r[2] = {static_cast<const Doc::Record*>(m.ops[0]), static_cast<const Doc::Record*>(m.ops[1])};
  uint32_t k[2] = {0, 0};
  static const std::vector<std::optional<JVal>> noProps(1);
  while (k[0] < m.n_ops[0] || k[1] < m.n_ops[1]) {
    for (int v = 0; v < 2; v++)
      while (k[v] < m.n_ops[v] && r[v][k[v]].type != 6) vec[v]->applyRecordParsed(r[v][k[v]++], nullptr, noProps);
    if (k[0] >= m.n_ops[0] || k[1] >= m.n_ops[1]) continue;
    const Doc::Record& a = r[0][k[0]++];
    const Doc::Record& b = r[1][k[1]++];
    const int ar = rows.adjustPosition((int)a.pos1, (int)a.refSeq, rows.getLongClientId(a.client));
    if (ar < 0) continue;
    const int ac = cols.adjustPosition((int)b.pos1, (int)b.refSeq, cols.getLongClientId(b.client));
    if (ac < 0) continue;
    rows.getAllocatedHandle(ar);
    cols.getAllocatedHandle(ac);
  }
  ck[0] = fnv1a64(rows.dumpSegments());
  ck[1] = fnv1a64(cols.dumpSegments());
}

double loggen_matrix_cpu_replay(const loggen_cfg* cfg, const loggen_matrix* mats, uint32_t n, int threads, int32_t* mismatches) {
  if (threads < 1) threads = 1;
  std::vector<int> bad(threads, 0);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; t++)
    ts.emplace_back([&, t] {
      for (uint32_t i = t; i < n; i += threads) {
        uint64_t ck[2];
        try {
          matrix_cpu_one(*cfg, mats[i], ck);
          if (ck[0] != mats[i].checksum[0] || ck[1] != mats[i].checksum[1]) bad[t]++;
        } catch (const OracleError&) {
          bad[t]++;
        }
      }
    });
  for (auto& th : ts) th.join();
  auto t1 = std::chrono::steady_clock::now();
  int b = 0;
  for (int v : bad) b += v;
  if (mismatches) *mismatches = b;
  return std::chrono::duration<double>(t1 - t0).count();
}

void loggen_free(loggen_doc* d) {
  free(d->ops);
  free(d->text);
  d->ops = nullptr;
  d->text = nullptr;
}

// JSON text of props id `i` for the generator's table (for engines that intern by JSON).
int loggen_props_count(int n_clients, int annotate_keys) { return (int)props_table(n_clients, std::max(1, annotate_keys)).size(); }
int loggen_props_json(int n_clients, int annotate_keys, int i, char* buf, int cap) {
  auto t = props_table(n_clients, std::max(1, annotate_keys));
  if (i < 0 || i >= (int)t.size()) return -1;
  int n = (int)t[i].size();
  if (n + 1 > cap) return -1;
  memcpy(buf, t[i].c_str(), n + 1);
  return n;
}

// CPU baseline: replay docs [0,n) of pre-generated logs through the oracle on `threads` threads.
// Returns wall seconds (log generation excluded), and the xor of final checksums.
double loggen_cpu_replay(const loggen_cfg* cfg, const loggen_doc* docs, uint32_t n, int threads, uint64_t* checksum_xor,
                         int32_t* errors) {
  std::vector<std::optional<JVal>> props = parse_table(props_table(cfg->n_clients, std::max(1, cfg->annotate_keys)));
  std::vector<std::unique_ptr<Doc>> done(n);
  std::vector<int> errs(threads, 0);
  if (threads < 1) threads = 1;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; t++) {
    ts.emplace_back([&, t] {
      for (uint32_t i = t; i < n; i += threads) {
        Options o;
        o.newLengthCalc = cfg->new_length_calc != 0;
        auto doc = std::make_unique<Doc>(o);
        const loggen_doc& d = docs[i];
        try {
          if (d.initial_len > 0)
            doc->insertTextLocal(0, u16str(reinterpret_cast<const char16_t*>(d.text), d.initial_len), std::nullopt);
          doc->startOrUpdateCollaboration("obs", 0, 0);
          for (uint32_t s = 1; s < d.n_short; s++) doc->getOrAddShortClientId("c" + std::to_string(d.client_writer[s]));
          const Doc::Record* r = static_cast<const Doc::Record*>(d.ops);
          for (uint32_t k = 0; k < d.n_ops; k++) doc->applyRecordParsed(r[k], d.text, props);
          done[i] = std::move(doc);
        } catch (const OracleError&) {
          errs[t]++;
        }
      }
    });
  }
  for (auto& th : ts) th.join();
  auto t1 = std::chrono::steady_clock::now();
  uint64_t x = 0;
  for (auto& d : done)
    if (d) x ^= fnv1a64(d->dumpSegments());
  if (checksum_xor) *checksum_xor = x;
  int e = 0;
  for (int v : errs) e += v;
  if (errors) *errors = e;
  return std::chrono::duration<double>(t1 - t0).count();
}

// CPU baseline of Client.summarize -> SnapshotV1: every document of the sample is replayed first
// (not timed), then summarizeV1 runs over all of them on `threads` threads (timed).  mismatches: summaries whose
// fingerprint differs from the generator's (docs[i].summary_fnv).
double loggen_cpu_summarize(const loggen_cfg* cfg, const loggen_doc* docs, uint32_t n, int threads, int32_t* mismatches) {
  std::vector<std::optional<JVal>> props = parse_table(props_table(cfg->n_clients, std::max(1, cfg->annotate_keys)));
  std::vector<std::unique_ptr<Doc>> done(n);
  if (threads < 1) threads = 1;
  auto run = [&](auto&& body) {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++)
      ts.emplace_back([&, t] {
        for (uint32_t i = t; i < n; i += threads) body(i);
      });
    for (auto& th : ts) th.join();
  };
  run([&](uint32_t i) {
    Options o;
    o.newLengthCalc = cfg->new_length_calc != 0;
    auto doc = std::make_unique<Doc>(o);
    const loggen_doc& d = docs[i];
    try {
      if (d.initial_len > 0)
        doc->insertTextLocal(0, u16str(reinterpret_cast<const char16_t*>(d.text), d.initial_len), std::nullopt);
      doc->startOrUpdateCollaboration("obs", 0, 0);
      for (uint32_t s = 1; s < d.n_short; s++) doc->getOrAddShortClientId("c" + std::to_string(d.client_writer[s]));
      const Doc::Record* r = static_cast<const Doc::Record*>(d.ops);
      for (uint32_t k = 0; k < d.n_ops; k++) doc->applyRecordParsed(r[k], d.text, props);
      done[i] = std::move(doc);
    } catch (const OracleError&) {
    }
  });
  std::vector<uint64_t> fp(n, 0);
  auto t0 = std::chrono::steady_clock::now();
  run([&](uint32_t i) {
    if (!done[i]) return;
    std::string summary;
    const auto blobs = done[i]->summarizeV1(&summary);
    uint64_t h = 1469598103934665603ull;
    auto add = [&](const std::string& x, bool zero) {
      for (unsigned char c : x) {
        h ^= c;
        h *= 1099511628211ull;
      }
      if (zero) h *= 1099511628211ull;
    };
    for (auto& bl : blobs) {
      add(bl.first, true);
      add(bl.second, true);
    }
    add(summary, false);
    fp[i] = h;
  });
  auto t1 = std::chrono::steady_clock::now();
  int32_t bad = 0;
  for (uint32_t i = 0; i < n; i++) bad += !done[i] || fp[i] != docs[i].summary_fnv;
  if (mismatches) *mismatches = bad;
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
