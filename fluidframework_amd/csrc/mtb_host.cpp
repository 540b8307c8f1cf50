// Host side of the MI355X merge-tree batch replay engine: the C ABI declared in include/mtb.h.
//
//  * mtb_apply_msg_json packs an ISequencedDocumentMessage (client.ts:858) into 32-byte op records,
//    interning long client ids (client.ts:673, first-seen order), property keys/values and props
//    objects into batch-wide tables that the kernel reads.
//  * mtb_replay sizes per-document HBM slices, uploads records / payload / tables, launches one
//    64-lane wavefront per document (mtb_replay.hip) and reads back the document headers.
//  * Read-outs (text, canonical segment dump, SnapshotV1 summary) download a document's slices and
//    walk its tree on the host.  There is no CPU replay path: without a GPU every compute entry point
//    fails with MTB_E_NODEV.
#include <functional>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <atomic>
#include <charconv>
#include <map>
#include <condition_variable>
#include <mutex>
#include <optional>
#include <cmath>
#include <thread>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <set>
#include <vector>

#include "../../include/mtb.h"
#include "hjson.hpp"
#include "mtb_dev.h"
#include "mtb_device.h"

// defined in mtb_replay.hip
hipError_t mtb_launch_move_words(hipStream_t stream, const uint32_t* src, const uint64_t* src_off, uint32_t* dst,
                                 const uint64_t* dst_off, const uint32_t* len, uint32_t n);
hipError_t mtb_launch_move_u16(hipStream_t stream, const uint16_t* src, const uint64_t* src_off, uint16_t* dst,
                               const uint64_t* dst_off, const uint32_t* len, uint32_t n);
hipError_t mtb_launch_rewind(hipStream_t stream, uint32_t ndocs, DocState* docs, const DocState* pristine, uint32_t* segp,
                             const uint32_t* psegp, FBlk* blks, const FBlk* pblk);
hipError_t mtb_launch_replay(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp,
                             FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                             Tables tables, int variant);  // 0 replay, 1 live clients, 2 marker ids
int mtb_sched_waves_per_cu();
hipError_t mtb_launch_replay_ticks(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops,
                                   uint32_t* segp, FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux,
                                   uint32_t* freel, Tables tables, uint32_t* sched, uint32_t nchunks, uint32_t nq);
hipError_t mtb_launch_replay_passes(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops,
                                    uint32_t* segp, FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux,
                                    uint32_t* freel, Tables tables, uint32_t first, uint32_t count, uint32_t nchunks);
hipError_t mtb_launch_load(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp,
                           FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                           Tables tables, int perm);
hipError_t mtb_launch_matrix(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp,
                             FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                             Tables tables);
hipError_t mtb_launch_extract_v1(hipStream_t stream, const DocState* docs, const uint32_t* list, uint32_t n,
                                 const FBlk* blks, const uint16_t* text, const uint32_t* aux, const uint32_t* pool,
                                 const Tables& tab, uint32_t* cnt, const uint64_t* off, uint32_t* items,
                                 uint16_t* otext, uint32_t* owords);
hipError_t mtb_launch_digest(hipStream_t stream, uint32_t ndocs, const DocState* docs, const FBlk* blks,
                             const uint16_t* text, const uint32_t* aux, const uint32_t* pool, const uint64_t* khash,
                             const uint64_t* vhash, uint64_t* out);

namespace {

using hj::U16;

uint64_t fnv_bytes(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

struct MtbError {
  int code;
  std::string msg;
};
[[noreturn]] void raise(int code, const std::string& m) { throw MtbError{code, m}; }

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) raise(MTB_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

// matchProperties (properties.ts:71-96) restated on parsed JSON values (JS semantics for the keys of
// primitives: strings expose their indices, other primitives none)
std::vector<U16> js_keys_of(const hj::Value* v) {
  std::vector<U16> k;
  if (!v) return k;
  if (v->kind == hj::Value::kObj) for (auto& m : v->members) k.push_back(m.first);
  else if (v->kind == hj::Value::kArr) for (size_t i = 0; i < v->items.size(); i++) { std::string t = std::to_string(i); k.push_back(U16(t.begin(), t.end())); }
  else if (v->kind == hj::Value::kStr) for (size_t i = 0; i < v->s.size(); i++) { std::string t = std::to_string(i); k.push_back(U16(t.begin(), t.end())); }
  return k;
}
bool js_get_of(const hj::Value* v, const U16& key, hj::Value& tmp, const hj::Value*& out) {
  out = nullptr;
  if (!v) return false;
  if (v->kind == hj::Value::kObj) { out = v->find(key.c_str()); return out != nullptr; }
  uint32_t idx;
  if (!hj::array_index(key, &idx)) return false;
  if (v->kind == hj::Value::kArr && idx < v->items.size()) { out = &v->items[idx]; return true; }
  if (v->kind == hj::Value::kStr && idx < v->s.size()) { tmp.kind = hj::Value::kStr; tmp.s = U16(1, v->s[idx]); out = &tmp; return true; }
  return false;
}
bool js_strict_eq(const hj::Value* a, const hj::Value* b) {
  if (!a || !b) return a == b;
  if (a->kind != b->kind) return false;
  switch (a->kind) {
    case hj::Value::kNull: case hj::Value::kUndef: return true;
    case hj::Value::kBool: return a->b == b->b;
    case hj::Value::kNum: return a->n == b->n;
    case hj::Value::kStr: return a->s == b->s;
    default: return a == b;  // object identity
  }
}
bool js_match_props(const hj::Value* a, const hj::Value* b) {
  if ((!a || !a->truthy()) && (!b || !b->truthy())) return true;
  const auto ka = js_keys_of(a), kb = js_keys_of(b);
  if (ka.size() != kb.size()) return false;
  for (auto& k : ka) {
    hj::Value ta, tb;
    const hj::Value *av = nullptr, *bv = nullptr;
    if (!js_get_of(b, k, tb, bv) || !bv || bv->kind == hj::Value::kUndef) return false;
    js_get_of(a, k, ta, av);
    if (bv->kind == hj::Value::kObj || bv->kind == hj::Value::kArr || bv->kind == hj::Value::kNull) {
      if (!js_match_props(av, bv)) return false;
    } else if (!js_strict_eq(bv, av)) {
      return false;
    }
  }
  return true;
}
// one key's step of matchProperties (properties.ts:84-92): b's value an object, array or null recurses,
// anything else compares strictly
bool js_match_value(const hj::Value* a, const hj::Value* b) {
  if (!b || b->kind == hj::Value::kUndef) return false;
  if (b->kind == hj::Value::kObj || b->kind == hj::Value::kArr || b->kind == hj::Value::kNull) return js_match_props(a, b);
  return js_strict_eq(b, a);
}

// ------------------------------------------------------------------ interning
// The property values one document can hold, per key (value ids): those of the props ids it met (its ops, a loaded
// summary's segments, host-made consensus values; noted lazily) and the results of its incr tables.  An incr
// annotate's result table covers these only, so its size and the refusal limit are per document, not per batch.
struct DocVals {
  std::vector<uint32_t> propsSeen;  // props ids, appended as met (load threads included), noted by Interner::note
  size_t noted = 0;
  std::unordered_map<uint32_t, std::vector<uint32_t>> keyVals;
  std::unordered_set<uint32_t> seen;
  void add(uint32_t k, uint32_t v) {
    if (seen.insert(v).second) keyVals[k].push_back(v);
  }
};

struct Interner {
  std::vector<U16> keys;
  std::vector<std::string> keyJson;  // each key quoted as a JSON string (the summary serializers' props)
  std::map<U16, uint32_t> keyId;
  std::vector<uint32_t> keyRank;
  std::vector<std::string> valJson;
  std::unordered_map<std::string, uint32_t> valId;  // "<key id>:" + JSON -> value id (values are per key)
  std::vector<uint32_t> valClass;
  std::vector<uint8_t> valFalsy;
  std::unordered_map<std::string, uint32_t> classId;
  std::vector<uint32_t> pool{0};   // offset 0 reserved
  std::vector<uint32_t> pidx{0, 0};  // props id 0 = none
  std::unordered_map<std::string, uint32_t> propsByJson;
  bool dirty = true;
  // matchProperties (properties.ts:71-96) exactly.  A value id belongs to one key.  A key is regular when, at
  // each path inside its values, one kind occurs (primitive, object-like, null) and no member is undefined:
  // matchProperties between its values is then the equality of their canonical forms (valClass, symmetric and
  // reflexive).  Any other key is irregular -- a primitive against an object ({k:5} vs {k:{}} matches, the
  // reverse does not), a nested null, a consensus value's undefined member -- and matchProperties(a, b) of each
  // ordered pair of its values is tabulated (irrRows; a = the run head's, zamboni.ts:155, snapshotV1.ts:240).
  static constexpr uint32_t kIrrMax = 4096;  // values of one irregular key (the table is n^2 bits)
  std::vector<std::unordered_map<std::string, uint8_t>> keyPaths;  // path -> kinds (1 prim, 2 object, 4 null, 8 undef)
  std::vector<uint8_t> keyIrr;
  std::vector<std::vector<uint32_t>> keyVals;              // the key's value ids, in interning order
  std::vector<std::vector<std::vector<uint8_t>>> irrRows;  // irregular key: [i][j] = matchProperties(v_i, v_j)
  std::vector<uint32_t> valLocal;                          // value -> index in its key's list
  std::vector<hj::Value> valStore;
  uint32_t nIrr = 0;
  uint32_t nIrrKeys() const {
    uint32_t n = 0;
    for (uint8_t x : keyIrr) n += x;
    return n;
  }
  // consensus values ({value: undefined, seq}) are matched by nothing as the second argument, and as the first
  // only by a two-key object {value: null | {} | [], seq: <that seq>} ("cv-like"): such values are refused on a
  // key that holds consensus values, so a set holding one matches no set (valFalsy bit 3, like NaN)
  std::vector<uint8_t> keyCv, keyCvLike;
  // keys an incr annotate names (they can hold NaN).  matchProperties(NaN, v) is true for an object or array v
  // without own keys and false otherwise, matchProperties(v, NaN) always false: such a key that also holds object
  // or array values is irregular (its pairs with NaN are decided on the device from val_falsy bits 3 and 4)
  std::vector<uint8_t> keyNaN;

  uint32_t key(const U16& k) {
    auto it = keyId.find(k);
    if (it != keyId.end()) return it->second;
    uint32_t id = (uint32_t)keys.size();
    keys.push_back(k);
    keyJson.emplace_back();
    hj::quote(keyJson.back(), k);
    keyId[k] = id;
    uint32_t r;
    keyRank.push_back(hj::array_index(k, &r) ? r : MTB_NONE);
    keyPaths.emplace_back();
    keyIrr.push_back(0);
    keyCv.push_back(0);
    keyCvLike.push_back(0);
    keyNaN.push_back(0);
    keyVals.emplace_back();
    irrRows.emplace_back();
    dirty = true;
    return id;
  }
  // canonical form: arrays compare like objects with index keys
  static void canon(std::string& o, const hj::Value& v) {
    switch (v.kind) {
      case hj::Value::kBool: o += v.b ? "b1" : "b0"; return;
      case hj::Value::kNum: o += "n" + hj::number(v.n); return;
      case hj::Value::kStr: o += "s"; hj::quote(o, v.s); return;
      case hj::Value::kNull: o += "z"; return;
      case hj::Value::kUndef: o += "u"; return;
      case hj::Value::kArr:
      case hj::Value::kObj: {
        std::vector<std::pair<U16, const hj::Value*>> m;
        if (v.kind == hj::Value::kArr) {
          for (size_t i = 0; i < v.items.size(); i++) {
            std::string s = std::to_string(i);
            m.push_back({U16(s.begin(), s.end()), &v.items[i]});
          }
        } else {
          for (auto& e : v.members) m.push_back({e.first, &e.second});
        }
        std::sort(m.begin(), m.end(), [](auto& a, auto& b) { return a.first < b.first; });
        o += "{";
        for (auto& e : m) {
          hj::quote(o, e.first);
          o += ":";
          canon(o, *e.second);
          o += ",";
        }
        o += "}";
        return;
      }
    }
  }
  void note_paths(uint32_t k, const hj::Value& v, std::string& path) {
    const bool objLike = v.kind == hj::Value::kObj || v.kind == hj::Value::kArr;
    const uint8_t kind = v.kind == hj::Value::kNull ? 4 : v.kind == hj::Value::kUndef ? 8 : objLike ? 2 : 1;
    uint8_t& m = keyPaths[k][path];
    m |= kind;
    if ((m & (m - 1)) || (m & 8)) keyIrr[k] = 1;
    if (!objLike) return;
    const size_t n0 = path.size();
    auto step = [&](const U16& key, const hj::Value& x) {
      path += std::to_string(key.size());
      path += ':';
      for (char16_t c : key) { path += (char)(c & 0xFF); path += (char)(c >> 8); }
      note_paths(k, x, path);
      path.resize(n0);
    };
    if (v.kind == hj::Value::kArr) {
      for (size_t i = 0; i < v.items.size(); i++) {
        std::string t = std::to_string(i);
        step(U16(t.begin(), t.end()), v.items[i]);
      }
    } else {
      for (auto& e : v.members) step(e.first, e.second);
    }
  }
  static bool cv_like(const hj::Value& v) {
    if (v.kind != hj::Value::kObj || v.members.size() != 2) return false;
    const hj::Value* val = v.find(u"value");
    const hj::Value* sq = v.find(u"seq");
    if (!val || !sq || sq->kind != hj::Value::kNum) return false;
    return val->kind == hj::Value::kNull || (val->kind == hj::Value::kObj && val->members.empty()) ||
           (val->kind == hj::Value::kArr && val->items.empty());
  }
  // `js`: the JSON the summaries write for the value (JSON.stringify drops undefined members); `cv`: a consensus
  // value (no paths noted: it never makes its key irregular)
  uint32_t add_value(uint32_t k, const std::string& idKey, const std::string& js, const hj::Value& v, bool cv = false) {
    std::string path;
    if (cv) {
      if (keyCvLike[k]) raise(MTB_E_UNSUPPORTED, "unsupported: consensus on a key holding a {value, seq} object value");
      keyCv[k] = 1;
    } else {
      if (cv_like(v)) {
        if (keyCv[k]) raise(MTB_E_UNSUPPORTED, "unsupported: a {value, seq} object value on a key holding consensus values");
        keyCvLike[k] = 1;
      }
      note_paths(k, v, path);
      if (keyNaN[k] && (v.kind == hj::Value::kObj || v.kind == hj::Value::kArr)) keyIrr[k] = 1;
    }
    if (keyIrr[k] && keyVals[k].size() + 1 > kIrrMax)  // (before the value is interned: only this message fails)
      raise(MTB_E_UNSUPPORTED, "unsupported: more than 4096 distinct values under one property key whose values "
                               "matchProperties does not compare as an equivalence");
    std::string c = std::to_string(k) + ":";
    canon(c, v);
    auto ci = classId.find(c);
    uint32_t cls;
    if (ci == classId.end()) {
      cls = (uint32_t)classId.size();
      classId[c] = cls;
    } else {
      cls = ci->second;
    }
    uint32_t id = (uint32_t)valJson.size();
    valJson.push_back(js);
    valId[idKey] = id;
    valClass.push_back(cls);
    // bit 0: JS falsy; bit 1: incr makes it NaN (number / boolean + undefined, properties.ts:38-45); bit 2: an
    // object whose seq is -1 (consensus completes it in place, properties.ts:56-60)
    const hj::Value* sq = v.kind == hj::Value::kObj ? v.find(u"seq") : nullptr;
    // bit 4: an object or array without own keys (Object.keys is empty: matchProperties(NaN, it) is true)
    const bool noKeys = (v.kind == hj::Value::kObj && v.members.empty()) || (v.kind == hj::Value::kArr && v.items.empty());
    valFalsy.push_back((v.truthy() ? 0 : 1) | (v.kind == hj::Value::kNum || v.kind == hj::Value::kBool ? 2 : 0) |
                       (sq && sq->kind == hj::Value::kNum && sq->n == -1 ? 4 : 0) | (cv ? 8 : 0) | (noKeys ? 16 : 0));
    valLocal.push_back((uint32_t)keyVals[k].size());
    keyVals[k].push_back(id);
    valStore.push_back(v);
    dirty = true;
    return id;
  }
  uint32_t value(uint32_t k, const hj::Value& v) {
    std::string js = hj::dump(v);
    std::string idKey = std::to_string(k) + ":" + js;
    auto it = valId.find(idKey);
    if (it != valId.end()) return it->second;
    return add_value(k, idKey, js, v);
  }
  // combine(consensus, undefined, undefined, seq) (properties.ts:46-55): a fresh {value: undefined, seq} --
  // {"seq":seq} in JSON, and never matched as the second argument of matchProperties (its undefined member)
  uint32_t consensus_value(uint32_t k, int seq) {
    std::string idKey = "\x02" + std::to_string(k) + ":" + std::to_string(seq);
    auto it = valId.find(idKey);
    if (it != valId.end()) return it->second;
    hj::Value v;
    v.kind = hj::Value::kObj;
    v.members.push_back({u"value", hj::Value()});
    hj::Value sv;
    sv.kind = hj::Value::kNum;
    sv.n = seq;
    v.members.push_back({u"seq", sv});
    nan();  // (the device's no-match check on new sets runs once a NaN value exists)
    anyCv = true;
    return add_value(k, idKey, "{\"seq\":" + std::to_string(seq) + "}", v, true);
  }
  // matchProperties(value a, value b) of two values of key k (properties.ts:84-92)
  bool value_match(uint32_t k, uint32_t a, uint32_t b) {
    if (!keyIrr[k]) return valClass[a] == valClass[b];
    irr_rows(k);
    return irrRows[k][valLocal[a]][valLocal[b]] != 0;
  }
  void irr_rows(uint32_t k) {
    auto& M = irrRows[k];
    const auto& vs = keyVals[k];
    const size_t n0 = M.size(), n = vs.size();
    if (n0 == n) return;
    for (auto& row : M) row.resize(n);
    M.resize(n);
    for (size_t i = 0; i < n; i++) {
      M[i].resize(n);
      for (size_t j = i < n0 ? n0 : 0; j < n; j++) M[i][j] = js_match_value(&valStore[vs[i]], &valStore[vs[j]]) ? 1 : 0;
    }
  }
  // device tables: keyOff[k] = 1 + offset of [n, bits of n x n (row a, column b)] in bits, 0 for a regular key
  void irr_tables(std::vector<uint32_t>& keyOff, std::vector<uint32_t>& localOf, std::vector<uint32_t>& bits) {
    keyOff.assign(keys.size(), 0);
    localOf.assign(valJson.size(), MTB_NONE);
    bits.assign(1, 0);
    nIrr = 0;
    for (uint32_t k = 0; k < keys.size(); k++) {
      if (!keyIrr[k]) continue;
      nIrr++;
      irr_rows(k);
      const auto& vs = keyVals[k];
      const size_t n = vs.size();
      keyOff[k] = (uint32_t)bits.size() + 1;
      bits.push_back((uint32_t)n);
      const size_t o = bits.size();
      bits.resize(o + (n * n + 31) / 32, 0);
      for (size_t i = 0; i < n; i++) {
        localOf[vs[i]] = (uint32_t)i;
        for (size_t j = 0; j < n; j++)
          if (irrRows[k][i][j]) bits[o + (i * n + j) / 32] |= 1u << ((i * n + j) % 32);
      }
    }
  }
  // an annotate's consensus op-props (properties.ts:46-62, a sequenced op at `seq`; the op's values are never
  // read): each key of props id `pid` holds what a segment lacking the key gets -- {value: undefined, seq} with
  // no defaultValue, else the defaultValue (its seq completed when -1: the op's own object, shared by the op's
  // segments alone), or MTB_NONE for a null defaultValue (the reference throws reading its seq).  A segment that
  // has the key keeps its value (the device; one whose value is an object with seq -1 fails, DERR_CONSENSUS).
  uint32_t consensus_props(uint32_t pid, const hj::Value* dv, int seq) {
    const std::string memo = "\x03" + std::to_string(pid) + ":" + std::to_string(seq) + ":" + (dv ? hj::dump(*dv) : "-");
    auto it = propsByJson.find(memo);
    if (it != propsByJson.end()) return it->second;
    const uint32_t off = pidx[2 * pid], n = pool[off];
    std::vector<std::pair<uint32_t, uint32_t>> kv;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t k = pool[off + 1 + 2 * i];
      uint32_t v;
      if (!dv || dv->kind == hj::Value::kUndef) {
        v = consensus_value(k, seq);
      } else if (dv->kind == hj::Value::kNull) {
        v = MTB_NONE;
      } else {
        hj::Value d = *dv;
        if (d.kind == hj::Value::kObj)
          for (auto& m : d.members)
            if (m.first == u"seq" && m.second.kind == hj::Value::kNum && m.second.n == -1) m.second.n = seq;
        v = value(k, d);
      }
      kv.push_back({k, v});
    }
    return props_kv(memo, kv);
  }
  // an incr annotate's op-props (properties.ts:24-45 through combine(op, previous, undefined), the op's values
  // never read): each key's value slot names a pool table [absent result, n, (value, result) * n]
  // (MTB_INCR_TAB).  On the device a number / boolean / NaN previous value becomes NaN; a string, object or array
  // v becomes String(v) + "undefined" -- and minValue when that is a string, object or array and the result sorts
  // below its string form (JS string order; a number or boolean minValue compares with NaN: never) -- looked up
  // here for every such value the key holds in the batch so far (a document's values were all interned before
  // its op is packed); an absent key gets defaultValue + undefined (NaN, or a string).
  // String(v) (ECMA-262 ToString): objects "[object Object]", arrays join(",") with undefined / null elements as ""
  static U16 js_string(const hj::Value& v) {
    switch (v.kind) {
      case hj::Value::kBool: return v.b ? U16(u"true") : U16(u"false");
      case hj::Value::kNum: {
        if (std::isnan(v.n)) return U16(u"NaN");
        if (std::isinf(v.n)) return v.n < 0 ? U16(u"-Infinity") : U16(u"Infinity");
        const std::string t = hj::number(v.n);
        return U16(t.begin(), t.end());
      }
      case hj::Value::kStr: return v.s;
      case hj::Value::kNull: return U16(u"null");
      case hj::Value::kUndef: return U16(u"undefined");
      case hj::Value::kObj: return U16(u"[object Object]");
      case hj::Value::kArr: {
        U16 o;
        for (size_t i = 0; i < v.items.size(); i++) {
          if (i) o += u",";
          if (v.items[i].kind != hj::Value::kUndef && v.items[i].kind != hj::Value::kNull) o += js_string(v.items[i]);
        }
        return o;
      }
    }
    return U16();
  }
  // the values of the props ids `dv` met since the last call (both the op list and the property set of each)
  void note(DocVals& dv) {
    for (; dv.noted < dv.propsSeen.size(); dv.noted++) {
      const uint32_t pid = dv.propsSeen[dv.noted];
      if (!pid || 2 * pid + 1 >= pidx.size()) continue;
      for (int w = 0; w < 2; w++) {
        const uint32_t off = pidx[2 * pid + w];
        if (!off) continue;
        const uint32_t n = pool[off];
        for (uint32_t i = 0; i < n; i++) {
          const uint32_t v = pool[off + 2 + 2 * i];
          if (v != MTB_NONE && !(v & MTB_INCR_TAB) && v < valJson.size()) dv.add(pool[off + 1 + 2 * i], v);
        }
      }
    }
  }
  static constexpr uint32_t kIncrStrMax = 4096;
  // (doc: the document's values; null: every value of the batch, e.g. records appended without a document context)
  uint32_t incr_props(uint32_t pid, const hj::Value* dv, const hj::Value* mv, DocVals* doc = nullptr) {
    const uint32_t off = pidx[2 * pid], n = pool[off];
    if (doc) note(*doc);
    std::string memo = "\x04" + std::to_string(pid) + ":" + (dv ? hj::dump(*dv) : "-") + ":" + (mv ? hj::dump(*mv) : "-");
    for (uint32_t i = 0; i < n; i++) memo += ":" + std::to_string(keyVals[pool[off + 1 + 2 * i]].size());
    auto it = doc ? propsByJson.end() : propsByJson.find(memo);  // (per-document tables are not shared)
    if (it != propsByJson.end()) return it->second;
    // minValue (when truthy) compares with a string result as its string form (ToPrimitive; a number or boolean
    // compares NaN: never), and replaces it, itself (an object stays an object), when the result sorts below it
    const bool minStr = mv && mv->truthy() &&
                        (mv->kind == hj::Value::kStr || mv->kind == hj::Value::kObj || mv->kind == hj::Value::kArr);
    const U16 minS = minStr ? js_string(*mv) : U16();
    // previous values that concatenate: strings, objects and arrays (numbers, booleans and NaN give NaN)
    auto concat = [](const hj::Value& v) {
      return v.kind == hj::Value::kStr || v.kind == hj::Value::kObj || v.kind == hj::Value::kArr;
    };
    auto result = [&](uint32_t k, const U16& s) {
      hj::Value r;
      r.kind = hj::Value::kStr;
      r.s = s + U16(u"undefined");
      if (minStr && r.s < minS) return value(k, *mv);
      return value(k, r);
    };
    std::vector<std::pair<uint32_t, uint32_t>> kv;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t k = pool[off + 1 + 2 * i];
      if (!keyNaN[k]) {  // the key can hold NaN from now on
        keyNaN[k] = 1;
        auto root = keyPaths[k].find(std::string());
        if (root != keyPaths[k].end() && (root->second & 2) && !keyIrr[k]) {
          keyIrr[k] = 1;
          dirty = true;
        }
      }
      std::vector<uint32_t> strs;
      for (uint32_t v : doc ? doc->keyVals[k] : keyVals[k])
        if (concat(valStore[v])) strs.push_back(v);
      if (strs.size() > kIncrStrMax)  // (checked before anything is interned: the refusal changes no state)
        raise(MTB_E_UNSUPPORTED, "unsupported: incr over a key holding more than 4096 distinct string / object values "
                                 "in one document");
      uint32_t absent = nan();
      if (dv && concat(*dv)) absent = result(k, js_string(*dv));
      std::vector<uint32_t> tab{absent, (uint32_t)strs.size()};
      for (uint32_t v : strs) {
        const U16 sv = js_string(valStore[v]);  // (value() may grow valStore)
        const uint32_t r = result(k, sv);
        tab.push_back(v);
        tab.push_back(r);
      }
      if (doc) {  // the document can hold the results from now on
        if (absent != nanVal) doc->add(k, absent);
        for (size_t j = 3; j < tab.size(); j += 2) doc->add(k, tab[j]);
      }
      const uint32_t t = (uint32_t)pool.size();
      pool.insert(pool.end(), tab.begin(), tab.end());
      kv.push_back({k, MTB_INCR_TAB | t});
      if (doc) memo += "@" + std::to_string(t);  // (a per-document table is its own props id)
    }
    dirty = true;
    return props_kv(memo, kv);
  }
  // NaN, the value an incr annotate gives a numeric key: JSON null (JSON.stringify), its own matchProperties
  // class; a set holding it is flagged MTB_PNAN by the device and matches nothing (NaN !== NaN)
  uint32_t nanVal = MTB_NONE;
  bool anyCv = false;  // consensus values interned (Tables::nan_val | MTB_NAN_CV)
  uint32_t nan() {
    if (nanVal != MTB_NONE) return nanVal;
    nanVal = (uint32_t)valJson.size();
    valJson.push_back("null");  // (null itself is never a stored value: it deletes)
    const uint32_t cls = (uint32_t)classId.size();
    classId["\x01NaN"] = cls;
    valClass.push_back(cls);
    valFalsy.push_back(1 | 2 | 8);
    valLocal.push_back(MTB_NONE);
    valStore.push_back(hj::Value());
    dirty = true;
    return nanVal;
  }
  // props object -> id with (a) op-props list for annotate, (b) property set for insert specs.
  uint32_t props(const hj::Value& obj) {
    if (obj.kind != hj::Value::kObj) raise(MTB_E_PARSE, "props is not an object");
    return props_keyed(hj::dump(obj), obj);
  }
  // `js` = hj::dump(obj) (computed by the caller, e.g. outside a lock)
  uint32_t props_keyed(const std::string& js, const hj::Value& obj) {
    auto it = propsByJson.find(js);
    if (it != propsByJson.end()) return it->second;
    std::vector<std::pair<uint32_t, uint32_t>> kv;
    for (auto& m : obj.members) {
      const uint32_t k = key(m.first);
      const uint32_t v = m.second.kind == hj::Value::kNull ? MTB_NONE : value(k, m.second);
      kv.push_back({k, v});
    }
    return props_kv(js, kv);
  }
  // a props id from (key, value id) pairs (MTB_NONE: null); `memo` names it for reuse
  uint32_t props_kv(const std::string& memo, const std::vector<std::pair<uint32_t, uint32_t>>& kv) {
    auto it = propsByJson.find(memo);
    if (it != propsByJson.end()) return it->second;
    const uint32_t opOff = (uint32_t)pool.size();
    pool.push_back((uint32_t)kv.size());
    for (auto& e : kv) { pool.push_back(e.first); pool.push_back(e.second); }
    const uint32_t setOff = (uint32_t)pool.size();
    uint32_t n = 0;  // (the set holds values: no nulls, no incr result tables)
    for (auto& e : kv) n += !(e.second & MTB_INCR_TAB);
    pool.push_back(n);
    for (auto& e : kv)
      if (!(e.second & MTB_INCR_TAB)) { pool.push_back(e.first); pool.push_back(e.second); }
    const uint32_t id = (uint32_t)(pidx.size() / 2);
    pidx.push_back(opOff);
    pidx.push_back(setOff);
    propsByJson[memo] = id;
    dirty = true;
    return id;
  }
};

// ------------------------------------------------------------------ SnapshotV1 load image
// A segment read from a summary chunk by SnapshotLoader.specToSegment (snapshotLoader.ts:94-131).
struct LoadSeg {
  uint32_t len = 0;     // cachedLength (markers 1)
  uint32_t text = 0;    // text offset (header: initial-text arena, body: payload) or MTB_MARKER | (refType + 1)
  uint32_t props = 0;   // props id (0 = none)
  int32_t seq = 0;      // UniversalSequenceNumber unless the spec carries merge info
  int32_t rseq = -1;    // removedSeq, -1 = not removed
  int16_t client = -2;  // NonCollabClient unless the spec names one
  int16_t rc0 = -1;     // removedClientIds[0] (-1 = none)
  uint32_t rcx = 0;     // aux offset of the further removers [n, c1..cn] (0 = none)
  bool marker = false;
  uint32_t mord = 0;    // marker id ordinal + 1 (0: no id)
};
// The header segments rebuilt as a tree (reloadFromSegments, mergeTree.ts:678-721) with the window
// lists startCollaboration's recursive combine gives every internal block (partialLengths.ts:256-338),
// laid out as the device slices hold them.
struct LoadImage {
  std::vector<uint32_t> segp;  // parent block of each header segment
  std::vector<FBlk> blks;
  std::vector<WEnt> lists;     // entry 0..MTB_LIST_RESERVED-1: the free-list heads
  std::vector<uint32_t> aux;   // word 0 unused, then the overlapping-remover lists
  uint32_t root = 0;
  uint32_t mk_map = 0, mk_n = 0;  // idToSegment of the live header markers (in `aux`)
  uint32_t mk_all = 0;            // DocState.mk_all: the live header markers with an id (in `aux`)
  uint32_t ph = 0;                // DocState.ph: the phantom partial-length table (in `aux`; 0 = none)
};

// ------------------------------------------------------------------ SharedMatrix cells
// SparseArray2D (matrix/src/sparsearray2d.ts) as the host keeps it for a matrix batch: every (row, col)
// handle pair ever written, with its current value id (0 = undefined).  The Morton-keyed tile levels
// the reference allocates on a write (getLevel, :226-231) are exactly the prefixes of the written keys,
// so the snapshot JSON is rebuilt from the sorted keys.  Written from the kernel's cell events.
struct CellStore {
  std::unordered_map<uint64_t, uint32_t> cells;  // (row << 32 | col) -> value id
  std::unordered_map<uint32_t, std::vector<uint32_t>> rowCols, colRows;
  uint64_t rootLen = 1;  // the root array's JS length (`[undefined]`, grown by writes or a load)
  static uint32_t spread(uint32_t x) {  // interlaceBitsX16: the low 16 bits onto the even positions
    x &= 0xffff;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
  }
  static uint32_t morton(uint32_t r, uint32_t c) { return (spread(r) << 1) | spread(c); }  // r0c0ToMorton2x16
  void set(uint32_t r, uint32_t c, uint32_t v) {
    rootLen = std::max<uint64_t>(rootLen, (uint64_t)morton(r >> 16, c >> 16) + 1);
    auto [it, fresh] = cells.try_emplace(((uint64_t)r << 32) | c, v);
    if (!fresh) {
      it->second = v;
      return;
    }
    rowCols[r].push_back(c);
    colRows[c].push_back(r);
  }
  void clearRow(uint32_t r) {  // clearRows(r, 1) (:150-174): leaves only, tiles stay
    auto it = rowCols.find(r);
    if (it != rowCols.end())
      for (uint32_t c : it->second) cells[((uint64_t)r << 32) | c] = 0;
  }
  void clearCol(uint32_t c) {
    auto it = colRows.find(c);
    if (it != colRows.end())
      for (uint32_t r : it->second) cells[((uint64_t)r << 32) | c] = 0;
  }
  // JSON.stringify(snapshot()): the root array (holes -> null) of 256-entry levels
  std::string snapshot_json(const std::vector<std::string>& vals) const {
    std::vector<std::pair<uint64_t, uint32_t>> keys;  // (keyHi << 32 | keyLo, value id)
    keys.reserve(cells.size());
    for (auto& [k, v] : cells) {
      const uint32_t r = (uint32_t)(k >> 32), c = (uint32_t)k;
      keys.push_back({((uint64_t)morton(r >> 16, c >> 16) << 32) | morton(r, c), v});
    }
    std::sort(keys.begin(), keys.end());
    std::string o = "[";
    size_t i = 0;

    // level `lv` (0..3) of the tile whose key prefix is `pre`: 256 entries, byte `lv` of keyLo
    auto level = [&](auto& self, int lv, uint64_t pre) -> void {
      o += '[';
      for (uint32_t e = 0; e < 256; e++) {
        if (e) o += ',';
        const int shift = 24 - 8 * lv;
        const uint64_t want = pre | ((uint64_t)e << shift);
        const uint64_t mask = ~((1ull << shift) - 1);
        if (i < keys.size() && (keys[i].first & mask) == want) {
          if (lv == 3) {
            o += keys[i].second ? vals[keys[i].second] : std::string("null");
            i++;
          } else {
            self(self, lv + 1, want);
          }
        } else {
          o += "null";
        }
      }
      o += ']';
    };
    for (uint64_t hi = 0; hi < rootLen; hi++) {
      if (hi) o += ',';
      if (i < keys.size() && (keys[i].first >> 32) == hi) level(level, 0, hi << 32);
      else o += "null";
    }
    return o + "]";
  }
};

// ------------------------------------------------------------------ host mirror of a document
struct HostDoc {
  DocVals vals;  // property values the document can hold (incr result tables)
  std::set<std::string> pendingConsensus;  // Client.pendingConsensus: marker ids (JSON) of annotateMarkerNotifyConsensus
  std::vector<std::string> longIds;
  std::unordered_map<std::string, uint16_t> shortOf;
  std::string observer;
  bool inited = false;
  std::vector<uint16_t> initText;
  uint32_t min0 = 0, cur0 = 0;
  std::vector<mtb_op> pending;
  std::vector<uint16_t> payload;  // payload of pending ops
  // the records (and payload) of the last replay, consumed before its host post-processing runs so
  // that a post-processing failure can never make a later replay apply them twice
  std::vector<mtb_op> applied;
  std::vector<uint16_t> appliedPayload;
  std::string hostErr;            // message of a sticky host-side failure (DERR_HOST)
  int64_t lastSeq = 0;            // last appended message seq (host-side 0x038 check)
  uint64_t totalOps = 0;          // all records ever appended (capacity sizing)
  uint64_t totalLocal = 0;        // local-op records, and groups a REGEN may re-queue (aux sizing)
  uint64_t totalDetached = 0;     // records of detached edits (mtb_detached_op_json), all before the first message
  uint64_t totalPayload = 0;
  // SnapshotV1 load (mtb_doc_load_v1): the reloaded header; the body segments are LOADSEG records
  bool loaded = false;
  bool phantom = false;  // a loaded summary with removed collaborator-inserted body segments (DSF_PHANTOM)
  // SharedSegmentSequence.messagesSinceMSNChange (MTB_BATCH_CATCHUP, sequence.ts:697-748): stored
  // messages; a lagging one is rewritten from the delta entries of its records (pending[first, +count))
  struct CatchMsg {
    hj::Value msg;
    bool resolved = true;
    uint32_t first = 0, count = 0;
  };
  std::vector<CatchMsg> catchup;
  // PermutationVector (matrix batches): segments carry handles; the handle table lives in the text arena
  bool perm = false;
  uint64_t totalSetcell = 0;
  std::unique_ptr<CellStore> cells;  // rows vector of a matrix: the matrix's cells (matrix.ts:96)
  LoadImage img;
  // idToSegment keys (mergeTree.ts:549): marker id -> per-document ordinal (first-seen order).  An id met on
  // a second marker is reused: blockUpdate's re-mapping (:296-306) decides which marker it names, which the
  // marker and live kernels reproduce (DSF_MKDUP).
  std::unordered_map<std::string, uint32_t> markerOrd;
  std::vector<uint8_t> markerAmbig;
  bool markerDup = false;      // some id is reused
  bool markerIdAnnot = false;  // an annotate names markerId (assert 0x5ad is checked on the device)
  // device mirror
  DocState st{};
  bool onDevice = false;
  // read-back cache
  bool cached = false;
  std::vector<Seg> segs;
  std::vector<Blk> blks;
  std::vector<uint16_t> text;
  std::vector<uint32_t> aux;

  uint16_t client(const std::string& id) {
    auto it = shortOf.find(id);
    if (it != shortOf.end()) return it->second;
    if (longIds.size() >= 0x7FFF) raise(MTB_E_UNSUPPORTED, "unsupported: more than 32767 clients in one document");
    uint16_t s = (uint16_t)longIds.size();
    shortOf[id] = s;
    longIds.push_back(id);
    return s;
  }
  std::string longId(int s) const { return s >= 0 && s < (int)longIds.size() ? longIds[s] : std::string("original"); }
  // The engine numbers the document's own client (the observer / live client) 0.  A loaded summary names its
  // clients first (snapshotLoader.ts:94-131), so the reference gives the observer a later short id: obsRef.
  // Engine ids 0 and obsRef are swapped against the reference's; ref_id maps either way (an involution) where
  // short ids leave the engine (segment dumps, map_range, getLongClientId, the GPU digest).
  uint16_t obsRef = 0;
  int ref_id(int c) const { return c < 0 ? c : c == 0 ? obsRef : c == obsRef ? 0 : c; }
};

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void ensure(size_t want) {
    if (want <= n) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    HIPCHK(hipMalloc((void**)&p, std::max<size_t>(want, 1) * sizeof(T)));
    n = want;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// A list of (src offset, dst offset, length) chunks moved by one kernel launch.
struct Chunks {
  std::vector<uint64_t> src, dst;
  std::vector<uint32_t> len;
  void add(uint64_t s, uint64_t d, uint64_t n) {
    if (!n) return;
    src.push_back(s);
    dst.push_back(d);
    len.push_back((uint32_t)n);
  }
};

}  // namespace

struct mtb_dev {
  mtb_options opts{};
  uint32_t ndocs = 0;
  int device = 0;
  std::vector<HostDoc> docs;
  Interner in;
  std::string err;
  bool devInit = false;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  DevBuf<DocState> dDocs;
  DevBuf<mtb_op> dOps;
  DevBuf<uint32_t> dSegs;  // parent block of each segment
  DevBuf<FBlk> dBlks;
  DevBuf<WEnt> dLists;
  DevBuf<uint16_t> dText;
  DevBuf<Lru> dHeap;
  DevBuf<uint32_t> dAux, dFree;
  DevBuf<uint32_t> dPool, dPidx, dValClass, dKeyRank, dKeyIrr, dValLocal, dIrr;
  DevBuf<uint8_t> dValFalsy;
  // host staging of the SnapshotV1 extraction (extract_docs), kept and reused by later summaries: a call does
  // not pay for freeing (or re-faulting) the previous call's hundreds of MB
  std::unique_ptr<uint32_t[]> exItems, exWords;
  std::unique_ptr<uint16_t[]> exText;
  size_t exItemsCap = 0, exWordsCap = 0, exTextCap = 0;
  DevBuf<uint32_t> dExItems, dExWords;  // ... and its device output (no hipFree, which waits for the device, per call)
  DevBuf<uint16_t> dExText;
  DevBuf<uint64_t> dKHash, dVHash;  // state digest: FNV-1a of each key's UTF-8 / each value's JSON text
  DevBuf<uint64_t> dDigest;         // per document {digest, segments, observer length} of the last replay
  std::vector<uint64_t> digests;
  std::vector<DocState> hst;
  double lastKernelMs = 0;
  // rewind support: state right after the first upload of every document's records
  bool haveRewind = false;
  bool tightCaps = false;
  uint32_t variantDocs = 0;  // documents flagged DSF_VARIANT by the last mark_variant_docs  // slices sized by caps_for's tight formula (large batches; capacity retry in replay())
  std::vector<DocState> hPristine;
  DevBuf<DocState> dPristine;
  DevBuf<uint32_t> dPSeg;
  DevBuf<FBlk> dPBlk;
  DevBuf<uint32_t> dPX;             // loaded documents: initial blocks / segp / lists / aux words
  DevBuf<uint32_t> dDelta;          // catch-up delta entries (4 words each), per-document slices
  DevBuf<uint32_t> dSched;          // ticket scheduler words (mtb_replay_tick_kernel)
  uint32_t waveSlots = 0;           // resident replay waves of the device (CUs x the sched kernel's occupancy)
  uint32_t nXcc = 0;                // XCDs of the device (the ticket scheduler's queues)
  mtb_launch_info launch{};         // what the last replay launched (mtb_launch_info)
  uint32_t schedWords[MTB_SCHED_BAD + 5 - MTB_SCHED_ABORT] = {};  // sched[MTB_SCHED_ABORT ..] after the launch
  uint32_t schedSpins = 0;  // (source of the wait bound's copy to the device)
  std::vector<uint32_t> schedPlan;  // the ticket scheduler's chunk plan (host copy of the uploaded one)
  Chunks pxSave[5], pxRestore[5];
  std::vector<std::array<uint64_t, 10>> pxDoc;  // per document: dPX offset and words of each pool's saved image
  bool residentLoad = false;        // the resident records start with LOADSEG records
  bool live = false;                // a document of the batch has made local ops (mtb_local_op_json)
  bool matrix = false;              // MTB_BATCH_MATRIX: documents 2m / 2m+1 are matrix m's rows / cols
  std::vector<std::string> cellVals{"null"};                 // setCell values (JSON text), id 0 = undefined
  std::unordered_map<std::string, uint32_t> cellValIds;
  // batched moves: chunk tables and host->device staging
  DevBuf<uint64_t> dMvSrc, dMvDst;
  DevBuf<uint32_t> dMvLen, dStageW;
  DevBuf<uint16_t> dStageH;
  ~mtb_dev() {
    dDocs.release(); dOps.release(); dSegs.release(); dBlks.release(); dLists.release(); dText.release();
    dHeap.release(); dAux.release(); dFree.release(); dPool.release(); dPidx.release(); dValClass.release();
    dKeyIrr.release(); dValLocal.release(); dIrr.release();
    dKeyRank.release(); dValFalsy.release(); dPristine.release(); dPSeg.release(); dPBlk.release(); dPX.release(); dDelta.release(); dSched.release(); dKHash.release(); dVHash.release(); dDigest.release();
    dMvSrc.release(); dMvDst.release(); dMvLen.release(); dStageW.release(); dStageH.release();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

template <class F>
int guarded(mtb_dev* b, F&& f) {
  if (!b) return MTB_E_ARG;
  // HIP's current device is per host thread: a batch driven from several threads (the multi-device
  // front end replays its shards in parallel) selects its device on every entry
  if (b->stream) (void)hipSetDevice(b->device);
  try {
    f();
    return MTB_OK;
  } catch (const MtbError& e) {
    b->err = e.msg;
    return e.code;
  } catch (const hj::ParseError& e) {
    b->err = std::string("JSON: ") + e.what();
    return MTB_E_PARSE;
  } catch (const std::exception& e) {
    b->err = e.what();
    return MTB_E_ARG;
  }
}

HostDoc& docref(mtb_dev* b, uint32_t doc) {
  if (doc >= b->ndocs) raise(MTB_E_ARG, "document index out of range");
  return b->docs[doc];
}

const hj::Value* member(const hj::Value& o, const char16_t* k) { return o.kind == hj::Value::kObj ? o.find(k) : nullptr; }

uint32_t u32field(const hj::Value& o, const char16_t* k, const char* what) {
  const hj::Value* v = member(o, k);
  if (!v || v->kind != hj::Value::kNum || v->n < 0 || v->n > 4294967295.0 || v->n != std::floor(v->n))
    raise(MTB_E_PARSE, std::string("missing or invalid ") + what);
  return (uint32_t)v->n;
}

// Map keys of marker ids (Marker.getId, mergeTreeNodes.ts:612-617; idToSegment, mergeTree.ts:549): the
// JS Map identity of the primitive values a JSON id can hold; falsy ids are no ids, object ids never match
std::optional<std::string> marker_key(const hj::Value* v) {
  if (!v || !v->truthy()) return std::nullopt;
  switch (v->kind) {
    case hj::Value::kStr: return "s" + hj::to_utf8(v->s.data(), v->s.size());
    case hj::Value::kNum: return "n" + hj::number(v->n);
    case hj::Value::kBool: return std::string("t");
    default: return std::nullopt;
  }
}
// The ordinal + 1 of the id of a marker inserted with `props` (0: no id); a reused id becomes ambiguous.
uint32_t marker_ord(HostDoc& d, const hj::Value* props) {
  if (!props || props->kind != hj::Value::kObj) return 0;
  auto key = marker_key(member(*props, u"markerId"));
  if (!key) return 0;
  auto [it, fresh] = d.markerOrd.try_emplace(*key, (uint32_t)d.markerAmbig.size());
  if (fresh) d.markerAmbig.push_back(0);
  else d.markerAmbig[it->second] = d.markerDup = true;
  return it->second + 1;
}
uint32_t marker_key_id(const Interner& in) {
  auto k = in.keyId.find(U16(u"markerId"));
  return k == in.keyId.end() ? MTB_NONE : k->second;
}
// the JSON text of an interned props id's markerId (property set, or op-props list), or nullptr
const std::string* props_marker_json(const Interner& in, uint32_t props, bool opList) {
  if (!props || props >= in.pidx.size() / 2) return nullptr;
  auto k = in.keyId.find(U16(u"markerId"));
  if (k == in.keyId.end()) return nullptr;
  const uint32_t off = in.pidx[2 * props + (opList ? 0 : 1)];
  for (uint32_t i = 0; i < in.pool[off]; i++)
    if (in.pool[off + 1 + 2 * i] == k->second) {
      static const std::string null = "null";
      const uint32_t v = in.pool[off + 2 + 2 * i];
      if (v != MTB_NONE && v >= in.valJson.size()) return nullptr;  // (an incr's result table, not a value)
      return v == MTB_NONE ? &null : &in.valJson[v];
    }
  return nullptr;
}

// getValidOpRange (client.ts:527-547): `pos1` / `pos2` when present, else the IRelativePosition
// `relativePos1` / `relativePos2` (ops.ts:77-92), packed as a descriptor the kernel resolves with
// posFromRelativePos (mergeTree.ts:1371-1395) in the op's view (MTB_F_RELPOS, mtb_device.h).
uint32_t position(const hj::Value& op, const char16_t* k, const char16_t* rel, HostDoc* d = nullptr, mtb_op* r = nullptr) {
  const hj::Value* v = member(op, k);
  if (v && v->kind == hj::Value::kNum) return (uint32_t)v->n;
  const hj::Value* rp = member(op, rel);
  if (rp && rp->truthy()) {
    if (!d) raise(MTB_E_UNSUPPORTED, "unsupported: relative positions in a matrix batch");
    if (rp->kind != hj::Value::kObj) raise(MTB_E_UNSUPPORTED, "unsupported: relative position is not an object");
    auto key = marker_key(member(*rp, u"id"));
    if (!key) raise(MTB_E_UNSUPPORTED, "unsupported: relative position without a marker id (posFromRelativePos -1)");
    auto it = d->markerOrd.find(*key);
    if (it == d->markerOrd.end())
      raise(MTB_E_UNSUPPORTED, "unsupported: relative position names no marker of the document (posFromRelativePos -1)");
    const hj::Value* off = member(*rp, u"offset");
    double o = 0;
    if (off && off->kind != hj::Value::kNull) {
      if (off->kind != hj::Value::kNum || off->n != std::floor(off->n) || std::fabs(off->n) > 1e9)
        raise(MTB_E_UNSUPPORTED, "unsupported: non-integer relative position offset");
      o = off->n;
    }
    const hj::Value* before = member(*rp, u"before");
    const uint32_t ord = it->second, ov = (uint32_t)(int32_t)o;
    const uint32_t at = (uint32_t)d->payload.size();
    const uint16_t desc[6] = {(uint16_t)ord, (uint16_t)(ord >> 16), (uint16_t)(before && before->truthy()), 0,
                              (uint16_t)ov, (uint16_t)(ov >> 16)};
    d->payload.insert(d->payload.end(), desc, desc + 6);
    r->flags |= MTB_F_RELPOS;
    return MTB_RELPOS | at;
  }
  raise(MTB_E_UNSUPPORTED, "unsupported: op without numeric position");
}

// An annotate's props.markerId as the device compares it with an annotated marker's own id (JS ===): 1 = a
// primitive (equal iff the interned value ids are), 2 = null, an object or an array (equal to nothing).
uint32_t annot_marker_test(const hj::Value* v) {
  return (v->kind == hj::Value::kStr || v->kind == hj::Value::kNum || v->kind == hj::Value::kBool) ? 1u : 2u;
}

// One delta op -> record (client.ts:489-524 insert, :430 remove, :457 annotate)
void pack_delta(mtb_dev* b, HostDoc& d, const hj::Value& op, mtb_op base, std::vector<mtb_op>& out) {
  const hj::Value* t = member(op, u"type");
  const int type = t && t->kind == hj::Value::kNum ? (int)t->n : -1;
  mtb_op r = base;
  // relative positions: SharedString batches (catch-up tracking included: a message that saw everything before
  // it is stored verbatim, relative positions and all, and a lagging one is rewritten from its delta entries,
  // sequence.ts:704-726); not in matrix batches
  HostDoc* rel = b->matrix ? nullptr : &d;
  if (type == 0) {
    r.pos1 = position(op, u"pos1", u"relativePos1", rel, &r);
    const hj::Value* seg = member(op, u"seg");
    if (!seg || !seg->truthy()) {  // applyInsertOp: `if (op.seg)` -> no-op member
      r.type = MTB_OP_NOOP;
      out.push_back(r);
      return;
    }
    r.type = MTB_OP_INSERT;
    const U16* text = nullptr;
    const hj::Value* props = nullptr;
    if (d.perm) {  // PermutationSegment.fromJSONObject([length, start]) (permutationvector.ts:45-48)
      if (seg->kind != hj::Value::kArr || seg->items.empty() || seg->items[0].kind != hj::Value::kNum ||
          seg->items[0].n < 0 || seg->items[0].n > 1e9 || seg->items[0].n != std::floor(seg->items[0].n))
        raise(MTB_E_PARSE, "PermutationVector insert without a [length, start] segment");
      r.flags |= MTB_F_PERMSEG;
      r.pos2 = (uint32_t)seg->items[0].n;
      out.push_back(r);
      return;
    }
    if (seg->kind == hj::Value::kStr) {
      text = &seg->s;
    } else if (seg->kind == hj::Value::kObj && member(*seg, u"text")) {
      const hj::Value* tv = member(*seg, u"text");
      if (tv->kind != hj::Value::kStr) raise(MTB_E_UNSUPPORTED, "unsupported: non-string text segment");
      text = &tv->s;
      props = member(*seg, u"props");
      r.flags |= MTB_F_SEGOBJ;
    } else if (seg->kind == hj::Value::kObj && member(*seg, u"marker")) {
      r.flags |= MTB_F_MARKER;
      const hj::Value* mk = member(*seg, u"marker");
      const hj::Value* rt = mk ? member(*mk, u"refType") : nullptr;
      r.pos2 = (rt && rt->kind == hj::Value::kNum) ? (uint32_t)rt->n : 0xFFFFFFFFu;
      props = member(*seg, u"props");
      r.payload = marker_ord(d, props && props->truthy() ? props : nullptr);
    } else {
      raise(MTB_E_PARSE, "Unrecognized IJSONSegment type");
    }
    if (text) {
      r.pos2 = (uint32_t)text->size();
      r.payload = (uint32_t)d.payload.size();
      d.payload.insert(d.payload.end(), text->begin(), text->end());
    }
    if (props && props->truthy()) {
      if (props->kind != hj::Value::kObj) raise(MTB_E_UNSUPPORTED, "unsupported: non-object segment props");
      r.props = b->in.props(*props);
      d.vals.propsSeen.push_back(r.props);
    }
    out.push_back(r);
  } else if (type == 1 || type == 2) {
    r.type = type == 1 ? MTB_OP_REMOVE : MTB_OP_ANNOTATE;
    r.pos1 = position(op, u"pos1", u"relativePos1", rel, &r);
    r.pos2 = position(op, u"pos2", u"relativePos2", rel, &r);
    if (type == 2) {
      const hj::Value* props = member(op, u"props");
      if (props && props->kind == hj::Value::kObj)
        if (const hj::Value* mid = member(*props, u"markerId")) {  // assert 0x5ad's operand (mergeTree.ts:1912-1918)
          d.markerIdAnnot = true;
          r.payload = annot_marker_test(mid);
        }
      hj::Value empty;
      empty.kind = hj::Value::kObj;
      r.props = b->in.props(props && props->kind == hj::Value::kObj ? *props : empty);
      d.vals.propsSeen.push_back(r.props);
      const hj::Value* comb = member(op, u"combiningOp");
      if (comb && comb->kind == hj::Value::kObj) {
        const hj::Value* name = member(*comb, u"name");
        if (name && name->kind == hj::Value::kStr && name->s == u"rewrite") {
          r.flags |= MTB_F_REWRITE;
        } else if (name && name->kind == hj::Value::kStr && name->s == u"incr") {
          // combine(op, previous, undefined) (segmentPropertiesManager.ts:145-147, properties.ts:24-69): NaN for a
          // number / boolean / absent previous value (defaultValue absent or numeric), string concatenation for a
          // string, object or array one (its String() form; Interner::incr_props)
          const hj::Value* dv = member(*comb, u"defaultValue");
          const hj::Value* mv = member(*comb, u"minValue");
          r.flags |= MTB_F_INCR;
          b->in.nan();
          r.props = b->in.incr_props(r.props, dv, mv, &d.vals);
        } else if (name && name->kind == hj::Value::kStr && name->s == u"consensus") {
          // A live client's own consensus annotate is its value {value: undefined, seq: -1}, completed in place at
          // the ack through Client.pendingConsensus (client.ts:1050-1058), which only annotateMarkerNotifyConsensus
          // fills (:155-181; the op createAnnotateMarkerOp makes, flagged "notifyConsensus": true by the caller).
          // Any other local consensus annotate leaves a minimum-sequence-number listener that dereferences the
          // missing entry: the reference throws later, refused here.
          int cseq = (int)r.seq;
          if (r.client == (uint16_t)MTB_LOCAL_CLIENT)
            raise(MTB_E_UNSUPPORTED, "unsupported: consensus annotate on a detached client");
          if (r.flags & MTB_F_LOCAL) {
            const hj::Value* nc = member(op, u"notifyConsensus");
            const hj::Value* r1 = member(op, u"relativePos1");
            const hj::Value* id = r1 && r1->kind == hj::Value::kObj ? member(*r1, u"id") : nullptr;
            if (!nc || nc->kind != hj::Value::kBool || !nc->b || !id || member(*comb, u"defaultValue"))
              raise(MTB_E_UNSUPPORTED, "unsupported: local consensus annotate other than annotateMarkerNotifyConsensus "
                                       "(the reference throws at a later minimum sequence number update)");
            d.pendingConsensus.insert(hj::dump(*id));
            cseq = -1;  // UnassignedSequenceNumber
          }
          r.flags |= MTB_F_CONSENSUS;
          r.props = b->in.consensus_props(r.props, member(*comb, u"defaultValue"), cseq);
          d.vals.propsSeen.push_back(r.props);
        } else {
          raise(MTB_E_UNSUPPORTED, "unsupported: combiningOp other than rewrite / incr / consensus");
        }
      }
    }
    out.push_back(r);
  } else if (type == 3) {
    const hj::Value* ops = member(op, u"ops");
    if (ops && ops->kind == hj::Value::kArr)
      for (auto& m : ops->items) pack_delta(b, d, m, base, out);
  } else {
    r.type = MTB_OP_NOOP;
    out.push_back(r);
  }
}

// ------------------------------------------------------------------ SnapshotV1 load (host side)
// specToSegment (snapshotLoader.ts:94-131) over the segment spec of textSegment.ts / Marker.make: a
// spec with merge info is {json, client?, seq?, removedSeq?, removedClient?, removedClientIds?}; its
// client ids are interned in the order they are met.  Text goes to `sink` (offsets are into it).
// Props interning for parallel loads: a per-thread cache in front of the batch's (locked) props table.
struct PropsCache {
  std::mutex* mu = nullptr;
  std::unordered_map<std::string, uint32_t> ids;
};

LoadSeg load_spec(mtb_dev* b, HostDoc& d, const hj::Value& spec, std::vector<uint16_t>& sink, PropsCache* pc) {
  LoadSeg g;
  const bool mergeInfo = spec.kind == hj::Value::kObj && member(spec, u"json");
  const hj::Value& js = mergeInfo ? *member(spec, u"json") : spec;
  const hj::Value* props = nullptr;
  const U16* text = nullptr;
  if (d.perm) {  // PermutationSegment.fromJSONObject([length, start]) (permutationvector.ts:45-48)
    if (js.kind != hj::Value::kArr || js.items.size() < 2 || js.items[0].kind != hj::Value::kNum)
      raise(MTB_E_PARSE, "Unrecognized PermutationSegment spec");
    g.len = (uint32_t)js.items[0].n;
    g.text = js.items[1].kind == hj::Value::kNum ? (uint32_t)(int32_t)js.items[1].n : MTB_HANDLE_UNALLOC;
  } else if (js.kind == hj::Value::kStr) {
    text = &js.s;
  } else if (js.kind == hj::Value::kObj && member(js, u"text")) {
    const hj::Value* tv = member(js, u"text");
    if (tv->kind != hj::Value::kStr) raise(MTB_E_UNSUPPORTED, "unsupported: non-string text segment");
    text = &tv->s;
    props = member(js, u"props");
  } else if (js.kind == hj::Value::kObj && member(js, u"marker")) {
    const hj::Value* mk = member(js, u"marker");
    const hj::Value* rt = mk ? member(*mk, u"refType") : nullptr;
    g.marker = true;
    g.len = 1;
    g.text = MTB_MARKER | ((rt && rt->kind == hj::Value::kNum) ? (uint32_t)rt->n + 1 : 0u);
    props = member(js, u"props");
    g.mord = marker_ord(d, props && props->truthy() ? props : nullptr);
  } else {
    raise(MTB_E_PARSE, "Unrecognized IJSONSegment type");
  }
  if (text) {
    g.len = (uint32_t)text->size();
    g.text = (uint32_t)sink.size();
    sink.insert(sink.end(), text->begin(), text->end());
  }
  if (props && props->truthy()) {
    if (props->kind != hj::Value::kObj) raise(MTB_E_UNSUPPORTED, "unsupported: non-object segment props");
    if (pc) {  // parallel loads share the batch's props table
      std::string js = hj::dump(*props);
      auto it = pc->ids.find(js);
      if (it != pc->ids.end()) {
        g.props = it->second;
      } else {
        {
          std::lock_guard<std::mutex> lk(*pc->mu);
          g.props = b->in.props_keyed(js, *props);
        }
        pc->ids.emplace(std::move(js), g.props);
      }
    } else {
      g.props = b->in.props(*props);
    }
    d.vals.propsSeen.push_back(g.props);
  }
  if (!mergeInfo) return g;  // seq = UniversalSequenceNumber, client = NonCollabClient
  auto cid = [&](const hj::Value& v) -> int16_t {
    if (v.kind != hj::Value::kStr) raise(MTB_E_PARSE, "client id in a segment spec is not a string");
    return (int16_t)d.client(hj::to_utf8(v.s.data(), v.s.size()));
  };
  const hj::Value* c = member(spec, u"client");
  if (c && c->kind == hj::Value::kStr) g.client = cid(*c);
  const hj::Value* sq = member(spec, u"seq");
  if (sq && sq->kind == hj::Value::kNum) g.seq = (int32_t)sq->n;
  const hj::Value* rs = member(spec, u"removedSeq");
  if (rs && rs->kind == hj::Value::kNum) g.rseq = (int32_t)rs->n;
  std::vector<int16_t> rcs;
  const hj::Value* rc = member(spec, u"removedClient");
  if (rc && rc->kind == hj::Value::kStr) rcs = {cid(*rc)};
  const hj::Value* rcl = member(spec, u"removedClientIds");
  if (rcl && rcl->kind == hj::Value::kArr) {
    rcs.clear();
    for (auto& x : rcl->items) rcs.push_back(cid(x));
  }
  if (!rcs.empty()) g.rc0 = rcs[0];
  if (rcs.size() > 1) {
    if (d.img.aux.empty()) d.img.aux.push_back(0);  // aux word 0 means "no list"
    g.rcx = (uint32_t)d.img.aux.size();
    d.img.aux.push_back((uint32_t)(rcs.size() - 1));
    for (size_t i = 1; i < rcs.size(); i++) d.img.aux.push_back((uint32_t)(int32_t)rcs[i]);
  }
  return g;
}

uint32_t seg_cli_word(const LoadSeg& g) { return ((uint32_t)(uint16_t)g.client) | ((uint32_t)(uint16_t)g.rc0 << 16); }

// reloadFromSegments (mergeTree.ts:678-721): the segments bottom-up, MaxNodesInBlock-1 = 7 children per
// block, followed by startCollaboration's combine of every block (the window list of a block whose
// children are blocks holds, per child slot, the entries derived from that child's leaves: insert
// (seq, client, +len) for seq > minSeq, removal (removedSeq, removedClientIds[0], -len) and overlapping
// removers (removedSeq, c, OVERLAP, +len) for removedSeq > minSeq — the same derivation the kernel's
// list rebuild uses).
void build_load_image(HostDoc& d, const std::vector<LoadSeg>& hdr) {
  LoadImage& im = d.img;
  if (im.aux.empty()) im.aux.push_back(0);
  const int32_t minSeq = (int32_t)d.min0;
  im.segp.assign(hdr.size(), MTB_NONE);
  im.blks.clear();
  im.lists.assign(MTB_LIST_RESERVED, WEnt{});
  for (auto& e : im.lists) e.seq = e.ck = e.delta = e.pad = (int32_t)MTB_NONE;  // empty free-list heads
  auto blank = [] {
    FBlk f{};
    for (int k = 0; k < MTB_MAXCH; k++) f.f[F_ID][k] = MTB_NONE;
    f.parent = MTB_NONE;
    f.scour = -1;  // needsScour undefined
    f.lseq = MTB_NOKEY;
    return f;
  };
  struct Node {
    uint32_t id;
    int32_t olen;
    uint32_t loff = 0, lcnt = 0, lcap = 0;
    std::vector<WEnt> ents;  // untagged entries of the subtree
  };
  auto derived = [&](const LoadSeg& g, std::vector<WEnt>& out) {
    if (g.seq > minSeq) out.push_back(WEnt{g.seq, (int32_t)WE_KEY((uint32_t)(uint16_t)g.client, WK_MAIN, 0), (int32_t)g.len, 0});
    if (g.rseq >= 0 && g.rseq > minSeq) {
      out.push_back(WEnt{g.rseq, (int32_t)WE_KEY((uint32_t)(uint16_t)g.rc0, WK_MAIN, 0), -(int32_t)g.len, 0});
      if (g.rcx)
        for (uint32_t i = 0; i < im.aux[g.rcx]; i++)
          out.push_back(WEnt{g.rseq, (int32_t)WE_KEY(im.aux[g.rcx + 1 + i] & 0xFFFF, WK_OVERLAP, 0), (int32_t)g.len, 0});
    }
  };
  std::vector<Node> level;
  for (size_t i = 0; i < hdr.size(); i++) {
    Node n;
    n.id = MTB_LEAF | (uint32_t)i;
    n.olen = hdr[i].rseq >= 0 ? 0 : (int32_t)hdr[i].len;  // localNetLength ?? 0
    derived(hdr[i], n.ents);
    level.push_back(std::move(n));
  }
  const uint32_t maxChildren = MTB_MAXCH - 1;
  while (true) {
    std::vector<Node> up;
    const size_t nb = level.empty() ? 1 : (level.size() + maxChildren - 1) / maxChildren;
    size_t ni = 0;
    for (size_t bi = 0; bi < nb; bi++) {
      const uint32_t id = (uint32_t)im.blks.size();
      FBlk f = blank();
      Node n;
      n.id = id;
      n.olen = 0;
      bool internal = false;
      uint32_t k = 0;
      for (; k < maxChildren && ni < level.size(); k++, ni++) {
        Node& c = level[ni];
        f.f[F_ID][k] = c.id;
        if (c.id & MTB_LEAF) {
          const LoadSeg& g = hdr[c.id & ~MTB_LEAF];
          f.f[F_LEN][k] = g.len;
          f.f[F_SEQ][k] = (uint32_t)g.seq;
          f.f[F_RSEQ][k] = (uint32_t)g.rseq;
          f.f[F_CLI][k] = seg_cli_word(g);
          f.f[F_RCX][k] = g.rcx;
          f.f[F_PROPS][k] = g.props;  // props id; resolve_load_props turns it into the device handle
          f.f[F_TEXT][k] = g.text;
          im.segp[c.id & ~MTB_LEAF] = id;
        } else {
          internal = true;
          f.f[F_LEN][k] = (uint32_t)c.olen;
          f.f[F_SEQ][k] = c.loff;
          f.f[F_RSEQ][k] = c.lcnt;
          f.f[F_CLI][k] = c.lcap;
          im.blks[c.id].parent = id;
          im.blks[c.id].index = k;
        }
        n.olen += c.olen;
      }
      f.count = k;
      f.len = n.olen;
      if (internal) {
        // the block's window list: its children's entries tagged with their slot
        uint32_t cnt = 0;
        for (size_t j = ni - k; j < ni; j++) cnt += (uint32_t)level[j].ents.size();
        uint32_t cap = 8;
        while (cap < cnt + cnt / 2 + 4) cap <<= 1;
        n.loff = (uint32_t)im.lists.size();
        n.lcnt = cnt;
        n.lcap = cap;
        for (size_t j = ni - k; j < ni; j++)
          for (WEnt e : level[j].ents) {
            e.ck |= (int32_t)((j - (ni - k)) << 20);
            im.lists.push_back(e);
          }
        // window lists are kept in seq order (MTB_LUNSORTED clear): views read only their tail
        std::stable_sort(im.lists.begin() + n.loff, im.lists.end(), [](const WEnt& a, const WEnt& b) { return a.seq < b.seq; });
        im.lists.resize(n.loff + cap, WEnt{});
      }
      for (size_t j = ni - k; j < ni; j++) {
        n.ents.insert(n.ents.end(), level[j].ents.begin(), level[j].ents.end());
        std::vector<WEnt>().swap(level[j].ents);
      }
      im.blks.push_back(f);
      up.push_back(std::move(n));
    }
    if (up.size() == 1) {
      im.root = up[0].id;
      FBlk& r = im.blks[im.root];
      r.loff = up[0].loff;
      r.lcnt = up[0].lcnt;
      r.lcap = up[0].lcap;
      break;
    }
    level = std::move(up);
  }
}

// Header segments' props ids -> global property-set handles (after every parallel load has interned).
void resolve_load_props(mtb_dev* b, HostDoc& d) {
  for (FBlk& f : d.img.blks)
    for (uint32_t k = 0; k < f.count; k++)
      if ((f.f[F_ID][k] & MTB_LEAF) && f.f[F_PROPS][k]) f.f[F_PROPS][k] = MTB_GPROPS | b->in.pidx[2 * f.f[F_PROPS][k] + 1];
}

// toLatestVersion (snapshotChunks.ts:151-175): a SnapshotLegacy chunk (no "version"; MergeTreeChunkLegacy)
// read as the V1 chunk the loader expects -- segments = segmentTexts, segmentCount = chunkSegmentCount -- and a
// legacy header's metadata from buildHeaderMetadataForLegacyChunk (:178-199): [header] + [body] when
// chunkLengthChars < totalLengthChars, minSequenceNumber = chunkMinSequenceNumber (absent in SnapshotLegacy's
// output: the loader then takes sequenceNumber), sequenceNumber = chunkSequenceNumber.
hj::Value to_latest_version(const std::string& path, hj::Value chunk) {
  if (chunk.kind != hj::Value::kObj) raise(MTB_E_PARSE, "summary chunk is not an object");
  const hj::Value* ver = member(chunk, u"version");
  if (ver && ver->kind == hj::Value::kStr && ver->s == u"1") return chunk;
  if (ver && ver->kind != hj::Value::kUndef) raise(MTB_E_PARSE, "Unsupported chunk path: " + path);
  hj::Value v;
  v.kind = hj::Value::kObj;
  auto put = [&](hj::Value& o, const char16_t* k, const hj::Value* x) {
    if (x) o.members.push_back({k, *x});
  };
  hj::Value one;
  one.kind = hj::Value::kStr;
  one.s = u"1";
  v.members.push_back({u"version", one});
  put(v, u"segmentCount", member(chunk, u"chunkSegmentCount"));
  if (path == "header") {
    if (const hj::Value* hm = member(chunk, u"headerMetadata")) {
      put(v, u"headerMetadata", hm);
    } else {
      hj::Value md, ids;
      md.kind = hj::Value::kObj;
      ids.kind = hj::Value::kArr;
      auto idv = [](const char16_t* id) {
        hj::Value o, sv;
        o.kind = hj::Value::kObj;
        sv.kind = hj::Value::kStr;
        sv.s = id;
        o.members.push_back({u"id", sv});
        return o;
      };
      ids.items.push_back(idv(u"header"));
      const hj::Value* cl = member(chunk, u"chunkLengthChars");
      const hj::Value* tl = member(chunk, u"totalLengthChars");
      if (cl && tl && cl->kind == hj::Value::kNum && tl->kind == hj::Value::kNum && cl->n < tl->n)
        ids.items.push_back(idv(u"body"));
      md.members.push_back({u"orderedChunkMetadata", ids});
      put(md, u"minSequenceNumber", member(chunk, u"chunkMinSequenceNumber"));
      put(md, u"sequenceNumber", member(chunk, u"chunkSequenceNumber"));
      put(md, u"totalSegmentCount", member(chunk, u"totalSegmentCount"));
      v.members.push_back({u"headerMetadata", md});
    }
  }
  put(v, u"segments", member(chunk, u"segmentTexts"));
  return v;
}

// Client.load of one SnapshotV1 (or SnapshotLegacy) summary into the fresh document d (client.ts:1007 ->
// SnapshotLoader, snapshotLoader.ts:41-257).  `mu` guards the batch's props table when documents load in
// parallel.  The catch-up messages blob of a legacy summary is the caller's (SharedSegmentSequence.loadCore
// applies it, sequence.ts:568-610).
void load_one(mtb_dev* b, HostDoc& d, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id,
              PropsCache* pc, const std::string& prefix = std::string()) {
  if (b->matrix && !d.perm) raise(MTB_E_ARG, "matrix batch: use mtb_matrix_load");
  if (d.inited || d.onDevice) raise(MTB_E_ARG, "document already initialised");
  if (!observer_long_id) raise(MTB_E_ARG, "observer long client id required");
  if (nblobs && !blobs) raise(MTB_E_ARG, "null blob array");
  auto blob = [&](const std::string& path) -> hj::Value {
    for (uint32_t i = 0; i < nblobs; i++)
      if (blobs[i].path && prefix + path == blobs[i].path) {
        if (!blobs[i].content && blobs[i].content_len) raise(MTB_E_ARG, "null blob content");
        return hj::parse(blobs[i].content ? blobs[i].content : "", blobs[i].content_len);
      }
    raise(MTB_E_ARG, "summary blob not found: " + prefix + path);
  };
  // loadHeader (snapshotLoader.ts:133-167)
  const hj::Value header = to_latest_version("header", blob("header"));
  const hj::Value* hsegs = member(header, u"segments");
  const hj::Value* md = member(header, u"headerMetadata");
  if (!hsegs || hsegs->kind != hj::Value::kArr || !md || md->kind != hj::Value::kObj)
    raise(MTB_E_PARSE, "header metadata not available");
  std::vector<LoadSeg> hdr;
  hdr.reserve(hsegs->items.size());
  for (auto& sp : hsegs->items) hdr.push_back(load_spec(b, d, sp, d.initText, pc));
  auto num = [&](const char16_t* k, double dflt) {
    const hj::Value* v = member(*md, k);
    return v && v->kind == hj::Value::kNum ? v->n : dflt;
  };
  const double seqNum = num(u"sequenceNumber", 0);
  const double minSeqNum = num(u"minSequenceNumber", seqNum);
  if (seqNum < 0 || minSeqNum < 0 || seqNum > 2147483647.0 || minSeqNum > seqNum)
    raise(MTB_E_PARSE, "invalid header sequence numbers");
  // startOrUpdateCollaboration(runtime.clientId ?? "snapshot", minSeq, seq) (snapshotLoader.ts:154)
  d.observer = observer_long_id;
  d.client(d.observer);
  d.min0 = (uint32_t)minSeqNum;
  d.cur0 = (uint32_t)seqNum;
  d.lastSeq = (int64_t)seqNum;
  // loadBody (snapshotLoader.ts:169-220): chunks 1.. of orderedChunkMetadata, appended at the end
  std::vector<LoadSeg> body;
  const hj::Value* ocm = member(*md, u"orderedChunkMetadata");
  // (chunk1.segmentCount === headerMetadata.totalSegmentCount: nothing more to load, snapshotLoader.ts:180)
  const hj::Value* hsc = member(header, u"segmentCount");
  const hj::Value* tsc = member(*md, u"totalSegmentCount");
  const bool complete = hsc && tsc && hsc->kind == hj::Value::kNum && tsc->kind == hj::Value::kNum && hsc->n == tsc->n;
  if (ocm && ocm->kind == hj::Value::kArr && !complete)
    for (size_t ci = 1; ci < ocm->items.size(); ci++) {
      const hj::Value* id = member(ocm->items[ci], u"id");
      if (!id || id->kind != hj::Value::kStr) raise(MTB_E_PARSE, "chunk metadata without an id");
      const std::string path = hj::to_utf8(id->s.data(), id->s.size());
      const hj::Value chunk = to_latest_version(path, blob(path));
      const hj::Value* cs = member(chunk, u"segments");
      if (cs && cs->kind == hj::Value::kArr)
        for (auto& sp : cs->items) body.push_back(load_spec(b, d, sp, d.payload, pc));
    }
  // the observer becomes engine id 0 (HostDoc::obsRef): swap it with the header's first client everywhere
  const uint16_t so = d.client(d.observer);
  if (so != 0) {
    auto sw = [&](int16_t& c) { c = (int16_t)(c == 0 ? so : c == (int16_t)so ? 0 : c); };
    auto swap_seg = [&](LoadSeg& g) {
      sw(g.client);
      sw(g.rc0);
      if (g.rcx)
        for (uint32_t i = 0; i < d.img.aux[g.rcx]; i++) {
          int16_t c = (int16_t)(int32_t)d.img.aux[g.rcx + 1 + i];
          sw(c);
          d.img.aux[g.rcx + 1 + i] = (uint32_t)(int32_t)c;
        }
    };
    for (auto& g : hdr) swap_seg(g);
    for (auto& g : body) swap_seg(g);
    std::swap(d.longIds[0], d.longIds[so]);
    d.shortOf[d.longIds[0]] = 0;
    d.shortOf[d.longIds[so]] = so;
    d.obsRef = so;
  }
  build_load_image(d, hdr);
  // body segments inserted by collaborating clients take blockUpdateLength's incremental path: the removed ones
  // leave phantom partial lengths, and an update that meets an entry at its own seq below newer ones leaves
  // deficits (mtb_replay.hip "phantom partial lengths"); the table starts empty and grows on the device
  {
    size_t nph = 0, ncol = 0;
    for (const LoadSeg& g : body) {
      nph += g.rseq >= 0 && g.client != -2;
      ncol += g.client != -2;
    }
    if (ncol && !d.perm) {
      const uint32_t cap = (uint32_t)std::min<size_t>(8 * nph + 2 * ncol + 16, 1u << 20);
      d.img.ph = (uint32_t)d.img.aux.size();
      d.img.aux.push_back(0);
      d.img.aux.push_back(cap);
      d.img.aux.resize(d.img.aux.size() + 8ull * cap, 0u);
      d.phantom = true;
    }
  }
  // idToSegment after reloadFromSegments: blockUpdate maps the live header markers (mergeTree.ts:296-306)
  if (!d.markerAmbig.empty()) {
    LoadImage& im = d.img;
    im.mk_map = (uint32_t)im.aux.size();
    im.mk_n = (uint32_t)d.markerAmbig.size();
    im.aux.resize(im.aux.size() + im.mk_n, MTB_NONE);
    std::vector<uint32_t> all;
    for (size_t i = 0; i < hdr.size(); i++)
      if (hdr[i].mord && hdr[i].rseq < 0) {
        im.aux[im.mk_map + hdr[i].mord - 1] = (uint32_t)i;
        all.push_back((uint32_t)i);
        all.push_back(hdr[i].mord - 1);
      }
    if (!all.empty()) {  // [n, cap, (segment, ordinal)*] for blockUpdate's re-mapping of reused ids
      im.mk_all = (uint32_t)im.aux.size();
      im.aux.push_back((uint32_t)all.size() / 2);
      im.aux.push_back((uint32_t)all.size() / 2);
      im.aux.insert(im.aux.end(), all.begin(), all.end());
    }
  }
  // body: runs of NonCollab/UniversalSeq segments share one insertSegments call; any other segment is
  // inserted alone with its own client and seq (snapshotLoader.ts:201-220)
  std::vector<mtb_op>& recs = d.pending;
  recs.reserve(body.size());
  size_t i = 0;
  while (i < body.size()) {
    const bool universal = body[i].client == -2 && body[i].seq == 0;
    size_t j = i + 1;
    if (universal)
      while (j < body.size() && body[j].client == -2 && body[j].seq == 0) j++;
    for (size_t k = i; k < j; k++) {
      const LoadSeg& g = body[k];
      if (g.rseq >= 0 && g.client != -2 && d.perm)
        raise(MTB_E_UNSUPPORTED, "unsupported: removed PermutationVector body segment inserted by a collaborating "
                                 "client (blockUpdateLength's incremental path, mergeTree.ts:2419-2431)");
      mtb_op r{};
      r.type = MTB_OP_LOADSEG;
      r.flags = (uint8_t)((g.marker ? MTB_F_MARKER : 0) | (k == i ? MTB_F_LDFIRST : 0) | (k + 1 == j ? MTB_F_LDLAST : 0));
      r.client = (uint16_t)g.client;
      r.seq = (uint32_t)g.seq;
      r.ref_seq = (uint32_t)g.rseq;
      r.msn = (uint16_t)g.rc0;
      r.pos1 = g.rcx;
      r.pos2 = g.marker ? (g.text & ~MTB_MARKER) - 1 : g.len;  // marker: refType (0xFFFFFFFF = undefined)
      r.payload = g.marker ? g.mord : g.text;  // marker: id ordinal + 1
      r.props = g.props;
      recs.push_back(r);
    }
    i = j;
  }
  d.totalOps += recs.size();
  d.totalPayload = d.payload.size();
  d.loaded = true;
  d.inited = true;
}

// ------------------------------------------------------------------ device management
void ensure_stream(mtb_dev* b) {
  if (b->stream) return;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) raise(MTB_E_NODEV, "no HIP device available (the engine has no CPU fallback)");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreate(&b->ev0));
  HIPCHK(hipEventCreate(&b->ev1));
}

void upload_chunks(mtb_dev* b, const Chunks& c) {
  b->dMvSrc.ensure(c.src.size());
  b->dMvDst.ensure(c.dst.size());
  b->dMvLen.ensure(c.len.size());
  HIPCHK(hipMemcpyAsync(b->dMvSrc.p, c.src.data(), c.src.size() * 8, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipMemcpyAsync(b->dMvDst.p, c.dst.data(), c.dst.size() * 8, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipMemcpyAsync(b->dMvLen.p, c.len.data(), c.len.size() * 4, hipMemcpyHostToDevice, b->stream));
}
// device words -> device words
void move_words(mtb_dev* b, const void* src, void* dst, const Chunks& c) {
  if (c.len.empty()) return;
  upload_chunks(b, c);
  HIPCHK(mtb_launch_move_words(b->stream, (const uint32_t*)src, b->dMvSrc.p, (uint32_t*)dst, b->dMvDst.p, b->dMvLen.p,
                               (uint32_t)c.len.size()));
  HIPCHK(hipStreamSynchronize(b->stream));
}
void move_u16(mtb_dev* b, const uint16_t* src, uint16_t* dst, const Chunks& c) {
  if (c.len.empty()) return;
  upload_chunks(b, c);
  HIPCHK(mtb_launch_move_u16(b->stream, src, b->dMvSrc.p, dst, b->dMvDst.p, b->dMvLen.p, (uint32_t)c.len.size()));
  HIPCHK(hipStreamSynchronize(b->stream));
}
// host words -> device (via one staging upload)
void scatter_words(mtb_dev* b, const std::vector<uint32_t>& host, void* dst, const Chunks& c) {
  if (c.len.empty()) return;
  b->dStageW.ensure(host.size());
  HIPCHK(hipMemcpyAsync(b->dStageW.p, host.data(), host.size() * 4, hipMemcpyHostToDevice, b->stream));
  move_words(b, b->dStageW.p, dst, c);
}
void scatter_u16(mtb_dev* b, const uint16_t* host, size_t n, uint16_t* dst, const Chunks& c) {
  if (c.len.empty()) return;
  b->dStageH.ensure(n);
  HIPCHK(hipMemcpyAsync(b->dStageH.p, host, n * 2, hipMemcpyHostToDevice, b->stream));
  move_u16(b, b->dStageH.p, dst, c);
}
void scatter_u16(mtb_dev* b, const std::vector<uint16_t>& host, uint16_t* dst, const Chunks& c) {
  scatter_u16(b, host.data(), host.size(), dst, c);
}
// f(i) for every document i, on up to 16 host threads (documents are independent)
template <class F>
void parallel_docs(uint32_t n, F&& f) {
  const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
  const uint32_t nt = std::min<uint32_t>(std::min<uint32_t>(16, hw), std::max<uint32_t>(1, n / 64));
  if (nt <= 1) {
    for (uint32_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<uint32_t> next{0};
  auto work = [&] {
    for (uint32_t i = next.fetch_add(64); i < n; i = next.fetch_add(64))
      for (uint32_t j = i; j < std::min(n, i + 64); j++) f(j);
  };
  std::vector<std::thread> ts;
  for (uint32_t t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

// Per-document slice capacities from the record count (see DESIGN.md "HBM layout").  `n` is the
// number of records the slices must hold (all records appended so far, times a growth margin).
struct Caps {
  uint32_t seg, blk, list, text, heap, aux;
};
// Two sizings.  Generous (batches whose slices take little HBM in total): several-fold headroom over the measured
// maxima -- bench documents (10k records) 15.7k segments, 743 blocks, 4.4k list entries, 10.5k aux words; the
// reference replay logs (2k records, long collab windows) 11.8k list entries, 21k aux words.  Tight (large batches,
// mtb_dev::tightCaps): about twice the maxima measured per record on the bench workload (MTB_USAGE_OUT: blocks
// 0.075, list entries 0.43, aux words 1.03, heap entries 0.014 per record), so 10,000 cfg2 documents take ~14 GiB
// instead of 44; a document that outgrows them in its first replay is laid out again with larger slices and
// replayed from its pristine state (replay(), "capacity retry"), so tight caps never change a result.  Segments
// never exceed 2 per record (+ the initial one) in either sizing.
double caps_scale() {  // MTB_CAPS_SCALE: scales the tight caps (tests force the capacity retry with small values)
  const char* v = getenv("MTB_CAPS_SCALE");
  return v ? std::max(0.0, atof(v)) : 1.0;
}
Caps caps_for(uint64_t n, uint64_t payload, uint64_t init, bool tight = false) {
  Caps c;
  c.seg = (uint32_t)(2 * n + 64);
  if (tight) {
    const double f = caps_scale();
    c.blk = (uint32_t)std::max<double>(8, f * (double)(n / 8 + 128));
    c.list = (uint32_t)std::max<double>(MTB_LIST_RESERVED + 16, f * (double)(n + 4096));
    c.text = (uint32_t)std::min<uint64_t>(10 * payload + 15 * init + 4096, 0xFFFFFFF0u);
    c.heap = (uint32_t)std::max<double>(4, f * (double)(n / 16 + 256));
    c.aux = (uint32_t)std::max<double>(64, f * (double)(2 * n + 2048));
    return c;
  }
  c.blk = (uint32_t)(n / 2 + 256);
  c.list = (uint32_t)(8 * n + 8192);
  // text: scour's appends re-copy merged runs, so the arena outgrows the payload (cfg2 documents use ~5.7x their
  // payload, the 1M-char cfg4 document ~16x: its long initial segments are split and re-merged); the initial
  // text counts 15x for that reason (these were the caps every batch ran with through round 3)
  c.text = (uint32_t)std::min<uint64_t>(10 * payload + 15 * init + 4096, 0xFFFFFFF0u);
  c.heap = (uint32_t)(n + 256);
  c.aux = (uint32_t)(16 * n + 4096);
  return c;
}
// caps_for plus what a loaded summary already occupies (header segments, blocks, lists, aux words)
Caps doc_caps(const HostDoc& d, uint64_t n, uint64_t payload, bool tight = false) {
  Caps c = caps_for(n, payload, d.initText.size(), tight);
  if (d.perm) c.text = (uint32_t)(2 * (d.totalSetcell + d.initText.size() / 2 + 4) + 64);  // the handle table (u32 words)
  if (d.loaded) {
    c.seg += (uint32_t)d.img.segp.size();
    c.blk += (uint32_t)d.img.blks.size() + (uint32_t)d.img.segp.size() / 4;
    c.list += (uint32_t)d.img.lists.size() * 2;
    c.aux += (uint32_t)d.img.aux.size();
  }
  // a live client's pending groups: directory entries (8 words, doubling) and member lists
  c.aux += (uint32_t)std::min<uint64_t>(48 * d.totalLocal, 1u << 30);
  if (!d.markerAmbig.empty()) c.aux += (uint32_t)std::min<uint64_t>(8 * n, 1u << 30);  // the id map and mk_all
  return c;
}
bool fits(const DocState& s, const Caps& c) {
  return s.seg_cap >= c.seg && s.blk_cap >= c.blk && s.list_cap >= c.list && s.text_cap >= c.text &&
         s.heap_cap >= c.heap && s.aux_cap >= c.aux;
}

// (Re)lay out every document's slices so that each holds at least `want[i]`, copying live state.
void layout(mtb_dev* b, const std::vector<Caps>& want) {
  b->haveRewind = false;  // slice bases move: the pristine snapshot is no longer valid
  std::vector<DocState> ns = b->hst;
  uint64_t seg = 0, blk = 0, lst = 0, txt = 0, hp = 0, ax = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    DocState& s = ns[i];
    const Caps& c = want[i];
    s.seg_cap = std::max(s.seg_cap, c.seg);
    s.blk_cap = std::max(s.blk_cap, c.blk);
    s.list_cap = std::max(s.list_cap, c.list);
    s.text_cap = std::max(s.text_cap, (c.text + 1) & ~1u);  // even: text slices stay u32-aligned (handle tables)
    s.heap_cap = std::max(s.heap_cap, c.heap);
    s.aux_cap = std::max(s.aux_cap, c.aux);
    s.seg_base = seg; seg += s.seg_cap;
    s.blk_base = blk; blk += s.blk_cap;
    s.list_base = lst; lst += s.list_cap;
    s.text_base = txt; txt += s.text_cap;
    s.heap_base = hp; hp += s.heap_cap;
    s.aux_base = ax; ax += s.aux_cap;
    s.free_base = s.blk_base;
  }
  // allocate the new pools and move every document's live prefix with one kernel per pool
  auto move = [&](auto& buf, uint64_t total, auto getBase, auto getUsed) {
    using T = std::remove_pointer_t<decltype(buf.p)>;
    T* np = nullptr;
    HIPCHK(hipMalloc((void**)&np, std::max<uint64_t>(total, 1) * sizeof(T)));
    if (buf.p) {
      Chunks c;
      const uint64_t w = sizeof(T) / 4;  // words per element (u16 handled separately)
      for (uint32_t i = 0; i < b->ndocs; i++) c.add(getBase(b->hst[i]) * w, getBase(ns[i]) * w, getUsed(b->hst[i]) * w);
      move_words(b, buf.p, np, c);
      (void)hipFree(buf.p);
    }
    buf.p = np;
    buf.n = total;
  };
  auto move_text = [&](uint64_t total) {
    uint16_t* np = nullptr;
    HIPCHK(hipMalloc((void**)&np, std::max<uint64_t>(total, 1) * 2));
    if (b->dText.p) {
      Chunks c;
      for (uint32_t i = 0; i < b->ndocs; i++) c.add(b->hst[i].text_base, ns[i].text_base, b->hst[i].text_used);
      move_u16(b, b->dText.p, np, c);
      (void)hipFree(b->dText.p);
    }
    b->dText.p = np;
    b->dText.n = total;
  };
  move(b->dSegs, seg, [](const DocState& s) { return s.seg_base; }, [](const DocState& s) { return (uint64_t)s.seg_used; });
  move(b->dBlks, blk, [](const DocState& s) { return s.blk_base; }, [](const DocState& s) { return (uint64_t)s.blk_used; });
  move(b->dLists, lst, [](const DocState& s) { return s.list_base; }, [](const DocState& s) { return (uint64_t)s.list_used; });
  move_text(txt);
  move(b->dHeap, hp, [](const DocState& s) { return s.heap_base; }, [](const DocState& s) { return (uint64_t)s.heap_cnt + 1; });
  move(b->dAux, ax + 8, [](const DocState& s) { return s.aux_base; }, [](const DocState& s) { return (uint64_t)s.aux_used; });
  move(b->dFree, blk, [](const DocState& s) { return s.free_base; }, [](const DocState& s) { return (uint64_t)s.free_top; });
  b->hst = ns;
}

void device_init(mtb_dev* b) {
  ensure_stream(b);
  b->hst.assign(b->ndocs, DocState{});
  std::vector<Caps> want(b->ndocs);
  // tight caps when the generous ones would take more than 8 GiB (MTB_CAPS=tight / generous forces either)
  double gen = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    const Caps c = doc_caps(d, d.totalOps, std::max<uint64_t>(d.totalPayload, d.payload.size()));
    gen += 4.0 * c.seg + (double)sizeof(FBlk) * c.blk + (double)sizeof(WEnt) * c.list + 2.0 * c.text +
           (double)sizeof(Lru) * c.heap + 4.0 * c.aux + 4.0 * c.blk;
  }
  const char* cm = getenv("MTB_CAPS");
  b->tightCaps = cm ? !strcmp(cm, "tight") : gen > 8.0 * (1ull << 30);
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    want[i] = doc_caps(d, d.totalOps, std::max<uint64_t>(d.totalPayload, d.payload.size()), b->tightCaps);
  }
  layout(b, want);
  // initial state: root block (+ the detached initial text segment), collaboration started
  std::vector<uint32_t> recs;
  std::vector<uint16_t> texts;
  Chunks segc, blkc, txtc, lstc, auxc;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    DocState& s = b->hst[i];
    s.new_mode = b->opts.new_length_calc;
    s.min_seq = (int32_t)d.min0;
    s.cur_seq = (int32_t)d.cur0;
    if (d.loaded) {
      // the reloaded header tree, its window lists and overlap lists, and the header text
      const LoadImage& im = d.img;
      s.root = im.root;
      s.blk_used = (uint32_t)im.blks.size();
      s.seg_used = (uint32_t)im.segp.size();
      s.list_used = (uint32_t)im.lists.size();
      s.aux_used = (uint32_t)im.aux.size();
      s.mk_map = im.mk_map;
      s.mk_n = im.mk_n;
      s.mk_all = im.mk_all;
      s.ph = im.ph;
      if (d.phantom) s.flags |= DSF_PHANTOM;
      s.heap_cnt = 0;
      s.text_used = (uint32_t)d.initText.size();
      segc.add(recs.size(), s.seg_base, im.segp.size());
      recs.insert(recs.end(), im.segp.begin(), im.segp.end());
      blkc.add(recs.size(), s.blk_base * (sizeof(FBlk) / 4), im.blks.size() * (sizeof(FBlk) / 4));
      const uint32_t* bwds = reinterpret_cast<const uint32_t*>(im.blks.data());
      recs.insert(recs.end(), bwds, bwds + im.blks.size() * (sizeof(FBlk) / 4));
      lstc.add(recs.size(), s.list_base * (sizeof(WEnt) / 4), im.lists.size() * (sizeof(WEnt) / 4));
      const uint32_t* lwds = reinterpret_cast<const uint32_t*>(im.lists.data());
      recs.insert(recs.end(), lwds, lwds + im.lists.size() * (sizeof(WEnt) / 4));
      auxc.add(recs.size(), s.aux_base, im.aux.size());
      recs.insert(recs.end(), im.aux.begin(), im.aux.end());
      txtc.add(texts.size(), s.text_base, d.initText.size());
      texts.insert(texts.end(), d.initText.begin(), d.initText.end());
      if (d.perm) s.flags |= DSF_PERM;  // a loaded PermutationVector: initText is its handle table
      d.onDevice = true;
      continue;
    }
    if (d.perm) {
      s.flags |= DSF_PERM;
      const uint16_t ht[4] = {1, 0, 1, 0};  // u32 [length 1, handles[0] = 1] (handletable.ts:22)
      txtc.add(texts.size(), s.text_base, 4);
      texts.insert(texts.end(), ht, ht + 4);
    }
    s.root = 0;
    s.blk_used = 1;
    s.aux_used = 1;
    s.heap_cnt = 0;
    s.list_used = 0;
    FBlk root{};
    for (int k = 0; k < MTB_MAXCH; k++) root.f[F_ID][k] = MTB_NONE;
    root.parent = MTB_NONE;
    root.scour = -1;
    root.lseq = (int32_t)0x80000000;
    if (!d.initText.empty()) {
      // the detached initial text: one segment, LocalClientId, seq 0 (client.replay.spec.ts:27)
      root.f[F_ID][0] = MTB_LEAF | 0;
      root.f[F_LEN][0] = (uint32_t)d.initText.size();
      root.f[F_SEQ][0] = 0;
      root.f[F_RSEQ][0] = (uint32_t)-1;
      root.f[F_CLI][0] = 0xFFFFu | 0xFFFF0000u;  // client -1, no remover
      root.f[F_TEXT][0] = 0;
      root.count = 1;
      root.len = (int32_t)d.initText.size();
      s.seg_used = 1;
      segc.add(recs.size(), s.seg_base, 1);
      recs.push_back(0);  // parent: root block 0
      txtc.add(texts.size(), s.text_base, d.initText.size());
      texts.insert(texts.end(), d.initText.begin(), d.initText.end());
    }
    s.text_used = d.perm ? 4u : (uint32_t)d.initText.size();
    blkc.add(recs.size(), s.blk_base * (sizeof(FBlk) / 4), sizeof(FBlk) / 4);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&root);
    recs.insert(recs.end(), w, w + sizeof(FBlk) / 4);
    d.onDevice = true;
  }
  if (!recs.empty()) {  // one upload, then one move per pool
    b->dStageW.ensure(recs.size());
    HIPCHK(hipMemcpyAsync(b->dStageW.p, recs.data(), recs.size() * 4, hipMemcpyHostToDevice, b->stream));
    move_words(b, b->dStageW.p, b->dSegs.p, segc);
    move_words(b, b->dStageW.p, b->dBlks.p, blkc);
    move_words(b, b->dStageW.p, b->dLists.p, lstc);
    move_words(b, b->dStageW.p, b->dAux.p, auxc);
  }
  scatter_u16(b, texts, b->dText.p, txtc);
  b->dDocs.ensure(b->ndocs);
  b->devInit = true;
}

void upload_tables(mtb_dev* b) {
  Interner& in = b->in;
  if (!in.dirty && b->dPool.p) return;
  auto up = [&](auto& buf, const auto& vec) {
    buf.ensure(vec.size() + 8);  // tail padding: the kernel reads property sets 5 words at a time
    if (!vec.empty())
      HIPCHK(hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice, b->stream));
  };
  up(b->dPool, in.pool);
  up(b->dPidx, in.pidx);
  up(b->dValClass, in.valClass);
  up(b->dValFalsy, in.valFalsy);
  up(b->dKeyRank, in.keyRank);
  {  // matchProperties of irregular keys' value pairs (Interner::irr_tables)
    std::vector<uint32_t> keyOff, localOf, bits;
    in.irr_tables(keyOff, localOf, bits);
    up(b->dKeyIrr, keyOff);
    up(b->dValLocal, localOf);
    up(b->dIrr, bits);
  }
  // state digest hashes of every interned key and value (DESIGN.md "State digest")
  std::vector<uint64_t> kh(in.keys.size()), vh(in.valJson.size());
  for (size_t k = 0; k < kh.size(); k++) kh[k] = fnv_bytes(hj::to_utf8(in.keys[k].data(), in.keys[k].size()));
  for (size_t v = 0; v < vh.size(); v++) vh[v] = fnv_bytes(in.valJson[v]);
  up(b->dKHash, kh);
  up(b->dVHash, vh);
  in.dirty = false;
}

Tables make_tables(mtb_dev* b) {
  Tables t;
  t.pool = b->dPool.p;
  t.pidx = b->dPidx.p;
  t.val_class = b->dValClass.p;
  t.val_falsy = b->dValFalsy.p;
  t.nan_val = b->in.nanVal == MTB_NONE ? MTB_NONE : b->in.nanVal | (b->in.anyCv ? MTB_NAN_CV : 0u);
  t.key_rank = b->dKeyRank.p;
  t.key_irr = b->dKeyIrr.p;
  t.val_local = b->dValLocal.p;
  t.irr = b->dIrr.p;
  t.irr_any = b->in.nIrr;
  t.delta = b->dDelta.p;
  t.class_trivial = b->in.classId.size() == b->in.valJson.size() && !b->in.nIrr ? 1u : 0u;
  t.mk_key = marker_key_id(b->in);
  return t;
}

// State digest v1 of every document (mtb_digest_kernel) after a replay: fills the stats' segments_final,
// text_units_final and checksum (sum of the per-document digests mod 2^64) and keeps the per-document
// values for mtb_doc_digests.
void run_digest(mtb_dev* b, mtb_stats& st) {
  b->dDigest.ensure(3ull * b->ndocs);
  HIPCHK(mtb_launch_digest(b->stream, b->ndocs, b->dDocs.p, b->dBlks.p, b->dText.p, b->dAux.p, b->dPool.p, b->dKHash.p,
                           b->dVHash.p, b->dDigest.p));
  b->digests.resize(3ull * b->ndocs);
  HIPCHK(hipMemcpyAsync(b->digests.data(), b->dDigest.p, b->digests.size() * 8, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  st.segments_final = st.text_units_final = st.checksum = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    st.checksum += b->digests[3ull * i];
    st.segments_final += b->digests[3ull * i + 1];
    st.text_units_final += b->digests[3ull * i + 2];
  }
  // + 24 B per final segment record + 2 B per final text unit (the state write-back term)
  st.bytes_alg += 24ull * st.segments_final + 2ull * st.text_units_final;
}

// Host views of a document from its downloaded slices: blocks from the records, segments from their
// parent's slot (hot fields live inline).
void populate_doc(HostDoc& d, const DocState& s, const FBlk* fb, const uint32_t* segp) {
  d.blks.assign(s.blk_used, Blk{});
  d.segs.assign(s.seg_used, Seg{});
  for (uint32_t k = 0; k < s.seg_used; k++) d.segs[k].parent = MTB_NONE;
  for (uint32_t bi = 0; bi < s.blk_used; bi++) {
    const FBlk& F = fb[bi];
    Blk& B = d.blks[bi];
    B.count = (uint8_t)std::min<uint32_t>(F.count, MTB_MAXCH);
    B.parent = F.parent;
    B.len = F.len;
    B.index = (uint8_t)F.index;
    B.scour = (int8_t)F.scour;
    for (int k = 0; k < MTB_MAXCH; k++) B.child[k] = k < B.count ? F.f[F_ID][k] : MTB_NONE;
    for (int k = 0; k < B.count; k++) {
      const uint32_t c = F.f[F_ID][k];
      if (!(c & MTB_LEAF)) continue;
      const uint32_t sid = c & ~MTB_LEAF;
      if (sid >= s.seg_used || segp[sid] != bi) continue;  // stale slot of a freed block
      Seg& g = d.segs[sid];
      g.len = (int32_t)F.f[F_LEN][k];
      g.seq = (int32_t)F.f[F_SEQ][k];
      g.rseq = (int32_t)F.f[F_RSEQ][k];
      g.props = F.f[F_PROPS][k];
      g.text = F.f[F_TEXT][k];
      g.parent = bi;
      g.rcx = F.f[F_RCX][k];
      g.client = (int16_t)(F.f[F_CLI][k] & 0xFFFF);
      g.rc0 = (int16_t)(F.f[F_CLI][k] >> 16);
    }
  }
  d.cached = true;
}

void download_doc(mtb_dev* b, uint32_t i) {
  if (i >= b->ndocs) raise(MTB_E_ARG, "document index out of range");
  HostDoc& d = b->docs[i];
  if (d.cached) return;
  if (!d.onDevice || !b->devInit || i >= b->hst.size()) raise(MTB_E_ARG, "document has not been replayed");
  const DocState& s = b->hst[i];
  std::vector<FBlk> fb(s.blk_used);
  std::vector<uint32_t> segp(s.seg_used);
  d.text.resize(s.text_used);
  d.aux.resize(s.aux_used);
  if (s.seg_used) HIPCHK(hipMemcpyAsync(segp.data(), b->dSegs.p + s.seg_base, s.seg_used * 4, hipMemcpyDeviceToHost, b->stream));
  if (s.blk_used) HIPCHK(hipMemcpyAsync(fb.data(), b->dBlks.p + s.blk_base, s.blk_used * sizeof(FBlk), hipMemcpyDeviceToHost, b->stream));
  if (s.text_used) HIPCHK(hipMemcpyAsync(d.text.data(), b->dText.p + s.text_base, s.text_used * 2, hipMemcpyDeviceToHost, b->stream));
  if (s.aux_used) HIPCHK(hipMemcpyAsync(d.aux.data(), b->dAux.p + s.aux_base, s.aux_used * 4, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  populate_doc(d, s, fb.data(), segp.data());
}

// download_doc for many documents at once: every listed document's used slices are gathered on the
// device into one staging buffer per element width (one kernel per pool), copied with two transfers,
// and the host views are built on host threads.
void download_docs(mtb_dev* b, const std::vector<uint32_t>& docs) {
  std::vector<uint32_t> todo;
  for (uint32_t i : docs) {
    if (i >= b->ndocs) raise(MTB_E_ARG, "document index out of range");
    if (b->docs[i].cached) continue;
    if (!b->docs[i].onDevice || !b->devInit || i >= b->hst.size()) raise(MTB_E_ARG, "document has not been replayed");
    todo.push_back(i);
  }
  if (todo.empty()) return;
  const uint64_t bw = sizeof(FBlk) / 4;
  Chunks seg, blk, aux, txt;
  std::vector<uint64_t> oSeg(todo.size()), oBlk(todo.size()), oAux(todo.size()), oTxt(todo.size());
  uint64_t nw = 0, nh = 0;
  for (size_t k = 0; k < todo.size(); k++) {
    const DocState& s = b->hst[todo[k]];
    oSeg[k] = nw; seg.add(s.seg_base, nw, s.seg_used); nw += s.seg_used;
    oBlk[k] = nw; blk.add(s.blk_base * bw, nw, (uint64_t)s.blk_used * bw); nw += (uint64_t)s.blk_used * bw;
    oAux[k] = nw; aux.add(s.aux_base, nw, s.aux_used); nw += s.aux_used;
    oTxt[k] = nh; txt.add(s.text_base, nh, s.text_used); nh += s.text_used;
  }
  DevBuf<uint32_t> dw;
  DevBuf<uint16_t> dh;
  dw.ensure(nw + 1);
  dh.ensure(nh + 1);
  move_words(b, b->dSegs.p, dw.p, seg);
  move_words(b, b->dBlks.p, dw.p, blk);
  move_words(b, b->dAux.p, dw.p, aux);
  move_u16(b, b->dText.p, dh.p, txt);
  std::vector<uint32_t> hw(nw + 1);
  std::vector<uint16_t> hh(nh + 1);
  if (nw) HIPCHK(hipMemcpyAsync(hw.data(), dw.p, nw * 4, hipMemcpyDeviceToHost, b->stream));
  if (nh) HIPCHK(hipMemcpyAsync(hh.data(), dh.p, nh * 2, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  dw.release();
  dh.release();
  parallel_docs((uint32_t)todo.size(), [&](uint32_t k) {
    HostDoc& d = b->docs[todo[k]];
    const DocState& s = b->hst[todo[k]];
    d.text.assign(hh.begin() + (long)oTxt[k], hh.begin() + (long)(oTxt[k] + s.text_used));
    d.aux.assign(hw.begin() + (long)oAux[k], hw.begin() + (long)(oAux[k] + s.aux_used));
    populate_doc(d, s, reinterpret_cast<const FBlk*>(hw.data() + oBlk[k]), hw.data() + oSeg[k]);
  });
}

std::string derr_text(int e) {
  switch (e) {
    case DERR_INSERT: return "MergeTree insert failed";
    case DERR_CAP_SEG: return "capacity: segment slice exhausted";
    case DERR_CAP_BLK: return "capacity: block slice exhausted";
    case DERR_CAP_LIST: return "capacity: window-list slice exhausted";
    case DERR_CAP_TEXT: return "capacity: text arena exhausted";
    case DERR_CAP_HEAP: return "capacity: LRU heap exhausted";
    case DERR_CAP_AUX: return "capacity: aux arena exhausted";
    case DERR_CAP_DELTA: return "capacity: catch-up delta / cell-event slice exhausted";
    case DERR_ASSERT_SEQ: return "0x038 Incoming op sequence# < local collabWindow's currentSequence#";
    case DERR_ASSERT_MSN: return "0x04e/0x04f/0x039 minimum sequence number out of order";
    case DERR_DEPTH: return "tree depth limit exceeded";
    case DERR_HOST: return "host post-processing of the replay failed";
    case DERR_REGEN: return "0x033/0x035 regeneratePendingOp: segment group not at the head of the pending queue";
    case DERR_SCHED: return "internal: the document's records did not all run (replay scheduler invariant)";
    case DERR_ASSERT_MKID: return "0x5ad Cannot change the markerId of an existing marker";
    case DERR_RELPOS: return "unsupported: relative position whose marker is not in the document (posFromRelativePos -1) or resolves below 0";
    case DERR_INCR: return "internal: incr annotate over a value missing from its result table (Interner::incr_props)";
    case DERR_CONSENSUS: return "unsupported: consensus annotate over an object value whose seq is -1 (the reference completes "
                                "it in place, shared with split clones)";
    case DERR_CONS_NULL: return "TypeError: Cannot read properties of null (reading 'seq') (properties.ts:56-57: a consensus "
                                "annotate with a null defaultValue over a segment lacking the key; the reference throws here)";
    case DERR_STALE: return "internal: stale cumulative partial lengths in a loaded document without a deficit table "
                            "(partialLengths.ts:543-577; the host gives every load with collaborating body segments one)";
    default: return "device error " + std::to_string(e);
  }
}
int derr_code(int e) {
  if (e == DERR_INSERT) return MTB_E_INSERT;
  if ((e >= DERR_CAP_SEG && e <= DERR_CAP_AUX) || e == DERR_CAP_DELTA || e == DERR_CAP_PEND) return MTB_E_CAPACITY;
  if (e == DERR_ASSERT_SEQ || e == DERR_ASSERT_MSN || e == DERR_ASSERT_MKID || e == DERR_CONS_NULL) return MTB_E_ASSERT;
  if (e == DERR_SCHED || e == DERR_STALE || e == DERR_INCR) return MTB_E_INTERNAL;
  return MTB_E_UNSUPPORTED;
}

// word offset of a document's slice in pool k of the pristine images (blks, segs, lists, aux, text as u32 words)
uint64_t px_base(const DocState& s, int k) {
  switch (k) {
    case 0: return s.blk_base * (sizeof(FBlk) / 4);
    case 1: return s.seg_base;
    case 2: return s.list_base * (sizeof(WEnt) / 4);
    case 3: return s.aux_base;
    default: return s.text_base / 2;
  }
}
// the pristine images' way back into the (current) slices
void px_restore_chunks(mtb_dev* b, const std::vector<uint32_t>* only = nullptr) {
  for (auto& c : b->pxRestore) c = Chunks{};
  auto add = [&](uint32_t i) {
    if (i >= b->pxDoc.size()) return;
    for (int k = 0; k < 5; k++) b->pxRestore[k].add(b->pxDoc[i][k], px_base(b->hPristine[i], k), b->pxDoc[i][5 + k]);
  };
  if (only)
    for (uint32_t i : *only) add(i);
  else
    for (uint32_t i = 0; i < b->ndocs; i++) add(i);
}

// Snapshot the freshly initialised documents (before their first replay) for mtb_rewind.
void capture_pristine(mtb_dev* b) {
  b->hPristine = b->hst;
  b->dPristine.ensure(b->ndocs);
  b->dPSeg.ensure(b->ndocs);
  b->dPBlk.ensure(b->ndocs);
  HIPCHK(hipMemcpyAsync(b->dPristine.p, b->hst.data(), b->ndocs * sizeof(DocState), hipMemcpyHostToDevice, b->stream));
  Chunks bc, sc;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    const DocState& s = b->hst[i];
    bc.add((s.blk_base + s.root) * (sizeof(FBlk) / 4), (uint64_t)i * (sizeof(FBlk) / 4), sizeof(FBlk) / 4);
    sc.add(s.seg_base, (uint64_t)i, 1);
  }
  move_words(b, b->dBlks.p, b->dPBlk.p, bc);
  move_words(b, b->dSegs.p, b->dPSeg.p, sc);
  // documents loaded from a summary: their whole initial tree, window lists and overlap lists
  for (auto& c : b->pxSave) c = Chunks{};
  for (auto& c : b->pxRestore) c = Chunks{};
  b->pxDoc.assign(b->ndocs, std::array<uint64_t, 10>{});
  uint64_t px = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    if (!b->docs[i].loaded && !b->docs[i].perm) continue;
    const DocState& s = b->hst[i];
    const bool ld = b->docs[i].loaded;
    // loaded documents: their whole initial tree; PermutationVectors: their handle table (text words)
    const uint64_t len[5] = {ld ? (uint64_t)s.blk_used * (sizeof(FBlk) / 4) : 0, ld ? s.seg_used : 0,
                             ld ? (uint64_t)s.list_used * (sizeof(WEnt) / 4) : 0, ld ? s.aux_used : 0,
                             b->docs[i].perm ? s.text_used / 2 : 0};
    for (int k = 0; k < 5; k++) {
      b->pxSave[k].add(px_base(s, k), px, len[k]);
      b->pxDoc[i][k] = px;
      b->pxDoc[i][5 + k] = len[k];
      px += len[k];
    }
  }
  px_restore_chunks(b);
  if (px) {
    b->dPX.ensure(px);
    void* pools[5] = {b->dBlks.p, b->dSegs.p, b->dLists.p, b->dAux.p, b->dText.p};
    for (int k = 0; k < 5; k++) move_words(b, pools[k], b->dPX.p, b->pxSave[k]);
  }
  b->haveRewind = true;
}

// MTB_TIMING=1: host-side phase times of each replay call on stderr
struct PhaseClock {
  bool on = getenv("MTB_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string line;
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    char buf[96];
    snprintf(buf, sizeof buf, " %s %.1f", what, std::chrono::duration<double, std::milli>(n - t).count());
    line += buf;
    t = n;
  }
  ~PhaseClock() {
    if (on) fprintf(stderr, "mtb_timing ms:%s\n", line.c_str());
  }
};

void resolve_catch_up(mtb_dev* b, uint32_t i);
void apply_cell_events(mtb_dev* b, uint32_t matrix);

// the batch's replay kernel: matrix pairs, live clients (local ops anywhere in the batch so far), or the
// observer replay engine
// the scheduler's abort flag, copied back with the stream's next synchronization
// (and the hand-over invariant's words: tick_check, mtb_replay.hip)
void sched_readback(mtb_dev* b) {
  std::fill(std::begin(b->schedWords), std::end(b->schedWords), 0u);
  if (b->launch.kernel == MTB_KERNEL_TICKS)
    HIPCHK(hipMemcpyAsync(b->schedWords, b->dSched.p + MTB_SCHED_ABORT, sizeof b->schedWords, hipMemcpyDeviceToHost,
                          b->stream));
}
// after the stream synchronized: the abort flag and hand-over violations into the launch info
void sched_result(mtb_dev* b) {
  if (b->launch.kernel != MTB_KERNEL_TICKS) return;
  const uint32_t* w = b->schedWords - MTB_SCHED_ABORT;
  b->launch.aborted = w[MTB_SCHED_ABORT];
  b->launch.handover_bad = w[MTB_SCHED_BAD];
  if (w[MTB_SCHED_BAD])
    fprintf(stderr,
            "mtb: %u ticket hand-over(s) found a stale document state (first: document %u chunk %u, op_next %u expected "
            "%u); those documents were finished by mtb_replay_finish_kernel\n",
            w[MTB_SCHED_BAD], w[MTB_SCHED_BAD + 1], w[MTB_SCHED_BAD + 2], w[MTB_SCHED_BAD + 4], w[MTB_SCHED_BAD + 3]);
}

// Which kernel replays each document (DocState.flags DSF_VARIANT): the marker variant for a document that met a
// marker id, loaded phantom partial lengths or uses a property key whose matchProperties is no equivalence
// (irregular in the batch), the observer kernels for every other -- so one such document no longer moves the whole
// batch onto the marker variant (the observer kernels skip flagged documents, the marker kernel the others).
// Live batches replay every document on the live kernel (no flags).
// the marker kernel over the flagged documents (the others return at once), before the observer kernels' launch
void launch_variant_docs(mtb_dev* b, const Tables& t) {
  HIPCHK(mtb_launch_replay(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                           b->dHeap.p, b->dAux.p, b->dFree.p, t, 2));
}
void mark_variant_docs(mtb_dev* b) {
  uint32_t nv = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    DocState& s = b->hst[i];
    bool v = false;
    if (!b->live && !b->matrix) {
      v = !d.markerAmbig.empty() || d.markerIdAnnot || d.phantom;
      if (!v && b->in.nIrrKeys()) {
        b->in.note(d.vals);
        for (const auto& kv : d.vals.keyVals)
          if (b->in.keyIrr[kv.first]) { v = true; break; }
      }
    }
    s.flags = v ? (s.flags | DSF_VARIANT) : (s.flags & ~DSF_VARIANT);
    nv += v;
  }
  b->variantDocs = nv;
}

void launch_main(mtb_dev* b, const Tables& t) {
  if (getenv("MTB_DEBUG_POOLS")) {  // (fault triage: the pools' address ranges, to place a faulting address)
    const struct { const char* name; const void* p; size_t bytes; } pools[] = {
        {"docs", b->dDocs.p, b->dDocs.n * sizeof(DocState)}, {"ops", b->dOps.p, b->dOps.n * sizeof(mtb_op)},
        {"segs", b->dSegs.p, b->dSegs.n * 4}, {"blks", b->dBlks.p, b->dBlks.n * sizeof(FBlk)},
        {"lists", b->dLists.p, b->dLists.n * sizeof(WEnt)}, {"text", b->dText.p, b->dText.n * 2},
        {"heap", b->dHeap.p, b->dHeap.n * sizeof(Lru)}, {"aux", b->dAux.p, b->dAux.n * 4},
        {"free", b->dFree.p, b->dFree.n * 4}, {"pool", t.pool, b->dPool.n * 4}, {"sched", b->dSched.p, b->dSched.n * 4}};
    for (const auto& q : pools)
      fprintf(stderr, "mtb_pool %-6s %p .. %p (%zu bytes)\n", q.name, q.p, (const void*)((const char*)q.p + q.bytes), q.bytes);
  }
  if (b->matrix) {
    HIPCHK(mtb_launch_matrix(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                             b->dHeap.p, b->dAux.p, b->dFree.p, t));
    b->launch = mtb_launch_info{};
    b->launch.kernel = MTB_KERNEL_MATRIX;
  } else
  {
    // the live-client kernel carries the marker code too; otherwise the marker variant runs only for
    // batches where some document met a marker id
    // (the marker variant carries the phantom tables and the irregular-key matchProperties too)
    // (mark_variant_docs: every document on the marker variant, some, or none)
    const bool markers = b->variantDocs != 0 && b->variantDocs == b->ndocs;
    const bool someMarkers = b->variantDocs != 0 && !markers;
    if (someMarkers) launch_variant_docs(b, t);
    // more documents than wave slots: tickets, one per workgroup (mtb_replay_tick_kernel, the default;
    // MTB_CHUNKS / MTB_CHUNK_PLAN set the tickets per document) or passes of equal chunks (MTB_SCHED=passes);
    // MTB_SCHED=0 launches one wave per whole document
    if (!b->live && !markers && !b->waveSlots) {
      hipDeviceProp_t prop;
      HIPCHK(hipGetDeviceProperties(&prop, b->device));
      b->waveSlots = (uint32_t)prop.multiProcessorCount * (uint32_t)mtb_sched_waves_per_cu();  // (16: 4 per SIMD)
      int nx = 1;
      if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, b->device) != hipSuccess) nx = 1;
      b->nXcc = (uint32_t)std::max(1, std::min(8, nx));
    }
    b->launch = mtb_launch_info{};
    b->launch.wave_slots = b->waveSlots;
    const char* sv = getenv("MTB_SCHED");
    const bool many = !b->live && !markers && b->ndocs > b->waveSlots && !(sv && sv[0] == '0');
    if (many && sv && !strcmp(sv, "passes")) {
      // Passes: the ndocs * m tasks (chunk c of document x, chunk-major) cut into launches of whole rounds
      // of the resident slots, at most ndocs tasks each (a document's chunks land in successive launches).
      // m (chunks per document, MTB_PASS_CHUNKS) leaves the smallest fraction of a round idle at the end.
      const uint64_t S = b->waveSlots, D = b->ndocs;
      uint32_t m = 0;
      if (const char* cv = getenv("MTB_PASS_CHUNKS")) m = (uint32_t)std::max(1, std::min(64, atoi(cv)));
      if (!m) {
        double best = 1e30;
        for (uint32_t k = 4; k <= 10; k++) {
          const double rounds = (double)(k * D) / (double)S;
          const double cost = std::ceil(rounds) / rounds + 0.004 * k;  // idle share of the last round + per-chunk setup
          if (cost < best) {
            best = cost;
            m = k;
          }
        }
      }
      while (m > 1 && (uint64_t)m * D > 0x7FFFFFFFull) m--;
      const uint64_t T = (uint64_t)m * D;
      const uint64_t P = std::max<uint64_t>(1, D / S) * S;  // tasks per launch: whole rounds, <= ndocs
      uint32_t passes = 0;
      for (uint64_t first = 0; first < T; first += P, passes++)
        HIPCHK(mtb_launch_replay_passes(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p,
                                        b->dText.p, b->dHeap.p, b->dAux.p, b->dFree.p, t, (uint32_t)first,
                                        (uint32_t)std::min<uint64_t>(P, T - first), m));
      b->launch.kernel = MTB_KERNEL_PASSES;
      b->launch.chunks = m;
      b->launch.passes = passes;
      return;
    }
    if (many) {
      // the chunk plan: cumulative fractions (1/4096) of every document's records per ticket; MTB_CHUNKS=n
      // makes n equal chunks, MTB_CHUNK_PLAN="a,b,..." (relative chunk sizes) any other split.  Chunk c's
      // ticket comes ndocs tickets after chunk c-1's, so a chunk at most ~2x the next keeps waits rare.
      std::vector<double> sizes;
      if (const char* pv = getenv("MTB_CHUNK_PLAN")) {
        for (const char* q = pv; *q;) {
          char* end = nullptr;
          const double v = strtod(q, &end);
          if (end == q) break;
          if (v > 0) sizes.push_back(v);
          q = *end ? end + 1 : end;
        }
      }
      if (sizes.empty()) {
        if (const char* cv = getenv("MTB_CHUNKS"))
          sizes.assign((size_t)std::max(1, std::min(64, atoi(cv))), 1.0);
        else  // default: 12/16, 3/16 and 1/16 of every document: three tickets, a fine tail (round-4 sweep)
          sizes = {12, 3, 1};
      }
      if (sizes.size() > 64) sizes.resize(64);
      while (sizes.size() > 1 && (uint64_t)sizes.size() * b->ndocs > 0x7FFFFFFFull) sizes.pop_back();  // tickets fit 31 bits
      const uint32_t nchunks = (uint32_t)sizes.size();
      double tot = 0, run = 0;
      for (double v : sizes) tot += v;
      std::vector<uint32_t> plan(nchunks);
      for (uint32_t c = 0; c < nchunks; c++) {
        run += sizes[c];
        plan[c] = c + 1 == nchunks ? 4096u : std::max<uint32_t>(1, std::min<uint32_t>(4096, (uint32_t)(4096.0 * run / tot)));
      }
      // queues: one per XCD (L2 affinity); MTB_SCHED_QUEUES overrides (1 = one global queue)
      uint32_t nq = b->nXcc ? b->nXcc : 1;
      if (const char* qv = getenv("MTB_SCHED_QUEUES")) nq = (uint32_t)std::max(1, std::min(8, atoi(qv)));
      // a wait bound far above any chunk (about a minute); MTB_SCHED_SPINS lowers it (tests force the abort)
      uint32_t spins = 1u << 27;
      if (const char* sp = getenv("MTB_SCHED_SPINS")) spins = (uint32_t)std::max(0L, std::min(1L << 30, atol(sp)));
      const size_t nw = MTB_SCHED_HDR + 2 * (size_t)b->ndocs + nchunks;  // progress, plan, hand-over op_next
      b->dSched.ensure(nw);
      HIPCHK(hipMemsetAsync(b->dSched.p, 0, (MTB_SCHED_HDR + (size_t)b->ndocs) * sizeof(uint32_t), b->stream));
      b->schedPlan = plan;  // (kept alive until the stream has consumed the copies)
      b->schedSpins = spins;
      HIPCHK(hipMemcpyAsync(b->dSched.p + MTB_SCHED_HDR + b->ndocs, b->schedPlan.data(), nchunks * sizeof(uint32_t),
                            hipMemcpyHostToDevice, b->stream));
      HIPCHK(hipMemcpyAsync(b->dSched.p + MTB_SCHED_SPINS, &b->schedSpins, sizeof(uint32_t), hipMemcpyHostToDevice,
                            b->stream));
      HIPCHK(mtb_launch_replay_ticks(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p,
                                     b->dText.p, b->dHeap.p, b->dAux.p, b->dFree.p, t, b->dSched.p, nchunks, nq));
      b->launch.kernel = MTB_KERNEL_TICKS;
      b->launch.chunks = nchunks;
      b->launch.queues = nq;
      return;
    }
    HIPCHK(mtb_launch_replay(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                             b->dHeap.p, b->dAux.p, b->dFree.p, t, b->live ? 1 : markers ? 2 : 0));
    b->launch.kernel = b->live ? MTB_KERNEL_LIVE : markers ? MTB_KERNEL_MARKERS
                       : b->ndocs <= 1024 ? MTB_KERNEL_FEW : MTB_KERNEL_REPLAY;
  }
}

// Capacity retry.  A document whose first replay overflowed one of its slices (DERR_CAP_*, never a result the
// reference produces) is laid out again with that slice four times larger and replayed from its pristine state, up
// to MTB_CAP_RETRIES (default 12) times; the other documents keep their state (layout() moves it) and have nothing left
// to run.  Only documents whose pristine snapshot is their state before this replay qualify (`fresh`); any other
// overflow stays a sticky MTB_E_CAPACITY.  Returns the number of relaunches.
int capacity_retry(mtb_dev* b, bool anyLoad, const std::vector<uint8_t>& fresh) {
  const char* rv = getenv("MTB_CAP_RETRIES");
  const int maxTries = rv ? std::max(0, atoi(rv)) : 12;
  int tries = 0;
  for (; tries < maxTries; tries++) {
    std::vector<uint32_t> redo;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      const int e = b->hst[i].err;
      if (fresh[i] && e >= DERR_CAP_SEG && e <= DERR_CAP_AUX) redo.push_back(i);
    }
    if (redo.empty()) break;
    if (getenv("MTB_TIMING"))
      fprintf(stderr, "mtb_capacity_retry %d: %zu document(s), first %u (error %d, caps seg %u blk %u list %u text %u heap %u aux %u)\n",
              tries, redo.size(), redo[0], b->hst[redo[0]].err, b->hst[redo[0]].seg_cap, b->hst[redo[0]].blk_cap,
              b->hst[redo[0]].list_cap, b->hst[redo[0]].text_cap, b->hst[redo[0]].heap_cap, b->hst[redo[0]].aux_cap);
    std::vector<Caps> want(b->ndocs, Caps{0, 0, 0, 0, 0, 0});
    for (uint32_t i : redo) {
      DocState& s = b->hst[i];
      Caps c{s.seg_cap, s.blk_cap, s.list_cap, s.text_cap, s.heap_cap, s.aux_cap};
      auto dbl = [](uint32_t& v) { v = (uint32_t)std::min<uint64_t>(4ull * v + 16, 0xFFFFFFF0u); };
      switch (s.err) {
        case DERR_CAP_SEG: dbl(c.seg); break;
        case DERR_CAP_BLK: dbl(c.blk); dbl(c.heap); break;
        case DERR_CAP_LIST: dbl(c.list); break;
        case DERR_CAP_TEXT: dbl(c.text); break;
        case DERR_CAP_HEAP: dbl(c.heap); break;
        default: dbl(c.aux); break;
      }
      want[i] = c;
      // layout() moves only the pristine prefix of a document that starts over
      const DocState& p = b->hPristine[i];
      s.seg_used = p.seg_used, s.blk_used = p.blk_used, s.list_used = p.list_used, s.text_used = p.text_used;
      s.heap_cnt = p.heap_cnt, s.aux_used = p.aux_used, s.free_top = p.free_top;
    }
    layout(b, want);
    // the pristine snapshot follows the new slices (rewind restores into them)
    for (uint32_t i = 0; i < b->ndocs; i++) {
      DocState& p = b->hPristine[i];
      const DocState& s = b->hst[i];
      p.seg_base = s.seg_base, p.blk_base = s.blk_base, p.list_base = s.list_base, p.text_base = s.text_base;
      p.heap_base = s.heap_base, p.aux_base = s.aux_base, p.free_base = s.free_base;
      p.seg_cap = s.seg_cap, p.blk_cap = s.blk_cap, p.list_cap = s.list_cap, p.text_cap = s.text_cap;
      p.heap_cap = s.heap_cap, p.aux_cap = s.aux_cap;
    }
    HIPCHK(hipMemcpyAsync(b->dPristine.p, b->hPristine.data(), b->ndocs * sizeof(DocState), hipMemcpyHostToDevice, b->stream));
    px_restore_chunks(b);
    b->haveRewind = true;
    // the documents that start over: pristine header, root block, initial segment and (loaded) initial tree
    Chunks bc, sc;
    for (uint32_t i : redo) {
      const DocState& p = b->hPristine[i];
      b->hst[i] = p;
      b->docs[i].cached = false;
      bc.add((uint64_t)i * (sizeof(FBlk) / 4), (p.blk_base + p.root) * (sizeof(FBlk) / 4), sizeof(FBlk) / 4);
      sc.add(i, p.seg_base, 1);
    }
    HIPCHK(hipMemcpyAsync(b->dDocs.p, b->hst.data(), b->ndocs * sizeof(DocState), hipMemcpyHostToDevice, b->stream));
    move_words(b, b->dPBlk.p, b->dBlks.p, bc);
    move_words(b, b->dPSeg.p, b->dSegs.p, sc);
    Chunks all[5];
    for (int k = 0; k < 5; k++) all[k] = b->pxRestore[k];
    px_restore_chunks(b, &redo);
    void* pools[5] = {b->dBlks.p, b->dSegs.p, b->dLists.p, b->dAux.p, b->dText.p};
    for (int k = 0; k < 5; k++) move_words(b, b->dPX.p, pools[k], b->pxRestore[k]);
    for (int k = 0; k < 5; k++) b->pxRestore[k] = all[k];
    const Tables t = make_tables(b);
    if (anyLoad)
      HIPCHK(mtb_launch_load(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                             b->dHeap.p, b->dAux.p, b->dFree.p, t, b->matrix ? 1 : 0));
    launch_main(b, t);
    sched_readback(b);
    HIPCHK(hipMemcpyAsync(b->hst.data(), b->dDocs.p, b->ndocs * sizeof(DocState), hipMemcpyDeviceToHost, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    sched_result(b);
    for (uint32_t i = 0; i < b->ndocs; i++)
      if (!b->hst[i].err && b->hst[i].op_next != b->hst[i].n_ops) b->hst[i].err = DERR_SCHED;
  }
  return tries;
}

void replay(mtb_dev* b, mtb_stats* out) {
  PhaseClock pc;
  // documents that failed in an earlier replay stay failed (sticky) and are counted in the stats, but
  // only a failure of this replay is reported as the call's error (the reference throws once, from
  // the applyMsg that failed)
  std::vector<uint8_t> failedBefore(b->ndocs);
  for (uint32_t i = 0; i < b->ndocs && i < b->hst.size(); i++) failedBefore[i] = b->hst[i].err != 0;
  // the matrix kernel's two waves meet at one barrier per SETCELL record: both vectors of a matrix must
  // carry the same number of them (checked before anything runs)
  if (b->matrix)
    for (uint32_t i = 0; i + 1 < b->ndocs; i += 2) {
      size_t n[2] = {0, 0};
      for (int v = 0; v < 2; v++)
        for (const mtb_op& o : b->docs[i + v].pending) n[v] += o.type == MTB_OP_SETCELL;
      if (n[0] != n[1])
        raise(MTB_E_ARG, "matrix " + std::to_string(i / 2) + ": rows and cols vectors hold different numbers of SETCELL records");
    }
  if (!b->devInit) device_init(b);
  pc.mark("device_init");
  upload_tables(b);
  pc.mark("tables");
  // grow the slices of documents whose appended records no longer fit (2x headroom)
  {
    std::vector<Caps> want(b->ndocs);
    bool grow = false;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      HostDoc& d = b->docs[i];
      const DocState& s = b->hst[i];
      // (the same requirement device_init laid the slices out for: caps_for's text term already counts the
      // initial text, so adding text_used here made every fresh batch re-lay out at twice the caps)
      Caps need = doc_caps(d, d.totalOps, std::max<uint64_t>(d.totalPayload, d.payload.size()), b->tightCaps);
      // ... and what the slices already hold plus the per-record margin for the pending records: a document can
      // outgrow the record-count formula (a live client holding thousands of unacked inserts keeps an entry per
      // insert in every ancestor's window list, and list rebuilds allocate before they free)
      if (s.seg_cap && d.totalOps != d.pending.size()) {  // (a fresh document's slices are the formula's)
        // (caps_for's per-record terms without its constants, which the formula above already carries)
        const uint64_t np = d.pending.size();
        auto at_least = [](uint32_t& c, uint64_t v) { c = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(c, v), 0xFFFFFFF0u); };
        at_least(need.seg, (uint64_t)s.seg_used + 2 * np);
        at_least(need.blk, (uint64_t)s.blk_used + np / 2);
        at_least(need.list, (uint64_t)s.list_used + s.list_used / 2 + 8 * np);
        at_least(need.heap, (uint64_t)s.heap_cnt + np);
        at_least(need.aux, (uint64_t)s.aux_used + s.aux_used / 4 + 16 * np);
      }
      if (!fits(s, need) || s.text_used + d.payload.size() > s.text_cap ||
          (d.perm && 2 * (d.totalSetcell + d.initText.size() / 2 + 4) > s.text_cap)) {
        want[i] = doc_caps(d, 2 * d.totalOps, 2 * (d.totalPayload + s.text_used), b->tightCaps);
        auto twice = [](uint32_t& c, uint32_t v) { c = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(c, 2ull * v), 0xFFFFFFF0u); };
        twice(want[i].seg, need.seg);
        twice(want[i].blk, need.blk);
        twice(want[i].list, need.list);
        twice(want[i].heap, need.heap);
        twice(want[i].aux, need.aux);
        grow = true;
      } else {
        want[i] = Caps{0, 0, 0, 0, 0, 0};
      }
    }
    if (grow) layout(b, want);
  }
  // a matrix whose vector failed is failed as a whole (its waves must agree on every setCell barrier)
  if (b->matrix)
    for (uint32_t i = 0; i + 1 < b->ndocs; i += 2) {
      const int e = b->hst[i].err ? b->hst[i].err : b->hst[i + 1].err;
      if (e) b->hst[i].err = b->hst[i + 1].err = e;
    }
  // gather pending ops of every document into one buffer
  // per-document offsets first, then every document's records and payload copied in parallel
  bool anyLoad = false;
  Chunks payc;
  std::vector<uint64_t> opOff(b->ndocs, 0), payOff(b->ndocs, 0);
  uint64_t nOps = 0, nPay = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    DocState& s = b->hst[i];
    if (s.err) {  // sticky: nothing more runs for this document
      s.n_ops = 0;
      s.op_next = 0;
      continue;
    }
    opOff[i] = nOps;
    payOff[i] = nPay;
    // payload goes after the text already in the arena
    payc.add(nPay, s.text_base + s.text_used, d.payload.size());
    nOps += d.pending.size();
    nPay += d.payload.size();
    if (!d.pending.empty() && d.pending[0].type == MTB_OP_LOADSEG) anyLoad = true;
  }
  std::unique_ptr<mtb_op[]> ops(new mtb_op[nOps + 1]);
  std::unique_ptr<uint16_t[]> pay(new uint16_t[nPay + 1]);
  parallel_docs(b->ndocs, [&](uint32_t i) {
    HostDoc& d = b->docs[i];
    DocState& s = b->hst[i];
    if (s.err) return;
    const uint32_t base = s.text_used;  // rebase record payload offsets into the arena
    std::copy(d.payload.begin(), d.payload.end(), pay.get() + payOff[i]);
    s.text_used += (uint32_t)d.payload.size();
    if (!(s.flags & DSF_NEWLINE)) {
      bool nl = std::find(d.payload.begin(), d.payload.end(), (uint16_t)'\n') != d.payload.end();
      if (!nl) nl = std::find(d.initText.begin(), d.initText.end(), (uint16_t)'\n') != d.initText.end();
      if (nl) s.flags |= DSF_NEWLINE;
    }
    s.op_base = opOff[i];
    s.n_ops = (uint32_t)d.pending.size();
    s.op_next = 0;
    mtb_op* out = ops.get() + opOff[i];
    s.mk_cap = (uint32_t)d.markerAmbig.size();
    if (d.markerDup) s.flags |= DSF_MKDUP;
    s.flags = (s.flags & 0xFFFFu) | ((uint32_t)d.obsRef << DSF_OBS_SHIFT);
    for (mtb_op o : d.pending) {
      // text offsets move with the arena; a PermutationSegment's LOADSEG payload is its handle start
      if ((o.type == MTB_OP_INSERT || o.type == MTB_OP_LOADSEG) && !(o.flags & MTB_F_MARKER) && !d.perm) o.payload += base;
      if ((o.flags & MTB_F_RELPOS) && o.type != MTB_OP_LOADSEG) {  // relative-position descriptors
        if (o.pos1 & MTB_RELPOS) o.pos1 += base;
        if (o.pos2 & MTB_RELPOS) o.pos2 += base;
      }
      *out++ = o;
    }
  });
  mark_variant_docs(b);
  // catch-up delta slices: a record's delta has at most one entry per unit of its range
  {
    uint64_t tot = 0;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      DocState& s = b->hst[i];
      s.delta_base = tot;
      s.delta_used = 0;
      uint64_t cap = 0;
      if (!s.err && b->matrix) {
        // cell events: one per setCell, one per segment unlinked with handles (live segments plus at most
        // three created per record)
        cap = s.seg_cap + 4ull * b->docs[i].pending.size() + 1;
      } else if (!s.err) {
        // a marker-relative range is resolved on the device: bound it by the document's length, itself bounded
        // by the text and segments it holds plus what the records before it insert
        // (a marker's pos2 is its refType, 0xFFFFFFFF when undefined: it adds 1).  A delta holds one entry per
        // segment the record touches, so a range is also bounded by the segments the document can hold by then:
        // those it holds plus two per record before it (the record's own boundary splits).
        uint64_t lenBound = (uint64_t)s.text_used + s.seg_used + 1, segBound = (uint64_t)s.seg_used + 1;
        for (const mtb_op& o : b->docs[i].pending) {
          if (o.type == MTB_OP_INSERT) lenBound += (o.flags & MTB_F_MARKER) ? 1 : o.pos2;
          segBound += 2;
          const uint64_t range =
              std::min((o.flags & MTB_F_RELPOS) ? lenBound : (o.pos2 > o.pos1 ? o.pos2 - o.pos1 : 0), segBound);
          if (o.flags & MTB_F_DELTA)  // (a rewrite annotate's segments get a second entry: the set before)
            cap += o.type == MTB_OP_INSERT ? 1
                   : (range + 1) * (o.type == MTB_OP_ANNOTATE && (o.flags & MTB_F_COMB) == MTB_F_REWRITE ? 2 : 1);
          if (o.type == MTB_OP_REGEN) cap += (uint64_t)o.pos1 * (s.seg_used + 16);  // one entry per regenerated op
        }
      }
      if (cap > 0xFFFFFFF0ull) {  // the device's cap is 32-bit: such a batch of lagging ops fails its document
        s.err = DERR_CAP_DELTA;
        s.err_op = 0;
        s.n_ops = 0;
        cap = 0;
      }
      s.delta_cap = (uint32_t)cap;
      tot += cap;
    }
    b->dDelta.ensure(4 * tot + 4);
  }
  pc.mark("gather");
  scatter_u16(b, pay.get(), nPay, b->dText.p, payc);
  b->dOps.ensure(nOps + 1);
  if (nOps) HIPCHK(hipMemcpyAsync(b->dOps.p, ops.get(), nOps * sizeof(mtb_op), hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipMemcpyAsync(b->dDocs.p, b->hst.data(), b->ndocs * sizeof(DocState), hipMemcpyHostToDevice, b->stream));
  pc.mark("upload");
  // documents whose pristine snapshot (taken now) is their state before this replay: the capacity retry's
  std::vector<uint8_t> fresh(b->ndocs, 0);
  if (!b->haveRewind) {
    capture_pristine(b);
    if (!b->matrix)
      for (uint32_t i = 0; i < b->ndocs; i++)
        fresh[i] = !failedBefore[i] && b->docs[i].totalOps == b->docs[i].pending.size() && b->hst[i].op_next == 0;
  }
  pc.mark("pristine");
  const Tables t = make_tables(b);
  b->residentLoad = anyLoad;
  HIPCHK(hipEventRecord(b->ev0, b->stream));
  if (anyLoad)  // summary bodies first (LOADSEG records head their documents' records)
    HIPCHK(mtb_launch_load(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                           b->dHeap.p, b->dAux.p, b->dFree.p, t, b->matrix ? 1 : 0));
  launch_main(b, t);
  HIPCHK(hipEventRecord(b->ev1, b->stream));
  sched_readback(b);
  HIPCHK(hipMemcpyAsync(b->hst.data(), b->dDocs.p, b->ndocs * sizeof(DocState), hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->lastKernelMs = ms;
  sched_result(b);
  pc.mark("kernels");
  if (b->matrix)
    for (uint32_t i = 0; i + 1 < b->ndocs; i += 2) {
      const int e = b->hst[i].err ? b->hst[i].err : b->hst[i + 1].err;
      if (e) b->hst[i].err = b->hst[i + 1].err = e;
    }
  // every document without an error ran all of its records (after a scheduler abort the finish kernel ran
  // the rest): an engine invariant, checked
  for (uint32_t i = 0; i < b->ndocs; i++)
    if (!b->hst[i].err && b->hst[i].op_next != b->hst[i].n_ops) b->hst[i].err = DERR_SCHED;
  if (getenv("MTB_TIMING")) {
    uint32_t nf = 0, ne = 0;
    for (uint32_t i = 0; i < b->ndocs; i++) nf += fresh[i], ne += b->hst[i].err != 0;
    fprintf(stderr, "mtb_capacity: %u fresh documents, %u with errors, tight caps %d\n", nf, ne, (int)b->tightCaps);
  }
  const uint32_t retries = (uint32_t)capacity_retry(b, anyLoad, fresh);
  b->launch.cap_retries = retries;
  pc.mark("capacity retry");
  // the records are consumed now: whatever the host post-processing below does, they never run again
  for (uint32_t i = 0; i < b->ndocs; i++) {
    HostDoc& d = b->docs[i];
    d.applied.clear();
    d.appliedPayload.clear();
    d.applied.swap(d.pending);
    d.appliedPayload.swap(d.payload);
    d.cached = false;
  }
  // host post-processing (cell events, catch-up rewriting): a failure is sticky for its document
  auto post = [&](uint32_t i, auto&& f) {
    try {
      f();
    } catch (const MtbError& e) {
      b->hst[i].err = DERR_HOST;
      b->docs[i].hostErr = e.msg;
    } catch (const std::exception& e) {
      b->hst[i].err = DERR_HOST;
      b->docs[i].hostErr = e.what();
    }
  };
  if (b->matrix)
    for (uint32_t i = 0; i + 1 < b->ndocs; i += 2)
      if (!b->hst[i].err) {
        post(i, [&] { apply_cell_events(b, i / 2); });
        if (b->hst[i].err) {
          b->hst[i + 1].err = b->hst[i].err;
          b->docs[i + 1].hostErr = b->docs[i].hostErr;
        }
      }
  for (uint32_t i = 0; i < b->ndocs; i++) {
    if (b->hst[i].err) continue;
    bool open = false;
    for (auto& m : b->docs[i].catchup) open |= !m.resolved;
    if (open) post(i, [&] { resolve_catch_up(b, i); });
  }
  mtb_stats st{};
  st.kernel_ms = ms;
  int firstErr = 0;
  uint32_t errDoc = 0;
  for (uint32_t i = 0; i < b->ndocs; i++) {
    DocState& s = b->hst[i];
    st.docs++;
    st.ops_applied += s.ops_applied;
    st.bytes_alg += 32ull * s.ops_applied + s.text_bytes + 24ull * s.n_mod;
    if (s.err) {
      st.errors++;
      if (!firstErr && !failedBefore[i]) { firstErr = s.err; errDoc = i; }
    }
  }
  run_digest(b, st);
  if (getenv("MTB_USAGE_OUT")) {  // slice use against capacity per pool (max, 99th percentile, mean), for sizing caps
    struct P { const char* name; uint32_t DocState::*used; uint32_t DocState::*cap; size_t bytes; };
    const P pools[] = {{"segs", &DocState::seg_used, &DocState::seg_cap, 4}, {"blks", &DocState::blk_used, &DocState::blk_cap, sizeof(FBlk)},
                       {"lists", &DocState::list_used, &DocState::list_cap, sizeof(WEnt)}, {"text", &DocState::text_used, &DocState::text_cap, 2},
                       {"heap", &DocState::heap_cnt, &DocState::heap_cap, sizeof(Lru)}, {"aux", &DocState::aux_used, &DocState::aux_cap, 4}};
    for (const P& q : pools) {
      std::vector<double> u, f;
      double capb = 0;
      for (uint32_t i = 0; i < b->ndocs; i++) {
        const DocState& s = b->hst[i];
        const double ops = std::max<double>(1, (double)b->docs[i].totalOps);
        u.push_back((double)(s.*q.used) / ops);
        f.push_back((double)(s.*q.used) / std::max<double>(1, (double)(s.*q.cap)));
        capb += (double)(s.*q.cap) * (double)q.bytes;
      }
      std::sort(u.begin(), u.end());
      std::sort(f.begin(), f.end());
      const size_t n = u.size();
      if (!n) continue;
      fprintf(stderr, "mtb_usage %-5s per record: max %.3f p99 %.3f mean %.3f | of cap: max %.3f p99 %.3f | cap %.1f MiB/doc\n",
              q.name, u[n - 1], u[n * 99 / 100], std::accumulate(u.begin(), u.end(), 0.0) / n, f[n - 1], f[n * 99 / 100],
              capb / n / 1048576.0);
    }
  }
  if (getenv("MTB_PROFILE_OUT")) {  // MTB_PROFILE builds: per-phase device cycles and events per op, summed over documents
    double p[11] = {0}, c[9] = {0};
    for (uint32_t i = 0; i < b->ndocs; i++) {
      for (int k = 0; k < 7; k++) p[k] += (double)b->hst[i].prof[k];
      for (int k = 0; k < 4; k++) p[7 + k] += (double)b->hst[i].prof2[k];
      for (int k = 0; k < 5; k++) c[k] += b->hst[i].cnt[k];
      for (int k = 0; k < 4; k++) c[5 + k] += b->hst[i].cnt2[k];
    }
    const double n = (double)std::max<uint64_t>(1, st.ops_applied);
    fprintf(stderr, "mtb_profile cycles/op: boundary %.0f insert %.0f nodemap %.0f zamboni %.0f total %.0f | view %.0f scour %.0f (ops %llu)\n",
            p[0] / n, p[1] / n, p[2] / n, p[3] / n, p[4] / n, p[5] / n, p[6] / n, (unsigned long long)st.ops_applied);
    fprintf(stderr, "mtb_profile zamboni cycles/op: heap %.0f stage %.0f place %.0f pack %.0f\n", p[7] / n, p[8] / n, p[9] / n, p[10] / n);
    fprintf(stderr, "mtb_profile events/op: scour %.3f pack %.3f rebuild %.3f view %.3f entries %.2f zcalls %.3f pops %.3f popskips %.3f psig %.3f\n",
            c[0] / n, c[1] / n, c[2] / n, c[3] / n, c[4] / n, c[5] / n, c[6] / n, c[7] / n, c[8] / n);
    uint64_t mx[7] = {0, 0, 0, 0, 0, 0, 0}, mxo = 0;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      const DocState& q = b->hst[i];
      const uint64_t v[7] = {q.seg_used, q.blk_used, q.list_used, q.text_used, q.heap_cnt, q.aux_used, q.n_ops};
      for (int k = 0; k < 7; k++) mx[k] = std::max(mx[k], v[k]);
      mxo = std::max<uint64_t>(mxo, q.ops_applied);
    }
    fprintf(stderr, "mtb_profile max usage: seg %llu blk %llu list %llu text %llu heap %llu aux %llu (records %llu, ops %llu)\n",
            (unsigned long long)mx[0], (unsigned long long)mx[1], (unsigned long long)mx[2], (unsigned long long)mx[3],
            (unsigned long long)mx[4], (unsigned long long)mx[5], (unsigned long long)mx[6], (unsigned long long)mxo);
  }
  if (getenv("MTB_SLICE_TRACE")) {  // per-document slice use after each replay (capacity debugging)
    for (uint32_t i = 0; i < b->ndocs && i < 4; i++) {
      const DocState& s = b->hst[i];
      fprintf(stderr, "mtb_slices doc %u ops %llu: seg %u/%u blk %u/%u list %u/%u text %u/%u heap %u/%u aux %u/%u\n", i,
              (unsigned long long)b->docs[i].totalOps, s.seg_used, s.seg_cap, s.blk_used, s.blk_cap, s.list_used,
              s.list_cap, s.text_used, s.text_cap, s.heap_cnt, s.heap_cap, s.aux_used, s.aux_cap);
    }
  }
  if (getenv("MTB_CHECK_OUT")) {  // MTB_CHECK builds: slice-bound violations per document (DocState.pad3)
    static const char* pools[4] = {"segp", "blk", "lst", "aux"};
    uint32_t nbad = 0;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      const uint32_t* r = b->hst[i].pad3;
      if (!r[0]) continue;
      if (nbad++ < 16)
        fprintf(stderr, "mtb_check doc %u: %u out-of-slice accesses, first %s[%u] (capacity %u), op_next %u\n", i, r[0],
                pools[r[3] & 3], r[1], r[2], b->hst[i].op_next);
    }
    fprintf(stderr, "mtb_check: %u of %u documents with out-of-slice accesses\n", nbad, b->ndocs);
  }
  if (out) *out = st;
  if (firstErr == DERR_HOST) raise(MTB_E_ARG, "document " + std::to_string(errDoc) + ": " + b->docs[errDoc].hostErr);
  if (firstErr)
    raise(derr_code(firstErr), "document " + std::to_string(errDoc) + " op " + std::to_string(b->hst[errDoc].err_op) + ": " +
                                   derr_text(firstErr));
}

// ------------------------------------------------------------------ read-out helpers
struct FlatSeg {
  uint32_t id;
  std::vector<int> path;
};
void flatten(const HostDoc& d, uint32_t root, std::vector<FlatSeg>& out, bool withPath) {
  std::vector<int> path;
  struct Fr { uint32_t b; int i; };
  if (root >= d.blks.size()) raise(MTB_E_INTERNAL, "corrupt tree: root block outside the slice");
  std::vector<Fr> st{{root, 0}};
  size_t entered = 1;
  while (!st.empty()) {
    Fr& f = st.back();
    const Blk& B = d.blks[f.b];
    if (f.i >= B.count) {
      st.pop_back();
      if (!path.empty()) path.pop_back();
      continue;
    }
    const int i = f.i++;
    const uint32_t c = B.child[i];
    if (c & MTB_LEAF) {
      FlatSeg fs;
      fs.id = c & ~MTB_LEAF;
      if (withPath) {
        fs.path = path;
        fs.path.push_back(i);
      }
      out.push_back(std::move(fs));
    } else {
      // a child outside the slice or a cycle (more blocks entered than exist) is an engine fault, not input
      if (c >= d.blks.size() || ++entered > d.blks.size()) raise(MTB_E_INTERNAL, "corrupt tree: bad block child");
      path.push_back(i);
      st.push_back({c, 0});
    }
  }
}

bool seg_removed(const Seg& s) { return s.rseq >= 0; }
// a live client's unacked insert / remove (F_SEQ / F_RSEQ = MTB_PEND + localSeq): UnassignedSequenceNumber
bool seg_pending(int32_t seq) { return seq >= MTB_PEND; }
int32_t seq_out(int32_t seq) { return seg_pending(seq) ? -1 : seq; }
bool is_marker(const Seg& s) { return (s.text & MTB_MARKER) != 0; }

struct PropView {
  const uint32_t* p = nullptr;  // [n, (k, v)*n]
  uint32_t n() const { return p ? p[0] : 0; }
};
PropView props_of(mtb_dev* b, const HostDoc& d, uint32_t h) {
  PropView v;
  if (!h) return v;
  if (h & MTB_GPROPS) v.p = b->in.pool.data() + (h & ~MTB_GPROPS);
  else v.p = d.aux.data() + (h & ~MTB_PNAN);
  return v;
}
void props_json(mtb_dev* b, std::string& o, PropView v) {
  o += '{';
  for (uint32_t i = 0; i < v.n(); i++) {
    if (i) o += ',';
    o += b->in.keyJson[v.p[1 + 2 * i]];
    o += ':';
    o += b->in.valJson[v.p[2 + 2 * i]];
  }
  o += '}';
}
// matchProperties(a, c) (properties.ts:71-96): a is the run head's set
// NaN and consensus values (valFalsy bit 3) never match as c's; as a's, NaN (no own keys) matches an object or array
// without own keys (bit 4) and a consensus value nothing (its cv-like partners are refused)
bool props_match(mtb_dev* b, PropView a, PropView c) {
  if (a.n() != c.n()) return false;
  const auto& F = b->in.valFalsy;
  for (uint32_t i = 0; i < a.n(); i++) {
    bool found = false;
    for (uint32_t q = 0; q < c.n(); q++) {
      if (c.p[1 + 2 * q] == a.p[1 + 2 * i]) {
        found = true;
        const uint32_t va = a.p[2 + 2 * i], vc = c.p[2 + 2 * q];
        if (F[vc] & 8) return false;
        if (F[va] & 8) {
          if (!(va == b->in.nanVal && (F[vc] & 16))) return false;
        } else if (!b->in.value_match(a.p[1 + 2 * i], va, vc)) {
          return false;
        }
      }
    }
    if (!found) return false;
  }
  return true;
}

void rc_list(const HostDoc& d, const Seg& s, std::vector<int>& out) {
  out.clear();
  if (!seg_removed(s)) return;
  out.push_back(s.rc0);
  if (s.rcx)
    for (uint32_t i = 0; i < d.aux[s.rcx]; i++) out.push_back((int)d.aux[s.rcx + 1 + i]);
}

// PermutationSegment.toJSONObject (permutationvector.ts:107): [length, start]
std::string perm_json(int len, uint32_t start) { return "[" + std::to_string(len) + "," + std::to_string((int32_t)start) + "]"; }
// HandleTable.getSummaryContent (handletable.ts:82): the handles array, from the text-arena words
std::string handle_table_json(const HostDoc& d) {
  auto word = [&](size_t k) { return (uint32_t)d.text[2 * k] | ((uint32_t)d.text[2 * k + 1] << 16); };
  const uint32_t L = d.text.size() >= 2 ? word(0) : 0;
  std::string o = "[";
  for (uint32_t k = 0; k < L && 2 * (k + 2) <= d.text.size(); k++) {
    if (k) o += ',';
    o += std::to_string(word(1 + k));
  }
  return o + "]";
}

std::string dump_doc(mtb_dev* b, uint32_t i) {
  download_doc(b, i);
  const HostDoc& d = b->docs[i];
  const DocState& s = b->hst[i];
  std::string o = "{\"minSeq\":" + std::to_string(s.min_seq) + ",\"currentSeq\":" + std::to_string(s.cur_seq) +
                  ",\"length\":" + std::to_string(d.blks[s.root].len);
  if (d.perm) o += ",\"handles\":" + handle_table_json(d);
  o += "}\n";
  std::vector<FlatSeg> fl;
  flatten(d, s.root, fl, true);
  std::vector<int> rc;
  for (auto& f : fl) {
    const Seg& g = d.segs[f.id];
    o += "[[";
    for (size_t k = 0; k < f.path.size(); k++) {
      if (k) o += ',';
      o += std::to_string(f.path[k]);
    }
    o += "],";
    if (d.perm) {
      o += "\"P\"," + perm_json(g.len, g.text);
    } else if (is_marker(g)) {
      const uint32_t rt = g.text & ~MTB_MARKER;
      o += "\"M\",";
      o += rt == 0 ? "null" : std::to_string(rt - 1);
    } else {
      o += "\"T\",";
      hj::quote(o, reinterpret_cast<const char16_t*>(d.text.data() + g.text), (size_t)g.len);
    }
    // PermutationVectors name clients by long id: their short ids depend on setCell interning order
    auto cl = [&](int c) {
      if (!d.perm) return std::to_string(d.ref_id(c));
      std::string q;
      hj::quote_u8(q, d.longId(c));
      return q;
    };
    o += ',' + std::to_string(seq_out(g.seq)) + ',' + cl(g.client) + ',' + std::to_string(seg_removed(g) ? seq_out(g.rseq) : -1) + ",[";
    rc_list(d, g, rc);
    for (size_t k = 0; k < rc.size(); k++) {
      if (k) o += ',';
      o += cl(rc[k]);
    }
    o += "],";
    PropView pv = props_of(b, d, g.props);
    if (g.props && pv.n() > 0) props_json(b, o, pv);
    else o += "null";
    o += "]\n";
  }
  return o;
}

uint64_t fnv(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

// utf8ByteLength (runtime-utils summaryUtils.ts:56-71) evaluated on the JS string of `utf8`
uint64_t utf8_byte_length(const std::string& utf8) {
  {  // well-formed UTF-8 without encoded surrogates (the serializers' output): its own byte count
    const uint8_t* p = reinterpret_cast<const uint8_t*>(utf8.data());
    const uint8_t* const e = p + utf8.size();
    size_t n = 1;
    while (p < e) {
      uint64_t w8;
      if (e - p >= 8 && (memcpy(&w8, p, 8), (w8 & 0x8080808080808080ull) == 0)) {  // eight ASCII bytes
        p += 8;
        continue;
      }
      if ((n = *p < 0x80 ? 1 : hj::utf8_seq(p, e)) == 0) break;
      p += n;
    }
    if (p == e) return utf8.size();
  }
  U16 s = hj::from_utf8(utf8);
  int64_t n = (int64_t)s.size();
  for (int64_t k = (int64_t)s.size() - 1; k >= 0; k--) {
    const uint32_t c = s[(size_t)k];
    if (c > 0x7f && c <= 0x7ff) n++;
    else if (c > 0x7ff && c <= 0xffff) n += 2;
    if (c >= 0xdc00 && c <= 0xdfff) k--;
  }
  return (uint64_t)n;
}

void emit_v1_chunks(mtb_dev* b, int minSeq, int curSeq, const std::vector<std::string>& segJson, const std::vector<int>& segLen,
                    std::vector<std::pair<std::string, std::string>>& blobs, std::string& tree, uint64_t& totalBytes);
#define EX_INLINE_HOST 0x40000000u  // mtb_extract_v1_kernel: a property set copied into the words output
void summarize_items(mtb_dev* b, uint32_t i, const uint32_t* items, uint32_t nwords, const uint16_t* txt, const uint32_t* words,
                     std::vector<std::pair<std::string, std::string>>& blobs, std::string& summaryJson);

// SnapshotV1.extractSync + emit (snapshotV1.ts:122-312) over the downloaded document.
void summarize(mtb_dev* b, uint32_t i, std::vector<std::pair<std::string, std::string>>& blobs, std::string& summaryJson) {
  download_doc(b, i);
  const HostDoc& d = b->docs[i];
  const DocState& s = b->hst[i];
  const int minSeq = s.min_seq, curSeq = s.cur_seq;
  std::vector<FlatSeg> fl;
  flatten(d, s.root, fl, false);
  std::vector<std::string> segJson;
  std::vector<int> segLen;
  struct Prev {
    bool live = false;
    U16 text;
    int len = 0;
    bool marker = false;
    uint32_t refType = 0;
    uint32_t props = 0;
    uint32_t start = 0;  // PermutationSegment
  };
  auto textOf = [&](const Seg& g) { return U16(reinterpret_cast<const char16_t*>(d.text.data() + g.text), (size_t)g.len); };
  const bool perm = d.perm;
  auto json_of = [&](bool marker, uint32_t refType, const U16& text, uint32_t props) {
    std::string o;
    PropView pv = props_of(b, d, props);
    const bool hasProps = props && pv.n() > 0;  // empty props normalized to undefined (snapshotV1.ts:199-206)
    if (marker) {
      o += "{\"marker\":{";
      if (refType) o += "\"refType\":" + std::to_string(refType - 1);
      o += "}";
      if (hasProps) { o += ",\"props\":"; props_json(b, o, pv); }
      o += "}";
    } else if (hasProps) {
      o += "{\"text\":";
      hj::quote(o, text);
      o += ",\"props\":";
      props_json(b, o, pv);
      o += "}";
    } else {
      hj::quote(o, text);
    }
    return o;
  };
  std::unique_ptr<Prev> prev;
  auto pushPrev = [&]() {
    if (!prev) return;
    segJson.push_back(perm ? perm_json(prev->len, prev->start) : json_of(prev->marker, prev->refType, prev->text, prev->props));
    segLen.push_back(prev->len);
    prev.reset();
  };
  std::vector<int> rc;
  for (auto& f : fl) {
    const Seg& g = d.segs[f.id];
    if (seg_pending(g.seq)) continue;                         // seq === UnassignedSequenceNumber
    // elided: removedSeq <= minSeq, which includes an unacked local removal (removedSeq ===
    // UnassignedSequenceNumber = -1, snapshotV1.ts:218)
    if (seg_removed(g) && (seg_pending(g.rseq) || g.rseq <= minSeq)) continue;
    if (g.seq <= minSeq && (!seg_removed(g) || seg_pending(g.rseq))) {
      const bool marker = !perm && is_marker(g);
      if (perm) {  // PermutationSegment.canAppend: both unallocated, or contiguous handles
        if (prev && (prev->start == MTB_HANDLE_UNALLOC ? g.text == MTB_HANDLE_UNALLOC : g.text == prev->start + (uint32_t)prev->len)) {
          prev->len += g.len;
          prev->live = false;
        } else {
          pushPrev();
          prev.reset(new Prev());
          prev->live = true;
          prev->len = g.len;
          prev->start = g.text;
        }
        continue;
      }
      if (!prev) {
        prev.reset(new Prev());
        prev->live = true;
        prev->marker = marker;
        prev->refType = marker ? (g.text & ~MTB_MARKER) : 0;
        if (!marker) prev->text = textOf(g);
        prev->len = g.len;
        prev->props = g.props;
        continue;
      }
      // TextSegment.canAppend (textSegment.ts:71-78) + matchProperties
      bool can = !prev->marker && !marker && !(prev->len > 0 && prev->text.back() == u'\n') &&
                 (prev->len <= 256 || g.len <= 256) && props_match(b, props_of(b, d, prev->props), props_of(b, d, g.props));
      if (can) {
        prev->text += textOf(g);
        prev->len += g.len;
        prev->live = false;
      } else {
        pushPrev();
        prev.reset(new Prev());
        prev->live = true;
        prev->marker = marker;
        prev->refType = marker ? (g.text & ~MTB_MARKER) : 0;
        if (!marker) prev->text = textOf(g);
        prev->len = g.len;
        prev->props = g.props;
      }
      continue;
    }
    pushPrev();
    std::string o = "{\"json\":";
    if (perm) o += perm_json(g.len, g.text);
    else o += json_of(is_marker(g), is_marker(g) ? (g.text & ~MTB_MARKER) : 0, is_marker(g) ? U16() : textOf(g), g.props);
    if (g.seq > minSeq) {
      o += ",\"seq\":" + std::to_string(g.seq) + ",\"client\":";
      hj::quote_u8(o, d.longId(g.client));
    }
    if (seg_removed(g)) {
      if (seg_pending(g.rseq)) raise(MTB_E_ASSERT, "0x065 invalid removed seq");
      rc_list(d, g, rc);
      o += ",\"removedSeq\":" + std::to_string(g.rseq) + ",\"removedClient\":";
      hj::quote_u8(o, d.longId(rc[0]));
      o += ",\"removedClientIds\":[";
      for (size_t k = 0; k < rc.size(); k++) {
        if (k) o += ',';
        hj::quote_u8(o, d.longId(rc[k]));
      }
      o += "]";
    }
    o += "}";
    segJson.push_back(o);
    segLen.push_back(g.len);
  }
  pushPrev();
  std::string tree;
  uint64_t totalBytes = 0;
  emit_v1_chunks(b, minSeq, curSeq, segJson, segLen, blobs, tree, totalBytes);
  if (perm) {
    // PermutationVector.summarize (permutationvector.ts:310-325): {segments: <SnapshotV1>, handleTable}
    const std::string ht = handle_table_json(d);
    std::string outer = "{\"segments\":{\"type\":1,\"tree\":" + tree + "},\"handleTable\":{\"type\":2,\"content\":";
    hj::quote_u8(outer, ht);
    outer += "}}";
    totalBytes += utf8_byte_length(ht);
    summaryJson = "{\"summary\":{\"type\":1,\"tree\":" + outer + "},\"stats\":{\"treeNodeCount\":2,\"blobNodeCount\":" +
                  std::to_string(blobs.size() + 1) + ",\"handleNodeCount\":0,\"totalBlobSize\":" + std::to_string(totalBytes) +
                  ",\"unreferencedBlobSize\":0}}";
    for (auto& bl : blobs) bl.first = "segments/" + bl.first;
    blobs.push_back({"handleTable", ht});
    return;
  }
  summaryJson = "{\"summary\":{\"type\":1,\"tree\":" + tree + "},\"stats\":{\"treeNodeCount\":1,\"blobNodeCount\":" +
                std::to_string(blobs.size()) + ",\"handleNodeCount\":0,\"totalBlobSize\":" + std::to_string(totalBytes) +
                ",\"unreferencedBlobSize\":0}}";
}

// SnapshotV1.emit (snapshotV1.ts:122-178): the serialized segments cut into chunks of about chunkSize
// UTF-16 units (header + body_i) and the summary tree's blobs (runtime-utils summaryUtils.ts:138-198)
struct V1Chunk {
  int start = 0, count = 0, length = 0;
};
struct V1Chunks {
  std::vector<V1Chunk> c;
  int totalCount = 0, totalLength = 0;
};
void append_int(std::string& o, int64_t v) {
  char buf[24];
  const auto r = std::to_chars(buf, buf + sizeof buf, v);
  o.append(buf, (size_t)(r.ptr - buf));
}
V1Chunks v1_chunks(mtb_dev* b, const std::vector<int>& segLen) {
  const int chunkSize = b->opts.chunk_size > 0 ? b->opts.chunk_size : 10000;
  V1Chunks r;
  do {
    V1Chunk c;
    c.start = r.totalCount;
    while (c.length < chunkSize && c.start + c.count < (int)segLen.size()) {
      c.length += segLen[c.start + c.count];
      c.count++;
    }
    r.c.push_back(c);
    r.totalCount += c.count;
    r.totalLength += c.length;
  } while (r.totalCount < (int)segLen.size());
  return r;
}
void v1_chunk_open(std::string& o, const V1Chunk& c) {
  o += "{\"version\":\"1\",\"segmentCount\":";
  append_int(o, c.count);
  o += ",\"length\":";
  append_int(o, c.length);
  o += ",\"segments\":[";
}
void v1_chunk_close(std::string& o, const V1Chunks& cs, size_t k, int minSeq, int curSeq) {
  o += "],\"startIndex\":";
  append_int(o, cs.c[k].start);
  if (k == 0) {
    o += ",\"headerMetadata\":{\"minSequenceNumber\":";
    append_int(o, minSeq);
    o += ",\"sequenceNumber\":";
    append_int(o, curSeq);
    o += ",\"orderedChunkMetadata\":[";
    for (size_t q = 0; q < cs.c.size(); q++) {
      if (q) o += ',';
      if (q == 0) {
        o += "{\"id\":\"header\"}";
      } else {
        o += "{\"id\":\"body_";
        append_int(o, (int64_t)q - 1);
        o += "\"}";
      }
    }
    o += "],\"totalLength\":";
    append_int(o, cs.totalLength);
    o += ",\"totalSegmentCount\":";
    append_int(o, cs.totalCount);
    o += "}";
  }
  o += "}";
}
std::string v1_blob_name(size_t k) { return k == 0 ? std::string("header") : "body_" + std::to_string(k - 1); }
// ISummaryTreeWithStats.summary.tree of the blobs (runtime-utils summaryUtils.ts:138-198), appended to o
void v1_tree(std::string& o, const std::vector<std::pair<std::string, std::string>>& blobs, uint64_t& totalBytes) {
  o += '{';
  totalBytes = 0;
  for (size_t k = 0; k < blobs.size(); k++) {
    if (k) o += ',';
    o += '"';
    o += blobs[k].first;
    o += "\":{\"type\":2,\"content\":";
    hj::quote_u8(o, blobs[k].second);
    o += '}';
    totalBytes += utf8_byte_length(blobs[k].second);
  }
  o += '}';
}
void v1_stats(std::string& o, int treeNodeCount, size_t blobNodeCount, uint64_t totalBytes) {
  o += "},\"stats\":{\"treeNodeCount\":";
  append_int(o, treeNodeCount);
  o += ",\"blobNodeCount\":";
  append_int(o, (int64_t)blobNodeCount);
  o += ",\"handleNodeCount\":0,\"totalBlobSize\":";
  append_int(o, (int64_t)totalBytes);
  o += ",\"unreferencedBlobSize\":0}}";
}
void emit_v1_chunks(mtb_dev* b, int minSeq, int curSeq, const std::vector<std::string>& segJson, const std::vector<int>& segLen,
                    std::vector<std::pair<std::string, std::string>>& blobs, std::string& tree, uint64_t& totalBytes) {
  const V1Chunks cs = v1_chunks(b, segLen);
  blobs.clear();
  for (size_t k = 0; k < cs.c.size(); k++) {
    const V1Chunk& c = cs.c[k];
    size_t bytes = 256 + 24 * cs.c.size();
    for (int q = 0; q < c.count; q++) bytes += segJson[c.start + q].size() + 1;
    std::string o;
    o.reserve(bytes);
    v1_chunk_open(o, c);
    for (int q = 0; q < c.count; q++) {
      if (q) o += ',';
      o += segJson[c.start + q];
    }
    v1_chunk_close(o, cs, k, minSeq, curSeq);
    blobs.push_back({v1_blob_name(k), std::move(o)});
  }
  tree.clear();
  v1_tree(tree, blobs, totalBytes);
}

// SnapshotV1 of a SharedString document from the device extraction (mtb_extract_v1_kernel): the same JSON
// as summarize() without downloading the tree.
void summarize_items(mtb_dev* b, uint32_t i, const uint32_t* items, uint32_t nwords, const uint16_t* txt, const uint32_t* words,
                     std::vector<std::pair<std::string, std::string>>& blobs, std::string& summaryJson) {
  const HostDoc& d = b->docs[i];
  const DocState& s = b->hst[i];
  const int minSeq = s.min_seq, curSeq = s.cur_seq;
  auto pview = [&](uint32_t h) {
    PropView v;
    if (!h) return v;
    if (h & MTB_GPROPS) v.p = b->in.pool.data() + (h & ~MTB_GPROPS);
    else v.p = words + (h & ~EX_INLINE_HOST);
    return v;
  };
  // the chunks first (they depend on the segment lengths only), then every segment's JSON written straight
  // into its chunk's blob: the bytes of summarize()'s segJson + emit_v1_chunks, without the per-segment strings
  // items are 4 words, 8 with merge info (EX_META): their starts first
  std::vector<uint32_t> at;
  at.reserve(nwords / 4 + 1);
  for (uint32_t w = 0; w + 4 <= nwords; w += (items[w] & 1u) ? 8u : 4u) at.push_back(w);
  const uint32_t ni = (uint32_t)at.size();
  std::vector<int> segLen(ni);
  for (uint32_t k = 0; k < ni; k++) segLen[k] = (int)items[at[k] + 1];
  const V1Chunks cs = v1_chunks(b, segLen);
  auto seg_json = [&](std::string& o, const uint32_t* it) {
    const uint32_t fl = it[0], len = it[1], toff = it[2];
    const bool marker = (fl & 2u) != 0;
    const uint32_t refType = fl >> 8;
    PropView pv = pview(it[3]);
    const bool hasProps = pv.n() > 0;  // empty props normalized to undefined (snapshotV1.ts:199-206)
    const bool info = (fl & 1u) != 0;  // else a coalesced (or single) segment below the MSN: its JSON alone
    if (info) o += "{\"json\":";
    if (marker) {
      o += "{\"marker\":{";
      if (refType) {
        o += "\"refType\":";
        append_int(o, (int64_t)refType - 1);
      }
      o += "}";
      if (hasProps) { o += ",\"props\":"; props_json(b, o, pv); }
      o += "}";
    } else if (hasProps) {
      o += "{\"text\":";
      hj::quote(o, reinterpret_cast<const char16_t*>(txt + toff), len);
      o += ",\"props\":";
      props_json(b, o, pv);
      o += "}";
    } else {
      hj::quote(o, reinterpret_cast<const char16_t*>(txt + toff), len);
    }
    if (!info) return;
    const int seq = (int)it[4], rseq = (int)it[6];
    const uint32_t cli = it[5];
    if (seq > minSeq) {
      o += ",\"seq\":";
      append_int(o, seq);
      o += ",\"client\":";
      hj::quote_u8(o, d.longId((int)(int16_t)(cli & 0xFFFF)));
    }
    if (rseq >= 0) {
      const int rc0 = (int)(int16_t)(cli >> 16);
      o += ",\"removedSeq\":";
      append_int(o, rseq);
      o += ",\"removedClient\":";
      hj::quote_u8(o, d.longId(rc0));
      o += ",\"removedClientIds\":[";
      hj::quote_u8(o, d.longId(rc0));
      if (it[7] != MTB_NONE) {
        const uint32_t* rc = words + it[7];
        for (uint32_t q = 0; q < rc[0]; q++) {
          o += ',';
          hj::quote_u8(o, d.longId((int)rc[1 + q]));
        }
      }
      o += "]";
    }
    o += "}";
  };
  blobs.clear();
  size_t blobBytes = 0;
  for (size_t k = 0; k < cs.c.size(); k++) {
    const V1Chunk& c = cs.c[k];
    std::string o;
    o.reserve((size_t)c.length + (size_t)c.length / 8 + 64 * (size_t)c.count + 256 + 24 * cs.c.size());
    v1_chunk_open(o, c);
    for (int q = 0; q < c.count; q++) {
      if (q) o += ',';
      seg_json(o, items + at[c.start + q]);
    }
    v1_chunk_close(o, cs, k, minSeq, curSeq);
    blobBytes += o.size();
    blobs.push_back({v1_blob_name(k), std::move(o)});
  }
  summaryJson.clear();
  summaryJson.reserve(blobBytes + blobBytes / 4 + 256);
  summaryJson += "{\"summary\":{\"type\":1,\"tree\":";
  uint64_t totalBytes = 0;
  v1_tree(summaryJson, blobs, totalBytes);
  v1_stats(summaryJson, 1, blobs.size(), totalBytes);
}

// ok[k]: document ids[k] was extracted (a SharedString document replayed without error).
struct Extracted {  // (items / text / words point into the batch's staging buffers)
  std::vector<uint8_t> ok;
  std::vector<uint32_t> cnt;
  std::vector<uint64_t> off;
  const uint32_t* items = nullptr;
  const uint32_t* words = nullptr;
  const uint16_t* text = nullptr;
  // Download in pieces (extract_docs with pieces > 1): piece p holds the outputs of the extracted documents
  // [first[p], first[p + 1]) in extraction order; copy_piece() downloads one and marks it ready, and a
  // serializer thread waits (wait_doc) only for the piece of the document it takes.
  uint32_t npieces = 0;
  std::vector<uint32_t> pieceOf;               // position in ids -> piece (extracted documents)
  std::vector<std::array<uint64_t, 3>> first;  // per piece + 1: items word, text unit, words word offsets
  uint32_t* hItems = nullptr;
  uint32_t* hWords = nullptr;
  uint16_t* hText = nullptr;
  std::unique_ptr<std::atomic<int>[]> ready;   // 1 copied, -1 failed
  std::mutex mu;
  std::condition_variable cv;
  bool wait_doc(uint32_t k) {  // false: the download failed
    if (!npieces) return true;
    std::atomic<int>& r = ready[pieceOf[k]];
    if (r.load(std::memory_order_acquire) == 0) {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return r.load(std::memory_order_acquire) != 0; });
    }
    return r.load(std::memory_order_acquire) > 0;
  }
  void mark(uint32_t p, int v) {
    {
      std::lock_guard<std::mutex> lk(mu);
      ready[p].store(v, std::memory_order_release);
    }
    cv.notify_all();
  }
};
template <class T>
T* staging(std::unique_ptr<T[]>& p, size_t& cap, size_t need) {
  if (need > cap) {
    p.reset();
    p.reset(new T[need]);
    cap = need;
  }
  return p.get();
}
void copy_piece(mtb_dev* b, Extracted& ex, uint32_t p) {
  const auto& a = ex.first[p];
  const auto& z = ex.first[p + 1];
  if (z[0] > a[0])
    HIPCHK(hipMemcpyAsync(ex.hItems + a[0], b->dExItems.p + a[0], (z[0] - a[0]) * sizeof(uint32_t), hipMemcpyDeviceToHost, b->stream));
  if (z[1] > a[1])
    HIPCHK(hipMemcpyAsync(ex.hText + a[1], b->dExText.p + a[1], (z[1] - a[1]) * sizeof(uint16_t), hipMemcpyDeviceToHost, b->stream));
  if (z[2] > a[2])
    HIPCHK(hipMemcpyAsync(ex.hWords + a[2], b->dExWords.p + a[2], (z[2] - a[2]) * sizeof(uint32_t), hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
}
// mtb_extract_v1_kernel over documents `ids` (count pass, offsets, emit pass).  pieces <= 1: the outputs are
// downloaded before it returns; else the caller downloads them with copy_piece(0 .. ex.npieces - 1).
void extract_docs(mtb_dev* b, const std::vector<uint32_t>& ids, Extracted& ex, uint32_t pieces = 1) {
  const uint32_t n = (uint32_t)ids.size();
  ex.ok.assign(n, 0);
  ex.cnt.assign(3 * (size_t)n + 3, 0);
  ex.off.assign(3 * (size_t)n + 3, 0);
  ex.npieces = 0;
  std::vector<uint32_t> dev;  // positions in ids
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t i = ids[k];
    if (b->devInit && i < b->hst.size() && b->docs[i].onDevice && !b->docs[i].perm && !b->hst[i].err &&
        !getenv("MTB_HOST_SUMMARY"))
      dev.push_back(k);
  }
  const uint32_t nf = (uint32_t)dev.size();
  if (!nf) return;
  std::vector<uint32_t> di(nf), cnt(3 * (size_t)nf);
  for (uint32_t f = 0; f < nf; f++) di[f] = ids[dev[f]];
  DevBuf<uint32_t> dl, dc;
  DevBuf<uint64_t> doff;
  dl.ensure(nf);
  dc.ensure(3 * (size_t)nf);
  HIPCHK(hipMemcpyAsync(dl.p, di.data(), nf * sizeof(uint32_t), hipMemcpyHostToDevice, b->stream));
  HIPCHK(mtb_launch_extract_v1(b->stream, b->dDocs.p, dl.p, nf, b->dBlks.p, b->dText.p, b->dAux.p, b->dPool.p,
                               make_tables(b), dc.p, nullptr, nullptr, nullptr, nullptr));
  HIPCHK(hipMemcpyAsync(cnt.data(), dc.p, 3 * (size_t)nf * sizeof(uint32_t), hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  std::vector<uint64_t> off(3 * (size_t)nf);
  uint64_t ti = 0, tt = 0, tw = 0;
  for (uint32_t f = 0; f < nf; f++) {
    const bool good = cnt[3 * f] != MTB_NONE;  // else the device walk did not trust the tree: host path
    if (!good) cnt[3 * f] = cnt[3 * f + 1] = cnt[3 * f + 2] = 0;
    off[3 * f] = ti;
    off[3 * f + 1] = tt;
    off[3 * f + 2] = tw;
    ti += cnt[3 * f];
    tt += cnt[3 * f + 1];
    tw += cnt[3 * f + 2];
    const uint32_t k = dev[f];
    ex.ok[k] = good;
    ex.cnt[3 * k] = cnt[3 * f];
    for (int q = 0; q < 3; q++) ex.off[3 * k + q] = off[3 * f + q];
  }
  b->dExItems.ensure(ti + 8);
  b->dExText.ensure(tt + 1);
  b->dExWords.ensure(tw + 1);
  doff.ensure(3 * (size_t)nf);
  HIPCHK(hipMemcpyAsync(doff.p, off.data(), 3 * (size_t)nf * sizeof(uint64_t), hipMemcpyHostToDevice, b->stream));
  HIPCHK(mtb_launch_extract_v1(b->stream, b->dDocs.p, dl.p, nf, b->dBlks.p, b->dText.p, b->dAux.p, b->dPool.p,
                               make_tables(b), dc.p, doff.p, b->dExItems.p, b->dExText.p, b->dExWords.p));
  ex.hItems = staging(b->exItems, b->exItemsCap, ti + 8);
  ex.hText = staging(b->exText, b->exTextCap, tt + 1);
  ex.hWords = staging(b->exWords, b->exWordsCap, tw + 1);
  ex.items = ex.hItems;
  ex.text = ex.hText;
  ex.words = ex.hWords;
  const uint32_t P = std::max<uint32_t>(1, std::min<uint32_t>(pieces, nf));
  ex.first.assign(P + 1, {0, 0, 0});
  ex.pieceOf.assign(n, 0);
  for (uint32_t p = 0; p < P; p++) {
    const uint32_t fa = (uint32_t)((uint64_t)p * nf / P), fb = (uint32_t)((uint64_t)(p + 1) * nf / P);
    for (uint32_t f = fa; f < fb; f++) ex.pieceOf[dev[f]] = p;
    ex.first[p] = {off[3 * fa], off[3 * fa + 1], off[3 * fa + 2]};
  }
  ex.first[P] = {ti, tt, tw};
  if (pieces <= 1) {
    copy_piece(b, ex, 0);
    return;
  }
  ex.npieces = P;
  ex.ready.reset(new std::atomic<int>[P]);
  for (uint32_t p = 0; p < P; p++) ex.ready[p].store(0);
}

// SnapshotV1 of one document: the device extraction when it applies, else the host path
void summarize_any(mtb_dev* b, uint32_t doc, std::vector<std::pair<std::string, std::string>>& blobs, std::string& summary) {
  Extracted ex;
  extract_docs(b, {doc}, ex);
  if (ex.ok[0]) summarize_items(b, doc, ex.items, ex.cnt[0], ex.text, ex.words, blobs, summary);
  else summarize(b, doc, blobs, summary);
}

// processMinSequenceNumberChanged (sequence.ts:737-748)
void drop_catch_up(HostDoc& d, int64_t minSeq) {
  size_t i = 0;
  for (; i < d.catchup.size(); i++) {
    const hj::Value* sq = member(d.catchup[i].msg, u"sequenceNumber");
    if (sq && sq->n > (double)minSeq) break;
  }
  d.catchup.erase(d.catchup.begin(), d.catchup.begin() + (long)i);
}

// Client.applyMsg (client.ts:858-887) -> records appended to d
void apply_msg(mtb_dev* b, HostDoc& d, const hj::Value& msg) {
  {
    if (msg.kind != hj::Value::kObj) raise(MTB_E_PARSE, "message is not an object");
    const hj::Value* cid = member(msg, u"clientId");
    if (!cid || cid->kind != hj::Value::kStr) raise(MTB_E_UNSUPPORTED, "unsupported: message without a string clientId");
    const std::string longId = hj::to_utf8(cid->s.data(), cid->s.size());
    mtb_op base{};
    base.client = d.client(longId);
    base.seq = u32field(msg, u"sequenceNumber", "sequenceNumber");
    base.ref_seq = u32field(msg, u"referenceSequenceNumber", "referenceSequenceNumber");
    base.msn = u32field(msg, u"minimumSequenceNumber", "minimumSequenceNumber");
    if ((int64_t)base.seq < d.lastSeq) raise(MTB_E_ASSERT, "0x038 Incoming op sequence# < local collabWindow's currentSequence#");
    if (base.msn > base.seq) raise(MTB_E_ASSERT, "0x039 Incoming op sequence# < minSequence#");
    std::vector<mtb_op> recs;
    const size_t payloadBefore = d.payload.size();
    const hj::Value* type = member(msg, u"type");
    const bool isOp = type && type->kind == hj::Value::kStr && type->s == u"op";
    const hj::Value* contents = member(msg, u"contents");
    const size_t recFirst = d.pending.size();
    if (isOp) {
      if (!contents || contents->kind != hj::Value::kObj) raise(MTB_E_PARSE, "op message without contents");
      if (longId == d.observer) {
        // the client's own op: Client.ackPendingSegment (client.ts:641-662), one MergeTree.ackPendingSegment
        // (mergeTree.ts:1283-1322: the oldest pending group, then zamboni) per member; pos2 = its op type
        auto ack = [&](const hj::Value& op) {
          const hj::Value* t = member(op, u"type");
          mtb_op r = base;
          r.type = MTB_OP_ACK;
          r.pos2 = t && t->kind == hj::Value::kNum ? (uint32_t)(int)t->n : 0xFFFFFFFFu;
          // updateConsensusProperty (client.ts:1050-1058): the registered marker's values at the ack's seq
          const hj::Value* comb = member(op, u"combiningOp");
          const hj::Value* cname = comb && comb->kind == hj::Value::kObj ? member(*comb, u"name") : nullptr;
          if (r.pos2 == 2 && cname && cname->kind == hj::Value::kStr && cname->s == u"consensus") {
            const hj::Value* r1 = member(op, u"relativePos1");
            const hj::Value* id = r1 && r1->kind == hj::Value::kObj ? member(*r1, u"id") : nullptr;
            if (!id || !d.pendingConsensus.count(hj::dump(*id)))
              raise(MTB_E_UNSUPPORTED, "unsupported: consensus ack without annotateMarkerNotifyConsensus (the reference "
                                       "throws at a later minimum sequence number update)");
            const hj::Value* props = member(op, u"props");
            hj::Value empty;
            empty.kind = hj::Value::kObj;
            r.props = b->in.consensus_props(b->in.props(props && props->kind == hj::Value::kObj ? *props : empty),
                                            nullptr, (int)r.seq);
            d.vals.propsSeen.push_back(r.props);
            r.flags |= MTB_F_CONSENSUS;
            // the registered marker (consensusInfo.marker), by its id's ordinal + 1: completed whether or not the
            // op's range reached it (a removed marker's relative range covers the next segment)
            auto key = marker_key(id);
            auto mo = key ? d.markerOrd.find(*key) : d.markerOrd.end();
            r.payload = mo == d.markerOrd.end() ? 0u : mo->second + 1;
          }
          recs.push_back(r);
        };
        const hj::Value* t = member(*contents, u"type");
        if (t && t->kind == hj::Value::kNum && (int)t->n == 3) {
          const hj::Value* ops = member(*contents, u"ops");
          if (ops && ops->kind == hj::Value::kArr)
            for (auto& m : ops->items) ack(m);
        } else {
          ack(*contents);
        }
      } else {
        pack_delta(b, d, *contents, base, recs);
      }
    }
    if (recs.empty()) {
      mtb_op r = base;
      r.type = MTB_OP_NOOP;
      recs.push_back(r);
    }
    recs.back().flags |= MTB_F_LAST;
    if (isOp && (b->opts.flags & MTB_BATCH_CATCHUP) && !d.perm) {
      // processMergeTreeMsg (sequence.ts:697-733)
      HostDoc::CatchMsg cm;
      cm.msg = msg;
      cm.first = (uint32_t)recFirst;
      cm.count = (uint32_t)recs.size();
      if ((int64_t)base.ref_seq != (int64_t)base.seq - 1) {
        cm.resolved = false;
        for (mtb_op& r : recs)
          if (r.type == MTB_OP_INSERT || r.type == MTB_OP_REMOVE || r.type == MTB_OP_ANNOTATE) r.flags |= MTB_F_DELTA;
      }
      d.catchup.push_back(std::move(cm));
      if (d.catchup.size() > 20) {  // "Do GC every once in a while"
        const hj::Value* s20 = member(d.catchup[20].msg, u"sequenceNumber");
        if (s20 && s20->n < (double)base.msn) drop_catch_up(d, (int64_t)base.msn);
      }
    }
    d.totalPayload += d.payload.size() - payloadBefore;
    d.pending.insert(d.pending.end(), recs.begin(), recs.end());
    d.totalOps += recs.size();
    d.lastSeq = base.seq;
  }
}


// Replay one matrix's cell events of this replay into its CellStore.  Both vectors' record streams hold
// every setCell; a clear logged at record k of either stream happened after the setCells before k and
// before the next one, and clears commute with each other, so events are merged by setCell ordinal.
void apply_cell_events(mtb_dev* b, uint32_t m) {
  HostDoc& R = b->docs[2 * m];
  if (!R.cells) R.cells.reset(new CellStore());
  struct Ev { uint32_t epoch, kind, a, n; };
  std::vector<Ev> ev[2];
  std::vector<uint32_t> setVal;
  for (int v = 0; v < 2; v++) {
    const DocState& s = b->hst[2 * m + v];
    const std::vector<mtb_op>& recs = b->docs[2 * m + v].applied;
    std::vector<uint32_t> ent(4 * (size_t)s.delta_used);
    if (!ent.empty())
      HIPCHK(hipMemcpy(ent.data(), b->dDelta.p + 4 * s.delta_base, ent.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> ordinal(recs.size() + 1, 0);  // setCells before record k
    for (size_t k = 0; k < recs.size(); k++) {
      ordinal[k + 1] = ordinal[k] + (recs[k].type == MTB_OP_SETCELL);
      if (v == 0 && recs[k].type == MTB_OP_SETCELL) setVal.push_back(recs[k].props);
    }
    for (uint32_t e = 0; e < s.delta_used; e++) {
      const uint32_t k = ent[4 * e], kind = ent[4 * e + 1];
      if (k >= recs.size()) raise(MTB_E_ASSERT, "cell event names no record");
      // handles recycled while a summary body loads clear the cells of the store that loadCore replaces
      // afterwards (matrix.ts:611-634: rows and cols load before the cells blob), so they touch nothing
      if (recs[k].type == MTB_OP_LOADSEG) continue;
      ev[v].push_back({ordinal[k], kind, ent[4 * e + 2], ent[4 * e + 3]});
    }
  }
  CellStore& cs = *R.cells;
  size_t p[2] = {0, 0};
  for (uint32_t j = 0;; j++) {
    uint32_t h[2] = {0, 0};
    bool have[2] = {false, false};
    for (int v = 0; v < 2; v++)
      for (; p[v] < ev[v].size() && ev[v][p[v]].epoch == j; p[v]++) {
        const Ev& x = ev[v][p[v]];
        if (x.kind == MTB_CELL_CLEAR) {
          for (uint32_t q = 0; q < x.n; q++) v == 0 ? cs.clearRow(x.a + q) : cs.clearCol(x.a + q);
        } else {  // the setCell with ordinal j: its record's events follow the clears logged before it
          h[v] = x.a;
          have[v] = true;
        }
      }
    if (have[0] != have[1]) raise(MTB_E_ASSERT, "setCell allocated in one vector only");
    if (have[0]) cs.set(h[0], h[1], setVal[j]);
    if (p[0] == ev[0].size() && p[1] == ev[1].size()) break;
  }
}

// Rewrite the lagging catch-up messages of this replay from their records' delta entries:
// SharedSegmentSequence.createOpsFromDelta (sequence.ts:120-172) per delta event, the message then
// stored with referenceSequenceNumber = seq - 1 and the ops (a GROUP unless exactly one) as contents.
void resolve_catch_up(mtb_dev* b, uint32_t i) {
  HostDoc& d = b->docs[i];
  const DocState& s = b->hst[i];
  std::vector<uint32_t> ent(4 * (size_t)s.delta_used);
  HIPCHK(hipMemcpy(ent.data(), b->dDelta.p + 4 * s.delta_base, ent.size() * 4, hipMemcpyDeviceToHost));
  d.cached = false;
  download_doc(b, i);
  std::unordered_map<uint32_t, std::vector<uint32_t>> byRec;  // (MTB_DELTA_OLD-tagged: a rewrite's sets before)
  for (uint32_t e = 0; e < s.delta_used; e++) byRec[ent[4 * e]].push_back(e);
  for (auto& m : d.catchup) {
    if (m.resolved) continue;
    std::vector<std::string> ops;
    for (uint32_t k = m.first; k < m.first + m.count && k < d.applied.size(); k++) {
      const mtb_op& r = d.applied[k];
      auto it = byRec.find(k);
      if (it == byRec.end()) continue;  // no delta segments: no event
      struct Ev { int pos1, pos2; std::string props; hj::Value pv; bool hasPos2, nan; std::string json; };
      std::vector<Ev> ev;
      const bool rewrite = r.type == MTB_OP_ANNOTATE && (r.flags & MTB_F_COMB) == MTB_F_REWRITE;
      const std::vector<uint32_t>* before = nullptr;  // a rewrite's entries with the sets before it, same order
      if (rewrite) {
        auto ot = byRec.find(k | MTB_DELTA_OLD);
        if (ot == byRec.end() || ot->second.size() != it->second.size()) raise(MTB_E_ASSERT, "catch-up: rewrite delta entries unpaired");
        before = &ot->second;
      }
      for (size_t ei = 0; ei < it->second.size(); ei++) {
        const uint32_t e = it->second[ei];
        const int position = (int)ent[4 * e + 1];
        const int len = (int)ent[4 * e + 2];
        const uint32_t ph = ent[4 * e + 3];
        if (r.type == MTB_OP_INSERT) {
          std::string seg;
          if (r.flags & MTB_F_MARKER) {
            seg = "{\"marker\":{";
            if (r.pos2 != 0xFFFFFFFFu) seg += "\"refType\":" + std::to_string(r.pos2);
            seg += "}";
            if (r.props) { seg += ",\"props\":"; props_json(b, seg, props_of(b, d, ph)); }
            seg += "}";
          } else {
            U16 text(reinterpret_cast<const char16_t*>(d.appliedPayload.data() + r.payload), r.pos2);
            if (r.props) {
              seg = "{\"text\":";
              hj::quote(seg, text);
              seg += ",\"props\":";
              props_json(b, seg, props_of(b, d, ph));
              seg += "}";
            } else {
              hj::quote(seg, text);
            }
          }
          Ev x{};
          x.json = "{\"pos1\":" + std::to_string(position) + ",\"seg\":" + seg + ",\"type\":0}";
          ev.push_back(std::move(x));
        } else if (r.type == MTB_OP_REMOVE) {
          if (!ev.empty() && ev.back().pos1 == position) {
            ev.back().pos2 += len;
          } else {
            Ev x{};
            x.pos1 = position;
            x.pos2 = position + len;
            ev.push_back(std::move(x));
          }
        } else {  // ANNOTATE: props[key] = segment.properties?.[key] ?? null over the propertyDeltas keys
          // (segmentPropertiesManager.ts:107-154: a rewrite's keys are first the old keys it deleted -- those
          // its props leave falsy -- in their order, then the op's keys; otherwise the op's keys)
          const uint32_t* opl = b->in.pool.data() + b->in.pidx[2 * r.props];
          const PropView sv = props_of(b, d, ph);
          std::vector<uint32_t> keys;
          if (rewrite) {
            const PropView ov = props_of(b, d, ent[4 * (*before)[ei] + 3]);
            for (uint32_t z = 0; z < ov.n(); z++) {
              const uint32_t key = ov.p[1 + 2 * z];
              bool truthy = false;
              for (uint32_t q = 0; q < opl[0]; q++)
                if (opl[1 + 2 * q] == key) truthy = opl[2 + 2 * q] != MTB_NONE && !(b->in.valFalsy[opl[2 + 2 * q]] & 1);
              if (!truthy) keys.push_back(key);
            }
          }
          for (uint32_t q = 0; q < opl[0]; q++)
            if (std::find(keys.begin(), keys.end(), opl[1 + 2 * q]) == keys.end()) keys.push_back(opl[1 + 2 * q]);
          std::string pj = "{";
          bool nan = false;  // an incr's NaN (JSON null): matchProperties never equal (NaN !== NaN)
          hj::Value pv;      // the values themselves (a consensus value's undefined member included)
          pv.kind = hj::Value::kObj;
          for (size_t q = 0; q < keys.size(); q++) {
            if (q) pj += ',';
            hj::quote(pj, b->in.keys[keys[q]]);
            pj += ':';
            std::string val = "null";
            hj::Value x;
            x.kind = hj::Value::kNull;
            for (uint32_t z = 0; z < sv.n(); z++)
              if (sv.p[1 + 2 * z] == keys[q]) {
                const uint32_t v = sv.p[2 + 2 * z];
                val = b->in.valJson[v];
                nan |= v == b->in.nanVal;
                if (v != b->in.nanVal) x = b->in.valStore[v];
              }
            pj += val;
            pv.members.push_back({b->in.keys[keys[q]], std::move(x)});
          }
          pj += "}";
          if (!ev.empty() && ev.back().hasPos2 && ev.back().pos2 == position && !nan && !ev.back().nan &&
              js_match_props(&ev.back().pv, &pv)) {
            ev.back().pos2 += len;
          } else {
            Ev x{};
            x.pos1 = position;
            x.pos2 = position + len;
            x.hasPos2 = true;
            x.nan = nan;
            x.props = pj;
            x.pv = std::move(pv);
            ev.push_back(std::move(x));
          }
        }
      }
      for (auto& x : ev) {
        if (r.type == MTB_OP_INSERT) ops.push_back(x.json);
        else if (r.type == MTB_OP_REMOVE)
          ops.push_back("{\"pos1\":" + std::to_string(x.pos1) + ",\"pos2\":" + std::to_string(x.pos2) + ",\"type\":1}");
        else
          ops.push_back("{\"pos1\":" + std::to_string(x.pos1) + ",\"pos2\":" + std::to_string(x.pos2) + ",\"props\":" +
                        x.props + ",\"type\":2}");
      }
    }
    std::string contents;
    if (ops.size() == 1) {
      contents = ops[0];
    } else {
      contents = "{\"ops\":[";
      for (size_t q = 0; q < ops.size(); q++) {
        if (q) contents += ',';
        contents += ops[q];
      }
      contents += "],\"type\":3}";
    }
    const hj::Value* sq = member(m.msg, u"sequenceNumber");
    for (auto& mem : m.msg.members) {
      if (mem.first == u"referenceSequenceNumber") {
        mem.second = hj::Value();
        mem.second.kind = hj::Value::kNum;
        mem.second.n = sq->n - 1;
      } else if (mem.first == u"contents") {
        mem.second = hj::parse(contents.data(), contents.size());
      }
    }
    m.resolved = true;
  }
}

// SnapshotLegacy.extractSync + emit (snapshotlegacy.ts:122-259) over the downloaded document: every
// segment in the MSN view (inserted at or below the MSN, not removed at or below it), coalesced with
// canAppend + matchProperties, split into "header" (first mergeTreeSnapshotChunkSize chars) and "body",
// plus the catch-up messages blob (sequence.ts:680-692) when given.
void summarize_legacy(mtb_dev* b, uint32_t i, const std::string& catchUp, std::vector<std::pair<std::string, std::string>>& blobs,
                      std::string& summaryJson) {
  download_doc(b, i);
  const HostDoc& d = b->docs[i];
  const DocState& s = b->hst[i];
  if (d.perm) raise(MTB_E_UNSUPPORTED, "unsupported: SnapshotLegacy of a PermutationVector (it forces SnapshotV1)");
  const int seq = s.min_seq;
  std::vector<FlatSeg> fl;
  flatten(d, s.root, fl, false);
  struct Piece {
    bool marker = false;
    uint32_t refType = 0;
    U16 text;
    int len = 0;
    uint32_t props = 0;
  };
  std::vector<Piece> segs;
  auto textOf = [&](const Seg& g) { return U16(reinterpret_cast<const char16_t*>(d.text.data() + g.text), (size_t)g.len); };
  bool havePrev = false;
  Piece prev;
  for (auto& f : fl) {
    const Seg& g = d.segs[f.id];
    if (g.len == 0) continue;  // mapRange skips zero-length nodes
    if (!(g.seq <= seq && (!seg_removed(g) || g.rseq > seq))) continue;
    const bool marker = is_marker(g);
    if (havePrev) {
      // TextSegment.canAppend (textSegment.ts:71-78) + matchProperties
      const bool can = !prev.marker && !marker && !(prev.len > 0 && prev.text.back() == u'\n') &&
                       (prev.len <= 256 || g.len <= 256) && props_match(b, props_of(b, d, prev.props), props_of(b, d, g.props));
      if (can) {
        prev.text += textOf(g);
        prev.len += g.len;
        continue;
      }
      segs.push_back(prev);
    }
    prev = Piece();
    prev.marker = marker;
    prev.refType = marker ? (g.text & ~MTB_MARKER) : 0;
    if (!marker) prev.text = textOf(g);
    prev.len = g.len;
    prev.props = g.props;
    havePrev = true;
  }
  if (havePrev) segs.push_back(prev);
  auto json_of = [&](const Piece& p) {
    std::string o;
    PropView pv = props_of(b, d, p.props);
    const bool hasProps = p.props && pv.n() > 0;  // {} -> undefined (snapshotlegacy.ts:236-243)
    if (p.marker) {
      o += "{\"marker\":{";
      if (p.refType) o += "\"refType\":" + std::to_string(p.refType - 1);
      o += "}";
      if (hasProps) { o += ",\"props\":"; props_json(b, o, pv); }
      o += "}";
    } else if (hasProps) {
      o += "{\"text\":";
      hj::quote(o, p.text);
      o += ",\"props\":";
      props_json(b, o, pv);
      o += "}";
    } else {
      hj::quote(o, p.text);
    }
    return o;
  };
  int total = 0;
  for (auto& p : segs) total += p.len;
  const int n = (int)segs.size();
  const int chunkSize = b->opts.chunk_size > 0 ? b->opts.chunk_size : 10000;
  struct Chunk { int start = 0, count = 0, length = 0; };
  auto take = [&](int approx, int start) {  // getSeqLengthSegs
    Chunk c;
    c.start = start;
    while (c.length < approx && start + c.count < n) c.length += segs[start + c.count++].len;
    return c;
  };
  auto chunkText = [&](const Chunk& c, bool header) {
    std::string o = "{\"chunkStartSegmentIndex\":" + std::to_string(c.start) + ",\"chunkSegmentCount\":" + std::to_string(c.count) +
                    ",\"chunkLengthChars\":" + std::to_string(c.length) + ",\"totalLengthChars\":" + std::to_string(total) +
                    ",\"totalSegmentCount\":" + std::to_string(n) + ",\"chunkSequenceNumber\":" + std::to_string(seq) +
                    ",\"segmentTexts\":[";
    for (int k = 0; k < c.count; k++) {
      if (k) o += ',';
      o += json_of(segs[c.start + k]);
    }
    o += "]";
    if (header) {  // buildHeaderMetadataForLegacyChunk (snapshotChunks.ts:178-200); minSequenceNumber undefined
      o += ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}";
      if (c.length < total) o += ",{\"id\":\"body\"}";
      o += "],\"sequenceNumber\":" + std::to_string(seq) + ",\"totalLength\":" + std::to_string(total) +
           ",\"totalSegmentCount\":" + std::to_string(n) + "}";
    }
    return o + "}";
  };
  blobs.clear();
  const Chunk c1 = take(chunkSize, 0);
  blobs.push_back({"header", chunkText(c1, true)});
  if (c1.count < n) blobs.push_back({"body", chunkText(take(total, c1.count), false)});
  std::string tracked;
  if (catchUp.empty() && (b->opts.flags & MTB_BATCH_CATCHUP)) {
    // SharedSegmentSequence.summarizeCore (sequence.ts:676-692)
    HostDoc& dm = b->docs[i];
    drop_catch_up(dm, seq);
    tracked = "[";
    for (size_t k = 0; k < dm.catchup.size(); k++) {
      for (auto& mem : dm.catchup[k].msg.members)
        if (mem.first == u"minimumSequenceNumber") mem.second.n = seq;
      if (k) tracked += ',';
      tracked += hj::dump(dm.catchup[k].msg);
    }
    tracked += "]";
  }
  const std::string& cuText = catchUp.empty() ? tracked : catchUp;
  if (!cuText.empty()) {
    hj::Value cu = hj::parse(cuText.data(), cuText.size());
    if (cu.kind != hj::Value::kArr) raise(MTB_E_PARSE, "catch-up messages must be a JSON array");
    if (!cu.items.empty()) blobs.push_back({"catchupOps", hj::dump(cu)});
  }
  std::string tree = "{";
  uint64_t totalBytes = 0;
  for (size_t k = 0; k < blobs.size(); k++) {
    if (k) tree += ',';
    tree += "\"" + blobs[k].first + "\":{\"type\":2,\"content\":";
    hj::quote_u8(tree, blobs[k].second);
    tree += "}";
    totalBytes += utf8_byte_length(blobs[k].second);
  }
  tree += "}";
  summaryJson = "{\"summary\":{\"type\":1,\"tree\":" + tree + "},\"stats\":{\"treeNodeCount\":1,\"blobNodeCount\":" +
                std::to_string(blobs.size()) + ",\"handleNodeCount\":0,\"totalBlobSize\":" + std::to_string(totalBytes) +
                ",\"unreferencedBlobSize\":0}}";
}

char* dup(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

int mtbx_batch_create(const mtb_options* opts, uint32_t ndocs, uint32_t device_mask, mtb_dev** out) {
  if (!out || ndocs == 0) return MTB_E_ARG;
  auto* b = new mtb_dev();
  if (opts) b->opts = *opts;
  b->matrix = (b->opts.flags & MTB_BATCH_MATRIX) != 0;
  if (b->matrix && (ndocs & 1)) {
    delete b;
    return MTB_E_ARG;  // a matrix batch holds (rows, cols) pairs
  }
  b->ndocs = ndocs;
  b->docs.resize(ndocs);
  b->device = 0;
  for (int k = 0; k < 32; k++)
    if (device_mask & (1u << k)) { b->device = k; break; }
  *out = b;
  return MTB_OK;
}

void mtbx_batch_destroy(mtb_dev* b) { delete b; }
const char* mtbx_last_error(mtb_dev* b) { return b ? b->err.c_str() : "null batch"; }
void mtb_free(void* p) { free(p); }

int mtbx_doc_init(mtb_dev* b, uint32_t doc, const uint16_t* initial_text, size_t n_units, const char* observer_long_id,
                 uint32_t min_seq, uint32_t cur_seq) {
  return guarded(b, [&] {
    if (b->matrix) raise(MTB_E_ARG, "matrix batch: use mtb_matrix_init");
    HostDoc& d = docref(b, doc);
    if (d.inited || d.onDevice) raise(MTB_E_ARG, "document already initialised");
    if (!observer_long_id) raise(MTB_E_ARG, "observer long client id required");
    d.initText.assign(initial_text, initial_text + n_units);
    d.observer = observer_long_id;
    d.client(d.observer);  // startOrUpdateCollaboration: observer gets short id 0 (client.ts:1133)
    d.min0 = min_seq;
    d.cur0 = cur_seq;
    d.lastSeq = cur_seq;
    d.inited = true;
  });
}

// Client.load of a SnapshotV1 summary (client.ts:1007 -> SnapshotLoader.initialize, snapshotLoader.ts:41-257).
int mtbx_doc_load_v1(mtb_dev* b, uint32_t doc, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    try {
      load_one(b, d, blobs, nblobs, observer_long_id, nullptr);
    } catch (...) {
      if (!d.onDevice) d = HostDoc{};  // leave the slot fresh
      throw;
    }
    resolve_load_props(b, d);
  });
}

// Many documents at once: blobs are parsed and headers rebuilt on `threads` host threads (the batch's
// props table is shared under a lock).  On failure the first failing document's error is returned and
// that document (and every other failing one) is left fresh; the others are loaded.
int mtbx_docs_load_v1(mtb_dev* b, uint32_t n, const uint32_t* docs, const mtb_blob* const* blobs,
                     const uint32_t* nblobs, const char* const* observer_long_ids, uint32_t threads) {
  return guarded(b, [&] {
    if (n && (!docs || !blobs || !nblobs || !observer_long_ids)) raise(MTB_E_ARG, "null argument");
    for (uint32_t i = 0; i < n; i++) docref(b, docs[i]);
    std::vector<uint8_t> seen(b->ndocs, 0);
    for (uint32_t i = 0; i < n; i++) {
      if (seen[docs[i]]) raise(MTB_E_ARG, "document listed twice");
      seen[docs[i]] = 1;
    }
    std::mutex mu;
    std::atomic<uint32_t> next{0};
    std::vector<int> codes(n, 0);
    std::vector<std::string> msgs(n);
    auto work = [&] {
      PropsCache pc;
      pc.mu = &mu;
      for (uint32_t i = next++; i < n; i = next++) {
        HostDoc& d = b->docs[docs[i]];
        try {
          load_one(b, d, blobs[i], nblobs[i], observer_long_ids[i], &pc);
        } catch (const MtbError& e) {
          codes[i] = e.code;
          msgs[i] = e.msg;
        } catch (const hj::ParseError& e) {
          codes[i] = MTB_E_PARSE;
          msgs[i] = std::string("JSON: ") + e.what();
        } catch (const std::exception& e) {
          codes[i] = MTB_E_ARG;
          msgs[i] = e.what();
        }
        if (codes[i] && !d.onDevice) d = HostDoc{};
      }
    };
    const uint32_t nt = std::max<uint32_t>(1, std::min<uint32_t>(threads ? threads : 1, n));
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < nt; t++) ts.emplace_back(work);
    work();
    for (auto& t : ts) t.join();
    for (uint32_t i = 0; i < n; i++)
      if (!codes[i]) resolve_load_props(b, b->docs[docs[i]]);
    for (uint32_t i = 0; i < n; i++)
      if (codes[i]) raise(codes[i], "document " + std::to_string(docs[i]) + ": " + msgs[i]);
  });
}

int mtbx_add_client(mtb_dev* b, uint32_t doc, const char* long_id) {
  return guarded(b, [&] { docref(b, doc).client(long_id ? long_id : ""); });
}

int mtbx_intern_props(mtb_dev* b, const char* json, size_t len, uint32_t* id_out) {
  return guarded(b, [&] {
    hj::Value v = hj::parse(json, len);
    *id_out = b->in.props(v);
  });
}

int mtbx_apply_msg_json(mtb_dev* b, uint32_t doc, const char* json, size_t len) {
  return guarded(b, [&] {
    if (b->matrix) raise(MTB_E_ARG, "matrix batch: use mtb_matrix_apply_msg_json");
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    apply_msg(b, d, hj::parse(json, len));
  });
}

// A live client's own op (client.ts:196-247 insertSegmentLocal / removeRangeLocal): the IMergeTreeOp it
// sends, applied at the document's next replay in its own view with UnassignedSequenceNumber
// (DESIGN.md section 10).  Local rewrite annotates count as pending rewrites (pendingRewriteCount).
int mtbx_local_op_json(mtb_dev* b, uint32_t doc, const char* json, size_t len) {
  return guarded(b, [&] {
    if (b->matrix) raise(MTB_E_UNSUPPORTED, "unsupported: local ops on a matrix batch");
    if (b->opts.flags & MTB_BATCH_CATCHUP) raise(MTB_E_UNSUPPORTED, "unsupported: local ops in a catch-up batch");
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    const hj::Value op = hj::parse(json, len);
    if (op.kind != hj::Value::kObj) raise(MTB_E_PARSE, "op is not an object");
    mtb_op base{};
    base.flags = MTB_F_LOCAL;
    std::vector<mtb_op> recs;
    const size_t payloadBefore = d.payload.size();
    try {
      pack_delta(b, d, op, base, recs);
      for (const mtb_op& r : recs) {
        if (r.type != MTB_OP_INSERT && r.type != MTB_OP_REMOVE && r.type != MTB_OP_ANNOTATE)
          raise(MTB_E_ARG, "local op without an effect");
        if (r.type == MTB_OP_INSERT && !(r.flags & MTB_F_MARKER) && r.pos2 == 0) raise(MTB_E_ARG, "empty local insert");
      }
    } catch (...) {
      d.payload.resize(payloadBefore);
      throw;
    }
    b->live = true;
    d.totalPayload += d.payload.size() - payloadBefore;
    d.pending.insert(d.pending.end(), recs.begin(), recs.end());
    d.totalOps += recs.size();
    d.totalLocal += recs.size();
  });
}

// A detached client's edit before collaboration (client.ts:196-247 while not collaborating: seq
// UniversalSequenceNumber, clientId LocalClientId, refSeq 0): applied by the next replay like a sequenced op of
// client -1 at seq 0 -- every perspective it meets is the local one (everything is at seq 0), no LRU entry
// (seq 0 is not above the window), no zamboni (empty heap), no updateSeqNumbers.
int mtbx_detached_op_json(mtb_dev* b, uint32_t doc, const char* json, size_t len) {
  return guarded(b, [&] {
    if (b->matrix) raise(MTB_E_UNSUPPORTED, "unsupported: detached ops on a matrix batch");
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    if (d.totalOps != d.totalDetached || d.min0 != 0 || d.cur0 != 0 || d.loaded)
      raise(MTB_E_ARG, "detached ops come before the document's first message or local op");
    const hj::Value op = hj::parse(json, len);
    if (op.kind != hj::Value::kObj) raise(MTB_E_PARSE, "op is not an object");
    mtb_op base{};
    base.client = (uint16_t)MTB_LOCAL_CLIENT;
    std::vector<mtb_op> recs;
    const size_t payloadBefore = d.payload.size();
    try {
      pack_delta(b, d, op, base, recs);
      for (const mtb_op& r : recs)
        if (r.flags & MTB_F_RELPOS) raise(MTB_E_UNSUPPORTED, "unsupported: relative positions in a detached op");
    } catch (...) {
      d.payload.resize(payloadBefore);
      throw;
    }
    d.totalPayload += d.payload.size() - payloadBefore;
    d.pending.insert(d.pending.end(), recs.begin(), recs.end());
    d.totalOps += recs.size();
    d.totalDetached += recs.size();
  });
}

// zamboniSegments / packParent(root) as the reference's unit tests call them (an internal record; the live
// kernel, which carries every engine path, applies it)
int mtbx_maintenance(mtb_dev* b, uint32_t doc, uint32_t kind) {
  return guarded(b, [&] {
    if (b->matrix) raise(MTB_E_UNSUPPORTED, "unsupported: maintenance calls on a matrix batch");
    if (kind > 1) raise(MTB_E_ARG, "maintenance kind: 0 zamboniSegments, 1 packParent(root)");
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    mtb_op r{};
    r.type = MTB_OP_MAINT;
    r.pos1 = kind;
    d.pending.push_back(r);
    d.totalOps++;
    d.totalLocal++;
    b->live = true;
  });
}

// Client.regeneratePendingOp (client.ts:917-960): the op(s) a live client resubmits after a reconnect for
// its oldest pending op `op_json` (one pending segment group per member op).  Runs as a REGEN record on
// the GPU (normalizeSegmentsOnRebase, positions at the groups' localSeq, new pending groups); the ops are
// composed here from the kernel's entries as the reference's opBuilder writes them.
int mtbx_regenerate_pending_op(mtb_dev* b, uint32_t doc, const char* json, size_t len, char** out, size_t* out_len) {
  return guarded(b, [&] {
    if (!out) raise(MTB_E_ARG, "null output");
    if (b->matrix) raise(MTB_E_UNSUPPORTED, "unsupported: local ops on a matrix batch");
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    const hj::Value op = hj::parse(json, len);
    if (op.kind != hj::Value::kObj) raise(MTB_E_PARSE, "op is not an object");
    std::vector<const hj::Value*> members;
    const hj::Value* t = member(op, u"type");
    if (t && t->kind == hj::Value::kNum && (int)t->n == 3) {
      const hj::Value* ops = member(op, u"ops");
      if (ops && ops->kind == hj::Value::kArr)
        for (auto& m : ops->items) members.push_back(&m);
    } else {
      members.push_back(&op);
    }
    for (const hj::Value* m : members) {
      const hj::Value* mt = member(*m, u"type");
      const int ty = mt && mt->kind == hj::Value::kNum ? (int)mt->n : -1;
      if (ty < 0 || ty > 2) raise(MTB_E_ARG, "Invalid op type");
    }
    std::vector<std::string> ops;
    if (!members.empty()) {
      // flush the batch first, so that an error of another document (reported by the replay that hits it)
      // surfaces here before anything is regenerated; the REGEN record then runs alone
      bool pendingWork = false;
      for (uint32_t i = 0; i < b->ndocs && !pendingWork; i++) pendingWork = !b->docs[i].pending.empty();
      if (pendingWork || !b->devInit) {
        mtb_stats st0{};
        replay(b, &st0);
      }
      if (b->hst[doc].err) raise(derr_code(b->hst[doc].err), derr_text(b->hst[doc].err));
      mtb_op r{};
      r.type = MTB_OP_REGEN;
      r.pos1 = (uint32_t)members.size();
      d.pending.push_back(r);
      d.totalOps++;
      d.totalLocal += 4 * members.size();
      b->live = true;
      const uint32_t k = (uint32_t)d.pending.size() - 1;  // the record's index in this replay
      mtb_stats st{};
      replay(b, &st);
      const DocState& s = b->hst[doc];
      if (s.err) raise(derr_code(s.err), derr_text(s.err));
      std::vector<uint32_t> ent(4ull * s.delta_used);
      if (s.delta_used)
        HIPCHK(hipMemcpy(ent.data(), b->dDelta.p + 4ull * s.delta_base, ent.size() * 4, hipMemcpyDeviceToHost));
      download_doc(b, doc);
      for (uint32_t e = 0; e < s.delta_used; e++) {
        if (ent[4 * e] != k) continue;
        const uint32_t ty = ent[4 * e + 1] & 0xFF, g = ent[4 * e + 1] >> 8, sid = ent[4 * e + 2];
        const int pos = (int)ent[4 * e + 3];
        if (g >= members.size() || sid >= d.segs.size()) raise(MTB_E_HIP, "regenerate: bad kernel entry");
        const Seg& sg = d.segs[sid];
        const hj::Value& reset = *members[g];
        std::string o = "{\"pos1\":" + std::to_string(pos);
        if (ty == MTB_OP_ANNOTATE) {  // createAnnotateRangeOp(start, end, props, combiningOp) (opBuilder.ts:52-65)
          const hj::Value* comb = member(reset, u"combiningOp");
          if (comb && comb->kind != hj::Value::kUndef) o = "{\"combiningOp\":" + hj::dump(*comb) + ",\"pos1\":" + std::to_string(pos);
        }
        if (ty == MTB_OP_INSERT) {  // createInsertSegmentOp(pos, segment): segment.toJSONObject()
          const hj::Value* rseg = member(reset, u"seg");
          const hj::Value* rprops = rseg && rseg->kind == hj::Value::kObj ? member(*rseg, u"props") : nullptr;
          std::string pj;
          bool hasProps = false;
          if (rprops && rprops->kind != hj::Value::kUndef) {  // segment.clone() with resetOp.seg.props
            hasProps = rprops->kind == hj::Value::kObj;
            if (hasProps) pj = hj::dump(*rprops);
          } else if (sg.props) {
            hasProps = true;
            props_json(b, pj, props_of(b, d, sg.props));
          }
          o += ",\"seg\":";
          if (is_marker(sg)) {
            const uint32_t rt = sg.text & ~MTB_MARKER;
            o += "{\"marker\":{";
            if (rt) o += "\"refType\":" + std::to_string(rt - 1);
            o += "}";
            if (hasProps) o += ",\"props\":" + pj;
            o += "}";
          } else {
            const U16 text(reinterpret_cast<const char16_t*>(d.text.data() + sg.text), (size_t)sg.len);
            if (hasProps) {
              o += "{\"text\":";
              hj::quote(o, text);
              o += ",\"props\":" + pj + "}";
            } else {
              hj::quote(o, text);
            }
          }
          o += ",\"type\":0}";
        } else {
          o += ",\"pos2\":" + std::to_string(pos + sg.len);
          if (ty == MTB_OP_ANNOTATE) {
            const hj::Value* pr = member(reset, u"props");
            if (pr) o += ",\"props\":" + hj::dump(*pr);
            o += ",\"type\":2}";
          } else {
            o += ",\"type\":1}";
          }
        }
        ops.push_back(std::move(o));
      }
    }
    std::string res;
    if (ops.size() == 1) {
      res = ops[0];
    } else {  // createGroupOp(...ops)
      res = "{\"ops\":[";
      for (size_t i = 0; i < ops.size(); i++) res += (i ? "," : "") + ops[i];
      res += "],\"type\":3}";
    }
    *out = (char*)malloc(res.size() + 1);
    memcpy(*out, res.data(), res.size());
    (*out)[res.size()] = 0;
    if (out_len) *out_len = res.size();
  });
}

uint32_t intern_cell_value(mtb_dev* b, const std::string& json) {
  auto [it, fresh] = b->cellValIds.try_emplace(json, (uint32_t)b->cellVals.size());
  if (fresh) b->cellVals.push_back(json);
  return it->second;
}

// SharedMatrix.processCore (matrix.ts:636-697): a vector op goes to its PermutationVector's applyMsg
// (with that vector's updateSeqNumbers); a remote setCell becomes a SETCELL record in both vectors
// (adjusted, exchanged and allocated on the GPU); a local setCell is an ack with no vector effect.
int mtbx_matrix_apply_msg_json(mtb_dev* b, uint32_t matrix, const char* json, size_t len) {
  return guarded(b, [&] {
    if (!b->matrix) raise(MTB_E_ARG, "not a matrix batch (MTB_BATCH_MATRIX)");
    if (matrix >= b->ndocs / 2) raise(MTB_E_ARG, "matrix index out of range");
    HostDoc& R = b->docs[2 * matrix];
    HostDoc& C = b->docs[2 * matrix + 1];
    if (!R.inited || !C.inited) raise(MTB_E_ARG, "mtb_matrix_init must be called first");
    hj::Value msg = hj::parse(json, len);
    if (msg.kind != hj::Value::kObj) raise(MTB_E_PARSE, "message is not an object");
    const hj::Value* type = member(msg, u"type");
    const hj::Value* contents = member(msg, u"contents");
    if (!type || type->kind != hj::Value::kStr || type->s != u"op") return;  // not routed to processCore
    if (!contents || contents->kind != hj::Value::kObj) raise(MTB_E_PARSE, "op message without contents");
    const hj::Value* target = member(*contents, u"target");
    if (target && target->kind == hj::Value::kStr && (target->s == u"rows" || target->s == u"cols")) {
      apply_msg(b, target->s == u"rows" ? R : C, msg);
      return;
    }
    const hj::Value* t = member(*contents, u"type");
    if (!t || t->kind != hj::Value::kNum || (int)t->n != 2)
      raise(MTB_E_ASSERT, "0x021 SharedMatrix message contents have unexpected type!");
    const hj::Value* cid = member(msg, u"clientId");
    if (!cid || cid->kind != hj::Value::kStr) raise(MTB_E_UNSUPPORTED, "unsupported: message without a string clientId");
    const std::string longId = hj::to_utf8(cid->s.data(), cid->s.size());
    if (longId == R.observer) return;  // ack of a local set (matrix.ts:660-667)
    mtb_op base{};
    base.type = MTB_OP_SETCELL;
    base.seq = u32field(msg, u"sequenceNumber", "sequenceNumber");
    base.ref_seq = u32field(msg, u"referenceSequenceNumber", "referenceSequenceNumber");
    base.msn = u32field(msg, u"minimumSequenceNumber", "minimumSequenceNumber");
    const uint32_t row = u32field(*contents, u"row", "row"), col = u32field(*contents, u"col", "col");
    // the cell value (opaque JSON, matrix.ts:684), interned batch-wide; absent = undefined (id 0)
    if (const hj::Value* v = member(*contents, u"value")) base.props = intern_cell_value(b, hj::dump(*v));
    mtb_op r = base, c = base;
    r.client = R.client(longId);  // getOrAddShortClientId in adjustPosition (client.ts:1070)
    r.pos1 = row;
    r.pos2 = R.client(R.observer);
    c.client = C.client(longId);
    c.pos1 = col;
    c.pos2 = C.client(C.observer);
    R.pending.push_back(r);
    C.pending.push_back(c);
    for (HostDoc* d : {&R, &C}) {
      d->totalOps++;
      d->totalSetcell++;
    }
  });
}

// SharedMatrix observers (rows = document 2m, cols = 2m + 1) in a MTB_BATCH_MATRIX batch:
// startOrUpdateCollaboration on both PermutationVectors (matrix.ts:102-118 construct them empty).
int mtbx_matrix_init(mtb_dev* b, uint32_t matrix, const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq) {
  return guarded(b, [&] {
    if (!b->matrix) raise(MTB_E_ARG, "not a matrix batch (MTB_BATCH_MATRIX)");
    if (matrix >= b->ndocs / 2) raise(MTB_E_ARG, "matrix index out of range");
    if (!observer_long_id) raise(MTB_E_ARG, "observer long client id required");
    for (int k = 0; k < 2; k++) {
      HostDoc& d = b->docs[2 * matrix + k];
      if (d.inited || d.onDevice) raise(MTB_E_ARG, "matrix already initialised");
    }
    for (int k = 0; k < 2; k++) {
      HostDoc& d = b->docs[2 * matrix + k];
      d.perm = true;
      d.observer = observer_long_id;
      d.client(d.observer);
      d.min0 = min_seq;
      d.cur0 = cur_seq;
      d.lastSeq = cur_seq;
      d.inited = true;
    }
  });
}

int mtbx_append_ops(mtb_dev* b, uint32_t doc, const mtb_op* ops, uint32_t n, const uint16_t* payload, size_t payload_len) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (!d.inited) raise(MTB_E_ARG, "mtb_doc_init must be called first");
    if (n && !ops) raise(MTB_E_ARG, "null records");
    if (payload_len && !payload) raise(MTB_E_ARG, "null payload");
    // validate every record first, then commit records, payload and totals together (all or nothing)
    const uint32_t base = (uint32_t)d.payload.size();
    std::vector<mtb_op> staged;
    staged.reserve(n);
    uint64_t setcells = 0;
    for (uint32_t k = 0; k < n; k++) {
      mtb_op o = ops[k];
      if (o.type > MTB_OP_ACK && !(b->matrix && o.type == MTB_OP_SETCELL)) raise(MTB_E_ARG, "bad record type");
      if (d.perm && o.type == MTB_OP_INSERT && !(o.flags & MTB_F_PERMSEG)) raise(MTB_E_ARG, "PermutationVector insert without MTB_F_PERMSEG");
      if (!d.perm && (o.flags & MTB_F_PERMSEG)) raise(MTB_E_ARG, "MTB_F_PERMSEG outside a matrix batch");
      if (o.flags & (MTB_F_LOCAL | MTB_F_LDLAST)) raise(MTB_E_ARG, "record flags 0x10 / 0x20 are internal (local ops: mtb_local_op_json)");
      if (o.type == MTB_OP_SETCELL) {
        if (o.flags & MTB_F_LAST) raise(MTB_E_ARG, "SETCELL records never carry MTB_F_LAST");
        if (o.props >= b->cellVals.size()) raise(MTB_E_ARG, "SETCELL value id out of range (mtb_matrix_intern_value)");
        setcells++;
      }
      if (o.type == MTB_OP_INSERT && !(o.flags & (MTB_F_MARKER | MTB_F_PERMSEG))) {
        if ((uint64_t)o.payload + o.pos2 > payload_len) raise(MTB_E_ARG, "record payload out of range");
        o.payload += base;
      }
      if ((o.type == MTB_OP_INSERT || o.type == MTB_OP_ANNOTATE) && o.props >= b->in.pidx.size() / 2)
        raise(MTB_E_ARG, "record props id out of range");
      if (o.type == MTB_OP_INSERT && (o.flags & MTB_F_MARKER)) o.payload = 0;  // set below (marker id ordinal)
      if (o.client >= d.longIds.size() && o.type != MTB_OP_NOOP)
        raise(MTB_E_ARG, "record client id not registered (mtb_add_client)");
      staged.push_back(o);
    }
    for (mtb_op& o : staged) {  // idToSegment keys of markers / annotates setting markerId (as the JSON path)
      if (o.type == MTB_OP_INSERT && (o.flags & MTB_F_MARKER)) {
        if (const std::string* js = props_marker_json(b->in, o.props, false)) {
          hj::Value mp;
          mp.kind = hj::Value::kObj;
          mp.members.push_back({U16(u"markerId"), hj::parse(js->data(), js->size())});
          o.payload = marker_ord(d, &mp);
        }
      } else if (o.type == MTB_OP_ANNOTATE) {
        o.payload = 0;
        if (const std::string* js = props_marker_json(b->in, o.props, true)) {  // (the op's own values)
          const hj::Value v = hj::parse(js->data(), js->size());
          d.markerIdAnnot = true;
          o.payload = annot_marker_test(&v);
        }
        // combiningOps: the op-props values the device applies (records carry no defaultValue / minValue)
        if ((o.flags & MTB_F_COMB) == MTB_F_CONSENSUS) o.props = b->in.consensus_props(o.props, nullptr, (int)o.seq);
        if ((o.flags & MTB_F_COMB) == MTB_F_INCR) {
          b->in.nan();
          o.props = b->in.incr_props(o.props, nullptr, nullptr, &d.vals);
        }
      }
      if (o.type == MTB_OP_INSERT || o.type == MTB_OP_ANNOTATE) d.vals.propsSeen.push_back(o.props);
    }
    d.payload.insert(d.payload.end(), payload, payload + payload_len);
    d.totalPayload += payload_len;
    d.pending.insert(d.pending.end(), staged.begin(), staged.end());
    d.totalSetcell += setcells;
    d.totalOps += n;
  });
}

int mtbx_replay(mtb_dev* b, mtb_stats* out) {
  return guarded(b, [&] { replay(b, out); });
}

int mtbx_rewind(mtb_dev* b) {
  return guarded(b, [&] {
    if (!b->haveRewind) raise(MTB_E_ARG, "nothing to rewind: replay the batch first");
    for (auto& d : b->docs)
      if (!d.pending.empty()) raise(MTB_E_ARG, "rewind with pending (unreplayed) ops");
    HIPCHK(mtb_launch_rewind(b->stream, b->ndocs, b->dDocs.p, b->dPristine.p, b->dSegs.p, b->dPSeg.p, b->dBlks.p, b->dPBlk.p));
    void* pools[5] = {b->dBlks.p, b->dSegs.p, b->dLists.p, b->dAux.p, b->dText.p};
    for (int k = 0; k < 5; k++) move_words(b, b->dPX.p, pools[k], b->pxRestore[k]);
    HIPCHK(hipStreamSynchronize(b->stream));
    b->hst = b->hPristine;
    for (auto& d : b->docs) d.cached = false;
  });
}

// Replay the records already resident on the device (after mtb_rewind); no host->device traffic.
int mtbx_get_launch_info(mtb_dev* b, mtb_launch_info* out) {
  return guarded(b, [&] {
    if (!out) raise(MTB_E_ARG, "null output");
    *out = b->launch;
  });
}

int mtbx_replay_resident(mtb_dev* b, mtb_stats* out, uint32_t flags) {
  return guarded(b, [&] {
    if (!b->haveRewind) raise(MTB_E_ARG, "no resident records");
    const Tables t = make_tables(b);
    HIPCHK(hipEventRecord(b->ev0, b->stream));
    if (b->residentLoad)
      HIPCHK(mtb_launch_load(b->stream, b->ndocs, b->dDocs.p, b->dOps.p, b->dSegs.p, b->dBlks.p, b->dLists.p, b->dText.p,
                             b->dHeap.p, b->dAux.p, b->dFree.p, t, b->matrix ? 1 : 0));
    launch_main(b, t);
    HIPCHK(hipEventRecord(b->ev1, b->stream));
    sched_readback(b);
    HIPCHK(hipMemcpyAsync(b->hst.data(), b->dDocs.p, b->ndocs * sizeof(DocState), hipMemcpyDeviceToHost, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, b->ev0, b->ev1));
    sched_result(b);
    mtb_stats st{};
    st.kernel_ms = ms;
    uint32_t short_docs = 0;
    for (uint32_t i = 0; i < b->ndocs; i++) {
      DocState& s = b->hst[i];
      b->docs[i].cached = false;
      if (!s.err && s.op_next != s.n_ops) {  // the same invariant as replay(): every record ran
        s.err = DERR_SCHED;
        short_docs++;
      }
      st.docs++;
      st.ops_applied += s.ops_applied;
      st.bytes_alg += 32ull * s.ops_applied + s.text_bytes + 24ull * s.n_mod;
      if (s.err) st.errors++;
    }
    if (flags & MTB_REPLAY_NO_DIGEST)
      b->digests.clear();  // (mtb_refresh_digests)
    else
      run_digest(b, st);
    if (out) *out = st;
    if (short_docs)
      raise(MTB_E_INTERNAL, std::to_string(short_docs) + " document(s) did not run all of their records");
  });
}

int mtbx_get_text(mtb_dev* b, uint32_t doc, uint16_t* buf, size_t cap, size_t* len_out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    download_doc(b, doc);
    std::vector<FlatSeg> fl;
    flatten(d, b->hst[doc].root, fl, false);
    size_t n = 0;
    for (auto& f : fl) {
      const Seg& g = d.segs[f.id];
      if (seg_removed(g) || is_marker(g)) continue;  // MergeTreeTextHelper.gatherText on visible text segments
      if (buf && n + (size_t)g.len <= cap) memcpy(buf + n, d.text.data() + g.text, (size_t)g.len * 2);
      n += (size_t)g.len;
    }
    if (len_out) *len_out = n;
    if (buf && n > cap) raise(MTB_E_ARG, "buffer too small");
  });
}

// Test hook (include/mtb_testing.h): overwrite the child id in the root block's last slot with `value` and
// return the old id, so tests can give the device walks a tree they must refuse (an engine fault, never input).
int mtbx_test_set_root_child(mtb_dev* b, uint32_t doc, uint32_t value, uint32_t* old_out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (!d.onDevice || !b->devInit || doc >= b->hst.size()) raise(MTB_E_ARG, "document has not been replayed");
    const DocState& s = b->hst[doc];
    FBlk r;
    FBlk* dp = b->dBlks.p + s.blk_base + s.root;
    HIPCHK(hipMemcpy(&r, dp, sizeof r, hipMemcpyDeviceToHost));
    if (r.count == 0 || r.count > MTB_MAXCH) raise(MTB_E_ARG, "the root block has no child slot to change");
    if (old_out) *old_out = r.f[F_ID][r.count - 1];
    r.f[F_ID][r.count - 1] = value == 0xFFFFFFFEu ? s.root : value;
    HIPCHK(hipMemcpy(dp, &r, sizeof r, hipMemcpyHostToDevice));
    d.cached = false;
  });
}

int mtbx_get_length(mtb_dev* b, uint32_t doc, uint32_t* len_out) {
  return guarded(b, [&] {
    docref(b, doc);
    download_doc(b, doc);
    *len_out = (uint32_t)b->docs[doc].blks[b->hst[doc].root].len;
  });
}

int mtbx_get_seq(mtb_dev* b, uint32_t doc, uint32_t* cur_seq, uint32_t* min_seq) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (d.onDevice) {
      if (cur_seq) *cur_seq = (uint32_t)b->hst[doc].cur_seq;
      if (min_seq) *min_seq = (uint32_t)b->hst[doc].min_seq;
    } else {
      if (cur_seq) *cur_seq = d.cur0;
      if (min_seq) *min_seq = d.min0;
    }
  });
}

int mtbx_dump_segments(mtb_dev* b, uint32_t doc, char** out, size_t* out_len) {
  return guarded(b, [&] {
    docref(b, doc);
    std::string s = dump_doc(b, doc);
    *out = dup(s);
    if (out_len) *out_len = s.size();
  });
}

int mtbx_refresh_digests(mtb_dev* b, mtb_stats* out) {
  return guarded(b, [&] {
    if (!b->devInit) raise(MTB_E_ARG, "no replay yet");
    mtb_stats st{};
    run_digest(b, st);
    if (out) *out = st;
  });
}

int mtbx_doc_digests(mtb_dev* b, uint32_t first, uint32_t n, uint64_t* out) {
  return guarded(b, [&] {
    if (!out && n) raise(MTB_E_ARG, "null output");
    if ((uint64_t)first + n > b->ndocs) raise(MTB_E_ARG, "document range out of bounds");
    if (b->digests.size() != 3ull * b->ndocs) raise(MTB_E_ARG, "no digests: no replay yet, or one without them (mtb_refresh_digests)");
    for (uint32_t k = 0; k < n; k++) out[k] = b->digests[3ull * (first + k)];
  });
}

int mtbx_doc_checksum(mtb_dev* b, uint32_t doc, uint64_t* out) {
  return guarded(b, [&] {
    docref(b, doc);
    *out = fnv(dump_doc(b, doc));
  });
}

namespace {
void fill_blob_list(const std::vector<std::pair<std::string, std::string>>& blobs, const std::string& summary, mtb_blob_list* out) {
  out->count = (uint32_t)blobs.size();
  out->blobs = (mtb_blob*)calloc(blobs.size() ? blobs.size() : 1, sizeof(mtb_blob));
  for (size_t k = 0; k < blobs.size(); k++) {
    out->blobs[k].path = dup(blobs[k].first);
    out->blobs[k].content = dup(blobs[k].second);
    out->blobs[k].content_len = blobs[k].second.size();
  }
  out->summary_json = dup(summary);
  out->summary_json_len = summary.size();
}
void summary_catch_up(mtb_dev* b, HostDoc& d, int64_t msn, int64_t seq) {
  if (msn >= 0 && seq >= 0) {  // Client.summarize: updateSeqNumbers(deltaManager.MSN, lastSequenceNumber)
    mtb_op r{};
    r.type = MTB_OP_NOOP;
    r.flags = MTB_F_LAST;
    r.seq = (uint32_t)seq;
    r.msn = (uint32_t)msn;
    d.pending.push_back(r);
    d.totalOps++;
    replay(b, nullptr);
  }
}
}  // namespace

// Client.summarize without newMergeTreeSnapshotFormat (client.ts:999-1003)
int mtbx_summarize_legacy(mtb_dev* b, uint32_t doc, int64_t msn, int64_t seq, const char* catchup_json, size_t catchup_len,
                         mtb_blob_list* out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (!out) raise(MTB_E_ARG, "null output");
    summary_catch_up(b, d, msn, seq);
    std::vector<std::pair<std::string, std::string>> blobs;
    std::string summary;
    summarize_legacy(b, doc, catchup_json ? std::string(catchup_json, catchup_len) : std::string(), blobs, summary);
    fill_blob_list(blobs, summary, out);
  });
}

int mtbx_summarize_v1(mtb_dev* b, uint32_t doc, int64_t msn, int64_t seq, mtb_blob_list* out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (msn >= 0 && seq >= 0) {  // Client.summarize: updateSeqNumbers(deltaManager.MSN, lastSequenceNumber)
      mtb_op r{};
      r.type = MTB_OP_NOOP;
      r.flags = MTB_F_LAST;
      r.seq = (uint32_t)seq;
      r.msn = (uint32_t)msn;
      d.pending.push_back(r);
      d.totalOps++;
      replay(b, nullptr);
    }
    std::vector<std::pair<std::string, std::string>> blobs;
    std::string summary;
    summarize_any(b, doc, blobs, summary);
    out->count = (uint32_t)blobs.size();
    out->blobs = (mtb_blob*)calloc(blobs.size(), sizeof(mtb_blob));
    for (size_t k = 0; k < blobs.size(); k++) {
      out->blobs[k].path = dup(blobs[k].first);
      out->blobs[k].content = dup(blobs[k].second);
      out->blobs[k].content_len = blobs[k].second.size();
    }
    out->summary_json = dup(summary);
    out->summary_json_len = summary.size();
  });
}

// Client.summarize (SnapshotV1) of many documents: one replay for the optional updateSeqNumbers, one
// bulk download of every listed document, and the summaries serialized on `threads` host threads.
int mtbx_summarize_v1_many(mtb_dev* b, uint32_t n, const uint32_t* docs, int64_t msn, int64_t seq, uint32_t threads,
                          mtb_blob_list* out) {
  return guarded(b, [&] {
    if (n && (!docs || !out)) raise(MTB_E_ARG, "null argument");
    std::vector<uint32_t> list(docs, docs + n);
    for (uint32_t i : list) docref(b, i);
    if (msn >= 0 && seq >= 0) {  // updateSeqNumbers(deltaManager.MSN, lastSequenceNumber) (client.ts:979)
      for (uint32_t i : list) {
        mtb_op r{};
        r.type = MTB_OP_NOOP;
        r.flags = MTB_F_LAST;
        r.seq = (uint32_t)seq;
        r.msn = (uint32_t)msn;
        b->docs[i].pending.push_back(r);
        b->docs[i].totalOps++;
      }
      replay(b, nullptr);
    }
    PhaseClock pc;
    // SharedString documents: extractSync on the device (mtb_extract_v1_kernel), only its output comes back;
    // PermutationVectors and failed documents take the host path over the downloaded tree
    std::vector<uint32_t> ids(list);
    Extracted ex;
    // MTB_SUMMARY_PIECES=P > 1: the outputs come back in P pieces while the serializer threads start on the
    // first ones.  Off by default: on the 16-CPU share of a GPU box the runtime's pageable staging copies compete
    // with the serializer threads and the overlap gained nothing (profiles/r04/summary/: 1 / 8 / 32 pieces
    // 0.216-0.222 / 0.226-0.244 / 0.210-0.216 s for 10,000 summaries)
    uint32_t pieces = 1;
    if (const char* e = getenv("MTB_SUMMARY_PIECES")) pieces = (uint32_t)std::max(1, atoi(e));
    extract_docs(b, ids, ex, pieces);
    pc.mark("extract");
    std::vector<uint32_t> fast, slow;
    for (uint32_t k = 0; k < n; k++) (ex.ok[k] ? fast : slow).push_back(k);
    const uint32_t nf = (uint32_t)fast.size();
    (void)nf;
    if (!slow.empty()) {
      std::vector<uint32_t> sl;
      for (uint32_t k : slow) sl.push_back(list[k]);
      download_docs(b, sl);
    }
    std::vector<std::string> errs(n);
    std::atomic<uint32_t> next{0};
    auto work = [&] {
      for (uint32_t k = next++; k < n; k = next++) {
        try {
          std::vector<std::pair<std::string, std::string>> blobs;
          std::string summary;
          if (ex.ok[k]) {
            if (!ex.wait_doc(k)) raise(MTB_E_HIP, "SnapshotV1 extraction download failed");
            summarize_items(b, list[k], ex.items + ex.off[3 * k], ex.cnt[3 * k], ex.text + ex.off[3 * k + 1],
                            ex.words + ex.off[3 * k + 2], blobs, summary);
          } else {
            summarize(b, list[k], blobs, summary);
          }
          fill_blob_list(blobs, summary, &out[k]);
        } catch (const MtbError& e) {
          errs[k] = e.msg;
          out[k] = mtb_blob_list{};
        } catch (const std::exception& e) {
          errs[k] = e.what();
          out[k] = mtb_blob_list{};
        }
      }
    };
    const uint32_t nt = std::max<uint32_t>(1, std::min<uint32_t>(threads ? threads : 1, n));
    std::vector<std::thread> ts;
    // on any exit (a thread that cannot start included): fail the pieces nobody marked, so no worker waits
    // for them, and join every worker before the vector is destroyed
    struct JoinGuard {
      Extracted& ex;
      std::vector<std::thread>& ts;
      ~JoinGuard() {
        for (uint32_t q = 0; q < ex.npieces; q++)
          if (ex.ready[q].load(std::memory_order_acquire) == 0) ex.mark(q, -1);
        for (auto& t : ts)
          if (t.joinable()) t.join();
      }
    } guard{ex, ts};
    for (uint32_t t = 1; t < nt; t++) ts.emplace_back(work);
    std::string copyErr;
    for (uint32_t p = 0; p < ex.npieces; p++) {  // (this thread downloads, then serializes too)
      try {
        copy_piece(b, ex, p);
        ex.mark(p, 1);
      } catch (const MtbError& e) {
        copyErr = e.msg;
        for (uint32_t q = p; q < ex.npieces; q++) ex.mark(q, -1);
        break;
      } catch (...) {  // (bad_alloc, system_error): no worker may wait for a piece that never comes
        copyErr = "SnapshotV1 extraction download failed";
        for (uint32_t q = p; q < ex.npieces; q++) ex.mark(q, -1);
        break;
      }
    }
    work();
    for (auto& t : ts) t.join();
    pc.mark("serialize");
    if (!copyErr.empty()) raise(MTB_E_HIP, copyErr);
    for (uint32_t k = 0; k < n; k++)
      if (!errs[k].empty()) raise(MTB_E_ARG, "document " + std::to_string(list[k]) + ": " + errs[k]);
  });
}

int mtbx_export_pending(mtb_dev* b, uint32_t doc, mtb_op* ops, uint32_t cap, uint32_t* n_out, uint16_t* payload,
                       size_t pcap, size_t* plen_out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (n_out) *n_out = (uint32_t)d.pending.size();
    if (plen_out) *plen_out = d.payload.size();
    if (ops) {
      if (cap < d.pending.size()) raise(MTB_E_ARG, "record buffer too small");
      memcpy(ops, d.pending.data(), d.pending.size() * sizeof(mtb_op));
    }
    if (payload) {
      if (pcap < d.payload.size()) raise(MTB_E_ARG, "payload buffer too small");
      memcpy(payload, d.payload.data(), d.payload.size() * 2);
    }
  });
}

int mtbx_props_json(mtb_dev* b, uint32_t id, char* buf, size_t cap, size_t* len_out) {
  return guarded(b, [&] {
    for (auto& kv : b->in.propsByJson) {
      if (kv.second == id) {
        if (len_out) *len_out = kv.first.size();
        if (buf) {
          if (cap < kv.first.size() + 1) raise(MTB_E_ARG, "buffer too small");
          memcpy(buf, kv.first.c_str(), kv.first.size() + 1);
        }
        return;
      }
    }
    raise(MTB_E_ARG, "unknown props id");
  });
}

int mtbx_client_long_id(mtb_dev* b, uint32_t doc, uint32_t short_id, char* buf, size_t cap, size_t* len_out) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (short_id >= d.longIds.size()) raise(MTB_E_ARG, "unknown short client id");
    const std::string& s = d.longIds[d.ref_id((int)short_id)];
    if (len_out) *len_out = s.size();
    if (buf) {
      if (cap < s.size() + 1) raise(MTB_E_ARG, "buffer too small");
      memcpy(buf, s.c_str(), s.size() + 1);
    }
  });
}

// FNV-1a 64 over a blob list: for each blob its path, a 0 byte, its content, a 0 byte; then the summary
// JSON (the same definition as the checker's summary hash, oracle/loggen.cpp)
int mtb_blob_list_fnv(const mtb_blob_list* l, uint64_t* out) {
  if (!l || !out) return MTB_E_ARG;
  uint64_t h = 1469598103934665603ull;
  auto add = [&](const char* p, size_t n) {
    for (size_t i = 0; i < n; i++) {
      h ^= (unsigned char)p[i];
      h *= 1099511628211ull;
    }
  };
  const char z = 0;
  for (uint32_t k = 0; k < l->count; k++) {
    add(l->blobs[k].path, strlen(l->blobs[k].path));
    add(&z, 1);
    add(l->blobs[k].content, l->blobs[k].content_len);
    add(&z, 1);
  }
  if (l->summary_json) add(l->summary_json, l->summary_json_len);
  *out = h;
  return MTB_OK;
}

void mtb_blob_list_free(mtb_blob_list* l) {
  if (!l) return;
  for (uint32_t k = 0; k < l->count; k++) {
    free((void*)l->blobs[k].path);
    free((void*)l->blobs[k].content);
  }
  free(l->blobs);
  free((void*)l->summary_json);
  l->blobs = nullptr;
  l->summary_json = nullptr;
  l->count = 0;
}

}  // extern "C"

// ------------------------------------------------------------------ SharedMatrix cells and summary
namespace {
// PermutationVector.getMaybeHandle (permutationvector.ts:200-207, handlecache.ts): the handle stored
// at local position `pos` of vector document i (start + offset; HandleUnallocated when none).
uint32_t vector_handle_at(mtb_dev* b, uint32_t i, uint32_t pos) {
  download_doc(b, i);
  const HostDoc& d = b->docs[i];
  uint32_t p = pos, found = MTB_NONE;
  auto visit = [&](auto& self, uint32_t bi) -> bool {  // segments in order; true once pos is reached
    const Blk& B = d.blks[bi];
    for (int k = 0; k < B.count; k++) {
      const uint32_t c = B.child[k];
      if (!(c & MTB_LEAF)) {
        if (self(self, c)) return true;
        continue;
      }
      const Seg& g = d.segs[c & ~MTB_LEAF];
      const uint32_t len = g.rseq < 0 ? (uint32_t)g.len : 0u;  // local view: removed segments are empty
      if (p < len) {
        found = g.text == MTB_HANDLE_UNALLOC ? MTB_HANDLE_UNALLOC : g.text + p;
        return true;
      }
      p -= len;
    }
    return false;
  };
  if (!visit(visit, b->hst[i].root)) raise(MTB_E_ARG, "0x027 position out of range");  // ensureRange (matrix.ts:189)
  return found;
}
}  // namespace

int mtbx_matrix_intern_value(mtb_dev* b, const char* json, size_t len, uint32_t* id_out) {
  return guarded(b, [&] {
    if (!json || !id_out) raise(MTB_E_ARG, "null argument");
    hj::Value v = hj::parse(json, len);
    *id_out = intern_cell_value(b, hj::dump(v));
  });
}

int mtbx_matrix_get_cell(mtb_dev* b, uint32_t matrix, uint32_t row, uint32_t col, char* buf, size_t cap, size_t* len_out) {
  return guarded(b, [&] {
    if (!b->matrix) raise(MTB_E_ARG, "not a matrix batch (MTB_BATCH_MATRIX)");
    if (matrix >= b->ndocs / 2) raise(MTB_E_ARG, "matrix index out of range");
    if (!b->docs[2 * matrix].inited) raise(MTB_E_ARG, "mtb_matrix_init must be called first");
    if (!b->devInit || !b->docs[2 * matrix].onDevice || !b->docs[2 * matrix + 1].onDevice)
      raise(MTB_E_ARG, "matrix has not been replayed");
    if (b->hst[2 * matrix].err) raise(derr_code(b->hst[2 * matrix].err), derr_text(b->hst[2 * matrix].err));
    std::string v;
    const uint32_t rh = vector_handle_at(b, 2 * matrix, row);
    const uint32_t ch = vector_handle_at(b, 2 * matrix + 1, col);  // bounds-checked even for an unallocated row
    const HostDoc& R = b->docs[2 * matrix];
    if (rh != MTB_HANDLE_UNALLOC && ch != MTB_HANDLE_UNALLOC && R.cells) {
      auto it = R.cells->cells.find(((uint64_t)rh << 32) | ch);
      if (it != R.cells->cells.end() && it->second) v = b->cellVals[it->second];
    }
    if (len_out) *len_out = v.size();
    if (buf && cap) snprintf(buf, cap, "%s", v.c_str());
  });
}

// SharedMatrix.summarizeCore (matrix.ts:449-463) through SummaryTreeBuilder (summaryUtils.ts:138-198):
// addWithStats(rows), addWithStats(cols) (PermutationVector.summarize), addBlob(cells)
int mtbx_matrix_summarize(mtb_dev* b, uint32_t matrix, mtb_blob_list* out) {
  return guarded(b, [&] {
    if (!b->matrix) raise(MTB_E_ARG, "not a matrix batch (MTB_BATCH_MATRIX)");
    if (matrix >= b->ndocs / 2) raise(MTB_E_ARG, "matrix index out of range");
    if (!out) raise(MTB_E_ARG, "null output");
    std::vector<std::pair<std::string, std::string>> all, vb[2];
    std::string vs[2];
    for (int v = 0; v < 2; v++) summarize(b, 2 * matrix + v, vb[v], vs[v]);
    const HostDoc& R = b->docs[2 * matrix];
    const std::string cells = "[" + (R.cells ? R.cells->snapshot_json(b->cellVals) : std::string("[null]")) + ",[null]]";
    for (int v = 0; v < 2; v++)
      for (auto& x : vb[v]) all.push_back({(v ? "cols/" : "rows/") + x.first, x.second});
    all.push_back({"cells", cells});
    uint64_t st[3] = {1, 1, utf8_byte_length(cells)};  // treeNodeCount, blobNodeCount, totalBlobSize
    std::string tree = "{";
    for (int v = 0; v < 2; v++) {
      const hj::Value sj = hj::parse(vs[v].data(), vs[v].size());
      const hj::Value* stats = member(sj, u"stats");
      st[0] += (uint64_t)member(*stats, u"treeNodeCount")->n;
      st[1] += (uint64_t)member(*stats, u"blobNodeCount")->n;
      st[2] += (uint64_t)member(*stats, u"totalBlobSize")->n;
      tree += v ? ",\"cols\":" : "\"rows\":";
      tree += hj::dump(*member(sj, u"summary"));
    }
    tree += ",\"cells\":{\"type\":2,\"content\":";
    hj::quote_u8(tree, cells);
    tree += "}}";
    const std::string summary = "{\"summary\":{\"type\":1,\"tree\":" + tree + "},\"stats\":{\"treeNodeCount\":" +
                                std::to_string(st[0]) + ",\"blobNodeCount\":" + std::to_string(st[1]) +
                                ",\"handleNodeCount\":0,\"totalBlobSize\":" + std::to_string(st[2]) +
                                ",\"unreferencedBlobSize\":0}}";
    fill_blob_list(all, summary, out);
  });
}

// ------------------------------------------------------------------ segment queries (Client reads)
namespace {
// nodeLength of a leaf (mergeTree.ts:916-1004) in the (refSeq R, client C) view; -1 = undefined.
// C == the observer is the local view (localNetLength, :613-634).  A live client's unacked insert /
// remove holds MTB_PEND + localSeq, above every refSeq (UnassignedSequenceNumber).
int leaf_length(const HostDoc& d, const Seg& g, int R, int C, bool newMode, int minSeq, std::vector<int>& rc) {
  const bool removed = seg_removed(g);
  if (C == 0) {
    if (!removed) return g.len;
    return newMode ? 0 : (g.rseq > minSeq ? 0 : -1);
  }
  bool cRemoved = false;
  if (removed) {
    rc_list(d, g, rc);
    cRemoved = std::find(rc.begin(), rc.end(), C) != rc.end();
  }
  if (newMode) {
    if (removed && g.rseq <= minSeq) return -1;
    if (removed && (g.rseq <= R || cRemoved)) return 0;
    return (g.seq <= R || g.client == C) ? g.len : 0;
  }
  if (removed && g.rseq <= R) return -1;
  if (g.client == C || g.seq <= R) return removed ? (cRemoved ? 0 : g.len) : g.len;
  return removed && !seg_pending(g.rseq) ? -1 : 0;
}
}  // namespace

// MergeTree.mapRange / nodeMap (mergeTree.ts:2456-2474, 2531-2582) over [start, end) in a perspective:
// Client.walkSegments (client.ts:286, the local view), getContainingSegment (:1065, mergeTree.ts:787-813)
// and getPropertiesAtPosition (client.ts:1101) are views of it.  Output: a JSON array of
// {"pos", "start", "end", "segment"} per visited leaf (start / end relative to the segment, as the
// reference's handler receives them), at most `limit` entries (0 = all).
namespace {
// The phantom surplus less the deficits of each block of a loaded document (mtb_replay.hip "phantom partial
// lengths") in the (R, C) view; empty for the local view and for documents without a table.
std::unordered_map<uint32_t, int64_t> phantom_surplus(const HostDoc& d, const DocState& s, int R, int C) {
  std::unordered_map<uint32_t, int64_t> sur;
  if (!s.ph || !(s.flags & DSF_PHANTOM) || C == 0 || (size_t)s.ph + 2 > d.aux.size()) return sur;
  const uint32_t n = d.aux[s.ph];
  if ((size_t)s.ph + 2 + 8ull * n > d.aux.size()) raise(MTB_E_INTERNAL, "corrupt phantom table");
  const int Rl = std::max(R, (int)s.min_seq);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t* e = d.aux.data() + s.ph + 2 + 8ull * i;
    if (e[0] == MTB_NONE) continue;  // (a dead deficit)
    if (e[6] == PH_PHANTOM) {
      bool vis = (int)e[1] <= Rl || (int)(int16_t)e[3] == C;
      if (!vis && e[4] && e[4] < d.aux.size())
        for (uint32_t r = 0; r < d.aux[e[4]] && e[4] + 1 + r < d.aux.size() && !vis; r++)
          vis = (int)d.aux[e[4] + 1 + r] == C;
      if (vis) sur[e[0]] += e[2];
    } else if (e[6] == PH_DEF_MIN || (e[6] == PH_DEF_MAIN && Rl >= (int)e[1]) ||
               (e[6] == PH_DEF_CLI && (int)(int16_t)e[3] == C && Rl < (int)e[1])) {
      sur[e[0]] -= e[2];  // (getPartialLength's shortfall, mtb_replay.hip ph_view)
    }
  }
  return sur;
}
}  // namespace

int mtbx_debug_blocks(mtb_dev* b, uint32_t doc, int64_t ref_seq, const char* long_client_id, char** out,
                      size_t* out_len) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (!out) raise(MTB_E_ARG, "null output");
    if (!d.onDevice || !b->devInit) raise(MTB_E_ARG, "document has not been replayed");
    if (b->hst[doc].err) raise(derr_code(b->hst[doc].err), derr_text(b->hst[doc].err));
    download_doc(b, doc);
    const DocState& s = b->hst[doc];
    const bool newMode = b->opts.new_length_calc != 0;
    const int R = ref_seq < 0 ? (int)s.cur_seq : (int)ref_seq;
    int C = 0;
    if (long_client_id) {
      auto it = d.shortOf.find(long_client_id);
      C = it == d.shortOf.end() ? -3 : it->second;
    }
    std::unordered_map<uint32_t, int64_t> sur = phantom_surplus(d, s, R, C);
    std::vector<int> rc;
    std::function<int64_t(uint32_t)> leafsum = [&](uint32_t c) -> int64_t {
      if (c & MTB_LEAF) {
        const int l = leaf_length(d, d.segs[c & ~MTB_LEAF], R, C, newMode, (int)s.min_seq, rc);
        return l > 0 ? l : 0;
      }
      const Blk& B = d.blks.at(c);
      int64_t t = 0;
      for (int i = 0; i < B.count; i++) t += leafsum(B.child[i]);
      return t;
    };
    std::string o;
    std::function<void(uint32_t, const std::string&)> visit = [&](uint32_t bi, const std::string& path) {
      const Blk& B = d.blks.at(bi);
      o += "{\"path\":[" + path + "],\"kids\":[";
      for (int i = 0; i < B.count; i++) {
        const uint32_t c = B.child[i];
        if (i) o += ",";
        if (c & MTB_LEAF) {
          o += "null";
        } else {
          const int64_t ls = leafsum(c);
          auto it = sur.find(c);
          o += "[" + std::to_string(ls + (it == sur.end() ? 0 : it->second)) + "," + std::to_string(ls) + "]";
        }
      }
      o += "],\"table\":[";
      bool first = true;
      if (s.ph && (size_t)s.ph + 2 <= d.aux.size()) {
        const uint32_t n = d.aux[s.ph];
        for (uint32_t i = 0; i < n && (size_t)s.ph + 2 + 8ull * (i + 1) <= d.aux.size(); i++) {
          const uint32_t* e = d.aux.data() + s.ph + 2 + 8ull * i;
          if (e[0] != bi) continue;
          o += std::string(first ? "" : ",") + "[" + std::to_string(e[6]) + "," + std::to_string((int)e[1]) + "," +
               std::to_string((int)e[2]) + "," + std::to_string((int)(int16_t)e[3]) + "]";
          first = false;
        }
      }
      o += "]}\n";
      for (int i = 0; i < B.count; i++)
        if (!(B.child[i] & MTB_LEAF)) visit(B.child[i], path + (path.empty() ? "" : ",") + std::to_string(i));
    };
    visit(s.root, "");
    *out = dup(o);
    if (out_len) *out_len = o.size();
  });
}

int mtbx_map_range(mtb_dev* b, uint32_t doc, int64_t start, int64_t end, int64_t ref_seq, const char* long_client_id,
                  uint32_t limit, char** out, size_t* out_len) {
  return guarded(b, [&] {
    HostDoc& d = docref(b, doc);
    if (!out) raise(MTB_E_ARG, "null output");
    if (!d.onDevice || !b->devInit) raise(MTB_E_ARG, "document has not been replayed");
    if (b->hst[doc].err) raise(derr_code(b->hst[doc].err), derr_text(b->hst[doc].err));
    download_doc(b, doc);
    const DocState& s = b->hst[doc];
    const bool newMode = b->opts.new_length_calc != 0;
    const int R = ref_seq < 0 ? (int)s.cur_seq : (int)ref_seq;
    int C = 0;
    if (long_client_id) {  // getClientSequenceArgsForMessage: a client not seen yet owns nothing
      auto it = d.shortOf.find(long_client_id);
      C = it == d.shortOf.end() ? -3 : it->second;
    }
    std::vector<FlatSeg> fl;
    flatten(d, s.root, fl, false);
    std::vector<int> rc;
    int64_t total = 0;
    std::vector<int> lens(fl.size());
    for (size_t k = 0; k < fl.size(); k++) {
      lens[k] = leaf_length(d, d.segs[fl[k].id], R, C, newMode, (int)s.min_seq, rc);
      if (lens[k] > 0) total += lens[k];
    }
    // nodeMap (mergeTree.ts:2531-2582) visits leaves in order; a block is skipped whole when `start` lies past
    // its length.  Block lengths are the sums of their leaves' except for a loaded document's phantom surplus,
    // which moves the position past a skipped block (and the default end, the root's length): those documents
    // take the walk over the blocks (visit[k] = leaf k's position, -1 = skipped or past the end)
    std::unordered_map<uint32_t, int64_t> sur = phantom_surplus(d, s, R, C);
    std::vector<int64_t> at;
    int64_t endPos = end < 0 ? total : end;
    if (!sur.empty()) {
      std::unordered_map<uint32_t, int64_t> blen;  // leaf sums + surplus, post-order
      {
        struct Fr { uint32_t b; int i; int64_t acc; };
        std::vector<Fr> st{{s.root, 0, 0}};
        size_t k = 0;
        while (!st.empty()) {
          Fr& f = st.back();
          const Blk& B = d.blks.at(f.b);
          if (f.i >= B.count) {
            const uint32_t fb = f.b;
            const int64_t acc = f.acc;
            auto it = sur.find(fb);
            blen[fb] = acc + (it == sur.end() ? 0 : it->second);
            st.pop_back();
            if (!st.empty()) st.back().acc += acc;  // (the parent's exact part: its leaves only)
            continue;
          }
          const uint32_t c = B.child[f.i++];
          if (c & MTB_LEAF) {
            f.acc += lens[k] > 0 ? lens[k] : 0;
            k++;
          } else {
            st.push_back({c, 0, 0});
          }
        }
      }
      if (end < 0) endPos = blen[s.root];
      at.assign(fl.size(), -1);
      int64_t pos = 0;
      bool exit = false;
      struct Fr { uint32_t b; int i; };
      std::vector<Fr> st{{s.root, 0}};
      size_t k = 0;
      // (leaf indices follow flatten's order: a skipped block's leaves are counted past)
      auto count_leaves = [&](uint32_t b0) {
        std::vector<uint32_t> q{b0};
        size_t c = 0;
        while (!q.empty()) {
          const Blk& B = d.blks.at(q.back());
          q.pop_back();
          for (int i = B.count - 1; i >= 0; i--) {
            if (B.child[i] & MTB_LEAF) c++;
            else q.push_back(B.child[i]);
          }
        }
        return c;
      };
      while (!st.empty() && !exit) {
        Fr& f = st.back();
        const Blk& B = d.blks.at(f.b);
        if (f.i >= B.count) {
          st.pop_back();
          continue;
        }
        const uint32_t c = B.child[f.i++];
        if (endPos <= pos) { exit = true; break; }
        if (c & MTB_LEAF) {
          const int len = lens[k];
          if (len > 0) {
            if (start >= pos + len) {
              pos += len;
            } else {
              at[k] = pos;
              pos += len;
            }
          }
          k++;
        } else {
          const int64_t len = blen[c];
          if (len == 0) { k += count_leaves(c); continue; }
          if (start >= pos + len) {
            pos += len;
            k += count_leaves(c);
            continue;
          }
          st.push_back({c, 0});
        }
      }
    }
    std::string o = "[";
    uint32_t n = 0;
    int64_t base = 0;
    if (endPos != start)
      for (size_t k = 0; k < fl.size(); k++) {
        const int len = lens[k];
        int64_t pos = base;
        if (!sur.empty()) {
          if (at[k] < 0) continue;
          pos = at[k];
        }
        if (pos >= endPos) break;
        if (len <= 0) continue;  // undefined or zero: Skip
        const int64_t next = pos + len;
        base += len;
        if (start >= next) continue;
        const Seg& g = d.segs[fl[k].id];
        if (n) o += ',';
        o += "{\"pos\":" + std::to_string(pos) + ",\"start\":" + std::to_string(start - pos) + ",\"end\":" +
             std::to_string(endPos - pos) + ",\"segment\":{\"type\":";
        if (d.perm) {
          o += "\"PermutationSegment\",\"start\":" + std::to_string(g.text == MTB_HANDLE_UNALLOC ? INT32_MIN : (int64_t)g.text);
        } else if (is_marker(g)) {
          const uint32_t rt = g.text & ~MTB_MARKER;
          o += "\"Marker\",\"refType\":" + (rt == 0 ? std::string("null") : std::to_string(rt - 1));
        } else {
          o += "\"TextSegment\",\"text\":";
          hj::quote(o, reinterpret_cast<const char16_t*>(d.text.data() + g.text), (size_t)g.len);
        }
        o += ",\"cachedLength\":" + std::to_string(g.len) + ",\"seq\":" + std::to_string(seq_out(g.seq)) +
             ",\"clientId\":" + std::to_string(d.ref_id(g.client));
        if (seg_removed(g)) {
          o += ",\"removedSeq\":" + std::to_string(seq_out(g.rseq)) + ",\"removedClientIds\":[";
          rc_list(d, g, rc);
          for (size_t q = 0; q < rc.size(); q++) o += (q ? "," : "") + std::to_string(d.ref_id(rc[q]));
          o += "]";
        }
        PropView pv = props_of(b, d, g.props);
        if (g.props && pv.n() > 0) {
          o += ",\"properties\":";
          props_json(b, o, pv);
        }
        o += "}}";
        if (++n == limit) break;
      }
    o += "]";
    *out = dup(o);
    if (out_len) *out_len = o.size();
  });
}

// ------------------------------------------------------------------ SharedMatrix load
namespace {
uint32_t compact_even(uint32_t x) {  // inverse of CellStore::spread: the even bits, packed
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0f0f0f0fu;
  x = (x | (x >> 4)) & 0x00ff00ffu;
  x = (x | (x >> 8)) & 0x0000ffffu;
  return x;
}
// SparseArray2D.load (sparsearray2d.ts:233-236) into a CellStore: every non-null leaf becomes a written
// key; a 256-leaf tile whose leaves are all null keeps its place through one written-undefined key
void load_cells(mtb_dev* b, CellStore& cs, const hj::Value& root) {
  if (root.kind != hj::Value::kArr) raise(MTB_E_PARSE, "cells snapshot is not an array");
  cs.rootLen = std::max<uint64_t>(1, root.items.size());
  for (size_t hi = 0; hi < root.items.size(); hi++) {
    const hj::Value& l0 = root.items[hi];
    if (l0.kind == hj::Value::kNull) continue;
    auto key = [&](uint32_t lo, uint32_t v) {
      const uint32_t khi = (uint32_t)hi;
      const uint32_t r = compact_even(lo >> 1) | (compact_even(khi >> 1) << 16);
      const uint32_t c = compact_even(lo) | (compact_even(khi) << 16);
      cs.set(r, c, v);
    };
    // levels 0..2 hold arrays, level 3 values; a level array with no children cannot be represented
    auto walk = [&](auto& self, const hj::Value& a, int lv, uint32_t pre) -> void {
      if (a.kind != hj::Value::kArr) raise(MTB_E_PARSE, "cells level is not an array");
      bool any = false;
      for (size_t e = 0; e < a.items.size() && e < 256; e++) {
        const hj::Value& x = a.items[e];
        if (x.kind == hj::Value::kNull) continue;
        const uint32_t k = pre | ((uint32_t)e << (24 - 8 * lv));
        if (lv == 3) key(k, intern_cell_value(b, hj::dump(x)));
        else self(self, x, lv + 1, k);
        any = true;
      }
      if (!any) {
        if (lv < 3) raise(MTB_E_UNSUPPORTED, "unsupported: an empty SparseArray2D level above the leaves");
        key(pre, 0);
      }
    };
    walk(walk, l0, 0, 0);
  }
}
}  // namespace

// SharedMatrix.loadCore (matrix.ts:611-634): rows / cols PermutationVector.load (permutationvector.ts:
// 327-345: HandleTable.load of "handleTable", then Client.load of "segments/...") and SparseArray2D.load
// of "cells"; blob paths as mtb_matrix_summarize writes them.
int mtbx_matrix_load(mtb_dev* b, uint32_t matrix, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id) {
  return guarded(b, [&] {
    if (!b->matrix) raise(MTB_E_ARG, "not a matrix batch (MTB_BATCH_MATRIX)");
    if (matrix >= b->ndocs / 2) raise(MTB_E_ARG, "matrix index out of range");
    if (!observer_long_id) raise(MTB_E_ARG, "observer long client id required");
    if (nblobs && !blobs) raise(MTB_E_ARG, "null blob array");
    for (int v = 0; v < 2; v++) {
      const HostDoc& d = b->docs[2 * matrix + v];
      if (d.inited || d.onDevice) raise(MTB_E_ARG, "matrix already initialised");
    }
    auto blob = [&](const std::string& path) -> hj::Value {
      for (uint32_t i = 0; i < nblobs; i++)
        if (blobs[i].path && path == blobs[i].path) return hj::parse(blobs[i].content ? blobs[i].content : "", blobs[i].content_len);
      raise(MTB_E_ARG, "summary blob not found: " + path);
    };
    HostDoc fresh[2];
    for (int v = 0; v < 2; v++) {
      HostDoc& d = fresh[v];
      d.perm = true;
      const std::string pre = v ? "cols/" : "rows/";
      const hj::Value ht = blob(pre + "handleTable");
      if (ht.kind != hj::Value::kArr || ht.items.empty()) raise(MTB_E_PARSE, "bad handleTable blob");
      load_one(b, d, blobs, nblobs, observer_long_id, nullptr, pre + "segments/");
      d.initText.clear();  // the text arena of a PermutationVector holds its handle table: u32 [length, handles]
      auto word = [&](uint32_t w) {
        d.initText.push_back((uint16_t)(w & 0xFFFF));
        d.initText.push_back((uint16_t)(w >> 16));
      };
      word((uint32_t)ht.items.size());
      for (auto& h : ht.items) word(h.kind == hj::Value::kNum ? (uint32_t)(int64_t)h.n : 0u);
      resolve_load_props(b, d);
    }
    const hj::Value cd = blob("cells");
    if (cd.kind != hj::Value::kArr || cd.items.size() < 2) raise(MTB_E_PARSE, "bad cells blob");
    std::unique_ptr<CellStore> cs(new CellStore());
    load_cells(b, *cs, cd.items[0]);
    const hj::Value& pend = cd.items[1];  // the observer's pending local writes must be empty
    if (pend.kind != hj::Value::kArr || pend.items.size() != 1 || pend.items[0].kind != hj::Value::kNull)
      raise(MTB_E_UNSUPPORTED, "unsupported: pending local cell writes in a summary");
    fresh[0].cells = std::move(cs);
    for (int v = 0; v < 2; v++) b->docs[2 * matrix + v] = std::move(fresh[v]);
  });
}
