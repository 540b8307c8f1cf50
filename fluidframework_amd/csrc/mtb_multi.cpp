// Public C ABI (include/mtb.h) over one or more devices.
//
// A batch created with a device mask of k devices holds k per-device engines (mtb_host.cpp, one HIP
// device with its own HBM pools and stream each; more per device with MTB_SHARDS_PER_DEVICE).  Documents
// are independent, so they are spread by the same document hash the multi-process path uses
// (fluidframework_amd/sharding.py: FNV-1a of the 8 little-endian bytes of the index, mod the shard
// count); a SharedMatrix batch spreads whole matrices (both vectors stay together).  Document-level calls
// go to the owning shard with the document's index there; mtb_replay / mtb_rewind / mtb_replay_resident
// run every shard on its own host thread (each device busy at once) and merge the statistics; interning
// calls are applied to every shard in the same order so props / value ids agree everywhere.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <regex>
#include <string>
#include <thread>
#include <vector>

#include "mtb_dev.h"
#include "../../include/mtb_testing.h"

struct mtb_batch {
  uint32_t ndocs = 0;
  bool matrix = false;
  std::vector<mtb_dev*> shards;
  std::vector<uint32_t> shardOf, localOf;   // global document -> (shard, index in the shard)
  std::vector<std::vector<uint32_t>> globalOf;  // shard -> its documents' global indices
  std::string err;
};

namespace {

uint32_t fnv32(uint64_t x) {
  uint32_t h = 2166136261u;
  for (int i = 0; i < 8; i++) {
    h ^= (uint32_t)((x >> (8 * i)) & 0xFF);
    h *= 16777619u;
  }
  return h;
}

// The shard's error text with its local document indices ("document 12") rewritten to global ones.
void take_error(mtb_batch* b, uint32_t s) {
  std::string m = mtbx_last_error(b->shards[s]);
  if (b->shards.size() > 1) {
    static const std::regex re("document ([0-9]+)");
    std::string out;
    std::sregex_iterator it(m.begin(), m.end(), re), end;
    size_t last = 0;
    for (; it != end; ++it) {
      const auto& mm = *it;
      const unsigned long li = std::stoul(mm[1].str());
      out += m.substr(last, (size_t)mm.position(0) - last);
      out += "document " + (li < b->globalOf[s].size() ? std::to_string(b->globalOf[s][li]) : mm[1].str());
      last = (size_t)(mm.position(0) + mm.length(0));
    }
    out += m.substr(last);
    m = out;
  }
  b->err = m;
}

template <class F>
int on_shard(mtb_batch* b, uint32_t s, F&& f) {
  const int rc = f(b->shards[s]);
  if (rc) take_error(b, s);
  return rc;
}

int doc_call(mtb_batch* b, uint32_t doc, uint32_t& s, uint32_t& local) {
  if (!b) return MTB_E_ARG;
  if (doc >= b->ndocs) {
    b->err = "document index out of range";
    return MTB_E_ARG;
  }
  s = b->shardOf[doc];
  local = b->localOf[doc];
  return MTB_OK;
}

#define DOC_CALL(doc, expr)                          \
  do {                                               \
    uint32_t s_, l_;                                 \
    const int rc_ = doc_call(b, (doc), s_, l_);      \
    if (rc_) return rc_;                             \
    return on_shard(b, s_, [&](mtb_dev* d_) { return expr; }); \
  } while (0)

// matrix m lives in the shard of its rows document 2m, as local matrix (local rows index) / 2
int matrix_call(mtb_batch* b, uint32_t m, uint32_t& s, uint32_t& lm) {
  if (!b) return MTB_E_ARG;
  if (!b->matrix) {
    b->err = "not a matrix batch (MTB_BATCH_MATRIX)";
    return MTB_E_ARG;
  }
  if (m >= b->ndocs / 2) {
    b->err = "matrix index out of range";
    return MTB_E_ARG;
  }
  s = b->shardOf[2 * m];
  lm = b->localOf[2 * m] / 2;
  return MTB_OK;
}

#define MATRIX_CALL(m, expr)                         \
  do {                                               \
    uint32_t s_, l_;                                 \
    const int rc_ = matrix_call(b, (m), s_, l_);     \
    if (rc_) return rc_;                             \
    return on_shard(b, s_, [&](mtb_dev* d_) { return expr; }); \
  } while (0)

// f(shard) on every shard, each on its own host thread; the first failure (by shard order) is reported
template <class F>
int all_shards(mtb_batch* b, F&& f) {
  const size_t n = b->shards.size();
  std::vector<int> rc(n, 0);
  if (n == 1) {
    rc[0] = f(0u);
  } else {
    std::vector<std::thread> ts;
    for (size_t s = 0; s < n; s++) ts.emplace_back([&, s] { rc[s] = f((uint32_t)s); });
    for (auto& t : ts) t.join();
  }
  for (size_t s = 0; s < n; s++)
    if (rc[s]) {
      take_error(b, (uint32_t)s);
      return rc[s];
    }
  return MTB_OK;
}

void merge_stats(mtb_stats& a, const mtb_stats& x) {
  a.ops_applied += x.ops_applied;
  a.docs += x.docs;
  a.segments_final += x.segments_final;
  a.text_units_final += x.text_units_final;
  a.bytes_alg += x.bytes_alg;
  a.checksum += x.checksum;
  a.errors += x.errors;
  if (x.kernel_ms > a.kernel_ms) a.kernel_ms = x.kernel_ms;
}

}  // namespace

extern "C" {

int mtb_batch_create(const mtb_options* opts, uint32_t ndocs, uint32_t device_mask, mtb_batch** out) {
  if (!out || ndocs == 0) return MTB_E_ARG;
  const bool matrix = opts && (opts->flags & MTB_BATCH_MATRIX);
  if (matrix && (ndocs & 1)) return MTB_E_ARG;  // a matrix batch holds (rows, cols) pairs
  std::vector<int> devs;
  for (int k = 0; k < 32; k++)
    if (device_mask & (1u << k)) devs.push_back(k);
  if (devs.empty()) devs.push_back(0);
  int per = 1;
  if (const char* e = getenv("MTB_SHARDS_PER_DEVICE")) per = std::max(1, std::min(64, atoi(e)));
  std::vector<int> shardDev;
  for (int d : devs)
    for (int k = 0; k < per; k++) shardDev.push_back(d);
  const uint32_t units = matrix ? ndocs / 2 : ndocs;  // documents, or matrices
  const uint32_t ns = (uint32_t)std::min<size_t>(shardDev.size(), units);
  auto* b = new mtb_batch();
  b->ndocs = ndocs;
  b->matrix = matrix;
  b->shardOf.assign(ndocs, 0);
  b->localOf.assign(ndocs, 0);
  std::vector<std::vector<uint32_t>> members(ns);
  for (uint32_t u = 0; u < units; u++) members[ns == 1 ? 0 : fnv32(u) % ns].push_back(u);
  for (uint32_t s = 0; s < ns; s++) {
    if (members[s].empty()) continue;
    const uint32_t si = (uint32_t)b->shards.size();
    std::vector<uint32_t> g;
    for (uint32_t u : members[s]) {
      if (matrix) {
        for (uint32_t v = 0; v < 2; v++) {
          b->shardOf[2 * u + v] = si;
          b->localOf[2 * u + v] = (uint32_t)g.size();
          g.push_back(2 * u + v);
        }
      } else {
        b->shardOf[u] = si;
        b->localOf[u] = (uint32_t)g.size();
        g.push_back(u);
      }
    }
    mtb_dev* d = nullptr;
    const int rc = mtbx_batch_create(opts, (uint32_t)g.size(), 1u << shardDev[s], &d);
    if (rc) {
      for (mtb_dev* x : b->shards) mtbx_batch_destroy(x);
      delete b;
      return rc;
    }
    b->shards.push_back(d);
    b->globalOf.push_back(std::move(g));
  }
  *out = b;
  return MTB_OK;
}

void mtb_batch_destroy(mtb_batch* b) {
  if (!b) return;
  for (mtb_dev* d : b->shards) mtbx_batch_destroy(d);
  delete b;
}

const char* mtb_last_error(mtb_batch* b) { return b ? b->err.c_str() : "null batch"; }

int mtb_doc_init(mtb_batch* b, uint32_t doc, const uint16_t* initial_text, size_t n_units, const char* observer_long_id,
                 uint32_t min_seq, uint32_t cur_seq) {
  DOC_CALL(doc, mtbx_doc_init(d_, l_, initial_text, n_units, observer_long_id, min_seq, cur_seq));
}

int mtb_doc_load_v1(mtb_batch* b, uint32_t doc, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id) {
  DOC_CALL(doc, mtbx_doc_load_v1(d_, l_, blobs, nblobs, observer_long_id));
}

int mtb_docs_load_v1(mtb_batch* b, uint32_t n, const uint32_t* docs, const mtb_blob* const* blobs, const uint32_t* nblobs,
                     const char* const* observer_long_ids, uint32_t threads) {
  if (!b) return MTB_E_ARG;
  if (n && (!docs || !blobs || !nblobs || !observer_long_ids)) {
    b->err = "null argument";
    return MTB_E_ARG;
  }
  for (uint32_t i = 0; i < n; i++)
    if (docs[i] >= b->ndocs) {
      b->err = "document index out of range";
      return MTB_E_ARG;
    }
  // every shard loads its documents (failures are reported after all shards ran, like one engine)
  const size_t ns = b->shards.size();
  std::vector<std::vector<uint32_t>> ld(ns), pos(ns);
  for (uint32_t i = 0; i < n; i++) {
    ld[b->shardOf[docs[i]]].push_back(b->localOf[docs[i]]);
    pos[b->shardOf[docs[i]]].push_back(i);
  }
  int first = MTB_OK;
  for (size_t s = 0; s < ns; s++) {
    if (ld[s].empty()) continue;
    std::vector<const mtb_blob*> bl;
    std::vector<uint32_t> nb;
    std::vector<const char*> ob;
    for (uint32_t i : pos[s]) {
      bl.push_back(blobs[i]);
      nb.push_back(nblobs[i]);
      ob.push_back(observer_long_ids[i]);
    }
    const int rc = mtbx_docs_load_v1(b->shards[s], (uint32_t)ld[s].size(), ld[s].data(), bl.data(), nb.data(), ob.data(), threads);
    if (rc && !first) {
      first = rc;
      take_error(b, (uint32_t)s);
    }
  }
  return first;
}

int mtb_add_client(mtb_batch* b, uint32_t doc, const char* long_id) { DOC_CALL(doc, mtbx_add_client(d_, l_, long_id)); }

int mtb_intern_props(mtb_batch* b, const char* json_utf8, size_t len, uint32_t* id_out) {
  if (!b) return MTB_E_ARG;
  uint32_t id0 = 0;
  for (uint32_t s = 0; s < b->shards.size(); s++) {
    uint32_t id = 0;
    const int rc = on_shard(b, s, [&](mtb_dev* d) { return mtbx_intern_props(d, json_utf8, len, &id); });
    if (rc) return rc;
    if (s == 0) id0 = id;
    else if (id != id0) {
      b->err = "props ids diverged between devices";
      return MTB_E_ARG;
    }
  }
  if (id_out) *id_out = id0;
  return MTB_OK;
}

int mtb_apply_msg_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len) {
  DOC_CALL(doc, mtbx_apply_msg_json(d_, l_, json_utf8, len));
}
int mtb_local_op_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len) {
  DOC_CALL(doc, mtbx_local_op_json(d_, l_, json_utf8, len));
}
int mtb_detached_op_json(mtb_batch* b, uint32_t doc, const char* json_utf8, size_t len) {
  DOC_CALL(doc, mtbx_detached_op_json(d_, l_, json_utf8, len));
}
int mtb_maintenance(mtb_batch* b, uint32_t doc, uint32_t kind) {
  DOC_CALL(doc, mtbx_maintenance(d_, l_, kind));
}
int mtb_regenerate_pending_op(mtb_batch* b, uint32_t doc, const char* op_json, size_t len, char** out, size_t* out_len) {
  DOC_CALL(doc, mtbx_regenerate_pending_op(d_, l_, op_json, len, out, out_len));
}

int mtb_append_ops(mtb_batch* b, uint32_t doc, const mtb_op* ops, uint32_t n, const uint16_t* payload, size_t payload_len) {
  DOC_CALL(doc, mtbx_append_ops(d_, l_, ops, n, payload, payload_len));
}

int mtb_matrix_init(mtb_batch* b, uint32_t matrix, const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq) {
  MATRIX_CALL(matrix, mtbx_matrix_init(d_, l_, observer_long_id, min_seq, cur_seq));
}

int mtb_matrix_apply_msg_json(mtb_batch* b, uint32_t matrix, const char* json_utf8, size_t len) {
  MATRIX_CALL(matrix, mtbx_matrix_apply_msg_json(d_, l_, json_utf8, len));
}

int mtb_matrix_intern_value(mtb_batch* b, const char* json_utf8, size_t len, uint32_t* id_out) {
  if (!b) return MTB_E_ARG;
  uint32_t id0 = 0;
  for (uint32_t s = 0; s < b->shards.size(); s++) {
    uint32_t id = 0;
    const int rc = on_shard(b, s, [&](mtb_dev* d) { return mtbx_matrix_intern_value(d, json_utf8, len, &id); });
    if (rc) return rc;
    if (s == 0) id0 = id;
    else if (id != id0) {
      b->err = "value ids diverged between devices";
      return MTB_E_ARG;
    }
  }
  if (id_out) *id_out = id0;
  return MTB_OK;
}

int mtb_matrix_load(mtb_batch* b, uint32_t matrix, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id) {
  MATRIX_CALL(matrix, mtbx_matrix_load(d_, l_, blobs, nblobs, observer_long_id));
}

int mtb_matrix_summarize(mtb_batch* b, uint32_t matrix, mtb_blob_list* out) {
  MATRIX_CALL(matrix, mtbx_matrix_summarize(d_, l_, out));
}

int mtb_matrix_get_cell(mtb_batch* b, uint32_t matrix, uint32_t row, uint32_t col, char* buf, size_t cap, size_t* len_out) {
  MATRIX_CALL(matrix, mtbx_matrix_get_cell(d_, l_, row, col, buf, cap, len_out));
}

int mtb_replay(mtb_batch* b, mtb_stats* out) {
  if (!b) return MTB_E_ARG;
  std::vector<mtb_stats> st(b->shards.size());
  const int rc = all_shards(b, [&](uint32_t s) { return mtbx_replay(b->shards[s], &st[s]); });
  if (out) {
    *out = mtb_stats{};
    for (auto& x : st) merge_stats(*out, x);
  }
  return rc;
}

int mtb_rewind(mtb_batch* b) {
  if (!b) return MTB_E_ARG;
  return all_shards(b, [&](uint32_t s) { return mtbx_rewind(b->shards[s]); });
}

int mtb_replay_resident(mtb_batch* b, mtb_stats* out) { return mtb_replay_resident_ex(b, out, 0); }

int mtb_replay_resident_ex(mtb_batch* b, mtb_stats* out, uint32_t flags) {
  if (!b) return MTB_E_ARG;
  std::vector<mtb_stats> st(b->shards.size());
  const int rc = all_shards(b, [&](uint32_t s) { return mtbx_replay_resident(b->shards[s], &st[s], flags); });
  if (out) {
    *out = mtb_stats{};
    for (auto& x : st) merge_stats(*out, x);
  }
  return rc;
}

int mtb_refresh_digests(mtb_batch* b, mtb_stats* out) {
  if (!b) return MTB_E_ARG;
  std::vector<mtb_stats> st(b->shards.size());
  const int rc = all_shards(b, [&](uint32_t s) { return mtbx_refresh_digests(b->shards[s], &st[s]); });
  if (out) {
    *out = mtb_stats{};
    for (auto& x : st) merge_stats(*out, x);
  }
  return rc;
}

int mtb_get_text(mtb_batch* b, uint32_t doc, uint16_t* buf, size_t cap, size_t* len_out) {
  DOC_CALL(doc, mtbx_get_text(d_, l_, buf, cap, len_out));
}

int mtb_get_length(mtb_batch* b, uint32_t doc, uint32_t* len_out) { DOC_CALL(doc, mtbx_get_length(d_, l_, len_out)); }

int mtb_test_set_root_child(mtb_batch* b, uint32_t doc, uint32_t value, uint32_t* old_out) {
  DOC_CALL(doc, mtbx_test_set_root_child(d_, l_, value, old_out));
}

int mtb_get_seq(mtb_batch* b, uint32_t doc, uint32_t* cur_seq, uint32_t* min_seq) {
  DOC_CALL(doc, mtbx_get_seq(d_, l_, cur_seq, min_seq));
}

int mtb_dump_segments(mtb_batch* b, uint32_t doc, char** out, size_t* out_len) {
  DOC_CALL(doc, mtbx_dump_segments(d_, l_, out, out_len));
}

int mtb_doc_checksum(mtb_batch* b, uint32_t doc, uint64_t* out) { DOC_CALL(doc, mtbx_doc_checksum(d_, l_, out)); }

int mtb_get_launch_info(mtb_batch* b, mtb_launch_info* out) {
  if (!b || !out) return MTB_E_ARG;
  mtb_launch_info acc{};
  for (uint32_t s = 0; s < (uint32_t)b->shards.size(); s++) {
    mtb_launch_info x{};
    const int rc = on_shard(b, s, [&](mtb_dev* d) { return mtbx_get_launch_info(d, &x); });
    if (rc) return rc;
    if (s == 0) acc = x;
    acc.aborted |= x.aborted;
    acc.handover_bad += x.handover_bad;
    acc.cap_retries = std::max(acc.cap_retries, x.cap_retries);
  }
  *out = acc;
  return 0;
}

int mtb_doc_digests(mtb_batch* b, uint32_t first, uint32_t n, uint64_t* out) {
  if (!b) return MTB_E_ARG;
  if (!out && n) {
    b->err = "null output";
    return MTB_E_ARG;
  }
  if ((uint64_t)first + n > b->ndocs) {
    b->err = "document range out of bounds";
    return MTB_E_ARG;
  }
  for (uint32_t s = 0; s < b->shards.size(); s++) {
    const auto& g = b->globalOf[s];
    std::vector<uint64_t> v(g.size());
    const int rc = on_shard(b, s, [&](mtb_dev* d) { return mtbx_doc_digests(d, 0, (uint32_t)g.size(), v.data()); });
    if (rc) return rc;
    for (size_t k = 0; k < g.size(); k++)
      if (g[k] >= first && g[k] < first + n) out[g[k] - first] = v[k];
  }
  return MTB_OK;
}

int mtb_map_range(mtb_batch* b, uint32_t doc, int64_t start, int64_t end, int64_t ref_seq, const char* long_client_id,
                  uint32_t limit, char** out, size_t* out_len) {
  DOC_CALL(doc, mtbx_map_range(d_, l_, start, end, ref_seq, long_client_id, limit, out, out_len));
}

int mtb_debug_blocks(mtb_batch* b, uint32_t doc, int64_t ref_seq, const char* long_client_id, char** out,
                     size_t* out_len) {
  DOC_CALL(doc, mtbx_debug_blocks(d_, l_, ref_seq, long_client_id, out, out_len));
}

int mtb_summarize_v1(mtb_batch* b, uint32_t doc, int64_t msn, int64_t seq, mtb_blob_list* out) {
  DOC_CALL(doc, mtbx_summarize_v1(d_, l_, msn, seq, out));
}

int mtb_summarize_v1_many(mtb_batch* b, uint32_t n, const uint32_t* docs, int64_t msn, int64_t seq, uint32_t threads,
                          mtb_blob_list* out) {
  if (!b) return MTB_E_ARG;
  if (n && (!docs || !out)) {
    b->err = "null argument";
    return MTB_E_ARG;
  }
  const size_t ns = b->shards.size();
  std::vector<std::vector<uint32_t>> ld(ns), pos(ns);
  for (uint32_t i = 0; i < n; i++) {
    if (docs[i] >= b->ndocs) {
      b->err = "document index out of range";
      return MTB_E_ARG;
    }
    ld[b->shardOf[docs[i]]].push_back(b->localOf[docs[i]]);
    pos[b->shardOf[docs[i]]].push_back(i);
  }
  std::vector<std::vector<mtb_blob_list>> res(ns);
  const uint32_t per = ns > 1 ? std::max<uint32_t>(1, threads / (uint32_t)ns) : threads;
  const int rc = all_shards(b, [&](uint32_t s) {
    res[s].assign(ld[s].size(), mtb_blob_list{});
    if (ld[s].empty()) return (int)MTB_OK;
    return mtbx_summarize_v1_many(b->shards[s], (uint32_t)ld[s].size(), ld[s].data(), msn, seq, per, res[s].data());
  });
  for (size_t s = 0; s < ns; s++)
    for (size_t k = 0; k < pos[s].size(); k++) out[pos[s][k]] = res[s][k];
  return rc;
}

int mtb_summarize_legacy(mtb_batch* b, uint32_t doc, int64_t msn, int64_t seq, const char* catchup_json, size_t catchup_len,
                         mtb_blob_list* out) {
  DOC_CALL(doc, mtbx_summarize_legacy(d_, l_, msn, seq, catchup_json, catchup_len, out));
}

int mtb_export_pending(mtb_batch* b, uint32_t doc, mtb_op* ops, uint32_t cap, uint32_t* n_out, uint16_t* payload, size_t pcap,
                       size_t* plen_out) {
  DOC_CALL(doc, mtbx_export_pending(d_, l_, ops, cap, n_out, payload, pcap, plen_out));
}

int mtb_props_json(mtb_batch* b, uint32_t id, char* buf, size_t cap, size_t* len_out) {
  if (!b || b->shards.empty()) return MTB_E_ARG;
  return on_shard(b, 0, [&](mtb_dev* d) { return mtbx_props_json(d, id, buf, cap, len_out); });
}

int mtb_client_long_id(mtb_batch* b, uint32_t doc, uint32_t short_id, char* buf, size_t cap, size_t* len_out) {
  DOC_CALL(doc, mtbx_client_long_id(d_, l_, short_id, buf, cap, len_out));
}

}  // extern "C"
