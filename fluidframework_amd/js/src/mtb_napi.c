/*
 * mtb_napi.c — Node N-API addon over the engine's C ABI (include/mtb.h).
 *
 * This is the thin native layer the JavaScript drop-in package (../index.js) calls; it exposes one
 * function per mtb_* entry point and does nothing but argument marshalling:
 *   JS string  <-> UTF-8 (JSON messages, ids) or UTF-16 (document text, napi_*_string_utf16)
 *   mtb_stats  ->  plain object;  mtb_blob_list -> {blobs: [[path, content], ...], summary: string}
 *   rc < 0     ->  thrown Error whose message is mtb_last_error() (the reference's assert code /
 *                  error text), with .code = rc and .name = "UsageError" for MTB_E_INSERT
 *                  (mergeTree.ts:1671 throws UsageError("MergeTree insert failed")).
 * replayAsync runs mtb_replay on the libuv thread pool and returns a Promise (SURVEY.md 8(b)
 * "Threading"); the batch handle must not be used from JS until it settles.
 */
#define NAPI_VERSION 3
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/mtb.h"

#define CHECK_NAPI(env, call)                                   \
  do {                                                          \
    if ((call) != napi_ok) {                                    \
      napi_throw_error((env), NULL, "N-API call failed: " #call); \
      return NULL;                                              \
    }                                                           \
  } while (0)

static napi_value throw_rc(napi_env env, mtb_batch* b, int rc) {
  const char* msg = b ? mtb_last_error(b) : "mtb call failed";
  napi_value m, e, code, name;
  napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &m);
  napi_create_error(env, NULL, m, &e);
  napi_create_int32(env, rc, &code);
  napi_set_named_property(env, e, "code", code);
  napi_create_string_utf8(env, rc == MTB_E_INSERT ? "UsageError" : "MergeTreeBatchError", NAPI_AUTO_LENGTH, &name);
  napi_set_named_property(env, e, "name", name);
  napi_throw(env, e);
  return NULL;
}

static napi_value undef(napi_env env) {
  napi_value u;
  napi_get_undefined(env, &u);
  return u;
}

/* ---- argument helpers ------------------------------------------------------------------------ */
static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
  size_t argc = want;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < want) {
    napi_throw_type_error(env, NULL, "wrong number of arguments");
    return 0;
  }
  return 1;
}
static mtb_batch* get_batch(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "expected a batch handle");
    return NULL;
  }
  return (mtb_batch*)p;
}
static int get_u32(napi_env env, napi_value v, uint32_t* out) {
  if (napi_get_value_uint32(env, v, out) != napi_ok) {
    napi_throw_type_error(env, NULL, "expected a number");
    return 0;
  }
  return 1;
}
static int get_i64(napi_env env, napi_value v, int64_t* out) {
  if (napi_get_value_int64(env, v, out) != napi_ok) {
    napi_throw_type_error(env, NULL, "expected a number");
    return 0;
  }
  return 1;
}
/* UTF-8 copy of a JS string (malloc'd, NUL-terminated). */
static char* get_utf8(napi_env env, napi_value v, size_t* len) {
  size_t n = 0;
  if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "expected a string");
    return NULL;
  }
  char* s = (char*)malloc(n + 1);
  napi_get_value_string_utf8(env, v, s, n + 1, &n);
  if (len) *len = n;
  return s;
}
/* UTF-16 copy of a JS string (malloc'd): lone surrogates survive, as in the reference's JS strings. */
static uint16_t* get_utf16(napi_env env, napi_value v, size_t* len) {
  size_t n = 0;
  if (napi_get_value_string_utf16(env, v, NULL, 0, &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "expected a string");
    return NULL;
  }
  uint16_t* s = (uint16_t*)malloc((n + 1) * 2);
  napi_get_value_string_utf16(env, v, (char16_t*)s, n + 1, &n);
  *len = n;
  return s;
}
static void set_num(napi_env env, napi_value o, const char* k, double x) {
  napi_value v;
  napi_create_double(env, x, &v);
  napi_set_named_property(env, o, k, v);
}
static napi_value stats_obj(napi_env env, const mtb_stats* st) {
  napi_value o;
  napi_create_object(env, &o);
  set_num(env, o, "opsApplied", (double)st->ops_applied);
  set_num(env, o, "docs", (double)st->docs);
  set_num(env, o, "segmentsFinal", (double)st->segments_final);
  set_num(env, o, "textUnitsFinal", (double)st->text_units_final);
  set_num(env, o, "bytesAlg", (double)st->bytes_alg);
  set_num(env, o, "errors", (double)st->errors);
  set_num(env, o, "kernelMs", st->kernel_ms);
  char hex[24];
  snprintf(hex, sizeof hex, "%016llx", (unsigned long long)st->checksum);
  napi_value h;
  napi_create_string_utf8(env, hex, NAPI_AUTO_LENGTH, &h);
  napi_set_named_property(env, o, "checksum", h);
  return o;
}

/* ---- entry points ---------------------------------------------------------------------------- */
static void batch_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  mtb_batch_destroy((mtb_batch*)data);
}

/* create(ndocs, newLengthCalc, chunkSize, device, flags?, deviceMask?) -> handle   client.ts:107 ctor */
static napi_value js_create(napi_env env, napi_callback_info info) {
  napi_value argv[6];
  size_t argc = 6;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 4) {
    napi_throw_type_error(env, NULL, "wrong number of arguments");
    return NULL;
  }
  uint32_t ndocs, nl, chunk, dev, flags = 0, mask = 0;
  if (!get_u32(env, argv[0], &ndocs) || !get_u32(env, argv[1], &nl) || !get_u32(env, argv[2], &chunk) ||
      !get_u32(env, argv[3], &dev) || (argc > 4 && !get_u32(env, argv[4], &flags)) ||
      (argc > 5 && !get_u32(env, argv[5], &mask)))
    return NULL;
  mtb_options o;
  memset(&o, 0, sizeof o);
  o.new_length_calc = (int32_t)nl;
  o.chunk_size = (int32_t)chunk;
  o.threads_per_doc = 64;
  o.flags = (int32_t)flags;
  mtb_batch* b = NULL;
  int rc = mtb_batch_create(&o, ndocs, mask ? mask : 1u << dev, &b);
  if (rc) return throw_rc(env, b, rc);
  napi_value h;
  CHECK_NAPI(env, napi_create_external(env, b, batch_finalize, NULL, &h));
  return h;
}

/* docInit(h, doc, initialText, observerLongId, minSeq, curSeq)         client.ts:1133 */
static napi_value js_doc_init(napi_env env, napi_callback_info info) {
  napi_value argv[6];
  if (!get_args(env, info, 6, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, mn, cur;
  if (!b || !get_u32(env, argv[1], &doc) || !get_u32(env, argv[4], &mn) || !get_u32(env, argv[5], &cur)) return NULL;
  size_t n = 0;
  uint16_t* text = get_utf16(env, argv[2], &n);
  if (!text) return NULL;
  char* id = get_utf8(env, argv[3], NULL);
  if (!id) {
    free(text);
    return NULL;
  }
  int rc = mtb_doc_init(b, doc, text, n, id, mn, cur);
  free(text);
  free(id);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* loadV1(h, doc, [[path, content], ...], observerLongId)               client.ts:1007, snapshotLoader.ts:41 */
static napi_value load_blobs(napi_env env, napi_callback_info info, int matrix);
static napi_value js_load_v1(napi_env env, napi_callback_info info) { return load_blobs(env, info, 0); }
/* matrixLoad(h, matrix, [[path, content], ...], observerLongId)          matrix.ts:611-634 */
static napi_value js_matrix_load(napi_env env, napi_callback_info info) { return load_blobs(env, info, 1); }
static napi_value load_blobs(napi_env env, napi_callback_info info, int matrix) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, n = 0;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  if (napi_get_array_length(env, argv[2], &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "expected an array of [path, content] pairs");
    return NULL;
  }
  mtb_blob* blobs = (mtb_blob*)calloc(n ? n : 1, sizeof(mtb_blob));
  char* id = NULL;
  int ok = 1;
  for (uint32_t i = 0; i < n && ok; i++) {
    napi_value pair, p, c;
    ok = napi_get_element(env, argv[2], i, &pair) == napi_ok && napi_get_element(env, pair, 0, &p) == napi_ok &&
         napi_get_element(env, pair, 1, &c) == napi_ok;
    if (!ok) {
      napi_throw_type_error(env, NULL, "expected [path, content]");
      break;
    }
    size_t len = 0;
    blobs[i].path = get_utf8(env, p, NULL);
    blobs[i].content = blobs[i].path ? get_utf8(env, c, &len) : NULL;
    blobs[i].content_len = len;
    ok = blobs[i].path && blobs[i].content;
  }
  int rc = 0;
  if (ok) {
    id = get_utf8(env, argv[3], NULL);
    if (id) rc = matrix ? mtb_matrix_load(b, doc, blobs, n, id) : mtb_doc_load_v1(b, doc, blobs, n, id);
    else ok = 0;
  }
  for (uint32_t i = 0; i < n; i++) {
    free((void*)blobs[i].path);
    free((void*)blobs[i].content);
  }
  free(blobs);
  free(id);
  if (!ok) return NULL;
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* matrixInit(h, matrix, observerLongId, minSeq, curSeq)                matrix.ts:102-118 */
static napi_value js_matrix_init(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t m, mn, cur;
  if (!b || !get_u32(env, argv[1], &m) || !get_u32(env, argv[3], &mn) || !get_u32(env, argv[4], &cur)) return NULL;
  char* id = get_utf8(env, argv[2], NULL);
  if (!id) return NULL;
  int rc = mtb_matrix_init(b, m, id, mn, cur);
  free(id);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* matrixApplyMsg(h, matrix, JSON.stringify(ISequencedDocumentMessage))  matrix.ts:636 */
static napi_value js_matrix_apply_msg(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t m;
  if (!b || !get_u32(env, argv[1], &m)) return NULL;
  size_t n = 0;
  char* json = get_utf8(env, argv[2], &n);
  if (!json) return NULL;
  int rc = mtb_matrix_apply_msg_json(b, m, json, n);
  free(json);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* applyMsg(h, doc, JSON.stringify(ISequencedDocumentMessage))          client.ts:858 */
static napi_value js_apply_msg(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  size_t n = 0;
  char* s = get_utf8(env, argv[2], &n);
  if (!s) return NULL;
  int rc = mtb_apply_msg_json(b, doc, s, n);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* localOp(h, doc, JSON.stringify(IMergeTreeOp)): a live client's own op     client.ts:196-247 */
static napi_value js_local_op(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  size_t n = 0;
  char* s = get_utf8(env, argv[2], &n);
  if (!s) return NULL;
  int rc = mtb_local_op_json(b, doc, s, n);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* detachedOp(h, doc, JSON.stringify(IMergeTreeOp)): an edit before collaboration (seq 0, LocalClientId) */
static napi_value js_detached_op(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  size_t n = 0;
  char* s = get_utf8(env, argv[2], &n);
  if (!s) return NULL;
  int rc = mtb_detached_op_json(b, doc, s, n);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* maintenance(h, doc, kind): 0 zamboniSegments, 1 packParent(root)              zamboni.ts:19-120 */
static napi_value js_maintenance(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, kind;
  if (!b || !get_u32(env, argv[1], &doc) || !get_u32(env, argv[2], &kind)) return NULL;
  int rc = mtb_maintenance(b, doc, kind);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* regeneratePendingOp(h, doc, JSON.stringify(resetOp)) -> JSON of the op(s) to resubmit   client.ts:917-960 */
static napi_value js_regenerate(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  size_t n = 0;
  char* s = get_utf8(env, argv[2], &n);
  if (!s) return NULL;
  char* out = NULL;
  size_t on = 0;
  int rc = mtb_regenerate_pending_op(b, doc, s, n, &out, &on);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  napi_value r;
  napi_status ok = napi_create_string_utf8(env, out, on, &r);
  mtb_free(out);
  CHECK_NAPI(env, ok);
  return r;
}

/* appendOps(h, doc, records: Uint8Array (32 B each), payload: Uint16Array) */
static napi_value js_append_ops(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  napi_typedarray_type t1, t2;
  size_t n1, n2, off;
  void *p1, *p2;
  napi_value ab;
  if (napi_get_typedarray_info(env, argv[2], &t1, &n1, &p1, &ab, &off) != napi_ok || t1 != napi_uint8_array ||
      n1 % sizeof(mtb_op) != 0 ||
      napi_get_typedarray_info(env, argv[3], &t2, &n2, &p2, &ab, &off) != napi_ok || t2 != napi_uint16_array) {
    napi_throw_type_error(env, NULL, "expected (Uint8Array records, Uint16Array payload)");
    return NULL;
  }
  int rc = mtb_append_ops(b, doc, (const mtb_op*)p1, (uint32_t)(n1 / sizeof(mtb_op)), (const uint16_t*)p2, n2);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* addClient(h, doc, longId) -> registers the next short id            client.ts:673 */
static napi_value js_add_client(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  char* s = get_utf8(env, argv[2], NULL);
  if (!s) return NULL;
  int rc = mtb_add_client(b, doc, s);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}

/* internProps(h, json) -> id */
static napi_value js_intern_props(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  if (!b) return NULL;
  size_t n = 0;
  char* s = get_utf8(env, argv[1], &n);
  if (!s) return NULL;
  uint32_t id = 0;
  int rc = mtb_intern_props(b, s, n, &id);
  free(s);
  if (rc) return throw_rc(env, b, rc);
  napi_value v;
  napi_create_uint32(env, id, &v);
  return v;
}

/* replay(h) -> stats (blocking) */
static napi_value js_replay(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  if (!b) return NULL;
  mtb_stats st;
  memset(&st, 0, sizeof st);
  int rc = mtb_replay(b, &st);
  if (rc) return throw_rc(env, b, rc);
  return stats_obj(env, &st);
}

/* replayAsync(h) -> Promise<stats>, mtb_replay on the libuv thread pool */
typedef struct {
  mtb_batch* b;
  napi_deferred deferred;
  napi_async_work work;
  mtb_stats st;
  int rc;
} ReplayJob;
static void replay_execute(napi_env env, void* data) {
  (void)env;
  ReplayJob* j = (ReplayJob*)data;
  memset(&j->st, 0, sizeof j->st);
  j->rc = mtb_replay(j->b, &j->st);
}
static void replay_complete(napi_env env, napi_status status, void* data) {
  ReplayJob* j = (ReplayJob*)data;
  if (status == napi_ok && j->rc == 0) {
    napi_resolve_deferred(env, j->deferred, stats_obj(env, &j->st));
  } else {
    napi_value m, e, code;
    napi_create_string_utf8(env, status == napi_ok ? mtb_last_error(j->b) : "replay cancelled", NAPI_AUTO_LENGTH, &m);
    napi_create_error(env, NULL, m, &e);
    napi_create_int32(env, j->rc, &code);
    napi_set_named_property(env, e, "code", code);
    napi_reject_deferred(env, j->deferred, e);
  }
  napi_delete_async_work(env, j->work);
  free(j);
}
static napi_value js_replay_async(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  if (!b) return NULL;
  ReplayJob* j = (ReplayJob*)calloc(1, sizeof(ReplayJob));
  j->b = b;
  napi_value promise, name;
  CHECK_NAPI(env, napi_create_promise(env, &j->deferred, &promise));
  napi_create_string_utf8(env, "mtb_replay", NAPI_AUTO_LENGTH, &name);
  CHECK_NAPI(env, napi_create_async_work(env, NULL, name, replay_execute, replay_complete, j, &j->work));
  CHECK_NAPI(env, napi_queue_async_work(env, j->work));
  return promise;
}

/* getText(h, doc) -> string                                            testClient.ts:185 */
static napi_value js_get_text(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  size_t n = 0;
  int rc = mtb_get_text(b, doc, NULL, 0, &n);
  if (rc) return throw_rc(env, b, rc);
  uint16_t* buf = (uint16_t*)malloc((n + 1) * 2);
  rc = mtb_get_text(b, doc, buf, n, &n);
  if (rc) {
    free(buf);
    return throw_rc(env, b, rc);
  }
  napi_value s;
  napi_status ok = napi_create_string_utf16(env, (const char16_t*)buf, n, &s);
  free(buf);
  CHECK_NAPI(env, ok);
  return s;
}

/* getLength(h, doc)                                                    client.ts:1129 */
static napi_value js_get_length(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, n = 0;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  int rc = mtb_get_length(b, doc, &n);
  if (rc) return throw_rc(env, b, rc);
  napi_value v;
  napi_create_uint32(env, n, &v);
  return v;
}

/* getSeq(h, doc) -> [currentSeq, minSeq]                               client.ts:1122, :348 */
static napi_value js_get_seq(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, cur = 0, mn = 0;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  int rc = mtb_get_seq(b, doc, &cur, &mn);
  if (rc) return throw_rc(env, b, rc);
  napi_value arr, v0, v1;
  napi_create_array_with_length(env, 2, &arr);
  napi_create_uint32(env, cur, &v0);
  napi_create_uint32(env, mn, &v1);
  napi_set_element(env, arr, 0, v0);
  napi_set_element(env, arr, 1, v1);
  return arr;
}

/* dumpSegments(h, doc) -> canonical segment dump (JSON lines) */
static napi_value js_dump_segments(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  char* out = NULL;
  size_t n = 0;
  int rc = mtb_dump_segments(b, doc, &out, &n);
  if (rc) return throw_rc(env, b, rc);
  napi_value s;
  napi_status ok = napi_create_string_utf8(env, out, n, &s);
  mtb_free(out);
  CHECK_NAPI(env, ok);
  return s;
}

/* mapRange(h, doc, start, end, refSeq, longClientId | null, limit) -> JSON text   mergeTree.ts:2456 */
static napi_value js_map_range(napi_env env, napi_callback_info info) {
  napi_value argv[7];
  if (!get_args(env, info, 7, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, limit;
  int64_t start, end, ref;
  if (!b || !get_u32(env, argv[1], &doc) || !get_i64(env, argv[2], &start) || !get_i64(env, argv[3], &end) ||
      !get_i64(env, argv[4], &ref) || !get_u32(env, argv[6], &limit))
    return NULL;
  napi_valuetype t;
  napi_typeof(env, argv[5], &t);
  char* id = NULL;
  if (t == napi_string) {
    id = get_utf8(env, argv[5], NULL);
    if (!id) return NULL;
  }
  char* out = NULL;
  size_t n = 0;
  int rc = mtb_map_range(b, doc, start, end, ref, id, limit, &out, &n);
  free(id);
  if (rc) return throw_rc(env, b, rc);
  napi_value s;
  napi_status ok = napi_create_string_utf8(env, out, n, &s);
  mtb_free(out);
  CHECK_NAPI(env, ok);
  return s;
}

/* checksum(h, doc) -> 16-digit hex string */
static napi_value js_checksum(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  if (!b || !get_u32(env, argv[1], &doc)) return NULL;
  uint64_t c = 0;
  int rc = mtb_doc_checksum(b, doc, &c);
  if (rc) return throw_rc(env, b, rc);
  char hex[24];
  snprintf(hex, sizeof hex, "%016llx", (unsigned long long)c);
  napi_value s;
  napi_create_string_utf8(env, hex, NAPI_AUTO_LENGTH, &s);
  return s;
}

/* summarizeV1(h, doc, msn, seq) -> {blobs: [[path, content]...], summary: JSON text}   client.ts:966 */
static napi_value blob_list_object(napi_env env, mtb_blob_list* lp);
static napi_value js_summarize_v1(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  int64_t msn, seq;
  if (!b || !get_u32(env, argv[1], &doc) || !get_i64(env, argv[2], &msn) || !get_i64(env, argv[3], &seq)) return NULL;
  mtb_blob_list l;
  memset(&l, 0, sizeof l);
  int rc = mtb_summarize_v1(b, doc, msn, seq, &l);
  if (rc) return throw_rc(env, b, rc);
  return blob_list_object(env, &l);
}

/* summarizeV1Many(h, docs: number[], msn, seq, threads) -> [{blobs, summary}]: many channels at once */
static napi_value js_summarize_v1_many(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  int64_t msn, seq;
  uint32_t threads, n = 0;
  if (!b || !get_i64(env, argv[2], &msn) || !get_i64(env, argv[3], &seq) || !get_u32(env, argv[4], &threads)) return NULL;
  CHECK_NAPI(env, napi_get_array_length(env, argv[1], &n));
  uint32_t* docs = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
  mtb_blob_list* ls = (mtb_blob_list*)calloc(n ? n : 1, sizeof(mtb_blob_list));
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    if (napi_get_element(env, argv[1], i, &e) != napi_ok || !get_u32(env, e, &docs[i])) {
      free(docs);
      free(ls);
      return NULL;
    }
  }
  int rc = mtb_summarize_v1_many(b, n, docs, msn, seq, threads, ls);
  free(docs);
  if (rc) {
    /* the documents (and shards) that succeeded filled their lists before the call failed */
    for (uint32_t i = 0; i < n; i++)
      if (ls[i].count || ls[i].blobs || ls[i].summary_json) mtb_blob_list_free(&ls[i]);
    free(ls);
    return throw_rc(env, b, rc);
  }
  napi_value arr;
  napi_create_array_with_length(env, n, &arr);
  for (uint32_t i = 0; i < n; i++) napi_set_element(env, arr, i, blob_list_object(env, &ls[i]));
  free(ls);
  return arr;
}

/* digests(h, first, n) -> 16-digit hex strings: per-document state digests (mtb_doc_digests) */
static napi_value js_digests(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t first, n;
  if (!b || !get_u32(env, argv[1], &first) || !get_u32(env, argv[2], &n)) return NULL;
  uint64_t* d = (uint64_t*)calloc(n ? n : 1, sizeof(uint64_t));
  int rc = mtb_doc_digests(b, first, n, d);
  if (rc) {
    free(d);
    return throw_rc(env, b, rc);
  }
  napi_value arr;
  napi_create_array_with_length(env, n, &arr);
  for (uint32_t i = 0; i < n; i++) {
    char hex[24];
    snprintf(hex, sizeof hex, "%016llx", (unsigned long long)d[i]);
    napi_value s;
    napi_create_string_utf8(env, hex, NAPI_AUTO_LENGTH, &s);
    napi_set_element(env, arr, i, s);
  }
  free(d);
  return arr;
}

/* summarizeLegacy(h, doc, msn, seq, catchupJson | null) -> {blobs, summary}   client.ts:999-1003,
 * snapshotlegacy.ts:122-259; null catch-up = the messages the batch tracked (MTB_BATCH_CATCHUP) */
static napi_value js_summarize_legacy(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc;
  int64_t msn, seq;
  if (!b || !get_u32(env, argv[1], &doc) || !get_i64(env, argv[2], &msn) || !get_i64(env, argv[3], &seq)) return NULL;
  napi_valuetype t;
  napi_typeof(env, argv[4], &t);
  char* cu = NULL;
  size_t cul = 0;
  if (t == napi_string) {
    cu = get_utf8(env, argv[4], &cul);
    if (!cu) return NULL;
  }
  mtb_blob_list l;
  memset(&l, 0, sizeof l);
  int rc = mtb_summarize_legacy(b, doc, msn, seq, cu, cul, &l);
  free(cu);
  if (rc) return throw_rc(env, b, rc);
  return blob_list_object(env, &l);
}

/* matrixSummarize(h, matrix) -> {blobs, summary}                        matrix.ts:449-463 */
static napi_value js_matrix_summarize(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t m;
  if (!b || !get_u32(env, argv[1], &m)) return NULL;
  mtb_blob_list l;
  memset(&l, 0, sizeof l);
  int rc = mtb_matrix_summarize(b, m, &l);
  if (rc) return throw_rc(env, b, rc);
  return blob_list_object(env, &l);
}

/* matrixGetCell(h, matrix, row, col) -> JSON text | undefined           matrix.ts:173-189 */
static napi_value js_matrix_get_cell(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t m, r, c;
  if (!b || !get_u32(env, argv[1], &m) || !get_u32(env, argv[2], &r) || !get_u32(env, argv[3], &c)) return NULL;
  size_t n = 0;
  int rc = mtb_matrix_get_cell(b, m, r, c, NULL, 0, &n);
  if (rc) return throw_rc(env, b, rc);
  if (n == 0) return undef(env);
  char* buf = (char*)malloc(n + 1);
  rc = mtb_matrix_get_cell(b, m, r, c, buf, n + 1, &n);
  if (rc) {
    free(buf);
    return throw_rc(env, b, rc);
  }
  napi_value v;
  napi_create_string_utf8(env, buf, n, &v);
  free(buf);
  return v;
}

/* {blobs: [[path, content]...], summary: JSON text}; frees the list */
static napi_value blob_list_object(napi_env env, mtb_blob_list* lp) {
  mtb_blob_list l = *lp;
  napi_value o, arr, sum;
  napi_create_object(env, &o);
  napi_create_array_with_length(env, l.count, &arr);
  for (uint32_t i = 0; i < l.count; i++) {
    napi_value pair, p, c;
    napi_create_array_with_length(env, 2, &pair);
    napi_create_string_utf8(env, l.blobs[i].path, NAPI_AUTO_LENGTH, &p);
    napi_create_string_utf8(env, l.blobs[i].content, l.blobs[i].content_len, &c);
    napi_set_element(env, pair, 0, p);
    napi_set_element(env, pair, 1, c);
    napi_set_element(env, arr, i, pair);
  }
  napi_create_string_utf8(env, l.summary_json, l.summary_json_len, &sum);
  napi_set_named_property(env, o, "blobs", arr);
  napi_set_named_property(env, o, "summary", sum);
  mtb_blob_list_free(lp);
  return o;
}

/* rewind(h) / replayResident(h) -> stats: benchmark re-replay utilities */
static napi_value js_rewind(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  if (!b) return NULL;
  int rc = mtb_rewind(b);
  if (rc) return throw_rc(env, b, rc);
  return undef(env);
}
static napi_value js_replay_resident(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  if (!b) return NULL;
  mtb_stats st;
  memset(&st, 0, sizeof st);
  int rc = mtb_replay_resident(b, &st);
  if (rc) return throw_rc(env, b, rc);
  return stats_obj(env, &st);
}

/* clientLongId(h, doc, shortId)                                        client.ts:682 */
static napi_value js_client_long_id(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mtb_batch* b = get_batch(env, argv[0]);
  uint32_t doc, sid;
  if (!b || !get_u32(env, argv[1], &doc) || !get_u32(env, argv[2], &sid)) return NULL;
  size_t n = 0;
  int rc = mtb_client_long_id(b, doc, sid, NULL, 0, &n);
  if (rc) return throw_rc(env, b, rc);
  char* buf = (char*)malloc(n + 1);
  rc = mtb_client_long_id(b, doc, sid, buf, n + 1, &n);
  if (rc) {
    free(buf);
    return throw_rc(env, b, rc);
  }
  napi_value s;
  napi_create_string_utf8(env, buf, n, &s);
  free(buf);
  return s;
}

static napi_value init(napi_env env, napi_value exports) {
  static const struct {
    const char* name;
    napi_callback fn;
  } fns[] = {
      {"create", js_create},           {"docInit", js_doc_init},       {"loadV1", js_load_v1},
      {"matrixInit", js_matrix_init},  {"matrixApplyMsg", js_matrix_apply_msg},
      {"matrixSummarize", js_matrix_summarize}, {"matrixGetCell", js_matrix_get_cell},
      {"matrixLoad", js_matrix_load},  {"summarizeLegacy", js_summarize_legacy},
      {"applyMsg", js_apply_msg},      {"appendOps", js_append_ops},
      {"localOp", js_local_op},        {"summarizeV1Many", js_summarize_v1_many},
      {"detachedOp", js_detached_op},  {"maintenance", js_maintenance},
      {"digests", js_digests},
      {"addClient", js_add_client},    {"internProps", js_intern_props},
      {"replay", js_replay},           {"replayAsync", js_replay_async},
      {"getText", js_get_text},        {"getLength", js_get_length},
      {"getSeq", js_get_seq},          {"dumpSegments", js_dump_segments},
      {"mapRange", js_map_range},      {"regeneratePendingOp", js_regenerate},
      {"checksum", js_checksum},       {"summarizeV1", js_summarize_v1},
      {"rewind", js_rewind},           {"replayResident", js_replay_resident},
      {"clientLongId", js_client_long_id},
  };
  for (size_t i = 0; i < sizeof fns / sizeof fns[0]; i++) {
    napi_value f;
    CHECK_NAPI(env, napi_create_function(env, fns[i].name, NAPI_AUTO_LENGTH, fns[i].fn, NULL, &f));
    CHECK_NAPI(env, napi_set_named_property(env, exports, fns[i].name, f));
  }
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
