// Internal interface between the public C ABI (mtb_multi.cpp: a batch spread over one or more devices)
// and the per-device engine (mtb_host.cpp: one device, its HBM pools and stream).  Each mtbx_* function
// is the per-device implementation of the include/mtb.h entry point of the same name.
#pragma once
#include "../../include/mtb.h"

typedef struct mtb_dev mtb_dev;

#ifdef __cplusplus
extern "C" {
#endif
int mtbx_batch_create(const mtb_options* opts, uint32_t ndocs, uint32_t device_mask, mtb_dev** out);
void mtbx_batch_destroy(mtb_dev* b);
const char* mtbx_last_error(mtb_dev* b);
int mtbx_doc_init(mtb_dev* b, uint32_t doc, const uint16_t* initial_text, size_t n_units,
                 const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq);
int mtbx_doc_load_v1(mtb_dev* b, uint32_t doc, const mtb_blob* blobs, uint32_t nblobs,
                    const char* observer_long_id);
int mtbx_docs_load_v1(mtb_dev* b, uint32_t n, const uint32_t* docs, const mtb_blob* const* blobs,
                     const uint32_t* nblobs, const char* const* observer_long_ids, uint32_t threads);
int mtbx_apply_msg_json(mtb_dev* b, uint32_t doc, const char* json_utf8, size_t len);
int mtbx_local_op_json(mtb_dev* b, uint32_t doc, const char* json_utf8, size_t len);
int mtbx_detached_op_json(mtb_dev* b, uint32_t doc, const char* json_utf8, size_t len);
int mtbx_maintenance(mtb_dev* b, uint32_t doc, uint32_t kind);
int mtbx_regenerate_pending_op(mtb_dev* b, uint32_t doc, const char* json, size_t len, char** out, size_t* out_len);
int mtbx_append_ops(mtb_dev* b, uint32_t doc, const mtb_op* ops, uint32_t n,
                   const uint16_t* payload, size_t payload_len);
int mtbx_add_client(mtb_dev* b, uint32_t doc, const char* long_id);
int mtbx_intern_props(mtb_dev* b, const char* json_utf8, size_t len, uint32_t* id_out);
int mtbx_matrix_init(mtb_dev* b, uint32_t matrix, const char* observer_long_id, uint32_t min_seq, uint32_t cur_seq);
int mtbx_matrix_apply_msg_json(mtb_dev* b, uint32_t matrix, const char* json_utf8, size_t len);
int mtbx_matrix_intern_value(mtb_dev* b, const char* json_utf8, size_t len, uint32_t* id_out);
int mtbx_matrix_load(mtb_dev* b, uint32_t matrix, const mtb_blob* blobs, uint32_t nblobs, const char* observer_long_id);
int mtbx_matrix_summarize(mtb_dev* b, uint32_t matrix, mtb_blob_list* out);
int mtbx_matrix_get_cell(mtb_dev* b, uint32_t matrix, uint32_t row, uint32_t col, char* buf, size_t cap,
                        size_t* len_out);
int mtbx_replay(mtb_dev* b, mtb_stats* out);
int mtbx_get_text(mtb_dev* b, uint32_t doc, uint16_t* buf, size_t cap, size_t* len_out);
int mtbx_get_length(mtb_dev* b, uint32_t doc, uint32_t* len_out);
int mtbx_test_set_root_child(mtb_dev* b, uint32_t doc, uint32_t value, uint32_t* old_out);
int mtbx_get_seq(mtb_dev* b, uint32_t doc, uint32_t* cur_seq, uint32_t* min_seq);
int mtbx_dump_segments(mtb_dev* b, uint32_t doc, char** out, size_t* out_len);
int mtbx_doc_checksum(mtb_dev* b, uint32_t doc, uint64_t* out);
int mtbx_doc_digests(mtb_dev* b, uint32_t first, uint32_t n, uint64_t* out);
int mtbx_get_launch_info(mtb_dev* b, mtb_launch_info* out);
int mtbx_debug_blocks(mtb_dev* b, uint32_t doc, int64_t ref_seq, const char* long_client_id, char** out,
                      size_t* out_len);
int mtbx_map_range(mtb_dev* b, uint32_t doc, int64_t start, int64_t end, int64_t ref_seq,
                  const char* long_client_id, uint32_t limit, char** out, size_t* out_len);
int mtbx_summarize_v1(mtb_dev* b, uint32_t doc, int64_t msn, int64_t seq,
                     mtb_blob_list* out);
int mtbx_summarize_v1_many(mtb_dev* b, uint32_t n, const uint32_t* docs, int64_t msn, int64_t seq, uint32_t threads,
                          mtb_blob_list* out);
int mtbx_summarize_legacy(mtb_dev* b, uint32_t doc, int64_t msn, int64_t seq, const char* catchup_json,
                         size_t catchup_len, mtb_blob_list* out);
int mtbx_rewind(mtb_dev* b);
int mtbx_replay_resident(mtb_dev* b, mtb_stats* out, uint32_t flags = 0);
int mtbx_refresh_digests(mtb_dev* b, mtb_stats* out);
int mtbx_export_pending(mtb_dev* b, uint32_t doc, mtb_op* ops, uint32_t cap, uint32_t* n_out,
                       uint16_t* payload, size_t pcap, size_t* plen_out);
int mtbx_props_json(mtb_dev* b, uint32_t id, char* buf, size_t cap, size_t* len_out);
int mtbx_client_long_id(mtb_dev* b, uint32_t doc, uint32_t short_id, char* buf, size_t cap, size_t* len_out);
#ifdef __cplusplus
}
#endif
