/* Test hooks of libmtb.so: not part of the drop-in boundary (include/mtb.h), no reference counterpart.
 * They let the parity tests put the engine into states that valid input never produces. */
#ifndef MTB_TESTING_H
#define MTB_TESTING_H
#include "mtb.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Overwrite the block child id in the last slot of the document's root block with `value` (old id in
 * *old_out; value 0xFFFFFFFE = the root's own id): an out-of-slice id or the root's own id (a cycle) makes
 * the device extraction walk refuse the tree (tests/test_gpu_summary_guard.py).  Write the old id back to
 * repair it. */
int mtb_test_set_root_child(mtb_batch* b, uint32_t doc, uint32_t value, uint32_t* old_out);

#ifdef __cplusplus
}
#endif
#endif
