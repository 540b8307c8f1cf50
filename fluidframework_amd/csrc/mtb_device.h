// Device-side data layout of the MI355X merge-tree batch replay engine.
//
// Every document owns disjoint slices of a few batch-wide pools in HBM (structure of arrays per
// node type, array of structures per node so one wave-instruction fetches a whole record):
//   segs   : Seg  (32 B)  leaf segments           (reference: BaseSegment, mergeTreeNodes.ts:367)
//   blks   : Blk  (64 B)  internal blocks          (reference: MergeBlock, mergeTreeNodes.ts:332)
//   lists  : WEnt (16 B)  per-block window lists   (replaces PartialSequenceLengths, partialLengths.ts:239)
//   text   : u16          per-document UTF-16 text arena (insert payloads + zamboni appends)
//   heap   : Lru  (8 B)   zamboni LRU heap         (reference: Heap<LRUSegment>, collections/heap.ts)
//   aux    : u32          property sets and overlapping-remove client lists
//   freel  : u32          free-block stack
// A DocState header (256 B) holds each document's slice bases, bump pointers and collab window.
#pragma once
#include <stdint.h>

#define MTB_NONE 0xFFFFFFFFu
#define MTB_LEAF 0x80000000u
#define MTB_MAXCH 8          // MaxNodesInBlock (mergeTreeNodes.ts:330)
#define MTB_MAXDEPTH 24
#define MTB_UNDEF (-1)
#define MTB_MARKER 0x80000000u  // Seg.text flag: marker, low bits = refType + 1 (0 = undefined)
#define MTB_GPROPS 0x80000000u  // props handle flag: batch-global table (else per-doc aux arena)

struct Seg {          // 32 bytes
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

struct Blk {          // 64 bytes
  uint32_t child[MTB_MAXCH];  // MTB_LEAF | seg id, or block id
  uint32_t parent;
  int32_t len;        // cachedLength: observer-view length (mergeTree.ts:2392 blockUpdate)
  uint32_t loff;      // window list: offset / count / capacity in the doc's list slice
  uint32_t lcnt;
  uint32_t lcap;
  uint8_t count;      // childCount
  uint8_t index;      // index in parent
  int8_t scour;       // needsScour: -1 undefined, 0 false, 1 true
  uint8_t pad0;
  int32_t lseq;       // key (seq, ck) of the list's last entry, so appends can merge without a
  int32_t lck;        //   dependent load of the entry (lseq = INT32_MIN: unknown, never merge)
};

// Window-list entry.  For a query (R, C):  length(block) = len - sum(w(e) for e.seq > R), where
// w = delta if (kind == MAIN && client != C) or (kind == OVERLAP && client == C), else 0.
struct WEnt {
  int32_t seq;
  int32_t ck;         // client | (kind << 16)
  int32_t delta;
  int32_t pad;
};
#define WK_MAIN 0
#define WK_OVERLAP 1

struct Lru {
  uint32_t seg;
  int32_t maxSeq;
};

struct DocState {     // 256 bytes
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
  uint32_t pad[10];
};

// Batch-global interned tables (read-only on the device).
struct Tables {
  const uint32_t* pool;      // u32 pool: op-props lists [n, (key, val)*n] (val MTB_NONE = null/delete)
                             //           and property sets [n, (key, val)*n]
  const uint32_t* pidx;      // props id i -> pidx[2i] = op-props list offset, pidx[2i+1] = property set offset
  const uint32_t* val_class; // matchProperties equivalence class of each value id
  const uint8_t* val_falsy;  // JS falsiness of each value id
  const uint32_t* key_rank;  // array-index keys: numeric value; other keys: MTB_NONE
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
