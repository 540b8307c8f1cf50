// MI355X (gfx950) batched merge-tree replay kernel.
//
// One 64-lane wavefront owns one document and applies that document's sequenced ops in order,
// exactly as the reference observer `Client.applyMsg` would (packages/dds/merge-tree/src/client.ts:858).
// Control flow is wave-uniform (every lane walks the same tree path); the lanes parallelise the
// per-op inner loops: the <=8 children of a block, the block's window list, the segments of a
// leaf-level block touched by a remove / annotate, scour decisions, list rebuilds and text copies.
// No MFMA: nothing here is a contraction.
//
// Data structures (mtb_device.h) and how they differ from the reference (results are identical):
//  * A tree node is one 320-byte record holding its children's hot fields inline (segment: length,
//    seq, removal info, props, text; block: cachedLength and the child's window-list metadata), so a
//    walk fetches one record per level and never touches a separate segment record.
//  * PartialSequenceLengths (partialLengths.ts:239) is replaced by slot-tagged window lists: block B's
//    list holds, for each of B's block children, the (seq, client, kind, delta) changes below it.  The
//    length of B's child k in the (refSeq R, client C) perspective is
//        childLen[k] - sum_{e in list(B), e.slot == k, e.seq > R} w(e)
//    with w(e) = e.delta for MAIN entries of other clients and for OVERLAP entries of C -- the quantity
//    getPartialLength (partialLengths.ts:698) returns, equal to the sum of the leaf visibilities
//    (mergeTree.ts:916-1004); the oracle verifies that identity on every query.  Blocks whose
//    children are segments need no list: their children's visibility is computed directly.  A block's
//    list metadata lives in its parent's slot, so a block and its list are fetched together.
//  * The recursive insertingWalk (mergeTree.ts:1740) and depthFirstNodeWalk (mergeTreeNodeWalk.ts:35)
//    run iteratively; every block an op visits is cached in LDS per tree depth ("view") together with
//    its children's lengths in the op's (R, C) perspective, and all walks of one op share the cache.
//  * Length/list bookkeeping is applied incrementally along the cached path instead of the
//    reference's combine/update rebuilds; split, root growth and packParent rebuild the lists of the
//    blocks whose children changed.
//  * The zamboni LRU heap (collections/heap.ts) lives in LDS while it fits.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <algorithm>

#include "../../include/mtb.h"
#include "mtb_device.h"

// The kernels are compiled in groups (build.py compiles this file once per group, in parallel, with
// -DMTB_TU=g; MTB_TU 0 or undefined = every kernel in one translation unit).  Each group instantiates the
// engine for its own variants only.
#ifndef MTB_TU
#define MTB_TU 0
#endif
#define MTB_TU_HAS(g) (MTB_TU == 0 || MTB_TU == (g))
#define MTB_TU_OBS 1      // observer replay: one wave per document, ticket-scheduled, few documents
#define MTB_TU_LIVE 2     // live clients
#define MTB_TU_MARKERS 3  // marker ids / relative positions
#define MTB_TU_LOADMAT 4  // SnapshotV1 body load, SharedMatrix
#define MTB_TU_MISC 5     // digest, rewind, moves, launch dispatch
#define MTB_TU_FEW 6      // the few-document kernel (its own code-generation flags, build.py GROUP_FLAGS)

namespace mtbk {
// matchProperties(va, vb) (properties.ts:84-92) of two values of key k, with irregular keys in the batch
// (Tables::key_irr; a regular key's values compare by class)
__device__ __forceinline__ bool irr_value_match(const Tables& t, uint32_t k, uint32_t va, uint32_t vb) {
  // NaN and consensus values (val_falsy bit 3) never match as the second argument; as the first, NaN (falsy: no own
  // keys) matches an object or array without own keys (bit 4), a consensus value nothing (cv-like values refused)
  if (t.val_falsy[vb] & 8) return false;
  if (t.val_falsy[va] & 8) return va == (t.nan_val & ~MTB_NAN_CV) && (t.val_falsy[vb] & 16) != 0;
  const uint32_t o = t.key_irr[k];
  if (!o) return va == vb || t.val_class[va] == t.val_class[vb];
  const uint32_t n = t.irr[o - 1];
  const uint32_t bit = t.val_local[va] * n + t.val_local[vb];
  return ((t.irr[o + bit / 32] >> (bit % 32)) & 1u) != 0;
}

// MTB_PROFILE builds accumulate s_memtime cycles per replay phase and event counts into DocState
// (diagnostic only; `MTB_PROFILE_OUT=1` prints them per op).
#ifdef MTB_PROFILE
#define PROF_T() ((uint64_t)__builtin_amdgcn_s_memtime())
#define PROF_ADD(i, t0) (prof[i] += PROF_T() - (t0))
#define PROF_CNT(i, n) ((i) < NCN ? (void)(evc[(i) < NCN ? (i) : 0] += (n)) : (void)0)
#ifdef MTB_PROFILE_PACK  // the heap / stage / place slots time packParent's staging, scour and placement instead
#define PROF_ZADD(i, t0) ((void)(t0))
#define PROF_PADD(i, t0) PROF_ADD(i, t0)
#else
#define PROF_ZADD(i, t0) PROF_ADD(i, t0)
#define PROF_PADD(i, t0) ((void)(t0))
#endif
#else
#define PROF_T() ((uint64_t)0)
#define PROF_ADD(i, t0) ((void)(t0))
#define PROF_CNT(i, n) ((void)0)
#define PROF_ZADD(i, t0) ((void)(t0))
#define PROF_PADD(i, t0) ((void)(t0))
#endif
enum { PH_BOUNDARY = 0, PH_INSERT = 1, PH_NODEMAP = 2, PH_ZAMBONI = 3, PH_TOTAL = 4, PH_VIEW = 5, PH_SCOUR = 6, PH_HEAP = 7,
       PH_STAGE = 8, PH_PLACE = 9, PH_PACK = 10, NPH = 11 };
enum { CN_SCOUR = 0, CN_PACK = 1, CN_REBUILD = 2, CN_VIEW = 3, CN_ENTRIES = 4, CN_ZCALL = 5, CN_POP = 6, CN_PSKIP = 7, CN_PSIG = 8,
       NCN = 9, CN_SPLIT = 99, CN_GROW = 99, CN_ZRECORD = 99 };

#ifndef MTB_LDS_HEAP
#define MTB_LDS_HEAP 128        // LRU heap entries kept in LDS by the batch kernels (more spill to HBM)
#endif
#define MTB_LDS_HEAP_LONG 2048  // ... by the few-document kernel (long documents keep big heaps)
#define MTB_VDEPTH 12  // depth of the LDS path cache; 4^12 segments per document is far beyond any input

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// Cross-lane hand-off inside the single wave that owns a document.  A wavefront's vector-memory and
// LDS instructions are performed in program order for the whole wave, so a wavefront-scope fence
// (no instruction; it only stops the compiler from moving memory operations across it) is enough
// to make one lane's store visible to another lane's later load of the same document state.
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// MTB_CRUMBS builds (fault triage only): every scheduled ticket leaves breadcrumbs in host-pinned memory, which the
// host can still read after a device fault has killed the context: crumbs[d] = stage | chunk << 8 (1 ticket taken,
// 2 replaying, 3 replayed, 4 progress published), crumbs[ndocs + d] = the record the document's wave is applying.
#ifdef MTB_CRUMBS
__device__ uint32_t* mtb_crumbs;
#define CRUMB(i, v) \
  do { if (lane_id() == 0) __hip_atomic_store(mtb_crumbs + (i), (uint32_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#else
#define CRUMB(i, v) ((void)0)
#endif

// Cross-lane primitives.  Every scan / sum in this kernel runs over the <=8 children of one block,
// i.e. lanes 0..7 of DPP row 0, so it is three DPP row_shr steps (plain VALU, no LDS round trip);
// values are read from a uniform lane with v_readlane (SGPR result) instead of ds_bpermute.
template <int CTRL>
__device__ __forceinline__ int dpp_shr_t(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);  // bound_ctrl: out-of-row source -> 0
}
// inclusive scan over lanes 0..7 (lanes >= count must hold 0)
__device__ __forceinline__ int cscan8(int v) {
  v += dpp_shr_t<0x111>(v);  // row_shr:1
  v += dpp_shr_t<0x112>(v);  // row_shr:2
  v += dpp_shr_t<0x114>(v);  // row_shr:4
  return v;
}
__device__ __forceinline__ int rl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ uint32_t rlu(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }
__device__ __forceinline__ int csum8(int v) { return rl(cscan8(v), 7); }
// Uniform values read from LDS or from a wave-uniform global address: readfirstlane moves them to
// SGPRs, so they cost no VGPR and branches on them stay scalar.
__device__ __forceinline__ int U(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t U(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
// Pointers kept in LDS or picked by a condition lose their address space and compile to flat_load /
// flat_store, which also count against lgkmcnt (every LDS wait then waits for them): GP() names the
// global address space explicitly, UP() also makes the pointer uniform.
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
using lptr = __attribute__((address_space(3))) T*;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ gptr<T> GP(T* p) { return (gptr<T>)p; }
template <class T>
__device__ __forceinline__ gptr<T> UP(T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = U((uint32_t)v), hi = U((uint32_t)(v >> 32));
  return (gptr<T>)(((uint64_t)hi << 32) | lo);
}
// number of set bits of m below this lane
__device__ __forceinline__ uint32_t rank_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int first_set(unsigned long long m) { return __ffsll((long long)m) - 1; }
// Branch hints: block splits, packParent, list re-allocation, overlapping removes, heap spills and errors
// are rare; marking them lets the register allocator place spill code on those paths.
#define COLD(x) __builtin_expect(!!(x), 0)
#define HOT(x) __builtin_expect(!!(x), 1)

__device__ __forceinline__ int cli_client(uint32_t cli) { return (int)(int16_t)(cli & 0xFFFF); }
__device__ __forceinline__ int cli_rc0(uint32_t cli) { return (int)(int16_t)(cli >> 16); }

// One block cached per tree depth: its record and its children's lengths in the op's (R, C) view.
struct View {
  uint32_t b;       // block id (MTB_NONE: empty)
  int32_t count;
  int32_t scour;
  int32_t len;
  uint32_t parent;
  int32_t rlv;      // rl[] valid
  int32_t pad[2];
  uint32_t f[8][MTB_MAXCH];
  int32_t rl[MTB_MAXCH];
};
// A block record staged for zamboni / rebuild.
struct Rec {
  uint32_t f[8][MTB_MAXCH];
  int32_t count;
  uint32_t parent;
  uint32_t index;
  int32_t scour;
};

template <int HEAPN>
#ifndef MTB_SORT_MIN
#define MTB_SORT_MIN 64  // rebuilt lists longer than this are counting-sorted (shorter ones are read whole)
#endif
#ifndef MTB_LSTK
#define MTB_LSTK 8    // capacity classes with an LDS stack of free lists
#endif
#ifndef MTB_LSTK_N
#define MTB_LSTK_N 4  // lists per stack
#endif
struct ScratchT {  // LDS, one per wave
  View v[MTB_VDEPTH];
  uint32_t path[MTB_VDEPTH];   // block at each depth of the current walk
  int32_t slot[MTB_VDEPTH];    // child slot taken at each depth
  int32_t pp[MTB_VDEPTH];      // remaining position at each depth of the last walk
  int32_t sidx[MTB_VDEPTH];    // node_map cursor
  int32_t acc[MTB_VDEPTH];     // node_map accumulated observer-length delta
  uint32_t rmeta[4];           // root window-list metadata (loff, lcnt, lcap)
  uint32_t lfree[MTB_LCLASSES];  // free window lists per capacity class (8 << c entries)
  uint32_t capv[8];              // the document's slice capacities (DocState seg, blk, list, text, heap, aux
                                 // caps, delta_cap): an allocation's bound check reads LDS, not HBM
#ifndef MTB_NO_LSTK
  uint32_t lstk[MTB_LSTK][MTB_LSTK_N];  // the last lists freed in the small classes, held in LDS: a pop
  uint32_t lstkn[MTB_LSTK];             // from here needs no dependent read of the next pointer in HBM
#endif
  int32_t corr[MTB_MAXCH];
  uint32_t nseg[8];            // staged fields of a child being inserted
  uint32_t sp[8];              // split_block results: cachedLength and list metadata of both halves
  int32_t ins[4];              // the segment placed by the last insert walk: block, slot, depth, needsScour
  uint32_t memo[3];            // per-op annotate memo: old props -> new props; [2] MODE_LIVE: overtaken blocks
  Tables tab;                  // batch-wide property tables
  Lru* gheap;                  // the document's global LRU heap slice
  uint32_t* gfree;             // free-block stack
  uint16_t* gtext;             // UTF-16 text arena
  Rec zr;                      // zamboni / pack / rebuild record
  union {
    Rec pr[MTB_MAXCH];         // scour inputs: the block(s) being scoured (packParent: all siblings)
    uint32_t hold[8][64];      // scour output: kept children, [field][i] (inputs are in registers by then)
    struct {
      uint32_t pk[64];         // props edit scratch (annotate; never live during a scour)
      uint32_t pv[64];
    };
  };
  alignas(16) Lru heap[HEAPN];  // LRU heap while it fits (index 0 unused; 16-byte child-pair reads)
};

using Scratch = ScratchT<MTB_LDS_HEAP>;
using ScratchBig = ScratchT<MTB_LDS_HEAP_LONG>;

// cold uniform state kept in LDS (frees scalar registers on the hot path)
#define sp_lenL sh->sp[0]
#define sp_lenR sh->sp[1]
#define sp_loffL sh->sp[2]
#define sp_lcntL sh->sp[3]
#define sp_lcapL sh->sp[4]
#define sp_loffR sh->sp[5]
#define sp_lcntR sh->sp[6]
#define sp_lcapR sh->sp[7]
#define ins_blk sh->ins[0]
#define ins_slot sh->ins[1]
#define ins_depth sh->ins[2]
#define ins_scour sh->ins[3]
#define memo_old sh->memo[0]
#define memo_new sh->memo[1]

// MTB_CHECK builds (diagnostic only): the engine's slice pointers are bounds-checked against the document's
// capacities (sh->capv); an index past its slice is replaced by 0 and reported in DocState.pad3 [count, index,
// capacity, pool (0 segp, 1 blk, 2 lst, 3 aux)], which the host prints with MTB_CHECK_OUT=1.
#ifdef MTB_CHECK
template <class T>
struct CP {
  T* p;
  const uint32_t* cap;  // LDS
  uint32_t* rep;        // DocState.pad3
  uint32_t pool;
  __device__ CP() : p(nullptr), cap(nullptr), rep(nullptr), pool(0) {}
  __device__ T& operator[](uint32_t i) const {
    const uint32_t c = *cap;
    if (COLD(i >= c)) {
      if (atomicAdd(rep, 1u) == 0) {
        rep[1] = i;
        rep[2] = c;
        rep[3] = pool;
      }
      i = 0;
    }
    return p[i];
  }
  __device__ operator T*() const { return p; }
};
#define SLICE(T) CP<T>
#define RAW(x) ((x).p)
#else
#define SLICE(T) T*
#define RAW(x) (x)
#endif

// Engine variants: MODE_REPLAY (mtb_replay_kernel); MODE_LOAD applies only the LOADSEG records at
// the head of each document's records (mtb_load_kernel); MODE_MATRIX replays SharedMatrix vector pairs
// with setCell handle allocation (mtb_matrix_kernel); MODE_LIVE is MODE_REPLAY plus the local ops, acks and
// pending segment groups of live clients (mtb_live_kernel); MODE_MARKERS is MODE_REPLAY
// plus marker ids and marker-relative positions (mtb_markers_kernel, for batches whose documents met a
// marker id).  Each variant carries only its own code.
// MODE_LOADPERM is MODE_LOAD for PermutationVector documents (a SharedMatrix summary with body chunks).
enum { MODE_REPLAY = 0, MODE_LOAD = 1, MODE_MATRIX = 2, MODE_LIVE = 3, MODE_MARKERS = 4, MODE_LOADPERM = 5 };
template <int MODE, class SCR>
struct Eng {
  DocState* ds;
  SLICE(uint32_t) segp;  // parent block of each segment
  SLICE(FBlk) blk;
  SLICE(WEnt) lst;
  SLICE(uint32_t) aux;
  SCR* sh;
  static constexpr uint32_t lheap_n = sizeof(SCR::heap) / sizeof(Lru);  // LDS heap capacity
  int lane;
  // uniform document state (mirrors DocState)
  int minSeq, curSeq;
  uint32_t root;
  bool newMode;
  bool hasNL;
  uint32_t seg_used, blk_used, free_top, list_used, text_used, heap_cnt, aux_used;
  int err;
  uint32_t n_mod, ops_applied, text_bytes;  // this launch's counts (added to DocState at the end)
  bool heap_lds;                // LRU heap lives in LDS (spills to the global slice when it outgrows it)
  int walk_depth;               // depth of the leaf-level block reached by the last walk (-1: none)
  uint32_t vmask;               // bit d: the LDS view of depth d may hold a fetched record (else it is empty)
  bool struct_changed;          // a block split / root growth happened since the last walk started
  bool sp_internal;
  int pending_fix;
  int ld_pos;                   // insertSegments' advancing insert position within a LOADSEG batch
  uint32_t cur_k;               // index of the record being applied (catch-up delta entries name it)
  bool delta_on;                // the record asks for its delta ranges (MTB_F_DELTA)
  bool mkDup;                   // DSF_MKDUP: leaf-block updates re-map marker ids (hasMk modes)
  uint32_t ann_mk;              // the annotate's markerId test (record payload): 0 none, 1 same value, 2 never
  uint32_t delta_used;          // entries written in this document's delta slice
  static constexpr bool isPerm = MODE == MODE_MATRIX || MODE == MODE_LOADPERM;  // PermutationVectors only
  static constexpr bool isLoad = MODE == MODE_LOAD || MODE == MODE_LOADPERM;  // LOADSEG records only
  static constexpr bool isLive = MODE == MODE_LIVE;    // local ops / acks of the document's own client (id 0)
  // idToSegment upkeep and relative positions (the observer-only replay kernel carries none of it)
  static constexpr bool hasMk = MODE == MODE_MARKERS || MODE == MODE_LIVE || MODE == MODE_LOAD;
  int local_seq;                // MODE_LIVE: collabWindow.localSeq
  uint32_t pend_dir, pend_head, pend_n, pend_cap;  // MODE_LIVE: pending segment-group FIFO (DocState)
  bool grp_open;                // MODE_LIVE: the current local op already has its group
  bool pk_rw;                   // MODE_LIVE: pending_keys found a pending local rewrite on the segment
  int32_t* xch;                 // MODE_MATRIX: the workgroup's setCell exchange slots [2 parities][2 waves]
  int wv;                       // MODE_MATRIX: 0 = rows vector, 1 = cols vector              // depth of a block that reached MaxNodesInBlock children (-1: none)
  // phantom partial lengths of loaded documents (see "phantom partial lengths" below)
  static constexpr bool hasPh = MODE == MODE_LOAD || MODE == MODE_MARKERS || MODE == MODE_LIVE;
  // property keys whose values matchProperties does not compare as an equivalence (Tables::irr_any): the host
  // runs such batches on the marker variant, so the observer kernel carries none of that code
  static constexpr bool hasIrr = MODE == MODE_LOAD || MODE == MODE_MARKERS || MODE == MODE_LIVE;
  uint32_t ph_off;              // DocState.ph: aux offset of the table (0: none)
  bool phDoc;                   // DSF_PHANTOM (hasPh modes)
  int ph_split_top;             // the topmost depth the last fix_overflow split (MTB_VDEPTH: none)
  bool ph_ow;                   // markRangeRemoved's _overwrite, set during the current op's nodeMap
  uint32_t ld_stale;            // MODE_LOAD: bit d = the walk's depth-d block holds entries newer than the segment
  uint64_t prof[NPH];
  uint32_t evc[NCN];
#ifdef MTB_TABCHECK  // fault triage (tools/build_variants.py tabcheck): the pointers the engine dereferences, as set up
  const void* x_sh;
  const void* x_ptr[4];
  const Tables* x_tab;
  __device__ __forceinline__ void tchk(uint32_t site) {
    const bool ok = (const void*)sh == x_sh && (const void*)RAW(segp) == x_ptr[0] && (const void*)RAW(blk) == x_ptr[1] &&
                    (const void*)RAW(lst) == x_ptr[2] && (const void*)RAW(aux) == x_ptr[3] && sh->tab.pool == x_tab->pool &&
                    sh->tab.pidx == x_tab->pidx && sh->tab.val_class == x_tab->val_class &&
                    sh->tab.val_falsy == x_tab->val_falsy && sh->tab.key_irr == x_tab->key_irr;
    if (__ballot(!ok) && !err) {
      if (lane == 0) {
        ds->pad3[0] = 1;
        ds->pad3[1] = site;
        ds->pad3[2] = cur_k;
        ds->pad3[3] = 0;
      }
      fail(DERR_SHAPE);
    }
  }
#define TCHK(site) tchk(site)
#else
#define TCHK(site) ((void)0)
#endif

  // ------------------------------------------------------------------ errors / allocation
  __device__ __forceinline__ void fail(int code) {
    if (!err) err = code;
  }
  __device__ __forceinline__ bool bad() const { return COLD(err != 0); }
  __device__ __forceinline__ uint32_t alloc_seg() {
    if (seg_used >= U(sh->capv[0])) { fail(DERR_CAP_SEG); return 0; }
    return seg_used++;
  }
  __device__ __forceinline__ uint32_t* bw(uint32_t b) const { return reinterpret_cast<uint32_t*>(&blk[b]); }
#ifdef MTB_CHECK
  __device__ __forceinline__ CP<u32x4> lst4() const {
    CP<u32x4> c;
    c.p = reinterpret_cast<u32x4*>(lst.p), c.cap = lst.cap, c.rep = lst.rep, c.pool = 2;
    return c;
  }
#else
  __device__ __forceinline__ u32x4* lst4() const { return reinterpret_cast<u32x4*>(lst); }
#endif
  __device__ __forceinline__ uint32_t alloc_blk() {
    uint32_t b;
    if (free_top > 0) {
      free_top--;
      b = U(UP(sh->gfree)[free_top]);
    } else {
      if (blk_used >= U(sh->capv[1])) { fail(DERR_CAP_BLK); return 0; }
      b = blk_used++;
    }
    uint32_t* w = bw(b);
    w[lane] = lane < MTB_MAXCH ? MTB_NONE : 0u;
    if (lane < 16) {
      uint32_t h = 0;
      if (lane == 1) h = MTB_NONE;             // parent
      if (lane == 3) h = (uint32_t)-1;         // needsScour: undefined
      if (lane == 8) h = (uint32_t)MTB_NOKEY;  // lseq
      w[FB_HDR + lane] = h;
    }
    wsync();
    return b;
  }
  __device__ __forceinline__ void free_blk(uint32_t b) {
    UP(sh->gfree)[free_top] = b;
    free_top++;
  }
  __device__ __forceinline__ uint32_t alloc_aux(uint32_t n) {
    if (aux_used + n > U(sh->capv[5])) { fail(DERR_CAP_AUX); return 1; }
    uint32_t o = aux_used;
    aux_used += n;
    return o;
  }
  __device__ __forceinline__ void view_clear() {
    if (lane < MTB_VDEPTH) sh->v[lane].b = MTB_NONE;
    vmask = 0;
    wsync();
  }

  // ------------------------------------------------------------------ visibility
  __device__ __forceinline__ bool rc_has(int rc0, uint32_t rcx, int C) const {
    if (rc0 == C) return true;
    if (rcx) {
      const uint32_t n = aux[rcx];
      for (uint32_t i = 0; i < n; i++)
        if ((int)aux[rcx + 1 + i] == C) return true;
    }
    return false;
  }
  // localNetLength (mergeTree.ts:613-634)
  __device__ __forceinline__ int local_len(int len, int rseq) const {
    if (rseq >= 0) {
      if (!newMode) return rseq > minSeq ? 0 : MTB_UNDEF;
      return 0;
    }
    return len;
  }
#ifdef MTB_VIS_V1
  // nodeLength for a leaf in a remote perspective (mergeTree.ts:935-1001)
  __device__ __forceinline__ int seg_vis(int len, int seq, int rseq, uint32_t cli, uint32_t rcx, int R, int C) const {
    const bool removed = rseq >= 0;
    const int client = cli_client(cli);
    if (newMode) {
      if (removed) {
        if (rseq <= minSeq) return MTB_UNDEF;
        if (rseq <= R || rc_has(cli_rc0(cli), rcx, C)) return 0;
      }
      return (seq <= R || client == C) ? len : 0;
    }
    if (removed && rseq <= R) return MTB_UNDEF;
    if (client == C || seq <= R) {
      if (removed) return rc_has(cli_rc0(cli), rcx, C) ? 0 : len;
      return len;
    }
    if (removed && !(isLive && rseq >= MTB_PEND)) return MTB_UNDEF;  // (removedSeq !== Unassigned)
    return 0;
  }
#else
  // the further removers [n, c1..cn] of a segment hold C (its removedClientIds[0] is checked by the caller)
  __device__ __forceinline__ bool rcx_has(uint32_t rcx, int C) const {
    const uint32_t n = aux[rcx];
    for (uint32_t i = 0; i < n; i++)
      if ((int)aux[rcx + 1 + i] == C) return true;
    return false;
  }
  // nodeLength for a leaf in a remote perspective (mergeTree.ts:935-1001).  Per lane and divergent: the
  // conditions are combined as masks, and only lanes that must read the further removers' list branch.
  __device__ __forceinline__ int seg_vis(int len, int seq, int rseq, uint32_t cli, uint32_t rcx, int R, int C) const {
    const bool removed = rseq >= 0;
    const bool seen = (seq <= R) | (cli_client(cli) == C);
    const bool rc0 = cli_rc0(cli) == C;
    if (newMode) {
      const bool und = removed & (rseq <= minSeq);
      bool gone = removed & ((rseq <= R) | rc0);
      if (COLD(removed & !und & !gone & (rcx != 0))) gone = rcx_has(rcx, C);
      return und ? MTB_UNDEF : (gone | !seen) ? 0 : len;
    }
    const bool remR = removed & (rseq <= R);
    bool rch = rc0;
    if (COLD(removed & !remR & seen & !rc0 & (rcx != 0))) rch = rcx_has(rcx, C);
    const bool und = remR | (!seen & removed & !(isLive && rseq >= MTB_PEND));  // (removedSeq !== Unassigned)
    return und ? MTB_UNDEF : (!seen | (removed & rch)) ? 0 : len;
  }
#endif
  // nodeLength of a leaf in the op's perspective: the local client's own view (mergeTree.ts:917-921) or a
  // remote one
  __device__ __forceinline__ int leaf_len(int len, int seq, int rseq, uint32_t cli, uint32_t rcx, int R, int C) const {
    if (isLive && C == 0) return local_len(len, rseq);
    return seg_vis(len, seq, rseq, cli, rcx, R, C);
  }
  // observer-view length contribution of a child (blockUpdate: cachedLength = sum localNetLength ?? 0)
  __device__ __forceinline__ int child_olen(uint32_t id, int len, int rseq) const {
    if (!(id & MTB_LEAF)) return len;
    const int l = local_len(len, rseq);
    return l == MTB_UNDEF ? 0 : l;
  }

  // ------------------------------------------------------------------ views
  // Window-list metadata of the block at depth d of the current path (root: rmeta).
  __device__ __forceinline__ void meta_of(int d, uint32_t& loff, uint32_t& lcnt, uint32_t& lcap) const {
    if (d == 0) {
      loff = U(sh->rmeta[0]);
      lcnt = U(sh->rmeta[1]);
      lcap = U(sh->rmeta[2]);
    } else {
      const View& P = sh->v[d - 1];
      const int k = U(sh->slot[d - 1]);
      loff = U(P.f[F_SEQ][k]);
      lcnt = U(P.f[F_RSEQ][k]);
      lcap = U(P.f[F_CLI][k]);
    }
  }
  // Slot `lane` of a block, in registers (lanes < count): child id, its F_SEQ / F_RSEQ / F_CLI fields
  // (segment: seq, removedSeq, client word; block: its list offset, count, capacity word) and the
  // child's length in the op's (R, C) view (MTB_UNDEF: undefined).
  struct Kid {
    uint32_t id, seq, rseq, cli;
    int rl;
  };
  // Fetch block b (depth d of the current path) together with its window list, and compute its
  // children's lengths in the (R, C) view.  Returns the child count; `k` receives slot `lane` in
  // registers (the walk decides from them without reading the LDS view back).  The record is also
  // stored as the LDS view of depth d for the op's later steps.  A caller that knows the block's list
  // metadata (the walk: its parent's slot fields, in registers) passes it in.
  __device__ __forceinline__ int load_view(int d, uint32_t b, int R, int C, Kid& k, bool haveMeta = false,
                                           uint32_t mloff = 0, uint32_t mlcnt = 0, uint32_t mlcap = 0) {
    View& V = sh->v[d];
    k.id = MTB_NONE;
    k.seq = k.rseq = k.cli = 0;
    k.rl = 0;
    if (vmask & (1u << d)) {
      const uint32_t vb = U(V.b);
      if (vb == b) {
        const int count = U(V.count);
        const int vrlv = U(V.rlv);
        if (lane < count) {
          k.id = V.f[F_ID][lane];
          k.seq = V.f[F_SEQ][lane];
          k.rseq = V.f[F_RSEQ][lane];
          k.cli = V.f[F_CLI][lane];
        }
        if (vrlv) {
          if (lane < count) k.rl = V.rl[lane];
          return count;
        }
        // record still valid (e.g. after a segment split): recompute the leaves' lengths from LDS
        if (__ballot(lane < count && !(k.id & MTB_LEAF)) == 0) {
          if (lane < count) {
            k.rl = leaf_len((int)V.f[F_LEN][lane], (int)k.seq, (int)k.rseq, k.cli, V.f[F_RCX][lane], R, C);
            V.rl[lane] = k.rl;
          }
          if (lane == 0) V.rlv = 1;
          wsync();
          return count;
        }
      }
    }
    PROF_CNT(CN_VIEW, 1);
    const uint64_t tv0 = PROF_T();
    uint32_t loff = mloff, lcnt = mlcnt, lcapw = mlcap;
    if (!haveMeta) meta_of(d, loff, lcnt, lcapw);
    if (isLive && C == 0) lcnt = 0;  // the local view: blocks' cachedLength as they are (no corrections)
    // remote-length corrections per child slot (partialLengths.ts:698 getPartialLength).  Entries at or
    // below minSeq sit in the reference's minLength whatever refSeq is, so the scan threshold is
    // max(refSeq, minSeq) (only a summary load's body inserts, at refSeq 0, ever see refSeq < minSeq).
    const int Rl = R > minSeq ? R : minSeq;
    const int Cm = C & 0xFFFF;
    // A sorted list's entries above Rl are its tail: it is read backwards from the end, one or two
    // 64-entry chunks in flight with the record (two when the op's view lags far behind the window),
    // more only while every entry read is still above Rl.  An unsorted list is read whole, front first.
    const bool sorted = !(lcapw & MTB_LUNSORTED);
    const bool two = lcnt > 64 && (!sorted || curSeq - Rl > 56);
    const uint32_t* src = bw(b);
    // the record twice: linear (lane i = dword i) for the LDS view, and slot-major on lanes 0..7
    const uint32_t w = src[lane];
    const uint32_t h = lane < 5 ? src[FB_HDR + lane] : 0u;
    uint32_t flen = 0, frcx = 0;
    if (lane < MTB_MAXCH) {
      flen = src[F_LEN * 8 + lane];
      k.seq = src[F_SEQ * 8 + lane];
      k.rseq = src[F_RSEQ * 8 + lane];
      k.cli = src[F_CLI * 8 + lane];
      frcx = src[F_RCX * 8 + lane];
    }
    const uint32_t i0 = sorted ? lcnt - 1 - (uint32_t)lane : (uint32_t)lane;
    const uint32_t i1 = sorted ? lcnt - 65 - (uint32_t)lane : 64u + (uint32_t)lane;
    const bool v0 = (uint32_t)lane < lcnt;
    const bool v1 = two && (uint32_t)lane + 64 < lcnt;
    WEnt e0, e1;
    e0.seq = e1.seq = MTB_NOKEY;
    e0.ck = e1.ck = 0;
    e0.delta = e1.delta = 0;
    if (v0) e0 = lst[loff + i0];
    if (v1) e1 = lst[loff + i1];
    if (lane < MTB_MAXCH) sh->corr[lane] = 0;
    (&V.f[0][0])[lane] = w;
    const int count = rl((int)h, 0);
    const uint32_t hpar = rlu(h, 1);
    const int hsc = rl((int)h, 3), hlen = rl((int)h, 4);
    wsync();
#ifdef MTB_VIS_V1
    auto correct = [&](const WEnt& e, bool v) {
      if (v && e.seq > Rl) {
        const int c = e.ck & 0xFFFF, kind = (e.ck >> 16) & 0xF;
        if ((kind == WK_MAIN && c != Cm) || (kind == WK_OVERLAP && c == Cm)) atomicAdd(&sh->corr[(e.ck >> 20) & 7], e.delta);
      }
    };
#else
    // (the entry's test as one mask: no nested exec-mask branches per entry chunk)
    auto correct = [&](const WEnt& e, bool v) {
      const uint32_t ck = (uint32_t)e.ck, kind = (ck >> 16) & 0xF;
      const bool same = (int)(ck & 0xFFFF) == Cm;
      const bool hit = v & (e.seq > Rl) & (((kind == WK_MAIN) & !same) | ((kind == WK_OVERLAP) & same));
      if (hit) atomicAdd(&sh->corr[(ck >> 20) & 7], e.delta);
    };
#endif
    correct(e0, v0);
    correct(e1, v1);
    uint32_t done = two ? 128u : 64u;  // entries fetched (from the end when sorted, from the front if not)
    if (sorted) {
      bool more = done < lcnt && __ballot((v0 && e0.seq <= Rl) || (v1 && e1.seq <= Rl)) == 0;
      while (COLD(more)) {
        const uint32_t i = lcnt - done - 1 - (uint32_t)lane;
        const bool v = (uint32_t)lane < lcnt - done;
        WEnt e;
        e.seq = MTB_NOKEY;
        if (v) e = lst[loff + i];
        correct(e, v);
        done += 64;
        more = done < lcnt && __ballot(v && e.seq <= Rl) == 0;
      }
    } else {
      for (; done < lcnt; done += 128) {
        const uint32_t ia = done + (uint32_t)lane, ib = ia + 64;
        WEnt ea, eb;
        if (ia < lcnt) ea = lst[loff + ia];
        if (ib < lcnt) eb = lst[loff + ib];
        correct(ea, ia < lcnt);
        correct(eb, ib < lcnt);
      }
    }
    PROF_CNT(CN_ENTRIES, done < lcnt ? done : lcnt);
    wsync();
    int phs = 0;  // the phantom surplus of a block child (loaded documents only)
    if constexpr (hasPh) {
      if (COLD(phDoc) && !(isLive && C == 0)) {
        const int c0 = lane < MTB_MAXCH ? sh->corr[lane] : 0;  // (ph_view reuses corr[])
        phs = ph_view(w, count, Rl, C);
        if (lane < MTB_MAXCH) sh->corr[lane] = c0;
        wsync();
      }
    }
    if (lane < count) {
      k.id = w;
      k.rl = (w & MTB_LEAF) ? leaf_len((int)flen, (int)k.seq, (int)k.rseq, k.cli, frcx, R, C) : (int)flen - sh->corr[lane] + phs;
      V.rl[lane] = k.rl;
    }
    if (lane == 0) {
      V.b = b;
      V.count = count;
      V.parent = hpar;
      V.scour = hsc;
      V.len = hlen;
      V.rlv = 1;
    }
    vmask |= 1u << d;
    wsync();
    PROF_ADD(PH_VIEW, tv0);
    return count;
  }
  __device__ __forceinline__ int load_view(int d, uint32_t b, int R, int C) {
    Kid k;
    return load_view(d, b, R, C, k);
  }

  // ------------------------------------------------------------------ window lists
  __device__ __forceinline__ static uint32_t list_class_cap(uint32_t want) {
    uint32_t c = 8;
    while (c < want) c <<= 1;
    return c;
  }
  __device__ __forceinline__ static int list_class(uint32_t cap) { return 28 - __builtin_clz(cap); }  // 8 -> 0
  // A list with room for `want` entries; `cap` receives its (power-of-two) capacity.
  __device__ __forceinline__ uint32_t list_alloc(uint32_t want, uint32_t& cap) {
    cap = list_class_cap(want);
    const int c = list_class(cap);
#ifndef MTB_NO_LSTK
    if (c < MTB_LSTK) {
      const uint32_t n = U(sh->lstkn[c]);
      if (n) {
        const uint32_t h = U(sh->lstk[c][n - 1]);
        wsync();
        if (lane == 0) sh->lstkn[c] = n - 1;
        wsync();
        return h;
      }
    }
#endif
    if (c < MTB_LCLASSES) {
      const uint32_t head = U(sh->lfree[c]);
      if (head != MTB_NONE) {
        const uint32_t next = U(reinterpret_cast<const uint32_t*>(&lst[head])[0]);
        wsync();
        if (lane == 0) sh->lfree[c] = next;
        wsync();
        return head;
      }
    }
    if (list_used + cap > U(sh->capv[2])) {
      fail(DERR_CAP_LIST);
      return 0;
    }
    const uint32_t o = list_used;
    list_used += cap;
    return o;
  }
  __device__ __forceinline__ void list_free(uint32_t off, uint32_t capw) {
    const uint32_t cap = capw & ~MTB_LUNSORTED;
    if (cap < 8 || (cap & (cap - 1))) return;
    const int c = list_class(cap);
    if (c >= MTB_LCLASSES) return;
#ifndef MTB_NO_LSTK
    if (c < MTB_LSTK) {
      const uint32_t n = U(sh->lstkn[c]);
      if (n < MTB_LSTK_N) {
        wsync();
        if (lane == 0) {
          sh->lstk[c][n] = off;
          sh->lstkn[c] = n + 1;
        }
        wsync();
        return;
      }
    }
#endif
    if (lane == 0) {
      reinterpret_cast<uint32_t*>(&lst[off])[0] = U(sh->lfree[c]);
      sh->lfree[c] = off;
    }
    wsync();
  }

  // Store the window-list metadata of the path block at depth d (its parent's slot, or the root
  // header).  Called by one lane.
  __device__ __forceinline__ void set_meta(int d, uint32_t loff, uint32_t lcnt, uint32_t lcap) {
    if (d == 0) {
      sh->rmeta[0] = loff;
      sh->rmeta[1] = lcnt;
      sh->rmeta[2] = lcap;
      FBlk& B = blk[sh->path[0]];
      B.loff = loff;
      B.lcnt = lcnt;
      B.lcap = lcap;
    } else {
      View& P = sh->v[d - 1];
      const int k = sh->slot[d - 1];
      P.f[F_SEQ][k] = loff;
      P.f[F_RSEQ][k] = lcnt;
      P.f[F_CLI][k] = lcap;
      FBlk& B = blk[sh->path[d - 1]];
      B.f[F_SEQ][k] = loff;
      B.f[F_RSEQ][k] = lcnt;
      B.f[F_CLI][k] = lcap;
    }
  }
  // Copy `cnt` entries at `off` into a fresh list with room for `extra` more, dropping entries at or
  // below minSeq.  Returns the new offset; `live` receives
  // the kept count, `cap` the capacity word: MTB_LUNSORTED unless the kept entries are in seq order
  // (a list rebuilt unsorted becomes sorted again once its out-of-order entries fall below minSeq).
  __device__ __forceinline__ uint32_t list_regrow(uint32_t off, uint32_t cnt, uint32_t ocap, uint32_t extra, uint32_t& live,
                                                   uint32_t& cap) {
    PROF_CNT(CN_GROW, 1);
    uint32_t n = 0;  // kept entries (the capacity follows them, not the stale ones)
    for (uint32_t base = 0; base < cnt; base += 64) {
      const uint32_t i = base + lane;
      const bool keep = i < cnt && lst[off + i].seq > minSeq;
      n += __popcll(__ballot(keep));
    }
    const uint32_t no = list_alloc(2 * (n + extra), cap);
    if (bad()) return 0;
    uint32_t w = 0;
    int carry = MTB_NOKEY;  // largest kept seq of the chunks before
    bool unsorted = false;
    for (uint32_t base = 0; base < cnt; base += 64) {
      const uint32_t i = base + lane;
      u32x4 e = {0u, 0u, 0u, 0u};  // (entries as vectors: struct copies here went through scratch)
      bool keep = false;
      if (i < cnt) {
        e = lst4()[off + i];
        keep = (int)e.x > minSeq;
      }
      const unsigned long long m = __ballot(keep);
      if (keep) lst4()[no + w + rank_below(m)] = e;
      w += __popcll(m);
      // order check: each kept entry against the largest kept seq before it (prefix max)
      int pm = keep ? (int)e.x : MTB_NOKEY;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(pm, o, 64);
        if (lane >= o) pm = max(pm, t);
      }
      int prev = __shfl_up(pm, 1, 64);
      if (lane == 0) prev = MTB_NOKEY;
      prev = max(prev, carry);
      if (keep && (int)e.x < prev) unsorted = true;
      carry = max(carry, rl(pm, 63));
    }
    live = w;
    if (__ballot(unsorted)) cap |= MTB_LUNSORTED;
    wsync();
    list_free(off, ocap);
    return no;
  }
  // Append (seqv, client, kind, delta) to the lists of the path blocks at depths [lo, hi), each entry
  // tagged with the slot the path takes at that depth.  One lane per depth; full lists are
  // re-allocated afterwards, one at a time.  A replay appends the current op's seq, never below any
  // entry, so the lists stay sorted; a summary load's body appends any seq, and a live document with
  // unacked local entries (MTB_PEND + localSeq) appends below them: both mark the lists unsorted.
  __device__ __forceinline__ void append_levels(int lo, int hi, int seqv, int client, int kind, int delta) {
    if (hi <= lo) return;
    bool need = false;
    const int i = lane;
    if (i >= lo && i < hi) {
      uint32_t loff, lcnt, lcap;
      if (i == 0) {
        loff = sh->rmeta[0];
        lcnt = sh->rmeta[1];
        lcap = sh->rmeta[2];
      } else {
        const View& P = sh->v[i - 1];
        const int k = sh->slot[i - 1];
        loff = P.f[F_SEQ][k];
        lcnt = P.f[F_RSEQ][k];
        lcap = P.f[F_CLI][k];
      }
      if (isLoad || (isLive && pend_n > 0)) {
        if (lcnt < (lcap & ~MTB_LUNSORTED) && !(lcap & MTB_LUNSORTED)) {
          lcap |= MTB_LUNSORTED;
          if (i == 0) {
            sh->rmeta[2] = lcap;
            blk[sh->path[0]].lcap = lcap;
          } else {
            const int k = sh->slot[i - 1];
            sh->v[i - 1].f[F_CLI][k] = lcap;
            blk[sh->path[i - 1]].f[F_CLI][k] = lcap;
          }
        }
      }
      if (lcnt < (lcap & ~MTB_LUNSORTED)) {
        WEnt e;
        e.seq = seqv;
        e.ck = WE_KEY(client, kind, sh->slot[i]);
        e.delta = delta;
        e.pad = 0;
        lst[loff + lcnt] = e;
        if (i == 0) {
          sh->rmeta[1] = lcnt + 1;
          blk[sh->path[0]].lcnt = lcnt + 1;
        } else {
          const int k = sh->slot[i - 1];
          sh->v[i - 1].f[F_RSEQ][k] = lcnt + 1;
          blk[sh->path[i - 1]].f[F_RSEQ][k] = lcnt + 1;
        }
      } else {
        need = true;
      }
    }
    unsigned long long m = __ballot(need);
    if (COLD(m))
    while (m) {
      const int d = first_set(m);
      m &= m - 1;
      uint32_t loff, lcnt, lcap;
      meta_of(d, loff, lcnt, lcap);
      uint32_t live, cap;
      const uint32_t no = list_regrow(loff, lcnt, lcap, 1, live, cap);
      if (bad()) return;
      // (cap carries the kept entries' order; pending MTB_PEND + localSeq entries may sit above this seq)
      const uint32_t flag = (isLoad || (isLive && pend_n > 0)) ? MTB_LUNSORTED : 0u;
      if (lane == 0) {
        WEnt e;
        e.seq = seqv;
        e.ck = WE_KEY(client, kind, sh->slot[d]);
        e.delta = delta;
        e.pad = 0;
        lst[no + live] = e;
        set_meta(d, no, live + 1, cap | flag);
      }
      wsync();
    }
  }
  // Insert an overlapping remover's (removedSeq, client, OVERLAP, +len) entry into the lists of the path
  // blocks at depths [lo, hi) at its seq position (removedSeq is older than the current op): the tail of
  // entries above it moves up by one, chunk by chunk from the end.  Rare (overlapping removes).
  __device__ __forceinline__ void insert_levels_sorted(int lo, int hi, int seqv, int client, int kind, int delta) {
    for (int dd = lo; dd < hi && !err; dd++) {
      uint32_t loff, lcnt, lcapw;
      meta_of(dd, loff, lcnt, lcapw);
      if (lcnt >= (lcapw & ~MTB_LUNSORTED)) {
        uint32_t live, cap;
        const uint32_t no = list_regrow(loff, lcnt, lcapw, 1, live, cap);
        if (bad()) return;
        lcapw = cap;
        if (lane == 0) set_meta(dd, no, live, lcapw);
        wsync();
        loff = no;
        lcnt = live;
      }
      uint32_t p = lcnt;
      if (!(lcapw & MTB_LUNSORTED)) {
        uint32_t top = lcnt;
        while (top > 0) {
          const uint32_t n = top < 64 ? top : 64u;
          const uint32_t i = top - n + (uint32_t)lane;
          const bool v = (uint32_t)lane < n;
          u32x4 e = {(uint32_t)MTB_NOKEY, 0u, 0u, 0u};
          if (v) e = lst4()[loff + i];
          const bool gt = v && (int)e.x > seqv;
          const unsigned long long m = __ballot(gt);
          if (gt) lst4()[loff + i + 1] = e;  // (sorted: the lanes above seqv are a suffix of the chunk)
          wsync();
          const uint32_t g = (uint32_t)__popcll(m);
          p = top - g;
          if (g < n) break;
          top -= n;
        }
      }
      if (lane == 0) {
        WEnt e;
        e.seq = seqv;
        e.ck = WE_KEY(client, kind, sh->slot[dd]);
        e.delta = delta;
        e.pad = 0;
        lst[loff + p] = e;
        set_meta(dd, loff, lcnt + 1, lcapw);
      }
      wsync();
    }
  }
  // Observer-length bookkeeping along the path: the path slot's childLen at depths [lo, hi) and the
  // block's own cachedLength at depths [lo, hdr_hi].
  __device__ __forceinline__ void add_len_levels(int lo, int hi, int hdr_hi, int dlen) {
    if (!dlen) return;
    const int i = lane;
    if (i >= lo && i < hi) {
      const int k = sh->slot[i];
      const int v = (int)sh->v[i].f[F_LEN][k] + dlen;
      sh->v[i].f[F_LEN][k] = (uint32_t)v;
      blk[sh->path[i]].f[F_LEN][k] = (uint32_t)v;
    }
    if (i >= lo && i <= hdr_hi) {
      const int v = sh->v[i].len + dlen;
      sh->v[i].len = v;
      blk[sh->path[i]].len = v;
    }
    wsync();
  }
  // Rebuild block P's window list from its children (after split / packParent / root growth): for
  // each block child k, the entries of k's own list plus entries derived from k's segment children
  // (the combine semantics of partialLengths.ts:256).  Returns the new metadata; the caller stores it
  // where P's metadata lives.
  // hold_nh >= 0 (packParent, every new child a block of segments): P's children are the hold_cc blocks packParent
  // just filled from sh->hold[.][0..hold_nh) in its order (the first hold_nh % hold_cc get one more), so their
  // segments are read from LDS instead of from the records written a moment before (two dependent round trips
  // fewer); such children have no lists of their own.
  // pv (a split's parent): P's record as the walk's LDS view of it holds it, instead of a read of the record.
  __device__ __forceinline__ void rebuild(uint32_t P, uint32_t old_loff, uint32_t old_lcap, uint32_t& loff_out,
                                         uint32_t& lcnt_out, uint32_t& lcap_out, int hold_nh = -1, int hold_cc = 0,
                                         const View* pv = nullptr) {
    PROF_CNT(CN_REBUILD, 1);
    Rec& Z = sh->zr;
    const bool fromHold = hold_nh >= 0;
    int count = hold_cc;
    if (!fromHold) {
      uint32_t w;
      if (pv) {
        w = (&pv->f[0][0])[lane];
        count = U(pv->count);
      } else {
        const uint32_t* src = bw(P);
        w = src[lane];
        count = U((int)src[FB_HDR]);
      }
      (&Z.f[0][0])[lane] = w;
      wsync();
    }
    // lane (k, s): segment child s of block child k
    const int k = lane >> 3, s = lane & 7;
    uint32_t ck = MTB_NONE;
    if (!fromHold && k < count) ck = Z.f[F_ID][k];
    const bool kblk = k < count && (fromHold || !(ck & MTB_LEAF));
    int ne = 0, nov = 0;
    int slen = 0, sseq = 0, srseq = -1;
    uint32_t scli = 0, srcx = 0;
    if (kblk) {
      if (fromHold) {
        const int base = hold_nh / hold_cc, rem = hold_nh % hold_cc;
        const int nk = base + (k < rem ? 1 : 0), start = k * base + (k < rem ? k : rem);
        if (s < nk) {
          const int i = start + s;
          slen = (int)sh->hold[F_LEN][i];
          sseq = (int)sh->hold[F_SEQ][i];
          srseq = (int)sh->hold[F_RSEQ][i];
          scli = sh->hold[F_CLI][i];
          srcx = sh->hold[F_RCX][i];
        }
      } else {
        const uint32_t* c = bw(ck);
        const int ccount = (int)c[FB_HDR];
        if (s < ccount) {
          const uint32_t sid = c[F_ID * 8 + s];
          if (sid & MTB_LEAF) {
            slen = (int)c[F_LEN * 8 + s];
            sseq = (int)c[F_SEQ * 8 + s];
            srseq = (int)c[F_RSEQ * 8 + s];
            scli = c[F_CLI * 8 + s];
            srcx = c[F_RCX * 8 + s];
          }
        }
      }
      if (sseq > minSeq) ne++;
      if (srseq >= 0 && srseq > minSeq) {
        ne++;
        if (srcx) nov = (int)aux[srcx];
      }
    }
    // the block children's own lists (metadata in P's slots), concatenated
    uint32_t lc = 0, lo = 0;
    if (!fromHold && lane < count && !(Z.f[F_ID][lane] & MTB_LEAF)) {
      lo = Z.f[F_SEQ][lane];
      lc = Z.f[F_RSEQ][lane];
    }
    const int lincl = cscan8((int)lc);
    const int ltotal = rl(lincl, 7);
    const int lexcl = lincl - (int)lc;
    int pre[MTB_MAXCH], off[MTB_MAXCH];
#pragma unroll
    for (int q = 0; q < MTB_MAXCH; q++) {
      pre[q] = rl(lexcl, q);
      off[q] = rl((int)lo, q);
    }
    const unsigned long long b1 = __ballot(ne >= 1), b2 = __ballot(ne >= 2);
    const int nder = __popcll(b1) + __popcll(b2);
    int novt = 0;
    if (__ballot(nov > 0)) {
      novt = nov;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) novt += __shfl_xor(novt, o, 64);
    }
    const uint32_t total = (uint32_t)(nder + novt + ltotal);
    uint32_t cap;
    const uint32_t no = list_alloc(total + total / 2 + 4, cap);
    if (bad()) return;
    // derived entries: insert (seq, client, +len), removal (removedSeq, rc0, -len)
    uint32_t wp = rank_below(b1) + rank_below(b2);
    if (ne) {
      WEnt e;
      e.pad = 0;
      if (sseq > minSeq) {
        e.seq = sseq;
        e.ck = WE_KEY(cli_client(scli), WK_MAIN, k);
        e.delta = slen;
        lst[no + wp++] = e;
      }
      if (srseq >= 0 && srseq > minSeq) {
        e.seq = srseq;
        e.ck = WE_KEY(cli_rc0(scli), WK_MAIN, k);
        e.delta = -slen;
        lst[no + wp++] = e;
      }
    }
    uint32_t wpos = (uint32_t)nder;
    // overlapping removers (rare): (removedSeq, c, OVERLAP, +len), lane by lane
    unsigned long long om = __ballot(nov > 0);
    if (COLD(om))
    while (om) {
      const int t = first_set(om);
      om &= om - 1;
      const uint32_t rcx = rlu(srcx, t);
      const int n = rl(nov, t);
      const int rseq = rl(srseq, t), len = rl(slen, t), kk = t >> 3;
      for (int i = lane; i < n; i += 64) {
        WEnt e;
        e.seq = rseq;
        e.ck = WE_KEY((int)aux[rcx + 1 + i], WK_OVERLAP, kk);
        e.delta = len;
        e.pad = 0;
        lst[no + wpos + i] = e;
      }
      wpos += (uint32_t)n;
    }
    // children's lists, retagged with the child's slot, entries above minSeq only
    for (int base = 0; base < ltotal; base += 64) {
      const int t = base + lane;
      bool keep = false;
      u32x4 e = {0u, 0u, 0u, 0u};
      if (t < ltotal) {
        int j = 0;
#pragma unroll
        for (int q = 1; q < MTB_MAXCH; q++)
          if (q < count && pre[q] <= t) j = q;
        int p = 0;
#pragma unroll
        for (int q = 0; q < MTB_MAXCH; q++)
          if (q == j) p = off[q] + (t - pre[q]);
        e = lst4()[p];
        keep = (int)e.x > minSeq;
        e.y = (e.y & 0xFFFFFu) | ((uint32_t)j << 20);
      }
      const unsigned long long m = __ballot(keep);
      if (keep) lst4()[no + wpos + rank_below(m)] = e;
      wpos += __popcll(m);
    }
    wsync();
    list_free(old_loff, old_lcap);
    // Sort the new list by seq (a counting sort over seq - minSeq - 1 into a second list) so that views
    // can read only its tail; lists of one chunk stay unsorted (list_regrow restores the order later).  The 1024 16-bit bucket counters live in the scour union, which no caller
    // holds live across a rebuild.  A seq window too wide for the buckets leaves the list unsorted.
    const uint32_t T = wpos;
    uint32_t outOff = no, outCap = cap | MTB_LUNSORTED;
    if (T <= 1) {
      outCap = cap;
    } else if (T > MTB_SORT_MIN && T < 65536) {  // (a list of one chunk is read whole anyway: left unsorted)
      uint32_t* hist = &sh->hold[0][0];
      for (int i = lane; i < MTB_SORT_BUCKETS / 2; i += 64) hist[i] = 0;
      wsync();
      bool over = false;
      for (uint32_t base = 0; base < T; base += 64) {
        const uint32_t i = base + (uint32_t)lane;
        if (i < T) {
          const int bk = lst[no + i].seq - minSeq - 1;
          if (bk < 0 || bk >= MTB_SORT_BUCKETS) over = true;
          else atomicAdd(&hist[bk >> 1], 1u << ((bk & 1) * 16));
        }
      }
      if (!__ballot(over)) {
        wsync();
        // exclusive scan of the counts: lane l owns buckets [16 l, 16 l + 16) = words [8 l, 8 l + 8)
        uint32_t wv[8];
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          wv[q] = hist[8 * lane + q];
          tot += (wv[q] & 0xFFFF) + (wv[q] >> 16);
        }
        int incl = (int)tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        uint32_t run = (uint32_t)incl - tot;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t c0 = run;
          run += wv[q] & 0xFFFF;
          hist[8 * lane + q] = c0 | (run << 16);
          run += wv[q] >> 16;
        }
        wsync();
        uint32_t cap2;
        const uint32_t no2 = list_alloc(T + T / 2 + 4, cap2);
        if (bad()) return;
        for (uint32_t base = 0; base < T; base += 64) {
          const uint32_t i = base + (uint32_t)lane;
          if (i < T) {
            const u32x4 e = lst4()[no + i];
            const int bk = (int)e.x - minSeq - 1;
            const uint32_t sft = (uint32_t)(bk & 1) * 16;
            const uint32_t old = atomicAdd(&hist[bk >> 1], 1u << sft);
            lst4()[no2 + ((old >> sft) & 0xFFFF)] = e;
          }
        }
        wsync();
        list_free(no, cap);
        outOff = no2;
        outCap = cap2;
      }
      wsync();
    }
    loff_out = outOff;
    lcnt_out = T;
    lcap_out = outCap;
  }

  // ------------------------------------------------------------------ tree primitives
  __device__ __forceinline__ void set_parent(uint32_t node, uint32_t b, int idx) {
    if (node & MTB_LEAF) {
      segp[node & ~MTB_LEAF] = b;
    } else {
      blk[node].parent = b;
      blk[node].index = (uint32_t)idx;
    }
  }
  // Insert a child with fields sh->nseg[] at slot k of the block cached at depth d
  // (insertingWalk shift, mergeTree.ts:1831-1837).  Updates the record, the view and the parents.
  __device__ __forceinline__ void insert_slot(int d, int k) {
    View& V = sh->v[d];
    const uint32_t b = U(V.b);
    const int count = U(V.count);
    const int fld = lane >> 3, s = lane & 7;
    uint32_t nv = (&V.f[0][0])[lane];
    if (s == k) nv = sh->nseg[fld];
    else if (s > k && s <= count) nv = V.f[fld][s - 1];
    wsync();
    if (s <= count) {
      (&V.f[0][0])[lane] = nv;
      bw(b)[lane] = nv;
    }
    wsync();
    // parents / indices of the new child and of the shifted block children
    if (lane < MTB_MAXCH && lane >= k && lane <= count) {
      const uint32_t c = V.f[F_ID][lane];
      if (lane == k || !(c & MTB_LEAF)) set_parent(c, b, lane);
    }
    if (lane == 0) {
      V.count = count + 1;
      V.rlv = 0;
      blk[b].count = (uint32_t)(count + 1);
    }
    wsync();
  }
  // split (mergeTree.ts:1858-1871): children 4..7 of the block at depth `level` move to a new block.
  // The halves' cachedLength and list metadata are left in sp_* for the caller, which links them in.
  __device__ __forceinline__ uint32_t split_block(int level) {
    PROF_CNT(CN_SPLIT, 1);
    struct_changed = true;
    const uint32_t nb = alloc_blk();
    if (bad()) return 0;
    View& V = sh->v[level];
    const uint32_t b = U(V.b);
    const int half = MTB_MAXCH / 2;
    const int fld = lane >> 3, s = lane & 7;
    const uint32_t val = (&V.f[0][0])[lane];
    if (s >= half) {
      bw(nb)[fld * 8 + s - half] = val;
      bw(b)[lane] = fld == F_ID ? MTB_NONE : 0u;
    }
    int ol = 0;
    bool isblk = false;
    if (lane < MTB_MAXCH) {
      const uint32_t c = V.f[F_ID][lane];
      ol = child_olen(c, (int)V.f[F_LEN][lane], (int)V.f[F_RSEQ][lane]);
      isblk = !(c & MTB_LEAF);
      if (lane >= half) set_parent(c, nb, lane - half);
    }
    const int lenAll = csum8(ol);
    const int lenL = csum8(lane < half ? ol : 0);
    const uint32_t vpar = U(V.parent);
    if (lane == 0) {
      blk[b].count = half;
      blk[b].len = lenL;
      blk[nb].count = half;
      blk[nb].len = lenAll - lenL;
      blk[nb].parent = vpar;
      V.count = half;  // (all views are cleared after fix_overflow)
    }
    wsync();
    sp_lenL = (uint32_t)lenL;
    sp_lenR = (uint32_t)(lenAll - lenL);
    sp_loffL = sp_lcntL = sp_lcapL = sp_loffR = sp_lcntR = sp_lcapR = 0;
    sp_internal = __ballot(isblk) != 0;  // the halves' lists are rebuilt by the caller
    // the segment placed by the insert walk moves with the right half
    if (level == U(ins_depth) && U(ins_slot) >= half) {
      ins_blk = nb;
      ins_slot -= half;
      ins_scour = -1;
    }
    return nb;
  }
  __device__ __forceinline__ void stage_block_child(uint32_t id, uint32_t len, uint32_t loff, uint32_t lcnt, uint32_t lcap) {
    if (lane < 8) {
      uint32_t v = 0;
      if (lane == F_ID) v = id;
      if (lane == F_LEN) v = len;
      if (lane == F_SEQ) v = loff;
      if (lane == F_RSEQ) v = lcnt;
      if (lane == F_CLI) v = lcap;
      sh->nseg[lane] = v;
    }
    wsync();
  }
  // After inserting into the block at depth d, split every full block on the path; a root split grows
  // the tree by one level (updateRoot, mergeTree.ts:1268-1277).
  __device__ __forceinline__ void fix_overflow(int d) {
    if (COLD(U(sh->v[d].count) >= MTB_MAXCH)) fix_overflow_slow(d);
  }
  // Split every full block on the path, from depth d upwards.  Written as a state machine with a
  // single list-rebuild site (the halves of an internal split, the new root, the parent).
  __device__ __forceinline__ void fix_overflow_slow(int d) {
    int level = d;
    int phase = 0;  // 0 split `level` | 1 rebuild left half | 2 rebuild right half | 3 link | 4 parent done | 5 root done
    uint32_t b = MTB_NONE, nb = MTB_NONE;
    while (!err) {
      if (phase == 0) {
        if (U(sh->v[level].count) < MTB_MAXCH) break;
        b = U(sh->v[level].b);
        nb = split_block(level);
        if (err) break;
        if constexpr (hasPh) {
          ph_split_top = level;  // (split halves are recombined: no stale update there, see apply_loadseg)
          if (COLD(phDoc)) {  // split (mergeTree.ts:1858-1871): both halves nodeUpdateLengthNewStructure
            ph_combine(b);
            ph_combine(nb);
            if (err) break;
          }
        }
        phase = sp_internal ? 1 : 3;
        continue;
      }
      uint32_t X, ooff = 0, ocnt = 0, ocap = 0;
      const int L = level - 1;
      const View* xv = nullptr;  // (the parent: its view is current)
      if (phase == 1) {
        X = b;
        meta_of(level, ooff, ocnt, ocap);
        phase = 2;
      } else if (phase == 2) {
        X = nb;
        phase = 3;
      } else if (level == 0) {
        // new root with children (b, nb) (updateRoot, mergeTree.ts:1268-1277)
        X = alloc_blk();
        if (err) break;
        if (lane == 0) {
          FBlk& Rb = blk[X];
          Rb.f[F_ID][0] = b;
          Rb.f[F_LEN][0] = sp_lenL;
          Rb.f[F_SEQ][0] = sp_loffL;
          Rb.f[F_RSEQ][0] = sp_lcntL;
          Rb.f[F_CLI][0] = sp_lcapL;
          Rb.f[F_ID][1] = nb;
          Rb.f[F_LEN][1] = sp_lenR;
          Rb.f[F_SEQ][1] = sp_loffR;
          Rb.f[F_RSEQ][1] = sp_lcntR;
          Rb.f[F_CLI][1] = sp_lcapR;
          Rb.count = 2;
          Rb.len = (int32_t)(sp_lenL + sp_lenR);
          blk[b].parent = X;
          blk[b].index = 0;
          blk[nb].parent = X;
          blk[nb].index = 1;
        }
        wsync();
        phase = 5;
      } else {
        // link (b, nb) into the parent at depth level-1, then rebuild the parent's list
        const int k = U(sh->slot[L]);
        View& P = sh->v[L];
        if (lane == 0) {
          P.f[F_LEN][k] = sp_lenL;
          P.f[F_SEQ][k] = sp_loffL;
          P.f[F_RSEQ][k] = sp_lcntL;
          P.f[F_CLI][k] = sp_lcapL;
          FBlk& PB = blk[P.b];
          PB.f[F_LEN][k] = sp_lenL;
          PB.f[F_SEQ][k] = sp_loffL;
          PB.f[F_RSEQ][k] = sp_lcntL;
          PB.f[F_CLI][k] = sp_lcapL;
        }
        wsync();
        stage_block_child(nb, sp_lenR, sp_loffR, sp_lcntR, sp_lcapR);
        insert_slot(L, k + 1);
        X = U(P.b);
        meta_of(L, ooff, ocnt, ocap);
        xv = &P;
        phase = 4;
      }
      uint32_t a, c2, e;
      rebuild(X, ooff, ocap, a, c2, e, -1, 0, xv);
      if (err) break;
      if (phase == 2) {
        sp_loffL = a;
        sp_lcntL = c2;
        sp_lcapL = e;
      } else if (phase == 3) {
        sp_loffR = a;
        sp_lcntR = c2;
        sp_lcapR = e;
      } else if (phase == 4) {
        if (lane == 0) set_meta(L, a, c2, e);
        wsync();
        level = L;
        phase = 0;
      } else {  // phase 5: the new root
        root = X;
        if (lane == 0) {
          sh->path[0] = X;
          sh->rmeta[0] = a;
          sh->rmeta[1] = c2;
          sh->rmeta[2] = e;
          blk[X].loff = a;
          blk[X].lcnt = c2;
          blk[X].lcap = e;
        }
        wsync();
        if constexpr (hasPh) {
          if (COLD(phDoc)) ph_combine(X);  // updateRoot (mergeTree.ts:1268-1277)
        }
        break;
      }
    }
    view_clear();
  }

  // Window-list entries for a summary segment placed by a LOADSEG insert: blockUpdateLength's combine
  // (mergeTree.ts:2419-2431) recomputes the path blocks' partials from their leaves, which is what the
  // derived entries give (the host admits removed body segments only for NonCollabClient, whose inserts
  // take that path; a client segment's incremental update equals the same entries when unremoved).
  __device__ __forceinline__ void load_entries(int d, int S, int C) {
    const int len = (int)U(sh->nseg[F_LEN]);
    const int rseq = (int)U(sh->nseg[F_RSEQ]);
    const uint32_t cli = U(sh->nseg[F_CLI]);
    const uint32_t rcx = U(sh->nseg[F_RCX]);
    if (S > minSeq) append_levels(0, d, S, C, WK_MAIN, len);
    if (rseq >= 0 && rseq > minSeq) {
      append_levels(0, d, rseq, cli_rc0(cli), WK_MAIN, -len);
      const uint32_t n = rcx ? U(aux[rcx]) : 0u;
      for (uint32_t i = 0; i < n && !err; i++) append_levels(0, d, rseq, (int)U(aux[rcx + 1 + i]), WK_OVERLAP, len);
    }
  }

  // ------------------------------------------------------------------ phantom partial lengths
  // A SnapshotV1 load appends a removed body segment P inserted by a collaborating client alone, through
  // blockUpdateLength's incremental path (snapshotLoader.ts:242-254 -> mergeTree.ts:2436-2453): every block
  // that update() reaches adds P's cachedLength at P's seq (removedSeq !== seq, partialLengths.ts:636-686) and
  // nothing ever records P's removal there.  The window lists stay exact; the surplus is a per-document table
  // in the aux arena (DocState.ph): [n, cap, entry * cap], 8 words an entry, word 6 its kind:
  //   PH_PHANTOM  (block, rseq, len, rc0, rcx, seq, 0, inserting client)
  //   PH_DEF_MAIN (block, t, d, -, -, seq, 1, -)   main-set deficit: lengths at refSeq >= t are short by d
  //   PH_DEF_CLI  (block, t, d, c, -, seq, 2, -)   client-set deficit: client c's lengths below t are short by d
  //   PH_DEF_MIN  (block, -, d, -, -, seq, 3, -)   a main-set deficit copied down into minLength: always short
  // A block child's length in a remote view then adds len(P) for each phantom whose exact-list removal would
  // count (rseq <= max(refSeq, minSeq), or the viewer is one of P's removers) and takes off each deficit that
  // applies.  Entries follow the reference's recombinations (PartialSequenceLengths.combine, :256-338): a
  // recombined block of segments has none (fromLeaves is exact), a recombined block of blocks the union of its
  // children's phantoms and copied-down deficits (combine sums the children's minLength, :304-308, and rebuilds
  // the entries from seglen, so every other shortfall is gone); update() leaves them.  Dead entries: block MTB_NONE.
  __device__ __forceinline__ void ph_add(uint32_t node, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                                         uint32_t w5 = 0, uint32_t kind = PH_PHANTOM, uint32_t w7 = 0) {
    const uint32_t n = U(aux[ph_off]), cap = U(aux[ph_off + 1]);
    if (n >= cap) {
      const uint32_t ncap = 2 * cap + 8;
      const uint32_t h = alloc_aux(2 + 8 * ncap);
      if (bad()) return;
      for (uint32_t i = lane; i < 8 * n; i += 64) aux[h + 2 + i] = aux[ph_off + 2 + i];
      if (lane == 0) {
        aux[h] = n;
        aux[h + 1] = ncap;
      }
      wsync();
      ph_off = h;
    }
    if (lane < 8) {
      const uint32_t v = lane == 0 ? node : lane == 1 ? w1 : lane == 2 ? w2 : lane == 3 ? w3 : lane == 4 ? w4
                         : lane == 5 ? w5 : lane == 6 ? kind : w7;
      aux[ph_off + 2 + 8 * n + lane] = v;
    }
    if (lane == 0) aux[ph_off] = n + 1;
    wsync();
  }
  __device__ __forceinline__ void ph_clear(uint32_t node) {
    const uint32_t n = U(aux[ph_off]);
    uint32_t w = 0;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      const bool v = i < n;
      uint32_t e[8];
#pragma unroll
      for (int q = 0; q < 8; q++) e[q] = v ? aux[ph_off + 2 + 8 * i + q] : 0u;
      const bool keep = v && e[0] != node;
      const unsigned long long m = __ballot(keep);
      wsync();  // (the chunk is read before its entries move down: w <= base)
      if (keep) {
        const uint32_t o = w + rank_below(m);
#pragma unroll
        for (int q = 0; q < 8; q++) aux[ph_off + 2 + 8 * o + q] = e[q];
      }
      w += (uint32_t)__popcll(m);
      wsync();
    }
    if (lane == 0) aux[ph_off] = w;
    wsync();
  }
  // nodeUpdateLengthNewStructure(X) / PartialSequenceLengths.combine(X) for the table
  __device__ __forceinline__ void ph_combine(uint32_t X) {
    ph_clear(X);
    if (bad()) return;
    const uint32_t cnt = U(blk[X].count);
    const uint32_t c0 = cnt ? U(blk[X].f[F_ID][0]) : (uint32_t)MTB_LEAF;
    if (c0 & MTB_LEAF) return;  // a block of segments: fromLeaves, exact
    const uint32_t kid = (uint32_t)lane < cnt ? blk[X].f[F_ID][lane] : MTB_NONE;
    const uint32_t n = U(aux[ph_off]);
    for (uint32_t base = 0; base < n && !err; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      const uint32_t node = i < n ? aux[ph_off + 2 + 8 * i] : MTB_NONE;
      const uint32_t kind = i < n ? aux[ph_off + 2 + 8 * i + 6] : PH_DEF_MAIN;
      bool match = false;
      for (uint32_t q = 0; q < cnt; q++) match |= node == rlu(kid, (int)q);
      match &= kind == PH_PHANTOM || kind == PH_DEF_MIN;
      unsigned long long m = __ballot(match);
      while (m && !err) {
        const uint32_t t = base + (uint32_t)first_set(m);
        m &= m - 1;
        const uint32_t o = ph_off + 2 + 8 * t;
        ph_add(X, U(aux[o + 1]), U(aux[o + 2]), U(aux[o + 3]), U(aux[o + 4]), U(aux[o + 5]), U(aux[o + 6]),
               U(aux[o + 7]));
      }
    }
  }
  // blockUpdatePathLengths(b, .., newStructure = true): b and every ancestor, bottom-up
  __device__ __forceinline__ void ph_up(uint32_t b) {
    for (int guard = 0; b != MTB_NONE && !err; guard++) {
      if (guard >= MTB_VDEPTH || b >= blk_used) { fail(DERR_SHAPE); return; }
      ph_combine(b);
      b = U(blk[b].parent);
    }
  }
  // update() of the blocks `a` and path[lo..hi] (partialLengths.ts:682-684 zamboni): copyDown moves the
  // main-set deficits whose first short entry is at or below minSeq into minLength
  __device__ __forceinline__ void ph_touch(uint32_t a, int lo, int hi) {
    const uint32_t n = U(aux[ph_off]);
    bool any = false;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      if (i < n && aux[ph_off + 2 + 8 * i + 6] == PH_DEF_MAIN && (int)aux[ph_off + 2 + 8 * i + 1] <= minSeq) {
        const uint32_t node = aux[ph_off + 2 + 8 * i];
        bool hit = node == a;
        for (int q = lo; q <= hi; q++) hit |= node == U(sh->path[q]);
        if (hit) {
          aux[ph_off + 2 + 8 * i + 6] = PH_DEF_MIN;
          any = true;
        }
      }
    }
    if (__ballot(any)) wsync();
  }
  __device__ __forceinline__ void ph_touch_up(uint32_t b) {
    for (int guard = 0; b != MTB_NONE && guard < MTB_VDEPTH; guard++) {
      ph_touch(b, 1, 0);
      b = U(blk[b].parent);
    }
  }
  // the surplus of each block child of the record on lanes 0..7 (ids `w`) in the (Rl, C) view, into corr[]
  __device__ __forceinline__ int ph_view(uint32_t w, int count, int Rl, int C) {
    if (lane < MTB_MAXCH) sh->corr[lane] = 0;
    wsync();
    const uint32_t n = U(aux[ph_off]);
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      uint32_t node = MTB_NONE, w1 = 0, len = 0, w3 = 0, rcx = 0, kind = 0;
      if (i < n) {
        const uint32_t o = ph_off + 2 + 8 * i;
        node = aux[o];
        w1 = aux[o + 1];
        len = aux[o + 2];
        w3 = aux[o + 3];
        rcx = aux[o + 4];
        kind = aux[o + 6];
      }
      int j = -1;
      for (int q = 0; q < count; q++)
        if (node == rlu(w, q) && !(node & MTB_LEAF)) j = q;
      if (j >= 0) {
        if (kind == PH_PHANTOM) {
          bool vis = (int)w1 <= Rl || (int)(int16_t)w3 == C;
          if (!vis && rcx) {
            const uint32_t nr = aux[rcx];
            for (uint32_t r = 0; r < nr && !vis; r++) vis = (int)aux[rcx + 1 + r] == C;
          }
          if (vis) atomicAdd(&sh->corr[j], (int)len);
        } else {
          // getPartialLength (partialLengths.ts:698-716): the main entry latestLeq(refSeq) is short from t on;
          // the client's cliLatest.len - precedingCli.len is short while precedingCli is below t
          const bool hit = kind == PH_DEF_MIN || (kind == PH_DEF_MAIN && Rl >= (int)w1) ||
                           (kind == PH_DEF_CLI && (int)(int16_t)w3 == C && Rl < (int)w1);
          if (hit) atomicAdd(&sh->corr[j], -(int)len);
        }
      }
    }
    wsync();
    return lane < MTB_MAXCH ? sh->corr[lane] : 0;
  }

  // PartialSequenceLengths.update(N, S) (partialLengths.ts:636-686) of a summary body insert: does N's main set
  // hold an entry AT S already, and which entries follow it?  addSeq (:543-577) then replaces that entry's
  // seglen and recomputes its len from the entry before it, while the later entries keep lengths built on the
  // old seglen: short by the segment from `t1` (N's first main entry above S) on, and client C's set the same
  // below `t1c` (C's first entry above S).  A new entry below newer ones is exact (PartialSequenceLengthsSet.
  // addOrUpdate raises them, :24-47).  N = the block at depth d of the walk (d >= 1); its entries are the list
  // entries of its parent tagged with N's slot, plus the phantom inserts of N's table.  A phantom's removal
  // entries (seq = its rseq) are in the exact list but not in the reference's partials: a removal seq counts
  // only when the removals of that op under N outweigh N's phantoms of it.  Checked as the walk places the
  // segment, before its own entries are appended; t1 / t1c = PH_NOSEQ when nothing follows.
  __device__ __forceinline__ static int wave_min(int v) {
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
  }
  __device__ __forceinline__ bool ph_later(int d, int S, int C, int& t1, int& t1c) {
    // N's entries: for d >= 1 the entries of its parent's list tagged with N's slot; for the root (d = 0) its own
    // list whole, or, when the root holds segments, those segments' inserts and removals (fromLeaves' view of
    // them, the segment being placed excluded)
    const uint32_t N = U(sh->path[d]);
    const uint32_t Cm = (uint32_t)C & 0xFFFF;
    const bool leafRoot = d == 0 && (U(sh->v[0].f[F_ID][0]) & MTB_LEAF);
    uint32_t loff = 0, lcnt = 0, lcap = 0, slot = MTB_NONE;
    if (leafRoot) {
      lcnt = (uint32_t)sh->v[0].count;
    } else if (d >= 1) {
      meta_of(d - 1, loff, lcnt, lcap);
      slot = U(sh->slot[d - 1]);
    } else {
      meta_of(0, loff, lcnt, lcap);
    }
    const int skip = leafRoot ? (int)U(ins_slot) : -1;
    // entry i of the source on this lane: up to two (insert, removal) for a segment; kind 0 insert, 1 removal
    // (amount = length removed by its first remover), 2 an overlapping remover (amount 0)
    auto entry = [&](uint32_t i, int which, int& seq, uint32_t& cl, int& kind, int& amt) -> bool {
      if (leafRoot) {
        if ((int)i == skip) return false;
        const uint32_t sq = sh->v[0].f[F_SEQ][i], rs = sh->v[0].f[F_RSEQ][i], ci = sh->v[0].f[F_CLI][i];
        if (which == 0) {
          seq = (int)sq;
          cl = (uint32_t)cli_client(ci) & 0xFFFF;
          kind = 0;
          amt = (int)sh->v[0].f[F_LEN][i];
          return (int)sq >= 0 && (int)sq < MTB_PEND;
        }
        if (!((int)rs >= 0 && (int)rs < MTB_PEND)) return false;
        seq = (int)rs;
        cl = (uint32_t)cli_rc0(ci) & 0xFFFF;
        kind = 1;
        amt = (int)sh->v[0].f[F_LEN][i];
        return true;
      }
      if (which != 0) return false;
      const WEnt e = lst[loff + i];
      const uint32_t ck = (uint32_t)e.ck, k = (ck >> 16) & 0xF;
      if (slot != MTB_NONE && (ck >> 20) != slot) return false;
      seq = e.seq;
      cl = ck & 0xFFFF;
      kind = k == WK_OVERLAP ? 2 : e.delta < 0 ? 1 : 0;
      amt = e.delta < 0 ? -e.delta : e.delta;
      return true;
    };
    // a leaf root's overlapping removers: client c removed at the segment's rseq too
    auto leaf_rc = [&](uint32_t i, uint32_t c) -> bool {
      const uint32_t rcx = sh->v[0].f[F_RCX][i];
      if (!rcx) return false;
      const uint32_t nr = aux[rcx];
      for (uint32_t r = 0; r < nr; r++)
        if (((uint32_t)aux[rcx + 1 + r] & 0xFFFF) == c) return true;
      return false;
    };
    bool atS = false;
    int mi = PH_NOSEQ, mc = PH_NOSEQ;
    for (uint32_t base = 0; base < lcnt; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      if (i < lcnt) {
        int seq, kind, amt;
        uint32_t cl;
        if (entry(i, 0, seq, cl, kind, amt) && kind == 0) {
          atS |= seq == S;
          if (seq > S && seq > minSeq) {
            mi = min(mi, seq);
            if (cl == Cm) mc = min(mc, seq);
          }
        }
      }
    }
    const uint32_t n = phDoc ? U(aux[ph_off]) : 0u;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      if (i < n && aux[ph_off + 2 + 8 * i] == N && aux[ph_off + 2 + 8 * i + 6] == PH_PHANTOM) {
        const int q = (int)aux[ph_off + 2 + 8 * i + 5];
        atS |= q == S;
        if (q > S) {
          mi = min(mi, q);
          if ((aux[ph_off + 2 + 8 * i + 7] & 0xFFFF) == Cm) mc = min(mc, q);
        }
      }
    }
    if (__ballot(atS) == 0) return false;
    // removal entries below the insert bounds, lowest seq first, until one is the reference's
    int floor = S;
    for (int guard = 0; guard < (1 << 20); guard++) {
      mi = wave_min(mi);
      mc = wave_min(mc);
      int q = PH_NOSEQ;
      for (uint32_t base = 0; base < lcnt; base += 64) {
        const uint32_t i = base + (uint32_t)lane;
        int seq, kind, amt;
        uint32_t cl;
        if (i < lcnt && entry(i, leafRoot ? 1 : 0, seq, cl, kind, amt) && kind != 0 && seq > floor && seq > minSeq &&
            (seq < mi || (seq < mc && (cl == Cm || (leafRoot && leaf_rc(i, Cm))))))
          q = min(q, seq);
      }
      q = wave_min(q);
      if (q == PH_NOSEQ) break;
      // removed under N at q, less N's phantom lengths removed at q; and whether client C removed there
      int acc = 0;
      bool byC = false;
      for (uint32_t base = 0; base < lcnt; base += 64) {
        const uint32_t i = base + (uint32_t)lane;
        if (i < lcnt) {
          int seq, kind, amt;
          uint32_t cl;
          if (entry(i, leafRoot ? 1 : 0, seq, cl, kind, amt) && kind != 0 && seq == q) {
            if (kind == 1) acc += amt;
            byC |= cl == Cm || (leafRoot && leaf_rc(i, Cm));
          }
        }
      }
      for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t i = base + (uint32_t)lane;
        if (i < n && aux[ph_off + 2 + 8 * i] == N && aux[ph_off + 2 + 8 * i + 6] == PH_PHANTOM &&
            (int)aux[ph_off + 2 + 8 * i + 1] == q)
          acc -= (int)aux[ph_off + 2 + 8 * i + 2];
      }
      for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
      byC = __ballot(byC) != 0;
      if (acc > 0) {
        mi = min(mi, q);
        if (byC) mc = min(mc, q);
      }
      floor = q;
    }
    t1 = wave_min(mi);
    t1c = wave_min(mc);
    return true;
  }
  // the load's update(N, S) with an entry at S (ph_later): the deficits that began at S's entry (recomputed now
  // from the entry before it) begin at the next one; the segment's own length, when it counts at S, leaves a
  // new main deficit from t1 and a client deficit below t1c
  __device__ __forceinline__ void ph_load_update(int d, int S, int C, int len, int t1, int t1c) {
    const uint32_t N = U(sh->path[d]);
    const uint32_t Cm = (uint32_t)C & 0xFFFF;
    const uint32_t n = U(aux[ph_off]);
    bool any = false;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      if (i < n && aux[ph_off + 2 + 8 * i] == N && (int)aux[ph_off + 2 + 8 * i + 1] == S) {
        const uint32_t o = ph_off + 2 + 8 * i, kind = aux[o + 6];
        const bool cli = kind == PH_DEF_CLI && (aux[o + 3] & 0xFFFF) == Cm;
        if (kind == PH_DEF_MAIN || cli) {
          const int t = kind == PH_DEF_MAIN ? t1 : t1c;
          if (t == PH_NOSEQ) aux[o] = MTB_NONE;
          else aux[o + 1] = (uint32_t)t;
          any = true;
        }
      }
    }
    if (__ballot(any)) wsync();
    if (len > 0 && t1 != PH_NOSEQ) ph_add(N, (uint32_t)t1, (uint32_t)len, 0u, 0u, (uint32_t)S, PH_DEF_MAIN);
    if (bad()) return;
    if (len > 0 && t1c != PH_NOSEQ) ph_add(N, (uint32_t)t1c, (uint32_t)len, Cm, 0u, (uint32_t)S, PH_DEF_CLI);
  }

  // blockInsert's continuePredicate (mergeTree.ts:1611-1615, forwardExcursion mergeTreeNodeWalk.ts:121-138):
  // is the first segment after block b in tree order an unacked local insert?  From each ancestor, the
  // next sibling's leftmost descent (an empty block there moves on to the following sibling).
  __device__ __forceinline__ bool next_leaf_pending(uint32_t b) {
    uint32_t cur = b;
    for (int guard = 0; guard < MTB_VDEPTH; guard++) {
      const uint32_t par = U(blk[cur].parent);
      if (par == MTB_NONE) return false;
      const uint32_t pc = U(blk[par].count);
      for (uint32_t i = U(blk[cur].index) + 1; i < pc; i++) {
        uint32_t c = U(blk[par].f[F_ID][i]);
        uint32_t seq = U(blk[par].f[F_SEQ][i]);
        while (!(c & MTB_LEAF)) {
          if (U(blk[c].count) == 0) { c = MTB_NONE; break; }
          seq = U(blk[c].f[F_SEQ][0]);
          c = U(blk[c].f[F_ID][0]);
        }
        if (c != MTB_NONE) return (int)seq >= MTB_PEND;
      }
      cur = par;
    }
    fail(DERR_DEPTH);
    return false;
  }

  // ------------------------------------------------------------------ insertingWalk
  // mode 0: ensureIntervalBoundary (seq = TreeMaintenance, leaf = splitLeafSegment)
  // mode 1: blockInsert of the staged segment sh->nseg (seq S).  Returns false if it was not placed.
  // `resume`: start at the leaf-level block reached by the previous walk (same (R, C) and position, no
  // block split since): internal-level decisions of both walks are identical (blocks tie-break the same
  // way in both modes and a segment split changes no block length).
  __device__ __forceinline__ bool walk(int pos, int R, int C, int S, bool insertMode, int candLen, bool resume = false) {
    uint32_t b = root;
    int p = pos;
    int d = 0;
    bool haveMeta = false;  // the list metadata of block b (its parent's slot fields, read from registers)
    uint32_t mo = 0, mc = 0, mk = 0;
    if (resume && walk_depth >= 0 && !struct_changed) {
      d = walk_depth;
      b = U(sh->path[d]);
      p = U(sh->pp[d]);
    }
    walk_depth = -1;
    struct_changed = false;
    int from = 0;  // MODE_LIVE: first slot to consider (a walk resumed past theUnfinishedNode)
    while (true) {
      if (d >= MTB_VDEPTH) { fail(DERR_DEPTH); return false; }
      if (lane == 0) {
        sh->path[d] = b;
        sh->pp[d] = p;
      }
      wsync();
      Kid k;
      const int count = load_view(d, b, R, C, k, haveMeta, mo, mc, mk);
      const View& V = sh->v[d];
      const int fromv = isLive ? from : 0;
      uint32_t cid = MTB_NONE;
      int clen = 0, cseq = 0;
      if (lane < count && lane >= fromv) {
        cid = k.id;
        clen = k.rl;
        cseq = (int)k.seq;
      }
      const int def = (lane < count && clen > 0) ? clen : 0;
      const int incl = cscan8(def);
      const int pj = p - (incl - def);
      const bool isBlk = lane < count && lane >= fromv && !(cid & MTB_LEAF);
      const bool tie = isBlk || (insertMode && pj == 0 && S > cseq);
      const bool qual = lane < count && lane >= fromv && clen != MTB_UNDEF && (pj < clen || (pj == clen && tie));
      const unsigned long long m = __ballot(qual);
      int at;
      if (m) {
        const int j = first_set(m);
        const uint32_t cj = rlu(cid, j);
        const int pjj = rl(pj, j);
        if (lane == 0) sh->slot[d] = j;
        wsync();
        if (!(cj & MTB_LEAF)) {
          haveMeta = true;
          mo = rlu(k.seq, j);
          mc = rlu(k.rseq, j);
          mk = rlu(k.cli, j);
          b = cj;
          p = pjj;
          d++;
          if (isLive) from = 0;
          continue;
        }
        walk_depth = d;
        if (!insertMode) {
          if (pjj <= 0) return true;  // splitLeafSegment: pos 0 -> no change
          if (!isPerm && (U(V.f[F_TEXT][j]) & MTB_MARKER)) return true;  // markers never split
          split_seg(d, j, pjj);
          if (bad()) return false;
          mk_remap_view(d);  // blockUpdateLength of the leaf block, or split's updates of its halves
          pending_fix = d;  // (handled by the caller, after the walk)
          return true;
        }
        at = j;
      } else {
        const int total = rl(incl, 7);
        if (isLive && p - total == 0 && insertMode && S < MTB_PEND && d > 0 && next_leaf_pending(b)) {
          // theUnfinishedNode (mergeTree.ts:1785-1787, 1816-1824): a sequenced insert at the end of this
          // block goes on past it when the next segment is an unacked local insert: the parent's scan
          // continues after this child at position 0
          d--;
          b = U(sh->path[d]);
          p = 0;
          from = U(sh->slot[d]) + 1;
          haveMeta = false;
          continue;
        }
        if (p - total == 0) walk_depth = d;
        if (p - total != 0 || !insertMode) return !insertMode;
        at = count;
      }
      // blockInsert: place the staged segment at slot `at` of the block at depth d
      ins_depth = d;
      ins_slot = at;
      ins_blk = b;
      ins_scour = U(V.scour);
      if (lane == 0) sh->slot[d] = at;
      wsync();
      insert_slot(d, at);
      mk_remap_view(d);
      add_len_levels(0, d, d, candLen);
      if constexpr (isLoad) {
        ld_stale = 0;
        // (a collaborating client's segment: update() on the path, see ph_later; one removed at its own seq adds
        // nothing at S, so it leaves no deficit, but its entry at S is still recomputed)
        if (C != -2) {
          const int own = (int)U(sh->nseg[F_RSEQ]) != S ? (int)U(sh->nseg[F_LEN]) : 0;  // (its cachedLength)
          for (int i = 0; i <= d && !err; i++) {
            if (!phDoc && i == 0) continue;  // (the root's partial lengths are never walked)
            int t1, t1c;
            if (!ph_later(i, S, C, t1, t1c)) continue;
            if (phDoc) ph_load_update(i, S, C, own, t1, t1c);
            else if (own > 0 && t1 != PH_NOSEQ) ld_stale |= 1u << i;
          }
          if (bad()) return false;
        }
        load_entries(d, S, C);
      } else {
        append_levels(0, d, S, C, WK_MAIN, candLen);
        if constexpr (hasPh) {
          if (COLD(phDoc) && S < MTB_PEND) ph_touch(MTB_NONE, 1, d);  // (blockInsert's update() of the path)
        }
      }
      pending_fix = d;
      return true;
    }
  }
  // BaseSegment.splitAt (mergeTreeNodes.ts:481-510) + TextSegment.createSplitSegmentAt (textSegment.ts:106):
  // the segment in slot j of the block at depth d is cut at offset `at`; the right half goes to slot j + 1.
  __device__ __forceinline__ void split_seg(int d, int j, int at) {
    const uint32_t r = alloc_seg();
    if (bad()) return;
    View& V = sh->v[d];
    if (lane < 8) {
      uint32_t v = V.f[lane][j];
      if (lane == F_ID) v = MTB_LEAF | r;
      if (lane == F_LEN) v = v - (uint32_t)at;
      // text offset + at; PermutationSegment: start + at unless unallocated (permutationvector.ts:126-140)
      if (lane == F_TEXT && !(isPerm && v == MTB_HANDLE_UNALLOC)) v = v + (uint32_t)at;
      sh->nseg[lane] = v;
    }
    wsync();
    if (lane == 0) {
      V.f[F_LEN][j] = (uint32_t)at;
      blk[V.b].f[F_LEN][j] = (uint32_t)at;
    }
    n_mod += 2;
    wsync();
    insert_slot(d, j + 1);
    if (isLive && (pend_n > 0 || COLD(U(ds->orphans) != 0))) grp_split(U(V.f[F_ID][j]) & ~MTB_LEAF, r);
  }

  // ------------------------------------------------------------------ LRU heap (collections/heap.ts)
  __device__ __forceinline__ Lru hget(uint32_t k) const {
    Lru x;
    if (heap_lds) {
      const u32x2 y = *reinterpret_cast<const u32x2*>(&sh->heap[k]);
      x.seg = y.x;
      x.maxSeq = (int)y.y;
    } else {
      const auto g = UP(sh->gheap) + k;
      x.seg = g->seg;
      x.maxSeq = g->maxSeq;
    }
    x.seg = U(x.seg);
    x.maxSeq = U(x.maxSeq);
    return x;
  }
  // children j and j + 1 (j even) with one round trip: a 16-byte LDS read, or two global loads in flight
  __device__ __forceinline__ void hget2(uint32_t j, Lru& a, Lru& b) const {
    if (heap_lds) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(&sh->heap[j]);
      a.seg = v.x;
      a.maxSeq = (int)v.y;
      b.seg = v.z;
      b.maxSeq = (int)v.w;
    } else {
      const auto g = UP(sh->gheap) + j;
      a.seg = g[0].seg;
      a.maxSeq = g[0].maxSeq;
      b.seg = g[1].seg;
      b.maxSeq = g[1].maxSeq;
    }
    a.seg = U(a.seg);
    a.maxSeq = U(a.maxSeq);
    b.seg = U(b.seg);
    b.maxSeq = U(b.maxSeq);
  }
  __device__ __forceinline__ void hset(uint32_t k, Lru v) {
    if (heap_lds) {
      u32x2 y;
      y.x = v.seg;
      y.y = (uint32_t)v.maxSeq;
      *reinterpret_cast<u32x2*>(&sh->heap[k]) = y;
    } else {
      const auto g = UP(sh->gheap) + k;
      g->seg = v.seg;
      g->maxSeq = v.maxSeq;
    }
  }
  __device__ __forceinline__ void heap_spill() {  // LDS -> global slice
    for (uint32_t i = 1 + lane; i <= heap_cnt; i += 64) {
      const u32x2 v = *reinterpret_cast<const u32x2*>(&sh->heap[i]);
      sh->gheap[i].seg = v.x;
      sh->gheap[i].maxSeq = (int)v.y;
    }
    heap_lds = false;
    wsync();
  }
  __device__ __forceinline__ void heap_add(uint32_t s, int maxSeq) {
    if (heap_cnt + 1 >= U(sh->capv[4])) { fail(DERR_CAP_HEAP); return; }
    if (COLD(heap_lds && heap_cnt + 1 >= lheap_n)) heap_spill();
    uint32_t k = ++heap_cnt;
    Lru x;
    x.seg = s;
    x.maxSeq = maxSeq;
    while (k > 1) {
      const Lru par = hget(k >> 1);
      if (!(par.maxSeq - x.maxSeq > 0)) break;
      hset(k, par);
      k >>= 1;
    }
    hset(k, x);
  }
  __device__ __forceinline__ Lru heap_get() {
    const Lru top = hget(1);
    const Lru last = hget(heap_cnt);
    heap_cnt--;
    const uint32_t count = heap_cnt;
    uint32_t k = 1;
    // fixDown with the last element placed at the root (collections/heap.ts:50-64)
    while ((k << 1) <= count) {
      uint32_t j = k << 1;
      Lru a, bb;
      hget2(j, a, bb);  // (j + 1 <= the old count: inside the heap's storage)
      if (j < count && a.maxSeq - bb.maxSeq > 0) {
        j++;
        a = bb;
      }
      if (last.maxSeq - a.maxSeq <= 0) break;
      hset(k, a);
      k = j;
    }
    if (count >= 1) hset(k, last);
    return top;
  }
  // addToLRUSet (mergeTree.ts:741-751); `b` is the segment's parent block, `scour` its needsScour
  __device__ __forceinline__ bool lru_add(uint32_t sid, uint32_t b, int scour, int seqv) {
    if (seqv > curSeq && scour != 1) {
      if (lane == 0) blk[b].scour = 1;
      heap_add(sid, seqv);
      return true;
    }
    return false;
  }

  // ------------------------------------------------------------------ pending segment groups (MODE_LIVE)
  // The FIFO of SegmentGroups (pendingSegments, mergeTree.ts:532): directory entry i (0 = oldest) is
  // [localSeq, member list offset, count, capacity, op type, op props id] in the aux arena.
  __device__ __forceinline__ gptr<uint32_t> grp_ent(uint32_t i) const {
    return UP(RAW(aux)) + pend_dir + MTB_PEND_ENT * ((pend_head + i) & (pend_cap - 1));
  }
  // room for one more group at the FIFO's tail: the directory starts at MTB_PEND_GROUPS entries and doubles
  // when full (the pending entries move to the front of the new one, oldest first)
  __device__ bool grp_room() {
    if (pend_n < pend_cap) return true;
    const uint32_t ncap = pend_cap ? 2 * pend_cap : MTB_PEND_GROUPS;
    if (ncap > MTB_PEND_MAX) { fail(DERR_CAP_PEND); return false; }
    const uint32_t nd = alloc_aux(MTB_PEND_ENT * ncap);
    if (bad()) return false;
    const auto dst = UP(RAW(aux)) + nd;
    for (uint32_t w = (uint32_t)lane; w < MTB_PEND_ENT * pend_n; w += 64) dst[w] = grp_ent(w / MTB_PEND_ENT)[w % MTB_PEND_ENT];  // (per lane)
    wsync();
    pend_dir = nd;
    pend_head = 0;
    pend_cap = ncap;
    return true;
  }
  // addToPendingList (mergeTree.ts:1324-1357): segment `sid` joins the current local op's group (made on
  // its first segment; `type` / `props` name the op: an ANNOTATE group's keys are pending on its members)
  __device__ __forceinline__ void grp_add(uint32_t sid, uint32_t type, uint32_t props) {
    if (!grp_open) {
      if (!grp_room()) return;
      const uint32_t off = alloc_aux(8);
      if (bad()) return;
      const auto e = grp_ent(pend_n);
      if (lane == 0) {
        e[0] = (uint32_t)local_seq;
        e[1] = off;
        e[2] = 0;
        e[3] = 8;
        e[4] = type;
        e[5] = props;
        if (type == MTB_OP_ANNOTATE) ds->pend_ann = ds->pend_ann + 1;
      }
      wsync();
      pend_n++;
      grp_open = true;
    }
    grp_push(pend_n - 1, sid);
  }
  // PropertiesManager.pendingKeyUpdateCount of segment `sid` (segmentPropertiesManager.ts:60-157): the keys
  // of the pending ANNOTATE groups holding it, collected at sh->hold[2] (at most 64); returns their number.
  // A group's props word carries MTB_GRP_REWRITE for a local rewrite: its null keys are not pending
  // (:126-131), and pk_rw reports pendingRewriteCount > 0 (a remote annotate then leaves the segment alone).
  __device__ __forceinline__ uint32_t pending_keys_of(uint32_t pw, uint32_t nk) {
    const bool rw = (pw & MTB_GRP_REWRITE) != 0;
    if (rw) pk_rw = true;
    const auto op = UP(sh->tab.pool) + U(UP(sh->tab.pidx)[2 * (pw & ~MTB_GRP_REWRITE)]);
    const uint32_t nop = U(op[0]);
    for (uint32_t q0 = 0; q0 < nop; q0 += 64) {
      const uint32_t q = q0 + (uint32_t)lane;
      const bool take = q < nop && !(rw && op[2 + 2 * q] == MTB_NONE);
      const unsigned long long m = __ballot(take);
      const uint32_t at = nk + rank_below(m);
      if (take && at < 64) sh->hold[2][at] = op[1 + 2 * q];
      nk += (uint32_t)__popcll(m);
      if (nk > 64) nk = 64;
    }
    wsync();
    return nk;
  }
  __device__ __forceinline__ uint32_t pending_keys(uint32_t sid) {
    uint32_t nk = 0;
    pk_rw = false;
    for (uint32_t i = 0; i < pend_n && !err; i++) {
      const auto e = grp_ent(i);
      if (U(e[4]) != MTB_OP_ANNOTATE) continue;
      const uint32_t off = U(e[1]), cnt = U(e[2]);
      bool found = false;
      for (uint32_t q = 0; q < cnt && !found; q += 64) found = __ballot(q + lane < cnt && aux[off + q + lane] == sid) != 0;
      if (!found) continue;
      nk = pending_keys_of(U(e[5]), nk);
    }
    const uint32_t orp = U(ds->orphans);
    if (COLD(orp != 0)) {  // keys a reconnect left pending without a group
      const uint32_t n = U(aux[orp]);
      for (uint32_t i = 0; i < n && !err; i++) {
        if (U(aux[orp + 3 + 2 * i]) != sid) continue;
        nk = pending_keys_of(U(aux[orp + 2 + 2 * i]), nk);
      }
    }
    return nk;
  }
  // hold mask for scourNode (zamboni.ts:122-193): a segment with pending groups stays as it is; pending
  // inserts / removes carry MTB_PEND tags, segments of pending annotates are found in their groups
  __device__ __forceinline__ bool annotate_pending(uint32_t id) {
    bool held = false;
    for (uint32_t i = 0; i < pend_n && !err; i++) {
      const auto e = grp_ent(i);
      if (U(e[4]) != MTB_OP_ANNOTATE) continue;
      const uint32_t off = U(e[1]), cnt = U(e[2]);
      for (uint32_t q = 0; q < cnt; q += 64) {
        const uint32_t m = q + lane < cnt ? aux[off + q + lane] : MTB_NONE;
        const uint32_t nq = cnt - q < 64 ? cnt - q : 64;
        for (uint32_t t = 0; t < nq; t++) held |= (id & ~MTB_LEAF) == rlu(m, (int)t) && (id & MTB_LEAF);
      }
    }
    return held;
  }
  // append a member to directory entry i (its list doubles when full)
  __device__ __forceinline__ void grp_push(uint32_t i, uint32_t sid) {
    const auto e = grp_ent(i);
    uint32_t off = U(e[1]);
    const uint32_t cnt = U(e[2]), cap = U(e[3]);
    if (cnt >= cap) {
      const uint32_t no = alloc_aux(2 * cap);
      if (bad()) return;
      for (uint32_t q = lane; q < cnt; q += 64) aux[no + q] = aux[off + q];
      wsync();
      if (lane == 0) {
        e[1] = no;
        e[3] = 2 * cap;
      }
      off = no;
    }
    if (lane == 0) {
      aux[off + cnt] = sid;
      e[2] = cnt + 1;
    }
    wsync();
  }
  // segmentGroups.copyTo (mergeTreeNodes.ts:239-245) for a split: the right half `r` joins every pending
  // group that holds the left half `s`
  __device__ __forceinline__ void grp_split(uint32_t s, uint32_t r) {
    for (uint32_t i = 0; i < pend_n && !err; i++) {
      const auto e = grp_ent(i);
      const uint32_t off = U(e[1]), cnt = U(e[2]);
      if (off + cnt > aux_used) { fail(DERR_SHAPE); return; }
      bool found = false;
      for (uint32_t q = 0; q < cnt; q += 64) found |= __ballot(q + lane < cnt && aux[off + q + lane] == s) != 0;
      if (found) grp_push(i, r);
    }
    // keys a reconnect left pending on `s` are copied too (PropertiesManager.copyTo)
    const uint32_t orp = U(ds->orphans);
    if (COLD(orp != 0)) {
      const uint32_t n = U(aux[orp]);
      for (uint32_t i = 0; i < n && !err; i++) {
        const uint32_t o = U(ds->orphans);  // (orphan_add may move the list)
        if (U(aux[o + 3 + 2 * i]) == s) orphan_add(U(aux[o + 2 + 2 * i]), r);
      }
    }
  }
  // The lists of every ancestor of block b from its parent up to the root, rebuilt bottom-up from their
  // children (nodeUpdateLengthNewStructure along blockUpdatePathLengths, mergeTree.ts:2419-2434).
  __device__ __forceinline__ void rebuild_up(uint32_t b) {
    if (b >= blk_used) { fail(DERR_SHAPE); return; }
    uint32_t X = U(blk[b].parent);
    for (int guard = 0; X != MTB_NONE && !err; guard++) {
      if (guard >= MTB_VDEPTH || X >= blk_used) { fail(DERR_SHAPE); return; }
      const uint32_t par = U(blk[X].parent), idx = U(blk[X].index);
      uint32_t ooff, ocap;
      if (par == MTB_NONE) {
        ooff = U(blk[X].loff);
        ocap = U(blk[X].lcap);
      } else {
        ooff = U(blk[par].f[F_SEQ][idx]);
        ocap = U(blk[par].f[F_CLI][idx]);
      }
      uint32_t a, c2, e;
      rebuild(X, ooff, ocap, a, c2, e);
      if (bad()) return;
      store_meta_of(X, par, idx, a, c2, e);
      X = par;
    }
  }
  // ackPendingSegment (mergeTree.ts:1283-1322, BaseSegment.ack mergeTreeNodes.ts:439-480) for the client's
  // own op sequenced at S: the oldest group's segments get seq S (insert) or removedSeq S (remove; already
  // set when a remote remove overtook it), join the LRU in group order, and their paths' lists are rebuilt.
  // cprops: the consensus completion of an acked annotateMarkerNotifyConsensus (the op's keys -> {value:
  // undefined, seq: S}, Interner::consensus_props; 0: none), applied to the registered marker -- `mk` = its id's
  // ordinal + 1 -- whether or not the op's range reached it (updateConsensusProperty, client.ts:1050-1058)
  __device__ __forceinline__ void ack_group(int S, int opType, uint32_t cprops = 0, uint32_t mk = 0) {
    if (pend_n == 0) return;
    bool ack_ow = false;
    const auto e = grp_ent(0);
    const uint32_t off = U(e[1]), cnt = U(e[2]);
    if (off + cnt > aux_used) { fail(DERR_SHAPE); return; }
    pend_head = (pend_head + 1) & (pend_cap - 1);
    pend_n--;
    if (opType != 0 && opType != 1 && opType != 2) { fail(DERR_LOCAL); return; }
    if (U(e[4]) == MTB_OP_ANNOTATE) {  // ackPendingProperties: the group's keys stop being pending
      if (lane == 0) ds->pend_ann = ds->pend_ann - 1;
      wsync();
    }
    for (uint32_t i = 0; i < cnt && !err; i++) {
      const uint32_t sid = U(aux[off + i]);
      if (sid >= seg_used) { fail(DERR_SHAPE); return; }
      const uint32_t b = U(segp[sid]);
      if (b >= blk_used) { fail(DERR_SHAPE); return; }
      const uint32_t* rec = bw(b);
      const uint32_t id = lane < MTB_MAXCH ? rec[F_ID * 8 + lane] : MTB_NONE;
      const unsigned long long m = __ballot(id == (MTB_LEAF | sid));
      if (!m) { fail(DERR_SHAPE); return; }
      const int j = first_set(m);
      const int sq = (int)U(rec[F_SEQ * 8 + j]), rs = (int)U(rec[F_RSEQ * 8 + j]);
      const int sc = (int)U(blk[b].scour);
      if (opType == 2) {
        // (annotate: no seq to stamp; the lengths are unchanged, so no list needs rebuilding below)
      } else if (opType == 0) {
        if (sq < MTB_PEND) { fail(DERR_ACK_INSERT); return; }
        if (lane == 0) blk[b].f[F_SEQ][j] = (uint32_t)S;
      } else {
        if (rs < 0) { fail(DERR_ACK_REMOVE); return; }
        if (rs >= MTB_PEND && lane == 0) blk[b].f[F_RSEQ][j] = (uint32_t)S;
        if (rs < MTB_PEND) ack_ow = true;  // a remote remove overtook it: overwrite (mergeTree.ts:1300-1312)
      }
      n_mod += 1;
      wsync();
      lru_add(sid, b, sc, S);  // addToLRUSet(segment, seq)
    }
    if constexpr (hasMk) {
      if (COLD(cprops != 0 && mk != 0)) {
        const uint32_t ord = mk - 1;
        const uint32_t sid = ord < U(ds->mk_n) ? U(aux[U(ds->mk_map) + ord]) : MTB_NONE;
        const uint32_t b = sid < seg_used ? U(segp[sid]) : MTB_NONE;
        if (b < blk_used) {
          const uint32_t id = lane < MTB_MAXCH ? blk[b].f[F_ID][lane] : MTB_NONE;
          const unsigned long long m = __ballot(id == (MTB_LEAF | sid));
          if (m) {
            const int j = first_set(m);
            const uint32_t np = props_apply_slow(U(blk[b].f[F_PROPS][j]), cprops, 5);
            if (bad()) return;
            memo_old = MTB_NONE;
            if (lane == 0) blk[b].f[F_PROPS][j] = np;
            wsync();
          }
        }
      }
    }
    // nodesToUpdate (distinct parents in first-appearance order): blockUpdate re-maps marker ids
    // (mergeTree.ts:1316 -> :2392), annotate acks included
    if constexpr (hasMk) {
      if (COLD(mkDup)) {
        for (uint32_t i = 0; i < cnt && !err; i++) {
          const uint32_t b = U(segp[U(aux[off + i])]);
          bool seen = false;
          for (uint32_t q = 0; q < i; q += 64) seen |= __ballot(q + lane < i && segp[aux[off + q + lane]] == b) != 0;
          if (!seen) mk_remap_blk(b);
        }
      }
    }
    // nodesToUpdate: the distinct parents, in order (a repeat only rebuilds again)
    uint32_t prev = MTB_NONE;
    for (uint32_t i = 0; i < cnt && !err && opType != 2; i++) {
      const uint32_t b = U(segp[U(aux[off + i])]);  // (ids checked above)
      if (b != prev) rebuild_up(b);
      prev = b;
    }
    if constexpr (hasPh) {
      // blockUpdatePathLengths(node, seq, clientId, overwrite): recombined only with overwrite
      // (and update() otherwise, annotate acks included: copyDown, ph_touch)
      if (COLD(phDoc)) {
        for (uint32_t i = 0; i < cnt && !err; i++) {
          const uint32_t b = U(segp[U(aux[off + i])]);
          bool seen = false;
          for (uint32_t q = 0; q < i; q++) seen |= U(segp[U(aux[off + q])]) == b;
          if (seen) continue;
          if (ack_ow) ph_up(b);
          else ph_touch_up(b);
        }
      }
    }
    view_clear();
  }

  // ------------------------------------------------------------------ reconnect (MODE_LIVE)
  // The leaf-level blocks (children are segments) in tree order: f(block) for each, over an explicit
  // stack in sh->path / sh->sidx (no walk is active while a REGEN record runs).
  template <class F>
  __device__ __forceinline__ void each_leaf_block(F&& f) {
    int d = 0;
    if (lane == 0) {
      sh->path[0] = root;
      sh->sidx[0] = 0;
    }
    wsync();
    for (int guard = 0; !err; guard++) {
      if (guard > (int)(4 * blk_used + 64)) { fail(DERR_SHAPE); return; }
      const uint32_t b = U(sh->path[d]);
      const int cnt = (int)U(blk[b].count);
      const uint32_t c0 = cnt ? U(blk[b].f[F_ID][0]) : MTB_NONE;
      int k = U(sh->sidx[d]);
      if (cnt == 0 || (c0 & MTB_LEAF)) {
        if (cnt && k == 0) f(b);
        k = cnt;
      }
      if (k >= cnt) {
        if (d == 0) return;
        d--;
        continue;
      }
      if (d + 1 >= MTB_VDEPTH) { fail(DERR_DEPTH); return; }
      const uint32_t c = U(blk[b].f[F_ID][k]);
      if (lane == 0) {
        sh->sidx[d] = k + 1;
        sh->path[d + 1] = c;
        sh->sidx[d + 1] = 0;
      }
      wsync();
      d++;
    }
  }
  // a new pending group with one member at the FIFO's tail (resetPendingDeltaToOps' newSegmentGroup)
  __device__ __forceinline__ void grp_new(uint32_t lseq, uint32_t type, uint32_t props, uint32_t sid) {
    if (!grp_room()) return;
    const uint32_t off = alloc_aux(8);
    if (bad()) return;
    const auto e = grp_ent(pend_n);
    if (lane == 0) {
      e[0] = lseq;
      e[1] = off;
      e[2] = 1;
      e[3] = 8;
      e[4] = type;
      e[5] = props;
      aux[off] = sid;
      if (type == MTB_OP_ANNOTATE) ds->pend_ann = ds->pend_ann + 1;
    }
    wsync();
    pend_n++;
  }
  // an annotate group member that a reconnect regenerated no op for keeps its pending keys
  __device__ __forceinline__ void orphan_add(uint32_t props, uint32_t sid) {
    uint32_t o = U(ds->orphans);
    const uint32_t n = o ? U(aux[o]) : 0, cap = o ? U(aux[o + 1]) : 0;
    if (n >= cap) {
      const uint32_t nc = cap ? 2 * cap : 8;
      const uint32_t no = alloc_aux(2 + 2 * nc);
      if (bad()) return;
      for (uint32_t i = lane; i < 2 * n; i += 64) aux[no + 2 + i] = aux[o + 2 + i];
      if (lane == 0) {
        aux[no + 1] = nc;
        ds->orphans = no;
      }
      o = no;
    }
    if (lane == 0) {
      aux[o] = n + 1;
      aux[o + 2 + 2 * n] = props;
      aux[o + 3 + 2 * n] = sid;
    }
    wsync();
  }
  // localNetLength(segment, currentSeq, localSeq) (mergeTree.ts:636-664): the local view as it was after
  // local op L (later local ops hidden; every sequenced op is at or below currentSeq)
  __device__ __forceinline__ int len_at(int len, int seq, int rseq, int L) const {
    const bool lrem = rseq >= MTB_PEND && rseq - MTB_PEND <= L;
    if (seq < MTB_PEND) return ((rseq >= 0 && rseq < MTB_PEND) || lrem) ? 0 : len;
    return (seq - MTB_PEND > L || lrem) ? 0 : len;
  }
  // cachedLength of leaf-level block b from its children, the difference carried up the ancestors
  __device__ __forceinline__ void fix_len(uint32_t b) {
    const uint32_t* r = bw(b);
    const int cnt = (int)U(r[FB_HDR]);
    int ol = 0;
    if (lane < cnt) ol = child_olen(r[F_ID * 8 + lane], (int)r[F_LEN * 8 + lane], (int)r[F_RSEQ * 8 + lane]);
    const int nl = csum8(ol);
    const int delta = nl - (int)U(blk[b].len);
    if (!delta) return;
    uint32_t X = b;
    if (lane == 0) blk[b].len = nl;
    for (int guard = 0; guard < MTB_VDEPTH; guard++) {
      const uint32_t P = U(blk[X].parent);
      if (P == MTB_NONE) break;
      const uint32_t ix = U(blk[X].index);
      if (lane == 0) {
        blk[P].f[F_LEN][ix] = (uint32_t)((int)blk[P].f[F_LEN][ix] + delta);
        blk[P].len = blk[P].len + delta;
      }
      wsync();
      X = P;
    }
    wsync();
  }
  // normalizeAdjacentSegments (mergeTree.ts:2234-2336) of run entries [0, n) at scratch `sc` (6 words
  // each: segment, block, slot, kind, localSeq, localRemovedSeq; kind 1 = removed and acked, 2 = removed);
  // the order list L is at sc + 6n, the gathered fields at sc + 7n.
  __device__ __forceinline__ void normalize_run(uint32_t sc, uint32_t n) {
    const auto E = [&](uint32_t i, int w) { return U(aux[sc + 6 * i + w]); };
    const uint32_t lo = sc + 6 * n;
    for (uint32_t i = lane; i < n; i += 64) aux[lo + i] = i;
    wsync();
    const auto Lr = [&](uint32_t i) { return U(aux[lo + i]); };
    const auto acked = [&](uint32_t e) { return (E(e, 3) & 1) != 0; };
    const auto idx = [&](uint32_t e) {
      uint32_t at = 0;
      for (uint32_t q = 0; q < n; q += 64) {
        const unsigned long long m = __ballot(q + lane < n && aux[lo + q + lane] == e);
        if (m) { at = q + (uint32_t)first_set(m); break; }
      }
      return at;
    };
    const auto erase = [&](uint32_t p) {
      for (uint32_t i = p; i + 1 < n; i++) {
        const uint32_t v = Lr(i + 1);
        if (lane == 0) aux[lo + i] = v;
        wsync();
      }
    };
    const auto insert = [&](uint32_t p, uint32_t e) {  // at index p of the n-1 remaining
      for (uint32_t i = n - 1; i > p; i--) {
        const uint32_t v = Lr(i - 1);
        if (lane == 0) aux[lo + i] = v;
        wsync();
      }
      if (lane == 0) aux[lo + p] = e;
      wsync();
    };
    int last = (int)n - 1;
    while (last >= 0 && acked(Lr((uint32_t)last))) last--;
    if (last < 0) return;
    const uint32_t lastLocal = Lr((uint32_t)last);
    uint32_t toSlide = lastLocal, nearer = last > 0 ? Lr((uint32_t)last - 1) : MTB_NONE;
    for (uint32_t guard = 0; toSlide != MTB_NONE && !err; guard++) {
      if (guard > n) { fail(DERR_SHAPE); return; }
      const uint32_t p = idx(toSlide);
      if (acked(toSlide)) {
        erase(p);
        insert(idx(lastLocal) + 1, toSlide);
      } else if (E(toSlide, 3) & 2) {
        const int lrs = (int)E(toSlide, 5);
        uint32_t cur = p;
        for (uint32_t sc2 = p + 1; sc2 < n; sc2++) {
          const uint32_t e = Lr(sc2);
          if (acked(e) || (int)E(e, 4) < 0 || (int)E(e, 4) <= lrs) break;
          cur = sc2;
        }
        if (cur != p) {
          erase(p);
          insert(cur, toSlide);
        }
      }
      toSlide = nearer;
      if (nearer != MTB_NONE) {
        const uint32_t q = idx(nearer);
        nearer = q > 0 ? Lr(q - 1) : MTB_NONE;
      }
    }
    // the run's slots keep their places; each takes the fields of its new segment
    const uint32_t F = sc + 7 * n;
    for (uint32_t t = lane; t < 8 * n; t += 64) {
      const uint32_t j = t >> 3, q = t & 7;
      aux[F + t] = blk[aux[sc + 6 * j + 1]].f[q][aux[sc + 6 * j + 2]];
    }
    wsync();
    for (uint32_t t = lane; t < 8 * n; t += 64) {
      const uint32_t i = t >> 3, q = t & 7;
      const uint32_t j = aux[lo + i];
      const uint32_t b = aux[sc + 6 * i + 1], sl = aux[sc + 6 * i + 2];
      blk[b].f[q][sl] = aux[F + 8 * j + q];
      if (q == 0) segp[aux[sc + 6 * j]] = b;
    }
    wsync();
    n_mod += n;
    // nodeUpdateLengthNewStructure of the ancestors: block lengths (and the leaf blocks' marker ids,
    // deepest first, in run order, mergeTree.ts:2320-2331), then the window lists
    uint32_t prev = MTB_NONE;
    for (uint32_t i = 0; i < n && !err; i++) {
      const uint32_t b = E(i, 1);
      if (b != prev) {
        fix_len(b);
        mk_remap_blk(b);
      }
      prev = b;
    }
    prev = MTB_NONE;
    for (uint32_t i = 0; i < n && !err; i++) {
      const uint32_t b = E(i, 1);
      if (b != prev) rebuild_up(b);
      prev = b;
    }
    if constexpr (hasPh) {
      if (COLD(phDoc)) {  // (mergeTree.ts:2320-2331: every ancestor of the moved segments recombined)
        prev = MTB_NONE;
        for (uint32_t i = 0; i < n && !err; i++) {
          const uint32_t b = E(i, 1);
          if (b != prev) ph_up(b);
          prev = b;
        }
      }
    }
  }
  // normalizeSegmentsOnRebase (mergeTree.ts:2357-2390): runs of removed / unacked segments holding both an
  // unacked insert and a remotely removed segment are normalized
  __device__ __forceinline__ void normalize() {
    const uint32_t save = aux_used;
    const uint32_t room = U(sh->capv[5]) > aux_used ? U(sh->capv[5]) - aux_used : 0;
    const uint32_t cap = room / 16 < 4096 ? room / 16 : 4096;  // run entries the scratch holds
    if (cap < 2) return;
    const uint32_t sc = alloc_aux(16 * cap);
    if (bad()) return;
    uint32_t rn = 0;
    bool hasLocal = false, hasRR = false;
    auto flush = [&]() {
      if (hasLocal && hasRR && rn > 1) {
        if (rn > cap) { fail(DERR_CAP_AUX); return; }
        normalize_run(sc, rn);
      }
      rn = 0;
      hasLocal = hasRR = false;
    };
    each_leaf_block([&](uint32_t b) {
      const uint32_t* r = bw(b);
      const int cnt = (int)U(r[FB_HDR]);
      uint32_t id = 0, sq = 0, rs = 0;
      if (lane < MTB_MAXCH) {
        id = r[F_ID * 8 + lane];
        sq = r[F_SEQ * 8 + lane];
        rs = r[F_RSEQ * 8 + lane];
      }
      for (int k = 0; k < cnt && !err; k++) {
        const int seq = rl((int)sq, k), rseq = rl((int)rs, k);
        if (rseq >= 0 || seq >= MTB_PEND) {
          const bool rr = rseq >= 0 && rseq < MTB_PEND;
          hasRR |= rr;
          hasLocal |= seq >= MTB_PEND;
          if (rn < cap && lane == 0) {
            const uint32_t o = sc + 6 * rn;
            aux[o] = rlu(id, k) & ~MTB_LEAF;
            aux[o + 1] = b;
            aux[o + 2] = (uint32_t)k;
            aux[o + 3] = (rr ? 1u : 0u) | (rseq >= 0 ? 2u : 0u);
            aux[o + 4] = (uint32_t)(seq >= MTB_PEND ? seq - MTB_PEND : -1);
            aux[o + 5] = (uint32_t)(rseq >= MTB_PEND ? rseq - MTB_PEND : -1);
          }
          wsync();
          rn++;
        } else {
          flush();
        }
      }
    });
    flush();
    aux_used = save;  // (the scratch is released; the rebuilds allocate list entries, not aux words)
    view_clear();
  }
  // Client.regeneratePendingOp (client.ts:917-960) / resetPendingDeltaToOps (:708-800) for the n groups at
  // the head of the FIFO (one per member op): each group's segments in tree order, each one's position in
  // the local view after the group's localSeq (findReconnectionPosition), an entry per regenerated op and a
  // new one-segment group for it at the FIFO's tail
  __device__ __forceinline__ void regen(uint32_t n) {
    if (curSeq != (int)U(ds->last_norm)) {
      normalize();
      if (bad()) return;
      if (lane == 0) ds->last_norm = curSeq;
      wsync();
    }
    for (uint32_t g = 0; g < n && !err; g++) {
      if (pend_n == 0) { fail(DERR_REGEN); return; }
      const auto e = grp_ent(0);
      const int L = (int)U(e[0]);
      const uint32_t off = U(e[1]), cnt = U(e[2]), type = U(e[4]), props = U(e[5]);
      pend_head = (pend_head + 1) & (pend_cap - 1);
      pend_n--;
      if (type == MTB_OP_ANNOTATE) {
        if (lane == 0) ds->pend_ann = ds->pend_ann - 1;
        wsync();
      }
      if (off + cnt > aux_used) { fail(DERR_SHAPE); return; }
      int pos = 0;
      uint32_t found = 0;
      each_leaf_block([&](uint32_t b) {
        const uint32_t* r = bw(b);
        const int bc = (int)U(r[FB_HDR]);
        uint32_t id = MTB_NONE;
        int l = 0, sq = 0, rs = -1;
        if (lane < bc) {
          id = r[F_ID * 8 + lane];
          sq = (int)r[F_SEQ * 8 + lane];
          rs = (int)r[F_RSEQ * 8 + lane];
          l = len_at((int)r[F_LEN * 8 + lane], sq, rs, L);
        }
        const int excl = cscan8(l) - l;
        unsigned mm = 0;  // slots of this block holding group members
        for (uint32_t q = 0; q < cnt; q += 64) {
          const uint32_t m = q + lane < cnt ? aux[off + q + lane] : MTB_NONE;
          for (int k = 0; k < bc; k++)
            if (__ballot(m == (rlu(id, k) & ~MTB_LEAF))) mm |= 1u << k;
        }
        while (mm && !err) {
          const int k = __ffs(mm) - 1;
          mm &= mm - 1;
          found++;
          const uint32_t sid = rlu(id, k) & ~MTB_LEAF;
          const int sqk = rl(sq, k), rsk = rl(rs, k);
          bool emit;
          if (type == MTB_OP_INSERT) {
            if (sqk < MTB_PEND) { fail(DERR_ACK_INSERT); return; }  // 0x037
            emit = true;
          } else if (type == MTB_OP_REMOVE) {
            emit = rsk >= MTB_PEND;
          } else {
            emit = rsk < 0 || rsk >= MTB_PEND;
          }
          if (emit) {
            if (delta_used + 1 > U(sh->capv[6])) { fail(DERR_CAP_DELTA); return; }
            if (lane == 0) {
              const auto o = dslice() + 4 * delta_used;
              o[0] = cur_k;
              o[1] = type | (g << 8);
              o[2] = sid;
              o[3] = (uint32_t)(pos + rl(excl, k));
            }
            wsync();
            delta_used++;
            grp_new((uint32_t)L, type, props, sid);
          } else if (type == MTB_OP_ANNOTATE) {
            orphan_add(props, sid);
          }
        }
        pos += rl(cscan8(l), 7);
      });
      if (!err && found != cnt) { fail(DERR_REGEN); return; }
    }
    view_clear();
  }

  // ------------------------------------------------------------------ properties
  __device__ __forceinline__ gptr<const uint32_t> props_ptr(uint32_t h) const {
    return (h & MTB_GPROPS) ? (gptr<const uint32_t>)(UP(sh->tab.pool) + (h & ~MTB_GPROPS))
                            : GP((const uint32_t*)RAW(aux) + (h & ~MTB_PNAN));
  }
  // Interner pair tables (mtbk::irr_value_match) with uniform operands, the table pointers in SGPRs
  __device__ __forceinline__ bool irr_match(uint32_t k, uint32_t va, uint32_t vb) const {
    const auto F = UP(sh->tab.val_falsy);  // (NaN / consensus values: irr_value_match)
    if (U((uint32_t)F[vb]) & 8) return false;
    if (U((uint32_t)F[va]) & 8) return va == (U(sh->tab.nan_val) & ~MTB_NAN_CV) && (U((uint32_t)F[vb]) & 16) != 0;
    const uint32_t o = U(UP(sh->tab.key_irr)[k]);
    if (!o) return va == vb || U(UP(sh->tab.val_class)[va]) == U(UP(sh->tab.val_class)[vb]);
    const auto T = UP(sh->tab.irr);
    const auto L = UP(sh->tab.val_local);
    const uint32_t bit = U(L[va]) * U(T[o - 1]) + U(L[vb]);
    return ((U(T[o + bit / 32]) >> (bit % 32)) & 1u) != 0;
  }
  // matchProperties (properties.ts:71-96) on interned property sets; a = the run head's set.  With irregular
  // keys in the batch (tab.irr_any) it is neither reflexive nor symmetric there: no shortcut on equal handles.
  __device__ __forceinline__ bool props_match(uint32_t a, uint32_t b) const {
    // NaN !== NaN: a set holding NaN or a consensus value matches nothing -- except, with irregular keys, a first
    // argument holding NaN under a key whose other value is an object or array without own keys (irr_match)
    const bool irr = hasIrr && U(sh->tab.irr_any) != 0;
    if ((irr ? b : (a | b)) & MTB_PNAN) return false;
    if (a == b && !irr) return true;
    const gptr<const uint32_t> pa = a ? props_ptr(a) : nullptr;
    const gptr<const uint32_t> pb = b ? props_ptr(b) : nullptr;
    const uint32_t na = pa ? pa[0] : 0, nb = pb ? pb[0] : 0;
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
      const uint32_t k = pa[1 + 2 * i];
      bool found = false;
      for (uint32_t q = 0; q < nb; q++) {
        if (pb[1 + 2 * q] == k) {
          found = true;
          const uint32_t va = pa[2 + 2 * i], vb = pb[2 + 2 * q];
          if (COLD(irr)) {
            if (!irr_match(U(k), U(va), U(vb))) return false;
          } else if (va != vb) {
            if (U(sh->tab.class_trivial)) return false;
            const auto vcl = UP(sh->tab.val_class);
            if (vcl[va] != vcl[vb]) return false;
          }
          break;
        }
      }
      if (!found) return false;
    }
    return true;
  }
  // PropertiesManager.addProperties for a sequenced remote op (segmentPropertiesManager.ts:60-157).
  // The key/value list is staged in LDS; all lanes run the (short) edit loop uniformly.
  // comb: 0 none, 1 rewrite, 2 incr, 3 consensus (the annotate's combiningOp)
  __device__ __forceinline__ uint32_t props_apply(uint32_t old, uint32_t opId, int comb) {
    const uint32_t mo = U(memo_old), mn = U(memo_new);
    if (HOT(old == mo && mn)) return mn;
    return props_apply_slow(old, opId, comb);
  }
  // nex > 0: the first nex words of sh->hold[2] are keys this edit leaves alone (pending local keys)
  __device__ __forceinline__ uint32_t props_apply_slow(uint32_t old, uint32_t opId, int comb, uint32_t nex = 0) {
    const bool rewrite = comb == 1;
    auto excluded = [&](uint32_t k) {
      bool x = false;
      for (uint32_t i = 0; i < nex; i++) x |= sh->hold[2][i] == k;
      return x;
    };
    const auto op = UP(sh->tab.pool) + U(UP(sh->tab.pidx)[2 * opId]);
    const uint32_t nop = U(op[0]);
    uint32_t n = 0;
    if (old) {
      const auto po = props_ptr(old);
      n = U(po[0]);
      if (n > 64) n = 64;
      for (uint32_t i = lane; i < n; i += 64) {
        sh->pk[i] = po[1 + 2 * i];
        sh->pv[i] = po[2 + 2 * i];
      }
    }
    wsync();
    if (rewrite) {
      // delete old keys whose new value is falsy/absent (the `!newProps[key]` test)
      uint32_t w = 0;
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = sh->pk[i], v0 = sh->pv[i];
        bool keep = false;
        for (uint32_t q = 0; q < nop; q++) {
          if (op[1 + 2 * q] == k) {
            const uint32_t v = op[2 + 2 * q];
            keep = v != MTB_NONE && !(sh->tab.val_falsy[v] & 1);
          }
        }
        if (!keep && nex && excluded(k)) keep = true;
        if (keep) {
          wsync();
          sh->pk[w] = k;
          sh->pv[w] = v0;
          wsync();
          w++;
        }
      }
      n = w;
    }
    for (uint32_t q = 0; q < nop; q++) {
      const uint32_t k = op[1 + 2 * q];
      uint32_t v = op[2 + 2 * q];
      if (nex && excluded(k)) continue;
      int at = -1;
      for (uint32_t i = 0; i < n; i++)
        if (sh->pk[i] == k) at = (int)i;
      if (COLD(comb == 2)) {
        // incr: combine(op, previous, undefined) (properties.ts:24-69) -- previous + undefined is NaN for numbers /
        // booleans / NaN; a string's, object's or array's result (String(v) + "undefined", minValue) and the absent
        // key's come from the op's table (Interner::incr_props; a value missing from it is an engine invariant)
        const uint32_t nanv = U(sh->tab.nan_val) & ~MTB_NAN_CV;
        const auto T = UP(sh->tab.pool) + (v & ~MTB_INCR_TAB);
        const bool tab = (v & MTB_INCR_TAB) != 0 && v != MTB_NONE;
        if (at < 0) {
          v = tab ? U(T[0]) : nanv;
        } else if (sh->tab.val_falsy[sh->pv[at]] & 2) {
          v = nanv;
        } else {
          const uint32_t pv0 = sh->pv[at], n = tab ? U(T[1]) : 0u;
          uint32_t r = MTB_NONE;
          for (uint32_t base = 0; base < n && r == MTB_NONE; base += 64) {
            const uint32_t i = base + (uint32_t)lane;
            const unsigned long long m = __ballot(i < n && T[2 + 2 * i] == pv0);
            if (m) r = U(T[3 + 2 * (base + (uint32_t)first_set(m))]);
          }
          if (r == MTB_NONE) { fail(DERR_INCR); return 0; }
          v = r;
        }
      } else if (COLD(comb >= 3)) {
        // consensus (properties.ts:46-62): a present value stays -- unless it is an object whose seq is -1,
        // completed in place by the reference (shared with split clones): refused; an absent one takes the
        // host-made value (Interner::consensus_props; MTB_NONE: a null defaultValue, the reference throws).
        // comb 4: a live client's own annotateMarkerNotifyConsensus (seq -1: such an object's seq stays -1);
        // comb 5: its completion at the ack (client.ts:1050-1058): the marker's own pending value {value:
        // undefined, seq: -1} (a consensus value with seq -1, val_falsy bits 2 and 3) takes the ack's seq
        if (at >= 0) {
          const uint32_t f = sh->tab.val_falsy[sh->pv[at]];
          if (!(comb == 5 && (f & 12) == 12)) {
            if (comb != 4 && (f & 4)) { fail(DERR_CONSENSUS); return 0; }
            continue;
          }
        } else if (v == MTB_NONE) {
          fail(DERR_CONS_NULL);
          return 0;
        }
      }
      if (v == MTB_NONE) {
        if (at >= 0) {
          for (uint32_t i = (uint32_t)at; i + 1 < n; i++) {
            const uint32_t kk = sh->pk[i + 1], vv = sh->pv[i + 1];
            wsync();
            sh->pk[i] = kk;
            sh->pv[i] = vv;
            wsync();
          }
          n--;
        }
      } else if (at >= 0) {
        sh->pv[at] = v;
        wsync();
      } else if (n < 64) {
        const uint32_t rank = sh->tab.key_rank[k];
        uint32_t ins = n;
        if (rank != MTB_NONE) {
          ins = 0;
          while (ins < n) {
            const uint32_t r2 = sh->tab.key_rank[sh->pk[ins]];
            if (r2 == MTB_NONE || r2 > rank) break;
            ins++;
          }
        }
        for (uint32_t i = n; i > ins; i--) {
          const uint32_t kk = sh->pk[i - 1], vv = sh->pv[i - 1];
          wsync();
          sh->pk[i] = kk;
          sh->pv[i] = vv;
          wsync();
        }
        sh->pk[ins] = k;
        sh->pv[ins] = v;
        wsync();
        n++;
      }
    }
    uint32_t h = alloc_aux(1 + 2 * n);
    if (bad()) return 0;
    aux[h] = n;
    for (uint32_t i = lane; i < n; i += 64) {
      aux[h + 1 + 2 * i] = sh->pk[i];
      aux[h + 2 + 2 * i] = sh->pv[i];
    }
    const uint32_t nanw = U(sh->tab.nan_val);
    if (COLD(nanw != MTB_NONE)) {  // a set holding NaN or a consensus value matches nothing: its handle says so
      bool hasNan = false;
      for (uint32_t i = lane; i < n; i += 64) hasNan |= sh->pv[i] == (nanw & ~MTB_NAN_CV);
      if (COLD(nanw & MTB_NAN_CV))  // consensus values exist: every no-match value (val_falsy bit 3)
        for (uint32_t i = lane; i < n; i += 64) hasNan |= (sh->tab.val_falsy[sh->pv[i]] & 8) != 0;
      if (__ballot(hasNan)) h |= MTB_PNAN;
    }
    wsync();
    memo_old = old;
    memo_new = h;
    return h;
  }

  // ------------------------------------------------------------------ catch-up deltas
  // SequenceDeltaEvent ranges (sequenceDelta.ts:43-56) for SharedSegmentSequence's rewriting of lagging
  // messages (sequence.ts:697-733): one entry per delta segment, in tree order: [record, segment id ->
  // local position after the op, cachedLength, property set after the op]; a rewrite annotate's segments
  // get a second entry each, tagged MTB_DELTA_OLD, holding the set before the op (its deleted keys).
  __device__ __forceinline__ gptr<uint32_t> dslice() const { return UP(sh->tab.delta) + ds->delta_base * 4; }
  __device__ __forceinline__ void delta_emit(bool sel, uint32_t sid, uint32_t len, uint32_t props, uint32_t tag = 0) {
    const unsigned long long m = __ballot(sel);
    if (!m) return;
    const uint32_t n = (uint32_t)__popcll(m);
    if (delta_used + n > U(sh->capv[6])) { fail(DERR_CAP_DELTA); return; }
    if (sel) {
      const auto e = dslice() + 4 * (delta_used + rank_below(m));
      e[0] = cur_k | tag;
      e[1] = sid;
      e[2] = len;
      e[3] = props;
    }
    delta_used += n;
    wsync();
  }
  // getPosition (mergeTree.ts:1240) of the segments named by entries [from, delta_used): the local
  // lengths left of the segment in its block and left of each ancestor in theirs
  __device__ __forceinline__ void delta_positions(uint32_t from) {
    const auto dl = dslice();
    for (uint32_t i = from; i < delta_used; i++) {
      const uint32_t sid = U(dl[4 * i + 1]);
      uint32_t child = MTB_LEAF | sid;
      uint32_t b = U(segp[sid]);
      int pos = 0;
      while (b != MTB_NONE) {
        const uint32_t* rec = bw(b);
        uint32_t id = MTB_NONE, ln = 0, rs = 0;
        if (lane < MTB_MAXCH) {
          id = rec[F_ID * 8 + lane];
          ln = rec[F_LEN * 8 + lane];
          rs = rec[F_RSEQ * 8 + lane];
        }
        const uint32_t cnt = U(rec[FB_HDR]);
        const uint32_t par = U(rec[FB_HDR + 1]);
        const int j = first_set(__ballot((uint32_t)lane < cnt && id == child));
        const int ol = lane < j ? child_olen(id, (int)ln, (int)rs) : 0;
        pos += csum8(ol);
        child = b;
        b = par;
      }
      if (lane == 0) dl[4 * i + 1] = (uint32_t)pos;
      wsync();
    }
  }

  // ------------------------------------------------------------------ nodeMap (remove / annotate)
  // The segments of one leaf-level block (depth d) touched by [start, end), all lanes at once (the
  // boundaries were split beforehand, so each segment is wholly in or out of the range).  `pos` is the
  // position at the start of the block; returns the block's total visible length.
  __device__ __forceinline__ int map_leaf_block(int d, int pos, int start, int end, int S, int C, bool remove, uint32_t opId,
                                int comb) {
    const bool rewrite = comb == 1;
    View& V = sh->v[d];
    const uint32_t b = U(V.b);
    const int count = U(V.count);
    int rlj = 0;
    if (lane < count) rlj = V.rl[lane];
    const int def = (lane < count && rlj > 0) ? rlj : 0;
    const int incl = cscan8(def);
    const int total = rl(incl, 7);
    const int sj = pos + incl - def;
    const bool visit = lane < count && rlj > 0 && sj < end && start < sj + rlj;
    const unsigned long long vm = __ballot(visit);
    if (!vm) return total;
    n_mod += (uint32_t)__popcll(vm);
    uint32_t id = MTB_NONE, cli = 0, props = 0;
    int len = 0, rseq = -1;
    if (lane < count) {
      id = V.f[F_ID][lane];
      len = (int)V.f[F_LEN][lane];
      rseq = (int)V.f[F_RSEQ][lane];
      cli = V.f[F_CLI][lane];
      props = V.f[F_PROPS][lane];
    }
    if (remove) {
      // fresh removes: removedSeq = S, removedClientIds = [C] (mergeTree.ts:1978-1995)
      const bool fresh = visit && rseq < 0;
      int dl = 0;
      if (fresh) {
        const uint32_t ncli = (cli & 0xFFFF) | ((uint32_t)C << 16);
        V.f[F_RSEQ][lane] = (uint32_t)S;
        V.f[F_CLI][lane] = ncli;
        V.f[F_RCX][lane] = 0;
        FBlk& B = blk[b];
        B.f[F_RSEQ][lane] = (uint32_t)S;
        B.f[F_CLI][lane] = ncli;
        B.f[F_RCX][lane] = 0;
        const int before = local_len(len, -1);
        const int after = local_len(len, S);
        dl = (after == MTB_UNDEF ? 0 : after) - (before == MTB_UNDEF ? 0 : before);
      }
      const int dsum = csum8(dl);
      if (lane == 0) sh->acc[d] += dsum;
      wsync();
      if (COLD(delta_on)) delta_emit(fresh, id & ~MTB_LEAF, (uint32_t)len, props);
      if (isLive && S >= MTB_PEND) {  // a local remove: its fresh segments join its group, in order
        unsigned long long fm = __ballot(fresh);
        while (fm && !err) {
          const int t = first_set(fm);
          fm &= fm - 1;
          grp_add(rlu(id, t) & ~MTB_LEAF, MTB_OP_REMOVE, 0);
        }
      }
      if (isLive) {
        // a remote remove of a segment removed by an unacked local op: the remote client goes to the
        // head of removedClientIds and its seq becomes removedSeq (mergeTree.ts:1980-1988); the lists of
        // the block's ancestors are rebuilt after the nodeMap (overwrite -> nodeUpdateLengthNewStructure)
        unsigned long long pm = __ballot(visit && rseq >= MTB_PEND && S < MTB_PEND);
        if (pm) {
          while (pm && !err) {
            const int t = first_set(pm);
            pm &= pm - 1;
            const uint32_t h = alloc_aux(2);
            if (bad()) return 0;
            if (lane == 0) {
              aux[h] = 1;
              aux[h + 1] = 0;  // the local client (short id 0)
              const uint32_t ncli = (U(V.f[F_CLI][t]) & 0xFFFF) | ((uint32_t)C << 16);
              V.f[F_RSEQ][t] = (uint32_t)S;
              V.f[F_CLI][t] = ncli;
              V.f[F_RCX][t] = h;
              blk[b].f[F_RSEQ][t] = (uint32_t)S;
              blk[b].f[F_CLI][t] = ncli;
              blk[b].f[F_RCX][t] = h;
            }
            wsync();
          }
          if (lane == 0) {
            const uint32_t nrb = sh->memo[2];
            if (nrb < 64) sh->pk[nrb] = b;
            sh->memo[2] = nrb + 1;
          }
          wsync();
        }
      }
      // overlapping removes (already removed): append C to removedClientIds (copy-on-write list) and an
      // OVERLAP entry on every ancestor list (no observer-length change)
      unsigned long long om = __ballot(visit && rseq >= 0 && !(isLive && rseq >= MTB_PEND));
      if constexpr (hasPh) {
        if (__ballot(visit && rseq >= 0)) ph_ow = true;  // _overwrite (mergeTree.ts:1978-1995)
      }
      if (COLD(om))
      while (om) {
        const int t = first_set(om);
        om &= om - 1;
        const uint32_t orcx = U(V.f[F_RCX][t]);
        const uint32_t oldn = orcx ? U(aux[orcx]) : 0;
        const uint32_t h = alloc_aux(oldn + 2);
        if (bad()) return 0;
        for (uint32_t i = lane; i < oldn; i += 64) aux[h + 1 + i] = aux[orcx + 1 + i];
        if (lane == 0) {
          aux[h] = oldn + 1;
          aux[h + 1 + oldn] = (uint32_t)C;
          V.f[F_RCX][t] = h;
          blk[b].f[F_RCX][t] = h;
        }
        wsync();
        insert_levels_sorted(0, d, rl(rseq, t), C, WK_OVERLAP, rl(len, t));
        if (bad()) return 0;
      }
      mk_remap_view(d);  // afterMarkRemoved: the leaf block's blockUpdateLength / nodeUpdateLengthNewStructure
    } else {
      if constexpr (hasMk)
        if (COLD(ann_mk != 0)) {
          mk_check_annot(vm, lane < count ? V.f[F_TEXT][lane] : 0u, props, opId);
          if (bad()) return 0;
        }
      // annotate: one new property set per distinct old set (memoized per op)
      unsigned long long am = vm, handled = 0;
      if (isLive && S >= MTB_PEND) {  // a local annotate: every annotated segment joins its group, in order
        unsigned long long gm = vm;
        while (gm && !err) {
          const int t = first_set(gm);
          gm &= gm - 1;
          grp_add(rlu(id, t) & ~MTB_LEAF, MTB_OP_ANNOTATE, opId | (rewrite ? MTB_GRP_REWRITE : 0u));
        }
      } else if (isLive && COLD((U(ds->pend_ann) | U(ds->orphans)) != 0)) {
        // a remote annotate leaves the keys of pending local annotates alone (shouldModifyKey,
        // segmentPropertiesManager.ts:95-106): segments holding pending keys get their own edit
        unsigned long long xm = vm;
        while (xm && !err) {
          const int t = first_set(xm);
          xm &= xm - 1;
          const uint32_t nk = pending_keys(rlu(id, t) & ~MTB_LEAF);
#ifndef MTB_NO_RWBLOCK  // (test builds: shows the rewrite farms depend on it)
          if (pk_rw) {  // pendingRewriteCount > 0: the remote annotate leaves the segment alone (:75-82)
            am &= ~(1ull << t);
            handled |= 1ull << t;
            continue;
          }
#endif
          if (!nk || comb >= 2) continue;  // (a combiningOp modifies pending keys too, shouldModifyKey :95-106)
          const uint32_t np = props_apply_slow(rlu(props, t), opId, comb, nk);
          if (bad()) return 0;
          memo_old = MTB_NONE;  // (an edit with exclusions is never reused)
          if (lane == t) {
            V.f[F_PROPS][lane] = np;
            blk[b].f[F_PROPS][lane] = np;
          }
          am &= ~(1ull << t);
          handled |= 1ull << t;
          wsync();
        }
      }
      while (am) {
        const int t = first_set(am);
        const uint32_t old = rlu(props, t);
        const uint32_t np = props_apply(old, opId, comb);
        if (bad()) return 0;
        const bool mine = visit && props == old && !((handled >> lane) & 1);
        if (mine) {
          V.f[F_PROPS][lane] = np;
          blk[b].f[F_PROPS][lane] = np;
        }
        am &= ~__ballot(mine);
        wsync();
      }
      if (COLD(delta_on)) {
        delta_emit(visit, id & ~MTB_LEAF, (uint32_t)len, lane < count ? V.f[F_PROPS][lane] : 0u);
        if (rewrite) delta_emit(visit, id & ~MTB_LEAF, (uint32_t)len, props, MTB_DELTA_OLD);
      }
    }
    // addToLRUSet for the first visited segment (the block's needsScour then becomes true)
    const int t = first_set(vm);
    const uint32_t tid = rlu(id, t);
    if (S > curSeq && U(V.scour) != 1 && !(isLive && S >= MTB_PEND)) {
      if (lane == 0) {
        V.scour = 1;
        blk[b].scour = 1;
      }
      wsync();
      heap_add(tid & ~MTB_LEAF, S);
    }
    if (lane == 0) V.rlv = 0;
    wsync();
    return total;
  }
  // markRangeRemoved (mergeTree.ts:1960-2052) when `remove`, else annotateRange (mergeTree.ts:1895-1958).
  // Emulates depthFirstNodeWalk (mergeTreeNodeWalk.ts:35) with an explicit stack; block post-actions
  // (blockUpdateLength) become one flush of the accumulated observer-length delta per block into its
  // parent's slot and list.  The walk's per-child loop (skip children of undefined / zero length or
  // wholly before `start`, stop at the first one at or after `end`) is one scan over the block's slots:
  // the next child descended into is the first slot at or after the cursor that overlaps the range.
  __device__ __forceinline__ void node_map(int start, int end, int R, int C, int S, bool remove, uint32_t opId, int comb) {
    if (end == start) return;
    ph_ow = false;
    int d = 0;
    bool exiting = false;  // a leaf block reached `end`: every open block is only flushed from here on
    walk_depth = -1;       // (pp[] holds the node_map block starts below)
    if (lane == 0) {
      sh->path[0] = root;
      sh->sidx[0] = 0;
      sh->acc[0] = 0;
      sh->pp[0] = 0;
    }
    wsync();
    load_view(0, root, R, C);
    while (!err) {
      View& V = sh->v[d];
      const int count = U(V.count);
      const int bpos = U(sh->pp[d]);  // position of the block's start in the (R, C) view
      const int idx = U(sh->sidx[d]);
      int walked = -1;  // a block of segments: the length of its leaves in the view (nodeMap's pos advance)
      if (!exiting) {
        if (idx == 0 && count > 0 && (U(V.f[F_ID][0]) & MTB_LEAF)) {
          // a block of segments: every touched segment at once
          const int tot = map_leaf_block(d, bpos, start, end, S, C, remove, opId, comb);
          if (bad()) return;
          walked = tot;
          if (bpos + tot >= end) exiting = true;
        } else {
          int rlj = 0;
          if (lane < count) rlj = V.rl[lane];
          const int def = (lane < count && rlj > 0) ? rlj : 0;
          const int sj = bpos + cscan8(def) - def;
          const unsigned long long m = __ballot(lane >= idx && def > 0 && start < sj + def && sj < end);
          if (m) {
            const int j = first_set(m);
            const uint32_t c = U(V.f[F_ID][j]);
            if (c & MTB_LEAF) { fail(DERR_SHAPE); return; }
            if (d + 1 >= MTB_VDEPTH) { fail(DERR_DEPTH); return; }
            const int cpos = rl(sj, j);
            if (lane == 0) {
              sh->sidx[d] = j + 1;
              sh->slot[d] = j;
              sh->path[d + 1] = c;
              sh->sidx[d + 1] = 0;
              sh->acc[d + 1] = 0;
              sh->pp[d + 1] = cpos;
            }
            wsync();
            d++;
            load_view(d, c, R, C);
            continue;
          }
        }
      }
      // post-order: flush this block's accumulated observer-length delta into its parent
      const int a = U(sh->acc[d]);
      if (a != 0) {
        if (d > 0) {
          const int L = d - 1;
          const int k = U(sh->slot[L]);
          if (lane == 0) {
            const int v = (int)sh->v[L].f[F_LEN][k] + a;
            sh->v[L].f[F_LEN][k] = (uint32_t)v;
            blk[sh->path[L]].f[F_LEN][k] = (uint32_t)v;
            sh->acc[L] += a;
          }
          wsync();
          append_levels(L, d, S, C, WK_MAIN, a);
        }
        if (lane == 0) {
          const int v = sh->v[d].len + a;
          sh->v[d].len = v;
          blk[sh->path[d]].len = v;
        }
        wsync();
      }
      if constexpr (hasPh) {
        // afterMarkRemoved (mergeTree.ts:2019-2026): once the op overwrote a removal, each block it finishes
        // is recombined (nodeUpdateLengthNewStructure), the earlier ones were updated
        if (COLD(phDoc && ph_ow)) {
          ph_combine(U(sh->path[d]));
          if (bad()) return;
        } else if (COLD(phDoc && remove && d > 0 && S < MTB_PEND)) {
          ph_touch(U(sh->path[d]), 1, 0);
        }
        // depthFirstNodeWalk moves nodeMap's pos past a block it descended into by what it counted there (leaf
        // lengths, and the partial lengths of the blocks it skipped), not by the block's own partial length:
        // phantoms and deficits make the two differ, so the parent's later siblings start from the former
        if (COLD(phDoc) && d > 0) {
          if (walked < 0) {
            const int r = lane < count ? V.rl[lane] : 0;
            walked = rl(cscan8(r > 0 ? r : 0), 7);
          }
          if (lane == 0) {
            sh->v[d - 1].rl[U(sh->slot[d - 1])] = walked;
            sh->v[d - 1].rlv = 0;  // (not the view's lengths any more: a later load_view recomputes them)
          }
          wsync();
        }
      }
      if (d == 0) break;
      d--;
    }
  }

  // ------------------------------------------------------------------ zamboni (zamboni.ts)
  __device__ __forceinline__ void copy_text(uint32_t dst, uint32_t src, uint32_t n) {
    const auto txt = UP(sh->gtext);
    for (uint32_t i = lane; i < n; i += 64) txt[dst + i] = txt[src + i];
  }
  __device__ __forceinline__ void stage_rec(uint32_t b) {
    PROF_CNT(CN_ZRECORD, 1);
    const uint32_t* src = bw(b);
    const uint32_t w = src[lane];
    const uint32_t h = lane < 4 ? src[FB_HDR + lane] : 0u;
    const int hc = rl((int)h, 0), hs = rl((int)h, 3);
    const uint32_t hp = rlu(h, 1), hi = rlu(h, 2);
    (&sh->zr.f[0][0])[lane] = w;
    if (lane == 0) {
      sh->zr.count = hc;
      sh->zr.parent = hp;
      sh->zr.index = hi;
      sh->zr.scour = hs;
    }
    wsync();
  }
  // Stage the records of blocks ids[r] (r < nrec, ids in lane r) into sh->pr[r]: lane (r, s) fetches
  // slot s of block r, so up to 8 blocks arrive with one round trip.
  __device__ __forceinline__ void stage_recs(int nrec, uint32_t ids) {
    const int r = lane >> 3, s = lane & 7;
    uint32_t id = MTB_NONE;
#pragma unroll
    for (int q = 0; q < MTB_MAXCH; q++)
      if (q == r) id = rlu(ids, q);
    uint32_t w[8];
    uint32_t h = 0;
    if (r < nrec) {
      const uint32_t* src = bw(id);
#pragma unroll
      for (int q = 0; q < 8; q++) w[q] = src[q * 8 + s];
      if (s < 4) h = src[FB_HDR + s];
    }
    if (r < nrec) {
#pragma unroll
      for (int q = 0; q < 8; q++) sh->pr[r].f[q][s] = w[q];
      if (s == 0) sh->pr[r].count = (int)h;
      if (s == 1) sh->pr[r].parent = h;
      if (s == 2) sh->pr[r].index = h;
      if (s == 3) sh->pr[r].scour = (int)h;
    }
    wsync();
  }
  // Property-set signature of a segment, for matchProperties (properties.ts:71-96) without
  // dependent loads: number of keys and up to two (key, value class) pairs.
  struct PSig {
    uint32_t n, k0, c0, k1, c1;
  };
  __device__ __forceinline__ PSig psig_of(uint32_t h) const {
    PSig g;
    g.n = 0;
    g.k0 = g.c0 = g.k1 = g.c1 = 0;
    if (h) {
      const auto p = props_ptr(h);  // pools carry >= 4 words of tail padding
      g.n = p[0];
      g.k0 = p[1];
      const uint32_t v0 = p[2];
      g.k1 = p[3];
      const uint32_t v1 = p[4];
      // (classes are the value ids themselves when no class holds two values: no dependent table load)
      if (U(sh->tab.class_trivial)) {
        g.c0 = g.n >= 1 ? v0 : 0u;
        g.c1 = g.n >= 2 ? v1 : 0u;
      } else {
        const auto vc = UP(sh->tab.val_class);
        if (g.n >= 1) g.c0 = vc[v0];
        if (g.n >= 2) g.c1 = vc[v1];
      }
    }
    return g;
  }
  // scourNode (zamboni.ts:122-193) over the staged records sh->pr[0..nrec), each one a block whose kept
  // children (all 8 fields) are appended, record after record, to sh->hold[.][nh..].  Lane (r, s)
  // evaluates child s of record r; the sequential keep/drop/append decisions then run on readlane
  // values, and the text of each run of appended segments is written with one parallel copy
  // (TextSegment.append, textSegment.ts:84).
  __device__ __forceinline__ int scour(int nrec, int nh) {
    const uint64_t ts0 = PROF_T();
    PROF_CNT(CN_SCOUR, nrec);
    const int r = lane >> 3, s = lane & 7;
    const int count = r < nrec ? sh->pr[r].count : 0;
    uint32_t f[8];
#pragma unroll
    for (int q = 0; q < 8; q++) f[q] = 0;
    f[F_ID] = MTB_NONE;
    int kind = 0;  // 0 hold+reset, 1 drop (tombstone below MSN), 2 acked text/marker (may append)
    uint16_t last = 0;
    PSig g;
    g.n = 0;
    g.k0 = g.c0 = g.k1 = g.c1 = 0;
    if (s < count) {
#pragma unroll
      for (int q = 0; q < 8; q++) f[q] = sh->pr[r].f[q][s];
      if (f[F_ID] & MTB_LEAF) {
        const int rseq = (int)f[F_RSEQ];
        if (rseq >= 0) kind = rseq > minSeq ? 0 : 1;
        else if ((int)f[F_SEQ] <= minSeq) kind = 2;
        if (kind == 2 && hasNL && !(f[F_TEXT] & MTB_MARKER) && (int)f[F_LEN] > 0)
          last = UP(sh->gtext)[f[F_TEXT] + f[F_LEN] - 1];
      }
    }
    if constexpr (isLive) {
      if (COLD(U(ds->pend_ann) != 0) && annotate_pending(s < count ? f[F_ID] : MTB_NONE)) kind = 0;
    }
    // property signatures only where matchProperties can decide a merge: an acked segment whose left
    // neighbour is also acked and carries a different property-set handle (equal handles match)
    {
      const bool k2 = s < count && kind == 2;
      const int lk2 = dpp_shr_t<0x111>((int)k2);
      const uint32_t lph = (uint32_t)dpp_shr_t<0x111>((int)f[F_PROPS]);
      const int rk2 = dpp_shr_t<0x101>((int)k2);
      const uint32_t rph = (uint32_t)dpp_shr_t<0x101>((int)f[F_PROPS]);
      const bool needL = s > 0 && lk2 != 0 && lph != f[F_PROPS];
      const bool needR = s < 7 && rk2 != 0 && rph != f[F_PROPS];
      if (__ballot(k2 && (needL || needR))) {
        PROF_CNT(CN_PSIG, 1);
        if (k2) g = psig_of(f[F_PROPS]);
      }
    }
    int target = -1;  // per lane: lane it was appended into (-1 kept / dropped)
    int newLen = 0;   // per lane: final length if it is an append target
    // Run decisions.  Lane-parallel: segment k joins the run of its left neighbour when both are acked
    // non-empty segments that may append (TextSegment.canAppend: no marker, no trailing newline;
    // matchProperties, an equivalence, so comparing with the left neighbour equals comparing with the
    // run's head; PermutationSegment.canAppend: contiguous handles).  The length rule (run length <= 256
    // or segment length <= 256) only cuts runs at segments longer than 256, and a cut there never
    // un-cuts a later one, so one segmented scan settles it.  Property sets with more than two keys that
    // need a full comparison fall back to the sequential form below.
    const int klen0 = (int)f[F_LEN];
    const bool cand = s < count && kind == 2 && klen0 > 0;
    bool compat = false;
    {
      // Every DPP read runs with all lanes active (a read from an inactive lane yields 0), so the
      // neighbour values are fetched in plain statements before any short-circuit combination.
      const bool hasLeft = s > 0;  // row_shr:1 also reaches lane 7 of the previous group for s == 0
      const int lcandv = dpp_shr_t<0x111>((int)cand);
      const bool lcand = hasLeft & (lcandv != 0);
      if (isPerm) {
        const uint32_t lst = (uint32_t)dpp_shr_t<0x111>((int)f[F_TEXT]);
        const int llen = dpp_shr_t<0x111>(klen0);
        compat = cand && lcand &&
                 (lst == MTB_HANDLE_UNALLOC ? f[F_TEXT] == MTB_HANDLE_UNALLOC : f[F_TEXT] == lst + (uint32_t)llen);
      } else {
        // each neighbour value is compared as soon as it is fetched: the results are lane masks (SGPRs)
        const bool mk = (f[F_TEXT] & MTB_MARKER) != 0;
        const int lmkv = dpp_shr_t<0x111>((int)mk);
        const int llastv = dpp_shr_t<0x111>((int)last);
        const bool base = cand & lcand & !mk & (lmkv == 0) & ((uint16_t)llastv != (uint16_t)'\n');
        const uint32_t lprops = (uint32_t)dpp_shr_t<0x111>((int)f[F_PROPS]);
        const bool sameH = f[F_PROPS] == lprops;
        const bool nanPair = ((f[F_PROPS] | lprops) & MTB_PNAN) != 0;  // a set holding NaN matches nothing
        const bool sameN = g.n == (uint32_t)dpp_shr_t<0x111>((int)g.n);
        const bool k0k0 = g.k0 == (uint32_t)dpp_shr_t<0x111>((int)g.k0);
        const bool c0c0 = g.c0 == (uint32_t)dpp_shr_t<0x111>((int)g.c0);
        const bool k1k1 = g.k1 == (uint32_t)dpp_shr_t<0x111>((int)g.k1);
        const bool c1c1 = g.c1 == (uint32_t)dpp_shr_t<0x111>((int)g.c1);
        const bool k0k1 = g.k0 == (uint32_t)dpp_shr_t<0x111>((int)g.k1);
        const bool c0c1 = g.c0 == (uint32_t)dpp_shr_t<0x111>((int)g.c1);
        const bool k1k0 = g.k1 == (uint32_t)dpp_shr_t<0x111>((int)g.k0);
        const bool c1c0 = g.c1 == (uint32_t)dpp_shr_t<0x111>((int)g.c0);
        bool eq = !nanPair && (sameH || (sameN && (g.n == 0 || (g.n == 1 && k0k0 && c0c0) ||
                                                   (g.n == 2 && ((k0k0 && c0c0 && k1k1 && c1c1) || (k0k1 && c0c1 && k1k0 && c1c0))))));
        // more than two keys: a full matchProperties, one neighbour pair at a time (rare).  With irregular keys in
        // the batch matchProperties is no equivalence: every candidate is compared with its run's head instead
        // (scourNode's prevSegment, zamboni.ts:151-177), block by block, the 256-unit length rule included.
        // (One loop, one inlined matchProperties: a second copy spills the hot scour.)
        const bool irrB = hasIrr && U(sh->tab.irr_any) != 0;
        const unsigned long long nf = __ballot(base && !sameH && !nanPair && sameN && g.n > 2);
        const unsigned long long cm = __ballot(cand), bm = __ballot(base);
        if (COLD(nf || irrB)) {
          unsigned long long todo = irrB ? cm : nf, okm = 0;
          int head = -1, runLen = 0, prev = -2;
          while (todo) {
            const int t = first_set(todo);
            todo &= todo - 1;
            int a = t - 1, lt = 0;
            bool need = true;
            if (irrB) {
              lt = rl(klen0, t);
              if (t != prev + 1 || (t & 7) == 0) head = -1;  // (a lane between, or a new block: no prevSegment)
              prev = t;
              need = head >= 0 && ((bm >> t) & 1) && (runLen <= 256 || lt <= 256);
              a = head;
            }
            const bool ok = need && props_match(rlu(f[F_PROPS], a), rlu(f[F_PROPS], t));
            if (ok) okm |= 1ull << t;
            if (irrB) {
              if (ok) {
                runLen += lt;
              } else {
                head = t;
                runLen = lt;
              }
            }
          }
          if (irrB || ((nf >> lane) & 1)) eq = ((okm >> lane) & 1) != 0;
        }
        compat = base && eq;
        // length rule: the run length before this segment (segmented scan restarting at run heads)
        int v = cand ? klen0 : 0;
        int st = (!cand || !compat) ? 1 : 0;
        {
          const int pv = dpp_shr_t<0x111>(v), pst = dpp_shr_t<0x111>(st);
          if (s >= 1 && !st) { v += pv; st = pst; }
        }
        {
          const int pv = dpp_shr_t<0x112>(v), pst = dpp_shr_t<0x112>(st);
          if (s >= 2 && !st) { v += pv; st = pst; }
        }
        {
          const int pv = dpp_shr_t<0x114>(v), pst = dpp_shr_t<0x114>(st);
          if (s >= 4 && !st) { v += pv; st = pst; }
        }
        const int cum = v - (cand ? klen0 : 0);
        if (compat && klen0 > 256 && cum > 256) compat = false;
      }
    }
    {
    // run heads and each member's head (prefix max of head lanes within the 8-lane group)
    const bool head = cand && !compat;
    int hv = head ? lane : -1;
    {
      const int pv = dpp_shr_t<0x111>(hv + 1) - 1;
      if (s >= 1) hv = max(hv, pv);
    }
    {
      const int pv = dpp_shr_t<0x112>(hv + 1) - 1;
      if (s >= 2) hv = max(hv, pv);
    }
    {
      const int pv = dpp_shr_t<0x114>(hv + 1) - 1;
      if (s >= 4) hv = max(hv, pv);
    }
    target = compat ? hv : -1;
    newLen = cand ? klen0 : 0;
    const int rcompat = dpp_shr_t<0x101>((int)compat);  // row_shl:1: does lane s + 1 join me?
      const bool follower = (s < 7) & (rcompat != 0);
    unsigned long long hm = __ballot(head && follower);
    while (hm) {
      const int t = first_set(hm);
      hm &= hm - 1;
      unsigned long long run = __ballot(target == t);
      int tot = rl(klen0, t);
      while (run) {
        const int q = first_set(run);
        run &= run - 1;
        tot += rl(klen0, q);
      }
      if (lane == t) newLen = tot;
    }
    }
    // targets that received appends: build their new text
    const bool isTarget = s < count && kind == 2 && target < 0 && newLen != (int)f[F_LEN];
    unsigned long long tm = __ballot(isTarget);
    if (isPerm) {  // BaseSegment.append: the length only (mergeTreeNodes.ts:527-545)
      if (isTarget) f[F_LEN] = (uint32_t)newLen;
      tm = 0;
      // unlinked tombstones return their handles, in scour order (permutationvector.ts:418-441)
      unsigned long long dm = __ballot(s < count && kind == 1 && (int)f[F_TEXT] >= 1);
      if (COLD(dm)) handles_free_lanes(dm, f[F_TEXT], (int)f[F_LEN]);
    }
    while (tm) {
      const int t = first_set(tm);
      tm &= tm - 1;
      // members of the run: t and every lane whose target is t, in order
      const unsigned long long run = __ballot(lane == t || target == t);
      const uint32_t ttext = rlu(f[F_TEXT], t);
      const int tlen = rl((int)f[F_LEN], t);
      const int total = rl(newLen, t);
      // contiguous in the arena already?
      bool contiguous = true;
      {
        uint32_t expect = ttext + (uint32_t)tlen;
        unsigned long long rm = run & ~(1ull << t);
        while (rm) {
          const int q = first_set(rm);
          rm &= rm - 1;
          const uint32_t qt = rlu(f[F_TEXT], q);
          if (qt != expect) contiguous = false;
          expect = qt + (uint32_t)rl((int)f[F_LEN], q);
        }
      }
      uint32_t dst = ttext;
      if (!contiguous) {
        const bool atEnd = ttext + (uint32_t)tlen == text_used;
        const uint32_t need = atEnd ? (uint32_t)(total - tlen) : (uint32_t)total;
        if (text_used + need > U(sh->capv[3])) { fail(DERR_CAP_TEXT); return nh; }
        uint32_t w = text_used;
        if (!atEnd) {
          copy_text(w, ttext, (uint32_t)tlen);
          dst = w;
          w += (uint32_t)tlen;
        } else {
          w = ttext + (uint32_t)tlen;
        }
        unsigned long long rm = run & ~(1ull << t);
        while (rm) {
          const int q = first_set(rm);
          rm &= rm - 1;
          const uint32_t qt = rlu(f[F_TEXT], q);
          const int ql = rl((int)f[F_LEN], q);
          copy_text(w, qt, (uint32_t)ql);
          w += (uint32_t)ql;
        }
        text_used += need;
      }
      if (lane == t) {
        f[F_TEXT] = dst;
        f[F_LEN] = (uint32_t)total;
      }
      wsync();
    }
    // unlink dropped / appended segments, compact the kept ones (record-major order) into hold[]
    const bool keep = s < count && kind != 1 && target < 0;
    if (s < count && !keep) segp[f[F_ID] & ~MTB_LEAF] = MTB_NONE;
    const unsigned long long km = __ballot(keep);
    if (keep) {
      const uint32_t at = nh + rank_below(km);
#pragma unroll
      for (int q = 0; q < 8; q++) sh->hold[q][at] = f[q];
    }
    wsync();
    PROF_ADD(PH_SCOUR, ts0);
    return nh + __popcll(km);
  }
  // Write hold[.][from, from+n) as the children of block nb (slots 0..n-1, the rest cleared), point the
  // children at nb and return their observer-view length.
  __device__ __forceinline__ int place_children(uint32_t nb, int from, int n) {
    const int fld = lane >> 3, s = lane & 7;
    uint32_t v = fld == F_ID ? MTB_NONE : 0u;
    if (s < n) v = sh->hold[fld][from + s];
    bw(nb)[lane] = v;
    int ol = 0;
    if (lane < n) {
      const uint32_t c = sh->hold[F_ID][from + lane];
      set_parent(c, nb, lane);
      ol = child_olen(c, (int)sh->hold[F_LEN][from + lane], (int)sh->hold[F_RSEQ][from + lane]);
    }
    const int len = csum8(ol);
    if (lane == 0) blk[nb].count = (uint32_t)n;
    wsync();
    return len;
  }
  // Store block P's window-list metadata where it lives (its parent's slot, or its own header).
  __device__ __forceinline__ void store_meta_of(uint32_t P, uint32_t parent, uint32_t index, uint32_t loff, uint32_t lcnt, uint32_t lcap) {
    if (lane == 0) {
      if (parent == MTB_NONE) {
        blk[P].loff = loff;
        blk[P].lcnt = lcnt;
        blk[P].lcap = lcap;
        if (P == root) {
          sh->rmeta[0] = loff;
          sh->rmeta[1] = lcnt;
          sh->rmeta[2] = lcap;
        }
      } else {
        FBlk& G = blk[parent];
        G.f[F_SEQ][index] = loff;
        G.f[F_RSEQ][index] = lcnt;
        G.f[F_CLI][index] = lcap;
      }
    }
    wsync();
  }
  // packParent (zamboni.ts:63-120), iterative over the recursion to the grandparent
  __device__ __forceinline__ void pack_parent(uint32_t parent) {
    while (!err) {
      PROF_CNT(CN_PACK, 1);
      uint64_t tp = PROF_T();
      stage_rec(parent);
      const int pc = U(sh->zr.count);
      const uint32_t pparent = U(sh->zr.parent), pindex = U(sh->zr.index);
      const uint32_t kids = lane < pc ? sh->zr.f[F_ID][lane] : MTB_NONE;
      const uint32_t kloff = lane < pc ? sh->zr.f[F_SEQ][lane] : 0u, kcap = lane < pc ? sh->zr.f[F_CLI][lane] : 0u;
      // P's own list metadata (its parent's slot, or the root header), in flight with the siblings
      const uint32_t* pm = pparent == MTB_NONE ? &blk[parent].loff : &blk[pparent].f[F_SEQ][pindex];
      const uint32_t ploff_v = pm[0], pcap_v = pparent == MTB_NONE ? pm[2] : pm[2 * MTB_MAXCH];
      stage_recs(pc, kids);
      TCHK(12);
      const uint32_t ploff = U(ploff_v), pcap = U(pcap_v);
      PROF_PADD(PH_HEAP, tp);
      tp = PROF_T();
      const int nh = scour(pc, 0);
      TCHK(13);
      if (bad()) return;
      PROF_PADD(PH_STAGE, tp);
      tp = PROF_T();
      int cc = 0;
      uint32_t nbs = 0;      // lane q: new block q, its observer length, whether its children are blocks
      int lens = 0, kbs = 0;
      if (nh > 0) {
        cc = nh / (MTB_MAXCH / 2);
        if (cc > MTB_MAXCH - 1) cc = MTB_MAXCH - 1;
        if (cc < 1) cc = 1;
      }
      // the new blocks reuse the siblings' records (block identity is not observable): no free-stack
      // round trip; siblings beyond the new count go back to the free stack
      for (int i = 0; i < pc; i++) {
        if (i >= cc) {
          free_blk(rlu(kids, i));
          if constexpr (hasPh) {
            if (COLD(phDoc)) ph_clear(rlu(kids, i));
          }
        }
        list_free(rlu(kloff, i), rlu(kcap, i));
      }
      if (nh > 0) {
        const int base = nh / cc;
        int rem = nh % cc;
        int taken = 0;
        // first every new block gets its children (the scour output in hold[] is consumed here) ...
        for (int q = 0; q < cc; q++) {
          int n = base;
          if (rem > 0) {
            n++;
            rem--;
          }
          const uint32_t nb = q < pc ? rlu(kids, q) : alloc_blk();
          if (bad()) return;
          const int len = place_children(nb, taken, n);
          if constexpr (hasPh) {
            if (COLD(phDoc)) {  // the packed block's nodeUpdateLengthNewStructure (zamboni.ts:103)
              ph_combine(nb);
              if (bad()) return;
            }
          }
          bool kblk = false;
          if (lane < n) kblk = !(sh->hold[F_ID][taken + lane] & MTB_LEAF);
          const int kb = __ballot(kblk) != 0;
          if (!kb) mk_remap_hold(taken, n);  // nodeUpdateLengthNewStructure(packedBlock) (zamboni.ts:103)
          if (lane == q) {
            nbs = nb;
            lens = len;
            kbs = kb;
          }
          if (lane == 0) {
            blk[nb].parent = parent;
            blk[nb].index = (uint32_t)q;
            blk[nb].len = len;
            blk[nb].scour = -1;  // a new block (makeBlock): needsScour undefined
          }
          wsync();
          taken += n;
        }
      }
      {
        const int fld = lane >> 3, s = lane & 7;
        if (s >= cc) bw(parent)[lane] = fld == F_ID ? MTB_NONE : 0u;
      }
      if (lane == 0) blk[parent].count = (uint32_t)cc;
      wsync();
      PROF_PADD(PH_PLACE, tp);
      // ... then the lists: of the new blocks whose children are blocks, and last of P itself (one rebuild
      // site; rebuild uses the union as scratch)
      uint32_t a = 0, c2 = 0, e = 0;
      // (every new child a block of segments: P's list is rebuilt from the scour output still in LDS)
      const bool leafKids = cc > 0 && __ballot(lane < cc && kbs != 0) == 0;
      for (int q = 0; q <= cc; q++) {
        const bool isP = q == cc;
        const uint32_t nb = isP ? parent : rlu(nbs, q);
        a = c2 = e = 0;
        if (isP || rl(kbs, q)) {
          rebuild(nb, isP ? ploff : 0u, isP ? pcap : 0u, a, c2, e, isP && leafKids ? nh : -1, cc);
          if (bad()) return;
        }
        if (isP) break;
        const int len = rl(lens, q);
        if (lane == 0) {
          FBlk& P = blk[parent];
          P.f[F_ID][q] = nb;
          P.f[F_LEN][q] = (uint32_t)len;
          P.f[F_SEQ][q] = a;
          P.f[F_RSEQ][q] = c2;
          P.f[F_CLI][q] = e;
          P.f[F_RCX][q] = 0;
          P.f[F_PROPS][q] = 0;
          P.f[F_TEXT][q] = 0;
        }
        wsync();
      }
      TCHK(14);
      store_meta_of(parent, pparent, pindex, a, c2, e);
      if (cc < MTB_MAXCH / 2 && pparent != MTB_NONE) {
        parent = pparent;
        continue;
      }
      if constexpr (hasPh) {
        if (COLD(phDoc)) ph_up(parent);  // blockUpdatePathLengths(parent, .., true) (zamboni.ts:116-118)
      }
      break;
    }
  }
  // ------------------------------------------------------------------ PermutationVector handles
  // HandleTable (matrix/src/handletable.ts) in the text arena: u32 [length, handles[0..length)].
  __device__ __forceinline__ gptr<uint32_t> htab() const { return (gptr<uint32_t>)UP(sh->gtext); }
  // free(start + i) for every lane of `m` in lane order (handletable.ts:55-58)
  __device__ __forceinline__ void handles_free_lanes(unsigned long long m, uint32_t start, int len) {
    const auto ht = htab();
    while (m) {
      const int t = first_set(m);
      m &= m - 1;
      const uint32_t st = rlu(start, t);
      const int n = rl(len, t);
      cell_event(MTB_CELL_CLEAR, st, (uint32_t)n);  // handlesRecycledCallback before the free
      if (lane == 0) {
        uint32_t head = ht[1];
        for (int i = 0; i < n; i++) {
          ht[1 + st + i] = head;  // handles[h] = next
          head = st + (uint32_t)i;
        }
        ht[1] = head;
      }
      wsync();
    }
  }
  // allocate (handletable.ts:36-41): the free-list head, growing the table when it is exhausted
  __device__ __forceinline__ uint32_t handle_alloc() {
    const auto ht = htab();
    const uint32_t L = U(ht[0]);
    const uint32_t fr = U(ht[1]);
    const uint32_t next = fr < L ? U(ht[1 + fr]) : fr + 1;  // handles[free] ?? free + 1
    if (fr >= L && 2u * (L + 2u) > U(sh->capv[3])) {
      fail(DERR_CAP_TEXT);
      return 0;
    }
    wsync();
    if (lane == 0) {
      ht[1] = next;
      ht[1 + fr] = 0;
      if (fr >= L) ht[0] = L + 1;
    }
    if (fr >= L) text_used = 2u * (L + 2u);
    wsync();
    return fr;
  }
  // getContainingSegment(pos, refSeq, clientId) (mergeTree.ts:787-813, nodeMap :2531-2582): the first
  // leaf with a non-zero (R, C) length whose span holds pos.  Leaves the path in the views; returns the
  // depth of the leaf-level block (or -1), its slot, the offset in the segment and the segment's local
  // position (getPosition in the observer's view, mergeTree.ts:1240).
  __device__ __forceinline__ int find_seg(int pos, int R, int C, int& slot, int& offset, int& lpos) {
    uint32_t b = root;
    int p = pos, d = 0, lp = 0;
    while (true) {
      if (d >= MTB_VDEPTH) { fail(DERR_DEPTH); return -1; }
      if (lane == 0) {
        sh->path[d] = b;
        sh->pp[d] = p;
      }
      wsync();
      const int count = load_view(d, b, R, C);
      const View& V = sh->v[d];
      int clen = 0, ol = 0;
      uint32_t cid = MTB_NONE;
      if (lane < count) {
        cid = V.f[F_ID][lane];
        clen = V.rl[lane];
        ol = child_olen(cid, (int)V.f[F_LEN][lane], (int)V.f[F_RSEQ][lane]);
      }
      const int def = clen > 0 ? clen : 0;  // nodeMap skips undefined and zero lengths
      const int incl = cscan8(def);
      const int pj = p - (incl - def);
      const unsigned long long m = __ballot(lane < count && def > 0 && pj < def);
      if (!m) return -1;
      const int j = first_set(m);
      lp += csum8(lane < j ? ol : 0);
      if (lane == 0) sh->slot[d] = j;
      wsync();
      const uint32_t cj = rlu(cid, j);
      const int pjj = rl(pj, j);
      if (!(cj & MTB_LEAF)) {
        b = cj;
        p = pjj;
        d++;
        continue;
      }
      slot = j;
      offset = pjj;
      lpos = lp + pjj;
      return d;
    }
  }
  // adjustPosition (permutationvector.ts:209-226): the op's position in the observer's view, or -1
  // when it lands on no segment or on a removed one
  __device__ __forceinline__ int adjust_position(int pos, int R, int C) {
    view_clear();
    int j, off, lp;
    const int d = find_seg(pos, R, C, j, off, lp);
    if (d < 0 || bad()) return -1;
    if ((int)U(sh->v[d].f[F_RSEQ][j]) >= 0) return -1;
    return lp;
  }
  // getAllocatedHandle (permutationvector.ts:183-207) at local position pos: nothing when the position
  // already has a handle, else walkSegments(pos, pos + 1, splitRange) isolates it and it gets one
  __device__ __forceinline__ int allocated_handle(int pos, int Cl) {  // the handle, or -1 on failure
    view_clear();
    int j, off, lp;
    int d = find_seg(pos, curSeq, Cl, j, off, lp);
    if (d < 0 || bad()) { fail(DERR_HANDLE); return -1; }
    const int st = (int)U(sh->v[d].f[F_TEXT][j]);
    if (st >= 1) return st + off;  // start + offset is valid
    walk(pos, curSeq, Cl, -2, false, 0);  // ensureIntervalBoundary(pos) and (pos + 1), local view
    settle();
    if (bad()) return -1;
    view_clear();
    walk(pos + 1, curSeq, Cl, -2, false, 0);
    settle();
    if (bad()) return -1;
    view_clear();
    d = find_seg(pos, curSeq, Cl, j, off, lp);
    if (d < 0 || bad() || off != 0 || (int)U(sh->v[d].f[F_LEN][j]) != 1) { fail(DERR_HANDLE); return -1; }
    const uint32_t h = handle_alloc();
    if (bad()) return -1;
    if (lane == 0) {
      sh->v[d].f[F_TEXT][j] = h;
      blk[sh->v[d].b].f[F_TEXT][j] = h;
    }
    n_mod += 1;
    wsync();
    return (int)h;
  }
  // SharedMatrix cell events in the document's delta slice, one 4-word entry each: [record, kind,
  // handle or first recycled handle, count].  The host replays them, with the setCell values, into the
  // matrix's SparseArray2D (matrix.ts:668-690 sets, :721-733 clears of recycled handles).
  __device__ __forceinline__ void cell_event(uint32_t kind, uint32_t a, uint32_t n) {
    if (delta_used + 1 > U(sh->capv[6])) { fail(DERR_CAP_DELTA); return; }
    if (lane == 0) {
      const auto e = dslice() + 4 * delta_used;
      e[0] = cur_k;
      e[1] = kind;
      e[2] = a;
      e[3] = n;
    }
    delta_used += 1;
  }
  // SharedMatrix setCell (matrix.ts:668-676) on this wave's vector: adjust, exchange with the partner
  // wave (the other vector of the same matrix) through LDS, allocate when both positions survive.
  // Both waves meet one barrier per setCell record, errors included.
  __device__ __forceinline__ void setcell(const mtb_op& o, int par) {
    const int adj = err ? -1 : adjust_position((int)o.pos1, (int)o.ref_seq, (int)(int16_t)o.client);
    if (lane == 0) xch[par * 2 + wv] = adj;
    __syncthreads();
    const int other = U(xch[par * 2 + (wv ^ 1)]);
    if (!err && adj >= 0 && other >= 0) {
      const int h = allocated_handle(adj, (int)o.pos2);
      if (h >= 0 && !err) cell_event(MTB_CELL_SET, (uint32_t)h, 1);
    }
  }

  // zamboniSegments (zamboni.ts:19-60)
  __device__ __forceinline__ void zamboni() {
    PROF_CNT(CN_ZCALL, 1);
    for (int i = 0; i < 2 && !err; i++) {
      if (heap_cnt == 0) break;
      const Lru top = hget(1);
      if (top.maxSeq > minSeq) break;
      PROF_CNT(CN_POP, 1);
      uint64_t tz = PROF_T();
      const uint32_t bp = segp[top.seg];  // in flight while the heap is fixed down
      heap_get();
      PROF_ZADD(PH_HEAP, tz);
      tz = PROF_T();
      const uint32_t b = U(bp);
      TCHK(7);
      if (b == MTB_NONE) { PROF_CNT(CN_PSKIP, 1); PROF_ZADD(PH_STAGE, tz); continue; }
      stage_recs(1, b);
      TCHK(8);
      const int sc = U(sh->pr[0].scour);
      PROF_ZADD(PH_STAGE, tz);
      if (sc == 0) { PROF_CNT(CN_PSKIP, 1); continue; }
      const int count = U(sh->pr[0].count);
      const uint32_t parent = U(sh->pr[0].parent);
      const int nh = scour(1, 0);
      TCHK(9);
      if (bad()) return;
      tz = PROF_T();
      if (lane == 0) blk[b].scour = 0;
      wsync();
      // nh == count: nothing was dropped or appended, the record is unchanged
      if (nh < count) {
        place_children(b, 0, nh);
        PROF_ZADD(PH_PLACE, tz);
        tz = PROF_T();
        TCHK(10);
        if (COLD(nh < MTB_MAXCH / 2 && parent != MTB_NONE)) {
          pack_parent(parent);
          TCHK(11);
        } else {
          mk_remap_hold(0, nh);  // blockUpdatePathLengths(block, .., true) (zamboni.ts:55)
          if constexpr (hasPh) {
            if (COLD(phDoc)) ph_up(b);
          }
        }
        PROF_ADD(PH_PACK, tz);
      } else {
        PROF_ZADD(PH_PLACE, tz);
      }
    }
  }

  // ------------------------------------------------------------------ marker ids (idToSegment)
  // mapIdToSegment (mergeTree.ts:668, from insertSegments :1658-1663): the marker inserted as segment `sid`
  // carries id ordinal `ord` (its record's payload - 1).  The map lives in the aux arena and grows to the
  // host's ordinal count; the host keeps every mapped id unique in its document (else relative positions
  // naming it are rejected at pack time), so blockUpdate's re-mapping (:296-306) never changes an entry.
  __device__ __forceinline__ void mk_set(uint32_t ord, uint32_t sid) {
    uint32_t map = U(ds->mk_map), n = U(ds->mk_n);
    if (ord >= n) {
      const uint32_t hc = U(ds->mk_cap);
      const uint32_t cap = hc > ord ? hc : ord + 1;
      const uint32_t nm = alloc_aux(cap);
      if (bad()) return;
      for (uint32_t i = lane; i < cap; i += 64) aux[nm + i] = i < n ? aux[map + i] : MTB_NONE;
      map = nm;
      n = cap;
      if (lane == 0) {
        ds->mk_map = map;
        ds->mk_n = n;
      }
    }
    if (lane == 0) aux[map + ord] = sid;
    wsync();
  }
  // Duplicate ids (DSF_MKDUP): every marker inserted with an id is listed as (segment, ordinal) in
  // DocState.mk_all [n, cap, pairs], so a leaf block's update can name the ids of its markers.
  __device__ __forceinline__ void mk_record(uint32_t ord, uint32_t sid) {
    uint32_t h = U(ds->mk_all);
    const uint32_t n = h ? U(aux[h]) : 0u, cap = h ? U(aux[h + 1]) : 0u;
    if (n >= cap) {
      const uint32_t nc = cap ? 2 * cap : 8u;
      const uint32_t nh = alloc_aux(2 + 2 * nc);
      if (bad()) return;
      for (uint32_t i = lane; i < 2 * n; i += 64) aux[nh + 2 + i] = aux[h + 2 + i];
      if (lane == 0) {
        aux[nh + 1] = nc;
        ds->mk_all = nh;
      }
      h = nh;
    }
    if (lane == 0) {
      aux[h + 2 + 2 * n] = sid;
      aux[h + 3 + 2 * n] = ord;
      aux[h] = n + 1;
    }
    wsync();
  }
  __device__ __forceinline__ uint32_t mk_ord_of(uint32_t sid) const {
    const uint32_t h = U(ds->mk_all);
    if (!h) return MTB_NONE;
    const uint32_t n = U(aux[h]);
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      const unsigned long long m = __ballot(i < n && aux[h + 2 + 2 * i] == sid);
      if (m) return U(aux[h + 3 + 2 * (base + (uint32_t)first_set(m))]);
    }
    return MTB_NONE;
  }
  // the value id of key k in property set h (MTB_NONE: absent); per lane
  __device__ __forceinline__ uint32_t props_val(uint32_t h, uint32_t k) const {
    if (!h || k == MTB_NONE) return MTB_NONE;
    const auto p = props_ptr(h);
    const uint32_t n = p[0];
    for (uint32_t i = 0; i < n; i++)
      if (p[1 + 2 * i] == k) return p[2 + 2 * i];
    return MTB_NONE;
  }
  // blockUpdate (mergeTree.ts:2392-2417) of a block of segments: addNodeReferences (:296-306) maps the id
  // of every child marker whose localNetLength is positive, in child order (the last one wins).  Lane i
  // holds child i (i < n).  Only documents with a reused id need it: otherwise an id's one marker is
  // already mapped by its insert and the map is never pruned.
  __device__ __forceinline__ void mk_remap(int n, uint32_t id, uint32_t text, uint32_t props, int len, int rseq) {
    const uint32_t key = U(sh->tab.mk_key);
    const bool q = lane < n && (id & MTB_LEAF) && (text & MTB_MARKER) && props && key != MTB_NONE &&
                   local_len(len, rseq) > 0 && props_val(props, key) != MTB_NONE;
    unsigned long long m = __ballot(q);
    while (m && !err) {
      const int t = first_set(m);
      m &= m - 1;
      const uint32_t sid = rlu(id, t) & ~MTB_LEAF;
      const uint32_t ord = mk_ord_of(sid);
      if (ord != MTB_NONE) mk_set(ord, sid);
    }
  }
  __device__ __forceinline__ void mk_remap_view(int d) {
    if constexpr (hasMk) {
      if (COLD(mkDup)) {
        const View& V = sh->v[d];
        const int n = U(V.count);
        uint32_t id = MTB_NONE, text = 0, props = 0;
        int len = 0, rseq = -1;
        if (lane < n) {
          id = V.f[F_ID][lane];
          text = V.f[F_TEXT][lane];
          props = V.f[F_PROPS][lane];
          len = (int)V.f[F_LEN][lane];
          rseq = (int)V.f[F_RSEQ][lane];
        }
        mk_remap(n, id, text, props, len, rseq);
      }
    }
  }
  // blockUpdate of leaf-level block b read from its record (MODE_LIVE: acks, normalizeAdjacentSegments)
  __device__ __forceinline__ void mk_remap_blk(uint32_t b) {
    if constexpr (hasMk) {
      if (COLD(mkDup)) {
        const uint32_t* r = bw(b);
        const int n = (int)U(r[FB_HDR]);
        uint32_t id = MTB_NONE, text = 0, props = 0;
        int len = 0, rseq = -1;
        if (lane < n) {
          id = r[F_ID * 8 + lane];
          text = r[F_TEXT * 8 + lane];
          props = r[F_PROPS * 8 + lane];
          len = (int)r[F_LEN * 8 + lane];
          rseq = (int)r[F_RSEQ * 8 + lane];
        }
        mk_remap(n, id, text, props, len, rseq);
      }
    }
  }
  __device__ __forceinline__ void mk_remap_hold(int from, int n) {  // children placed from sh->hold[.][from..)
    if constexpr (hasMk) {
      if (COLD(mkDup)) {
        uint32_t id = MTB_NONE, text = 0, props = 0;
        int len = 0, rseq = -1;
        if (lane < n) {
          id = sh->hold[F_ID][from + lane];
          text = sh->hold[F_TEXT][from + lane];
          props = sh->hold[F_PROPS][from + lane];
          len = (int)sh->hold[F_LEN][from + lane];
          rseq = (int)sh->hold[F_RSEQ][from + lane];
        }
        mk_remap(n, id, text, props, len, rseq);
      }
    }
  }
  // assert 0x5ad (annotateRange, mergeTree.ts:1912-1918): an annotate whose props name markerId must carry
  // each annotated marker's own id (JS ===; the host reduced the op's value to ann_mk: 1 = a primitive,
  // compared as its value id, 2 = null / object, equal to nothing).  Lanes of `vm` hold the visited children.
  __device__ __forceinline__ void mk_check_annot(unsigned long long vm, uint32_t text, uint32_t props, uint32_t opId) {
    const bool mk = ((vm >> lane) & 1) && (text & MTB_MARKER);
    if (!__ballot(mk)) return;
    if (ann_mk != 1) { fail(DERR_ASSERT_MKID); return; }
    const uint32_t key = U(sh->tab.mk_key);
    const auto op = UP(sh->tab.pool) + U(UP(sh->tab.pidx)[2 * opId]);
    uint32_t vop = MTB_NONE;
    const uint32_t nop = U(op[0]);
    for (uint32_t q = 0; q < nop; q++)
      if (U(op[1 + 2 * q]) == key) vop = U(op[2 + 2 * q]);
    if (__ballot(mk && props_val(props, key) != vop)) fail(DERR_ASSERT_MKID);
  }
  // posFromRelativePos (mergeTree.ts:1371-1395) of a record position field `v` in the op's (R, C) view:
  // v itself, or for MTB_RELPOS | descriptor offset: getPosition (:768-785) of the mapped marker (0 once
  // zamboni unlinked it), then `before` / `offset`.  An unmapped marker or a negative result fails the
  // document (DERR_RELPOS).  The views loaded on the way up stay valid for the op's walks.
  __device__ __forceinline__ int rel_pos(uint32_t v, int R, int C) {
    if (!(v & MTB_RELPOS)) return (int)v;
    const auto t = UP(sh->gtext) + (v & ~MTB_RELPOS);
    const uint32_t ord = U((uint32_t)t[0] | ((uint32_t)t[1] << 16));
    const uint32_t before = U((uint32_t)t[2]);
    const int off = (int)U((uint32_t)t[4] | ((uint32_t)t[5] << 16));
    if (ord >= U(ds->mk_n)) { fail(DERR_RELPOS); return 0; }
    const uint32_t sid = U(aux[U(ds->mk_map) + ord]);
    if (sid == MTB_NONE) { fail(DERR_RELPOS); return 0; }
    int pos = 0;
    const uint32_t b0 = U(segp[sid]);
    if (b0 != MTB_NONE) {
      uint32_t mine = MTB_NONE;  // lane i: the i-th ancestor block from the bottom
      int n = 0;
      for (uint32_t x = b0; x != MTB_NONE; x = U(blk[x].parent)) {
        if (n >= MTB_VDEPTH) { fail(DERR_DEPTH); return 0; }
        if (lane == n) mine = x;
        n++;
      }
      for (int d = 0; d < n; d++) {
        const uint32_t bd = rlu(mine, n - 1 - d);
        if (d > 0) {
          if (lane == 0) sh->slot[d - 1] = (int)blk[bd].index;
          wsync();
        }
        Kid k;
        const int cnt = load_view(d, bd, R, C, k);
        const uint32_t target = d + 1 < n ? rlu(mine, n - 2 - d) : (MTB_LEAF | sid);
        const int j = first_set(__ballot(lane < cnt && k.id == target));
        if (j < 0) { fail(DERR_SHAPE); return 0; }
        pos += csum8(lane < j && k.rl != MTB_UNDEF ? k.rl : 0);
      }
    }
    pos += before ? -off : 1 + off;  // marker.cachedLength = 1
    if (pos < 0) fail(DERR_RELPOS);
    return pos;
  }

  // ------------------------------------------------------------------ ops
  __device__ __forceinline__ void set_min_seq(int msn) {  // mergeTree.ts:1025-1044
    if (!(msn <= curSeq) || !(minSeq <= msn)) { fail(DERR_ASSERT_MSN); return; }
    if (msn > minSeq) {
      minSeq = msn;
      zamboni();
    }
  }
  // block splits requested by the last walk (one call site keeps the split code out of the walk)
  __device__ __forceinline__ void settle() {
    if (COLD(pending_fix >= 0)) {
      const int d = pending_fix;
      pending_fix = -1;
      if (!err) fix_overflow(d);
    }
  }
  __device__ __forceinline__ void zamboni_p() {
    const uint64_t t0 = PROF_T();
    zamboni();
    PROF_ADD(PH_ZAMBONI, t0);
  }
  // One body segment of a SnapshotV1 load: insertSegments(root length, batch, UniversalSeq, C, S)
  // (snapshotLoader.ts:201-220, mergeTree.ts:1397-1427): ensureIntervalBoundary at the batch start, the
  // segment placed at the batch's advancing position in the (refSeq 0, C) view, zamboni at the batch end.
  __device__ __forceinline__ void apply_loadseg(const mtb_op& o, int S, int C) {
    view_clear();
    const bool first = (o.flags & MTB_F_LDFIRST) != 0;
    if (first) {
      ld_pos = U(blk[root].len);
      walk(ld_pos, 0, C, -2, false, 0);
      settle();
      if (bad()) return;
    }
    const bool marker = !isPerm && (o.flags & MTB_F_MARKER) != 0;
    const int len = marker ? 1 : (int)o.pos2;
    const int rseq = (int)o.ref_seq;
    if (len > 0) {
      const uint32_t sid = alloc_seg();
      if (bad()) return;
      if (lane < 8) {
        uint32_t v = 0;
        if (lane == F_ID) v = MTB_LEAF | sid;
        if (lane == F_LEN) v = (uint32_t)len;
        if (lane == F_SEQ) v = (uint32_t)S;
        if (lane == F_RSEQ) v = (uint32_t)rseq;
        if (lane == F_CLI) v = ((uint32_t)C & 0xFFFF) | (o.msn << 16);
        if (lane == F_RCX) v = o.pos1;
        if (lane == F_PROPS) v = o.props ? (MTB_GPROPS | UP(sh->tab.pidx)[2 * o.props + 1]) : 0;
        if (lane == F_TEXT) v = marker ? (MTB_MARKER | (o.pos2 == 0xFFFFFFFFu ? 0u : o.pos2 + 1)) : o.payload;
        sh->nseg[lane] = v;
      }
      wsync();
      n_mod += 1;
      if (COLD(marker && o.payload != 0)) {  // body markers are mapped whatever their removal (:1658-1663)
        mk_set(o.payload - 1, sid);
        if (bad()) return;
        mk_record(o.payload - 1, sid);
        if (bad()) return;
      }
      const bool ok = walk(ld_pos, 0, C, S, true, rseq >= 0 ? 0 : len, first);
      if (!ok) {
        fail(DERR_INSERT);
        return;
      }
      const int dins = U(ins_depth);
      ph_split_top = MTB_VDEPTH;
      settle();
      if (bad()) return;
      // a collaborating client's segment takes update() on every path block that did not split (the split halves
      // and a new root were recombined, which clears their deficits again); a document without a deficit table
      // (the host gives one to every load with collaborating body segments) refuses a stale update instead
      const int top = ph_split_top < dins + 1 ? ph_split_top : dins + 1;
      if (C != -2 && (ld_stale & ((1u << top) - 1u))) { fail(DERR_STALE); return; }
      if constexpr (hasPh) {
        if (COLD(phDoc)) {
          if (C == -2) {
            // NonCollabClient: blockUpdateLength recombines every block of the path (mergeTree.ts:2447-2452)
            ph_up(U(ins_blk));
          } else if (rseq >= 0) {
            // a removed segment of a collaborating client: update() records its insert, never its removal
            for (int i = 0; i < top && !err; i++)
              ph_add(U(sh->path[i]), (uint32_t)rseq, (uint32_t)len, o.msn, o.pos1, (uint32_t)S, PH_PHANTOM,
                     (uint32_t)C & 0xFFFF);
          }
          if (bad()) return;
        }
      }
      if (S > minSeq) lru_add(sid, U(ins_blk), U(ins_scour), S);
      ld_pos += len;
    }
    if (o.flags & MTB_F_LDLAST) zamboni_p();
  }
  // A live client's own op (client.ts:196-247 insertSegmentLocal / removeRangeLocal): applied in its own
  // view at (currentSeq, own id) with UnassignedSequenceNumber (here MTB_PEND + the new localSeq), after
  // getValidOpRange's bounds check (client.ts:527-592); no LRU, no zamboni, no sequence-number update.
  __device__ __forceinline__ void apply_local(const mtb_op& oin) {
    grp_open = false;
    const int len = (int)U(blk[root].len);  // the local view's length
    mtb_op o = oin;
    if (COLD(o.flags & MTB_F_RELPOS)) {  // getValidOpRange in the client's own view (Client.annotateMarker)
      view_clear();
      const int p1 = rel_pos(o.pos1, curSeq, 0);
      const int p2 = o.type == MTB_OP_INSERT ? 0 : rel_pos(o.pos2, curSeq, 0);
      if (err == DERR_RELPOS) err = DERR_RANGE;  // an unknown marker is -1: RangeOutOfBounds
      if (bad()) return;
      o.pos1 = (uint32_t)p1;
      if (o.type != MTB_OP_INSERT) o.pos2 = (uint32_t)p2;
      o.flags &= (uint8_t)~MTB_F_RELPOS;
    }
    if (o.type == MTB_OP_INSERT) {
      if ((int)o.pos1 < 0 || (int)o.pos1 > len) { fail(DERR_RANGE); return; }
    } else if (o.type == MTB_OP_REMOVE || o.type == MTB_OP_ANNOTATE) {
      // getValidOpRange (client.ts:550-585): start in [0, length), end > start (end past the length is
      // not checked; nodeMap stops at the tree's end)
      if ((int)o.pos1 < 0 || (int)o.pos1 >= len || (int)o.pos2 <= (int)o.pos1) { fail(DERR_RANGE); return; }
    } else {
      fail(DERR_LOCAL);
      return;
    }
    mtb_op l = o;
    l.seq = (uint32_t)(MTB_PEND + local_seq + 1);
    l.ref_seq = (uint32_t)curSeq;
    l.client = 0;
    l.flags &= (uint8_t)~MTB_F_LAST;
    local_seq++;  // (insertSegments / markRangeRemoved: ++collabWindow.localSeq)
    if (o.type == MTB_OP_INSERT && !(o.flags & MTB_F_MARKER) && o.pos2 == 0) local_seq--;  // nothing inserted
    apply_op(l);
  }
  __device__ __forceinline__ void apply(const mtb_op& o) {
    if (isLive && (o.flags & MTB_F_LOCAL)) {
      apply_local(o);
      return;
    }
    apply_op(o);
  }
  __device__ __forceinline__ void apply_op(const mtb_op& o) {
    const uint64_t tA = PROF_T();
    memo_old = MTB_NONE;
    memo_new = 0;
    const int S = (int)o.seq, R = (int)o.ref_seq, C = (int)(int16_t)o.client;
    const bool local = isLive && S >= MTB_PEND;
    if constexpr (MODE == MODE_REPLAY || MODE == MODE_MARKERS || MODE == MODE_LIVE) delta_on = (o.flags & MTB_F_DELTA) != 0;
    else delta_on = false;
    if constexpr (isLoad) {
      apply_loadseg(o, S, C);
      return;
    }
    switch (o.type) {
      case MTB_OP_INSERT: {
        ops_applied++;
        TCHK(1);
        view_clear();
        uint64_t t0 = PROF_T();
        int p1 = (int)o.pos1;
        if constexpr (hasMk)
          if (COLD(o.flags & MTB_F_RELPOS)) {  // getValidOpRange (client.ts:531-537)
            p1 = rel_pos(o.pos1, R, C);
            if (bad()) return;
          }
        walk(p1, R, C, -2, false, 0);  // ensureIntervalBoundary
        settle();
        PROF_ADD(PH_BOUNDARY, t0);
        TCHK(2);
        if (bad()) return;
        const bool marker = (o.flags & MTB_F_MARKER) != 0;
        const int len = marker ? 1 : (int)o.pos2;
        if (len > 0) {
          t0 = PROF_T();
          const uint32_t sid = alloc_seg();
          if (bad()) return;
          if (lane < 8) {
            uint32_t v = 0;
            if (lane == F_ID) v = MTB_LEAF | sid;
            if (lane == F_LEN) v = (uint32_t)len;
            if (lane == F_SEQ) v = (uint32_t)S;
            if (lane == F_RSEQ) v = (uint32_t)-1;
            if (lane == F_CLI) v = ((uint32_t)C & 0xFFFF) | 0xFFFF0000u;  // removedClientIds[0] = none
            if (lane == F_PROPS) v = o.props ? (MTB_GPROPS | UP(sh->tab.pidx)[2 * o.props + 1]) : 0;
            if (lane == F_TEXT)
              v = marker ? (MTB_MARKER | (o.pos2 == 0xFFFFFFFFu ? 0u : o.pos2 + 1))
                         : ((o.flags & MTB_F_PERMSEG) ? MTB_HANDLE_UNALLOC : o.payload);  // onDelta resets remote handles
            sh->nseg[lane] = v;
          }
          wsync();
          n_mod += 1;
          text_bytes += (marker || (o.flags & MTB_F_PERMSEG)) ? 0u : 2u * (uint32_t)len;
          if constexpr (hasMk)
            if (COLD(marker && o.payload != 0)) {
              mk_set(o.payload - 1, sid);
              if (bad()) return;
              mk_record(o.payload - 1, sid);
              if (bad()) return;
            }
          if (!walk(p1, R, C, S, true, len, true)) {
            fail(DERR_INSERT);
            return;
          }
          TCHK(3);
          settle();
          TCHK(4);
          if (local) grp_add(sid, MTB_OP_INSERT, 0);  // saveIfLocal (mergeTree.ts:1617-1637)
          else if (S > minSeq) lru_add(sid, U(ins_blk), U(ins_scour), S);
          if (COLD(delta_on)) {
            const uint32_t from = delta_used;
            delta_emit(lane == 0, sid, (uint32_t)len, o.props ? (MTB_GPROPS | UP(sh->tab.pidx)[2 * o.props + 1]) : 0u);
            delta_positions(from);
            if (bad()) return;
          }
          PROF_ADD(PH_INSERT, t0);
        }
        if (!local) zamboni_p();
        break;
      }
      case MTB_OP_REMOVE:
      case MTB_OP_ANNOTATE: {
        ops_applied++;
        view_clear();
        if constexpr (hasMk) ann_mk = o.type == MTB_OP_ANNOTATE ? (o.payload & 3u) : 0u;
        uint64_t t0 = PROF_T();
        int p1 = (int)o.pos1, p2 = (int)o.pos2;
        if constexpr (hasMk)
          if (COLD(o.flags & MTB_F_RELPOS)) {  // getValidOpRange (client.ts:531-547)
            p1 = rel_pos(o.pos1, R, C);
            if (bad()) return;
            p2 = rel_pos(o.pos2, R, C);
            if (bad()) return;
          }
        walk(p1, R, C, -2, false, 0);
        settle();
        walk(p2, R, C, -2, false, 0);
        settle();
        PROF_ADD(PH_BOUNDARY, t0);
        if (bad()) return;
        t0 = PROF_T();
        const uint32_t dfrom = delta_used;
        if (isLive) sh->memo[2] = 0;
        // 1 rewrite, 2 incr, 3 consensus, 4 a live client's own consensus (annotateMarkerNotifyConsensus)
        int comb = o.type != MTB_OP_ANNOTATE ? 0 : (o.flags & MTB_F_COMB) >> 2;
        if (isLive && comb == 3 && local) comb = 4;
        TCHK(5);
        node_map(p1, p2, R, C, S, o.type == MTB_OP_REMOVE, o.props, comb);
        TCHK(6);
        if (COLD(delta_on)) {
          if (bad()) return;
          delta_positions(dfrom);
        }
        if (isLive) {  // blocks whose segments a remote remove took over from unacked local removes
          const uint32_t nrb = U(sh->memo[2]);
          if (nrb > 64) { fail(DERR_CAP_PEND); return; }
          const uint32_t mine = (uint32_t)lane < nrb ? sh->pk[lane] : MTB_NONE;  // (pk shares the rebuild scratch)
          wsync();
          for (uint32_t i = 0; i < nrb && !err; i++) rebuild_up(rlu(mine, (int)i));
          if (nrb) view_clear();
        }
        PROF_ADD(PH_NODEMAP, t0);
        if (!local) zamboni_p();
        break;
      }
      case MTB_OP_ACK:
        if (isLive) ack_group(S, (int)o.pos2, (o.flags & MTB_F_COMB) == MTB_F_CONSENSUS ? o.props : 0u, o.payload);
        zamboni_p();
        break;
      case MTB_OP_REGEN:
        if constexpr (isLive) regen(o.pos1);
        break;
      case MTB_OP_MAINT:  // zamboniSegments / packParent(root) called directly (mergeTree.zamboni.spec.ts)
        if constexpr (isLive) {
          view_clear();
          if (o.pos1 == 0) {
            zamboni();
          } else {
            const uint32_t rc = U(blk[root].count);
            if (rc > 0 && (U(blk[root].f[F_ID][0]) & MTB_LEAF)) { fail(DERR_SHAPE); return; }  // children must be blocks
            pack_parent(root);
          }
          view_clear();
        }
        break;
      default:
        break;
    }
    if (bad()) return;
    if ((o.flags & MTB_F_LAST) && !local) {  // updateSeqNumbers (client.ts:877-887)
      if (!(curSeq <= S)) { fail(DERR_ASSERT_SEQ); return; }
      curSeq = S;
      if (!((int)o.msn <= S)) { fail(DERR_ASSERT_MSN); return; }
      const uint64_t t0 = PROF_T();
      set_min_seq((int)o.msn);
      PROF_ADD(PH_ZAMBONI, t0);
    }
    PROF_ADD(PH_TOTAL, tA);
  }
};

}  // namespace mtbk

using namespace mtbk;

#ifndef MTB_WAVES_PER_SIMD
#define MTB_WAVES_PER_SIMD 4
#endif
__device__ __forceinline__ uint32_t ds_word(uint32_t w0, uint32_t w1, uint32_t i) { return i < 64 ? rlu(w0, i) : rlu(w1, i - 64); }
// Replays document `doc` from its op_next; returns the op_next it leaves (the record after the last one applied).
template <int MODE, class SCR>
__device__ __forceinline__ uint32_t replay_doc(SCR& sh, uint32_t doc, int32_t* xch, int wv,
                                           DocState* docs,  // (no __restrict__: see mtb_replay_tick_kernel)
                                           uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks, WEnt* lists,
                                           uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                                           const Tables& tables, uint32_t upto = 0) {
  if (doc >= ndocs) return 0;
  DocState* ds = &docs[doc];
  Eng<MODE, SCR> e;
  e.xch = xch;
  e.wv = wv;
  e.ds = ds;
  // The DocState arrives as two vector loads (lane i: dwords i and 64 + i) read out with v_readlane, never
  // through the scalar cache: within one launch of mtb_replay_tick_kernel another workgroup wrote it (the
  // previous chunk's), and the hand-over's acquire does not invalidate the scalar cache.
  const uint32_t dw0 = reinterpret_cast<const uint32_t*>(ds)[lane_id()];
  const uint32_t dw1 = lane_id() < (int)(sizeof(DocState) / 4 - 64) ? reinterpret_cast<const uint32_t*>(ds)[64 + lane_id()] : 0u;
#define DSF(f) ds_word(dw0, dw1, offsetof(DocState, f) / 4)
#define DSF64(f) (((uint64_t)ds_word(dw0, dw1, offsetof(DocState, f) / 4 + 1) << 32) | ds_word(dw0, dw1, offsetof(DocState, f) / 4))
  // a document on the marker variant (DSF_VARIANT, mtb_host.cpp mark_variant_docs) is the marker kernel's; every
  // other document of such a batch the observer kernels'
  if constexpr (MODE == MODE_REPLAY) {
    if (DSF(flags) & DSF_VARIANT) return DSF(op_next);
  } else if constexpr (MODE == MODE_MARKERS) {
    if (!(DSF(flags) & DSF_VARIANT)) return DSF(op_next);
  }
#ifdef MTB_CHECK
  {
    uint32_t* rep = &ds->pad3[0];
    e.segp.p = segp + DSF64(seg_base), e.segp.cap = &sh.capv[0], e.segp.rep = rep, e.segp.pool = 0;
    e.blk.p = blks + DSF64(blk_base), e.blk.cap = &sh.capv[1], e.blk.rep = rep, e.blk.pool = 1;
    e.lst.p = lists + DSF64(list_base), e.lst.cap = &sh.capv[2], e.lst.rep = rep, e.lst.pool = 2;
    e.aux.p = aux + DSF64(aux_base), e.aux.cap = &sh.capv[5], e.aux.rep = rep, e.aux.pool = 3;
  }
#else
  e.segp = segp + DSF64(seg_base);
  e.blk = blks + DSF64(blk_base);
  e.lst = lists + DSF64(list_base);
  e.aux = aux + DSF64(aux_base);
#endif
  Lru* const gheap = heap + DSF64(heap_base);
  const mtb_op* const dops = ops + DSF64(op_base);
  sh.tab = tables;  // (every lane stores the same values)
  sh.gheap = gheap;
  sh.gfree = freel + DSF64(free_base);
  sh.gtext = text + DSF64(text_base);
  e.sh = &sh;
#ifdef MTB_TABCHECK
  e.x_sh = &sh;
  e.x_ptr[0] = RAW(e.segp);
  e.x_ptr[1] = RAW(e.blk);
  e.x_ptr[2] = RAW(e.lst);
  e.x_ptr[3] = RAW(e.aux);
  e.x_tab = &tables;
#endif
  e.lane = lane_id();
  e.minSeq = (int)DSF(min_seq);
  e.curSeq = (int)DSF(cur_seq);
  e.root = DSF(root);
  e.newMode = DSF(new_mode) != 0;
  e.hasNL = (DSF(flags) & DSF_NEWLINE) != 0;
  e.seg_used = DSF(seg_used);
  e.blk_used = DSF(blk_used);
  e.free_top = DSF(free_top);
  e.list_used = DSF(list_used);
  e.text_used = DSF(text_used);
  e.heap_cnt = DSF(heap_cnt);
  e.aux_used = DSF(aux_used);
  e.err = (int)DSF(err);
  e.n_mod = 0;
  e.ops_applied = 0;
  e.text_bytes = 0;
  uint32_t k = DSF(op_next);
  const uint32_t n = DSF(n_ops);
  // a scheduler ticket replays up to upto/4096 of the document's records (0: all of them)
  const uint32_t kend = upto ? (uint32_t)(((uint64_t)n * upto + 4095) >> 12) : n;
  uint32_t errk = n;  // MODE_MATRIX: index after the record that failed
  e.walk_depth = -1;
  e.vmask = 0;
  e.struct_changed = false;
  e.pending_fix = -1;
  e.ld_pos = 0;
  e.delta_on = false;
#ifdef MTB_NO_MKREMAP  // (test builds: shows the reused-id tests depend on the re-mapping)
  e.mkDup = false;
#else
  e.mkDup = (DSF(flags) & DSF_MKDUP) != 0;
#endif
  e.ann_mk = 0;
  e.delta_used = DSF(delta_used);
  e.ph_off = DSF(ph);
  e.phDoc = Eng<MODE, SCR>::hasPh && (DSF(flags) & DSF_PHANTOM) != 0 && e.ph_off != 0;
  e.ph_split_top = MTB_VDEPTH;
  e.ph_ow = false;
  e.ld_stale = 0;
  e.cur_k = 0;
  e.sp_internal = false;
  e.local_seq = (int)DSF(local_seq);
  e.pend_dir = DSF(pend_dir);
  e.pend_head = DSF(pend_head);
  e.pend_n = DSF(pend_n);
  e.pend_cap = DSF(pend_cap);
  e.grp_open = false;
  e.pk_rw = false;
  if (e.lane < 6) sh.capv[e.lane] = (&ds->seg_cap)[e.lane];
  if (e.lane == 6) sh.capv[6] = DSF(delta_cap);
  sh.ins[0] = (int32_t)MTB_NONE;  // (every lane stores the same values)
  sh.ins[1] = sh.ins[2] = sh.ins[3] = -1;
  for (int i = 0; i < NPH; i++) e.prof[i] = 0;
  for (int i = 0; i < NCN; i++) e.evc[i] = 0;
  // root window-list metadata, the list free heads and the LRU heap (while it fits) into LDS
  if (e.lane < 3) sh.rmeta[e.lane] = (&e.blk[e.root].loff)[e.lane];
  if (e.list_used == 0) {
    if (e.lane < MTB_LCLASSES) sh.lfree[e.lane] = MTB_NONE;
    e.list_used = MTB_LIST_RESERVED;
  } else if (e.lane < MTB_LCLASSES) {
    sh.lfree[e.lane] = reinterpret_cast<const uint32_t*>(RAW(e.lst))[e.lane];
  }
#ifndef MTB_NO_LSTK
  if (e.lane < MTB_LSTK) sh.lstkn[e.lane] = 0;
#endif
  if (e.lane == 0) sh.path[0] = e.root;
  e.heap_lds = e.heap_cnt + 1 < e.lheap_n;
  if (e.heap_lds)
    for (uint32_t i = 1 + e.lane; i <= e.heap_cnt; i += 64) {
      u32x2 v;
      v.x = gheap[i].seg;
      v.y = (uint32_t)gheap[i].maxSeq;
      *reinterpret_cast<u32x2*>(&sh.heap[i]) = v;
    }
  e.view_clear();
  __syncthreads();
  if (k < n) {
    // op records are read one dword per lane (lanes 0..7), the next one in flight while applying
    const uint32_t* opw = reinterpret_cast<const uint32_t*>(dops);
    uint32_t cw = e.lane < 8 ? opw[k * 8 + e.lane] : 0u;
    int par = 0;  // MODE_MATRIX: setCell exchange parity
    // a matrix wave keeps walking its records after an error: its partner waits for it at every setCell
    for (; k < kend && k < n && (MODE == MODE_MATRIX || !e.err); k++) {
      const uint32_t nk = k + 1 < n ? k + 1 : k;
      const uint32_t nw = e.lane < 8 ? opw[nk * 8 + e.lane] : 0u;  // prefetch the next record
      mtb_op cur;
      const uint32_t w0 = rlu(cw, 0);
      cur.type = (uint8_t)(w0 & 0xFF);
      cur.flags = (uint8_t)((w0 >> 8) & 0xFF);
      cur.client = (uint16_t)(w0 >> 16);
      cur.seq = rlu(cw, 1);
      cur.ref_seq = rlu(cw, 2);
      cur.msn = rlu(cw, 3);
      cur.pos1 = rlu(cw, 4);
      cur.pos2 = rlu(cw, 5);
      cur.payload = rlu(cw, 6);
      cur.props = rlu(cw, 7);
      if constexpr (MODE == MODE_LOAD || MODE == MODE_LOADPERM) {
        if (cur.type != MTB_OP_LOADSEG) break;  // the summary body precedes every op
      }
      e.cur_k = k;
      CRUMB(ndocs + doc, k);
#ifdef MTB_TABCHECK  // (fault triage, DESIGN.md section 4: is the LDS copy of the batch tables intact at each op?)
      {
        const bool ok = sh.tab.pool == tables.pool && sh.tab.pidx == tables.pidx && sh.tab.val_class == tables.val_class &&
                        sh.tab.val_falsy == tables.val_falsy && sh.tab.key_rank == tables.key_rank &&
                        sh.tab.key_irr == tables.key_irr && sh.tab.val_local == tables.val_local &&
                        sh.tab.irr == tables.irr && sh.gheap == gheap && sh.gtext == text + DSF64(text_base);
        if (__ballot(!ok)) {
          if (e.lane == 0) {
            ds->pad3[0] = 1;
            ds->pad3[1] = k;
            ds->pad3[2] = (uint32_t)(uintptr_t)sh.tab.val_falsy;
            ds->pad3[3] = 0;
          }
          e.fail(DERR_SHAPE);
          break;
        }
      }
#endif
      if constexpr (MODE == MODE_MATRIX) {
        if (cur.type == MTB_OP_SETCELL) {
          e.setcell(cur, par);
          par ^= 1;
          cw = nw;
          continue;
        }
        if (e.err) {
          cw = nw;
          continue;
        }
      }
      e.apply(cur);
      if constexpr (MODE == MODE_MATRIX) {
        if (e.err && errk == n) errk = k + 1;
      }
      cw = nw;
    }
  }
  if (e.heap_lds)
    for (uint32_t i = 1 + e.lane; i <= e.heap_cnt; i += 64) {
      const u32x2 v = *reinterpret_cast<const u32x2*>(&sh.heap[i]);
      gheap[i].seg = v.x;
      gheap[i].maxSeq = (int)v.y;
    }
#ifndef MTB_NO_LSTK
  // the LDS stacks go back onto the free lists in HBM (lane c: class c)
  if (e.lane < MTB_LSTK) {
    uint32_t head = sh.lfree[e.lane];
    const uint32_t n = sh.lstkn[e.lane];
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t off = sh.lstk[e.lane][i];
      reinterpret_cast<uint32_t*>(&e.lst[off])[0] = head;
      head = off;
    }
    sh.lfree[e.lane] = head;
  }
  __syncthreads();
#endif
  if (e.lane < MTB_LCLASSES) reinterpret_cast<uint32_t*>(RAW(e.lst))[e.lane] = sh.lfree[e.lane];
  __syncthreads();
  if (e.lane == 0) {
    ds->min_seq = e.minSeq;
    ds->cur_seq = e.curSeq;
    ds->root = e.root;
    ds->seg_used = e.seg_used;
    ds->blk_used = e.blk_used;
    ds->free_top = e.free_top;
    ds->list_used = e.list_used;
    ds->text_used = e.text_used;
    ds->heap_cnt = e.heap_cnt;
    ds->aux_used = e.aux_used;
    ds->delta_used = e.delta_used;
    ds->ph = e.ph_off;
    if (MODE == MODE_LIVE) {
      ds->local_seq = e.local_seq;
      ds->pend_dir = e.pend_dir;
      ds->pend_head = e.pend_head;
      ds->pend_n = e.pend_n;
      ds->pend_cap = e.pend_cap;
    }
    ds->n_mod += e.n_mod;
    ds->ops_applied += e.ops_applied;
    ds->text_bytes += e.text_bytes;
#ifdef MTB_PROFILE
    for (int i = 0; i < NPH; i++) {
      if (i < 7) ds->prof[i] += e.prof[i];
      else ds->prof2[i - 7] += e.prof[i];
    }
    for (int i = 0; i < NCN; i++) {
      if (i < 5) ds->cnt[i] += e.evc[i];
      else ds->cnt2[i - 5] += e.evc[i];
    }
#endif
    if (e.err && !ds->err) {
      ds->err = e.err;
      ds->err_op = MODE == MODE_MATRIX ? errk : k;
    }
    ds->op_next = k;
  }
  return k;
}

#define KARGS docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables
#if MTB_TU_HAS(MTB_TU_OBS)
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_replay_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                      WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  replay_doc<MODE_REPLAY>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
// Batches with more documents than wave slots, as a sequence of launches ("passes"): the tasks (chunk c of
// document x) are ordered chunk-major, task i = c * ndocs + x, and pass p runs tasks [first, first + grid): one
// workgroup per task, which replays document x up to the fraction (c + 1) / nchunks of its records.  A pass
// holds at most one chunk per document (grid <= ndocs) and a chunk's predecessor sits ndocs tasks earlier, in
// an earlier pass, so the launch boundary orders them.  The host sizes passes as multiples of the resident
// wave slots: every pass is whole rounds of equal tasks.
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_replay_pass_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                           WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables,
                           uint32_t first, uint32_t nchunks) {
  __shared__ Scratch sh;
  const uint32_t t = first + blockIdx.x;
  const uint32_t c = t / ndocs;
  const uint32_t upto = c + 1 >= nchunks ? 0u : (uint32_t)(((c + 1) * 4096u) / nchunks);
  replay_doc<MODE_REPLAY>(sh, t - c * ndocs, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables,
                          upto);
}
// Batches with more documents than wave slots: tickets (chunk c, document d), one per workgroup (grid =
// documents x chunks).  Ticket c replays document d's records up to the fraction plan[c] / 4096 of them (the
// host's chunk plan), so every document advances at the same pace and the launch ends within about one ticket
// of the ideal, instead of a last partial "round" of whole documents (10,000 documents on 4,096 slots = 2.44
// rounds).  A workgroup takes the next ticket of its XCD's queue (HW_REG_XCC_ID; or of the next queue with
// tickets left) as it starts, waits for the document's previous chunk, replays its chunk and exits.
//
// Queues (L2 affinity, speed only): documents are split into nq queues (d mod nq, nq = the device's XCD
// count), so a document's chunks normally run on one XCD.  Correctness never depends on where a workgroup
// runs: every hand-over is an agent-scope release (after the chunk's stores) and acquire (before the next
// chunk's loads).  In queue q, ticket t = c * n_q + j names document d = j * nq + q; it waits for ticket
// t - n_q (the same document's previous chunk), which a workgroup that started earlier took and is running,
// so the waits always drain.  The DocState is read with vector loads (replay_doc): the scalar cache is not
// invalidated by the acquire.  A wait longer than `spins` polls raises the abort flag; later workgroups leave
// at once, and mtb_replay_finish_kernel, launched right after, replays the rest of every document (each
// document's state is consistent at its op_next).
// sched: [32 q] next ticket of queue q (one line each), [MTB_SCHED_ABORT] abort flag, [MTB_SCHED_SPINS] the
// wait bound, [MTB_SCHED_HDR + d] chunks of document d completed (zeroed before launch), [MTB_SCHED_HDR +
// ndocs + c] the plan: cumulative record fraction of chunk c in 1/4096 (the last one 4096), [MTB_SCHED_HDR + ndocs +
// nchunks + d] the op_next document d's last completed chunk left (tick_check).
//
// (Rounds 2-3 ran the tickets on persistent waves, the engine a called function between them.  In round 4 that
// kernel faulted in some builds; its replacement keeps the plain replay kernel's register allocation.  The
// wait is a called function: inlined, its loop and acquire fence made the engine spill.)
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}
// The hand-over helpers are called functions in the product build (inlined, their spin loop and fence made the
// engine spill).  Builds whose engine spills anyway (MTB_PROFILE) inline them: a kernel that both uses scratch and
// makes calls faulted deterministically in the MTB_PROFILE_PACK build (DESIGN.md §4 "Round 6": independent of
// hand-overs, gone with the calls inlined); tests/test_code_object.py keeps the product kernel free of scratch.
#if defined(MTB_TICK_INLINE) || defined(MTB_PROFILE)
#define TICK_FN __device__ __forceinline__
#else
#define TICK_FN __device__ __attribute__((noinline))
#endif
TICK_FN bool tick_wait(uint32_t* sched, uint32_t* prog, uint32_t c, uint32_t spins) {
  uint32_t n = 0;
  while (U(__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < c) {
    if (++n > spins) {
      if (lane_id() == 0) __hip_atomic_store(&sched[MTB_SCHED_ABORT], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(16);
    if (COLD((n & 1023) == 0) &&
        U(__hip_atomic_load(&sched[MTB_SCHED_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
      return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // one acquire per hand-over (the spin reads relaxed)
  return true;
}
// The hand-over invariant, checked at every chunk's entry after the acquire: the document's DocState is the one
// the previous chunk left (its op_next equals the record index that chunk returned, published beside the progress
// word).  A mismatch means this workgroup would resume from a stale state (round 4's scalar-cache fault had that
// shape): the chunk is not run, the first mismatch is recorded ([MTB_SCHED_BAD] count, then document, chunk,
// expected, seen) and the abort flag hands the rest to mtb_replay_finish_kernel, a new launch that reads every
// DocState afresh.  Both words are read with agent-scope atomic loads (vector memory, never the scalar cache).
TICK_FN bool tick_check(uint32_t* sched, uint32_t* hand, uint32_t* opn, uint32_t d, uint32_t c) {
  const uint32_t want = U(__hip_atomic_load(hand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t have = U(__hip_atomic_load(opn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (want == have) return true;
  if (lane_id() == 0) {
    if (atomicAdd(&sched[MTB_SCHED_BAD], 1u) == 0) {
      __hip_atomic_store(&sched[MTB_SCHED_BAD + 1], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sched[MTB_SCHED_BAD + 2], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sched[MTB_SCHED_BAD + 3], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sched[MTB_SCHED_BAD + 4], have, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(&sched[MTB_SCHED_ABORT], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return false;
}
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_replay_tick_kernel(DocState* docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                           WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables,
                           uint32_t* sched, uint32_t nchunks, uint32_t nq) {
  __shared__ Scratch sh;
  const uint32_t home = xcc_id() % nq;
  uint32_t d = MTB_NONE, c = 0;
  for (uint32_t qi = 0; qi < nq && d == MTB_NONE; qi++) {
    const uint32_t q = (home + qi) % nq;
    if (q >= ndocs) continue;
    const uint32_t nqd = (ndocs - q + nq - 1) / nq;  // documents of queue q
    uint32_t t = 0;
    if (lane_id() == 0) t = atomicAdd(&sched[MTB_SCHED_TICK * q], 1u);
    t = U(t);
    if (t >= nqd * nchunks) continue;
    c = t / nqd;
    d = (t - c * nqd) * nq + q;
  }
  if (d == MTB_NONE) return;
  CRUMB(d, 1 | c << 8);
  if (U(__hip_atomic_load(&sched[MTB_SCHED_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0) return;
  uint32_t* prog = &sched[MTB_SCHED_HDR + d];
  uint32_t* hand = &sched[MTB_SCHED_HDR + ndocs + nchunks + d];  // op_next the previous chunk left
  if (c > 0) {
    if (!tick_wait(sched, prog, c, U(sched[MTB_SCHED_SPINS]))) return;
    if (!tick_check(sched, hand, &docs[d].op_next, d, c)) return;
  }
  CRUMB(d, 2 | c << 8);
  const uint32_t k = replay_doc<MODE_REPLAY>(sh, d, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel,
                                             tables, U(sched[MTB_SCHED_HDR + ndocs + c]));
  CRUMB(d, 3 | c << 8);
  if (c + 1 < nchunks && lane_id() == 0) *hand = k;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (MI355X guide: the write-back completes before the flag)
  if (lane_id() == 0) __hip_atomic_store(prog, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  CRUMB(d, 4 | c << 8);
}
// After an aborted scheduled launch: every document continues from its op_next (one wave per document;
// documents that finished have nothing left).  Without an abort every wave leaves at once.
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_replay_finish_kernel(DocState* docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                             WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables,
                             const uint32_t* sched) {
  __shared__ Scratch sh;
  if (U(sched[MTB_SCHED_ABORT]) == 0) return;
  replay_doc<MODE_REPLAY>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
#endif
#if MTB_TU_HAS(MTB_TU_FEW)
// The same engine for batches of few documents (at most a few per CU, e.g. BASELINE configs[3]'s single
// long document): LDS is not what limits occupancy there, so the zamboni LRU heap keeps up to 2,047
// entries in LDS instead of spilling to HBM past 127.
extern "C" __global__ void __launch_bounds__(64, 1)
    mtb_replay_few_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                          WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ ScratchBig sh;
  replay_doc<MODE_REPLAY>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
#endif
// Batches holding live clients (local ops, acks of them): the replay engine with the local-op paths.
#if MTB_TU_HAS(MTB_TU_LIVE)
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_live_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                    WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  replay_doc<MODE_LIVE>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
#endif
// Batches whose documents carry marker ids: the replay engine with idToSegment and relative positions.
#if MTB_TU_HAS(MTB_TU_MARKERS)
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_markers_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                       WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  replay_doc<MODE_MARKERS>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
#endif
// SnapshotV1 body append (LOADSEG records), run before mtb_replay_kernel when a load is pending.
#if MTB_TU_HAS(MTB_TU_LOADMAT)
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_load_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                    WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  replay_doc<MODE_LOAD>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
// The same for the PermutationVectors of a matrix batch (segments carry handle starts, no text).
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD)
    mtb_load_perm_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                         WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  replay_doc<MODE_LOADPERM>(sh, blockIdx.x, nullptr, 0, docs, ndocs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
// SharedMatrix batches: one 128-lane workgroup per matrix, wave 0 = rows vector (document 2m), wave 1 =
// cols vector (document 2m + 1); setCell records meet at a workgroup barrier (matrix.ts:668-676).
extern "C" __global__ void __launch_bounds__(128, MTB_WAVES_PER_SIMD)
    mtb_matrix_kernel(DocState* __restrict__ docs, uint32_t ndocs, const mtb_op* ops, uint32_t* segp, FBlk* blks,
                      WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  __shared__ Scratch sh[2];
  __shared__ int32_t xch[4];
  const int wv = (int)(threadIdx.x >> 6);
  replay_doc<MODE_MATRIX>(sh[wv], 2 * blockIdx.x + (uint32_t)wv, xch, wv, docs, ndocs, ops, segp, blks, lists, text, heap,
                          aux, freel, tables);
}

hipError_t mtb_launch_matrix(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp,
                             FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                             Tables tables) {
  hipLaunchKernelGGL(mtb_matrix_kernel, dim3((ndocs + 1) / 2), dim3(128), 0, stream, KARGS);
  return hipGetLastError();
}
hipError_t mtb_launch_load(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp,
                           FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel,
                           Tables tables, int perm) {
  if (perm)
    hipLaunchKernelGGL(mtb_load_perm_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  else
    hipLaunchKernelGGL(mtb_load_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  return hipGetLastError();
}
#endif
#define KPARAMS hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, uint32_t* segp, FBlk* blks, \
                WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables
#if MTB_TU_HAS(MTB_TU_FEW)
hipError_t mtb_launch_few(KPARAMS) {
  hipLaunchKernelGGL(mtb_replay_few_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  return hipGetLastError();
}
#endif
#if MTB_TU_HAS(MTB_TU_OBS)
// Up to MTB_FEW_DOCS documents (at most ~4 per CU) replay on the large-LDS-heap variant.
#define MTB_FEW_DOCS 1024
hipError_t mtb_launch_few(KPARAMS);
hipError_t mtb_launch_observer(KPARAMS) {
  if (ndocs <= MTB_FEW_DOCS)
    return mtb_launch_few(stream, ndocs, docs, ops, segp, blks, lists, text, heap, aux, freel, tables);
  else
    hipLaunchKernelGGL(mtb_replay_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  return hipGetLastError();
}
// resident waves of the scheduled kernel per CU (its grid is exactly the device's resident slots)
int mtb_sched_waves_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(mtb_replay_tick_kernel), 64, 0) !=
          hipSuccess || n <= 0)
    return 16;
  return n;
}
// tickets, then mtb_replay_finish_kernel (it replays the rest of every document after an abort, else exits)
hipError_t mtb_launch_replay_ticks(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops,
                                   uint32_t* segp, FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux,
                                   uint32_t* freel, Tables tables, uint32_t* sched, uint32_t nchunks, uint32_t nq) {
#ifdef MTB_CRUMBS
  static uint32_t* hc = nullptr;
  static size_t hn = 0;
  if (hn < 2 * (size_t)ndocs) {
    if (hc) (void)hipHostFree(hc);
    if (hipHostMalloc((void**)&hc, 2 * (size_t)ndocs * 4, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return hipErrorOutOfMemory;
    hn = 2 * (size_t)ndocs;
  }
  memset(hc, 0, 2 * (size_t)ndocs * 4);
  uint32_t* dc = nullptr;
  (void)hipHostGetDevicePointer((void**)&dc, hc, 0);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(mtb_crumbs), &dc, sizeof dc);
#endif
  hipLaunchKernelGGL(mtb_replay_tick_kernel, dim3(ndocs * nchunks), dim3(64), 0, stream, KARGS, sched, nchunks, nq);
  hipError_t e = hipGetLastError();
#ifdef MTB_CRUMBS
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  {
    uint32_t cnt[5] = {0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < ndocs; i++) cnt[std::min<uint32_t>(hc[i] & 0xFF, 4)]++;
    fprintf(stderr, "mtb_crumbs after the tick kernel (%s): stage 0 %u, 1 %u, 2 %u, 3 %u, 4 %u\n", hipGetErrorString(e), cnt[0],
            cnt[1], cnt[2], cnt[3], cnt[4]);
    uint32_t shown = 0;
    for (uint32_t i = 0; i < ndocs; i++) {
      const uint32_t st = hc[i] & 0xFF;
      if ((st == 1 || st == 3 || (e != hipSuccess && st == 2)) && shown++ < 40)
        fprintf(stderr, "mtb_crumbs doc %u stage %u chunk %u record %u\n", i, st, hc[i] >> 8, hc[ndocs + i]);
    }
  }
#endif
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mtb_replay_finish_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS, (const uint32_t*)sched);
  return hipGetLastError();
}
hipError_t mtb_launch_replay_passes(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops,
                                    uint32_t* segp, FBlk* blks, WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux,
                                    uint32_t* freel, Tables tables, uint32_t first, uint32_t count, uint32_t nchunks) {
  hipLaunchKernelGGL(mtb_replay_pass_kernel, dim3(count), dim3(64), 0, stream, KARGS, first, nchunks);
  return hipGetLastError();
}
#endif
#if MTB_TU_HAS(MTB_TU_LIVE)
hipError_t mtb_launch_live(KPARAMS) {
  hipLaunchKernelGGL(mtb_live_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  return hipGetLastError();
}
#endif
#if MTB_TU_HAS(MTB_TU_MARKERS)
hipError_t mtb_launch_markers(KPARAMS) {
  hipLaunchKernelGGL(mtb_markers_kernel, dim3(ndocs), dim3(64), 0, stream, KARGS);
  return hipGetLastError();
}
#endif
#if MTB_TU_HAS(MTB_TU_MISC)
hipError_t mtb_launch_observer(KPARAMS);
hipError_t mtb_launch_live(KPARAMS);
hipError_t mtb_launch_markers(KPARAMS);
hipError_t mtb_launch_replay(KPARAMS, int variant) {
  if (variant == 1) return mtb_launch_live(stream, ndocs, docs, ops, segp, blks, lists, text, heap, aux, freel, tables);
  if (variant == 2) return mtb_launch_markers(stream, ndocs, docs, ops, segp, blks, lists, text, heap, aux, freel, tables);
  return mtb_launch_observer(stream, ndocs, docs, ops, segp, blks, lists, text, heap, aux, freel, tables);
}
// ---------------------------------------------------------------------- state digest v1
// One wave per document folds the replayed state -- every segment in tree order with its tree path,
// text (or marker / handle span), seq, client, removal info and properties -- into 64 bits
// (DESIGN.md "State digest"; the checker restates the same definition over its own tree, Doc::digest).
// Per document out[3d..3d+2] = {digest, segments in the tree, observer length}; a failed document or a
// tree the walk cannot trust (depth > 16, a block id out of range, a text span outside the arena)
// reports digest 0.
namespace mtbk {
__device__ __forceinline__ uint64_t dg_fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ uint64_t dg_mix(uint64_t h, uint64_t x) {
  return dg_fmix(h ^ (x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
}  // namespace mtbk

#define MTB_DG_DEPTH 16
extern "C" __global__ void __launch_bounds__(64)
    mtb_digest_kernel(const DocState* __restrict__ docs, uint32_t ndocs, const FBlk* blks, const uint16_t* text,
                      const uint32_t* aux, const uint32_t* pool, const uint64_t* khash, const uint64_t* vhash,
                      uint64_t* out) {
  __shared__ uint32_t ids[MTB_DG_DEPTH][MTB_MAXCH];
  __shared__ int32_t cnt[MTB_DG_DEPTH], nxt[MTB_DG_DEPTH];
  __shared__ uint32_t rec[64];
  const uint32_t doc = blockIdx.x;
  const int lane = threadIdx.x;
  if (doc >= ndocs) return;
  const DocState& s = docs[doc];
  const int32_t derr = s.err;
  if (derr) {
    if (lane < 3) out[3 * doc + lane] = 0;
    return;
  }
  const FBlk* B = blks + s.blk_base;
  const uint16_t* T = text + s.text_base;
  const uint32_t* A = aux + s.aux_base;
  const uint32_t blk_used = s.blk_used, text_cap = s.text_cap, aux_used = s.aux_used;
  const bool perm = (s.flags & DSF_PERM) != 0;
  const uint32_t root = s.root;
  // client ids as the reference numbers them: engine id 0 and the observer's reference id swap places
  const int obs = (int)(s.flags >> DSF_OBS_SHIFT);
  auto rid = [&](int c) -> uint32_t { return (uint32_t)(c < 0 ? c : c == 0 ? obs : c == obs ? 0 : c); };
  const int sg = lane >> 3, q = lane & 7;  // leaf blocks: lane (segment slot, part)
  uint64_t acc = 0;
  uint64_t nsegs = 0;
  bool bad = root >= blk_used;
  int d = 0;
  uint32_t entered = 1;  // a block is entered once per walk: more entries than blocks is a corrupt tree
  // fetch block b as depth d of the walk: children ids + count, the whole record into rec[]
  auto enter = [&](uint32_t b, int dd) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(B + b);
    const uint32_t v = w[lane];
    const uint32_t c = w[FB_HDR];
    rec[lane] = v;
    if (lane < MTB_MAXCH) ids[dd][lane] = v;
    if (lane == 0) {
      cnt[dd] = (int32_t)(c > MTB_MAXCH ? MTB_MAXCH : c);
      nxt[dd] = 0;
    }
    __syncthreads();
  };
  if (!bad) enter(root, 0);
  while (!bad) {
    const int c = cnt[d], k = nxt[d];
    if (k >= c) {
      if (d == 0) break;
      d--;
      continue;
    }
    const uint32_t child = ids[d][k];
    if (child & MTB_LEAF) {
      // a leaf-level block (the one entered last): all its segments at once, 8 lanes per segment
      uint64_t P = 0;
      for (int l = 0; l < d; l++) P += (uint64_t)(nxt[l]) << (4 * l);  // nxt[l] = slot taken + 1
      uint64_t t = 0;
      bool kbad = false;
      uint32_t len = 0, seq = 0, rseq = 0, cli = 0, rcx = 0, props = 0, txt = 0, id = MTB_NONE;
      if (sg < c) {
        id = rec[F_ID * 8 + sg];
        len = rec[F_LEN * 8 + sg];
        seq = rec[F_SEQ * 8 + sg];
        rseq = rec[F_RSEQ * 8 + sg];
        cli = rec[F_CLI * 8 + sg];
        rcx = rec[F_RCX * 8 + sg];
        props = rec[F_PROPS * 8 + sg];
        txt = rec[F_TEXT * 8 + sg];
        if (!(id & MTB_LEAF)) kbad = true;
        if (!perm && !(txt & MTB_MARKER)) {
          if ((uint64_t)txt + len > text_cap) kbad = true;
          else
            for (uint32_t j = (uint32_t)q; j < len; j += 8)
              t += dg_fmix((((uint64_t)j << 16) | T[txt + j]) + 0x632BE59BD9B4E019ull);
        }
      }
      t += shfl_xor64(t, 1);
      t += shfl_xor64(t, 2);
      t += shfl_xor64(t, 4);
      if (sg < c && q == 0) {
        uint64_t K = 0;
        if (perm) {
          K = 2;
          t = dg_fmix(((uint64_t)txt << 32) | len);
        } else if (txt & MTB_MARKER) {
          K = 1;
          t = dg_fmix(0x4D00000000ull | (txt & ~MTB_MARKER));
        }
        uint64_t Rc = 0;
        if ((int32_t)rseq >= 0) {
          Rc = dg_mix(1, rid((int16_t)(cli >> 16)));
          if (rcx) {
            const uint32_t n = rcx < aux_used ? A[rcx] : 0;
            for (uint32_t i = 0; i < n && rcx + 1 + i < aux_used; i++) Rc += dg_mix(i + 2, rid((int32_t)A[rcx + 1 + i]));
          }
        }
        uint64_t Ph = 0;
        if (props) {
          const uint32_t* ps = (props & MTB_GPROPS) ? pool + (props & ~MTB_GPROPS) : A + (props & ~MTB_PNAN);
          const uint32_t n = ps[0];
          for (uint32_t i = 0; i < n; i++) Ph += dg_mix(dg_mix(i + 1, khash[ps[1 + 2 * i]]), vhash[ps[2 + 2 * i]]);
        }
        uint64_t h = 0;
        h = dg_mix(h, P + ((uint64_t)(sg + 1) << (4 * d)));
        h = dg_mix(h, K);
        h = dg_mix(h, t);
        h = dg_mix(h, len);
        h = dg_mix(h, (int32_t)seq >= MTB_PEND ? 0xFFFFFFFFu : seq);  // unacked: UnassignedSequenceNumber
        h = dg_mix(h, rid((int16_t)(cli & 0xFFFF)));
        h = dg_mix(h, (int32_t)rseq >= MTB_PEND ? 0xFFFFFFFFu : rseq);
        h = dg_mix(h, Rc);
        h = dg_mix(h, Ph);
        acc += dg_fmix(h + (nsegs + (uint64_t)sg + 1) * 0xD6E8FEB86659FD93ull);
      }
      if (__ballot(kbad)) bad = true;
      nsegs += (uint64_t)c;
      __syncthreads();
      if (lane == 0) nxt[d] = c;
      __syncthreads();
      continue;
    }
    if (lane == 0) nxt[d] = k + 1;
    __syncthreads();
    if (d + 1 >= MTB_DG_DEPTH || child >= blk_used || ++entered > blk_used) {
      bad = true;
      break;
    }
    d++;
    enter(child, d);
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) acc += shfl_xor64(acc, m);
  if (lane == 0) {
    uint64_t D = 0;
    uint32_t len = 0;
    if (!bad) {
      len = (uint32_t)B[root].len;
      D = 0x4D544231ull;
      D = dg_mix(D, (uint32_t)s.min_seq);
      D = dg_mix(D, (uint32_t)s.cur_seq);
      D = dg_mix(D, len);
      D = dg_mix(D, nsegs);
      D = dg_mix(D, acc);
    }
    out[3 * doc] = D;
    out[3 * doc + 1] = bad ? 0 : nsegs;
    out[3 * doc + 2] = len;
  }
}

hipError_t mtb_launch_digest(hipStream_t stream, uint32_t ndocs, const DocState* docs, const FBlk* blks,
                             const uint16_t* text, const uint32_t* aux, const uint32_t* pool, const uint64_t* khash,
                             const uint64_t* vhash, uint64_t* out) {
  hipLaunchKernelGGL(mtb_digest_kernel, dim3(ndocs), dim3(64), 0, stream, docs, ndocs, blks, text, aux, pool, khash,
                     vhash, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------- SnapshotV1 extraction
// SnapshotV1.extractSync (snapshotV1.ts:180-312) on the device, one wave per listed document: the leaves in
// tree order, elided (unacked inserts; removedSeq <= minSeq, which includes an unacked removal), coalesced
// (below the MSN and not removed: TextSegment.canAppend + matchProperties, or PermutationSegment.canAppend)
// or kept with their merge info.  The host serializes the result (mtb_host.cpp summarize_items) instead of
// downloading the whole tree.  Per document the output is
//   items : per snapshot segment [flags (EX_META, EX_MARKER | refType+1 << 8), length, text offset
//           (PermutationSegment: its start), props (0; MTB_GPROPS | pool offset; EX_INLINE | word offset of a
//           copied [n, (k, v)*n] set)], and when it keeps its merge info (EX_META) 4 more words [seq, client |
//           removedClientIds[0] << 16, removedSeq, word offset of [n, c1..cn] further removers (MTB_NONE:
//           none)]: 4 or 8 words, read in order
//   text  : the UTF-16 of every item (a coalesced run's pieces back to back)
//   words : inlined per-document property sets and remover lists
// Pass 1 (off == nullptr) counts (item words, text units, words) into cnt[3 k]; pass 2 writes at off[3 k..].
#define EX_META 1u
#define EX_MARKER 2u
#define EX_INLINE 0x40000000u
namespace mtbk {
__device__ __forceinline__ bool ex_props_match(uint32_t a, uint32_t b, const uint32_t* pool, const uint32_t* A,
                                               const Tables& tab) {
  if ((tab.irr_any ? b : (a | b)) & MTB_PNAN) return false;  // NaN !== NaN (a's NaN: irr_value_match)
  if (a == b && !tab.irr_any) return true;
  const uint32_t* pa = a ? ((a & MTB_GPROPS) ? pool + (a & ~MTB_GPROPS) : A + (a & ~MTB_PNAN)) : nullptr;
  const uint32_t* pb = b ? ((b & MTB_GPROPS) ? pool + (b & ~MTB_GPROPS) : A + (b & ~MTB_PNAN)) : nullptr;
  const uint32_t na = pa ? pa[0] : 0, nb = pb ? pb[0] : 0;
  if (na != nb) return false;
  for (uint32_t i = 0; i < na; i++) {
    const uint32_t k = pa[1 + 2 * i];
    bool found = false;
    for (uint32_t q = 0; q < nb; q++)
      if (pb[1 + 2 * q] == k) {
        if (tab.irr_any ? !irr_value_match(tab, k, pa[2 + 2 * i], pb[2 + 2 * q])
                        : tab.val_class[pa[2 + 2 * i]] != tab.val_class[pb[2 + 2 * q]])
          return false;
        found = true;
        break;
      }
    if (!found) return false;
  }
  return true;
}
}  // namespace mtbk
extern "C" __global__ void __launch_bounds__(64)
    mtb_extract_v1_kernel(const DocState* __restrict__ docs, const uint32_t* list, uint32_t n, const FBlk* blks,
                          const uint16_t* text, const uint32_t* aux, const uint32_t* pool, const Tables tab,
                          uint32_t* cnt, const uint64_t* off, uint32_t* items, uint16_t* otext, uint32_t* owords) {
  __shared__ uint32_t ids[MTB_DG_DEPTH][MTB_MAXCH];
  __shared__ int32_t bc[MTB_DG_DEPTH], nxt[MTB_DG_DEPTH];
  __shared__ uint32_t rec[64];
  const uint32_t k = blockIdx.x;
  const int lane = threadIdx.x;
  if (k >= n) return;
  const bool emit = off != nullptr;
  // emit pass: a document the count pass could not trust (MTB_NONE, still in cnt) got no room in the outputs
  // (its offsets are the next document's); the host serializes it from its slices, so write nothing
  if (emit && cnt[3 * k] == MTB_NONE) return;
  const DocState& s = docs[list[k]];
  const FBlk* B = blks + s.blk_base;
  const uint16_t* T = text + s.text_base;
  const uint32_t* A = aux + s.aux_base;
  const bool perm = (s.flags & DSF_PERM) != 0;
  const int minSeq = s.min_seq;
  uint32_t* I = emit ? items + off[3 * k] : nullptr;
  uint16_t* OT = emit ? otext + off[3 * k + 1] : nullptr;
  uint32_t* OW = emit ? owords + off[3 * k + 2] : nullptr;
  uint32_t ni = 0, nt = 0, nw = 0;  // item words, text units, words so far (uniform)
  // the open coalescing candidate (`prev`): its item index, length, last UTF-16 unit, marker, props
  bool open = false;
  uint32_t p_item = 0, p_len = 0, p_props = 0, p_start = 0;
  uint16_t p_last = 0;
  bool p_marker = false;
  // inline a per-document property set (global ones are referenced by pool offset)
  auto props_out = [&](uint32_t h) -> uint32_t {
    if (!h || (h & MTB_GPROPS)) return h;
    h &= ~MTB_PNAN;  // (the host serializes the copy; NaN is JSON null)
    const uint32_t m = 1 + 2 * U(A[h]);
    if (emit)
      for (uint32_t i = (uint32_t)lane; i < m; i += 64) OW[nw + i] = A[h + i];
    const uint32_t o = EX_INLINE | nw;
    nw += m;
    return o;
  };
  auto copy_text = [&](uint32_t src, uint32_t len) {
    if (emit)
      for (uint32_t i = (uint32_t)lane; i < len; i += 64) OT[nt + i] = T[src + i];
    nt += len;
  };
  auto close_prev = [&]() {
    if (open && emit && lane == 0) I[p_item + 1] = p_len;
    open = false;
  };
  int d = 0;
  auto enter = [&](uint32_t b, int dd) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(B + b);
    const uint32_t v = w[lane];
    const uint32_t c = w[FB_HDR];
    rec[lane] = v;
    if (lane < MTB_MAXCH) ids[dd][lane] = v;
    if (lane == 0) {
      bc[dd] = (int32_t)(c > MTB_MAXCH ? MTB_MAXCH : c);
      nxt[dd] = 0;
    }
    __syncthreads();
  };
  // a tree the walk cannot trust (too deep, a child id outside the slice, a cycle: the digest kernel's
  // conditions) reports MTB_NONE and the host serializes the document from its downloaded slices instead
  bool bad = s.err != 0 || s.root >= s.blk_used;
  uint32_t entered = 0;
  if (!bad) enter(s.root, 0);
  while (!bad) {
    const int c = bc[d], kk = nxt[d];
    if (kk >= c) {
      if (d == 0) break;
      d--;
      continue;
    }
    const uint32_t child = ids[d][kk];
    if (!(child & MTB_LEAF)) {
      if (lane == 0) nxt[d] = kk + 1;
      __syncthreads();
      if (d + 1 >= MTB_DG_DEPTH || child >= s.blk_used || ++entered > s.blk_used) {
        bad = true;
        break;
      }
      d++;
      enter(child, d);
      continue;
    }
    // a leaf-level block: its segments in order (uniform decisions, lane-parallel copies)
    for (int j = 0; j < c; j++) {
      const uint32_t len = U(rec[F_LEN * 8 + j]);
      const int seq = (int)U(rec[F_SEQ * 8 + j]);
      const int rseq = (int)U(rec[F_RSEQ * 8 + j]);
      const uint32_t cli = U(rec[F_CLI * 8 + j]);
      const uint32_t rcx = U(rec[F_RCX * 8 + j]);
      const uint32_t props = U(rec[F_PROPS * 8 + j]);
      const uint32_t txt = U(rec[F_TEXT * 8 + j]);
      const bool removed = rseq >= 0;
      if (seq >= MTB_PEND) continue;                                    // unacked insert
      if (removed && (rseq >= MTB_PEND || rseq <= minSeq)) continue;    // removedSeq <= minSeq (-1 unacked)
      const bool marker = !perm && (txt & MTB_MARKER);
      if (seq <= minSeq && !removed) {
        bool append = false;
        if (open) {
          if (perm) {
            append = p_start == MTB_HANDLE_UNALLOC ? txt == MTB_HANDLE_UNALLOC : txt == p_start + p_len;
          } else {
            append = !p_marker && !marker && !(p_len > 0 && p_last == u'\n') && (p_len <= 256 || len <= 256) &&
                     ex_props_match(p_props, props, pool, A, tab);
          }
        }
        if (append) {
          if (!perm) {
            copy_text(txt, len);
            if (len) p_last = U((uint32_t)T[txt + len - 1]);
          }
          p_len += len;
          continue;
        }
        close_prev();
        // a new candidate item (its length is written when it closes)
        const uint32_t po = perm ? 0u : props_out(props);
        if (emit && lane < 4) {
          const uint32_t v = lane == 0 ? (marker ? (EX_MARKER | (((txt & ~MTB_MARKER)) << 8)) : 0u)
                             : lane == 2 ? (perm ? txt : marker ? 0u : nt) : lane == 3 ? po : 0u;
          I[ni + lane] = v;
        }
        open = true;
        p_item = ni;
        ni += 4;
        p_len = len;
        p_props = props;
        p_start = txt;
        p_marker = marker;
        p_last = 0;
        if (!perm && !marker) {
          copy_text(txt, len);
          if (len) p_last = U((uint32_t)T[txt + len - 1]);
        }
        continue;
      }
      // merge info kept: the candidate is emitted first
      close_prev();
      const uint32_t po = perm ? 0u : props_out(props);
      uint32_t ro = MTB_NONE;
      if (removed && rcx) {
        const uint32_t m = 1 + U(A[rcx]);
        if (emit)
          for (uint32_t i = (uint32_t)lane; i < m; i += 64) OW[nw + i] = A[rcx + i];
        ro = nw;
        nw += m;
      }
      const uint32_t toff = nt;
      if (!perm && !marker) copy_text(txt, len);
      if (emit && lane < 8) {
        const uint32_t v = lane == 0 ? (EX_META | (marker ? (EX_MARKER | (((txt & ~MTB_MARKER)) << 8)) : 0u))
                           : lane == 1 ? len : lane == 2 ? (perm ? txt : toff) : lane == 3 ? po
                           : lane == 4 ? (uint32_t)seq : lane == 5 ? cli : lane == 6 ? (uint32_t)rseq : ro;
        I[ni + lane] = v;
      }
      ni += 8;
    }
    __syncthreads();
    if (lane == 0) nxt[d] = c;
    __syncthreads();
  }
  close_prev();
  if (!emit && lane == 0) {
    cnt[3 * k] = bad ? MTB_NONE : ni;
    cnt[3 * k + 1] = nt;
    cnt[3 * k + 2] = nw;
  }
}
hipError_t mtb_launch_extract_v1(hipStream_t stream, const DocState* docs, const uint32_t* list, uint32_t n,
                                 const FBlk* blks, const uint16_t* text, const uint32_t* aux, const uint32_t* pool,
                                 const Tables& tab, uint32_t* cnt, const uint64_t* off, uint32_t* items,
                                 uint16_t* otext, uint32_t* owords) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(mtb_extract_v1_kernel, dim3(n), dim3(64), 0, stream, docs, list, n, blks, text, aux, pool, tab, cnt,
                     off, items, otext, owords);
  return hipGetLastError();
}

// Rewind every document to its post-init state (benchmark / re-replay utility): restores the
// DocState header, the root block and the initial segment's parent; ops and payload stay resident.
extern "C" __global__ void mtb_rewind_kernel(DocState* docs, const DocState* pristine, uint32_t ndocs, uint32_t* segp,
                                             const uint32_t* psegp, FBlk* blks, const FBlk* pblk) {
  // one 64-lane wave per document: lanes copy the DocState header and the 320-byte root block
  const uint32_t i = blockIdx.x;
  const int l = threadIdx.x;
  if (i >= ndocs) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(pristine + i);
  uint32_t* dst = reinterpret_cast<uint32_t*>(docs + i);
  dst[l] = src[l];
  if (l < (int)(sizeof(DocState) / 4 - 64)) dst[64 + l] = src[64 + l];
  const uint64_t bb = pristine[i].blk_base, sb = pristine[i].seg_base;
  const uint32_t* ps = reinterpret_cast<const uint32_t*>(pblk + i);
  uint32_t* bd = reinterpret_cast<uint32_t*>(blks + bb);
  bd[l] = ps[l];
  if (l < 16) bd[64 + l] = ps[64 + l];
  if (pristine[i].seg_used && l == 0) segp[sb] = psegp[i];
}

hipError_t mtb_launch_rewind(hipStream_t stream, uint32_t ndocs, DocState* docs, const DocState* pristine, uint32_t* segp,
                             const uint32_t* psegp, FBlk* blks, const FBlk* pblk) {
  hipLaunchKernelGGL(mtb_rewind_kernel, dim3(ndocs), dim3(64), 0, stream, docs, pristine, ndocs, segp, psegp, blks, pblk);
  return hipGetLastError();
}

// ---------------------------------------------------------------------- batched host<->slice moves
// One launch moves every document's piece instead of one hipMemcpy per document.
// Chunk i: `len[i]` 32-bit words from src + src_off[i] to dst + dst_off[i]; one wave per chunk.
extern "C" __global__ void mtb_move_words_kernel(const uint32_t* src, const uint64_t* src_off, uint32_t* dst,
                                                 const uint64_t* dst_off, const uint32_t* len, uint32_t n) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t* s = src + src_off[i];
  uint32_t* d = dst + dst_off[i];
  for (uint32_t k = threadIdx.x; k < len[i]; k += blockDim.x) d[k] = s[k];
}
extern "C" __global__ void mtb_move_u16_kernel(const uint16_t* src, const uint64_t* src_off, uint16_t* dst,
                                               const uint64_t* dst_off, const uint32_t* len, uint32_t n) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint16_t* s = src + src_off[i];
  uint16_t* d = dst + dst_off[i];
  for (uint32_t k = threadIdx.x; k < len[i]; k += blockDim.x) d[k] = s[k];
}

hipError_t mtb_launch_move_words(hipStream_t stream, const uint32_t* src, const uint64_t* src_off, uint32_t* dst,
                                 const uint64_t* dst_off, const uint32_t* len, uint32_t n) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(mtb_move_words_kernel, dim3(n), dim3(64), 0, stream, src, src_off, dst, dst_off, len, n);
  return hipGetLastError();
}
hipError_t mtb_launch_move_u16(hipStream_t stream, const uint16_t* src, const uint64_t* src_off, uint16_t* dst,
                               const uint64_t* dst_off, const uint32_t* len, uint32_t n) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(mtb_move_u16_kernel, dim3(n), dim3(64), 0, stream, src, src_off, dst, dst_off, len, n);
  return hipGetLastError();
}
#endif  // MTB_TU_HAS(MTB_TU_MISC)
