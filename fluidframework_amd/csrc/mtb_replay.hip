// MI355X (gfx950) batched merge-tree replay kernel.
//
// One 64-lane wavefront owns one document and applies that document's sequenced ops in order,
// exactly as the reference observer `Client.applyMsg` would (packages/dds/merge-tree/src/client.ts:858).
// Control flow is wave-uniform (every lane walks the same tree path); the lanes parallelise the
// per-op inner loops: the <=8 children of a block, the concatenated window lists of those children,
// scour decisions, list/segment rebuilds and text copies.  No MFMA: nothing here is a contraction.
//
// Differences from the reference data structures (results are identical):
//  * PartialSequenceLengths (partialLengths.ts:239) is replaced by one flat window list per block.
//    A block's length in the (refSeq R, client C) perspective is
//        cachedLength - sum_{e in list, e.seq > R} w(e)
//    where w(e) = e.delta for MAIN entries of other clients and for OVERLAP entries of C.  This is the
//    same quantity getPartialLength (partialLengths.ts:698) returns and the sum of the leaf
//    visibilities (mergeTree.ts:916-1004) - the oracle verifies that identity on every query.
//  * The recursive insertingWalk (mergeTree.ts:1740) runs iteratively with an explicit path; all walks
//    of one op share an LDS cache of the children lengths (they use the same (R, C)).
//  * Length/list bookkeeping is propagated incrementally along the recorded path instead of the
//    reference's combine/update rebuilds; split/pack blocks rebuild their list from their children.
//  * The zamboni LRU heap (collections/heap.ts) lives in LDS while it fits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtb.h"
#include "mtb_device.h"

namespace mtbk {

#define MTB_LDS_HEAP 256
#define MTB_NOKEY ((int32_t)0x80000000)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// Cross-lane hand-off inside the single wave that owns a document.  A wavefront's vector-memory and
// LDS instructions are performed in program order for the whole wave, so a wavefront-scope fence
// (no instruction; it only stops the compiler from moving memory operations across it) is enough
// to make one lane's store visible to another lane's later load of the same document state.
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

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
// sum over lanes 0..7
__device__ __forceinline__ int csum8(int v) { return rl(cscan8(v), 7); }
// number of set bits of m below this lane
__device__ __forceinline__ uint32_t rank_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int first_set(unsigned long long m) { return __ffsll((long long)m) - 1; }

struct Scratch {  // LDS, one per wave
  // per-op child-info cache, one slot per tree depth (all walks of one op share (R, C))
  uint32_t cb[MTB_MAXDEPTH];                 // block cached in the slot (MTB_NONE: empty)
  int32_t ccount[MTB_MAXDEPTH];
  int32_t cscour[MTB_MAXDEPTH];
  uint32_t cid[MTB_MAXDEPTH][MTB_MAXCH];
  int32_t clen[MTB_MAXDEPTH][MTB_MAXCH];
  int32_t cseq[MTB_MAXDEPTH][MTB_MAXCH];
  int32_t corr[MTB_MAXCH];                   // list-scan accumulators
  // walk / nodeMap stacks
  uint32_t path[MTB_MAXDEPTH];
  int32_t pp[MTB_MAXDEPTH];                  // remaining position at each level of the last walk
  int32_t sidx[MTB_MAXDEPTH];
  int32_t acc[MTB_MAXDEPTH];
  // scour / pack / props scratch
  uint32_t hold[64];
  uint32_t pk[64];
  uint32_t pv[64];
  Lru heap[MTB_LDS_HEAP];                    // LRU heap while it fits (index 0 unused)
};

struct Eng {
  DocState* ds;
  Seg* seg;
  Blk* blk;
  WEnt* lst;
  uint16_t* txt;
  Lru* heap;
  uint32_t* aux;
  uint32_t* fre;
  const mtb_op* ops;
  Tables T;
  Scratch* sh;
  int lane;
  // uniform document state (mirrors DocState)
  int minSeq, curSeq;
  uint32_t root;
  bool newMode;
  uint32_t seg_used, blk_used, free_top, list_used, text_used, heap_cnt, aux_used;
  int err;
  uint64_t n_mod, ops_applied, text_bytes;
  uint32_t memo_old, memo_new;  // per-op annotate memo (old props -> new props)
  bool heap_lds;                // LRU heap lives in LDS (spills to the global slice when it outgrows it)
  int walk_depth;               // depth of the leaf-level block reached by the last walk (-1: none)
  bool struct_changed;          // a block split / root growth happened since the last walk started

  // ------------------------------------------------------------------ errors / allocation
  __device__ __forceinline__ void fail(int code) {
    if (!err) err = code;
  }
  __device__ __forceinline__ uint32_t alloc_seg() {
    if (seg_used >= ds->seg_cap) { fail(DERR_CAP_SEG); return 0; }
    return seg_used++;
  }
  __device__ __forceinline__ uint32_t alloc_blk() {
    uint32_t b;
    if (free_top > 0) {
      free_top--;
      b = fre[free_top];
    } else {
      if (blk_used >= ds->blk_cap) { fail(DERR_CAP_BLK); return 0; }
      b = blk_used++;
    }
    Blk& B = blk[b];
    if (lane < MTB_MAXCH) B.child[lane] = MTB_NONE;
    B.parent = MTB_NONE;
    B.len = 0;
    B.loff = 0;
    B.lcnt = 0;
    B.lcap = 0;
    B.count = 0;
    B.index = 0;
    B.scour = -1;
    B.lseq = MTB_NOKEY;
    B.lck = 0;
    wsync();
    return b;
  }
  __device__ __forceinline__ void free_blk(uint32_t b) {
    fre[free_top] = b;
    free_top++;
  }
  __device__ __forceinline__ uint32_t alloc_aux(uint32_t n) {
    if (aux_used + n > ds->aux_cap) { fail(DERR_CAP_AUX); return 1; }
    uint32_t o = aux_used;
    aux_used += n;
    return o;
  }
  __device__ __forceinline__ void cache_clear() {
    if (lane < MTB_MAXDEPTH) sh->cb[lane] = MTB_NONE;
    wsync();
  }

  // ------------------------------------------------------------------ visibility
  __device__ __forceinline__ bool rc_has(const Seg& s, int C) const {
    if (s.rc0 == C) return true;
    if (s.rcx) {
      uint32_t n = aux[s.rcx];
      for (uint32_t i = 0; i < n; i++)
        if ((int)aux[s.rcx + 1 + i] == C) return true;
    }
    return false;
  }
  // localNetLength (mergeTree.ts:613-634)
  __device__ __forceinline__ int local_len(const Seg& s) const {
    if (s.rseq >= 0) {
      if (!newMode) return s.rseq > minSeq ? 0 : MTB_UNDEF;
      return 0;
    }
    return s.len;
  }
  // nodeLength for a leaf in a remote perspective (mergeTree.ts:935-1001)
  __device__ __forceinline__ int seg_vis(const Seg& s, int R, int C) const {
    const bool removed = s.rseq >= 0;
    if (newMode) {
      if (removed) {
        if (s.rseq <= minSeq) return MTB_UNDEF;
        if (s.rseq <= R || rc_has(s, C)) return 0;
      }
      return (s.seq <= R || s.client == C) ? s.len : 0;
    }
    if (removed && s.rseq <= R) return MTB_UNDEF;
    if (s.client == C || s.seq <= R) {
      if (removed) return rc_has(s, C) ? 0 : s.len;
      return s.len;
    }
    if (removed) return MTB_UNDEF;
    return 0;
  }

  // Children of block b (tree depth d) in the (R, C) perspective: lane j < count receives the child id,
  // its length (UNDEF allowed) and, for leaves, the segment's seq.  Results are cached in LDS slot d for
  // the rest of the op.
  __device__ __forceinline__ int child_info(uint32_t b, int d, int R, int C, uint32_t& cid, int& clen, int& cseq) {
    if (sh->cb[d] == b) {
      const int count = sh->ccount[d];
      cid = lane < count ? sh->cid[d][lane] : MTB_NONE;
      clen = lane < count ? sh->clen[d][lane] : 0;
      cseq = lane < count ? sh->cseq[d][lane] : 0;
      return count;
    }
    const Blk& B = blk[b];
    const int count = B.count;
    const int scour = B.scour;
    cid = MTB_NONE;
    clen = 0;
    cseq = 0;
    uint32_t loff = 0, lcnt = 0;
    if (lane < count) {
      cid = B.child[lane];
      if (cid & MTB_LEAF) {
        const Seg s = seg[cid & ~MTB_LEAF];
        clen = seg_vis(s, R, C);
        cseq = s.seq;
      } else {
        const Blk& cb = blk[cid];
        clen = cb.len;
        loff = cb.loff;
        lcnt = cb.lcnt;
      }
    }
    // concatenated scan of the children's window lists, accumulated per child in LDS
    const int incl = cscan8((int)lcnt);
    const int total = rl(incl, 7);
    if (total > 0) {
      const int excl = incl - (int)lcnt;
      if (lane < MTB_MAXCH) sh->corr[lane] = 0;
      int pre[MTB_MAXCH], off[MTB_MAXCH];
#pragma unroll
      for (int k = 0; k < MTB_MAXCH; k++) {
        pre[k] = rl(excl, k);
        off[k] = rl((int)loff, k);
      }
      wsync();
      for (int t = lane; t < total; t += 64) {
        int j = 0;
#pragma unroll
        for (int k = 1; k < MTB_MAXCH; k++)
          if (k < count && pre[k] <= t) j = k;
        int base = 0;
#pragma unroll
        for (int k = 0; k < MTB_MAXCH; k++)
          if (k == j) base = off[k] + (t - pre[k]);
        const WEnt e = lst[base];
        if (e.seq > R) {
          const int c = e.ck & 0xFFFF;
          const int kind = e.ck >> 16;
          if ((kind == WK_MAIN && c != C) || (kind == WK_OVERLAP && c == C)) atomicAdd(&sh->corr[j], e.delta);
        }
      }
      wsync();
      if (lane < count && !(cid & MTB_LEAF)) clen -= sh->corr[lane];
    }
    if (lane < count) {
      sh->cid[d][lane] = cid;
      sh->clen[d][lane] = clen;
      sh->cseq[d][lane] = cseq;
    }
    sh->ccount[d] = count;
    sh->cscour[d] = scour;
    sh->cb[d] = b;
    wsync();
    return count;
  }

  // ------------------------------------------------------------------ window lists
  __device__ __forceinline__ uint32_t list_alloc(uint32_t cap) {
    if (list_used + cap > ds->list_cap) { fail(DERR_CAP_LIST); return 0; }
    uint32_t o = list_used;
    list_used += cap;
    return o;
  }
  // Add `dlen` to the cachedLength of the `n` blocks sh->path[0..n) and append (seq, client, kind,
  // delta) to their window lists.  One lane per block; blocks whose list is full are re-allocated
  // afterwards, one at a time.
  __device__ __forceinline__ void path_update(int n, int dlen, int seqv, int client, int kind, int delta) {
    const int ck = (client & 0xFFFF) | (kind << 16);
    bool need = false;
    if (lane < n) {
      const uint32_t b = sh->path[lane];
      Blk& B = blk[b];
      const uint32_t cnt = B.lcnt, cap = B.lcap, off = B.loff;
      const int ls = B.lseq, lk = B.lck;
      if (dlen) B.len = B.len + dlen;
      if (cnt > 0 && ls == seqv && lk == ck) {
        lst[off + cnt - 1].delta += delta;  // same (seq, client, kind) as the last entry (GROUP members)
      } else if (cnt < cap) {
        WEnt e;
        e.seq = seqv;
        e.ck = ck;
        e.delta = delta;
        e.pad = 0;
        lst[off + cnt] = e;
        B.lcnt = cnt + 1;
        B.lseq = seqv;
        B.lck = ck;
      } else {
        need = true;
      }
    }
    unsigned long long m = __ballot(need);
    wsync();
    while (m) {
      const int i = first_set(m);
      m &= m - 1;
      const uint32_t b = sh->path[i];
      list_grow(b, 1);
      if (err) return;
      Blk& B = blk[b];
      WEnt e;
      e.seq = seqv;
      e.ck = ck;
      e.delta = delta;
      e.pad = 0;
      const uint32_t cnt = B.lcnt;
      lst[B.loff + cnt] = e;
      B.lcnt = cnt + 1;
      B.lseq = seqv;
      B.lck = ck;
      wsync();
    }
  }
  // Re-allocate block b's list with room for `extra` more entries, dropping entries <= minSeq.
  __device__ __forceinline__ void list_grow(uint32_t b, uint32_t extra) {
    Blk& B = blk[b];
    const uint32_t cnt = B.lcnt, off = B.loff;
    uint32_t live = 0;
    for (uint32_t base = 0; base < cnt; base += 64) {
      const uint32_t i = base + lane;
      const bool keep = i < cnt && lst[off + i].seq > minSeq;
      live += __popcll(__ballot(keep));
    }
    uint32_t cap = live + extra;
    cap = cap < 8 ? 8 : cap * 2;
    const uint32_t no = list_alloc(cap);
    if (err) return;
    uint32_t w = 0;
    for (uint32_t base = 0; base < cnt; base += 64) {
      const uint32_t i = base + lane;
      WEnt e;
      bool keep = false;
      if (i < cnt) {
        e = lst[off + i];
        keep = e.seq > minSeq;
      }
      const unsigned long long m = __ballot(keep);
      const uint32_t rank = rank_below(m);
      if (keep) lst[no + w + rank] = e;
      w += __popcll(m);
    }
    B.loff = no;
    B.lcnt = w;
    B.lcap = cap;
    B.lseq = MTB_NOKEY;
    wsync();
  }
  // Rebuild block b's window list from its children (after split / pack / root growth) and its
  // cachedLength (blockUpdate, mergeTree.ts:2392).
  __device__ __forceinline__ void rebuild(uint32_t b) {
    Blk& B = blk[b];
    const int count = B.count;
    int nent = 0, olen = 0;
    uint32_t cid = MTB_NONE;
    Seg s;
    uint32_t coff = 0, ccnt = 0;
    if (lane < count) {
      cid = B.child[lane];
      if (cid & MTB_LEAF) {
        s = seg[cid & ~MTB_LEAF];
        const int l = local_len(s);
        olen = l == MTB_UNDEF ? 0 : l;
        if (s.seq > minSeq) nent++;
        if (s.rseq >= 0 && s.rseq > minSeq) {
          nent++;
          if (s.rcx) nent += (int)aux[s.rcx];
        }
      } else {
        const Blk& cb = blk[cid];
        olen = cb.len;
        coff = cb.loff;
        ccnt = cb.lcnt;
      }
    }
    const int totalLen = csum8(olen);
    const int cincl = cscan8((int)ccnt);
    const int cexcl = cincl - (int)ccnt;
    const int ctotal = rl(cincl, 7);
    int pre[MTB_MAXCH], off[MTB_MAXCH];
#pragma unroll
    for (int k = 0; k < MTB_MAXCH; k++) {
      pre[k] = rl(cexcl, k);
      off[k] = rl((int)coff, k);
    }
    int live_from_children = 0;
    for (int base = 0; base < ctotal; base += 64) {
      const int t = base + lane;
      bool keep = false;
      if (t < ctotal) {
        int j = 0;
#pragma unroll
        for (int k = 1; k < MTB_MAXCH; k++)
          if (k < count && pre[k] <= t) j = k;
        int p = 0;
#pragma unroll
        for (int k = 0; k < MTB_MAXCH; k++)
          if (k == j) p = off[k] + (t - pre[k]);
        keep = lst[p].seq > minSeq;
      }
      live_from_children += __popcll(__ballot(keep));
    }
    const int segEnt = csum8(nent);
    const int total = segEnt + live_from_children;
    uint32_t cap = (uint32_t)total;
    cap = cap < 8 ? 8 : cap + cap / 2 + 4;
    const uint32_t no = list_alloc(cap);
    if (err) return;
    const int sincl = cscan8(nent);
    int w = sincl - nent;
    if (lane < count && (cid & MTB_LEAF)) {
      WEnt e;
      e.pad = 0;
      if (s.seq > minSeq) {
        e.seq = s.seq;
        e.ck = (s.client & 0xFFFF) | (WK_MAIN << 16);
        e.delta = s.len;
        lst[no + w++] = e;
      }
      if (s.rseq >= 0 && s.rseq > minSeq) {
        e.seq = s.rseq;
        e.ck = (s.rc0 & 0xFFFF) | (WK_MAIN << 16);
        e.delta = -s.len;
        lst[no + w++] = e;
        if (s.rcx) {
          const uint32_t n = aux[s.rcx];
          for (uint32_t i = 0; i < n; i++) {
            e.ck = ((int)aux[s.rcx + 1 + i] & 0xFFFF) | (WK_OVERLAP << 16);
            e.delta = s.len;
            lst[no + w++] = e;
          }
        }
      }
    }
    uint32_t wpos = (uint32_t)segEnt;
    for (int base = 0; base < ctotal; base += 64) {
      const int t = base + lane;
      bool keep = false;
      WEnt e;
      if (t < ctotal) {
        int j = 0;
#pragma unroll
        for (int k = 1; k < MTB_MAXCH; k++)
          if (k < count && pre[k] <= t) j = k;
        int p = 0;
#pragma unroll
        for (int k = 0; k < MTB_MAXCH; k++)
          if (k == j) p = off[k] + (t - pre[k]);
        e = lst[p];
        keep = e.seq > minSeq;
      }
      const unsigned long long m = __ballot(keep);
      const uint32_t rank = rank_below(m);
      if (keep) lst[no + wpos + rank] = e;
      wpos += __popcll(m);
    }
    B.loff = no;
    B.lcnt = (uint32_t)total;
    B.lcap = cap;
    B.len = totalLen;
    B.lseq = MTB_NOKEY;
    wsync();
  }

  // ------------------------------------------------------------------ tree primitives
  __device__ __forceinline__ void set_parent(uint32_t node, uint32_t b, int idx) {
    if (node & MTB_LEAF) {
      seg[node & ~MTB_LEAF].parent = b;
    } else {
      blk[node].parent = b;
      blk[node].index = (uint8_t)idx;
    }
  }
  // Insert `node` at child index k of block b (insertingWalk shift, mergeTree.ts:1831-1837).  `d` is the
  // depth of b in the current walk (its cache slot holds the children), or -1.
  __device__ __forceinline__ void insert_child(uint32_t b, int k, uint32_t node, int d) {
    Blk& B = blk[b];
    int count;
    uint32_t c = MTB_NONE;
    if (d >= 0 && sh->cb[d] == b) {
      count = sh->ccount[d];
      if (lane < count) c = sh->cid[d][lane];
      sh->cb[d] = MTB_NONE;  // children change
    } else {
      count = B.count;
      if (lane < count) c = B.child[lane];
    }
    wsync();
    if (lane < count && lane >= k) {
      B.child[lane + 1] = c;
      if (!(c & MTB_LEAF)) blk[c].index = (uint8_t)(lane + 1);
    }
    B.child[k] = node;
    set_parent(node, b, k);
    B.count = (uint8_t)(count + 1);
    wsync();
  }
  // split (mergeTree.ts:1858-1871): children 4..7 move to a new block.
  __device__ __forceinline__ uint32_t split_block(uint32_t b) {
    struct_changed = true;
    const uint32_t nb = alloc_blk();
    if (err) return 0;
    Blk& B = blk[b];
    Blk& N = blk[nb];
    const int half = MTB_MAXCH / 2;
    if (lane < half) {
      const uint32_t c = B.child[half + lane];
      N.child[lane] = c;
      set_parent(c, nb, lane);
      B.child[half + lane] = MTB_NONE;
    }
    B.count = (uint8_t)half;
    N.count = (uint8_t)half;
    N.parent = B.parent;
    wsync();
    rebuild(b);
    rebuild(nb);
    return nb;
  }
  // updateRoot (mergeTree.ts:1268-1277)
  __device__ __forceinline__ void grow_root(uint32_t left, uint32_t right) {
    const uint32_t r = alloc_blk();
    if (err) return;
    Blk& R = blk[r];
    R.child[0] = left;
    R.child[1] = right;
    R.count = 2;
    blk[left].parent = r;
    blk[left].index = 0;
    blk[right].parent = r;
    blk[right].index = 1;
    wsync();
    rebuild(r);
    root = r;
  }
  // After inserting into block sh->path[d] (the leaf-level block), split every full block on the path.
  __device__ __forceinline__ void fix_overflow(int d) {
    int level = d;
    uint32_t cur = sh->path[level];
    while (!err && blk[cur].count >= MTB_MAXCH) {
      const uint32_t nb = split_block(cur);
      if (err) return;
      if (level == 0) {
        grow_root(cur, nb);
        break;
      }
      const uint32_t p = sh->path[level - 1];
      insert_child(p, blk[cur].index + 1, nb, -1);
      cur = p;
      level--;
    }
    if (struct_changed) cache_clear();
  }

  // BaseSegment.splitAt (mergeTreeNodes.ts:481-510) + TextSegment.createSplitSegmentAt
  __device__ __forceinline__ uint32_t split_seg(uint32_t sid, int at) {
    const uint32_t r = alloc_seg();
    if (err) return 0;
    Seg t = seg[sid];
    t.len -= at;
    t.text += (uint32_t)at;
    seg[r] = t;
    seg[sid].len = at;
    n_mod += 2;
    wsync();
    return r;
  }

  // ------------------------------------------------------------------ insertingWalk
  // mode 0: ensureIntervalBoundary (seq = TreeMaintenance, leaf = splitLeafSegment)
  // mode 1: blockInsert of candidate `cand` (seq S).  Returns false if the candidate was not placed.
  // `resume`: start at the leaf-level block reached by the previous walk (same (R, C) and position, no
  // block split since): internal-level decisions of both walks are identical (blocks tie-break the same
  // way in both modes and a segment split changes no block length).
  __device__ __forceinline__ bool walk(int pos, int R, int C, int S, bool insertMode, uint32_t cand, int candLen,
                                       bool resume = false) {
    uint32_t b = root;
    int p = pos;
    int d = 0;
    if (resume && walk_depth >= 0 && !struct_changed) {
      d = walk_depth;
      b = sh->path[d];
      p = sh->pp[d];
    }
    walk_depth = -1;
    struct_changed = false;
    while (true) {
      if (d >= MTB_MAXDEPTH) { fail(DERR_DEPTH); return false; }
      sh->path[d] = b;
      sh->pp[d] = p;
      uint32_t cid;
      int clen, cseq;
      const int count = child_info(b, d, R, C, cid, clen, cseq);
      const int def = (lane < count && clen > 0) ? clen : 0;
      const int incl = cscan8(def);
      const int pj = p - (incl - def);
      const bool isBlk = lane < count && !(cid & MTB_LEAF);
      const bool tie = isBlk || (insertMode && pj == 0 && S > cseq);
      const bool qual = lane < count && clen != MTB_UNDEF && (pj < clen || (pj == clen && tie));
      const unsigned long long m = __ballot(qual);
      if (m) {
        const int j = first_set(m);
        const uint32_t cj = rlu(cid, j);
        const int pjj = rl(pj, j);
        if (!(cj & MTB_LEAF)) {
          b = cj;
          p = pjj;
          d++;
          continue;
        }
        walk_depth = d;
        if (insertMode) {
          insert_child(b, j, cand | MTB_LEAF, d);
        } else {
          if (pjj <= 0) return true;  // splitLeafSegment: pos 0 -> no change
          const uint32_t sid = cj & ~MTB_LEAF;
          if (seg[sid].text & MTB_MARKER) return true;  // markers never split
          const uint32_t r = split_seg(sid, pjj);
          if (err) return false;
          insert_child(b, j + 1, r | MTB_LEAF, d);
          fix_overflow(d);
          return true;
        }
      } else {
        const int total = rl(incl, 7);
        if (p - total == 0) walk_depth = d;
        if (p - total != 0 || !insertMode) return !insertMode;
        insert_child(b, count, cand | MTB_LEAF, d);
      }
      // candidate inserted into block b at depth d: propagate its length and window entry
      cache_clear();
      path_update(d + 1, candLen, S, C, WK_MAIN, candLen);
      fix_overflow(d);
      return true;
    }
  }

  // ------------------------------------------------------------------ LRU heap (collections/heap.ts)
  __device__ __forceinline__ Lru hget(uint32_t k) const { return heap_lds ? sh->heap[k] : heap[k]; }
  __device__ __forceinline__ void hset(uint32_t k, Lru v) {
    if (heap_lds) sh->heap[k] = v;
    else heap[k] = v;
  }
  __device__ __forceinline__ void heap_spill() {  // LDS -> global slice
    for (uint32_t i = 1 + lane; i <= heap_cnt; i += 64) heap[i] = sh->heap[i];
    heap_lds = false;
    wsync();
  }
  __device__ __forceinline__ void heap_add(uint32_t s, int maxSeq) {
    if (heap_cnt + 1 >= ds->heap_cap) { fail(DERR_CAP_HEAP); return; }
    if (heap_lds && heap_cnt + 1 >= MTB_LDS_HEAP) heap_spill();
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
    // fixDown with the last element placed at the root
    while ((k << 1) <= count) {
      uint32_t j = k << 1;
      Lru a = hget(j);
      if (j < count) {
        const Lru bb = hget(j + 1);
        if (a.maxSeq - bb.maxSeq > 0) {
          j++;
          a = bb;
        }
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
      blk[b].scour = 1;
      heap_add(sid, seqv);
      return true;
    }
    return false;
  }

  // ------------------------------------------------------------------ properties
  __device__ __forceinline__ const uint32_t* props_ptr(uint32_t h) const {
    return (h & MTB_GPROPS) ? (T.pool + (h & ~MTB_GPROPS)) : (aux + h);
  }
  // matchProperties (properties.ts:71-96) on interned property sets
  __device__ __forceinline__ bool props_match(uint32_t a, uint32_t b) const {
    if (a == b) return true;
    const uint32_t* pa = a ? props_ptr(a) : nullptr;
    const uint32_t* pb = b ? props_ptr(b) : nullptr;
    const uint32_t na = pa ? pa[0] : 0, nb = pb ? pb[0] : 0;
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
      const uint32_t k = pa[1 + 2 * i];
      bool found = false;
      for (uint32_t q = 0; q < nb; q++) {
        if (pb[1 + 2 * q] == k) {
          found = true;
          if (T.val_class[pa[2 + 2 * i]] != T.val_class[pb[2 + 2 * q]]) return false;
          break;
        }
      }
      if (!found) return false;
    }
    return true;
  }
  // PropertiesManager.addProperties for a sequenced remote op (segmentPropertiesManager.ts:60-157).
  // The key/value list is staged in LDS; all lanes run the (short) edit loop uniformly.
  __device__ __forceinline__ uint32_t props_apply(uint32_t old, uint32_t opId, bool rewrite) {
    if (old == memo_old && memo_new) return memo_new;
    const uint32_t* op = T.pool + T.pidx[2 * opId];
    const uint32_t nop = op[0];
    uint32_t n = 0;
    if (old) {
      const uint32_t* po = props_ptr(old);
      n = po[0];
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
            keep = v != MTB_NONE && !T.val_falsy[v];
          }
        }
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
      const uint32_t v = op[2 + 2 * q];
      int at = -1;
      for (uint32_t i = 0; i < n; i++)
        if (sh->pk[i] == k) at = (int)i;
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
        const uint32_t rank = T.key_rank[k];
        uint32_t ins = n;
        if (rank != MTB_NONE) {
          ins = 0;
          while (ins < n) {
            const uint32_t r2 = T.key_rank[sh->pk[ins]];
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
    const uint32_t h = alloc_aux(1 + 2 * n);
    if (err) return 0;
    aux[h] = n;
    for (uint32_t i = lane; i < n; i += 64) {
      aux[h + 1 + 2 * i] = sh->pk[i];
      aux[h + 2 + 2 * i] = sh->pv[i];
    }
    wsync();
    memo_old = old;
    memo_new = h;
    return h;
  }

  // ------------------------------------------------------------------ nodeMap (remove / annotate)
  // markRangeRemoved (mergeTree.ts:1960-2052) when `remove`, else annotateRange (mergeTree.ts:1895-1958).
  // Emulates depthFirstNodeWalk (mergeTreeNodeWalk.ts:35) with an explicit stack; block post-actions
  // (blockUpdateLength) become one flush of the accumulated observer-length delta per block.
  __device__ __forceinline__ void node_map(int start, int end, int R, int C, int S, bool remove, uint32_t opId,
                                           bool rewrite) {
    if (end == start) return;
    int pos = 0;
    int d = 0;
    bool exiting = false;
    auto enter = [&](uint32_t b) {
      uint32_t cid;
      int clen, cseq;
      child_info(b, d, R, C, cid, clen, cseq);
      sh->path[d] = b;
      sh->sidx[d] = 0;
      sh->acc[d] = 0;
      wsync();
    };
    enter(root);
    while (!err) {
      const int idx = sh->sidx[d];
      if (exiting || idx >= sh->ccount[d]) {
        // post-order: flush this block's accumulated observer-length delta
        const int a = sh->acc[d];
        if (a != 0) {
          const uint32_t b = sh->path[d];
          const uint32_t keep = sh->path[0];
          sh->path[0] = b;
          wsync();
          path_update(1, a, S, C, WK_MAIN, a);
          sh->path[0] = keep;
          if (d > 0) sh->acc[d - 1] += a;
          wsync();
        }
        if (d == 0) break;
        d--;
        continue;
      }
      sh->sidx[d] = idx + 1;
      wsync();
      if (end <= pos) {
        exiting = true;
        continue;
      }
      const int len = sh->clen[d][idx];
      if (len == MTB_UNDEF || len == 0) continue;
      const int nextPos = pos + len;
      if (start >= nextPos) {
        pos = nextPos;
        continue;
      }
      const uint32_t c = sh->cid[d][idx];
      if (!(c & MTB_LEAF)) {
        if (d + 1 >= MTB_MAXDEPTH) { fail(DERR_DEPTH); return; }
        d++;
        enter(c);
        continue;
      }
      const uint32_t sid = c & ~MTB_LEAF;
      const Seg s = seg[sid];
      n_mod += 1;
      if (remove) {
        if (s.rseq >= 0) {
          // overlapping remove: append C to removedClientIds (copy-on-write list) and add an OVERLAP
          // window entry on every ancestor (no observer-length change)
          const uint32_t oldn = s.rcx ? aux[s.rcx] : 0;
          const uint32_t h = alloc_aux(oldn + 2);
          if (err) return;
          for (uint32_t i = lane; i < oldn; i += 64) aux[h + 1 + i] = aux[s.rcx + 1 + i];
          aux[h] = oldn + 1;
          aux[h + 1 + oldn] = (uint32_t)C;
          seg[sid].rcx = h;
          wsync();
          path_update(d + 1, 0, s.rseq, C, WK_OVERLAP, s.len);
        } else {
          const int before = local_len(s);
          seg[sid].rseq = S;
          seg[sid].rc0 = (int16_t)C;
          seg[sid].rcx = 0;
          Seg s2 = s;
          s2.rseq = S;
          const int after = local_len(s2);
          const int dl = (after == MTB_UNDEF ? 0 : after) - (before == MTB_UNDEF ? 0 : before);
          sh->acc[d] += dl;
          wsync();
        }
      } else {
        const uint32_t np = props_apply(s.props, opId, rewrite);
        if (err) return;
        seg[sid].props = np;
      }
      if (lru_add(sid, sh->path[d], sh->cscour[d], S)) sh->cscour[d] = 1;
      wsync();
      pos = nextPos;
    }
  }

  // ------------------------------------------------------------------ zamboni (zamboni.ts)
  __device__ __forceinline__ void copy_text(uint32_t dst, uint32_t src, uint32_t n) {
    for (uint32_t i = lane; i < n; i += 64) txt[dst + i] = txt[src + i];
  }
  // scourNode (zamboni.ts:122-193) for block `node`: kept children are appended to sh->hold[nh..].
  // Every child record (and the last UTF-16 unit of every text) is fetched at once, lane-parallel;
  // the sequential keep/drop/append decisions then run on registers (shuffles), and the text of each
  // run of appended segments is written with one parallel copy (TextSegment.append, textSegment.ts:84).
  __device__ __forceinline__ int scour(uint32_t node, int nh) {
    const Blk& B = blk[node];
    const int count = B.count;
    uint32_t c = MTB_NONE;
    Seg s;
    s.len = 0;
    s.seq = 0;
    s.rseq = -1;
    s.props = 0;
    s.text = 0;
    uint16_t last = 0;
    int kind = 0;  // 0 hold+reset, 1 drop (tombstone below MSN), 2 acked text/marker (may append)
    if (lane < count) {
      c = B.child[lane];
      if (c & MTB_LEAF) {
        s = seg[c & ~MTB_LEAF];
        if (s.rseq >= 0) kind = s.rseq > minSeq ? 0 : 1;
        else if (s.seq <= minSeq) kind = 2;
        if (kind == 2 && !(s.text & MTB_MARKER) && s.len > 0) last = txt[s.text + s.len - 1];
      }
    }
    // sequential decisions (uniform), values pulled from lane k by shuffles
    int prev = -1;            // lane index of the current append target
    int prevLen = 0;          // its (growing) length
    uint16_t prevLast = 0;    // its (growing) last unit
    bool prevMarker = false;
    uint32_t prevProps = 0;
    int target = -1;          // per lane: lane it was appended into (-1 kept / dropped)
    int newLen = 0;           // per lane: final length if it is an append target
    for (int k = 0; k < count; k++) {
      const int kk = rl(kind, k);
      const int klen = rl(s.len, k);
      const uint32_t ktext = rlu(s.text, k);
      const uint32_t kprops = rlu(s.props, k);
      const uint16_t klast = (uint16_t)rl((int)last, k);
      if (kk == 1) {
        prev = -1;
        continue;
      }
      if (kk == 2) {
        const bool kmarker = (ktext & MTB_MARKER) != 0;
        bool ok = false;
        if (prev >= 0 && klen > 0 && !prevMarker && !kmarker && prevLast != (uint16_t)'\n' &&
            (prevLen <= 256 || klen <= 256))
          ok = props_match(prevProps, kprops);
        if (ok) {
          if (lane == k) target = prev;
          prevLen += klen;
          prevLast = klast;
          if (lane == prev) newLen = prevLen;
        } else {
          prev = klen > 0 ? k : -1;
          prevLen = klen;
          prevLast = klast;
          prevMarker = kmarker;
          prevProps = kprops;
          if (lane == k) newLen = klen;
        }
        continue;
      }
      prev = -1;
    }
    // targets that received appends: build their new text
    const bool isTarget = lane < count && kind == 2 && target < 0 && newLen != s.len;
    unsigned long long tm = __ballot(isTarget);
    while (tm) {
      const int t = first_set(tm);
      tm &= tm - 1;
      // members of the run: t and every lane whose target is t, in order
      const unsigned long long run = __ballot(lane == t || target == t);
      const uint32_t ttext = rlu(s.text, t);
      const int tlen = rl(s.len, t);
      const int total = rl(newLen, t);
      // contiguous in the arena already?
      bool contiguous = true;
      {
        uint32_t expect = ttext + (uint32_t)tlen;
        unsigned long long r = run & ~(1ull << t);
        while (r) {
          const int q = first_set(r);
          r &= r - 1;
          const uint32_t qt = rlu(s.text, q);
          const int ql = rl(s.len, q);
          if (qt != expect) contiguous = false;
          expect = qt + (uint32_t)ql;
        }
      }
      uint32_t dst = ttext;
      if (!contiguous) {
        const bool atEnd = ttext + (uint32_t)tlen == text_used;
        const uint32_t need = atEnd ? (uint32_t)(total - tlen) : (uint32_t)total;
        if (text_used + need > ds->text_cap) { fail(DERR_CAP_TEXT); return nh; }
        uint32_t w = text_used;
        if (!atEnd) {
          copy_text(w, ttext, (uint32_t)tlen);
          dst = w;
          w += (uint32_t)tlen;
        } else {
          w = ttext + (uint32_t)tlen;
        }
        unsigned long long r = run & ~(1ull << t);
        while (r) {
          const int q = first_set(r);
          r &= r - 1;
          const uint32_t qt = rlu(s.text, q);
          const int ql = rl(s.len, q);
          copy_text(w, qt, (uint32_t)ql);
          w += (uint32_t)ql;
        }
        text_used += need;
      }
      if (lane == t) {
        seg[c & ~MTB_LEAF].text = dst;
        seg[c & ~MTB_LEAF].len = total;
      }
      wsync();
    }
    // unlink dropped / appended segments, compact the kept ones into hold[]
    const bool keep = lane < count && kind != 1 && target < 0;
    if (lane < count && !keep) seg[c & ~MTB_LEAF].parent = MTB_NONE;
    const unsigned long long km = __ballot(keep);
    if (keep) sh->hold[nh + rank_below(km)] = c;
    wsync();
    return nh + __popcll(km);
  }
  // packParent (zamboni.ts:63-120), iterative over the recursion to the grandparent
  __device__ __forceinline__ void pack_parent(uint32_t parent) {
    while (!err) {
      Blk& P = blk[parent];
      const int pc = P.count;
      int nh = 0;
      for (int i = 0; i < pc; i++) {
        const uint32_t cb = P.child[i];
        nh = scour(cb, nh);
        free_blk(cb);
      }
      wsync();
      int cc = 0;
      if (nh > 0) {
        cc = nh / (MTB_MAXCH / 2);
        if (cc > MTB_MAXCH - 1) cc = MTB_MAXCH - 1;
        if (cc < 1) cc = 1;
        const int base = nh / cc;
        int rem = nh % cc;
        int taken = 0;
        for (int q = 0; q < cc; q++) {
          int n = base;
          if (rem > 0) {
            n++;
            rem--;
          }
          const uint32_t nb = alloc_blk();
          if (err) return;
          Blk& N = blk[nb];
          if (lane < n) {
            const uint32_t c = sh->hold[taken + lane];
            N.child[lane] = c;
            set_parent(c, nb, lane);
          }
          N.count = (uint8_t)n;
          N.parent = parent;
          N.index = (uint8_t)q;
          P.child[q] = nb;
          wsync();
          taken += n;
          rebuild(nb);
        }
      }
      if (lane < MTB_MAXCH && lane >= cc) P.child[lane] = MTB_NONE;
      P.count = (uint8_t)cc;
      wsync();
      if (cc < MTB_MAXCH / 2 && P.parent != MTB_NONE) {
        parent = P.parent;
        continue;
      }
      break;
    }
  }
  // zamboniSegments (zamboni.ts:19-60)
  __device__ __forceinline__ void zamboni() {
    for (int i = 0; i < 2 && !err; i++) {
      if (heap_cnt == 0) break;
      const Lru top = hget(1);
      if (top.maxSeq > minSeq) break;
      heap_get();
      const uint32_t b = seg[top.seg].parent;
      if (b != MTB_NONE && blk[b].scour != 0) {
        const int count = blk[b].count;
        const int nh = scour(b, 0);
        Blk& B = blk[b];
        B.scour = 0;
        if (nh < count) {
          if (lane < nh) {
            const uint32_t c = sh->hold[lane];
            B.child[lane] = c;
            if (!(c & MTB_LEAF)) blk[c].index = (uint8_t)lane;
          }
          if (lane < MTB_MAXCH && lane >= nh) B.child[lane] = MTB_NONE;
          B.count = (uint8_t)nh;
          wsync();
          if (nh < MTB_MAXCH / 2 && B.parent != MTB_NONE) pack_parent(B.parent);
        }
        wsync();
      }
    }
  }

  // ------------------------------------------------------------------ ops
  __device__ __forceinline__ void set_min_seq(int msn) {  // mergeTree.ts:1025-1044
    if (!(msn <= curSeq) || !(minSeq <= msn)) { fail(DERR_ASSERT_MSN); return; }
    if (msn > minSeq) {
      minSeq = msn;
      zamboni();
    }
  }
  __device__ __forceinline__ void apply(const mtb_op& o) {
    memo_old = MTB_NONE;
    memo_new = 0;
    const int S = (int)o.seq, R = (int)o.ref_seq, C = (int)o.client;
    switch (o.type) {
      case MTB_OP_INSERT: {
        ops_applied++;
        cache_clear();
        walk((int)o.pos1, R, C, -2, false, 0, 0);  // ensureIntervalBoundary
        if (err) return;
        const bool marker = (o.flags & MTB_F_MARKER) != 0;
        const int len = marker ? 1 : (int)o.pos2;
        if (len > 0) {
          const uint32_t sid = alloc_seg();
          if (err) return;
          Seg s;
          s.len = len;
          s.seq = S;
          s.rseq = -1;
          s.props = o.props ? (MTB_GPROPS | T.pidx[2 * o.props + 1]) : 0;
          s.text = marker ? (MTB_MARKER | (o.pos2 == 0xFFFFFFFFu ? 0u : o.pos2 + 1)) : o.payload;
          s.parent = MTB_NONE;
          s.rcx = 0;
          s.client = (int16_t)C;
          s.rc0 = -1;
          seg[sid] = s;
          wsync();
          n_mod += 1;
          text_bytes += marker ? 0 : 2ull * (uint64_t)len;
          if (!walk((int)o.pos1, R, C, S, true, sid, len, true)) {
            fail(DERR_INSERT);
            return;
          }
          if (S > minSeq) {  // saveIfLocal (mergeTree.ts:1617-1637)
            const uint32_t pb = seg[sid].parent;
            lru_add(sid, pb, blk[pb].scour, S);
          }
        }
        zamboni();
        break;
      }
      case MTB_OP_REMOVE:
      case MTB_OP_ANNOTATE: {
        ops_applied++;
        cache_clear();
        walk((int)o.pos1, R, C, -2, false, 0, 0);
        walk((int)o.pos2, R, C, -2, false, 0, 0);
        if (err) return;
        node_map((int)o.pos1, (int)o.pos2, R, C, S, o.type == MTB_OP_REMOVE, o.props, (o.flags & MTB_F_REWRITE) != 0);
        zamboni();
        break;
      }
      case MTB_OP_ACK:
        zamboni();
        break;
      default:
        break;
    }
    if (err) return;
    if (o.flags & MTB_F_LAST) {  // updateSeqNumbers (client.ts:877-887)
      if (!(curSeq <= S)) { fail(DERR_ASSERT_SEQ); return; }
      curSeq = S;
      if (!((int)o.msn <= S)) { fail(DERR_ASSERT_MSN); return; }
      set_min_seq((int)o.msn);
    }
  }
};

}  // namespace mtbk

using namespace mtbk;

#ifndef MTB_WAVES_PER_SIMD
#define MTB_WAVES_PER_SIMD 3
#endif
extern "C" __global__ void __launch_bounds__(64, MTB_WAVES_PER_SIMD) mtb_replay_kernel(DocState* __restrict__ docs, uint32_t ndocs,
                                                                   const mtb_op* ops, Seg* segs, Blk* blks, WEnt* lists,
                                                                   uint16_t* text, Lru* heap, uint32_t* aux,
                                                                   uint32_t* freel, Tables tables) {
  __shared__ Scratch sh;
  const uint32_t doc = blockIdx.x;
  if (doc >= ndocs) return;
  DocState* ds = &docs[doc];
  Eng e;
  e.ds = ds;
  e.seg = segs + ds->seg_base;
  e.blk = blks + ds->blk_base;
  e.lst = lists + ds->list_base;
  e.txt = text + ds->text_base;
  e.heap = heap + ds->heap_base;
  e.aux = aux + ds->aux_base;
  e.fre = freel + ds->free_base;
  e.ops = ops + ds->op_base;
  e.T = tables;
  e.sh = &sh;
  e.lane = lane_id();
  e.minSeq = ds->min_seq;
  e.curSeq = ds->cur_seq;
  e.root = ds->root;
  e.newMode = ds->new_mode != 0;
  e.seg_used = ds->seg_used;
  e.blk_used = ds->blk_used;
  e.free_top = ds->free_top;
  e.list_used = ds->list_used;
  e.text_used = ds->text_used;
  e.heap_cnt = ds->heap_cnt;
  e.aux_used = ds->aux_used;
  e.err = ds->err;
  e.n_mod = ds->n_mod;
  e.ops_applied = ds->ops_applied;
  e.text_bytes = ds->text_bytes;
  uint32_t k = ds->op_next;
  const uint32_t n = ds->n_ops;
  e.walk_depth = -1;
  e.struct_changed = false;
  // bring the LRU heap into LDS when it fits
  e.heap_lds = e.heap_cnt + 1 < MTB_LDS_HEAP;
  if (e.heap_lds)
    for (uint32_t i = 1 + e.lane; i <= e.heap_cnt; i += 64) sh.heap[i] = e.heap[i];
  __syncthreads();
  if (k < n) {
    mtb_op cur = e.ops[k];
    for (; k < n && !e.err; k++) {
      const mtb_op nxt = e.ops[k + 1 < n ? k + 1 : k];  // prefetch the next record
      e.apply(cur);
      cur = nxt;
    }
  }
  if (e.heap_lds)
    for (uint32_t i = 1 + e.lane; i <= e.heap_cnt; i += 64) e.heap[i] = sh.heap[i];
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
    ds->n_mod = e.n_mod;
    ds->ops_applied = e.ops_applied;
    ds->text_bytes = e.text_bytes;
    if (e.err && !ds->err) {
      ds->err = e.err;
      ds->err_op = k;
    }
    ds->op_next = e.err ? k : n;
  }
}

hipError_t mtb_launch_replay(hipStream_t stream, uint32_t ndocs, DocState* docs, const mtb_op* ops, Seg* segs, Blk* blks,
                             WEnt* lists, uint16_t* text, Lru* heap, uint32_t* aux, uint32_t* freel, Tables tables) {
  hipLaunchKernelGGL(mtb_replay_kernel, dim3(ndocs), dim3(64), 0, stream, docs, ndocs, ops, segs, blks, lists, text, heap,
                     aux, freel, tables);
  return hipGetLastError();
}

// Rewind every document to its post-init state (benchmark / re-replay utility): restores the
// DocState header, the root block and the initial segment; ops and payload stay resident.
extern "C" __global__ void mtb_rewind_kernel(DocState* docs, const DocState* pristine, uint32_t ndocs, Seg* segs,
                                             const Seg* pseg, Blk* blks, const Blk* pblk) {
  // one 64-lane wave per document: lanes copy the 256-byte header, the root block and the initial segment
  const uint32_t i = blockIdx.x;
  const int l = threadIdx.x;
  if (i >= ndocs) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(pristine + i);
  uint32_t* dst = reinterpret_cast<uint32_t*>(docs + i);
  dst[l] = src[l];
  const uint64_t bb = pristine[i].blk_base, sb = pristine[i].seg_base;
  if (l < 16) reinterpret_cast<uint32_t*>(blks + bb)[l] = reinterpret_cast<const uint32_t*>(pblk + i)[l];
  if (pristine[i].seg_used && l < 8) reinterpret_cast<uint32_t*>(segs + sb)[l] = reinterpret_cast<const uint32_t*>(pseg + i)[l];
}

hipError_t mtb_launch_rewind(hipStream_t stream, uint32_t ndocs, DocState* docs, const DocState* pristine, Seg* segs,
                             const Seg* pseg, Blk* blks, const Blk* pblk) {
  hipLaunchKernelGGL(mtb_rewind_kernel, dim3(ndocs), dim3(64), 0, stream, docs, pristine, ndocs, segs, pseg, blks, pblk);
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
