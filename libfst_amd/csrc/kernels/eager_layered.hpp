// eager_layered.hpp -- batched fst_shortest_path(fst_compose_frozen(chain_i, rhs))
// for lattices that are layered by input position (gfx950 / CDNA4).
//
// Replaces, for one linear-chain lhs per string, the loops of
//   src/ops/compose.zig:64-195       (FIFO BFS: lattice state id = discovery index)
//   src/ops/shortest-path.zig:64-136 (Dijkstra, best final, backtrace)
// and the rhs lookup src/fst.zig:112-136 (arcsByIlabel).
//
// Why a level-synchronous kernel reproduces the sequential reference exactly
// (DESIGN.md §4.1):
//  * With no epsilon moves (rhs has no ilabel-0 arcs, inputs have no label 0),
//    every lattice arc goes from layer k to layer k+1, so BFS level == input
//    position and compose.zig's discovery order is: layer by layer, and inside a
//    layer the order of FIRST occurrence among candidates enumerated as
//    (source id, arc index) -- a stable-dedup prefix sum.
//  * shortestPath's result depends on Dijkstra only through d(X) (the float
//    minimum over in-arcs of d(s) + w, algorithm independent for non-negative
//    weights) and the final back-pointer, which the tie rule
//    (shortest-path.zig:74-84: take iff nd < old, or nd == old and s < prev)
//    makes the lexicographic minimum (s, arc index) over "tight" in-arcs
//    (d(s) + w == d(X)).  In candidate order that is the minimum candidate index
//    among tight candidates.
//  * Best final (shortest-path.zig:88-104): lexmin (total, id) over finite nodes.
//
// Layout: one workgroup owns one string at a time (persistent, atomic work
// counter).  The current layer (s2, dist, span) and the next layer's open-
// addressing hash table live either in LDS (fast tier, <= FCAP tuples per layer)
// or in a per-workgroup HBM slab (overflow tier, capacity chosen at launch).
// Back-pointers of every layer go to a per-workgroup HBM slab that the final
// backtrace walks.
#pragma once

#include "device_common.hpp"

namespace fstamd {

// Pointers to one workgroup's layer tables (LDS or HBM).
struct LayerTables {
  uint32_t* s2[2];
  double* d[2];
  uint32_t* lo;                  // current layer: first matching rhs arc
  uint32_t* cnt;                 // current layer: number of matching rhs arcs
  uint32_t* h_key;               // next layer hash: rhs state (kEmptyKey = free)
  uint32_t* h_first;             // first candidate index that reached the key, then
                                 // 0x80000000 | rank of the tuple in the next layer
  unsigned long long* h_dmin;    // minimum distance (order-preserving bits)
  uint32_t* h_bmin;              // minimum tight candidate index (back-pointer)
  uint32_t* nslot;               // next layer rank -> slot
  uint32_t fcap, hcap, hbits;
  // select, not index: a dynamically indexed pointer array would live in scratch
  __device__ __forceinline__ uint32_t* s2p(uint32_t i) const { return i ? s2[1] : s2[0]; }
  __device__ __forceinline__ double* dp(uint32_t i) const { return i ? d[1] : d[0]; }
};

template <int FCAP, int HCAP>
struct LayerLds {
  uint32_t s2[2][FCAP];
  double d[2][FCAP];
  uint32_t lo[FCAP];
  uint32_t cnt[FCAP];
  uint32_t h_key[HCAP];
  uint32_t h_first[HCAP];
  unsigned long long h_dmin[HCAP];
  uint32_t h_bmin[HCAP];
  uint32_t nslot[FCAP];
};

// Bytes of one workgroup's HBM table slab for the overflow tier.
// Rounded to 256 B: workgroup slabs are carved at blockIdx * this stride, and the
// 64-bit atomics on h_dmin fault on a misaligned address.
__host__ __device__ inline size_t layer_slab_bytes(uint32_t fcap, uint32_t hcap) {
  const size_t raw =
      (size_t)fcap * (2 * 4 + 2 * 8 + 4 + 4 + 4) + (size_t)hcap * (4 + 4 + 8 + 4) + 256;
  return (raw + 255) & ~(size_t)255;
}

__device__ inline LayerTables carve_slab(uint8_t* base, uint32_t fcap, uint32_t hcap) {
  LayerTables t;
  uint8_t* p = base;
  auto take = [&](size_t bytes) {
    uint8_t* r = p;
    p += (bytes + 15) & ~(size_t)15;
    return r;
  };
  t.d[0] = (double*)take((size_t)fcap * 8);
  t.d[1] = (double*)take((size_t)fcap * 8);
  t.h_dmin = (unsigned long long*)take((size_t)hcap * 8);
  t.s2[0] = (uint32_t*)take((size_t)fcap * 4);
  t.s2[1] = (uint32_t*)take((size_t)fcap * 4);
  t.lo = (uint32_t*)take((size_t)fcap * 4);
  t.cnt = (uint32_t*)take((size_t)fcap * 4);
  t.nslot = (uint32_t*)take((size_t)fcap * 4);
  t.h_key = (uint32_t*)take((size_t)hcap * 4);
  t.h_first = (uint32_t*)take((size_t)hcap * 4);
  t.h_bmin = (uint32_t*)take((size_t)hcap * 4);
  t.fcap = fcap;
  t.hcap = hcap;
  t.hbits = __builtin_ctz(hcap);
  return t;
}

__device__ __forceinline__ uint32_t lhash(uint32_t k, uint32_t hbits) {
  return (k * 2654435761u) >> (32 - hbits);
}

// Insert-or-find `k`; returns the slot or kEmptyKey if the probe bound is hit.
__device__ __forceinline__ uint32_t tbl_insert(const LayerTables& T, uint32_t k, bool& created) {
  uint32_t i = lhash(k, T.hbits);
  created = false;
  for (uint32_t probe = 0; probe < T.hcap; ++probe) {
    const uint32_t old = atomicCAS(&T.h_key[i], kEmptyKey, k);
    if (old == kEmptyKey) {
      created = true;
      return i;
    }
    if (old == k) return i;
    i = (i + 1) & (T.hcap - 1);
  }
  return kEmptyKey;
}

__device__ __forceinline__ uint32_t tbl_find(const LayerTables& T, uint32_t k) {
  uint32_t i = lhash(k, T.hbits);
  for (uint32_t probe = 0; probe < T.hcap; ++probe) {
    if (T.h_key[i] == k) return i;
    i = (i + 1) & (T.hcap - 1);
  }
  return (uint32_t)FB(kEmptyKey, T.hcap, 10);  // a key inserted in phase B must be found
}

__device__ __forceinline__ void tbl_clear_slot(const LayerTables& T, uint32_t s) {
  s = (uint32_t)FB(s, T.hcap, 19);
  T.h_key[s] = kEmptyKey;
  T.h_first[s] = kEmptyKey;
  T.h_dmin[s] = kMaxU64;
  T.h_bmin[s] = kEmptyKey;
}

struct LayerShared {
  uint32_t scan[16];
  uint32_t item;
  uint32_t expired;  // watchdog verdict of thread 0 for this item (uniform for all waves)
  unsigned long long t_item;  // when this item started (thread 0's clock): the watchdog
                              // is per string, so every string gets the full limit
  uint32_t nnext;
  uint32_t flag;
  uint32_t bestp;
  unsigned long long best;
};

struct EagerLaunch {
  const uint32_t* items;         // null: item i is string i
  const uint32_t* num_items_dev; // null: use num_items
  uint32_t num_items;
  uint8_t* slab;                 // HBM tier tables (null for the LDS tier)
  uint32_t fcap, hcap;           // HBM tier capacities
  uint2* back_ws;                // [grid * back_cap] {source id, rhs arc}
  uint32_t back_cap;
  unsigned long long wd_ticks;   // wall-clock watchdog (s_memrealtime ticks)
};

__device__ __forceinline__ void write_status(const BatchOutDev& out, uint32_t si, int32_t st,
                                             uint32_t tuples, uint32_t relax) {
  out.status[si] = st;
  if (out.first_status) out.first_status[si] = st;  // the streamed batch's parts (pull tiers)
  out.path_len[si] = 0;
  out.path_off[si] = 0;
  out.final_w[si] = w_zero();
  if (out.work) {
    out.work[2 * si] = tuples;
    out.work[2 * si + 1] = relax;
  }
}

template <int WG, int FCAP, int HCAP, bool kLds>
__global__ void __launch_bounds__(WG)
eager_layered_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                     EagerLaunch lp, BatchOutDev out) {
  __shared__ LayerShared SH;
  LayerTables T;
  if constexpr (kLds) {
    __shared__ LayerLds<FCAP, HCAP> L;
    T.s2[0] = L.s2[0];
    T.s2[1] = L.s2[1];
    T.d[0] = L.d[0];
    T.d[1] = L.d[1];
    T.lo = L.lo;
    T.cnt = L.cnt;
    T.h_key = L.h_key;
    T.h_first = L.h_first;
    T.h_dmin = L.h_dmin;
    T.h_bmin = L.h_bmin;
    T.nslot = L.nslot;
    T.fcap = FCAP;
    T.hcap = HCAP;
    T.hbits = __builtin_ctz(HCAP);
  } else {
    T = carve_slab(lp.slab + (size_t)blockIdx.x * layer_slab_bytes(lp.fcap, lp.hcap), lp.fcap,
                   lp.hcap);
  }
  const uint32_t tid = threadIdx.x;
  uint2* back = lp.back_ws + (size_t)blockIdx.x * lp.back_cap;
  const uint32_t num_items = lp.num_items_dev ? *lp.num_items_dev : lp.num_items;

  for (uint32_t i = tid; i < T.hcap; i += WG) tbl_clear_slot(T, i);

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      SH.item = atomicAdd(next_item, 1u);
      SH.expired = 0;
      SH.t_item = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t item = SH.item;
    if (item >= num_items) break;
    FT(item, 0xFFFFFFFFu, 0, 0);
    const uint32_t si = lp.items ? lp.items[item] : item;
    const uint64_t off = in.offsets[si];
    const uint32_t L = (uint32_t)(in.offsets[si + 1] - off);

    // compose.zig:33-35 / shortest-path.zig:21-24 (n checked after the empty checks)
    if (rhs.start == kNoState || n_best != 1) {
      if (tid == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }

    if (tid == 0) {
      T.s2[0][0] = rhs.start;
      T.d[0][0] = w_one();
    }
    uint32_t cur = 0, n_cur = 1, cur_base = 0;
    uint32_t tuples = 1, relax = 0;
    int32_t fail = kPathOk;
    __syncthreads();

    for (uint32_t k = 0; k < L; ++k) {
      const uint32_t label = in.labels[off + k];
      if (label == kEpsilon) {  // lhs epsilon output: not a layered lattice
        fail = kPathUnsupported;
        break;
      }
      // Each thread owns a contiguous chunk of the layer: candidate order, i.e.
      // (source id, arc index), equals thread order then chunk order.
      const uint32_t E = (n_cur + WG - 1) / WG;
      const uint32_t p0 = min(tid * E, n_cur), p1 = min(p0 + E, n_cur);

      FT(item, si, k, 1);
      // ---- (A) rhs spans (arcsByIlabel) of the chunk ----
      uint32_t tsum = 0;
      for (uint32_t p = p0; p < p1; ++p) {
        uint32_t a, b;
        span_by_ilabel(rhs, T.s2p(cur)[p], label, a, b);
        T.lo[p] = a;
        T.cnt[p] = b - a;
        tsum += b - a;
      }
      if (tid == 0) {
        SH.nnext = 0;
        SH.flag = 0;
      }
      uint32_t ctot;
      const uint32_t cbase = block_excl_scan<WG>(tsum, SH.scan, ctot);
      relax += ctot;

      FT(item, si, k, 2);
      // ---- (B) dedup targets, first occurrence, minimum distance ----
      uint32_t c = cbase;
      for (uint32_t p = p0; p < p1; ++p) {
        const double dp = T.dp(cur)[p];
        const uint32_t a0 = T.lo[p], n = T.cnt[p];
        for (uint32_t j = 0; j < n; ++j, ++c) {
          const ArcRec r = rhs.rec[FB(a0 + j, rhs.num_arcs, 14)];
          const double nd = w_times(dp, w_times(w_one(), r.weight));  // compose.zig:104
          bool created;
          const uint32_t slot = tbl_insert(T, r.next, created);
          if (slot == kEmptyKey) {
            SH.flag = 1;
            continue;
          }
          if (created && atomicAdd(&SH.nnext, 1u) >= T.fcap) SH.flag = 1;
          atomicMin(&T.h_first[slot], c);
          atomicMin(&T.h_dmin[slot], (unsigned long long)okey(nd));
        }
      }
      // Watchdog, per string: no bug may keep a workgroup resident forever (INTERNAL).
      // Thread 0's verdict goes through LDS, so every wave takes the same path.
      if (tid == 0 && (k & 15u) == 0 &&
          __builtin_amdgcn_s_memrealtime() - SH.t_item > lp.wd_ticks)
        SH.expired = 1;
      __syncthreads();
      if (SH.expired) {
        fail = kPathInternal;
        break;
      }
      const uint32_t n_next = SH.nnext;
      if (SH.flag || (uint64_t)cur_base + n_cur + n_next > lp.back_cap) {
        fail = kPathOverflow;
        break;
      }
      if (n_next == 0) {  // nothing reachable beyond this layer: no final state
        n_cur = 0;
        break;
      }

      FT(item, si, k, 3);
      // ---- (C) tight candidates -> back-pointer; count first occurrences ----
      uint32_t nf = 0;
      c = cbase;
      for (uint32_t p = p0; p < p1; ++p) {
        const double dp = T.dp(cur)[p];
        const uint32_t a0 = T.lo[p], n = T.cnt[p];
        for (uint32_t j = 0; j < n; ++j, ++c) {
          const ArcRec r = rhs.rec[a0 + j];
          const double nd = w_times(dp, w_times(w_one(), r.weight));
          const uint32_t slot = tbl_find(T, r.next);
          if (okey(nd) == T.h_dmin[slot]) atomicMin(&T.h_bmin[slot], c);
          if (T.h_first[slot] == c) ++nf;
        }
      }
      uint32_t nftot;
      uint32_t rank = block_excl_scan<WG>(nf, SH.scan, nftot);

      FT(item, si, k, 4);
      // ---- (D) ids of the next layer in first-occurrence order ----
      const uint32_t nxt = cur ^ 1;
      c = cbase;
      for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t a0 = T.lo[p], n = T.cnt[p];
        for (uint32_t j = 0; j < n; ++j, ++c) {
          const uint32_t t = rhs.rec[a0 + j].next;
          const uint32_t slot = tbl_find(T, t);
          if (T.h_first[slot] == c) {
            // the slot's rank replaces its first-candidate index (tag bit 31: candidate
            // indices are < 2^31, so no other candidate can match it any more)
            T.h_first[slot] = 0x80000000u | rank;
            T.nslot[FB(rank, T.fcap, 17)] = slot;
            T.s2p(nxt)[FB(rank, T.fcap, 18)] = t;
            ++rank;
          }
        }
      }
      __syncthreads();

      FT(item, si, k, 5);
      // ---- (E) back-pointer records of the next layer ----
      const uint32_t next_base = cur_base + n_cur;
      c = cbase;
      for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t a0 = T.lo[p], n = T.cnt[p];
        for (uint32_t j = 0; j < n; ++j, ++c) {
          const uint32_t t = rhs.rec[a0 + j].next;
          const uint32_t slot = tbl_find(T, t);
          if (T.h_bmin[slot] == c)
            back[FB(next_base + (T.h_first[slot] & 0x7FFFFFFFu), lp.back_cap, 11)] =
                make_uint2(cur_base + p, a0 + j);
        }
      }
      __syncthreads();

      FT(item, si, k, 6);
      // ---- (F) next-layer distances, clear the used slots ----
      for (uint32_t r = tid; r < n_next; r += WG) {
        const uint32_t slot = T.nslot[FB(r, T.fcap, 15)];
        T.dp(nxt)[r] = from_okey(T.h_dmin[FB(slot, T.hcap, 16)]);
        tbl_clear_slot(T, slot);
      }
      __syncthreads();
      cur = nxt;
      cur_base = next_base;
      n_cur = n_next;
      tuples += n_next;
    }

    if (fail != kPathOk) {
      // Leave the tables clean for the next string.
      __syncthreads();
      for (uint32_t i = tid; i < T.hcap; i += WG) tbl_clear_slot(T, i);
      if (tid == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }

    FT(item, si, L, 7);
    // ---- best final over the last layer (only final(L) is non-Zero on a chain) ----
    if (tid == 0) {
      SH.best = kMaxU64;
      SH.bestp = kEmptyKey;
    }
    __syncthreads();
    for (uint32_t p = tid; p < n_cur; p += WG) {
      const double d = T.dp(cur)[p];
      const double fw2 = rhs.final_w[FB(T.s2p(cur)[p], rhs.num_states, 20)];
      if (!w_is_zero(d) && !w_is_zero(fw2))
        atomicMin(&SH.best, (unsigned long long)okey(w_times(d, w_times(w_one(), fw2))));
    }
    __syncthreads();
    const unsigned long long best = SH.best;
    if (best != kMaxU64) {
      for (uint32_t p = tid; p < n_cur; p += WG) {
        const double d = T.dp(cur)[p];
        const double fw2 = rhs.final_w[FB(T.s2p(cur)[p], rhs.num_states, 20)];
        if (!w_is_zero(d) && !w_is_zero(fw2) &&
            okey(w_times(d, w_times(w_one(), fw2))) == best)
          atomicMin(&SH.bestp, p);
      }
    }
    __syncthreads();

    if (tid == 0) {
      const uint32_t bp = SH.bestp;
      if (n_cur == 0 || best == kMaxU64 || bp == kEmptyKey) {
        write_status(out, si, kPathEmpty, tuples, relax);
      } else {
        const double fw = w_times(w_one(), rhs.final_w[T.s2p(cur)[bp]]);  // compose.zig:73
        const unsigned long long o = reserve_path(out, si, L);
        if (o + L > out.arc_cap) {
          write_status(out, si, kPathOutputFull, tuples, relax);
        } else {
          FT(item, si, L, 8);
          // shortest-path.zig:109-136: walk back-pointers, one layer per hop.
          uint32_t id = cur_base + bp;
          for (uint32_t k = L; k > 0; --k) {
            const uint2 b = back[FB(id, lp.back_cap, 12)];
            const ArcRec r = rhs.rec[FB(b.y, rhs.num_arcs, 13)];
            out.out_il[o + k - 1] = in.labels[off + k - 1];
            out.out_ol[o + k - 1] = r.olabel;
            out.out_w[o + k - 1] = w_times(w_one(), r.weight);
            id = b.x;
          }
          out.status[si] = kPathOk;
          out.path_len[si] = L;
          out.path_off[si] = o;
          out.final_w[si] = fw;
          if (out.work) {
            out.work[2 * si] = tuples;
            out.work[2 * si + 1] = relax;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// LDS tier, v2: same phases and the same results as the generic kernel above, with
// the per-layer latency cut down:
//  * each thread owns <= EMAX = FCAP/WG tuples of a layer; the distance and hash
//    slot of each of their first KMAX candidates stay in registers from phase B to
//    E (no re-reads of rhs arcs, no re-probing of the hash);
//  * the next layer's arcsByIlabel spans are computed while the layer is finished
//    (span loads issued in E, ilabel search in F), so a layer starts with its
//    spans already in LDS.
// Per layer the critical path holds two global round trips (arc records in B,
// ilabels in F) instead of six.
// ---------------------------------------------------------------------------------
template <int WG, int FCAP, int HCAP, int KMAX>
__global__ void __launch_bounds__(WG)
eager_layered_lds_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                         EagerLaunch lp, BatchOutDev out) {
  constexpr int EMAX = FCAP / WG;
  static_assert(FCAP % WG == 0, "FCAP must be a multiple of WG");
  __shared__ LayerShared SH;
  __shared__ LayerLds<FCAP, HCAP> L;
  LayerTables T;
  T.s2[0] = L.s2[0];
  T.s2[1] = L.s2[1];
  T.d[0] = L.d[0];
  T.d[1] = L.d[1];
  T.lo = L.lo;
  T.cnt = L.cnt;
  T.h_key = L.h_key;
  T.h_first = L.h_first;
  T.h_dmin = L.h_dmin;
  T.h_bmin = L.h_bmin;
  T.nslot = L.nslot;
  T.fcap = FCAP;
  T.hcap = HCAP;
  T.hbits = __builtin_ctz(HCAP);
  const uint32_t tid = threadIdx.x;
  uint2* back = lp.back_ws + (size_t)blockIdx.x * lp.back_cap;
  const uint32_t num_items = lp.num_items_dev ? *lp.num_items_dev : lp.num_items;

  for (uint32_t i = tid; i < HCAP; i += WG) tbl_clear_slot(T, i);

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      SH.item = atomicAdd(next_item, 1u);
      SH.expired = 0;
      SH.t_item = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t item = SH.item;
    if (item >= num_items) break;
    const uint32_t si = lp.items ? lp.items[item] : item;
    const uint64_t off = in.offsets[si];
    const uint32_t Lk = (uint32_t)(in.offsets[si + 1] - off);

    if (rhs.start == kNoState || n_best != 1) {  // compose.zig:33-35, shortest-path.zig:21-24
      if (tid == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }
    if (tid == 0) {
      T.s2[0][0] = rhs.start;
      T.d[0][0] = w_one();
      if (Lk > 0) {
        uint32_t a, b;
        span_by_ilabel(rhs, rhs.start, in.labels[off], a, b);
        T.lo[0] = a;
        T.cnt[0] = b - a;
      }
    }
    uint32_t cur = 0, n_cur = 1, cur_base = 0;
    uint32_t tuples = 1, relax = 0;
    int32_t fail = kPathOk;
    __syncthreads();

    for (uint32_t k = 0; k < Lk; ++k) {
      const uint32_t label = in.labels[off + k];
      if (label == kEpsilon) {  // lhs epsilon output: not a layered lattice
        fail = kPathUnsupported;
        break;
      }
      const uint32_t E = (n_cur + WG - 1) / WG;  // <= EMAX because n_cur <= FCAP
      const uint32_t p0 = min(tid * E, n_cur);
      uint32_t lo[EMAX], cnt[EMAX];
      double dd[EMAX];
      uint32_t tsum = 0;
      bool too_long = false;  // > KMAX arcs with one label: HBM tier handles the string
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        const uint32_t p = p0 + e;
        const bool v = (uint32_t)e < E && p < n_cur;
        lo[e] = v ? T.lo[p] : 0u;
        cnt[e] = v ? T.cnt[p] : 0u;
        dd[e] = v ? T.dp(cur)[p] : 0.0;
        too_long |= cnt[e] > (uint32_t)KMAX;
        tsum += cnt[e];
      }
      if (tid == 0) {
        SH.nnext = 0;
        SH.flag = 0;
      }
      uint32_t ctot;
      const uint32_t cbase = block_excl_scan<WG>(tsum, SH.scan, ctot);
      relax += ctot;
      if (too_long) SH.flag = 1;  // after the scan's barriers: the reset above is done

      // ---- (B) dedup targets, first occurrence, minimum distance ----
      double rnd[EMAX][KMAX];
      uint32_t rslot[EMAX][KMAX];
      uint32_t c = cbase;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        const double dp = dd[e];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          rslot[e][j] = kEmptyKey;
          rnd[e][j] = 0.0;
          if ((uint32_t)j < cnt[e]) {
            const ArcRec r = rhs.rec[FB(lo[e] + j, rhs.num_arcs, 24)];
            const double nd = w_times(dp, w_times(w_one(), r.weight));  // compose.zig:104
            bool created;
            const uint32_t slot = tbl_insert(T, r.next, created);
            if (slot == kEmptyKey) {
              SH.flag = 1;
            } else {
              if (created && atomicAdd(&SH.nnext, 1u) >= (uint32_t)FCAP) SH.flag = 1;
              atomicMin(&T.h_first[slot], c + j);
              atomicMin(&T.h_dmin[slot], (unsigned long long)okey(nd));
            }
            rslot[e][j] = slot;
            rnd[e][j] = nd;
          }
        }
        c += cnt[e];
      }
      if (tid == 0 && (k & 15u) == 0 &&
          __builtin_amdgcn_s_memrealtime() - SH.t_item > lp.wd_ticks)
        SH.expired = 1;  // per-string watchdog, as in eager_layered_kernel
      __syncthreads();
      if (SH.expired) {
        fail = kPathInternal;
        break;
      }
      const uint32_t n_next = SH.nnext;
      if (SH.flag || (uint64_t)cur_base + n_cur + n_next > lp.back_cap) {
        fail = kPathOverflow;
        break;
      }
      if (n_next == 0) {
        n_cur = 0;
        break;
      }

      // ---- (C) tight candidates -> back-pointer; count first occurrences ----
      uint32_t nf = 0;
      c = cbase;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if ((uint32_t)j < cnt[e]) {
            const uint32_t slot = rslot[e][j];
            if (okey(rnd[e][j]) == T.h_dmin[slot]) atomicMin(&T.h_bmin[slot], c + j);
            if (T.h_first[slot] == c + j) ++nf;
          }
        }
        c += cnt[e];
      }
      uint32_t nftot;
      uint32_t rank = block_excl_scan<WG>(nf, SH.scan, nftot);

      // ---- (D) ids of the next layer in first-occurrence order ----
      const uint32_t nxt = cur ^ 1;
      c = cbase;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if ((uint32_t)j < cnt[e]) {
            const uint32_t slot = rslot[e][j];
            if (T.h_first[slot] == c + j) {
              T.h_first[slot] = 0x80000000u | rank;
              T.nslot[rank] = slot;
              T.s2p(nxt)[rank] = T.h_key[slot];
              ++rank;
            }
          }
        }
        c += cnt[e];
      }
      __syncthreads();

      // ---- (E) back-pointer records; start loading the next layer's spans ----
      const uint32_t next_base = cur_base + n_cur;
      c = cbase;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if ((uint32_t)j < cnt[e]) {
            const uint32_t slot = rslot[e][j];
            if (T.h_bmin[slot] == c + j)
              back[FB(next_base + (T.h_first[slot] & 0x7FFFFFFFu), lp.back_cap, 21)] =
                  make_uint2(cur_base + p0 + e, lo[e] + j);
          }
        }
        c += cnt[e];
      }
      const bool more = k + 1 < Lk;
      const uint32_t next_label = more ? in.labels[off + k + 1] : 0u;
      uint2 sp[EMAX];
#pragma unroll
      for (int i = 0; i < EMAX; ++i) {
        const uint32_t r = tid + i * WG;
        sp[i] = (more && r < n_next) ? rhs.span[T.s2p(nxt)[r]] : make_uint2(0, 0);
      }
      __syncthreads();

      // ---- (F) next-layer distances, clear used slots, next-layer spans ----
#pragma unroll
      for (int i = 0; i < EMAX; ++i) {
        const uint32_t r = tid + i * WG;
        if (r < n_next) {
          const uint32_t slot = T.nslot[r];
          T.dp(nxt)[r] = from_okey(T.h_dmin[slot]);
          tbl_clear_slot(T, slot);
          if (more) {
            // Fst.arcsByIlabel over [sp.x, sp.x + sp.y) (src/fst.zig:112-136)
            const uint32_t o = sp[i].x, n = sp[i].y;
            uint32_t a, b;
            if (n <= 8) {
              uint32_t cl = 0, ch = 0;
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                const uint32_t x = (uint32_t)q < n ? rhs.il[o + q] : 0xFFFFFFFFu;
                cl += ((uint32_t)q < n && x < next_label) ? 1u : 0u;
                ch += ((uint32_t)q < n && x <= next_label) ? 1u : 0u;
              }
              a = o + cl;
              b = o + ch;
            } else {
              span_by_ilabel(rhs, T.s2p(nxt)[r], next_label, a, b);
            }
            T.lo[r] = a;
            T.cnt[r] = b - a;
          }
        }
      }
      __syncthreads();
      cur = nxt;
      cur_base = next_base;
      n_cur = n_next;
      tuples += n_next;
    }

    if (fail != kPathOk) {
      __syncthreads();
      for (uint32_t i = tid; i < HCAP; i += WG) tbl_clear_slot(T, i);
      if (tid == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }

    // ---- best final over the last layer (shortest-path.zig:88-104) ----
    if (tid == 0) {
      SH.best = kMaxU64;
      SH.bestp = kEmptyKey;
    }
    __syncthreads();
    unsigned long long mykey = kMaxU64;
    uint32_t myp = kEmptyKey;
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      const uint32_t p = tid + i * WG;
      if (p < n_cur) {
        const double d = T.dp(cur)[p];
        const double fw2 = rhs.final_w[FB(T.s2p(cur)[p], rhs.num_states, 20)];
        if (!w_is_zero(d) && !w_is_zero(fw2)) {
          const unsigned long long kk = okey(w_times(d, w_times(w_one(), fw2)));
          if (kk < mykey) {
            mykey = kk;
            myp = p;
          }
        }
      }
    }
    if (mykey != kMaxU64) atomicMin(&SH.best, mykey);
    __syncthreads();
    const unsigned long long best = SH.best;
    if (best != kMaxU64 && mykey == best) atomicMin(&SH.bestp, myp);
    __syncthreads();

    if (tid == 0) {
      const uint32_t bp = SH.bestp;
      if (n_cur == 0 || best == kMaxU64 || bp == kEmptyKey) {
        write_status(out, si, kPathEmpty, tuples, relax);
      } else {
        const double fw = w_times(w_one(), rhs.final_w[T.s2p(cur)[bp]]);  // compose.zig:73
        const unsigned long long o = reserve_path(out, si, Lk);
        if (o + Lk > out.arc_cap) {
          write_status(out, si, kPathOutputFull, tuples, relax);
        } else {
          uint32_t id = cur_base + bp;  // shortest-path.zig:109-136
          for (uint32_t k = Lk; k > 0; --k) {
            const uint2 b = back[FB(id, lp.back_cap, 22)];
            const ArcRec r = rhs.rec[FB(b.y, rhs.num_arcs, 23)];
            out.out_il[o + k - 1] = in.labels[off + k - 1];
            out.out_ol[o + k - 1] = r.olabel;
            out.out_w[o + k - 1] = w_times(w_one(), r.weight);
            id = b.x;
          }
          out.status[si] = kPathOk;
          out.path_len[si] = Lk;
          out.path_off[si] = o;
          out.final_w[si] = fw;
          if (out.work) {
            out.work[2 * si] = tuples;
            out.work[2 * si + 1] = relax;
          }
        }
      }
    }
  }
}

// Appends every string whose status is `code` to a device list (retry tier input).
[[maybe_unused]] static __global__ void collect_status_kernel(const int32_t* status, uint32_t num, int32_t code,
                                      uint32_t* list, uint32_t* count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < num && status[i] == code) list[atomicAdd(count, 1u)] = i;
}

}  // namespace fstamd
