// eager_bfs.hpp -- general eager compose (+ shortestPath) on the GPU (gfx950 / CDNA4).
//
// Covers what the layered kernels cannot: rhs epsilon arcs, label-0 (epsilon) inputs,
// general lhs FSTs (single-call C ABI), and the lattice output of fst_compose_frozen.
//
// compose (src/ops/compose.zig:29-198) as a level-synchronous BFS.  The reference pops
// tuples from a FIFO queue in id order and gives a newly seen target the next id.  A
// FIFO BFS visits tuples level by level, so level l+1 holds exactly the tuples first
// seen while expanding level l, numbered in the order of their first candidate, where
// candidates are enumerated by (source id, compose.zig's 4 phases, arc order).  Per
// level: count candidates per tuple (scan -> arc offsets), write every candidate as an
// arc and insert its target into a per-string hash (atomicMin keeps the first candidate
// of a new key), rank the first occurrences (scan), then resolve every arc's target id.
// The arcs of a tuple are contiguous and in phase order, so arc ai of tuple s is the
// ai-th arc compose.zig appends to s.
//
// shortestPath (src/ops/shortest-path.zig:18-139) for non-negative weights without the
// heap.  Its dist is the least fixpoint of d(X) = min over in-arcs fl(d(s) + w) (every
// Dijkstra distance is a path sum and no path sum is smaller; fl(d + w) >= d keeps the
// float recurrence monotone), computed here by Gauss-Seidel sweeps over the BFS levels
// until nothing changes.  Relaxations also reach settled nodes (:70-84), so the final
// back-pointer of X is the tight in-arc (fl(d(s) + w) == d(X)) with the smallest
// (s, arc index) -- later ties replace only for a smaller s, and a later arc of the
// same s never does -- which holds for the start too.  Best final: lexmin (total, id)
// (:88-104).  The backtrace (:109-122) is bounded by the node count: a back-pointer
// cycle (zero-weight ties, where the reference would not terminate) reports CYCLE.
#pragma once

#include "device_common.hpp"
#include "eager_layered.hpp"  // write_status, LayerShared-style helpers

namespace fstamd {

struct BfsWs {
  uint8_t* slab;            // [grid] per-workgroup slabs of `stride` bytes
  size_t stride;
  uint32_t ncap, acap, hcap, lcap;  // nodes, arcs, hash slots (pow2), levels
  uint32_t* hdr;            // [grid * 8]: n_nodes, n_arcs, n_levels, status, item
  unsigned long long wd_ticks;
  uint32_t lattice_only;    // 1: stop after compose (fst_compose_frozen)
};

struct BfsTables {
  unsigned long long* hkey;  // [hcap] tuple key, ~0 = free
  uint32_t* hval;            // [hcap] id (< 2^31) or 0x80000000 | first candidate arc
  unsigned long long* nkey;  // [ncap] key of node id
  uint32_t* aoff;            // [ncap + 1] first arc of node id
  uint32_t* lvl;             // [lcap + 2] first node id of each BFS level
  unsigned long long* nd;    // [ncap] okey of the distance
  unsigned long long* nback; // [ncap] (source id << 32) | arc index, ~0 = none
  double* nfin;              // [ncap] final weight of node id
  uint32_t* anext;           // [acap]
  uint32_t* ail;
  uint32_t* aol;
  double* aw;
  uint32_t* cslot;           // [acap] hash slot of the arc's target (level scratch)
};

__host__ __device__ inline size_t bfs_slab_bytes(uint32_t ncap, uint32_t acap, uint32_t hcap,
                                                 uint32_t lcap) {
  auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return r((size_t)hcap * 8) + r((size_t)hcap * 4) + r((size_t)ncap * 8) +
         r(((size_t)ncap + 1) * 4) + r(((size_t)lcap + 2) * 4) + r((size_t)ncap * 8) +
         r((size_t)ncap * 8) + r((size_t)ncap * 8) + r((size_t)acap * 4) * 3 +
         r((size_t)acap * 8) + r((size_t)acap * 4);
}

__device__ inline BfsTables bfs_carve(uint8_t* p, uint32_t ncap, uint32_t acap, uint32_t hcap,
                                      uint32_t lcap) {
  auto take = [&](size_t b) {
    uint8_t* q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  BfsTables t;
  t.hkey = (unsigned long long*)take((size_t)hcap * 8);
  t.hval = (uint32_t*)take((size_t)hcap * 4);
  t.nkey = (unsigned long long*)take((size_t)ncap * 8);
  t.aoff = (uint32_t*)take(((size_t)ncap + 1) * 4);
  t.lvl = (uint32_t*)take(((size_t)lcap + 2) * 4);
  t.nd = (unsigned long long*)take((size_t)ncap * 8);
  t.nback = (unsigned long long*)take((size_t)ncap * 8);
  t.nfin = (double*)take((size_t)ncap * 8);
  t.anext = (uint32_t*)take((size_t)acap * 4);
  t.ail = (uint32_t*)take((size_t)acap * 4);
  t.aol = (uint32_t*)take((size_t)acap * 4);
  t.aw = (double*)take((size_t)acap * 8);
  t.cslot = (uint32_t*)take((size_t)acap * 4);
  return t;
}

// Product tuple (s1, s2, filter) <-> 64-bit key; s1 < 2^30.
__device__ __forceinline__ unsigned long long bfs_key(uint32_t s1, uint32_t s2, uint32_t f) {
  return ((unsigned long long)s2 << 32) | ((unsigned long long)s1 << 2) | f;
}
__device__ __forceinline__ uint32_t bfs_hash(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// Coherent reads of words other threads update with atomics (bypass the CU's L1).
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The lhs of one item: a linear chain acceptor (batch API, compileString semantics:
// label k on arc k -> k+1, weight One, final(L) = One) or a general MutableFst (CSR).
template <bool kGraph>
struct BfsLhs {
  const uint32_t* labels;
  uint32_t L;
  GraphInput g;
  __device__ uint32_t start() const { return kGraph ? g.start : 0u; }
  __device__ uint32_t deg(uint32_t s1) const {
    if constexpr (kGraph) return g.state_off[s1 + 1] - g.state_off[s1];
    return s1 < L ? 1u : 0u;
  }
  __device__ void arc(uint32_t s1, uint32_t i, uint32_t& il, uint32_t& ol, double& w,
                      uint32_t& nx) const {
    if constexpr (kGraph) {
      const uint32_t a = g.state_off[s1] + i;
      il = g.arc_il[a];
      ol = g.arc_ol[a];
      w = g.arc_w[a];
      nx = g.arc_next[a];
    } else {
      il = ol = labels[s1];
      w = w_one();
      nx = s1 + 1;
    }
  }
  __device__ double final_w(uint32_t s1) const {
    if constexpr (kGraph) return g.final_w[s1];
    return s1 == L ? w_one() : w_zero();
  }
};

// The candidates of tuple (s1, s2, f) in compose.zig's order (phases :95-121, :124-134,
// :136-157, :160-194); emit(il, ol, w, target key).
template <bool kGraph, class Emit>
__device__ __forceinline__ void bfs_expand(const RhsView& rhs, const BfsLhs<kGraph>& lhs,
                                           uint32_t s1, uint32_t s2, uint32_t f, Emit&& emit) {
  const uint32_t deg = lhs.deg(s1);
  for (uint32_t i = 0; i < deg; ++i) {  // phase 1: non-epsilon lhs output x rhs ilabel
    uint32_t il, ol, nx;
    double w;
    lhs.arc(s1, i, il, ol, w, nx);
    if (ol == kEpsilon) continue;
    uint32_t lo, hi;
    span_by_ilabel(rhs, s2, ol, lo, hi);
    for (uint32_t a = lo; a < hi; ++a) {
      const ArcRec r = rhs.rec[a];
      emit(il, r.olabel, w_times(w, r.weight), bfs_key(nx, r.next, 0));
    }
  }
  if (f != 1) {  // phase 2: lhs epsilon output alone
    const uint32_t nf = f == 0 ? 2u : f;
    for (uint32_t i = 0; i < deg; ++i) {
      uint32_t il, ol, nx;
      double w;
      lhs.arc(s1, i, il, ol, w, nx);
      if (ol != kEpsilon) continue;
      emit(il, kEpsilon, w, bfs_key(nx, s2, nf));
    }
  }
  uint32_t elo, ehi;
  span_by_ilabel(rhs, s2, kEpsilon, elo, ehi);
  if (f != 2) {  // phase 3: rhs epsilon input alone
    const uint32_t nf = f == 0 ? 1u : f;
    for (uint32_t a = elo; a < ehi; ++a) {
      const ArcRec r = rhs.rec[a];
      emit(kEpsilon, r.olabel, r.weight, bfs_key(s1, r.next, nf));
    }
  }
  if (f == 0 && ehi > elo) {  // phase 4: both epsilon
    for (uint32_t i = 0; i < deg; ++i) {
      uint32_t il, ol, nx;
      double w;
      lhs.arc(s1, i, il, ol, w, nx);
      if (ol != kEpsilon) continue;
      for (uint32_t a = elo; a < ehi; ++a) {
        const ArcRec r = rhs.rec[a];
        emit(il, r.olabel, w_times(w, r.weight), bfs_key(nx, r.next, 0));
      }
    }
  }
}

struct BfsShared {
  uint32_t scan[16];
  uint32_t item;
  uint32_t expired;
  uint32_t flag;
  uint32_t changed;
  unsigned long long best;
  uint32_t bestid;
};

// shortestPath on a lattice held in BfsTables (aoff / anext / aw / ail / aol / nfin, BFS
// levels in lvl[0..n_levels]); the whole workgroup calls it; thread 0 writes the result.
template <int WG>
__device__ void bfs_shortest_path(const BfsTables& T, uint32_t n_nodes, uint32_t n_arcs,
                                  uint32_t n_levels, uint32_t start, const BatchOutDev& out,
                                  uint32_t si, BfsShared& SH, unsigned long long deadline) {
  const uint32_t tid = threadIdx.x;
  int32_t fail = kPathOk;
  // ---- shortestPath: Gauss-Seidel sweeps to the least fixpoint ----
  for (uint32_t i = tid; i < n_nodes; i += WG) {
    T.nd[i] = i == start ? okey(w_one()) : okey(w_zero());
    T.nback[i] = ~0ull;
  }
  __syncthreads();
  for (uint32_t sweep = 0;; ++sweep) {
    if (tid == 0) SH.changed = 0;
    __syncthreads();
    for (uint32_t l = 0; l < n_levels; ++l) {
      const uint32_t b0 = T.lvl[l], b1 = T.lvl[l + 1];
      for (uint32_t s = b0 + tid; s < b1; s += WG) {
        const double ds = from_okey(ld_agent(&T.nd[s]));
        if (w_is_zero(ds)) continue;
        for (uint32_t a = T.aoff[s]; a < T.aoff[s + 1]; ++a) {
          const unsigned long long v = okey(w_times(ds, T.aw[a]));  // shortest-path.zig:72
          const unsigned long long old = atomicMin(&T.nd[T.anext[a]], v);
          if (v < old) SH.changed = 1;
        }
      }
      __syncthreads();
    }
    // read the verdicts into registers, then a barrier: thread 0 resets SH.changed for
    // the next sweep only after every thread has read it (uniform exit)
    if (tid == 0) SH.flag = __builtin_amdgcn_s_memrealtime() > deadline;
    __syncthreads();
    const bool changed = SH.changed != 0, expired = SH.flag != 0;
    __syncthreads();
    if (!changed) break;
    if (expired || sweep > n_nodes) {  // sweep > n_nodes cannot happen for weights >= 0
      fail = kPathInternal;
      break;
    }
  }
  if (fail != kPathOk) {
    if (tid == 0) write_status(out, si, fail, n_nodes, n_arcs);
    return;
  }
  // back-pointers: tight in-arc with the smallest (source, arc index)
  for (uint32_t s = tid; s < n_nodes; s += WG) {
    const double ds = from_okey(ld_agent(&T.nd[s]));
    if (w_is_zero(ds)) continue;
    const uint32_t a0 = T.aoff[s], a1 = T.aoff[s + 1];
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t x = T.anext[a];
      const unsigned long long v = okey(w_times(ds, T.aw[a]));
      if (v == ld_agent(&T.nd[x]))
        atomicMin(&T.nback[x], ((unsigned long long)s << 32) | (a - a0));
    }
  }
  // best final: lexmin (total, id)
  if (tid == 0) {
    SH.best = kMaxU64;
    SH.bestid = kEmptyKey;
  }
  __syncthreads();
  unsigned long long mk = kMaxU64;
  uint32_t mid = kEmptyKey;
  for (uint32_t s = tid; s < n_nodes; s += WG) {
    const double ds = from_okey(ld_agent(&T.nd[s]));
    const double fw = T.nfin[s];
    if (w_is_zero(ds) || w_is_zero(fw)) continue;
    const unsigned long long k = okey(w_times(ds, fw));
    if (k < mk) {  // s ascending per thread: equal keys keep the smaller id
      mk = k;
      mid = s;
    }
  }
  if (mk != kMaxU64) atomicMin(&SH.best, mk);
  __syncthreads();
  if (mk != kMaxU64 && mk == SH.best) atomicMin(&SH.bestid, mid);
  __syncthreads();

  if (tid == 0) {
    const uint32_t best = SH.bestid;
    if (best == kEmptyKey) {
      write_status(out, si, kPathEmpty, n_nodes, n_arcs);
    } else {
      // walk 1: length and termination (bounded: a cycle reports CYCLE)
      uint32_t cur = best, hops = 0;
      bool cyc = false;
      for (;;) {
        const unsigned long long b = ld_agent(&T.nback[cur]);
        if (b == ~0ull) break;
        if (++hops > n_nodes) {
          cyc = true;
          break;
        }
        cur = (uint32_t)(b >> 32);
      }
      if (cyc) {
        write_status(out, si, kPathCycle, n_nodes, n_arcs);
      } else if (cur != start) {  // shortest-path.zig:120-122
        write_status(out, si, kPathEmpty, n_nodes, n_arcs);
      } else {
        const unsigned long long o = atomicAdd(out.cursor, (unsigned long long)hops);
        if (o + hops > out.arc_cap) {
          write_status(out, si, kPathOutputFull, n_nodes, n_arcs);
        } else {
          cur = best;
          for (uint32_t k = hops; k > 0; --k) {  // walk 2: emit arcs back to front
            const unsigned long long b = ld_agent(&T.nback[cur]);
            const uint32_t s = (uint32_t)(b >> 32);
            const uint32_t a = T.aoff[s] + (uint32_t)b;
            out.out_il[o + k - 1] = T.ail[a];
            out.out_ol[o + k - 1] = T.aol[a];
            out.out_w[o + k - 1] = T.aw[a];
            cur = s;
          }
          out.status[si] = kPathOk;
          out.path_len[si] = hops;
          out.path_off[si] = o;
          out.final_w[si] = T.nfin[best];
          if (out.work) {
            out.work[2 * si] = n_nodes;
            out.work[2 * si + 1] = n_arcs;
          }
        }
      }
    }
  }
}

template <int WG, bool kGraph>
__global__ void __launch_bounds__(WG)
eager_bfs_kernel(RhsView rhs, ChainInput in, GraphInput graph, uint32_t n_best,
                 unsigned int* next_item, const uint32_t* items, const uint32_t* num_items_dev,
                 uint32_t num_items_host, BfsWs ws, BatchOutDev out) {
  __shared__ BfsShared SH;
  const uint32_t tid = threadIdx.x;
  BfsTables T = bfs_carve(ws.slab + (size_t)blockIdx.x * ws.stride, ws.ncap, ws.acap, ws.hcap,
                          ws.lcap);
  uint32_t* hdr = ws.hdr + (size_t)blockIdx.x * 8;
  const uint32_t num_items = num_items_dev ? *num_items_dev : num_items_host;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t hmask = ws.hcap - 1;

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      SH.item = atomicAdd(next_item, 1u);
      SH.expired = __builtin_amdgcn_s_memrealtime() - t0 > ws.wd_ticks;
    }
    __syncthreads();
    const uint32_t item = SH.item;
    if (item >= num_items) break;
    const uint32_t si = items ? items[item] : item;

    BfsLhs<kGraph> lhs;
    lhs.g = graph;
    lhs.labels = nullptr;
    lhs.L = 0;
    if constexpr (!kGraph) {
      const uint64_t off = in.offsets[si];
      lhs.labels = in.labels + off;
      lhs.L = (uint32_t)(in.offsets[si + 1] - off);
    }
    const bool no_start = rhs.start == kNoState || lhs.start() == kNoState;
    if (!ws.lattice_only && (no_start || n_best != 1)) {
      // shortest-path.zig:21-24 on the (empty if no start) lattice
      if (tid == 0) write_status(out, si, (no_start || n_best == 0) ? kPathEmpty : kPathErrorN, 0, 0);
      continue;
    }
    if (ws.lattice_only && no_start) {  // compose.zig:33-35: empty result
      if (tid == 0) {
        hdr[0] = 0;
        hdr[1] = 0;
        hdr[2] = 0;
        hdr[3] = kPathOk;
        hdr[4] = si;
      }
      continue;
    }
    if (SH.expired) {
      if (tid == 0) write_status(out, si, kPathInternal, 0, 0);
      continue;
    }

    // ---- compose: level-synchronous BFS ----
    for (uint32_t i = tid; i < ws.hcap; i += WG) {
      T.hkey[i] = ~0ull;
      T.hval[i] = ~0u;
    }
    __syncthreads();
    const unsigned long long k0 = bfs_key(lhs.start(), rhs.start, 0);
    if (tid == 0) {
      uint32_t h = bfs_hash(k0) & hmask;
      T.hkey[h] = k0;
      T.hval[h] = 0;
      T.nkey[0] = k0;
      T.lvl[0] = 0;
      T.lvl[1] = 1;
      T.aoff[0] = 0;
    }
    __syncthreads();
    uint32_t n_nodes = 1, n_arcs = 0, level = 0;
    int32_t fail = kPathOk;
    while (true) {
      const uint32_t f0 = level == 0 ? 0u : ld_agent(&T.lvl[level]);
      const uint32_t f1 = n_nodes;
      if (f0 >= f1) break;
      if (level + 2 > ws.lcap) {
        fail = kPathOverflow;
        break;
      }
      // (A) candidate counts -> arc offsets; final weights of the level's tuples
      uint32_t carry = 0;
      for (uint32_t b = f0; b < f1; b += WG) {
        const uint32_t p = b + tid;
        uint32_t cnt = 0;
        if (p < f1) {
          const unsigned long long k = T.nkey[p];
          const uint32_t s1 = (uint32_t)(k >> 2) & 0x3FFFFFFFu, s2 = (uint32_t)(k >> 32),
                         f = (uint32_t)k & 3u;
          bfs_expand<kGraph>(rhs, lhs, s1, s2, f,
                             [&](uint32_t, uint32_t, double, unsigned long long) { ++cnt; });
          // compose.zig:69-74: final = fw1 (x) fw2 when both are non-Zero
          const double fw1 = lhs.final_w(s1), fw2 = rhs.final_w[s2];
          T.nfin[p] = (!w_is_zero(fw1) && !w_is_zero(fw2)) ? w_times(fw1, fw2) : w_zero();
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<WG>(cnt, SH.scan, tot);
        if (p < f1) T.aoff[p] = n_arcs + carry + ex;
        carry += tot;
      }
      if ((uint64_t)n_arcs + carry > ws.acap) {
        fail = kPathOverflow;
        break;
      }
      if (tid == 0) T.aoff[f1] = n_arcs + carry;
      __syncthreads();
      // (B) write arcs, insert targets (first candidate of a new key wins)
      if (tid == 0) SH.flag = 0;
      __syncthreads();
      for (uint32_t p = f0 + tid; p < f1; p += WG) {
        const unsigned long long k = T.nkey[p];
        const uint32_t s1 = (uint32_t)(k >> 2) & 0x3FFFFFFFu, s2 = (uint32_t)(k >> 32),
                       f = (uint32_t)k & 3u;
        uint32_t a = T.aoff[p];
        bfs_expand<kGraph>(rhs, lhs, s1, s2, f,
                           [&](uint32_t il, uint32_t ol, double w, unsigned long long key) {
                             T.ail[a] = il;
                             T.aol[a] = ol;
                             T.aw[a] = w;
                             uint32_t h = bfs_hash(key) & hmask, slot = kEmptyKey;
                             for (uint32_t probe = 0; probe <= hmask; ++probe) {
                               const unsigned long long old = atomicCAS(&T.hkey[h], ~0ull, key);
                               if (old == ~0ull || old == key) {
                                 slot = h;
                                 break;
                               }
                               h = (h + 1) & hmask;
                             }
                             if (slot == kEmptyKey) {
                               SH.flag = 1;
                             } else {
                               atomicMin(&T.hval[slot], 0x80000000u | a);  // ids stay smaller
                             }
                             T.cslot[a] = slot;
                             ++a;
                           });
      }
      __syncthreads();
      if (SH.flag) {
        fail = kPathOverflow;
        break;
      }
      // (C) ids of first occurrences, in candidate order (contiguous chunks per thread)
      const uint32_t c0 = n_arcs, c1 = n_arcs + carry;
      constexpr uint32_t K = 4;
      uint32_t newc = 0;
      for (uint32_t b = c0; b < c1; b += WG * K) {
        const uint32_t a0 = b + tid * K;
        uint32_t nf = 0;
#pragma unroll
        for (uint32_t q = 0; q < K; ++q) {
          const uint32_t a = a0 + q;
          if (a < c1 && ld_agent(&T.hval[T.cslot[a]]) == (0x80000000u | a)) ++nf;
        }
        uint32_t tot;
        uint32_t rank = block_excl_scan<WG>(nf, SH.scan, tot);
        if ((uint64_t)n_nodes + newc + tot > ws.ncap) {
          SH.flag = 1;  // read after the loop (uniform: every thread sees the same tot)
        } else {
#pragma unroll
          for (uint32_t q = 0; q < K; ++q) {
            const uint32_t a = a0 + q;
            if (a < c1) {
              const uint32_t slot = T.cslot[a];
              if (ld_agent(&T.hval[slot]) == (0x80000000u | a)) {
                const uint32_t id = n_nodes + newc + rank++;
                T.hval[slot] = id;
                T.nkey[id] = ld_agent(&T.hkey[slot]);
              }
            }
          }
        }
        newc += tot;
        if ((uint64_t)n_nodes + newc > ws.ncap) break;
      }
      __syncthreads();
      if ((uint64_t)n_nodes + newc > ws.ncap) {
        fail = kPathOverflow;
        break;
      }
      // (D) arc targets
      for (uint32_t a = c0 + tid; a < c1; a += WG) T.anext[a] = ld_agent(&T.hval[T.cslot[a]]);
      n_arcs = c1;
      n_nodes += newc;
      ++level;
      if (tid == 0) T.lvl[level + 1] = n_nodes;
      __syncthreads();
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2 * ws.wd_ticks) {  // uniform per wave...
        if (tid == 0) SH.flag = 1;
      }
      __syncthreads();
      if (SH.flag) {  // ...made uniform for the workgroup through LDS
        fail = kPathInternal;
        break;
      }
    }
    const uint32_t n_levels = level;

    if (ws.lattice_only) {
      if (tid == 0) {
        hdr[0] = n_nodes;
        hdr[1] = n_arcs;
        hdr[2] = n_levels;
        hdr[3] = (uint32_t)fail;
        hdr[4] = si;
      }
      continue;
    }
    if (fail != kPathOk) {
      if (tid == 0) write_status(out, si, fail, n_nodes, n_arcs);
      continue;
    }

    bfs_shortest_path<WG>(T, n_nodes, n_arcs, n_levels, 0u, out, si, SH, t0 + 2 * ws.wd_ticks);
  }
}

// fst_shortest_path on an explicit FST held as a lattice (T.aoff/anext/ail/aol/aw/nfin
// are the FST's own CSR, T.lvl = {0, N}: one "level", Jacobi-style sweeps).
template <int WG>
__global__ void __launch_bounds__(WG)
sp_graph_kernel(BfsTables T, uint32_t n_nodes, uint32_t start, uint32_t n_best, BatchOutDev out,
                unsigned long long wd_ticks) {
  __shared__ BfsShared SH;
  if (start == kNoState || n_best == 0 || n_nodes == 0) {  // shortest-path.zig:21-23
    if (threadIdx.x == 0) write_status(out, 0, kPathEmpty, 0, 0);
    return;
  }
  if (n_best != 1) {  // :24
    if (threadIdx.x == 0) write_status(out, 0, kPathErrorN, 0, 0);
    return;
  }
  bfs_shortest_path<WG>(T, n_nodes, T.aoff[n_nodes], 1u, start, out, 0u, SH,
                        __builtin_amdgcn_s_memrealtime() + wd_ticks);
}

}  // namespace fstamd
