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
  uint32_t lazy;            // 1: composeShortestPath semantics (bfs_lazy_path)
  unsigned long long* prof; // [grid * 8] phase ticks (FSTAMD_BFS_PROF) or null
  uint8_t* replay;          // non-null: exact heap replay (negative weights); per workgroup
                            // (acap + 1) * 16 B of heap, then ncap B of settled flags
};

// Phase profile (thread 0): prof[slot] += ticks since *tp; *tp = now.  Slots: 0 compose,
// 1 fixpoint, 2 lazy rounds, 3 back/best/backtrace, 4 items, 5 rounds, 6 sum of active
// list lengths, 7 sum of members.
__device__ __forceinline__ void prof_mark(unsigned long long* prof, int slot,
                                          unsigned long long* tp) {
  if (prof && threadIdx.x == 0) {
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    prof[slot] += now - *tp;
    *tp = now;
  }
}
__device__ __forceinline__ void prof_add(unsigned long long* prof, int slot,
                                         unsigned long long v) {
  if (prof && threadIdx.x == 0) prof[slot] += v;
}

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
  uint32_t* cslot;           // [acap + ncap] hash slot of the arc's target (level scratch)
};

__host__ __device__ constexpr size_t bfs_slab_bytes(uint32_t ncap, uint32_t acap, uint32_t hcap,
                                                    uint32_t lcap, size_t align = 256) {
  auto r = [align](size_t b) { return (b + align - 1) & ~(align - 1); };
  return r((size_t)hcap * 8) + r((size_t)hcap * 4) + r((size_t)ncap * 8) +
         r(((size_t)ncap + 1) * 4) + r(((size_t)lcap + 2) * 4) + r((size_t)ncap * 8) +
         r((size_t)ncap * 8) + r((size_t)ncap * 8) + r((size_t)acap * 4) * 3 +
         r((size_t)acap * 8) + r(((size_t)acap + ncap) * 4);
}

__device__ inline BfsTables bfs_carve(uint8_t* p, uint32_t ncap, uint32_t acap, uint32_t hcap,
                                      uint32_t lcap, size_t align = 256) {
  auto take = [&](size_t b) {
    uint8_t* q = p;
    p += (b + align - 1) & ~(align - 1);
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
  t.cslot = (uint32_t*)take(((size_t)acap + ncap) * 4);
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
    uint32_t lo, cnt;
    span_summary<kGraph>(rhs, s2, ol, lo, cnt);
    for (uint32_t a = lo; a < lo + cnt; ++a) {
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
  uint32_t elo, ecnt;
  span_summary<kGraph>(rhs, s2, kEpsilon, elo, ecnt);
  const uint32_t ehi = elo + ecnt;
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
  unsigned long long red[16];  // per-wave partials of block reductions
  uint32_t item;
  unsigned long long t_item;   // when thread 0 fetched the item: the per-string watchdog
  uint32_t flag;
  uint32_t changed;
  unsigned long long best;
  uint32_t bestid;
  uint32_t count;              // lazy rounds: next active list length
};

// Least fixpoint of d(X) = min fl(d(s) + w) from d(start) = One, by Gauss-Seidel sweeps
// over the BFS levels (lvl[0..n_levels]); also clears nback.  The whole workgroup calls
// it; false = the deadline passed (uniform).  `init`: start from d = (One at the start,
// Zero elsewhere); otherwise nd already holds path sums (compose relaxed every level in
// order), and `dag` (every arc goes to the next level) means they are already final.
template <int WG>
__device__ bool bfs_fixpoint(const BfsTables& T, uint32_t n_nodes, uint32_t n_levels,
                             uint32_t start, BfsShared& SH, unsigned long long deadline,
                             bool init = true, bool dag = false) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < n_nodes; i += WG) {
    if (init) T.nd[i] = i == start ? okey(w_one()) : okey(w_zero());
    T.nback[i] = ~0ull;
  }
  __syncthreads();
  if (dag) return true;
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
    if (!changed) return true;
    if (expired || sweep > n_nodes) return false;  // sweep > n_nodes: impossible for w >= 0
  }
}

// shortestPath on a lattice held in BfsTables (aoff / anext / aw / ail / aol / nfin, BFS
// levels in lvl[0..n_levels]); the whole workgroup calls it; thread 0 writes the result.
template <int WG>
__device__ void bfs_shortest_path(const BfsTables& T, uint32_t n_nodes, uint32_t n_arcs,
                                  uint32_t n_levels, uint32_t start, const BatchOutDev& out,
                                  uint32_t si, BfsShared& SH, unsigned long long deadline,
                                  bool init = true, bool dag = false) {
  const uint32_t tid = threadIdx.x;
  if (!bfs_fixpoint<WG>(T, n_nodes, n_levels, start, SH, deadline, init, dag)) {
    if (tid == 0) write_status(out, si, kPathInternal, n_nodes, n_arcs);
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
        const unsigned long long o = reserve_path(out, si, hops);
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

// ---------------------------------------------------------------------------------------
// composeShortestPath (src/ops/compose-shortest-path.zig:26-401) for finite weights >= 0,
// on the lattice compose built (same tuples, same arcs in the same candidate order: the
// lazy expansion at :182-365 follows compose.zig's 4 phases).  Its answer depends on the
// heap order only through the ids, which are assigned at first touch in pop order; so:
//   dist  = the least fixpoint (bfs_fixpoint), as for shortestPath;
//   lid   = first-touch ids in pop order, computed in parallel rounds (below);
//   back  = lexmin (lid(source), il, ol, candidate order) over tight in-arcs (relax at
//           :107-141: a lexicographic min on (dist, source id, il, ol); a full tie keeps
//           the earlier relaxation);
//   best  = lexmin (total, lid) over nodes with both finals non-Zero (:165-179);
//   path  = back-pointers from best until the start id (:368-380).
// Rounds.  A node is poppable ("active") once a popped in-neighbour reaches it tightly
// (its tentative dist is then final), the start from the outset; with weights >= 0 the
// heap minimum is always an active node at the minimum active dist dmin.  A round takes
// the active nodes at dmin in lid order and pops the longest prefix that no member's
// "joiner" undercuts: popping u activates an older, inactive node x at dmin (0-weight
// arc) that must pop before every member with a larger lid.  Targets first touched in
// the round get fresh lids in (popper order, candidate order) -- larger than every
// existing lid, so they never undercut.  tests/lazy_model.py is the executable model,
// checked against the sequential replay on random tie-heavy inputs.
// ---------------------------------------------------------------------------------------

// Wavefront-then-workgroup reductions / scans through SH (all threads call).
template <int WG>
__device__ __forceinline__ unsigned long long block_min_u64(unsigned long long v, BfsShared& SH) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = y < v ? y : v;
  }
  if constexpr (WG == 64) {
    return v;
  } else {
    if ((threadIdx.x & 63) == 0) SH.red[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long m = SH.red[0];
#pragma unroll
    for (int i = 1; i < WG / 64; ++i) m = SH.red[i] < m ? SH.red[i] : m;
    __syncthreads();
    return m;
  }
}

// Exclusive prefix minimum in thread order (identity ~0u); `total` = the block minimum.
template <int WG>
__device__ __forceinline__ uint32_t block_excl_min(uint32_t v, BfsShared& SH, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc = y < inc ? y : inc;
  }
  uint32_t ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = ~0u;
  if constexpr (WG == 64) {
    total = __shfl(inc, 63, 64);
    return ex;
  } else {
    if (lane == 63) SH.scan[w] = inc;
    __syncthreads();
    uint32_t base = ~0u, tot = ~0u;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) {
      const uint32_t t = SH.scan[i];
      if (i < w) base = t < base ? t : base;
      tot = t < tot ? t : tot;
    }
    __syncthreads();
    total = tot;
    return base < ex ? base : ex;
  }
}

// Round tables, carved from the BFS tables compose no longer needs (hkey / hval / nkey /
// lvl / cslot; the fixpoint has finished with lvl).
struct LazyTables {
  uint32_t* lid;    // [n] first-touch id, ~0 = untouched
  uint32_t* inv;    // [n] lid -> node
  uint32_t* flg;    // [n] kLzActive | kLzPopped
  uint32_t* touch;  // [n] smallest candidate rank touching an untouched node this round
  uint32_t* act;    // [n] active nodes (unordered)
  uint32_t* act2;   // [n] next round's active nodes
  uint32_t* slist;  // [n] this round's dmin members in lid order
  uint32_t* mbase;  // [n] rank of each member's header entry in rk
  uint32_t* bmap;   // [n / 32 + 1] lid bitmap of the members (clear between rounds)
  uint32_t* rk;     // [arcs + n] per member: header (kLzHdr | member), then its arcs
};
constexpr uint32_t kLzHdr = 0x80000000u;
constexpr uint32_t kLzActive = 1u, kLzPopped = 2u;

__device__ inline LazyTables lazy_carve(const BfsTables& T, uint32_t ncap) {
  LazyTables L;
  uint32_t* h = (uint32_t*)T.hkey;  // 8 * hcap >= 16 * ncap bytes
  L.lid = h;
  L.inv = h + ncap;
  L.flg = h + 2 * (size_t)ncap;
  L.touch = h + 3 * (size_t)ncap;
  L.act = T.hval;                   // 4 * hcap >= 8 * ncap bytes
  L.act2 = T.hval + ncap;
  L.slist = (uint32_t*)T.nkey;      // 8 * ncap bytes
  L.mbase = (uint32_t*)T.nkey + ncap;
  L.bmap = T.lvl;                   // 4 * (ncap + 2) bytes
  L.rk = T.cslot;
  return L;
}

template <int WG>
__device__ void bfs_lazy_path(const BfsTables& T, uint32_t ncap, uint32_t n_nodes,
                              uint32_t n_arcs, uint32_t n_levels, uint32_t start,
                              const BatchOutDev& out, uint32_t si, BfsShared& SH,
                              unsigned long long deadline, unsigned long long* prof,
                              unsigned long long* tp, bool dag) {
  const uint32_t tid = threadIdx.x;
  const bool fix_ok = bfs_fixpoint<WG>(T, n_nodes, n_levels, start, SH, deadline, false, dag);
  prof_mark(prof, 1, tp);
  if (!fix_ok) {
    if (tid == 0) write_status(out, si, kPathInternal, n_nodes, n_arcs);
    return;
  }
  const LazyTables L = lazy_carve(T, ncap);
  for (uint32_t i = tid; i < n_nodes; i += WG) {
    L.lid[i] = i == start ? 0u : ~0u;
    L.flg[i] = i == start ? kLzActive : 0u;
    L.touch[i] = ~0u;
  }
  for (uint32_t i = tid; i <= n_nodes / 32; i += WG) L.bmap[i] = 0;
  if (tid == 0) {
    L.inv[0] = start;
    L.act[0] = start;
  }
  __syncthreads();

  uint32_t* A = L.act;
  uint32_t* A2 = L.act2;
  uint32_t na = 1, nxt = 1, popped = 0;
  int32_t fail = kPathOk;
  while (na > 0) {
    prof_add(prof, 5, 1);
    prof_add(prof, 6, na);
    // (1) dmin over the active nodes
    unsigned long long m = kMaxU64;
    for (uint32_t i = tid; i < na; i += WG) {
      const unsigned long long d = ld_agent(&T.nd[A[i]]);
      m = d < m ? d : m;
    }
    const unsigned long long dmin = block_min_u64<WG>(m, SH);
    // (2) members (active at dmin) into the lid bitmap; lid range
    uint32_t lo = ~0u, hi = 0;
    for (uint32_t i = tid; i < na; i += WG) {
      const uint32_t u = A[i];
      if (ld_agent(&T.nd[u]) != dmin) continue;
      const uint32_t l = L.lid[u];
      atomicOr(&L.bmap[l >> 5], 1u << (l & 31));
      lo = l < lo ? l : lo;
      hi = l > hi ? l : hi;
    }
    lo = (uint32_t)(block_min_u64<WG>(lo, SH));
    hi = ~(uint32_t)(block_min_u64<WG>((unsigned long long)(~hi), SH));
    // (3) members in lid order: compact the bitmap words [lo/32, hi/32], clearing them
    uint32_t ns = 0;
    const uint32_t w0 = lo >> 5, w1 = hi >> 5;
    for (uint32_t b = w0; b <= w1; b += WG) {
      const uint32_t w = b + tid;
      uint32_t bits = w <= w1 ? ld_agent(&L.bmap[w]) : 0u;
      uint32_t tot;
      uint32_t pos = ns + block_excl_scan<WG>((uint32_t)__builtin_popcount(bits), SH.scan, tot);
      if (w <= w1) L.bmap[w] = 0;
      while (bits) {
        const uint32_t bit = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1;
        L.slist[pos++] = L.inv[(w << 5) | bit];
      }
      ns += tot;
    }
    prof_add(prof, 7, ns);
    __syncthreads();
    // (4) rank list: per member (lid order) a header entry, then its arcs (candidate
    // order); the batch's candidates are the ranks before the first unpopped header
    uint32_t RA = 0;
    for (uint32_t b = 0; b < ns; b += WG) {
      const uint32_t p = b + tid;
      uint32_t a0 = 0, deg = 0;
      if (p < ns) {
        const uint32_t u = L.slist[p];
        a0 = T.aoff[u];
        deg = T.aoff[u + 1] - a0;
      }
      uint32_t tot;
      const uint32_t base = RA + block_excl_scan<WG>(p < ns ? deg + 1 : 0u, SH.scan, tot);
      if (p < ns) {
        L.mbase[p] = base;
        L.rk[base] = kLzHdr | p;
        for (uint32_t i = 0; i < deg; ++i) L.rk[base + 1 + i] = a0 + i;
      }
      RA += tot;
    }
    __syncthreads();
    // (5) batch = longest lid-ordered prefix no earlier member's joiner undercuts: per
    // arc the joiner lid (an older, inactive node it reaches tightly at dmin), an
    // exclusive prefix minimum in rank order, checked at every member's header
    const double dminw = from_okey(dmin);
    uint32_t k = ns, carry = ~0u;
    for (uint32_t b = 0; b < RA; b += WG) {
      const uint32_t r = b + tid;
      uint32_t j = ~0u, my = 0, hp = ~0u;
      if (r < RA) {
        const uint32_t e = L.rk[r];
        if (e & kLzHdr) {
          hp = e & ~kLzHdr;
          my = L.lid[L.slist[hp]];
        } else {
          const uint32_t x = T.anext[e];
          if (okey(w_times(dminw, T.aw[e])) == dmin && ld_agent(&T.nd[x]) == dmin) {
            const uint32_t lx = L.lid[x];
            if (lx != ~0u && (ld_agent(&L.flg[x]) & (kLzActive | kLzPopped)) == 0) j = lx;
          }
        }
      }
      uint32_t tot;
      uint32_t ex = block_excl_min<WG>(j, SH, tot);
      ex = carry < ex ? carry : ex;
      const uint32_t viol = (hp != ~0u && my > ex) ? hp : ~0u;
      const uint32_t cut = (uint32_t)block_min_u64<WG>(viol, SH);
      if (cut != ~0u) {
        k = cut;
        break;
      }
      carry = tot < carry ? tot : carry;
    }
    const uint32_t R = k < ns ? L.mbase[k] : RA;
    for (uint32_t p = tid; p < k; p += WG) L.flg[L.slist[p]] = kLzPopped;
    if (tid == 0) SH.count = 0;
    __syncthreads();
    // (6) first touches; tight targets become active; survivors of the old list stay
    for (uint32_t r = tid; r < R; r += WG) {
      const uint32_t a = L.rk[r];
      if (a & kLzHdr) continue;
      const uint32_t x = T.anext[a];
      if (L.lid[x] == ~0u) atomicMin(&L.touch[x], r);
      if (okey(w_times(dminw, T.aw[a])) == ld_agent(&T.nd[x]) &&
          (ld_agent(&L.flg[x]) & kLzPopped) == 0) {
        const uint32_t old = atomicOr(&L.flg[x], kLzActive);
        if ((old & kLzActive) == 0) A2[atomicAdd(&SH.count, 1u)] = x;
      }
    }
    for (uint32_t i = tid; i < na; i += WG) {
      const uint32_t u = A[i];
      if ((ld_agent(&L.flg[u]) & kLzPopped) == 0) A2[atomicAdd(&SH.count, 1u)] = u;
    }
    __syncthreads();
    // (7) fresh lids for the first touches, in rank order (K contiguous ranks per thread)
    constexpr uint32_t K = 4;
    uint32_t newc = 0;
    for (uint32_t b = 0; b < R; b += WG * K) {
      const uint32_t r0 = b + tid * K;
      uint32_t mask = 0, nf = 0;
#pragma unroll
      for (uint32_t q = 0; q < K; ++q) {
        const uint32_t r = r0 + q;
        const uint32_t a = r < R ? L.rk[r] : kLzHdr;
        if (!(a & kLzHdr)) {
          const uint32_t x = T.anext[a];
          if (ld_agent(&L.touch[x]) == r && L.lid[x] == ~0u) {
            mask |= 1u << q;
            ++nf;
          }
        }
      }
      uint32_t tot;
      uint32_t rank = nxt + newc + block_excl_scan<WG>(nf, SH.scan, tot);
#pragma unroll
      for (uint32_t q = 0; q < K; ++q) {
        if (mask & (1u << q)) {
          const uint32_t x = T.anext[L.rk[r0 + q]];
          L.lid[x] = rank;
          L.inv[rank] = x;
          ++rank;
        }
      }
      newc += tot;
    }
    nxt += newc;
    popped += k;
    if (tid == 0) SH.flag = __builtin_amdgcn_s_memrealtime() > deadline;
    __syncthreads();
    na = SH.count;
    const bool expired = SH.flag != 0;
    __syncthreads();
    uint32_t* t = A;
    A = A2;
    A2 = t;
    if (expired || popped > n_nodes || nxt > n_nodes) {
      fail = kPathInternal;
      break;
    }
  }
  prof_mark(prof, 2, tp);
  if (fail == kPathOk && (popped != n_nodes || nxt != n_nodes)) fail = kPathInternal;
  if (fail != kPathOk) {
    if (tid == 0) write_status(out, si, fail, n_nodes, n_arcs);
    return;
  }

  // back-pointers: lexmin (lid(source), il, ol, candidate order) over tight in-arcs; a
  // source contributes only its own best tight arc into each target
  for (uint32_t s = tid; s < n_nodes; s += WG) {
    const double ds = from_okey(ld_agent(&T.nd[s]));
    const uint32_t a0 = T.aoff[s], a1 = T.aoff[s + 1];
    const unsigned long long ls = (unsigned long long)L.lid[s] << 32;
    if (a1 - a0 <= 8) {  // registers: independent loads, then a tight-arc bitmask
      constexpr int M = 8;
      uint32_t nx[M], tight = 0;
#pragma unroll
      for (int i = 0; i < M; ++i) nx[i] = a0 + i < a1 ? T.anext[a0 + i] : ~0u;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (nx[i] == ~0u) continue;
        if (okey(w_times(ds, T.aw[a0 + i])) == ld_agent(&T.nd[nx[i]])) tight |= 1u << i;
      }
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (!(tight & (1u << i))) continue;
        uint32_t rivals = 0;  // other tight arcs of s into the same target
#pragma unroll
        for (int c = 0; c < M; ++c)
          if (c != i && (tight & (1u << c)) && nx[c] == nx[i]) rivals |= 1u << c;
        bool win = true;
        if (rivals) {
          const uint32_t il = T.ail[a0 + i], ol = T.aol[a0 + i];
          for (int c = 0; c < M && win; ++c) {
            if (!(rivals & (1u << c))) continue;
            const uint32_t cil = T.ail[a0 + c], col = T.aol[a0 + c];
            if (cil < il || (cil == il && (col < ol || (col == ol && c < i)))) win = false;
          }
        }
        if (win) atomicMin(&T.nback[nx[i]], ls | (uint32_t)i);
      }
      continue;
    }
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t x = T.anext[a];
      const unsigned long long dx = ld_agent(&T.nd[x]);
      if (okey(w_times(ds, T.aw[a])) != dx) continue;
      const uint32_t il = T.ail[a], ol = T.aol[a];
      bool win = true;
      for (uint32_t c = a0; c < a1 && win; ++c) {
        if (c == a || T.anext[c] != x) continue;
        const uint32_t cil = T.ail[c], col = T.aol[c];
        const bool before = cil < il || (cil == il && (col < ol || (col == ol && c < a)));
        if (before && okey(w_times(ds, T.aw[c])) == dx) win = false;
      }
      if (win) atomicMin(&T.nback[x], ls | (a - a0));
    }
  }
  // best final: lexmin (total, lid)
  if (tid == 0) {
    SH.best = kMaxU64;
    SH.bestid = kEmptyKey;
  }
  __syncthreads();
  unsigned long long mk = kMaxU64;
  uint32_t ml = kEmptyKey;
  for (uint32_t s = tid; s < n_nodes; s += WG) {
    const double fw = T.nfin[s];
    if (w_is_zero(fw)) continue;
    const unsigned long long kk = okey(w_times(from_okey(ld_agent(&T.nd[s])), fw));
    const uint32_t l = L.lid[s];
    if (kk < mk || (kk == mk && l < ml)) {
      mk = kk;
      ml = l;
    }
  }
  if (mk != kMaxU64) atomicMin(&SH.best, mk);
  __syncthreads();
  if (mk != kMaxU64 && mk == SH.best) atomicMin(&SH.bestid, ml);
  __syncthreads();

  if (tid == 0) {
    if (SH.bestid == kEmptyKey) {
      write_status(out, si, kPathEmpty, n_nodes, n_arcs);
      return;
    }
    const uint32_t best = L.inv[SH.bestid];
    // walk 1 (compose-shortest-path.zig:372-380): until the start id; bounded
    uint32_t cur = best, hops = 0;
    int32_t st = kPathOk;
    while (cur != start) {
      const unsigned long long b = ld_agent(&T.nback[cur]);
      if (b == ~0ull) {
        st = kPathEmpty;
        break;
      }
      if (++hops > n_nodes) {
        st = kPathCycle;
        break;
      }
      cur = L.inv[(uint32_t)(b >> 32)];
    }
    if (st != kPathOk) {
      write_status(out, si, st, n_nodes, n_arcs);
      return;
    }
    const unsigned long long o = reserve_path(out, si, hops);
    if (o + hops > out.arc_cap) {
      write_status(out, si, kPathOutputFull, n_nodes, n_arcs);
      return;
    }
    cur = best;
    for (uint32_t k = hops; k > 0; --k) {  // walk 2: emit arcs back to front
      const unsigned long long b = ld_agent(&T.nback[cur]);
      const uint32_t s = L.inv[(uint32_t)(b >> 32)];
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

// ---------------------------------------------------------------------------------------
// Exact replay of shortestPath (src/ops/shortest-path.zig:18-139) for weights of any sign
// (fst_shortest_path, or the eager batch, with a negative weight).  With a negative arc Dijkstra is no longer
// the least fixpoint: a settled state's dist and back-pointer still move (:70-84) but its
// arcs are never relaxed again, so the answer depends on the pop order.  The queue order
// is total -- (dist, state) lexicographic (:56-62) -- and two entries equal in both are
// interchangeable (the second is skipped as settled), so any binary heap pops the same
// sequence; one lane replays it.  Pushes happen once per relaxation of an unsettled
// target, at most once per arc per settle, so the heap never holds more than
// n_arcs + 1 entries.  Latency-bound by construction: it only serves rhs / graphs with a
// negative weight, and the deadline turns a runaway into INTERNAL.
// ---------------------------------------------------------------------------------------
struct SpHeapEnt {
  double d;
  uint32_t s, pad;
};
__device__ __forceinline__ bool sp_heap_less(const SpHeapEnt& a, const SpHeapEnt& b) {
  return a.d < b.d || (a.d == b.d && a.s < b.s);  // W.compare = IEEE order, then the id
}

// The whole workgroup calls it (it initialises with every thread); thread 0 replays.
__device__ void sp_replay(const BfsTables& T, uint32_t n_nodes, uint32_t n_arcs,
                          uint32_t start, SpHeapEnt* heap, uint64_t hcap, uint8_t* settled,
                          const BatchOutDev& out, uint32_t si, unsigned long long deadline) {
  const uint32_t lane = threadIdx.x;
  double* dist = reinterpret_cast<double*>(T.nd);
  for (uint32_t s = lane; s < n_nodes; s += blockDim.x) {  // :35-37, :45-49
    dist[s] = __builtin_huge_val();
    T.nback[s] = ~0ull;
    settled[s] = 0;
  }
  __syncthreads();
  if (lane != 0) return;
  dist[start] = 0.0;
  uint64_t hn = 1;
  heap[0] = SpHeapEnt{0.0, start, 0};
  uint64_t pops = 0;
  while (hn > 0) {  // :65
    const SpHeapEnt item = heap[0];
    const SpHeapEnt last = heap[--hn];
    uint64_t k = 0;  // sift `last` down from the root
    for (;;) {
      uint64_t c = 2 * k + 1;
      if (c >= hn) break;
      if (c + 1 < hn && sp_heap_less(heap[c + 1], heap[c])) ++c;
      if (!sp_heap_less(heap[c], last)) break;
      heap[k] = heap[c];
      k = c;
    }
    if (hn) heap[k] = last;
    if ((++pops & 1023) == 0 && __builtin_amdgcn_s_memrealtime() > deadline) {
      write_status(out, si, kPathInternal, n_nodes, n_arcs);
      return;
    }
    const uint32_t s = item.s;
    if (settled[s]) continue;
    if (!(item.d == dist[s])) continue;  // stale entry (:68)
    settled[s] = 1;
    const double ds = dist[s];
    const uint32_t a0 = T.aoff[s], a1 = T.aoff[s + 1];
    for (uint32_t a = a0; a < a1; ++a) {  // :71-84
      const uint32_t x = T.anext[a];
      const double nd = w_times(ds, T.aw[a]);
      const double od = dist[x];
      const unsigned long long b = T.nback[x];
      const uint32_t prev = b == ~0ull ? kNoState : (uint32_t)(b >> 32);
      const bool tie = nd == od && (prev == kNoState || s < prev);
      if (w_is_zero(od) || nd < od || tie) {
        dist[x] = nd;
        T.nback[x] = ((unsigned long long)s << 32) | (a - a0);
        if (!settled[x]) {
          if (hn >= hcap) {  // cannot happen (<= one push per arc per settle + 1)
            write_status(out, si, kPathInternal, n_nodes, n_arcs);
            return;
          }
          uint64_t j = hn++;  // sift up
          const SpHeapEnt e{nd, x, 0};
          while (j > 0) {
            const uint64_t pj = (j - 1) / 2;
            if (!sp_heap_less(e, heap[pj])) break;
            heap[j] = heap[pj];
            j = pj;
          }
          heap[j] = e;
        }
      }
    }
  }
  // best final: lexmin (total, id) over reachable states (:88-104)
  uint32_t best = kNoState;
  double bt = __builtin_huge_val();
  for (uint32_t s = 0; s < n_nodes; ++s) {
    if (w_is_zero(dist[s]) || w_is_zero(T.nfin[s])) continue;
    const double t = w_times(dist[s], T.nfin[s]);
    if (best == kNoState || t < bt) {  // equal totals keep the smaller id
      best = s;
      bt = t;
    }
  }
  if (best == kNoState) {
    write_status(out, si, kPathEmpty, n_nodes, n_arcs);
    return;
  }
  uint32_t cur = best, hops = 0;  // backtrace (:109-122), bounded: a cycle reports CYCLE
  for (;;) {
    const unsigned long long b = T.nback[cur];
    if (b == ~0ull) break;
    if (++hops > n_nodes) {
      write_status(out, si, kPathCycle, n_nodes, n_arcs);
      return;
    }
    cur = (uint32_t)(b >> 32);
  }
  if (cur != start) {
    write_status(out, si, kPathEmpty, n_nodes, n_arcs);
    return;
  }
  const unsigned long long o = reserve_path(out, si, hops);
  if (o + hops > out.arc_cap) {
    write_status(out, si, kPathOutputFull, n_nodes, n_arcs);
    return;
  }
  cur = best;
  for (uint32_t k = hops; k > 0; --k) {
    const unsigned long long b = T.nback[cur];
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


#ifndef FSTAMD_BFS_WAVES64  // waves per SIMD of the one-wavefront instance (config 4 eager:
// 6 waves, 84 B of spills, engine 39.5 ms vs 47.2 ms at 4 waves spill-free; 8: 40.0 ms)
#define FSTAMD_BFS_WAVES64 6
#endif
// The tiny tier: small lattices (config 4's tagger and verbalizer: 43 / 72 tuples per
// utterance on average) keep every table in LDS instead of an HBM slab, so a BFS level
// costs LDS round trips rather than HBM ones, and no string clears a 384 KB HBM hash.
// Strings that outgrow it report OVERFLOW and move on to tier 0.  The caps are the
// host's ws.* values for this tier (device_engine.hip run_bfs_chain).
// Two sizes (config 4's lattices: at most 87 / 159 tuples, 1.0-1.3 arcs per tuple, and up
// to ~150 BFS levels: a verbalizer word is an epsilon chain of 3-5 levels; what outgrows the
// first size finishes in the second rather than in HBM):
// kTiny = 1: 128 tuples / 176 arcs / 256 slots / 256 levels, ~14.6 KB, 10-11 per CU;
// kTiny = 2: 256 tuples / 384 arcs / 512 slots / 512 levels, ~28 KB, 5 per CU.
// Both hold chains of up to 126 labels in LDS.
struct TinyCaps {
  uint32_t n, a, h, l, lab;
};
__host__ __device__ constexpr TinyCaps tiny_caps(int k) {
  return k == 1 ? TinyCaps{128, 176, 256, 256, 128} : TinyCaps{256, 384, 512, 512, 128};
}
constexpr size_t kTinyAlign = 16;
__host__ __device__ constexpr size_t tiny_bytes(int k) {
  return bfs_slab_bytes(tiny_caps(k).n, tiny_caps(k).a, tiny_caps(k).h, tiny_caps(k).l,
                        kTinyAlign);
}
__host__ __device__ constexpr int tiny_waves(int k) { return k == 1 ? 3 : 2; }  // per SIMD
// (A/B on config 4: with the ~3 KB rhs copied into LDS as well a string took 143 / 288 us
// instead of 178 / 338 us, but 6 workgroups fit per CU instead of 8: no faster overall)

template <int WG, bool kGraph, int kTiny = 0>
__global__ void __launch_bounds__(WG, WG == 64 ? (kTiny ? tiny_waves(kTiny) : FSTAMD_BFS_WAVES64) : 1)
eager_bfs_kernel(RhsView rhs, ChainInput in, GraphInput graph, uint32_t n_best,
                 unsigned int* next_item, const uint32_t* items, const uint32_t* num_items_dev,
                 uint32_t num_items_host, BfsWs ws, BatchOutDev out) {
  static_assert(kTiny == 0 || (!kGraph && WG == 64), "the tiny tiers are the chain batch's");
  __shared__ BfsShared SH;
  const uint32_t tid = threadIdx.x;
  BfsTables T;
  [[maybe_unused]] uint32_t* tiny_lab = nullptr;
  constexpr TinyCaps kTC = tiny_caps(kTiny);
  if constexpr (kTiny != 0) {
    __shared__ __attribute__((aligned(16))) uint8_t tiny_slab[tiny_bytes(kTiny)];
    __shared__ uint32_t tiny_labels[kTC.lab];
    T = bfs_carve(tiny_slab, kTC.n, kTC.a, kTC.h, kTC.l, kTinyAlign);
    tiny_lab = tiny_labels;
  } else {
    T = bfs_carve(ws.slab + (size_t)blockIdx.x * ws.stride, ws.ncap, ws.acap, ws.hcap, ws.lcap);
  }
  uint32_t* hdr = ws.hdr + (size_t)blockIdx.x * 8;
  unsigned long long* prof = ws.prof ? ws.prof + (size_t)blockIdx.x * 8 : nullptr;
  const uint32_t num_items = num_items_dev ? *num_items_dev : num_items_host;
  const uint32_t hmask = ws.hcap - 1;

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      SH.item = atomicAdd(next_item, 1u);
      SH.t_item = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t item = SH.item;
    if (item >= num_items) break;
    // the watchdog is per string: each string gets the full limit from its own start,
    // however long the launch has been running (INTERNAL past it)
    const unsigned long long t0 = SH.t_item;
    const uint32_t si = items ? items[item] : item;

    unsigned long long tp = __builtin_amdgcn_s_memrealtime();
    prof_add(prof, 4, 1);
    BfsLhs<kGraph> lhs;
    lhs.g = graph;
    lhs.labels = nullptr;
    lhs.L = 0;
    if constexpr (!kGraph) {
      const uint64_t off = in.offsets[si];
      lhs.labels = in.labels + off;
      lhs.L = (uint32_t)(in.offsets[si + 1] - off);
      if constexpr (kTiny != 0) {  // the labels in LDS; a chain this long needs more levels
        if (lhs.L + 2 > kTC.lab) {
          if (tid == 0) write_status(out, si, kPathOverflow, 0, 0);
          continue;
        }
        for (uint32_t i = tid; i < lhs.L; i += WG) tiny_lab[i] = lhs.labels[i];
        lhs.labels = tiny_lab;
        __syncthreads();
      }
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
      T.nd[0] = okey(w_one());
      T.lvl[0] = 0;
      T.lvl[1] = 1;
      T.aoff[0] = 0;
    }
    __syncthreads();
    uint32_t n_nodes = 1, n_arcs = 0, level = 0;
    int32_t fail = kPathOk;
    if (tid == 0) SH.changed = 0;  // (E) sets it on a backward arc
    __syncthreads();
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
      // (B) write arcs, insert targets (first candidate of a new key wins).  A thread
      // expands its tuples' candidates (arcs, and each target's key parked in anext/cslot),
      // then every thread inserts candidates of the level in parallel: a tuple's dozen
      // hash inserts are no longer a chain of dependent atomics on one thread
      if (tid == 0) SH.flag = 0;
      const uint32_t c0 = n_arcs, c1 = n_arcs + carry;
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
                             T.anext[a] = (uint32_t)(key >> 32);  // (D) overwrites it
                             T.cslot[a] = (uint32_t)key;
                             ++a;
                           });
      }
      __syncthreads();
      for (uint32_t a = c0 + tid; a < c1; a += WG) {
        const unsigned long long key = ((unsigned long long)T.anext[a] << 32) | T.cslot[a];
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
      }
      __syncthreads();
      if (SH.flag) {
        fail = kPathOverflow;
        break;
      }
      // (C) ids of first occurrences, in candidate order (contiguous chunks per thread)
      constexpr uint32_t K = 4;
      uint32_t newc = 0;
      for (uint32_t b = c0; b < c1; b += WG * K) {
        const uint32_t a0 = b + tid * K;
        uint32_t nf = 0, slots[K];
        bool first[K];  // (kept from the count pass: no second round of dependent loads)
#pragma unroll
        for (uint32_t q = 0; q < K; ++q) {
          const uint32_t a = a0 + q;
          slots[q] = a < c1 ? T.cslot[a] : 0u;
          first[q] = a < c1 && ld_agent(&T.hval[slots[q]]) == (0x80000000u | a);
          nf += first[q] ? 1u : 0u;
        }
        uint32_t tot;
        uint32_t rank = block_excl_scan<WG>(nf, SH.scan, tot);
        if ((uint64_t)n_nodes + newc + tot > ws.ncap) {
          SH.flag = 1;  // read after the loop (uniform: every thread sees the same tot)
        } else {
#pragma unroll
          for (uint32_t q = 0; q < K; ++q) {
            {
              const uint32_t slot = slots[q];
              if (first[q]) {
                const uint32_t id = n_nodes + newc + rank++;
                T.hval[slot] = id;
                T.nkey[id] = ld_agent(&T.hkey[slot]);
                T.nd[id] = okey(w_zero());
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
      // (E) relax the level's arcs in level order (exact for a DAG by levels: no arc into
      // this or an earlier level); a backward arc leaves the rest to bfs_fixpoint's sweeps
      if (!ws.lattice_only) {
        __syncthreads();
        bool back = false;
        for (uint32_t p = f0 + tid; p < f1; p += WG) {
          const double ds = from_okey(ld_agent(&T.nd[p]));
          const uint32_t a1 = T.aoff[p + 1];
          for (uint32_t a = T.aoff[p]; a < a1; ++a) {
            const uint32_t x = T.anext[a];
            back |= x < f1;
            if (!w_is_zero(ds)) atomicMin(&T.nd[x], okey(w_times(ds, T.aw[a])));
          }
        }
        if (back) SH.changed = 1;  // reset before the level loop
      }
      n_arcs = c1;
      n_nodes += newc;
      ++level;
      if (tid == 0) T.lvl[level + 1] = n_nodes;
      __syncthreads();
      // the watchdog every 8 levels (a level's work is bounded by its tuples and arcs; the
      // s_memrealtime round trip and its barrier had sat in every level's latency)
      if ((level & 7u) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ws.wd_ticks) {  // uniform per wave...
          if (tid == 0) SH.flag = 1;
        }
        __syncthreads();
        if (SH.flag) {  // ...made uniform for the workgroup through LDS
          fail = kPathInternal;
          break;
        }
      }
    }
    const uint32_t n_levels = level;
    prof_mark(prof, 0, &tp);
    __syncthreads();
    const bool dag = SH.changed == 0;

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

    if (ws.lazy) {
      bfs_lazy_path<WG>(T, ws.ncap, n_nodes, n_arcs, n_levels, 0u, out, si, SH,
                        t0 + ws.wd_ticks, prof, &tp, dag);
      prof_mark(prof, 3, &tp);
    } else if (ws.replay) {
      uint8_t* r = ws.replay + (size_t)blockIdx.x * ((size_t)(ws.acap + 1) * 16 + ws.ncap);
      sp_replay(T, n_nodes, n_arcs, 0u, (SpHeapEnt*)r, (uint64_t)ws.acap + 1,
                r + (size_t)(ws.acap + 1) * 16, out, si, t0 + ws.wd_ticks);
    } else
      bfs_shortest_path<WG>(T, n_nodes, n_arcs, n_levels, 0u, out, si, SH,
                            t0 + ws.wd_ticks, false, dag);
  }
}

// fst_shortest_path on an explicit FST held as a lattice (T.aoff/anext/ail/aol/aw/nfin
// are the FST's own CSR, T.lvl = {0, N}: one "level", Jacobi-style sweeps).
// Distances of fst_shortest_path (weights >= 0) by label correcting over a frontier, one
// workgroup: a round relaxes the out-arcs of the nodes whose distance dropped in the
// previous round (atomicMin on the order-preserving key); a node whose key drops joins the
// next frontier once per round (stamp).  It converges to the least fixpoint, which is
// Dijkstra's distance for weights >= 0, after as many rounds as the
// longest shortest path has arcs, touching only the frontier's arcs: on config 1's lattice
// (781 K states, 10 M arcs, ~4,200 levels) the sweeps over every arc took 34 s.
// A round takes the frontier WG nodes at a time: their spans and distances go to LDS with a
// scan of the out-degrees, then the chunk's ARCS are spread over the threads (binary
// search of the arc's node in LDS), kArcUnroll at a time so that their loads and atomics
// are in flight together.  *expired = 1 when the watchdog stops it.
constexpr int kSpArcUnroll = 4;

template <int WG>
__global__ void __launch_bounds__(WG)
sp_frontier_kernel(BfsTables T, uint32_t n_nodes, uint32_t start, uint32_t* mark,
                   uint32_t* fa, uint32_t* fb, uint32_t* expired, unsigned long long wd_ticks) {
  __shared__ uint32_t cnt[3];
  __shared__ uint32_t stop;
  __shared__ uint32_t scan[16];
  __shared__ uint32_t c_off[WG + 1];   // chunk: first arc (chunk-relative) of each node
  __shared__ uint32_t c_a0[WG];        // its first arc in the graph
  __shared__ double c_ds[WG];          // its distance
  const uint32_t tid = threadIdx.x;
  if (start >= n_nodes) return;
  for (uint32_t i = tid; i < n_nodes; i += WG) {
    T.nd[i] = i == start ? okey(w_one()) : okey(w_zero());
    mark[i] = ~0u;
  }
  if (tid == 0) {
    fa[0] = start;
    cnt[0] = 1;  // round 0's frontier
    cnt[1] = 0;
    cnt[2] = 0;
    stop = 0;
  }
  __syncthreads();
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + wd_ticks;
  uint32_t* cur = fa;
  uint32_t* nxt = fb;
  for (uint32_t r = 0;; ++r) {
    const uint32_t fsize = cnt[r % 3];  // written before the last barrier
    if (fsize == 0 || stop) break;
    // the counter round r + 1 pushes into was last read before the previous barrier
    if (tid == 0) {
      cnt[(r + 1) % 3] = 0;
      if ((r & 63u) == 63u && __builtin_amdgcn_s_memrealtime() > deadline) stop = 1;
    }
    uint32_t* const push = &cnt[(r + 1) % 3];
    for (uint32_t c0 = 0; c0 < fsize; c0 += WG) {
      // (1) the chunk's nodes: span and distance into LDS, out-degree scan
      uint32_t deg = 0;
      const uint32_t q = c0 + tid;
      if (q < fsize) {
        const uint32_t s = ld_agent(&cur[q]);
        const uint32_t a0 = T.aoff[s];
        deg = T.aoff[s + 1] - a0;
        c_a0[tid] = a0;
        c_ds[tid] = from_okey(ld_agent(&T.nd[s]));
      }
      uint32_t total;
      const uint32_t ex = block_excl_scan<WG>(deg, scan, total);  // (its barriers publish LDS)
      c_off[tid] = ex;
      if (tid == 0) c_off[WG] = total;
      const uint32_t nn = min(WG, fsize - c0);
      __syncthreads();
      // (2) the chunk's arcs, kSpArcUnroll per thread at a time
      for (uint32_t b = 0; b < total; b += WG * kSpArcUnroll) {
        uint32_t x[kSpArcUnroll];
        unsigned long long v[kSpArcUnroll];
        bool act[kSpArcUnroll];
#pragma unroll
        for (int u = 0; u < kSpArcUnroll; ++u) {
          const uint32_t i = b + (uint32_t)u * WG + tid;
          act[u] = i < total;
          x[u] = 0;
          v[u] = ~0ull;
          if (act[u]) {
            uint32_t lo = 0, hi = nn;  // the node whose arc range holds i
            while (hi - lo > 1) {
              const uint32_t mid = (lo + hi) >> 1;
              if (c_off[mid] <= i) lo = mid;
              else hi = mid;
            }
            const uint32_t a = c_a0[lo] + (i - c_off[lo]);
            x[u] = T.anext[a];
            v[u] = okey(w_times(c_ds[lo], T.aw[a]));  // shortest-path.zig:72
          }
        }
        unsigned long long old[kSpArcUnroll];
#pragma unroll
        for (int u = 0; u < kSpArcUnroll; ++u)
          old[u] = act[u] ? atomicMin(&T.nd[x[u]], v[u]) : 0ull;
#pragma unroll
        for (int u = 0; u < kSpArcUnroll; ++u)
          if (act[u] && v[u] < old[u] && atomicExch(&mark[x[u]], r) != r)
            nxt[atomicAdd(push, 1u)] = x[u];
      }
      __syncthreads();  // the chunk's LDS is reused by the next one
    }
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (tid == 0 && stop) *expired = 1;
}

// Distances of fst_shortest_path (weights >= 0) settled in distance order, one workgroup:
// every node at the smallest open distance dcur is final (no arc can lower it), so a round
// settles the frontier at dcur and relaxes each settled node's arcs exactly once; targets
// reached at dcur (0-weight arcs) form the next round's frontier, the others go to a
// pending list.  When the frontier is empty the pending list is scanned for the next
// distance (its settled and stale entries dropped).  Unlike label correcting this does no
// rework (config 1's lattice: label correcting took every node 33 times); its cost is one
// pending scan per distinct distance, so after max_adv advances it gives up (*fallback = 1)
// and the host runs sp_frontier_kernel instead.  pend holds at most one entry per arc.
template <int WG>
__global__ void __launch_bounds__(WG)
sp_settle_kernel(BfsTables T, uint32_t n_nodes, uint32_t start, uint32_t* mark, uint32_t* st,
                 uint32_t* fa, uint32_t* fb, uint32_t* pend, uint32_t* flags, uint32_t max_adv,
                 unsigned long long wd_ticks) {
  __shared__ uint32_t cnt[3];
  __shared__ uint32_t stop, pcount;
  __shared__ unsigned long long dmin_s;
  __shared__ uint32_t scan[16];
  __shared__ uint32_t c_off[WG + 1];
  __shared__ uint32_t c_a0[WG];
  const uint32_t tid = threadIdx.x;
  if (start >= n_nodes) return;
  for (uint32_t i = tid; i < n_nodes; i += WG) {
    T.nd[i] = i == start ? okey(w_one()) : okey(w_zero());
    mark[i] = ~0u;
    st[i] = 0;
  }
  if (tid == 0) {
    fa[0] = start;
    cnt[0] = 1;
    cnt[1] = 0;
    cnt[2] = 0;
    stop = 0;
    pcount = 0;
  }
  __syncthreads();
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + wd_ticks;
  unsigned long long dcur = okey(w_one());
  uint32_t* cur = fa;
  uint32_t* nxt = fb;
  uint32_t r = 0, adv = 0, rounds = 0;
  for (;;) {
    // ---- settle rounds at dcur ----
    for (;; ++r) {
      const uint32_t fsize = cnt[r % 3];
      if (fsize == 0 || stop) break;
      ++rounds;
      if (tid == 0) {
        cnt[(r + 1) % 3] = 0;
        if ((rounds & 63u) == 63u && __builtin_amdgcn_s_memrealtime() > deadline) stop = 1;
      }
      uint32_t* const push = &cnt[(r + 1) % 3];
      const double ds = from_okey(dcur);
      for (uint32_t c0 = 0; c0 < fsize; c0 += WG) {
        uint32_t deg = 0;
        const uint32_t q = c0 + tid;
        if (q < fsize) {
          const uint32_t s = ld_agent(&cur[q]);
          if (atomicExch(&st[s], 1u) == 0u) {  // settle s once; its arcs are relaxed once
            const uint32_t a0 = T.aoff[s];
            deg = T.aoff[s + 1] - a0;
            c_a0[tid] = a0;
          }
        }
        uint32_t total;
        const uint32_t ex = block_excl_scan<WG>(deg, scan, total);
        c_off[tid] = ex;
        const uint32_t nn = min(WG, fsize - c0);
        __syncthreads();
        for (uint32_t b = 0; b < total; b += WG * kSpArcUnroll) {
          uint32_t x[kSpArcUnroll];
          unsigned long long v[kSpArcUnroll];
          bool act[kSpArcUnroll];
#pragma unroll
          for (int u = 0; u < kSpArcUnroll; ++u) {
            const uint32_t i = b + (uint32_t)u * WG + tid;
            act[u] = i < total;
            x[u] = 0;
            v[u] = ~0ull;
            if (act[u]) {
              uint32_t lo = 0, hi = nn;
              while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (c_off[mid] <= i) lo = mid;
                else hi = mid;
              }
              const uint32_t a = c_a0[lo] + (i - c_off[lo]);
              x[u] = T.anext[a];
              v[u] = okey(w_times(ds, T.aw[a]));  // shortest-path.zig:72
            }
          }
          unsigned long long old[kSpArcUnroll];
#pragma unroll
          for (int u = 0; u < kSpArcUnroll; ++u)
            old[u] = act[u] ? atomicMin(&T.nd[x[u]], v[u]) : 0ull;
#pragma unroll
          for (int u = 0; u < kSpArcUnroll; ++u) {
            if (!act[u] || !(v[u] < old[u])) continue;
            if (v[u] == dcur) {  // reached at dcur: settled next round
              if (atomicExch(&mark[x[u]], r) != r) nxt[atomicAdd(push, 1u)] = x[u];
            } else {
              pend[atomicAdd(&pcount, 1u)] = x[u];
            }
          }
        }
        __syncthreads();
      }
      uint32_t* t = cur;
      cur = nxt;
      nxt = t;
    }
    if (stop) break;
    // ---- advance: the smallest open distance among the pending entries ----
    const uint32_t pn = pcount;
    unsigned long long m = ~0ull;
    for (uint32_t i = tid; i < pn; i += WG) {
      const uint32_t x = ld_agent(&pend[i]);
      if (ld_agent(&st[x]) == 0u) {
        const unsigned long long d = ld_agent(&T.nd[x]);
        m = d < m ? d : m;
      }
    }
    if (tid == 0) dmin_s = ~0ull;
    __syncthreads();
    if (m != ~0ull) atomicMin(&dmin_s, m);
    __syncthreads();
    const unsigned long long dmin = dmin_s;
    if (dmin == ~0ull || dmin == okey(w_zero())) break;  // nothing open: done
    if (++adv > max_adv) {
      if (tid == 0) flags[0] = 1;  // fallback: label correcting
      return;
    }
    // entries at dmin -> the frontier (once per node), the rest stay (compacted in place)
    ++r;
    if (tid == 0) {
      cnt[r % 3] = 0;
      cnt[(r + 1) % 3] = 0;
    }
    __syncthreads();
    uint32_t kept = 0;
    for (uint32_t c0 = 0; c0 < pn; c0 += WG) {
      const uint32_t i = c0 + tid;
      uint32_t x = 0, keep = 0;
      if (i < pn) {
        x = ld_agent(&pend[i]);
        if (ld_agent(&st[x]) == 0u) {
          if (ld_agent(&T.nd[x]) == dmin) {
            if (atomicExch(&mark[x], r) != r) cur[atomicAdd(&cnt[r % 3], 1u)] = x;
          } else {
            keep = 1;
          }
        }
      }
      uint32_t tot;
      const uint32_t rank = block_excl_scan<WG>(keep, scan, tot);  // reads done: barrier
      if (keep) pend[kept + rank] = x;  // kept + rank <= c0 + tid: never an unread entry
      kept += tot;
    }
    if (tid == 0) pcount = kept;
    dcur = dmin;
    __syncthreads();
  }
  if (tid == 0) {
    if (stop) flags[1] = 1;
    flags[2] = rounds;
    flags[3] = adv;
  }
}

template <int WG>
__global__ void __launch_bounds__(WG)
sp_graph_kernel(BfsTables T, uint32_t n_nodes, uint32_t start, uint32_t n_best, BatchOutDev out,
                unsigned long long wd_ticks, const uint32_t* have_dist) {
  __shared__ BfsShared SH;
  if (start == kNoState || n_best == 0 || n_nodes == 0) {  // shortest-path.zig:21-23
    if (threadIdx.x == 0) write_status(out, 0, kPathEmpty, 0, 0);
    return;
  }
  if (n_best != 1) {  // :24
    if (threadIdx.x == 0) write_status(out, 0, kPathErrorN, 0, 0);
    return;
  }
  // have_dist: sp_frontier_kernel left the distances in T.nd ([1]: its watchdog fired)
  if (have_dist && have_dist[1]) {
    if (threadIdx.x == 0) write_status(out, 0, kPathInternal, n_nodes, T.aoff[n_nodes]);
    return;
  }
  bfs_shortest_path<WG>(T, n_nodes, T.aoff[n_nodes], 1u, start, out, 0u, SH,
                        __builtin_amdgcn_s_memrealtime() + wd_ticks, !have_dist, have_dist != nullptr);
}

__global__ void __launch_bounds__(64)
sp_replay_kernel(BfsTables T, uint32_t n_nodes, uint32_t start, uint32_t n_best,
                 SpHeapEnt* heap, uint64_t hcap, uint8_t* settled, BatchOutDev out,
                 unsigned long long wd_ticks) {
  if (start == kNoState || n_best == 0 || n_nodes == 0) {  // :21-23
    if (threadIdx.x == 0) write_status(out, 0, kPathEmpty, 0, 0);
    return;
  }
  if (n_best != 1) {  // :24
    if (threadIdx.x == 0) write_status(out, 0, kPathErrorN, 0, 0);
    return;
  }
  sp_replay(T, n_nodes, T.aoff[n_nodes], start, heap, hcap, settled, out, 0u,
            __builtin_amdgcn_s_memrealtime() + wd_ticks);
}

}  // namespace fstamd
