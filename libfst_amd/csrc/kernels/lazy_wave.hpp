// lazy_wave.hpp -- batched composeShortestPath (FST_SEM_LAZY), exact replay.
//
// Replaces src/ops/compose-shortest-path.zig:26-401 (and the arcsByIlabel inner
// loop src/fst.zig:112-136) for many lhs at once: one wavefront per string.
//
// The lazy algorithm's answer depends on the id each product tuple receives at
// FIRST TOUCH (getOrCreate, :70-89) in Dijkstra pop order, so it is replayed
// exactly rather than re-derived:
//  * priority queue: a 64-ary min-heap on (dist, id) in HBM; pop = one coalesced
//    64-child load + a wave argmin per level.  Pop order equals the reference's
//    binary heap with lazy deletion because (dist, id) is a total order and stale
//    or settled entries are skipped identically (:159-163).
//  * one pop's candidates (4 fixed phases, :181-365) are enumerated across lanes in
//    reference order, 64 at a time; hash lookups run in parallel; NEW tuples get
//    ids by first occurrence in lane order (ballot + popcount), exactly getOrCreate.
//  * relaxations that hit the same tuple inside a chunk are folded in lane order
//    by the group's first lane with the reference rule (:110-128), which is the
//    sequential result; one push per (pop, tuple) is equivalent to the
//    reference's push-per-take because earlier entries become stale.
//  * a candidate that targets the popped tuple itself (self-loop) switches the
//    chunk to a one-lane sequential path, since it may rewrite dist[curr].
#pragma once

#include "device_common.hpp"

extern "C" __device__ double __ockl_wfred_min_f64(double);
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

namespace fstamd {

struct LazyWs {
  uint4* hslot;                  // [waves * hcap] {key lo, key hi, id, stamp}
  unsigned long long* nkey;      // [waves * ncap] (s2 << 32) | (s1 << 2) | filter
  double* ndist;                 // [waves * ncap]
  uint4* nback;                  // [waves * ncap] {prev, ilabel, olabel, flags}
  double* nbw;                   // [waves * ncap] back-pointer edge weight
  double* qd;                    // [waves * qcap] heap dist
  uint32_t* qid;                 // [waves * qcap] heap id
  uint4* gscratch;               // [waves * gcap] graph-lhs enumeration table
  uint32_t hcap, ncap, qcap, gcap;
  uint32_t stamp_base;
  uint32_t max_pops;             // hard bound per string: pops <= pushes <= qcap
  unsigned long long wd_ticks;   // wall-clock watchdog (s_memrealtime, 100 MHz ticks)
  uint32_t* dbg;                 // optional [waves * 8] diagnostics, may be null
};

// Every loop of the kernel polls this: no input, bug or corruption can keep a
// wave resident longer than wd_ticks.
__device__ __forceinline__ bool wd_expired(unsigned long long t0, unsigned long long lim) {
  return __builtin_amdgcn_s_memrealtime() - t0 > lim;
}

constexpr uint32_t kSettled = 1u;
constexpr uint32_t kHasBack = 2u;

// The kernel runs one wavefront per workgroup and all of a string's state is
// private to that wave.  A wave's vector memory and LDS operations execute in
// program order, so its own stores are visible to its later loads (LLVM AMDGPU
// memory model: wavefront scope needs no cache or counter synchronisation).  The
// fence below therefore only stops the compiler from reordering accesses across
// phases -- no s_waitcnt for store acknowledgements on the critical path.
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ unsigned long long tuple_key(uint32_t s1, uint32_t s2, uint32_t f) {
  return ((unsigned long long)s2 << 32) | ((unsigned long long)s1 << 2) | f;
}
__device__ __forceinline__ uint32_t hmix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

// (dist, id) order of queueCompare (compose-shortest-path.zig:55-61); NaN out of contract.
__device__ __forceinline__ bool qless(double da, uint32_t ia, double db, uint32_t ib) {
  return da < db || (da == db && ia < ib);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ unsigned long long lanemask_lt() {
  const uint32_t l = lane_id();
  return l ? (~0ull >> (64 - l)) : 0ull;
}

// ---- lhs accessors -------------------------------------------------------------

// One linear-chain acceptor of the batch (src/string.zig:24-50 semantics).
struct ChainLhs {
  const uint32_t* labels;
  uint32_t L;
  __device__ uint32_t start() const { return 0; }
  __device__ double final_w(uint32_t s1) const { return s1 == L ? w_one() : w_zero(); }
};

// Per-pop candidate enumeration state, uniform across the wave.
struct PopCands {
  uint32_t s1, s2, f;
  uint32_t n1, n2, n3, n4;   // phase sizes
  uint32_t lo1, lo3;         // chain: phase-1 span start, rhs-epsilon span start
  uint32_t label;            // chain: the lhs arc label (if s1 < L)
  uint32_t deg;              // graph: lhs out-degree of s1
  uint32_t e_cnt;            // graph: number of epsilon-output lhs arcs
};

struct Cand {
  unsigned long long key;
  uint32_t il, ol;
  double w;
};

// Chain: phase sizes in closed form (at most one lhs arc per state).
__device__ __forceinline__ void prepare_chain(const RhsView& rhs, const ChainLhs& lhs,
                                              PopCands& P) {
  const bool has_arc = P.s1 < lhs.L;
  P.label = has_arc ? lhs.labels[P.s1] : 0u;
  // arcsByIlabel for the epsilon and the label runs of the (wave-uniform) popped state:
  // up to 64 arcs, every lane reads one ilabel and both runs come from ballots (one round
  // trip; ilabels ascending, epsilon = 0 first); beyond, the binary searches
  // (the state summary first: a state whose arcs share one ilabel -- most of a tagger's
  // -- needs no ilabel loads, so its arc records are the next and last round trip)
  const uint4 ss = rhs.sspan[FB(P.s2, rhs.num_states, 30)];
  const uint32_t off = ss.x, n = ss.y;
  uint32_t lo3, hi3, lo1 = 0, hi1 = 0;
  if (ss.z != kSpanMixed) {  // one ilabel (or no arc)
    const bool eps = ss.z == kEpsilon;
    lo3 = off;
    hi3 = eps ? off + n : off;
    lo1 = off;
    hi1 = !eps && ss.z == P.label ? off + n : off;
  } else if (n <= 64) {
    const uint32_t lane = lane_id();
    const bool v = lane < n;
    const uint32_t x = v ? rhs.il[FB(off + lane, rhs.num_arcs, 2)] : 0u;
    lo3 = off;
    hi3 = off + (uint32_t)__popcll(__ballot(v && x == kEpsilon));
    lo1 = off + (uint32_t)__popcll(__ballot(v && x < P.label));
    hi1 = off + (uint32_t)__popcll(__ballot(v && x <= P.label));
  } else {  // many arcs: the leading epsilon run from the summary, the label's run counted
    lo3 = off;
    hi3 = off + ss.w;
    if (has_arc && P.label != kEpsilon) wave_span_by_ilabel(rhs, off, n, P.label, lo1, hi1);
  }
  P.lo3 = lo3;
  const uint32_t ne = hi3 - lo3;
  P.n1 = 0;
  P.lo1 = 0;
  if (has_arc && P.label != kEpsilon) {  // :182-224
    P.lo1 = lo1;
    P.n1 = hi1 - lo1;
  }
  P.n2 = (has_arc && P.label == kEpsilon && P.f != 1) ? 1u : 0u;       // :227-252
  P.n3 = (P.f != 2) ? ne : 0u;                                          // :254-305
  P.n4 = (has_arc && P.label == kEpsilon && P.f == 0) ? ne : 0u;       // :307-365
}

__device__ __forceinline__ Cand chain_cand(const RhsView& rhs, const PopCands& P, uint32_t c) {
  Cand x;
  if (c < P.n1) {
    const ArcRec r = rhs.rec[P.lo1 + c];
    x.key = tuple_key(P.s1 + 1, r.next, 0);
    x.il = P.label;
    x.ol = r.olabel;
    x.w = w_times(w_one(), r.weight);
    return x;
  }
  c -= P.n1;
  if (c < P.n2) {
    x.key = tuple_key(P.s1 + 1, P.s2, P.f == 0 ? 2u : P.f);
    x.il = P.label;
    x.ol = kEpsilon;
    x.w = w_one();
    return x;
  }
  c -= P.n2;
  if (c < P.n3) {
    const ArcRec r = rhs.rec[P.lo3 + c];
    x.key = tuple_key(P.s1, r.next, P.f == 0 ? 1u : P.f);
    x.il = kEpsilon;
    x.ol = r.olabel;
    x.w = r.weight;
    return x;
  }
  c -= P.n3;
  const ArcRec r = rhs.rec[P.lo3 + c];
  x.key = tuple_key(P.s1 + 1, r.next, 0);
  x.il = P.label;
  x.ol = r.olabel;
  x.w = w_times(w_one(), r.weight);
  return x;
}

// Graph: per-pop table over the lhs arcs of s1 in gscratch:
//   tbl[i] = {phase-1 base, phase-1 span lo, phase-1 count, arc index} for i < deg
//   tbl[deg + e].w = arc index of the e-th epsilon-output lhs arc.
__device__ void prepare_graph(const RhsView& rhs, const GraphInput& g, uint4* tbl, PopCands& P) {
  const uint32_t a0 = g.state_off[P.s1];
  P.deg = g.state_off[P.s1 + 1] - a0;
  uint32_t base1 = 0, ebase = 0;
  for (uint32_t i0 = 0; i0 < P.deg; i0 += 64) {
    const uint32_t i = i0 + lane_id();
    const bool v = i < P.deg;
    uint32_t lo = 0, cnt = 0;
    bool eps_out = false;
    if (v) {
      const uint32_t ol = g.arc_ol[a0 + i];
      eps_out = ol == kEpsilon;
      if (!eps_out) {
        uint32_t hi;
        span_by_ilabel(rhs, P.s2, ol, lo, hi);
        cnt = hi - lo;
      }
    }
    const uint32_t inc = wave_incl_scan(cnt);
    const unsigned long long em = __ballot(v && eps_out);
    const uint32_t erank = __popcll(em & lanemask_lt());
    if (v) {
      tbl[i] = make_uint4(base1 + inc - cnt, lo, cnt, a0 + i);
      if (eps_out) tbl[P.deg + ebase + erank].w = a0 + i;
    }
    base1 += __shfl(inc, 63, 64);
    ebase += __popcll(em);
  }
  wave_fence();
  uint32_t lo3, hi3;
  span_by_ilabel(rhs, P.s2, kEpsilon, lo3, hi3);
  P.lo3 = lo3;
  const uint32_t ne = hi3 - lo3;
  P.e_cnt = ebase;
  P.n1 = base1;
  P.n2 = (P.f != 1) ? ebase : 0u;
  P.n3 = (P.f != 2) ? ne : 0u;
  P.n4 = (P.f == 0) ? ebase * ne : 0u;
}

__device__ __forceinline__ Cand graph_cand(const RhsView& rhs, const GraphInput& g,
                                           const uint4* tbl, const PopCands& P, uint32_t c) {
  Cand x;
  if (c < P.n1) {  // find the lhs arc whose phase-1 range holds c
    uint32_t a = 0, b = P.deg;
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (tbl[m].x <= c) a = m;
      else b = m;
    }
    while (tbl[a].z == 0 || c >= tbl[a].x + tbl[a].z) ++a;  // skip empty ranges
    const uint4 t = tbl[a];
    const ArcRec r = rhs.rec[t.y + (c - t.x)];
    x.key = tuple_key(g.arc_next[t.w], r.next, 0);
    x.il = g.arc_il[t.w];
    x.ol = r.olabel;
    x.w = w_times(g.arc_w[t.w], r.weight);
    return x;
  }
  c -= P.n1;
  if (c < P.n2) {
    const uint32_t ai = tbl[P.deg + c].w;
    x.key = tuple_key(g.arc_next[ai], P.s2, P.f == 0 ? 2u : P.f);
    x.il = g.arc_il[ai];
    x.ol = kEpsilon;
    x.w = g.arc_w[ai];
    return x;
  }
  c -= P.n2;
  if (c < P.n3) {
    const ArcRec r = rhs.rec[P.lo3 + c];
    x.key = tuple_key(P.s1, r.next, P.f == 0 ? 1u : P.f);
    x.il = kEpsilon;
    x.ol = r.olabel;
    x.w = r.weight;
    return x;
  }
  c -= P.n3;
  const uint32_t ne = P.n3 ? P.n3 : (P.n4 / (P.e_cnt ? P.e_cnt : 1));
  const uint32_t ai = tbl[P.deg + c / ne].w;
  const ArcRec r = rhs.rec[P.lo3 + c % ne];
  x.key = tuple_key(g.arc_next[ai], r.next, 0);
  x.il = g.arc_il[ai];
  x.ol = r.olabel;
  x.w = w_times(g.arc_w[ai], r.weight);
  return x;
}

// ---- the kernel ----------------------------------------------------------------

struct LazyLds {
  double nd[64];
  double w[64];
  uint32_t il[64];
  uint32_t ol[64];
  uint32_t id[64];
};

#ifndef FSTAMD_REPLAY_WAVES  // waves per SIMD of the hashed replay (config 4 lazy: 4 spill-free
// 18.4 ms per call, 6 and 8 with spills 20.4 ms)
#define FSTAMD_REPLAY_WAVES 4
#endif
// LDS sizes of the LDS replay (kernels/lazy_tiny.hpp): size t holds 64 << t tuples.
constexpr uint32_t lz_tiny_n(int t) { return 64u << t; }

template <bool kGraph>
__global__ void __launch_bounds__(64, FSTAMD_REPLAY_WAVES)
lazy_wave_kernel(RhsView rhs, ChainInput chain, GraphInput graph, uint32_t n_best,
                 unsigned int* next_item, const uint32_t* items, uint32_t num_items, LazyWs ws,
                 BatchOutDev out) {
  __shared__ LazyLds S;
  const uint32_t lane = lane_id();
  const size_t w = blockIdx.x;
  uint4* const hslot = ws.hslot + w * ws.hcap;
  unsigned long long* const nkey = ws.nkey + w * ws.ncap;
  double* const ndist = ws.ndist + w * ws.ncap;
  uint4* const nback = ws.nback + w * ws.ncap;
  double* const nbw = ws.nbw + w * ws.ncap;
  double* const qd = ws.qd + w * ws.qcap;
  uint32_t* const qid = ws.qid + w * ws.qcap;
  uint4* const tbl = ws.gscratch + w * ws.gcap;
  const uint32_t hmask = ws.hcap - 1;
  // per-string watchdog: both are reset when a string starts, so every string gets the
  // full limit however long the launch has been running
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool dead = false;  // watchdog fired for the current string: it reports INTERNAL
  uint32_t dbg_pops = 0, dbg_cb = 0, dbg_C = 0, dbg_qn = 0, dbg_nn = 0;
#define LZ_WD(code)                                                                  \
  if (!dead && wd_expired(t0, ws.wd_ticks)) {                                        \
    dead = true;                                                                     \
    if (ws.dbg && lane == 0) {                                                       \
      uint32_t* d_ = ws.dbg + w * 8;                                                 \
      d_[0] = (code);                                                                \
      d_[1] = dbg_pops;                                                              \
      d_[2] = dbg_cb;                                                                \
      d_[3] = dbg_C;                                                                 \
      d_[4] = dbg_qn;                                                                \
      d_[5] = dbg_nn;                                                                \
    }                                                                                \
  }

  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(next_item, 1u);
    item = __shfl(item, 0, 64);
    if (item >= num_items) break;
    const uint32_t si = items ? items[item] : item;
    t0 = __builtin_amdgcn_s_memrealtime();
    dead = false;
    const uint32_t stamp = ws.stamp_base + item + 1;

    ChainLhs cl{nullptr, 0};
    uint32_t start1;
    if constexpr (kGraph) {
      start1 = graph.start;
    } else {
      const uint64_t off = chain.offsets[si];
      cl.labels = chain.labels + off;
      cl.L = (uint32_t)(chain.offsets[si + 1] - off);
      start1 = 0;
    }
    auto lhs_final = [&](uint32_t s1) -> double {
      if constexpr (kGraph) return graph.final_w[s1];
      else return cl.final_w(s1);
    };

    // compose-shortest-path.zig:30-33
    if (start1 == kNoState || rhs.start == kNoState || n_best == 0 || n_best != 1) {
      if (lane == 0) {
        const bool empty = start1 == kNoState || rhs.start == kNoState || n_best == 0;
        out.status[si] = empty ? kPathEmpty : kPathErrorN;
        out.path_len[si] = 0;
        out.path_off[si] = 0;
        out.final_w[si] = w_zero();
        if (out.work) {
          out.work[2 * si] = 0;
          out.work[2 * si + 1] = 0;
        }
      }
      continue;
    }

    // init tuple, id 0 (:146-153)
    uint32_t nn = 1, qn = 1;
    if (lane == 0) {
      const unsigned long long k0 = tuple_key(start1, rhs.start, 0);
      nkey[0] = k0;
      ndist[0] = w_one();
      nback[0] = make_uint4(0, 0, 0, 0);
      uint32_t h = hmix(k0) & hmask;
      hslot[h] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), 0u, stamp);
      qd[0] = w_one();
      qid[0] = 0;
    }
    wave_fence();

    uint32_t best_id = kNoState;
    double best_fw = w_zero(), best_total = w_zero();
    uint32_t relax_count = 0;
    int32_t fail = kPathOk;

    uint32_t pops = 0, pushes = 1;
    uint32_t wd_work = 256;  // candidates since the last watchdog read (read at once)
    while (qn > 0) {
      dbg_pops = pops;
      dbg_qn = qn;
      dbg_nn = nn;
      // the watchdog once per ~256 candidates (16 pops of 16; a pop with more candidates
      // also reads it every 64 chunks below): an s_memrealtime round trip per inner loop
      // iteration had sat on the pop's critical path, and the loops inside one chunk
      // (sift-down, dedup, grouping: at most the heap depth or 64 iterations) need none
      if (wd_work >= 256u) {
        wd_work = 0;
        LZ_WD(1);
      }
      if (dead || ++pops > ws.max_pops) {  // a heap yields only as many items as were pushed
        fail = kPathInternal;
        break;
      }
      // ---- pop (64-ary heap, wave-cooperative sift-down) ----
      const double pd = qd[0];
      const uint32_t pid = qid[0];
      --qn;
      if (qn > 0) {
        const double xd = qd[qn];
        const uint32_t xi = qid[qn];
        uint32_t i = 0;
        for (;;) {
          const uint32_t c0 = i * 64 + 1;
          if (c0 >= qn) break;
          const uint32_t cc = c0 + lane;
          const bool v = cc < qn;
          const double cd = v ? qd[cc] : 0.0;
          const uint32_t ci = v ? qid[cc] : 0u;
          // the minimum child by (dist, id), duplicates of one (dist, id) (an equal-dist tie
          // takes push again) by heap position: three DPP reductions (min dist, then min id
          // among those, then min position), the winner's exact dist read from its lane
          // (-0.0 == +0.0 as in qless); lane 0 (child c0 < qn) is always valid
          const double dmn = __ockl_wfred_min_f64(v ? cd : __builtin_huge_val());
          const bool c1 = v && cd == dmn;
          const uint32_t mi = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_u32(c1 ? ci : ~0u));
          const uint32_t mp = __builtin_amdgcn_readfirstlane(
              __ockl_wfred_min_u32(c1 && ci == mi ? cc : ~0u));
          const uint32_t wl = mp - c0;
          const unsigned long long cb = (unsigned long long)__double_as_longlong(cd);
          const double md = __longlong_as_double(
              (long long)(((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(cb >> 32), wl) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((uint32_t)cb, wl)));
          // all lanes now hold the minimum child
          if (qless(md, mi, xd, xi)) {
            if (lane == 0) {
              qd[i] = md;
              qid[i] = mi;
            }
            i = mp;
          } else {
            break;
          }
        }
        if (lane == 0) {
          qd[i] = xd;
          qid[i] = xi;
        }
      }
      wave_fence();

      if (pid >= nn) {  // cannot happen on a consistent heap; never spin on garbage
        fail = kPathInternal;
        break;
      }
      // ---- settled / stale (:161-163) ----
      const uint4 pb = nback[pid];
      const double pdist = ndist[pid];
      if (pb.w & kSettled) continue;
      if (!(pd == pdist)) continue;
      if (lane == 0) nback[pid].w = pb.w | kSettled;
      const unsigned long long pk = nkey[pid];
      PopCands P;
      P.s1 = (uint32_t)(pk & 0xFFFFFFFFull) >> 2;
      P.f = (uint32_t)pk & 3u;
      P.s2 = (uint32_t)(pk >> 32);
      if (P.s2 >= rhs.num_states) {  // invariant guard (see pid check above)
        fail = kPathInternal;
        break;
      }

      // ---- best final (:165-179) ----
      const double fw1 = lhs_final(P.s1);
      const double fw2 = rhs.final_w[P.s2];
      if (!w_is_zero(fw1) && !w_is_zero(fw2)) {
        const double fw = w_times(fw1, fw2);
        const double total = w_times(pdist, fw);
        if (best_id == kNoState || total < best_total || (total == best_total && pid < best_id)) {
          best_id = pid;
          best_fw = fw;
          best_total = total;
        }
      }

      // ---- candidates of the 4 phases in reference order ----
      if constexpr (kGraph) prepare_graph(rhs, graph, tbl, P);
      else prepare_chain(rhs, cl, P);
      const uint32_t C = P.n1 + P.n2 + P.n3 + P.n4;
      relax_count += C;
      wd_work += C + 16u;
      double cur_dist = pdist;  // dist[curr_id]; changes only through a self-loop

      dbg_C = C;
      for (uint32_t cb = 0; cb < C; cb += 64) {
        dbg_cb = cb;
        if (cb != 0 && (cb & 4095u) == 0) {
          LZ_WD(2);
        }
        if (dead) {
          fail = kPathInternal;
          break;
        }
        const uint32_t c = cb + lane;
        const bool act = c < C;
        Cand x{0, 0, 0, 0.0};
        if (act) {
          if constexpr (kGraph) x = graph_cand(rhs, graph, tbl, P, c);
          else x = chain_cand(rhs, P, c);
        }
        // lookup (getOrCreate's get)
        uint32_t tid = kNoState;
        uint32_t slot = hmix(x.key) & hmask;
        if (act) {
          for (uint32_t probe = 0; probe <= hmask; ++probe) {
            const uint4 s = hslot[slot];
            if (s.w != stamp) break;
            if (s.x == (uint32_t)x.key && s.y == (uint32_t)(x.key >> 32)) {
              tid = s.z;
              break;
            }
            slot = (slot + 1) & hmask;
          }
        }
        // first-occurrence dedup of new tuples in lane order
        bool need = act && tid == kNoState;
        uint32_t leader = lane;
        unsigned long long pending = __ballot(need);
        while (pending) {
          const uint32_t l = (uint32_t)__ffsll((long long)pending) - 1;
          const unsigned long long lk =
              ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(x.key >> 32), l) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((uint32_t)x.key, l);
          const bool same = need && x.key == lk;
          const unsigned long long m = __ballot(same);
          if (same) leader = l;
          pending &= ~m;
        }
        const bool is_new_leader = need && leader == lane;
        const unsigned long long nlm = __ballot(is_new_leader);
        const uint32_t n_new = (uint32_t)__popcll(nlm);
        if (nn + n_new > ws.ncap || 2 * (nn + n_new) > ws.hcap) {
          fail = kPathOverflow;
          break;
        }
        if (is_new_leader) {
          tid = nn + (uint32_t)__popcll(nlm & lanemask_lt());
          // claim a slot (the table is private to this wave)
          uint32_t s = slot;
          for (uint32_t probe = 0; probe <= hmask; ++probe) {  // load <= 1/2: always ends
            const uint32_t old = atomicExch(&hslot[s].w, stamp);
            if (old != stamp) break;
            s = (s + 1) & hmask;
          }
          hslot[s] = make_uint4((uint32_t)x.key, (uint32_t)(x.key >> 32), tid, stamp);
          nkey[tid] = x.key;
          ndist[tid] = w_zero();
          nback[tid] = make_uint4(0, 0, 0, 0);
        }
        const uint32_t lt = __shfl(tid, (int)leader, 64);
        if (need) tid = lt;
        nn += n_new;
        wave_fence();

        // self-loop onto the popped tuple: rare, exact one-lane path
        const unsigned long long selfm = __ballot(act && tid == pid);
        if (selfm) {
          S.id[lane] = tid;
          S.w[lane] = x.w;
          S.il[lane] = x.il;
          S.ol[lane] = x.ol;
          wave_fence();
          const uint32_t cnt = C - cb < 64 ? C - cb : 64;
          if (lane == 0) {
            for (uint32_t i = 0; i < cnt; ++i) {
              const uint32_t t = S.id[i];
              const double nd = w_times(cur_dist, S.w[i]);
              const double od = ndist[t];
              uint4 b = nback[t];
              bool take = w_is_zero(od) || nd < od;
              if (!take && nd == od) {
                take = !(b.w & kHasBack) || pid < b.x ||
                       (pid == b.x && (S.il[i] < b.y || (S.il[i] == b.y && S.ol[i] < b.z)));
              }
              if (take) {
                ndist[t] = nd;
                nbw[t] = S.w[i];
                nback[t] = make_uint4(pid, S.il[i], S.ol[i], b.w | kHasBack);
                if (t == pid) cur_dist = nd;
                if (!(b.w & kSettled)) {
                  if (qn >= ws.qcap) {
                    fail = kPathOverflow;
                  } else {  // push + sift-up
                    uint32_t q = qn++;
                    ++pushes;
                    while (q > 0) {
                      const uint32_t pq = (q - 1) >> 6;
                      const double qpd = qd[pq];
                      const uint32_t qpi = qid[pq];
                      if (!qless(nd, t, qpd, qpi)) break;
                      qd[q] = qpd;
                      qid[q] = qpi;
                      q = pq;
                    }
                    qd[q] = nd;
                    qid[q] = t;
                  }
                }
              }
            }
          }
          cur_dist = __shfl(cur_dist, 0, 64);
          qn = __shfl(qn, 0, 64);
          fail = __shfl(fail, 0, 64);
          wave_fence();
          if (fail != kPathOk) break;
          continue;
        }

        // group by target: the first lane of each group folds its members in lane order
        const double nd = w_times(cur_dist, x.w);
        S.nd[lane] = nd;
        S.w[lane] = x.w;
        S.il[lane] = x.il;
        S.ol[lane] = x.ol;
        S.id[lane] = act ? tid : kNoState;
        wave_fence();
        unsigned long long gmask = 0;
        {
          unsigned long long pend = __ballot(act);
          while (pend) {
            const uint32_t l = (uint32_t)__ffsll((long long)pend) - 1;
            const uint32_t lt2 = __builtin_amdgcn_readlane(tid, l);
            const bool same = act && tid == lt2;
            const unsigned long long m = __ballot(same);
            if (lane == l) gmask = m;
            pend &= ~m;
          }
        }
        bool push = false;
        double push_d = 0.0;
        if (gmask) {  // group leader
          const uint32_t t = tid;
          double od = ndist[t];
          uint4 b = nback[t];
          double bw = 0.0;
          bool took = false;
          unsigned long long m = gmask;
          while (m) {
            const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
            m &= m - 1;
            const double cnd = S.nd[i];
            const uint32_t cil = S.il[i], col = S.ol[i];
            bool take = w_is_zero(od) || cnd < od;
            if (!take && cnd == od) {
              take = !(b.w & kHasBack) || pid < b.x ||
                     (pid == b.x && (cil < b.y || (cil == b.y && col < b.z)));
            }
            if (take) {
              od = cnd;
              b = make_uint4(pid, cil, col, b.w | kHasBack);
              bw = S.w[i];
              took = true;
            }
          }
          if (took) {
            ndist[t] = od;
            nback[t] = b;
            nbw[t] = bw;
            if (!(b.w & kSettled)) {
              push = true;
              push_d = od;
            }
          }
        }
        wave_fence();
        // pushes in lane order, one lane at a time (sift-up is short in practice)
        unsigned long long pm = __ballot(push);
        while (pm) {
          const uint32_t l = (uint32_t)__ffsll((long long)pm) - 1;
          pm &= pm - 1;
          const unsigned long long pb2 = (unsigned long long)__double_as_longlong(push_d);
          const double xd = __longlong_as_double(
              (long long)(((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(pb2 >> 32), l) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((uint32_t)pb2, l)));
          const uint32_t xi = __builtin_amdgcn_readlane(tid, l);
          if (qn >= ws.qcap) {
            fail = kPathOverflow;
            break;
          }
          if (lane == 0) {
            uint32_t q = qn;
            while (q > 0) {
              const uint32_t pq = (q - 1) >> 6;
              const double qpd = qd[pq];
              const uint32_t qpi = qid[pq];
              if (!qless(xd, xi, qpd, qpi)) break;
              qd[q] = qpd;
              qid[q] = qpi;
              q = pq;
            }
            qd[q] = xd;
            qid[q] = xi;
          }
          ++qn;
          ++pushes;
        }
        wave_fence();
        if (fail != kPathOk) break;
      }
      if (fail != kPathOk) break;
    }

    // ---- result (:368-400) ----
    if (lane == 0) {
      int32_t st = fail;
      uint32_t P = 0;
      unsigned long long o = 0;
      double fin = w_zero();
      if (st == kPathOk) {
        if (best_id == kNoState) {
          st = kPathEmpty;
        } else {
          uint32_t cur = best_id;
          bool empty = false;
          while (cur != 0) {  // init_id == 0
            const uint4 b = nback[cur];
            if (!(b.w & kHasBack)) {
              empty = true;
              break;
            }
            if (++P > nn) {
              st = kPathCycle;
              break;
            }
            cur = b.x;
          }
          if (st == kPathOk && empty) {
            st = kPathEmpty;
            P = 0;
          }
          if (st == kPathOk) {
            o = reserve_path(out, si, P);
            if (o + P > out.arc_cap) {
              st = kPathOutputFull;
            } else {
              uint32_t k = P;
              cur = best_id;
              while (cur != 0) {
                const uint4 b = nback[cur];
                --k;
                out.out_il[o + k] = b.y;
                out.out_ol[o + k] = b.z;
                out.out_w[o + k] = nbw[cur];
                cur = b.x;
              }
              fin = best_fw;
            }
          }
        }
      }
      if (st != kPathOk) {
        P = 0;
        o = 0;
        fin = w_zero();
      }
      out.status[si] = st;
      out.path_len[si] = st == kPathInternal ? pops : P;  // diagnostics on a bug path
      out.path_off[si] = st == kPathInternal ? pushes : o;
      out.final_w[si] = fin;
      if (out.work) {
        out.work[2 * si] = nn;
        out.work[2 * si + 1] = relax_count;
      }
    }
  }
}
#undef LZ_WD

}  // namespace fstamd
