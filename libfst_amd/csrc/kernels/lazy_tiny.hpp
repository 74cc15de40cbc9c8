// lazy_tiny.hpp -- composeShortestPath (FST_SEM_LAZY) for small lattices with every table of
// the string in LDS: the first engine of the lazy chain batch (config 4's tagger and
// verbalizer, coalesced single calls).
//
// Replaces src/ops/compose-shortest-path.zig:26-401 for one linear-chain lhs per wavefront,
// like lazy_wave.hpp (its candidate enumeration, first-touch id assignment and lane-order
// folding are shared and documented there), but laid out for occupancy: the replay waits
// on two dependent rhs reads per pop, so the rate is resident strings per CU, and that is
// LDS per string.  34 B per tuple instead of lazy_wave's 108 B:
//  * hash slots are one word, (generation << 16) | id; the key is checked in nkey[id].  The
//    generation advances per string (the table is cleared when it wraps), so nothing is
//    cleared between strings;
//  * the back pointer is 8 B: {prev id | flags, rhs arc index}.  The ilabel is the popped
//    tuple's lhs label when the move consumed it (phases 1, 2, 4) and epsilon otherwise;
//    the olabel and the weight are the rhs arc's (phase 2 has none: epsilon, One), read
//    back from the frozen rhs when the path is written -- the tie-break of :110-128 needs
//    the olabel only on an exact tie from the same pop and then reads it;
//  * the queue is the frontier itself: an unordered array of the ids pushed and not yet
//    settled (2 B each, an in-frontier flag in the back pointer), popped by one wave
//    argmin of (dist[id], id) and appended to in parallel (no sift, no per-push lane-0
//    loop; a better dist needs no queue update at all).  Its pop order is the reference's
//    lazy-deletion binary heap's: both pop the minimum (dist, id) over the ids pushed and
//    not yet settled -- a stale entry of the lazy heap has a dist above dist[id], a
//    settled id is skipped there and absent here -- so the ids, the paths and the weights
//    are the same bits.  Frontier size <= tuples: no queue overflow.
//  * one loop groups a chunk's candidates by tuple key: its leaders are the first-touch
//    owners of new tuples (getOrCreate in lane order) and the folding lanes alike.
// LDS indices that come from the tables themselves pass FB() (sites 170-181: checked and
// clamped in DEBUG_BOUNDS builds).
// Sizes: tier t holds 64 << t tuples at 34 B; 1 (128) = 5.9 KB, 2 (256) = 10.2 KB, 3 (512)
// = 18.9 KB, 4 (1024) = 36.4 KB.  A string that outgrows its tier ends OVERFLOW and the host reruns
// it in the next (DeviceEngine::run_chain).
#pragma once

#include "lazy_wave.hpp"

namespace fstamd {

constexpr uint32_t kTyPrev = 0xFFFFu;       // nback.x bits 0..15: the previous tuple's id
constexpr uint32_t kTySettled = 1u << 16;
constexpr uint32_t kTyHasBack = 1u << 17;
constexpr uint32_t kTyConsumed = 1u << 18;  // the move read the lhs label (phases 1, 2, 4)
constexpr uint32_t kTyArc = 1u << 19;       // nback.y is an rhs arc index (not phase 2)
constexpr uint32_t kTyInQ = 1u << 20;       // in the frontier
constexpr uint32_t kTyKeep = kTySettled | kTyInQ;  // kept when the back pointer changes

// FSTAMD_TINY_PROF (a debug build): cycles per phase summed over every wave, printed by
// DeviceEngine::run_lazy_tiny -- [0] pop, [1] popped tuple + final + arc spans, [2] candidate
// records + lookups, [3] dedup + new tuples, [4] grouping + fold, [5] heap updates, [6]
// result, [7] pops
#ifdef FSTAMD_TINY_PROF
__device__ unsigned long long g_tiny_prof[8];
#define TY_T(k)                                                  \
  do {                                                           \
    const unsigned long long t_ = __builtin_readcyclecounter();  \
    prof[k] += t_ - tl;                                          \
    tl = t_;                                                     \
  } while (0)
#else
#define TY_T(k) \
  do {          \
  } while (0)
#endif

template <int kTier>
struct TinyLds {
  static constexpr uint32_t N = lz_tiny_n(kTier), H = 2 * N;
  // the rhs state summary (RhsView::sspan) of each tuple's s2, loaded when the tuple is
  // created (its latency hidden behind the rest of that chunk) so that a pop starts with
  // no global round trip: the latency-bound sizes only (3, 4: small batches, single calls)
#ifdef FSTAMD_TY_NOCACHE  // A/B builds
  static constexpr bool kCache = false;
#else
  static constexpr bool kCache = kTier >= 3;
#endif
  uint4 span[kCache ? N : 1];
  unsigned long long nkey[N];  // (s2 << 32) | (s1 << 2) | filter
  double ndist[N];
  double cnd[64];              // one chunk's candidates, read by the group leaders (the
                               // arc weights on the self-loop path)
  uint2 nback[N];
  uint32_t hs[H];
  uint32_t carc[64];
  uint32_t col[64];
  uint32_t ccode[64];
  uint32_t cid[64];
  uint16_t qid[N];             // the frontier (unordered), then the path's ids
  uint8_t own[256];            // a chunk's lane per key hash (the all-distinct test)
};

struct TyCand {
  unsigned long long key;
  uint32_t arc, ol, code;
  double w;
};

// Candidate c of a pop in reference order (chain_cand, lazy_wave.hpp): its rhs arc (phases
// 1, 3, 4; none in phase 2), its code and the s1 / filter of its target key.
__device__ __forceinline__ void tiny_cand_arc(const PopCands& P, uint32_t c, uint32_t& arc,
                                              uint32_t& code, uint32_t& ks1, uint32_t& kf) {
  if (c < P.n1) {  // :182-224
    arc = P.lo1 + c;
    code = kTyConsumed | kTyArc;
    ks1 = P.s1 + 1;
    kf = 0;
    return;
  }
  c -= P.n1;
  if (c < P.n2) {  // :227-252
    arc = 0;
    code = kTyConsumed;
    ks1 = P.s1 + 1;
    kf = P.f == 0 ? 2u : P.f;
    return;
  }
  c -= P.n2;
  if (c < P.n3) {  // :254-305
    arc = P.lo3 + c;
    code = kTyArc;
    ks1 = P.s1;
    kf = P.f == 0 ? 1u : P.f;
    return;
  }
  c -= P.n3;  // :307-365
  arc = P.lo3 + c;
  code = kTyConsumed | kTyArc;
  ks1 = P.s1 + 1;
  kf = 0;
}

// the olabel of a stored back pointer (phase 2: epsilon)
__device__ __forceinline__ uint32_t tiny_back_ol(const RhsView& rhs, uint2 b) {
  return (b.x & kTyArc) ? rhs.rec[b.y].olabel : kEpsilon;
}

// The relax rule of :110-128 for a candidate (nd, il, ol) from pop `pid` against the
// target's (od, b): the sequential reference's decision.  bol / bol_known cache b's olabel.
__device__ __forceinline__ bool tiny_take(const RhsView& rhs, double nd, uint32_t il, uint32_t ol,
                                          double od, uint2 b, uint32_t pid, uint32_t label,
                                          uint32_t& bol, bool& bol_known) {
  if (w_is_zero(od) || nd < od) return true;
  if (!(nd == od)) return false;
  if (!(b.x & kTyHasBack)) return true;
  const uint32_t bp = b.x & kTyPrev;
  if (pid != bp) return pid < bp;
  const uint32_t bil = (b.x & kTyConsumed) ? label : kEpsilon;
  if (il != bil) return il < bil;
  if (!bol_known) {
    bol = tiny_back_ol(rhs, b);
    bol_known = true;
  }
  return ol < bol;
}

template <int kTier>
__global__ void __launch_bounds__(64, kTier == 1 ? 5 : kTier == 2 ? 4 : kTier == 3 ? 2 : 1)
lazy_tiny_kernel(RhsView rhs, ChainInput chain, uint32_t n_best, unsigned int* next_item,
                 const uint32_t* items, uint32_t num_items, LazyWs ws, BatchOutDev out) {
  constexpr uint32_t N = TinyLds<kTier>::N, H = TinyLds<kTier>::H, hmask = H - 1;
  static_assert(N <= 1024 && (H & (H - 1)) == 0, "ids are 16-bit, the table a power of two");
  __shared__ TinyLds<kTier> S;
  const uint32_t lane = lane_id();
  const size_t w = blockIdx.x;
  for (uint32_t i = lane; i < H; i += 64) S.hs[i] = 0u;
  uint32_t gen = ws.stamp_base & 0xFFFFu;  // the cleared table is generation 0 (< any
                                           // generation a string uses)
  wave_fence();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool dead = false;
  uint32_t dbg_pops = 0, dbg_cb = 0, dbg_C = 0, dbg_qn = 0, dbg_nn = 0;
#ifdef FSTAMD_TINY_PROF
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tl = __builtin_readcyclecounter();
#endif
#define TY_WD(code)                                                                  \
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
    if (++gen == 0x10000u) {
      for (uint32_t i = lane; i < H; i += 64) S.hs[i] = 0u;
      gen = 1;
      wave_fence();
    }
    const uint64_t off = chain.offsets[si];
    const ChainLhs cl{chain.labels + off, (uint32_t)(chain.offsets[si + 1] - off)};

    // compose-shortest-path.zig:30-33 (a chain always has a start)
    if (rhs.start == kNoState || n_best != 1) {
      if (lane == 0) {
        out.status[si] = (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN;
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
      const unsigned long long k0 = tuple_key(0, rhs.start, 0);
      S.nkey[0] = k0;
      S.ndist[0] = w_one();
      S.nback[0] = make_uint2(kTyInQ, 0u);
      S.hs[hmix(k0) & hmask] = gen << 16;
      S.qid[0] = 0;
      if constexpr (TinyLds<kTier>::kCache) S.span[0] = rhs.sspan[rhs.start];
    }
    wave_fence();

    uint32_t best_id = kNoState;
    double best_fw = w_zero(), best_total = w_zero();
    uint32_t relax_count = 0;
    int32_t fail = kPathOk;
    uint32_t pops = 0, pushes = 1;
    uint32_t wd_work = 256;
    while (qn > 0) {
      dbg_pops = pops;
      dbg_qn = qn;
      dbg_nn = nn;
      if (wd_work >= 256u) {
        wd_work = 0;
        TY_WD(1);
      }
      if (dead || ++pops > N) {  // every id is popped at most once
        fail = kPathInternal;
        break;
      }
      // ---- pop: the frontier's minimum (dist, id) (ids distinct), the last entry moves
      // into its place ----
      double bd = __builtin_huge_val();
      uint32_t bi = kNoState, bp = 0;
      for (uint32_t c0 = 0; c0 < qn; c0 += 64) {
        const uint32_t cc = c0 + lane;
        if (cc < qn) {
          const uint32_t id = S.qid[cc];
          const double d = S.ndist[FB(id, N, 170)];
          if (bi == kNoState || qless(d, id, bd, bi)) {
            bd = d;
            bi = id;
            bp = cc;
          }
        }
      }
      // min dist, then min id among those; -0.0 == +0.0 as in qless (the exact dist is
      // read back from ndist below)
      const double dmn = __ockl_wfred_min_f64(bi != kNoState ? bd : __builtin_huge_val());
      const bool c1 = bi != kNoState && bd == dmn;
      const uint32_t pid = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_u32(c1 ? bi : ~0u));
      const uint32_t wl = (uint32_t)__ffsll((long long)__ballot(c1 && bi == pid)) - 1;
      const uint32_t ppos = __builtin_amdgcn_readlane(bp, wl);
      --qn;
      if (lane == 0) S.qid[FB(ppos, N, 171)] = S.qid[FB(qn, N, 171)];
      wave_fence();
      TY_T(0);
#ifdef FSTAMD_TINY_PROF
      prof[7] += 1;
#endif
      if (pid >= nn) {  // cannot happen on a consistent heap; never read past the tables
        fail = kPathInternal;
        break;
      }
      const uint2 pb = S.nback[FB(pid, N, 172)];
      const double pdist = S.ndist[pid];
      if ((pb.x & kTySettled) || !(pb.x & kTyInQ)) {
        fail = kPathInternal;
        break;
      }
      if (lane == 0) S.nback[pid].x = (pb.x & ~kTyInQ) | kTySettled;
      const unsigned long long pk = S.nkey[pid];
      PopCands P;
      P.s1 = (uint32_t)(pk & 0xFFFFFFFFull) >> 2;
      P.f = (uint32_t)pk & 3u;
      P.s2 = (uint32_t)(pk >> 32);
      if (P.s2 >= rhs.num_states) {
        fail = kPathInternal;
        break;
      }

      // ---- best final (:165-179): a chain's only final state is s1 == L ----
      if (P.s1 == cl.L) {
        const double fw2 = rhs.final_w[P.s2];
        if (!w_is_zero(fw2)) {
          const double fw = w_times(w_one(), fw2);
          const double total = w_times(pdist, fw);
          if (best_id == kNoState || total < best_total ||
              (total == best_total && pid < best_id)) {
            best_id = pid;
            best_fw = fw;
            best_total = total;
          }
        }
      }

      // ---- arcsByIlabel for the lhs label and epsilon (prepare_chain, lazy_wave.hpp): a
      // state of <= 64 arcs has its records and ilabels loaded together, arc j in lane j ----
      uint4 ss;
      if constexpr (TinyLds<kTier>::kCache) ss = S.span[pid];
      else ss = rhs.sspan[P.s2];
      const uint32_t off = ss.x, na = ss.y;
      // (the batch sizes 1, 2 load each candidate's record itself: the shuffles measured
      // 3 % slower there, where other waves hide the second round trip)
      const bool inl = TinyLds<kTier>::kCache && na <= 64;
      const bool has_arc = P.s1 < cl.L;
      P.label = has_arc ? cl.labels[P.s1] : 0u;
      ArcRec lr{0u, 0u, 0.0};
      uint32_t lil = 0;
      if (na <= 64 && lane < na) {
        if (inl) lr = rhs.rec[off + lane];
        if (ss.z == kSpanMixed) lil = rhs.il[off + lane];
      }
      {
        uint32_t lo3, hi3, lo1 = 0, hi1 = 0;
        if (ss.z != kSpanMixed) {  // one ilabel (or no arc)
          const bool eps = ss.z == kEpsilon;
          lo3 = off;
          hi3 = eps ? off + na : off;
          lo1 = off;
          hi1 = !eps && ss.z == P.label ? off + na : off;
        } else if (na <= 64) {
          const bool v = lane < na;
          lo3 = off;
          hi3 = off + (uint32_t)__popcll(__ballot(v && lil == kEpsilon));
          lo1 = off + (uint32_t)__popcll(__ballot(v && lil < P.label));
          hi1 = off + (uint32_t)__popcll(__ballot(v && lil <= P.label));
        } else {  // many arcs: the leading epsilon run from the summary, the label counted
          lo3 = off;
          hi3 = off + ss.w;
          if (has_arc && P.label != kEpsilon) wave_span_by_ilabel(rhs, off, na, P.label, lo1, hi1);
        }
        const uint32_t ne = hi3 - lo3;
        P.lo3 = lo3;
        P.n1 = 0;
        P.lo1 = 0;
        if (has_arc && P.label != kEpsilon) {  // :182-224
          P.lo1 = lo1;
          P.n1 = hi1 - lo1;
        }
        P.n2 = (has_arc && P.label == kEpsilon && P.f != 1) ? 1u : 0u;  // :227-252
        P.n3 = (P.f != 2) ? ne : 0u;                                     // :254-305
        P.n4 = (has_arc && P.label == kEpsilon && P.f == 0) ? ne : 0u;  // :307-365
      }
      const uint32_t C = P.n1 + P.n2 + P.n3 + P.n4;
      TY_T(1);
      relax_count += C;
      wd_work += C + 16u;
      double cur_dist = pdist;  // dist[curr_id]; changes only through a self-loop
      dbg_C = C;
      for (uint32_t cb = 0; cb < C; cb += 64) {
        dbg_cb = cb;
        if (cb != 0 && (cb & 4095u) == 0) {
          TY_WD(2);
        }
        if (dead) {
          fail = kPathInternal;
          break;
        }
        const uint32_t c = cb + lane;
        const bool act = c < C;
        TyCand x{0, 0, 0, 0, 0.0};
        {
          uint32_t ks1, kf;
          tiny_cand_arc(P, c, x.arc, x.code, ks1, kf);
          ArcRec r{0u, 0u, 0.0};
          if (inl) {  // from the lane holding the arc (every lane takes part in the shuffles)
            const int j = (int)((x.arc - off) & 63u);
            r.next = __shfl(lr.next, j, 64);
            r.olabel = __shfl(lr.olabel, j, 64);
            r.weight = __shfl(lr.weight, j, 64);
          } else if (act && (x.code & kTyArc)) {
            r = rhs.rec[x.arc];
          }
          if (x.code & kTyArc) {
            x.key = tuple_key(ks1, r.next, kf);
            x.ol = r.olabel;
            x.w = (x.code & kTyConsumed) ? w_times(w_one(), r.weight) : r.weight;
          } else {
            x.key = tuple_key(ks1, P.s2, kf);
            x.ol = kEpsilon;
            x.w = w_one();
          }
          if (!act) x = TyCand{0, 0, 0, 0, 0.0};
        }
        // lookup (getOrCreate's get): the slot names an id, the id's key decides
        uint32_t tid = kNoState;
        const uint32_t h0 = hmix(x.key);
        uint32_t slot = h0 & hmask;
        if (act) S.own[h0 & 255u] = (uint8_t)lane;
        if (act) {
          for (uint32_t probe = 0; probe <= hmask; ++probe) {
            const uint32_t v = S.hs[slot];
            if ((v >> 16) != gen) break;
            const uint32_t id = v & 0xFFFFu;
            if (S.nkey[FB(id, N, 173)] == x.key) {
              tid = id;
              break;
            }
            slot = (slot + 1) & hmask;
          }
        }
        TY_T(2);
        // group the chunk by tuple key in lane order: a group's first lane leads it --
        // the first touch of a new tuple (getOrCreate: ids by first occurrence in lane
        // order) and the lane that folds the group's relaxations
        unsigned long long gmask = 0;
        uint32_t leader = lane;
        // the common case first: every active lane wrote its own entry of the 256-entry
        // owner table, so no two share a key (two lanes of one key share an entry; keys that
        // merely collide take the loop below, which is exact in any case)
#ifdef FSTAMD_TY_NOFAST  // A/B builds: always the loop
        const bool single = false;
#else
        const bool single = !__ballot(act && S.own[h0 & 255u] != lane);
#endif
        if (single) {
          gmask = act ? 1ull << lane : 0ull;
        } else {
          unsigned long long pend = __ballot(act);
          while (pend) {
            const uint32_t l = (uint32_t)__ffsll((long long)pend) - 1;
            const unsigned long long lk =
                ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(x.key >> 32), l) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((uint32_t)x.key, l);
            const bool same = act && x.key == lk;
            const unsigned long long m = __ballot(same);
            if (lane == l) gmask = m;
            if (same) leader = l;
            pend &= ~m;
          }
        }
        const bool is_new_leader = gmask && tid == kNoState;
        const unsigned long long nlm = __ballot(is_new_leader);
        const uint32_t n_new = (uint32_t)__popcll(nlm);
        if (nn + n_new > N) {
          fail = kPathOverflow;
          break;
        }
        if (is_new_leader) {
          tid = nn + (uint32_t)__popcll(nlm & lanemask_lt());
          // claim the first free slot from where the lookup ended (load <= 1/2)
          const uint32_t mine = (gen << 16) | tid;
          uint32_t s = slot;
          for (uint32_t probe = 0; probe <= hmask; ++probe) {
            const uint32_t old = S.hs[s];
            if ((old >> 16) != gen && atomicCAS(&S.hs[s], old, mine) == old) break;
            s = (s + 1) & hmask;
          }
          S.nkey[tid] = x.key;
          S.ndist[tid] = w_zero();
          S.nback[tid] = make_uint2(0u, 0u);
        }
        uint4 new_span = make_uint4(0u, 0u, 0u, 0u);
        if constexpr (TinyLds<kTier>::kCache) {
          if (is_new_leader) new_span = rhs.sspan[(uint32_t)(x.key >> 32)];
        }
        if (n_new) {
          const uint32_t lt = __shfl(tid, (int)leader, 64);
          if (act) tid = lt;
        }
        nn += n_new;
        wave_fence();
        TY_T(3);

        // self-loop onto the popped tuple: rare, exact one-lane path
        const unsigned long long selfm = __ballot(act && tid == pid);
        if (selfm) {
          S.cid[lane] = tid;
          S.cnd[lane] = x.w;
          S.col[lane] = x.ol;
          S.ccode[lane] = x.code;
          S.carc[lane] = x.arc;
          wave_fence();
          const uint32_t cnt = C - cb < 64 ? C - cb : 64;
          if (lane == 0) {
            for (uint32_t i = 0; i < cnt; ++i) {
              const uint32_t t = S.cid[i];
              const double nd = w_times(cur_dist, S.cnd[i]);
              const double od = S.ndist[FB(t, N, 174)];
              const uint2 b = S.nback[t];
              const uint32_t code = S.ccode[i];
              uint32_t bol = 0;
              bool bol_known = false;
              if (tiny_take(rhs, nd, (code & kTyConsumed) ? P.label : kEpsilon, S.col[i], od, b,
                            pid, P.label, bol, bol_known)) {
                const bool add = !(b.x & kTyKeep);  // neither settled nor in the frontier
                S.ndist[t] = nd;
                S.nback[t] = make_uint2(pid | (b.x & kTyKeep) | (add ? kTyInQ : 0u) | kTyHasBack |
                                            code, S.carc[i]);
                if (t == pid) cur_dist = nd;
                if (add) S.qid[FB(qn++, N, 175)] = (uint16_t)t;
                if (!(b.x & kTySettled)) ++pushes;
              }
            }
          }
          cur_dist = __shfl(cur_dist, 0, 64);
          qn = __shfl(qn, 0, 64);
          pushes = __shfl(pushes, 0, 64);
          if constexpr (TinyLds<kTier>::kCache) {
            if (is_new_leader) S.span[tid] = new_span;
          }
          wave_fence();
          continue;
        }

        // group by target: the first lane of each group folds its members in lane order
        const double nd = w_times(cur_dist, x.w);
        if (!single) {  // the groups' members, for their leaders
          S.cnd[lane] = nd;
          S.col[lane] = x.ol;
          S.ccode[lane] = x.code;
          S.carc[lane] = x.arc;
          wave_fence();
        }
        bool push = false, app = false;
        if (gmask) {  // group leader
          const uint32_t t = tid;
          double od = S.ndist[FB(t, N, 176)];
          uint2 b = S.nback[t];
          uint32_t bol = 0;
          bool bol_known = false;
          bool took = false;
          if (single) {  // the group is this lane
            if (tiny_take(rhs, nd, (x.code & kTyConsumed) ? P.label : kEpsilon, x.ol, od, b, pid,
                          P.label, bol, bol_known)) {
              od = nd;
              b = make_uint2(pid | (b.x & kTyKeep) | kTyHasBack | x.code, x.arc);
              took = true;
            }
          }
          unsigned long long m = single ? 0ull : gmask;
          while (m) {
            const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
            m &= m - 1;
            const double cnd = S.cnd[i];
            const uint32_t code = S.ccode[i], col = S.col[i];
            if (tiny_take(rhs, cnd, (code & kTyConsumed) ? P.label : kEpsilon, col, od, b, pid,
                          P.label, bol, bol_known)) {
              od = cnd;
              b = make_uint2(pid | (b.x & kTyKeep) | kTyHasBack | code, S.carc[i]);
              bol = col;
              bol_known = true;
              took = true;
            }
          }
          if (took) {
            push = !(b.x & kTySettled);
            app = !(b.x & kTyKeep);  // pushed, and not yet in the frontier
            if (app) b.x |= kTyInQ;
            S.ndist[t] = od;
            S.nback[t] = b;
          }
        }
        TY_T(4);
        // pushes: new frontier entries appended in lane order (a better dist of an id in
        // the frontier needs nothing: the pop reads dist[id])
        pushes += (uint32_t)__popcll(__ballot(push));
        const unsigned long long am = __ballot(app);
        if (app) S.qid[FB(qn + (uint32_t)__popcll(am & lanemask_lt()), N, 177)] = (uint16_t)tid;
        qn += (uint32_t)__popcll(am);
        if constexpr (TinyLds<kTier>::kCache) {
          if (is_new_leader) S.span[tid] = new_span;
        }
        wave_fence();
        TY_T(5);
      }
      if (fail != kPathOk) break;
    }

    // ---- result (:368-400): the path's ids in LDS, then written by all lanes ----
    int32_t st = fail;
    uint32_t P = 0;
    unsigned long long o = 0;
    if (lane == 0 && st == kPathOk) {
      if (best_id == kNoState) {
        st = kPathEmpty;
      } else {
        uint32_t cur = best_id;
        while (cur != 0) {  // init_id == 0
          const uint2 b = S.nback[FB(cur, N, 178)];
          if (!(b.x & kTyHasBack)) {
            st = kPathEmpty;
            break;
          }
          if (++P > nn) {
            st = kPathCycle;
            break;
          }
          S.qid[FB(P - 1, N, 179)] = (uint16_t)cur;  // the heap is empty: its ids hold the path
          cur = b.x & kTyPrev;
        }
        if (st == kPathOk) {
          o = reserve_path(out, si, P);
          if (o + P > out.arc_cap) st = kPathOutputFull;
        }
      }
    }
    st = __shfl(st, 0, 64);
    wave_fence();
    if (st == kPathOk) {
      P = __shfl(P, 0, 64);
      o = __shfl(o, 0, 64);
      for (uint32_t k = lane; k < P; k += 64) {
        const uint32_t id = S.qid[k];
        const uint2 b = S.nback[FB(id, N, 180)];
        const uint32_t prev = b.x & kTyPrev;
        uint32_t il = kEpsilon, ol = kEpsilon;
        double aw = w_one();
        if (b.x & kTyConsumed) il = cl.labels[(uint32_t)(S.nkey[FB(prev, N, 181)] & 0xFFFFFFFFull) >> 2];
        if (b.x & kTyArc) {
          const ArcRec r = rhs.rec[b.y];
          ol = r.olabel;
          aw = (b.x & kTyConsumed) ? w_times(w_one(), r.weight) : r.weight;
        }
        const unsigned long long at = o + (P - 1 - k);
        out.out_il[at] = il;
        out.out_ol[at] = ol;
        out.out_w[at] = aw;
      }
    } else {
      P = 0;
      o = 0;
    }
    if (lane == 0) {
      out.status[si] = st;
      out.path_len[si] = st == kPathInternal ? pops : P;  // diagnostics on a bug path
      out.path_off[si] = st == kPathInternal ? pushes : o;
      out.final_w[si] = st == kPathOk ? best_fw : w_zero();
      if (out.work) {
        out.work[2 * si] = nn;
        out.work[2 * si + 1] = relax_count;
      }
    }
    wave_fence();
    TY_T(6);
  }
#ifdef FSTAMD_TINY_PROF
  if (lane < 8) {
    unsigned long long v = 0;
    for (int k = 0; k < 8; ++k) v = lane == (uint32_t)k ? prof[k] : v;
    atomicAdd(&g_tiny_prof[lane], v);
  }
#endif
}
#undef TY_WD
#undef TY_T

}  // namespace fstamd
