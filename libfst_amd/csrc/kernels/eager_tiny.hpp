// eager_tiny.hpp -- the compact LDS tier of the general engine's chain batch: eager
// semantics (compose, src/ops/compose.zig:29-198, then shortestPath,
// src/ops/shortest-path.zig:18-139) on lattices of up to 128 / 256 tuples, one wavefront
// per string, every table in LDS.
//
// Same algorithm and same answers as eager_bfs_kernel's tiny tiers (kernels/eager_bfs.hpp:
// level-synchronous BFS with ids in first-candidate order, the least fixpoint by sweeps
// over the levels when an arc goes backwards, back-pointer = tight in-arc with the
// smallest (source id, arc index), best final = lexmin (total, id)); only the tables are
// narrower, because the utterances of a WeText-scale tagger (~140 tuples, 95 % under 256)
// are latency-bound and their workgroups per CU were set by LDS: eager_bfs_kernel<64,
// false, 2> holds ~110 B per tuple (28 KB at 256 tuples, 5 per CU); this one ~52 B
// (13.1 KB, 12 per CU; 6.8 KB and 23 per CU at 128):
//   - a tuple key is one word, (s2 << 9) | (s1 << 2) | filter: the lhs is a chain of at
//     most 126 labels (s1 < 128) and the host sends only an rhs of fewer than 2^23 states;
//   - ids, arc offsets and levels are 16-bit; a back-pointer is (source << 16) | arc index;
//   - an arc keeps its target and weight (f64, relaxed every level), not its labels: the
//     path's arcs read theirs back by expanding their source tuples again;
//   - the hash has 1.5 slots per tuple (any size: multiply-shift home slots);
//   - final weights are recomputed for the tuples with s1 = L instead of being stored.
#pragma once

#include "eager_bfs.hpp"

namespace fstamd {

constexpr uint32_t kCtPhase2 = 0xFFFFFFFFu;  // arc code: the lhs epsilon-output arc alone
constexpr uint32_t kCtPhase3 = 0x80000000u;  // arc code flag: the rhs epsilon-input arc alone
constexpr uint32_t kCtLab = 128;             // lhs labels held in LDS (chains of <= 126)
constexpr uint32_t kCtMaxStates = 1u << 23;  // rhs states a one-word key can name

__host__ __device__ constexpr int ct_waves(int n) { return n <= 128 ? 5 : 3; }  // per SIMD

__device__ __forceinline__ uint32_t ct_key(uint32_t s1, uint32_t s2, uint32_t f) {
  return (s2 << 9) | (s1 << 2) | f;
}
// Home slot of key k in a table of H slots (any H: multiply-shift of a mixed hash).
template <uint32_t H>
__device__ __forceinline__ uint32_t ct_slot(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  return (uint32_t)(((uint64_t)k * H) >> 32);
}
// Insert key into the hash (linear probing); its slot, or kEmptyKey when the table is full.
template <uint32_t H>
__device__ __forceinline__ uint32_t ct_insert(uint32_t* hkey, uint32_t key) {
  uint32_t h = ct_slot<H>(key);
  for (uint32_t probe = 0; probe < H; ++probe) {
    const uint32_t old = atomicCAS(&hkey[h], kEmptyKey, key);
    if (old == kEmptyKey || old == key) return h;
    h = h + 1 < H ? h + 1 : 0u;
  }
  return kEmptyKey;
}

// bfs_expand (eager_bfs.hpp) for a chain lhs (label lab[s1] on arc s1 -> s1 + 1, weight One),
// in two steps: ct_spans finds the tuple's rhs spans (the dependent loads: the state
// summary, a search on a multi-label state), ct_emit walks them and emits the same
// candidates in the same order, each as emit(code, weight, target key, olabel).  The level loop
// keeps a lane's spans from the count pass (A) for the arc pass (B).
struct CtSpans {
  uint32_t lo, cnt;    // phase 1's arcs (cnt = 0: none)
  uint32_t elo, ecnt;  // the state's epsilon-input arcs
  uint32_t s1, s2, f, c;
  bool arc;            // s1 < L
  __device__ uint32_t count() const {
    const bool e = arc && c == kEpsilon;
    return cnt + ((f != 1 && e) ? 1u : 0u) + (f != 2 ? ecnt : 0u) + ((f == 0 && e) ? ecnt : 0u);
  }
};

__device__ __forceinline__ CtSpans ct_spans(const RhsView& rhs, const uint32_t* lab, uint32_t L,
                                            uint32_t k) {
  CtSpans sp;
  sp.s1 = (k >> 2) & 127u;
  sp.s2 = k >> 9;
  sp.f = k & 3u;
  sp.arc = sp.s1 < L;
  sp.c = sp.arc ? lab[sp.s1] : 0u;
  sp.lo = 0;
  sp.cnt = 0;
  if (sp.arc && sp.c != kEpsilon) span_summary<false>(rhs, sp.s2, sp.c, sp.lo, sp.cnt);
  span_summary<false>(rhs, sp.s2, kEpsilon, sp.elo, sp.ecnt);
  return sp;
}

// ct_spans for the whole wave (every lane calls it; `valid` lanes get their tuple's spans).
// Phase 1's arcsByIlabel on a multi-label state of more than 8 arcs was a binary search per
// lane: ~2 log2(n) dependent loads, 10-14 round trips on a WeText-scale tagger's lead-byte
// and char-boundary states (17-110 arcs), every BFS level.  Here lanes in 16-lane groups
// count the state's ilabels below / up to the label instead, 64 per round trip, four
// lanes' searches at a time.
__device__ __forceinline__ CtSpans ct_spans_wave(const RhsView& rhs, const uint32_t* lab,
                                                 uint32_t L, uint32_t k, bool valid) {
  CtSpans sp;
  sp.s1 = (k >> 2) & 127u;
  sp.s2 = k >> 9;
  sp.f = k & 3u;
  sp.arc = valid && sp.s1 < L;
  sp.c = sp.arc ? lab[sp.s1] : 0u;
  sp.lo = sp.cnt = sp.elo = sp.ecnt = 0;
  uint4 ss = make_uint4(0, 0, 0, 0);
  if (valid) {
    ss = rhs.sspan[sp.s2];  // span_summary's cases, from one load
    sp.elo = ss.x;
    sp.ecnt = ss.z == kEpsilon ? ss.y : ss.z == kSpanMixed ? ss.w : 0u;
  }
  bool need = false;
  if (sp.arc && sp.c != kEpsilon) {
    sp.lo = ss.x;
    if (ss.z == sp.c) {
      sp.cnt = ss.y;
    } else if (ss.z == kSpanMixed) {
      if (ss.y <= 8) {  // span_by_ilabel's independent loads
        uint32_t x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (uint32_t)i < ss.y ? rhs.il[ss.x + i] : 0xFFFFFFFFu;
        uint32_t cl = 0, ch = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bool v = (uint32_t)i < ss.y;
          cl += (v && x[i] < sp.c) ? 1u : 0u;
          ch += (v && x[i] <= sp.c) ? 1u : 0u;
        }
        sp.lo = ss.x + cl;
        sp.cnt = ch - cl;
      } else {
        need = true;
      }
    }
  }
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, sub = lane & 15;
  uint64_t mask = __ballot(need);
  while (mask) {  // uniform: up to four searches per round, one per 16-lane group
    uint64_t m = mask;
    for (uint32_t i = 0; i < g; ++i) m &= m - 1;
    const bool has = m != 0;
    const uint32_t t = has ? (uint32_t)__ffsll((long long)m) - 1 : 0u;
    // (the shuffles run on every lane: a lane that skipped one would not provide its value)
    const uint32_t off = __shfl(ss.x, t), nt = __shfl(ss.y, t), label = __shfl(sp.c, t);
    const uint32_t n = has ? nt : 0u;
    uint32_t lt = 0, le = 0;
    for (uint32_t base = 0; __ballot(base < n); base += 64) {
      uint32_t x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t i = base + sub + 16 * q;
        x[q] = i < n ? rhs.il[off + i] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool v = base + sub + 16 * q < n;
        lt += __popcll((__ballot(v && x[q] < label) >> (16 * g)) & 0xFFFFull);
        le += __popcll((__ballot(v && x[q] <= label) >> (16 * g)) & 0xFFFFull);
      }
    }
    // each searching lane takes its group's counts: job j = its rank among the set bits
    const uint32_t j = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    const bool mine = ((mask >> lane) & 1ull) && j < 4;
    const uint32_t src = mine ? 16 * j : 0u;
    const uint32_t mlt = __shfl(lt, src), mle = __shfl(le, src);
    if (mine) {
      sp.lo = ss.x + mlt;
      sp.cnt = mle - mlt;
    }
    for (int i = 0; i < 4 && mask; ++i) mask &= mask - 1;
  }
  return sp;
}

template <class Emit>
__device__ __forceinline__ void ct_emit(const RhsView& rhs, const CtSpans& sp, Emit&& emit) {
  const uint32_t s1 = sp.s1, s2 = sp.s2, f = sp.f;
  for (uint32_t a = sp.lo; a < sp.lo + sp.cnt; ++a) {  // phase 1 (compose.zig:95-121)
    const ArcRec r = rhs.rec[a];
    emit(a, w_times(w_one(), r.weight), ct_key(s1 + 1, r.next, 0), r.olabel);
  }
  const bool e = sp.arc && sp.c == kEpsilon;
  if (f != 1 && e)  // phase 2 (:124-134)
    emit(kCtPhase2, w_one(), ct_key(s1 + 1, s2, f == 0 ? 2u : f), kEpsilon);
  if (f != 2) {  // phase 3 (:136-157)
    const uint32_t nf = f == 0 ? 1u : f;
    for (uint32_t a = sp.elo; a < sp.elo + sp.ecnt; ++a) {
      const ArcRec r = rhs.rec[a];
      emit(a | kCtPhase3, r.weight, ct_key(s1, r.next, nf), r.olabel);
    }
  }
  if (f == 0 && e) {  // phase 4 (:160-194)
    for (uint32_t a = sp.elo; a < sp.elo + sp.ecnt; ++a) {
      const ArcRec r = rhs.rec[a];
      emit(a, w_times(w_one(), r.weight), ct_key(s1 + 1, r.next, 0), r.olabel);
    }
  }
}

struct CtShared {
  uint32_t item;
  uint32_t flag;
  uint32_t changed;
  uint32_t bestid;
  unsigned long long t_item;
  unsigned long long best;
  unsigned long long path_o;  // the path's arena offset (thread 0 -> the wave)
  uint32_t hops;
  int32_t verdict;            // kPathOk: write the path; else the status to report
};

// Final weight of tuple key k (compose.zig:69-74 with the chain's final(L) = One).
__device__ __forceinline__ double ct_final(const RhsView& rhs, uint32_t k, uint32_t L) {
  if (((k >> 2) & 127u) != L) return w_zero();
  const double fw1 = w_one(), fw2 = rhs.final_w[k >> 9];
  return (!w_is_zero(fw1) && !w_is_zero(fw2)) ? w_times(fw1, fw2) : w_zero();
}

template <int kN>
__global__ void __launch_bounds__(64, ct_waves(kN))
eager_tiny_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                  const uint32_t* items, const uint32_t* num_items_dev,
                  unsigned long long wd_ticks, BatchOutDev out) {
  constexpr uint32_t N = kN, A = kN * 3 / 2, H = kN * 3 / 2;
  static_assert(N <= 256 && A < 65536 && H < 65535, "16-bit ids, offsets and slots");
  __shared__ CtShared SH;
  __shared__ uint32_t hkey[H], hval[H], nkey[N], nback[N], lab[kCtLab];
  __shared__ unsigned long long nd[N];
  __shared__ double aw[A];
  __shared__ uint16_t aoff[N + 2], lvl[N + 2], anext[A], cslot[A];
  const uint32_t tid = threadIdx.x;
  const uint32_t num_items = *num_items_dev;

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      SH.item = atomicAdd(next_item, 1u);
      SH.t_item = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t item = SH.item;
    if (item >= num_items) break;
    const unsigned long long t0 = SH.t_item;  // per-string watchdog, as eager_bfs_kernel
    const uint32_t si = items[item];
    const uint64_t off = in.offsets[si];
    const uint32_t L = (uint32_t)(in.offsets[si + 1] - off);
    if (L + 2 > kCtLab) {
      if (tid == 0) write_status(out, si, kPathOverflow, 0, 0);
      continue;
    }
    for (uint32_t i = tid; i < L; i += 64) lab[i] = in.labels[off + i];
    if (rhs.start == kNoState || n_best != 1) {  // shortest-path.zig:21-24
      if (tid == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }

    // ---- compose: level-synchronous BFS (eager_bfs_kernel's phases A-E) ----
    for (uint32_t i = tid; i < H; i += 64) {
      hkey[i] = kEmptyKey;
      hval[i] = ~0u;
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t k0 = ct_key(0, rhs.start, 0), h = ct_slot<H>(k0);
      hkey[h] = k0;
      hval[h] = 0;
      nkey[0] = k0;
      nd[0] = okey(w_one());
      lvl[0] = 0;
      lvl[1] = 1;
      aoff[0] = 0;
      SH.changed = 0;
    }
    __syncthreads();
    uint32_t n_nodes = 1, n_arcs = 0, level = 0;
    int32_t fail = kPathOk;
    while (true) {
      const uint32_t f0 = level == 0 ? 0u : lvl[level];
      const uint32_t f1 = n_nodes;
      if (f0 >= f1) break;
      // (A) candidate counts -> arc offsets (written only while they fit: 16-bit)
      uint32_t carry = 0;
      CtSpans sp0;  // the lane's first tuple of the level (p = f0 + tid), kept for (B)
      for (uint32_t b = f0; b < f1; b += 64) {
        const uint32_t p = b + tid;
        const CtSpans sp = ct_spans_wave(rhs, lab, L, p < f1 ? nkey[p] : 0u, p < f1);
        const uint32_t cnt = p < f1 ? sp.count() : 0u;
        if (b == f0) sp0 = sp;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<64>(cnt, nullptr, tot);
        if (p < f1 && n_arcs + carry + ex <= A) aoff[p] = (uint16_t)(n_arcs + carry + ex);
        carry += tot;
      }
      if ((uint64_t)n_arcs + carry > A) {
        fail = kPathOverflow;
        break;
      }
      if (tid == 0) {
        aoff[f1] = (uint16_t)(n_arcs + carry);
        SH.flag = 0;
      }
      __syncthreads();
      // (B) the level's arcs (weights; their labels are read back for the path only), each
      // candidate's target into the hash by the lane that emits it (the first candidate of
      // a new key keeps the smallest arc index; a tagger level has a handful of tuples with
      // one or two candidates each, so parking the keys for a parallel insert cost LDS and
      // saved nothing)
      const uint32_t c0 = n_arcs, c1 = n_arcs + carry;
      for (uint32_t p = f0 + tid; p < f1; p += 64) {
        uint32_t a = aoff[p];
        ct_emit(rhs, p == f0 + tid ? sp0 : ct_spans(rhs, lab, L, nkey[p]),
                [&](uint32_t, double w, uint32_t key, uint32_t) {
                  aw[a] = w;
                  const uint32_t slot = ct_insert<H>(hkey, key);
                  if (slot == kEmptyKey) SH.flag = 1;
                  else atomicMin(&hval[slot], 0x80000000u | a);
                  cslot[a] = (uint16_t)slot;
                  ++a;
                });
      }
      __syncthreads();
      if (SH.flag) {
        fail = kPathOverflow;
        break;
      }
      // (C) ids of first occurrences, in candidate order (4 candidates per lane per round)
      constexpr uint32_t K = 4;
      uint32_t newc = 0;
      for (uint32_t b = c0; b < c1; b += 64 * K) {
        const uint32_t a0 = b + tid * K;
        uint32_t nf = 0, slots[K];
        bool first[K];
#pragma unroll
        for (uint32_t q = 0; q < K; ++q) {
          const uint32_t a = a0 + q;
          slots[q] = a < c1 ? cslot[a] : 0u;
          first[q] = a < c1 && hval[slots[q]] == (0x80000000u | a);
          nf += first[q] ? 1u : 0u;
        }
        uint32_t tot;
        uint32_t rank = block_excl_scan<64>(nf, nullptr, tot);
        if (n_nodes + newc + tot <= N) {
#pragma unroll
          for (uint32_t q = 0; q < K; ++q) {
            if (first[q]) {
              const uint32_t id = n_nodes + newc + rank++;
              hval[slots[q]] = id;
              nkey[id] = hkey[slots[q]];
              nd[id] = okey(w_zero());
            }
          }
        }
        newc += tot;
        if (n_nodes + newc > N) break;
      }
      __syncthreads();
      if (n_nodes + newc > N) {
        fail = kPathOverflow;
        break;
      }
      // (D) arc targets; (E) relax the level's arcs in level order (a backward arc leaves
      // the rest to the fixpoint sweeps)
      for (uint32_t a = c0 + tid; a < c1; a += 64) anext[a] = (uint16_t)hval[cslot[a]];
      __syncthreads();
      bool back = false;
      for (uint32_t p = f0 + tid; p < f1; p += 64) {
        const double ds = from_okey(nd[p]);
        const uint32_t a1 = aoff[p + 1];
        for (uint32_t a = aoff[p]; a < a1; ++a) {
          const uint32_t x = anext[a];
          back |= x < f1;
          if (!w_is_zero(ds)) atomicMin(&nd[x], okey(w_times(ds, aw[a])));
        }
      }
      if (back) SH.changed = 1;
      n_arcs = c1;
      n_nodes += newc;
      ++level;
      if (tid == 0) lvl[level + 1] = (uint16_t)n_nodes;
      __syncthreads();
      if ((level & 7u) == 0) {  // the watchdog every 8 levels
        if (__builtin_amdgcn_s_memrealtime() - t0 > wd_ticks) {
          if (tid == 0) SH.flag = 1;
        }
        __syncthreads();
        if (SH.flag) {
          fail = kPathInternal;
          break;
        }
      }
    }
    __syncthreads();
    if (fail != kPathOk) {
      if (tid == 0) write_status(out, si, fail, n_nodes, n_arcs);
      continue;
    }
    const uint32_t n_levels = level;
    const bool dag = SH.changed == 0;
    const unsigned long long deadline = t0 + wd_ticks;

    // ---- shortestPath: the least fixpoint (bfs_fixpoint), nd already holds path sums ----
    for (uint32_t i = tid; i < n_nodes; i += 64) nback[i] = ~0u;
    __syncthreads();
    bool ok = true;
    if (!dag) {
      for (uint32_t sweep = 0;; ++sweep) {
        if (tid == 0) SH.changed = 0;
        __syncthreads();
        for (uint32_t l = 0; l < n_levels; ++l) {
          const uint32_t b0 = lvl[l], b1 = lvl[l + 1];
          for (uint32_t s = b0 + tid; s < b1; s += 64) {
            const double ds = from_okey(nd[s]);
            if (w_is_zero(ds)) continue;
            for (uint32_t a = aoff[s]; a < aoff[s + 1]; ++a) {
              const unsigned long long v = okey(w_times(ds, aw[a]));  // shortest-path.zig:72
              const unsigned long long old = atomicMin(&nd[anext[a]], v);
              if (v < old) SH.changed = 1;
            }
          }
          __syncthreads();
        }
        if (tid == 0) SH.flag = __builtin_amdgcn_s_memrealtime() > deadline;
        __syncthreads();
        const bool changed = SH.changed != 0, expired = SH.flag != 0;
        __syncthreads();
        if (!changed) break;
        if (expired || sweep > n_nodes) {  // sweep > n_nodes: impossible for w >= 0
          ok = false;
          break;
        }
      }
    }
    if (!ok) {
      if (tid == 0) write_status(out, si, kPathInternal, n_nodes, n_arcs);
      continue;
    }
    // back-pointers: the tight in-arc with the smallest (source, arc index)
    for (uint32_t s = tid; s < n_nodes; s += 64) {
      const double ds = from_okey(nd[s]);
      if (w_is_zero(ds)) continue;
      const uint32_t a0 = aoff[s], a1 = aoff[s + 1];
      for (uint32_t a = a0; a < a1; ++a) {
        const uint32_t x = anext[a];
        if (okey(w_times(ds, aw[a])) == nd[x]) atomicMin(&nback[x], (s << 16) | (a - a0));
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
    for (uint32_t s = tid; s < n_nodes; s += 64) {
      const double ds = from_okey(nd[s]);
      const double fw = ct_final(rhs, nkey[s], L);
      if (w_is_zero(ds) || w_is_zero(fw)) continue;
      const unsigned long long k = okey(w_times(ds, fw));
      if (k < mk) {  // s ascending per lane: equal keys keep the smaller id
        mk = k;
        mid = s;
      }
    }
    if (mk != kMaxU64) atomicMin(&SH.best, mk);
    __syncthreads();
    if (mk != kMaxU64 && mk == SH.best) atomicMin(&SH.bestid, mid);
    __syncthreads();
    // backtrace: thread 0 walks the back-pointers in LDS (bounded: a cycle reports CYCLE)
    // and parks the path's (source, arc index) pairs in anext / cslot; then one lane per
    // path arc expands its source tuple again up to that arc for the arc's labels (the
    // tables keep no labels), all in parallel
    const uint32_t best = SH.bestid;
    if (tid == 0) {
      int32_t verdict = kPathOk;
      uint32_t hops = 0;
      if (best == kEmptyKey) {
        verdict = kPathEmpty;
      } else {
        uint32_t cur = best;
        for (;;) {
          const uint32_t b = nback[cur];
          if (b == ~0u) break;
          if (++hops > n_nodes) {
            verdict = kPathCycle;
            break;
          }
          cur = b >> 16;
        }
        if (verdict == kPathOk && cur != 0u) verdict = kPathEmpty;  // shortest-path.zig:120-122
      }
      if (verdict == kPathOk) {
        const unsigned long long o = reserve_path(out, si, hops);
        if (o + hops > out.arc_cap) {
          verdict = kPathOutputFull;
        } else {
          uint32_t cur = best;
          for (uint32_t k = hops; k > 0; --k) {
            const uint32_t b = nback[cur], s = b >> 16;
            anext[k - 1] = (uint16_t)s;
            cslot[k - 1] = (uint16_t)b;
            cur = s;
          }
          SH.path_o = o;
        }
      }
      SH.hops = hops;
      SH.verdict = verdict;
    }
    __syncthreads();
    const int32_t verdict = SH.verdict;
    if (verdict != kPathOk) {
      if (tid == 0) write_status(out, si, verdict, n_nodes, n_arcs);
      continue;
    }
    const uint32_t hops = SH.hops;
    const unsigned long long o = SH.path_o;
    for (uint32_t kb = 0; kb < hops; kb += 64) {  // uniform (ct_spans_wave)
      const uint32_t k = kb + tid;
      const bool v = k < hops;
      const uint32_t s = v ? anext[k] : 0u, ai = v ? cslot[k] : 0u, k1 = nkey[s];
      const CtSpans sp = ct_spans_wave(rhs, lab, L, k1, v);
      if (!v) continue;
      uint32_t i = 0, code = 0, ol = 0;
      ct_emit(rhs, sp, [&](uint32_t c, double, uint32_t, uint32_t l) {
        if (i++ == ai) {
          code = c;
          ol = l;
        }
      });
      const bool ph3 = code != kCtPhase2 && (code & kCtPhase3) != 0u;
      out.out_il[o + k] = ph3 ? kEpsilon : lab[(k1 >> 2) & 127u];
      out.out_ol[o + k] = ol;
      out.out_w[o + k] = aw[aoff[s] + ai];
    }
    if (tid == 0) {
      out.status[si] = kPathOk;
      out.path_len[si] = hops;
      out.path_off[si] = o;
      out.final_w[si] = ct_final(rhs, nkey[best], L);
      if (out.work) {
        out.work[2 * si] = n_nodes;
        out.work[2 * si + 1] = n_arcs;
      }
    }
  }
}

}  // namespace fstamd
