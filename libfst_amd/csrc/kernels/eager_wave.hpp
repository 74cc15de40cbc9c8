// eager_wave.hpp -- eager compose + shortestPath on layered lattices, one wavefront per
// string (gfx950 / CDNA4).  Tier 1 of the eager engine since round 1 (v3).
//
// Same results as eager_layered.hpp (and so as compose.zig:64-195 + shortest-path.zig:
// 64-136, see the proof there and DESIGN.md §4.1): per layer the next tuples are the
// distinct rhs targets in first-occurrence order of the candidates (source position,
// arc index); d = min over candidate sums; the back-pointer is the tight candidate with
// the smallest index; the best final is lexmin (total, position).
//
// Why one wave per string.  A layer of the metric holds <= 257 tuples and ~635
// candidates: a 64-lane wave covers it with <= 5 tuples and <= 25 candidates per lane,
// and a single wave needs no s_barrier -- LDS operations of one wave complete in order,
// so a wavefront-scope fence (compiler ordering only) separates the phases.  The LDS
// footprint per string is 12.6 KB (vs 39 KB for the 256-thread tier), so ~12 strings
// are in flight per CU instead of 4, and their phases overlap.
//
// Per layer k (label = labels[k]); lane l owns the contiguous tuple chunk
// [l*E, l*E + E), E = ceil(n/64), in registers (rhs state, distance, arc span), and its
// candidates' rhs records (target, weight) were loaded at the end of layer k-1:
//   B  insert targets into the LDS hash; atomicMin first candidate and distance
//   C  tight candidates -> atomicMin of the packed (index, source, arc); creators counted
//   D  ranks of created tuples (wave scan) -> rank->slot table
//   E  each lane takes ranks [l*E', l*E' + E') of the next layer: back record to HBM,
//      slot cleared, and the next layer's spans and arc records loaded.
#pragma once

#include "device_common.hpp"
#include "eager_layered.hpp"  // EagerLaunch, write_status, lhash

namespace fstamd {

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int FCAP, int HCAP>
struct WaveLds {
  uint32_t key[HCAP];              // rhs state; kEmptyKey = free
  uint32_t first[HCAP];            // first (smallest) candidate index reaching the key
  unsigned long long dmin[HCAP];   // okey of the minimum candidate distance
  unsigned long long bpack[HCAP];  // (index << 48) | (source position << 32) | rhs arc of
                                   // the tight candidate with the smallest index
  uint16_t nslot[FCAP];            // next-layer rank -> slot
  unsigned long long best;         // best-final reduction words
  uint32_t bestp;
};

// Exclusive prefix sum over the wave of a value < 2^BITS, from bit-plane ballots:
// prefix = sum_b popcount(ballot(bit b) & lanes below) << b.  No LDS, no bpermute
// address registers; `total` is wave-uniform.
template <int BITS>
__device__ __forceinline__ uint32_t wave_excl_scan_small(uint32_t v, uint32_t& total) {
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const unsigned long long m = __ballot((v >> b) & 1u);
    pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    tot += (uint32_t)__popcll(m) << b;
  }
  total = tot;
  return pre;
}

__device__ __forceinline__ void wave_span(const RhsView& r, uint32_t s, uint32_t label,
                                          uint32_t& lo, uint32_t& cnt) {
  span_summary(r, s, label, lo, cnt);
}

// Spans of the owned tuples for `label` (row e holds position e*64 + lane), then the
// (target, weight) of their first KMAX arcs.  The loads are unconditional: the arc
// mirror is padded by kRecPad >= KMAX records, so rec[lo + j] is in bounds for any
// lo <= num_arcs; lanes mask what they do not own.
template <int EMAX, int KMAX>
__device__ __forceinline__ bool wave_load_layer(const RhsView& rhs, uint32_t label,
                                                uint32_t lane, uint32_t n_cur,
                                                const uint32_t (&s2)[EMAX], uint32_t (&lo)[EMAX],
                                                uint32_t (&cnt)[EMAX], uint32_t (&ct)[EMAX][KMAX],
                                                double (&cw)[EMAX][KMAX]) {
  bool too_long = false;
  // all span summaries in flight at once (one round trip), then the rare mixed-label
  // states fall back to the binary search
  uint4 ss[EMAX];
#pragma unroll
  for (int e = 0; e < EMAX; ++e) {
    const bool own = (uint32_t)e * 64 + lane < n_cur;
    ss[e] = rhs.sspan[own ? s2[e] : 0u];
    if (!own) ss[e] = make_uint4(0u, 0u, kSpanNone, 0u);
  }
#pragma unroll
  for (int e = 0; e < EMAX; ++e) {
    uint32_t l = ss[e].x, c = ss[e].y;
    if (ss[e].z != label) {
      c = 0;
      if (ss[e].z == kSpanMixed) {
        uint32_t a0, b0;
        span_by_ilabel(rhs, s2[e], label, a0, b0);
        l = a0;
        c = b0 - a0;
      }
    }
    lo[e] = l;
    cnt[e] = c;
    too_long |= c > (uint32_t)KMAX;
  }
#pragma unroll
  for (int e = 0; e < EMAX; ++e) {
    const ArcRec* b = rhs.rec + lo[e];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      ct[e][j] = b[j].next;
      cw[e][j] = b[j].weight;
    }
  }
  return too_long;
}

// Slot hash: the identity on state ids below HCAP (banded transducers -- the metric's --
// then fill the table without a single collision, and lanes holding neighbouring
// positions hit neighbouring banks), higher bits folded in above.
template <int HCAP>
__device__ __forceinline__ uint32_t wave_slot(uint32_t t) {
  constexpr uint32_t kBits = __builtin_ctz(HCAP);
  return (t ^ (t >> kBits) ^ (t >> (2 * kBits))) & (HCAP - 1);
}

// Best final = lexmin (total, position) over the last layer (shortest-path.zig:88-104).
// `best_w` / `bestp_w` are the wave's LDS reduction words.
// One final candidate of a lane: tuple at position p with state s and distance d.  Keeps
// the lane's lexmin (total, position); positions must arrive in ascending order.
__device__ __forceinline__ void wave_final_candidate(const RhsView& rhs, uint32_t p, uint32_t s,
                                                     double d, unsigned long long& mykey,
                                                     uint32_t& myp, double& myfw) {
  const double fw2 = rhs.final_w[FB(s, rhs.num_states, 33)];
  if (!w_is_zero(d) && !w_is_zero(fw2)) {
    const unsigned long long kk = okey(d + fw2);  // times(d, times(One, fw2))
    if (kk < mykey) {
      mykey = kk;
      myp = p;
      myfw = fw2;
    }
  }
}

// The lanes' final candidates -> the wave's best (lexmin (total, position)).  Returns
// whether there is one; `bp` = its position in the last layer, `fw2` = its rhs final weight
// (uniform).
__device__ __forceinline__ bool wave_pick_best(unsigned long long& best_w, uint32_t& bestp_w,
                                               uint32_t lane, unsigned long long mykey,
                                               uint32_t myp, double myfw, uint32_t& bp,
                                               double& fw2) {
  if (lane == 0) {
    best_w = kMaxU64;
    bestp_w = kEmptyKey;
  }
  wave_lds_sync();
  if (mykey != kMaxU64) atomicMin(&best_w, mykey);
  wave_lds_sync();
  const unsigned long long best = best_w;
  if (best != kMaxU64 && mykey == best) atomicMin(&bestp_w, myp);
  wave_lds_sync();
  bp = __builtin_amdgcn_readfirstlane(bestp_w);
  // final weight of the best tuple: its owner lane (bp % 64) has myp == bp; readlane
  // moves 32 bits, so the f64 goes as two words
  const uint32_t bl = bp & 63u;
  const unsigned long long fwbits = (unsigned long long)__double_as_longlong(myfw);
  const uint32_t fw_lo = __builtin_amdgcn_readlane((uint32_t)fwbits, bl);
  const uint32_t fw_hi = __builtin_amdgcn_readlane((uint32_t)(fwbits >> 32), bl);
  fw2 = __longlong_as_double((long long)(((unsigned long long)fw_hi << 32) | fw_lo));
  return best != kMaxU64;
}

// The lanes' final candidates -> the wave's best (lexmin (total, position)), then the
// backtrace through the back slab (shortest-path.zig:109-136) by lane 0.
__device__ __forceinline__ void wave_pick_and_backtrace(
    const RhsView& rhs, const ChainInput& in, const BatchOutDev& out, const uint2* back,
    uint32_t back_cap, unsigned long long& best_w, uint32_t& bestp_w, uint32_t si, uint64_t off,
    uint32_t L, uint32_t lane, uint32_t cur_base, unsigned long long mykey, uint32_t myp,
    double myfw, uint32_t tuples, uint32_t relax) {
  uint32_t bp;
  double fw2;
  const bool hit = wave_pick_best(best_w, bestp_w, lane, mykey, myp, myfw, bp, fw2);

  if (lane == 0) {
    if (!hit) {
      write_status(out, si, kPathEmpty, tuples, relax);
    } else {
      const unsigned long long o = reserve_path(out, si, L);
      if (o + L > out.arc_cap) {
        write_status(out, si, kPathOutputFull, tuples, relax);
      } else {
        uint32_t id = cur_base + bp;  // shortest-path.zig:109-136
        for (uint32_t k = L; k > 0; --k) {
          const uint2 b = back[FB(id, back_cap, 34)];
          const ArcRec r = rhs.rec[FB(b.y, rhs.num_arcs, 35)];
          out.out_il[o + k - 1] = in.labels[off + k - 1];
          out.out_ol[o + k - 1] = r.olabel;
          out.out_w[o + k - 1] = r.weight;  // times(One, w) == w for w >= +0
          id = b.x;
        }
        out.status[si] = kPathOk;
        out.path_len[si] = L;
        out.path_off[si] = o;
        out.final_w[si] = fw2;  // compose.zig:73: times(One, fw2) == fw2
        if (out.work) {
          out.work[2 * si] = tuples;
          out.work[2 * si + 1] = relax;
        }
      }
    }
  }
}

template <int EMAX>
__device__ __forceinline__ void wave_best_and_backtrace(
    const RhsView& rhs, const ChainInput& in, const BatchOutDev& out, const uint2* back,
    uint32_t back_cap, unsigned long long& best_w, uint32_t& bestp_w, uint32_t si, uint64_t off,
    uint32_t L, uint32_t lane, uint32_t n_cur, uint32_t cur_base, const uint32_t (&s2)[EMAX],
    const double (&dd)[EMAX], uint32_t tuples, uint32_t relax) {
  unsigned long long mykey = kMaxU64;
  uint32_t myp = kEmptyKey;
  double myfw = 0.0;
#pragma unroll
  for (int e = 0; e < EMAX; ++e) {  // e ascending = position ascending within the lane
    const uint32_t p = e * 64 + lane;
    if (p < n_cur) wave_final_candidate(rhs, p, s2[e], dd[e], mykey, myp, myfw);
  }
  wave_pick_and_backtrace(rhs, in, out, back, back_cap, best_w, bestp_w, si, off, L, lane,
                          cur_base, mykey, myp, myfw, tuples, relax);
}

template <int FCAP, int HCAP, int EMAX, int KMAX>
__global__ void __launch_bounds__(64, 3)
eager_wave_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                  EagerLaunch lp, BatchOutDev out) {
  static_assert(FCAP == 64 * EMAX, "FCAP = 64 lanes x EMAX rows");
  static_assert(EMAX * KMAX <= 64, "creator mask is 64 bits");
  static_assert(KMAX <= kRecPad, "arc mirror padding covers KMAX records");
  static_assert(HCAP >= FCAP && (HCAP & (HCAP - 1)) == 0, "HCAP: power of two >= FCAP");
  constexpr unsigned long long kFree = ~0ull;
  // per-lane, per-row candidate counts are <= KMAX
  constexpr int kRowBits = 32 - __builtin_clz((unsigned)KMAX);
  __shared__ WaveLds<FCAP, HCAP> S;
  const uint32_t lane = threadIdx.x;
  uint2* back = lp.back_ws + (size_t)blockIdx.x * lp.back_cap;
  const uint32_t num_items = __builtin_amdgcn_readfirstlane(
      lp.num_items_dev ? *lp.num_items_dev : lp.num_items);

#pragma unroll 1
  for (uint32_t i = lane; i < HCAP; i += 64) {
    S.key[i] = kEmptyKey;
    S.first[i] = kEmptyKey;
    S.dmin[i] = kFree;
    S.bpack[i] = kFree;
  }
  wave_lds_sync();

  for (;;) {
    // work item: fetched by the first active lane, broadcast through an SGPR
    uint32_t item = 0;
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) ==
        (uint32_t)(__ffsll((long long)__ballot(1)) - 1))
      item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readlane(item, __ffsll((long long)__ballot(1)) - 1);
    if (item >= num_items) break;
    FT(item, 0xFFFFFFFFu, 0, 0);
    const uint32_t si = __builtin_amdgcn_readfirstlane(lp.items ? lp.items[item] : item);
    // every value that steers control flow is made provably wave-uniform (SGPR), so the
    // compiler emits scalar branches and no divergent-loop structure
    const uint64_t off0 = in.offsets[si];
    const uint64_t off = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(off0 >> 32)) << 32) |
                         __builtin_amdgcn_readfirstlane((uint32_t)off0);
    const uint32_t L = __builtin_amdgcn_readfirstlane((uint32_t)(in.offsets[si + 1] - off));

    if (rhs.start == kNoState || n_best != 1) {  // compose.zig:33-35, shortest-path.zig:21-24
      if (lane == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }
    // per-string watchdog: every string gets the full limit (INTERNAL past it)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();

    // layer 0: the start tuple, position 0 (lane 0, row 0)
    uint32_t n_cur = 1, cur_base = 0;
    uint32_t tuples = 1, relax = 0;
    uint32_t s2[EMAX];
    double dd[EMAX];
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      s2[e] = rhs.start;
      dd[e] = w_one();
    }
    int32_t fail = kPathOk;

    for (uint32_t k = 0; k < L; ++k) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > lp.wd_ticks) {  // no wave stays forever
        fail = kPathInternal;
        tuples = 0x10000u | k;
        relax = n_cur;
        break;
      }
      FT(item, si, k, 1);
      const uint32_t lab = __builtin_amdgcn_readfirstlane(in.labels[off + k]);
      if (lab == kEpsilon) {  // lhs epsilon output: not a layered lattice
        fail = kPathUnsupported;
        break;
      }
      uint32_t lo[EMAX], cnt[EMAX];
      uint32_t ct[EMAX][KMAX];
      double cw[EMAX][KMAX];
      if (__ballot(wave_load_layer<EMAX, KMAX>(rhs, lab, lane, n_cur, s2, lo, cnt, ct, cw))) {
        fail = kPathOverflow;  // a span longer than KMAX: the next tier takes the string
        break;
      }
      FT(item, si, k, 2);
      // Candidate index of (row e, lane, j) = rows before e + lanes before in row e + j:
      // candidates enumerate (source position, arc index) and position = e * 64 + lane.
      const uint32_t rows = (n_cur + 63) / 64;
      uint32_t cbase[EMAX];
      uint32_t rbase = 0;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        uint32_t tot = 0;
        cbase[e] = rbase;
        if ((uint32_t)e < rows) {
          cbase[e] += wave_excl_scan_small<kRowBits>(cnt[e], tot);
          rbase += tot;
        }
      }
      relax += rbase;

      // ---- (B) insert targets; first occurrence and minimum distance ----
      // Linear probing in uniform rounds: in round r every still-pending candidate tries
      // slot (hash + r), so no per-candidate probe state is needed besides a pending bit.
      // Tier A only sees rhs weights >= +0 (no -0, NaN, -inf): there
      // times(d, times(One, w)) (compose.zig:104, shortest-path.zig:72) is exactly d + w.
      // Per row: all compare-and-swaps in flight, then one wait, then the atomics.
      unsigned long long pend = 0;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if ((uint32_t)e >= rows) continue;  // uniform
        uint32_t old[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          cw[e][j] = dd[e] + cw[e][j];
          old[j] = kEmptyKey - 1u;  // "not inserted" for idle slots
          if ((uint32_t)j < cnt[e]) old[j] = atomicCAS(&S.key[wave_slot<HCAP>(ct[e][j])], kEmptyKey, ct[e][j]);
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if ((uint32_t)j < cnt[e]) {
            const uint32_t t = ct[e][j];
            if (old[j] == kEmptyKey || old[j] == t) {
              const uint32_t i = wave_slot<HCAP>(t);
              ct[e][j] = i;
              atomicMin(&S.first[i], cbase[e] + j);
              atomicMin(&S.dmin[i], (unsigned long long)okey(cw[e][j]));
            } else {
              pend |= 1ull << (e * KMAX + j);
            }
          }
        }
      }
      FT(item, si, k, 3);
#pragma unroll 1
      for (uint32_t r = 1; __ballot(pend != 0) && r < (uint32_t)HCAP; ++r) {
#pragma unroll
        for (int e = 0; e < EMAX; ++e) {
#pragma unroll
          for (int j = 0; j < KMAX; ++j) {
            if (pend & (1ull << (e * KMAX + j))) {
              const uint32_t t = ct[e][j];
              const uint32_t i = (wave_slot<HCAP>(t) + r) & (HCAP - 1);
              const uint32_t old = atomicCAS(&S.key[i], kEmptyKey, t);
              if (old == kEmptyKey || old == t) {
                ct[e][j] = i;
                atomicMin(&S.first[i], cbase[e] + j);
                atomicMin(&S.dmin[i], (unsigned long long)okey(cw[e][j]));
                pend &= ~(1ull << (e * KMAX + j));
              }
            }
          }
        }
      }
      if (__ballot(pend != 0)) {  // table full
        fail = kPathOverflow;
        break;
      }
      wave_lds_sync();
      FT(item, si, k, 4);

      // ---- (C) tight candidates -> packed back-pointer; creators ----
      unsigned long long creators = 0;
      uint32_t nf[EMAX];
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        nf[e] = 0;
        if ((uint32_t)e >= rows) continue;  // uniform
        unsigned long long dm[KMAX];
        uint32_t fi[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {  // reads in flight together
          const uint32_t slot = (uint32_t)j < cnt[e] ? ct[e][j] : 0u;
          dm[j] = S.dmin[slot];
          fi[j] = S.first[slot];
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if ((uint32_t)j < cnt[e]) {
            const uint32_t ci = cbase[e] + j;
            if (okey(cw[e][j]) == dm[j])
              atomicMin(&S.bpack[ct[e][j]], ((unsigned long long)ci << 48) |
                                                ((unsigned long long)(e * 64 + lane) << 32) |
                                                (lo[e] + j));
            if (fi[j] == ci) {
              creators |= 1ull << (e * KMAX + j);
              ++nf[e];
            }
          }
        }
      }
      // ---- (D) ranks of the created tuples (candidate order = row, lane, j) ----
      uint32_t n_next = 0;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if ((uint32_t)e < rows) {
          uint32_t tot;
          uint32_t rank = n_next + wave_excl_scan_small<kRowBits>(nf[e], tot);
          n_next += tot;
          if (n_next <= (uint32_t)FCAP) {
#pragma unroll
            for (int j = 0; j < KMAX; ++j)
              if (creators & (1ull << (e * KMAX + j))) S.nslot[rank++] = (uint16_t)ct[e][j];
          }
        }
      }
      if (n_next > (uint32_t)FCAP || (uint64_t)cur_base + n_cur + n_next > lp.back_cap) {
        fail = kPathOverflow;
        break;
      }
      wave_lds_sync();
      FT(item, si, k, 6);

      // ---- (E) next layer: back records, slot reset (rank e * 64 + lane) ----
      const uint32_t next_base = cur_base + n_cur;
      const uint32_t rows_n = (n_next + 63) / 64;
      uint32_t es[EMAX];
      unsigned long long ebp[EMAX];
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {  // rank -> slot, all rows in flight
        const uint32_t r = e * 64 + lane;
        es[e] = (uint32_t)e < rows_n ? S.nslot[r < n_next ? r : 0] : 0u;
      }
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if ((uint32_t)e < rows_n) {
          s2[e] = S.key[es[e]];
          dd[e] = from_okey(S.dmin[es[e]]);
          ebp[e] = S.bpack[es[e]];
        }
      }
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        const uint32_t r = e * 64 + lane;
        if ((uint32_t)e < rows_n && r < n_next) {
          back[FB(next_base + r, lp.back_cap, 32)] =
              make_uint2(cur_base + (uint32_t)((ebp[e] >> 32) & 0xFFFFu), (uint32_t)ebp[e]);
          S.key[es[e]] = kEmptyKey;
          S.first[es[e]] = kEmptyKey;
          S.dmin[es[e]] = kFree;
          S.bpack[es[e]] = kFree;
        }
      }
      cur_base = next_base;
      n_cur = n_next;
      tuples += n_next;
      wave_lds_sync();
    }

    if (fail != kPathOk) {
      // leave the table clean for the next string
      wave_lds_sync();
#pragma unroll 1
      for (uint32_t i = lane; i < HCAP; i += 64) {
        S.key[i] = kEmptyKey;
        S.first[i] = kEmptyKey;
        S.dmin[i] = kFree;
        S.bpack[i] = kFree;
      }
      wave_lds_sync();
      if (lane == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }

    FT(item, si, L, 7);
    wave_best_and_backtrace<EMAX>(rhs, in, out, back, lp.back_cap, S.best, S.bestp, si, off, L,
                                  lane, n_cur, cur_base, s2, dd, tuples, relax);
  }
}

}  // namespace fstamd
