// eager_window.hpp -- eager compose + shortestPath on layered lattices, one wavefront per
// string, with a DIRECT-MAPPED target window instead of a hash (gfx950 / CDNA4).  Tier A0
// of the eager engine: it runs first and hands the strings it cannot hold to the hashed
// wave tier (eager_wave.hpp) through a device-side list.
//
// Results: identical to eager_wave.hpp (same candidate enumeration, same first-occurrence
// ids, same tight-candidate back-pointers, same best final), so the proof in
// eager_layered.hpp / DESIGN.md §4.1 carries over unchanged.  What differs is the table:
//
//   * Per layer the wave reduces the min and max target state of its candidates.  If they
//     span fewer than W = 64 * EW states, target t lives in slot t - tmin: no keys, no
//     compare-and-swap, no probing, and the next layer's state is tmin + slot.  (A layer of
//     a banded transducer -- the reference bench's ambiguous chain, a tagger's left-to-right
//     states -- always fits: the metric's widest layer spans 257 states.)  A wider layer
//     reports OVERFLOW and the string moves on to the hashed tier.
//   * Candidates that do not exist (j >= span count) aim their LDS atomics at a per-lane
//     trash slot W + lane instead of branching, so the phase loops carry no exec-mask
//     branches at all.
//   * At most W distinct targets fit a window, so a layer never holds more than W tuples.
//     Only layers that are expanded again live in registers (<= 64 * EMAX tuples); the
//     last layer (the metric's 257 tuples) is reduced to its best final straight from the
//     LDS table, so EMAX = 4 rows suffice for the metric and the wave fits 128 VGPRs.
//
// The LDS image is 8.3 KB per wave (12.9 KB for the hashed tier), so LDS no longer caps
// the wave count: registers do (__launch_bounds__ below).
#pragma once

#include "device_common.hpp"
#include "eager_layered.hpp"  // EagerLaunch, write_status
#include "eager_wave.hpp"     // wave_lds_sync, wave_excl_scan_small, wave_load_layer,
                              // wave_final_candidate, wave_pick_and_backtrace

extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_max_u32(uint32_t);

namespace fstamd {

// Backtraces are walked in batches: a wave finishes kChaseBatch strings (each into its own
// back slab), then lane r walks the path of string r -- the 1-dependent-load-per-arc chase
// (shortest-path.zig:109-136) is paid once per batch instead of once per string.
constexpr int kChaseBatch = 16;

// A finished string whose backtrace is pending (see the batched chase in the kernel).
struct ChaseJob {
  uint32_t si, L, id, tuples, relax, pad;
  unsigned long long o, off;
  double fw;
};

template <int W>
struct WindowLds {
  uint32_t first[W + 64];            // first (smallest) candidate index reaching the slot
  unsigned long long dmin[W + 64];   // okey of the minimum candidate distance
  unsigned long long bpack[W + 64];  // (index << 48) | (source position << 32) | rhs arc of
                                     // the tight candidate with the smallest index
  uint16_t nslot[W + 64];            // next-layer rank -> slot (+ trash slots)
  double dcur[W];                    // distance of each position of the current layer
                                     // (LDS, not registers: it lives across the loads)
  unsigned long long best;           // best-final reduction words
  uint32_t bestp;
  ChaseJob job[kChaseBatch];         // strings whose backtrace is pending, one slab each
};

// EMAX: register rows of a layer that is expanded (<= 64 * EMAX tuples); EW: rows of the
// window (W = 64 * EW target states, so <= W tuples in the last layer, which is never
// expanded: its best final is taken straight from the LDS table).
template <int EMAX, int EW, int KMAX, int WAVES_PER_EU>
__global__ void __launch_bounds__(64, WAVES_PER_EU)
eager_window_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                    EagerLaunch lp, BatchOutDev out) {
  constexpr int W = 64 * EW;
  static_assert(EW >= EMAX, "the window holds every expandable layer");
  static_assert(EMAX * KMAX <= 64, "creator mask is 64 bits");
  static_assert(KMAX <= kRecPad, "arc mirror padding covers KMAX records");
  constexpr unsigned long long kFree = ~0ull;
  constexpr int kRowBits = 32 - __builtin_clz((unsigned)KMAX);
  __shared__ WindowLds<W> S;
  const uint32_t lane = threadIdx.x;
  const uint32_t trash = W + lane;  // where non-existent candidates aim their atomics
  uint2* const slabs = lp.back_ws + (size_t)blockIdx.x * kChaseBatch * lp.back_cap;
  uint32_t njobs = 0;  // uniform: pending backtraces (slab j belongs to job j)
  // lane r < njobs walks job r's path: outputs, status, final weight, work counters
  auto chase_batch = [&]() {
    wave_lds_sync();
    uint32_t maxL = 0;
    ChaseJob jb{};
    if (lane < njobs) {
      jb = S.job[lane];
      maxL = jb.L;
    }
    maxL = __builtin_amdgcn_readfirstlane(__ockl_wfred_max_u32(maxL));
    const uint2* sl = slabs + (size_t)lane * lp.back_cap;
    uint32_t id = jb.id;
    for (uint32_t t = 0; t < maxL; ++t) {  // uniform trip count; lanes mask themselves
      if (lane < njobs && t < jb.L) {
        const uint32_t k = jb.L - 1 - t;
        const uint2 b = sl[FB(id, lp.back_cap, 34)];
        const ArcRec r = rhs.rec[FB(b.y, rhs.num_arcs, 35)];
        out.out_il[jb.o + k] = in.labels[jb.off + k];
        out.out_ol[jb.o + k] = r.olabel;
        out.out_w[jb.o + k] = r.weight;  // times(One, w) == w for w >= +0
        id = b.x;
      }
    }
    if (lane < njobs) {
      out.status[jb.si] = kPathOk;
      out.path_len[jb.si] = jb.L;
      out.path_off[jb.si] = jb.o;
      out.final_w[jb.si] = jb.fw;  // compose.zig:73: times(One, fw2) == fw2
      if (out.work) {
        out.work[2 * jb.si] = jb.tuples;
        out.work[2 * jb.si + 1] = jb.relax;
      }
    }
    njobs = 0;
    wave_lds_sync();
  };
  const uint32_t num_items = __builtin_amdgcn_readfirstlane(
      lp.num_items_dev ? *lp.num_items_dev : lp.num_items);

#pragma unroll 1
  for (uint32_t i = lane; i < (uint32_t)W + 64; i += 64) {
    S.first[i] = kEmptyKey;
    S.dmin[i] = kFree;
    S.bpack[i] = kFree;
  }
  wave_lds_sync();

  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readfirstlane(item);
    if (item >= num_items) break;
    const uint32_t si = __builtin_amdgcn_readfirstlane(lp.items ? lp.items[item] : item);
    uint2* const back = slabs + (size_t)njobs * lp.back_cap;
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
    // the watchdog is per string: every string gets the full limit, however long the
    // launch has been running (a string that exceeds it reports INTERNAL)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();

    uint32_t n_cur = 1, cur_base = 0;
    uint32_t tuples = 1, relax = 0;
    uint32_t s2[EMAX];
#pragma unroll
    for (int e = 0; e < EMAX; ++e) s2[e] = rhs.start;
    if (lane == 0) S.dcur[0] = w_one();  // the start tuple
    int32_t fail = kPathOk;
    uint32_t cmin = rhs.start, cmax = rhs.start;  // bounds of the current layer's states
    unsigned long long mykey = kMaxU64;  // this lane's best final candidate
    uint32_t myp = kEmptyKey;
    double myfw = 0.0;

    // the string's labels, 64 at a time, one per lane (no load on the layer's chain)
    uint32_t labs = 0;
    for (uint32_t k = 0; k < L; ++k) {
      // watchdog every 16 layers (the clock read is an SMEM round trip)
      if ((k & 15u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > lp.wd_ticks) {
        fail = kPathInternal;
        break;
      }
      if ((k & 63u) == 0) labs = k + lane < L ? in.labels[off + k + lane] : 0u;
      const uint32_t lab = __builtin_amdgcn_readlane(labs, k & 63u);
      if (lab == kEpsilon) {  // lhs epsilon output: not a layered lattice
        fail = kPathUnsupported;
        break;
      }
      uint32_t lo[EMAX], cnt[EMAX];
      uint32_t ct[EMAX][KMAX];
      double cw[EMAX][KMAX];
      if (__ballot(wave_load_layer<EMAX, KMAX>(rhs, lab, lane, n_cur, s2, lo, cnt, ct, cw))) {
        fail = kPathOverflow;
        break;
      }
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
      if (rbase == 0) {  // no candidate: the lattice dies here, no final is reachable
        n_cur = 0;
        break;
      }

      // ---- window of this layer's targets ----
      // Banded rhs (RhsView::jump_*): the targets lie in [cmin - jump_back, cmax +
      // jump_fwd], where [cmin, cmax] bounds this layer's states; if that fits the window
      // no per-candidate pass is needed.  Otherwise the exact min / max of the targets.
      uint32_t tmin, tmax;
      {
        const uint32_t blo = cmin >= rhs.jump_back ? cmin - rhs.jump_back : 0u;
        const uint64_t bhi = min((uint64_t)cmax + rhs.jump_fwd, (uint64_t)rhs.num_states - 1);
        if (bhi - blo < (uint64_t)W) {
          tmin = blo;
          tmax = (uint32_t)bhi;
        } else {
          uint32_t mn = kEmptyKey, mx = 0;
#pragma unroll
          for (int e = 0; e < EMAX; ++e) {
            if ((uint32_t)e >= rows) continue;  // uniform
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
              const bool v = (uint32_t)j < cnt[e];
              mn = v ? min(mn, ct[e][j]) : mn;
              mx = v ? max(mx, ct[e][j]) : mx;
            }
          }
          tmin = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_u32(mn));
          tmax = __builtin_amdgcn_readfirstlane(__ockl_wfred_max_u32(mx));
        }
      }
      if (tmax - tmin >= (uint32_t)W) {
        fail = kPathOverflow;  // the hashed tier takes the string
        break;
      }

      // ---- (B) first occurrence and minimum distance per slot ----
      // Tier A0 only sees rhs weights >= +0 (no -0, NaN, -inf): there
      // times(d, times(One, w)) (compose.zig:104, shortest-path.zig:72) is exactly d + w.
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if ((uint32_t)e >= rows) continue;  // uniform
        const double de = S.dcur[e * 64 + lane];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          const uint32_t slot = (uint32_t)j < cnt[e] ? ct[e][j] - tmin : trash;
          ct[e][j] = slot;
          cw[e][j] = de + cw[e][j];
          atomicMin(&S.first[slot], cbase[e] + j);
          atomicMin(&S.dmin[slot], (unsigned long long)okey(cw[e][j]));
        }
      }
      wave_lds_sync();

      // ---- (C) tight candidates -> packed back-pointer; creators; (D) their ranks
      // (candidate order = row, lane, j), one row at a time ----
      uint32_t n_next = 0;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if ((uint32_t)e >= rows) continue;  // uniform
        unsigned long long dm[KMAX];
        uint32_t fi[KMAX];
        // opaque copy: stops the compiler from keeping phase B's cbase + j values alive
        // across the sync (16 VGPRs at the register peak); recomputing costs 1 VALU each
        uint32_t cb = cbase[e], lc = lo[e];
        asm volatile("" : "+v"(cb), "+v"(lc));
        const uint32_t phi = (cb << 16) | (uint32_t)(e * 64 + lane);
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          dm[j] = S.dmin[ct[e][j]];
          fi[j] = S.first[ct[e][j]];
        }
        bool cr[KMAX];
        uint32_t nf = 0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          const bool v = (uint32_t)j < cnt[e];
          const uint32_t ci = cb + j;
          const bool tight = v && okey(cw[e][j]) == dm[j];
          // (index << 48) | (position << 32) | rhs arc, from a per-row high word
          const uint32_t hi = phi + ((uint32_t)j << 16);
          atomicMin(&S.bpack[tight ? ct[e][j] : trash],
                    ((unsigned long long)hi << 32) | (lc + j));
          cr[j] = v && fi[j] == ci;
          nf += cr[j] ? 1u : 0u;
        }
        uint32_t tot;
        uint32_t rank = n_next + wave_excl_scan_small<kRowBits>(nf, tot);
        n_next += tot;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {  // branch-free: non-creators write a trash slot
          S.nslot[cr[j] ? rank : trash] = (uint16_t)ct[e][j];
          rank += cr[j] ? 1u : 0u;
        }
      }
      const bool last = k + 1 == L;
      if ((!last && n_next > (uint32_t)(64 * EMAX)) ||
          (uint64_t)cur_base + n_cur + n_next > lp.back_cap) {
        fail = kPathOverflow;
        break;
      }
      wave_lds_sync();

      // ---- (E) next layer: back records, slot reset (rank e * 64 + lane); the rows of
      // the next layer, or on the last layer its final candidates ----
      const uint32_t next_base = cur_base + n_cur;
      const uint32_t rows_n = (n_next + 63) / 64;
      uint32_t es[EW];
      unsigned long long edm[EW], ebp[EW];
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        const uint32_t r = e * 64 + lane;
        es[e] = (uint32_t)e < rows_n && r < n_next ? (uint32_t)S.nslot[r] : trash;
      }
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        if ((uint32_t)e < rows_n) {
          edm[e] = S.dmin[es[e]];
          ebp[e] = S.bpack[es[e]];
        }
      }
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        const uint32_t r = e * 64 + lane;
        if ((uint32_t)e < rows_n) {
          if (r < n_next)
            back[FB(next_base + r, lp.back_cap, 40)] =
                make_uint2(cur_base + (uint32_t)((ebp[e] >> 32) & 0xFFFFu), (uint32_t)ebp[e]);
          S.first[es[e]] = kEmptyKey;
          S.dmin[es[e]] = kFree;
          S.bpack[es[e]] = kFree;
          if (last) {
            if (r < n_next)  // e ascending = position ascending within the lane
              wave_final_candidate(rhs, r, tmin + es[e], from_okey(edm[e]), mykey, myp, myfw);
          } else if (e < EMAX) {
            s2[e] = tmin + es[e];
            S.dcur[e * 64 + lane] = from_okey(edm[e]);
          }
        }
      }
      cur_base = next_base;
      n_cur = n_next;
      tuples += n_next;
      cmin = tmin;  // the next layer's states lie within this layer's target window
      cmax = tmax;
      wave_lds_sync();
    }

    if (fail != kPathOk) {
      // leave the table clean for the next string
      wave_lds_sync();
#pragma unroll 1
      for (uint32_t i = lane; i < (uint32_t)W + 64; i += 64) {
        S.first[i] = kEmptyKey;
        S.dmin[i] = kFree;
        S.bpack[i] = kFree;
      }
      wave_lds_sync();
      if (lane == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }
    if (L == 0 && lane == 0)  // the start tuple is the whole lattice
      wave_final_candidate(rhs, 0, rhs.start, w_one(), mykey, myp, myfw);
    uint32_t bp;
    double fw2;
    if (!wave_pick_best(S.best, S.bestp, lane, mykey, myp, myfw, bp, fw2)) {
      if (lane == 0) write_status(out, si, kPathEmpty, tuples, relax);
      continue;
    }
    unsigned long long o = 0;
    if (lane == 0) o = reserve_path(out, si, L);
    o = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(o >> 32)) << 32) |
        __builtin_amdgcn_readfirstlane((uint32_t)o);
    if (o + L > out.arc_cap) {
      if (lane == 0) write_status(out, si, kPathOutputFull, tuples, relax);
      continue;
    }
    if (lane == 0) {
      ChaseJob& j = S.job[njobs];
      j.si = si;
      j.L = L;
      j.id = cur_base + bp;  // shortest-path.zig:109-136 starts at the best final
      j.tuples = tuples;
      j.relax = relax;
      j.o = o;
      j.off = off;
      j.fw = fw2;
    }
    if (++njobs == (uint32_t)kChaseBatch) chase_batch();
  }
  if (njobs) chase_batch();
}

}  // namespace fstamd
