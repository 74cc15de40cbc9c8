// eager_pull.hpp -- eager compose + shortestPath on layered lattices, one wavefront per
// string, PULL formulation (gfx950 / CDNA4).  Tier P of the eager engine: it runs first
// when the rhs has a reverse mirror (DeviceFst::rev) and hands the strings it cannot hold
// to the push tiers (A0 eager_window.hpp, then A, B, C) through a device-side list.
//
// Same results as the push tiers (compose.zig:64-195 + shortest-path.zig:64-136, proof
// in eager_layered.hpp / DESIGN.md §4.1): with no epsilon move every lattice arc goes
// from layer k to layer k+1, and
//   * the tuples of layer k+1 are numbered by their first candidate in the order
//     (source id, position of the arc in the source's arcsByIlabel run) -- compose.zig's
//     FIFO discovery order;
//   * d(t) = min over candidates of d(s) + w (weights >= +0: Dijkstra's distance);
//   * back(t) = the tight candidate with the smallest (source id, arc position) -- the
//     tie rule of shortest-path.zig:74-84 applied by every relaxation;
//   * best final = lexmin (d + final, id) over the last layer (shortest-path.zig:88-104).
//
// What differs is who does the work.  The push tiers give each lane SOURCE tuples and
// merge candidates per target with LDS atomics (first index, min distance, then a second
// pass for the tight back-pointer).  Here each lane owns TARGET states of the layer's
// window [tmin', tmin' + wn) and pulls their in-arcs from the reverse mirror: one 16-B
// record per in-arc (source, arc position j, weight) and one LDS read of the source's
// cell (distance, rank).  The merge is then private to the lane:
//   pk    = rank(s) << 20 | j << 17 | m << 13 | 8 * source slot  (order = candidate order)
//   first = min pk                      -> the target exists iff first is a real candidate
//   d     = min (d(s) + w)
//   back  = min pk over the in-arcs with d(s) + w == d
// No atomics, no per-target table, no second pass over LDS.  Ids (ranks) of layer k+1
// come from a bitmap over the first keys (rank << 3 | j < 8 W): one LDS OR per target,
// a popcount prefix over <= 40 words (DPP scan), one read per target.
//
// A slot with no tuple holds {+inf, kPullAbsent}: its candidates have distance +inf and
// a key above every real one, so they never win -- the merge needs no validity selects.
// Reverse records hold 8 * source state, so the source's cell offset is one subtraction:
// slots outside the current layer's window (and the null block's padding records) are
// clamped to slot W, which never holds a tuple.
//
// The back record of a tuple is the reverse record of its back arc (4 B); the record's
// source state and the source layer's {slab base, window origin} (one 8-B entry per layer)
// give the source's slab position: the batched backtrace walks two dependent loads per arc
// (back record, then the reverse record it reads anyway for the olabel and weight).
#pragma once

#include <type_traits>

#include "device_common.hpp"
#include "eager_layered.hpp"  // EagerLaunch, write_status
#include "eager_wave.hpp"     // wave_lds_sync, wave_pick_best
#include "eager_window.hpp"   // ChaseJob, kChaseBatch

namespace fstamd {

constexpr uint32_t kPullAbsent = 0xFFFF0000u;  // rank word of a slot that holds no tuple
#ifdef FSTAMD_P_TIGHT_SELECT  // A/B builds: tier P's back key by compare-and-select
constexpr bool kTightSelect = true;
#else
constexpr bool kTightSelect = false;
#endif
// integer cells (the F32 kernels: every distance an integer below 2^24): the distance of a
// slot with no tuple.  Far above every real distance, and a weight below 2^24 added to it
// stays below 2^31, so a candidate from such a slot never wins and never wraps
constexpr uint32_t kDistAbsent = 0x7F000000u;
// +inf of the cells' distance type
template <typename DT>
__device__ __forceinline__ DT dist_inf() {
  if constexpr (sizeof(DT) == 4) return (DT)kDistAbsent;
  else return (DT)__builtin_huge_val();
}
template <typename DT>
__device__ __forceinline__ DT dist_min(DT a, DT b) {
  if constexpr (sizeof(DT) == 4) return min(a, b);
  else return fmin(a, b);
}


template <int W, bool F32 = false, int WT = kPullWt>
struct PullLds {
  static constexpr int kWords = W * 8 / 64;  // first keys rank << 3 | j < 8 W
  // the current layer's cells, slot W never holds a tuple.  Two arrays of 8-B entries
  // (one byte offset addresses both): 16-B cells cost ~12 K LDS bank-conflict cycles per
  // metric string
  double d[W + 1];                 // distance of the slot's tuple (+inf: no tuple)
  unsigned long long rk[W + 1];    // rank << 20 (kPullAbsent: no tuple) in the low word
  unsigned long long bits[kWords];
  uint4 pre[kWords];                         // per 32-bit half {keys before it, its bits}
  unsigned long long best;
  uint32_t bestp;
  ChaseJob job[kChaseBatch];
  double wt[WT];                   // RK 4 / 5: the rhs's distinct arc weights (rv_weight_table)
};
// integer cells (every distance an integer below 2^24; round 3 kept them as f32, round 4 as
// u32, whose add takes the 8-B record's weight byte as an SDWA operand): one 8-B cell
// {distance, rank word} per slot, read by one ds_read_b64 per in-arc; 4.3 KB instead of 6.9 KB
template <int W>
struct PullLds<W, true> {
  static constexpr int kWords = W * 8 / 64;
  uint2 cell[W + 1];               // {distance (kDistAbsent: no tuple), rank << 20}
  unsigned long long bits[kWords];
  uint4 pre[kWords];
  unsigned long long best;
  uint32_t bestp;
  ChaseJob job[kChaseBatch];
};

// The back key: the smallest key among the tight candidates (nd == b), as selects then a
// tree of 3-input mins (v_min3_u32) -- the running min(c, tight ? key : ~0) compiles to a
// compare, a min and a select per candidate (the lazy pull uses it)
template <int KP, typename DT>
__device__ __forceinline__ uint32_t tight_min(const DT (&nd)[KP], DT b, const uint32_t (&pk)[KP]) {
  uint32_t t[KP];
#pragma unroll
  for (int m = 0; m < KP; ++m) t[m] = nd[m] == b ? pk[m] : 0xFFFFFFFFu;
  uint32_t c = t[0];
#pragma unroll
  for (int m = 1; m < KP; m += 2) c = m + 1 < KP ? min(min(c, t[m]), t[m + 1]) : min(c, t[m]);
  return c;
}

// A load at a 32-bit byte offset from a kernel-argument base: global_load's SGPR-base +
// VGPR-offset form, no 64-bit address arithmetic per lane (the caller guarantees the
// offset fits: tables of < 4 GB)
template <typename T>
__device__ __forceinline__ const T* at_byte(const T* base, uint32_t byte_off) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// One in-arc record against the current layer's cells: its candidate key and distance.
template <int W>
__device__ __forceinline__ void pull_candidate(const PullLds<W>& S, const RevRec& r,
                                               uint32_t tmin8, uint32_t& pk, double& nd,
                                               uint32_t& rank_word) {
  // byte offset of the source's cell; outside the window (or padding): slot W
  const uint32_t off = min(r.src - tmin8, 8u * W);
  const double d = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(S.d) + FB(off, 8 * (W + 1), 150));
  const uint32_t rw = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(S.rk) + FB(off, 8 * (W + 1), 151));
  // (folding the pad c.w into the OR makes the compiler read the cell with one
  // ds_read2_b64 instead of b64 + b32, but costs a register and spills: 19.1 vs 20.1 M
  // strings/s)
  pk = rw | r.y | off;
  rank_word = rw;
  // times(d, times(One, w)) for w >= +0 (compose.zig:104, shortest-path.zig:72); +inf
  // stays +inf
  nd = d + r.weight;
}
// The same on tier P's 4-B records whose low byte indexes the rhs's table of distinct
// weights (RK 4: weights that no power-of-two scale makes integers; the cells stay f64):
// the source's offset as in the integer RK 3 below, the weight read from the LDS table --
// the same f64 value the reference adds
template <int W, int WT>
__device__ __forceinline__ void pull_candidate(const PullLds<W, false, WT>& S, const uint32_t& r,
                                               uint32_t base8, uint32_t& pk, double& nd,
                                               uint32_t& rank_word) {
  const uint32_t off = min(base8 - (r >> 16), 8u * W);
  const double d = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(S.d) + FB(off, 8 * (W + 1), 150));
  const uint32_t rw = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(S.rk) + FB(off, 8 * (W + 1), 151));
  pk = rw | (r & 0xFFFFu);
  rank_word = rw;
  nd = d + S.wt[FB(r & (WT - 1u), WT, 149)];
}
// The same on integer cells and the integer record copy {src, y, weight, olabel}: the
// distances are integers below 2^24, so the u32 sum, min and compare equal the f64 ones.
template <int W>
__device__ __forceinline__ void pull_candidate(const PullLds<W, true>& S, const uint4& r,
                                               uint32_t tmin8, uint32_t& pk, uint32_t& nd,
                                               uint32_t& rank_word) {
  const uint32_t off = min(r.x - tmin8, 8u * W);
  const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(S.cell) + FB(off, 8 * (W + 1), 152));
  pk = c.y | r.y | off;
  rank_word = c.y;
  nd = c.x + r.z;
}
// The same on the 8-B records {src, y | weight} (RevView::rrec8): the weight, an integer
// <= 7, sits in y's low 3 bits, below the byte offset (a multiple of 8), so it rides in the
// key's bits that never decide a comparison; y's bits 3..7 are zero, so the weight is
// y's low byte
__device__ __forceinline__ uint32_t rec8_weight(uint32_t y) { return y & 0xFFu; }
template <int W>
__device__ __forceinline__ void pull_candidate(const PullLds<W, true>& S, const uint2& r,
                                               uint32_t tmin8, uint32_t& pk, uint32_t& nd,
                                               uint32_t& rank_word) {
  const uint32_t off = min(r.x - tmin8, 8u * W);
  const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(S.cell) + FB(off, 8 * (W + 1), 152));
  pk = c.y | r.y | off;
  rank_word = c.y;
  nd = c.x + rec8_weight(r.y);  // (one v_add_u32 with a byte-0 SDWA operand)
}

// The same on tier P's 4-B records (RevView::rrec4, RK 3): base8 = 8 * (target - window
// origin) + rbias8 for this lane, the record's high half = 8 * (target - source) + rbias8,
// so their difference is the source's cell offset (a wrap or a padding record's 0xFFFF
// lands past slot W); the key keeps the record's low half (j << 13 | m << 9 | pos << 8 |
// weight) under the rank word (rank << 16), and the weight is its low byte.  Each of the
// three steps is one VALU with an SDWA operand, as with the 8-B records.
template <int W>
__device__ __forceinline__ void pull_candidate(const PullLds<W, true>& S, const uint32_t& r,
                                               uint32_t base8, uint32_t& pk, uint32_t& nd,
                                               uint32_t& rank_word) {
  const uint32_t off = min(base8 - (r >> 16), 8u * W);
  const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(S.cell) + FB(off, 8 * (W + 1), 152));
  pk = c.y | (r & 0xFFFFu);
  rank_word = c.y;
  nd = c.x + (r & 0xFFu);
}

// The in-arc group of target t for input label `lab`: the index of its first record and
// its block count (nb = 0: no in-arc with that label).  rspan is padded past the last
// state, so t may run past the window (such targets have no in-arc from the layer).
__device__ __forceinline__ void pull_group(const RevView& rv, uint32_t lab, uint32_t t,
                                           uint32_t& rec0, uint32_t& nb) {
  const uint4 rs = rv.rspan[t];
  // (labels >= kSpanMixed always go through gtab: they collide with the markers)
  const bool hit = rs.z == lab && lab < kSpanMixed;
  rec0 = hit ? rs.x : 0u;
  nb = hit ? rs.y : 0u;
  // several in-labels: binary search of gtab (gsearch == 0: the rhs has no such state)
  if (rv.gsearch && __ballot(rs.z == kSpanMixed)) {
    if (rs.z == kSpanMixed) {
      uint32_t a = rs.x, b = rs.x + rs.y;
      for (uint32_t it = 0; it < rv.gsearch; ++it) {
        if (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (rv.gtab[mid].x < lab) a = mid + 1;
          else b = mid;
        }
      }
      if (a < rs.x + rs.y) {
        const uint4 g = rv.gtab[a];
        if (g.x == lab) {
          rec0 = g.y;
          nb = g.z;
        }
      }
    }
  }
}

// DIRECT (RevView::direct): block 0 of target t is records [t * KP, t * KP + KP), loaded
// together with rspan[t] (which then only confirms the label); otherwise the group is
// looked up first (pull_group) and its records loaded after.
// RK (records): 0 RevRec, f64 cells; 1 and 2 (F32): cells and merge in f32, records from
// RevView::rrec32 (1) or the 8-B RevView::rrec8 (2, weights <= 7) -- chosen by the host when
// every distance of the launch is an integer below 2^24 (pull_f32: integer arc weights,
// max_len * max weight < 2^24), where every f32 sum, min and compare equals the f64 one.
// Strings longer than in.max_len (a caller's wrong bound) are handed on, so the bound
// always holds.
template <int EW, int KP, bool DIRECT, int WAVES_PER_EU, int RK = 0>
__global__ void __launch_bounds__(64, WAVES_PER_EU)
eager_pull_kernel(RhsView rhs, RevView rv, ChainInput in, uint32_t n_best,
                  unsigned int* next_item, EagerLaunch lp, BatchOutDev out) {
  constexpr int W = 64 * EW;
  constexpr bool F32 = RK != 0 && RK != 4 && RK != 5;
  constexpr bool REC4 = RK >= 3;  // tier P's 4-B records (RK 4 / 5: f64 cells)
  constexpr int WT = RK == 5 ? (int)kPullWtMax : (int)kPullWt;  // weight-table entries
  using DT = typename std::conditional<F32, uint32_t, double>::type;  // (F32: integer cells)
  using RT = typename std::conditional<
      REC4, uint32_t,
      typename std::conditional<RK == 2, uint2,
                                typename std::conditional<F32, uint4, RevRec>::type>::type>::type;
  // key layout: rank word rank << 20 over y = j << 17 | m << 13 (RK 3: rank << 16 over
  // j << 13 | m << 9): the first key (rank << 3 | j) and m sit at these shifts
  constexpr uint32_t kRankShift = REC4 ? 16 : 20;
  constexpr uint32_t kFirstShift = kRankShift - 3;
  constexpr uint32_t kMShift = kFirstShift - 4;
  constexpr int kWords = PullLds<W, F32, WT>::kWords;
  static_assert(KP <= 16, "m is 4 bits of the key");
  static_assert(W < 512, "8 * slot is 12 bits of the key, ranks 9 bits");
  __shared__ PullLds<W, F32, WT> S;
  const uint32_t lane = threadIdx.x;
  const DT kInf = dist_inf<DT>();
  // a cell: {distance, rank word}
  auto set_cell = [&](uint32_t i, DT d, uint32_t rw) {
    if constexpr (F32) {
      S.cell[FB(i, W + 1, 153)] = make_uint2(d, rw);
    } else {
      S.d[FB(i, W + 1, 154)] = d;
      S.rk[FB(i, W + 1, 155)] = rw;
    }
  };
  auto rec = [&](uint32_t r) -> RT {
    if constexpr (REC4) return rv.rrec4[r];
    else if constexpr (RK == 2) return rv.rrec8[r];
    else if constexpr (F32) return rv.rrec32[r];
    else return rv.rrec[r];
  };
  uint2* const slabs = lp.back_ws + (size_t)blockIdx.x * kChaseBatch * lp.back_cap;
  uint32_t njobs = 0;  // uniform: pending backtraces (slab j belongs to job j)

  // lane r < njobs walks job r's path (shortest-path.zig:109-136): one 8-B back record
  // per arc, {reverse record of the arc, slab position of the source}
  auto chase_batch = [&]() {
    wave_lds_sync();
    uint32_t maxL = 0;
    ChaseJob jb{};
    if (lane < njobs) {
      jb = S.job[FB(lane, kChaseBatch, 156)];
      maxL = jb.L;
    }
    maxL = __builtin_amdgcn_readfirstlane(__ockl_wfred_max_u32(maxL));
    // slab: 4-B back records (the reverse record of each tuple's back arc) in its first
    // half, per layer k {slab base, window origin} of layer k in its second half: the
    // record's source state gives the source's slab position
    const uint32_t* sl = reinterpret_cast<const uint32_t*>(slabs + (size_t)lane * lp.back_cap);
    const uint2* hdr = slabs + (size_t)lane * lp.back_cap + lp.back_cap / 2;
    uint32_t id = jb.id;
    uint32_t tcur = jb.pad;  // RK 3: the state of the tuple at slab position id
    for (uint32_t t = 0; t < maxL; ++t) {  // uniform trip count; lanes mask themselves
      if (lane < njobs && t < jb.L) {
        const uint32_t k = jb.L - 1 - t;
        uint32_t b;
        if constexpr (REC4) {  // the byte x * KP + m of the tuple at slab position id,
                                  // whose state is tcur: block 0 at tcur * KP, blocks 1.. at
                                  // rxrec[tcur].x (eager_pull.hip)
          const uint32_t v = reinterpret_cast<const uint8_t*>(sl)[FB(id, lp.back_cap, 60)];
          b = FB(v < (uint32_t)KP ? tcur * KP + v : rv.rxrec[tcur].x + v - KP, rv.nrec, 63);
        } else {
          b = FB(sl[FB(id, lp.back_cap, 60)], rv.nrec, 63);
        }
        const uint2 h = hdr[k];
        if (!out.host_ol) out.out_il[jb.o + k] = in.labels[jb.off + k];
        uint32_t src8;
        if constexpr (REC4) {
          const uint32_t r = rv.rrec4[b];
          out.out_ol[jb.o + k] = rv.rolab[b];
          if constexpr (RK >= 4)
            out.out_w[jb.o + k] = rv_weight_table(rv)[r & (WT - 1u)];  // the f64 weight
          else
            out.out_w[jb.o + k] = (double)(r & 0xFFu) * rv.winv;  // exact: the f64 weight
          tcur -= (uint32_t)(((int32_t)(r >> 16) - (int32_t)rv.rbias8) >> 3);  // the source
          src8 = tcur << 3;
        } else if constexpr (RK == 2) {
          const uint2 r = rv.rrec8[b];
          out.out_ol[jb.o + k] = rv.rolab[b];
          out.out_w[jb.o + k] = (double)rec8_weight(r.y) * rv.winv;  // exact: the f64 weight
          src8 = r.x;
        } else if constexpr (F32) {
          const uint4 r = rv.rrec32[b];
          out.out_ol[jb.o + k] = r.w;
          out.out_w[jb.o + k] = (double)r.z * rv.winv;  // exact: the f64 weight
          src8 = r.x;
        } else {
          const RevRec r = rv.rrec[b];
          out.out_ol[jb.o + k] = rv.rolab[b];
          out.out_w[jb.o + k] = r.weight;  // times(One, w) == w for w >= +0
          src8 = r.src;
        }
        id = h.x + ((src8 >> 3) - h.y);
      }
    }
    if (lane < njobs) {
      out.status[jb.si] = kPathOk;
      if (out.first_status) out.first_status[jb.si] = kPathOk;
      out.path_len[jb.si] = jb.L;
      out.path_off[jb.si] = jb.o;
      out.final_w[jb.si] = jb.fw;  // compose.zig:73: times(One, fw2) == fw2
      if (out.work) {
        out.work[2 * jb.si] = jb.tuples;
        out.work[2 * jb.si + 1] = jb.relax;
      }
    }
    if (out.host_ol) copy_out_paths(out, njobs, jb.o, jb.L, lane);
    njobs = 0;
    wave_lds_sync();
  };
  const uint32_t num_items = __builtin_amdgcn_readfirstlane(
      lp.num_items_dev ? *lp.num_items_dev : lp.num_items);
  // (an SGPR word made opaque at each test: as a bool the compiler kept it as a spilled lane
  // mask, reloaded per row with two readlanes)
  const uint32_t want_work_w = __builtin_amdgcn_readfirstlane(out.work != nullptr ? 1u : 0u);
  auto want_work = [&]() -> bool {
    uint32_t w = __builtin_amdgcn_readfirstlane(want_work_w);
    asm volatile("" : "+s"(w));
    return w != 0u;
  };

#pragma unroll 1
  for (uint32_t i = lane; i < (uint32_t)W + 1; i += 64) set_cell(i, kInf, kPullAbsent);
  if (lane < (uint32_t)kWords) S.bits[FB(lane, kWords, 157)] = 0;
  if constexpr (RK >= 4)
    for (uint32_t i = lane; i < (uint32_t)WT; i += 64) S.wt[i] = rv_weight_table(rv)[i];
  wave_lds_sync();
  uint32_t wlast = 0;  // uniform: cells [wlast, W] hold no tuple

  for (;;) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readfirstlane(item);
    if (item >= num_items) break;
    const uint32_t si = __builtin_amdgcn_readfirstlane(lp.items ? lp.items[item] : item);
    uint32_t* const back = reinterpret_cast<uint32_t*>(slabs + (size_t)njobs * lp.back_cap);
    uint2* const hdr = slabs + (size_t)njobs * lp.back_cap + lp.back_cap / 2;
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
    // the watchdog is per string (a string that exceeds it reports INTERNAL)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();

    // layer 0: the start tuple alone, slot 0 of a window at the start state
#pragma unroll 1
    for (uint32_t i = lane; i < wlast; i += 64) set_cell(i, kInf, kPullAbsent);
    wave_lds_sync();
    if (lane == 0) set_cell(0, (DT)w_one(), 0u);
    wave_lds_sync();
    uint32_t tmin = rhs.start, wk = 1, base = 0, n_cur = 1;
    uint32_t cmin = rhs.start, cmax = rhs.start;  // bounds of the current layer's states
    uint32_t tuples = 1, relax = 0;
    int32_t fail = F32 && L > in.max_len ? kPathOverflow : kPathOk;
    unsigned long long mykey = kMaxU64;  // this lane's best final candidate
    uint32_t myp = kEmptyKey;
    double myfw = 0.0;

    uint32_t labs = 0;
    for (uint32_t k = 0; k < L && fail == kPathOk; ++k) {
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
      // ---- window of the next layer: every target of a state in [cmin, cmax] lies in
      // [cmin - jump_back, cmax + jump_fwd] (RhsView) ----
      const uint32_t tn = cmin >= rhs.jump_back ? cmin - rhs.jump_back : 0u;
      // (32-bit: the pull tiers take rhs of fewer than 2^27 states, so cmax + jump_fwd
      // cannot wrap, and the compares stay scalar -- u64 ones went to the VALU)
      const uint32_t hi = min(cmax + rhs.jump_fwd, rhs.num_states - 1);
      const uint32_t nbase = base + wk;
      // (the slab's second half holds one header entry per layer: k < back_cap / 2)
      if (hi - tn >= (uint32_t)W || nbase + (hi - tn + 1) > lp.back_cap ||
          k >= lp.back_cap / 2) {
        fail = kPathOverflow;  // the push tiers take the string
        break;
      }
      const uint32_t wn = hi - tn + 1;
      const uint32_t rows_n = (wn + 63) / 64;

      // ---- (P1) pull: every target slot of the window merges its in-arcs ----
      uint32_t fst[EW], bk[EW], bra[EW];
      DT bd[EW];
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        fst[e] = kEmptyKey;
        bk[e] = kEmptyKey;
        bra[e] = 0;
        bd[e] = kInf;
        if ((uint32_t)e >= rows_n) continue;  // uniform
        // (looking up every row's group before the row loop measured no faster)
        const uint32_t i = (uint32_t)e * 64 + lane;
        const uint32_t t = tn + i;
        uint32_t rec0, nb, xrec = 0;
        uint32_t tmin8 = tmin << 3;
        if constexpr (DIRECT) {
          const uint32_t rs = *at_byte(rv.rlab, t * 4u);  // ilabel | min(nblocks, 255) << 24
          // block 0 holds the arcs of another label: shifting the window origin by 2^31
          // sends every source of the row past slot W (8 * state < 2^30), so the row
          // merges to "no tuple" with no per-result selects
          const bool hit = (rs & 0xFFFFFFu) == lab && lab < kSpanMixed;
          tmin8 = hit ? tmin8 : tmin8 + 0x80000000u;
          rec0 = t * KP;
          nb = hit ? rs >> 24 : 0u;
        } else {
          pull_group(rv, lab, t, rec0, nb);
        }
        // RK 3: the records hold the source relative to the target, so the lane's base is
        // 8 * (t - window origin) + rbias8 (the 2^31 shift of a miss applies the same)
        if constexpr (REC4) tmin8 = (t << 3) - (tmin << 3) + rv.rbias8 + (tmin8 - (tmin << 3));
        RT rr[KP];
        // one base address, the records at immediate offsets
        const RT* R;
        // (RK 2, 3: the byte offset in 32 bits -- fewer than 2^28 records, eager_pull.hip)
        if constexpr (REC4) R = at_byte(rv.rrec4, rec0 * 4u);
        else if constexpr (RK == 2) R = at_byte(rv.rrec8, rec0 * 8u);
        else if constexpr (F32) R = rv.rrec32 + rec0;
        else R = rv.rrec + rec0;
#pragma unroll
        for (int m = 0; m < KP; ++m) rr[m] = R[m];
        uint32_t pk[KP], rw[KP];
        DT nd[KP];
        uint32_t f = kEmptyKey;
        DT b = kInf;
        uint32_t c = kEmptyKey;
        // (one 64-bit min of (distance bits, key) per in-arc instead of fmin + the tight
        // pass: 25 fewer VALU per unrolled row, same 41.4 ms per 1M metric strings, round 4)
#pragma unroll
        for (int m = 0; m < KP; ++m) {
          pull_candidate<W>(S, rr[m], tmin8, pk[m], nd[m], rw[m]);
          f = min(f, pk[m]);
          b = dist_min(b, nd[m]);
        }
        // the back key: the smallest key among the tight in-arcs (nd == b).  Integer cells:
        // b - nd has its sign bit set exactly for the in-arcs above b (every nd >= b, and
        // nd - b < 2^31), and a real key's bit 31 is clear (rank << 16, rank < 512), so
        // OR-ing that bit into the key leaves only the tight ones in the running min -- one
        // subtract and one v_and_or per in-arc instead of a compare (+ its SGPR-mask wait
        // states) and a select: 26.70 -> 26.56 ms per 1M metric strings (A/B, one box).
        // (tight_min's select-then-min3 tree measured 0.5 % slower here.)
        if constexpr (F32 && !kTightSelect) {
#pragma unroll
          for (int m = 0; m < KP; ++m) c = min(c, pk[m] | ((b - nd[m]) & 0x80000000u));
        } else {
#pragma unroll
          for (int m = 0; m < KP; ++m) c = min(c, nd[m] == b ? pk[m] : kEmptyKey);
        }
        if (want_work()) {
#pragma unroll
          for (int m = 0; m < KP; ++m) relax += (uint32_t)__popcll(__ballot(rw[m] < kPullAbsent));
        }
        // the back record: RK 3 (direct layout) keeps one byte, the in-arc's position
        // x * KP + m in its target's group (block x, slot m; the chase re-derives the record
        // from the target state); the other kinds the record index itself
        uint32_t ra = (REC4 ? 0u : rec0) + ((c >> kMShift) & 15u);
        // groups of more than KP in-arcs: the further blocks, rare (a hub state)
        if (__ballot(nb > 1)) {
          if constexpr (DIRECT) {  // block 1's record; the true count past 255 blocks
            const uint2 xr = nb > 1 ? rv.rxrec[t] : make_uint2(0u, nb);
            xrec = xr.x;
            nb = xr.y;
          }
          for (uint32_t x = 1;; ++x) {
            const bool act = nb > x;
            if (!__ballot(act)) break;
            // inactive lanes read a padding block (indirect: block 0; direct: the block of
            // the first padding state past the last one)
            const uint32_t rx = act ? (DIRECT ? xrec + (x - 1) * KP : rec0 + x * KP)
                                    : (DIRECT ? rhs.num_states * KP : 0u);
#pragma unroll
            for (int m = 0; m < KP; ++m) {
              uint32_t p2, w2;
              DT n2;
              pull_candidate<W>(S, rec(rx + m), tmin8, p2, n2, w2);
              f = min(f, p2);
              if (n2 < b || (n2 == b && p2 < c)) {
                b = n2;
                c = p2;
                ra = REC4 ? x * KP + m : rx + m;
              }
              if (want_work()) relax += (uint32_t)__popcll(__ballot(w2 < kPullAbsent));
            }
          }
        }
        fst[e] = f;
        bd[e] = b;
        bk[e] = c;
        bra[e] = ra;
        if (f < kPullAbsent) {  // a tuple: mark its first key (rank << 3 | j)
          const uint32_t key = f >> kFirstShift;
          // (a 32-bit OR into the word's half: ~4 lanes of a row share an address instead
          // of ~8, and same-address LDS atomics serialise -- they were all of the kernel's
          // LDS conflict cycles)
          atomicOr(reinterpret_cast<uint32_t*>(S.bits) + FB(key >> 5, 2 * kWords, 158), 1u << (key & 31u));
        }
      }
      wave_lds_sync();

      // ---- (P2) ranks: popcount prefix over the first-key bitmap ----
      const uint32_t nw = (n_cur * 8 + 63) / 64;  // keys < 8 * n_cur
      unsigned long long word = 0;
      if (lane < nw) word = S.bits[FB(lane, kWords, 159)];
      const uint32_t pc = (uint32_t)__popcll(word);
      const uint32_t inc = wave_incl_scan_dpp(pc);
      const uint32_t n_next = __builtin_amdgcn_readlane(inc, 63);
      if (lane < nw) {
        // per 32-bit half: {popcount of the keys before it, its bits}, so P3's lookup is one
        // 32-bit mask and count
        S.pre[FB(lane, kWords, 160)] = make_uint4(inc - pc, (uint32_t)word,
                                 inc - pc + (uint32_t)__popc((uint32_t)word), (uint32_t)(word >> 32));
        S.bits[FB(lane, kWords, 161)] = 0;
      }
      wave_lds_sync();
      if (n_next == 0) {  // no candidate: the lattice dies here, no final is reachable
        n_cur = 0;
        break;
      }

      // ---- (P3) the next layer's cells (rewriting every row the current one used), back
      // records, and on the last layer the final candidates ----
      const bool last = k + 1 == L;
      if (lane == 0) hdr[k] = make_uint2(base, tmin);  // layer k: where its sources sit
      const uint32_t rows_w = max(rows_n, (wk + 63) / 64);
      uint32_t lo_slot = kEmptyKey, hi_slot = 0;  // uniform: present slots of the next layer
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        if ((uint32_t)e >= rows_w) continue;  // uniform
        const uint32_t i = (uint32_t)e * 64 + lane;
        if ((uint32_t)e >= rows_n) {  // uniform: a row past the next layer's window, emptied
          set_cell(i, bd[e], kPullAbsent);
          continue;
        }
        // (the row test as its own uniform branch: folded into pres, the compiler kept it
        // as a lane mask and rebuilt masks from it per row, 2 VALU each)
        uint32_t fe = fst[e];
        asm volatile("" : "+v"(fe));  // (a fresh compare here: P1's, kept across P2 under
                                      // another exec mask, was rebuilt with 2 VALU)
        const bool pres = fe < kPullAbsent;
        const uint32_t key = pres ? fe >> kFirstShift : 0u;
        const uint2 p = reinterpret_cast<const uint2*>(S.pre)[FB(key >> 5, 2 * kWords, 162)];
        const uint32_t rank = p.x + (uint32_t)__popc(p.y & ((1u << (key & 31u)) - 1u));
        // (an absent slot keeps its merged distance, +inf or >= kDistAbsent: no select; the
        // rank word alone marks it absent)
        set_cell(i, bd[e], pres ? rank << kRankShift : kPullAbsent);
        const unsigned long long pm = __ballot(pres);
        if (pm) {
          lo_slot = min(lo_slot, (uint32_t)e * 64 + (uint32_t)__builtin_ctzll(pm));
          hi_slot = max(hi_slot, (uint32_t)e * 64 + 63u - (uint32_t)__builtin_clzll(pm));
        }
        if (pres) {
          if constexpr (REC4)
            reinterpret_cast<uint8_t*>(back)[FB(nbase + i, lp.back_cap, 61)] = (uint8_t)bra[e];
          else
            *const_cast<uint32_t*>(at_byte(back, FB(nbase + i, lp.back_cap, 61) * 4u)) = bra[e];
          if (last) {  // final candidates, lexmin (total, rank) within the lane
            const uint32_t t = tn + i;
            const double fw2 = rhs.final_w[FB(t, rhs.num_states, 62)];
            if (!w_is_zero((double)bd[e]) && !w_is_zero(fw2)) {
              // times(d, times(One, fw2)), in f64 (f32 cells hold d exactly, scaled by 2^k)
              const unsigned long long kk = okey((double)bd[e] * (F32 ? rv.winv : 1.0) + fw2);
              const uint32_t pp = (rank << 9) | i;
              if (kk < mykey || (kk == mykey && pp < myp)) {
                mykey = kk;
                myp = pp;
                myfw = fw2;
              }
            }
          }
        }
      }
      tmin = tn;
      base = nbase;
      wk = wn;
      n_cur = n_next;
      tuples += n_next;
      cmin = tn + lo_slot;
      cmax = tn + hi_slot;
      wave_lds_sync();
    }
    wlast = wk;

    if (fail != kPathOk) {
      if (lane == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }
    if (L == 0 && lane == 0) {  // the start tuple is the whole lattice
      const double fw2 = rhs.final_w[rhs.start];
      if (!w_is_zero(fw2)) {
        mykey = okey(w_one() + fw2);
        myp = 0;
        myfw = fw2;
      }
    }
    uint32_t bp;
    double fw2;
    if (n_cur == 0 || !wave_pick_best(S.best, S.bestp, lane, mykey, myp, myfw, bp, fw2)) {
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
      ChaseJob& j = S.job[FB(njobs, kChaseBatch, 163)];
      j.si = si;
      j.L = L;
      j.id = base + (bp & 511u);  // shortest-path.zig:109-136 starts at the best final
      j.pad = tmin + (bp & 511u);  // (its state: RK 3's records hold sources relative to it)
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
