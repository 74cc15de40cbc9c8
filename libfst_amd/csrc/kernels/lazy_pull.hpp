// lazy_pull.hpp -- composeShortestPath (FST_SEM_LAZY) on layered lattices, one wavefront
// per string, PULL formulation over the reverse mirror of tier P (gfx950 / CDNA4).
//
// Domain: chain inputs without label 0 against an rhs without input epsilons, finite
// weights >= 0 (every lattice arc goes from layer k to layer k+1).  The reference
// (src/ops/compose-shortest-path.zig:26-401) pops min (dist, id) with ids given at first
// touch (getOrCreate, :70-89); the answer depends on the ids through the tie rules of
// relax (:107-141) and of the best final (:165-179).  tests/lazy_pull_model.py states the
// argument and is checked against the oracle's sequential replay:
//
//   C  if every tuple x but the start has a tight in-neighbour u that pops before it --
//      d(u) < d(x), or d(u) == d(x) and id(u) < id(x) -- the pop order is exactly the
//      sort by (dist, id).
//
// Under C every piece of the answer is layer-local, so a layer costs a pull merge like
// tier P's plus one sort:
//   * p_k  = pop rank within layer k = rank of (d, r_k)           -- stable LSD split sort
//   * r_k+1 (id order within layer k+1) = order of (p_k(u*), j*), u* = the first toucher
//     (the in-neighbour popped first), j* its candidate position    -- first-key bitmap
//   * back(x) = lexmin (r_k(u), j) over tight in-arcs (relax's (id, il, ol) order with il
//     fixed by the layer; the reverse mirror is built only when, for arcs of one source
//     into one target, candidate order = ol order)
//   * best = lexmin (total, r_L)
// C needs id(u) < id(x) across adjacent layers: id(u) < id(x) iff u's first toucher popped
// before x's, recursively down the chains of first touchers.  Each cell keeps tb = d(u*)
// (-1 for the start) and run = the length of the initial run of equal distances in its
// chain; a tight u certifies x when tb(u) < tb(x), or tb equal and run(u) < run(x).  A
// string with an uncertified tuple ends OVERFLOW and the rounds engine (lazy_layered.hpp)
// takes it.
#pragma once

#include <type_traits>

#include "eager_pull.hpp"  // RevView helpers, pull_group, wave_incl_scan_dpp, ChaseJob

extern "C" __device__ double __ockl_wfred_min_f64(double);
extern "C" __device__ double __ockl_wfred_max_f64(double);
extern "C" __device__ unsigned long long __ockl_wfred_or_u64(unsigned long long);

namespace fstamd {

constexpr uint32_t kLpAbsent = 0xFFF00000u;  // rank words of a slot that holds no tuple
constexpr uint32_t kLpRunMask = 0xFFFu;      // run (<= 4095 layers) below the pop rank
constexpr uint32_t kLpMaxLen = 4095;
// counting sort of the pop order: integer keys d - dmin below this (f32 cells: 128, so that
// 5 waves' LDS fits a CU; f64 cells: 64, so that 4 do -- round 6, was 256 at 3 waves)
template <typename DT>
constexpr int lp_bins() { return sizeof(DT) == 4 ? 128 : 64; }
// f32 cells keep d - tb (the first toucher's distance) in 8 bits of the pop word: the lazy
// pull takes f32 cells only when every arc weight is at most this
constexpr double kLpF32WMax = 255.0;
constexpr int kLpChase = 15;  // backtraces batched per wave (<= kChaseBatch: slabs)

// DT: the cells' distance storage.  double in general; uint32_t when every distance is an
// integer below 2^24 (integer -- or 2^k-scaled dyadic -- arc weights with L * max weight
// < 2^24, checked on the host: DeviceFst::int_wmax), which is exact and saves 2.5 KB.
// The current layer's cells (slot W never holds a tuple) in arrays of 8-B entries addressed
// by one byte offset o = 8 * slot.  Per cell: the distance d (+inf: no tuple), the id-rank
// word idw = id rank << 20 (kLpAbsent: no tuple), the pop word pw = pop rank << 20 | run
// (kLpAbsent: no tuple) and tb = the first toucher's distance (-1: the start).
template <int W, typename DT>
struct LazyPullCells {  // f64 distances: d, {idw, pw}, tb
  double d[W + 1];
  unsigned long long rp[W + 1];    // lo: idw; hi: pw
  double tb[W + 1];
  __device__ __forceinline__ const char* base(const void* a) const { return (const char*)a; }
  // (DEBUG_BOUNDS: byte offsets o < 8 (W + 1), slots i <= W, as every LDS index below)
  __device__ __forceinline__ double get_d(uint32_t o) const { return *(const double*)(base(d) + FB(o, 8 * (W + 1), 100)); }
  __device__ __forceinline__ uint32_t get_idw(uint32_t o) const { return *(const uint32_t*)(base(rp) + FB(o, 8 * (W + 1), 101)); }
  __device__ __forceinline__ uint32_t get_pw(uint32_t o) const { return *(const uint32_t*)(base(rp) + FB(o, 8 * (W + 1), 102) + 4); }
  __device__ __forceinline__ double get_tb(uint32_t o) const { return *(const double*)(base(tb) + FB(o, 8 * (W + 1), 103)); }
  __device__ __forceinline__ void set(uint32_t i, double dd, uint32_t idw, uint32_t pw, double t) {
    i = FB(i, W + 1, 104);
    d[i] = dd;
    rp[i] = ((unsigned long long)pw << 32) | idw;
    tb[i] = t;
  }
  __device__ __forceinline__ void set_pop(uint32_t i, uint32_t q) {  // pop rank q
    uint32_t* w = (uint32_t*)&rp[FB(i, W + 1, 105)] + 1;
    *w = (*w & kLpRunMask) | (q << 20);
  }
};
// integer distances (below 2^24; the F32 kernels, named for round 3's f32 cells -- u32
// since round 5: the add takes the 8-B record's weight byte as an operand, no conversion;
// kDistAbsent for no tuple): {d, idw} (8 B) and one 4-B pop word
// pw = pop rank << 20 | (255 - (d - tb)) << 12 | run, so the merge reads one 8-B word per in-arc
// (as tier P).  d - tb lies in [0, the largest arc weight]: the first toucher u* pops no
// later than a tight in-neighbour (d(u*) <= d), and d <= d(u*) + w; the start's tb = -1
// gives 1.  5 waves' cells, sort and jobs fit a CU's LDS (7.4 KB per wave).
// the pop word of an f32 cell: pop rank << 20 | cf << 12 | run, cf = 255 - (d - tb)
constexpr uint32_t kLpCfShift = 12, kLpCfMask = 0xFFu, kLpCkeyMask = 0xFFFFFu;
template <int W>
struct LazyPullCells<W, uint32_t> {
  uint2 a[W + 1];                  // {d, idw}
  uint32_t b[W + 1];               // pw
  __device__ __forceinline__ uint2 get_a(uint32_t o) const { return *(const uint2*)((const char*)a + FB(o, 8 * (W + 1), 106)); }
  __device__ __forceinline__ uint32_t get_d(uint32_t o) const { return get_a(o).x; }
  __device__ __forceinline__ uint32_t get_idw(uint32_t o) const { return get_a(o).y; }
  __device__ __forceinline__ uint32_t get_pw(uint32_t o) const {
    return *(const uint32_t*)((const char*)b + (FB(o, 8 * (W + 1), 107) >> 1));
  }
  // d - tb of the cell's tuple
  __device__ __forceinline__ uint32_t get_delta(uint32_t o) const {
    return kLpCfMask - ((get_pw(o) >> kLpCfShift) & kLpCfMask);
  }
  // an empty slot (the cells carry no tb: d - delta)
  __device__ __forceinline__ void set(uint32_t i, uint32_t dd, uint32_t idw, uint32_t pw, uint32_t) {
    i = FB(i, W + 1, 108);
    a[i] = make_uint2(dd, idw);
    b[i] = pw;
  }
  // pw carries the run in its low 12 bits and cf = 255 - (d - tb) above it
  __device__ __forceinline__ void set_packed(uint32_t i, uint32_t dd, uint32_t idw, uint32_t pwd) {
    i = FB(i, W + 1, 109);
    a[i] = make_uint2(dd, idw);
    b[i] = pwd;
  }
  __device__ __forceinline__ void set_pop(uint32_t i, uint32_t q) {
    i = FB(i, W + 1, 110);
    b[i] = (b[i] & 0xFFFFFu) | (q << 20);
  }
};

template <int W, typename DT>
struct LazyPullLds {
  static constexpr int kWords = W * 8 / 64;  // first keys p << 3 | j < 8 W
  // the sort buffers' entries: f64 cells keep slots (and counting keys < 64 above them) in
  // 16 bits, their split sort reads its keys from the cells: 10.0 KB of LDS per wave, so 4
  // waves per SIMD fit a CU (round 6; 32-bit entries and 256 bins were 12.8 KB, 3 waves)
  using OrdT = typename std::conditional<sizeof(DT) == 4, uint32_t, uint16_t>::type;
  LazyPullCells<W, DT> c;
  OrdT ord0[W];                    // (key << 9 |) slot in id order (f32 cells: first d)
  // P1-P3 use {bits, pre}; the sorts (P4, after P3 read pre) overlay the split sort's
  // second buffer ord1 or the counting sort's {mask, hist} on them.  bits must be all zero
  // when P1 starts: the counting sort leaves mask zero, the split sort re-zeroes bits.
  union {
    struct {
      unsigned long long bits[kWords];
      uint4 pre[kWords];
    };
    OrdT ord1[W];                  // split sort: the other buffer
    struct {
      unsigned long long mask[lp_bins<DT>()];  // lanes of the current 64-chunk holding key b
      uint32_t hist[lp_bins<DT>()];            // running count of key b, then its prefix
    };
  };
  unsigned long long best;
  uint32_t bestp;
  ChaseJob job[kLpChase];
};

// RK: the records, as in eager_pull_kernel (0 RevRec, 1 rrec32, 2 rrec8).  B1 (direct
// layout, DeviceFst::byte_back): 1-B back records, the back arc's position x * KP + m in its
// target's in-arc group (block x, slot m), as tier P's; the chase walks the states back from
// the best final's and re-derives each record from its target (block 0 at t * KP, blocks
// 1.. from rxrec[t].x).  Else 4-B records: the reverse record's index.
template <int EW, int KP, bool DIRECT, int WAVES_PER_EU, int RK, bool B1 = false>
__global__ void __launch_bounds__(64, WAVES_PER_EU)
lazy_pull_kernel(RhsView rhs, RevView rv, ChainInput in, uint32_t n_best,
                 unsigned int* next_item, EagerLaunch lp, BatchOutDev out) {
  constexpr int W = 64 * EW;
  constexpr bool F32 = RK != 0;
  // DT: the distance type of cells and of the merge's arithmetic (f32: exact for the
  // integer distances below 2^24 the host checked)
  using DT = typename std::conditional<F32, uint32_t, double>::type;
  // records: RevRec, or with f32 cells RevView::rrec32 {src, y, f32 weight, olabel} or
  // RevView::rrec8 {src, y | weight}.  The keys carry y: with rrec8 the weight sits in their
  // low 3 bits, so a cell offset taken from a key is masked with 0xFF8
  using RT = typename std::conditional<RK == 2, uint2,
                                       typename std::conditional<F32, uint4, RevRec>::type>::type;
  auto rec = [&](uint32_t r) -> RT {
    if constexpr (RK == 2) return rv.rrec8[r];
    else if constexpr (F32) return rv.rrec32[r];
    else return rv.rrec[r];
  };
  auto r_src = [](const RT& r) -> uint32_t {
    if constexpr (F32) return r.x;
    else return r.src;
  };
  auto r_w = [](const RT& r) -> DT {
    if constexpr (RK == 2) return rec8_weight(r.y);
    else if constexpr (F32) return r.z;  // (rrec32 holds the integer weight)
    else return r.weight;
  };
  constexpr int kWords = LazyPullLds<W, DT>::kWords;
  static_assert(KP <= 16 && W < 512, "key layout as in eager_pull.hpp");
  static_assert(!B1 || DIRECT, "byte back records need the direct layout");
  __shared__ LazyPullLds<W, DT> S;
  auto& CL = S.c;
#ifdef FSTAMD_LP_PAD  // occupancy experiment only: LDS padding to cut waves per SIMD
  __shared__ uint32_t pad_[FSTAMD_LP_PAD];
  if (threadIdx.x == 1000) pad_[0] = 0;
#endif
  const uint32_t lane = threadIdx.x;
  const DT kInf = dist_inf<DT>();
  // min of two distances >= +0 (no NaN: finite weights)
  auto lp_dmin = [](DT x, DT y) -> DT { return dist_min(x, y); };
  uint2* const slabs = lp.back_ws + (size_t)blockIdx.x * kChaseBatch * lp.back_cap;
  uint32_t njobs = 0;

  // the batched backtrace of tier P (shortest-path.zig:109-136 / compose-shortest-
  // path.zig:368-380: the path has exactly L arcs, one per layer)
  auto chase_batch = [&]() {
    wave_lds_sync();
    uint32_t maxL = 0;
    ChaseJob jb{};
    if (lane < njobs) {
      jb = S.job[FB(lane, kLpChase, 111)];
      maxL = jb.L;
    }
    maxL = __builtin_amdgcn_readfirstlane(__ockl_wfred_max_u32(maxL));
    // slab: back records (B1: 1 B, else the 4-B reverse record index of each tuple's back
    // arc) in its first half, per layer k {slab base, window origin} of layer k in its
    // second half: the record's source state gives the source's slab position
    const uint32_t* sl = reinterpret_cast<const uint32_t*>(slabs + (size_t)lane * lp.back_cap);
    const uint2* hdr = slabs + (size_t)lane * lp.back_cap + lp.back_cap / 2;
    uint32_t id = jb.id;
    uint32_t tcur = jb.pad;  // B1: the state of the tuple at slab position id
    for (uint32_t t = 0; t < maxL; ++t) {  // uniform trip count; lanes mask themselves
      if (lane < njobs && t < jb.L) {
        const uint32_t k = jb.L - 1 - t;
        uint32_t b;
        if constexpr (B1) {
          const uint32_t v = reinterpret_cast<const uint8_t*>(sl)[FB(id, lp.back_cap, 70)];
          b = FB(v < (uint32_t)KP ? tcur * KP + v : rv.rxrec[tcur].x + v - KP, rv.nrec, 73);
        } else {
          b = FB(sl[FB(id, lp.back_cap, 70)], rv.nrec, 73);
        }
        const uint2 h = hdr[k];
        if (!out.host_ol) out.out_il[jb.o + k] = in.labels[jb.off + k];
        uint32_t src8;
        if constexpr (RK == 2) {
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
        tcur = src8 >> 3;
        id = h.x + (tcur - h.y);
      }
    }
    if (lane < njobs) {
      out.status[jb.si] = kPathOk;
      if (out.first_status) out.first_status[jb.si] = kPathOk;
      out.path_len[jb.si] = jb.L;
      out.path_off[jb.si] = jb.o;
      out.final_w[jb.si] = jb.fw;
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
  // mask and rebuilt it per row with two readlanes, a select and a compare)
  const uint32_t want_work_w = __builtin_amdgcn_readfirstlane(out.work != nullptr ? 1u : 0u);
  auto want_work = [&]() -> bool {
    uint32_t w = __builtin_amdgcn_readfirstlane(want_work_w);
    asm volatile("" : "+s"(w));
    return w != 0u;
  };

#pragma unroll 1
  for (uint32_t i = lane; i < (uint32_t)W + 1; i += 64) CL.set(i, kInf, kLpAbsent, kLpAbsent, kInf);
  if (lane < (uint32_t)kWords) S.bits[FB(lane, kWords, 112)] = 0;
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
                         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)off0);  // (no sign ext.)
    const uint32_t L = __builtin_amdgcn_readfirstlane((uint32_t)(in.offsets[si + 1] - off));

    if (rhs.start == kNoState || n_best != 1) {  // compose-shortest-path.zig:30-33
      if (lane == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();

    // layer 0: the start tuple (id 0, pop rank 0, tb -1 < every distance)
#pragma unroll 1
    for (uint32_t i = lane; i < wlast; i += 64) CL.set(i, kInf, kLpAbsent, kLpAbsent, kInf);
    wave_lds_sync();
    if (lane == 0) {
      if constexpr (F32) CL.set_packed(0, 0u, 0u, (kLpCfMask - 1u) << kLpCfShift);  // d - tb = 1
      else CL.set(0, (DT)w_one(), 0u, 0u, (DT)-1.0);
    }
    wave_lds_sync();
    uint32_t tmin = rhs.start, wk = 1, base = 0, n_cur = 1;
    uint32_t cmin = rhs.start, cmax = rhs.start;
    uint32_t tuples = 1, relax = 0;
    int32_t fail = L > kLpMaxLen || (F32 && L > in.max_len) ? kPathOverflow : kPathOk;
    unsigned long long mykey = kMaxU64;
    uint32_t myp = kEmptyKey;
    double myfw = 0.0;

    uint32_t labs = 0;
    // uniform: the current layer's pop ranks equal its id ranks (layer 0; every layer the
    // sort below finds already in order, or with at most one tuple): the merge's first
    // toucher is then its smallest candidate key, read from the id-rank words alone
    bool io = true;
    for (uint32_t k = 0; k < L && fail == kPathOk; ++k) {
      if ((k & 15u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > lp.wd_ticks) {
        fail = kPathInternal;
        break;
      }
      if ((k & 63u) == 0) labs = k + lane < L ? in.labels[off + k + lane] : 0u;
      const uint32_t lab = __builtin_amdgcn_readlane(labs, k & 63u);
      if (lab == kEpsilon) {
        fail = kPathUnsupported;
        break;
      }
      const uint32_t tn = cmin >= rhs.jump_back ? cmin - rhs.jump_back : 0u;
      // (32-bit: the pull tiers take rhs of fewer than 2^27 states, so cmax + jump_fwd
      // cannot wrap, and the compares stay scalar -- u64 ones went to the VALU)
      const uint32_t hi = min(cmax + rhs.jump_fwd, rhs.num_states - 1);
      const uint32_t nbase = base + wk;
      // (the slab's second half holds one header entry per layer: k < back_cap / 2)
      if (hi - tn >= (uint32_t)W || nbase + (hi - tn + 1) > lp.back_cap ||
          k >= lp.back_cap / 2) {
        fail = kPathOverflow;
        break;
      }
      const uint32_t wn = hi - tn + 1;
      const uint32_t rows_n = (wn + 63) / 64;
      const bool check_c = k + 1 < L;  // the last layer's pop order is never used

      // ---- (P1) pull merge per target: first toucher, distance, back-pointer, C ----
      uint32_t fst[EW], bk[EW], bra[EW], runx[EW];
      DT bd[EW], tbx[EW];
      // f32 cells: the distance (an integer below 2^24) and d - tb (<= 255) share one word,
      // the run sits in fst's low 17 bits (P3 reads only fst >> 17): 3 words per row live
      // across P2 instead of 6 (5 waves per SIMD)
      uint32_t bdp[EW];
      bool uncert = false;
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        fst[e] = kEmptyKey;
        bk[e] = kEmptyKey;
        bra[e] = 0;
        bd[e] = kInf;
        tbx[e] = kInf;
        runx[e] = 0;
        bdp[e] = 0;
        if ((uint32_t)e >= rows_n) continue;  // uniform
        const uint32_t i = (uint32_t)e * 64 + lane;
        const uint32_t t = tn + i;
        uint32_t rec0, nb, xrec = 0;
        uint32_t tmin8 = tmin << 3;
        if constexpr (DIRECT) {
          const uint32_t rs = *at_byte(rv.rlab, t * 4u);  // ilabel | min(nblocks, 255) << 24
          const bool hit = (rs & 0xFFFFFFu) == lab && lab < kSpanMixed;
          tmin8 = hit ? tmin8 : tmin8 + 0x80000000u;  // no in-arc of this label (tier P)
          rec0 = t * KP;
          nb = hit ? rs >> 24 : 0u;
        } else {
          pull_group(rv, lab, t, rec0, nb);
        }
        // first record of block x >= 1 of a group longer than one block (a hub state);
        // lanes without one read a padding block
        auto block_rec = [&](uint32_t x) -> uint32_t {
          if (nb > x) return DIRECT ? xrec + (x - 1) * KP : rec0 + x * KP;
          return DIRECT ? rhs.num_states * KP : 0u;
        };
        const bool hubs = __ballot(nb > 1) != 0;  // uniform
        RT rr[KP];
        // one base address, the records at immediate offsets
        const RT* R;
        if constexpr (RK == 2) R = at_byte(rv.rrec8, rec0 * 8u);  // (32-bit byte offset)
        else if constexpr (F32) R = rv.rrec32 + rec0;
        else R = rv.rrec + rec0;
#pragma unroll
        for (int m = 0; m < KP; ++m) rr[m] = R[m];
        uint32_t bpk[KP];
        DT nd[KP];
        uint32_t ff = kEmptyKey;
        DT b = kInf;
        if (io) {  // pop ranks = id ranks: the first toucher is the smallest candidate key
#pragma unroll
          for (int m = 0; m < KP; ++m) {
            const uint32_t o = min(r_src(rr[m]) - tmin8, 8u * W);
            nd[m] = CL.get_d(o) + r_w(rr[m]);  // times(d, w) for finite w >= 0 (:108)
            bpk[m] = CL.get_idw(o) | rr[m].y | o;
            ff = min(ff, bpk[m]);
            b = lp_dmin(b, nd[m]);
          }
        } else {
#pragma unroll
          for (int m = 0; m < KP; ++m) {
            const uint32_t o = min(r_src(rr[m]) - tmin8, 8u * W);
            nd[m] = CL.get_d(o) + r_w(rr[m]);
            bpk[m] = CL.get_idw(o) | rr[m].y | o;
            ff = min(ff, (CL.get_pw(o) & kLpAbsent) | rr[m].y | o);
            b = lp_dmin(b, nd[m]);
          }
        }
        if (want_work()) {  // (one uniform branch per row; an absent source's key >= kLpAbsent)
#pragma unroll
          for (int m = 0; m < KP; ++m) relax += (uint32_t)__popcll(__ballot(bpk[m] < kLpAbsent));
        }
        // the back key: tier P's sign-bit form on the integer cells (b - nd has its sign bit
        // set exactly for the non-tight in-arcs, a real key's bit 31 is clear; round 5: the
        // u32 cells and this key 46.7 -> 45.3 ms per 1M metric strings, A/B on one box; on
        // round 4's f32 bit patterns it was 2 % slower than the select tree)
        uint32_t c;
#ifndef FSTAMD_LP_TIGHTSEL  // A/B: the select tree (tight_min) on every cell type
        if constexpr (F32) {
          c = kEmptyKey;
#pragma unroll
          for (int m = 0; m < KP; ++m) c = min(c, bpk[m] | ((b - nd[m]) & 0x80000000u));
        } else {
          c = tight_min<KP>(nd, b, bpk);
        }
#else
        c = tight_min<KP>(nd, b, bpk);
#endif
        uint32_t ra = (B1 ? 0u : rec0) + ((c >> 13) & 15u);
        if (hubs) {  // the further blocks: first toucher, distance, back-pointer
          // (block 1's record, loaded here: a branch before the row's record loads would
          // hold them behind the label load)
          if constexpr (DIRECT) {  // block 1's record; the true count past 255 blocks
            const uint2 xr = nb > 1 ? rv.rxrec[t] : make_uint2(0u, nb);
            xrec = xr.x;
            nb = xr.y;
          }
          for (uint32_t x = 1;; ++x) {
            if (!__ballot(nb > x)) break;
            const uint32_t rxx = block_rec(x);
#pragma unroll
            for (int m = 0; m < KP; ++m) {
              const RT r2 = rec(rxx + m);
              const uint32_t o = min(r_src(r2) - tmin8, 8u * W);
              const DT n2 = CL.get_d(o) + r_w(r2);
              const uint32_t iw = CL.get_idw(o);
              const uint32_t p2 = iw | r2.y | o;
              ff = min(ff, (CL.get_pw(o) & kLpAbsent) | r2.y | o);
              if (n2 < b || (n2 == b && p2 < c)) {
                b = n2;
                c = p2;
                ra = B1 ? x * KP + m : rxx + m;
              }
              if (want_work()) relax += (uint32_t)__popcll(__ballot(iw < kLpAbsent));
            }
          }
        }
        const bool pres = ff < kLpAbsent;
        // the first toucher's cell: tb(x) = d(u*), run(x) = 1 + run(u*) if tb(u*) == tb(x)
        // (no select for absent lanes: their keys' offsets are in-bounds LDS addresses too,
        // and nothing they read is used)
        const uint32_t ou = ff & 0xFF8u;
        const DT du = CL.get_d(ou);
        const uint32_t pwu = CL.get_pw(ou);
        const uint32_t ruu = pwu & kLpRunMask;
        // the back-pointer source's cell (a tight in-neighbour), read in the same LDS
        // round trip: its certificate alone usually settles C
        const uint32_t ob = c & 0xFF8u;
        const uint32_t pwb = CL.get_pw(ob);
        const DT tx = du;
        // C: a tight in-arc of positive weight pops before x; else a tight 0-weight
        // source certified by (tb, run).  The back arc is tight, so its own certificate
        // (positive weight: kRevPos in its key, or its source's (tb, run)) is sufficient;
        // the loop over every tight in-arc runs only for rows where some lane is left
        // without one.
        // f32 cells: a tight 0-weight source u sits at d(u) = b, so tb(u) < tb(x) iff
        // d(u) - tb(u) > b - tb(x): with the cell field cf = 255 - (d - tb), (tb, run)(u) <
        // (tb, run)(x) is one integer compare of (cf << 12 | run), the pop word's low 20
        // bits (a positive-weight in-arc certifies by itself, so its field never decides)
        uint32_t rx, ckx = 0;
        DT tbu = 0;
        bool fast;
        if constexpr (F32) {
          rx = 1u + (((pwu >> kLpCfShift) & kLpCfMask) == kLpCfMask ? ruu : 0u);  // tb(u*) == d(u*)
          ckx = ((kLpCfMask - (uint32_t)(b - du)) << kLpCfShift) | rx;
          fast = !pres || (c & kRevPos) || (pwb & kLpCkeyMask) < ckx;
        } else {
          tbu = CL.get_tb(ou);
          rx = 1u + (tbu == tx ? ruu : 0u);
          const DT tbb = CL.get_tb(ob);
          const uint32_t rbb = pwb & kLpRunMask;
          fast = !pres || (c & kRevPos) || tbb < tx || (tbb == tx && rbb < rx);
        }
        // the lanes whose back arc does not certify them, as SALU ANDs of compare masks (a
        // ballot of the OR-ed predicate costs two VALU to materialise it)
        auto lanes_without = [](bool pr, uint32_t cc, uint32_t pwbb, uint32_t ck,
                                bool fst_) -> unsigned long long {
          if constexpr (F32)
            return __ballot(pr) & ~__ballot((cc & kRevPos) != 0u) &
                   ~__ballot((pwbb & kLpCkeyMask) < ck);
          else return __ballot(!fst_);
        };
        auto certifies = [&](uint32_t pw_src, DT tb_src) -> bool {  // a tight 0-weight source
          if constexpr (F32) return (pw_src & kLpCkeyMask) < ckx;
          else return tb_src < tx || (tb_src == tx && (pw_src & kLpRunMask) < rx);
        };
#ifdef FSTAMD_LP_NOCERT  // timing experiment only: no certificate check
        if (false) {
#elif defined(FSTAMD_LP_FULLCERT)  // A/B: the full loop on every row that needs it
        if (check_c && __ballot(pres && (!(c & kRevPos) || nb > 1))) {
#else
        uint32_t ff2 = ff;  // (a fresh compare for the ballot, as in P3 below)
        asm volatile("" : "+v"(ff2));
        if (check_c && lanes_without(ff2 < kLpAbsent, c, pwb, ckx, fast)) {
#endif
#ifdef FSTAMD_LP_FULLCERT
          bool cert = !pres || (c & kRevPos);
#else
          bool cert = fast;
#endif
#pragma unroll
          for (int m = 0; m < KP; ++m) {
            const uint32_t o = bpk[m] & 0xFF8u;
            DT tbm = 0;
            if constexpr (!F32) tbm = CL.get_tb(o);
            // (short-circuit: two exec-mask branches per in-arc, but the LDS read only for
            // tight 0-weight in-arcs; the bitwise form that reads every pop word measured
            // 2 % slower, round 5)
            cert |= nd[m] == b && ((bpk[m] & kRevPos) || certifies(CL.get_pw(o), tbm));
          }
          if (hubs) {  // the further blocks' tight in-arcs
            for (uint32_t x = 1;; ++x) {
              if (!__ballot(nb > x)) break;
              const uint32_t rxx = block_rec(x);
#pragma unroll
              for (int m = 0; m < KP; ++m) {
                const RT r2 = rec(rxx + m);
                const uint32_t o = min(r_src(r2) - tmin8, 8u * W);
                const DT d = CL.get_d(o);
                DT tbm = 0;
                if constexpr (!F32) tbm = CL.get_tb(o);
                cert |= d + r_w(r2) == b && (r_w(r2) > (DT)0 || certifies(CL.get_pw(o), tbm));
              }
            }
          }
          uncert |= !cert;
        }
        bk[e] = c;
        bra[e] = ra;
        if constexpr (F32) {
          // (an absent lane keeps ff's high bits, >= kLpAbsent; its bdp is never read)
          fst[e] = (ff & ~0x1FFFFu) | rx;
          bdp[e] = (uint32_t)b | ((ckx >> kLpCfShift) << 24);
        } else {
          fst[e] = ff;
          bd[e] = b;
          tbx[e] = tx;
          runx[e] = rx;
        }
        if (pres) {
          const uint32_t key = ff >> 17;  // pop rank << 3 | j
          // (a 32-bit OR into the word's half: ~4 lanes of a row share an address instead
          // of ~8, and same-address LDS atomics serialise -- they were all of the kernel's
          // LDS conflict cycles)
          atomicOr(reinterpret_cast<uint32_t*>(S.bits) + FB(key >> 5, 2 * kWords, 113), 1u << (key & 31u));
        }
      }
      wave_lds_sync();

      // ---- (P2) id ranks of the next layer: popcount prefix over the first keys ----
      const uint32_t nw = (n_cur * 8 + 63) / 64;
      unsigned long long word = 0;
      if (lane < nw) word = S.bits[FB(lane, kWords, 114)];
      const uint32_t pc = (uint32_t)__popcll(word);
      const uint32_t inc = wave_incl_scan_dpp(pc);
      const uint32_t n_next = __builtin_amdgcn_readlane(inc, 63);
      if (lane < nw) {
        // per 32-bit half: {popcount of the keys before it, its bits}, so P3's lookup is one
        // 32-bit mask and count
        S.pre[FB(lane, kWords, 115)] = make_uint4(inc - pc, (uint32_t)word,
                                 inc - pc + (uint32_t)__popc((uint32_t)word), (uint32_t)(word >> 32));
        S.bits[FB(lane, kWords, 116)] = 0;
      }
      wave_lds_sync();
      // an uncertified tuple: the rounds engine takes the string
      if (__ballot(uncert)) {
        fail = kPathOverflow;
        break;
      }
      if (n_next == 0) {
        n_cur = 0;
        break;
      }

      // ---- (P3) the next layer's cells (pop ranks after the sort), back records, and the
      // id order's slots for P4 ----
      const bool last = k + 1 == L;
      if (lane == 0) hdr[k] = make_uint2(base, tmin);  // layer k: where its sources sit
      const bool sort = !last && n_next > 1;  // the last layer's pop order is never used
      const uint32_t rows_w = max(rows_n, (wk + 63) / 64);
      uint32_t lo_slot = kEmptyKey, hi_slot = 0;
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        if ((uint32_t)e >= rows_w) continue;
        const uint32_t i = (uint32_t)e * 64 + lane;
        // a fresh compare (rows past rows_n keep fst = kEmptyKey): P1's mask, kept across P2,
        // came back as a select and a compare per row (round 6: 43.0 -> 42.4 ms, A/B)
        uint32_t fe = fst[e];
        asm volatile("" : "+v"(fe));
        const bool pres = fe < kLpAbsent;
        uint32_t rank = 0;
        if ((uint32_t)e < rows_n) {
          const uint32_t key = pres ? fst[e] >> 17 : 0u;
          const uint2 p = reinterpret_cast<const uint2*>(S.pre)[FB(key >> 5, 2 * kWords, 117)];
          rank = p.x + (uint32_t)__popc(p.y & ((1u << (key & 31u)) - 1u));
        }
        // pop rank: identity until the sort below fills it in
        DT dx;
        if constexpr (F32) {
          // (branch-free: an absent slot's words are OR-ed with kLpAbsent, which covers
          // rank << 20; readers of an absent cell's pop word look only at those high bits)
          const uint32_t gone = pres ? 0u : kLpAbsent;
          dx = pres ? (DT)(bdp[e] & 0xFFFFFFu) : kInf;
          CL.set_packed(i, dx, (rank << 20) | gone,
                        (rank << 20) | ((bdp[e] >> 24) << kLpCfShift) | (fst[e] & kLpRunMask) |
                            gone);
        } else {
          dx = bd[e];
          CL.set(i, pres ? bd[e] : kInf, pres ? rank << 20 : kLpAbsent,
                 pres ? (rank << 20) | runx[e] : kLpAbsent, pres ? tbx[e] : kInf);
        }
        // (f32 cells: the distance's bits, ordered as the non-negative distances are; P4
        // rebuilds the slots from the cells' id-rank words when the layer needs its sort)
        if (pres && sort) S.ord0[FB(rank, W, 118)] = F32 ? (uint32_t)dx : i;
        const unsigned long long pm = __ballot(pres);
        if (pm) {
          lo_slot = min(lo_slot, (uint32_t)e * 64 + (uint32_t)__builtin_ctzll(pm));
          hi_slot = max(hi_slot, (uint32_t)e * 64 + 63u - (uint32_t)__builtin_clzll(pm));
        }
        if (pres) {
          if constexpr (B1)
            reinterpret_cast<uint8_t*>(back)[FB(nbase + i, lp.back_cap, 71)] = (uint8_t)bra[e];
          else
            *const_cast<uint32_t*>(at_byte(back, FB(nbase + i, lp.back_cap, 71) * 4u)) = bra[e];
          if (last) {  // best final: lexmin (total, id) (compose-shortest-path.zig:165-179)
            const uint32_t t = tn + i;
            const double fw2 = rhs.final_w[FB(t, rhs.num_states, 72)];
            if (!w_is_zero(fw2)) {
              const unsigned long long kk = okey((double)dx * (RK ? rv.winv : 1.0) + fw2);
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
      wave_lds_sync();

      // ---- (P4) pop ranks: stable sort of the id order by distance.  Integer distances
      // (integer weights, the metric's) are keyed as d - dmin; keys < 256 take a counting
      // sort, the rest a stable LSD split sort (one bit per pass, only the bits that
      // differ; f64 bit patterns when the distances are not integers) ----
#ifdef FSTAMD_LP_NOSORT  // timing experiment only: wrong pop ranks
      if (false) {
#else
      if (sort) {
#endif
        const uint32_t rows_s = (n_next + 63) / 64;
        // already in order (the metric's layers, every one of them): the id order is the
        // pop order and the identity ranks written in P3 stand; nothing below runs (no
        // reductions, no keys: the check compares the cells' distances in id order)
        // (round 6: the check as SALU ORs of per-row ballots with a uniform lane bound
        // measured 42.45 vs 42.37 ms, not kept)
        bool unsorted = false;
#pragma unroll
        for (int e = 0; e < EW; ++e) {
          if ((uint32_t)e >= rows_s) continue;  // uniform
          const uint32_t q = (uint32_t)e * 64 + lane;
          if (q + 1 < n_next) {
            if constexpr (F32) unsorted |= S.ord0[FB(q, W, 119)] > S.ord0[FB(q + 1, W, 120)];
            else unsorted |= CL.get_d(8 * S.ord0[FB(q, W, 119)]) > CL.get_d(8 * S.ord0[FB(q + 1, W, 120)]);
          }
        }
        const bool in_order = !__ballot(unsorted);
        if (!in_order) {
        if constexpr (F32) {  // the id order's slots, from the cells' id ranks
          wave_lds_sync();
#pragma unroll
          for (int e = 0; e < EW; ++e) {
            if ((uint32_t)e >= rows_n) continue;  // uniform
            const uint32_t i = (uint32_t)e * 64 + lane;
            const uint32_t iw = CL.get_idw(8 * i);
            if (iw < kLpAbsent) S.ord0[FB(iw >> 20, W, 121)] = i;
          }
          wave_lds_sync();
        }
        // keys: integer distances with d - dmin < 2^23 (ik) sort by d - dmin, others by
        // their f64 bit patterns; dmin / dmax over the layer, then key << 9 | slot in ord0
        DT mn = kInf, mx = F32 ? (DT)0 : -kInf;
        bool nonint = false;
        uint32_t cs[EW];
        DT cd[EW];
#pragma unroll
        for (int e = 0; e < EW; ++e) {
          cs[e] = 0;
          cd[e] = (DT)0;
          if ((uint32_t)e >= rows_s) continue;  // uniform
          const uint32_t q = (uint32_t)e * 64 + lane;
          if (q < n_next) {
            cs[e] = S.ord0[FB(q, W, 122)];
            cd[e] = CL.get_d(8 * cs[e]);
            mn = dist_min(mn, cd[e]);
            if constexpr (F32) mx = max(mx, cd[e]);
            else mx = fmax(mx, cd[e]);
            if (!F32) nonint |= cd[e] != __builtin_trunc(cd[e]);
          }
        }
        if constexpr (F32) {
          mn = __ockl_wfred_min_u32(mn);
          mx = __ockl_wfred_max_u32(mx);
        } else {
          mn = __ockl_wfred_min_f64(mn);
          mx = __ockl_wfred_max_f64(mx);
        }
        // (f64 cells: integer keys only where the counting sort takes them -- their 16-bit
        // sort entries hold key << 9 | slot for keys < 64; the split sort reads f64 bit
        // patterns from the cells otherwise)
        const bool ik = __ballot(nonint) == 0 &&
                        (double)mx - (double)mn < (F32 ? 8388608.0 : (double)lp_bins<DT>());
        const unsigned long long mnb = (unsigned long long)__double_as_longlong((double)mn);
        uint32_t kacc = 0;            // OR of the integer keys
        unsigned long long diff = 0;  // OR of the f64 patterns' differences from dmin's
#pragma unroll
        for (int e = 0; e < EW; ++e) {
          if ((uint32_t)e >= rows_s) continue;  // uniform
          const uint32_t q = (uint32_t)e * 64 + lane;
          if (q < n_next) {
            const uint32_t key = ik ? (uint32_t)(cd[e] - mn) : 0u;  // exact: integers < 2^23
            S.ord0[FB(q, W, 123)] = (key << 9) | cs[e];
            kacc |= key;
            if constexpr (!F32)  // (f32 cells: integer distances, ik)
              diff |= ik ? 0ull : (unsigned long long)__double_as_longlong((double)cd[e]) ^ mnb;
          }
        }
        wave_lds_sync();
#ifdef FSTAMD_LP_SPLIT_ONLY  // A/B: the split sort for every layer
        const bool counting = false;
#else
        const bool counting = ik && mx - mn < (DT)lp_bins<DT>();
#endif
        unsigned long long vary;
        if (ik) {
          vary = (unsigned long long)__builtin_amdgcn_readfirstlane(__ockl_wfred_or_u32(kacc)) << 9;
        } else {
          const unsigned long long dv = __ockl_wfred_or_u64(diff);
          vary = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(dv >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)dv);
        }
        if (counting) {
          // stable counting sort, 64 ids at a time in id order: the lanes holding key b
          // meet in mask[b] (LDS OR), a lane's rank among them = the equal keys before
          // it in the chunk; hist[b] carries the count from earlier chunks.  One wave's
          // LDS operations complete in order, so the fences below separate the steps.
#pragma unroll
          for (int b = 0; b < lp_bins<DT>() / 64; ++b) {
            S.mask[FB(b * 64 + lane, lp_bins<DT>(), 124)] = 0;
            S.hist[FB(b * 64 + lane, lp_bins<DT>(), 125)] = 0;
          }
          wave_lds_sync();
          uint32_t ck[EW], cw[EW];
#pragma unroll
          for (int e = 0; e < EW; ++e) {  // every row's (key, slot) in one LDS round trip
            ck[e] = 0;
            if ((uint32_t)e < rows_s && (uint32_t)e * 64 + lane < n_next) ck[e] = S.ord0[FB(e * 64 + lane, W, 126)];
          }
#pragma unroll
          for (int e = 0; e < EW; ++e) {
            cw[e] = 0;
            if ((uint32_t)e >= rows_s) continue;  // uniform
            const uint32_t q = (uint32_t)e * 64 + lane;
            const bool valid = q < n_next;
            const uint32_t key = ck[e] >> 9;
            if (valid) atomicOr(&S.mask[FB(key, lp_bins<DT>(), 127)], 1ull << lane);
            wave_lds_sync();
            const unsigned long long peers = valid ? S.mask[FB(key, lp_bins<DT>(), 128)] : 0ull;
            const uint32_t hb = valid ? S.hist[FB(key, lp_bins<DT>(), 129)] : 0u;
            wave_lds_sync();
            const unsigned long long lt = peers & ((1ull << lane) - 1ull);
            cw[e] = hb + (uint32_t)__popcll(lt);
            if (valid && lt == 0) {  // the key's first lane in this chunk
              S.hist[FB(key, lp_bins<DT>(), 130)] = hb + (uint32_t)__popcll(peers);
              S.mask[FB(key, lp_bins<DT>(), 131)] = 0;
            }
            wave_lds_sync();
          }
          // exclusive prefix of the counts: lane l holds keys 4l .. 4l+3 (256 bins), 2l,
          // 2l+1 (128 bins, f32 cells) or l (64 bins, f64 cells) -- never past hist, which
          // ends the union: the pending chase jobs follow it
          static_assert(lp_bins<DT>() == 256 || lp_bins<DT>() == 128 || lp_bins<DT>() == 64,
                        "bins per lane");
          if constexpr (lp_bins<DT>() == 64) {
            const uint32_t h = S.hist[FB(lane, lp_bins<DT>(), 142)];
            S.hist[FB(lane, lp_bins<DT>(), 143)] = wave_incl_scan_dpp(h) - h;
          } else if constexpr (lp_bins<DT>() == 256) {
            static_assert(4 * 64 == lp_bins<DT>(), "4 bins per lane cover hist exactly");
            const uint4 h = reinterpret_cast<const uint4*>(S.hist)[FB(lane, lp_bins<DT>() / 4, 132)];
            const uint32_t s4 = h.x + h.y + h.z + h.w;
            const uint32_t ex = wave_incl_scan_dpp(s4) - s4;
            reinterpret_cast<uint4*>(S.hist)[FB(lane, lp_bins<DT>() / 4, 133)] =
                make_uint4(ex, ex + h.x, ex + h.x + h.y, ex + h.x + h.y + h.z);
          } else {
            static_assert(2 * 64 == lp_bins<DT>(), "2 bins per lane cover hist exactly");
            const uint2 h = reinterpret_cast<const uint2*>(S.hist)[FB(lane, lp_bins<DT>() / 2, 134)];
            const uint32_t s2 = h.x + h.y;
            const uint32_t ex = wave_incl_scan_dpp(s2) - s2;
            reinterpret_cast<uint2*>(S.hist)[FB(lane, lp_bins<DT>() / 2, 135)] = make_uint2(ex, ex + h.x);
          }
          wave_lds_sync();
#pragma unroll
          for (int e = 0; e < EW; ++e) {  // pop rank -> the cell's high word
            if ((uint32_t)e >= rows_s) continue;
            if ((uint32_t)e * 64 + lane < n_next) {
              const uint32_t q = S.hist[FB(ck[e] >> 9, lp_bins<DT>(), 136)] + cw[e];
              CL.set_pop(ck[e] & 511u, q);
            }
          }
          wave_lds_sync();
          vary = 0;  // the split sort below has nothing to do
        }
        wave_lds_sync();
        uint32_t cur = 0;
        while (vary) {
          const uint32_t bit = (uint32_t)__builtin_ctzll(vary);
          vary &= vary - 1;
          uint32_t el[EW], v[EW];
          unsigned long long z[EW];
          uint32_t Z = 0;
#pragma unroll
          for (int e = 0; e < EW; ++e) {
            el[e] = 0;
            v[e] = 0;
            z[e] = 0;
            if ((uint32_t)e >= rows_s) continue;
            const uint32_t q = (uint32_t)e * 64 + lane;
            const bool valid = q < n_next;
            el[e] = valid ? (cur ? S.ord1 : S.ord0)[FB(q, W, 138)] : 0u;
            if (ik) {
              v[e] = (el[e] >> bit) & 1u;
            } else {
              const unsigned long long key =
                  (unsigned long long)__double_as_longlong((double)CL.get_d(8 * (el[e] & 511u)));
              v[e] = (uint32_t)(key >> bit) & 1u;
            }
            z[e] = __ballot(valid && !v[e]);
            Z += (uint32_t)__popcll(z[e]);
          }
          uint32_t zb = 0, ob = 0;
#pragma unroll
          for (int e = 0; e < EW; ++e) {
            if ((uint32_t)e >= rows_s) continue;
            const uint32_t q = (uint32_t)e * 64 + lane;
            const bool valid = q < n_next;
            const unsigned long long o = __ballot(valid && v[e]);
            const uint32_t below0 = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(z[e] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)z[e], 0u));
            const uint32_t below1 = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(o >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)o, 0u));
            const uint32_t dst = v[e] ? Z + ob + below1 : zb + below0;
            if (valid) (cur ? S.ord0 : S.ord1)[FB(dst, W, 139)] = el[e];
            zb += (uint32_t)__popcll(z[e]);
            ob += (uint32_t)__popcll(o);
          }
          cur ^= 1u;
          wave_lds_sync();
        }
        for (uint32_t q = lane; q < n_next && !counting; q += 64) {  // pop rank q -> cell
          CL.set_pop((cur ? S.ord1 : S.ord0)[FB(q, W, 140)] & 511u, q);
        }
        wave_lds_sync();
        if (!counting && lane < (uint32_t)kWords) S.bits[FB(lane, kWords, 137)] = 0;  // (ord1 overlays bits)
        wave_lds_sync();
        }  // !in_order
        io = in_order;
      } else {
        io = true;  // at most one tuple (or the last layer): identity pop ranks
      }
      tmin = tn;
      base = nbase;
      wk = wn;
      n_cur = n_next;
      tuples += n_next;
      cmin = tn + lo_slot;
      cmax = tn + hi_slot;
    }
    wlast = wk;

    if (fail != kPathOk) {
      // leave every cell empty for the next string (a failed string may stop mid-layer)
      wave_lds_sync();
#pragma unroll 1
      for (uint32_t i = lane; i < (uint32_t)W + 1; i += 64) CL.set(i, kInf, kLpAbsent, kLpAbsent, kInf);
      if (lane < (uint32_t)kWords) S.bits[FB(lane, kWords, 112)] = 0;
      wave_lds_sync();
      wlast = 0;
      if (lane == 0) write_status(out, si, fail, tuples, relax);
      continue;
    }
    if (L == 0 && lane == 0) {
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
        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)o);
    if (o + L > out.arc_cap) {
      if (lane == 0) write_status(out, si, kPathOutputFull, tuples, relax);
      continue;
    }
    if (lane == 0) {
      ChaseJob& j = S.job[FB(njobs, kLpChase, 141)];
      j.si = si;
      j.L = L;
      j.id = base + (bp & 511u);
      j.pad = tmin + (bp & 511u);  // (its state: B1's chase walks the states back from it)
      j.tuples = tuples;
      j.relax = relax;
      j.o = o;
      j.off = off;
      j.fw = fw2;
    }
    if (++njobs == (uint32_t)kLpChase) chase_batch();
  }
  if (njobs) chase_batch();
}

}  // namespace fstamd
