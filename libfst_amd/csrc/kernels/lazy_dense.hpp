// lazy_dense.hpp -- composeShortestPath (FST_SEM_LAZY) as an exact replay of the
// reference's pop sequence, one wavefront per string (gfx950 / CDNA4).
//
// Domain: chain inputs without label 0 against an rhs whose arc weights are finite and
// >= 0, WITH or without rhs input epsilons (the epsilon-dense lattices of config 3).  It
// replays src/ops/compose-shortest-path.zig:26-401 pop by pop -- the answer depends on
// the id each tuple gets at first touch (getOrCreate, :70-89) in (dist, id) pop order,
// and on epsilon-dense lattices almost every tuple sits at one distance, so the parallel
// rounds engines degenerate to one pop per round.  What makes a pop cheap here:
//   * tuple (k, s2, f) -- input position, rhs state, filter (0, or 1 after an rhs
//     epsilon; a chain without label 0 never reaches 2) -- lives at the dense index
//     (s2 * (L + 1) + k) * 2 + f: no hash, no probing.  State-major: on epsilon-dense
//     lattices the pops sweep the rhs states with every input position open at once, so
//     the live tuples of a wave stay in a few pages (position-major, they spread over
//     L + 1 pages of 2 * NS * 16 B: at T = 65,536 with ~250 waves resident, TLB misses made
//     a pop 6x slower).  rec[x] = {dist, id | settled, back
//     source id}: one 16-B load answers getOrCreate and relax (:99-141) for a target;
//   * the heap is split by distance.  With weights >= 0 the popped distances never
//     decrease, and the reference pops min (dist, id) among open tuples (stale and
//     settled entries skipped, :159-163), so:
//       - the open tuples AT the current distance dcur are a bitmap over ids (leaf words
//         in HBM, one summary bit per leaf in LDS); pop = lowest set bit.  Pops run in
//         near-id order, so the lowest non-empty leaf stays in registers and a pop costs
//         no memory access at all;
//       - tuples above dcur go to an unsorted list of (dist, tuple) entries.  When the
//         bitmap empties, one scan finds the smallest live distance (live: not settled,
//         dist unchanged), moves every live entry at that distance into the bitmap and
//         compacts the rest away;
//   * one pop's candidates (phase 1: rhs arcs labelled labels[k]; phase 3: rhs epsilon
//     arcs, :181-305) are read lane-parallel from the L2-resident rhs, permuted into the
//     reference's relax order through LDS and relaxed together: relaxations that hit the
//     same tuple are folded in order by the group's first lane with the reference's rule
//     (:110-128), new tuples are numbered by first occurrence (ballot + popcount).
// tests/lazy_model.py (lazy_via_buckets) is the executable model of this engine; it
// matches the oracle's sequential replay on random tie-heavy epsilon inputs.
//
// The per-wave dense arrays are clean between strings (rec id word ~0, leaves 0): each
// string resets what it touched, whatever its status.  Strings this engine does not take
// (label-0 inputs, an overflowing future list) end UNSUPPORTED / OVERFLOW and go to the
// general rounds engine.
#pragma once

#include "device_common.hpp"
#include "eager_layered.hpp"  // write_status
#include "eager_wave.hpp"     // wave_lds_sync
#include "lazy_wave.hpp"      // wave_fence, lanemask_lt

extern "C" __device__ double __ockl_wfred_min_f64(double);
extern "C" __device__ unsigned long long __ockl_wfred_or_u64(unsigned long long);
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

namespace fstamd {

struct LdWs {
  uint4* rec;                 // [grid * dn] {dist lo, dist hi, id | kLdSettled, back source}
  uint32_t* barc;             // [grid * dn] rhs arc index of the back-pointer
  uint32_t* ids;              // [grid * dn] id -> dense index
  unsigned long long* leaf;   // [grid * nleaf] open-at-dcur bitmap over ids
  uint4* fut;                 // [grid * fcap] {dist lo, dist hi, dense index, 0}
  unsigned long long dn;      // dense tuples per wave = NS * (lcap + 1) * 2
  uint32_t nleaf, nsum, fcap, lcap;
  unsigned long long wd_ticks;
  // the watchdog grows with the string's lattice: a pop takes ~2.5 us (4 us with every
  // wave resident), and config 3 at T = 65,536 pops up to 33 M tuples per string
  unsigned long long wd_tuple_ticks;
  unsigned long long* prof;   // [grid * 8] (FSTAMD_BFS_PROF): pops, advances, scanned, items
  const uint32_t* items;      // this launch's strings (a length bucket), or nullptr = all
  uint32_t num_items;         // entries of items (ignored when items is nullptr)
};

constexpr uint32_t kLdUntouched = 0xFFFFFFFFu;  // rec id word of an untouched tuple
constexpr uint32_t kLdSettled = 0x80000000u;
constexpr uint32_t kLdNoPrev = 0xFFFFFFFFu;     // no back-pointer (the start; new tuples)
constexpr uint64_t kLdDenseMax = 0x7FFFFF00ull;  // ids and dense indices fit 31 bits

// The id -> dense index map of the newest kLdRing ids also lives in LDS: pops follow the
// creation frontier closely (near-id order), so most pops find their tuple there.
constexpr uint32_t kLdRing = 512;

struct LdLds {
  uint32_t ring[kLdRing];  // ids[id] for id >= nn - kLdRing
  uint32_t x[64];    // candidates in relax order: target dense index
  uint32_t a[64];    // rhs arc index
  uint32_t il[64];
  uint32_t ol[64];
  double w[64];      // arc weight as relaxed (W.times(lhs arc, rhs arc) for phase 1)
  double nd[64];     // dist[curr] (x) w
};

__device__ __forceinline__ double ld_dist(uint4 r) {
  return __hiloint2double((int)r.y, (int)r.x);
}
__device__ __forceinline__ uint4 ld_rec(double d, uint32_t id, uint32_t prev) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return make_uint4((uint32_t)b, (uint32_t)(b >> 32), id, prev);
}

// Wave reductions over DPP (the ockl ones) and uniform-lane reads (v_readlane): no
// ds_bpermute round trips on the pop's serial path.
__device__ __forceinline__ double wave_min_f64(double v) { return __ockl_wfred_min_f64(v); }
__device__ __forceinline__ unsigned long long wave_or_u64(unsigned long long v) {
  return __ockl_wfred_or_u64(v);
}
__device__ __forceinline__ uint32_t wave_min_u32d(uint32_t v) { return __ockl_wfred_min_u32(v); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) {  // l uniform
  return __builtin_amdgcn_readlane(v, l);
}
// (readlane returns int: both halves go through uint32_t, or a low half with bit 31 set
// would sign-extend over the high half)
__device__ __forceinline__ unsigned long long lane_read64(unsigned long long v, uint32_t l) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
  return ((unsigned long long)hi << 32) | lo;
}
// Leaf words are updated with L2 atomics (several lanes may set bits of one word in one
// instruction), so they are read with agent-scope loads, which skip the vector L1.
__device__ __forceinline__ unsigned long long ld_leaf(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait until every memory operation this wave issued is complete (gfx9 counts stores in
// vmcnt), so later loads of any lane see the wave's earlier stores and atomics.
__device__ __forceinline__ void ld_drain() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
  return ((unsigned long long)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
__device__ __forceinline__ double uni_f64(double v) {
  return __longlong_as_double((long long)uni64((unsigned long long)__double_as_longlong(v)));
}

// Per-wave workspace pointers (slices of LdWs) and LDS, passed to the per-string body.
struct LdWave {
  uint4* R;
  uint32_t* barc;
  uint32_t* ids;
  unsigned long long* leaf;
  uint4* fut;
  unsigned long long* sum;
  const uint32_t* lab;
  LdLds* S;
  unsigned long long* prof;
  unsigned long long t0;
};

// One string (index `item` into the batch), start to finish.
__device__ __forceinline__ void lazy_dense_string(const RhsView& rhs, const ChainInput& in,
                                               const LdWs& ws, const BatchOutDev& out,
                                               const LdWave& V, uint32_t item, uint32_t L) {
  const uint32_t lane = threadIdx.x;
  const uint32_t si = item;
  uint4* R = V.R;
  uint32_t* Rw = (uint32_t*)R;
  uint32_t* barc = V.barc;
  uint32_t* ids = V.ids;
  unsigned long long* leaf = V.leaf;
  uint4* fut = V.fut;
  unsigned long long* sum = V.sum;
  const uint32_t* lab = V.lab;
  LdLds& S = *V.S;
  unsigned long long* prof = V.prof;
  const unsigned long long t0 = V.t0;
  const uint32_t NS = rhs.num_states;
  const uint32_t LC = L + 1;  // the dense index's position stride (state-major)
#ifdef FSTAMD_LD_KMAJOR  // A/B: position-major (k * NS + s2) * 2 + f
  auto dix = [&](uint32_t k_, uint32_t s_) { return k_ * NS + s_; };
#else
  auto dix = [&](uint32_t k_, uint32_t s_) { return s_ * LC + k_; };
#endif
  if (prof && lane == 0) prof[3] += 1;
  const uint32_t nsum_s = (uint32_t)(((uint64_t)LC * 2 * NS + 4095) / 4096);
  const unsigned long long wd = ws.wd_ticks + (uint64_t)LC * 2 * NS * ws.wd_tuple_ticks;

  // ---- init tuple (fst1.start, fst2.start, 0), id 0, dist One (:146-153) ----
  const uint32_t x0 = 2 * dix(0, rhs.start);
  if (lane == 0) {
    R[x0] = ld_rec(w_one(), 0u, kLdNoPrev);
    ids[0] = x0;
    S.ring[0] = x0;
    leaf[0] = 1ull;
    sum[0] = 1ull;
  }
  wave_lds_sync();
  uint32_t nn = 1, fn = 0, pops = 0, advances = 0, scur = 0;
  uint32_t cur_leaf = 0;
  unsigned long long cur_bits = 1ull;
  bool cache = true;  // no open id below leaf cur_leaf; cur_bits = its word
  double dcur = w_one();
  uint32_t best_id = kNoState;
  double best_fw = w_zero(), best_total = w_zero();
  int32_t fail = kPathOk;
  uint32_t site = 0;  // INTERNAL diagnostics: where it stopped (path_off), pops (path_len)
  uint64_t relax = 0, scanned = 0;

  // bucket insert of lane-held ids (`ins` lanes): leaf word (HBM), summary bit (LDS),
  // the cached leaf in registers; an id below the cached leaf invalidates the cache
  auto bucket_insert = [&](bool ins, uint32_t id) {
    const uint32_t li = id >> 6;
    const unsigned long long bit = 1ull << (id & 63);
    if (ins) {
      atomicOr(&leaf[li], bit);
      atomicOr(&sum[li >> 6], 1ull << (li & 63));
    }
    // ids at or above the cached leaf keep it the lowest non-empty one (scur <= its
    // summary word already); only an id below it forces a rescan (rare: a joiner)
    if (__ballot(ins && li == cur_leaf)) cur_bits = uni64(cur_bits | wave_or_u64(ins && li == cur_leaf ? bit : 0ull));
    if (__ballot(ins && li < cur_leaf)) {
      cache = false;
      scur = min(scur, uni(wave_min_u32d(ins ? (li >> 6) : ~0u)));
    }
  };

  for (;;) {
    // ---- the lowest open id at dcur ----
    bool have = uni(cache && cur_bits != 0ull ? 1u : 0u) != 0u;
    while (!have) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > wd) {
        fail = kPathInternal;
        site = 1;
        break;
      }
      uint32_t found = kNoState;
      for (uint32_t s0 = scur; s0 < nsum_s; s0 += 64) {
        const uint32_t i = s0 + lane;
        const unsigned long long v = i < nsum_s ? sum[i] : 0ull;
        const unsigned long long nz = __ballot(v != 0ull);
        if (nz) {
          const uint32_t l = (uint32_t)__ffsll((long long)nz) - 1;
          const unsigned long long vv = lane_read64(v, l);
          scur = s0 + l;
          found = (s0 + l) * 64 + (uint32_t)__ffsll((long long)vv) - 1;
          break;
        }
      }
      found = uni(found);
      if (found == kNoState) break;
      const unsigned long long word = uni64(ld_leaf(&leaf[found]));
      if (word == 0ull) {  // summary bit left by a leaf that emptied: drop it
        if (lane == 0) atomicAnd(&sum[found >> 6], ~(1ull << (found & 63)));
        wave_lds_sync();
        continue;
      }
      cur_leaf = found;
      cur_bits = word;
      cache = true;
      have = true;
    }
    if (fail != kPathOk) break;
    if (!have) {
      // ---- advance: smallest live distance in the future list (:159-163) ----
      ++advances;
      FT(item, si, fn, 4);
      scanned += fn;
      double dmin = w_zero();
      bool any = false;
      uint32_t wpos = 0;
      for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
        const uint32_t e = e0 + lane;
        const bool v = e < fn;
        const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
        const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
        const double ed = __hiloint2double((int)en.y, (int)en.x);
        const bool live = v && rv.z != kLdUntouched && !(rv.z & kLdSettled) && ld_dist(rv) == ed;
        if (live) {
          any = true;
          dmin = ed < dmin ? ed : dmin;
        }
        const unsigned long long lm = __ballot(live);
        if (live) fut[wpos + (uint32_t)__popcll(lm & lanemask_lt())] = en;
        wpos += (uint32_t)__popcll(lm);
      }
      wave_fence();
      fn = wpos;
      if (!__ballot(any)) break;  // the queue is empty: done
      dcur = uni_f64(wave_min_f64(dmin));
      wpos = 0;
      cache = false;
      for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
        const uint32_t e = e0 + lane;
        const bool v = e < fn;
        const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
        const double ed = __hiloint2double((int)en.y, (int)en.x);
        const bool hit = v && ed == dcur;
        const uint32_t id = hit ? (Rw[4 * (size_t)en.z + 2] & ~kLdSettled) : 0u;
        const bool keep = v && !hit;
        const unsigned long long km = __ballot(keep);
        if (keep) fut[wpos + (uint32_t)__popcll(km & lanemask_lt())] = en;
        wpos += (uint32_t)__popcll(km);
        bucket_insert(hit, id);
      }
      fn = wpos;
      wave_fence();
      wave_lds_sync();
      continue;
    }

    // ---- pop (:159-163: an open id is never stale nor settled) ----
    // (No wait for the previous pop's stores: a wave's vector memory operations to one
    // address are performed in order, so its later loads see them.)
    const uint32_t pid = uni(cur_leaf * 64 + (uint32_t)__ffsll((long long)cur_bits) - 1);
    cur_bits = uni64(cur_bits & (cur_bits - 1));
    const uint32_t x = uni(pid + kLdRing >= nn ? S.ring[pid & (kLdRing - 1)] : ids[pid]);
    if (lane == 0) {
      atomicAnd(&leaf[cur_leaf], ~(1ull << (pid & 63)));
      if (cur_bits == 0ull) atomicAnd(&sum[cur_leaf >> 6], ~(1ull << (cur_leaf & 63)));
      Rw[4 * (size_t)x + 2] = pid | kLdSettled;
    }
    ++pops;
    FT(item, si, pops, 3);
    if ((pops & 255u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > wd) {
      fail = kPathInternal;
      site = 2;
      break;
    }
#ifdef FSTAMD_LD_KMAJOR
    const uint32_t k = (x >> 1) / NS;
    const uint32_t s = (x >> 1) - k * NS;
#else
    const uint32_t s = (x >> 1) / LC;
    const uint32_t k = (x >> 1) - s * LC;
#endif
    if (k > L || s >= NS || pid >= nn) {  // invariant guard: never walk on garbage
      fail = kPathInternal;
      site = 3;
      break;
    }

    // ---- best final (:165-179): lhs final only at k == L (string.zig:24-50) ----
    if (k == L) {
      const double fw2 = rhs.final_w[s];
      if (!w_is_zero(fw2)) {
        const double fw = w_times(w_one(), fw2);
        const double total = w_times(dcur, fw);
        if (best_id == kNoState || total < best_total || (total == best_total && pid < best_id)) {
          best_id = pid;
          best_fw = fw;
          best_total = total;
        }
      }
    }

    // ---- candidates: phase 1 (labels[k] arcs) then phase 3 (epsilon arcs) ----
    const bool has1 = k < L;
    const uint32_t label = has1 ? lab[k] : 0u;
    const uint2 sp = rhs.span[s];
    const uint32_t aoff = sp.x, na = sp.y;
    uint32_t C = 0, lo1 = 0, n1 = 0, lo3 = 0;
    const bool small = na <= 64;
    if (small) {
      const bool v = lane < na;
      const uint32_t il = v ? rhs.il[aoff + lane] : 0xFFFFFFFFu;
      const ArcRec r = v ? rhs.rec[aoff + lane] : ArcRec{0u, 0u, 0.0};
      const bool p1 = v && has1 && il == label;
      const bool p3 = v && il == kEpsilon;
      const unsigned long long m1 = __ballot(p1), m3 = __ballot(p3);
      n1 = (uint32_t)__popcll(m1);
      C = n1 + (uint32_t)__popcll(m3);
      if (p1 || p3) {
        const uint32_t rank = p1 ? (uint32_t)__popcll(m1 & lanemask_lt())
                                 : n1 + (uint32_t)__popcll(m3 & lanemask_lt());
        S.x[rank] = p1 ? 2 * dix(k + 1, r.next) : 2 * dix(k, r.next) + 1;
        S.a[rank] = aoff + lane;
        S.il[rank] = il;
        S.ol[rank] = r.olabel;
        S.w[rank] = p1 ? w_times(w_one(), r.weight) : r.weight;
      }
      wave_lds_sync();
    } else {
      uint32_t hi;  // many arcs: counted by the whole wave (no dependent search chain)
      if (has1) {
        wave_span_by_ilabel(rhs, aoff, na, label, lo1, hi);
        n1 = hi - lo1;
      }
      wave_span_by_ilabel(rhs, aoff, na, kEpsilon, lo3, hi);
      C = n1 + (hi - lo3);
    }
    relax += C;

    for (uint32_t cb = 0; cb < C; cb += 64) {
      const uint32_t cnt = min(64u, C - cb);
      if (!small) {  // this chunk's candidates into LDS, in relax order
        const uint32_t c = cb + lane;
        if (lane < cnt) {
          const bool p1 = c < n1;
          const uint32_t a = p1 ? lo1 + c : lo3 + (c - n1);
          const ArcRec r = rhs.rec[a];
          S.x[lane] = p1 ? 2 * dix(k + 1, r.next) : 2 * dix(k, r.next) + 1;
          S.a[lane] = a;
          S.il[lane] = p1 ? label : kEpsilon;
          S.ol[lane] = r.olabel;
          S.w[lane] = p1 ? w_times(w_one(), r.weight) : r.weight;
        }
        wave_lds_sync();
      }
      // room for this chunk's future entries: compact the list first if needed
      if (fn + 64 > ws.fcap) {
        uint32_t wpos = 0;
        for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
          const uint32_t e = e0 + lane;
          const bool v = e < fn;
          const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
          const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
          const double ed = __hiloint2double((int)en.y, (int)en.x);
          const bool live =
              v && rv.z != kLdUntouched && !(rv.z & kLdSettled) && ld_dist(rv) == ed;
          const unsigned long long lm = __ballot(live);
          if (live) fut[wpos + (uint32_t)__popcll(lm & lanemask_lt())] = en;
          wpos += (uint32_t)__popcll(lm);
        }
        wave_fence();
        scanned += fn;
        fn = wpos;
        if (fn + 64 > ws.fcap) {
          fail = kPathOverflow;
          break;
        }
      }
      const bool act = lane < cnt;
      const uint32_t tx = act ? S.x[lane] : 0u;
      const double nd = act ? w_times(dcur, S.w[lane]) : 0.0;
      S.nd[lane] = nd;
      const uint4 rv = act ? R[tx] : make_uint4(0, 0, kLdUntouched, 0);
      // group candidates by target: the group's first lane folds it in order
      unsigned long long gmask = 0;
      {
        unsigned long long pend = __ballot(act);
        while (pend) {
          const uint32_t l = (uint32_t)__ffsll((long long)pend) - 1;
          const uint32_t xl = lane_read(tx, l);
          const unsigned long long m = __ballot(act && tx == xl);
          if (lane == l) gmask = m;
          pend &= ~m;
        }
      }
      wave_lds_sync();
      const bool leader = gmask != 0ull;
      const bool untouched = rv.z == kLdUntouched;
      const double od = untouched ? w_zero() : ld_dist(rv);
      double cd = od;
      uint32_t bprev = untouched ? kLdNoPrev : rv.w;
      uint32_t bil = 0, bol = 0, ba = 0;
      bool took = false;
      if (leader) {
        if (!untouched && bprev == pid) {  // back set earlier in this pop: its labels
          const uint32_t a0 = barc[tx];
          bil = rhs.il[a0];
          bol = rhs.rec[a0].olabel;
        }
        unsigned long long m = gmask;
        while (m) {  // relax (:99-141) in candidate order
          const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
          m &= m - 1;
          const double cnd = S.nd[i];
          const uint32_t cil = S.il[i], col = S.ol[i];
          bool take = w_is_zero(cd) || cnd < cd;
          if (!take && cnd == cd)
            take = pid < bprev || (pid == bprev && (cil < bil || (cil == bil && col < bol)));
          if (take) {
            cd = cnd;
            bprev = pid;
            bil = cil;
            bol = col;
            ba = S.a[i];
            took = true;
          }
        }
      }
      // getOrCreate: new tuples numbered by first occurrence (leaders in lane order)
      const bool fresh = leader && untouched;
      const unsigned long long fm = __ballot(fresh);
      const uint32_t id = fresh ? nn + (uint32_t)__popcll(fm & lanemask_lt()) : (rv.z & ~kLdSettled);
      nn += (uint32_t)__popcll(fm);
      const bool settled = !untouched && (rv.z & kLdSettled);
      if (took) {
        R[tx] = ld_rec(cd, untouched ? id : rv.z, pid);
        barc[tx] = ba;
        if (fresh) {
          ids[id] = tx;
          S.ring[id & (kLdRing - 1)] = tx;
        }
      }
      // push (:136-140): open at dcur -> bitmap, above -> future list.  An equal-dist
      // take (a tie) is already queued at that distance.
      const bool q = took && !settled && (untouched || cd < od);
      const bool tob = q && cd == dcur;
      const bool tof = q && !tob;
      const unsigned long long fmk = __ballot(tof);
      if (tof) fut[fn + (uint32_t)__popcll(fmk & lanemask_lt())] = ld_rec(cd, tx, 0u);
      fn += (uint32_t)__popcll(fmk);
      bucket_insert(tob, id);
      wave_fence();
      wave_lds_sync();
    }
    if (fail != kPathOk) break;
  }

  // ---- result (:368-400) ----
  FT(item, si, nn, 5);
  ld_drain();
  uint32_t P = 0;
  unsigned long long o = 0;
  double fin = w_zero();
  int32_t st = fail;
  if (lane == 0) {
    if (st == kPathOk) {
      if (best_id == kNoState) {
        st = kPathEmpty;
      } else {
        uint32_t cur = best_id;
        while (cur != 0) {  // init_id == 0
          const uint32_t prev = Rw[4 * (size_t)ids[cur] + 3];
          if (prev == kLdNoPrev) {
            st = kPathEmpty;
            break;
          }
          if (++P > nn) {
            st = kPathCycle;
            break;
          }
          cur = prev;
        }
        if (st == kPathOk) {
          o = reserve_path(out, si, P);
          if (o + P > out.arc_cap) {
            st = kPathOutputFull;
          } else {
            uint32_t kk = P;
            cur = best_id;
            while (cur != 0 && kk > 0) {
              const uint32_t xx = ids[cur];
              const uint32_t a = barc[xx];
              const uint32_t il = rhs.il[a];
              const ArcRec r = rhs.rec[a];
              --kk;
              out.out_il[o + kk] = il;
              out.out_ol[o + kk] = r.olabel;
              out.out_w[o + kk] = il == kEpsilon ? r.weight : w_times(w_one(), r.weight);
              cur = Rw[4 * (size_t)xx + 3];
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
    out.path_len[si] = st == kPathInternal ? pops : P;
    out.path_off[si] = st == kPathInternal ? site : o;
    out.final_w[si] = fin;
    if (out.work) {
      out.work[2 * si] = nn;
      out.work[2 * si + 1] = (uint32_t)relax;
    }
    if (prof) {
      prof[0] += pops;
      prof[1] += advances;
      prof[2] += scanned;
    }
  }
  // ---- leave the dense arrays clean ----
  FT(item, si, nn, 6);
  wave_fence();
  for (uint32_t i = lane; i < nn; i += 64) Rw[4 * (size_t)ids[i] + 2] = kLdUntouched;
  for (uint32_t i = lane; i < (nn + 63) / 64; i += 64) leaf[i] = 0ull;
  for (uint32_t i = lane; i < nsum_s; i += 64) sum[i] = 0ull;
  wave_fence();
  wave_lds_sync();
  FT(item, si, nn, 7);
}

__global__ void __launch_bounds__(64)
lazy_dense_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                  LdWs ws, BatchOutDev out) {
  extern __shared__ unsigned long long ld_dyn[];
  __shared__ LdLds S;
  unsigned long long* sum = ld_dyn;                    // [nsum] one bit per leaf word
  uint32_t* lab = (uint32_t*)(ld_dyn + ws.nsum);       // [lcap] the string's labels
  const uint32_t lane = threadIdx.x;
  const size_t w = blockIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  LdWave V;
  V.R = ws.rec + w * ws.dn;
  V.barc = ws.barc + w * ws.dn;
  V.ids = ws.ids + w * ws.dn;
  V.leaf = ws.leaf + w * (size_t)ws.nleaf;
  V.fut = ws.fut + w * (size_t)ws.fcap;
  V.sum = sum;
  V.lab = lab;
  V.S = &S;
  V.prof = ws.prof ? ws.prof + w * 8 : nullptr;
  V.t0 = t0;

  for (uint32_t i = lane; i < ws.nsum; i += 64) sum[i] = 0ull;
  wave_lds_sync();

  const uint32_t num_items = ws.items ? ws.num_items : in.num_strings;
  uint32_t passes = 0;
  for (;;) {
    // The structurizer may turn this loop into nested divergent loops in which lane 0
    // leaves to fetch work while the others re-run the old item (it did, with a lane-0
    // fetch + shfl: a wave replayed item 0 forever).  Hence the first-active-lane fetch
    // below (tier-A post-mortem).
    // hard stop: every pass of this loop consumes a fresh item, so a wave whose control
    // flow went wrong (re-running an item) ends after num_strings passes
    if (++passes > num_items + 1) return;
    // work item: fetched by the FIRST ACTIVE lane and broadcast with readlane, so every
    // subset of lanes the compiler's loop structure may run fetches its own item
    uint32_t item = 0;
    const uint32_t first = (uint32_t)__ffsll((long long)__ballot(1)) - 1;
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == first)
      item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readlane(item, first);
    if (item >= num_items) break;
    const uint32_t si = ws.items ? uni(ws.items[item]) : item;
    const uint64_t off = in.offsets[si];
    const uint32_t L = uni((uint32_t)(in.offsets[si + 1] - off));
    FT(item, si, L, 1);
    int32_t pre = kPathOk;
    if (rhs.start == kNoState || n_best != 1)  // compose-shortest-path.zig:30-33
      pre = (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN;
    else if (L > ws.lcap)
      pre = kPathUnsupported;
    V.t0 = __builtin_amdgcn_s_memrealtime();  // the string's watchdog starts now
    if (pre == kPathOk) {
      bool zero_label = false;
      for (uint32_t i = lane; i < L; i += 64) {
        const uint32_t x = in.labels[off + i];
        lab[i] = x;
        zero_label |= x == kEpsilon;
      }
      // label-0 input: lhs epsilon phases (general engine)
      if (__ballot(zero_label) != 0ull) pre = kPathUnsupported;
      wave_lds_sync();
    }
    pre = (int32_t)uni((uint32_t)pre);
    if (pre != kPathOk) {
      if (lane == 0) write_status(out, si, pre, 0, 0);
      FT(item, si, pre, 2);
    } else {
      lazy_dense_string(rhs, in, ws, out, V, si, L);
    }
  }
  FT(0xFFFFFFFFu, 0, 0, 8);
}

}  // namespace fstamd
