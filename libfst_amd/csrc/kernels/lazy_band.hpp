// lazy_band.hpp -- composeShortestPath (FST_SEM_LAZY) as an exact pop-by-pop replay over a
// sliding window of rhs states, one wavefront per string (gfx950 / CDNA4).
//
// Same replay as lazy_dense.hpp (the reference's pops of src/ops/compose-shortest-path.zig:
// 26-401 one by one, heap split by distance, candidates read lane-parallel and folded in
// relax order), for the same domain, with a per-wave footprint ~14x smaller so that many
// more strings run at once.  The dense replay is latency-bound: its throughput scales
// with the waves in flight (T = 16,384, L = 87: 20 / 40 / 78 / 142 strings/s at 128 / 256 /
// 512 / 1,024 waves, profiles/r03/dense_waves.log), and at config 3's full size its 28 B
// per dense tuple (0.93 GB per wave at L = 251) cap them near 250.
//
// What lives where (per wave):
//   * the tuple records {dist, id | settled, back source id} (16 B) only for rhs states in
//     a window [slo, slo + Ws): index ((s mod Ws) (L + 1) + k) 2 + f.  With every rhs arc
//     going forward (t >= s, RhsView::jump_back == 0), a pop at state s only touches states
//     >= s, so a tuple whose state lies below every open tuple's can never be touched or
//     relaxed again (its record is final): the window slides up to the lowest state with an
//     open tuple (found by walking the open set, rare) when a target falls beyond its end.  On
//     epsilon-dense lattices the open tuples span L + 2 states (a diagonal across the input
//     positions, tests/lazy_model.py), so Ws = 2 (L + 1) rounded up to a power of two;
//   * per tuple (every state, not just the window), written on every take: the back
//     pointer packed in 1 B (2 or 4 B when the rhs needs it) -- the source tuple's filter, its
//     state distance (t - s <= jump_fwd) and the arc's index within the source state's
//     arcs; the source position follows from the target's filter (0: a labelled arc,
//     k - 1; 1: an epsilon arc, k).  All the backtrace (:368-400) needs, walked by tuple;
//   * the open-at-dcur set as a bitmap over the newest R ids (LDS): the open tuples' ids lie
//     within ~12 L of the newest (2,997 at L = 251, T = 1,024); an id falling R behind
//     while open, or a window overflow, hands the string to the dense replay (OVERFLOW);
//   * id -> window index for the newest R ids (HBM ring, the newest 512 also in LDS).
#pragma once

#include "lazy_dense.hpp"

namespace fstamd {

// FSTAMD_BAND_TIMING (debug builds): cycles per phase into prof[300 + i]
#ifdef FSTAMD_BAND_TIMING
#define LB_T(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    tacc[i] += t_ - tlast; tlast = t_; } while (0)
#else
#define LB_T(i) do { } while (0)
#endif
#if defined(FSTAMD_BAND_DEBUG) || defined(FSTAMD_BAND_TIMING)
constexpr uint32_t kLbProf = 512;  // per-wave profile words (+ the phase timing)
#else
constexpr uint32_t kLbProf = 20;
#endif

struct LbWs {
  uint4* win;                 // [grid * wn] window records (lazy_dense.hpp ld_rec layout)
  void* bk;                   // [grid * tn] per tuple back pointer (bkb bytes each)
  uint32_t* idr;              // [grid * ring] id -> window index (id mod ring)
  uint4* fut;                 // [grid * fcap] {dist lo, dist hi, window index, id}
  unsigned long long wn;      // window records per wave = ws * (lcap + 1) * 2
  unsigned long long tn;      // tuples per wave = num_states * (lcap + 1) * 2
  uint32_t bkb;               // bytes per back pointer: 1, 2 or 4
  uint32_t dbits;             // bits of the state distance in a back pointer
  uint32_t ws;                // window states (power of two)
  uint32_t ring;              // ids kept (power of two, multiple of 4096)
  uint32_t fcap, lcap;
  uint32_t scap;              // back pointers for states [start, start + scap) (a target
                              // beyond: OVERFLOW, the next launch has the whole rhs)
  uint32_t early;             // 1: exact early exit (weights and finals >= +0, finite)
  unsigned long long wd_ticks, wd_tuple_ticks;
  unsigned long long* prof;   // [grid * kLbProf] (FSTAMD_BFS_PROF): pops, advances, slides,
                              // items, overflows by site (4..7), the wave's last overflow
                              // (8..15), early exits (16), overflows past scap (17)
  const uint32_t* items;      // this launch's strings, or nullptr = all
  uint32_t num_items;
  // the rhs's arcs at a fixed stride per state (DeviceFst::band_il / band_rec: 2^ssh slots,
  // padding slots with ilabel 0xFFFFFFFF), or nullptr: a pop reads its state's arcs without
  // first reading the state's span
  const uint32_t* sil;
  const ArcRec* srec;
  uint32_t ssh;
};

// The id -> window index map of the newest kLbRing ids also lives in LDS (the rest: the
// per-wave HBM ring).  Small, so that 32 waves fit a CU's 160 KB of LDS (~5 KB each).
#ifndef FSTAMD_BAND_LDS_RING
#define FSTAMD_BAND_LDS_RING 256
#endif
constexpr uint32_t kLbRing = FSTAMD_BAND_LDS_RING;
// the per-wave id ring (HBM, power of two) and future list: compile-time sizes, so the
// loop holds no registers for them
constexpr uint32_t kLbIdRing = 4096;
constexpr uint32_t kLbFcap = 65536;
// FSTAMD_BAND_STATS (debug builds, implied by FSTAMD_BAND_DEBUG / _TIMING): advances, slides
// and the failing state/id in the FSTAMD_BFS_PROF words (they cost the loop registers)
#if defined(FSTAMD_BAND_DEBUG) || defined(FSTAMD_BAND_TIMING)
#define FSTAMD_BAND_STATS 1
#endif
#ifdef FSTAMD_BAND_STATS
#define LB_STAT(x) x
#else
#define LB_STAT(x) do { } while (0)
#endif
// 7 waves per SIMD (72 VGPRs): 42.1 K vs 39.5 K strings/s at the compiler's 73 VGPRs and 6
// waves (config 3 sample, profiles/r06/band/ab_v5.txt)
#ifndef FSTAMD_BAND_ATTR
#define FSTAMD_BAND_ATTR __attribute__((amdgpu_waves_per_eu(7)))
#endif

struct LbLds {
  uint32_t ring[kLbRing];  // id -> window index for id >= nn - kLbRing
  uint32_t x[64];    // candidates in relax order: target window index
  uint32_t a[64];    // rhs arc index
  uint32_t il[64];
  uint32_t ol[64];
  double w[64];      // arc weight as relaxed (W.times(lhs arc, rhs arc) for phase 1)
  uint32_t fut_lb;   // <= every live future entry's id (LDS min per push; read when needed)
  union {
    double nd[64];                // dist[curr] (x) w
    unsigned long long key[64];   // the slot path: per slot min (distance bits | lane)
  };
};

// FP: the host guarantees the strided arc table and jump_fwd < 32 (the slot path's
// preconditions), so neither is tested per pop
template <uint32_t BKB, bool FP>
__device__ __forceinline__ void lazy_band_string(const RhsView& rhs, const ChainInput& in,
                                                 const LbWs& ws, const BatchOutDev& out,
                                                 uint4* R, void* bkv, uint32_t* idr, uint4* fut,
                                                 unsigned long long* bm,
                                                 const uint32_t* lab, LbLds& S,
                                                 unsigned long long* prof, uint32_t si,
                                                 uint32_t L) {
  const uint32_t lane = threadIdx.x;
  uint32_t* Rw = (uint32_t*)R;
  const uint32_t NS = rhs.num_states;
  const uint32_t LC = L + 1;
  const uint32_t WS = ws.ws, wmask = WS - 1;
  constexpr uint32_t RING = kLbIdRing, rmask = RING - 1;
  constexpr uint32_t nbw = RING / 64;  // bitmap words
  // open ids stay within the newest LS = RING - 64 (an older one hands the string on):
  // then a scan over [nn - LS, nn) never meets one physical bitmap word twice, and the
  // ring slot of an open id is never reused
  constexpr uint32_t LS = RING - 64;
  const uint32_t S0 = rhs.start;  // every reachable state is >= S0 (arcs go forward)
  const uint32_t SCAP = ws.scap;
  const bool jf32 = FP || rhs.jump_fwd < 32;  // a pop's targets fit 2 x 32 slots (the slot path)
  auto wix = [&](uint32_t k_, uint32_t s_) { return (s_ & wmask) * LC + k_; };  // x 2 + f
  // v / LC for window indices v < 2^26 (the host plan checks WS * LC < 2^26): one 64-bit
  // multiply instead of a ~35-instruction integer division, exact since 2^38 >= v * LC
  const uint64_t mlc = ((1ull << 38) + LC - 1) / LC;
  auto div_lc = [&](uint32_t v_) -> uint32_t { return (uint32_t)(((uint64_t)v_ * mlc) >> 38); };
  auto gix = [&](uint32_t k_, uint32_t s_) { return (s_ - S0) * LC + k_; };     // x 2 + f
  // back pointers: f_src | ds << 1 | local arc << (1 + dbits)
  uint8_t* bk8 = (uint8_t*)bkv;
  uint16_t* bk16 = (uint16_t*)bkv;
  uint32_t* bk32 = (uint32_t*)bkv;
  constexpr uint32_t bkb = BKB;  // bytes per back pointer: 1, 2 or 4
  const uint32_t dbits = ws.dbits, dmask = (1u << dbits) - 1;
  auto bk_get = [&](uint32_t g_) -> uint32_t {
    if constexpr (bkb == 1) return (uint32_t)bk8[g_];
    else if constexpr (bkb == 2) return (uint32_t)bk16[g_];
    else return bk32[g_];
  };
  auto bk_put = [&](uint32_t g_, uint32_t c_) {
    if constexpr (bkb == 1) bk8[g_] = (uint8_t)c_;
    else if constexpr (bkb == 2) bk16[g_] = (uint16_t)c_;
    else bk32[g_] = c_;
  };
  if (prof && lane == 0) prof[3] += 1;
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + ws.wd_ticks +
                                     (uint64_t)LC * 2 * NS * ws.wd_tuple_ticks;

  uint32_t slo = rhs.start;  // window: states [slo, slo + WS)
  // a pop at s >= near_lim may reach past the window or the back pointers' states
  // (s + jump_fwd >= min(slo + WS, S0 + SCAP)); recomputed when the window slides
  auto near_limit = [&]() -> uint32_t {
    const uint64_t e = min((uint64_t)slo + WS, (uint64_t)S0 + SCAP);
    return e > rhs.jump_fwd ? (uint32_t)min<uint64_t>(e - rhs.jump_fwd, 0xFFFFFFFFull) : 0u;
  };
  uint32_t near_lim = near_limit();
  const uint32_t x0 = 2 * wix(0, rhs.start);
  if (lane == 0) {
    R[x0] = ld_rec(w_one(), 0u, kLdNoPrev);
    idr[0] = x0;
    S.ring[0] = x0;
    bm[0] = 1ull;
  }
  wave_lds_sync();
  uint32_t nn = 1, fn = 0, pops = 0;
#ifdef FSTAMD_BAND_STATS
  uint32_t advances = 0, slides = 0;
#endif
  uint32_t lowp = 0;                 // every open id at dcur is >= lowp
  uint32_t cur_base = 0;             // cached word: ids [cur_base, cur_base + 64)
  unsigned long long cur_bits = 1ull;
  bool cache = true;
  double dcur = w_one();
  uint32_t best_id = kNoState, best_g = 0;
  double best_fw = w_zero(), best_total = w_zero();
  int32_t fail = kPathOk;
  uint32_t site = 0;  // INTERNAL / OVERFLOW: where it stopped (FSTAMD_BFS_PROF)
#ifdef FSTAMD_BAND_STATS
  uint32_t dbg_s = 0, dbg_t = 0;
#endif
  uint32_t relax = 0;
  // exact early exit (ws.early): once the next pop is at dcur == best_total
  // and every tuple with an id <= emax is settled, where emax bounds the ids on the best
  // tuple's back chain, no later pop can change the best or a back pointer on that chain
  const bool early = ws.early != 0;
  uint32_t emax = 0;       // the largest id on the back chain when last walked (grows)
  if (lane == 0) S.fut_lb = ~0u;  // (S.fut_lb: <= every live future entry's id)
  uint32_t nn_slid = 0;    // every tuple that left the window has an id < nn_slid
  uint32_t scan_gate = 0;  // pops before the next exact scan of the future list
  bool stop = false;       // early exit taken
  // back chain step by tuple (the result's walk below): g_'s back source tuple, a_ its arc
  auto step = [&](uint32_t g_, uint32_t& a_) -> uint32_t {
    const uint32_t c = bk_get(g_);
    const uint32_t rs_ = (g_ >> 1) / LC, kk_ = (g_ >> 1) - rs_ * LC;
    const uint32_t sp_ = S0 + rs_ - ((c >> 1) & dmask);
    a_ = rhs.span[sp_].x + (c >> (1 + dbits));
    return 2 * gix(kk_ - ((g_ & 1) ? 0u : 1u), sp_) + (c & 1);
  };

  // open-at-dcur insert of lane-held ids: LDS bitmap bits (ds_or_b64, no return), the
  // cached word (one reduction when an id falls in it), lowp
  auto bucket_insert = [&](bool ins, uint32_t id) {
    if (ins) atomicOr(&bm[(id & rmask) >> 6], 1ull << (id & 63));
    // both cases relative to the cached word have id < cur_base + 64: one test for the
    // common insert above it.  (lowp is not tied to cur_base: after an advance the cached
    // word is stale and lowp = nn, so its test stays separate.)
    if (__ballot(ins && id < cur_base + 64)) {
      if (__ballot(ins && (id & ~63u) == cur_base)) {  // the cached word: read back (LDS
        wave_fence();                                   // operations of a wave run in order)
        cur_bits = uni64(bm[(cur_base & rmask) >> 6]);
      }
      if (__ballot(ins && id < cur_base)) cache = false;
    }
    if (__ballot(ins && id < lowp)) lowp = uni(wave_min_u32d(ins ? id : ~0u));
  };

#ifdef FSTAMD_BAND_TIMING
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  for (;;) {
    LB_T(5);
    // ---- the lowest open id at dcur: the cached word, else a scan of the bitmap over
    // ids [lowp, nn) ----
    bool have = uni(cache && cur_bits != 0ull ? 1u : 0u) != 0u;
    if (cache && !have) lowp = max(lowp, cur_base + 64);  // the lowest word is exhausted
    if (!have) {
      if (__builtin_amdgcn_s_memrealtime() > deadline) {
        fail = kPathInternal;
        site = 1;
        break;
      }
      uint32_t found = kNoState;
      unsigned long long fw = 0ull;
      const uint32_t lo = max(lowp, nn > LS ? nn - LS : 0u);
      for (uint32_t b0 = lo & ~63u; b0 < nn; b0 += 64 * 64) {
        const uint32_t id0 = b0 + lane * 64;
        const unsigned long long v = id0 < nn ? bm[(id0 & rmask) >> 6] : 0ull;
        const unsigned long long nz = __ballot(v != 0ull);
        if (nz) {
          const uint32_t l = (uint32_t)__ffsll((long long)nz) - 1;
          fw = lane_read64(v, l);
          found = b0 + l * 64;
          break;
        }
      }
      found = uni(found);
      if (found != kNoState) {
        cur_base = found;
        cur_bits = uni64(fw);
        lowp = found;
        cache = true;
        have = true;
      } else {
        lowp = nn;
      }
    }
    if (!have) {
      // ---- advance: smallest live distance in the future list (:159-163) ----
      LB_STAT(++advances);
      double dmin = w_zero();
      bool any = false;
      uint32_t wpos = 0;
      for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
        const uint32_t e = e0 + lane;
        const bool v = e < fn;
        const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
        const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
        const double ed = __hiloint2double((int)en.y, (int)en.x);
        // live: the window slot still holds this id, unsettled, at this distance
        const bool live = v && rv.z == en.w && ld_dist(rv) == ed;
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
      // every later pop is at dcur > best_total: its total (final >= 0) and its relaxations
      // of the chain (whose distances are <= best_total) can no longer win
      if (early && best_id != kNoState && dcur > best_total) {
        stop = true;
        break;
      }
      wpos = 0;
      cache = false;
      bool old = false;
      for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
        const uint32_t e = e0 + lane;
        const bool v = e < fn;
        const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
        const double ed = __hiloint2double((int)en.y, (int)en.x);
        const bool hit = v && ed == dcur;
        old |= hit && en.w + LS <= nn;  // fell out of the id ring
        const bool keep = v && !hit;
        const unsigned long long km = __ballot(keep);
        if (keep) fut[wpos + (uint32_t)__popcll(km & lanemask_lt())] = en;
        wpos += (uint32_t)__popcll(km);
        bucket_insert(hit, en.w);
      }
      fn = wpos;
      wave_fence();
      wave_lds_sync();
      if (__ballot(old)) {
        fail = kPathOverflow;
        site = 7;
        break;
      }
      continue;
    }

    LB_T(0);  // finding the next id (scans, advances)
    if (early && best_id != kNoState && dcur == best_total &&
        cur_base + (uint32_t)__ffsll((long long)cur_bits) - 1 > emax) {
      // the next pop (the smallest open id at dcur) is past emax; the future list's live
      // ids (above dcur) must be too -- its bound first, an exact scan (amortised) if not
      if (uni(S.fut_lb) <= emax && pops >= scan_gate) {
        uint32_t wpos = 0, mn = ~0u;
        for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
          const uint32_t e = e0 + lane;
          const bool v = e < fn;
          const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
          const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
          const double ed = __hiloint2double((int)en.y, (int)en.x);
          const bool live = v && rv.z == en.w && ld_dist(rv) == ed;
          if (live) mn = min(mn, en.w);
          const unsigned long long lm = __ballot(live);
          if (live) fut[wpos + (uint32_t)__popcll(lm & lanemask_lt())] = en;
          wpos += (uint32_t)__popcll(lm);
        }
        wave_fence();
        fn = wpos;
        mn = uni(wave_min_u32d(mn));
        wave_lds_sync();
        if (lane == 0) S.fut_lb = mn;
        wave_lds_sync();
        scan_gate = pops + max(64u, fn / 16u);
      }
      if (uni(S.fut_lb) > emax) {
        // the chain's ids now (lane 0 walks it): a tuple still in the window holds its id
        // in its record; one that left it has an id < nn_slid
        uint32_t m = best_id;
        if (lane == 0) {
          uint32_t g = best_g, a = 0, n = 0;
          while (g != 0u && n++ <= nn) {
            g = step(g, a);
            const uint32_t rs = (g >> 1) / LC, kk = (g >> 1) - rs * LC, st = S0 + rs;
            if (st >= slo && st - slo < WS)
              m = max(m, Rw[4 * (size_t)(2 * wix(kk, st) + (g & 1)) + 2] & ~kLdSettled);
            else
              m = max(m, nn_slid);
          }
        }
        m = uni(m);
        if (m <= emax) {
          stop = true;
          break;
        }
        emax = m;
      }
    }
    // ---- pop (:159-163) ----
    const uint32_t pid = uni(cur_base + (uint32_t)__ffsll((long long)cur_bits) - 1);
    cur_bits = uni64(cur_bits & (cur_bits - 1));
    const uint32_t x = uni(pid + kLbRing >= nn ? S.ring[pid & (kLbRing - 1)] : idr[pid & rmask]);
    const uint32_t sslot = div_lc(x >> 1);
    const uint32_t k = (x >> 1) - sslot * LC;
    const uint32_t s = slo + ((sslot - slo) & wmask);
#ifdef FSTAMD_BAND_DEBUG
    {
      const unsigned long long wbits = uni64(bm[(pid & rmask) >> 6]);
      const uint32_t zz = uni(Rw[4 * (size_t)x + 2]);
      if (!((wbits >> (pid & 63)) & 1ull) || zz != pid) {
        fail = kPathInternal;
        site = ((wbits >> (pid & 63)) & 1ull) ? 9 : 8;
        LB_STAT((dbg_s = zz, dbg_t = pid));
        break;
      }
    }
#endif
    // every lane stores the same values (no exec branch): the popped id's bitmap word is
    // the cached word, which now holds the rest of its open ids (44.6 -> 46.3 K strings/s
    // against lane 0's atomicAnd, profiles/r06/band/ab_v10.txt)
    bm[(cur_base & rmask) >> 6] = cur_bits;
    Rw[4 * (size_t)x + 2] = pid | kLdSettled;
    ++pops;
    if ((pops & 255u) == 0 && __builtin_amdgcn_s_memrealtime() > deadline) {
      fail = kPathInternal;
      site = 2;
      break;
    }
    if (k > L || s >= NS || pid >= nn) {  // invariant guard: never walk on garbage
      fail = kPathInternal;
      site = 3;
      LB_STAT((dbg_s = s, dbg_t = pid));
      break;
    }

    // ---- best final (:165-179): lhs final only at k == L ----
    if (k == L) {
      const double fw2 = rhs.final_w[s];
      if (!w_is_zero(fw2)) {
        const double fw = w_times(w_one(), fw2);
        const double total = w_times(dcur, fw);
        if (best_id == kNoState || total < best_total || (total == best_total && pid < best_id)) {
          best_id = pid;
          best_g = 2 * gix(k, s) + (x & 1);
          emax = max(emax, pid);
          best_fw = fw;
          best_total = total;
        }
      }
    }

    LB_T(1);  // pop bookkeeping, best final
    // ---- candidates: phase 1 (labels[k] arcs) then phase 3 (epsilon arcs) ----
    const bool has1 = k < L;
    const uint32_t label = has1 ? lab[k] : 0u;
    // with the strided table a state's arcs sit at s << ssh (aoff 0: every use of an arc
    // index below is relative to the state's first arc), else behind its span
    const bool tab = FP || ws.sil != nullptr;
    const uint2 sp = tab ? make_uint2(0u, 1u << ws.ssh) : rhs.span[s];
    const uint32_t aoff = sp.x, na = sp.y;
    uint32_t C = 0, lo1 = 0, n1 = 0, lo3 = 0, tmax = s;
    const bool small = na <= 64;
    // the targets' largest state only matters near the window's end (t - s <= jump_fwd)
    const bool near_end = s >= near_lim;
    // slot path (below): this lane's candidate, kept in registers
    bool fast = false, fc = false, fp1 = false;
    uint32_t fnext = 0;
    double fnd = 0.0;
    if (small) {
      const bool v = lane < na;
      // unconditional loads: a lane past the span reads its last arc (or the padding
      // record past the arc mirror's end when the span is empty) and is masked off
      const uint32_t ai = (tab ? s << ws.ssh : aoff) + min(lane, max(na, 1u) - 1u);
      const uint32_t il = v ? (tab ? ws.sil[ai] : rhs.il[ai]) : 0xFFFFFFFFu;
      const ArcRec r = tab ? ws.srec[ai] : rhs.rec[ai];
      const bool p1 = v && has1 && il == label;
      const bool p3 = v && il == kEpsilon;
      const unsigned long long m1 = __ballot(p1), m3 = __ballot(p3);
      n1 = (uint32_t)__popcll(m1);
      C = n1 + (uint32_t)__popcll(m3);
      if (near_end) tmax = max(tmax, __ockl_wfred_max_u32((p1 || p3) ? r.next : 0u));
      if (jf32) {
        // the slot path takes the pop when every candidate distance is finite, >= +0 and
        // has its 6 low mantissa bits clear (integer costs do): then (bits | lane) orders
        // the candidates of one target exactly as (distance, relax order)
        fnd = w_times(dcur, p1 ? w_times(w_one(), r.weight) : r.weight);
        const unsigned long long b = (unsigned long long)__double_as_longlong(fnd);
        const bool nice = (b & 0x800000000000003Full) == 0ull && b < 0x7FF0000000000000ull;
        fast = __ballot((p1 || p3) && !nice) == 0ull;
        fc = p1 || p3;
        fp1 = p1;
        fnext = r.next;
      }
      if ((p1 || p3) && !fast) {  // (a window index does not depend on slo: valid after any slide)
        const uint32_t rank = p1 ? (uint32_t)__popcll(m1 & lanemask_lt())
                                 : n1 + (uint32_t)__popcll(m3 & lanemask_lt());
        S.x[rank] = p1 ? 2 * wix(k + 1, r.next) : 2 * wix(k, r.next) + 1;
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
      if (near_end) {
        for (uint32_t c = lane; c < C; c += 64) {
          const uint32_t a = c < n1 ? lo1 + c : lo3 + (c - n1);
          tmax = max(tmax, rhs.rec[a].next);
        }
        tmax = __ockl_wfred_max_u32(tmax);
      }
    }
    tmax = uni(tmax);
    relax += C;
    if (tmax - S0 >= SCAP) {  // beyond the back pointers' states: the next launch's
      fail = kPathOverflow;
      site = 10;
      LB_STAT((dbg_s = s, dbg_t = tmax));
      break;
    }

    LB_T(2);  // candidates
    // ---- the window must hold every target: slide it up to the lowest state with an
    // open tuple (a pop at state s only ever touches states >= s) ----
    if (tmax >= slo + WS) {
      LB_STAT(++slides);
      // lowest state with an open tuple: the ids open at dcur (bitmap) and the live future
      // entries (compacted on the way); none below: the popped state s.  Slides are rare
      // (every ~Ws - L states), so the open set is walked rather than counted per pop.
      uint32_t smin = s;
      {
        auto state_of = [&](uint32_t xw) { return slo + ((div_lc(xw >> 1) - slo) & wmask); };
        const uint32_t lo = max(lowp, nn > LS ? nn - LS : 0u);
        for (uint32_t b0 = lo & ~63u; b0 < nn; b0 += 64 * 64) {
          const uint32_t id0 = b0 + lane * 64;
          unsigned long long v = id0 < nn ? bm[(id0 & rmask) >> 6] : 0ull;
          while (v) {
            const uint32_t id = id0 + (uint32_t)__ffsll((long long)v) - 1;
            v &= v - 1;
            const uint32_t xw = id + kLbRing >= nn ? S.ring[id & (kLbRing - 1)] : idr[id & rmask];
            smin = min(smin, state_of(xw));
          }
        }
        uint32_t wpos = 0;
        for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
          const uint32_t e = e0 + lane;
          const bool v = e < fn;
          const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
          const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
          const double ed = __hiloint2double((int)en.y, (int)en.x);
          const bool live = v && rv.z == en.w && ld_dist(rv) == ed;
          if (live) smin = min(smin, state_of(en.z));
          const unsigned long long lm = __ballot(live);
          if (live) fut[wpos + (uint32_t)__popcll(lm & lanemask_lt())] = en;
          wpos += (uint32_t)__popcll(lm);
        }
        wave_fence();
        fn = wpos;
        smin = uni(wave_min_u32d(smin));
      }
      if (tmax >= smin + WS) {  // the open tuples span more than the window
        fail = kPathOverflow;
        site = 4;
        LB_STAT((dbg_s = s, dbg_t = smin));
        break;
      }
      // clear the leaving states' records (every tuple there is final)
      const uint32_t nclear = (smin - slo) * LC * 2;
      for (uint32_t i = lane; i < nclear; i += 64) {
        const uint32_t st = slo + div_lc(i >> 1);
        const uint32_t r = i - (st - slo) * (LC * 2);
        Rw[4 * (size_t)(2 * ((st & wmask) * LC) + r) + 2] = kLdUntouched;
      }
      wave_fence();
      slo = smin;
      near_lim = near_limit();
      nn_slid = nn;
    }

    LB_T(3);  // slides
    for (uint32_t cb = 0; cb < C; cb += 64) {
      const uint32_t cnt_c = min(64u, C - cb);
      if (!small) {  // this chunk's candidates into LDS, in relax order
        const uint32_t c = cb + lane;
        if (lane < cnt_c) {
          const bool p1 = c < n1;
          const uint32_t a = p1 ? lo1 + c : lo3 + (c - n1);
          const ArcRec r = rhs.rec[a];
          S.x[lane] = p1 ? 2 * wix(k + 1, r.next) : 2 * wix(k, r.next) + 1;
          S.a[lane] = a;
          S.il[lane] = p1 ? label : kEpsilon;
          S.ol[lane] = r.olabel;
          S.w[lane] = p1 ? w_times(w_one(), r.weight) : r.weight;
        }
        wave_lds_sync();
      }
      // room for this chunk's future entries: compact the list first if needed
      if (fn + 64 > kLbFcap) {
        uint32_t wpos = 0;
        for (uint32_t e0 = 0; e0 < fn; e0 += 64) {
          const uint32_t e = e0 + lane;
          const bool v = e < fn;
          const uint4 en = v ? fut[e] : make_uint4(0, 0, 0, 0);
          const uint4 rv = v ? R[en.z] : make_uint4(0, 0, kLdUntouched, 0);
          const double ed = __hiloint2double((int)en.y, (int)en.x);
          const bool live = v && rv.z == en.w && ld_dist(rv) == ed;
          const unsigned long long lm = __ballot(live);
          if (live) fut[wpos + (uint32_t)__popcll(lm & lanemask_lt())] = en;
          wpos += (uint32_t)__popcll(lm);
        }
        wave_fence();
        fn = wpos;
        if (fn + 64 > kLbFcap) {
          fail = kPathOverflow;
          site = 6;
          break;
        }
      }
      // per target, one writer lane holds the folded relax (:99-141) of its candidates
      uint32_t tx = 0, tg = 0, id = 0, bkw = 0;
      uint4 rv;
      bool took = false, fresh = false;
      double cd, od;
      if (fast) {
        // slot path: a target's candidates share one slot (phase, t - s < 32); one LDS
        // min of (distance bits | lane) per slot finds the fold's winner, the first in
        // relax order among the least distances.  Its fold against the record is the
        // whole group's: an earlier candidate at a larger distance is overtaken by it,
        // a later one at the same distance has an olabel >= its own (arcs sort by
        // (ilabel, olabel)) and loses the tie, and the record cannot hold this pop's id
        // (each target is met by one phase of one pop).  A min of lanes finds the
        // slot's first candidate, which numbers a new tuple (getOrCreate order).
        const bool act = fc;
        // (a lane without a candidate reads the popped tuple's record: no branch)
        const uint32_t sl = ((fp1 ? 0u : 32u) + (fnext - s)) & 63u;
        const uint32_t kk = fp1 ? k + 1 : k;
        tx = act ? 2 * wix(kk, fnext) + (fp1 ? 0u : 1u) : x;
        tg = 2 * gix(kk, fnext) + (fp1 ? 0u : 1u);
        rv = R[tx];
        unsigned long long* K = S.key;
        uint32_t* F = S.x;  // per slot: its first candidate's lane
        const unsigned long long key =
            (unsigned long long)__double_as_longlong(fnd) | (unsigned long long)lane;
        K[lane] = ~0ull;
        F[lane] = ~0u;
        wave_fence();
        if (act) {  // (LDS atomics of many lanes on one word serialise: candidates only)
          atomicMin(&K[sl], key);
          atomicMin(&F[sl], lane);
        }
        wave_fence();
        const unsigned long long kmin = K[sl];
        const uint32_t first = F[sl];
        wave_lds_sync();
        const bool untouched = rv.z == kLdUntouched;
        od = untouched ? w_zero() : ld_dist(rv);
        const uint32_t bprev = untouched ? kLdNoPrev : rv.w;
        const bool win = act && kmin == key;
        took = win && (w_is_zero(od) || fnd < od || (fnd == od && pid < bprev));
        cd = took ? fnd : od;
        const bool ff = act && first == lane && untouched;
        const unsigned long long fm1 = __ballot(ff && fp1), fm3 = __ballot(ff && !fp1);
        const unsigned long long below = (1ull << (first & 63)) - 1;
        fresh = win && untouched;
        id = fresh ? nn + (fp1 ? (uint32_t)__popcll(fm1 & below)
                               : (uint32_t)__popcll(fm1) + (uint32_t)__popcll(fm3 & below))
                   : (rv.z & ~kLdSettled);
        nn += (uint32_t)__popcll(fm1) + (uint32_t)__popcll(fm3);
        bkw = (x & 1) | ((fnext - s) << 1) | (lane << (1 + dbits));
      } else {
        const bool act = lane < cnt_c;
        tx = act ? S.x[lane] : 0u;
        // the target's tuple index (its state from the window slot: targets lie in the window)
        const uint32_t tslot = div_lc(tx >> 1);
        const uint32_t tstate = slo + ((tslot - slo) & wmask);
        tg = 2 * gix((tx >> 1) - tslot * LC, tstate) + (tx & 1);
        const double nd = act ? w_times(dcur, S.w[lane]) : 0.0;
        S.nd[lane] = nd;
        rv = act ? R[tx] : make_uint4(0, 0, kLdUntouched, 0);
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
        od = untouched ? w_zero() : ld_dist(rv);
        cd = od;
        uint32_t bprev = untouched ? kLdNoPrev : rv.w;
        uint32_t bil = 0, bol = 0, ba = 0;
        if (leader) {
          if (!untouched && bprev == pid) {  // back set earlier in this pop: its labels
            const uint32_t a0 = (tab ? rhs.span[s].x : aoff) + (bk_get(tg) >> (1 + dbits));
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
        fresh = leader && untouched;
        const unsigned long long fm = __ballot(fresh);
        id = fresh ? nn + (uint32_t)__popcll(fm & lanemask_lt()) : (rv.z & ~kLdSettled);
        nn += (uint32_t)__popcll(fm);
        bkw = (x & 1) | ((tstate - s) << 1) | ((ba - aoff) << (1 + dbits));
      }
      const bool untouched = rv.z == kLdUntouched;
      // the live span: every id open at dcur is >= pid (pops go in id order) or was
      // re-opened by this pop (checked below); one open above dcur is checked when it joins
      // the bitmap.  So the span holds while the newest id stays below pid + LS.
      bool clash = (uint64_t)pid + LS <= nn;
      const bool settled = !untouched && (rv.z & kLdSettled);
      if (took) {
        R[tx] = ld_rec(cd, untouched ? id : rv.z, pid);
        bk_put(tg, bkw);
        if (fresh) {
          idr[id & rmask] = tx;
          S.ring[id & (kLbRing - 1)] = tx;
        }
      }
      // push (:136-140): open at dcur -> bitmap, above -> future list.  An equal-dist
      // take (a tie) is already queued at that distance.
      const bool q = took && !settled && (untouched || cd < od);
      const bool tob = q && cd == dcur;
      const bool tof = q && !tob;
      clash |= tob && !fresh && id + LS <= nn;
      const unsigned long long fmk = __ballot(tof);
      if (tof) fut[fn + (uint32_t)__popcll(fmk & lanemask_lt())] = ld_rec(cd, tx, id);
      fn += (uint32_t)__popcll(fmk);
      if (tof && early) atomicMin(&S.fut_lb, id);
      bucket_insert(tob, id);
      wave_fence();
      wave_lds_sync();
      if (__ballot(clash)) {
        fail = kPathOverflow;
        site = 5;
        LB_STAT((dbg_s = s, dbg_t = uni(wave_min_u32d(clash ? id : ~0u))));
        break;
      }
    }
    LB_T(4);  // relax
    if (fail != kPathOk) break;
  }
#ifdef FSTAMD_BAND_TIMING
  if (prof && lane == 0)
    for (int i = 0; i < 6; ++i) prof[300 + i] += tacc[i];
#endif

  // ---- result (:368-400): the back chain, walked by tuple ----
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
        // by tuple: the start tuple (0, start, 0) is id 0 (init_id, :372), index 0
        const uint32_t g0 = 0;
        uint32_t cur = best_g, arc = 0;
        while (cur != g0) {
          if (++P > nn) {
            st = kPathCycle;
            break;
          }
          cur = step(cur, arc);
        }
        if (st == kPathOk) {
          o = reserve_path(out, si, P);
          if (o + P > out.arc_cap) {
            st = kPathOutputFull;
          } else {
            uint32_t kk = P;
            cur = best_g;
            while (cur != g0 && kk > 0) {
              cur = step(cur, arc);
              const uint32_t il = rhs.il[arc];
              const ArcRec r = rhs.rec[arc];
              --kk;
              out.out_il[o + kk] = il;
              out.out_ol[o + kk] = r.olabel;
              out.out_w[o + kk] = il == kEpsilon ? r.weight : w_times(w_one(), r.weight);
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
      out.work[2 * si + 1] = relax;
    }
    if (prof) {
      if (stop) prof[16] += 1;
      prof[0] += pops;
#ifdef FSTAMD_BAND_STATS
      prof[1] += advances;
      prof[2] += slides;
#endif
      if (fail != kPathOk && site != 0) {
        if (site >= 4 && site < 8) prof[site] += 1;
        if (site == 10) prof[17] += 1;
        prof[8] = pops;  // the last failure of this wave
        prof[9] = site;
#ifdef FSTAMD_BAND_STATS
        prof[10] = dbg_s;
        prof[11] = dbg_t;
#endif
        prof[12] = slo;
        prof[13] = nn;
        prof[14] = fn;
        prof[15] = L;
      }
    }
  }
  // ---- leave the window, the bitmap and the counts clean ----
  wave_fence();
  for (uint32_t i = lane; i < WS * LC * 2; i += 64) Rw[4 * (size_t)i + 2] = kLdUntouched;
  for (uint32_t i = lane; i < nbw; i += 64) bm[i] = 0ull;
  wave_fence();
  wave_lds_sync();
}

template <uint32_t BKB, bool FP>
__global__ void __launch_bounds__(64) FSTAMD_BAND_ATTR
lazy_band_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item, LbWs ws,
                 BatchOutDev out) {
  extern __shared__ unsigned long long lb_dyn[];
  __shared__ LbLds S;
  unsigned long long* bm = lb_dyn;                        // [ring / 64] open-at-dcur bitmap
  uint32_t* lab = (uint32_t*)(lb_dyn + kLbIdRing / 64);  // [lcap] the string's labels
  const uint32_t lane = threadIdx.x;
  const size_t w = blockIdx.x;
  uint4* R = ws.win + w * ws.wn;
  void* bk = (void*)((uint8_t*)ws.bk + w * ws.tn * ws.bkb);
  uint32_t* idr = ws.idr + w * (size_t)kLbIdRing;
  uint4* fut = ws.fut + w * (size_t)kLbFcap;
  unsigned long long* prof = ws.prof ? ws.prof + w * kLbProf : nullptr;

  for (uint32_t i = lane; i < kLbIdRing / 64; i += 64) bm[i] = 0ull;
  wave_lds_sync();

  const uint32_t num_items = ws.items ? ws.num_items : in.num_strings;
  uint32_t passes = 0;
  for (;;) {
    // one fresh item per pass, fetched by the first active lane (lazy_dense.hpp's loop)
    if (++passes > num_items + 1) return;
    uint32_t item = 0;
    const uint32_t first = (uint32_t)__ffsll((long long)__ballot(1)) - 1;
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == first)
      item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readlane(item, first);
    if (item >= num_items) break;
    const uint32_t si = ws.items ? uni(ws.items[item]) : item;
    const uint64_t off = in.offsets[si];
    const uint32_t L = uni((uint32_t)(in.offsets[si + 1] - off));
    int32_t pre = kPathOk;
    if (rhs.start == kNoState || n_best != 1)  // compose-shortest-path.zig:30-33
      pre = (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN;
    else if (L > ws.lcap)
      pre = kPathUnsupported;
    if (pre == kPathOk) {
      bool zero_label = false;
      for (uint32_t i = lane; i < L; i += 64) {
        const uint32_t x = in.labels[off + i];
        lab[i] = x;
        zero_label |= x == kEpsilon;
      }
      if (__ballot(zero_label) != 0ull) pre = kPathUnsupported;  // lhs epsilon phases
      wave_lds_sync();
    }
    pre = (int32_t)uni((uint32_t)pre);
    if (pre != kPathOk) {
      if (lane == 0) write_status(out, si, pre, 0, 0);
    } else {
      lazy_band_string<BKB, FP>(rhs, in, ws, out, R, bk, idr, fut, bm, lab, S, prof, si, L);
    }
  }
}

}  // namespace fstamd
