// eager_pull.hip -- the pull tier's reverse arc mirror (host build + upload) and launches.
// Kernel and proof: kernels/eager_pull.hpp.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "device_engine.hpp"
#include "host_fst.hpp"
#include "kernels/eager_pull.hpp"
#include "kernels/lazy_pull.hpp"

namespace fstamd {

namespace {
// Waves per SIMD the compiler targets: 5 fit spill-free with blocks of <= 5 records (the
// metric: 5 waves 20.3 M strings/s, 4 waves 18.5 M, 6 waves 19.8 M with spills);
// 8-record blocks need 4.

// RK: the records the kernel reads -- 0 RevRec (f64 cells), 1 rrec32, 2 rrec8 (f32 cells)
template <int KP, int WV, int RK>
const void* pull_kernel_ptr(bool direct) {
  return direct ? (const void*)eager_pull_kernel<kPullRows, KP, true, WV, RK>
                : (const void*)eager_pull_kernel<kPullRows, KP, false, WV, RK>;
}
#ifndef FSTAMD_PULL_WAVES_SMALL  // A/B builds: waves per SIMD for blocks of <= 5 records
#define FSTAMD_PULL_WAVES_SMALL 5
#endif
#ifndef FSTAMD_PULL_WAVES_F32  // A/B builds: the same with f32 cells (8-B cells, f32 merge)
#define FSTAMD_PULL_WAVES_F32 6
#endif
// ... and with the 8-B records: 7 waves (3 VGPRs spilled outside the layer loop) measured
// 37.1 ms per 1M metric strings, 6 waves 37.7 ms, 8 waves (10 spilled) 38.9 ms
#ifndef FSTAMD_PULL_WAVES_R8
#define FSTAMD_PULL_WAVES_R8 7
#endif
template <int RK>
const void* pull_kernel_for(const RevView& rv) {
  const bool dir = rv.direct != 0;
  constexpr int wv = RK == 5 ? 4  // (f64 cells and a 2 KB weight table: 8.9 KB of LDS)
                   : RK == 4 ? FSTAMD_PULL_WAVES_SMALL  // (f64 cells)
                   : RK >= 2 ? FSTAMD_PULL_WAVES_R8 : RK ? FSTAMD_PULL_WAVES_F32 : FSTAMD_PULL_WAVES_SMALL;
  switch (rv.kp) {
    case 4: return pull_kernel_ptr<4, wv, RK>(dir);
    case 5: return pull_kernel_ptr<5, wv, RK>(dir);
    default: return pull_kernel_ptr<8, 4, RK>(dir);
  }
}
// the 8-B records when the rhs has them (every weight an integer <= kRec8WMax)
bool use_rec8(const RevView& rv) { return rv.rrec8 && !std::getenv("FSTAMD_NO_REC8"); }
// FSTAMD_ROUTE_LOG: which records the pull kernel reads (0 RevRec / f64 cells, 1 rrec32,
// 2 rrec8, 3 rrec4, 4 rrec4 with weight indices and f64 cells, 5 the same with a 256-entry
// table) and the weight scale 2^k of
// the integer records (tests)
int route_rk(const char* sem, int rk, const RevView& rv, bool log) {
  if (log && std::getenv("FSTAMD_ROUTE_LOG"))
    std::fprintf(stderr, "[libfst_amd route] %s pull: records %d, weight scale %g\n", sem, rk,
                 rk && rk < 4 ? 1.0 / rv.winv : 1.0);
  return rk;
}
int pull_rk(const DeviceFst& rhs, uint32_t max_len) {
  if (!pull_f32(rhs, max_len) || std::getenv("FSTAMD_P_F64"))  // f64 cells
    return rhs.rev.rrec4 && rhs.widx && !std::getenv("FSTAMD_NO_REC4")
               ? (rhs.wt_n <= kPullWt ? 4 : 5)
               : 0;
  if (rhs.rev.rrec4 && use_rec8(rhs.rev) && !std::getenv("FSTAMD_NO_REC4")) return 3;
  return use_rec8(rhs.rev) ? 2 : 1;
}
const void* pull_kernel_for(const DeviceFst& rhs, uint32_t max_len, bool log = false) {
  switch (route_rk("eager", pull_rk(rhs, max_len), rhs.rev, log)) {
    case 0: return pull_kernel_for<0>(rhs.rev);
    case 5: return pull_kernel_for<5>(rhs.rev);
    case 4: return pull_kernel_for<4>(rhs.rev);
    case 3: return pull_kernel_for<3>(rhs.rev);
    case 2: return pull_kernel_for<2>(rhs.rev);
    default: return pull_kernel_for<1>(rhs.rev);
  }
}
// Lazy pull: 4 waves per SIMD with f64 cells (10.0 KB of LDS; round 5: 3 at 12.8 KB), 5
// with f32 cells (7.4 KB; round 3: 4 at 10.2 KB) when every distance is an integer below
// 2^24.
#ifndef FSTAMD_LP_WAVES_F32  // A/B builds
#define FSTAMD_LP_WAVES_F32 5
#endif
#ifndef FSTAMD_LP_WAVES_F64
#define FSTAMD_LP_WAVES_F64 4
#endif
constexpr int kLazyPullWaves = 3;
// B1: 1-B back records (DeviceFst::byte_back; the direct layout only)
template <int KP, int RK>
const void* lazy_pull_ptr(bool direct, bool b1) {
  constexpr int wv = KP > 5 ? kLazyPullWaves  // (8-record blocks spill at 4)
                   : RK ? FSTAMD_LP_WAVES_F32 : FSTAMD_LP_WAVES_F64;
  if (!direct) return (const void*)lazy_pull_kernel<kPullRows, KP, false, wv, RK, false>;
  return b1 ? (const void*)lazy_pull_kernel<kPullRows, KP, true, wv, RK, true>
            : (const void*)lazy_pull_kernel<kPullRows, KP, true, wv, RK, false>;
}
template <int RK>
const void* lazy_pull_kernel_for(const DeviceFst& rhs) {
  const bool dir = rhs.rev.direct != 0, b1 = dir && rhs.byte_back;
  switch (rhs.rev.kp) {
    case 4: return lazy_pull_ptr<4, RK>(dir, b1);
    case 5: return lazy_pull_ptr<5, RK>(dir, b1);
    default: return lazy_pull_ptr<8, RK>(dir, b1);
  }
}
const void* lazy_pull_kernel_for(const DeviceFst& rhs, uint32_t max_len, bool log = false) {
  const int rk = !lazy_pull_f32(rhs, max_len) ? 0 : use_rec8(rhs.rev) ? 2 : 1;
  if (log && std::getenv("FSTAMD_ROUTE_LOG"))
    std::fprintf(stderr, "[libfst_amd route] lazy pull: back records %d B\n",
                 rhs.rev.direct && rhs.byte_back ? 1 : 4);
  switch (route_rk("lazy", rk, rhs.rev, log)) {
    case 0: return lazy_pull_kernel_for<0>(rhs);
    case 2: return lazy_pull_kernel_for<2>(rhs);
    default: return lazy_pull_kernel_for<1>(rhs);
  }
}
}  // namespace

void free_reverse_mirror(DeviceFst* d) {
  for (void*& p : d->rev_bufs) {
    if (p) (void)hipFree(p);
    p = nullptr;
  }
  d->rev = RevView{};
  d->pull_ok = false;
  d->widx = false;
  d->wt_n = 0;
}

bool build_reverse_mirror(DeviceFst* d, const FrozenFst& f) {
  d->pull_ok = false;
  d->lazy_pull_ok = false;
  if (std::getenv("FSTAMD_NO_PULL")) return true;
  // the pull tier's contract: layered lattices (no input epsilon) and the push tiers'
  // weights (>= +0, no NaN)
  if (d->has_eps || !d->nonneg || d->nan) return true;
  const uint32_t ns = f.num_states(), na = f.header().num_arcs;
  if (ns == 0 || ns >= (1u << 27)) return true;  // records hold 8 * state < 2^30
  const StateEntry* se = f.states();
  const PackedArc* pa = f.arcs();
  // the device numbering (DeviceFst::perm): sources and targets by their device ids
  const std::vector<uint32_t>& perm = d->perm;
  auto pid = [&](uint32_t s) { return perm.empty() ? s : perm[s]; };

  // j of every arc: its position in the source's run of equal ilabels (spans are sorted
  // by ilabel, fst.zig:258-265).  A run longer than 8 does not fit the key's 3 bits.
  std::vector<uint8_t> jpos(na);
  std::vector<uint32_t> src(na);
  std::vector<uint32_t> indeg(ns + 1, 0);
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t run = se[s].arc_offset;
    for (uint32_t a = se[s].arc_offset; a < se[s].arc_offset + se[s].num_arcs; ++a) {
      if (a > se[s].arc_offset && pa[a].ilabel != pa[a - 1].ilabel) run = a;
      if (a - run >= 8) return true;
      jpos[a] = (uint8_t)(a - run);
      src[a] = pid(s);
      ++indeg[pid(pa[a].nextstate)];
    }
  }
  // lazy pull: within a same-ilabel run, arcs into one target must come in olabel order
  // (fromMutable sorts by (ilabel, olabel, weight, nextstate); a fromBytes blob may not)
  bool ol_ordered = true;
  for (uint32_t s = 0; s < ns && ol_ordered; ++s)
    for (uint32_t a = se[s].arc_offset; a < se[s].arc_offset + se[s].num_arcs && ol_ordered; ++a)
      for (uint32_t b = a - jpos[a]; b < a; ++b)
        if (pa[b].nextstate == pa[a].nextstate && pa[b].olabel > pa[a].olabel) {
          ol_ordered = false;
          break;
        }
  // in-arcs by target (counting sort), then by (ilabel, source, j) within a target
  std::vector<uint32_t> ioff(ns + 1, 0);
  for (uint32_t t = 0; t < ns; ++t) ioff[t + 1] = ioff[t] + indeg[t];
  std::vector<uint32_t> in(na), fill(ioff.begin(), ioff.end() - 1);
  for (uint32_t a = 0; a < na; ++a) in[fill[pid(pa[a].nextstate)]++] = a;
  for (uint32_t t = 0; t < ns; ++t)
    std::sort(in.begin() + ioff[t], in.begin() + ioff[t + 1], [&](uint32_t x, uint32_t y) {
      if (pa[x].ilabel != pa[y].ilabel) return pa[x].ilabel < pa[y].ilabel;
      if (src[x] != src[y]) return src[x] < src[y];
      return jpos[x] < jpos[y];
    });
  // groups: runs of equal ilabel within a target's in-arcs
  struct Group { uint32_t t, label, first, n; };
  std::vector<Group> groups;
  for (uint32_t t = 0; t < ns; ++t)
    for (uint32_t i = ioff[t]; i < ioff[t + 1];) {
      uint32_t e = i + 1;
      while (e < ioff[t + 1] && pa[in[e]].ilabel == pa[in[i]].ilabel) ++e;
      groups.push_back(Group{t, pa[in[i]].ilabel, i, e - i});
      i = e;
    }
  // block size: the fewest record slots, a further block of a group counted double (the
  // kernel visits it in a separate loop)
  uint32_t kp = 8;
  uint64_t best_cost = ~0ull;
  for (uint32_t cand : {4u, 5u, 8u}) {
    uint64_t cost = 0;
    for (const Group& g : groups) {
      const uint64_t nb = (g.n + cand - 1) / cand;
      cost += nb * cand + (nb - 1) * cand;
    }
    if (cost < best_cost) {
      best_cost = cost;
      kp = cand;
    }
  }
  // Direct layout: when every state has at most one in-label group (and no label collides
  // with the kSpan* markers), the first block of state t sits at record t * kp, so the
  // kernel loads it together with rspan[t] instead of after it (one L2 round trip per
  // target row instead of two).  Further blocks follow the direct region.
  bool direct = !std::getenv("FSTAMD_PULL_INDIRECT");
  for (size_t g = 0; g < groups.size() && direct; ++g)
    if ((g > 0 && groups[g].t == groups[g - 1].t) || groups[g].label >= (1u << 24)) direct = false;
  const uint64_t ndirect = direct ? (uint64_t)ns + kPullW : 0;  // rows may run past the last state
  uint64_t nblocks = direct ? ndirect : 1;  // indirect: block 0 is the null block
  for (const Group& g : groups) nblocks += (g.n + kp - 1) / kp - (direct ? 1 : 0);
  if (nblocks * kp * sizeof(RevRec) > (4ull << 30) || nblocks * kp >= 0xFFFFFFFFull) return true;

  std::vector<RevRec> rrec(nblocks * kp, RevRec{0xFFFFFFF8u, 0u, 0.0});  // padding
  std::vector<uint32_t> rtgt(nblocks * kp, 0u);  // each record's target state (rrec4)
  std::vector<uint32_t> rolab(nblocks * kp, 0u);
  // padded by kPullW entries: a window row may run past the last state
  std::vector<uint4> rspan((size_t)ns + kPullW, make_uint4(0u, 0u, kSpanNone, 0u));
  std::vector<uint4> gtab;
  uint32_t max_groups = 0;
  uint64_t blk = direct ? ndirect : 1;  // next free block past the fixed ones
  for (size_t gi = 0; gi < groups.size();) {
    const uint32_t t = groups[gi].t;
    size_t ge = gi;
    while (ge < groups.size() && groups[ge].t == t) ++ge;
    const uint32_t ng = (uint32_t)(ge - gi);
    // one group whose label is an ordinary one: found from rspan alone; several (or a
    // label that collides with the kSpan* markers): binary search over gtab
    const bool single = ng == 1 && groups[gi].label < kSpanMixed;
    if (!single) {
      rspan[t] = make_uint4((uint32_t)gtab.size(), ng, kSpanMixed, 0u);
      max_groups = std::max(max_groups, ng);
    }
    for (size_t g = gi; g < ge; ++g) {
      const Group& G = groups[g];
      const uint32_t nb = (G.n + kp - 1) / kp;
      // direct: block 0 at t * kp, blocks 1.. from `blk` on (rspan.x = their first record)
      const uint32_t rec0 = (uint32_t)(blk * kp);
      if (single) rspan[t] = make_uint4(rec0, nb, G.label, 0u);
      else gtab.push_back(make_uint4(G.label, rec0, nb, 0u));
      for (uint32_t r = 0; r < G.n; ++r) {
        const uint32_t a = in[G.first + r];
        const uint64_t slot = direct ? (r < kp ? (uint64_t)t * kp + r : blk * kp + (r - kp))
                                     : blk * kp + r;
        const uint32_t m = r % kp;
        rrec[slot] = RevRec{src[a] << 3,
                            ((uint32_t)jpos[a] << 17) | (m << 13) | (pa[a].weight > 0.0 ? kRevPos : 0u),
                            pa[a].weight};
        rolab[slot] = pa[a].olabel;
        rtgt[slot] = t;
      }
      blk += nb - (direct ? 1 : 0);
    }
    gi = ge;
  }
  uint32_t gsearch = 0;  // 0: no state has several in-labels (the kernel skips the search)
  if (!gtab.empty())
    while ((1u << gsearch) < max_groups + 1) ++gsearch;

  // integer arc weights in [0, 2^24): the pull tiers may keep their cells' distances in f32
  // (exact while L * int_wmax < 2^24, pull_f32), reading the f32 copy of the records.
  // Dyadic weights (0.5, 1.25, ...: integers after a power-of-two scale 2^k, k <= 8) take
  // the same tiers: f64 sums of such weights are exact (multiples of 2^-k far below 2^53),
  // so integer sums of the scaled weights order and tie exactly as the reference's f64 sums,
  // and the kernels multiply by 2^-k (RevView::winv, exact) only what they output.
  double wscale = 0.0;
  for (int k = 0; k <= 8 && wscale == 0.0; ++k) {
    const double sc = (double)(1u << k);
    bool ok = true;
    for (uint32_t a = 0; a < na && ok; ++a) {
      const double w = pa[a].weight * sc;  // (exact: a power of two)
      ok = w >= 0.0 && w == __builtin_trunc(w) && w < 16777216.0;
    }
    if (ok) wscale = sc;
  }
  d->int_wmax = wscale > 0.0 ? 0.0 : -1.0;
  for (uint32_t a = 0; a < na && d->int_wmax >= 0.0; ++a)
    d->int_wmax = std::max(d->int_wmax, pa[a].weight * wscale);
  if (wscale == 0.0) wscale = 1.0;
  auto wsc = [wscale](double w) { return (uint32_t)(w * wscale); };  // scaled integer weight
  // direct layout: per state one 4-B row word ilabel | min(nblocks, 255) << 24 (labels
  // below 2^24, else the layout is indirect), and {block 1's record, nblocks} for hub rows
  std::vector<uint32_t> rlab;
  std::vector<uint2> rxrec;
  if (direct) {
    rlab.resize(rspan.size());
    rxrec.resize(rspan.size());
    for (size_t t = 0; t < rspan.size(); ++t) {
      rlab[t] = (rspan[t].z & 0xFFFFFFu) | (std::min<uint32_t>(rspan[t].y, 255u) << 24);
      rxrec[t] = make_uint2(rspan[t].x, rspan[t].y);
    }
  }
  // 1-B back records: the direct layout, every in-arc group within 255 / kp blocks
  uint64_t max_nb = 0;
  for (const uint4& r : rspan)
    if (r.z != kSpanMixed) max_nb = std::max<uint64_t>(max_nb, r.y);
  const bool byte_back = direct && max_nb * kp <= 255 && !std::getenv("FSTAMD_NO_BYTE_BACK");
  std::vector<uint4> rrec32;
  std::vector<uint2> rrec8;
  if (d->int_wmax >= 0.0 && d->int_wmax <= kRec8WMax) {
    rrec8.resize(rrec.size());
    for (size_t r = 0; r < rrec.size(); ++r)
      rrec8[r] = make_uint2(rrec[r].src, rrec[r].y | wsc(rrec[r].weight));
  }
  // 4-B records for tier P: {8 * (t - source + bias) << 16 | j << 13 | m << 9 | pos << 8 |
  // weight} -- the source as an offset from the target (every arc stays within the rhs's
  // jump range), the key bits in the low half.  Padding: 0xFFFF0000 (an offset past every
  // window).  Only with the 8-B records' weights (integers <= 7) or the weight table's
  // indices (< kPullWtMax), and offsets below 2^13.
  // Weights that are not dyadic (0.1, ln 3): with at most kPullWtMax distinct values the
  // 4-B records hold the value's index in a table instead (RK 4 up to kPullWt = 64 values,
  // RK 5 up to 256: tier P with f64 cells adds the table's f64 value, the very value the
  // reference adds; FSTAMD_NO_WIDX: off)
  std::vector<double> wtab;
  std::unordered_map<uint64_t, uint32_t> widx_of;
  if (d->int_wmax < 0.0 && !std::getenv("FSTAMD_NO_WIDX")) {
    bool ok = true;
    for (uint32_t a = 0; a < na && ok; ++a) {
      const double w = pa[a].weight;
      uint64_t bits;
      std::memcpy(&bits, &w, 8);
      if (widx_of.count(bits)) continue;
      if (!(w >= 0.0) || !std::isfinite(w) || wtab.size() == kPullWtMax) ok = false;
      else {
        widx_of.emplace(bits, (uint32_t)wtab.size());
        wtab.push_back(w);
      }
    }
    if (!ok) {
      wtab.clear();
      widx_of.clear();
    }
  }
  const bool widx = !wtab.empty();
  auto low_weight = [&](double w) -> uint32_t {  // the 4-B record's low byte
    if (!widx) return wsc(w);
    uint64_t bits;
    std::memcpy(&bits, &w, 8);
    return widx_of.at(bits);
  };
  std::vector<uint32_t> rrec4;
  uint32_t rbias8 = 0;
  if (!rrec8.empty() || widx) {
    int64_t dlo = 0, dhi = 0;
    for (size_t r = 0; r < rrec.size(); ++r) {
      if (rrec[r].src == 0xFFFFFFF8u) continue;
      const int64_t dl = (int64_t)rtgt[r] - (int64_t)(rrec[r].src >> 3);
      dlo = std::min(dlo, dl);
      dhi = std::max(dhi, dl);
    }
    // Both halves of the bound: the offsets fit the high half, and the largest lane base
    // of a window, 8 * (kPullW - 1) + rbias8, stays below a padding record's 0xFFFF, so
    // base - 0xFFFF always wraps past slot W (a backward jump of ~7,900 states would
    // otherwise turn padding into an in-window cell)
    // Tier P then keeps 1-B back records (x * kp + m, eager_pull.hpp): byte_back below
    if ((dhi - dlo) * 8 < 0xFFF0 && -dlo * 8 + 8 * (int64_t)kPullW <= 0xFFFF && byte_back) {
      rbias8 = (uint32_t)(-dlo * 8);
      rrec4.resize(rrec.size());
      for (size_t r = 0; r < rrec.size(); ++r) {
        const uint32_t y = rrec[r].y;
        if (rrec[r].src == 0xFFFFFFF8u) {
          rrec4[r] = 0xFFFF0000u;
        } else {
          const uint32_t low = (((y >> 17) & 7u) << 13) | (((y >> 13) & 15u) << 9) |
                               (((y >> 12) & 1u) << 8) | low_weight(rrec[r].weight);
          const int64_t dl = (int64_t)rtgt[r] - (int64_t)(rrec[r].src >> 3);
          rrec4[r] = ((uint32_t)((dl - dlo) * 8) << 16) | low;
        }
      }
    }
  }
  if (d->int_wmax >= 0.0) {
    rrec32.resize(rrec.size());
    for (size_t r = 0; r < rrec.size(); ++r)  // the weight: an integer below 2^24
      rrec32[r] = make_uint4(rrec[r].src, rrec[r].y, wsc(rrec[r].weight), rolab[r]);
  }
  if (rrec4.empty()) wtab.clear();  // (the table serves the 4-B records only)
  if (!wtab.empty()) {  // appended to the records (rv_weight_table)
    d->wt_n = (uint32_t)wtab.size();
    wtab.resize(kPullWtMax, 0.0);
    rrec4.resize((rrec4.size() + 1) & ~(size_t)1, 0xFFFF0000u);
    const size_t at = rrec4.size();
    rrec4.resize(at + 2 * kPullWtMax);
    std::memcpy(rrec4.data() + at, wtab.data(), kPullWtMax * sizeof(double));
  }
  d->widx = !wtab.empty();
  auto up = [&](int i, const void* src_p, size_t bytes) -> bool {
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&d->rev_bufs[i], bytes) != hipSuccess) return false;
    return hipMemcpy(d->rev_bufs[i], src_p, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
  if (gtab.empty()) gtab.push_back(zero4);
  if (!up(0, rspan.data(), rspan.size() * sizeof(uint4)) ||
      !up(1, gtab.data(), gtab.size() * sizeof(uint4)) ||
      !up(2, rrec.data(), rrec.size() * sizeof(RevRec)) ||
      !up(3, rolab.data(), rolab.size() * sizeof(uint32_t)) ||
      (!rrec32.empty() && !up(4, rrec32.data(), rrec32.size() * sizeof(uint4))) ||
      (!rrec8.empty() && !up(5, rrec8.data(), rrec8.size() * sizeof(uint2))) ||
      (direct && (!up(6, rlab.data(), rlab.size() * sizeof(uint32_t)) ||
                  !up(7, rxrec.data(), rxrec.size() * sizeof(uint2)))) ||
      (!rrec4.empty() && !up(8, rrec4.data(), rrec4.size() * sizeof(uint32_t)))) {
    free_reverse_mirror(d);
    return false;
  }
  d->rev = RevView{(const uint4*)d->rev_bufs[0], (const uint4*)d->rev_bufs[1],
                   (const RevRec*)d->rev_bufs[2], (const uint32_t*)d->rev_bufs[3], kp, gsearch,
                   direct ? 1u : 0u, (const uint4*)d->rev_bufs[4], (const uint2*)d->rev_bufs[5],
                   (const uint32_t*)d->rev_bufs[6], (const uint2*)d->rev_bufs[7],
                   (uint32_t)(nblocks * kp), (const uint32_t*)d->rev_bufs[8], rbias8,
                   1.0 / wscale};
  d->byte_back = byte_back;
  d->pull_ok = true;
  d->lazy_pull_ok = ol_ordered && d->finite && !std::getenv("FSTAMD_NO_LAZY_PULL");
  return true;
}

bool pull_f32(const DeviceFst& rhs, uint32_t max_len) {
  return rhs.int_wmax >= 0.0 && rhs.rev.rrec32 && (double)max_len * rhs.int_wmax < 16777216.0;
}

int pull_waves_per_cu(const DeviceFst& rhs, uint32_t max_len) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pull_kernel_for(rhs, max_len), 64, 0) !=
      hipSuccess)
    occ = 1;
  return std::max(occ, 1);
}

hipError_t launch_eager_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n_best,
                             unsigned int* next_item, const EagerLaunch& lp,
                             const BatchOutDev& out, uint32_t grid, hipStream_t stream) {
  void* args[] = {(void*)&rhs.view, (void*)&rhs.rev, (void*)&in, (void*)&n_best,
                  (void*)&next_item, (void*)&lp, (void*)&out};
  return hipLaunchKernel(pull_kernel_for(rhs, in.max_len, true), dim3(grid), dim3(64), args, 0, stream);
}

bool lazy_pull_f32(const DeviceFst& rhs, uint32_t max_len) {
  // (the f32 cells keep d - tb <= the largest arc weight in 8 bits, kernels/lazy_pull.hpp)
  return pull_f32(rhs, max_len) && rhs.int_wmax <= kLpF32WMax && !std::getenv("FSTAMD_LP_F64");
}

int lazy_pull_waves_per_cu(const DeviceFst& rhs, uint32_t max_len) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, lazy_pull_kernel_for(rhs, max_len), 64, 0) !=
      hipSuccess)
    occ = 1;
  return std::max(occ, 1);
}

hipError_t launch_lazy_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n_best,
                            unsigned int* next_item, const EagerLaunch& lp,
                            const BatchOutDev& out, uint32_t grid, hipStream_t stream) {
  void* args[] = {(void*)&rhs.view, (void*)&rhs.rev, (void*)&in, (void*)&n_best,
                  (void*)&next_item, (void*)&lp, (void*)&out};
  return hipLaunchKernel(lazy_pull_kernel_for(rhs, in.max_len, true), dim3(grid), dim3(64), args, 0,
                         stream);
}

}  // namespace fstamd
