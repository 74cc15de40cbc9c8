// device_common.hpp -- device helpers shared by the gfx950 batch kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "../device_engine.hpp"
#include "../fst_core.hpp"

namespace fstamd {

constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;
constexpr unsigned long long kMaxU64 = ~0ull;

// Debug builds (make DEBUG_BOUNDS=1) check every indexed access FB(i, cap, site):
// an out-of-range index is reported with device printf and clamped to 0, so a bug
// shows up as a message instead of a GPU memory fault.  Release builds: no-op.
#ifdef FSTAMD_DEBUG_BOUNDS
#define FSTAMD_DEBUG_FB 1
#define FSTAMD_DEBUG_FT 1
#define FSTAMD_DEBUG_WAIT 1
#endif

#ifdef FSTAMD_DEBUG_FB
__device__ __forceinline__ uint64_t fst_bound(uint64_t i, uint64_t cap, int site) {
  if (i >= cap) {
    printf("[fstamd OOB] site %d index %llu cap %llu block %u thread %u\n", site,
           (unsigned long long)i, (unsigned long long)cap, blockIdx.x, threadIdx.x);
    return 0;
  }
  return i;
}
#define FB(i, cap, site) fst_bound((uint64_t)(i), (uint64_t)(cap), (site))
#else
#define FB(i, cap, site) (i)
#endif

#if defined(FSTAMD_DEBUG_FT) || defined(FSTAMD_DEBUG_WAIT)
// Progress trace into fine-grained host memory (survives a queue abort): thread 0 of
// each workgroup records (item, string, layer, phase) before every phase.
__device__ uint32_t* g_fst_trace;
#endif
#ifdef FSTAMD_DEBUG_FT
__device__ __forceinline__ void fst_trace(uint32_t item, uint32_t si, uint32_t k, uint32_t ph) {
  uint32_t* t = g_fst_trace;
  if (t && threadIdx.x == 0) {
    volatile uint32_t* w = t + blockIdx.x * 4;
    w[0] = item; w[1] = si; w[2] = k; w[3] = ph;
    __threadfence_system();
  }
}
#define FT(item, si, k, ph) fst_trace((item), (si), (k), (ph))
#else
#define FT(item, si, k, ph) ((void)0)
#endif

// The arena slot of string si's path of P arcs: the next P slots of the batch's cursor,
// or, in the streamed host batch (BatchOutDev::slots), the string's fixed slot.
__device__ __forceinline__ unsigned long long reserve_path(const BatchOutDev& out, uint32_t si,
                                                           uint32_t P) {
  return out.slots ? out.slots[si] : atomicAdd(out.cursor, (unsigned long long)P);
}

// Streamed host batches (BatchOutDev::host_ol): after a batched chase, the wave copies the
// finished paths' olabels and weights from their arena slots to the host-mapped result,
// one string at a time so every store writes whole lines (the chase's own stores are one
// lane per string, scattered).  The chase's stores come from other lanes of this same wave,
// so a work-group-scope fence orders them before the reads (on gfx950 it emits nothing: a
// wave's vector memory operations go through one L1 in order).  Round 5 first used an
// agent-scope acquire here -- s_waitcnt vmcnt(0) + buffer_inv sc1 per chase, a cache
// invalidate every 16 strings on every wave.
// Round 6, measured and not kept (FSTAMD_COPYOUT_WIDE builds): 16-B units.  A string's
// olabels and weights (L = 64: 256 + 512 B) went out as 16-B lane stores -- 48 lanes, one
// load and one store instruction per string -- instead of 4- and 8-B lane stores.  The
// copy-out holds the pull tier back by ~1 ms per part of the streamed batch (its trace with
// and without it): device-initiated writes over PCIe run at ~30 GB/s.  The
// wide stores were slower still (A/B on one box, 1M metric strings through the host entry:
// 31.0-31.3 vs 29.9-30.4 ms, profiles/r06/ab_copyout_wide.txt).  The head and tail elements
// before / after the 16-B aligned middle go out one element per lane in the same pass; the
// device arena and the host result share each element's address modulo 16 (run_streamed
// shifts the arena's base pointers to match the shard's first label).
#ifdef FSTAMD_COPYOUT_WIDE
__device__ __forceinline__ void copy_out_paths(const BatchOutDev& out, uint32_t njobs,
                                               uint64_t my_o, uint32_t my_L, uint32_t lane) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  for (uint32_t j = 0; j < njobs; ++j) {  // uniform
    const uint32_t Lj = __builtin_amdgcn_readlane(my_L, j);
    const uint64_t oj = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(my_o >> 32), j) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((uint32_t)my_o, j);
    const uint32_t* dol = out.out_ol + oj;
    uint32_t* hol = out.host_ol + oj;
    const double* dw = out.out_w + oj;
    double* hw = out.host_w + oj;
    // olabels: ha head elements, nq 16-B units, then the tail; weights: hb, nw, tail
    const uint32_t ha = min(Lj, (4u - (uint32_t)(((uintptr_t)hol >> 2) & 3u)) & 3u);
    const uint32_t nq = (Lj - ha) >> 2, ta = Lj - ha - 4 * nq;
    const uint32_t hb = min(Lj, (uint32_t)(((uintptr_t)hw >> 3) & 1u));
    const uint32_t nw = (Lj - hb) >> 1, tb = Lj - hb - 2 * nw;
    const uint32_t units = nq + nw + ha + ta + hb + tb;
    for (uint32_t u = lane; u < units; u += 64) {
      if (u < nq) {
        *reinterpret_cast<u32x4*>(hol + ha + 4 * u) =
            *reinterpret_cast<const u32x4*>(dol + ha + 4 * u);
      } else if (u < nq + nw) {
        const uint32_t v = u - nq;
        *reinterpret_cast<u32x4*>(hw + hb + 2 * v) =
            *reinterpret_cast<const u32x4*>(dw + hb + 2 * v);
      } else {  // single elements: olabel head, olabel tail, weight head, weight tail
        uint32_t r = u - nq - nw;
        if (r < ha) {
          hol[r] = dol[r];
        } else if ((r -= ha) < ta) {
          hol[ha + 4 * nq + r] = dol[ha + 4 * nq + r];
        } else if ((r -= ta) < hb) {
          hw[0] = dw[0];
        } else {
          hw[hb + 2 * nw] = dw[hb + 2 * nw];
        }
      }
    }
  }
}
#else
__device__ __forceinline__ void copy_out_paths(const BatchOutDev& out, uint32_t njobs,
                                               uint64_t my_o, uint32_t my_L, uint32_t lane) {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  for (uint32_t j = 0; j < njobs; ++j) {  // uniform
    const uint32_t Lj = __builtin_amdgcn_readlane(my_L, j);
    const uint64_t oj = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(my_o >> 32), j) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((uint32_t)my_o, j);
    for (uint32_t x = lane; x < Lj; x += 64) {
      __builtin_nontemporal_store(out.out_ol[oj + x], out.host_ol + oj + x);
      __builtin_nontemporal_store(out.out_w[oj + x], out.host_w + oj + x);
    }
  }
}
#endif

// Fst.arcsByIlabel (src/fst.zig:112-136): global arc range [lo, hi) of the arcs of
// state `s` whose ilabel == label.  Spans of <= 8 arcs are counted with independent
// loads (no dependent binary-search chain); longer spans use the two binary searches.
__device__ __forceinline__ void span_by_ilabel(const RhsView& r, uint32_t s, uint32_t label,
                                               uint32_t& lo, uint32_t& hi) {
  const uint2 sp = r.span[FB(s, r.num_states, 1)];
  const uint32_t off = sp.x, n = sp.y;
  if (n <= 8) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      x[i] = (uint32_t)i < n ? r.il[FB(off + i, r.num_arcs, 2)] : 0xFFFFFFFFu;
    uint32_t cl = 0, ch = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool v = (uint32_t)i < n;
      cl += (v && x[i] < label) ? 1u : 0u;
      ch += (v && x[i] <= label) ? 1u : 0u;
    }
    lo = off + cl;
    hi = off + ch;
    return;
  }
  uint32_t a = 0, b = n;
  while (a < b) {
    const uint32_t m = a + ((b - a) >> 1);
    if (r.il[FB(off + m, r.num_arcs, 3)] < label) a = m + 1;
    else b = m;
  }
  const uint32_t first = a;
  b = n;
  while (a < b) {
    const uint32_t m = a + ((b - a) >> 1);
    if (r.il[FB(off + m, r.num_arcs, 4)] <= label) a = m + 1;
    else b = m;
  }
  lo = off + first;
  hi = off + a;
}

// arcsByIlabel for a wave-uniform state with many arcs (the wave-per-string replays: a
// tagger's root and boundary states carry ~100-300 arcs, one per UTF-8 lead byte).  The
// two binary searches above are chains of ~2 log2(n) dependent loads (the root of the
// WeText-scale stand-in: ~18 round trips per pop); here the whole wave counts the arcs
// below / up to `label`, 8 chunks of 64 ilabels per round trip, and past 512 arcs a first
// round samples 64 evenly spaced ilabels to narrow each bound to one window of n / 64.
// Every lane must be active (uniform control flow); lo, hi come out wave-uniform.
__device__ __forceinline__ void wave_count_ilabels(const RhsView& r, uint32_t base, uint32_t n,
                                                   uint32_t label, uint32_t& lt, uint32_t& le) {
  const uint32_t lane = threadIdx.x & 63;
  lt = 0;
  le = 0;
  for (uint32_t b0 = 0; b0 < n; b0 += 512) {
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t i = b0 + k * 64 + lane;
      x[k] = i < n ? r.il[FB(base + i, r.num_arcs, 5)] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool v = b0 + k * 64 + lane < n;
      lt += (uint32_t)__popcll(__ballot(v && x[k] < label));
      le += (uint32_t)__popcll(__ballot(v && x[k] <= label));
    }
  }
}
__device__ __forceinline__ void wave_span_by_ilabel(const RhsView& r, uint32_t off, uint32_t n,
                                                    uint32_t label, uint32_t& lo, uint32_t& hi) {
  if (n <= 512) {
    uint32_t lt, le;
    wave_count_ilabels(r, off, n, label, lt, le);
    lo = off + lt;
    hi = off + le;
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  auto q = [n](uint32_t k) { return (uint32_t)(((uint64_t)k * n) >> 6); };
  const uint32_t smp = r.il[FB(off + q(lane), r.num_arcs, 6)];
  const uint32_t klt = (uint32_t)__popcll(__ballot(smp < label));
  const uint32_t kle = (uint32_t)__popcll(__ballot(smp <= label));
  // the first arc with ilabel >= label lies in [q(k - 1) + 1, q(k)] for k = klt (q(64) = n)
  const uint32_t a0 = klt ? q(klt - 1) + 1 : 0, a1 = klt < 64 ? q(klt) : n;
  const uint32_t b0 = kle ? q(kle - 1) + 1 : 0, b1 = kle < 64 ? q(kle) : n;
  uint32_t lt, le, dummy;
  wave_count_ilabels(r, off + a0, a1 - a0, label, lt, dummy);
  wave_count_ilabels(r, off + b0, b1 - b0, label, dummy, le);
  lo = off + a0 + lt;
  hi = off + b0 + le;
}

// arcsByIlabel (src/fst.zig:112-136) with the per-state summary: one 16-B load when all
// arcs of the state share an ilabel (or it has none), binary search otherwise.
// kTwo: answer a two-label state (RhsView::sspan2) without the search.  Only the general
// engine's graph-lhs expansion asks for it (config 1's epsilon-dense lattice: every state
// is an epsilon run then label 1; kernel 133.6 -> 123.6 ms); on the batch tiers' small
// lattices the extra branch measured 2-3 % slower.
template <bool kTwo = false>
__device__ __forceinline__ void span_summary(const RhsView& r, uint32_t s, uint32_t label,
                                             uint32_t& lo, uint32_t& cnt) {
  const uint4 ss = r.sspan[FB(s, r.num_states, 30)];
  if (ss.z == label) {
    lo = ss.x;
    cnt = ss.y;
  } else if (ss.z != kSpanMixed) {
    lo = ss.x;
    cnt = 0;
  } else if (label == 0u) {  // kEpsilon: a mixed state's leading epsilon run, ss.w arcs
    lo = ss.x;
    cnt = ss.w;
  } else if (!kTwo) {
    uint32_t a, b;
    span_by_ilabel(r, s, label, a, b);
    lo = a;
    cnt = b - a;
  } else if (const uint4 s2 = r.sspan2[FB(s, r.num_states, 31)]; label == s2.x) {
    lo = ss.x;  // the first ilabel's run
    cnt = s2.z;
  } else if (s2.w) {  // two labels: a run of a, then z (ilabels ascending)
    lo = label < s2.x ? ss.x : label <= s2.y ? ss.x + s2.z : ss.x + ss.y;
    cnt = label == s2.y ? ss.y - s2.z : 0u;
  } else {
    uint32_t a, b;
    span_by_ilabel(r, s, label, a, b);
    lo = a;
    cnt = b - a;
  }
}

// Inclusive prefix sum over the 64 lanes with DPP (row_shr 1/2/4/8, row_bcast 15/31):
// six VALU ops, no LDS round trip; every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

// Wavefront inclusive prefix sum (64 lanes): DPP when the whole wave is active (the
// callers' usual case: uniform control flow), else shuffles (six ds_bpermute round trips).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  if (__builtin_amdgcn_read_exec() == ~0ull) return wave_incl_scan_dpp(x);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// Workgroup exclusive scan in thread order; `scratch` holds WG/64 words.
template <int WG>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch,
                                                    uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if constexpr (WG == 64) {
    total = __builtin_amdgcn_readlane(inc, 63);
    return inc - v;
  } else {
    if (lane == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) {
      const uint32_t t = scratch[i];
      base += (i < w) ? t : 0u;
      tot += t;
    }
    __syncthreads();
    total = tot;
    return base + inc - v;
  }
}

}  // namespace fstamd
