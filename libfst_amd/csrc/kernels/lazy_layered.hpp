// lazy_layered.hpp -- composeShortestPath on layered lattices, one wavefront per string
// (gfx950 / CDNA4).  The lazy engine for the tier-A domain: chain inputs without label 0
// against an rhs without input epsilons and with finite weights >= 0 (the metric's shape).
//
// Same decomposition as bfs_lazy_path (kernels/eager_bfs.hpp; tests/lazy_model.py is the
// executable model): dist = least fixpoint, lid = first-touch order from the pop rounds,
// back = lexmin (lid(source), il, ol, candidate) over tight in-arcs, best = lexmin
// (total, lid), path = back-pointers until the start (compose-shortest-path.zig:26-401).
// What the layered shape buys:
//   * tuple (k, s2) -- input position k, rhs state s2; filter 0 throughout -- lives at the
//     dense index k * NS + s2 of per-wave arrays: no hash, no BFS ids (the lazy answer
//     never uses compose's ids, only lids);
//   * the arcs of (k, s2) are the rhs arcs of s2 labelled labels[k], read straight from
//     the L2-resident rhs (span summary + records), never stored;
//   * every arc goes from layer k to k+1, so one pass in layer order gives the exact
//     distances;
//   * the round state (active list, members in lid order) stays in LDS and registers:
//     a round costs a handful of dependent global accesses, not dozens.
// The dense arrays are clean (~0 / 0) between strings: each string resets the entries it
// touched before taking the next one, whatever its status.
#pragma once

#include "device_common.hpp"
#include "eager_layered.hpp"  // write_status
#include "eager_bfs.hpp"      // kLzActive / kLzPopped, prof_mark
#include "eager_wave.hpp"     // wave_lds_sync, wave_excl_scan_small

namespace fstamd {

struct LlWs {
  unsigned long long* dk;    // [grid * dn] okey(dist); ~0 = untouched
  unsigned long long* back;  // [grid * dn] (lid(source) << 32) | candidate index; ~0 = none
  uint32_t* lidf;            // [grid * dn] ~0 untouched, kLlPend | rank touched this round, else lid
  uint32_t* flg;             // [grid * dn] kLzActive | kLzPopped
  uint32_t* nodes;           // [grid * ncap] touched tuples, layer by layer (ncap = dn)
  uint32_t* inv;             // [grid * ncap] lid -> tuple
  uint32_t* loff;            // [grid * (lcap + 2)] layer offsets into nodes
  uint4* act;                // [grid * 2 * acap] active lists {tuple, lid, okey(dist)}
  unsigned long long dn;     // dense tuples per wave = (lcap + 1) * num_states
  uint32_t ncap, lcap, acap;
  unsigned long long wd_ticks;
  unsigned long long* prof;  // [grid * 8] (FSTAMD_BFS_PROF): ticks of layers, rounds,
                             // backs/best/output, reset; items; rounds
  const uint32_t* items;     // null: item i is string i; else the strings to take
  const uint32_t* num_items_dev;  // entries of items (device count)
};

constexpr uint32_t kLlPend = 0x80000000u;
constexpr int kLlCap = 256;          // members per round (LDS)
constexpr uint32_t kLlSpanMax = 64;    // same-label arcs per rhs state (64-bit masks)
constexpr uint64_t kLlDenseMax = 1ull << 24;  // lids and tuples fit 24 bits

struct LlLds {
  uint32_t mnode[kLlCap];            // this round's members: tuple, lid
  uint32_t mlid[kLlCap];
  uint32_t mlo[kLlCap];              // ... and their arcs: rhs span, next layer base
  uint32_t mcnt[kLlCap];
  uint32_t mnb[kLlCap];
  uint32_t keys[kLlCap];             // members (lid << 8 | member), sorted
  uint32_t count;                    // appends (tuples of a layer / activations)
};

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = y < v ? y : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(v, o, 64);
    v = y < v ? y : v;
  }
  return v;
}

// Exclusive prefix minimum over lanes (identity ~0u).
__device__ __forceinline__ uint32_t wave_excl_min_u32(uint32_t v, uint32_t lane) {
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc = y < inc ? y : inc;
  }
  const uint32_t ex = __shfl_up(inc, 1, 64);
  return lane == 0 ? ~0u : ex;
}

// Ascending bitonic sort of one key per lane (64 lanes).
__device__ __forceinline__ uint32_t wave_sort64(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t p = __shfl_xor(v, j, 64);
      const bool up = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == up) ? (p < v ? p : v) : (p > v ? p : v);
    }
  }
  return v;
}

// Ascending bitonic sort of keys[0..P) in LDS, P a power of two <= kLlCap.
__device__ __forceinline__ void lds_sort(uint32_t* keys, uint32_t P, uint32_t lane) {
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < P; i += 64) {
        const uint32_t ij = i ^ j;
        if (ij > i) {
          const uint32_t a = keys[i], b = keys[ij];
          if ((a > b) == ((i & k) == 0)) {
            keys[i] = b;
            keys[ij] = a;
          }
        }
      }
      wave_lds_sync();
    }
  }
}

__device__ __forceinline__ uint32_t rd_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long rd_u64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void global_sync() {  // this wave's global stores -> visible
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// The arcs of one tuple are processed in chunks of kLlKB with every load of a chunk
// issued before any is used (records, then target words): a lane's arcs cost one
// dependent round trip per kind of word, not one per arc.  rec[lo + c] is in bounds for
// c < cnt + kRecPad (padded mirror), so chunk loads are unconditional and masked.
constexpr int kLlKB = 8;

// Waves per SIMD the layered rounds engine is compiled for (5 and 6 measured the same as
// 4 on the metric: the rounds are bound by the memory system's scattered transactions,
// not by resident waves).
#ifndef FSTAMD_LL_WAVES
#define FSTAMD_LL_WAVES 4
#endif
static_assert(kLlKB <= (int)kRecPad, "chunk loads rely on the mirror padding");

__global__ void __launch_bounds__(64, FSTAMD_LL_WAVES)
lazy_layered_kernel(RhsView rhs, ChainInput in, uint32_t n_best, unsigned int* next_item,
                    LlWs ws, BatchOutDev out) {
  __shared__ LlLds S;
  const uint32_t lane = threadIdx.x;
  const size_t w = blockIdx.x;
  unsigned long long* dk = ws.dk + w * ws.dn;
  unsigned long long* back = ws.back + w * ws.dn;
  uint32_t* lidf = ws.lidf + w * ws.dn;
  uint32_t* flg = ws.flg + w * ws.dn;
  uint32_t* nodes = ws.nodes + w * ws.ncap;
  uint32_t* inv = ws.inv + w * ws.ncap;
  uint32_t* loff = ws.loff + w * (ws.lcap + 2);
  const uint32_t NS = rhs.num_states;
  unsigned long long* prof = ws.prof ? ws.prof + w * 8 : nullptr;

  const uint32_t num_items =
      __builtin_amdgcn_readfirstlane(ws.items ? *ws.num_items_dev : in.num_strings);
  for (uint32_t guard = 0;; ++guard) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(next_item, 1u);
    item = __builtin_amdgcn_readfirstlane(item);
    if (item >= num_items) break;
    const uint32_t si = __builtin_amdgcn_readfirstlane(ws.items ? ws.items[item] : item);
    const uint64_t off = in.offsets[si];
    const uint32_t L = __builtin_amdgcn_readfirstlane((uint32_t)(in.offsets[si + 1] - off));
    const uint32_t* labels = in.labels + off;
    const unsigned long long now0 = __builtin_amdgcn_s_memrealtime();
    if (rhs.start == kNoState || n_best != 1) {  // compose-shortest-path.zig:30-33
      if (lane == 0)
        write_status(out, si, (rhs.start == kNoState || n_best == 0) ? kPathEmpty : kPathErrorN,
                     0, 0);
      continue;
    }
    if (L > ws.lcap) {
      if (lane == 0) write_status(out, si, kPathOverflow, 0, 0);
      continue;
    }
    // per-string watchdog: the limit starts with the string, not with the launch
    const unsigned long long deadline = now0 + ws.wd_ticks;
    int32_t fail = kPathOk;
    uint64_t relax = 0;
    unsigned long long tp = now0;
    prof_add(prof, 4, 1);

    // ---- distances, layer by layer (tuples of layer k+1 appended at first touch) ----
    const uint32_t start = rhs.start;  // layer 0: (0, rhs.start)
    if (lane == 0) {
      dk[start] = okey(w_one());
      nodes[0] = start;
      loff[0] = 0;
      loff[1] = 1;
    }
    uint32_t n = 1;
    global_sync();
    for (uint32_t k = 0; k < L && fail == kPathOk; ++k) {
      const uint32_t label = __builtin_amdgcn_readfirstlane(labels[k]);
      if (label == kEpsilon) {  // label-0 input: not layered (general engine)
        fail = kPathUnsupported;
        break;
      }
      const uint32_t f0 = __builtin_amdgcn_readfirstlane(rd_u32(&loff[k]));
      if (lane == 0) S.count = 0;
      wave_lds_sync();
      const size_t nb = (size_t)(k + 1) * NS;
      const uint32_t f1 = n;
      // relax the arcs of one tuple (records then atomics, each batch issued at once)
      auto relax_tuple = [&](uint32_t u, double du, uint4 ss) {
        if (u == kNoState) return;
        uint32_t lo = ss.x, cnt = ss.z == label ? ss.y : 0u;
        if (ss.z == kSpanMixed) {
          uint32_t a, b2;
          span_by_ilabel(rhs, u - k * NS, label, a, b2);
          lo = a;
          cnt = b2 - a;
        }
        relax += cnt;
        for (uint32_t c0 = 0; c0 < cnt; c0 += kLlKB) {
          ArcRec r[kLlKB];
#pragma unroll
          for (int i = 0; i < kLlKB; ++i) r[i] = rhs.rec[lo + c0 + i];
          unsigned long long old[kLlKB];
#pragma unroll
          for (int i = 0; i < kLlKB; ++i)
            old[i] = c0 + i < cnt ? atomicMin(&dk[nb + r[i].next], okey(w_times(du, r[i].weight)))
                                  : 0ull;
          uint32_t fresh = 0;
#pragma unroll
          for (int i = 0; i < kLlKB; ++i) fresh |= (old[i] == ~0ull ? 1u : 0u) << i;
          if (fresh) {
            uint32_t qq = atomicAdd(&S.count, (uint32_t)__popc(fresh));
            while (fresh) {
              const int i = __builtin_ctz(fresh);
              fresh &= fresh - 1;
              nodes[f1 + qq++] = (uint32_t)(nb + rhs.rec[lo + c0 + i].next);  // no r[i]:
                                                                               // dynamic index
            }
          }
        }
      };
      for (uint32_t g0 = f0; g0 < f1; g0 += 4 * 64) {
        // a lane's (up to) 4 tuples: every load issued before any is used
        const uint32_t p0 = g0 + lane, p1 = p0 + 64, p2 = p0 + 128, p3 = p0 + 192;
        const uint32_t u0 = p0 < f1 ? nodes[p0] : kNoState, u1 = p1 < f1 ? nodes[p1] : kNoState,
                       u2 = p2 < f1 ? nodes[p2] : kNoState, u3 = p3 < f1 ? nodes[p3] : kNoState;
        const uint4 none = make_uint4(0u, 0u, kSpanNone, 0u);
        const double d0 = u0 != kNoState ? from_okey(rd_u64(&dk[u0])) : 0.0;
        const double d1 = u1 != kNoState ? from_okey(rd_u64(&dk[u1])) : 0.0;
        const double d2 = u2 != kNoState ? from_okey(rd_u64(&dk[u2])) : 0.0;
        const double d3 = u3 != kNoState ? from_okey(rd_u64(&dk[u3])) : 0.0;
        const uint4 s0 = u0 != kNoState ? rhs.sspan[u0 - k * NS] : none;
        const uint4 s1 = u1 != kNoState ? rhs.sspan[u1 - k * NS] : none;
        const uint4 s2 = u2 != kNoState ? rhs.sspan[u2 - k * NS] : none;
        const uint4 s3 = u3 != kNoState ? rhs.sspan[u3 - k * NS] : none;
        relax_tuple(u0, d0, s0);
        relax_tuple(u1, d1, s1);
        relax_tuple(u2, d2, s2);
        relax_tuple(u3, d3, s3);
      }
      wave_lds_sync();
      n += __builtin_amdgcn_readfirstlane(S.count);
      if (lane == 0) loff[k + 2] = n;
      global_sync();
      if (__builtin_amdgcn_s_memrealtime() > deadline) fail = kPathInternal;
      fail = __builtin_amdgcn_readfirstlane(fail);
    }

    prof_mark(prof, 0, &tp);
    // ---- lazy ids: pop rounds (members = active at dmin, in lid order) ----
    // The active list lives in HBM as {tuple, lid, okey(dist)} entries, double-buffered:
    // each round scans it (coalesced), moves the members into LDS and every other entry
    // into the next list, then appends the activations and the unpopped members.
    uint4* A = ws.act + w * 2 * (size_t)ws.acap;
    uint4* B = A + ws.acap;
    uint32_t nxt = 1, popped = 0, na = 1;
    if (fail == kPathOk) {
      if (lane == 0) {
        lidf[start] = 0;
        inv[0] = start;
        flg[start] = kLzActive;
        const unsigned long long d0 = okey(w_one());
        A[0] = make_uint4(start, 0u, (uint32_t)d0, (uint32_t)(d0 >> 32));
      }
      global_sync();
    }
    while (fail == kPathOk && na > 0) {
      prof_add(prof, 5, 1);
      // (1) dmin over the active entries
      unsigned long long m = ~0ull;
      uint4 reg[4];  // the first 256 entries stay in registers for (2)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t e = q * 64 + lane;
        reg[q] = e < na ? A[e] : make_uint4(0u, 0u, ~0u, ~0u);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned long long d = ((unsigned long long)reg[q].w << 32) | reg[q].z;
        m = d < m ? d : m;
      }
      for (uint32_t e = 256 + lane; e < na; e += 64) {
        const uint4 a = A[e];
        const unsigned long long d = ((unsigned long long)a.w << 32) | a.z;
        m = d < m ? d : m;
      }
      const unsigned long long dmin = wave_min_u64(m);
      // (2) members -> LDS (keys lid << 8 | member), everything else -> B[0..nsv)
      uint32_t M = 0, nsv = 0;
      auto place = [&](const uint4 a, bool valid) {
        const unsigned long long d = ((unsigned long long)a.w << 32) | a.z;
        const bool mem = valid && d == dmin, sv = valid && !mem;
        uint32_t t1, t2;
        const uint32_t pm = M + wave_excl_scan_small<1>(mem ? 1u : 0u, t1);
        const uint32_t ps = nsv + wave_excl_scan_small<1>(sv ? 1u : 0u, t2);
        if (mem && pm < (uint32_t)kLlCap) {
          S.mnode[pm] = a.x;
          S.mlid[pm] = a.y;
          S.keys[pm] = (a.y << 8) | pm;
        }
        if (sv) B[ps] = a;
        M += t1;
        nsv += t2;
      };
#pragma unroll
      for (int q = 0; q < 4; ++q) place(reg[q], (uint32_t)q * 64 + lane < na);
      for (uint32_t b = 256; b < na; b += 64) {
        const uint32_t e = b + lane;
        place(e < na ? A[e] : make_uint4(0u, 0u, 0u, 0u), e < na);
      }
      if (M > (uint32_t)kLlCap) {
        fail = kPathOverflow;
        break;
      }
      wave_lds_sync();
      if (M <= 64) {
        uint32_t v = lane < M ? S.keys[lane] : ~0u;
        v = wave_sort64(v, lane);
        if (lane < M) S.keys[lane] = v;
      } else {
        uint32_t P = 128;
        while (P < M) P <<= 1;
        for (uint32_t i = M + lane; i < P; i += 64) S.keys[i] = ~0u;
        wave_lds_sync();
        lds_sort(S.keys, P, lane);
      }
      wave_lds_sync();
      const double dminw = from_okey(dmin);
      // (3) batch cut: exclusive prefix minimum of joiner lids in member order
      uint32_t kcut = M, carry = ~0u;
      for (uint32_t b = 0; b < M; b += 64) {
        const uint32_t pos = b + lane;
        uint32_t j = ~0u, my = 0;
        if (pos < M) {
          const uint32_t key = S.keys[pos], mi = key & 255u, u = S.mnode[mi];
          my = key >> 8;
          const uint32_t k = u / NS;
          uint32_t lo = 0, cnt = 0;
          if (k < L) span_summary(rhs, u - k * NS, labels[k], lo, cnt);
          const size_t nb = (size_t)(k + 1) * NS;
          S.mlo[mi] = lo;
          S.mcnt[mi] = cnt;
          S.mnb[mi] = (uint32_t)nb;
          {
            for (uint32_t c0 = 0; c0 < cnt; c0 += kLlKB) {
              uint32_t x[kLlKB];
              bool t[kLlKB];
#pragma unroll
              for (int i = 0; i < kLlKB; ++i) {
                const ArcRec r = rhs.rec[lo + c0 + i];
                x[i] = (uint32_t)(nb + r.next);
                t[i] = c0 + i < cnt && okey(w_times(dminw, r.weight)) == dmin;
              }
              unsigned long long dx[kLlKB];
              uint32_t lx[kLlKB], fx[kLlKB];
#pragma unroll
              for (int i = 0; i < kLlKB; ++i) {
                dx[i] = t[i] ? rd_u64(&dk[x[i]]) : 0ull;
                lx[i] = t[i] ? rd_u32(&lidf[x[i]]) : ~0u;
                fx[i] = t[i] ? rd_u32(&flg[x[i]]) : 0u;
              }
#pragma unroll
              for (int i = 0; i < kLlKB; ++i)
                if (t[i] && dx[i] == dmin && lx[i] < kLlPend &&
                    (fx[i] & (kLzActive | kLzPopped)) == 0)
                  j = lx[i] < j ? lx[i] : j;
            }
          }
        }
        uint32_t ex = wave_excl_min_u32(j, lane);
        ex = carry < ex ? carry : ex;
        const unsigned long long vb = __ballot(pos < M && my > ex);
        if (vb) {
          kcut = b + (uint32_t)__builtin_ctzll(vb);
          break;
        }
        const uint32_t jm = wave_min_u32(j);
        carry = jm < carry ? jm : carry;
      }
      kcut = __builtin_amdgcn_readfirstlane(kcut);
      // (4) pop the batch: popped flags first, then touches and activations (-> B)
      for (uint32_t pos = lane; pos < kcut; pos += 64)
        flg[S.mnode[S.keys[pos] & 255u]] = kLzPopped;
      if (lane == 0) S.count = 0;
      global_sync();
      wave_lds_sync();
      const uint32_t room = ws.acap - nsv;
      for (uint32_t pos = lane; pos < kcut; pos += 64) {
        const uint32_t mi = S.keys[pos] & 255u;
        const uint32_t lo = S.mlo[mi], cnt = S.mcnt[mi];
        const size_t nb = S.mnb[mi];
        for (uint32_t c0 = 0; c0 < cnt; c0 += kLlKB) {
          uint32_t x[kLlKB];
          unsigned long long v[kLlKB];
#pragma unroll
          for (int i = 0; i < kLlKB; ++i) {
            const ArcRec r = rhs.rec[lo + c0 + i];
            x[i] = (uint32_t)(nb + r.next);
            v[i] = okey(w_times(dminw, r.weight));
          }
          unsigned long long dx[kLlKB];
          uint32_t fx[kLlKB];
#pragma unroll
          for (int i = 0; i < kLlKB; ++i) {
            if (c0 + i < cnt)  // no-op once x has a lid
              atomicMin(&lidf[x[i]], kLlPend | (pos << 12) | (c0 + i));
            dx[i] = c0 + i < cnt ? rd_u64(&dk[x[i]]) : ~0ull;
            fx[i] = c0 + i < cnt ? rd_u32(&flg[x[i]]) : kLzPopped;
          }
          uint32_t old[kLlKB];
#pragma unroll
          for (int i = 0; i < kLlKB; ++i)
            old[i] = (v[i] == dx[i] && (fx[i] & kLzPopped) == 0)
                         ? atomicOr(&flg[x[i]], kLzActive)
                         : kLzActive;
#pragma unroll
          for (int i = 0; i < kLlKB; ++i) {
            if ((old[i] & (kLzActive | kLzPopped)) == 0) {
              const uint32_t q = atomicAdd(&S.count, 1u);
              if (q < room)
                B[nsv + q] = make_uint4(x[i], 0u, (uint32_t)dx[i], (uint32_t)(dx[i] >> 32));
            }
          }
        }
      }
      global_sync();
      wave_lds_sync();
      const uint32_t nadd = __builtin_amdgcn_readfirstlane(S.count);
      if (nadd + (M - kcut) > room) {
        fail = kPathOverflow;
        break;
      }
      // (5) fresh lids in (member, candidate) order
      uint32_t newc = 0;
      for (uint32_t b = 0; b < kcut; b += 64) {
        const uint32_t pos = b + lane;
        unsigned long long mask = 0;
        uint32_t lo = 0, cnt = 0;
        size_t nb = 0;
        if (pos < kcut) {
          const uint32_t mi = S.keys[pos] & 255u;
          lo = S.mlo[mi];
          cnt = S.mcnt[mi];
          nb = S.mnb[mi];
          {
            for (uint32_t c0 = 0; c0 < cnt; c0 += kLlKB) {  // cnt <= kLlSpanMax (host check)
              uint32_t lx[kLlKB];
#pragma unroll
              for (int i = 0; i < kLlKB; ++i)
                lx[i] = c0 + i < cnt ? rd_u32(&lidf[nb + rhs.rec[lo + c0 + i].next]) : 0u;
#pragma unroll
              for (int i = 0; i < kLlKB; ++i)
                if (lx[i] == (kLlPend | (pos << 12) | (c0 + i))) mask |= 1ull << (c0 + i);
            }
          }
        }
        uint32_t tot;
        uint32_t rank = nxt + newc + wave_excl_scan_small<7>((uint32_t)__popcll(mask), tot);
        while (mask) {
          const uint32_t c = (uint32_t)__builtin_ctzll(mask);
          mask &= mask - 1;
          const uint32_t x = (uint32_t)(nb + rhs.rec[lo + c].next);
          lidf[x] = rank;
          inv[rank] = x;
          ++rank;
        }
        newc += tot;
      }
      nxt += newc;
      popped += kcut;
      global_sync();
      // (6) the activations' lids (fresh ones were just assigned); unpopped members
      for (uint32_t q = lane; q < nadd; q += 64) B[nsv + q].y = rd_u32(&lidf[B[nsv + q].x]);
      for (uint32_t pos = kcut + lane; pos < M; pos += 64) {
        const uint32_t mi = S.keys[pos] & 255u;
        B[nsv + nadd + (pos - kcut)] =
            make_uint4(S.mnode[mi], S.mlid[mi], (uint32_t)dmin, (uint32_t)(dmin >> 32));
      }
      na = nsv + nadd + (M - kcut);
      global_sync();
      wave_lds_sync();
      uint4* t = A;
      A = B;
      B = t;
      if (__builtin_amdgcn_s_memrealtime() > deadline || popped > n) fail = kPathInternal;
      fail = __builtin_amdgcn_readfirstlane(fail);
    }
    if (fail == kPathOk && (popped != n || nxt != n)) fail = kPathInternal;

    prof_mark(prof, 1, &tp);
    {
      uint32_t r32 = (uint32_t)relax;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) r32 += __shfl_xor(r32, o, 64);
      relax = r32;
    }
    // ---- back-pointers (lexmin (lid(source), ol, candidate): il is the layer's label) ----
    if (fail == kPathOk) {
      for (uint32_t k = 0; k < L; ++k) {
        const uint32_t label = __builtin_amdgcn_readfirstlane(labels[k]);
        const uint32_t f0 = __builtin_amdgcn_readfirstlane(rd_u32(&loff[k]));
        const uint32_t f1 = __builtin_amdgcn_readfirstlane(rd_u32(&loff[k + 1]));
        const size_t nb = (size_t)(k + 1) * NS;
        for (uint32_t p = f0 + lane; p < f1; p += 64) {
          const uint32_t u = nodes[p];
          const double du = from_okey(rd_u64(&dk[u]));
          const unsigned long long lu = (unsigned long long)rd_u32(&lidf[u]) << 32;
          uint32_t lo, cnt;
          span_summary(rhs, u - k * NS, label, lo, cnt);
          if (cnt <= (uint32_t)kLlKB) {  // registers: records, target dists, tight mask
            ArcRec r[kLlKB];
            unsigned long long dx[kLlKB];
#pragma unroll
            for (int i = 0; i < kLlKB; ++i) r[i] = rhs.rec[lo + i];
#pragma unroll
            for (int i = 0; i < kLlKB; ++i) dx[i] = (uint32_t)i < cnt ? rd_u64(&dk[nb + r[i].next]) : 0ull;
            uint32_t tight = 0;
#pragma unroll
            for (int i = 0; i < kLlKB; ++i)
              if ((uint32_t)i < cnt && okey(w_times(du, r[i].weight)) == dx[i]) tight |= 1u << i;
#pragma unroll
            for (int i = 0; i < kLlKB; ++i) {
              if (!(tight & (1u << i))) continue;
              bool win = true;  // another tight arc into the same target, smaller (ol, index)?
#pragma unroll
              for (int c = 0; c < kLlKB; ++c)
                if (c != i && (tight & (1u << c)) && r[c].next == r[i].next &&
                    (r[c].olabel < r[i].olabel || (r[c].olabel == r[i].olabel && c < i)))
                  win = false;
              if (win) atomicMin(&back[nb + r[i].next], lu | (uint32_t)i);
            }
            continue;
          }
          for (uint32_t c = 0; c < cnt; ++c) {
            const ArcRec r = rhs.rec[lo + c];
            const uint32_t x = (uint32_t)(nb + r.next);
            const unsigned long long dx = rd_u64(&dk[x]);
            if (okey(w_times(du, r.weight)) != dx) continue;
            bool win = true;
            for (uint32_t c2 = 0; c2 < cnt && win; ++c2) {
              if (c2 == c) continue;
              const ArcRec r2 = rhs.rec[lo + c2];
              if (r2.next != r.next || okey(w_times(du, r2.weight)) != dx) continue;
              if (r2.olabel < r.olabel || (r2.olabel == r.olabel && c2 < c)) win = false;
            }
            if (win) atomicMin(&back[x], lu | c);
          }
        }
      }
      global_sync();
      // best final: layer L, lexmin (dist + fw2, lid) -- the lhs final is One
      const uint32_t f0 = __builtin_amdgcn_readfirstlane(rd_u32(&loff[L]));
      const uint32_t f1 = __builtin_amdgcn_readfirstlane(rd_u32(&loff[L + 1]));
      unsigned long long bk = ~0ull;
      uint32_t bl = ~0u, bn = 0;
      for (uint32_t p = f0 + lane; p < f1; p += 64) {
        const uint32_t u = nodes[p];
        const double fw = rhs.final_w[u - L * NS];
        if (w_is_zero(fw)) continue;
        const unsigned long long t = okey(w_times(from_okey(rd_u64(&dk[u])), fw));
        const uint32_t l = rd_u32(&lidf[u]);
        if (t < bk || (t == bk && l < bl)) {
          bk = t;
          bl = l;
          bn = u;
        }
      }
      const unsigned long long best = wave_min_u64(bk);
      const uint32_t bestl = wave_min_u32(bk == best ? bl : ~0u);
      if (best == ~0ull) {
        if (lane == 0) write_status(out, si, kPathEmpty, n, (uint32_t)relax);
      } else {
        const unsigned long long own = __ballot(bk == best && bl == bestl);
        const uint32_t bnode = __shfl(bn, (int)__builtin_ctzll(own), 64);
        if (lane == 0) {
          // the path has exactly L arcs: each back-pointer steps back one layer, and
          // layer 0 holds only the start (compose-shortest-path.zig:372-380)
          const unsigned long long o = reserve_path(out, si, L);
          if (o + L > out.arc_cap) {
            write_status(out, si, kPathOutputFull, n, (uint32_t)relax);
          } else {
            uint32_t x = bnode;
            int32_t st = kPathOk;
            for (uint32_t k = L; k > 0; --k) {
              const unsigned long long bp = rd_u64(&back[x]);
              if (bp == ~0ull) {
                st = kPathInternal;  // every popped tuple but the start has a tight in-arc
                break;
              }
              const uint32_t src = inv[(uint32_t)(bp >> 32)], c = (uint32_t)bp;
              const uint32_t lab = labels[k - 1];
              uint32_t lo, cnt;
              span_summary(rhs, src - (k - 1) * NS, lab, lo, cnt);
              const ArcRec r = rhs.rec[lo + c];
              out.out_il[o + k - 1] = lab;
              out.out_ol[o + k - 1] = r.olabel;
              out.out_w[o + k - 1] = w_times(w_one(), r.weight);
              x = src;
            }
            if (st == kPathOk && x != start) st = kPathInternal;
            if (st != kPathOk) {
              write_status(out, si, st, n, (uint32_t)relax);
            } else {
              out.status[si] = kPathOk;
              out.path_len[si] = L;
              out.path_off[si] = o;
              out.final_w[si] = w_times(w_one(), rhs.final_w[bnode - L * NS]);
              if (out.work) {
                out.work[2 * si] = n;
                out.work[2 * si + 1] = (uint32_t)relax;
              }
            }
          }
        }
      }
    } else {
      if (lane == 0) write_status(out, si, fail, n, (uint32_t)relax);
    }
    // ---- reset every tuple this string touched ----
    global_sync();
    prof_mark(prof, 2, &tp);
    for (uint32_t p = lane; p < n; p += 64) {
      const uint32_t x = nodes[p];
      dk[x] = ~0ull;
      back[x] = ~0ull;
      lidf[x] = ~0u;
      flg[x] = 0u;
    }
    global_sync();
    prof_mark(prof, 3, &tp);
    if (guard > in.num_strings) break;  // cannot happen: one item per iteration
  }
}

}  // namespace fstamd
