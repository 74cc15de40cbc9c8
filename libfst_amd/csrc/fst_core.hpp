// fst_core.hpp -- value types, weights and the frozen binary layout shared by
// host and device code of libfst_amd.
//
// Layout and semantics follow ontypehq/libfst:
//   Label/StateId/epsilon/no_state  src/arc.zig:4-13
//   Arc(W)                          src/arc.zig:17-63 (compareByIlabel :46-54)
//   TropicalWeight times/compare     src/weight.zig:5-65 (LogWeight :68-132: identical
//                                    times/compare/isZero; plus() is never used on
//                                    the compose / shortest-path path)
//   Header/StateEntry/PackedArc      src/fst.zig:12-47
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>

#if defined(__HIPCC__)
#define FST_HD __host__ __device__ __forceinline__
#else
#define FST_HD inline
#endif

namespace fstamd {

using Label = uint32_t;
using StateId = uint32_t;
constexpr Label kEpsilon = 0;
constexpr StateId kNoState = 0xFFFFFFFFu;

constexpr uint32_t kMagic = 0x46535421u;  // "FST!"
constexpr uint16_t kVersion = 1;
constexpr uint8_t kWeightTropical = 0;
constexpr uint8_t kWeightLog = 1;

struct Header {          // 24 bytes, little endian, 8-aligned blob start
  uint32_t magic;
  uint16_t version;
  uint8_t weight_type;
  uint8_t flags;
  uint32_t num_states;
  uint32_t num_arcs;
  uint32_t start_state;
  uint32_t pad;
};
struct StateEntry {      // 16 bytes
  uint32_t arc_offset;
  uint32_t num_arcs;
  double final_weight;
};
struct PackedArc {       // 24 bytes (extern struct: 4 trailing pad bytes)
  uint32_t ilabel;
  uint32_t olabel;
  double weight;
  uint32_t nextstate;
  uint32_t pad;
};
static_assert(sizeof(Header) == 24, "Header must be 24 bytes");
static_assert(sizeof(StateEntry) == 16, "StateEntry must be 16 bytes");
static_assert(sizeof(PackedArc) == 24, "PackedArc must be 24 bytes");

struct Arc {
  Label ilabel;
  Label olabel;
  double weight;
  StateId nextstate;
};

// ---- semiring (tropical; log shares times/compare/isZero on this path) ----
FST_HD double w_zero() { return __builtin_huge_val(); }
FST_HD double w_one() { return 0.0; }
FST_HD bool w_is_zero(double v) { return __builtin_isinf(v); }  // -inf counts as Zero too
FST_HD double w_times(double a, double b) {
  return (__builtin_isinf(a) || __builtin_isinf(b)) ? __builtin_huge_val() : a + b;
}

// Order-preserving u64 key of a non-negative, non-NaN double (the eager
// engines' contract): IEEE bits of +0..+inf are already ordered.
FST_HD uint64_t okey(double v) { return (uint64_t)__builtin_bit_cast(uint64_t, v); }
FST_HD double from_okey(uint64_t k) { return __builtin_bit_cast(double, k); }

// Arc.compareByIlabel, src/arc.zig:46-54
inline bool arc_less(const Arc& a, const Arc& b) {
  if (a.ilabel != b.ilabel) return a.ilabel < b.ilabel;
  if (a.olabel != b.olabel) return a.olabel < b.olabel;
  if (a.weight < b.weight) return true;
  if (a.weight > b.weight) return false;
  return a.nextstate < b.nextstate;
}

// Device SoA mirror record of one rhs arc: everything a relaxation needs in one
// 16-byte load (ilabels live in their own array for the span search).
struct alignas(16) ArcRec {
  uint32_t next;
  uint32_t olabel;
  double weight;
};

// Per-string status codes written by the batch engines (include/fst_batch.h).
enum PathStatus : int32_t {
  kPathOk = 0,           // a path (possibly zero arcs)
  kPathEmpty = 1,        // result FST has no states (no path / n == 0 / no start)
  kPathErrorN = 2,       // n not in {0,1}: the reference returns FST_INVALID_HANDLE
  kPathCycle = 3,        // back-pointer cycle: the reference would loop forever
  kPathOverflow = 4,     // engine capacity exceeded (host retries on a larger engine)
  kPathUnsupported = 5,  // input outside this engine's contract (host reroutes)
  kPathOutputFull = 6,   // output arc arena exhausted
  kPathInternal = 7,     // engine invariant violated (a bug); never silently wrong
};

}  // namespace fstamd
