// device_engine.hpp -- device-resident frozen FSTs and the batch engines.
//
// Engines:
//   eager-layered : FST_SEM_EAGER on lattices that are layered by input position
//                   (rhs without epsilon input arcs, inputs without label 0).
//                   One workgroup per string, per-layer LDS hash tables; ids,
//                   distances and back-pointers reproduce compose.zig's BFS ids and
//                   shortest-path.zig's tie rules.
//   lazy-wave     : FST_SEM_LAZY, exact replay of composeShortestPath's Dijkstra
//                   (one wavefront per string, workspace in HBM).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <new>
#include <vector>

#include "fst_core.hpp"

namespace fstamd {

class FrozenFst;

// RhsView::sspan[s].z when the state's arcs carry more than one ilabel / no arcs.
constexpr uint32_t kSpanMixed = 0xFFFFFFFEu;
constexpr uint32_t kSpanNone = 0xFFFFFFFFu;
// The device arc mirror (RhsView::rec) has kRecPad zeroed records past num_arcs, so a
// kernel may read rec[lo + j] for any lo <= num_arcs and j < kRecPad unconditionally.
constexpr uint32_t kRecPad = 16;
// Input label no rhs arc carries: a pipeline string that failed an earlier stage.
constexpr uint32_t kDeadLabel = 0xFFFFFFFFu;

// Read-only view of a device-resident rhs (the kernels' only rhs interface).
struct RhsView {
  const uint2* span;        // [num_states] (arc_offset, num_arcs)
  const double* final_w;    // [num_states]
  const uint32_t* il;       // [num_arcs] sorted ilabels per state span
  const ArcRec* rec;        // [num_arcs] {nextstate, olabel, weight}
  const uint4* sspan;       // [num_states] {arc_offset, num_arcs, ilabel shared by all
                            //  arcs of the state | kSpanMixed | kSpanNone, leading epsilon
                            //  arcs of a kSpanMixed state (ilabel 0 sorts first) else 0}
  uint32_t num_states;
  uint32_t num_arcs;
  uint32_t start;
  uint32_t max_span;        // largest per-state arc count
  uint32_t jump_back;       // max (s - t) over arcs s -> t (0 if none goes backwards)
  uint32_t jump_fwd;        // max (t - s) over arcs s -> t: a layer's targets lie within
                            // [min state - jump_back, max state + jump_fwd]
  // [num_states] for states with several ilabels: {first ilabel a, last ilabel z, arcs
  // carrying a, 1 when every other arc carries z}: a two-label state (an epsilon run then
  // one label, the epsilon-dense rhs) answers arcsByIlabel without a search
  const uint4* sspan2;
};

// Reverse arc mirror for the pull tier (kernels/eager_pull.hpp): the in-arcs of every rhs
// state t, grouped by ilabel, each group in padded blocks of `kp` records.  Record m of a
// block: 8 * the source state (its LDS cell offset before the window shift), y = (j << 17)
// | (m << 13) with j = the arc's position in its source's run of equal ilabels (the
// candidate order of compose.zig:93-121) | kRevPos when the weight is > 0, and the weight.
// Padding records have src = 0xFFFFFFF8.  Block 0 is all padding (the null block).
// y's flag of a positive-weight arc: bit 12, below m; the pull keys OR y with the cell's
// byte offset (< 4096), so the flag never decides a key comparison (keys of two in-arcs
// always differ in rank, j or m) and is masked off with the offset (& 0xFFF)
constexpr uint32_t kRevPos = 0x1000u;
struct RevRec {
  uint32_t src;
  uint32_t y;
  double weight;
};
static_assert(sizeof(RevRec) == 16, "RevRec is one 16-byte load");
struct RevView {
  const uint4* rspan;     // [num_states + kPullW] one group: {first record, nblocks, ilabel,
                          // 0}; several: {first gtab entry, groups, kSpanMixed, 0}; none (and
                          // the padding past the last state): {0, 0, kSpanNone, 0}
  const uint4* gtab;      // groups of multi-label states {ilabel, first record, nblocks, 0}
  const RevRec* rrec;     // [nblocks * kp]
  const uint32_t* rolab;  // [nblocks * kp] olabel of each record (backtrace only)
  uint32_t kp;            // records per block
  uint32_t gsearch;       // binary-search steps over the longest gtab run (0: no gtab)
  uint32_t direct;        // 1: block 0 of state t at record t * kp (every state has at most
                          // one in-label group); rspan.x = the record of its block 1
  // [nblocks * kp] the same records with an f32 weight and the olabel: {src, y, f32 bits of
  // the weight, olabel}; only when every arc weight is an integer in [0, 2^24) (exact in
  // f32; DeviceFst::int_wmax), else null
  const uint4* rrec32;
  // [nblocks * kp] the records in 8 B: {src, y | weight}, only when every arc weight is an
  // integer in [0, kRec8WMax] (it sits in y's low 3 bits, below the byte offset the keys OR
  // in), else null
  const uint2* rrec8;
  // direct layout: rspan split for the row loads, ilabel | min(nblocks, 255) << 24 per
  // state (4 B; labels below 2^24) and {the record of its block 1, nblocks} (read only for
  // states with more than one block)
  const uint32_t* rlab;
  const uint2* rxrec;
  uint32_t nrec;  // records (nblocks * kp)
  // [nblocks * kp] tier P's 4-B records (eager_pull.hip: the source as 8 * (target - source)
  // + rbias8 in the high half, the key bits and weight in the low half), else null
  const uint32_t* rrec4;
  uint32_t rbias8;
  // 2^-k: the compact records (rrec32 / rrec8 / rrec4) hold every weight times 2^k, the
  // smallest power of two that makes them all integers (DeviceFst::int_wmax); the kernels
  // multiply back what they output (exact).  1 for integer weights.  (The view's layout
  // steers tier P's register allocation: one more 8-B field here cost it 3 %, so the weight
  // table below has no pointer of its own.)
  double winv;
  // (weights no such scale makes integers, DeviceFst::widx: rrec4's low byte indexes a
  // table of the rhs's distinct arc weights stored after the records, rv_weight_table)
};
constexpr uint32_t kPullWt = 64;  // (a power of two: the kernels mask the index)
// rhs with 65..256 distinct weights: tier P's RK 5 (the same records, a 256-entry LDS
// table, 4 waves per SIMD instead of 5); the global copy always holds kPullWtMax entries
constexpr uint32_t kPullWtMax = 256;
// the weight table of an rhs with DeviceFst::widx: kPullWtMax doubles right after the
// rrec4 records (their count rounded up to 8-B alignment)
__host__ __device__ inline const double* rv_weight_table(const RevView& rv) {
  return reinterpret_cast<const double*>(rv.rrec4 + ((rv.nrec + 1u) & ~1u));
}
constexpr double kRec8WMax = 7.0;

struct DeviceFst {
  int dev = 0;
  uint8_t* blob = nullptr;  // the frozen blob itself, byte-identical to the host copy
  size_t blob_size = 0;
  uint2* span = nullptr;
  double* final_w = nullptr;
  uint32_t* il = nullptr;
  ArcRec* rec = nullptr;
  uint4* sspan = nullptr;
  RhsView view{};
  bool has_eps = false;
  bool nonneg = true;        // every arc and final weight >= +0
  bool nan = false;          // some arc or final weight is NaN
  bool finite = true;        // every arc weight finite
  uint8_t weight_type = 0;
  // pull tier (kernels/eager_pull.hpp): reverse mirror, built when the rhs qualifies
  // (no input epsilon, weights >= +0, every same-ilabel run of a state <= 8 arcs)
  bool pull_ok = false;
  // lazy pull tier (kernels/lazy_pull.hpp) too: for arcs of one source into one target
  // within a same-ilabel run, candidate order = olabel order (relax's (id, il, ol) rule
  // then reduces to (id, candidate))
  bool lazy_pull_ok = false;
  double int_wmax = -1.0;    // largest arc weight times RevView::winv^-1 when every scaled
                             // weight is an integer >= 0 below 2^24, else -1
  bool widx = false;         // rrec4 holds weight-table indices (RK 4 / 5; rv_weight_table)
  uint32_t wt_n = 0;         // distinct arc weights in that table (<= kPullWtMax)
  // the direct layout with every in-arc group within 255 / kp blocks: a back record can be
  // one byte, the in-arc's position x * kp + m in its target's group (the chases re-derive
  // the record from the target state: tier P with rrec4, the lazy pull with any records)
  bool byte_back = false;
  // Routing hints learnt from earlier batches on this rhs: a small-lattice (LDS) tier that
  // handed on nearly every string is skipped next time (config 3's lattices never fit).
  mutable std::atomic<int> skip_tiny_lazy{0}, skip_tiny_eager{0};
  // ... and one whose 128-tuple LDS size handed on over a third of a batch starts at 256
  mutable std::atomic<int> tiny_lazy_256{0}, tiny_eager_256{0};
  // ... counted over small batches too (coalesced single calls: batches of a few strings
  // never reach the per-batch thresholds): strings the 128-tuple LDS replay saw / handed on
  mutable std::atomic<uint64_t> tiny_lazy_seen{0}, tiny_lazy_over{0};
  RevView rev{};
  void* rev_bufs[9] = {};
  // band replay (kernels/lazy_band.hpp): the arcs at a fixed stride of 2^band_sh slots per
  // state (device numbering), built when the rhs takes the band replay (arcs forward, input
  // epsilon, <= 64 arcs per state) and the table stays small; padding slots: ilabel
  // 0xFFFFFFFF, a zero record
  uint32_t* band_il = nullptr;
  ArcRec* band_rec = nullptr;
  uint32_t band_sh = 0;
  // The device's state numbering (old id -> new id; empty = the blob's own ids): a
  // breadth-first renumbering of an rhs with scattered ids (device_engine.hip
  // bfs_renumbering).  Every device view (RhsView, RevView) uses it; results do not.
  std::vector<uint32_t> perm;

  static DeviceFst* create(const FrozenFst& f, int dev);
  // Blob already in device memory on `dev` (e.g. after an RCCL broadcast).
  static DeviceFst* adopt(const void* d_blob, const FrozenFst& host_view, int dev);
  static void destroy(DeviceFst* d);
};

// Device pointers of one batch's outputs (mirrors FstDeviceBatch in fst_batch.h).
struct BatchOutDev {
  int32_t* status;
  uint32_t* path_len;
  uint64_t* path_off;
  double* final_w;
  uint32_t* out_il;
  uint32_t* out_ol;
  double* out_w;
  uint64_t arc_cap;
  unsigned long long* cursor;
  uint32_t* work;
  // The host batch's streamed mode (c_api.cpp run_streamed; rhs without input epsilons, so
  // every path has exactly L arcs):
  //   slots: string si's path sits at arena slot slots[si] (the batch's own label offsets:
  //     no cursor, no compaction);
  //   host_ol / host_w (pull tiers only): each finished path's olabels and weights are
  //     also copied into these host-mapped result arrays (whole lines per store), and the
  //     chase skips the ilabels (the host stages them: on an OK path il[k] = label k).
  const uint64_t* slots = nullptr;
  uint32_t* host_ol = nullptr;
  double* host_w = nullptr;
  // (host side, not read by kernels) when set, run_chain copies the statuses right after
  // the first tier here: which strings the pull tier finished (and copied out) itself
  int32_t* first_status = nullptr;
};

// Chain inputs (batch API) or one general lhs FST (single-call C ABI).
struct ChainInput {
  const uint32_t* labels;
  const uint64_t* offsets;
  uint32_t num_strings;
  uint32_t max_len;
};
struct GraphInput {       // CSR of a MutableFst lhs, arcs in insertion order
  const uint32_t* state_off;   // [ns + 1]
  const uint32_t* arc_il;
  const uint32_t* arc_ol;
  const double* arc_w;
  const uint32_t* arc_next;
  const double* final_w;   // [ns]
  uint32_t num_states;
  uint32_t start;
  uint32_t max_outdeg;     // largest lhs out-degree (sizes the per-pop table)
  uint32_t ncap;           // product-tuple capacity for this run (power of two)
  uint32_t eps_out;        // 1: some lhs arc has output epsilon (filter-2 tuples exist)
};

// Lattice of one fst_compose_frozen call, downloaded from the device (CSR by source id).
// Pooled pinned host memory (c_api.cpp): D2H / H2D of it is one DMA, without the
// runtime's staging copies.
void* pin_host_alloc(size_t bytes);
void pin_host_release(void* p);
// Frees the device block pool's cached blocks of `dev` (c_api.cpp), so that a free-HBM query
// sees them as free.
void device_pool_release(int dev);
template <class T>
struct PinnedAllocator {
  using value_type = T;
  PinnedAllocator() = default;
  template <class U>
  PinnedAllocator(const PinnedAllocator<U>&) {}
  T* allocate(size_t n) {
    void* p = pin_host_alloc(n * sizeof(T));
    if (!p) throw std::bad_alloc();
    return (T*)p;
  }
  void deallocate(T* p, size_t) { pin_host_release(p); }
  template <class U>
  bool operator==(const PinnedAllocator<U>&) const { return true; }
  template <class U>
  bool operator!=(const PinnedAllocator<U>&) const { return false; }
};
template <class T>
using PinnedVec = std::vector<T, PinnedAllocator<T>>;

struct HostLattice {
  int32_t status = 0;  // PathStatus of the compose (kPathOk or kPathOverflow/kPathInternal)
  uint32_t n_nodes = 0, n_arcs = 0;
  PinnedVec<uint32_t> aoff, anext, ail, aol;  // downloaded from the device (config 1: 10 M arcs)
  PinnedVec<double> aw, nfin;
};

struct LaunchStats {
  double kernel_ms = 0;
  uint32_t launches = 0;
  uint32_t engine = 0;
  uint32_t grid = 0;
  // set by the caller: run_chain records its events but does not wait for them; the caller
  // synchronises the stream itself and then calls DeviceEngine::finish_deferred
  bool defer = false;
};

// ---- pull tier (eager_pull.hip, kernels/eager_pull.hpp) ----
struct EagerLaunch;
// Window rows of the pull tier: W = 64 * kPullRows target states per layer.
constexpr int kPullRows = 5;
constexpr uint32_t kPullW = 64 * kPullRows;
// Builds d->rev from the host copy when the rhs qualifies (sets d->pull_ok); false only
// on a device allocation failure.
bool build_reverse_mirror(DeviceFst* d, const FrozenFst& f);
void free_reverse_mirror(DeviceFst* d);
// Resident waves per CU of the pull kernel for this rhs.
int pull_waves_per_cu(const DeviceFst& rhs, uint32_t max_len);
// f32 cells for the pull tiers: every distance of a string of <= max_len labels is an
// integer below 2^24 (exact in f32)
bool pull_f32(const DeviceFst& rhs, uint32_t max_len);
hipError_t launch_eager_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n_best,
                             unsigned int* next_item, const EagerLaunch& lp,
                             const BatchOutDev& out, uint32_t grid, hipStream_t stream);
// Lazy pull tier (eager_pull.hip, kernels/lazy_pull.hpp): resident waves per CU, launch.
int lazy_pull_waves_per_cu(const DeviceFst& rhs, uint32_t max_len);
bool lazy_pull_f32(const DeviceFst& rhs, uint32_t max_len);
hipError_t launch_lazy_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n_best,
                            unsigned int* next_item, const EagerLaunch& lp,
                            const BatchOutDev& out, uint32_t grid, hipStream_t stream);

// Per-device engine state: persistent workspaces (grown on demand), its own non-blocking
// HIP stream and events.  A device has a small pool of engines (FSTAMD_ENGINES, default
// 4): concurrent C-ABI calls each lease one, so they run side by side on separate streams
// and synchronise only their own stream (src/c-api.zig:776-787 runs compute outside its
// lock; include/fst.h:11-26).
class DeviceEngine {
 public:
  // Exclusive use of one engine of `dev` for the lifetime of the lease.  use(s) binds the
  // stream the call's work goes on (the engine's own stream for synchronous entries, the
  // caller's for the async device entries): a stream other than the previous user's first
  // waits for that user's work (an event), and the lease records the event when it ends,
  // so an engine's workspaces are never reused while earlier work on them still runs.
  class Lease {
   public:
    Lease() = default;
    Lease(Lease&& o) noexcept : e_(o.e_), s_(o.s_), used_(o.used_) { o.e_ = nullptr; }
    Lease& operator=(Lease&& o) noexcept {
      if (this != &o) {
        release();
        e_ = o.e_;
        s_ = o.s_;
        used_ = o.used_;
        o.e_ = nullptr;
      }
      return *this;
    }
    ~Lease() { release(); }
    DeviceEngine* operator->() const { return e_; }
    DeviceEngine& operator*() const { return *e_; }
    explicit operator bool() const { return e_ != nullptr; }
    hipStream_t use(hipStream_t s);
    hipStream_t stream() { return used_ ? s_ : use(own_stream()); }

   private:
    friend class DeviceEngine;
    explicit Lease(DeviceEngine* e) : e_(e) {}
    void release();  // records the end event, returns the engine to its pool
    hipStream_t own_stream() const;
    DeviceEngine* e_ = nullptr;
    hipStream_t s_ = nullptr;
    bool used_ = false;
  };
  // Blocks while every engine of the device is leased.  An empty lease on failure.
  static Lease acquire(int dev);
  // The same without blocking: an empty lease when every engine of the device is leased.
  static Lease try_acquire(int dev);

  // All launches are asynchronous on `stream`; stats are filled when `stats` is
  // non-null (this synchronises on the stream's end event).
  hipError_t run_chain(const DeviceFst& rhs, const ChainInput& in, uint32_t n, int semantics,
                       const BatchOutDev& out, hipStream_t stream, LaunchStats* stats);
  // Whether run_chain's first tier for these semantics is a pull tier (eager tier P, the
  // lazy pull): only those wait for streamed labels (ChainInput::ready) and copy their
  // paths out (BatchOutDev::host_ol), so the streamed host batch needs it.  run_chain
  // refuses streamed inputs otherwise.
  static bool pull_first(const DeviceFst& rhs, int semantics);
  // kernel_ms of a deferred LaunchStats, once the caller has synchronised the stream
  hipError_t finish_deferred(LaunchStats* stats);
  // The streamed host batch's parts (c_api.cpp run_streamed): the pull tier alone on `in`
  // (pull_first must hold), no fills or copies on `stream` (a fill or copy is a blit that
  // waits for CU slots behind the other engine's persistent kernel) and no host
  // synchronisation; item_ctr zeroed and statuses filled by the caller.  The later tiers
  // then run once over the whole batch: run_chain with set_after_pull(true).
  hipError_t launch_pull_part(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                              int semantics, const BatchOutDev& out, hipStream_t stream,
                              unsigned int* item_ctr);
  // run_chain after launch_pull_part: the statuses are the pull tier's (no INTERNAL fill,
  // no pull launch); the later tiers take the strings it handed on.
  void set_after_pull(bool v) { after_pull_ = v; }
  // Out of HBM: the workspaces of the device's idle engines (kept per engine between calls)
  // go back to the device (all but `except`'s; hipFree outside the pool lock).
  static void trim_idle(int dev, const DeviceEngine* except = nullptr);
  hipError_t run_graph(const DeviceFst& rhs, const GraphInput& in, uint32_t n, int semantics,
                       const BatchOutDev& out, hipStream_t stream, LaunchStats* stats);
  // fst_compose_frozen: the whole lattice of one general lhs (kernels/eager_bfs.hpp), on
  // `stream` (synchronised: the lattice is downloaded).
  hipError_t compose_lattice(const DeviceFst& rhs, const GraphInput& lhs, HostLattice* lat,
                             LaunchStats* stats, hipStream_t stream);
  // Output tape of each path of a finished stage as the next stage's chain inputs
  // (printOutputString + compileString on device): next_labels = the path's non-epsilon
  // olabels.  A string whose status is not OK, or whose output has a label > 256, gets
  // the single input label kDeadLabel (no rhs arc matches it: the next stage reports
  // EMPTY) and its reason in proj_status.  Synchronises on `stream` (returns max_len).
  hipError_t project_output(const BatchOutDev& stage, uint32_t num, uint32_t* next_labels,
                            uint64_t* next_offsets, int32_t* proj_status, uint32_t* max_len,
                            hipStream_t stream);
  // The batch result in CSR order, on the device: status (with `fail`, when given, taking
  // precedence: a pipeline's first failing stage), path offsets over the OK strings'
  // paths, the arcs gathered from the arena, final weights (+inf unless OK).  il / ol / w
  // hold out_cap arcs (the arena's used arcs); no path is written past them.  Synchronises
  // on `stream`; *total = arcs (> out_cap only if an engine broke its arena invariant).
  hipError_t compact_paths(const BatchOutDev& s, uint32_t num, const int32_t* fail,
                           int32_t* status, uint64_t* offsets, uint32_t* il, uint32_t* ol,
                           double* w, double* fin, uint64_t out_cap, uint64_t* total,
                           hipStream_t stream);
  // fail[i] = st[i] where fail[i] is still OK (the first failing stage wins).
  hipError_t merge_status(int32_t* fail, const int32_t* st, uint32_t num, hipStream_t stream);
  // fst_shortest_path on an explicit graph; `g` holds the FST itself (CSR, arcs in
  // insertion order).  nonneg: every weight >= +0 (parallel fixpoint); otherwise the exact
  // one-lane replay of the reference's heap order (sp_replay_kernel).  No NaN weights.
  // Runs on `stream` and synchronises it.
  hipError_t shortest_path_graph(const GraphInput& g, uint32_t n, const BatchOutDev& out,
                                 LaunchStats* stats, hipStream_t stream, bool nonneg = true);

  int dev() const { return dev_; }
  int num_cus() const { return num_cus_; }

 private:
  explicit DeviceEngine(int dev);
  hipStream_t stream_ = nullptr;   // the engine's own stream (non-blocking)
  bool after_pull_ = false;        // run_chain: the pull tier already ran (set_after_pull)
  void take_scratch(std::vector<void*>* out);  // an idle engine's workspaces, to be freed
  hipEvent_t done_ = nullptr;      // recorded when a lease ends (on the stream it used)
  hipStream_t done_stream_ = nullptr;
  bool done_valid_ = false;
  // General engine (kernels/eager_bfs.hpp) over the strings of `in` whose status is
  // UNSUPPORTED or OVERFLOW after the layered tiers (all strings when `all`); eager
  // shortestPath or, with `lazy`, composeShortestPath semantics (finite weights >= 0).
  // Grows its per-string workspace in tiers.  Synchronises on `stream` to size the tiers.
  hipError_t run_bfs_chain(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                           const BatchOutDev& out, hipStream_t stream, bool all,
                           bool lazy = false, bool replay = false);
  // composeShortestPath on layered lattices (kernels/lazy_layered.hpp); strings it does
  // not take end UNSUPPORTED / OVERFLOW for run_bfs_chain.
  hipError_t run_lazy_layered(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                              const BatchOutDev& out, hipStream_t stream,
                              const uint32_t* items = nullptr,
                              const uint32_t* num_items_dev = nullptr);
  // composeShortestPath on layered lattices by the layer-local pull (kernels/lazy_pull.hpp);
  // the strings it hands on (OVERFLOW) are listed in *list, their count at *count_dev.
  hipError_t run_lazy_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                           const BatchOutDev& out, hipStream_t stream, uint32_t** list,
                           uint32_t** count_dev, bool launch = true);
  // composeShortestPath as a dense-indexed exact replay (kernels/lazy_dense.hpp), for rhs
  // with input epsilons; strings it does not take end UNSUPPORTED / OVERFLOW for
  // run_bfs_chain.  *ran = false: it took none (the lattice exceeds its dense index).
  // subset_dev (device, subset_n entries): only those strings (nullptr: all).
  hipError_t run_lazy_dense(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                            const BatchOutDev& out, hipStream_t stream, bool* ran,
                            const uint32_t* subset_dev = nullptr, uint32_t subset_n = 0);
  // composeShortestPath with the wave's tables in LDS (kernels/lazy_tiny.hpp, tier t holds
  // 64 << t tuples: 1 = 128 ... 4 = 1024) over a device list of strings (nullptr: all);
  // strings whose lattice outgrows it end OVERFLOW.
  // The band replay (kernels/lazy_band.hpp); *ran = false when the rhs or the batch is not
  // its (arcs going backwards, lengths > 4095); strings it hands on end OVERFLOW.  capped:
  // back pointers only for the first 2 x window states past the start (the early exit's
  // footprint), strings reaching beyond end OVERFLOW.
  hipError_t run_lazy_band(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                           const BatchOutDev& out, hipStream_t stream, bool* ran,
                           const uint32_t* subset_dev = nullptr, uint32_t subset_n = 0,
                           bool capped = false);
  hipError_t launch_lazy_hashed(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                const BatchOutDev& out, hipStream_t stream, uint64_t want_nodes,
                                const uint32_t* items, uint32_t num_items, unsigned int* ctr,
                                uint32_t* grid_out);
  hipError_t run_lazy_tiny(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                           const BatchOutDev& out, hipStream_t stream, int tier,
                           const uint32_t* items, uint32_t num_items, unsigned int* ctr,
                           uint32_t* grid_out);
  void* scratch(size_t idx, size_t bytes);
  int dev_;
  int num_cus_ = 0;
  std::vector<void*> bufs_;
  std::vector<size_t> sizes_;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  size_t lazy_hash_bytes_ = 0;   // hash table stamps are valid for this allocation
  uint32_t lazy_stamp_ = 0;      // next stamp base (bumped per launch)
  void* ll_clean_ = nullptr;     // lazy-layered dense arrays initialised for this allocation
  size_t ll_clean_bytes_ = 0;
  void* ld_clean_ = nullptr;     // lazy-dense rec / leaf arrays initialised for these allocations
  size_t ld_clean_bytes_ = 0;
  void* ld_leaf_ = nullptr;
  size_t ld_leaf_bytes_ = 0;
  void* lb_clean_ = nullptr;     // band-replay window initialised for this allocation
  size_t lb_clean_bytes_ = 0;
};

}  // namespace fstamd
