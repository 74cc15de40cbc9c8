// device_engine.hip -- device copies of frozen FSTs and the batch engine launches.
#include "device_engine.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>

#include <hipcub/hipcub.hpp>

#include "host_fst.hpp"
#include "kernels/eager_bfs.hpp"
#include "kernels/eager_tiny.hpp"
#include "kernels/lazy_dense.hpp"
#include "kernels/lazy_band.hpp"
#include "kernels/lazy_layered.hpp"
#include "kernels/eager_layered.hpp"
#include "kernels/eager_wave.hpp"
#include "kernels/eager_window.hpp"
#include "kernels/lazy_wave.hpp"
#include "kernels/lazy_tiny.hpp"

#define HIP_TRY(x)                              \
  do {                                          \
    hipError_t e_ = (x);                        \
    if (e_ != hipSuccess) return e_;            \
  } while (0)

namespace fstamd {

// ---------------------------------------------------------------------------------
// Frozen FST on the device: the blob itself (byte-identical, the HBM-resident
// Fst(W) layout) plus an SoA mirror derived from it on the device.
// ---------------------------------------------------------------------------------

// perm (optional): the device's state numbering (old id -> new id, DeviceFst::perm).
// The band replay's strided arc table: slot i of state s (device numbering) holds the
// state's i-th arc, or padding past its last one.
__global__ void build_band_table_kernel(const uint2* span, const uint32_t* il, const ArcRec* rec,
                                        uint32_t ns, uint32_t sh, uint32_t* bil, ArcRec* brec) {
  const uint64_t total = (uint64_t)ns << sh;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t st = (uint32_t)(i >> sh), j = (uint32_t)(i & ((1u << sh) - 1));
    const uint2 sp = span[st];
    const bool v = j < sp.y;
    bil[i] = v ? il[sp.x + j] : 0xFFFFFFFFu;
    brec[i] = v ? rec[sp.x + j] : ArcRec{0u, 0u, 0.0};
  }
}

__global__ void build_mirror_kernel(const uint8_t* blob, uint32_t ns, uint32_t na,
                                    const uint32_t* perm, uint2* span, double* fin, uint32_t* il,
                                    ArcRec* rec, uint4* sspan, uint4* sspan2) {
  const StateEntry* se = reinterpret_cast<const StateEntry*>(blob + sizeof(Header));
  const PackedArc* pa =
      reinterpret_cast<const PackedArc*>(blob + sizeof(Header) + (size_t)ns * sizeof(StateEntry));
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
    const StateEntry e = se[i];
    const uint32_t ni = perm ? perm[i] : i;
    span[ni] = make_uint2(e.arc_offset, e.num_arcs);
    fin[ni] = e.final_weight;
    // arcs are sorted by ilabel (fst.zig:258-265): first == last <=> one shared ilabel
    uint32_t uniq = kSpanNone;
    if (e.num_arcs > 0) {
      const uint32_t a = pa[e.arc_offset].ilabel, z = pa[e.arc_offset + e.num_arcs - 1].ilabel;
      uniq = a == z ? a : kSpanMixed;
    }
    uint4 two = make_uint4(kSpanNone, kSpanNone, 0u, 0u);
    uint32_t neps = 0;  // mixed states: the leading epsilon run (ilabel 0 sorts first)
    if (uniq == kSpanMixed) {
      const uint32_t a = pa[e.arc_offset].ilabel, z = pa[e.arc_offset + e.num_arcs - 1].ilabel;
      uint32_t na_ = 1;
      while (na_ < e.num_arcs && pa[e.arc_offset + na_].ilabel == a) ++na_;
      two = make_uint4(a, z, na_, pa[e.arc_offset + na_].ilabel == z ? 1u : 0u);
      neps = a == 0u ? na_ : 0u;
    }
    sspan[ni] = make_uint4(e.arc_offset, e.num_arcs, uniq, neps);
    sspan2[ni] = two;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) {
    const PackedArc a = pa[i];
    il[i] = a.ilabel;
    ArcRec r;
    r.next = perm ? perm[a.nextstate] : a.nextstate;
    r.olabel = a.olabel;
    r.weight = a.weight;
    rec[i] = r;
  }
}

// Eager batch on an rhs no eager engine covers yet: per-string UNSUPPORTED
// (after the reference's empty / n checks, which need no search).
__global__ void mark_status_kernel(uint32_t num, uint32_t n_best, uint32_t rhs_start,
                                   BatchOutDev out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num) return;
  int32_t st = kPathUnsupported;
  if (rhs_start == kNoState || n_best == 0) st = kPathEmpty;
  else if (n_best != 1) st = kPathErrorN;
  out.status[i] = st;
  out.path_len[i] = 0;
  out.path_off[i] = 0;
  out.final_w[i] = w_zero();
  if (out.work) {
    out.work[2 * i] = 0;
    out.work[2 * i + 1] = 0;
  }
}

// Bandwidth reduction of the device's state numbering.  No kernel orders anything by rhs
// state id: candidates go in (lattice id, arc position) order, arcs keep their span order
// (sorted by the ORIGINAL nextstate, fst.zig:160-224), and outputs carry labels and
// weights only -- so renumbering the device copy changes no result, only locality.  A
// grammar whose ids are scattered (a WeText asset, or any rhs built without regard to
// numbering) gets breadth-first ids from the start state when that shrinks the widest
// arc jump at least 4x: the pull tiers' 320-state windows then hold its layers again
// (metric rhs with scattered ids: P / LP instead of the hash tiers).  FSTAMD_RENUMBER=0
// keeps the blob's ids, =1 forces BFS ids.
static std::vector<uint32_t> bfs_renumbering(const FrozenFst& f, uint32_t* jf_out,
                                             uint32_t* jb_out) {
  const uint32_t ns = f.num_states();
  const StateEntry* se = f.states();
  const PackedArc* pa = f.arcs();
  auto band = [&](const uint32_t* perm, uint32_t* jf, uint32_t* jb) {
    *jf = *jb = 0;
    for (uint32_t i = 0; i < ns; ++i) {
      const uint32_t pi = perm ? perm[i] : i;
      for (uint32_t a = se[i].arc_offset; a < se[i].arc_offset + se[i].num_arcs; ++a) {
        const uint32_t t = perm ? perm[pa[a].nextstate] : pa[a].nextstate;
        if (t >= pi) *jf = std::max(*jf, t - pi);
        else *jb = std::max(*jb, pi - t);
      }
    }
  };
  band(nullptr, jf_out, jb_out);
  const char* e = std::getenv("FSTAMD_RENUMBER");
  const int mode = e ? std::atoi(e) : -1;  // -1 auto, 0 off, 1 force
  const uint64_t id_band = (uint64_t)*jf_out + *jb_out;
  if (mode == 0 || ns < 2 || f.start() >= ns || (mode < 0 && id_band <= 64)) return {};
  std::vector<uint32_t> perm(ns, 0xFFFFFFFFu), queue;
  queue.reserve(ns);
  uint32_t next = 0;
  auto visit = [&](uint32_t s) {
    if (perm[s] == 0xFFFFFFFFu) {
      perm[s] = next++;
      queue.push_back(s);
    }
  };
  visit(f.start());
  for (size_t q = 0; q < queue.size(); ++q) {
    const uint32_t s = queue[q];
    for (uint32_t a = se[s].arc_offset; a < se[s].arc_offset + se[s].num_arcs; ++a)
      visit(pa[a].nextstate);
  }
  for (uint32_t s = 0; s < ns; ++s) visit(s);  // unreachable states last, in id order
  uint32_t jf = 0, jb = 0;
  band(perm.data(), &jf, &jb);
  if (mode < 0 && ((uint64_t)jf + jb) * 4 > id_band) return {};
  *jf_out = jf;
  *jb_out = jb;
  return perm;
}

static DeviceFst* finish_device(DeviceFst* d, const FrozenFst& f) {
  const Header& h = f.header();
  const uint32_t ns = h.num_states, na = h.num_arcs;
  uint32_t jf = 0, jb = 0;
  d->perm = bfs_renumbering(f, &jf, &jb);
  uint32_t* d_perm = nullptr;
  if (!d->perm.empty() &&
      (hipMalloc(&d_perm, ns * 4ull) != hipSuccess ||
       hipMemcpy(d_perm, d->perm.data(), ns * 4ull, hipMemcpyHostToDevice) != hipSuccess)) {
    if (d_perm) (void)hipFree(d_perm);
    DeviceFst::destroy(d);
    return nullptr;
  }
  bool ok = hipMalloc(&d->span, sizeof(uint2) * std::max<uint32_t>(ns, 1)) == hipSuccess &&
            hipMalloc(&d->final_w, sizeof(double) * std::max<uint32_t>(ns, 1)) == hipSuccess &&
            hipMalloc(&d->il, sizeof(uint32_t) * std::max<uint32_t>(na, 1)) == hipSuccess &&
            hipMalloc(&d->rec, sizeof(ArcRec) * ((size_t)na + kRecPad)) == hipSuccess &&
            hipMemset(d->rec + na, 0, sizeof(ArcRec) * kRecPad) == hipSuccess &&
            hipMalloc(&d->sspan, sizeof(uint4) * 2 * (size_t)std::max<uint32_t>(ns, 1)) ==
                hipSuccess;  // sspan, then sspan2
  if (!ok) {
    DeviceFst::destroy(d);
    return nullptr;
  }
  const uint32_t work = std::max(ns, na);
  const uint32_t blocks = std::min<uint32_t>((work + 255) / 256, 4096);
  if (work > 0) {
    build_mirror_kernel<<<std::max<uint32_t>(blocks, 1), 256>>>(d->blob, ns, na, d_perm, d->span,
                                                                d->final_w, d->il, d->rec,
                                                                d->sspan, d->sspan + ns);
  }
  const bool synced = hipStreamSynchronize(nullptr) == hipSuccess;  // the null stream only:
  if (d_perm) (void)hipFree(d_perm);          // other calls' engines run on their own streams
  if (!synced) {
    DeviceFst::destroy(d);
    return nullptr;
  }
  uint32_t max_span = 0;
  const StateEntry* se = f.states();
  for (uint32_t i = 0; i < ns; ++i) max_span = std::max(max_span, se[i].num_arcs);
  const uint32_t start = (d->perm.empty() || h.start_state >= ns) ? h.start_state
                                                                  : d->perm[h.start_state];
  d->view = RhsView{d->span, d->final_w, d->il,       d->rec,     d->sspan,
                    ns,      na,         start,        max_span,   jb, jf, d->sspan + ns};
  d->has_eps = f.has_epsilon_input();
  d->nonneg = f.weights_nonnegative();
  d->nan = f.has_nan_weight();
  d->finite = f.arc_weights_finite();
  d->weight_type = f.weight_type();
  // band replay's strided arc table (<= 1 GB; without it the band reads spans first)
  if (d->has_eps && jb == 0 && max_span > 0 && max_span <= 64 && ns > 0 &&
      !std::getenv("FSTAMD_NO_BAND_TABLE")) {
    uint32_t sh = 0;
    while ((1u << sh) < max_span) ++sh;
    const uint64_t slots = (uint64_t)ns << sh;
    if (slots * (4 + sizeof(ArcRec)) <= (1ull << 30)) {
      // (an optimisation only: without the HBM for it the band reads spans first)
      if (hipMalloc(&d->band_il, slots * 4) != hipSuccess ||
          hipMalloc(&d->band_rec, slots * sizeof(ArcRec)) != hipSuccess) {
        (void)hipGetLastError();  // clear the failed allocation's error
        if (d->band_il) (void)hipFree(d->band_il);
        if (d->band_rec) (void)hipFree(d->band_rec);
        d->band_il = nullptr;
        d->band_rec = nullptr;
      } else {
        d->band_sh = sh;
        const uint32_t bb = (uint32_t)std::min<uint64_t>((slots + 255) / 256, 8192);
        build_band_table_kernel<<<bb, 256>>>(d->span, d->il, d->rec, ns, sh, d->band_il,
                                             d->band_rec);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess) {
          DeviceFst::destroy(d);
          return nullptr;
        }
      }
    }
  }
  // pull tier (eager_pull.hip); false = device OOM.  Its uploads go to the null stream:
  // wait for them before engines on their own streams read the mirror
  if (!build_reverse_mirror(d, f) || hipStreamSynchronize(nullptr) != hipSuccess) {
    DeviceFst::destroy(d);
    return nullptr;
  }
  return d;
}

DeviceFst* DeviceFst::create(const FrozenFst& f, int dev) {
  if (hipSetDevice(dev) != hipSuccess) return nullptr;
  DeviceFst* d = new DeviceFst();
  d->dev = dev;
  d->blob_size = f.size();
  if (hipMalloc(&d->blob, d->blob_size) != hipSuccess ||
      hipMemcpy(d->blob, f.bytes(), d->blob_size, hipMemcpyHostToDevice) != hipSuccess) {
    destroy(d);
    return nullptr;
  }
  return finish_device(d, f);
}

DeviceFst* DeviceFst::adopt(const void* d_blob, const FrozenFst& f, int dev) {
  if (hipSetDevice(dev) != hipSuccess) return nullptr;
  DeviceFst* d = new DeviceFst();
  d->dev = dev;
  d->blob_size = f.size();
  if (hipMalloc(&d->blob, d->blob_size) != hipSuccess ||
      hipMemcpy(d->blob, d_blob, d->blob_size, hipMemcpyDeviceToDevice) != hipSuccess) {
    destroy(d);
    return nullptr;
  }
  return finish_device(d, f);
}

void DeviceFst::destroy(DeviceFst* d) {
  if (!d) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(d->dev);
  if (d->blob) (void)hipFree(d->blob);
  if (d->span) (void)hipFree(d->span);
  if (d->final_w) (void)hipFree(d->final_w);
  if (d->il) (void)hipFree(d->il);
  if (d->rec) (void)hipFree(d->rec);
  if (d->sspan) (void)hipFree(d->sspan);
  if (d->band_il) (void)hipFree(d->band_il);
  if (d->band_rec) (void)hipFree(d->band_rec);
  free_reverse_mirror(d);
  (void)hipSetDevice(cur);
  delete d;
}

// ---------------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------------

namespace {
// eager-layered geometry: 256 threads (4 waves) per string, <= 512 tuples per layer.
constexpr int kElWG = 256;
constexpr int kElFcap = 512;
constexpr int kElHcap = 1024;
constexpr int kElKmax = 8;  // candidates per tuple kept in registers across phases
// eager-wave geometry (tier 1): one wavefront per string, <= 320 tuples per layer
// (5 per lane), <= 8 same-label arcs per tuple, 512-slot LDS hash.
constexpr int kEwEmax = 5;
constexpr int kEwFcap = 64 * kEwEmax;
constexpr int kEwHcap = 512;
constexpr int kEwKmax = 5;
// eager-window geometry (tier A0): one wavefront per string, direct-mapped target window of
// kEwinW = 64 * kEwinRows states, <= 64 * kEwinEmax tuples in a layer that is expanded,
// <= kEwinKmax same-label arcs per tuple, kEwinWaves waves per SIMD.
constexpr int kEwinEmax = 4;
constexpr int kEwinRows = 5;
constexpr int kEwinW = 64 * kEwinRows;
constexpr int kEwinKmax = 5;
constexpr int kEwinWaves = 3;
static_assert((uint32_t)kEwinW == kPullW, "tiers P and A0 share the back slab geometry");

// Item counters and list counts, one 256-B block shared by the engines (word ranges):
// run_chain [0..6] and [14..15] (pull tier), run_lazy_pull [34..35], lazy replay retry
// tiers [6..13], run_bfs_chain [8..11] (never in the
// same call as the replay tiers), run_lazy_layered [32], run_lazy_dense [33].
constexpr size_t kCounterBytes = 256;

enum Scratch : size_t {
  kCounter = 0,
  kElBack,
  kLzHash,
  kLzNkey,
  kLzNdist,
  kLzNback,
  kLzNbw,
  kLzQd,
  kLzQid,
  kLzG,
  kItems,
  kDebug,
  kElSlab,
  kElBack2,
  kElBackB,
  kItems2,
  kBfsSlab,
  kBfsHdr,
  kBfsList,
  kBfsList2,
  kProjCount,
  kProjTemp,
  kLlDk,
  kLlBack,
  kLlLidf,
  kLlFlg,
  kLlNodes,
  kLlInv,
  kLlLoff,
  kLlAct,
  kElBackW,
  kItems3,
  kLdRec,
  kLdBarc,
  kLdIds,
  kLdLeaf,
  kLdFut,
  kLdItems,
  kLbWin,
  kLbBk,
  kLbIdr,
  kLbFut,
  kLbItems,
  kBfsHeap,
  kPullBack,
  kItems4,
  kLpBack,
  kItems5,
  kNumScratch
};

// Lazy-engine watchdog: 60 s of s_memrealtime (100 MHz) per wave, far beyond any
// legitimate string; it exists so that no bug can leave a wave resident forever.
constexpr unsigned long long kWatchdogTicks = 6000000000ull;

unsigned long long watchdog_ticks() {
  const char* e = std::getenv("FSTAMD_WATCHDOG_MS");  // test/debug override
  if (e && *e) return (unsigned long long)std::strtoull(e, nullptr, 10) * 100000ull;
  return kWatchdogTicks;
}

void dump_debug(const uint32_t* d_dbg, uint32_t grid, hipStream_t stream) {
  std::vector<uint32_t> h((size_t)grid * 8);
  if (hipStreamSynchronize(stream) != hipSuccess) return;
  if (hipMemcpy(h.data(), d_dbg, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return;
  for (uint32_t w = 0; w < grid; ++w)
    if (h[w * 8])
      std::fprintf(stderr,
                   "[fstamd lazy dbg] wave %u: watchdog at site %u pops=%u cb=%u C=%u qn=%u nn=%u\n",
                   w, h[w * 8], h[w * 8 + 1], h[w * 8 + 2], h[w * 8 + 3], h[w * 8 + 4],
                   h[w * 8 + 5]);
}

#ifdef FSTAMD_DEBUG_WAIT
// Debug builds: kernels record per-workgroup progress (FT) into fine-grained host memory,
// which the host can read while a kernel runs or after its queue aborted.
uint32_t* g_host_trace = nullptr;
constexpr size_t kTraceWords = 65536 * 4;

hipError_t debug_trace_arm() {
  if (!g_host_trace) {
    HIP_TRY(hipHostMalloc((void**)&g_host_trace, kTraceWords * 4, hipHostMallocCoherent));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_fst_trace), &g_host_trace, sizeof(g_host_trace)));
  }
  std::memset(g_host_trace, 0xEE, kTraceWords * 4);
  return hipSuccess;
}

// Waits up to FSTAMD_DEBUG_WAIT_S (default 20) seconds; on a fault or a timeout prints the
// progress of every workgroup and (timeout) exits the process, so a hang becomes a report.
hipError_t debug_wait(hipStream_t stream, uint32_t grid, const char* what) {
  const char* ws = std::getenv("FSTAMD_DEBUG_WAIT_S");
  const double limit = ws ? std::atof(ws) : 20.0;
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  bool timed_out = false;
  while ((e = hipStreamQuery(stream)) == hipErrorNotReady) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      timed_out = true;
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  std::fprintf(stderr, "[fstamd dbg] %s: %s\n", what,
               timed_out ? "TIMEOUT" : hipGetErrorString(e));
  if (timed_out || e != hipSuccess) {
    for (uint32_t b = 0; b < grid && b < 65536; ++b) {
      const uint32_t* w = g_host_trace + b * 4;
      if (w[0] != 0xEEEEEEEEu)
        std::fprintf(stderr, "[fstamd dbg]   wg %u item %u si %d k %u phase %u\n", b, w[0],
                     (int)w[1], w[2], w[3]);
    }
    std::fflush(stderr);
    if (timed_out) std::_Exit(3);
  }
  return e == hipErrorNotReady ? hipSuccess : e;
}
#endif

uint32_t next_pow2(uint64_t x) {
  uint32_t p = 1;
  while (p < x && p < 0x80000000u) p <<= 1;
  return p;
}
}  // namespace

namespace {
// The engines of one device: created on demand up to max_engines(), leased LIFO (a single
// caller keeps reusing the same warm engine).
struct EnginePool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::unique_ptr<DeviceEngine>> all;
  std::vector<DeviceEngine*> idle;
  std::mutex heavy;  // dense-replay plans sized from free HBM: query + allocate one at a time
};
EnginePool& engine_pool(int dev) {
  static std::mutex mu;
  static std::vector<std::unique_ptr<EnginePool>>* pools =
      new std::vector<std::unique_ptr<EnginePool>>();  // never destroyed (static teardown)
  std::lock_guard<std::mutex> g(mu);
  if ((int)pools->size() <= dev) pools->resize(dev + 1);
  if (!(*pools)[dev]) (*pools)[dev].reset(new EnginePool());
  return *(*pools)[dev];
}
size_t max_engines() {
  static const size_t k = [] {
    const char* e = std::getenv("FSTAMD_ENGINES");
    const int v = e ? std::atoi(e) : 4;
    return (size_t)std::max(1, std::min(v, 64));
  }();
  return k;
}
}  // namespace

DeviceEngine::Lease DeviceEngine::acquire(int dev) {
  if (dev < 0) return Lease();
  EnginePool& P = engine_pool(dev);
  std::unique_lock<std::mutex> lk(P.mu);
  for (;;) {
    if (!P.idle.empty()) {
      DeviceEngine* e = P.idle.back();
      P.idle.pop_back();
      return Lease(e);
    }
    if (P.all.size() < max_engines()) {
      P.all.emplace_back(new DeviceEngine(dev));
      return Lease(P.all.back().get());
    }
    P.cv.wait(lk);
  }
}

DeviceEngine::Lease DeviceEngine::try_acquire(int dev) {
  if (dev < 0) return Lease();
  EnginePool& P = engine_pool(dev);
  std::lock_guard<std::mutex> lk(P.mu);
  if (!P.idle.empty()) {
    DeviceEngine* e = P.idle.back();
    P.idle.pop_back();
    return Lease(e);
  }
  if (P.all.size() < max_engines()) {
    P.all.emplace_back(new DeviceEngine(dev));
    return Lease(P.all.back().get());
  }
  return Lease();
}

hipStream_t DeviceEngine::Lease::own_stream() const { return e_ ? e_->stream_ : nullptr; }

hipStream_t DeviceEngine::Lease::use(hipStream_t s) {
  if (!e_) return s;
  (void)hipSetDevice(e_->dev_);
  // work of the engine's previous user on another stream finishes before ours starts
  if (e_->done_valid_ && e_->done_stream_ != s) (void)hipStreamWaitEvent(s, e_->done_, 0);
  s_ = s;
  used_ = true;
  return s;
}

// Workspaces above this many bytes (96 GB: the dense and band replays size theirs from the free
// HBM) go back to the device when the lease ends: kept by an idle engine, they would leave
// the next heavy plan on this device -- another engine's, maybe another shard's of the same
// streamed call -- only the reserve to size itself from.  FSTAMD_RETAIN_GB overrides.
static size_t retain_bytes() {
  static const size_t b = [] {
    const char* e = std::getenv("FSTAMD_RETAIN_GB");
    return (size_t)(e ? std::max(0, std::atoi(e)) : 96) << 30;
  }();
  return b;
}

void DeviceEngine::Lease::release() {
  if (!e_) return;
  if (used_) {
    (void)hipSetDevice(e_->dev_);
    e_->done_valid_ = hipEventRecord(e_->done_, s_) == hipSuccess;
    e_->done_stream_ = s_;
  }
  size_t held = 0;
  for (size_t b : e_->sizes_) held += b;
  if (held > retain_bytes()) {  // (hipFree waits for the device's work, this lease's too)
    std::vector<void*> drop;
    e_->take_scratch(&drop);
    (void)hipSetDevice(e_->dev_);
    for (void* q : drop) (void)hipFree(q);
  }
  EnginePool& P = engine_pool(e_->dev_);
  {
    std::lock_guard<std::mutex> g(P.mu);
    P.idle.push_back(e_);
  }
  P.cv.notify_one();
  e_ = nullptr;
  used_ = false;
}

DeviceEngine::DeviceEngine(int dev) : dev_(dev) {
  (void)hipSetDevice(dev);
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) == hipSuccess) num_cus_ = p.multiProcessorCount;
  if (num_cus_ <= 0) num_cus_ = 256;
  bufs_.assign(kNumScratch, nullptr);
  sizes_.assign(kNumScratch, 0);
  (void)hipEventCreate(&ev0_);
  (void)hipEventCreate(&ev1_);
  (void)hipEventCreateWithFlags(&done_, hipEventDisableTiming);
  // non-blocking: the legacy null stream (other libraries, torch's default) never
  // serialises with it, and calls on other engines run concurrently
  if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) stream_ = nullptr;
}

// The idle engines' workspaces leave them under the pool lock; hipFree (it waits for the
// device's work, other engines' running kernels included) runs after the lock is released,
// so acquire / try_acquire on this device never wait behind it.
void DeviceEngine::trim_idle(int dev, const DeviceEngine* except) {
  if (dev < 0) return;
  EnginePool& P = engine_pool(dev);
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> g(P.mu);
    for (DeviceEngine* e : P.idle)
      if (e != except) e->take_scratch(&drop);
  }
  if (drop.empty()) return;
  (void)hipSetDevice(dev);
  for (void* p : drop) (void)hipFree(p);
}

void DeviceEngine::take_scratch(std::vector<void*>* out) {
  for (size_t i = 0; i < bufs_.size(); ++i) {
    if (bufs_[i]) out->push_back(bufs_[i]);
    bufs_[i] = nullptr;
    sizes_[i] = 0;
  }
  // the arrays that are initialised once per allocation must be initialised again: a new
  // allocation of the same size may come back at the same address, dirty
  ll_clean_ = ld_clean_ = ld_leaf_ = lb_clean_ = nullptr;
  ll_clean_bytes_ = ld_clean_bytes_ = ld_leaf_bytes_ = lb_clean_bytes_ = 0;
}

void* DeviceEngine::scratch(size_t idx, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (sizes_[idx] >= bytes) return bufs_[idx];
  if (bufs_[idx]) (void)hipFree(bufs_[idx]);
  bufs_[idx] = nullptr;
  sizes_[idx] = 0;
  if (hipMalloc(&bufs_[idx], bytes) != hipSuccess) {
    // out of HBM: the scratch of the device's idle engines (workspaces grow and are kept
    // per engine, so up to max_engines() sets of them) and the cached pool blocks go back,
    // then once more (this engine's own buffers may be in use by this call's launches)
    (void)hipGetLastError();
    trim_idle(dev_, this);
    device_pool_release(dev_);
    (void)hipSetDevice(dev_);
    if (hipMalloc(&bufs_[idx], bytes) != hipSuccess) {
      (void)hipGetLastError();
      bufs_[idx] = nullptr;
      return nullptr;
    }
  }
  sizes_[idx] = bytes;
  return bufs_[idx];
}

// A synchronous copy ordered with the engine's work on `stream` (the legacy synchronous
// hipMemcpy goes to the null stream, which a non-blocking engine stream does not wait for).
static hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind,
                            hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, kind, stream));
  return hipStreamSynchronize(stream);
}

// Test knob: caps a persistent kernel's grid, so that each wave takes many strings and
// keeps chase jobs pending across them (tests/test_gpu_lazy_pull.py, test_gpu_eager_pull.py)
static uint32_t grid_cap(const char* env) {
  const char* g = std::getenv(env);
  return g && std::atoi(g) > 0 ? (uint32_t)std::atoi(g) : 0xFFFFFFFFu;
}

__global__ void collect_list_kernel(const uint32_t* in_list, const uint32_t* in_count,
                                    const int32_t* status, int32_t code, uint32_t* list,
                                    uint32_t* count);

static hipError_t finish_stats(hipEvent_t e0, hipEvent_t e1, LaunchStats* stats) {
  if (!stats || stats->defer) return hipSuccess;  // (defer: DeviceEngine::finish_deferred)
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  stats->kernel_ms = ms;
  return hipSuccess;
}

bool DeviceEngine::pull_first(const DeviceFst& rhs, int semantics) {
  if (rhs.has_eps) return false;
  if (semantics == 1) {  // run_chain's eager tier chain: use_p
    if (rhs.nan || !rhs.nonneg || !rhs.pull_ok) return false;
    return std::getenv("FSTAMD_EAGER_TIER1") == nullptr;
  }
  const char* le = std::getenv("FSTAMD_LAZY_ENGINE");  // the lazy dispatch below: use_lp
  if (le && *le) return false;
  return rhs.nonneg && rhs.finite && rhs.lazy_pull_ok;
}

hipError_t DeviceEngine::finish_deferred(LaunchStats* stats) {
  if (!stats || !stats->defer) return hipSuccess;
  float ms = 0.f;
  const hipError_t e = hipEventElapsedTime(&ms, ev0_, ev1_);
  stats->kernel_ms = e == hipSuccess ? ms : 0.0;
  stats->defer = false;
  return e;
}

namespace {
template <int T>
int lazy_tiny_per_cu();
}  // namespace

hipError_t DeviceEngine::run_chain(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                   int semantics, const BatchOutDev& out, hipStream_t stream,
                                   LaunchStats* stats) {
  HIP_TRY(hipSetDevice(dev_));
  // the pull tiers alone copy paths out to the host (they must come first)
  if (out.host_ol && !pull_first(rhs, semantics)) return hipErrorInvalidValue;
  unsigned int* counter = (unsigned int*)scratch(kCounter, kCounterBytes);
  if (!counter) return hipErrorOutOfMemory;
  HIP_TRY(hipMemsetAsync(counter, 0, 64, stream));
  HIP_TRY(hipMemsetAsync(out.cursor, 0, sizeof(unsigned long long), stream));
  if (in.num_strings == 0) return hipSuccess;
  // every string starts as INTERNAL: a string no kernel finished can never read as a result
  // (after launch_pull_part the statuses are the pull tier's)
  if (!after_pull_)
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)out.status, kPathInternal, in.num_strings, stream));

  // Eager semantics on a layered lattice -> eager-layered engine.
  if (semantics == 1) {
    if (rhs.nan) {  // NaN has no order in the reference's compare: UNSUPPORTED
      mark_status_kernel<<<(in.num_strings + 255) / 256, 256, 0, stream>>>(in.num_strings, n,
                                                                           rhs.view.start, out);
      return hipGetLastError();
    }
    if (!rhs.nonneg) {
      // Negative weights: shortest-path.zig's Dijkstra is then not the exact SSSP the
      // parallel engines compute; the general engine builds each lattice and replays
      // the heap order on it (sp_replay, kernels/eager_bfs.hpp).
      if (stats) {
        stats->engine = 6;
        HIP_TRY(hipEventRecord(ev0_, stream));
      }
      HIP_TRY(run_bfs_chain(rhs, in, n, out, stream, true, false, true));
      if (stats) {
        HIP_TRY(hipEventRecord(ev1_, stream));
        HIP_TRY(finish_stats(ev0_, ev1_, stats));
      }
      return hipSuccess;
    }
    if (rhs.has_eps) {  // not layered: the general BFS engine takes every string
      if (stats) {
        stats->engine = 2;
        HIP_TRY(hipEventRecord(ev0_, stream));
      }
      HIP_TRY(run_bfs_chain(rhs, in, n, out, stream, true));
      if (stats) {
        HIP_TRY(hipEventRecord(ev1_, stream));
        HIP_TRY(finish_stats(ev0_, ev1_, stats));
      }
      return hipSuccess;
    }
    // Tier chain for layered lattices (each tier takes the strings the previous one
    // reports as OVERFLOW, through a device-side list):
    //   P  one wavefront per string, pull over the reverse mirror, window of kPullW states
    //      (when the rhs has one: DeviceFst::pull_ok)
    //   A0 one wavefront per string, direct-mapped LDS window of kEwinW target states
    //   A  one wavefront per string, LDS hash, <= kEwFcap tuples/layer, spans <= kEwKmax
    //   B  256 threads per string, LDS tables, <= kElFcap tuples/layer, spans <= kElKmax
    //   C  256 threads per string, HBM tables sized by the rhs (any layer)
    // FSTAMD_EAGER_TIER1=window starts at A0, =wave at A, =wg at B (A/B comparisons).  A
    // tier is skipped when the previous one provably cannot overflow on this rhs.
    const char* t1 = std::getenv("FSTAMD_EAGER_TIER1");
    const bool start_b = t1 && std::strcmp(t1, "wg") == 0;
    const bool use_w = !start_b && !(t1 && std::strcmp(t1, "wave") == 0);
    const bool use_p = use_w && rhs.pull_ok && !(t1 && std::strcmp(t1, "window") == 0);
    const uint32_t ns = rhs.view.num_states, ms = rhs.view.max_span;
    auto back_cap_for = [&](uint32_t fcap, uint64_t limit, bool* capped) {
      const uint64_t want = (uint64_t)(in.max_len + 1) * fcap;
      *capped = want > limit;
      return (uint32_t)std::min<uint64_t>(want, limit);
    };
    bool cap_w = false, cap_a = false, cap_b = false;
    const uint32_t back_cap_w = back_cap_for(kEwinW, 1u << 22, &cap_w);
    const uint32_t back_cap_a = back_cap_for(kEwFcap, 1u << 22, &cap_a);
    const uint32_t back_cap_b = back_cap_for(kElFcap, 1u << 22, &cap_b);
    // A0 overflows on a window wider than kEwinW or an expanded layer of more than
    // 64 * kEwinEmax tuples (both impossible with <= 64 * kEwinEmax states), on a span
    // longer than kEwinKmax and on its back slab; only the first two are A's business.
    const bool use_a = !start_b && (!use_w || ns > (uint32_t)(64 * kEwinEmax));
    const bool need_b = !(use_w || use_a) || ns > (uint32_t)kEwFcap || ms > (uint32_t)kEwKmax ||
                        (use_a && cap_a) || (use_w && (ms > (uint32_t)kEwinKmax || cap_w));
    const bool need_c = need_b && (ns > (uint32_t)kElFcap || ms > (uint32_t)kElKmax || cap_b);
    auto k_win = eager_window_kernel<kEwinEmax, kEwinRows, kEwinKmax, kEwinWaves>;
    if (const char* ww = std::getenv("FSTAMD_EWIN_WAVES")) {  // occupancy experiments
      if (std::strcmp(ww, "2") == 0) k_win = eager_window_kernel<kEwinEmax, kEwinRows, kEwinKmax, 2>;
      if (std::strcmp(ww, "4") == 0) k_win = eager_window_kernel<kEwinEmax, kEwinRows, kEwinKmax, 4>;
    }
    auto k_wave = eager_wave_kernel<kEwFcap, kEwHcap, kEwEmax, kEwKmax>;
    auto k_wg = eager_layered_lds_kernel<kElWG, kElFcap, kElHcap, kElKmax>;
    auto grid_for = [&](const void* k, int block, uint32_t back_cap) -> uint32_t {
      int occ = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, block, 0) != hipSuccess) occ = 1;
      uint32_t g = (uint32_t)std::min<uint64_t>((uint64_t)std::max(occ, 1) * num_cus_,
                                                in.num_strings);
      while (g > 1 && (uint64_t)g * back_cap * sizeof(uint2) > (4ull << 30)) g /= 2;
      return std::max<uint32_t>(g, 1);
    };
    // A0 keeps kChaseBatch back slabs per wave (backtraces are walked in batches)
    uint32_t grid_w = 0;
    if (use_w) {
      int occ = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_win, 64, 0) !=
          hipSuccess)
        occ = 1;
      grid_w = (uint32_t)std::min<uint64_t>((uint64_t)std::max(occ, 1) * num_cus_, in.num_strings);
      // behind tier P, A0 only takes P's overflows: 2 waves per CU keep its slabs small
      if (use_p) grid_w = std::min<uint32_t>(grid_w, 2u * (uint32_t)num_cus_);
      while (grid_w > 1 && (uint64_t)grid_w * kChaseBatch * back_cap_w * 8 > (24ull << 30))
        grid_w /= 2;
      grid_w = std::max<uint32_t>(grid_w, 1);
    }
    // P: kChaseBatch back slabs per wave too, kPullW slots per layer
    uint32_t grid_p = 0;
    uint2* back_p = nullptr;
    uint32_t* list_pw = nullptr;
    if (use_p) {
      grid_p = (uint32_t)std::min<uint64_t>((uint64_t)pull_waves_per_cu(rhs, in.max_len) * num_cus_,
                                            in.num_strings);
      grid_p = std::min<uint32_t>(grid_p, grid_cap("FSTAMD_P_GRID"));
      while (grid_p > 1 && (uint64_t)grid_p * kChaseBatch * back_cap_w * 8 > (24ull << 30))
        grid_p /= 2;
      grid_p = std::max<uint32_t>(grid_p, 1);
      back_p = (uint2*)scratch(kPullBack, (size_t)grid_p * kChaseBatch * back_cap_w * 8);
      list_pw = (uint32_t*)scratch(kItems4, (size_t)in.num_strings * 4);
      if (!back_p || !list_pw) return hipErrorOutOfMemory;
    }
    const uint32_t grid_a = use_a ? grid_for((const void*)k_wave, 64, back_cap_a) : 0;
    const uint32_t grid_b = need_b ? grid_for((const void*)k_wg, kElWG, back_cap_b) : 0;
    uint2* back_w =
        use_w ? (uint2*)scratch(kElBackW, (size_t)grid_w * kChaseBatch * back_cap_w * 8) : nullptr;
    uint2* back_a = use_a ? (uint2*)scratch(kElBack, (size_t)grid_a * back_cap_a * 8) : nullptr;
    uint2* back_b = need_b ? (uint2*)scratch(kElBackB, (size_t)grid_b * back_cap_b * 8) : nullptr;
    if ((use_w && !back_w) || (use_a && !back_a) || (need_b && !back_b))
      return hipErrorOutOfMemory;
    uint32_t* list_wa = (use_w && use_a) ? (uint32_t*)scratch(kItems3, (size_t)in.num_strings * 4)
                                         : nullptr;
    uint32_t* list_ab = ((use_w || use_a) && need_b)
                            ? (uint32_t*)scratch(kItems, (size_t)in.num_strings * 4)
                            : nullptr;
    uint32_t* list_bc = need_c ? (uint32_t*)scratch(kItems2, (size_t)in.num_strings * 4) : nullptr;
    if ((use_w && use_a && !list_wa) || ((use_w || use_a) && need_b && !list_ab) ||
        (need_c && !list_bc))
      return hipErrorOutOfMemory;
    uint32_t grid_c = 0, fcap_c = 0, hcap_c = 0, back_cap_c = 0;
    uint8_t* slab_c = nullptr;
    uint2* back_c = nullptr;
    if (need_c) {
      fcap_c = std::max<uint32_t>(ns, 1);
      hcap_c = next_pow2(2ull * fcap_c);
      back_cap_c = (uint32_t)std::min<uint64_t>((uint64_t)(in.max_len + 1) * fcap_c, 1u << 28);
      const uint64_t per_wg = layer_slab_bytes(fcap_c, hcap_c) + (uint64_t)back_cap_c * 8;
      grid_c = (uint32_t)std::min<uint64_t>(num_cus_, std::max<uint64_t>(1, (8ull << 30) / per_wg));
      slab_c = (uint8_t*)scratch(kElSlab, (size_t)grid_c * layer_slab_bytes(fcap_c, hcap_c));
      back_c = (uint2*)scratch(kElBack2, (size_t)grid_c * back_cap_c * sizeof(uint2));
      if (!slab_c || !back_c) return hipErrorOutOfMemory;
    }
    if (stats) {
      stats->engine = 0;
      stats->grid = use_p ? grid_p : use_w ? grid_w : use_a ? grid_a : grid_b;
      stats->launches = (use_p ? 2 : 0) + (use_w ? 1 : 0) + (use_a ? (use_w ? 2 : 1) : 0) +
                        (need_b ? ((use_w || use_a) ? 2 : 1) : 0) + (need_c ? 2 : 0);
      HIP_TRY(hipEventRecord(ev0_, stream));
    }
    const unsigned long long wd = watchdog_ticks();
    const uint32_t blocks = (in.num_strings + 255) / 256;
    // counters: [14] item counter of tier P, [15] |list_pw|; [5] item counter of tier A0,
    // [6] |list_wa|; [0..2] item counters of tiers A, B, C; [3] |list_ab|; [4] |list_bc|
    if (use_p) {
      EagerLaunch lp{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back_p, back_cap_w, wd};
      if (!after_pull_) HIP_TRY(launch_eager_pull(rhs, in, n, counter + 14, lp, out, grid_p, stream));
      // test hook: FSTAMD_EAGER_ONLY_FIRST leaves tier P's OVERFLOW / UNSUPPORTED strings
      // as they are, so a test can tell what the tier itself took
      if (std::getenv("FSTAMD_EAGER_ONLY_FIRST")) {
        if (stats) {
          HIP_TRY(hipEventRecord(ev1_, stream));
          HIP_TRY(finish_stats(ev0_, ev1_, stats));
        }
        return hipSuccess;
      }
    }
    if (use_w) {
      EagerLaunch lw{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back_w, back_cap_w, wd};
      if (use_p) {
        collect_status_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                          kPathOverflow, list_pw, counter + 15);
        lw.items = list_pw;
        lw.num_items_dev = counter + 15;
      }
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_trace_arm());
#endif
      k_win<<<grid_w, 64, 0, stream>>>(rhs.view, in, n, counter + 5, lw, out);
      HIP_TRY(hipGetLastError());
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_wait(stream, grid_w, "tierA0"));
#endif
    }
    if (use_a) {
      EagerLaunch la{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back_a, back_cap_a, wd};
      if (use_w) {
        collect_status_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                          kPathOverflow, list_wa, counter + 6);
        la.items = list_wa;
        la.num_items_dev = counter + 6;
      }
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_trace_arm());
#endif
      k_wave<<<grid_a, 64, 0, stream>>>(rhs.view, in, n, counter, la, out);
      HIP_TRY(hipGetLastError());
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_wait(stream, grid_a, "tierA"));
#endif
    }
    if (need_b) {
      EagerLaunch lb{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back_b, back_cap_b, wd};
      if (use_w || use_a) {
        collect_status_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                          kPathOverflow, list_ab, counter + 3);
        lb.items = list_ab;
        lb.num_items_dev = counter + 3;
      }
      k_wg<<<grid_b, kElWG, 0, stream>>>(rhs.view, in, n, counter + 1, lb, out);
      HIP_TRY(hipGetLastError());
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_wait(stream, grid_b, "tierB"));
#endif
    }
    if (need_c) {
      collect_status_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                        kPathOverflow, list_bc, counter + 4);
      EagerLaunch lc{list_bc, counter + 4, 0, slab_c, fcap_c, hcap_c, back_c, back_cap_c, wd};
      eager_layered_kernel<kElWG, kElFcap, kElHcap, false>
          <<<grid_c, kElWG, 0, stream>>>(rhs.view, in, n, counter + 2, lc, out);
      HIP_TRY(hipGetLastError());
#ifdef FSTAMD_DEBUG_WAIT
      HIP_TRY(debug_wait(stream, grid_c, "tierC"));
#endif
    }
    if (std::getenv("FSTAMD_ROUTE_LOG")) {  // how many strings each fallback tier took
      unsigned int h[16] = {};
      HIP_TRY(hipMemcpyAsync(h, counter, sizeof(h), hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      std::fprintf(stderr,
                   "[libfst_amd route] eager: %u strings, tiers P %d A0 %d A %d B %d C %d | "
                   "handed on: P->A0 %u, A0->A %u, ->B %u, ->C %u\n",
                   in.num_strings, (int)use_p, (int)use_w, (int)use_a, (int)need_b, (int)need_c,
                   use_p && use_w ? h[15] : 0u, use_w && use_a ? h[6] : 0u,
                   need_b && (use_w || use_a) ? h[3] : 0u, need_c ? h[4] : 0u);
    }
    // Strings the layered tiers cannot take (label-0 inputs -> UNSUPPORTED, tier-2
    // OVERFLOW) go to the general BFS engine.
    HIP_TRY(run_bfs_chain(rhs, in, n, out, stream, false));
    if (stats) {
      HIP_TRY(hipEventRecord(ev1_, stream));
      HIP_TRY(finish_stats(ev0_, ev1_, stats));
    }
    return hipSuccess;
  }

  // Lazy semantics.  Finite weights >= 0 -> the parallel rounds engines or the dense
  // replay; otherwise (+inf arcs, negative weights) the hashed exact replay.
  //  * rhs without input epsilons: the layered rounds engine (kernels/lazy_layered.hpp),
  //    then the general rounds engine (eager_bfs.hpp, bfs_lazy_path) for its leftovers;
  //  * rhs with input epsilons: the dense replay (kernels/lazy_dense.hpp) -- on epsilon-
  //    dense lattices nearly every tuple sits at one distance and the rounds degenerate to
  //    one pop each -- with the general rounds engine for its leftovers.  Small lattices
  //    too (config 4's tagger and verbalizer: 15.2 ms per two-stage call of 64K
  //    utterances vs 18.4 ms in the hashed replay, whose per-wave tables live in HBM).
  // FSTAMD_LAZY_ENGINE=rounds | replay | dense forces one engine (A/B runs, tests).
  const char* le = std::getenv("FSTAMD_LAZY_ENGINE");
  const bool force_rounds = le && std::strcmp(le, "rounds") == 0;
  const bool force_replay = le && std::strcmp(le, "replay") == 0;
  const bool force_dense = le && std::strcmp(le, "dense") == 0;
  // "lds": the LDS replay first whatever the rhs (tests: rhs without input epsilons)
  const bool force_lds = le && std::strcmp(le, "lds") == 0;
  // The hashed replay (below) starts small lattices with its tables in LDS, then HBM for
  // what outgrows them; FSTAMD_LAZY_TINY=0 skips that.  (As the engine for config 4's small
  // epsilon lattices it measured level with the dense replay, 15.8 vs 15.0 ms per two-stage
  // call: the pop's rhs reads and shuffles bind, not the tables.)
  const char* lte = std::getenv("FSTAMD_LAZY_TINY");
  const bool tiny_ok = !(lte && std::strcmp(lte, "0") == 0) &&
                       (uint64_t)(in.max_len + 1) * rhs.view.num_states <= 16384;
  const bool exact_ok = rhs.nonneg && rhs.finite && !force_replay;
  const bool use_dense = exact_ok && !force_rounds && (force_dense || force_lds || rhs.has_eps);
  const bool use_rounds = exact_ok && !use_dense;
  if (use_dense) {
    if (stats) {
      stats->engine = 5;
      stats->launches = 1;
      HIP_TRY(hipEventRecord(ev0_, stream));
    }
    // Small lattices first, whatever the rhs size: the replay with the wave's tables in
    // LDS at 128, then 256 tuples.  A WeText-scale tagger has 0.4 M states but ~140 tuples
    // per utterance, while the dense replay's per-wave index is (L + 1) * NS * 2 tuples (1.6
    // GB per wave there): it takes only what outgrows the LDS.  An rhs whose strings nearly
    // all outgrow it (config 3's lattices of millions of tuples) skips the LDS pass from
    // then on (DeviceFst::skip_tiny_lazy); FSTAMD_LAZY_TINY=0 skips it always.
    const bool small = !force_dense && !(lte && std::strcmp(lte, "0") == 0) &&
                       rhs.skip_tiny_lazy.load(std::memory_order_relaxed) == 0 &&
                       in.num_strings > 0;
    const uint32_t* todo = nullptr;  // the dense replay's strings (nullptr: all)
    uint32_t todo_n = in.num_strings;
    if (small) {
      const uint32_t num = in.num_strings;
      uint32_t* la = (uint32_t*)scratch(kItems, (size_t)num * 4);
      uint32_t* lb = (uint32_t*)scratch(kItems2, (size_t)num * 4);
      if (!la || !lb) return hipErrorOutOfMemory;
      unsigned int* c = counter + 40;  // [40] items (LDS 128), [41] |la|, [42] items (256), [43] |lb|
      HIP_TRY(hipMemsetAsync(c, 0, 16, stream));
      uint32_t g = 0;
      // the 128-tuple size first, unless it handed on over a third of an earlier batch on
      // this rhs (DeviceFst::tiny_lazy_256: the WeText-scale tagger's lattices, 54 % over
      // 128 tuples: tagger stage 46.7 -> 40.0 ms per 64 K utterances starting at 256);
      // FSTAMD_LAZY_TINY_START=1|2 forces the first size
      const char* ts = std::getenv("FSTAMD_LAZY_TINY_START");
      const bool first128 = ts && *ts ? std::strcmp(ts, "2") != 0
                                      : rhs.tiny_lazy_256.load(std::memory_order_relaxed) == 0;
      uint32_t cnt[2] = {0, 0};
      // A batch that the largest LDS size holds at once (coalesced single calls, small host
      // batches) starts every string there: one wave per string whichever the size, so a
      // long utterance no longer pays a replay at 256 tuples before its rerun at 512 or 1024
      // (36 B per tuple: 1024 tuples are 38 KB, 4 waves per CU)
      const bool direct = !(ts && *ts) &&
                          (uint64_t)num <= (uint64_t)num_cus_ * lazy_tiny_per_cu<4>();
      if (direct) {
        HIP_TRY(run_lazy_tiny(rhs, in, n, out, stream, 4, nullptr, num, c + 2, &g));
        if (stats) stats->grid = g;
        collect_status_kernel<<<(num + 255) / 256, 256, 0, stream>>>(out.status, num,
                                                                    kPathOverflow, lb, c + 3);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&cnt[1], c + 3, 4, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        if (num >= 64 && (uint64_t)cnt[1] * 10 > (uint64_t)num * 9)
          rhs.skip_tiny_lazy.store(1, std::memory_order_relaxed);
      } else if (first128) {
        HIP_TRY(run_lazy_tiny(rhs, in, n, out, stream, 1, nullptr, num, c, &g));
        if (stats) stats->grid = g;
        collect_status_kernel<<<(num + 255) / 256, 256, 0, stream>>>(out.status, num,
                                                                    kPathOverflow, la, c + 1);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&cnt[0], c + 1, 4, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
      } else {
        cnt[0] = num;
      }
      if (!direct && cnt[0] > 0) {
        HIP_TRY(run_lazy_tiny(rhs, in, n, out, stream, 2, first128 ? la : nullptr, cnt[0], c + 2, &g));
        if (first128) {
          collect_list_kernel<<<(cnt[0] + 255) / 256, 256, 0, stream>>>(la, c + 1, out.status,
                                                                        kPathOverflow, lb, c + 3);
        } else {
          collect_status_kernel<<<(num + 255) / 256, 256, 0, stream>>>(out.status, num,
                                                                      kPathOverflow, lb, c + 3);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&cnt[1], c + 3, 4, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        if (stats) stats->launches += 1;
      }
      if (!direct && first128 && num >= 1024 && (uint64_t)cnt[0] * 3 > (uint64_t)num)
        rhs.tiny_lazy_256.store(1, std::memory_order_relaxed);
      if (!direct && first128 && num < 1024) {  // small batches: the same rule over their sum
        const uint64_t seen = rhs.tiny_lazy_seen.fetch_add(num) + num;
        const uint64_t over = rhs.tiny_lazy_over.fetch_add(cnt[0]) + cnt[0];
        if (seen >= 1024 && over * 3 > seen) rhs.tiny_lazy_256.store(1, std::memory_order_relaxed);
      }
      if (!direct && first128 && num >= 64 && (uint64_t)cnt[0] * 10 > (uint64_t)num * 9)
        rhs.skip_tiny_lazy.store(1, std::memory_order_relaxed);
      todo = lb;
      todo_n = cnt[1];
      uint32_t* rest = lb;             // the strings still OVERFLOW, and their count (device)
      unsigned int* rest_cnt = c + 3;
      uint32_t* spare = la;
      unsigned int* spare_cnt = c + 1;
      // Larger LDS sizes for the outliers of the LDS replays, or for every string of a small
      // batch (a coalesced single call: a long utterance, ~400-900 tuples, went to the dense
      // replay's HBM index -- 2.7 ms for 63 labels of the WeText-scale tagger): 512 tuples
      // (~55 KB, 2 waves per CU), then 1024 (~110 KB, 1 per CU), one string per wave.
      uint32_t cnt_big[2] = {0, 0};
      for (int t = 3; !direct && t <= 4 && todo_n > 0 && ((uint64_t)todo_n * 4 <= num || num <= 64);
           ++t) {
        unsigned int* ci = counter + 48 + 2 * (t - 3);  // [48|50] items, [49|51] |next list|
        HIP_TRY(hipMemsetAsync(ci, 0, 8, stream));
        HIP_TRY(run_lazy_tiny(rhs, in, n, out, stream, t, rest, todo_n, ci, &g));
        collect_list_kernel<<<(todo_n + 255) / 256, 256, 0, stream>>>(rest, rest_cnt, out.status,
                                                                      kPathOverflow, spare, ci + 1);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&todo_n, ci + 1, 4, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        cnt_big[t - 3] = todo_n;
        std::swap(rest, spare);
        spare_cnt = rest_cnt;
        rest_cnt = ci + 1;
        todo = rest;
        if (stats) stats->launches += 1;
      }
      // The LDS replays took most strings (>= 3/4): the rest are small-lattice outliers,
      // served by the hashed replay (HBM tables sized by the lattice, x8 per retry) rather
      // than by the dense index sized by (L + 1) * NS (a WeText-scale tagger: 1.6 GB per
      // wave).  When they took few (large lattices), the dense replay takes the rest.
      if (todo_n > 0 && (uint64_t)todo_n * 4 <= num) {
        uint32_t* cur = rest;
        unsigned int* cur_cnt = rest_cnt;
        uint32_t* nxt = spare;
        unsigned int* nxt_cnt = spare_cnt;
        uint64_t want = 4096;
        for (int t = 0; t < 4 && todo_n > 0; ++t, want *= 8) {
          HIP_TRY(hipMemsetAsync(c + 4, 0, 4, stream));  // [44] item counter
          if (launch_lazy_hashed(rhs, in, n, out, stream, want, cur, todo_n, c + 4, &g) !=
              hipSuccess)
            break;  // beyond its budget: the strings stay OVERFLOW for the dense replay
          HIP_TRY(hipMemsetAsync(nxt_cnt, 0, 4, stream));
          collect_list_kernel<<<(todo_n + 255) / 256, 256, 0, stream>>>(
              cur, cur_cnt, out.status, kPathOverflow, nxt, nxt_cnt);
          HIP_TRY(hipGetLastError());
          HIP_TRY(hipMemcpyAsync(&todo_n, nxt_cnt, 4, hipMemcpyDeviceToHost, stream));
          HIP_TRY(hipStreamSynchronize(stream));
          std::swap(cur, nxt);
          std::swap(cur_cnt, nxt_cnt);
          if (stats) stats->launches += 1;
        }
        todo = cur;
      }
      if (std::getenv("FSTAMD_ROUTE_LOG"))
        std::fprintf(stderr,
                     "[libfst_amd route] lazy: %u strings, LDS-128 handed on %u, LDS-256 %u, "
                     "LDS-512 %u, LDS-1024 %u, to the dense replay %u\n",
                     num, cnt[0], cnt[1], cnt_big[0], cnt_big[1], todo_n);
    }
    // the LDS (and hashed) replays took every string: they leave none UNSUPPORTED, so there
    // is nothing for the band, dense or general engines -- and the general engine's count
    // readback would cost the call a synchronisation (the band and dense replays do mark
    // strings UNSUPPORTED, so this holds only when neither runs)
    const bool all_done = small && todo_n == 0;
    bool ran = true;
    if (todo_n > 0) {
      // the band replay first (rhs whose arcs all go forward: config 3), the dense replay
      // for what it hands on
      // With the exact early exit a string only reaches ~2 L states past the start
      // (config 3: DESIGN.md §4.2c), so the first launch keeps back pointers for a few
      // windows of states; what reaches further runs again over the whole rhs.
      const bool early_ok = rhs.nonneg && rhs.finite && !std::getenv("FSTAMD_NO_EARLY");
      for (int pass = early_ok ? 0 : 1; pass < 2 && todo_n > 0; ++pass) {
        bool band = false;
        HIP_TRY(run_lazy_band(rhs, in, n, out, stream, &band, todo, todo ? todo_n : 0,
                              pass == 0));
        if (!band) break;
        if (stats) stats->launches += 1;
        // (the list `todo` may be kItems or kItems2: the next one goes elsewhere)
        uint32_t* la = (uint32_t*)scratch(pass == 0 ? kItems3 : kItems4,
                                          (size_t)in.num_strings * 4);
        if (!la) return hipErrorOutOfMemory;
        unsigned int* c = counter + 46;  // [46] |la|
        HIP_TRY(hipMemsetAsync(c, 0, 4, stream));
        collect_status_kernel<<<(in.num_strings + 255) / 256, 256, 0, stream>>>(
            out.status, in.num_strings, kPathOverflow, la, c);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&todo_n, c, 4, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        todo = la;
        if (std::getenv("FSTAMD_ROUTE_LOG"))
          std::fprintf(stderr, "[libfst_amd route] lazy: band replay (%s) handed on %u\n",
                       pass == 0 ? "capped, early exit" : "whole rhs", todo_n);
      }
    }
    if (todo_n > 0) {
      HIP_TRY(run_lazy_dense(rhs, in, n, out, stream, &ran, todo, todo ? todo_n : 0));
      if (stats) stats->launches += 1;
    }
    if (stats && !ran) stats->engine = 3;  // too large for the dense engine: rounds only
    if (!std::getenv("FSTAMD_DENSE_NOFALLBACK") && !all_done)  // debug: leave UNSUPPORTED
      HIP_TRY(run_bfs_chain(rhs, in, n, out, stream, !ran && !small, true));
    if (stats) {
      HIP_TRY(hipEventRecord(ev1_, stream));
      HIP_TRY(finish_stats(ev0_, ev1_, stats));
    }
    return hipSuccess;
  }
  if (use_rounds) {
    if (stats) {
      stats->engine = 3;
      HIP_TRY(hipEventRecord(ev0_, stream));
    }
    // Layered lattices (no rhs input epsilon; label-0 inputs are sent on as UNSUPPORTED):
    // the one-wave dense engine (kernels/lazy_layered.hpp), FSTAMD_LAZY_LAYERED=0 skips
    // it; the general rounds engine takes everything else and its leftovers.
    const char* ll = std::getenv("FSTAMD_LAZY_LAYERED");
    const bool layered = !rhs.has_eps && rhs.view.max_span <= kLlSpanMax &&
                         (uint64_t)(in.max_len + 1) * rhs.view.num_states <= kLlDenseMax &&
                         !(ll && std::strcmp(ll, "0") == 0);
    // Layer-local pull first (kernels/lazy_pull.hpp) when the rhs has a reverse mirror
    // that suits it; the strings it hands on go to the rounds engines.
    const bool use_lp = !rhs.has_eps && rhs.lazy_pull_ok && !force_rounds;
    uint32_t* lp_list = nullptr;
    uint32_t* lp_count = nullptr;
    if (use_lp) {
      if (stats) stats->engine = 7;
      HIP_TRY(run_lazy_pull(rhs, in, n, out, stream, &lp_list, &lp_count, !after_pull_));
      if (std::getenv("FSTAMD_LAZY_ONLY_FIRST")) {  // test hook: what the pull took alone
        if (stats) {
          HIP_TRY(hipEventRecord(ev1_, stream));
          HIP_TRY(finish_stats(ev0_, ev1_, stats));
        }
        return hipSuccess;
      }
    }
    if (layered) {
      if (stats && !use_lp) stats->engine = 4;
      HIP_TRY(run_lazy_layered(rhs, in, n, out, stream, lp_list, lp_count));
    }
    HIP_TRY(run_bfs_chain(rhs, in, n, out, stream, !layered && !use_lp, true));
    if (stats) {
      HIP_TRY(hipEventRecord(ev1_, stream));
      HIP_TRY(finish_stats(ev0_, ev1_, stats));
    }
    return hipSuccess;
  }
  // Replay: the per-wave workspace is sized from max_len; strings that outgrow it
  // (OVERFLOW) are re-run from a list with 8x the capacity and fewer waves, until they
  // fit or the budget is exhausted.
  auto launch_lazy = [&](uint64_t want_nodes, const uint32_t* items, uint32_t num_items,
                         unsigned int* ctr, uint32_t* grid_out) -> hipError_t {
    return launch_lazy_hashed(rhs, in, n, out, stream, want_nodes, items, num_items, ctr,
                              grid_out);
  };
  uint64_t want = std::max<uint64_t>(4096, (uint64_t)256 * (in.max_len + 1));
  if (stats) {
    stats->engine = 1;
    stats->launches = 1;
    HIP_TRY(hipEventRecord(ev0_, stream));
  }
  uint32_t grid0 = 0;
  const bool tiny_first = tiny_ok;
  if (tiny_first) {  // LDS tables (kernels/lazy_wave.hpp, 128 tuples)
    HIP_TRY(run_lazy_tiny(rhs, in, n, out, stream, 1, nullptr, in.num_strings, counter, &grid0));
  } else {
    HIP_TRY(launch_lazy(want, nullptr, in.num_strings, counter, &grid0));
  }
  if (stats) stats->grid = grid0;
  // retry tiers for OVERFLOW strings (host reads the count: this path is for outliers)
  uint32_t* list = (uint32_t*)scratch(kItems, (size_t)in.num_strings * 4);
  if (!list) return hipErrorOutOfMemory;
  for (int tier = 1; tier <= 4; ++tier) {
    unsigned int* ctr = counter + 4 + 2 * tier;  // [item counter, list count] per tier
    HIP_TRY(hipMemsetAsync(ctr, 0, 8, stream));
    collect_status_kernel<<<(in.num_strings + 255) / 256, 256, 0, stream>>>(
        out.status, in.num_strings, kPathOverflow, list, ctr + 1);
    HIP_TRY(hipGetLastError());
    uint32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, ctr + 1, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (cnt == 0) break;
    if (!(tiny_first && tier == 1)) want *= 8;  // after the tiny launch: HBM at `want` first
    uint32_t g = 0;
    if (launch_lazy(want, list, cnt, ctr, &g) != hipSuccess) break;  // stays OVERFLOW
    if (stats) stats->launches += 2;
  }
  if (stats) {
    HIP_TRY(hipEventRecord(ev1_, stream));
    HIP_TRY(finish_stats(ev0_, ev1_, stats));
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------------
// General eager engine (kernels/eager_bfs.hpp)
// ---------------------------------------------------------------------------------

namespace {
// Per-string workspace tiers: nodes / arcs grow x8 until one slab would exceed the
// budget.  Tier 0 (16K tuples, 256K arcs, ~4 MB) covers metric-like strings with
// 4 workgroups per CU in flight; eps-dense T=4096 L=96 (781K tuples, 10M arcs) needs
// tier 2.
constexpr uint32_t kBfsNcap0 = 1u << 14;
constexpr uint32_t kBfsAcap0 = 1u << 18;
constexpr uint32_t kBfsWgPerCu0 = 4;
constexpr uint64_t kBfsBudget = 40ull << 30;  // bytes of BFS workspace per launch
constexpr int kBfsWG = 256;

struct BfsCaps {
  uint32_t ncap, acap, hcap, lcap;
  size_t stride;
};
BfsCaps bfs_caps(int tier) {
  BfsCaps c;
  uint64_t n = (uint64_t)kBfsNcap0 << (3 * tier), a = (uint64_t)kBfsAcap0 << (3 * tier);
  c.ncap = (uint32_t)std::min<uint64_t>(n, 1u << 30);
  c.acap = (uint32_t)std::min<uint64_t>(a, 0x7FFFFFFFu);
  c.hcap = next_pow2(2ull * c.ncap);
  c.lcap = c.ncap;
  c.stride = bfs_slab_bytes(c.ncap, c.acap, c.hcap, c.lcap);
  return c;
}
}  // namespace

__global__ void collect_status2_kernel(const int32_t* status, uint32_t num, int32_t a, int32_t b,
                                       uint32_t* list, uint32_t* count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < num && (status[i] == a || status[i] == b)) list[atomicAdd(count, 1u)] = i;
}

__global__ void collect_list_kernel(const uint32_t* in_list, const uint32_t* in_count,
                                    const int32_t* status, int32_t code, uint32_t* list,
                                    uint32_t* count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *in_count && status[in_list[i]] == code) list[atomicAdd(count, 1u)] = in_list[i];
}

// One-wave dense lazy engine for layered lattices.  Its per-wave dense arrays are left
// clean by every string, so they are initialised only when (re)allocated.
hipError_t DeviceEngine::run_lazy_pull(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                       const BatchOutDev& out, hipStream_t stream,
                                       uint32_t** list, uint32_t** count_dev, bool launch) {
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);  // [34..35] are ours
  if (!ctr) return hipErrorOutOfMemory;
  // kChaseBatch back slabs per wave, kPullW slots per layer (as tier P)
  const uint32_t back_cap =
      (uint32_t)std::min<uint64_t>((uint64_t)(in.max_len + 1) * kPullW, 1u << 22);
  uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)lazy_pull_waves_per_cu(rhs, in.max_len) * num_cus_,
                                               in.num_strings);
  grid = std::min<uint32_t>(grid, grid_cap("FSTAMD_LP_GRID"));
  while (grid > 1 && (uint64_t)grid * kChaseBatch * back_cap * 8 > (24ull << 30)) grid /= 2;
  grid = std::max<uint32_t>(grid, 1);
  uint2* back = (uint2*)scratch(kLpBack, (size_t)grid * kChaseBatch * back_cap * 8);
  uint32_t* lst = (uint32_t*)scratch(kItems5, (size_t)in.num_strings * 4);
  if (!back || !lst) return hipErrorOutOfMemory;
  HIP_TRY(hipMemsetAsync(ctr + 34, 0, 8, stream));
  EagerLaunch lp{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back, back_cap, watchdog_ticks()};
  if (launch) HIP_TRY(launch_lazy_pull(rhs, in, n, ctr + 34, lp, out, grid, stream));
  collect_status_kernel<<<(in.num_strings + 255) / 256, 256, 0, stream>>>(
      out.status, in.num_strings, kPathOverflow, lst, ctr + 35);
  HIP_TRY(hipGetLastError());
  *list = lst;
  *count_dev = ctr + 35;
  return hipSuccess;
}

hipError_t DeviceEngine::launch_pull_part(const DeviceFst& rhs, const ChainInput& in,
                                          uint32_t n, int semantics, const BatchOutDev& out,
                                          hipStream_t stream, unsigned int* item_ctr) {
  HIP_TRY(hipSetDevice(dev_));
  if (!pull_first(rhs, semantics)) return hipErrorInvalidValue;
  if (in.num_strings == 0) return hipSuccess;
  const bool lazy = semantics != 1;
  const int per_cu = lazy ? lazy_pull_waves_per_cu(rhs, in.max_len) : pull_waves_per_cu(rhs, in.max_len);
  const uint32_t back_cap =
      (uint32_t)std::min<uint64_t>((uint64_t)(in.max_len + 1) * kPullW, 1u << 22);
  // the back slabs sized for a full grid whatever this part's size, so no later part
  // reallocates them (a free waits for the device) while an earlier one runs
  uint32_t full = (uint32_t)std::max<uint64_t>((uint64_t)per_cu * num_cus_, 1);
  while (full > 1 && (uint64_t)full * kChaseBatch * back_cap * 8 > (24ull << 30)) full /= 2;
  uint2* back = (uint2*)scratch(lazy ? kLpBack : kPullBack, (size_t)full * kChaseBatch * back_cap * 8);
  if (!back) return hipErrorOutOfMemory;
  const uint32_t grid = std::max<uint32_t>(std::min<uint32_t>(full, in.num_strings), 1);
  EagerLaunch lp{nullptr, nullptr, in.num_strings, nullptr, 0, 0, back, back_cap, watchdog_ticks()};
  return lazy ? launch_lazy_pull(rhs, in, n, item_ctr, lp, out, grid, stream)
              : launch_eager_pull(rhs, in, n, item_ctr, lp, out, grid, stream);
}

hipError_t DeviceEngine::run_lazy_layered(const DeviceFst& rhs, const ChainInput& in,
                                          uint32_t n, const BatchOutDev& out,
                                          hipStream_t stream, const uint32_t* items,
                                          const uint32_t* num_items_dev) {
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);  // [32] is ours
  if (!ctr) return hipErrorOutOfMemory;
  LlWs ws{};
  ws.lcap = in.max_len;
  ws.dn = (uint64_t)(in.max_len + 1) * rhs.view.num_states;
  ws.ncap = (uint32_t)ws.dn;
  ws.wd_ticks = watchdog_ticks();
  ws.items = items;
  ws.num_items_dev = num_items_dev;
  ws.acap = (uint32_t)std::min<uint64_t>(ws.dn, 1u << 15);
  const uint64_t per_wave = ws.dn * (8 + 8 + 4 + 4 + 4 + 4) + ((uint64_t)ws.lcap + 2) * 4 +
                            (uint64_t)ws.acap * 32;
  const uint64_t budget = 48ull << 30;  // of the 288 GB: all 16 waves per CU at the metric
  // behind the lazy pull (items != null) it takes only the pull's fallbacks: 2 waves per
  // CU keep its dense workspaces small
  uint32_t grid = (uint32_t)std::min<uint64_t>(
      {(uint64_t)num_cus_ * (items ? 2 : 16), (uint64_t)in.num_strings,
       std::max<uint64_t>(1, budget / per_wave)});
  grid = std::max<uint32_t>(grid, 1);
  const size_t g = grid;
  ws.dk = (unsigned long long*)scratch(kLlDk, g * ws.dn * 8);
  ws.back = (unsigned long long*)scratch(kLlBack, g * ws.dn * 8);
  ws.lidf = (uint32_t*)scratch(kLlLidf, g * ws.dn * 4);
  ws.flg = (uint32_t*)scratch(kLlFlg, g * ws.dn * 4);
  ws.nodes = (uint32_t*)scratch(kLlNodes, g * ws.dn * 4);
  ws.inv = (uint32_t*)scratch(kLlInv, g * ws.dn * 4);
  ws.loff = (uint32_t*)scratch(kLlLoff, g * ((size_t)ws.lcap + 2) * 4);
  ws.act = (uint4*)scratch(kLlAct, g * 2 * (size_t)ws.acap * sizeof(uint4));
  if (!ws.dk || !ws.back || !ws.lidf || !ws.flg || !ws.nodes || !ws.inv || !ws.loff || !ws.act)
    return hipErrorOutOfMemory;
  if (ll_clean_ != bufs_[kLlDk] || ll_clean_bytes_ != sizes_[kLlDk]) {  // new allocation
    HIP_TRY(hipMemsetAsync(ws.dk, 0xFF, sizes_[kLlDk], stream));
    HIP_TRY(hipMemsetAsync(ws.back, 0xFF, sizes_[kLlBack], stream));
    HIP_TRY(hipMemsetAsync(ws.lidf, 0xFF, sizes_[kLlLidf], stream));
    HIP_TRY(hipMemsetAsync(ws.flg, 0, sizes_[kLlFlg], stream));
    ll_clean_ = bufs_[kLlDk];
    ll_clean_bytes_ = sizes_[kLlDk];
  }
  HIP_TRY(hipMemsetAsync(ctr + 32, 0, 4, stream));
  const bool prof = std::getenv("FSTAMD_BFS_PROF") != nullptr;
  ws.prof = prof ? (unsigned long long*)scratch(kDebug, g * 64) : nullptr;
  if (ws.prof) HIP_TRY(hipMemsetAsync(ws.prof, 0, g * 64, stream));
  lazy_layered_kernel<<<grid, 64, 0, stream>>>(rhs.view, in, n, ctr + 32, ws, out);
  HIP_TRY(hipGetLastError());
  if (ws.prof) {  // phase profile: sums over waves, ticks at 100 MHz
    std::vector<unsigned long long> h(g * 8);
    HIP_TRY(hipMemcpyAsync(h.data(), ws.prof, h.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    unsigned long long sum[8] = {};
    for (size_t i = 0; i < h.size(); ++i) sum[i % 8] += h[i];
    const double it = (double)std::max(1ull, sum[4]);
    std::fprintf(stderr,
                 "[lazy-layered prof] grid %u items %llu | us/item: layers %.1f rounds %.1f "
                 "back/best/out %.1f reset %.1f | rounds/item %.1f\n",
                 grid, sum[4], sum[0] / 100.0 / it, sum[1] / 100.0 / it, sum[2] / 100.0 / it,
                 sum[3] / 100.0 / it, sum[5] / it);
  }
  return hipSuccess;
}

// The hashed exact replay (kernels/lazy_wave.hpp) with per-wave HBM tables sized for
// want_nodes tuples, over a device list of strings (nullptr: all of `in`).
hipError_t DeviceEngine::launch_lazy_hashed(const DeviceFst& rhs, const ChainInput& in,
                                            uint32_t n, const BatchOutDev& out,
                                            hipStream_t stream, uint64_t want_nodes,
                                            const uint32_t* items, uint32_t num_items,
                                            unsigned int* ctr, uint32_t* grid_out) {
  GraphInput none{};
  const bool debug = std::getenv("FSTAMD_LAZY_DEBUG") != nullptr;
  LazyWs ws{};
  ws.ncap = next_pow2(want_nodes);
  ws.hcap = ws.ncap * 2;
  ws.qcap = ws.ncap * 4;
  ws.gcap = 64;
  const uint64_t per_wave = (uint64_t)ws.hcap * sizeof(uint4) +
                            (uint64_t)ws.ncap * (8 + 8 + 16 + 8) +
                            (uint64_t)ws.qcap * (8 + 4) + (uint64_t)ws.gcap * sizeof(uint4);
  if (per_wave > (24ull << 30)) return hipErrorOutOfMemory;
  uint32_t grid =
      (uint32_t)std::min<uint64_t>((uint64_t)num_cus_ * 4 * FSTAMD_REPLAY_WAVES, num_items);
  // latency-bound: as many waves in flight as the SIMDs hold (4/SIMD), within 20 GB of
  // the 288 GB HBM
  const uint64_t budget = 20ull << 30;
  while (grid > 1 && (uint64_t)grid * per_wave > budget) grid /= 2;
  grid = std::max<uint32_t>(grid, 1);
  ws.hslot = (uint4*)scratch(kLzHash, (size_t)grid * ws.hcap * sizeof(uint4));
  ws.nkey = (unsigned long long*)scratch(kLzNkey, (size_t)grid * ws.ncap * 8);
  ws.ndist = (double*)scratch(kLzNdist, (size_t)grid * ws.ncap * 8);
  ws.nback = (uint4*)scratch(kLzNback, (size_t)grid * ws.ncap * 16);
  ws.nbw = (double*)scratch(kLzNbw, (size_t)grid * ws.ncap * 8);
  ws.qd = (double*)scratch(kLzQd, (size_t)grid * ws.qcap * 8);
  ws.qid = (uint32_t*)scratch(kLzQid, (size_t)grid * ws.qcap * 4);
  ws.gscratch = (uint4*)scratch(kLzG, (size_t)grid * ws.gcap * sizeof(uint4));
  if (!ws.hslot || !ws.nkey || !ws.ndist || !ws.nback || !ws.nbw || !ws.qd || !ws.qid ||
      !ws.gscratch)
    return hipErrorOutOfMemory;
  // Stamps: zero the table whenever it was (re)allocated or the stamp would wrap.
  if (lazy_hash_bytes_ != (size_t)grid * ws.hcap * sizeof(uint4) ||
      (uint64_t)lazy_stamp_ + num_items + 2 > 0xFFFFFFF0ull) {
    HIP_TRY(hipMemsetAsync(ws.hslot, 0, (size_t)grid * ws.hcap * sizeof(uint4), stream));
    lazy_hash_bytes_ = (size_t)grid * ws.hcap * sizeof(uint4);
    lazy_stamp_ = 0;
  }
  ws.stamp_base = lazy_stamp_;
  ws.max_pops = ws.qcap + 1;
  lazy_stamp_ += num_items + 1;
  ws.wd_ticks = watchdog_ticks();
  ws.dbg = debug ? (uint32_t*)scratch(kDebug, (size_t)grid * 8 * 4) : nullptr;
  if (ws.dbg) HIP_TRY(hipMemsetAsync(ws.dbg, 0, (size_t)grid * 8 * 4, stream));
  lazy_wave_kernel<false><<<grid, 64, 0, stream>>>(rhs.view, in, none, n, ctr, items,
                                                   num_items, ws, out);
  HIP_TRY(hipGetLastError());
  if (debug) dump_debug(ws.dbg, grid, stream);
  *grid_out = grid;
  return hipSuccess;
}

namespace {
template <int T>
int lazy_tiny_per_cu() {  // resident LDS-replay waves per CU, asked of the runtime once
  static const int occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &o, (const void*)lazy_tiny_kernel<T>, 64, 0) != hipSuccess)
      o = 1;
    return std::max(o, 1);
  }();
  return occ;
}
template <int N>
int ctiny_per_cu() {
  static const int occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (const void*)eager_tiny_kernel<N>, 64,
                                                     0) != hipSuccess)
      o = 1;
    return std::max(o, 1);
  }();
  return occ;
}
}  // namespace

hipError_t DeviceEngine::run_lazy_tiny(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                       const BatchOutDev& out, hipStream_t stream, int tier,
                                       const uint32_t* items, uint32_t num_items,
                                       unsigned int* ctr, uint32_t* grid_out) {
  // (lazy_tiny_kernel sizes its tables from the tier; of LazyWs it reads the watchdog and
  // the first hash generation)
  LazyWs ws{};
  // test knobs: FSTAMD_TINY_GEN0 = the hash generation lazy_tiny_kernel starts from (its wrap
  // at 65536 strings per wave, within reach); FSTAMD_TINY_WAVES caps the grid
  const char* eg = std::getenv("FSTAMD_TINY_GEN0");
  const char* ew = std::getenv("FSTAMD_TINY_WAVES");
  ws.stamp_base = eg ? (uint32_t)std::strtoul(eg, nullptr, 10) & 0xFFFFu : 0u;
  const uint32_t cap_waves = ew ? (uint32_t)std::strtoul(ew, nullptr, 10) : 0u;
  ws.wd_ticks = watchdog_ticks();
  const int occ = tier == 1 ? lazy_tiny_per_cu<1>() : tier == 2 ? lazy_tiny_per_cu<2>()
                 : tier == 3 ? lazy_tiny_per_cu<3>() : lazy_tiny_per_cu<4>();
  uint32_t grid =
      (uint32_t)std::min<uint64_t>((uint64_t)num_cus_ * occ, std::max(num_items, 1u));
  if (cap_waves) grid = std::min(grid, cap_waves);
  if (tier == 1)
    lazy_tiny_kernel<1><<<grid, 64, 0, stream>>>(rhs.view, in, n, ctr, items, num_items, ws, out);
  else if (tier == 2)
    lazy_tiny_kernel<2><<<grid, 64, 0, stream>>>(rhs.view, in, n, ctr, items, num_items, ws, out);
  else if (tier == 3)
    lazy_tiny_kernel<3><<<grid, 64, 0, stream>>>(rhs.view, in, n, ctr, items, num_items, ws, out);
  else
    lazy_tiny_kernel<4><<<grid, 64, 0, stream>>>(rhs.view, in, n, ctr, items, num_items, ws, out);
  HIP_TRY(hipGetLastError());
#ifdef FSTAMD_TINY_PROF
  {
    unsigned long long p[8];
    HIP_TRY(hipStreamSynchronize(stream));
    HIP_TRY(hipMemcpyFromSymbol(p, HIP_SYMBOL(g_tiny_prof), sizeof(p)));
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_tiny_prof), z, sizeof(z)));
    const double pops = p[7] ? (double)p[7] : 1.0;
    std::fprintf(stderr,
                 "[tiny prof] tier %d: %u strings, %llu pops; cycles per pop: pop %.0f, tuple+spans "
                 "%.0f, records+lookup %.0f, dedup %.0f, group+fold %.0f, heap %.0f, result %.0f\n",
                 tier, num_items, p[7], p[0] / pops, p[1] / pops, p[2] / pops, p[3] / pops,
                 p[4] / pops, p[5] / pops, p[6] / pops);
  }
#endif
  if (grid_out) *grid_out = grid;
  return hipSuccess;
}

constexpr size_t kLdMaxDynLds = 150 * 1024;

// Band replay (kernels/lazy_band.hpp): the dense replay over a sliding window of rhs
// states, for an rhs whose arcs all go forward (jump_back == 0).  Per wave: the window's
// records (16 B x ws x (L + 1) x 2), 8 B per possible id, a 16K-id ring, a 64K-entry
// future list.  Strings it hands on end OVERFLOW / UNSUPPORTED (the dense replay, then
// the rounds engine, take them).  subset_dev: the strings to run (nullptr: all).
hipError_t DeviceEngine::run_lazy_band(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                       const BatchOutDev& out, hipStream_t stream, bool* ran,
                                       const uint32_t* subset_dev, uint32_t subset_n,
                                       bool capped) {
  *ran = false;
  if (rhs.view.jump_back != 0 || std::getenv("FSTAMD_NO_BAND")) return hipSuccess;
  if (rhs.view.start >= rhs.view.num_states) capped = false;  // (no start: all EMPTY)
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);  // [36] is ours
  if (!ctr) return hipErrorOutOfMemory;
  // the strings and their lengths on the host (plans, buckets, longest first)
  std::vector<uint64_t> off((size_t)in.num_strings + 1);
  HIP_TRY(hipMemcpyAsync(off.data(), in.offsets, off.size() * 8, hipMemcpyDeviceToHost, stream));
  std::vector<uint32_t> order;
  if (subset_dev) {
    order.resize(subset_n);
    if (subset_n)
      HIP_TRY(hipMemcpyAsync(order.data(), subset_dev, subset_n * 4ull, hipMemcpyDeviceToHost,
                             stream));
  } else {
    order.resize(in.num_strings);
    for (uint32_t i = 0; i < in.num_strings; ++i) order[i] = i;
  }
  HIP_TRY(hipStreamSynchronize(stream));
  const uint32_t num = (uint32_t)order.size();
  if (num == 0) {
    *ran = true;
    return hipSuccess;
  }
  auto len = [&](uint32_t i) { return (uint32_t)std::min<uint64_t>(off[i + 1] - off[i], in.max_len); };
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return len(a) < len(b); });
  const uint32_t NS = rhs.view.num_states;
  constexpr uint32_t kRing = kLbIdRing, kFcap = kLbFcap;  // the kernel's compile-time sizes
  // states past the start (every reachable state is: arcs go forward)
  const uint32_t srange = rhs.view.start < NS ? NS - rhs.view.start : NS;
  struct Plan {
    uint32_t lcap, wstates, scap, grid, first, count;
    uint64_t wn, tn;
    size_t lds;
  };
  // back pointer width: f_src (1 bit) | state distance (dbits) | arc index within the source
  // state; 1, 2 or 4 B as that fits (config 3's rhs: 1 + 3 + 4 bits), else not this engine's
  uint32_t dbits = 1;
  while ((1ull << dbits) <= rhs.view.jump_fwd) ++dbits;
  uint32_t abits = 1;
  while ((1ull << abits) < rhs.view.max_span) ++abits;
  const uint32_t bits = 1 + dbits + abits;
  if (bits > 32) return hipSuccess;
  const uint32_t bkb = bits <= 8 ? 1 : bits <= 16 ? 2 : 4;
  // every launch's memory from one budget: free HBM (pooled blocks released first) less a
  // 24 GB reserve, 90 % of it; the plans are made one at a time per device (EnginePool::heavy)
  std::unique_lock<std::mutex> heavy(engine_pool(dev_).heavy);
  device_pool_release(dev_);
  uint64_t budget = 128ull << 30;
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) {
      uint64_t avail = fr;
      for (size_t b : {kLbWin, kLbBk, kLbIdr, kLbFut}) avail += sizes_[b];
      const uint64_t reserve = 24ull << 30;
      budget = avail > 2 * reserve ? (avail - reserve) / 10 * 9 : avail / 2;
    }
    if (const char* be = std::getenv("FSTAMD_DENSE_BUDGET_GB"))
      budget = (uint64_t)std::max(1, std::atoi(be)) << 30;
  }
  // waves per CU: ~5 KB of LDS and 61 VGPRs each, so 32 fit
  uint32_t wpc = 32;
  if (const char* we = std::getenv("FSTAMD_BAND_WAVES_PER_CU")) wpc = (uint32_t)std::max(1, std::atoi(we));
  const uint32_t max_waves = (uint32_t)num_cus_ * wpc;
  const char* ge = std::getenv("FSTAMD_DENSE_GRID");
  const char* wse = std::getenv("FSTAMD_BAND_WS");  // tests: a window too small (overflows)
  auto make_plan = [&](uint32_t max_len, uint32_t count, Plan& p) -> bool {
    p.lcap = std::max<uint32_t>(max_len, 1);
    if (p.lcap > 4095) return false;
    uint32_t w = 64;
    const uint64_t want = 2ull * (p.lcap + 1) + 2ull * (rhs.view.jump_fwd + 1);
    while (w < want) w <<= 1;
    if (wse) w = std::max<uint32_t>(64, 1u << (31 - __builtin_clz((uint32_t)std::max(1, std::atoi(wse)))));
    p.wstates = w;
    if ((uint64_t)w * (p.lcap + 1) >= (1ull << 26)) return false;  // the kernel's div_lc range
    p.wn = (uint64_t)w * (p.lcap + 1) * 2;
    p.scap = capped ? std::min<uint32_t>(srange, 2 * w) : srange;
    p.tn = (uint64_t)(p.lcap + 1) * p.scap * 2;  // ids and tuple indices fit 31 bits
    if (p.tn > kLdDenseMax) return false;
    p.lds = kRing / 8 + (size_t)p.lcap * 4;
    if (p.lds > kLdMaxDynLds) return false;
    const uint64_t per_wave = p.wn * 16 + p.tn * bkb + (uint64_t)kRing * 4 + (uint64_t)kFcap * 16;
    p.grid = (uint32_t)std::min<uint64_t>(
        {(uint64_t)max_waves, (uint64_t)count, std::max<uint64_t>(1, budget / per_wave)});
    if (ge) p.grid = std::min<uint32_t>(p.grid, (uint32_t)std::max(1, std::atoi(ge)));
    p.grid = std::max<uint32_t>(p.grid, 1);
    p.count = count;
    p.first = 0;
    return true;
  };
  Plan whole;
  if (!make_plan(len(order.back()), num, whole)) return hipSuccess;
  // length buckets (as the dense replay) when the longest string's footprint caps the
  // waves and the batch refills them many times; longest first inside each launch
  uint32_t nb = (whole.grid < max_waves && num >= 8ull * max_waves) ? 4u : 1u;
  if (const char* be = std::getenv("FSTAMD_DENSE_BUCKETS")) nb = (uint32_t)std::max(1, std::atoi(be));
  nb = std::min<uint32_t>(nb, num);
  std::vector<Plan> plans;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t lo = (uint32_t)((uint64_t)num * b / nb), hi = (uint32_t)((uint64_t)num * (b + 1) / nb);
    if (hi == lo) continue;
    Plan p;
    if (nb == 1 || !make_plan(len(order[hi - 1]), hi - lo, p)) p = whole;
    p.first = lo;
    p.count = hi - lo;
    std::reverse(order.begin() + lo, order.begin() + hi);
    plans.push_back(p);
  }
  uint64_t need_win = 0, need_bk = 0;
  uint32_t gmax = 0;
  for (const Plan& p : plans) {
    need_win = std::max<uint64_t>(need_win, (uint64_t)p.grid * p.wn);
    need_bk = std::max<uint64_t>(need_bk, (uint64_t)p.grid * p.tn);
    gmax = std::max(gmax, p.grid);
  }
  LbWs ws{};
  ws.win = (uint4*)scratch(kLbWin, need_win * 16);
  ws.bk = scratch(kLbBk, need_bk * bkb);
  ws.bkb = bkb;
  ws.dbits = dbits;
  ws.idr = (uint32_t*)scratch(kLbIdr, (size_t)gmax * kRing * 4);
  ws.fut = (uint4*)scratch(kLbFut, (size_t)gmax * kFcap * 16);
  uint32_t* d_order = (uint32_t*)scratch(kLbItems, (size_t)num * 4);
  if (!ws.win || !ws.bk || !ws.idr || !ws.fut || !d_order) return hipErrorOutOfMemory;
  if (lb_clean_ != bufs_[kLbWin] || lb_clean_bytes_ != sizes_[kLbWin]) {  // new allocation
    HIP_TRY(hipMemsetAsync(ws.win, 0xFF, sizes_[kLbWin], stream));
    lb_clean_ = bufs_[kLbWin];
    lb_clean_bytes_ = sizes_[kLbWin];
  }
  HIP_TRY(hipMemcpyAsync(d_order, order.data(), (size_t)num * 4, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));  // `order` is pageable and goes away
  heavy.unlock();  // the arrays are allocated: a concurrent plan sees the HBM they took
  const bool prof = std::getenv("FSTAMD_BFS_PROF") != nullptr;
  ws.prof = prof ? (unsigned long long*)scratch(kDebug, (size_t)gmax * kLbProf * 8) : nullptr;
  if (ws.prof) HIP_TRY(hipMemsetAsync(ws.prof, 0, (size_t)gmax * kLbProf * 8, stream));
  ws.ring = kRing;
  ws.fcap = kFcap;
  ws.sil = rhs.band_il;
  ws.srec = rhs.band_rec;
  ws.ssh = rhs.band_sh;
  if (std::getenv("FSTAMD_ROUTE_LOG"))
    for (const Plan& p : plans)
      std::fprintf(stderr, "[libfst_amd route] band plan: %u strings, lcap %u, grid %u of %u waves "
                   "(budget %.1f GB), window %u states, arc table %s\n", p.count, p.lcap, p.grid,
                   max_waves, budget / 1e9, p.wstates, ws.sil ? "on" : "off");
  // the exact early exit needs every arc and final weight >= +0, finite
  // arcs; FSTAMD_NO_EARLY=1 replays the whole product as the reference does (tests, A/B)
  ws.early = (rhs.nonneg && rhs.finite && !std::getenv("FSTAMD_NO_EARLY")) ? 1u : 0u;
  for (const Plan& p : plans) {
    ws.lcap = p.lcap;
    ws.scap = p.scap;
    ws.ws = p.wstates;
    ws.wn = p.wn;
    ws.tn = p.tn;
    ws.wd_ticks = watchdog_ticks();
    ws.wd_tuple_ticks = std::getenv("FSTAMD_WATCHDOG_MS") ? 0ull : 1000ull;
    ws.items = d_order + p.first;
    ws.num_items = p.count;
    HIP_TRY(hipMemsetAsync(ctr + 36, 0, 4, stream));
    // back pointers of 1, 2 or 4 B: one instance each
    // (and the slot path's preconditions as a compile-time fact when they hold)
    const bool fp = ws.sil != nullptr && rhs.view.jump_fwd < 32;
    auto* kern = fp ? (bkb == 1 ? lazy_band_kernel<1, true> : bkb == 2 ? lazy_band_kernel<2, true>
                                                                         : lazy_band_kernel<4, true>)
                    : (bkb == 1 ? lazy_band_kernel<1, false> : bkb == 2 ? lazy_band_kernel<2, false>
                                                                          : lazy_band_kernel<4, false>);
    if (p.lds > 64 * 1024)
      HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)p.lds));
    kern<<<p.grid, 64, p.lds, stream>>>(rhs.view, in, n, ctr + 36, ws, out);
    HIP_TRY(hipGetLastError());
  }
  *ran = true;
  if (ws.prof) {
    std::vector<unsigned long long> h((size_t)gmax * kLbProf);
    HIP_TRY(hipMemcpyAsync(h.data(), ws.prof, h.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    unsigned long long sum[8] = {}, ee = 0, oc = 0;
    for (size_t w = 0; w < gmax; ++w) {
      for (int j = 0; j < 8; ++j) sum[j] += h[w * kLbProf + j];
      ee += h[w * kLbProf + 16];
      oc += h[w * kLbProf + 17];
    }
    const double it = (double)std::max(1ull, sum[3]);
    std::fprintf(stderr, "[lazy-band prof] grid %u items %llu | per item: pops %.0f advances "
                 "%.1f slides %.1f | early exits %llu | overflows: window %llu ids %llu future "
                 "%llu ring %llu states %llu\n",
                 gmax, sum[3], sum[0] / it, sum[1] / it, sum[2] / it, ee, sum[4], sum[5], sum[6],
                 sum[7], oc);
    if (kLbProf > 306) {
      unsigned long long tt[6] = {};
      for (size_t w = 0; w < gmax; ++w)
        for (int j = 0; j < 6; ++j) tt[j] += h[w * kLbProf + 300 + j];
      const double tp = (double)std::max(1ull, sum[0]);
      std::fprintf(stderr, "[lazy-band prof] s_memtime ticks per pop: find %.1f pop %.1f "
                   "cand %.1f slide %.1f relax %.1f loop %.1f\n", tt[0] / tp, tt[1] / tp,
                   tt[2] / tp, tt[3] / tp, tt[4] / tp, tt[5] / tp);
    }
    int shown = 0;
    for (size_t w = 0; w < gmax && shown < 4; ++w) {
      const unsigned long long* q = &h[w * kLbProf];
      if (!q[9]) continue;
      if (kLbProf > 16 && shown == 0)
        for (uint32_t e = 0; e < (kLbProf - 16) / 2 && q[16 + 2 * e]; ++e)
          std::fprintf(stderr, "[lazy-band ev] tag %llu id %llu pop %llu word %016llx\n",
                       q[16 + 2 * e] >> 56, (q[16 + 2 * e] >> 24) & 0xFFFFFFFFull,
                       q[16 + 2 * e] & 0xFFFFFFull, q[17 + 2 * e]);
      ++shown;
      std::fprintf(stderr, "[lazy-band prof]   wave %zu: site %llu at pop %llu s %llu aux %llu "
                   "slo %llu nn %llu fn %llu L %llu | %llx %llu %llu %llx\n", w, q[9], q[8], q[10], q[11],
                   q[12], q[13], q[14], q[15], q[4], q[5], q[6], q[7]);
    }
  }
  uint64_t held = 0;
  for (size_t b : {kLbWin, kLbBk, kLbIdr, kLbFut}) held += sizes_[b];
  if (held > (64ull << 30)) {  // give large arrays back after the call
    HIP_TRY(hipStreamSynchronize(stream));
    for (size_t b : {kLbWin, kLbBk, kLbIdr, kLbFut}) {
      (void)hipFree(bufs_[b]);
      bufs_[b] = nullptr;
      sizes_[b] = 0;
    }
    lb_clean_ = nullptr;
  }
  return hipSuccess;
}

// Dense lazy replay (kernels/lazy_dense.hpp).  Per wave: rec 16 B + back arc 4 B + id map
// 4 B per dense tuple, the bitmap, and a future list of a quarter of the dense tuples
// (compacted when full; a string that still overflows goes to the rounds engine).  The
// dense arrays are left clean by every string, so they are initialised only when
// (re)allocated.  *ran = false when the lattice is too large for the engine at all.
// LDS of a gfx950 workgroup is 160 KB; the kernel's static LdLds takes ~4.6 KB of it.

hipError_t DeviceEngine::run_lazy_dense(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                        const BatchOutDev& out, hipStream_t stream, bool* ran,
                                        const uint32_t* subset_dev, uint32_t subset_n) {
  *ran = false;
  // the strings this call takes: all of `in`, or a device list (what the LDS replay of
  // small lattices handed on); with a list the plan is sized by its own longest string
  std::vector<uint32_t> subset;
  std::vector<uint64_t> off;
  uint32_t num = in.num_strings, max_len = in.max_len;
  if (subset_dev) {
    subset.resize(subset_n);
    off.resize((size_t)in.num_strings + 1);
    if (subset_n)
      HIP_TRY(hipMemcpyAsync(subset.data(), subset_dev, subset_n * 4ull, hipMemcpyDeviceToHost,
                             stream));
    HIP_TRY(hipMemcpyAsync(off.data(), in.offsets, off.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    num = subset_n;
    max_len = 0;
    for (uint32_t i : subset)
      max_len = std::max<uint32_t>(max_len, (uint32_t)std::min<uint64_t>(off[i + 1] - off[i], in.max_len));
    if (num == 0) {
      *ran = true;
      return hipSuccess;
    }
  }
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);  // [33] is ours
  if (!ctr) return hipErrorOutOfMemory;
  // One launch plan: the per-wave dense state is sized by the longest string it takes.
  struct Plan {
    uint32_t lcap, nleaf, nsum, fcap, grid, first, count;  // [first, first + count) of items
    uint64_t dn;
    size_t lds;
  };
  // Latency-bound: the waves in flight set the rate, and at large rhs (config 3, T =
  // 65,536: ~0.9 GB per wave) memory caps them.  The budget is what HBM has free (the
  // dense arrays already held count as free for them) less a 24 GB reserve, 90 % of it;
  // 128 GB when the runtime cannot say.  Arrays above 128 GB are released after the call
  // so that later calls of other engines find their memory.  FSTAMD_DENSE_BUDGET_GB sets it.
  // (the runtime is asked only when the plan could need more than 16 GB: small calls skip
  // the query)
  uint64_t budget = 128ull << 30;
  bool budget_known = false;
  if (const char* be = std::getenv("FSTAMD_DENSE_BUDGET_GB")) {
    budget = (uint64_t)std::max(1, std::atoi(be)) << 30;
    budget_known = true;
  }
  // plans that ask the runtime for free HBM are made (and their arrays allocated) one at a
  // time per device: two concurrent calls would otherwise both size themselves to it
  std::unique_lock<std::mutex> heavy(engine_pool(dev_).heavy, std::defer_lock);
  auto query_budget = [&] {
    if (!heavy.owns_lock()) heavy.lock();
    device_pool_release(dev_);  // idle pooled blocks count as free HBM
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) {
      uint64_t avail = fr;
      for (size_t b : {kLdRec, kLdBarc, kLdIds, kLdLeaf, kLdFut}) avail += sizes_[b];
      const uint64_t reserve = 24ull << 30;
      budget = avail > 2 * reserve ? (avail - reserve) / 10 * 9 : avail / 2;
    }
    budget_known = true;
  };
  const uint32_t max_waves = (uint32_t)num_cus_ * 16;
  const char* ge = std::getenv("FSTAMD_DENSE_GRID");  // debug: fewer waves
  auto make_plan = [&](uint32_t max_len, uint32_t count, Plan& p) -> bool {
    p.lcap = std::max<uint32_t>(max_len, 1);
    p.dn = (uint64_t)(p.lcap + 1) * 2 * rhs.view.num_states;
    if (p.dn > kLdDenseMax) return false;
    p.nleaf = (uint32_t)((p.dn + 63) / 64);
    p.nsum = (p.nleaf + 63) / 64;
    // dynamic LDS: the summary bitmap and the labels (config 3 at T = 65,536, L = 251:
    // 65 KB; the waves in flight there are capped by HBM long before LDS)
    p.lds = (size_t)p.nsum * 8 + (size_t)p.lcap * 4;
    if (const char* le = std::getenv("FSTAMD_DENSE_LDS_MIN"))  // tests: a > 64 KB launch
      p.lds = std::max<size_t>(p.lds, (size_t)std::max(0, std::atoi(le)));
    if (p.lds > kLdMaxDynLds) return false;
    p.fcap = (uint32_t)std::max<uint64_t>(4096, p.dn / 4);
    const uint64_t per_wave = p.dn * (16 + 4 + 4) + (uint64_t)p.nleaf * 8 + (uint64_t)p.fcap * 16;
    if (!budget_known &&
        std::min<uint64_t>(max_waves, count) * per_wave > (16ull << 30))
      query_budget();
    p.grid = (uint32_t)std::min<uint64_t>(
        {(uint64_t)max_waves, (uint64_t)count, std::max<uint64_t>(1, budget / per_wave)});
    if (ge) p.grid = std::min<uint32_t>(p.grid, (uint32_t)std::max(1, std::atoi(ge)));
    p.grid = std::max<uint32_t>(p.grid, 1);
    p.count = count;
    p.first = 0;
    return true;
  };
  Plan whole;
  if (!make_plan(max_len, num, whole)) return hipSuccess;
  // Length buckets.  When the dense state of the longest string caps the waves in flight
  // (budget / per-wave < max_waves: large rhs, e.g. config 3 at T >= 4096), the strings are
  // launched in buckets of similar length, each sized by its own longest string, so short
  // strings run many more waves at once.  Results do not depend on the launch a string is
  // in.  FSTAMD_DENSE_BUCKETS=k forces k buckets (tests), =1 turns them off.
  std::vector<Plan> plans;
  std::vector<uint32_t> order;  // string indices, bucket by bucket
  // Only for batches that refill every bucket's waves many times over: with fewer strings
  // a bucket runs one string per wave and its tail dominates (T = 4096, 4096 strings:
  // 14.1 s bucketed vs 9.2 s in one launch).
  uint32_t nb = (whole.grid < max_waves && num >= 8ull * max_waves) ? 4u : 1u;
  if (const char* be = std::getenv("FSTAMD_DENSE_BUCKETS"))
    nb = (uint32_t)std::max(1, std::atoi(be));
  nb = std::min<uint32_t>(nb, std::max<uint32_t>(num, 1));
  // Longest first inside a launch: work items are taken in order, so when a launch has
  // more strings than waves the long strings start first and the short ones fill the
  // tail (list scheduling, longest processing time first).  FSTAMD_DENSE_LPT=0 turns it
  // off (measurements).
  bool lpt = num > whole.grid;
  if (const char* le = std::getenv("FSTAMD_DENSE_LPT")) lpt = lpt && std::atoi(le) != 0;
  if (nb > 1 || lpt || subset_dev) {
    if (!subset_dev) {
      off.resize((size_t)in.num_strings + 1);
      HIP_TRY(hipMemcpyAsync(off.data(), in.offsets, off.size() * 8, hipMemcpyDeviceToHost,
                             stream));
      HIP_TRY(hipStreamSynchronize(stream));
      order.resize(in.num_strings);
      for (uint32_t i = 0; i < in.num_strings; ++i) order[i] = i;
    } else {
      order = subset;
    }
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      return off[a + 1] - off[a] < off[b + 1] - off[b];
    });
    for (uint32_t b = 0; b < nb; ++b) {  // equal-count buckets of the sorted lengths
      const uint32_t lo = (uint32_t)((uint64_t)num * b / nb);
      const uint32_t hi = (uint32_t)((uint64_t)num * (b + 1) / nb);
      if (hi == lo) continue;
      const uint32_t last = order[hi - 1];
      // a length above max_len (caller's bound) keeps the whole plan: the kernel passes
      // such a string on (UNSUPPORTED) exactly as without buckets
      const uint32_t blen = (uint32_t)std::min<uint64_t>(off[last + 1] - off[last], in.max_len);
      Plan p;
      if (nb == 1 || !make_plan(blen, hi - lo, p)) p = whole;
      p.first = lo;
      p.count = hi - lo;
      if (lpt) std::reverse(order.begin() + lo, order.begin() + hi);
      plans.push_back(p);
    }
  } else {
    plans.push_back(whole);
  }
  // one allocation per array, sized for the largest launch
  uint64_t need_rec = 0, need_leaf = 0, need_fut = 0;
  for (const Plan& p : plans) {
    need_rec = std::max<uint64_t>(need_rec, (uint64_t)p.grid * p.dn);
    need_leaf = std::max<uint64_t>(need_leaf, (uint64_t)p.grid * p.nleaf);
    need_fut = std::max<uint64_t>(need_fut, (uint64_t)p.grid * p.fcap);
  }
  LdWs ws{};
  ws.rec = (uint4*)scratch(kLdRec, need_rec * 16);
  ws.barc = (uint32_t*)scratch(kLdBarc, need_rec * 4);
  ws.ids = (uint32_t*)scratch(kLdIds, need_rec * 4);
  ws.leaf = (unsigned long long*)scratch(kLdLeaf, need_leaf * 8);
  ws.fut = (uint4*)scratch(kLdFut, need_fut * 16);
  uint32_t* d_order = nullptr;
  if (!order.empty()) d_order = (uint32_t*)scratch(kLdItems, order.size() * 4);
  if (!ws.rec || !ws.barc || !ws.ids || !ws.leaf || !ws.fut || (!order.empty() && !d_order))
    return hipErrorOutOfMemory;
  // every string leaves the rec / leaf words it touched clean, whatever the launch's
  // partition of the buffers, so they are initialised once per allocation
  if (ld_clean_ != bufs_[kLdRec] || ld_clean_bytes_ != sizes_[kLdRec] ||
      ld_leaf_ != bufs_[kLdLeaf] || ld_leaf_bytes_ != sizes_[kLdLeaf]) {  // new allocation
    HIP_TRY(hipMemsetAsync(ws.rec, 0xFF, sizes_[kLdRec], stream));
    HIP_TRY(hipMemsetAsync(ws.leaf, 0, sizes_[kLdLeaf], stream));
    ld_clean_ = bufs_[kLdRec];
    ld_clean_bytes_ = sizes_[kLdRec];
    ld_leaf_ = bufs_[kLdLeaf];
    ld_leaf_bytes_ = sizes_[kLdLeaf];
  }
  if (d_order) {  // pageable source: wait for the copy before `order` goes away
    HIP_TRY(hipMemcpyAsync(d_order, order.data(), order.size() * 4, hipMemcpyHostToDevice,
                           stream));
    HIP_TRY(hipStreamSynchronize(stream));
  }
  const bool prof = std::getenv("FSTAMD_BFS_PROF") != nullptr;
  uint32_t gmax = 0;
  for (const Plan& p : plans) gmax = std::max(gmax, p.grid);
  ws.prof = prof ? (unsigned long long*)scratch(kDebug, (size_t)gmax * 64) : nullptr;
  if (ws.prof) HIP_TRY(hipMemsetAsync(ws.prof, 0, (size_t)gmax * 64, stream));
  for (const Plan& p : plans) {
    ws.lcap = p.lcap;
    ws.dn = p.dn;
    ws.nleaf = p.nleaf;
    ws.nsum = p.nsum;
    ws.fcap = p.fcap;
    ws.wd_ticks = watchdog_ticks();
    // + 10 us per dense tuple (s_memrealtime: 100 MHz), unless a test set the watchdog
    ws.wd_tuple_ticks = std::getenv("FSTAMD_WATCHDOG_MS") ? 0ull : 1000ull;
    ws.items = d_order ? d_order + p.first : nullptr;
    ws.num_items = p.count;
    HIP_TRY(hipMemsetAsync(ctr + 33, 0, 4, stream));
#ifdef FSTAMD_DEBUG_WAIT
    HIP_TRY(debug_trace_arm());
#endif
    if (p.lds > 64 * 1024)  // beyond the default dynamic-LDS limit of a launch
      HIP_TRY(hipFuncSetAttribute((const void*)lazy_dense_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds));
    lazy_dense_kernel<<<p.grid, 64, p.lds, stream>>>(rhs.view, in, n, ctr + 33, ws, out);
    HIP_TRY(hipGetLastError());
#ifdef FSTAMD_DEBUG_WAIT
    HIP_TRY(debug_wait(stream, p.grid, "lazy_dense"));
#endif
  }
  const size_t g = gmax;
  const uint32_t grid = gmax;
  *ran = true;
  if (ws.prof) {
    std::vector<unsigned long long> h(g * 8);
    HIP_TRY(hipMemcpyAsync(h.data(), ws.prof, h.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    unsigned long long sum[8] = {};
    for (size_t i = 0; i < h.size(); ++i) sum[i % 8] += h[i];
    const double it = (double)std::max(1ull, sum[3]);
    std::fprintf(stderr,
                 "[lazy-dense prof] grid %u items %llu | per item: pops %.0f advances %.1f "
                 "future entries scanned %.0f\n",
                 grid, sum[3], sum[0] / it, sum[1] / it, sum[2] / it);
  }
  uint64_t held = 0;
  for (size_t b : {kLdRec, kLdBarc, kLdIds, kLdLeaf, kLdFut}) held += sizes_[b];
  if (held > (128ull << 30)) {  // beyond the old fixed budget: give it back after the call
    HIP_TRY(hipStreamSynchronize(stream));
    for (size_t b : {kLdRec, kLdBarc, kLdIds, kLdLeaf, kLdFut}) {
      (void)hipFree(bufs_[b]);
      bufs_[b] = nullptr;
      sizes_[b] = 0;
    }
    ld_clean_ = nullptr;
    ld_leaf_ = nullptr;
  }
  return hipSuccess;
}

namespace {
// resident tiny-tier workgroups per CU (LDS-bound), asked of the runtime once per size
template <int K>
int tiny_per_cu() {
  static const int occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &o, (const void*)eager_bfs_kernel<64, false, K>, 64, 0) != hipSuccess)
      o = 1;
    return std::max(o, 1);
  }();
  return occ;
}
}  // namespace

hipError_t DeviceEngine::run_bfs_chain(const DeviceFst& rhs, const ChainInput& in, uint32_t n,
                                       const BatchOutDev& out, hipStream_t stream, bool all,
                                       bool lazy, bool replay) {
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);  // [8..15] are ours
  uint32_t* list = (uint32_t*)scratch(kBfsList, (size_t)in.num_strings * 4);
  uint32_t* list2 = (uint32_t*)scratch(kBfsList2, (size_t)in.num_strings * 4);
  if (!ctr || !list || !list2) return hipErrorOutOfMemory;
  uint32_t* cnt = ctr + 8;
  HIP_TRY(hipMemsetAsync(cnt, 0, 32, stream));
  const uint32_t blocks = (in.num_strings + 255) / 256;
  if (all) {
    mark_status_kernel<<<blocks, 256, 0, stream>>>(in.num_strings, 1, rhs.view.start, out);
    collect_status2_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                       kPathUnsupported, kPathUnsupported, list,
                                                       cnt);
  } else {
    collect_status2_kernel<<<blocks, 256, 0, stream>>>(out.status, in.num_strings,
                                                       kPathUnsupported, kPathOverflow, list, cnt);
  }
  HIP_TRY(hipGetLastError());
  uint32_t count = 0;
  HIP_TRY(hipMemcpyAsync(&count, cnt, 4, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  // Tiers -2 and -1 (tiny, tables in LDS, kernels/eager_bfs.hpp tiny_caps) first when the lattices are
  // small by the product bound; not for the exact heap replay (negative weights), whose
  // heap lives in HBM.  FSTAMD_BFS_TINY=0 turns it off (A/B runs, tests).
  const char* te = std::getenv("FSTAMD_BFS_TINY");
  // Small lattices by the product bound always fit; beyond it the tiny tiers are tried too
  // (a WeText-scale rhs: 0.4 M states, ~140 tuples per utterance) unless an earlier batch
  // on this rhs handed nearly every string on (DeviceFst::skip_tiny_eager).
  const bool tiny = !replay && !(te && std::strcmp(te, "0") == 0) &&
                    ((uint64_t)(in.max_len + 1) * rhs.view.num_states <= 16384 ||
                     rhs.skip_tiny_eager.load(std::memory_order_relaxed) == 0);
  const uint32_t count0 = count;
  // Eager semantics on an rhs a one-word tuple key can name: the compact tiny tiers
  // (kernels/eager_tiny.hpp, ~52 B per tuple instead of ~110: 23 / 12 workgroups per CU
  // instead of 10 / 5).  FSTAMD_EAGER_CTINY=0 keeps eager_bfs_kernel's (A/B runs, tests).
  const char* cte = std::getenv("FSTAMD_EAGER_CTINY");
  const bool compact = tiny && !lazy && !(cte && std::strcmp(cte, "0") == 0) &&
                       rhs.view.num_states < kCtMaxStates && rhs.view.num_arcs < kCtPhase3;
  // tier -2: the 128-tuple tiny size, tier -1: the 256-tuple one, then the HBM tiers.
  // The 128-tuple size is skipped on an rhs where it handed on over a third of an earlier
  // batch (DeviceFst::tiny_eager_256); FSTAMD_BFS_TINY_START=1|2 forces the first size.
  const char* tse = std::getenv("FSTAMD_BFS_TINY_START");
  const bool first128 = tse && *tse ? std::strcmp(tse, "2") != 0
                                    : rhs.tiny_eager_256.load(std::memory_order_relaxed) == 0;
  for (int tier = tiny ? (first128 ? -2 : -1) : 0; count > 0; ++tier) {
    const TinyCaps tc = tiny_caps(tier == -2 ? 1 : 2);
    const BfsCaps c = tier < 0 ? BfsCaps{tc.n, tc.a, tc.h, tc.l, 0} : bfs_caps(tier);
    const uint64_t fit = tier < 0 ? ~0ull : std::max<uint64_t>(1, kBfsBudget / c.stride);
    if (kBfsBudget < c.stride) break;  // beyond the budget: those strings stay OVERFLOW
    // tier 0: small lattices -> one wavefront per string by default (wave-level
    // barriers, 4x the strings in flight); FSTAMD_BFS_WG0=256 for A/B runs
    const char* wge = std::getenv("FSTAMD_BFS_WG0");
    const bool wave = tier == 0 && !(wge && std::strcmp(wge, "256") == 0);
    const uint64_t per_cu = tier < 0 ? (uint64_t)(compact ? (tier == -2 ? ctiny_per_cu<128>()
                                                                        : ctiny_per_cu<256>())
                                                 : tier == -2 ? tiny_per_cu<1>() : tiny_per_cu<2>())
                            : tier == 0 ? (wave ? 4 * FSTAMD_BFS_WAVES64 : kBfsWgPerCu0) : 1;
    const uint32_t grid =
        (uint32_t)std::min<uint64_t>({(uint64_t)count, (uint64_t)num_cus_ * per_cu, fit});
    BfsWs ws{};
    ws.slab = tier < 0 ? nullptr : (uint8_t*)scratch(kBfsSlab, (size_t)grid * c.stride);
    ws.hdr = (uint32_t*)scratch(kBfsHdr, (size_t)grid * 8 * 4);
    if ((tier >= 0 && !ws.slab) || !ws.hdr) return hipErrorOutOfMemory;
    ws.stride = c.stride;
    ws.ncap = c.ncap;
    ws.acap = c.acap;
    ws.hcap = c.hcap;
    ws.lcap = c.lcap;
    ws.wd_ticks = watchdog_ticks();
    ws.lattice_only = 0;
    ws.lazy = lazy ? 1u : 0u;
    if (replay && !lazy) {  // heap + settled flags per workgroup (kernels/eager_bfs.hpp)
      ws.replay = (uint8_t*)scratch(kBfsHeap,
                                    (size_t)grid * ((size_t)(c.acap + 1) * 16 + c.ncap));
      if (!ws.replay) return hipErrorOutOfMemory;
    }
    const bool prof = std::getenv("FSTAMD_BFS_PROF") != nullptr;
    ws.prof = prof ? (unsigned long long*)scratch(kDebug, (size_t)grid * 64) : nullptr;
    if (ws.prof) HIP_TRY(hipMemsetAsync(ws.prof, 0, (size_t)grid * 64, stream));
    HIP_TRY(hipMemsetAsync(cnt + 1, 0, 8, stream));  // item counter + next list count
    GraphInput none{};
    if (tier < 0 && compact) {
      if (tier == -2)
        eager_tiny_kernel<128><<<grid, 64, 0, stream>>>(rhs.view, in, n, cnt + 1, list, cnt,
                                                        ws.wd_ticks, out);
      else
        eager_tiny_kernel<256><<<grid, 64, 0, stream>>>(rhs.view, in, n, cnt + 1, list, cnt,
                                                        ws.wd_ticks, out);
    } else if (tier == -2)
      eager_bfs_kernel<64, false, 1><<<grid, 64, 0, stream>>>(rhs.view, in, none, n, cnt + 1,
                                                              list, cnt, 0, ws, out);
    else if (tier == -1)
      eager_bfs_kernel<64, false, 2><<<grid, 64, 0, stream>>>(rhs.view, in, none, n, cnt + 1,
                                                              list, cnt, 0, ws, out);
    else if (wave)
      eager_bfs_kernel<64, false><<<grid, 64, 0, stream>>>(rhs.view, in, none, n, cnt + 1, list,
                                                           cnt, 0, ws, out);
    else
      eager_bfs_kernel<kBfsWG, false><<<grid, kBfsWG, 0, stream>>>(rhs.view, in, none, n, cnt + 1,
                                                                   list, cnt, 0, ws, out);
    HIP_TRY(hipGetLastError());
    if (ws.prof) {  // phase profile: sums over workgroups, ticks at 100 MHz
      std::vector<unsigned long long> h((size_t)grid * 8);
      HIP_TRY(hipMemcpyAsync(h.data(), ws.prof, h.size() * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      unsigned long long sum[8] = {};
      for (size_t i = 0; i < h.size(); ++i) sum[i % 8] += h[i];
      std::fprintf(stderr,
                   "[bfs prof] tier %d grid %u wg %d items %llu | us/item: compose %.1f "
                   "fixpoint %.1f rounds %.1f tail %.1f | rounds/item %.1f active/round %.1f "
                   "members/round %.1f\n",
                   tier, grid, (wave || tier < 0) ? 64 : kBfsWG, sum[4], sum[0] / 100.0 / sum[4],
                   sum[1] / 100.0 / sum[4], sum[2] / 100.0 / sum[4], sum[3] / 100.0 / sum[4],
                   (double)sum[5] / sum[4], (double)sum[6] / std::max(1ull, sum[5]),
                   (double)sum[7] / std::max(1ull, sum[5]));
    }
    // strings that overflowed this tier move on to the next one
    collect_list_kernel<<<(count + 255) / 256, 256, 0, stream>>>(list, cnt, out.status,
                                                                 kPathOverflow, list2, cnt + 2);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&count, cnt + 2, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(cnt, cnt + 2, 4, hipMemcpyDeviceToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    std::swap(list, list2);
    if (tier == -2 && count0 >= 1024 && (uint64_t)count * 3 > (uint64_t)count0)
      rhs.tiny_eager_256.store(1, std::memory_order_relaxed);
    // the 128-tuple tier handed on nearly every string: skip the tiny tiers on this rhs
    if (tier == -2 && count0 >= 64 && (uint64_t)count * 10 > (uint64_t)count0 * 9 &&
        (uint64_t)(in.max_len + 1) * rhs.view.num_states > 16384)
      rhs.skip_tiny_eager.store(1, std::memory_order_relaxed);
  }
  return hipSuccess;
}

hipError_t DeviceEngine::compose_lattice(const DeviceFst& rhs, const GraphInput& lhs,
                                         HostLattice* lat, LaunchStats* stats,
                                         hipStream_t stream) {
  HIP_TRY(hipSetDevice(dev_));
  unsigned int* ctr = (unsigned int*)scratch(kCounter, kCounterBytes);
  if (!ctr) return hipErrorOutOfMemory;
  BatchOutDev none_out{};
  // First tier: 128K tuples, or the smallest one that holds every tuple the product can
  // have -- |lhs| x |rhs| per filter value in use (compose.zig: filter 1 needs an rhs input
  // epsilon, filter 2 an lhs output epsilon) -- so a large lattice does not first run
  // until it overflows a small tier (config 1: 781K tuples, 78 ms lost in tier 1).
  const uint64_t bound = (uint64_t)lhs.num_states * rhs.view.num_states *
                         (1u + (rhs.has_eps ? 1u : 0u) + (lhs.eps_out ? 1u : 0u));
  // The bound is trusted only up to 1M tuples: a large sparse rhs (a WeText-scale tagger,
  // 0.43 M states) makes it ~14 M for a 15-label utterance whose lattice has ~140 tuples,
  // and clearing that tier's tables cost 17.7 ms per fst_compose_frozen call; such lattices
  // start at the first tier and grow on overflow.
  int tier0 = 1;
  while (bound <= (1u << 20) && bfs_caps(tier0).ncap < bound &&
         bfs_caps(tier0 + 1).stride <= kBfsBudget && bfs_caps(tier0).ncap < (1u << 30))
    ++tier0;
  // One 1024-thread workgroup: the ~4,200 BFS levels of config 1 are ~190 tuples wide
  // (kernel 182 vs 214 ms with 256 threads).  FSTAMD_LATTICE_WG=256 for A/B runs.
  const char* lwg = std::getenv("FSTAMD_LATTICE_WG");
  const bool wg1k = !(lwg && std::strcmp(lwg, "256") == 0);
  for (int tier = tier0;; ++tier) {
    const BfsCaps c = bfs_caps(tier);
    if (c.stride > kBfsBudget) {
      lat->status = kPathOverflow;
      return hipSuccess;
    }
    BfsWs ws{};
    ws.slab = (uint8_t*)scratch(kBfsSlab, c.stride);
    ws.hdr = (uint32_t*)scratch(kBfsHdr, 8 * 4);
    if (!ws.slab || !ws.hdr) return hipErrorOutOfMemory;
    ws.stride = c.stride;
    ws.ncap = c.ncap;
    ws.acap = c.acap;
    ws.hcap = c.hcap;
    ws.lcap = c.lcap;
    ws.wd_ticks = watchdog_ticks();
    ws.lattice_only = 1;
    HIP_TRY(hipMemsetAsync(ctr, 0, 64, stream));
    if (stats) HIP_TRY(hipEventRecord(ev0_, stream));
    ChainInput none{};
    if (wg1k)
      eager_bfs_kernel<1024, true><<<1, 1024, 0, stream>>>(rhs.view, none, lhs, 1, ctr, nullptr,
                                                            nullptr, 1, ws, none_out);
    else
      eager_bfs_kernel<kBfsWG, true><<<1, kBfsWG, 0, stream>>>(rhs.view, none, lhs, 1, ctr,
                                                                nullptr, nullptr, 1, ws, none_out);
    HIP_TRY(hipGetLastError());
    if (stats) {
      HIP_TRY(hipEventRecord(ev1_, stream));
      HIP_TRY(finish_stats(ev0_, ev1_, stats));
      stats->engine = 2;
      stats->grid = 1;
      stats->launches = tier - tier0 + 1;
    }
    uint32_t hdr[8];
    HIP_TRY(copy_sync(hdr, ws.hdr, sizeof(hdr), hipMemcpyDeviceToHost, stream));
    lat->status = (int32_t)hdr[3];
    if (lat->status == kPathOverflow) continue;
    lat->n_nodes = hdr[0];
    lat->n_arcs = hdr[1];
    if (lat->status != kPathOk) return hipSuccess;
    // copy the lattice out of the slab (same carve as the kernel)
    const size_t N = lat->n_nodes, A = lat->n_arcs;
    lat->aoff.resize(N + 1);
    lat->nfin.resize(N);
    lat->anext.resize(A);
    lat->ail.resize(A);
    lat->aol.resize(A);
    lat->aw.resize(A);
    if (N == 0) {
      lat->aoff.assign(1, 0);
      return hipSuccess;
    }
    auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint8_t* p = ws.slab;
    const size_t o_hkey = 0, o_hval = o_hkey + r((size_t)c.hcap * 8),
                 o_nkey = o_hval + r((size_t)c.hcap * 4), o_aoff = o_nkey + r((size_t)c.ncap * 8),
                 o_lvl = o_aoff + r(((size_t)c.ncap + 1) * 4),
                 o_nd = o_lvl + r(((size_t)c.lcap + 2) * 4), o_nback = o_nd + r((size_t)c.ncap * 8),
                 o_nfin = o_nback + r((size_t)c.ncap * 8), o_anext = o_nfin + r((size_t)c.ncap * 8),
                 o_ail = o_anext + r((size_t)c.acap * 4), o_aol = o_ail + r((size_t)c.acap * 4),
                 o_aw = o_aol + r((size_t)c.acap * 4);
    // pinned host arrays: asynchronous DMAs, one synchronisation
    const auto d2h = [&](void* dst, const void* src, size_t b) {
      return hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, stream);
    };
    HIP_TRY(d2h(lat->aoff.data(), p + o_aoff, (N + 1) * 4));
    HIP_TRY(d2h(lat->nfin.data(), p + o_nfin, N * 8));
    if (A) {
      HIP_TRY(d2h(lat->anext.data(), p + o_anext, A * 4));
      HIP_TRY(d2h(lat->ail.data(), p + o_ail, A * 4));
      HIP_TRY(d2h(lat->aol.data(), p + o_aol, A * 4));
      HIP_TRY(d2h(lat->aw.data(), p + o_aw, A * 8));
    }
    return hipStreamSynchronize(stream);
  }
}

hipError_t DeviceEngine::shortest_path_graph(const GraphInput& g, uint32_t n,
                                             const BatchOutDev& out, LaunchStats* stats,
                                             hipStream_t stream, bool nonneg) {
  HIP_TRY(hipSetDevice(dev_));
  const uint32_t N = g.num_states;
  if (!nonneg) {  // negative weights: exact replay of the heap order, one lane
    uint32_t A = 0;
    if (N) HIP_TRY(copy_sync(&A, g.state_off + N, 4, hipMemcpyDeviceToHost, stream));
    const uint64_t hcap = (uint64_t)A + 1;
    const size_t nd_b = ((size_t)N * 16 + 255) & ~(size_t)255;
    const size_t st_b = ((size_t)N + 255) & ~(size_t)255;
    uint8_t* w = (uint8_t*)scratch(kBfsSlab, nd_b + st_b + hcap * sizeof(SpHeapEnt));
    if (!w) return hipErrorOutOfMemory;
    HIP_TRY(hipMemsetAsync(out.cursor, 0, 8, stream));
    BfsTables T{};
    T.aoff = const_cast<uint32_t*>(g.state_off);
    T.anext = const_cast<uint32_t*>(g.arc_next);
    T.ail = const_cast<uint32_t*>(g.arc_il);
    T.aol = const_cast<uint32_t*>(g.arc_ol);
    T.aw = const_cast<double*>(g.arc_w);
    T.nfin = const_cast<double*>(g.final_w);
    T.nd = (unsigned long long*)w;
    T.nback = (unsigned long long*)(w + (size_t)N * 8);
    if (stats) HIP_TRY(hipEventRecord(ev0_, stream));
    sp_replay_kernel<<<1, 64, 0, stream>>>(T, N, g.start, n, (SpHeapEnt*)(w + nd_b + st_b),
                                            hcap, w + nd_b, out, watchdog_ticks());
    HIP_TRY(hipGetLastError());
    if (stats) {
      HIP_TRY(hipEventRecord(ev1_, stream));
      HIP_TRY(finish_stats(ev0_, ev1_, stats));
      stats->engine = 6;
      stats->grid = 1;
      stats->launches = 1;
    }
    return hipStreamSynchronize(stream);
  }
  // work arrays: distances, back-pointers, stamps, settled flags, two frontiers, the
  // pending list (one entry per arc at most); the one "level" [0, N) and the distance
  // kernels' flags in the header
  const size_t n_b = ((size_t)N * 4 + 255) & ~(size_t)255;
  uint32_t A = 0;
  if (N) HIP_TRY(copy_sync(&A, g.state_off + N, 4, hipMemcpyDeviceToHost, stream));
  uint8_t* w = (uint8_t*)scratch(kBfsSlab, (size_t)N * 16 + 256 + 4 * n_b + ((size_t)A + 64) * 4);
  uint32_t* lv = (uint32_t*)scratch(kBfsHdr, 32);
  if (!w || !lv) return hipErrorOutOfMemory;
  const uint32_t lvh[8] = {0, N, 0, 0, 0, 0, 0, 0};  // [2..3]: have_dist, expired; [4..5] prof
  HIP_TRY(copy_sync(lv, lvh, 32, hipMemcpyHostToDevice, stream));
  uint32_t* mark = (uint32_t*)(w + (((size_t)N * 16 + 255) & ~(size_t)255));
  uint32_t* fa = (uint32_t*)((uint8_t*)mark + n_b);
  uint32_t* fb = (uint32_t*)((uint8_t*)fa + n_b);
  uint32_t* stl = (uint32_t*)((uint8_t*)fb + n_b);
  uint32_t* pend = (uint32_t*)((uint8_t*)stl + n_b);
  HIP_TRY(hipMemsetAsync(out.cursor, 0, 8, stream));
  BfsTables T{};
  T.aoff = const_cast<uint32_t*>(g.state_off);
  T.anext = const_cast<uint32_t*>(g.arc_next);
  T.ail = const_cast<uint32_t*>(g.arc_il);
  T.aol = const_cast<uint32_t*>(g.arc_ol);
  T.aw = const_cast<double*>(g.arc_w);
  T.nfin = const_cast<double*>(g.final_w);
  T.lvl = lv;
  T.nd = (unsigned long long*)w;
  T.nback = (unsigned long long*)(w + (size_t)N * 8);
  if (stats) HIP_TRY(hipEventRecord(ev0_, stream));
  // FSTAMD_SP_SWEEP=1: the Gauss-Seidel sweeps over every arc instead of the frontier
  const bool sweep = std::getenv("FSTAMD_SP_SWEEP") != nullptr;
  const bool hprof = std::getenv("FSTAMD_HOST_PROF") != nullptr;
  hipEvent_t em = nullptr;
  if (hprof) {
    HIP_TRY(hipEventCreate(&em));
    HIP_TRY(hipEventRecord(ev0_, stream));
  }
  // distances: settled in distance order (sp_settle_kernel); after more than
  // FSTAMD_SP_MAX_ADV (256) distinct distances, label correcting (sp_frontier_kernel)
  uint32_t sf[4] = {0, 0, 0, 0};  // fallback, expired, rounds, advances
  if (!sweep && g.start < N && n == 1) {
    const char* ma = std::getenv("FSTAMD_SP_MAX_ADV");
    const uint32_t max_adv = ma ? (uint32_t)std::strtoul(ma, nullptr, 10) : 256u;
    sp_settle_kernel<1024><<<1, 1024, 0, stream>>>(T, N, g.start, mark, stl, fa, fb, pend,
                                                    lv + 4, max_adv, watchdog_ticks());
    HIP_TRY(hipGetLastError());
    HIP_TRY(copy_sync(sf, lv + 4, 16, hipMemcpyDeviceToHost, stream));
    if (sf[1]) {  // its watchdog fired: the path reports INTERNAL
      const uint32_t one = 1;
      HIP_TRY(copy_sync(lv + 3, &one, 4, hipMemcpyHostToDevice, stream));
    } else if (sf[0]) {
      sp_frontier_kernel<1024><<<1, 1024, 0, stream>>>(T, N, g.start, mark, fa, fb, lv + 3,
                                                        watchdog_ticks());
    }
  }
  if (hprof) HIP_TRY(hipEventRecord(em, stream));
  sp_graph_kernel<1024><<<1, 1024, 0, stream>>>(
      T, N, g.start, n, out, watchdog_ticks(), sweep || g.start >= N || n != 1 ? nullptr : lv + 2);
  if (hprof) {
    HIP_TRY(hipEventRecord(ev1_, stream));
    HIP_TRY(hipEventSynchronize(ev1_));
    float a = 0.f, b = 0.f;
    HIP_TRY(hipEventElapsedTime(&a, ev0_, em));
    HIP_TRY(hipEventElapsedTime(&b, em, ev1_));
    std::fprintf(stderr, "[libfst_amd host] fst_shortest_path: distances %.2f ms (settle: %u "
                 "rounds, %u advances%s), back-pointers + best + path %.2f ms (%u states)\n",
                 a, sf[2], sf[3], sf[0] ? ", then label correcting" : "", b, N);
    HIP_TRY(hipEventDestroy(em));
  }
  HIP_TRY(hipGetLastError());
  if (stats) {
    HIP_TRY(hipEventRecord(ev1_, stream));
    HIP_TRY(finish_stats(ev0_, ev1_, stats));
    stats->engine = 2;
    stats->grid = 1;
    stats->launches = 1;
  }
  return hipStreamSynchronize(stream);
}

// ---------------------------------------------------------------------------------
// Stage -> stage projection (src/string.zig:60-97 printOutputString, then :24-50
// compileString: label = byte + 1 on both sides, so the next input labels are the
// path's non-epsilon olabels; a label > 256 is not a byte -- the reference's @intCast
// would trap -- and is reported instead).
// ---------------------------------------------------------------------------------
__global__ void project_count_kernel(BatchOutDev s, uint32_t num, uint64_t* counts,
                                     int32_t* proj_status, uint32_t* max_len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > num) return;
  if (i == num) {  // the scan's last element: offsets[num] = total
    counts[i] = 0;
    return;
  }
  int32_t ps = s.status[i];
  uint64_t c = 0;
  if (ps == kPathOk) {
    const uint64_t o = s.path_off[i];
    const uint32_t L = s.path_len[i];
    for (uint32_t k = 0; k < L; ++k) {
      const uint32_t ol = s.out_ol[o + k];
      if (ol > 256u) {
        ps = kPathUnsupported;
        break;
      }
      c += ol != kEpsilon;
    }
  }
  if (ps != kPathOk) c = 1;  // kDeadLabel
  counts[i] = c;
  proj_status[i] = ps;
  atomicMax(max_len, (uint32_t)c);
}

__global__ void project_write_kernel(BatchOutDev s, uint32_t num, const uint64_t* offsets,
                                     const int32_t* proj_status, uint32_t* labels) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num) return;
  uint64_t w = offsets[i];
  if (proj_status[i] != kPathOk) {
    labels[w] = kDeadLabel;
    return;
  }
  const uint64_t o = s.path_off[i];
  const uint32_t L = s.path_len[i];
  for (uint32_t k = 0; k < L; ++k) {
    const uint32_t ol = s.out_ol[o + k];
    if (ol != kEpsilon) labels[w++] = ol;
  }
}

hipError_t DeviceEngine::project_output(const BatchOutDev& stage, uint32_t num,
                                        uint32_t* next_labels, uint64_t* next_offsets,
                                        int32_t* proj_status, uint32_t* max_len,
                                        hipStream_t stream) {
  HIP_TRY(hipSetDevice(dev_));
  uint64_t* counts = (uint64_t*)scratch(kProjCount, ((size_t)num + 1) * 8 + 16);
  uint32_t* ml = (uint32_t*)scratch(kCounter, kCounterBytes) + 15;
  if (!counts || !ml) return hipErrorOutOfMemory;
  HIP_TRY(hipMemsetAsync(ml, 0, 4, stream));
  project_count_kernel<<<(num + 256) / 256, 256, 0, stream>>>(stage, num, counts, proj_status,
                                                             ml);
  HIP_TRY(hipGetLastError());
  size_t tbytes = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, counts, next_offsets, num + 1,
                                           stream));
  void* temp = scratch(kProjTemp, tbytes + 16);
  if (!temp) return hipErrorOutOfMemory;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(temp, tbytes, counts, next_offsets, num + 1, stream));
  project_write_kernel<<<(num + 255) / 256, 256, 0, stream>>>(stage, num, next_offsets,
                                                             proj_status, next_labels);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(max_len, ml, 4, hipMemcpyDeviceToHost, stream));
  return hipStreamSynchronize(stream);
}

__global__ void csr_count_kernel(BatchOutDev s, uint32_t num, const int32_t* fail,
                                 int32_t* status, uint64_t* counts, double* fin) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > num) return;
  if (i == num) {  // the scan's last element: offsets[num] = the total
    counts[num] = 0;
    return;
  }
  int32_t st = s.status[i];
  if (fail && fail[i] != kPathOk) st = fail[i];
  status[i] = st;
  const bool ok = st == kPathOk;
  counts[i] = ok ? s.path_len[i] : 0u;
  fin[i] = ok ? s.final_w[i] : w_zero();
}

// One wavefront per string (grid-stride): the lanes copy its arcs, coalesced on both sides.
// A path that would read past the arena or write past `out_cap` is not copied (an engine
// bug; the host sees the total exceed the arena and fails the call).
__global__ void __launch_bounds__(64) csr_gather_kernel(BatchOutDev s, uint32_t num,
                                                        const int32_t* status,
                                                        const uint64_t* offsets, uint32_t* il,
                                                        uint32_t* ol, double* w,
                                                        uint64_t out_cap) {
  for (uint32_t i = blockIdx.x; i < num; i += gridDim.x) {
    if (status[i] != kPathOk) continue;
    const uint64_t src = s.path_off[i], dst = offsets[i];
    const uint32_t L = s.path_len[i];
    if (dst + L > out_cap || src + L > s.arc_cap) continue;
    for (uint32_t k = threadIdx.x; k < L; k += 64) {
      il[dst + k] = s.out_il[src + k];
      ol[dst + k] = s.out_ol[src + k];
      w[dst + k] = s.out_w[src + k];
    }
  }
}

__global__ void merge_status_kernel(int32_t* fail, const int32_t* st, uint32_t num) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < num && fail[i] == kPathOk && st[i] != kPathOk) fail[i] = st[i];
}

hipError_t DeviceEngine::compact_paths(const BatchOutDev& s, uint32_t num, const int32_t* fail,
                                       int32_t* status, uint64_t* offsets, uint32_t* il,
                                       uint32_t* ol, double* w, double* fin, uint64_t out_cap,
                                       uint64_t* total, hipStream_t stream) {
  HIP_TRY(hipSetDevice(dev_));
  uint64_t* counts = (uint64_t*)scratch(kProjCount, ((size_t)num + 1) * 8 + 16);
  if (!counts) return hipErrorOutOfMemory;
  csr_count_kernel<<<(num + 256) / 256, 256, 0, stream>>>(s, num, fail, status, counts, fin);
  HIP_TRY(hipGetLastError());
  size_t tbytes = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, counts, offsets, num + 1, stream));
  void* temp = scratch(kProjTemp, tbytes + 16);
  if (!temp) return hipErrorOutOfMemory;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(temp, tbytes, counts, offsets, num + 1, stream));
  if (num) {
    const uint32_t grid = std::min<uint32_t>(num, (uint32_t)num_cus_ * 32);
    csr_gather_kernel<<<grid, 64, 0, stream>>>(s, num, status, offsets, il, ol, w, out_cap);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpyAsync(total, offsets + num, 8, hipMemcpyDeviceToHost, stream));
  return hipStreamSynchronize(stream);
}

hipError_t DeviceEngine::merge_status(int32_t* fail, const int32_t* st, uint32_t num,
                                      hipStream_t stream) {
  HIP_TRY(hipSetDevice(dev_));
  if (num) merge_status_kernel<<<(num + 255) / 256, 256, 0, stream>>>(fail, st, num);
  HIP_TRY(hipGetLastError());
  return hipSuccess;
}

hipError_t DeviceEngine::run_graph(const DeviceFst& rhs, const GraphInput& in, uint32_t n,
                                   int semantics, const BatchOutDev& out, hipStream_t stream,
                                   LaunchStats* stats) {
  HIP_TRY(hipSetDevice(dev_));
  if (semantics != 0) return hipErrorInvalidValue;
  unsigned int* counter = (unsigned int*)scratch(kCounter, kCounterBytes);
  if (!counter) return hipErrorOutOfMemory;
  HIP_TRY(hipMemsetAsync(counter, 0, 64, stream));
  HIP_TRY(hipMemsetAsync(out.cursor, 0, sizeof(unsigned long long), stream));
  LazyWs ws{};
  ws.ncap = next_pow2(std::max<uint32_t>(in.ncap, 1024));
  ws.hcap = ws.ncap * 2;
  ws.qcap = ws.ncap * 4;
  ws.gcap = next_pow2(std::max<uint32_t>(64, 2 * in.max_outdeg + 2));
  const uint32_t grid = 1;
  ws.hslot = (uint4*)scratch(kLzHash, (size_t)grid * ws.hcap * sizeof(uint4));
  ws.nkey = (unsigned long long*)scratch(kLzNkey, (size_t)grid * ws.ncap * 8);
  ws.ndist = (double*)scratch(kLzNdist, (size_t)grid * ws.ncap * 8);
  ws.nback = (uint4*)scratch(kLzNback, (size_t)grid * ws.ncap * 16);
  ws.nbw = (double*)scratch(kLzNbw, (size_t)grid * ws.ncap * 8);
  ws.qd = (double*)scratch(kLzQd, (size_t)grid * ws.qcap * 8);
  ws.qid = (uint32_t*)scratch(kLzQid, (size_t)grid * ws.qcap * 4);
  ws.gscratch = (uint4*)scratch(kLzG, (size_t)grid * ws.gcap * sizeof(uint4));
  if (!ws.hslot || !ws.nkey || !ws.ndist || !ws.nback || !ws.nbw || !ws.qd || !ws.qid ||
      !ws.gscratch)
    return hipErrorOutOfMemory;
  HIP_TRY(hipMemsetAsync(ws.hslot, 0, (size_t)grid * ws.hcap * sizeof(uint4), stream));
  lazy_hash_bytes_ = 0;  // force a clear before the next chain launch
  ws.stamp_base = 0;
  ws.max_pops = ws.qcap + 1;
  ws.wd_ticks = watchdog_ticks();
  ws.dbg = nullptr;
  if (stats) {
    stats->engine = 1;
    stats->grid = grid;
    stats->launches = 1;
    HIP_TRY(hipEventRecord(ev0_, stream));
  }
  ChainInput none{};
  none.num_strings = 1;
  lazy_wave_kernel<true><<<grid, 64, 0, stream>>>(rhs.view, none, in, n, counter, nullptr, 1, ws,
                                                  out);
  HIP_TRY(hipGetLastError());
  if (stats) {
    HIP_TRY(hipEventRecord(ev1_, stream));
    HIP_TRY(finish_stats(ev0_, ev1_, stats));
  }
  return hipSuccess;
}

}  // namespace fstamd
