// c_api.cpp -- the fst.h / fst_batch.h C ABI of libfst_amd.
//
// Handle tables, snapshots and pinning follow src/c-api.zig:105-271: u64 handles
// (generation << 32 | slot), one global mutex for table bookkeeping only, compute
// outside the lock on a cloned lhs, the frozen rhs pinned (a shared_ptr copy here)
// so that fst_free() during a call defers destruction.
//
// Every compose / shortest-path entry computes on the GPU; there is no CPU
// fallback.  If no HIP device is usable the entry fails (FST_INVALID_HANDLE /
// FST_INVALID_ARG) and, once per process, says why on stderr.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <thread>
#include <vector>

#include "../../include/fst_batch.h"
#include "device_engine.hpp"
#include "host_fst.hpp"

using namespace fstamd;

namespace {

constexpr uint64_t kInvalid = UINT64_MAX;

// Handle tables (src/c-api.zig:132-271), sharded: a handle's low bits name one of kShards
// shards, each with its own reader-writer lock over its slots AND the contents of the
// objects they hold.  Queries take their shard shared, edits exclusive; threads working on
// their own handles (concurrent compose calls reading their results arc by arc) do not meet
// on one lock -- one table-wide lock cost a third of the calls/s at 256 threads.
template <class T>
class HandleTable {
 public:
  static constexpr uint32_t kShards = 64;
  using SharedLock = std::shared_lock<std::shared_mutex>;
  using ExclusiveLock = std::unique_lock<std::shared_mutex>;

  uint64_t insert(std::shared_ptr<T> p) {
    // a thread fills one shard (its own, by arrival order): inserts from many threads spread
    static std::atomic<uint32_t> next{0};
    thread_local uint32_t mine = next.fetch_add(1, std::memory_order_relaxed) % kShards;
    Shard& sh = shards_[mine];
    ExclusiveLock g(sh.mu);
    uint32_t local;
    if (!sh.free.empty()) {
      local = sh.free.back();
      sh.free.pop_back();
      if (++sh.gen[local] == 0) sh.gen[local] = 1;
      sh.slots[local] = std::move(p);
    } else {
      local = (uint32_t)sh.slots.size();
      if ((uint64_t)local * kShards + mine >= 0xFFFFFFFFull) return kInvalid;
      sh.slots.push_back(std::move(p));
      sh.gen.push_back(1);
    }
    return ((uint64_t)sh.gen[local] << 32) | (local * kShards + mine);
  }
  // the lock a query (shared) or an edit (exclusive) of handle h holds around get_locked
  SharedLock lock_shared(uint64_t h) const { return SharedLock(shard(h).mu); }
  ExclusiveLock lock(uint64_t h) const { return ExclusiveLock(shard(h).mu); }
  // the object of h, or null; the caller holds lock_shared(h) or lock(h)
  T* get_locked(uint64_t h) const {
    if (h == kInvalid) return nullptr;
    const uint32_t g = (uint32_t)(h >> 32), idx = (uint32_t)h;
    if (g == 0 || idx == 0xFFFFFFFFu) return nullptr;
    const Shard& sh = shard(h);
    const uint32_t local = idx / kShards;
    if (local >= sh.slots.size() || sh.gen[local] != g) return nullptr;
    return sh.slots[local].get();
  }
  // get/pin: a shared_ptr copy keeps the object alive outside the lock
  std::shared_ptr<T> get(uint64_t h) const {
    SharedLock g = lock_shared(h);
    if (!get_locked(h)) return nullptr;
    return shard(h).slots[(uint32_t)h / kShards];
  }
  bool remove(uint64_t h) {
    ExclusiveLock g = lock(h);
    if (!get_locked(h)) return false;
    Shard& sh = shard(h);
    const uint32_t local = (uint32_t)h / kShards;
    sh.slots[local].reset();
    if (++sh.gen[local] == 0) sh.gen[local] = 1;  // invalidateSlot
    sh.free.push_back(local);
    return true;
  }
  void clear() {
    for (Shard& sh : shards_) {
      ExclusiveLock g(sh.mu);
      sh.slots.clear();
      sh.gen.clear();
      sh.free.clear();
    }
  }

 private:
  struct alignas(64) Shard {
    mutable std::shared_mutex mu;
    std::vector<std::shared_ptr<T>> slots;
    std::vector<uint32_t> gen;
    std::vector<uint32_t> free;
  };
  Shard& shard(uint64_t h) { return shards_[(uint32_t)h % kShards]; }
  const Shard& shard(uint64_t h) const { return shards_[(uint32_t)h % kShards]; }
  Shard shards_[kShards];
};

HandleTable<MutableFst> g_mut;
HandleTable<FrozenFst> g_fst;

thread_local LaunchStats t_last_stats;

bool trace_enabled() {  // LIBFST_TRACE_COMPOSE, src/c-api.zig:55-64
  static const bool on = std::getenv("LIBFST_TRACE_COMPOSE") != nullptr;
  return on;
}

void trace(const char* tag, uint64_t a, uint64_t b, size_t in_s, size_t in_a, size_t out_s,
           size_t out_a, double us, double kernel_ms) {
  if (!trace_enabled()) return;
  std::fprintf(stderr,
               "[libfst] %s op=fst_compose_frozen a=%llu b=%llu in_states=%zu in_arcs=%zu "
               "out_states=%zu out_arcs=%zu elapsed_us=%lld kernel_us=%lld\n",
               tag, (unsigned long long)a, (unsigned long long)b, in_s, in_a, out_s, out_a,
               (long long)us, (long long)(kernel_ms * 1000.0));
}

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  return dev;
}

// Tests only: FSTAMD_FAULT_INJECT=<site> makes the named error branch fire after its work
// is in flight on the GPU (tests/test_gpu_error_paths.py: the buffers a failing call hands
// back to the pools must not still be in use by its copies or kernels).
bool fault_inject(const char* site) {
  const char* e = std::getenv("FSTAMD_FAULT_INJECT");
  return e && std::strcmp(e, site) == 0;
}

bool gpu_available() {
  static int ok = -1;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (ok < 0) {
    int n = 0;
    ok = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
    if (!ok)
      std::fprintf(stderr,
                   "[libfst_amd] no usable HIP device: compose/shortest-path entries fail "
                   "(there is no CPU fallback)\n");
  }
  return ok == 1;
}

// Device buffers of the batch calls come from a per-process pool of power-of-two blocks:
// hipMalloc / hipFree of tens of MB per call (inputs, arena, CSR results) cost up to
// ~20 ms of host time a call, and hipFree synchronises the device.  Every DevBuf user
// synchronises before the buffer goes back, so a block is never reused while a kernel
// still runs on it.  Blocks beyond kPoolMax bytes held are freed instead; fst_teardown
// empties the pool.
// Blocks above kPoolMaxBlock (multi-GB path arenas) are never cached: they would hold HBM
// the dense replay sizes its waves from (hipMemGetInfo).  A failed hipMalloc releases the
// device's cached blocks and retries once, so cached blocks of other size classes can never
// turn into an FST_OOM.
constexpr size_t kPoolMax = 8ull << 30;
constexpr size_t kPoolMaxBlock = 1ull << 30;
struct BufPool {
  std::mutex mu;
  std::multimap<std::pair<int, size_t>, void*> free;
  size_t held = 0;
};
BufPool& buf_pool() {
  static BufPool* p = new BufPool;  // never destroyed: DevBufs may outlive static teardown
  return *p;
}
// Frees the cached blocks of device `dev` (every device when dev < 0); the calling
// thread's current device is restored.
void pool_release(int dev) {
  BufPool& P = buf_pool();
  // the blocks leave the pool under the lock; hipFree (it synchronises the device) runs
  // after it, so other threads' DevBuf allocations never wait for a running kernel here
  std::vector<std::pair<int, void*>> drop;
  {
    std::lock_guard<std::mutex> g(P.mu);
    for (auto it = P.free.begin(); it != P.free.end();) {
      if (dev >= 0 && it->first.first != dev) {
        ++it;
        continue;
      }
      drop.emplace_back(it->first.first, it->second);
      P.held -= it->first.second;
      it = P.free.erase(it);
    }
  }
  if (drop.empty()) return;
  int cur = 0;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  for (auto& [d, p] : drop) {
    (void)hipSetDevice(d);
    (void)hipFree(p);
  }
  if (have_cur) (void)hipSetDevice(cur);
}
void pool_clear() { pool_release(-1); }

// RAII device buffer (pooled)
struct DevBuf {
  void* p = nullptr;
  size_t cls = 0;
  int dev = 0;
  explicit DevBuf(size_t n) {
    cls = 4096;
    while (cls < n) cls <<= 1;
    if (hipGetDevice(&dev) != hipSuccess) return;
    BufPool& P = buf_pool();
    {
      std::lock_guard<std::mutex> g(P.mu);
      auto it = P.free.find({dev, cls});
      if (it != P.free.end()) {
        p = it->second;
        P.free.erase(it);
        P.held -= cls;
        return;
      }
    }
    if (hipMalloc(&p, cls) == hipSuccess) return;
    p = nullptr;
    (void)hipGetLastError();
    pool_release(dev);  // cached blocks of other classes back to the device, then retry
    if (hipMalloc(&p, cls) == hipSuccess) return;
    (void)hipGetLastError();
    DeviceEngine::trim_idle(dev);  // and the idle engines' workspaces
    (void)hipSetDevice(dev);
    if (hipMalloc(&p, cls) != hipSuccess) p = nullptr;
  }
  ~DevBuf() {
    if (!p) return;
    BufPool& P = buf_pool();
    std::lock_guard<std::mutex> g(P.mu);
    if (cls <= kPoolMaxBlock && P.held + cls <= kPoolMax) {
      P.free.insert({{dev, cls}, p});
      P.held += cls;
    } else {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      (void)hipSetDevice(cur);
    }
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

// Result arrays of the batch entries (FstBatchResult) come from a pool of pinned host
// blocks: the device writes them by DMA, with no staging through the runtime's bounce
// buffers and no page faults on freshly malloc'd pages every call (config 4 returns ~50 MB
// of paths per 64 K utterances).  fst_batch_result_free gives them back; beyond
// kPinPoolMax held they are freed.  A failed pinned allocation falls back to malloc.
constexpr size_t kPinPoolMax = 4ull << 30;
struct PinPool {
  std::mutex mu;
  std::multimap<size_t, void*> free;       // size class -> pinned block
  std::map<void*, std::pair<size_t, bool>> live;  // block -> (size class, pinned)
  size_t held = 0;
};
PinPool& pin_pool() {
  static PinPool* p = new PinPool;  // never destroyed: results may outlive static teardown
  return *p;
}
void* pin_alloc(size_t n) {
  size_t c = 4096;
  while (c < n) c <<= 1;
  PinPool& P = pin_pool();
  std::lock_guard<std::mutex> g(P.mu);
  auto it = P.free.find(c);
  if (it != P.free.end()) {
    void* p = it->second;
    P.free.erase(it);
    P.held -= c;
    P.live[p] = {c, true};
    return p;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, c, hipHostMallocDefault) == hipSuccess && p) {
    P.live[p] = {c, true};
    return p;
  }
  p = std::malloc(c);
  if (p) P.live[p] = {c, false};
  return p;
}
void pin_release(void* p) {
  if (!p) return;
  PinPool& P = pin_pool();
  std::lock_guard<std::mutex> g(P.mu);
  auto it = P.live.find(p);
  if (it == P.live.end()) return;  // not ours (never happens through the API)
  const size_t c = it->second.first;
  const bool pinned = it->second.second;
  P.live.erase(it);
  if (!pinned) {
    std::free(p);
  } else if (P.held + c <= kPinPoolMax) {
    P.free.insert({c, p});
    P.held += c;
  } else {
    (void)hipHostFree(p);
  }
}
bool pin_is_pinned(const void* p) {  // a pooled block from hipHostMalloc (device-mapped)
  PinPool& P = pin_pool();
  std::lock_guard<std::mutex> g(P.mu);
  auto it = P.live.find(const_cast<void*>(p));
  return it != P.live.end() && it->second.second;
}
void pin_pool_clear() {
  PinPool& P = pin_pool();
  std::lock_guard<std::mutex> g(P.mu);
  for (auto& kv : P.free) (void)hipHostFree(kv.second);
  P.free.clear();
  P.held = 0;
}

struct HostPaths {  // pinned: each array is one DMA (single calls download all of them)
  PinnedVec<int32_t> status;
  PinnedVec<uint32_t> len;
  PinnedVec<uint64_t> off;
  PinnedVec<double> fin;
  PinnedVec<uint32_t> il, ol;
  PinnedVec<double> w;
};

// Device outputs for `num` strings with `arc_cap` arena slots.
struct DevOut {
  DevBuf status, len, off, fin, il, ol, w, cursor;
  BatchOutDev v{};
  DevOut(uint32_t num, uint64_t arc_cap)
      : status(num * 4ull), len(num * 4ull), off(num * 8ull), fin(num * 8ull), il(arc_cap * 4),
        ol(arc_cap * 4), w(arc_cap * 8), cursor(8) {
    v.status = (int32_t*)status.p;
    v.path_len = (uint32_t*)len.p;
    v.path_off = (uint64_t*)off.p;
    v.final_w = (double*)fin.p;
    v.out_il = (uint32_t*)il.p;
    v.out_ol = (uint32_t*)ol.p;
    v.out_w = (double*)w.p;
    v.arc_cap = arc_cap;
    v.cursor = (unsigned long long*)cursor.p;
    v.work = nullptr;
  }
  bool ok() const {
    return status.p && len.p && off.p && fin.p && il.p && ol.p && w.p && cursor.p;
  }
  bool download(uint32_t num, HostPaths* h, hipStream_t stream) const {
    h->status.resize(num);
    h->len.resize(num);
    h->off.resize(num);
    h->fin.resize(num);
    unsigned long long used = 0;
    if (hipMemcpyAsync(&used, cursor.p, 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return false;
    used = std::min<unsigned long long>(used, v.arc_cap);
    h->il.resize(used);
    h->ol.resize(used);
    h->w.resize(used);
    // HostPaths is pinned: the copies run asynchronously, one synchronisation for all
    const auto d2h = [stream](void* dst, const void* src, size_t b) {
      return hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, stream) == hipSuccess;
    };
    if (num && !(d2h(h->status.data(), status.p, num * 4ull) && d2h(h->len.data(), len.p, num * 4ull) &&
                 d2h(h->off.data(), off.p, num * 8ull) && d2h(h->fin.data(), fin.p, num * 8ull)))
      return false;
    if (used && !(d2h(h->il.data(), il.p, used * 4) && d2h(h->ol.data(), ol.p, used * 4) &&
                  d2h(h->w.data(), w.p, used * 8)))
      return false;
    return hipStreamSynchronize(stream) == hipSuccess;
  }
};

// Result FST of one string: linear chain, or the empty FST (src/ops/*:382-400).
MutableFst chain_result(const HostPaths& h, uint32_t i) {
  MutableFst r;
  if (h.status[i] != kPathOk) return r;
  const uint32_t P = h.len[i];
  r.add_states(P + 1);
  r.set_start(0);
  r.set_final(P, h.fin[i]);
  for (uint32_t k = 0; k < P; ++k) {
    const uint64_t o = h.off[i] + k;
    r.add_arc(k, Arc{h.il[o], h.ol[o], h.w[o], k + 1});
  }
  return r;
}

// A MutableFst uploaded as CSR (arcs in insertion order): the lhs of the single-call
// compose entries, or the FST itself for fst_shortest_path.
// A MutableFst flattened to CSR on the host (arcs in insertion order), the device upload's
// source.  Large FSTs are flattened on host threads by state ranges (fst_shortest_path on a
// 10 M-arc lattice: a deep copy plus a push_back pass took ~150 ms).
// Host array without value-initialisation (the flatten writes every element, on the
// threads that first touch its pages).
// The arrays live in the pinned host pool (pin_alloc), so their upload is one DMA per
// array without the runtime's staging copies (config 1's lattice, 10 M arcs: ~200 MB).
template <class T>
struct RawVec {
  T* p = nullptr;
  size_t n = 0;
  RawVec() = default;
  RawVec(const RawVec&) = delete;
  RawVec& operator=(const RawVec&) = delete;
  ~RawVec() { pin_release(p); }
  void resize(size_t k) {
    pin_release(p);
    p = k ? (T*)pin_alloc(k * sizeof(T)) : nullptr;
    if (k && !p) throw std::bad_alloc();  // as new T[k] did
    n = k;
  }
  size_t size() const { return n; }
  T* data() { return p; }
  const T* data() const { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};

struct HostGraph {
  std::vector<uint32_t> soff;
  RawVec<uint32_t> il, ol, nx;
  RawVec<double> w, fin;
  uint32_t start = kNoState, maxdeg = 0;
  bool nonneg = true;  // every arc and final weight >= +0.0 (no -0.0, no NaN)
  bool nan = false;    // some arc or final weight is NaN
  bool eps_out = false;

  explicit HostGraph(const MutableFst& a) {
    const uint32_t ns = (uint32_t)a.num_states();
    start = a.start();
    soff.assign(ns + 1, 0);
    fin.resize(ns);
    for (uint32_t s = 0; s < ns; ++s) {
      const uint32_t d = (uint32_t)a.num_arcs(s);
      soff[s + 1] = soff[s] + d;
      maxdeg = std::max(maxdeg, d);
    }
    const size_t na = soff[ns];
    il.resize(na);
    ol.resize(na);
    nx.resize(na);
    w.resize(na);
    auto neg = [](double x) { return x < 0.0 || std::isnan(x) || (x == 0.0 && std::signbit(x)); };
    const uint32_t nt = na < (1u << 18) ? 1u
                        : std::min<uint32_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<uint8_t> flags(nt, 0);  // per thread: 1 negative, 2 NaN, 4 output epsilon
    auto fill = [&](uint32_t t) {
      const uint32_t lo = (uint32_t)((uint64_t)ns * t / nt), hi = (uint32_t)((uint64_t)ns * (t + 1) / nt);
      uint8_t fl = 0;
      for (uint32_t s = lo; s < hi; ++s) {
        fin[s] = a.final_weight(s);
        if (neg(fin[s])) fl |= 1;
        if (std::isnan(fin[s])) fl |= 2;
        uint32_t k = soff[s];
        for (const Arc& x : a.arcs(s)) {
          il[k] = x.ilabel;
          ol[k] = x.olabel;
          w[k] = x.weight;
          nx[k] = x.nextstate;
          if (x.olabel == kEpsilon) fl |= 4;
          if (neg(x.weight)) fl |= 1;
          if (std::isnan(x.weight)) fl |= 2;
          ++k;
        }
      }
      flags[t] = fl;
    };
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < nt; ++t) th.emplace_back(fill, t);
    fill(0);
    for (auto& x : th) x.join();
    for (uint8_t fl : flags) {
      if (fl & 1) nonneg = false;
      if (fl & 2) nan = true;
      if (fl & 4) eps_out = true;
    }
  }
};

struct GraphUpload {
  DevBuf off, il, ol, w, nx, fin;
  GraphInput g{};
  bool ok = false;
  bool nonneg = true;
  bool nan = false;
  // Uploads on `stream` (the call's engine stream) and waits for them: the host arrays may
  // be a temporary.
  GraphUpload(const MutableFst& a, hipStream_t stream) : GraphUpload(HostGraph(a), stream) {}
  GraphUpload(const HostGraph& h, hipStream_t stream)
      : off(h.soff.size() * 4ull), il(h.il.size() * 4), ol(h.ol.size() * 4), w(h.w.size() * 8),
        nx(h.nx.size() * 4), fin(h.fin.size() * 8ull) {
    nonneg = h.nonneg;
    nan = h.nan;
    const uint32_t ns = (uint32_t)h.fin.size();
    const size_t na = h.il.size();
    if (!off.p || !il.p || !ol.p || !w.p || !nx.p || !fin.p) return;
    const auto h2d = [stream](void* d, const void* src, size_t b) {
      return b == 0 || hipMemcpyAsync(d, src, b, hipMemcpyHostToDevice, stream) == hipSuccess;
    };
    bool good = h2d(off.p, h.soff.data(), (ns + 1) * 4ull) && h2d(il.p, h.il.data(), na * 4) &&
                h2d(ol.p, h.ol.data(), na * 4) && h2d(w.p, h.w.data(), na * 8) &&
                h2d(nx.p, h.nx.data(), na * 4) && h2d(fin.p, h.fin.data(), ns * 8ull);
    good = hipStreamSynchronize(stream) == hipSuccess && good;
    g.state_off = (const uint32_t*)off.p;
    g.arc_il = (const uint32_t*)il.p;
    g.arc_ol = (const uint32_t*)ol.p;
    g.arc_w = (const double*)w.p;
    g.arc_next = (const uint32_t*)nx.p;
    g.final_w = (const double*)fin.p;
    g.num_states = ns;
    g.start = h.start;
    g.max_outdeg = h.maxdeg;
    g.eps_out = h.eps_out ? 1u : 0u;
    ok = good;
  }
};

// A single-call lhs that is exactly a compileString acceptor (src/string.zig:24-50: states
// 0..L, arc k = (c, c, One, k + 1), final(L) = One, no other final) is the batch API's chain
// input: its labels.  Such a call runs the batch engines on one string (the layered pull
// tiers, the dense replay), not the general-lhs hashed replay: 1^64 on the metric rhs took
// 93 ms there (one wave popping 8,385 tuples through HBM tables).
bool as_chain(const MutableFst& a, std::vector<uint32_t>* labels) {
  const size_t ns = a.num_states();
  if (ns == 0 || a.start() != 0 || ns > (1u << 30)) return false;
  auto bits = [](double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
  };
  const uint32_t L = (uint32_t)(ns - 1);
  labels->resize(L);
  for (uint32_t k = 0; k <= L; ++k) {
    const auto& arcs = a.arcs(k);
    if (k == L) {
      if (!arcs.empty() || bits(a.final_weight(k)) != bits(w_one())) return false;
      break;
    }
    if (arcs.size() != 1 || !std::isinf(a.final_weight(k)) || a.final_weight(k) < 0) return false;
    const Arc& x = arcs[0];
    if (x.nextstate != k + 1 || x.ilabel != x.olabel || bits(x.weight) != bits(w_one()))
      return false;
    (*labels)[k] = x.ilabel;
  }
  return true;
}

// Lazy 1-best of one general lhs on the GPU (single-call C ABI path).
int run_lazy_single(const MutableFst& a, FrozenFst& b, uint32_t n, MutableFst* result,
                    double* kernel_ms) {
  const int dev = current_device();
  if (dev < 0) return -1;
  DeviceFst* D = b.device(dev);
  if (!D) return -1;
  DeviceEngine::Lease E = DeviceEngine::acquire(dev);
  if (!E) return -1;
  const hipStream_t stream = E.stream();
  GraphUpload up(a, stream);
  if (!up.ok) return -1;
  GraphInput g = up.g;
  // Grow the tuple capacity on overflow (the reference has no limit but memory).
  for (uint32_t ncap = 1u << 14; ncap <= (1u << 26); ncap <<= 2) {
    g.ncap = ncap;
    const uint64_t arc_cap = std::max<uint64_t>(ncap, 1024);
    DevOut out(1, arc_cap);
    if (!out.ok()) return -1;
    LaunchStats st;
    if (E->run_graph(*D, g, n, 0, out.v, stream, &st) != hipSuccess) return -1;
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    HostPaths h;
    if (!out.download(1, &h, stream)) return -1;
    t_last_stats = st;
    if (kernel_ms) *kernel_ms = st.kernel_ms;
    const int32_t s = h.status[0];
    if (s == kPathOverflow || s == kPathOutputFull) continue;
    if (s == kPathErrorN) return 2;
    if (s == kPathCycle) return 3;
    *result = chain_result(h, 0);  // OK or EMPTY
    return 0;
  }
  return -1;
}

FstError run_chain_batch_dev(DeviceEngine::Lease& E, DeviceFst& D, const ChainInput& in,
                             uint64_t total_labels, uint32_t n, int semantics, HostPaths* h,
                             std::unique_ptr<DevOut>* keep);

// Chain batch on the GPU from host arrays; fills `h` in input order.
// FSTAMD_HOST_PROF=1: wall time per host phase of the batch calls, printed to stderr at
// the end of each call (where a host API call spends its time beside the kernels).
struct HostProf {
  bool on = std::getenv("FSTAMD_HOST_PROF") != nullptr;
  double ms[8] = {};  // inputs H2D, output alloc, engine + sync, download, project, result
  int runs = 0;       // engine runs (a full arena reruns the batch with 4x the arcs)
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(int i) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    ms[i] += std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
  }
  void print(const char* what) const {
    if (!on) return;
    std::fprintf(stderr,
                 "[libfst_amd host] %s: inputs %.2f alloc %.2f engine %.2f download %.2f "
                 "project %.2f result %.2f ms (engine: %d launch(es))\n",
                 what, ms[0], ms[1], ms[2], ms[3], ms[4], ms[5], runs);
  }
};
thread_local HostProf* t_prof = nullptr;

// ---- Small batches: the coalesced single calls (one utterance each) and small host
// batches.  Per call the regular path costs ~10 uploads / downloads / synchronisations of
// ~10-25 us each beside a ~160 us kernel (WeText-scale tagger, profiles/r05/s2): here the
// inputs go up in one copy from one pinned block, the outputs live in one device block
// that comes down in one copy (the whole arena: it is small), and the only host waits are
// the engines' own routing reads and that final download.  A result the arena could not
// hold (OUTPUT_FULL) reruns on the regular path.
constexpr uint64_t kSmallLabels = 1u << 16;
constexpr uint32_t kSmallStrings = 1u << 12;
constexpr int kSmallRetry = -2;

int run_small_batch(DeviceEngine::Lease& E, DeviceFst& D, const uint32_t* labels,
                    const uint64_t* offsets, uint32_t num, uint64_t total, uint32_t max_len,
                    uint32_t n, int semantics, HostPaths* h) {
  const hipStream_t stream = E.stream();
  const uint64_t cap = std::max<uint64_t>((D.has_eps ? 4 : 1) * total + 16, 1024);
  auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
  // device block: inputs [offsets | labels], then outputs [status | len | off | fin |
  // cursor | il | ol | w], each region 256-B aligned
  const uint64_t o_off = 0, o_lab = al((num + 1) * 8ull), in_bytes = o_lab + total * 4;
  const uint64_t o_st = al(in_bytes), o_len = o_st + al(num * 4ull), o_po = o_len + al(num * 4ull),
                 o_fin = o_po + al(num * 8ull), o_cur = o_fin + al(num * 8ull),
                 o_il = o_cur + 256, o_ol = o_il + al(cap * 4), o_w = o_ol + al(cap * 4),
                 end = o_w + cap * 8;
  DevBuf blk(end);
  PinnedVec<uint8_t> hin(in_bytes), hout(end - o_st);
  if (!blk.p) return FST_OOM;
  // every return before the final synchronisation drains the stream first: `blk`, `hin`
  // and `hout` go back to their pools on return, and an upload, a kernel (run_chain can
  // fail after launching some) or the download may still be using them
  struct Drain {
    hipStream_t s;
    bool done = false;
    ~Drain() {
      if (!done) (void)hipStreamSynchronize(s);
    }
  } drain{stream};
  uint64_t* ho = (uint64_t*)(hin.data() + o_off);
  for (uint32_t i = 0; i <= num; ++i) ho[i] = offsets[i] - offsets[0];
  if (total) std::memcpy(hin.data() + o_lab, labels + offsets[0], total * 4);
  uint8_t* p = (uint8_t*)blk.p;
  if (hipMemcpyAsync(p, hin.data(), in_bytes, hipMemcpyHostToDevice, stream) != hipSuccess)
    return FST_OOM;
  ChainInput in{(const uint32_t*)(p + o_lab), (const uint64_t*)(p + o_off), num, max_len};
  BatchOutDev v{(int32_t*)(p + o_st), (uint32_t*)(p + o_len), (uint64_t*)(p + o_po),
                (double*)(p + o_fin), (uint32_t*)(p + o_il), (uint32_t*)(p + o_ol),
                (double*)(p + o_w), cap, (unsigned long long*)(p + o_cur), nullptr};
  if (t_prof) t_prof->lap(0);
  LaunchStats st;
  st.defer = true;  // (kernel time read after the download's synchronisation)
  const bool launched = E->run_chain(D, in, n, semantics, v, stream, &st) == hipSuccess &&
                        !fault_inject("small_after_launch");
  if (!launched ||
      hipMemcpyAsync(hout.data(), p + o_st, end - o_st, hipMemcpyDeviceToHost, stream) !=
          hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return FST_OOM;
  drain.done = true;
  (void)E->finish_deferred(&st);
  t_last_stats = st;
  if (t_prof) {
    t_prof->lap(2);
    ++t_prof->runs;
  }
  const uint8_t* q = hout.data() - o_st;  // (offsets below are block offsets)
  const int32_t* status = (const int32_t*)(q + o_st);
  for (uint32_t i = 0; i < num; ++i)
    if (status[i] == kPathOutputFull) return kSmallRetry;
  const uint64_t used = std::min<uint64_t>(*(const uint64_t*)(q + o_cur), cap);
  h->status.resize(num);
  h->len.resize(num);
  h->off.resize(num);
  h->fin.resize(num);
  h->il.resize(used);
  h->ol.resize(used);
  h->w.resize(used);
  std::memcpy(h->status.data(), status, num * 4ull);
  std::memcpy(h->len.data(), q + o_len, num * 4ull);
  std::memcpy(h->off.data(), q + o_po, num * 8ull);
  std::memcpy(h->fin.data(), q + o_fin, num * 8ull);
  if (used) {
    std::memcpy(h->il.data(), q + o_il, used * 4);
    std::memcpy(h->ol.data(), q + o_ol, used * 4);
    std::memcpy(h->w.data(), q + o_w, used * 8);
  }
  if (t_prof) t_prof->lap(3);
  return FST_OK;
}

// The call runs on the engine `E` leases (its stream; E->dev() is the device).
FstError run_chain_batch_host(DeviceEngine::Lease& E, FrozenFst& b, const uint32_t* labels,
                              const uint64_t* offsets, uint32_t num, uint32_t n, int semantics,
                              HostPaths* h, std::unique_ptr<DevOut>* keep = nullptr) {
  const int dev = E->dev();
  if (hipSetDevice(dev) != hipSuccess) return FST_INVALID_ARG;
  DeviceFst* D = b.device(dev);
  if (!D) return FST_OOM;
  const hipStream_t stream = E.stream();
  const uint64_t total = num ? offsets[num] - offsets[0] : 0;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < num; ++i)
    max_len = std::max<uint32_t>(max_len, (uint32_t)(offsets[i + 1] - offsets[i]));
  if (!keep && num && total <= kSmallLabels && num <= kSmallStrings) {
    const int r = run_small_batch(E, *D, labels, offsets, num, total, max_len, n, semantics, h);
    if (r != kSmallRetry) return (FstError)r;
  }
  std::vector<uint64_t> rebased(num + 1);
  for (uint32_t i = 0; i <= num; ++i) rebased[i] = offsets[i] - offsets[0];
  DevBuf d_lab(total * 4), d_off((num + 1) * 8ull);
  if (!d_lab.p || !d_off.p) return FST_OOM;
  // (pageable sources: hipMemcpyAsync stages them before it returns)
  if (total && hipMemcpyAsync(d_lab.p, labels + offsets[0], total * 4, hipMemcpyHostToDevice,
                              stream) != hipSuccess)
    return FST_OOM;
  if (hipMemcpyAsync(d_off.p, rebased.data(), (num + 1) * 8ull, hipMemcpyHostToDevice, stream) !=
      hipSuccess)
    return FST_OOM;
  ChainInput in{(const uint32_t*)d_lab.p, (const uint64_t*)d_off.p, num, max_len};
  if (t_prof) t_prof->lap(0);
  return run_chain_batch_dev(E, *D, in, total, n, semantics, h, keep);
}

// ---- Host batches in shards (one device, or several: FST_BATCH_DEVICES) ---------------
// A shard is strings [s0, s1) of the caller's arrays on one device: computed on an engine
// lease (its device outputs kept), compacted to CSR on the device (count, scan, gather:
// DeviceEngine::compact_paths), then downloaded straight into the caller's result at the
// shard's string and arc offsets.
struct Shard {
  int dev = 0;
  uint32_t s0 = 0, s1 = 0;
  DeviceEngine::Lease E;
  std::unique_ptr<DevOut> keep;
  std::unique_ptr<DevBuf> fail;  // pipelines: the first failing stage per string
  std::unique_ptr<DevBuf> st, off, fin, il, ol, w;
  uint64_t tot = 0;
  FstError err = FST_OK;
  LaunchStats stats;
};

FstError shard_compact(Shard& S) {
  const uint32_t num = S.s1 - S.s0;
  const hipStream_t stream = S.E.stream();
  const DevOut& o = *S.keep;
  unsigned long long used = 0;
  if (hipMemcpyAsync(&used, o.cursor.p, 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return FST_OOM;
  used = std::min<unsigned long long>(used, o.v.arc_cap);
  S.st = std::make_unique<DevBuf>(num * 4ull);
  S.off = std::make_unique<DevBuf>((num + 1ull) * 8);
  S.fin = std::make_unique<DevBuf>(num * 8ull);
  S.il = std::make_unique<DevBuf>(used * 4);
  S.ol = std::make_unique<DevBuf>(used * 4);
  S.w = std::make_unique<DevBuf>(used * 8);
  if (!S.st->p || !S.off->p || !S.fin->p || !S.il->p || !S.ol->p || !S.w->p) return FST_OOM;
  if (S.E->compact_paths(o.v, num, S.fail ? (const int32_t*)S.fail->p : nullptr,
                         (int32_t*)S.st->p, (uint64_t*)S.off->p, (uint32_t*)S.il->p,
                         (uint32_t*)S.ol->p, (double*)S.w->p, (double*)S.fin->p, used, &S.tot,
                         stream) != hipSuccess)
    return FST_OOM;
  if (S.tot > used) return FST_OOM;  // an engine bug (the gather wrote nothing past `used`)
  return FST_OK;
}

bool alloc_result(FstBatchResult* out, uint32_t num, uint64_t tot) {
  out->num_strings = num;
  out->total_arcs = tot;
  out->status = (int32_t*)pin_alloc(std::max<size_t>(num, 1) * 4);
  out->path_offsets = (uint64_t*)pin_alloc((num + 1ull) * 8);
  out->final_weights = (double*)pin_alloc(std::max<size_t>(num, 1) * 8);
  out->ilabels = (uint32_t*)pin_alloc(std::max<uint64_t>(tot, 1) * 4);
  out->olabels = (uint32_t*)pin_alloc(std::max<uint64_t>(tot, 1) * 4);
  out->weights = (double*)pin_alloc(std::max<uint64_t>(tot, 1) * 8);
  return out->status && out->path_offsets && out->final_weights && out->ilabels &&
         out->olabels && out->weights;
}

// D2H of a compacted shard into the (pinned) result: asynchronous DMAs on the shard's
// stream, one synchronisation, then its path offsets moved by the shard's first arc.
FstError shard_download(Shard& S, FstBatchResult* out, uint64_t arc_base) {
  const uint32_t num = S.s1 - S.s0;
  const hipStream_t stream = S.E.stream();
  const auto d2h = [stream](void* dst, const void* src, size_t b) {
    return b == 0 || hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, stream) == hipSuccess;
  };
  if (!(d2h(out->status + S.s0, S.st->p, num * 4ull) &&
        d2h(out->final_weights + S.s0, S.fin->p, num * 8ull) &&
        d2h(out->path_offsets + S.s0, S.off->p, num * 8ull) &&
        d2h(out->ilabels + arc_base, S.il->p, S.tot * 4) &&
        d2h(out->olabels + arc_base, S.ol->p, S.tot * 4) &&
        d2h(out->weights + arc_base, S.w->p, S.tot * 8)) ||
      hipStreamSynchronize(stream) != hipSuccess)
    return FST_OOM;
  if (arc_base)
    for (uint32_t i = S.s0; i < S.s1; ++i) out->path_offsets[i] += arc_base;
  return FST_OK;
}

// Gives the calling thread its current HIP device back when it goes out of scope.
struct DeviceRestore_ {
  int dev = -1;
  DeviceRestore_() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceRestore_() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

// The same copies without the synchronisation or the offset fix-up, on `stream` (the
// pipelined host batch: the caller synchronises once at the end).
bool shard_download_async(Shard& S, FstBatchResult* out, uint64_t arc_base, hipStream_t stream) {
  const uint32_t num = S.s1 - S.s0;
  const auto d2h = [stream](void* dst, const void* src, size_t b) {
    return b == 0 || hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, stream) == hipSuccess;
  };
  return d2h(out->status + S.s0, S.st->p, num * 4ull) &&
         d2h(out->final_weights + S.s0, S.fin->p, num * 8ull) &&
         d2h(out->path_offsets + S.s0, S.off->p, num * 8ull) &&
         d2h(out->ilabels + arc_base, S.il->p, S.tot * 4) &&
         d2h(out->olabels + arc_base, S.ol->p, S.tot * 4) &&
         d2h(out->weights + arc_base, S.w->p, S.tot * 8);
}

// One device, one large batch on an rhs without input epsilons (a path has exactly L arcs,
// so the result is allocated before any shard finishes): the strings run as consecutive
// sub-shards on one engine, and the download of sub-shard j (a second stream, waiting for
// j's compaction only) runs while sub-shard j + 1 computes -- round 3's host batch ran its
// ~1 GB D2H after all the kernels.  Results are identical to the one-shard path.
FstError run_pipelined(int dev, FrozenFst& b, const uint32_t* labels, const uint64_t* offsets,
                       uint32_t num, uint32_t n, int semantics, uint32_t parts,
                       FstBatchResult* out) {
  if (hipSetDevice(dev) != hipSuccess) return FST_INVALID_ARG;
  DeviceFst* D = b.device(dev);
  if (!D) return FST_OOM;
  DeviceEngine::Lease E = DeviceEngine::acquire(dev);
  if (!E) return FST_INVALID_ARG;
  const hipStream_t stream = E.stream();
  struct CopyStream {  // the downloads' stream and the compaction events it waits for
    hipStream_t s = nullptr;
    std::vector<hipEvent_t> ev;
    ~CopyStream() {
      if (s) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
      }
      for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
  } C;
  if (hipStreamCreateWithFlags(&C.s, hipStreamNonBlocking) != hipSuccess) return FST_OOM;
  const uint64_t total = offsets[num] - offsets[0];
  std::vector<uint64_t> rebased(num + 1);
  for (uint32_t i = 0; i <= num; ++i) rebased[i] = offsets[i] - offsets[0];
  DevBuf d_lab(total * 4), d_off((num + 1) * 8ull);
  if (!d_lab.p || !d_off.p) return FST_OOM;
  if (hipMemcpyAsync(d_off.p, rebased.data(), (num + 1) * 8ull, hipMemcpyHostToDevice, stream) !=
      hipSuccess)
    return FST_OOM;
  std::vector<Shard> sh(parts);
  // every return drains the engine stream before the buffers its kernels use (d_lab, d_off,
  // the sub-shards' outputs: declared above, destroyed after this) go back to the pool
  struct SyncEngine {
    hipStream_t s;
    ~SyncEngine() { (void)hipStreamSynchronize(s); }
  } sync_engine{stream};
  for (uint32_t j = 0; j < parts; ++j) {
    sh[j].dev = dev;
    sh[j].s0 = (uint32_t)((uint64_t)num * j / parts);
    sh[j].s1 = (uint32_t)((uint64_t)num * (j + 1) / parts);
  }
  // The labels go up per sub-shard on a thread and stream of their own (a pageable source
  // is staged through pinned memory on the copying thread), so sub-shard j + 1's upload
  // runs while sub-shard j computes; the engine's stream waits on each upload's event.
  struct Uploader {
    hipStream_t s = nullptr;
    std::vector<hipEvent_t> ev;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t ready = 0;
    bool failed = false;
    std::thread th;
    ~Uploader() {
      if (th.joinable()) th.join();
      if (s) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
      }
      for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
  } U;
  if (hipStreamCreateWithFlags(&U.s, hipStreamNonBlocking) != hipSuccess) return FST_OOM;
  U.ev.assign(parts, nullptr);
  for (uint32_t j = 0; j < parts; ++j)
    if (hipEventCreateWithFlags(&U.ev[j], hipEventDisableTiming) != hipSuccess) return FST_OOM;
  U.th = std::thread([&, dev] {
    bool ok = hipSetDevice(dev) == hipSuccess;
    for (uint32_t j = 0; j < parts; ++j) {
      const uint64_t a = rebased[sh[j].s0], z = rebased[sh[j].s1];
      ok = ok && (z == a || hipMemcpyAsync((uint32_t*)d_lab.p + a, labels + offsets[0] + a,
                                           (z - a) * 4, hipMemcpyHostToDevice, U.s) == hipSuccess);
      ok = ok && hipEventRecord(U.ev[j], U.s) == hipSuccess;
      std::lock_guard<std::mutex> g(U.mu);
      if (!ok) {
        U.failed = true;
        U.cv.notify_all();
        return;
      }
      U.ready = j + 1;
      U.cv.notify_all();
    }
  });
  if (t_prof) t_prof->lap(0);
  if (!alloc_result(out, num, total)) return FST_OOM;  // paths of L arcs: <= total arcs
  // every return below first waits for the downloads in flight: on an error the caller
  // frees the result, whose pinned pages must not be written after that
  struct SyncOnExit {
    hipStream_t s;
    ~SyncOnExit() { (void)hipStreamSynchronize(s); }
  } sync_copies{C.s};
  uint64_t base = 0;
  for (uint32_t j = 0; j < parts; ++j) {
    Shard& S = sh[j];
    {
      std::unique_lock<std::mutex> g(U.mu);
      U.cv.wait(g, [&] { return U.failed || U.ready > j; });
      if (U.failed) return FST_OOM;
    }
    if (hipStreamWaitEvent(stream, U.ev[j], 0) != hipSuccess) return FST_OOM;
    uint32_t ml = 0;
    for (uint32_t i = S.s0; i < S.s1; ++i) ml = std::max<uint32_t>(ml, (uint32_t)(rebased[i + 1] - rebased[i]));
    // the sub-shard reads the whole upload: its offsets index the one label array
    ChainInput in{(const uint32_t*)d_lab.p, (const uint64_t*)d_off.p + S.s0, S.s1 - S.s0, ml};
    HostPaths h;
    if (FstError e = run_chain_batch_dev(E, *D, in, rebased[S.s1] - rebased[S.s0], n, semantics,
                                         &h, &S.keep);
        e != FST_OK)
      return e;
    S.stats = t_last_stats;
    S.E = std::move(E);  // shard_compact runs on the lease's stream
    const FstError ce = shard_compact(S);
    E = std::move(S.E);
    if (ce != FST_OK) return ce;
    if (base + S.tot > total) return FST_OOM;  // (a path longer than its string: impossible)
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return FST_OOM;
    C.ev.push_back(ev);
    if (hipEventRecord(ev, stream) != hipSuccess || hipStreamWaitEvent(C.s, ev, 0) != hipSuccess ||
        !shard_download_async(S, out, base, C.s))
      return FST_OOM;
    S.keep.reset();  // (the path arena: compaction copied what the download needs)
    base += S.tot;
  }
  if (hipStreamSynchronize(C.s) != hipSuccess) return FST_OOM;
  if (t_prof) t_prof->lap(3);
  uint64_t acc = 0;
  for (uint32_t j = 0; j < parts; ++j) {
    if (acc)
      for (uint32_t i = sh[j].s0; i < sh[j].s1; ++i) out->path_offsets[i] += acc;
    acc += sh[j].tot;
  }
  out->path_offsets[num] = base;
  out->total_arcs = base;
  LaunchStats agg = sh[0].stats;
  agg.kernel_ms = 0;
  agg.launches = 0;
  for (const Shard& S : sh) {
    agg.kernel_ms += S.stats.kernel_ms;
    agg.launches += S.stats.launches;
  }
  t_last_stats = agg;
  return FST_OK;
}

// ---- The streamed host batch --------------------------------------------------------
// One device, an rhs without input epsilons whose first tier is a pull tier (the metric's
// case: DeviceEngine::pull_first).  Every path then has exactly L arcs, so string i's path
// can sit at its own label offsets (BatchOutDev::slots) and the result's CSR offsets are
// the rebased input offsets.  The batch runs as a few parts of growing size (labels 1/43,
// 6/43, 36/43: each part's upload fits in the previous part's compute), alternating
// between two engines (streams), each part's launch waiting on its labels' upload event;
// the second engine's kernels fill the GPU while the first one's drain.  Meanwhile:
//  * other host threads copy the labels into result.ilabels (on an OK path il[k] = label
//    k: the result's ilabels are the input labels);
//  * the pull tier copies each finished path's olabels and weights into the (pinned,
//    device-mapped) result with whole-line stores as it goes (copy_out_paths): no D2H of
//    paths, no compaction pass on the device;
//  * statuses and final weights (12 B per string) come down per part;
//  * strings the pull tier handed on are finished by the later tiers in the device arena
//    (same slots) and downloaded after them; strings without a path are compacted out.
// No kernel ever waits on the host or another queue (only stream-ordered event waits).
// Labels read from host memory instead (zero-copy) measured 34.5 vs 30.6 ms per 1M metric
// strings: a PCIe read at every string's start.  Returns kStreamNotApplicable when the mode
// does not apply; the caller then takes the pipelined path.
constexpr int kStreamNotApplicable = -1;

struct StreamKit {  // per calling thread and device: the upload stream and its events
  hipStream_t up = nullptr;
  std::vector<hipEvent_t> ev;
  bool init(int dev) {
    if (!up && hipSetDevice(dev) == hipSuccess)
      (void)hipStreamCreateWithFlags(&up, hipStreamNonBlocking);
    return up != nullptr;
  }
  bool events(size_t n) {
    while (ev.size() < n) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
      ev.push_back(e);
    }
    return true;
  }
};

// StreamKits are leased per call from a process-wide pool per device (a kit per calling
// thread leaked a stream and its events for every thread that ever entered the batch
// API): the pool holds at most as many kits as calls ever ran at once on the device.
// (Never destroyed: the process may exit after the runtime's teardown.)
class KitLease {
 public:
  explicit KitLease(int dev) : dev_(dev) {
    Pool& P = pool();
    {
      std::lock_guard<std::mutex> g(P.mu);
      auto& v = P.free[dev];
      if (!v.empty()) {
        k_ = v.back();
        v.pop_back();
      }
    }
    if (!k_) k_ = new StreamKit;
    if (!k_->init(dev)) {
      give_back();
      k_ = nullptr;
    }
  }
  ~KitLease() { give_back(); }
  StreamKit* operator->() const { return k_; }
  explicit operator bool() const { return k_ != nullptr; }
  KitLease(const KitLease&) = delete;
  KitLease& operator=(const KitLease&) = delete;

 private:
  struct Pool {
    std::mutex mu;
    std::map<int, std::vector<StreamKit*>> free;
  };
  static Pool& pool() {
    static Pool* p = new Pool;
    return *p;
  }
  void give_back() {
    if (!k_) return;
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    P.free[dev_].push_back(k_);
    k_ = nullptr;
  }
  int dev_;
  StreamKit* k_ = nullptr;
};

// One shard of a streamed batch: strings [s0, s1) on device `dev`, everything but the
// result's final CSR compaction.  The result is already allocated and its offsets `poff`
// (the batch's rebased input offsets) filled; the shard's paths sit at those offsets (its
// labels at poff[s0] and up, its device buffers indexed from there), its statuses, final
// weights and pull-tier statuses at string s0 and up.
struct StreamShard {
  int dev = 0;
  uint32_t s0 = 0, s1 = 0;
  FstError err = FST_OK;
  double wall_ms = 0;
  uint32_t launches = 0;
};

FstError stream_shard(StreamShard& S, DeviceFst& D, const uint32_t* src, const uint64_t* poff,
                      uint32_t max_len, uint32_t n, int semantics, FstBatchResult* out,
                      int32_t* first_all, std::mutex* later_mu) {
  // the later tiers of the shards of one device run one shard at a time, each to the end of
  // its leases (declared after this lock, so released before it): the heavy replays size
  // their workspaces from the free HBM, which a concurrent shard's would have taken
  std::unique_lock<std::mutex> later_lock(*later_mu, std::defer_lock);
  const int dev = S.dev;
  if (hipSetDevice(dev) != hipSuccess) return FST_INVALID_ARG;
  const uint32_t num = S.s1 - S.s0;
  const uint64_t lbase = poff[S.s0], total = poff[S.s1] - lbase;
  if (num == 0) return FST_OK;
  KitLease K(dev);
  if (!K) return FST_OOM;
  const hipStream_t up = K->up;
  // the shard's offsets from its first label (shard 0 of the batch: poff itself)
  PinnedVec<uint64_t> loff_own(lbase ? num + 1 : 0);
  const uint64_t* loff = poff + S.s0;
  if (lbase) {
    for (uint32_t i = 0; i <= num; ++i) loff_own[i] = poff[S.s0 + i] - lbase;
    loff = loff_own.data();
  }
  const uint32_t* lsrc = src ? src + lbase : nullptr;
  uint32_t* const il_out = out->ilabels + lbase;
  struct Threads {  // joined on every return (declared after what they use)
    std::vector<std::thread> th;
    void join() {
      for (auto& t : th) t.join();
      th.clear();
    }
    ~Threads() { join(); }
  };

  // ---- parts: string ranges cut at these fractions of the labels (per mille; small
  // shards: one part): 1/43 and 7/43, so each part's upload fits in the previous part's
  // compute.  FSTAMD_STREAM_CUTS overrides (A/B, one box: "23,163" 30.9 ms per 1M metric
  // strings, "167" 31.2, "100,400" 31.0, "125" 31.5) ----
  std::vector<uint32_t> cut{0};
  if (total >= (1u << 22) && num >= (1u << 15)) {
    std::vector<uint64_t> pm{23, 163};
    if (const char* ce = std::getenv("FSTAMD_STREAM_CUTS")) {
      pm.clear();
      for (const char* q = ce; *q;) {
        char* e = nullptr;
        const unsigned long v = std::strtoul(q, &e, 10);
        if (e == q) break;
        if (v > 0 && v < 1000) pm.push_back(v);
        q = *e ? e + 1 : e;
      }
    }
    for (uint64_t f : pm) {
      const uint64_t want = total * f / 1000;
      const uint32_t i = (uint32_t)(std::upper_bound(loff, loff + num, want) - loff);
      if (i > cut.back() && i < num) cut.push_back(i);
    }
  }
  cut.push_back(num);
  const size_t parts = cut.size() - 1;
  if (parts > 64 || !K->events(parts)) return FST_OOM;  // one upload event a part

  // ---- engines and device buffers ----
  DeviceEngine::Lease EA = DeviceEngine::acquire(dev);
  if (!EA) return FST_INVALID_ARG;
  DeviceEngine::Lease EB;
  if (parts > 1) EB = DeviceEngine::try_acquire(dev);  // (none free: one engine in order)
  const hipStream_t sA = EA.stream(), sB = EB ? EB.stream() : nullptr;
  DevBuf d_lab(std::max<uint64_t>(total, 1) * 4), d_off((num + 1) * 8ull),
      d_first(std::max<size_t>(num, 1) * 4ull), d_ctr(64 * 4);  // item counter per part
  DevOut o(num, total + 4);
  if (!d_lab.p || !d_off.p || !d_first.p || !d_ctr.p || !o.ok()) return FST_OOM;
  // the arena's path arrays shifted so that each element shares its host twin's address
  // modulo 16 (the copy-out's 16-B units, kernels/device_common.hpp copy_out_paths)
  BatchOutDev vb = o.v;
  vb.out_il += lbase & 3u;
  vb.out_ol += lbase & 3u;
  vb.out_w += lbase & 1u;
  struct SyncAll {  // every return: no kernel or copy still uses the buffers or the result
    hipStream_t s[3];
    ~SyncAll() {
      for (hipStream_t x : s)
        if (x) (void)hipStreamSynchronize(x);
    }
  } sync_all{{up, sA, sB}};

  // ---- uploads (offsets, then each part's labels: one event per part) ----
  // Two ways to move the labels (FSTAMD_STREAM_STAGE): 0 = the runtime stages the pageable
  // source itself while other threads copy it into the result's ilabels (the labels cross
  // host DRAM twice); 1 = threads copy each chunk into the result's (pinned) ilabels and
  // the chunk's DMA reads it from there (once).
  const char* stage_env = std::getenv("FSTAMD_STREAM_STAGE");
  const int stage_mode = stage_env ? std::atoi(stage_env) : 0;
  struct Ready {
    std::mutex mu;
    std::condition_variable cv;
    size_t n = 0;
    bool failed = false;
  } R;
  Threads Th;
  Th.th.emplace_back([&] {
    // (the fills first, on the idle GPU: every string INTERNAL until a tier finishes it,
    // the parts' item counters zero; the parts wait on events recorded after them)
    bool ok = hipSetDevice(dev) == hipSuccess &&
              hipMemsetD32Async((hipDeviceptr_t)o.status.p, kPathInternal, num, up) == hipSuccess &&
              hipMemsetD32Async((hipDeviceptr_t)d_first.p, kPathInternal, num, up) == hipSuccess &&
              hipMemsetAsync(d_ctr.p, 0, 64 * 4, up) == hipSuccess &&
              hipMemcpyAsync(d_off.p, loff, (num + 1) * 8ull, hipMemcpyHostToDevice, up) ==
                  hipSuccess;
    constexpr uint64_t kChunk = 1ull << 21;  // labels per staged chunk (8 MB)
    for (size_t p = 0; p < parts && ok; ++p) {
      const uint64_t a = loff[cut[p]], z = loff[cut[p + 1]];
      if (stage_mode == 1) {
        for (uint64_t c = a; c < z && ok; c += kChunk) {
          const uint64_t e = std::min(z, c + kChunk), w = e - c;
          const uint64_t T = w >= (1u << 19) ? 4 : 1;
          std::vector<std::thread> cp;
          for (uint64_t t = 1; t < T; ++t)
            cp.emplace_back([&, t, T] {
              std::memcpy(il_out + c + w * t / T, lsrc + c + w * t / T,
                          (w * (t + 1) / T - w * t / T) * 4);
            });
          std::memcpy(il_out + c, lsrc + c, (w / T) * 4);
          for (auto& x : cp) x.join();
          ok = hipMemcpyAsync((uint32_t*)d_lab.p + c, il_out + c, w * 4, hipMemcpyHostToDevice,
                              up) == hipSuccess;
        }
      } else {
        // (a pageable source is staged through pinned memory before this returns)
        ok = z == a || hipMemcpyAsync((uint32_t*)d_lab.p + a, lsrc + a, (z - a) * 4,
                                      hipMemcpyHostToDevice, up) == hipSuccess;
      }
      ok = ok && hipEventRecord(K->ev[p], up) == hipSuccess;
      std::lock_guard<std::mutex> g(R.mu);
      if (ok) R.n = p + 1;
      R.cv.notify_all();
    }
    std::lock_guard<std::mutex> g(R.mu);
    if (!ok) R.failed = true;
    R.cv.notify_all();
  });
  if (stage_mode != 1) {
    // the result's ilabels, once the uploads are staged: the runtime's staging copies of
    // a pageable source read the same pages, and the kernels wait for them, not for these
    const uint64_t T = total >= (1u << 20) ? 3 : 1;
    for (uint64_t t = 0; t < T; ++t)
      Th.th.emplace_back([&, t, T] {
        {
          std::unique_lock<std::mutex> g(R.mu);
          R.cv.wait(g, [&] { return R.failed || R.n == parts; });
        }
        const uint64_t a = total * t / T, z = total * (t + 1) / T;
        if (z > a) std::memcpy(il_out + a, lsrc + a, (z - a) * 4);
      });
  }

  // ---- the parts: engine A takes parts 0, 2, .., engine B 1, 3, .. (A all without B) ----
  std::vector<FstError> perr(parts, FST_OK);
  // (A/B timing only: FSTAMD_STREAM_AB=1 drops the copy-out; the result then lacks paths)
  const char* abe = std::getenv("FSTAMD_STREAM_AB");
  const bool ab_nocopy = abe && std::atoi(abe) == 1;
  auto drive = [&](DeviceEngine::Lease& E, hipStream_t s, size_t p0, size_t step) {
    if (hipSetDevice(dev) != hipSuccess) {
      perr[p0] = FST_INVALID_ARG;
      return;
    }
    for (size_t p = p0; p < parts; p += step) {
      {
        std::unique_lock<std::mutex> g(R.mu);
        R.cv.wait(g, [&] { return R.failed || R.n > p; });
        if (R.n <= p) {
          perr[p] = FST_OOM;
          return;
        }
      }
      const uint32_t s0 = cut[p], np = cut[p + 1] - cut[p];
      ChainInput in{(const uint32_t*)d_lab.p, (const uint64_t*)d_off.p + s0, np, max_len};
      BatchOutDev v = vb;
      v.status += s0;
      v.path_len += s0;
      v.path_off += s0;
      v.final_w += s0;
      v.slots = (const uint64_t*)d_off.p + s0;
      v.host_ol = out->olabels + lbase;
      v.host_w = out->weights + lbase;
      if (ab_nocopy) v.host_ol = nullptr, v.host_w = nullptr;
      v.first_status = (int32_t*)d_first.p + s0;
      // the pull tier alone: no fill, copy or host synchronisation between parts (a fill
      // or copy is a blit kernel that waits for CU slots behind the other engine's
      // persistent kernel, and had held this engine's next part back); the later tiers
      // and the downloads come after the last part
      if (hipStreamWaitEvent(s, K->ev[p], 0) != hipSuccess ||
          E->launch_pull_part(D, in, n, semantics, v, s, (unsigned int*)d_ctr.p + p) !=
              hipSuccess) {
        perr[p] = FST_OOM;
        return;
      }
    }
  };
  const auto tk0 = std::chrono::steady_clock::now();
  {
    Threads P;
    if (EB) P.th.emplace_back([&] { drive(EB, sB, 1, 2); });
    drive(EA, sA, 0, EB ? 2 : 1);
    P.join();
  }
  for (hipStream_t x : {up, sA, sB})
    if (x && hipStreamSynchronize(x) != hipSuccess) return FST_OOM;
  for (size_t p = 0; p < parts; ++p)
    if (perr[p] != FST_OK) return perr[p];
  int32_t* const st_out = out->status + S.s0;
  double* const fin_out = out->final_weights + S.s0;
  int32_t* const first = first_all + S.s0;
  // statuses, final weights and the pull tier's statuses in one download each
  auto download = [&](bool with_first) {
    return (hipMemcpyAsync(st_out, o.status.p, num * 4ull, hipMemcpyDeviceToHost, sA) ==
                hipSuccess &&
            hipMemcpyAsync(fin_out, o.fin.p, num * 8ull, hipMemcpyDeviceToHost, sA) ==
                hipSuccess &&
            (!with_first || hipMemcpyAsync(first, d_first.p, num * 4ull, hipMemcpyDeviceToHost,
                                           sA) == hipSuccess) &&
            hipStreamSynchronize(sA) == hipSuccess);
  };
  if (!download(true) || fault_inject("stream_after_pull")) return FST_OOM;
  // the later tiers, once, over the strings the pull tier handed on (in the device arena,
  // the same slots) -- only when it handed some on (the metric: none), then the statuses
  // and final weights again
  bool handed = false;
  for (uint32_t i = 0; i < num && !handed; ++i) handed = first[i] != kPathOk && first[i] != kPathEmpty;
  uint32_t launches = (uint32_t)parts;
  if (handed) {
    later_lock.lock();
    ChainInput in{(const uint32_t*)d_lab.p, (const uint64_t*)d_off.p, num, max_len};
    BatchOutDev v = vb;
    v.slots = (const uint64_t*)d_off.p;
    EA->set_after_pull(true);
    const hipError_t e = EA->run_chain(D, in, n, semantics, v, sA, nullptr);
    EA->set_after_pull(false);
    if (e != hipSuccess || !download(false)) return FST_OOM;
    ++launches;
  }

  // ---- paths the later tiers wrote (device arena, same slots) ----
  uint64_t nfix = 0;
  for (uint32_t i = 0; i < num; ++i) nfix += st_out[i] == kPathOk && first[i] != kPathOk;
  if (nfix) {
    const auto d2h = [&](void* dst, const void* s, size_t bytes) {
      return bytes == 0 || hipMemcpyAsync(dst, s, bytes, hipMemcpyDeviceToHost, sA) == hipSuccess;
    };
    bool ok = true;
    const char* few_env = std::getenv("FSTAMD_STREAM_FIX_FEW");  // (tests: 0 = bulk copy)
    const uint64_t few = few_env ? std::strtoull(few_env, nullptr, 10) : 4096ull;
    if (nfix <= few) {
      for (uint32_t i = 0; i < num && ok; ++i)
        if (st_out[i] == kPathOk && first[i] != kPathOk) {
          const uint64_t a = loff[i], L = loff[i + 1] - a;
          ok = d2h(out->olabels + lbase + a, vb.out_ol + a, L * 4) &&
               d2h(out->weights + lbase + a, vb.out_w + a, L * 8);
        }
    } else {  // many: the whole arena (every pull-tier chase writes its path there too)
      ok = d2h(out->olabels + lbase, vb.out_ol, total * 4) &&
           d2h(out->weights + lbase, vb.out_w, total * 8);
    }
    if (!ok || hipStreamSynchronize(sA) != hipSuccess) return FST_OOM;
  }
  Th.join();
  S.launches = launches;
  S.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tk0)
                  .count();
  return FST_OK;
}

// The streamed host batch over `devices` (one shard per device, or `nsh` shards round
// robin: FST_BATCH_DEVICES): the result is allocated once, every shard streams into its own
// slice of it (fixed slots: no compaction between shards, no gather), then strings without
// a path are compacted out on the host.  Shards are contiguous string ranges of equal
// estimated cost (FrozenFst::chain_cost), as in run_sharded.
int run_streamed(const std::vector<int>& devices, uint32_t nsh, FrozenFst& b,
                 const uint32_t* labels, const uint64_t* offsets, uint32_t num, uint32_t n,
                 int semantics, FstBatchResult* out) {
  DeviceRestore_ restore;
  std::vector<DeviceFst*> Ds(devices.size(), nullptr);
  for (size_t d = 0; d < devices.size(); ++d) {  // (the rhs goes to every device first)
    if (hipSetDevice(devices[d]) != hipSuccess) return FST_INVALID_ARG;
    Ds[d] = b.device(devices[d]);
    if (!Ds[d]) return FST_OOM;
    if (Ds[d]->has_eps || !DeviceEngine::pull_first(*Ds[d], semantics))
      return kStreamNotApplicable;
  }
  const uint64_t base0 = offsets[0], total = offsets[num] - base0;
  if (!alloc_result(out, num, total)) return FST_OOM;
  if (!pin_is_pinned(out->ilabels) || !pin_is_pinned(out->olabels) ||
      !pin_is_pinned(out->weights) || !pin_is_pinned(out->path_offsets) ||
      !pin_is_pinned(out->status) || !pin_is_pinned(out->final_weights)) {
    fst_batch_result_free(out);
    return kStreamNotApplicable;
  }
  const uint32_t* src = labels ? labels + base0 : nullptr;

  // ---- the result's CSR offsets (= the rebased input offsets) and max_len ----
  uint64_t* const poff = out->path_offsets;
  uint32_t max_len = 0;
  {
    const uint32_t nt = num >= (1u << 18) ? 4 : 1;
    std::vector<uint32_t> mx(nt, 0);
    auto rebase = [&](uint32_t t) {
      uint32_t m = 0;
      for (uint64_t i = (uint64_t)num * t / nt, e = (uint64_t)num * (t + 1) / nt; i < e; ++i) {
        poff[i] = offsets[i] - base0;
        m = std::max<uint32_t>(m, (uint32_t)(offsets[i + 1] - offsets[i]));
      }
      mx[t] = m;
    };
    std::vector<std::thread> R;
    for (uint32_t t = 1; t < nt; ++t) R.emplace_back(rebase, t);
    rebase(0);
    for (auto& t : R) t.join();
    for (uint32_t m : mx) max_len = std::max(max_len, m);
    poff[num] = total;
  }

  // ---- shards: contiguous string ranges of equal estimated cost ----
  nsh = std::max<uint32_t>(1, std::min<uint32_t>(nsh, num));
  std::vector<StreamShard> sh(nsh);
  const bool shard_log = std::getenv("FSTAMD_SHARD_LOG") != nullptr;
  std::vector<double> pre;  // cost of strings [0, i) (chain_cost per distinct length)
  if (nsh > 1 || shard_log) {
    std::vector<double> cl(max_len + 1, -1.0);
    pre.assign(num + 1, 0.0);
    for (uint32_t i = 0; i < num; ++i) {
      const uint32_t L = (uint32_t)(poff[i + 1] - poff[i]);
      if (cl[L] < 0) cl[L] = b.chain_cost(L);
      pre[i + 1] = pre[i] + cl[L];
    }
  }
  {
    std::vector<uint32_t> cuts{0};
    if (nsh > 1) {
      for (uint32_t j = 1; j < nsh; ++j) {
        const double goal = pre[num] * j / nsh;
        uint32_t i = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), goal) - pre.begin());
        i = std::max(i, cuts.back() + 1);          // never empty
        i = std::min(i, num - (nsh - j));           // at least one string for each later one
        cuts.push_back(i);
      }
    }
    cuts.push_back(num);
    for (uint32_t j = 0; j < nsh; ++j) {
      sh[j].dev = devices[j % devices.size()];
      sh[j].s0 = cuts[j];
      sh[j].s1 = cuts[j + 1];
    }
  }
  if (shard_log)  // tests: the shard plan and the route
    for (uint32_t j = 0; j < nsh; ++j)
      std::fprintf(stderr, "[libfst_amd shard] %u dev %d strings %u..%u cost %.6g route streamed\n",
                   j, sh[j].dev, sh[j].s0, sh[j].s1, pre[sh[j].s1] - pre[sh[j].s0]);

  PinnedVec<int32_t> first(std::max<uint32_t>(num, 1));
  std::vector<std::mutex> later_mu(devices.size());  // (stream_shard: per device)
  if (t_prof) t_prof->lap(0);
  const auto tk0 = std::chrono::steady_clock::now();
  {
    auto run = [&](uint32_t j) {
      StreamShard& S = sh[j];
      const size_t d = (size_t)(j % devices.size());
      S.err = stream_shard(S, *Ds[d], src, poff, max_len, n, semantics, out, first.data(),
                           &later_mu[d]);
    };
    std::vector<std::thread> th;
    for (uint32_t j = 1; j < nsh; ++j) th.emplace_back(run, j);
    run(0);
    for (auto& t : th) t.join();
  }
  LaunchStats agg{};  // (the parts overlap on two streams: their wall time, not a sum)
  agg.engine = semantics == 1 ? 0 : 7;
  for (const StreamShard& S : sh) {
    if (S.err != FST_OK) return S.err;
    agg.launches += S.launches;
  }
  agg.kernel_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tk0).count();
  t_last_stats = agg;
  if (t_prof) t_prof->lap(2);

  // ---- strings without a path: their slots dropped (in order, moving left) ----
  uint64_t nbad = 0;
  for (uint32_t i = 0; i < num; ++i) nbad += out->status[i] != kPathOk;
  if (nbad) {
    uint64_t dst = 0;
    for (uint32_t i = 0; i < num; ++i) {
      const uint64_t a = poff[i], L = poff[i + 1] - a;
      poff[i] = dst;
      if (out->status[i] != kPathOk) continue;
      if (dst != a) {
        std::memmove(out->ilabels + dst, out->ilabels + a, L * 4);
        std::memmove(out->olabels + dst, out->olabels + a, L * 4);
        std::memmove(out->weights + dst, out->weights + a, L * 8);
      }
      dst += L;
    }
    poff[num] = dst;
  }
  out->total_arcs = poff[num];
  if (t_prof) {
    t_prof->runs = (int)agg.launches;
    t_prof->lap(3);
  }
  return FST_OK;
}

// Runs `compute` (the engines: it fills S.keep and, for pipelines, S.fail) over the shards
// of a batch and gathers their results into *out.  Shards are contiguous string ranges of
// equal estimated cost (cost[i]: the work estimate of string i); shard j runs on
// devices[j % devices.size()] on a host thread of its own (inline for one shard).
FstError run_sharded(const std::vector<int>& devices, uint32_t nsh, uint32_t num,
                     const std::vector<double>& cost,
                     const std::function<FstError(Shard&)>& compute, FstBatchResult* out) {
  // shard 0 runs on the calling thread and switches its current device: give the caller
  // its device back on every return (later calls that use current_device() rely on it)
  DeviceRestore_ restore;
  nsh = std::max<uint32_t>(1, std::min<uint32_t>(nsh, std::max<uint32_t>(num, 1)));
  std::vector<Shard> sh(nsh);
  if (nsh == 1) {
    sh[0].dev = devices[0];
    sh[0].s0 = 0;
    sh[0].s1 = num;
  } else {
    double total = 0;
    for (double c : cost) total += c;
    uint32_t i = 0;
    double acc = 0;
    for (uint32_t j = 0; j < nsh; ++j) {
      sh[j].dev = devices[j % devices.size()];
      sh[j].s0 = i;
      const double goal = total * (j + 1) / nsh;
      // leave at least one string for each later shard
      while (i < num && (j + 1 == nsh || (acc + cost[i] <= goal && num - i > nsh - 1 - j))) {
        acc += cost[i];
        ++i;
      }
      if (j + 1 < nsh && i == sh[j].s0 && i < num) acc += cost[i++];  // never empty
      sh[j].s1 = (j + 1 == nsh) ? num : i;
    }
  }
  if (std::getenv("FSTAMD_SHARD_LOG"))  // tests: the shard plan
    for (uint32_t j = 0; j < nsh; ++j) {
      double c = 0;
      for (uint32_t i = sh[j].s0; i < sh[j].s1 && i < cost.size(); ++i) c += cost[i];
      std::fprintf(stderr, "[libfst_amd shard] %u dev %d strings %u..%u cost %.6g route sharded\n", j,
                   sh[j].dev, sh[j].s0, sh[j].s1, c);
    }
  auto phase1 = [&](Shard& S) {
    if (hipSetDevice(S.dev) != hipSuccess) {
      S.err = FST_INVALID_ARG;
      return;
    }
    S.E = DeviceEngine::acquire(S.dev);
    if (!S.E) {
      S.err = FST_INVALID_ARG;
      return;
    }
    S.err = compute(S);
    S.stats = t_last_stats;
    if (S.err == FST_OK && !S.keep) S.err = FST_OOM;
    if (S.err == FST_OK) S.err = shard_compact(S);
    // no lease is held between the phases: a shard waiting for an engine never holds one
    // (two sharded calls on one device cannot deadlock)
    S.E = DeviceEngine::Lease();
  };
  auto phase2 = [&](Shard& S, uint64_t base) {
    if (hipSetDevice(S.dev) != hipSuccess) {
      S.err = FST_OOM;
      return;
    }
    S.E = DeviceEngine::acquire(S.dev);
    S.err = S.E ? shard_download(S, out, base) : FST_OOM;
    S.E = DeviceEngine::Lease();
  };
  auto each = [&](const std::function<void(uint32_t)>& f) {
    if (nsh == 1) return f(0);
    std::vector<std::thread> th;
    for (uint32_t j = 1; j < nsh; ++j) th.emplace_back(f, j);
    f(0);
    for (auto& x : th) x.join();
  };
  each([&](uint32_t j) { phase1(sh[j]); });
  uint64_t tot = 0;
  for (Shard& S : sh) {
    if (S.err != FST_OK) return S.err;
    tot += S.tot;
  }
  if (t_prof) t_prof->lap(4);
  if (!alloc_result(out, num, tot)) return FST_OOM;
  std::vector<uint64_t> base(nsh, 0);
  for (uint32_t j = 1; j < nsh; ++j) base[j] = base[j - 1] + sh[j - 1].tot;
  each([&](uint32_t j) { phase2(sh[j], base[j]); });
  out->path_offsets[num] = tot;
  LaunchStats agg = sh[0].stats;  // the slowest shard's kernel time, launches summed
  for (uint32_t j = 1; j < nsh; ++j) {
    agg.kernel_ms = std::max(agg.kernel_ms, sh[j].stats.kernel_ms);
    agg.launches += sh[j].stats.launches;
  }
  t_last_stats = agg;
  for (Shard& S : sh)
    if (S.err != FST_OK) return S.err;
  if (t_prof) t_prof->lap(3);
  return FST_OK;
}

// The devices and shard count of a host batch call (FstBatchOptions, fst_batch.h).
FstError batch_devices(const FstBatchOptions* opts, std::vector<int>* devices, uint32_t* nsh) {
  devices->clear();
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return FST_INVALID_ARG;
  if (opts && (opts->flags & FST_BATCH_DEVICES) && opts->device_mask) {
    for (int d = 0; d < 64; ++d)
      if (opts->device_mask >> d & 1) {
        if (d >= count) return FST_INVALID_ARG;
        devices->push_back(d);
      }
  } else {
    int dev = opts ? opts->device : -1;
    if (dev < 0) dev = current_device();
    if (dev < 0 || dev >= count) return FST_INVALID_ARG;
    devices->push_back(dev);
  }
  *nsh = (uint32_t)devices->size();
  if (opts && (opts->flags & FST_BATCH_DEVICES) && opts->num_shards)
    *nsh = std::max<uint32_t>(opts->num_shards, 1);
  return FST_OK;
}

// One batch on device inputs; the path arena grows on OUTPUT_FULL.  With `keep` the
// device outputs stay alive (pipelines) and `h` receives only the statuses.
FstError run_chain_batch_dev(DeviceEngine::Lease& E, DeviceFst& D, const ChainInput& in,
                             uint64_t total_labels, uint32_t n, int semantics, HostPaths* h,
                             std::unique_ptr<DevOut>* keep) {
  const uint32_t num = in.num_strings;
  const hipStream_t stream = E.stream();
  // Arena: chains without rhs epsilons produce exactly L arcs per path; with them a path
  // also carries the rhs epsilon arcs (a tagger's or verbalizer's multi-symbol outputs),
  // so start at 4 arcs per label rather than run the whole batch twice on OUTPUT_FULL.
  uint64_t arc_cap = std::max<uint64_t>((D.has_eps ? 4 : 1) * total_labels + 16, 1024);
  // test override: the first arena size, grown x4 per attempt (so that 6 attempts can run
  // out, tests/test_gpu_watchdog.py) instead of sized from the demand
  bool fixed_growth = false;
  if (const char* e = std::getenv("FSTAMD_ARENA_ARCS"))
    if (*e) {
      arc_cap = std::max<uint64_t>(std::strtoull(e, nullptr, 10), 1);
      fixed_growth = true;
    }
  constexpr int kAttempts = 6;
  for (int attempt = 0; attempt < kAttempts; ++attempt) {
    if (t_prof) t_prof->lap(7);
    auto out = std::make_unique<DevOut>(num, arc_cap);
    if (!out->ok()) return FST_OOM;
    if (t_prof) t_prof->lap(1);
    LaunchStats st;
    hipError_t err = E->run_chain(D, in, n, semantics, out->v, stream, &st);
    if (err == hipSuccess) err = hipStreamSynchronize(stream);
    if (t_prof) {
      t_prof->lap(2);
      ++t_prof->runs;
    }
    if (err != hipSuccess) {
      std::fprintf(stderr, "[libfst_amd] batch engine failed: %s\n", hipGetErrorString(err));
      return FST_OOM;
    }
    t_last_stats = st;
    bool full = false;
    if (keep) {
      h->status.resize(num);
      if (num && (hipMemcpyAsync(h->status.data(), out->v.status, num * 4ull,
                                 hipMemcpyDeviceToHost, stream) != hipSuccess ||
                  hipStreamSynchronize(stream) != hipSuccess))
        return FST_OOM;
    } else if (!out->download(num, h, stream)) {
      return FST_OOM;
    }
    if (t_prof) t_prof->lap(3);
    for (uint32_t i = 0; i < num; ++i) full |= h->status[i] == kPathOutputFull;
    // The last attempt's result stands: strings still OUTPUT_FULL keep that status (the
    // caller sees FST_PATH_OUTPUT_FULL per string), and `keep` is always set on FST_OK.
    if (!full || attempt + 1 == kAttempts) {
      if (keep) *keep = std::move(out);
      return FST_OK;
    }
    // every engine reserves a path with atomicAdd on the cursor before it checks the
    // capacity, so the cursor ends at the arcs the whole batch needs: one rerun suffices
    unsigned long long need = 0;
    if (hipMemcpyAsync(&need, out->v.cursor, 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return FST_OOM;
    arc_cap = fixed_growth ? arc_cap * 4 : std::max<uint64_t>(arc_cap * 2, need + 1024);
  }
  return FST_OOM;  // unreachable: the last attempt returns above
}

// ---- Coalesced single calls ----------------------------------------------------------
// fst_compose_frozen_shortest_path on a compileString lhs is one chain string.  Calls that
// arrive while a batch is in flight are combined (flat combining): the first caller of an
// idle device becomes a leader, takes every queued call (grouped by rhs and n), runs them
// as one batch on an engine lease and hands each caller its path; up to chain_leaders()
// batches run at once (separate engines and streams).  A lone caller runs its own string
// with no added latency; N concurrent callers share launches and host <-> device trips, so
// calls/s grows with N (the reference scales calls over threads, README.md:68-82).
// FSTAMD_COALESCE=0 runs every call on its own.
struct ChainCall {
  std::shared_ptr<FrozenFst> rhs;
  uint32_t n = 1;
  const std::vector<uint32_t>* labels = nullptr;
  // result
  FstError err = FST_OOM;
  int32_t status = kPathInternal;
  // the batch's host result, shared by its callers: each copies its own path out (the
  // leader allocating and the callers freeing one arc vector per call had the callers
  // queue on the leader's malloc arena)
  std::shared_ptr<const HostPaths> paths;
  uint32_t index = 0;
  double fin = 0;
  LaunchStats stats;
  // combiner hand-off: each caller sleeps on its own word (a futex), so a finished batch
  // wakes exactly its callers, which return without touching the combiner's lock, and one
  // queued caller to lead next.  The queue and the leader count stay under
  // ChainCombiner::mu; the lock-free word took the wake-ups of 256 waiting threads off it
  // (each had re-taken the lock on waking: half the process's CPU time at 256 threads).
  std::atomic<uint32_t> word{0};  // kCallWaiting / kCallLead / kCallDone
  bool taken = false;             // in a leader's batch (under ChainCombiner::mu)
};
constexpr uint32_t kCallWaiting = 0, kCallLead = 1, kCallDone = 2;

void call_wake(std::atomic<uint32_t>& w) {
  // after a post the caller may already have returned and its frame be reused: a wake on
  // that address is at most a spurious one, and every waiter re-checks its word
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}
void call_wait(std::atomic<uint32_t>& w) {  // until the word leaves kCallWaiting
  while (w.load(std::memory_order_acquire) == kCallWaiting)
    syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAIT_PRIVATE, kCallWaiting, nullptr,
            nullptr, 0);
}
// a queued caller (under ChainCombiner::mu): a leader slot is free
void call_hint_lead(ChainCall* c) {
  uint32_t z = kCallWaiting;
  if (c->word.compare_exchange_strong(z, kCallLead, std::memory_order_acq_rel)) call_wake(c->word);
}

struct ChainCombiner {
  std::mutex mu;
  std::deque<ChainCall*> q;
  int leaders = 0;
};
// leaders at once (each on its own engine lease); FSTAMD_CHAIN_LEADERS overrides (A/B)
int chain_leaders() {
  static const int n = [] {
    const char* e = std::getenv("FSTAMD_CHAIN_LEADERS");
    return e && std::atoi(e) > 0 ? std::atoi(e) : 2;
  }();
  return n;
}
constexpr size_t kChainMaxBatch = 1u << 16;

ChainCombiner& chain_combiner(int dev) {
  static std::mutex mu;
  static auto* cs = new std::vector<std::unique_ptr<ChainCombiner>>();  // never destroyed
  std::lock_guard<std::mutex> g(mu);
  if ((int)cs->size() <= dev) cs->resize(dev + 1);
  if (!(*cs)[dev]) (*cs)[dev].reset(new ChainCombiner());
  return *(*cs)[dev];
}

void run_chain_calls(int dev, std::vector<ChainCall*>& calls) {
  // group by (rhs, n): one batch per group, strings in arrival order
  std::stable_sort(calls.begin(), calls.end(), [](const ChainCall* x, const ChainCall* y) {
    return std::make_pair(x->rhs.get(), x->n) < std::make_pair(y->rhs.get(), y->n);
  });
  for (size_t g0 = 0; g0 < calls.size();) {
    size_t g1 = g0 + 1;
    while (g1 < calls.size() && calls[g1]->rhs == calls[g0]->rhs && calls[g1]->n == calls[g0]->n)
      ++g1;
    const uint32_t num = (uint32_t)(g1 - g0);
    std::vector<uint64_t> offs(num + 1, 0);
    for (uint32_t i = 0; i < num; ++i) offs[i + 1] = offs[i] + calls[g0 + i]->labels->size();
    std::vector<uint32_t> labels(offs[num]);
    for (uint32_t i = 0; i < num; ++i)
      std::copy(calls[g0 + i]->labels->begin(), calls[g0 + i]->labels->end(),
                labels.begin() + offs[i]);
    auto hp = std::make_shared<HostPaths>();
    HostPaths& h = *hp;
    FstError e = FST_INVALID_ARG;
    HostProf prof;  // FSTAMD_HOST_PROF=1: the phases of this coalesced batch
    t_prof = prof.on ? &prof : nullptr;
    {
      DeviceEngine::Lease E = DeviceEngine::acquire(dev);
      if (E)
        e = run_chain_batch_host(E, *calls[g0]->rhs, labels.data(), offs.data(), num,
                                 calls[g0]->n, FST_SEM_LAZY, &h);
    }
    if (t_prof) {
      prof.lap(5);
      char what[96];
      std::snprintf(what, sizeof(what), "chain call batch (%u string(s))", num);
      prof.print(what);
      t_prof = nullptr;
    }
    for (uint32_t i = 0; i < num; ++i) {
      ChainCall* c = calls[g0 + i];
      c->err = e;
      c->stats = t_last_stats;
      if (e != FST_OK) continue;
      c->status = h.status[i];
      if (c->status != kPathOk) continue;
      c->fin = h.fin[i];
      c->paths = hp;
      c->index = i;
    }
    g0 = g1;
  }
}

FstError coalesced_chain_call(int dev, ChainCall* c) {
  if (dev < 0) return FST_INVALID_ARG;
  static const bool on = [] {
    const char* e = std::getenv("FSTAMD_COALESCE");
    return !(e && std::atoi(e) == 0);
  }();
  if (!on) {
    std::vector<ChainCall*> one{c};
    run_chain_calls(dev, one);
    return c->err;
  }
  ChainCombiner& C = chain_combiner(dev);
  std::unique_lock<std::mutex> lk(C.mu);
  C.q.push_back(c);
  // a call leads when a leader slot is free and no leader has taken it yet; a slot is only
  // ever taken here, by the thread itself under the lock, and given back by the same thread
  // after its batch, so slots can be neither lost nor duplicated (round-3 ADVICE)
  while (c->taken || C.leaders >= chain_leaders()) {
    lk.unlock();
    call_wait(c->word);
    lk.lock();
    if (c->word.load(std::memory_order_acquire) == kCallDone) return c->err;
    uint32_t h = kCallLead;  // hinted: look again (a done word is never rewritten)
    c->word.compare_exchange_strong(h, kCallWaiting, std::memory_order_acq_rel);
  }
  ++C.leaders;
  // this call first, then the oldest queued ones
  auto it = std::find(C.q.begin(), C.q.end(), c);
  C.q.erase(it);
  C.q.push_front(c);
  const size_t take = std::min(C.q.size(), kChainMaxBatch);
  std::vector<ChainCall*> batch(C.q.begin(), C.q.begin() + take);
  C.q.erase(C.q.begin(), C.q.begin() + take);
  for (ChainCall* x : batch) x->taken = true;
  // a second free slot: let the oldest remaining caller lead a batch beside this one
  if (!C.q.empty() && C.leaders < chain_leaders()) call_hint_lead(C.q.front());
  lk.unlock();
  run_chain_calls(dev, batch);
  for (ChainCall* x : batch) {
    if (x == c) continue;
    x->word.store(kCallDone, std::memory_order_release);
    call_wake(x->word);
  }
  lk.lock();
  --C.leaders;
  if (!C.q.empty()) call_hint_lead(C.q.front());
  return c->err;
}

}  // namespace

namespace fstamd {  // the pools for device_engine.hip (HostLattice, the dense replay's budget)
void* pin_host_alloc(size_t bytes) { return pin_alloc(bytes); }
void pin_host_release(void* p) { pin_release(p); }
void device_pool_release(int dev) { pool_release(dev); }
}  // namespace fstamd

extern "C" {

// ---- MutableFst lifecycle -----------------------------------------------------------

FstMutableHandle fst_mutable_new(void) {
  return g_mut.insert(std::make_shared<MutableFst>());
}

FstMutableHandle fst_mutable_clone(FstMutableHandle handle) {
  std::shared_ptr<MutableFst> copy;
  {
    auto g = g_mut.lock_shared(handle);
    const MutableFst* m = g_mut.get_locked(handle);
    if (!m) return kInvalid;
    copy = std::make_shared<MutableFst>(*m);
  }
  return g_mut.insert(std::move(copy));
}

void fst_mutable_free(FstMutableHandle handle) { g_mut.remove(handle); }

uint32_t fst_mutable_add_state(FstMutableHandle handle) {
  auto g = g_mut.lock(handle);
  MutableFst* m = g_mut.get_locked(handle);
  if (!m) return FST_NO_STATE;
  return m->add_state();
}

FstError fst_mutable_set_start(FstMutableHandle handle, uint32_t state) {
  auto g = g_mut.lock(handle);
  MutableFst* m = g_mut.get_locked(handle);
  if (!m) return FST_INVALID_ARG;
  if (state >= m->num_states()) return FST_INVALID_STATE;
  m->set_start(state);
  return FST_OK;
}

FstError fst_mutable_set_final(FstMutableHandle handle, uint32_t state, double weight) {
  auto g = g_mut.lock(handle);
  MutableFst* m = g_mut.get_locked(handle);
  if (!m) return FST_INVALID_ARG;
  if (state >= m->num_states()) return FST_INVALID_STATE;
  m->set_final(state, weight);
  return FST_OK;
}

FstError fst_mutable_add_arc(FstMutableHandle handle, uint32_t src, uint32_t ilabel,
                             uint32_t olabel, double weight, uint32_t nextstate) {
  auto g = g_mut.lock(handle);
  MutableFst* m = g_mut.get_locked(handle);
  if (!m) return FST_INVALID_ARG;
  if (src >= m->num_states()) return FST_INVALID_STATE;
  if (nextstate >= m->num_states()) return FST_INVALID_STATE;
  m->add_arc(src, Arc{ilabel, olabel, weight, nextstate});
  return FST_OK;
}

uint32_t fst_mutable_start(FstMutableHandle handle) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  return m ? m->start() : FST_NO_STATE;
}

uint32_t fst_mutable_num_states(FstMutableHandle handle) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  return m ? (uint32_t)m->num_states() : 0;
}

uint32_t fst_mutable_num_arcs(FstMutableHandle handle, uint32_t state) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  if (!m || state >= m->num_states()) return 0;
  return (uint32_t)m->num_arcs(state);
}

double fst_mutable_final_weight(FstMutableHandle handle, uint32_t state) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  if (!m || state >= m->num_states()) return w_zero();
  return m->final_weight(state);
}

uint32_t fst_mutable_get_arcs(FstMutableHandle handle, uint32_t state, FstArc* buf,
                              uint32_t buf_len) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  if (!m || state >= m->num_states()) return 0;
  const auto& arcs = m->arcs(state);
  const uint32_t count = std::min<uint32_t>((uint32_t)arcs.size(), buf_len);
  if (buf)
    for (uint32_t i = 0; i < count; ++i)
      buf[i] = FstArc{arcs[i].ilabel, arcs[i].olabel, arcs[i].weight, arcs[i].nextstate};
  return count;
}

// ---- Freeze / frozen ----------------------------------------------------------------

FstHandle fst_freeze(FstMutableHandle mutable_handle) {
  std::shared_ptr<MutableFst> snap;
  {
    auto g = g_mut.lock_shared(mutable_handle);
    const MutableFst* m = g_mut.get_locked(mutable_handle);
    if (!m) return kInvalid;
    snap = std::make_shared<MutableFst>(*m);  // clone under the lock (c-api.zig:507-517)
  }
  auto f = FrozenFst::from_mutable(*snap, kWeightTropical);
  return g_fst.insert(std::move(f));
}

void fst_free(FstHandle handle) { g_fst.remove(handle); }

uint32_t fst_start(FstHandle handle) {
  auto f = g_fst.get(handle);
  return f ? f->start() : FST_NO_STATE;
}

uint32_t fst_num_states(FstHandle handle) {
  auto f = g_fst.get(handle);
  return f ? f->num_states() : 0;
}

uint32_t fst_num_arcs(FstHandle handle, uint32_t state) {
  auto f = g_fst.get(handle);
  if (!f || state >= f->num_states()) return 0;
  return f->num_arcs(state);
}

double fst_final_weight(FstHandle handle, uint32_t state) {
  auto f = g_fst.get(handle);
  if (!f || state >= f->num_states()) return w_zero();
  return f->final_weight(state);
}

uint32_t fst_get_arcs(FstHandle handle, uint32_t state, FstArc* buf, uint32_t buf_len) {
  auto f = g_fst.get(handle);
  if (!f || state >= f->num_states()) return 0;
  const StateEntry& e = f->states()[state];
  const uint32_t count = std::min(e.num_arcs, buf_len);
  if (buf)
    for (uint32_t i = 0; i < count; ++i) {
      const PackedArc& a = f->arcs()[e.arc_offset + i];
      buf[i] = FstArc{a.ilabel, a.olabel, a.weight, a.nextstate};
    }
  return count;
}

// ---- Binary I/O (src/io/binary.zig:9-36) ----------------------------------------------

FstHandle fst_load(const char* path) {
  if (!path) return kInvalid;
  auto f = FrozenFst::load_file(path, kWeightTropical, nullptr);  // binary.zig:16-36
  if (!f) return kInvalid;
  return g_fst.insert(std::move(f));
}

// src/c-api.zig:588-599: the whole file (at most 64 MiB, as readFileAlloc's limit there),
// parsed by readText; no label shift.
FstMutableHandle fst_read_text(const char* path) {
  if (!path) return kInvalid;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return kInvalid;
  std::vector<char> data;
  bool ok = std::fseek(fp, 0, SEEK_END) == 0;
  const long sz = ok ? std::ftell(fp) : -1;
  ok = sz >= 0 && sz <= (64l << 20);
  if (ok) {
    data.resize((size_t)sz);
    std::rewind(fp);
    ok = sz == 0 || std::fread(data.data(), 1, (size_t)sz, fp) == (size_t)sz;
  }
  std::fclose(fp);
  if (!ok) return kInvalid;
  auto m = std::make_shared<MutableFst>();
  if (!MutableFst::read_text(data.data(), data.size(), m.get())) return kInvalid;
  return g_mut.insert(std::move(m));
}

FstError fst_save(FstHandle handle, const char* path) {
  if (!path) return FST_INVALID_ARG;
  std::shared_ptr<FrozenFst> f;
  {
    f = g_fst.get(handle);
    if (!f) return FST_INVALID_ARG;
  }
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return FST_IO_ERROR;
  const bool ok = std::fwrite(f->bytes(), 1, f->size(), fp) == f->size();
  std::fclose(fp);
  return ok ? FST_OK : FST_IO_ERROR;
}

// ---- The hot path -----------------------------------------------------------------

FstMutableHandle fst_compose_frozen_shortest_path(FstMutableHandle a_handle, FstHandle b_handle,
                                                  uint32_t n) {
  const auto t0 = std::chrono::steady_clock::now();
  auto us = [&] {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  };
  std::shared_ptr<MutableFst> a;
  std::shared_ptr<FrozenFst> b;
  // a compileString acceptor is snapshotted as its labels alone (the chain route below
  // needs nothing else); any other lhs as a deep copy
  std::vector<uint32_t> chain;
  bool is_chain = false;
  size_t a_states = 0, a_arcs = 0;
  bool a_start = false;
  {
    auto g = g_mut.lock_shared(a_handle);
    const MutableFst* ha = g_mut.get_locked(a_handle);
    if (!ha) {
      trace("sp_invalid_a", a_handle, b_handle, 0, 0, 0, 0, us(), 0);
      return kInvalid;
    }
    is_chain = as_chain(*ha, &chain);
    if (!is_chain) a = std::make_shared<MutableFst>(*ha);  // snapshot (c-api.zig:754)
    a_states = ha->num_states();
    a_arcs = is_chain ? chain.size() : ha->total_arcs();
    a_start = ha->start() != kNoState;
    b = g_fst.get(b_handle);                // pin (c-api.zig:759)
    if (!b) {
      trace("sp_invalid_b", a_handle, b_handle, a_states, a_arcs, 0, 0, us(), 0);
      return kInvalid;
    }
  }
  MutableFst result;
  // compose-shortest-path.zig:30-33: empty checks first, then n.
  if (!a_start || b->start() == kNoState || n == 0) {
    // empty result
  } else if (n != 1) {
    trace("sp_compose_error", a_handle, b_handle, a_states, a_arcs, 0, 0, us(), 0);
    return kInvalid;
  } else {
    if (!gpu_available()) return kInvalid;
    double kms = 0;
    int rc = -1;
    if (is_chain) {  // the batch engines on one string, coalesced with the chain calls of
                     // other threads (ChainCombiner)
      ChainCall c;
      c.rhs = b;
      c.n = n;
      c.labels = &chain;
      const FstError e = coalesced_chain_call(current_device(), &c);
      if (e == FST_OK) {
        if (c.status == kPathOk) {
          const HostPaths& h = *c.paths;
          const uint32_t P = h.len[c.index];
          const uint64_t o = h.off[c.index];
          result.add_states(P + 1);
          result.set_start(0);
          result.set_final(P, c.fin);
          for (uint32_t k = 0; k < P; ++k)
            result.add_arc(k, Arc{h.il[o + k], h.ol[o + k], h.w[o + k], k + 1});
          rc = 0;
        } else if (c.status == kPathEmpty) {
          rc = 0;  // the empty FST
        } else if (c.status == kPathCycle) {
          rc = 3;  // as the general path: the reference would not terminate
        }
        t_last_stats = c.stats;
        kms = c.stats.kernel_ms;
      }
    }
    // anything else (a general lhs; a string the batch engines handed back): one general lhs
    if (rc < 0) {
      if (!a) a = std::make_shared<MutableFst>(MutableFst::compile_chain(chain));
      rc = run_lazy_single(*a, *b, n, &result, &kms);
    }
    if (rc != 0) {
      trace("sp_compose_error", a_handle, b_handle, a_states, a_arcs, 0, 0, us(), kms);
      return kInvalid;
    }
  }
  trace("sp_ok", a_handle, b_handle, a_states, a_arcs, result.num_states(),
        result.total_arcs(), us(), t_last_stats.kernel_ms);
  return g_mut.insert(std::make_shared<MutableFst>(std::move(result)));
}

FstMutableHandle fst_compose_frozen(FstMutableHandle a_handle, FstHandle b_handle) {
  // src/c-api.zig:675-742 -> src/ops/compose.zig:29-198 on the GPU (kernels/eager_bfs.hpp):
  // the whole lattice, states numbered in BFS discovery order, arcs in compose order.
  const auto t0 = std::chrono::steady_clock::now();
  auto us = [&] {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  };
  std::shared_ptr<MutableFst> a;
  std::shared_ptr<FrozenFst> b;
  {
    auto g = g_mut.lock_shared(a_handle);
    const MutableFst* ha = g_mut.get_locked(a_handle);
    if (!ha) {
      trace("invalid_a", a_handle, b_handle, 0, 0, 0, 0, us(), 0);
      return kInvalid;
    }
    a = std::make_shared<MutableFst>(*ha);  // snapshot (c-api.zig:686)
    b = g_fst.get(b_handle);                // pin (c-api.zig:691)
    if (!b) {
      trace("invalid_b", a_handle, b_handle, a->num_states(), a->total_arcs(), 0, 0, us(), 0);
      return kInvalid;
    }
  }
  if (!gpu_available()) return kInvalid;
  const int dev = current_device();
  DeviceFst* D = dev >= 0 ? b->device(dev) : nullptr;
  if (!D) return kInvalid;
  const bool hprof = std::getenv("FSTAMD_HOST_PROF") != nullptr;
  HostLattice lat;
  LaunchStats st;
  double t_up0 = 0, t_up1 = 0;
  {
    DeviceEngine::Lease E = DeviceEngine::acquire(dev);
    if (!E) return kInvalid;
    const hipStream_t stream = E.stream();
    t_up0 = us();
    GraphUpload up(*a, stream);
    if (!up.ok) return kInvalid;
    t_up1 = us();
    if (E->compose_lattice(*D, up.g, &lat, &st, stream) != hipSuccess || lat.status != kPathOk) {
      trace("compose_error", a_handle, b_handle, a->num_states(), a->total_arcs(), 0, 0, us(),
            st.kernel_ms);
      return kInvalid;
    }
  }
  t_last_stats = st;
  const double t_gpu = us();
  MutableFst result;
  if (lat.n_nodes > 0) {
    result.add_states(lat.n_nodes);
    result.set_start(0);
    // states in contiguous ranges, one host thread each (a 10 M-arc lattice: ~80 ms on
    // one thread); every state's arc vector is its own allocation
    auto build = [&](uint32_t lo, uint32_t hi) {
      for (uint32_t s2 = lo; s2 < hi; ++s2) {
        if (!w_is_zero(lat.nfin[s2])) result.set_final(s2, lat.nfin[s2]);
        const uint32_t k0 = lat.aoff[s2], k1 = lat.aoff[s2 + 1];
        result.reserve_arcs(s2, k1 - k0);
        for (uint32_t k = k0; k < k1; ++k)
          result.add_arc(s2, Arc{lat.ail[k], lat.aol[k], lat.aw[k], lat.anext[k]});
      }
    };
    const uint32_t nt = lat.n_arcs < (1u << 18) ? 1u
                        : std::min<uint32_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < nt; ++t)
      th.emplace_back(build, (uint32_t)((uint64_t)lat.n_nodes * t / nt),
                      (uint32_t)((uint64_t)lat.n_nodes * (t + 1) / nt));
    build(0, (uint32_t)((uint64_t)lat.n_nodes / nt));
    for (auto& x : th) x.join();
  }
  if (hprof)
    std::fprintf(stderr,
                 "[libfst_amd host] fst_compose_frozen: upload %.2f compose+download %.2f "
                 "(kernel %.2f, %u launch(es)) result %.2f ms\n",
                 (t_up1 - t_up0) / 1e3, (t_gpu - t_up1) / 1e3, st.kernel_ms, st.launches,
                 (us() - t_gpu) / 1e3);
  trace("ok", a_handle, b_handle, a->num_states(), a->total_arcs(), result.num_states(),
        result.total_arcs(), us(), st.kernel_ms);
  return g_mut.insert(std::make_shared<MutableFst>(std::move(result)));
}

FstMutableHandle fst_shortest_path(FstMutableHandle handle, uint32_t n) {
  // src/c-api.zig:897-916 -> src/ops/shortest-path.zig:18-139 on the GPU.
  const bool hprof = std::getenv("FSTAMD_HOST_PROF") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  std::unique_ptr<HostGraph> m;
  {
    auto g = g_mut.lock_shared(handle);
    const MutableFst* h = g_mut.get_locked(handle);
    if (!h) return kInvalid;
    m = std::make_unique<HostGraph>(*h);  // snapshot, flattened to CSR under the lock
  }
  const double t_snap = ms();
  MutableFst result;
  const uint32_t m_states = (uint32_t)m->fin.size();
  if (m->start == kNoState || n == 0) {  // :21-23 -> empty
  } else if (n != 1) {                   // :24 UnsupportedNShortest
    return kInvalid;
  } else {
    if (!gpu_available()) return kInvalid;
    const int dev = current_device();
    if (dev < 0) return kInvalid;
    DeviceEngine::Lease E = DeviceEngine::acquire(dev);
    if (!E) return kInvalid;
    const hipStream_t stream = E.stream();
    GraphUpload up(*m, stream);
    m.reset();
    const double t_up = ms();
    // Non-negative weights: the parallel fixpoint (eager_bfs.hpp); a negative weight:
    // the exact replay of the reference's heap order (sp_replay_kernel).  NaN has no
    // order in the reference's compare (std.math.order): reported as an error.
    if (!up.ok || up.nan) return kInvalid;
    const uint64_t cap = std::max<uint64_t>(m_states + 16, 1024);
    DevOut out(1, cap);
    if (!out.ok()) return kInvalid;
    LaunchStats st;
    HostPaths hp;
    if (E->shortest_path_graph(up.g, n, out.v, &st, stream, up.nonneg) != hipSuccess)
      return kInvalid;
    if (!out.download(1, &hp, stream)) return kInvalid;
    t_last_stats = st;
    if (hp.status[0] == kPathCycle || hp.status[0] == kPathInternal ||
        hp.status[0] == kPathOutputFull)
      return kInvalid;
    result = chain_result(hp, 0);  // OK or EMPTY
    if (hprof)
      std::fprintf(stderr,
                   "[libfst_amd host] fst_shortest_path call: snapshot %.2f upload %.2f engine + "
                   "result %.2f ms\n", t_snap, t_up - t_snap, ms() - t_up);
  }
  return g_mut.insert(std::make_shared<MutableFst>(std::move(result)));
}

// ---- Strings ------------------------------------------------------------------------

FstMutableHandle fst_compile_string(const uint8_t* input, uint32_t len) {
  if (!input) return kInvalid;
  return g_mut.insert(
      std::make_shared<MutableFst>(MutableFst::compile_string(input, len, input, len)));
}

static int32_t print_impl(FstMutableHandle handle, uint8_t* buf, uint32_t buf_len, bool out_tape) {
  auto g = g_mut.lock_shared(handle);
  const MutableFst* m = g_mut.get_locked(handle);
  if (!m) return -1;
  std::vector<uint8_t> s;
  if (!m->print_string(out_tape, &s)) return -1;
  if (s.size() > buf_len) return -1;
  if (buf && !s.empty()) std::memcpy(buf, s.data(), s.size());
  return (int32_t)s.size();
}

int32_t fst_print_string(FstMutableHandle handle, uint8_t* buf, uint32_t buf_len) {
  return print_impl(handle, buf, buf_len, false);
}

int32_t fst_print_output_string(FstMutableHandle handle, uint8_t* buf, uint32_t buf_len) {
  return print_impl(handle, buf, buf_len, true);
}

void fst_teardown(void) {
  g_mut.clear();
  g_fst.clear();
  pool_clear();
  pin_pool_clear();
}

// ---- Batched entries (fst_batch.h) ----------------------------------------------------

FstError fst_compose_frozen_shortest_path_batch(FstHandle b_handle, const uint32_t* labels,
                                                const uint64_t* offsets, uint32_t num_strings,
                                                uint32_t n, const FstBatchOptions* opts,
                                                FstBatchResult* out) {
  if (!out || !offsets || (!labels && num_strings && offsets[num_strings] != offsets[0]))
    return FST_INVALID_ARG;
  std::memset(out, 0, sizeof(*out));
  for (uint32_t i = 0; i < num_strings; ++i)
    if (offsets[i + 1] < offsets[i]) return FST_INVALID_ARG;
  if (opts && (opts->flags & ~FST_BATCH_DEVICES)) return FST_INVALID_ARG;
  std::shared_ptr<FrozenFst> b;
  {
    b = g_fst.get(b_handle);
  }
  if (!b) return FST_INVALID_ARG;
  if (!gpu_available()) return FST_INVALID_ARG;
  const int semantics = opts ? (int)opts->semantics : FST_SEM_LAZY;
  std::vector<int> devices;
  uint32_t nsh = 1;
  if (FstError e = batch_devices(opts, &devices, &nsh); e != FST_OK) return e;
  HostProf prof;
  t_prof = &prof;
  struct ProfScope {
    ~ProfScope() { t_prof = nullptr; }
  } prof_scope;
  // an rhs without input epsilons and a pull tier first: the streamed batch, on one device
  // or sharded over several (FSTAMD_STREAM=0 turns it off)
  if (num_strings > 0) {
    const char* se = std::getenv("FSTAMD_STREAM");
    if (!(se && std::strcmp(se, "0") == 0)) {
      const int e = run_streamed(devices, nsh, *b, labels, offsets, num_strings, n, semantics, out);
      if (e != kStreamNotApplicable) {
        if (e != FST_OK) {
          fst_batch_result_free(out);
          return (FstError)e;
        }
        prof.lap(5);
        prof.print("fst_compose_frozen_shortest_path_batch (streamed)");
        return FST_OK;
      }
    }
  }
  // one device and a large batch on an rhs without input epsilons: pipelined sub-shards
  // (FSTAMD_PIPELINE=0 keeps the one-shard path; FSTAMD_PIPELINE=k forces k sub-shards)
  {
    const char* pe = std::getenv("FSTAMD_PIPELINE");
    const int want = pe && *pe ? std::atoi(pe) : -1;
    uint32_t parts = want > 0 ? (uint32_t)want
                              : (uint32_t)std::min<uint64_t>(8, num_strings / (1u << 17));
    parts = std::min<uint32_t>(parts, std::max<uint32_t>(num_strings, 1));
    const bool single = devices.size() == 1 && nsh == 1;
    if (single && want != 0 && parts >= 2) {
      // (before hipSetDevice: every path out of this block gives the caller its device back)
      DeviceRestore_ restore;
      DeviceFst* D = nullptr;
      if (hipSetDevice(devices[0]) == hipSuccess) D = b->device(devices[0]);
      if (D && !D->has_eps) {
        const FstError e = run_pipelined(devices[0], *b, labels, offsets, num_strings, n,
                                         semantics, parts, out);
        if (e != FST_OK) {
          fst_batch_result_free(out);
          return e;
        }
        prof.lap(5);
        prof.print("fst_compose_frozen_shortest_path_batch (pipelined)");
        return FST_OK;
      }
    }
  }
  std::vector<double> cost(nsh > 1 ? num_strings : 0);
  for (size_t i = 0; i < cost.size(); ++i) cost[i] = b->chain_cost(offsets[i + 1] - offsets[i]);
  const FstError e = run_sharded(
      devices, nsh, num_strings, cost,
      [&](Shard& S) {
        HostPaths h;
        return run_chain_batch_host(S.E, *b, labels, offsets + S.s0, S.s1 - S.s0, n, semantics,
                                    &h, &S.keep);
      },
      out);
  if (e != FST_OK) {
    fst_batch_result_free(out);
    return e;
  }
  prof.lap(5);
  prof.print("fst_compose_frozen_shortest_path_batch");
  return FST_OK;
}

void fst_batch_result_free(FstBatchResult* r) {
  if (!r) return;
  pin_release(r->status);
  pin_release(r->path_offsets);
  pin_release(r->ilabels);
  pin_release(r->olabels);
  pin_release(r->weights);
  pin_release(r->final_weights);
  std::memset(r, 0, sizeof(*r));
}

FstError fst_device_project_output(const FstDeviceBatch* o, uint32_t num_strings,
                                   uint32_t* d_next_labels, uint64_t* d_next_offsets,
                                   int32_t* d_proj_status, uint32_t* max_len, void* stream) {
  if (!o || !d_next_offsets || !d_proj_status || (num_strings && !d_next_labels))
    return FST_INVALID_ARG;
  if (!gpu_available()) return FST_INVALID_ARG;
  const int dev = current_device();
  if (dev < 0) return FST_INVALID_ARG;
  BatchOutDev v{o->status, o->path_len, o->path_offset, o->final_weight, o->ilabels,
                o->olabels, o->weights, o->arc_capacity,
                (unsigned long long*)o->arc_cursor, o->work};
  uint32_t ml = 0;
  DeviceEngine::Lease E = DeviceEngine::acquire(dev);
  if (!E) return FST_INVALID_ARG;
  const hipStream_t s = E.use((hipStream_t)stream);
  if (E->project_output(v, num_strings, d_next_labels, d_next_offsets, d_proj_status, &ml, s) !=
      hipSuccess)
    return FST_OOM;
  if (max_len) *max_len = ml;
  return FST_OK;
}

namespace {
// One shard of a pipeline: every stage on the shard's device, each stage's 1-best output tape
// projected into the next stage's inputs on the device; S.keep = the last stage's outputs,
// S.fail = the first failing stage per string.
FstError run_pipeline_shard(Shard& S, const std::vector<std::shared_ptr<FrozenFst>>& fs,
                            const uint32_t* labels, const uint64_t* offsets, uint32_t n,
                            int semantics) {
  DeviceEngine::Lease& E = S.E;
  const int dev = S.dev;
  const uint32_t num_strings = S.s1 - S.s0;
  const hipStream_t stream = E.stream();
  // stage-1 inputs
  const uint64_t total = num_strings ? offsets[num_strings] - offsets[0] : 0;
  uint32_t max_len = 0;
  std::vector<uint64_t> rebased(num_strings + 1);
  for (uint32_t i = 0; i <= num_strings; ++i) rebased[i] = offsets[i] - offsets[0];
  for (uint32_t i = 0; i < num_strings; ++i)
    max_len = std::max<uint32_t>(max_len, (uint32_t)(rebased[i + 1] - rebased[i]));
  auto lab = std::make_unique<DevBuf>(total * 4), off = std::make_unique<DevBuf>((num_strings + 1ull) * 8);
  if (!lab->p || !off->p) return FST_OOM;
  if (total && hipMemcpyAsync(lab->p, labels + offsets[0], total * 4, hipMemcpyHostToDevice,
                              stream) != hipSuccess)
    return FST_OOM;
  if (hipMemcpyAsync(off->p, rebased.data(), (num_strings + 1ull) * 8, hipMemcpyHostToDevice,
                     stream) != hipSuccess)
    return FST_OOM;
  S.fail = std::make_unique<DevBuf>(num_strings * 4ull);  // first failing stage per string
  if (!S.fail->p || hipMemsetAsync(S.fail->p, 0, num_strings * 4ull, stream) != hipSuccess)
    return FST_OOM;
  uint64_t in_total = total;
  HostPaths h;
  if (t_prof) t_prof->lap(0);
  for (size_t k = 0; k < fs.size(); ++k) {
    DeviceFst* D = fs[k]->device(dev);
    if (!D) return FST_OOM;
    ChainInput in{(const uint32_t*)lab->p, (const uint64_t*)off->p, num_strings, max_len};
    S.keep.reset();
    FstError e = run_chain_batch_dev(E, *D, in, in_total, n, semantics, &h, &S.keep);
    if (e != FST_OK) return e;
    if (!S.keep) return FST_OOM;  // run_chain_batch_dev sets it on FST_OK
    if (k + 1 == fs.size()) break;
    // project this stage's outputs into the next stage's inputs, on the device
    unsigned long long used = 0;
    if (hipMemcpyAsync(&used, S.keep->v.cursor, 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return FST_OOM;
    auto nlab = std::make_unique<DevBuf>((used + num_strings) * 4);
    auto noff = std::make_unique<DevBuf>((num_strings + 1ull) * 8);
    DevBuf pst(num_strings * 4ull);
    if (!nlab->p || !noff->p || !pst.p) return FST_OOM;
    if (E->project_output(S.keep->v, num_strings, (uint32_t*)nlab->p, (uint64_t*)noff->p,
                          (int32_t*)pst.p, &max_len, stream) != hipSuccess ||
        E->merge_status((int32_t*)S.fail->p, (const int32_t*)pst.p, num_strings, stream) !=
            hipSuccess)
      return FST_OOM;
    uint64_t nt = 0;  // (synchronises: pst may go back to the pool)
    if (hipMemcpyAsync(&nt, (uint64_t*)noff->p + num_strings, 8, hipMemcpyDeviceToHost,
                       stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return FST_OOM;
    in_total = nt;
    lab = std::move(nlab);
    off = std::move(noff);
    if (t_prof) t_prof->lap(4);
  }
  return FST_OK;
}
}  // namespace

FstError fst_pipeline_batch(const FstHandle* stages, uint32_t num_stages, const uint32_t* labels,
                            const uint64_t* offsets, uint32_t num_strings, uint32_t n,
                            const FstBatchOptions* opts, FstBatchResult* out) {
  if (!out || !stages || num_stages == 0 || !offsets ||
      (!labels && num_strings && offsets[num_strings] != offsets[0]))
    return FST_INVALID_ARG;
  std::memset(out, 0, sizeof(*out));
  for (uint32_t i = 0; i < num_strings; ++i)
    if (offsets[i + 1] < offsets[i]) return FST_INVALID_ARG;
  if (opts && (opts->flags & ~FST_BATCH_DEVICES)) return FST_INVALID_ARG;
  std::vector<std::shared_ptr<FrozenFst>> fs(num_stages);
  {
    for (uint32_t k = 0; k < num_stages; ++k)
      if (!(fs[k] = g_fst.get(stages[k]))) return FST_INVALID_ARG;
  }
  if (!gpu_available()) return FST_INVALID_ARG;
  const int semantics = opts ? (int)opts->semantics : FST_SEM_LAZY;
  std::vector<int> devices;
  uint32_t nsh = 1;
  if (FstError e = batch_devices(opts, &devices, &nsh); e != FST_OK) return e;
  HostProf prof;
  t_prof = &prof;
  struct ProfScope {
    ~ProfScope() { t_prof = nullptr; }
  } prof_scope;
  // shards balanced by the first stage's work (later stages' inputs are not known yet)
  std::vector<double> cost(nsh > 1 ? num_strings : 0);
  for (size_t i = 0; i < cost.size(); ++i) cost[i] = fs[0]->chain_cost(offsets[i + 1] - offsets[i]);
  const FstError e = run_sharded(
      devices, nsh, num_strings, cost,
      [&](Shard& S) {
        return run_pipeline_shard(S, fs, labels, offsets + S.s0, n, semantics);
      },
      out);
  if (e != FST_OK) {
    fst_batch_result_free(out);
    return e;
  }
  prof.lap(5);
  prof.print("fst_pipeline_batch");
  return FST_OK;
}

FstError fst_device_compose_shortest_path(FstHandle b_handle, const uint32_t* d_labels,
                                          const uint64_t* d_offsets, uint32_t num_strings,
                                          uint32_t max_len, uint32_t n,
                                          const FstBatchOptions* opts, const FstDeviceBatch* o,
                                          void* stream) {
  if (!o || !d_offsets) return FST_INVALID_ARG;
  std::shared_ptr<FrozenFst> b;
  {
    b = g_fst.get(b_handle);
  }
  if (!b) return FST_INVALID_ARG;
  if (!gpu_available()) return FST_INVALID_ARG;
  int dev = opts && opts->device >= 0 ? opts->device : current_device();
  if (dev < 0 || hipSetDevice(dev) != hipSuccess) return FST_INVALID_ARG;
  DeviceFst* D = b->device(dev);
  if (!D) return FST_OOM;
  BatchOutDev v{o->status, o->path_len, o->path_offset, o->final_weight, o->ilabels,
                o->olabels, o->weights, o->arc_capacity,
                (unsigned long long*)o->arc_cursor, o->work};
  ChainInput in{d_labels, d_offsets, num_strings, max_len};
  DeviceEngine::Lease E = DeviceEngine::acquire(dev);
  if (!E) return FST_INVALID_ARG;
  const hipStream_t s = E.use((hipStream_t)stream);
  LaunchStats st;
  const int semantics = opts ? (int)opts->semantics : FST_SEM_LAZY;
  if (E->run_chain(*D, in, n, semantics, v, s, &st) != hipSuccess) return FST_OOM;
  t_last_stats = st;
  return FST_OK;
}

FstError fst_device_prepare(FstHandle b_handle, int32_t device) {
  std::shared_ptr<FrozenFst> b;
  {
    b = g_fst.get(b_handle);
  }
  if (!b) return FST_INVALID_ARG;
  if (!gpu_available()) return FST_INVALID_ARG;
  const int dev = device >= 0 ? device : current_device();
  return b->device(dev) ? FST_OK : FST_OOM;
}

FstHandle fst_device_adopt_blob(const void* d_blob, uint64_t len, int32_t device,
                                const void* host_copy) {
  if (!d_blob || len < sizeof(Header)) return kInvalid;
  if (!gpu_available()) return kInvalid;
  const int dev = device >= 0 ? device : current_device();
  if (hipSetDevice(dev) != hipSuccess) return kInvalid;
  std::vector<uint8_t> bytes(len);
  if (host_copy) std::memcpy(bytes.data(), host_copy, len);
  else if (hipMemcpy(bytes.data(), d_blob, len, hipMemcpyDeviceToHost) != hipSuccess)
    return kInvalid;
  Header h;
  std::memcpy(&h, bytes.data(), sizeof(h));
  // as fst_batch_load_bytes: only the two semirings of weight.zig (fst.zig:43-47)
  if (h.weight_type != kWeightTropical && h.weight_type != kWeightLog) return kInvalid;
  auto f = FrozenFst::from_bytes(bytes.data(), len, h.weight_type, nullptr);
  if (!f) return kInvalid;
  DeviceFst* D = DeviceFst::adopt(d_blob, *f, dev);
  if (!D) return kInvalid;
  f->adopt_device(dev, D);
  return g_fst.insert(std::move(f));
}

FstError fst_last_launch_stats(FstLaunchStats* out) {
  if (!out) return FST_INVALID_ARG;
  out->kernel_ms = t_last_stats.kernel_ms;
  out->launches = t_last_stats.launches;
  out->engine = t_last_stats.engine;
  out->grid = t_last_stats.grid;
  return FST_OK;
}

FstHandle fst_batch_load_bytes(const void* bytes, uint64_t len) {
  if (!bytes || len < sizeof(Header)) return kInvalid;
  Header h;
  std::memcpy(&h, bytes, sizeof(h));
  if (h.weight_type != kWeightTropical && h.weight_type != kWeightLog) return kInvalid;
  auto f = FrozenFst::from_bytes((const uint8_t*)bytes, len, h.weight_type, nullptr);
  if (!f) return kInvalid;
  return g_fst.insert(std::move(f));
}

FstHandle fst_batch_load(const char* path) {
  if (!path) return kInvalid;
  auto f = FrozenFst::load_file(path, FrozenFst::kAnyWeightType, nullptr);
  if (!f) return kInvalid;
  return g_fst.insert(std::move(f));
}

FstHandle fst_load_att(const char* path, uint32_t flags) {
  if (!path || (flags & ~FST_ATT_SHIFT_BYTE_LABELS)) return kInvalid;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return kInvalid;
  std::vector<char> data;
  bool ok = std::fseek(fp, 0, SEEK_END) == 0;
  const long sz = ok ? std::ftell(fp) : -1;
  ok = sz >= 0 && sz <= (256l << 20);  // att2lfst.zig:40-45 (.limited(256 MiB))
  if (ok) {
    data.resize((size_t)sz);
    std::rewind(fp);
    ok = sz == 0 || std::fread(data.data(), 1, (size_t)sz, fp) == (size_t)sz;
  }
  std::fclose(fp);
  if (!ok) return kInvalid;
  MutableFst m;
  if (!MutableFst::read_text(data.data(), data.size(), &m)) return kInvalid;
  if (flags & FST_ATT_SHIFT_BYTE_LABELS) m.shift_labels();
  auto f = FrozenFst::from_mutable(m, kWeightTropical);
  return g_fst.insert(std::move(f));
}

double fst_chain_cost(FstHandle b, uint64_t len) {
  auto f = g_fst.get(b);
  return f ? f->chain_cost(len) : -1.0;
}

int32_t fst_debug_coalescer_state(int32_t device, uint32_t* queued) {
  if (device < 0) return -1;
  ChainCombiner& C = chain_combiner(device);
  std::lock_guard<std::mutex> g(C.mu);
  if (queued) *queued = (uint32_t)C.q.size();
  return C.leaders;
}

int32_t fst_weight_type(FstHandle b) {
  auto f = g_fst.get(b);
  return f ? (int32_t)f->weight_type() : -1;
}

// Reference bench rhs generators (bench/optimize-bench.zig:219-306).
FstHandle fst_bench_transducer(uint32_t kind, uint32_t T, uint32_t B) {
  return fst_bench_transducer_wt(kind, T, B, kWeightTropical);
}

FstHandle fst_bench_transducer_wt(uint32_t kind, uint32_t T, uint32_t B, uint32_t weight_type) {
  if (weight_type != kWeightTropical && weight_type != kWeightLog) return kInvalid;
  MutableFst m;
  if (kind == 0) {  // buildAmbiguousChainTransducer, :250-277
    m.add_states(T + 1);
    m.set_start(0);
    for (uint32_t i = 0; i <= T; ++i) m.set_final(i, w_one());
    const uint32_t fan = std::max<uint32_t>(1, std::min<uint32_t>(B, 4));
    for (uint32_t i = 0; i <= T; ++i) {
      m.add_arc(i, Arc{1, 1, w_one(), i});
      for (uint32_t b = 0; b < fan; ++b)
        m.add_arc(i, Arc{1, ((i + b) % 255) + 1, (double)b, std::min(i + b + 1, T)});
    }
  } else if (kind == 1) {  // buildEpsilonDenseTransducer, :219-248
    m.add_states(T + 1);
    m.set_start(0);
    for (uint32_t i = 0; i <= T; ++i) m.set_final(i, w_one());
    for (uint32_t i = 0; i < T; ++i) {
      m.add_arc(i, Arc{0, 0, w_one(), i + 1});
      for (uint32_t b = 0; b < B; ++b)
        m.add_arc(i, Arc{1, ((i + b) % 255) + 1, (double)b, std::min(i + (b % 4) + 1, T)});
    }
  } else if (kind == 2) {  // transducer_for_freeze, :290-306
    if (T == 0) return kInvalid;
    m.add_states(T);
    m.set_start(0);
    for (uint32_t i = 0; i < T; ++i) {
      m.set_final(i, w_one());
      for (uint32_t b = 0; b < B; ++b)
        m.add_arc(i, Arc{(b % 255) + 1, ((i + b) % 255) + 1, (double)b,
                         (uint32_t)(((uint64_t)i + b + 1) % T)});
    }
  } else {
    return kInvalid;
  }
  auto f = FrozenFst::from_mutable(m, (uint8_t)weight_type);
  return g_fst.insert(std::move(f));
}

}  // extern "C"
