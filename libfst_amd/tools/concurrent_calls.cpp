// concurrent_calls -- N host threads calling the drop-in single-string entry
// fst_compose_frozen_shortest_path concurrently, the way the reference is used from many
// threads (include/fst.h:11-26, README.md:68-82).  A C-ABI client only.
//
// Every thread compiles its strings with fst_compile_string, composes each against one
// shared frozen rhs, reads the result chain back through fst_mutable_get_arcs and checks it
// against the batch entry's answer for the same string (the batch entry is itself
// bit-compared with the oracle by the test suite).  With --free-midway the rhs handle is
// freed while calls are in flight: calls already holding it finish correctly, later ones
// must return FST_INVALID_HANDLE.
//
// usage: concurrent_calls [--threads 32] [--calls 1000] [--len 64] [--rhs ambiguous|eps_dense]
//                         [--transducer-len 4096] [--varied] [--free-midway]
//                         [--rhs-file BLOB --strings-file CSR]
// --rhs-file / --strings-file: a frozen blob (fst_batch_load) and the strings to call it on
// (u32 count, u64 offsets[count + 1], u32 labels = byte + 1), e.g. the WeText-scale tagger
// stand-in and its utterances (scripts/concurrent_calls_bench.py --wetext).
// prints one JSON line: calls/s, mismatches, invalid results.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <sys/resource.h>
#include <vector>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include "../../include/fst_batch.h"

namespace {

struct Expect {
  int32_t status;
  std::vector<FstArc> arcs;
  double fin;
};

bool same(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

// CC_PROF=<file>: a CPU sampling profile of the timed region (SIGPROF every 200 us of process
// CPU time; the interrupted thread's program counter), written as "<object> <offset>" lines
// for addr2line.
constexpr int kMaxSamples = 1 << 16, kDepth = 12;
void* g_samples[kMaxSamples][kDepth];
std::atomic<int> g_nsamples{0};
void on_prof(int, siginfo_t*, void* ctx) {
  const int i = g_nsamples.fetch_add(1, std::memory_order_relaxed);
  if (i >= kMaxSamples) return;
  g_samples[i][0] = (void*)((ucontext_t*)ctx)->uc_mcontext.gregs[REG_RIP];
  void* fr[kDepth + 2] = {};
  const int n = backtrace(fr, kDepth + 2);  // [0] this handler, [1] the signal trampoline
  for (int k = 1; k < kDepth; ++k) g_samples[i][k] = k + 1 < n ? fr[k + 1] : nullptr;
}
void prof_start() {
  void* warm[4];
  backtrace(warm, 4);  // loads the unwinder outside the handler
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  itimerval it{{0, 200}, {0, 200}};
  setitimer(ITIMER_PROF, &it, nullptr);
}
void prof_stop(const char* path) {
  itimerval it{};
  setitimer(ITIMER_PROF, &it, nullptr);
  FILE* f = std::fopen(path, "w");
  if (!f) return;
  const int n = std::min(g_nsamples.load(), kMaxSamples);
  for (int i = 0; i < n; ++i) {  // one line per sample: "<object>:<offset>" frames, pc first
    for (int k = 0; k < kDepth && g_samples[i][k]; ++k) {
      Dl_info d{};
      void* pc = g_samples[i][k];
      if (dladdr(pc, &d) && d.dli_fname)
        std::fprintf(f, "%s%s:%#lx", k ? " " : "", d.dli_fname,
                     (unsigned long)((char*)pc - (char*)d.dli_fbase));
      else
        std::fprintf(f, "%s?:%p", k ? " " : "", pc);
    }
    std::fprintf(f, "\n");
  }
  std::fclose(f);
}

}  // namespace

int main(int argc, char** argv) {
  int threads = 32, calls = 1000, len = 64, T = 4096;
  bool varied = false, free_midway = false, light = false;
  std::string kind = "ambiguous", rhs_file, strings_file;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&] { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--threads") threads = std::atoi(next().c_str());
    else if (a == "--calls") calls = std::atoi(next().c_str());
    else if (a == "--len") len = std::atoi(next().c_str());
    else if (a == "--transducer-len") T = std::atoi(next().c_str());
    else if (a == "--rhs") kind = next();
    else if (a == "--varied") varied = true;
    else if (a == "--free-midway") free_midway = true;
    else if (a == "--light-check") light = true;  // state count only (no per-arc reads)
    else if (a == "--rhs-file") rhs_file = next();
    else if (a == "--strings-file") strings_file = next();
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  const FstHandle rhs = rhs_file.empty() ? fst_bench_transducer(kind == "eps_dense" ? 1 : 0, T, 12)
                                          : fst_batch_load(rhs_file.c_str());
  if (rhs == FST_INVALID_HANDLE) return 2;
  std::vector<std::vector<uint8_t>> texts;
  if (!strings_file.empty()) {  // the caller's strings (labels = byte + 1)
    FILE* f = std::fopen(strings_file.c_str(), "rb");
    if (!f) return 2;
    uint32_t num = 0;
    bool ok = std::fread(&num, 4, 1, f) == 1;
    std::vector<uint64_t> off(num + 1);
    ok = ok && std::fread(off.data(), 8, num + 1, f) == num + 1;
    std::vector<uint32_t> lab(ok ? off[num] : 0);
    ok = ok && std::fread(lab.data(), 4, lab.size(), f) == lab.size();
    std::fclose(f);
    if (!ok || num == 0) return 2;
    texts.resize(num);
    for (uint32_t d = 0; d < num; ++d)
      for (uint64_t k = off[d]; k < off[d + 1]; ++k) {
        if (lab[k] == 0 || lab[k] > 256) return 2;  // not a byte string
        texts[d].push_back((uint8_t)(lab[k] - 1));
      }
    kind = "file";
  } else {
    // the distinct strings: bytes 0 (label 1), lengths 1..len when varied, some dead (byte 1)
    const int nd = varied ? 64 : 1;
    texts.resize(nd);
    for (int d = 0; d < nd; ++d) {
      const int L = varied ? 1 + (d * 37) % len : len;
      texts[d].assign(L, 0);
      if (varied && d % 10 == 3) texts[d][L / 2] = 1;  // label 2: no rhs arc (empty result)
    }
  }
  const int distinct = (int)texts.size();
  // expected answers from the batch entry (lazy semantics, like the single call)
  std::vector<uint32_t> labels;
  std::vector<uint64_t> offs{0};
  for (auto& t : texts) {
    for (uint8_t c : t) labels.push_back(c + 1u);
    offs.push_back(labels.size());
  }
  FstBatchOptions opts{-1, FST_SEM_LAZY, 0};
  FstBatchResult br;
  if (fst_compose_frozen_shortest_path_batch(rhs, labels.data(), offs.data(), distinct, 1, &opts,
                                             &br) != FST_OK)
    return 3;
  std::vector<Expect> expect(distinct);
  for (int d = 0; d < distinct; ++d) {
    expect[d].status = br.status[d];
    expect[d].fin = br.final_weights[d];
    for (uint64_t k = br.path_offsets[d]; k < br.path_offsets[d + 1]; ++k)
      expect[d].arcs.push_back(FstArc{br.ilabels[k], br.olabels[k], br.weights[k],
                                      (uint32_t)(k - br.path_offsets[d] + 1)});
  }
  fst_batch_result_free(&br);

  std::atomic<long> mismatches{0}, invalid{0}, done_calls{0};
  std::atomic<bool> freed{false};
  auto worker = [&](int t) {
    std::vector<FstArc> buf(4096);
    for (int i = 0; i < calls; ++i) {
      const int d = (t * 7919 + i) % distinct;
      const FstMutableHandle a = fst_compile_string(texts[d].data(), (uint32_t)texts[d].size());
      const bool was_freed = freed.load();
      const FstMutableHandle r = fst_compose_frozen_shortest_path(a, rhs, 1);
      fst_mutable_free(a);
      done_calls.fetch_add(1);
      if (r == FST_INVALID_HANDLE) {
        // only legitimate once the rhs handle is gone
        if (!free_midway || !(was_freed || freed.load())) mismatches.fetch_add(1);
        else invalid.fetch_add(1);
        continue;
      }
      const Expect& e = expect[d];
      bool ok;
      if (e.status != 0) {  // FST_PATH_EMPTY: no states
        ok = fst_mutable_num_states(r) == 0;
      } else {
        const uint32_t P = (uint32_t)e.arcs.size();
        ok = fst_mutable_num_states(r) == P + 1 && fst_mutable_start(r) == 0 &&
             same(fst_mutable_final_weight(r, P), e.fin);
        for (uint32_t k = 0; ok && !light && k < P; ++k) {
          ok = fst_mutable_get_arcs(r, k, buf.data(), 2) == 1 && buf[0].ilabel == e.arcs[k].ilabel &&
               buf[0].olabel == e.arcs[k].olabel && same(buf[0].weight, e.arcs[k].weight) &&
               buf[0].nextstate == k + 1;
        }
      }
      if (!ok) mismatches.fetch_add(1);
      fst_mutable_free(r);
    }
  };
  auto cpu_now = [] {  // process CPU seconds (user + system), all threads
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return u.ru_utime.tv_sec + u.ru_stime.tv_sec + 1e-6 * (u.ru_utime.tv_usec + u.ru_stime.tv_usec);
  };
  const char* prof_path = std::getenv("CC_PROF");
  if (prof_path) prof_start();
  const double cpu0 = cpu_now();
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back(worker, t);
  if (free_midway) {
    while (done_calls.load() < (long)threads * calls / 2) std::this_thread::yield();
    freed.store(true);
    fst_free(rhs);
  }
  for (auto& x : th) x.join();
  const double secs =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double cpu_s = cpu_now() - cpu0;
  if (prof_path) prof_stop(prof_path);
  if (!free_midway) fst_free(rhs);
  std::printf(
      "{\"threads\": %d, \"calls_per_thread\": %d, \"len\": %d, \"rhs\": \"%s\", "
      "\"transducer_len\": %d, \"varied\": %s, \"free_midway\": %s, \"seconds\": %.4f, "
      "\"calls_per_s\": %.1f, \"cpu_seconds\": %.3f, \"mismatches\": %ld, "
      "\"invalid_after_free\": %ld}\n",
      threads, calls, len, kind.c_str(), T, varied ? "true" : "false",
      free_midway ? "true" : "false", secs, threads * (double)calls / secs, cpu_s,
      mismatches.load(), invalid.load());
  return mismatches.load() == 0 ? 0 : 1;
}
