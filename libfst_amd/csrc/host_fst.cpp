// host_fst.cpp -- MutableFst helpers and the frozen blob (see host_fst.hpp).
#include "host_fst.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cctype>
#include <exception>
#include <new>
#include <cstdlib>
#include <string>
#include <thread>

#include "device_engine.hpp"

namespace fstamd {

// ---- AT&T text (src/io/text.zig:20-123) ---------------------------------------------

namespace {

// std.fmt.parseInt(u32, s, 10): optional sign, decimal digits, '_' between digits;
// out of range (or a negative non-zero) is an error.
bool parse_u32(const char* b, const char* e, uint32_t* out) {
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = *b == '-';
    ++b;
  }
  if (b == e || *b == '_' || e[-1] == '_') return false;
  uint64_t x = 0;
  for (const char* c = b; c < e; ++c) {
    if (*c == '_') continue;
    if (*c < '0' || *c > '9') return false;
    x = x * 10 + (uint64_t)(*c - '0');
    if (x > 0xFFFFFFFFull) return false;
  }
  if (neg && x != 0) return false;
  *out = (uint32_t)x;
  return true;
}

// parseWeight (:117-123): "inf" / "Infinity" -> Zero, else std.fmt.parseFloat(f64).
bool parse_weight(const char* b, const char* e, double* out) {
  const std::string t(b, e);
  if (t == "inf" || t == "Infinity") {
    *out = w_zero();
    return true;
  }
  if (t.empty() || std::isspace((unsigned char)t[0])) return false;
  errno = 0;
  char* end = nullptr;
  const double v = std::strtod(t.c_str(), &end);
  if (end != t.c_str() + t.size()) return false;
  *out = v;
  return true;
}

}  // namespace

bool MutableFst::read_text(const char* data, size_t len, MutableFst* out) {
  // a state id asks for that many states (ensure below): a huge one fails the allocation,
  // which must come back as an error, not cross the C ABI as an exception
  try {
    return read_text_impl(data, len, out);
  } catch (const std::exception&) {
    return false;
  }
}

bool MutableFst::read_text_impl(const char* data, size_t len, MutableFst* out) {
  MutableFst f;
  bool start_set = false;
  // states up to the largest id named (the reference adds them one by one and fails with
  // OutOfMemory when they do not fit): a table larger than the host's physical memory is
  // refused up front instead of being left to the allocator and overcommit
  const size_t phys = (size_t)sysconf(_SC_PHYS_PAGES) * (size_t)sysconf(_SC_PAGESIZE);
  auto ensure = [&](uint32_t s) {
    if (f.num_states() > s) return;
    if (((size_t)s + 1) * sizeof(State) > phys) throw std::bad_alloc();
    f.add_states((size_t)s + 1 - f.num_states());
  };
  const char* p = data;
  const char* end = data + len;
  while (p <= end) {
    const char* nl = (const char*)std::memchr(p, '\n', (size_t)(end - p));
    const char* le = nl ? nl : end;
    // trim '\r', ' ', '\t' on both sides
    const char* b = p;
    const char* e = le;
    auto ws = [](char c) { return c == '\r' || c == ' ' || c == '\t'; };
    while (b < e && ws(*b)) ++b;
    while (e > b && ws(e[-1])) --e;
    p = le + 1;
    if (b == e) {
      if (!nl) break;
      continue;
    }
    // tokenizeAny(" \t")
    const char* tb[6];
    const char* te[6];
    int nt = 0;
    for (const char* c = b; c < e && nt < 6;) {
      while (c < e && (*c == ' ' || *c == '\t')) ++c;
      if (c == e) break;
      tb[nt] = c;
      while (c < e && *c != ' ' && *c != '\t') ++c;
      te[nt++] = c;
    }
    uint32_t src;
    if (!parse_u32(tb[0], te[0], &src)) return false;
    ensure(src);
    if (!start_set) {
      f.set_start(src);
      start_set = true;
    }
    if (nt == 1) {  // single field: final with One
      f.set_final(src, w_one());
    } else {
      uint32_t dest;
      if (!parse_u32(tb[1], te[1], &dest)) {  // "state weight"
        double w;
        if (!parse_weight(tb[1], te[1], &w) || nt > 2) return false;
        f.set_final(src, w);
      } else if (nt == 2) {
        double w;
        if (parse_weight(tb[1], te[1], &w)) {
          f.set_final(src, w);
        } else {  // "src dest": an epsilon arc
          ensure(dest);
          f.add_arc(src, Arc{kEpsilon, kEpsilon, w_one(), dest});
        }
      } else {
        ensure(dest);
        uint32_t il;
        if (!parse_u32(tb[2], te[2], &il) || nt > 5) return false;
        uint32_t ol = il;
        double w = w_one();
        if (nt >= 4) {
          if (!parse_u32(tb[3], te[3], &ol)) {  // the fourth field is the weight
            ol = il;
            if (!parse_weight(tb[3], te[3], &w)) return false;
            f.add_arc(src, Arc{il, ol, w, dest});
            if (!nl) break;
            continue;
          }
          if (nt == 5 && !parse_weight(tb[4], te[4], &w)) return false;
        }
        f.add_arc(src, Arc{il, ol, w, dest});
      }
    }
    if (!nl) break;
  }
  *out = std::move(f);
  return true;
}

void MutableFst::shift_labels() {
  for (State& s : states_)
    for (Arc& a : s.arcs) {
      if (a.ilabel != kEpsilon) a.ilabel += 1;
      if (a.olabel != kEpsilon) a.olabel += 1;
    }
}

MutableFst MutableFst::compile_string(const uint8_t* in, uint32_t in_len, const uint8_t* out,
                                      uint32_t out_len) {
  MutableFst f;
  const uint32_t max_len = std::max(in_len, out_len);
  if (max_len == 0) {  // empty string: one final state (src/string.zig:30-36)
    StateId s = f.add_state();
    f.set_start(s);
    f.set_final(s, w_one());
    return f;
  }
  f.add_states(max_len + 1);
  f.set_start(0);
  f.set_final(max_len, w_one());
  for (uint32_t i = 0; i < max_len; ++i) {
    Label il = i < in_len ? (Label)in[i] + 1 : kEpsilon;  // label = byte + 1
    Label ol = i < out_len ? (Label)out[i] + 1 : kEpsilon;
    f.add_arc(i, Arc{il, ol, w_one(), i + 1});
  }
  return f;
}

MutableFst MutableFst::compile_chain(const std::vector<Label>& labels) {
  MutableFst f;
  const uint32_t L = (uint32_t)labels.size();
  f.add_states((size_t)L + 1);
  f.set_start(0);
  f.set_final(L, w_one());
  for (uint32_t i = 0; i < L; ++i) f.add_arc(i, Arc{labels[i], labels[i], w_one(), i + 1});
  return f;
}

bool MutableFst::print_string(bool output_tape, std::vector<uint8_t>* bytes) const {
  StateId cur = start_;
  if (cur == kNoState) return false;
  bytes->clear();
  size_t steps = 0;
  for (;;) {
    const State& s = states_[cur];
    if (!w_is_zero(s.final_weight) && s.arcs.empty()) break;
    if (s.arcs.size() != 1) return false;  // not a linear chain
    const Arc& a = s.arcs[0];
    Label l = output_tape ? a.olabel : a.ilabel;
    if (l != kEpsilon) {
      if (l - 1 > 255u) return false;  // would be a safety panic in the reference
      bytes->push_back((uint8_t)(l - 1));
    }
    cur = a.nextstate;
    if (cur == kNoState || cur >= states_.size()) return false;
    if (++steps > states_.size()) return false;  // the reference would walk forever
  }
  return true;
}

std::shared_ptr<FrozenFst> FrozenFst::from_mutable(const MutableFst& m, uint8_t weight_type) {
  std::shared_ptr<FrozenFst> f(new FrozenFst());
  const uint32_t ns = (uint32_t)m.num_states();
  const uint64_t na = m.total_arcs();
  const size_t len = sizeof(Header) + (size_t)ns * sizeof(StateEntry) + (size_t)na * sizeof(PackedArc);
  if (!f->alloc(len)) throw std::bad_alloc();
  uint8_t* b = f->buf_;
  std::memset(b, 0, len);  // header and arc padding are zero (byte-identical blobs)
  Header* h = reinterpret_cast<Header*>(b);
  h->magic = kMagic;
  h->version = kVersion;
  h->weight_type = weight_type;
  h->flags = 0;
  h->num_states = ns;
  h->num_arcs = (uint32_t)na;
  h->start_state = m.start();
  StateEntry* se = reinterpret_cast<StateEntry*>(b + sizeof(Header));
  PackedArc* pa = reinterpret_cast<PackedArc*>(b + sizeof(Header) + (size_t)ns * sizeof(StateEntry));
  std::vector<Arc> work;
  uint32_t off = 0;
  for (uint32_t i = 0; i < ns; ++i) {
    work = m.arcs(i);
    std::stable_sort(work.begin(), work.end(), arc_less);
    se[i].arc_offset = off;
    se[i].num_arcs = (uint32_t)work.size();
    se[i].final_weight = m.final_weight(i);
    for (const Arc& a : work) {
      pa[off].ilabel = a.ilabel;
      pa[off].olabel = a.olabel;
      pa[off].weight = a.weight;
      pa[off].nextstate = a.nextstate;
      ++off;
    }
  }
  f->analyze();
  return f;
}

BlobError FrozenFst::validate(const uint8_t* b, size_t len, uint8_t expect_wt) {
  if (len < sizeof(Header)) return BlobError::kInvalidFormat;
  Header h;
  std::memcpy(&h, b, sizeof(h));
  if (h.magic != kMagic) return BlobError::kInvalidMagic;
  if (h.version != kVersion) return BlobError::kUnsupportedVersion;
  if (h.weight_type != expect_wt) return BlobError::kWeightTypeMismatch;
  const size_t expected = sizeof(Header) + (size_t)h.num_states * sizeof(StateEntry) +
                          (size_t)h.num_arcs * sizeof(PackedArc);
  if (len != expected) return BlobError::kInvalidFormat;
  if (h.num_states > 0 && h.start_state != kNoState && h.start_state >= h.num_states)
    return BlobError::kInvalidFormat;
  if (h.num_states == 0 && h.start_state != kNoState) return BlobError::kInvalidFormat;
  for (uint32_t i = 0; i < h.num_states; ++i) {
    StateEntry e;
    std::memcpy(&e, b + sizeof(Header) + (size_t)i * sizeof(StateEntry), sizeof(e));
    if (e.arc_offset > h.num_arcs) return BlobError::kInvalidFormat;
    if (e.num_arcs > h.num_arcs - e.arc_offset) return BlobError::kInvalidFormat;
    bool have_last = false;
    uint32_t last = 0;
    for (uint32_t k = 0; k < e.num_arcs; ++k) {
      PackedArc a;
      std::memcpy(&a,
                  b + sizeof(Header) + (size_t)h.num_states * sizeof(StateEntry) +
                      (size_t)(e.arc_offset + k) * sizeof(PackedArc),
                  sizeof(a));
      if (a.nextstate >= h.num_states) return BlobError::kInvalidFormat;
      if (have_last && a.ilabel < last) return BlobError::kInvalidFormat;
      last = a.ilabel;
      have_last = true;
    }
  }
  return BlobError::kOk;
}

std::shared_ptr<FrozenFst> FrozenFst::from_bytes(const uint8_t* bytes, size_t len,
                                                 uint8_t expect_wt, BlobError* err) {
  BlobError e = validate(bytes, len, expect_wt);
  if (err) *err = e;
  if (e != BlobError::kOk) return nullptr;
  std::shared_ptr<FrozenFst> f(new FrozenFst());
  if (!f->alloc(len)) return nullptr;
  std::memcpy(f->buf_, bytes, len);
  f->analyze();
  return f;
}

bool FrozenFst::alloc(size_t len) {
  const size_t cap = (len + 7) & ~(size_t)7;
  void* p = nullptr;
  // small blobs (test graphs, toy grammars) stay pageable: pinning costs a syscall and a
  // page per blob, and their upload is tiny either way
  if (cap >= (64u << 10) &&
      hipHostMalloc(&p, cap, hipHostMallocDefault) == hipSuccess && p) {
    pinned_ = true;
  } else {
    (void)hipGetLastError();  // no device: clear the runtime's sticky error
    p = std::aligned_alloc(8, std::max<size_t>(cap, 8));
    if (!p) return false;
    pinned_ = false;
  }
  buf_ = (uint8_t*)p;
  size_ = len;
  if (cap > len) std::memset(buf_ + len, 0, cap - len);
  return true;
}

std::shared_ptr<FrozenFst> FrozenFst::load_file(const char* path, uint8_t expect_wt,
                                                BlobError* err) {
  if (err) *err = BlobError::kInvalidFormat;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return nullptr;
  struct stat st;
  if (::fstat(fd, &st) != 0 || st.st_size < (off_t)sizeof(Header)) {
    ::close(fd);
    return nullptr;
  }
  const size_t len = (size_t)st.st_size;
  (void)::posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  std::shared_ptr<FrozenFst> f(new FrozenFst());
  if (!f->alloc(len)) {
    ::close(fd);
    return nullptr;
  }
  // pread straight into the pinned block; files of many MB on several threads (a WeText
  // tagger is tens of MB, config 3's rhs 21.5 MB)
  const size_t piece = 16ull << 20;
  const uint32_t nth = (uint32_t)std::min<size_t>(8, std::max<size_t>(1, len / piece));
  std::vector<uint8_t> ok(nth, 1);
  auto rd = [&](uint32_t t) {
    size_t lo = len * t / nth, hi = len * (t + 1) / nth;
    while (lo < hi) {
      const ssize_t r = ::pread(fd, f->buf_ + lo, hi - lo, (off_t)lo);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        ok[t] = 0;
        return;
      }
      lo += (size_t)r;
    }
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < nth; ++t) th.emplace_back(rd, t);
  rd(0);
  for (auto& x : th) x.join();
  ::close(fd);
  for (uint8_t o : ok)
    if (!o) return nullptr;
  uint8_t wt = expect_wt;
  if (expect_wt == kAnyWeightType) {
    wt = reinterpret_cast<const Header*>(f->buf_)->weight_type;
    if (wt != kWeightTropical && wt != kWeightLog) return nullptr;
  }
  const BlobError e = validate(f->buf_, len, wt);
  if (err) *err = e;
  if (e != BlobError::kOk) return nullptr;
  f->analyze();
  return f;
}

void FrozenFst::analyze() {
  has_eps_ = false;
  nonneg_ = true;
  nan_ = false;
  finite_ = true;
  const Header& h = header();
  const PackedArc* a = arcs();
  for (uint32_t i = 0; i < h.num_arcs; ++i) {
    if (a[i].ilabel == kEpsilon) has_eps_ = true;
    const double w = a[i].weight;
    if (!(w >= 0.0) || std::signbit(w)) nonneg_ = false;  // negative, -0.0 or NaN
    if (std::isnan(w)) nan_ = true;
    if (!std::isfinite(w)) finite_ = false;
  }
  const StateEntry* s = states();
  jump_fwd_ = jump_back_ = 0;
  for (uint32_t i = 0; i < h.num_states; ++i) {
    const double w = s[i].final_weight;
    if (!(w >= 0.0) || std::signbit(w)) nonneg_ = false;
    if (std::isnan(w)) nan_ = true;
    for (uint32_t k = s[i].arc_offset; k < s[i].arc_offset + s[i].num_arcs; ++k) {
      const uint32_t t = a[k].nextstate;
      if (t >= i) jump_fwd_ = std::max(jump_fwd_, t - i);
      else jump_back_ = std::max(jump_back_, i - t);
    }
  }
}

double FrozenFst::chain_cost(uint64_t L) const {
  // sum over input positions k = 0..L of the rhs states layer k can hold: min(NS, 1 + k J),
  // J = the widest forward + backward jump of one arc; an rhs with input epsilons can
  // spread a layer over every state (config 3: ~2 (T + 1) tuples per layer)
  const double ns = std::max<uint32_t>(num_states(), 1);
  if (has_eps_) return (double)(L + 1) * ns;
  const double J = std::max<uint32_t>(jump_fwd_ + jump_back_, 1);
  const double K = std::ceil((ns - 1) / J);  // layers below the cap
  const double l1 = (double)L + 1;
  if (l1 <= K) return l1 + J * (double)L * l1 / 2;
  return K + J * (K - 1) * K / 2 + (l1 - K) * ns;
}

void FrozenFst::arcs_by_ilabel(StateId s, Label label, uint32_t* lo_out, uint32_t* hi_out) const {
  const StateEntry& e = states()[s];
  const PackedArc* a = arcs() + e.arc_offset;
  uint32_t lo = 0, hi = e.num_arcs;
  while (lo < hi) {
    uint32_t mid = lo + (hi - lo) / 2;
    if (a[mid].ilabel < label) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t first = lo;
  hi = e.num_arcs;
  while (lo < hi) {
    uint32_t mid = lo + (hi - lo) / 2;
    if (a[mid].ilabel <= label) lo = mid + 1;
    else hi = mid;
  }
  *lo_out = e.arc_offset + first;
  *hi_out = e.arc_offset + lo;
}

DeviceFst* FrozenFst::device(int dev) {
  std::lock_guard<std::mutex> g(dev_mu_);
  if ((int)dev_.size() <= dev) dev_.resize(dev + 1, nullptr);
  if (!dev_[dev]) dev_[dev] = DeviceFst::create(*this, dev);
  return dev_[dev];
}

void FrozenFst::adopt_device(int dev, DeviceFst* d) {
  std::lock_guard<std::mutex> g(dev_mu_);
  if ((int)dev_.size() <= dev) dev_.resize(dev + 1, nullptr);
  if (dev_[dev]) DeviceFst::destroy(dev_[dev]);
  dev_[dev] = d;
}

FrozenFst::~FrozenFst() {
  for (DeviceFst* d : dev_)
    if (d) DeviceFst::destroy(d);
  if (buf_) {
    if (pinned_) (void)hipHostFree(buf_);
    else std::free(buf_);
  }
}

}  // namespace fstamd
