// host_fst.cpp -- MutableFst helpers and the frozen blob (see host_fst.hpp).
#include "host_fst.hpp"

#include <algorithm>

#include "device_engine.hpp"

namespace fstamd {

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
  f->size_ = sizeof(Header) + (size_t)ns * sizeof(StateEntry) + (size_t)na * sizeof(PackedArc);
  f->buf_.assign((f->size_ + 7) / 8, 0);
  uint8_t* b = reinterpret_cast<uint8_t*>(f->buf_.data());
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
  f->size_ = len;
  f->buf_.assign((len + 7) / 8, 0);
  std::memcpy(f->buf_.data(), bytes, len);
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
  for (uint32_t i = 0; i < h.num_states; ++i) {
    const double w = s[i].final_weight;
    if (!(w >= 0.0) || std::signbit(w)) nonneg_ = false;
    if (std::isnan(w)) nan_ = true;
  }
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
}

}  // namespace fstamd
