// host_fst.hpp -- host-side containers of libfst_amd.
//
//   MutableFst  : build-time graph used as lhs input and as result container
//                 (src/mutable-fst.zig:45-279; arcs kept in insertion order).
//   FrozenFst   : the frozen contiguous blob, byte-compatible with libfst's
//                 Fst(W) (src/fst.zig:51-288): fromMutable (sort + pack),
//                 fromBytes validation, arcsByIlabel.
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "fst_core.hpp"

namespace fstamd {

class MutableFst {
 public:
  struct State {
    double final_weight = w_zero();
    std::vector<Arc> arcs;
  };

  StateId add_state() {
    states_.emplace_back();
    return (StateId)(states_.size() - 1);
  }
  void add_states(size_t n) { states_.resize(states_.size() + n); }
  void set_start(StateId s) { start_ = s; }
  void set_final(StateId s, double w) { states_[s].final_weight = w; }
  void add_arc(StateId src, const Arc& a) { states_[src].arcs.push_back(a); }
  void reserve_arcs(StateId src, size_t n) { states_[src].arcs.reserve(n); }

  StateId start() const { return start_; }
  size_t num_states() const { return states_.size(); }
  size_t num_arcs(StateId s) const { return states_[s].arcs.size(); }
  double final_weight(StateId s) const { return states_[s].final_weight; }
  const std::vector<Arc>& arcs(StateId s) const { return states_[s].arcs; }
  size_t total_arcs() const {
    size_t t = 0;
    for (const auto& s : states_) t += s.arcs.size();
    return t;
  }

  // compileString / compileStringTransducer, src/string.zig:17-50
  static MutableFst compile_string(const uint8_t* in, uint32_t in_len, const uint8_t* out,
                                   uint32_t out_len);
  // The acceptor of a label chain (what c_api.cpp's as_chain recognises): states 0..L,
  // arc k = (c, c, One, k + 1), final(L) = One.
  static MutableFst compile_chain(const std::vector<Label>& labels);
  // printStringFromTape, src/string.zig:64-97.  Returns false for "null".
  bool print_string(bool output_tape, std::vector<uint8_t>* bytes) const;
  // readText, src/io/text.zig:20-115 (OpenFst AT&T text: "src dest il [ol] [w]" arcs,
  // "state [w]" finals, first source = start).  Returns false for error.InvalidFormat.
  static bool read_text(const char* data, size_t len, MutableFst* out);
  static bool read_text_impl(const char* data, size_t len, MutableFst* out);
  // att2lfst's label normalisation (src/tools/att2lfst.zig:54-60): every non-epsilon
  // ilabel / olabel + 1 (OpenFst byte labels -> libfst's byte + 1 convention).
  void shift_labels();

 private:
  std::vector<State> states_;
  StateId start_ = kNoState;
};

enum class BlobError { kOk, kInvalidFormat, kInvalidMagic, kUnsupportedVersion, kWeightTypeMismatch };

// Device-resident copy of one frozen FST on one HIP device (owned by FrozenFst).
struct DeviceFst;

class FrozenFst {
 public:
  // Fst.fromMutable, src/fst.zig:160-224 (sorts each state's arcs with
  // compareByIlabel -- a stable sort, like std.mem.sort -- then packs).
  static std::shared_ptr<FrozenFst> from_mutable(const MutableFst& m, uint8_t weight_type);
  // Fst.fromBytes, src/fst.zig:227-273 (copies the bytes into an owned buffer).
  static std::shared_ptr<FrozenFst> from_bytes(const uint8_t* bytes, size_t len,
                                               uint8_t expect_weight_type, BlobError* err);
  static BlobError validate(const uint8_t* bytes, size_t len, uint8_t expect_weight_type);
  // readBinary + fromBytes (src/io/binary.zig:16-36, src/fst.zig:227-273) without the
  // intermediate copy: the file is read straight into the blob's own pinned host block and
  // validated there, so the device copy is one DMA.  expect_weight_type 0xFF accepts either
  // semiring (the batch loaders); the reference's fst_load expects Tropical (0).
  static std::shared_ptr<FrozenFst> load_file(const char* path, uint8_t expect_weight_type,
                                              BlobError* err);
  static constexpr uint8_t kAnyWeightType = 0xFF;

  ~FrozenFst();

  const uint8_t* bytes() const { return buf_; }
  bool pinned() const { return pinned_; }
  size_t size() const { return size_; }
  const Header& header() const { return *reinterpret_cast<const Header*>(bytes()); }
  const StateEntry* states() const {
    return reinterpret_cast<const StateEntry*>(bytes() + sizeof(Header));
  }
  const PackedArc* arcs() const {
    return reinterpret_cast<const PackedArc*>(bytes() + sizeof(Header) +
                                              (size_t)header().num_states * sizeof(StateEntry));
  }
  StateId start() const { return header().start_state; }
  uint32_t num_states() const { return header().num_states; }
  uint32_t num_arcs(StateId s) const { return states()[s].num_arcs; }
  double final_weight(StateId s) const { return states()[s].final_weight; }
  uint8_t weight_type() const { return header().weight_type; }

  // Fst.arcsByIlabel, src/fst.zig:112-136: global arc index range [lo, hi).
  void arcs_by_ilabel(StateId s, Label label, uint32_t* lo, uint32_t* hi) const;

  // Properties the engines route on (computed once).
  bool has_epsilon_input() const { return has_eps_; }
  bool weights_nonnegative() const { return nonneg_; }
  bool has_nan_weight() const { return nan_; }
  bool arc_weights_finite() const { return finite_; }
  // Widest forward / backward state jump of one arc, and the estimated work of one chain
  // string of length L against this rhs (product tuples), for cost-balanced shards.
  uint32_t jump_fwd() const { return jump_fwd_; }
  uint32_t jump_back() const { return jump_back_; }
  double chain_cost(uint64_t L) const;

  // Lazily uploaded per-device copy (blob + SoA mirror); thread safe.
  DeviceFst* device(int dev);
  // Install a device copy built elsewhere (fst_device_adopt_blob); takes ownership.
  void adopt_device(int dev, DeviceFst* d);

 private:
  FrozenFst() = default;
  FrozenFst(const FrozenFst&) = delete;
  FrozenFst& operator=(const FrozenFst&) = delete;
  void analyze();
  // The blob's storage: a page-aligned pinned host block when the HIP runtime grants one
  // (device uploads are then one DMA, not staged through the runtime's bounce buffers),
  // 8-aligned malloc otherwise (no GPU).  Zero-filled past size_ to the next 8 bytes.
  bool alloc(size_t len);
  uint8_t* buf_ = nullptr;
  bool pinned_ = false;
  size_t size_ = 0;
  bool has_eps_ = false;
  bool nonneg_ = true;
  bool nan_ = false;
  bool finite_ = true;
  uint32_t jump_fwd_ = 0, jump_back_ = 0;
  std::mutex dev_mu_;
  std::vector<DeviceFst*> dev_;
};

}  // namespace fstamd
