// att2lfst -- OpenFst AT&T text -> libfst frozen blob (src/tools/att2lfst.zig), a client of
// the C ABI only: fst_load_att (readText + the +1 byte-label shift + fromMutable) and
// fst_save (writeBinary).  Output is byte-identical to the reference tool's.
//
// usage: att2lfst --input <att.txt> --output <libfst.fst>
#include <cstdio>
#include <cstring>

#include "../../include/fst_batch.h"

int main(int argc, char** argv) {
  if (argc != 5 || std::strcmp(argv[1], "--input") != 0 || std::strcmp(argv[3], "--output") != 0) {
    std::fprintf(stderr, "Usage: att2lfst --input <att.txt> --output <libfst.fst>\n");
    return 1;
  }
  const FstHandle h = fst_load_att(argv[2], FST_ATT_SHIFT_BYTE_LABELS);
  if (h == FST_INVALID_HANDLE) {
    std::fprintf(stderr, "error: InvalidFormat (%s)\n", argv[2]);
    return 1;
  }
  if (fst_save(h, argv[4]) != FST_OK) {
    std::fprintf(stderr, "error: cannot write %s\n", argv[4]);
    fst_free(h);
    return 1;
  }
  unsigned long long arcs = 0;
  const uint32_t ns = fst_num_states(h);
  for (uint32_t s = 0; s < ns; ++s) arcs += fst_num_arcs(h, s);
  std::fprintf(stderr, "Converted %s -> %s (states=%u, arcs=%llu)\n", argv[2], argv[4], ns, arcs);
  fst_free(h);
  return 0;
}
