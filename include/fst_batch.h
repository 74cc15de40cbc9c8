/*
 * fst_batch.h -- batched entry points of libfst_amd (new; no libfst counterpart).
 *
 * A batch is N linear-chain acceptors given as CSR label sequences
 * (labels[offsets[i] .. offsets[i+1]) for string i).  Each string is the FST
 * `fst_compile_string` would build (src/string.zig:24-50): state k --l:l/One-->
 * k+1, final(L) = One; labels are used as given (fst_compile_string's byte+1
 * encoding is the caller's choice).  Every string is composed against ONE
 * frozen rhs FstHandle and reduced to its 1-best path with either
 *   FST_SEM_LAZY : the result fst_compose_frozen_shortest_path(a, b, n) returns
 *                  (src/ops/compose-shortest-path.zig:26-401), or
 *   FST_SEM_EAGER: the result fst_shortest_path(fst_compose_frozen(a, b), n)
 *                  returns (src/ops/compose.zig:29-198 then
 *                  src/ops/shortest-path.zig:18-139) -- what the reference bench
 *                  scenario compose_frozen_shortest_path_* measures.
 * The two agree on weight but may pick different equal-weight paths.
 *
 * Per-string results use the FST_PATH_* codes; a string with FST_PATH_OK has a
 * result chain of path_len arcs (states 0..path_len, start 0, final(path_len) =
 * final_weight), FST_PATH_EMPTY is the reference's empty FST.
 */
#ifndef LIBFST_AMD_FST_BATCH_H
#define LIBFST_AMD_FST_BATCH_H

#include "fst.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    FST_SEM_LAZY = 0,
    FST_SEM_EAGER = 1,
} FstSemantics;

typedef enum {
    FST_PATH_OK = 0,           /* a 1-best chain */
    FST_PATH_EMPTY = 1,        /* empty result FST (no path, n == 0, or rhs has no start) */
    FST_PATH_ERROR_N = 2,      /* n not in {0, 1}: the reference returns FST_INVALID_HANDLE */
    FST_PATH_CYCLE = 3,        /* back-pointer cycle; the reference would not terminate */
    FST_PATH_OVERFLOW = 4,     /* internal: engine capacity exceeded (retried internally) */
    FST_PATH_UNSUPPORTED = 5,  /* input outside every available engine's contract */
    FST_PATH_OUTPUT_FULL = 6,  /* device arc arena too small */
    FST_PATH_INTERNAL = 7,     /* engine invariant violated (a bug), reported, never silent */
} FstPathStatus;

/* Host-memory result of a batch, allocated by the library (pooled pinned host blocks the
 * device writes by DMA) and valid until fst_batch_result_free(), which returns them. */
typedef struct {
    uint32_t num_strings;
    int32_t* status;          /* [num_strings] FstPathStatus */
    uint64_t* path_offsets;   /* [num_strings + 1] CSR offsets into the arc arrays */
    uint32_t* ilabels;        /* [total_arcs] */
    uint32_t* olabels;        /* [total_arcs] */
    double* weights;          /* [total_arcs] */
    double* final_weights;    /* [num_strings] */
    uint64_t total_arcs;
} FstBatchResult;

/* Multi-GPU batches inside the library: with FST_BATCH_DEVICES in flags the
 * host entries (fst_compose_frozen_shortest_path_batch, fst_pipeline_batch) split the
 * strings into contiguous shards balanced by estimated work (sum over the string's input
 * positions of the rhs states a layer can hold) and run one shard per device of
 * device_mask (bit d = HIP device d), each on its own host thread, with the frozen rhs
 * replicated to every device on first use (one DMA from its pinned host copy).  Results
 * are gathered into one FstBatchResult in input order, identical to a one-device run.
 * num_shards > popcount(device_mask) runs several shards per device (round robin) on
 * separate engines and streams; 0 = one per device.  No collective runs on the data path. */
#define FST_BATCH_DEVICES 1u

/* The work estimate the shard planner uses for one chain string of `len` labels against
 * rhs b (product tuples: the sum over input positions of the rhs states a layer can hold),
 * for callers that shard batches over processes themselves (one rank per GPU); < 0 for an
 * invalid handle. */
double fst_chain_cost(FstHandle b, uint64_t len);

typedef struct {
    int32_t device;           /* HIP device ordinal (-1: current device); without
                                 FST_BATCH_DEVICES the whole batch runs there */
    uint32_t semantics;       /* FstSemantics */
    uint32_t flags;           /* FST_BATCH_DEVICES or 0 */
    uint32_t num_shards;      /* with FST_BATCH_DEVICES: shards (0 = one per device) */
    uint64_t device_mask;     /* with FST_BATCH_DEVICES: the devices (0 = `device` only) */
} FstBatchOptions;

/* Host arrays in, host result out (H2D, kernels, D2H).  Returns FST_INVALID_ARG for an
 * invalid handle or malformed offsets; per-string outcomes are in out->status.  Once the
 * arguments are checked, *out is zeroed before anything else: on any error return it holds
 * nothing (a result the caller still owned in that struct must be freed beforehand). */
FstError fst_compose_frozen_shortest_path_batch(FstHandle b, const uint32_t* labels,
                                                const uint64_t* offsets, uint32_t num_strings,
                                                uint32_t n, const FstBatchOptions* opts,
                                                FstBatchResult* out);
void fst_batch_result_free(FstBatchResult* r);

/* Device-resident batch: every pointer is device memory on opts->device; the call is
 * asynchronous on `stream` (a hipStream_t, or NULL for the null stream).  Paths are
 * appended to the arc arena; *arc_cursor (device) is reset by the call.  `work`, if
 * non-NULL, receives two counters per string: product states and relaxations.
 * max_len (fst_device_compose_shortest_path) is the caller's bound on the strings'
 * lengths: it sizes workspaces and picks kernels (e.g. f32 cells when every distance
 * stays an exact integer below 2^24).  A string longer than max_len is still answered
 * exactly, by a slower tier. */
typedef struct {
    int32_t* status;            /* [num_strings] */
    uint32_t* path_len;         /* [num_strings] */
    uint64_t* path_offset;      /* [num_strings] offset of the string's first arc */
    double* final_weight;       /* [num_strings] */
    uint32_t* ilabels;          /* [arc_capacity] */
    uint32_t* olabels;          /* [arc_capacity] */
    double* weights;            /* [arc_capacity] */
    uint64_t arc_capacity;
    uint64_t* arc_cursor;       /* [1] */
    uint32_t* work;             /* [2 * num_strings] or NULL */
} FstDeviceBatch;

FstError fst_device_compose_shortest_path(FstHandle b, const uint32_t* d_labels,
                                          const uint64_t* d_offsets, uint32_t num_strings,
                                          uint32_t max_len, uint32_t n,
                                          const FstBatchOptions* opts, const FstDeviceBatch* out,
                                          void* stream);

/* Multi-stage pipelines (tagger -> verbalizer, README.md:177-214) without host round
 * trips.  The reference app does, per utterance and stage:
 *   print_output_string(best) -> compile_string(bytes) -> compose_frozen_shortest_path.
 * On a 1-best chain that is: next input labels = the path's non-epsilon olabels
 * (src/string.zig:60-97 then :24-50; label = byte + 1 on both sides).
 * fst_device_project_output does that for a whole batch on the device.  A string whose
 * stage status is not OK, or whose output holds a label > 256 (not a byte: the
 * reference's @intCast would trap), gets one input label no rhs carries (the next stage
 * reports EMPTY) and its reason in d_proj_status (the stage's status, or
 * FST_PATH_UNSUPPORTED for a non-byte label).  d_next_labels needs room for the sum of
 * path_len plus num_strings; d_next_offsets for num_strings + 1.  Synchronises `stream`
 * and returns the longest projected input in *max_len. */
FstError fst_device_project_output(const FstDeviceBatch* stage, uint32_t num_strings,
                                   uint32_t* d_next_labels, uint64_t* d_next_offsets,
                                   int32_t* d_proj_status, uint32_t* max_len, void* stream);

/* Host convenience: runs num_stages frozen FSTs in sequence on one device, each stage's
 * 1-best output tape feeding the next (fst_device_project_output in between).  The
 * result holds the last stage's paths; a string that failed at an earlier stage reports
 * that stage's status.  Semantics / device from opts (NULL: lazy, current device). */
FstError fst_pipeline_batch(const FstHandle* stages, uint32_t num_stages, const uint32_t* labels,
                            const uint64_t* offsets, uint32_t num_strings, uint32_t n,
                            const FstBatchOptions* opts, FstBatchResult* out);

/* Bring a frozen FST's device copy up on `device` (blob H2D + on-device SoA mirror). */
FstError fst_device_prepare(FstHandle b, int32_t device);
/* Adopt a blob that already sits in device memory on `device` (e.g. received by an
 * RCCL broadcast): validates the header, builds the SoA mirror, returns a new handle.
 * `host_copy` must hold the same bytes (used for host-side queries); may be NULL, in
 * which case the bytes are copied back from the device. */
FstHandle fst_device_adopt_blob(const void* d_blob, uint64_t len, int32_t device,
                                const void* host_copy);

/* Engine introspection for benchmarks (last device launch on this thread). */
typedef struct {
    double kernel_ms;           /* sum of kernel durations, HIP events on the launch stream */
    uint32_t launches;          /* kernel launches in the call */
    uint32_t engine;            /* 0 = eager-layered, 1 = lazy replay, 2 = eager-general,
                                   3 = lazy rounds, 4 = lazy layered (+ rounds for the rest),
                                   5 = lazy dense replay, 6 = shortest-path heap replay */
    uint32_t grid;              /* workgroups of the dominant kernel */
} FstLaunchStats;
FstError fst_last_launch_stats(FstLaunchStats* out);

/* Generators of the reference bench's synthetic rhs (bench/optimize-bench.zig:219-306),
 * built host-side and frozen: 0 = ambiguous chain, 1 = epsilon dense, 2 = branching. */
FstHandle fst_bench_transducer(uint32_t kind, uint32_t transducer_len, uint32_t branches);
/* Same, frozen with the given weight type (0 = tropical, 1 = log; src/fst.zig:43-47). */
FstHandle fst_bench_transducer_wt(uint32_t kind, uint32_t transducer_len, uint32_t branches,
                                  uint32_t weight_type);

/* Frozen blobs of either weight type for the batch entries ("weight_type
 * taken from the blob header").  fst_load stays Tropical-only like the reference c-api
 * (src/c-api.zig:601, W = TropicalWeight); these accept header weight_type 0 (tropical)
 * or 1 (log) and otherwise validate exactly like Fst.fromBytes (src/fst.zig:227-273).
 * On this path LogWeight's times / compare / isZero equal TropicalWeight's
 * (src/weight.zig:15-37 vs :88-104; log-add `plus` is never used), so both run through
 * the same engines. */
FstHandle fst_batch_load(const char* path);
FstHandle fst_batch_load_bytes(const void* bytes, uint64_t len);
/* OpenFst AT&T text -> frozen FST in one call: readText (src/io/text.zig:20-115; files up
 * to 256 MiB, src/tools/att2lfst.zig:40-45), then with FST_ATT_SHIFT_BYTE_LABELS every
 * non-epsilon ilabel / olabel + 1 (att2lfst.zig:54-60: OpenFst byte labels -> libfst's
 * byte + 1, so the asset matches fst_compile_string input), then fromMutable (Tropical).
 * tools/att2lfst (libfst_amd/att2lfst) is this plus fst_save. */
#define FST_ATT_SHIFT_BYTE_LABELS 1u
FstHandle fst_load_att(const char* path, uint32_t flags);

/* Header weight type of a frozen FST: 0 tropical, 1 log, -1 invalid handle. */
int32_t fst_weight_type(FstHandle b);

/* Diagnostics: the coalescer of single fst_compose_frozen_shortest_path calls on `device`
 * (leader slots in use, calls waiting in its queue).  Both are 0 when no call is in
 * flight; tests check that no slot leaks.  Returns -1 for a negative device. */
int32_t fst_debug_coalescer_state(int32_t device, uint32_t* queued);

#ifdef __cplusplus
}
#endif

#endif /* LIBFST_AMD_FST_BATCH_H */
