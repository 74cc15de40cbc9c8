/*
 * fst.h -- libfst_amd's drop-in C ABI for ontypehq/libfst's frozen-compose hot path.
 *
 * Every declaration keeps the signature, argument meaning and error behaviour of
 * the libfst function it replaces (reference file:line cited per entry; the
 * reference header is include/fst.h of ontypehq/libfst).  Only the subset the
 * compose/1-best path needs is exported: building the lhs, freezing/loading the
 * rhs, the two compose entries, shortest path, result readback and strings.
 * Grammar-construction operations (determinize, minimize, union, cdrewrite, ...)
 * are out of scope for this engine.
 *
 * Thread safety mirrors the reference: handle-table bookkeeping runs under one
 * global mutex; compute runs outside it on snapshots; frozen FSTs are pinned
 * (not copied) for the duration of a call and may be freed concurrently.
 */
#ifndef LIBFST_AMD_FST_H
#define LIBFST_AMD_FST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Handles: (generation << 32) | slot, generation >= 1 (src/c-api.zig:109-130). */
typedef uint64_t FstMutableHandle;
typedef uint64_t FstHandle;

typedef enum { /* include/fst.h:34-40 */
    FST_OK = 0,
    FST_OOM = 1,
    FST_INVALID_ARG = 2,
    FST_INVALID_STATE = 3,
    FST_IO_ERROR = 4,
} FstError;

typedef struct { /* include/fst.h:50-55 (24 bytes) */
    uint32_t ilabel;
    uint32_t olabel;
    double weight;
    uint32_t nextstate;
} FstArc;

#define FST_NO_STATE UINT32_MAX        /* include/fst.h:58 */
#define FST_EPSILON 0                  /* include/fst.h:59 */
#define FST_INVALID_HANDLE UINT64_MAX  /* include/fst.h:60 */

/* --- MutableFst lifecycle: src/c-api.zig:437-503 --- */
FstMutableHandle fst_mutable_new(void);                                   /* :437 */
FstMutableHandle fst_mutable_clone(FstMutableHandle handle);              /* :443 */
void fst_mutable_free(FstMutableHandle handle);                           /* :464 */
uint32_t fst_mutable_add_state(FstMutableHandle handle);                  /* :470 */
FstError fst_mutable_set_start(FstMutableHandle handle, uint32_t state);  /* :477 */
FstError fst_mutable_set_final(FstMutableHandle handle, uint32_t state, double weight); /* :486 */
FstError fst_mutable_add_arc(FstMutableHandle handle, uint32_t src, uint32_t ilabel,
                             uint32_t olabel, double weight, uint32_t nextstate);       /* :495 */

/* --- MutableFst query (result readback): src/c-api.zig:1376-1424 --- */
uint32_t fst_mutable_start(FstMutableHandle handle);
uint32_t fst_mutable_num_states(FstMutableHandle handle);
uint32_t fst_mutable_num_arcs(FstMutableHandle handle, uint32_t state);
double fst_mutable_final_weight(FstMutableHandle handle, uint32_t state);
uint32_t fst_mutable_get_arcs(FstMutableHandle handle, uint32_t state, FstArc* buf,
                              uint32_t buf_len);

/* --- Freeze / frozen Fst: src/c-api.zig:507-584 --- */
FstHandle fst_freeze(FstMutableHandle mutable_handle);                    /* :507 */
void fst_free(FstHandle handle);                                          /* :530 */
uint32_t fst_start(FstHandle handle);                                     /* :536 */
uint32_t fst_num_states(FstHandle handle);                                /* :543 */
uint32_t fst_num_arcs(FstHandle handle, uint32_t state);                  /* :550 */
double fst_final_weight(FstHandle handle, uint32_t state);                /* :558 */
uint32_t fst_get_arcs(FstHandle handle, uint32_t state, FstArc* buf, uint32_t buf_len); /* :566 */

/* --- Binary I/O of the frozen blob: src/c-api.zig:601-610, :625-640 --- */
/* (the file is read straight into a pinned host block and validated there, so the first
 * device use uploads it with one DMA) */
FstHandle fst_load(const char* path);                                     /* :601 */
FstError fst_save(FstHandle handle, const char* path);                    /* :625 */
/* --- AT&T text (src/io/text.zig:20-115) as the reference's fst_read_text: the asset path
 * of an OpenFst grammar (fstprint -> text -> fst_read_text -> fst_freeze); no label shift
 * (tools/att2lfst adds att2lfst.zig's +1, src/tools/att2lfst.zig:54-60) --- */
FstMutableHandle fst_read_text(const char* path);                         /* :588 */

/* --- The hot path --- */
/* Eager lattice compose(a, b) with b pinned: src/c-api.zig:675-742 -> src/ops/compose.zig:29-198 */
FstMutableHandle fst_compose_frozen(FstMutableHandle a, FstHandle b);
/* Lazy 1-best without the lattice: src/c-api.zig:744-811 -> src/ops/compose-shortest-path.zig:26-401.
 * Only n == 1 searches; n == 0 returns an empty FST; other n return FST_INVALID_HANDLE. */
FstMutableHandle fst_compose_frozen_shortest_path(FstMutableHandle a, FstHandle b, uint32_t n);
/* 1-best of a MutableFst: src/c-api.zig:897-916 -> src/ops/shortest-path.zig:18-139. */
FstMutableHandle fst_shortest_path(FstMutableHandle handle, uint32_t n);

/* --- Strings: src/c-api.zig:1334-1372 -> src/string.zig:17-97 --- */
FstMutableHandle fst_compile_string(const uint8_t* input, uint32_t len);
int32_t fst_print_string(FstMutableHandle handle, uint8_t* buf, uint32_t buf_len);
int32_t fst_print_output_string(FstMutableHandle handle, uint8_t* buf, uint32_t buf_len);

/* --- Global teardown: src/c-api.zig:295-329 --- */
void fst_teardown(void);

#ifdef __cplusplus
}
#endif

#endif /* LIBFST_AMD_FST_H */
