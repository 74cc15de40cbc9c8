/*
 * fst_oracle.h -- CPU restatement of ontypehq/libfst's frozen-compose hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker (and the
 * "port" CPU baseline timed by bench.py).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library
 * (libfst_amd/) never links, loads or calls anything in oracle/.
 *
 * Every function restates one reference function clause by clause; the file
 * and line it follows are cited next to it (paths relative to the reference
 * repository root).  The reference is Zig 0.16; no Zig toolchain exists in
 * this image, so the restatement is pinned by the reference's own known-answer
 * tests and corpus fixtures (see tests/test_oracle_known_answers.py).
 */
#ifndef FST_ORACLE_H
#define FST_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_NO_STATE 0xFFFFFFFFu /* src/arc.zig:13 */
#define OR_EPSILON 0u           /* src/arc.zig:10 */

/* Status codes of the restated algorithms. */
enum {
    OR_OK = 0,
    OR_ERR_UNSUPPORTED_N = 1, /* error.UnsupportedNShortest */
    OR_ERR_CYCLE = 2,         /* back-pointer cycle: the reference would loop forever */
    OR_ERR_NAN = 3,           /* NaN weight compare: `unreachable` in Zig */
    OR_ERR_OOM = 4,
    OR_ERR_INVALID = 5,
};

/* fromBytes validation results, src/fst.zig:227-273 */
enum {
    OR_BLOB_OK = 0,
    OR_BLOB_INVALID_FORMAT = 1,
    OR_BLOB_INVALID_MAGIC = 2,
    OR_BLOB_UNSUPPORTED_VERSION = 3,
    OR_BLOB_WEIGHT_TYPE_MISMATCH = 4,
};

typedef struct {
    uint32_t ilabel;
    uint32_t olabel;
    double weight;
    uint32_t nextstate;
} or_arc; /* Arc(W), src/arc.zig:17-23 */

typedef struct or_mfst or_mfst;

/* ---- MutableFst (src/mutable-fst.zig:45-279) ---- */
or_mfst* or_mfst_new(void);
void or_mfst_free(or_mfst* m);
uint32_t or_mfst_add_state(or_mfst* m);
void or_mfst_set_start(or_mfst* m, uint32_t s);
void or_mfst_set_final(or_mfst* m, uint32_t s, double w);
int or_mfst_add_arc(or_mfst* m, uint32_t src, uint32_t il, uint32_t ol, double w, uint32_t next);
uint32_t or_mfst_start(const or_mfst* m);
uint32_t or_mfst_num_states(const or_mfst* m);
uint32_t or_mfst_num_arcs(const or_mfst* m, uint32_t s);
uint64_t or_mfst_total_arcs(const or_mfst* m);
double or_mfst_final(const or_mfst* m, uint32_t s);
int or_mfst_get_arc(const or_mfst* m, uint32_t s, uint32_t i, or_arc* out);
/* test helper: CSR export (off[ns + 1], arcs[total], finals[ns]) */
void or_mfst_export(const or_mfst* m, uint64_t* off, or_arc* arcs, double* finals);

/* ---- string helpers (src/string.zig:17-97) ---- */
or_mfst* or_compile_string(const uint8_t* in, uint32_t len);
or_mfst* or_compile_string_transducer(const uint8_t* in, uint32_t in_len, const uint8_t* out,
                                      uint32_t out_len);
/* tape 0 = input, 1 = output.  Returns length, or -1 for "not a linear chain" (null). */
int32_t or_print_string(const or_mfst* m, int tape, uint8_t* buf, uint32_t cap);

/* ---- frozen blob (src/fst.zig:12-273) ---- */
uint8_t* or_freeze(const or_mfst* m, uint8_t weight_type, size_t* out_len);
void or_blob_free(uint8_t* blob);
int or_validate(const uint8_t* blob, size_t len, uint8_t expect_weight_type);
void or_arcs_by_ilabel(const uint8_t* blob, uint32_t s, uint32_t ilabel, uint32_t* lo, uint32_t* hi);
int or_find_arc(const uint8_t* blob, uint32_t s, uint32_t ilabel, or_arc* out);

/* ---- algorithms ----
 * rhs is either a frozen blob (rhs_blob != NULL: arcsByIlabel path) or a mutable
 * FST (rhs_mut: linear-scan path), mirroring `rhs_has_label_lookup`.
 * On success *out receives a new FST owned by the caller.  Work counters (optional):
 * stats[0] = product tuples / lattice states, stats[1] = relaxations / lattice arcs. */
int or_compose(const or_mfst* a, const or_mfst* rhs_mut, const uint8_t* rhs_blob, or_mfst** out,
               uint64_t* stats);
int or_shortest_path(const or_mfst* a, uint32_t n, or_mfst** out, uint64_t* stats);
int or_compose_shortest_path(const or_mfst* a, const or_mfst* rhs_mut, const uint8_t* rhs_blob,
                             uint32_t n, or_mfst** out, uint64_t* stats);

/* ---- bench generators (bench/optimize-bench.zig:160-328) ---- */
or_mfst* or_gen_linear_acceptor(uint32_t len, uint32_t alphabet);
or_mfst* or_gen_repeat_acceptor(uint32_t len, uint32_t label);
or_mfst* or_gen_branching_frozen_src(uint32_t T, uint32_t B);
or_mfst* or_gen_eps_dense(uint32_t T, uint32_t B);
or_mfst* or_gen_ambiguous(uint32_t T, uint32_t B);

/* ---- batch driver: one linear-chain acceptor per string ----
 * semantics 0 = lazy composeShortestPath, 1 = eager shortestPath(compose()).
 * The chain for string i has labels labels[offsets[i] .. offsets[i+1]) with
 * olabel = ilabel, weight One, final(L) = One (src/string.zig:24-50). */
typedef struct {
    uint32_t num_strings;
    int32_t* status;        /* OR_OK (check path_len / empty), or an OR_ERR_* code */
    uint8_t* empty;         /* 1 if the result FST has no states (start == no_state) */
    uint64_t* offsets;      /* num_strings + 1 */
    uint32_t* ilabels;
    uint32_t* olabels;
    double* weights;
    double* finals;
    uint64_t* tuples;       /* work counter X per string */
    uint64_t* relaxations;  /* work counter R per string */
    uint64_t total_arcs;
} or_batch_result;

or_batch_result* or_batch_run(const uint8_t* blob, const uint32_t* labels, const uint64_t* offsets,
                              uint32_t num_strings, int semantics, uint32_t n, int threads);
void or_batch_result_free(or_batch_result* r);

/* Throughput helper for the CPU baseline: runs the batch and returns wall seconds. */
double or_batch_time(const uint8_t* blob, const uint32_t* labels, const uint64_t* offsets,
                     uint32_t num_strings, int semantics, int threads, uint64_t* checksum);

#ifdef __cplusplus
}
#endif
#endif
