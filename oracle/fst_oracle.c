/*
 * fst_oracle.c -- CPU restatement of ontypehq/libfst's frozen-compose hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + "port" CPU baseline).  See
 * fst_oracle.h.  Nothing here is shipped in or called by libfst_amd/.
 *
 * The code keeps the reference's data structures on purpose (hash map
 * tuple->id, binary heap with lazy deletion, per-call arena-like growable
 * arrays, materialised lattice for the eager path) so that timing it is a
 * fair stand-in for the Zig CPU path, which cannot be built here (no Zig).
 */
#define _GNU_SOURCE
#include "fst_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* Weights: TropicalWeight, src/weight.zig:5-37 (LogWeight times/compare/isZero */
/* are identical, src/weight.zig:88-104; plus() never runs on this path).      */
/* ------------------------------------------------------------------------- */

typedef struct {
    int nan_seen;
} or_ctx;

static const double W_ZERO = INFINITY; /* src/weight.zig:8 */
static const double W_ONE = 0.0;       /* src/weight.zig:9 */

static inline int w_is_zero(double v) { return isinf(v); } /* :30-32 (-inf is Zero too) */

static inline double w_times(double a, double b) { /* :19-23 */
    if (w_is_zero(a) || w_is_zero(b)) return W_ZERO;
    return a + b;
}

/* math.order(a, b), :34-37.  NaN is `unreachable` in Zig; we flag it. */
static inline int w_cmp(or_ctx* c, double a, double b) {
    if (a == b) return 0;
    if (a < b) return -1;
    if (a > b) return 1;
    c->nan_seen = 1;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* MutableFst, src/mutable-fst.zig:45-279                                     */
/* ------------------------------------------------------------------------- */

typedef struct {
    double final_w;
    or_arc* arcs;
    uint32_t n, cap;
} or_state;

struct or_mfst {
    or_state* st;
    uint32_t n, cap;
    uint32_t start;
};

or_mfst* or_mfst_new(void) {
    or_mfst* m = (or_mfst*)calloc(1, sizeof(or_mfst));
    if (m) m->start = OR_NO_STATE; /* init(): start_state = no_state */
    return m;
}

void or_mfst_free(or_mfst* m) {
    if (!m) return;
    for (uint32_t i = 0; i < m->n; ++i) free(m->st[i].arcs);
    free(m->st);
    free(m);
}

static int mfst_reserve_states(or_mfst* m, uint32_t want) {
    if (want <= m->cap) return 0;
    uint32_t nc = m->cap ? m->cap : 8;
    while (nc < want) nc *= 2;
    or_state* ns = (or_state*)realloc(m->st, (size_t)nc * sizeof(or_state));
    if (!ns) return -1;
    m->st = ns;
    m->cap = nc;
    return 0;
}

uint32_t or_mfst_add_state(or_mfst* m) { /* addState(), :95-101 */
    if (mfst_reserve_states(m, m->n + 1)) return OR_NO_STATE;
    or_state* s = &m->st[m->n];
    s->final_w = W_ZERO; /* MutableState.init(): final = Zero */
    s->arcs = NULL;
    s->n = s->cap = 0;
    return m->n++;
}

static int mfst_add_states(or_mfst* m, uint32_t k) { /* addStates(), :103-109 */
    if (mfst_reserve_states(m, m->n + k)) return -1;
    for (uint32_t i = 0; i < k; ++i) or_mfst_add_state(m);
    return 0;
}

void or_mfst_set_start(or_mfst* m, uint32_t s) { m->start = s; }
void or_mfst_set_final(or_mfst* m, uint32_t s, double w) { m->st[s].final_w = w; }

int or_mfst_add_arc(or_mfst* m, uint32_t src, uint32_t il, uint32_t ol, double w, uint32_t next) {
    or_state* s = &m->st[src]; /* addArc(): append in insertion order, :124-127 */
    if (s->n == s->cap) {
        uint32_t nc = s->cap ? s->cap * 2 : 4;
        or_arc* na = (or_arc*)realloc(s->arcs, (size_t)nc * sizeof(or_arc));
        if (!na) return -1;
        s->arcs = na;
        s->cap = nc;
    }
    or_arc a = {il, ol, w, next};
    s->arcs[s->n++] = a;
    return 0;
}

uint32_t or_mfst_start(const or_mfst* m) { return m->start; }
uint32_t or_mfst_num_states(const or_mfst* m) { return m->n; }
uint32_t or_mfst_num_arcs(const or_mfst* m, uint32_t s) { return s < m->n ? m->st[s].n : 0; }
uint64_t or_mfst_total_arcs(const or_mfst* m) {
    uint64_t t = 0;
    for (uint32_t i = 0; i < m->n; ++i) t += m->st[i].n;
    return t;
}
double or_mfst_final(const or_mfst* m, uint32_t s) { return s < m->n ? m->st[s].final_w : W_ZERO; }
int or_mfst_get_arc(const or_mfst* m, uint32_t s, uint32_t i, or_arc* out) {
    if (s >= m->n || i >= m->st[s].n) return -1;
    *out = m->st[s].arcs[i];
    return 0;
}
/* Test helper (not in the reference): the whole FST as CSR in state order, arcs in
 * insertion order; off[num_states + 1], arcs[total_arcs], finals[num_states]. */
void or_mfst_export(const or_mfst* m, uint64_t* off, or_arc* arcs, double* finals) {
    uint64_t k = 0;
    for (uint32_t s = 0; s < m->n; ++s) {
        off[s] = k;
        finals[s] = m->st[s].final_w;
        if (m->st[s].n) memcpy(arcs + k, m->st[s].arcs, (size_t)m->st[s].n * sizeof(or_arc));
        k += m->st[s].n;
    }
    off[m->n] = k;
}

/* ------------------------------------------------------------------------- */
/* String helpers, src/string.zig:17-97                                       */
/* ------------------------------------------------------------------------- */

or_mfst* or_compile_string_transducer(const uint8_t* in, uint32_t in_len, const uint8_t* out,
                                      uint32_t out_len) { /* :24-50 */
    or_mfst* f = or_mfst_new();
    if (!f) return NULL;
    uint32_t max_len = in_len > out_len ? in_len : out_len;
    if (max_len == 0) { /* empty string: single final state */
        uint32_t s = or_mfst_add_state(f);
        or_mfst_set_start(f, s);
        or_mfst_set_final(f, s, W_ONE);
        return f;
    }
    mfst_add_states(f, max_len + 1);
    or_mfst_set_start(f, 0);
    or_mfst_set_final(f, max_len, W_ONE);
    for (uint32_t i = 0; i < max_len; ++i) {
        uint32_t il = i < in_len ? (uint32_t)in[i] + 1 : OR_EPSILON;   /* label = byte + 1 */
        uint32_t ol = i < out_len ? (uint32_t)out[i] + 1 : OR_EPSILON;
        or_mfst_add_arc(f, i, il, ol, W_ONE, i + 1);
    }
    return f;
}

or_mfst* or_compile_string(const uint8_t* in, uint32_t len) { /* :17-19 */
    return or_compile_string_transducer(in, len, in, len);
}

/* printStringFromTape, :64-97.  Returns -1 for null (not a linear chain),
 * -2 for a label that does not fit a byte (a safety panic in Zig), -3 if the
 * walk exceeds num_states steps (the reference would loop forever). */
int32_t or_print_string(const or_mfst* m, int tape, uint8_t* buf, uint32_t cap) {
    uint32_t cur = m->start;
    if (cur == OR_NO_STATE) return -1;
    uint32_t len = 0;
    uint64_t steps = 0;
    for (;;) {
        const or_state* s = &m->st[cur];
        if (!w_is_zero(s->final_w)) {
            if (s->n == 0) break;
        }
        if (s->n != 1) return -1;
        const or_arc* a = &s->arcs[0];
        uint32_t label = tape == 0 ? a->ilabel : a->olabel;
        if (label != OR_EPSILON) {
            if (label - 1 > 255u) return -2;
            if (len < cap && buf) buf[len] = (uint8_t)(label - 1);
            len++;
        }
        cur = a->nextstate;
        if (cur == OR_NO_STATE) return -1;
        if (++steps > (uint64_t)m->n) return -3;
    }
    return (int32_t)len;
}

/* ------------------------------------------------------------------------- */
/* Frozen blob, src/fst.zig:12-273                                            */
/* ------------------------------------------------------------------------- */

#define OR_MAGIC 0x46535421u /* "FST!", :12 */
#define OR_VERSION 1u        /* :13 */

typedef struct {
    uint32_t magic;
    uint16_t version;
    uint8_t weight_type;
    uint8_t flags;
    uint32_t num_states;
    uint32_t num_arcs;
    uint32_t start_state;
    uint32_t pad;
} or_header; /* Header, :31-40 (24 bytes) */

typedef struct {
    uint32_t arc_offset;
    uint32_t num_arcs;
    double final_weight;
} or_state_entry; /* StateEntry, :16-20 (16 bytes) */

typedef struct {
    uint32_t ilabel;
    uint32_t olabel;
    double weight;
    uint32_t nextstate;
    uint32_t pad;
} or_packed_arc; /* PackedArc, :23-28 (24 bytes as an extern struct) */

_Static_assert(sizeof(or_header) == 24, "Header is 24 bytes");
_Static_assert(sizeof(or_state_entry) == 16, "StateEntry is 16 bytes");
_Static_assert(sizeof(or_packed_arc) == 24, "PackedArc is 24 bytes");

static inline const or_header* blob_hdr(const uint8_t* b) { return (const or_header*)b; }
static inline const or_state_entry* blob_states(const uint8_t* b) {
    return (const or_state_entry*)(b + sizeof(or_header));
}
static inline const or_packed_arc* blob_arcs(const uint8_t* b) {
    return (const or_packed_arc*)(b + sizeof(or_header) +
                                  (size_t)blob_hdr(b)->num_states * sizeof(or_state_entry));
}

/* Arc.compareByIlabel, src/arc.zig:46-54: (ilabel, olabel, weight, nextstate). */
static int arc_less(const or_arc* a, const or_arc* b) {
    if (a->ilabel != b->ilabel) return a->ilabel < b->ilabel;
    if (a->olabel != b->olabel) return a->olabel < b->olabel;
    if (a->weight < b->weight) return 1;
    if (a->weight > b->weight) return 0;
    return a->nextstate < b->nextstate;
}

/* std.mem.sort is a stable block sort; a stable merge sort gives the same order. */
static void stable_sort_arcs(or_arc* a, uint32_t n, or_arc* tmp) {
    if (n < 2) return;
    if (n <= 16) { /* insertion sort (stable) */
        for (uint32_t i = 1; i < n; ++i) {
            or_arc x = a[i];
            uint32_t j = i;
            while (j > 0 && arc_less(&x, &a[j - 1])) {
                a[j] = a[j - 1];
                --j;
            }
            a[j] = x;
        }
        return;
    }
    uint32_t h = n / 2;
    stable_sort_arcs(a, h, tmp);
    stable_sort_arcs(a + h, n - h, tmp);
    uint32_t i = 0, j = h, k = 0;
    while (i < h && j < n) tmp[k++] = arc_less(&a[j], &a[i]) ? a[j++] : a[i++];
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, (size_t)n * sizeof(or_arc));
}

/* Fst.fromMutable, src/fst.zig:160-224 (sortAllArcs, then pack). */
uint8_t* or_freeze(const or_mfst* m, uint8_t weight_type, size_t* out_len) {
    uint64_t total = or_mfst_total_arcs(m);
    size_t sz = sizeof(or_header) + (size_t)m->n * sizeof(or_state_entry) +
                (size_t)total * sizeof(or_packed_arc);
    uint8_t* b = (uint8_t*)aligned_alloc(8, (sz + 7) & ~(size_t)7);
    if (!b) return NULL;
    memset(b, 0, sz);
    or_header* h = (or_header*)b;
    h->magic = OR_MAGIC;
    h->version = OR_VERSION;
    h->weight_type = weight_type;
    h->flags = 0;
    h->num_states = m->n;
    h->num_arcs = (uint32_t)total;
    h->start_state = m->start;
    or_state_entry* se = (or_state_entry*)(b + sizeof(or_header));
    or_packed_arc* pa = (or_packed_arc*)(b + sizeof(or_header) + (size_t)m->n * sizeof(or_state_entry));
    uint32_t maxn = 0;
    for (uint32_t i = 0; i < m->n; ++i)
        if (m->st[i].n > maxn) maxn = m->st[i].n;
    or_arc* work = (or_arc*)malloc((size_t)(maxn ? maxn : 1) * sizeof(or_arc));
    or_arc* tmp = (or_arc*)malloc((size_t)(maxn ? maxn : 1) * sizeof(or_arc));
    uint32_t off = 0;
    for (uint32_t i = 0; i < m->n; ++i) {
        const or_state* s = &m->st[i];
        memcpy(work, s->arcs, (size_t)s->n * sizeof(or_arc));
        stable_sort_arcs(work, s->n, tmp);
        se[i].arc_offset = off;
        se[i].num_arcs = s->n;
        se[i].final_weight = s->final_w;
        for (uint32_t k = 0; k < s->n; ++k) {
            pa[off + k].ilabel = work[k].ilabel;
            pa[off + k].olabel = work[k].olabel;
            pa[off + k].weight = work[k].weight;
            pa[off + k].nextstate = work[k].nextstate;
        }
        off += s->n;
    }
    free(work);
    free(tmp);
    *out_len = sz;
    return b;
}

void or_blob_free(uint8_t* blob) { free(blob); }

/* Fst.fromBytes, src/fst.zig:227-273 */
int or_validate(const uint8_t* b, size_t len, uint8_t expect_wt) {
    if (len < sizeof(or_header)) return OR_BLOB_INVALID_FORMAT;
    const or_header* h = blob_hdr(b);
    if (h->magic != OR_MAGIC) return OR_BLOB_INVALID_MAGIC;
    if (h->version != OR_VERSION) return OR_BLOB_UNSUPPORTED_VERSION;
    if (h->weight_type != expect_wt) return OR_BLOB_WEIGHT_TYPE_MISMATCH;
    size_t expected = sizeof(or_header) + (size_t)h->num_states * sizeof(or_state_entry) +
                      (size_t)h->num_arcs * sizeof(or_packed_arc);
    if (len != expected) return OR_BLOB_INVALID_FORMAT;
    if (h->num_states > 0 && h->start_state != OR_NO_STATE && h->start_state >= h->num_states)
        return OR_BLOB_INVALID_FORMAT;
    if (h->num_states == 0 && h->start_state != OR_NO_STATE) return OR_BLOB_INVALID_FORMAT;
    const or_state_entry* se = blob_states(b);
    const or_packed_arc* pa = blob_arcs(b);
    for (uint32_t i = 0; i < h->num_states; ++i) {
        if (se[i].arc_offset > h->num_arcs) return OR_BLOB_INVALID_FORMAT;
        if (se[i].num_arcs > h->num_arcs - se[i].arc_offset) return OR_BLOB_INVALID_FORMAT;
        int have_last = 0;
        uint32_t last = 0;
        for (uint32_t k = 0; k < se[i].num_arcs; ++k) {
            const or_packed_arc* a = &pa[se[i].arc_offset + k];
            if (a->nextstate >= h->num_states) return OR_BLOB_INVALID_FORMAT;
            if (have_last && a->ilabel < last) return OR_BLOB_INVALID_FORMAT;
            last = a->ilabel;
            have_last = 1;
        }
    }
    return OR_BLOB_OK;
}

/* Fst.arcsByIlabel, src/fst.zig:112-136: [lower_bound, upper_bound) in the span. */
void or_arcs_by_ilabel(const uint8_t* b, uint32_t s, uint32_t ilabel, uint32_t* lo_out,
                       uint32_t* hi_out) {
    const or_state_entry e = blob_states(b)[s];
    const or_packed_arc* arcs = blob_arcs(b) + e.arc_offset;
    uint32_t lo = 0, hi = e.num_arcs;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (arcs[mid].ilabel < ilabel) lo = mid + 1;
        else hi = mid;
    }
    uint32_t start = lo;
    hi = e.num_arcs;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (arcs[mid].ilabel <= ilabel) lo = mid + 1;
        else hi = mid;
    }
    *lo_out = e.arc_offset + start;
    *hi_out = e.arc_offset + lo;
}

/* Fst.findArc, src/fst.zig:140-155 */
int or_find_arc(const uint8_t* b, uint32_t s, uint32_t ilabel, or_arc* out) {
    const or_state_entry e = blob_states(b)[s];
    const or_packed_arc* arcs = blob_arcs(b) + e.arc_offset;
    uint32_t lo = 0, hi = e.num_arcs;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (arcs[mid].ilabel < ilabel) lo = mid + 1;
        else if (arcs[mid].ilabel > ilabel) hi = mid;
        else {
            out->ilabel = arcs[mid].ilabel;
            out->olabel = arcs[mid].olabel;
            out->weight = arcs[mid].weight;
            out->nextstate = arcs[mid].nextstate;
            return 1;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* rhs abstraction: frozen (arcsByIlabel) or mutable (linear scan), mirroring */
/* `rhs_has_label_lookup` (src/ops/compose.zig:31, compose-shortest-path.zig:28) */
/* ------------------------------------------------------------------------- */

typedef struct {
    const uint8_t* blob; /* non-NULL: frozen */
    const or_mfst* mut;
} or_rhs;

static uint32_t rhs_start(const or_rhs* r) {
    return r->blob ? blob_hdr(r->blob)->start_state : r->mut->start;
}
static double rhs_final(const or_rhs* r, uint32_t s) {
    return r->blob ? blob_states(r->blob)[s].final_weight : r->mut->st[s].final_w;
}

/* Iterate the rhs arcs of state s whose ilabel equals `label`, in the order the
 * reference visits them: the sorted span for a frozen rhs, insertion order with
 * an ilabel filter for a mutable rhs. */
typedef struct {
    const or_rhs* r;
    uint32_t s, label, i, end;
} rhs_iter;

static void rhs_iter_init(rhs_iter* it, const or_rhs* r, uint32_t s, uint32_t label) {
    it->r = r;
    it->s = s;
    it->label = label;
    if (r->blob) {
        or_arcs_by_ilabel(r->blob, s, label, &it->i, &it->end);
    } else {
        it->i = 0;
        it->end = r->mut->st[s].n;
    }
}

static int rhs_iter_next(rhs_iter* it, or_arc* out) {
    if (it->r->blob) {
        if (it->i >= it->end) return 0;
        const or_packed_arc* a = &blob_arcs(it->r->blob)[it->i++];
        out->ilabel = a->ilabel;
        out->olabel = a->olabel;
        out->weight = a->weight;
        out->nextstate = a->nextstate;
        return 1;
    }
    const or_state* st = &it->r->mut->st[it->s];
    while (it->i < it->end) {
        const or_arc* a = &st->arcs[it->i++];
        if (a->ilabel != it->label) continue;
        *out = *a;
        return 1;
    }
    return 0;
}

static uint32_t rhs_count(const or_rhs* r, uint32_t s, uint32_t label) {
    rhs_iter it;
    rhs_iter_init(&it, r, s, label);
    if (r->blob) return it.end - it.i;
    uint32_t n = 0;
    or_arc a;
    while (rhs_iter_next(&it, &a)) n++;
    return n;
}

/* ------------------------------------------------------------------------- */
/* Tuple hash map (std.AutoHashMapUnmanaged(StateTuple, u32) stand-in).        */
/* Results never depend on hash internals: lookups only, no iteration.        */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint32_t s1, s2;
    uint8_t f;
} or_tuple;

typedef struct {
    uint32_t s1, s2;
    uint32_t f;
    uint32_t id1; /* id + 1, 0 = empty */
} tslot;

typedef struct {
    tslot* slots; /* keys stored inline, like AutoHashMapUnmanaged */
    uint32_t cap; /* power of two */
    uint32_t count;
} tmap;

static inline uint64_t tuple_hash(or_tuple t) {
    uint64_t x = ((uint64_t)t.s1 << 32) ^ (uint64_t)t.s2 ^ ((uint64_t)t.f << 61);
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

static int tmap_init(tmap* m, uint32_t cap) {
    m->cap = cap;
    m->count = 0;
    m->slots = (tslot*)calloc(cap, sizeof(tslot));
    return m->slots ? 0 : -1;
}

/* Returns id or OR_NO_STATE. */
static uint32_t tmap_get(const tmap* m, or_tuple t) {
    uint32_t mask = m->cap - 1;
    uint32_t i = (uint32_t)tuple_hash(t) & mask;
    for (;;) {
        const tslot* s = &m->slots[i];
        if (!s->id1) return OR_NO_STATE;
        if (s->s1 == t.s1 && s->s2 == t.s2 && s->f == t.f) return s->id1 - 1;
        i = (i + 1) & mask;
    }
}

static void tmap_put_new(tmap* m, or_tuple t, uint32_t id) {
    uint32_t mask = m->cap - 1;
    uint32_t i = (uint32_t)tuple_hash(t) & mask;
    while (m->slots[i].id1) i = (i + 1) & mask;
    m->slots[i].s1 = t.s1;
    m->slots[i].s2 = t.s2;
    m->slots[i].f = t.f;
    m->slots[i].id1 = id + 1;
    m->count++;
}

static int tmap_grow(tmap* m) {
    uint32_t old_cap = m->cap;
    tslot* old = m->slots;
    if (tmap_init(m, old_cap * 2)) {
        m->slots = old;
        m->cap = old_cap;
        return -1;
    }
    for (uint32_t i = 0; i < old_cap; ++i) {
        if (old[i].id1) {
            or_tuple t = {old[i].s1, old[i].s2, (uint8_t)old[i].f};
            tmap_put_new(m, t, old[i].id1 - 1);
        }
    }
    free(old);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Binary heap (std.PriorityQueue stand-in).  Pop order is fully determined   */
/* by the (dist, id) total order, so the heap's internals do not matter.      */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint32_t id;
    double dist;
} hitem;

typedef struct {
    hitem* a;
    uint32_t n, cap;
    or_ctx* ctx;
} heap;

static inline int hless(or_ctx* c, hitem x, hitem y) { /* queueCompare: (dist, id) */
    int d = w_cmp(c, x.dist, y.dist);
    if (d != 0) return d < 0;
    return x.id < y.id;
}

static int heap_push(heap* h, hitem x) {
    if (h->n == h->cap) {
        uint32_t nc = h->cap ? h->cap * 2 : 64;
        hitem* na = (hitem*)realloc(h->a, (size_t)nc * sizeof(hitem));
        if (!na) return -1;
        h->a = na;
        h->cap = nc;
    }
    uint32_t i = h->n++;
    while (i > 0) {
        uint32_t p = (i - 1) / 2;
        if (!hless(h->ctx, x, h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = x;
    return 0;
}

static int heap_pop(heap* h, hitem* out) {
    if (!h->n) return 0;
    *out = h->a[0];
    hitem x = h->a[--h->n];
    uint32_t i = 0, n = h->n;
    for (;;) {
        uint32_t l = 2 * i + 1;
        if (l >= n) break;
        uint32_t c = l;
        if (l + 1 < n && hless(h->ctx, h->a[l + 1], h->a[l])) c = l + 1;
        if (!hless(h->ctx, h->a[c], x)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (n) h->a[i] = x;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Product-state table shared by compose and composeShortestPath.             */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint32_t prev_id;
    uint32_t ilabel, olabel;
    double weight;
    uint8_t has;
} or_backptr; /* BackPtr, compose-shortest-path.zig:44-49 */

typedef struct {
    or_tuple* tuples;
    double* dist;
    or_backptr* back;
    uint8_t* settled;
    uint32_t n, cap;
    tmap map;
} ptable;

static int ptable_init(ptable* t) {
    memset(t, 0, sizeof(*t));
    return tmap_init(&t->map, 1024);
}

static void ptable_free(ptable* t) {
    free(t->tuples);
    free(t->dist);
    free(t->back);
    free(t->settled);
    free(t->map.slots);
}

/* getOrCreate, compose-shortest-path.zig:70-89 (also compose.zig:77-91 for ids) */
static uint32_t ptable_get_or_create(ptable* t, or_tuple key, int* created) {
    uint32_t id = tmap_get(&t->map, key);
    if (created) *created = 0;
    if (id != OR_NO_STATE) return id;
    if (t->n == t->cap) {
        uint32_t nc = t->cap ? t->cap * 2 : 1024;
        or_tuple* a = (or_tuple*)realloc(t->tuples, (size_t)nc * sizeof(or_tuple));
        if (!a) return OR_NO_STATE;
        t->tuples = a;
        double* d = (double*)realloc(t->dist, (size_t)nc * sizeof(double));
        if (!d) return OR_NO_STATE;
        t->dist = d;
        or_backptr* b = (or_backptr*)realloc(t->back, (size_t)nc * sizeof(or_backptr));
        if (!b) return OR_NO_STATE;
        t->back = b;
        uint8_t* s = (uint8_t*)realloc(t->settled, nc);
        if (!s) return OR_NO_STATE;
        t->settled = s;
        t->cap = nc;
    }
    id = t->n++;
    t->tuples[id] = key;
    t->dist[id] = W_ZERO;
    t->back[id].has = 0;
    t->settled[id] = 0;
    if ((uint64_t)(t->map.count + 1) * 10 > (uint64_t)t->map.cap * 7) {
        if (tmap_grow(&t->map)) return OR_NO_STATE;
    }
    tmap_put_new(&t->map, key, id);
    if (created) *created = 1;
    return id;
}

/* ------------------------------------------------------------------------- */
/* composeShortestPath (lazy), src/ops/compose-shortest-path.zig:26-401       */
/* ------------------------------------------------------------------------- */

typedef struct {
    or_ctx* ctx;
    ptable* t;
    heap* q;
    uint64_t relax_count;
    int oom;
} lazy_state;

/* relax, compose-shortest-path.zig:91-144 */
static void lazy_relax(lazy_state* L, uint32_t curr_id, or_tuple next, uint32_t il, uint32_t ol,
                       double edge_w) {
    L->relax_count++;
    ptable* t = L->t;
    uint32_t next_id = ptable_get_or_create(t, next, NULL); /* :107 (first touch) */
    if (next_id == OR_NO_STATE) {
        L->oom = 1;
        return;
    }
    double new_dist = w_times(t->dist[curr_id], edge_w); /* :108 */
    double old_dist = t->dist[next_id];
    int by_dist = w_cmp(L->ctx, new_dist, old_dist); /* :110 */
    int take = 0;
    if (w_is_zero(old_dist) || by_dist < 0) { /* :113 */
        take = 1;
    } else if (by_dist == 0) { /* :115-126 */
        const or_backptr* bp = &t->back[next_id];
        if (bp->has) {
            if (curr_id < bp->prev_id ||
                (curr_id == bp->prev_id &&
                 (il < bp->ilabel || (il == bp->ilabel && ol < bp->olabel))))
                take = 1;
        } else {
            take = 1;
        }
    }
    if (!take) return;
    t->dist[next_id] = new_dist; /* :130-136: also for settled tuples */
    t->back[next_id].prev_id = curr_id;
    t->back[next_id].ilabel = il;
    t->back[next_id].olabel = ol;
    t->back[next_id].weight = edge_w;
    t->back[next_id].has = 1;
    if (!t->settled[next_id]) { /* :137-142 */
        hitem x = {next_id, new_dist};
        if (heap_push(L->q, x)) L->oom = 1;
    }
}

static int make_chain_result(or_mfst** out, const or_backptr* rev, uint32_t len, double final_w) {
    or_mfst* r = or_mfst_new(); /* compose-shortest-path.zig:382-398 */
    if (!r) return OR_ERR_OOM;
    if (mfst_add_states(r, len + 1)) {
        or_mfst_free(r);
        return OR_ERR_OOM;
    }
    or_mfst_set_start(r, 0);
    or_mfst_set_final(r, len, final_w);
    uint32_t out_idx = 0;
    for (uint32_t i = len; i > 0; --i) {
        const or_backptr* bp = &rev[i - 1];
        or_mfst_add_arc(r, out_idx, bp->ilabel, bp->olabel, bp->weight, out_idx + 1);
        out_idx++;
    }
    *out = r;
    return OR_OK;
}

int or_compose_shortest_path(const or_mfst* fst1, const or_mfst* rhs_mut, const uint8_t* rhs_blob,
                             uint32_t n, or_mfst** out, uint64_t* stats) {
    or_rhs R = {rhs_blob, rhs_mut};
    const or_rhs* fst2 = &R;
    or_ctx ctx = {0};
    *out = NULL;
    if (stats) stats[0] = stats[1] = 0;
    if (fst1->start == OR_NO_STATE || rhs_start(fst2) == OR_NO_STATE || n == 0) { /* :30-32 */
        *out = or_mfst_new();
        return OR_OK;
    }
    if (n != 1) return OR_ERR_UNSUPPORTED_N; /* :33 */

    ptable t;
    if (ptable_init(&t)) return OR_ERR_OOM;
    heap q = {NULL, 0, 0, &ctx};
    lazy_state L = {&ctx, &t, &q, 0, 0};
    int rc = OR_OK;

    or_tuple init = {fst1->start, rhs_start(fst2), 0}; /* :146-150 */
    uint32_t init_id = ptable_get_or_create(&t, init, NULL);
    t.dist[init_id] = W_ONE; /* :152 */
    hitem first = {init_id, W_ONE};
    heap_push(&q, first);

    uint32_t best_final_id = OR_NO_STATE; /* :155-157 */
    double best_final_weight = W_ZERO;
    double best_total = W_ZERO;

    hitem item;
    while (heap_pop(&q, &item)) { /* :159 */
        uint32_t curr_id = item.id;
        if (t.settled[curr_id]) continue;                           /* :161 */
        if (w_cmp(&ctx, item.dist, t.dist[curr_id]) != 0) continue; /* :162 stale */
        t.settled[curr_id] = 1;

        or_tuple tt = t.tuples[curr_id];
        double fw1 = fst1->st[tt.s1].final_w;
        double fw2 = rhs_final(fst2, tt.s2);
        if (!w_is_zero(fw1) && !w_is_zero(fw2)) { /* :168-179 */
            double final_w = w_times(fw1, fw2);
            double total = w_times(t.dist[curr_id], final_w);
            if (best_final_id == OR_NO_STATE || w_cmp(&ctx, total, best_total) < 0 ||
                (w_cmp(&ctx, total, best_total) == 0 && curr_id < best_final_id)) {
                best_final_id = curr_id;
                best_final_weight = final_w;
                best_total = total;
            }
        }

        const or_state* s1 = &fst1->st[tt.s1];
        /* Non-epsilon matches, :181-224 */
        for (uint32_t i = 0; i < s1->n; ++i) {
            or_arc a1 = s1->arcs[i];
            if (a1.olabel == OR_EPSILON) continue;
            rhs_iter it;
            or_arc a2;
            rhs_iter_init(&it, fst2, tt.s2, a1.olabel);
            while (rhs_iter_next(&it, &a2)) {
                or_tuple nx = {a1.nextstate, a2.nextstate, 0};
                lazy_relax(&L, curr_id, nx, a1.ilabel, a2.olabel, w_times(a1.weight, a2.weight));
            }
        }
        /* lhs epsilon-output moves, :227-252 */
        if (tt.f != 1) {
            for (uint32_t i = 0; i < s1->n; ++i) {
                or_arc a1 = s1->arcs[i];
                if (a1.olabel != OR_EPSILON) continue;
                uint8_t nf = tt.f == 0 ? 2 : tt.f;
                or_tuple nx = {a1.nextstate, tt.s2, nf};
                lazy_relax(&L, curr_id, nx, a1.ilabel, OR_EPSILON, a1.weight);
            }
        }
        /* rhs epsilon-input moves, :254-305 */
        if (tt.f != 2) {
            rhs_iter it;
            or_arc a2;
            rhs_iter_init(&it, fst2, tt.s2, OR_EPSILON);
            while (rhs_iter_next(&it, &a2)) {
                uint8_t nf = tt.f == 0 ? 1 : tt.f;
                or_tuple nx = {tt.s1, a2.nextstate, nf};
                lazy_relax(&L, curr_id, nx, OR_EPSILON, a2.olabel, a2.weight);
            }
        }
        /* simultaneous epsilon moves, :307-365 */
        if (tt.f == 0) {
            int go = rhs_blob ? rhs_count(fst2, tt.s2, OR_EPSILON) > 0 : 1;
            if (go) {
                for (uint32_t i = 0; i < s1->n; ++i) {
                    or_arc a1 = s1->arcs[i];
                    if (a1.olabel != OR_EPSILON) continue;
                    rhs_iter it;
                    or_arc a2;
                    rhs_iter_init(&it, fst2, tt.s2, OR_EPSILON);
                    while (rhs_iter_next(&it, &a2)) {
                        or_tuple nx = {a1.nextstate, a2.nextstate, 0};
                        lazy_relax(&L, curr_id, nx, a1.ilabel, a2.olabel,
                                   w_times(a1.weight, a2.weight));
                    }
                }
            }
        }
        if (L.oom) break;
    }

    if (stats) {
        stats[0] = t.n;
        stats[1] = L.relax_count;
    }
    if (L.oom) {
        rc = OR_ERR_OOM;
    } else if (ctx.nan_seen) {
        rc = OR_ERR_NAN;
    } else if (best_final_id == OR_NO_STATE) { /* :368-370 */
        *out = or_mfst_new();
    } else { /* backtrace, :372-380 */
        or_backptr* rev = (or_backptr*)malloc(((size_t)t.n + 1) * sizeof(or_backptr));
        uint32_t len = 0;
        uint32_t curr = best_final_id;
        int empty = 0;
        while (curr != init_id) {
            const or_backptr* bp = &t.back[curr];
            if (!bp->has) {
                empty = 1;
                break;
            }
            if (len > t.n) { /* the reference loops forever here */
                rc = OR_ERR_CYCLE;
                break;
            }
            rev[len++] = *bp;
            curr = bp->prev_id;
        }
        if (rc == OR_OK) {
            if (empty) *out = or_mfst_new();
            else rc = make_chain_result(out, rev, len, best_final_weight);
        }
        free(rev);
    }
    free(q.a);
    ptable_free(&t);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* compose (eager), src/ops/compose.zig:29-198                                */
/* ------------------------------------------------------------------------- */

int or_compose(const or_mfst* fst1, const or_mfst* rhs_mut, const uint8_t* rhs_blob, or_mfst** out,
               uint64_t* stats) {
    or_rhs R = {rhs_blob, rhs_mut};
    const or_rhs* fst2 = &R;
    *out = NULL;
    if (stats) stats[0] = stats[1] = 0;
    or_mfst* result = or_mfst_new();
    if (!result) return OR_ERR_OOM;
    if (fst1->start == OR_NO_STATE || rhs_start(fst2) == OR_NO_STATE) { /* :33-35 */
        *out = result;
        return OR_OK;
    }
    /* state_map + FIFO queue; result state id == BFS discovery index, :53-62 */
    ptable t;
    if (ptable_init(&t)) {
        or_mfst_free(result);
        return OR_ERR_OOM;
    }
    or_tuple init = {fst1->start, rhs_start(fst2), 0};
    uint32_t init_state = or_mfst_add_state(result);
    or_mfst_set_start(result, init_state);
    ptable_get_or_create(&t, init, NULL); /* id 0 == init_state */
    uint64_t narcs = 0;
    int oom = 0;

#define GET_OR_CREATE(NX, NS)                                   \
    do {                                                        \
        int created_;                                           \
        NS = ptable_get_or_create(&t, (NX), &created_);         \
        if (NS == OR_NO_STATE) oom = 1;                         \
        else if (created_) or_mfst_add_state(result); /* :86 */ \
    } while (0)

    for (uint32_t qi = 0; qi < t.n && !oom; ++qi) { /* :64-65 FIFO over discovery order */
        or_tuple tt = t.tuples[qi];
        uint32_t current = qi; /* :67 state_map.get(t) */
        double fw1 = fst1->st[tt.s1].final_w;
        double fw2 = rhs_final(fst2, tt.s2);
        if (!w_is_zero(fw1) && !w_is_zero(fw2)) or_mfst_set_final(result, current, w_times(fw1, fw2));

        const or_state* s1 = &fst1->st[tt.s1];
        for (uint32_t i = 0; i < s1->n && !oom; ++i) { /* :95-121 */
            or_arc a1 = s1->arcs[i];
            if (a1.olabel == OR_EPSILON) continue;
            rhs_iter it;
            or_arc a2;
            rhs_iter_init(&it, fst2, tt.s2, a1.olabel);
            while (rhs_iter_next(&it, &a2)) {
                or_tuple nx = {a1.nextstate, a2.nextstate, 0};
                uint32_t ns;
                GET_OR_CREATE(nx, ns);
                if (oom) break;
                or_mfst_add_arc(result, current, a1.ilabel, a2.olabel, w_times(a1.weight, a2.weight), ns);
                narcs++;
            }
        }
        if (tt.f != 1) { /* :124-134 */
            for (uint32_t i = 0; i < s1->n && !oom; ++i) {
                or_arc a1 = s1->arcs[i];
                if (a1.olabel != OR_EPSILON) continue;
                uint8_t nf = tt.f == 0 ? 2 : tt.f;
                or_tuple nx = {a1.nextstate, tt.s2, nf};
                uint32_t ns;
                GET_OR_CREATE(nx, ns);
                if (oom) break;
                or_mfst_add_arc(result, current, a1.ilabel, OR_EPSILON, a1.weight, ns);
                narcs++;
            }
        }
        if (tt.f != 2 && !oom) { /* :136-157 */
            rhs_iter it;
            or_arc a2;
            rhs_iter_init(&it, fst2, tt.s2, OR_EPSILON);
            while (rhs_iter_next(&it, &a2)) {
                uint8_t nf = tt.f == 0 ? 1 : tt.f;
                or_tuple nx = {tt.s1, a2.nextstate, nf};
                uint32_t ns;
                GET_OR_CREATE(nx, ns);
                if (oom) break;
                or_mfst_add_arc(result, current, OR_EPSILON, a2.olabel, a2.weight, ns);
                narcs++;
            }
        }
        if (tt.f == 0 && !oom) { /* :160-194 */
            int go = rhs_blob ? rhs_count(fst2, tt.s2, OR_EPSILON) > 0 : 1;
            if (go) {
                for (uint32_t i = 0; i < s1->n && !oom; ++i) {
                    or_arc a1 = s1->arcs[i];
                    if (a1.olabel != OR_EPSILON) continue;
                    rhs_iter it;
                    or_arc a2;
                    rhs_iter_init(&it, fst2, tt.s2, OR_EPSILON);
                    while (rhs_iter_next(&it, &a2)) {
                        or_tuple nx = {a1.nextstate, a2.nextstate, 0};
                        uint32_t ns;
                        GET_OR_CREATE(nx, ns);
                        if (oom) break;
                        or_mfst_add_arc(result, current, a1.ilabel, a2.olabel,
                                        w_times(a1.weight, a2.weight), ns);
                        narcs++;
                    }
                }
            }
        }
    }
#undef GET_OR_CREATE
    if (stats) {
        stats[0] = t.n;
        stats[1] = narcs;
    }
    ptable_free(&t);
    if (oom) {
        or_mfst_free(result);
        return OR_ERR_OOM;
    }
    *out = result;
    return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* shortestPath (n = 1), src/ops/shortest-path.zig:18-139                     */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint32_t prev_state;
    uint32_t arc_idx;
    uint8_t has;
} sp_back; /* BackPtr, :40-43 */

int or_shortest_path(const or_mfst* fst, uint32_t n, or_mfst** out, uint64_t* stats) {
    or_ctx ctx = {0};
    *out = NULL;
    if (stats) stats[0] = stats[1] = 0;
    if (fst->start == OR_NO_STATE || n == 0) { /* :21-23 */
        *out = or_mfst_new();
        return OR_OK;
    }
    if (n != 1) return OR_ERR_UNSUPPORTED_N; /* :24 */

    uint32_t ns = fst->n;
    double* dist = (double*)malloc((size_t)(ns ? ns : 1) * sizeof(double));
    sp_back* back = (sp_back*)calloc(ns ? ns : 1, sizeof(sp_back));
    uint8_t* settled = (uint8_t*)calloc(ns ? ns : 1, 1);
    if (!dist || !back || !settled) {
        free(dist);
        free(back);
        free(settled);
        return OR_ERR_OOM;
    }
    for (uint32_t i = 0; i < ns; ++i) dist[i] = W_ZERO;
    dist[fst->start] = W_ONE; /* :37 */
    heap q = {NULL, 0, 0, &ctx};
    hitem first = {fst->start, W_ONE};
    heap_push(&q, first);
    uint64_t relax = 0;
    int rc = OR_OK;

    hitem item;
    while (heap_pop(&q, &item)) { /* :64 */
        uint32_t s = item.id;
        if (settled[s]) continue;
        if (w_cmp(&ctx, item.dist, dist[s]) != 0) continue; /* stale */
        settled[s] = 1;
        const or_state* st = &fst->st[s];
        for (uint32_t ai = 0; ai < st->n; ++ai) { /* :70-85 */
            const or_arc* a = &st->arcs[ai];
            uint32_t next = a->nextstate;
            relax++;
            double new_dist = w_times(dist[s], a->weight);
            double old_dist = dist[next];
            int by_dist = w_cmp(&ctx, new_dist, old_dist);
            uint32_t prev_state = back[next].has ? back[next].prev_state : OR_NO_STATE;
            int better_tie = by_dist == 0 && (prev_state == OR_NO_STATE || s < prev_state);
            if (w_is_zero(old_dist) || by_dist < 0 || better_tie) {
                dist[next] = new_dist;
                back[next].prev_state = s;
                back[next].arc_idx = ai;
                back[next].has = 1;
                if (!settled[next]) {
                    hitem x = {next, new_dist};
                    if (heap_push(&q, x)) {
                        rc = OR_ERR_OOM;
                        break;
                    }
                }
            }
        }
        if (rc) break;
    }
    if (stats) {
        stats[0] = ns;
        stats[1] = relax;
    }

    uint32_t best_final = OR_NO_STATE; /* :88-104 */
    double best_total = W_ZERO;
    if (rc == OR_OK) {
        for (uint32_t s = 0; s < ns; ++s) {
            if (w_is_zero(dist[s])) continue;
            double fw = fst->st[s].final_w;
            if (w_is_zero(fw)) continue;
            double total = w_times(dist[s], fw);
            if (best_final == OR_NO_STATE || w_cmp(&ctx, total, best_total) < 0 ||
                (w_cmp(&ctx, total, best_total) == 0 && s < best_final)) {
                best_final = s;
                best_total = total;
            }
        }
    }
    if (rc == OR_OK && ctx.nan_seen) rc = OR_ERR_NAN;
    if (rc == OR_OK) {
        if (best_final == OR_NO_STATE) {
            *out = or_mfst_new(); /* :105-107 */
        } else {
            sp_back* rev = (sp_back*)malloc(((size_t)ns + 1) * sizeof(sp_back));
            uint32_t len = 0;
            uint32_t current = best_final;
            while (back[current].has) { /* :114-117 */
                if (len > ns) { /* the reference loops forever here */
                    rc = OR_ERR_CYCLE;
                    break;
                }
                rev[len++] = back[current];
                current = back[current].prev_state;
            }
            if (rc == OR_OK) {
                if (current != fst->start) { /* :120-122 */
                    *out = or_mfst_new();
                } else {
                    or_mfst* r = or_mfst_new(); /* :124-136 */
                    mfst_add_states(r, len + 1);
                    or_mfst_set_start(r, 0);
                    or_mfst_set_final(r, len, fst->st[best_final].final_w);
                    uint32_t out_idx = 0;
                    for (uint32_t i = len; i > 0; --i) {
                        const sp_back* bp = &rev[i - 1];
                        const or_arc* a = &fst->st[bp->prev_state].arcs[bp->arc_idx];
                        or_mfst_add_arc(r, out_idx, a->ilabel, a->olabel, a->weight, out_idx + 1);
                        out_idx++;
                    }
                    *out = r;
                }
            }
            free(rev);
        }
    }
    free(q.a);
    free(dist);
    free(back);
    free(settled);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Bench generators, bench/optimize-bench.zig:160-328                         */
/* ------------------------------------------------------------------------- */

or_mfst* or_gen_linear_acceptor(uint32_t len, uint32_t alphabet) { /* :164-180 */
    or_mfst* f = or_mfst_new();
    mfst_add_states(f, len + 1);
    or_mfst_set_start(f, 0);
    or_mfst_set_final(f, len, W_ONE);
    uint32_t alpha = alphabet ? alphabet : 1;
    for (uint32_t i = 0; i < len; ++i) {
        uint32_t label = (i % alpha) + 1;
        or_mfst_add_arc(f, i, label, label, W_ONE, i + 1);
    }
    return f;
}

or_mfst* or_gen_repeat_acceptor(uint32_t len, uint32_t label) { /* :182-196 */
    or_mfst* f = or_mfst_new();
    mfst_add_states(f, len + 1);
    or_mfst_set_start(f, 0);
    or_mfst_set_final(f, len, W_ONE);
    for (uint32_t i = 0; i < len; ++i) or_mfst_add_arc(f, i, label, label, W_ONE, i + 1);
    return f;
}

or_mfst* or_gen_branching_frozen_src(uint32_t T, uint32_t B) { /* :290-306 */
    or_mfst* f = or_mfst_new();
    if (T == 0) return f;
    mfst_add_states(f, T);
    or_mfst_set_start(f, 0);
    for (uint32_t i = 0; i < T; ++i) {
        or_mfst_set_final(f, i, W_ONE);
        for (uint32_t b = 0; b < B; ++b) {
            uint32_t il = (b % 255) + 1;
            uint32_t ol = ((i + b) % 255) + 1;
            uint32_t nx = (uint32_t)(((uint64_t)i + b + 1) % T);
            or_mfst_add_arc(f, i, il, ol, (double)b, nx);
        }
    }
    return f;
}

or_mfst* or_gen_eps_dense(uint32_t T, uint32_t B) { /* :219-248 */
    or_mfst* f = or_mfst_new();
    mfst_add_states(f, T + 1);
    or_mfst_set_start(f, 0);
    for (uint32_t i = 0; i <= T; ++i) or_mfst_set_final(f, i, W_ONE);
    for (uint32_t i = 0; i < T; ++i) {
        or_mfst_add_arc(f, i, 0, 0, W_ONE, i + 1);
        for (uint32_t b = 0; b < B; ++b) {
            uint32_t jump = (b % 4) + 1;
            uint32_t nx = i + jump < T ? i + jump : T;
            uint32_t ol = ((i + b) % 255) + 1;
            or_mfst_add_arc(f, i, 1, ol, (double)b, nx);
        }
    }
    return f;
}

or_mfst* or_gen_ambiguous(uint32_t T, uint32_t B) { /* :250-277 */
    or_mfst* f = or_mfst_new();
    mfst_add_states(f, T + 1);
    or_mfst_set_start(f, 0);
    for (uint32_t i = 0; i <= T; ++i) or_mfst_set_final(f, i, W_ONE);
    uint32_t fanout = B < 4 ? B : 4;
    if (fanout < 1) fanout = 1;
    for (uint32_t i = 0; i <= T; ++i) {
        or_mfst_add_arc(f, i, 1, 1, W_ONE, i); /* stay */
        for (uint32_t b = 0; b < fanout; ++b) {
            uint32_t jump = b + 1;
            uint32_t nx = i + jump < T ? i + jump : T;
            uint32_t ol = ((i + b) % 255) + 1;
            or_mfst_add_arc(f, i, 1, ol, (double)b, nx);
        }
    }
    return f;
}

/* ------------------------------------------------------------------------- */
/* Batch driver                                                               */
/* ------------------------------------------------------------------------- */

static or_mfst* chain_from_labels(const uint32_t* labels, uint32_t len) {
    /* compileString semantics (src/string.zig:24-50) over pre-encoded labels */
    or_mfst* f = or_mfst_new();
    mfst_add_states(f, len + 1);
    or_mfst_set_start(f, 0);
    or_mfst_set_final(f, len, W_ONE);
    for (uint32_t i = 0; i < len; ++i) or_mfst_add_arc(f, i, labels[i], labels[i], W_ONE, i + 1);
    return f;
}

typedef struct {
    int32_t status;
    uint8_t empty;
    uint32_t len;
    uint32_t* il;
    uint32_t* ol;
    double* w;
    double final_w;
    uint64_t tuples, relax;
} one_result;

static void run_one(const uint8_t* blob, const uint32_t* labels, uint32_t len, int semantics,
                    uint32_t n, one_result* res) {
    memset(res, 0, sizeof(*res));
    or_mfst* lhs = chain_from_labels(labels, len);
    or_mfst* out = NULL;
    uint64_t st[2] = {0, 0};
    int rc;
    if (semantics == 0) {
        rc = or_compose_shortest_path(lhs, NULL, blob, n, &out, st);
    } else {
        or_mfst* lat = NULL;
        rc = or_compose(lhs, NULL, blob, &lat, st);
        if (rc == OR_OK) {
            uint64_t st2[2];
            rc = or_shortest_path(lat, n, &out, st2);
        }
        or_mfst_free(lat);
    }
    or_mfst_free(lhs);
    res->status = rc;
    res->tuples = st[0];
    res->relax = st[1];
    if (rc != OR_OK) return;
    if (out->start == OR_NO_STATE) {
        res->empty = 1;
    } else {
        uint32_t P = out->n - 1;
        res->len = P;
        res->il = (uint32_t*)malloc((P ? P : 1) * sizeof(uint32_t));
        res->ol = (uint32_t*)malloc((P ? P : 1) * sizeof(uint32_t));
        res->w = (double*)malloc((P ? P : 1) * sizeof(double));
        for (uint32_t i = 0; i < P; ++i) {
            const or_arc* a = &out->st[i].arcs[0];
            res->il[i] = a->ilabel;
            res->ol[i] = a->olabel;
            res->w[i] = a->weight;
        }
        res->final_w = out->st[P].final_w;
    }
    or_mfst_free(out);
}

typedef struct {
    const uint8_t* blob;
    const uint32_t* labels;
    const uint64_t* offsets;
    uint32_t begin, end;
    int semantics;
    uint32_t n;
    one_result* res;  /* NULL in timing mode */
    uint64_t checksum;
} shard_job;

static void* shard_main(void* p) {
    shard_job* j = (shard_job*)p;
    for (uint32_t i = j->begin; i < j->end; ++i) {
        one_result r;
        run_one(j->blob, j->labels + j->offsets[i], (uint32_t)(j->offsets[i + 1] - j->offsets[i]),
                j->semantics, j->n, &r);
        if (j->res) {
            j->res[i] = r;
        } else {
            uint64_t h = (uint64_t)r.status * 31u + r.len;
            for (uint32_t k = 0; k < r.len; ++k) h = h * 1000003u + r.ol[k];
            j->checksum += h;
            free(r.il);
            free(r.ol);
            free(r.w);
        }
    }
    return NULL;
}

static void run_shards(const uint8_t* blob, const uint32_t* labels, const uint64_t* offsets,
                       uint32_t num, int semantics, uint32_t n, int threads, one_result* res,
                       uint64_t* checksum) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > num && num > 0) threads = (int)num;
    shard_job* jobs = (shard_job*)calloc((size_t)threads, sizeof(shard_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        jobs[t].blob = blob;
        jobs[t].labels = labels;
        jobs[t].offsets = offsets;
        jobs[t].begin = (uint32_t)((uint64_t)num * t / threads);
        jobs[t].end = (uint32_t)((uint64_t)num * (t + 1) / threads);
        jobs[t].semantics = semantics;
        jobs[t].n = n;
        jobs[t].res = res;
    }
    if (threads == 1) {
        shard_main(&jobs[0]);
    } else {
        for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, shard_main, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
    if (checksum) {
        *checksum = 0;
        for (int t = 0; t < threads; ++t) *checksum += jobs[t].checksum;
    }
    free(jobs);
    free(th);
}

or_batch_result* or_batch_run(const uint8_t* blob, const uint32_t* labels, const uint64_t* offsets,
                              uint32_t num, int semantics, uint32_t n, int threads) {
    one_result* res = (one_result*)calloc(num ? num : 1, sizeof(one_result));
    run_shards(blob, labels, offsets, num, semantics, n, threads, res, NULL);
    or_batch_result* r = (or_batch_result*)calloc(1, sizeof(or_batch_result));
    r->num_strings = num;
    r->status = (int32_t*)calloc(num ? num : 1, sizeof(int32_t));
    r->empty = (uint8_t*)calloc(num ? num : 1, 1);
    r->offsets = (uint64_t*)calloc((size_t)num + 1, sizeof(uint64_t));
    r->finals = (double*)calloc(num ? num : 1, sizeof(double));
    r->tuples = (uint64_t*)calloc(num ? num : 1, sizeof(uint64_t));
    r->relaxations = (uint64_t*)calloc(num ? num : 1, sizeof(uint64_t));
    uint64_t total = 0;
    for (uint32_t i = 0; i < num; ++i) {
        r->offsets[i] = total;
        total += res[i].len;
    }
    r->offsets[num] = total;
    r->total_arcs = total;
    r->ilabels = (uint32_t*)malloc((total ? total : 1) * sizeof(uint32_t));
    r->olabels = (uint32_t*)malloc((total ? total : 1) * sizeof(uint32_t));
    r->weights = (double*)malloc((total ? total : 1) * sizeof(double));
    for (uint32_t i = 0; i < num; ++i) {
        r->status[i] = res[i].status;
        r->empty[i] = res[i].empty;
        r->finals[i] = res[i].final_w;
        r->tuples[i] = res[i].tuples;
        r->relaxations[i] = res[i].relax;
        uint64_t o = r->offsets[i];
        for (uint32_t k = 0; k < res[i].len; ++k) {
            r->ilabels[o + k] = res[i].il[k];
            r->olabels[o + k] = res[i].ol[k];
            r->weights[o + k] = res[i].w[k];
        }
        free(res[i].il);
        free(res[i].ol);
        free(res[i].w);
    }
    free(res);
    return r;
}

void or_batch_result_free(or_batch_result* r) {
    if (!r) return;
    free(r->status);
    free(r->empty);
    free(r->offsets);
    free(r->ilabels);
    free(r->olabels);
    free(r->weights);
    free(r->finals);
    free(r->tuples);
    free(r->relaxations);
    free(r);
}

double or_batch_time(const uint8_t* blob, const uint32_t* labels, const uint64_t* offsets,
                     uint32_t num, int semantics, int threads, uint64_t* checksum) {
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    run_shards(blob, labels, offsets, num, semantics, 1, threads, NULL, checksum);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
