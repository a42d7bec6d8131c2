/*
 * refsem.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference
 * Keto Check/Expand engines, used as the parity oracle and as bench.py's
 * cpu_baseline ("port").  Never linked by the product.
 *
 * Schedule: the reference evaluates sub-checks through checkgroup with one
 * reservation per group (internal/check/checkgroup/concurrent_checkgroup.go:
 * 66-138): results are consumed in add order, but Add returns as soon as the
 * sub-check's goroutine is handed to the consumer (:150-159).  So in
 * checkExpandSubject's child loop (engine.go:151-162) the parent marks the NEXT
 * sibling visited right after starting child k -- in practice long before child
 * k's subtree does its first read -- and keeps marking siblings that were
 * already visited until it reaches one that was not; it then blocks in Add until
 * child k is done.  After a decisive (IsMember / error) child, Add no longer
 * blocks and the loop marks every remaining sibling before the result is sent.
 * The canonical order (SCHED_EAGER) is exactly that: mark siblings up to the
 * next unvisited one before running child k; drain the rest after a decisive
 * child.  Every other sub-check runs to completion in add order.
 * SCHED_SEQUENTIAL (each child completes before the next is even marked, the
 * round-1 order) is kept as the alternative legal schedule the schedule-
 * sensitivity report (rs_check_ex) compares against.
 */
#define _GNU_SOURCE
#include "refsem.h"

#include <sched.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#define MAX_RECURSION 4096
#define REACH_CAP_MAX 128 /* u_reach_prunes: RS_REACH_CAP (A/B runs; the product's KETO_REACH_CAP), default 32 */

typedef struct {
    uint32_t ns, obj, rel, kind, sid, sns, srel;
} key7;

struct rs_db {
    const rs_tuple *t; /* the caller's tuples: read while the indexes are built */
    size_t n;
    uint32_t *perm;    /* build only: tuple indices sorted by (ns, obj, rel, shard) */
    uint32_t *exq;     /* build only: tuple indices sorted by (ns, obj, rel, subject) */
    key7 *rt;          /* rows: (ns, obj, rel, subject) in (ns, obj, rel, shard) order */
    key7 *ex;          /* EXISTS keys, sorted */
    int shard_bytes;   /* shard_hi/lo hold the raw UUID bytes (product layout) */
    rs_ns *ns;
    rs_rel *rels;
    rs_ast *ast;
    int32_t *children;
    uint32_t *vclass;
    uint8_t *ssrel;    /* [n_ns * n_relnames]: some tuple of (ns, rel) has a subject set */
    uint8_t *sstarget; /* [n_ns * n_relnames]: some tuple's subject set is a (ns, ., rel) */
    int32_t aliased;   /* two relation slots share a visited class (the engine's vkey table) */
    int32_t no_reach;  /* rs_set_reach(db, 0) / RS_NO_REACH=1: the engine built without tables */
    uint32_t reach_cap;
    uint32_t n_ns, n_relnames, empty_rel, n_rels, n_ast, n_children;
    int32_t strict, max_depth, max_width;
};

/* ------------------------------------------------------------------ */
/* indexes: a parallel LSD radix sort of packed (ns, obj, rel) keys, then */
/* each equal-key run ordered by shard (rows) or by subject (EXISTS).     */

static int cmp_u32(uint32_t a, uint32_t b) { return a < b ? -1 : a > b; }
static int cmp_u64(uint64_t a, uint64_t b) { return a < b ? -1 : a > b; }

static uint64_t sh_hi(const rs_db *db, const rs_tuple *t) {
    return db->shard_bytes ? __builtin_bswap64(t->shard_hi) : t->shard_hi;
}
static uint64_t sh_lo(const rs_db *db, const rs_tuple *t) {
    return db->shard_bytes ? __builtin_bswap64(t->shard_lo) : t->shard_lo;
}

/* ORDER BY nid, shard_id  (traverser.go:88, relationtuples.go:216) within one row */
static int cmp_shard(const rs_db *db, uint32_t ia, uint32_t ib) {
    const rs_tuple *a = &db->t[ia], *b = &db->t[ib];
    int c;
    if ((c = cmp_u64(sh_hi(db, a), sh_hi(db, b)))) return c;
    if ((c = cmp_u64(sh_lo(db, a), sh_lo(db, b)))) return c;
    return cmp_u32(ia, ib);
}
static int cmp_subject(const rs_db *db, uint32_t ia, uint32_t ib) {
    const rs_tuple *a = &db->t[ia], *b = &db->t[ib];
    int c;
    if ((c = cmp_u32(a->kind, b->kind))) return c;
    if ((c = cmp_u32(a->sid, b->sid))) return c;
    if (a->kind == 1) {
        if ((c = cmp_u32(a->sns, b->sns))) return c;
        if ((c = cmp_u32(a->srel, b->srel))) return c;
    }
    return cmp_u32(ia, ib);
}

typedef int (*idx_cmp)(const rs_db *, uint32_t, uint32_t);

static void sift(const rs_db *db, idx_cmp cmp, uint32_t *a, size_t root, size_t len) {
    for (;;) {
        size_t c = 2 * root + 1;
        if (c >= len) return;
        if (c + 1 < len && cmp(db, a[c], a[c + 1]) < 0) c++;
        if (cmp(db, a[root], a[c]) >= 0) return;
        uint32_t x = a[root];
        a[root] = a[c];
        a[c] = x;
        root = c;
    }
}
static void sort_idx(const rs_db *db, idx_cmp cmp, uint32_t *a, size_t len) {
    if (len <= 24) {
        for (size_t i = 1; i < len; i++) {
            uint32_t x = a[i];
            size_t j = i;
            while (j > 0 && cmp(db, x, a[j - 1]) < 0) {
                a[j] = a[j - 1];
                j--;
            }
            a[j] = x;
        }
        return;
    }
    for (size_t r = len / 2; r-- > 0;) sift(db, cmp, a, r, len);
    for (size_t e = len - 1; e > 0; e--) {
        uint32_t x = a[0];
        a[0] = a[e];
        a[e] = x;
        sift(db, cmp, a, 0, e);
    }
}

static int build_threads(void) {
    const char *e = getenv("REFSEM_THREADS");
    if (e && atoi(e) > 0) return atoi(e);
    cpu_set_t cs;
    int n = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 1;
    return n < 1 ? 1 : (n > 16 ? 16 : n);
}

typedef struct {
    const rs_db *db;
    uint64_t *key, *key2;
    uint32_t *idx, *idx2;
    size_t n, b, e;
    int shift, nth, tid;
    size_t *hist; /* [nth][2048] */
    uint32_t bn, bo, br;
    uint32_t *runs_perm, *runs_exq;
} sort_job;

#define RADIX 11
#define NBUCKET (1u << RADIX)

static void *job_keys(void *p) {
    sort_job *j = p;
    for (size_t i = j->b; i < j->e; i++) {
        const rs_tuple *t = &j->db->t[i];
        j->key[i] = (((uint64_t)t->ns << j->bo | t->obj) << j->br) | t->rel;
        j->idx[i] = (uint32_t)i;
    }
    return NULL;
}
static void *job_hist(void *p) {
    sort_job *j = p;
    size_t *h = j->hist + (size_t)j->tid * NBUCKET;
    memset(h, 0, NBUCKET * sizeof *h);
    for (size_t i = j->b; i < j->e; i++) h[(j->key[i] >> j->shift) & (NBUCKET - 1)]++;
    return NULL;
}
static void *job_scatter(void *p) {
    sort_job *j = p;
    size_t *h = j->hist + (size_t)j->tid * NBUCKET; /* per-thread write cursors */
    for (size_t i = j->b; i < j->e; i++) {
        size_t o = h[(j->key[i] >> j->shift) & (NBUCKET - 1)]++;
        j->key2[o] = j->key[i];
        j->idx2[o] = j->idx[i];
    }
    return NULL;
}
/* order each equal-key run: rows by shard, EXISTS by subject */
static void *job_runs(void *p) {
    sort_job *j = p;
    size_t i = j->b;
    while (i > 0 && i < j->n && j->key[i] == j->key[i - 1]) i++; /* runs start in their own chunk */
    while (i < j->e) {
        size_t k = i + 1;
        while (k < j->n && j->key[k] == j->key[i]) k++;
        if (k - i > 1) {
            sort_idx(j->db, cmp_shard, j->runs_perm + i, k - i);
            sort_idx(j->db, cmp_subject, j->runs_exq + i, k - i);
        }
        i = k;
    }
    return NULL;
}

static key7 mk_key(const rs_tuple *t) {
    key7 k = {t->ns, t->obj, t->rel, t->kind, t->sid, 0, 0};
    if (t->kind == 1) {
        k.sns = t->sns;
        k.srel = t->srel;
    }
    return k;
}
static void *job_gather(void *p) {
    sort_job *j = p;
    for (size_t i = j->b; i < j->e; i++) {
        j->db->rt[i] = mk_key(&j->db->t[j->db->perm[i]]);
        j->db->ex[i] = mk_key(&j->db->t[j->db->exq[i]]);
    }
    return NULL;
}

static void run_jobs(sort_job *jobs, int nth, void *(*fn)(void *)) {
    pthread_t th[64];
    for (int t = 0; t < nth; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nth; t++) pthread_join(th[t], NULL);
}

static int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) b++;
    return b;
}

static void build_index(rs_db *db) {
    const size_t n = db->n;
    db->perm = malloc((n ? n : 1) * sizeof *db->perm);
    db->exq = malloc((n ? n : 1) * sizeof *db->exq);
    if (!n) {
        db->rt = malloc(sizeof *db->rt);
        db->ex = malloc(sizeof *db->ex);
        return;
    }
    uint32_t mns = 0, mobj = 0, mrel = 0;
    for (size_t i = 0; i < n; i++) {
        if (db->t[i].ns > mns) mns = db->t[i].ns;
        if (db->t[i].obj > mobj) mobj = db->t[i].obj;
        if (db->t[i].rel > mrel) mrel = db->t[i].rel;
    }
    const uint32_t bo = bits_for(mobj), br = bits_for(mrel), bn = bits_for(mns);
    const int total = bn + bo + br;
    int nth = build_threads();
    if (n < (1u << 16)) nth = 1;
    if (nth > 64) nth = 64;
    uint64_t *key = malloc(n * sizeof *key), *key2 = malloc(n * sizeof *key2);
    uint32_t *idx2 = malloc(n * sizeof *idx2);
    uint32_t *idx = db->perm;
    size_t *hist = malloc((size_t)nth * NBUCKET * sizeof *hist);
    sort_job jobs[64];
    for (int t = 0; t < nth; t++) {
        jobs[t] = (sort_job){db, key, key2, idx, idx2, n, n * t / nth, n * (t + 1) / nth, 0, nth, t, hist, bn, bo, br,
                             NULL, NULL};
    }
    run_jobs(jobs, nth, job_keys);
    for (int shift = 0; shift < total; shift += RADIX) {
        for (int t = 0; t < nth; t++) jobs[t].shift = shift;
        run_jobs(jobs, nth, job_hist);
        size_t acc = 0; /* bucket-major, thread-minor: a stable LSD pass */
        for (uint32_t b = 0; b < NBUCKET; b++)
            for (int t = 0; t < nth; t++) {
                size_t c = hist[(size_t)t * NBUCKET + b];
                hist[(size_t)t * NBUCKET + b] = acc;
                acc += c;
            }
        run_jobs(jobs, nth, job_scatter);
        for (int t = 0; t < nth; t++) {
            uint64_t *k = jobs[t].key;
            jobs[t].key = jobs[t].key2;
            jobs[t].key2 = k;
            uint32_t *x = jobs[t].idx;
            jobs[t].idx = jobs[t].idx2;
            jobs[t].idx2 = x;
        }
    }
    uint64_t *fk = jobs[0].key; /* after the passes: sorted keys and indices */
    if (jobs[0].idx != db->perm) memcpy(db->perm, jobs[0].idx, n * sizeof *idx);
    memcpy(db->exq, db->perm, n * sizeof *db->perm);
    for (int t = 0; t < nth; t++) {
        jobs[t].key = fk;
        jobs[t].runs_perm = db->perm;
        jobs[t].runs_exq = db->exq;
    }
    run_jobs(jobs, nth, job_runs);
    free(hist);
    free(key);
    free(key2);
    free(idx2);
    /* materialize both orders as compact records: sequential row scans, no indirection */
    db->rt = malloc(n * sizeof *db->rt);
    db->ex = malloc(n * sizeof *db->ex);
    run_jobs(jobs, nth, job_gather);
    free(db->perm);
    free(db->exq);
    db->perm = db->exq = NULL;
}

rs_db *rs_build(const rs_tuple *tuples, size_t n, const rs_config *cfg) {
    rs_db *db = calloc(1, sizeof *db);
    db->n = n;
    db->t = tuples;
    db->shard_bytes = cfg->shard_bytes;
    build_index(db);

    db->n_ns = cfg->n_ns;
    db->n_relnames = cfg->n_relnames;
    db->empty_rel = cfg->empty_rel;
    db->n_rels = cfg->n_rels;
    db->n_ast = cfg->n_ast;
    db->n_children = cfg->n_children;
#define DUP(field, cnt)                                                  \
    do {                                                                 \
        size_t sz = (size_t)(cnt) * sizeof *cfg->field;                  \
        db->field = malloc(sz ? sz : 1);                                 \
        if (sz) memcpy(db->field, cfg->field, sz);                       \
    } while (0)
    DUP(ns, cfg->n_ns);
    DUP(rels, cfg->n_rels);
    DUP(ast, cfg->n_ast);
    DUP(children, cfg->n_children);
    DUP(vclass, (size_t)cfg->n_ns * cfg->n_relnames);
#undef DUP
    db->strict = cfg->strict;
    db->max_depth = cfg->max_depth;
    db->max_width = cfg->max_width;
    const size_t NR = (size_t)db->n_ns * db->n_relnames;
    db->ssrel = calloc(NR + 1, 1);
    db->sstarget = calloc(NR + 1, 1);
    uint8_t *slot = calloc(NR + 1, 1); /* the engine's relation slots: declared or used pairs */
    for (size_t i = 0; i < n; i++) {
        const key7 *t = &db->rt[i];
        if (t->ns < db->n_ns && t->rel < db->n_relnames) slot[(size_t)t->ns * db->n_relnames + t->rel] = 1;
        if (t->kind != 1) continue;
        if (t->ns < db->n_ns && t->rel < db->n_relnames) db->ssrel[(size_t)t->ns * db->n_relnames + t->rel] = 1;
        if (t->sns < db->n_ns && t->srel < db->n_relnames) {
            db->sstarget[(size_t)t->sns * db->n_relnames + t->srel] = 1;
            slot[(size_t)t->sns * db->n_relnames + t->srel] = 1;
        }
    }
    for (uint32_t a = 0; a < db->n_ns; a++)
        if (db->ns[a].configured)
            for (int i = 0; i < db->ns[a].rel_count; i++) {
                const uint32_t r = db->rels[db->ns[a].rel_begin + i].name;
                if (r < db->n_relnames) slot[(size_t)a * db->n_relnames + r] = 1;
            }
    /* csrc/snapshot.cpp "visited keys": slots whose ns+"-"+rel strings are equal */
    uint32_t maxc = 0;
    for (size_t i = 0; i < NR; i++)
        if (slot[i] && db->vclass[i] > maxc) maxc = db->vclass[i];
    uint8_t *seen = calloc((size_t)maxc + 2, 1);
    for (size_t i = 0; i < NR; i++)
        if (slot[i]) {
            if (seen[db->vclass[i]]) db->aliased = 1;
            seen[db->vclass[i]] = 1;
        }
    free(seen);
    free(slot);
    const char *nr = getenv("RS_NO_REACH"); /* (the product's KETO_NO_REACH=1) */
    db->no_reach = nr && *nr == '1';
    const char *rc = getenv("RS_REACH_CAP");
    db->reach_cap = rc ? (uint32_t)atoi(rc) : 32;
    if (db->reach_cap < 1 || db->reach_cap > REACH_CAP_MAX) db->reach_cap = 32;
    return db;
}

void rs_free(rs_db *db) {
    if (!db) return;
    free(db->perm);
    free(db->exq);
    free(db->rt);
    free(db->ex);
    free(db->ns);
    free(db->rels);
    free(db->ast);
    free(db->children);
    free(db->vclass);
    free(db->sstarget);
    free(db->ssrel);
    free(db);
}

void rs_set_limits(rs_db *db, int32_t max_depth, int32_t max_width) {
    db->max_depth = max_depth;
    db->max_width = max_width;
}

static int cmp_row(const key7 *t, uint32_t ns, uint32_t obj, uint32_t rel) {
    int c = cmp_u32(t->ns, ns);
    if (!c) c = cmp_u32(t->obj, obj);
    if (!c) c = cmp_u32(t->rel, rel);
    return c;
}

/* rows of (ns,obj,rel): rt[lo, hi) in shard order */
static void node_rows(const rs_db *db, uint32_t ns, uint32_t obj, uint32_t rel, size_t *lo, size_t *hi) {
    size_t a = 0, b = db->n;
    while (a < b) {
        size_t m = (a + b) / 2;
        if (cmp_row(&db->rt[m], ns, obj, rel) < 0) a = m + 1;
        else b = m;
    }
    *lo = a;
    b = db->n;
    while (a < b) {
        size_t m = (a + b) / 2;
        if (cmp_row(&db->rt[m], ns, obj, rel) <= 0) a = m + 1;
        else b = m;
    }
    *hi = a;
}
static int cmp_key7(const void *pa, const void *pb) {
    const uint32_t *a = pa, *b = pb;
    for (int i = 0; i < 7; i++) {
        int c = cmp_u32(a[i], b[i]);
        if (c) return c;
    }
    return 0;
}
#define ROW(db, i) (&(db)->rt[i])

/* ------------------------------------------------------------------ */
/* per-query evaluation context                                         */

typedef struct {
    uint64_t *slot;
    int32_t *dep; /* rest depth at which each key was marked */
    size_t cap, cnt;
    /* schedule-sensitivity evidence of this visited scope: siblings pruned as already
     * visited (dskips: marked at another rest depth than the pruned occurrence), depth
     * truncation inside the scope, and the order-sensitive events (width truncation, errors,
     * AND / NOT evaluated) */
    uint32_t skips, dskips, trunc, events;
} vset;

enum { SCHED_EAGER = 0, SCHED_SEQUENTIAL = 1 };

typedef struct {
    const rs_db *db;
    uint32_t kind, sid, sns, srel; /* the query subject: never changes (traverser.go:102) */
    rs_stats *st;
    int depth_guard;
    int sched;
    uint32_t flags; /* RS_F_SENSITIVE */
    uint64_t mx_nodes; /* maximal exploration: checks built so far */
} qctx;

/* an order-sensitive event inside the current visited scope (if any) */
static void scope_event(vset *vs) {
    if (vs) vs->events++;
}
/* depth truncation inside the current scope: order-sensitive only where pruned nodes can be
 * reached at different rest depths */
static void scope_trunc(vset *vs) {
    if (vs) vs->trunc++;
}

typedef struct {
    int m;
    int err;
} res;

static const res R_UNK = {RS_UNKNOWN, 0};
static const res R_IS = {RS_IS_MEMBER, 0};
static const res R_NOT = {RS_NOT_MEMBER, 0};

static int decisive(res r) { return r.err != 0 || r.m == RS_IS_MEMBER; }

static vset *vset_new(void) {
    vset *v = calloc(1, sizeof *v);
    v->cap = 64;
    v->slot = calloc(v->cap, sizeof *v->slot);
    v->dep = calloc(v->cap, sizeof *v->dep);
    return v;
}
static void vset_free(vset *v) {
    if (v) {
        free(v->slot);
        free(v->dep);
        free(v);
    }
}
/* end of a scope owned by the ES that opened it.  Another legal schedule only changes WHICH
 * occurrence of a node reached twice is explored; that can change the scope's result only if
 * pruning meets an order-sensitive event -- width truncation, an error, AND / NOT -- or if the
 * occurrences carry different rest depths and some depth truncation happened in the scope. */
static void scope_close(uint32_t *flags, vset *own) {
    if (own && ((own->skips && own->events) || (own->dskips && own->trunc))) *flags |= RS_F_SENSITIVE;
    vset_free(own);
}
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}
/* stringSet.addNoDuplicate (x/graph/graph_utils.go:27-36): returns 1 if present (*prev = the
 * rest depth it was marked at), else inserts the key with rest depth d */
static int vset_add_d(vset *v, uint64_t key, int32_t d, int32_t *prev) {
    key += 1; /* 0 = empty slot */
    if (2 * (v->cnt + 1) > v->cap) {
        size_t nc = v->cap * 2;
        uint64_t *ns = calloc(nc, sizeof *ns);
        int32_t *nd = calloc(nc, sizeof *nd);
        for (size_t i = 0; i < v->cap; i++) {
            uint64_t k = v->slot[i];
            if (!k) continue;
            size_t h = mix64(k) & (nc - 1);
            while (ns[h]) h = (h + 1) & (nc - 1);
            ns[h] = k;
            nd[h] = v->dep[i];
        }
        free(v->slot);
        free(v->dep);
        v->slot = ns;
        v->dep = nd;
        v->cap = nc;
    }
    size_t h = mix64(key) & (v->cap - 1);
    while (v->slot[h]) {
        if (v->slot[h] == key) {
            if (prev) *prev = v->dep[h];
            return 1;
        }
        h = (h + 1) & (v->cap - 1);
    }
    v->slot[h] = key;
    v->dep[h] = d;
    v->cnt++;
    return 0;
}
static int vset_add(vset *v, uint64_t key) { return vset_add_d(v, key, 0, NULL); }

/* SubjectSet.UniqueID = UUIDv5(obj, ns+"-"+rel) (relationtuple/definitions.go:114-116) */
static uint64_t vkey(const rs_db *db, uint32_t ns, uint32_t obj, uint32_t rel) {
    /* ids outside the tables name a (namespace, relation) no tuple holds: a class of its own */
    if (ns >= db->n_ns || rel >= db->n_relnames) return ((uint64_t)obj << 32) | (0x80000000u | (ns << 16) | (rel & 0xFFFFu));
    uint32_t cls = db->vclass[(size_t)ns * db->n_relnames + rel];
    return ((uint64_t)obj << 32) | cls;
}

/* ExistsRelationTuples (persistence/sql/relationtuples.go:249-261) for the query subject */
static int exists(const qctx *c, uint32_t ns, uint32_t obj, uint32_t rel) {
    key7 k = {ns, obj, rel, c->kind, c->sid, 0, 0};
    if (c->kind == 1) {
        k.sns = c->sns;
        k.srel = c->srel;
    }
    c->st->probes++;
    return bsearch(&k, c->db->ex, c->db->n, sizeof k, cmp_key7) != NULL;
}

/* namespace.ASTRelationFor (internal/namespace/definitions.go:37-62).
 * Returns relation index or -1 (nil relation); *err on "does not exist". */
static int ast_relation_for(const rs_db *db, uint32_t ns, uint32_t rel, int *err) {
    *err = 0;
    if (rel == db->empty_rel) return -1;                   /* :40-42 */
    if (ns >= db->n_ns || !db->ns[ns].configured) return -1; /* :43-48 */
    if (db->ns[ns].rel_count == 0) return -1;              /* :52-54 */
    for (int i = 0; i < db->ns[ns].rel_count; i++) {
        int ri = db->ns[ns].rel_begin + i;
        if (db->rels[ri].name == rel) return ri;           /* :56-60 */
    }
    *err = RS_ERR_NO_RELATION;                             /* :61 */
    return -1;
}

static res check_is_allowed(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip_direct,
                            vset *vs);
static res check_rewrite(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs);
static res check_inverted(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs);

/* checkDirect (internal/check/engine.go:167-208) */
static res check_direct(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, vset *vs) {
    if (d <= 0) { /* :168-173 */
        scope_trunc(vs);
        return R_UNK;
    }
    return exists(c, ns, obj, rel) ? R_IS : R_NOT;
}

/* checkExpandSubject's child list: the kept subject-set rows of [lo, hi) in shard order */
typedef struct {
    size_t i, hi, left; /* next row, row end, children not yet reached */
} kids;

/* CheckAndAddVisited over the next children until one was not visited (engine.go:157-160);
 * 1 + its row index in *at, or 0 when the list is exhausted */
static int advance(qctx *c, kids *k, vset *vs, int d, size_t *at) {
    const rs_db *db = c->db;
    while (k->left && k->i < k->hi) {
        const key7 *t = ROW(db, k->i);
        const size_t i = k->i++;
        if (t->kind != 1) continue;
        k->left--;
        int32_t prev = d;
        if (vset_add_d(vs, vkey(db, t->sns, t->sid, t->srel), d, &prev)) {
            vs->skips++;
            if (prev != d) vs->dskips++;
            continue;
        }
        *at = i;
        return 1;
    }
    return 0;
}

/* checkExpandSubject (engine.go:102-164) + TraverseSubjectSetExpansion (traverser.go:53-121) */
static res check_expand_subject(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, vset *vs) {
    if (d <= 0) { /* :103-108 */
        scope_trunc(vs);
        return R_UNK;
    }
    const rs_db *db = c->db;
    vset *own = NULL;
    if (!vs) vs = own = vset_new(); /* graph.InitVisited (graph_utils.go:38-43) */
    size_t lo, hi;
    node_rows(db, ns, obj, rel, &lo, &hi);
    c->st->rows++;
    /* subject-set rows in shard order, each with EXISTS(found) lookahead; stop at first found */
    size_t nres = 0;
    for (size_t i = lo; i < hi; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue; /* current.subject_id IS NULL (traverser.go:87) */
        c->st->edges++;
        nres++;
        if (exists(c, t->sns, t->sid, t->srel)) { /* :109-111, engine.go:133-138 */
            scope_close(&c->flags, own);
            return R_IS;
        }
    }
    /* width truncation: results[:maxWidth-1] (engine.go:141-150) */
    size_t keep = nres;
    if ((long)nres > (long)db->max_width) {
        keep = db->max_width > 0 ? (size_t)(db->max_width - 1) : 0;
        scope_event(vs);
    }
    kids k = {lo, hi, keep};
    res out = R_NOT;
    size_t at;
    if (c->sched == SCHED_SEQUENTIAL) {
        while (advance(c, &k, vs, d, &at)) {
            const key7 *t = ROW(db, at);
            res r = check_is_allowed(c, t->sns, t->sid, t->srel, d, 1, vs); /* :161 */
            if (decisive(r)) {
                out = r;
                break;
            }
        }
        scope_close(&c->flags, own);
        return out;
    }
    /* SCHED_EAGER: g.Add(check_k) returns once check_k is handed to the group's consumer
     * (concurrent_checkgroup.go:150-159), so the loop marks the following siblings -- up to
     * and including the next one that was not visited yet -- before check_k runs, then
     * waits in the next Add for check_k's result. */
    size_t next;
    int have = advance(c, &k, vs, d, &next);
    while (have) {
        const key7 *t = ROW(db, next);
        have = advance(c, &k, vs, d, &next);
        res r = check_is_allowed(c, t->sns, t->sid, t->srel, d, 1, vs); /* :161 */
        if (decisive(r)) {
            /* the group is done, so every later Add returns at once: the loop still marks
             * every remaining sibling before its deferred result is sent (:119, :151-162).
             * Marks in a scope this ES owns die with it. */
            if (!own)
                while (advance(c, &k, vs, d, &at)) {
                }
            out = r;
            break;
        }
    }
    scope_close(&c->flags, own);
    return out;
}

/* checkComputedSubjectSet (rewrites.go:208-230) */
static res check_css(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, vset *vs) {
    if (d < 0) { /* :214-217 */
        scope_trunc(vs);
        return R_UNK;
    }
    return check_is_allowed(c, ns, obj, rel, d, 0, vs);
}

/* checkTupleToSubjectSet (rewrites.go:242-293) + GetRelationTuples (relationtuples.go:207-247) */
static res check_ttu(qctx *c, uint32_t ns, uint32_t obj, const rs_ast *a, int d, vset *vs) {
    if (d < 0) { /* :247-250 */
        scope_trunc(vs);
        return R_UNK;
    }
    const rs_db *db = c->db;
    size_t lo, hi;
    node_rows(db, ns, obj, a->rel, &lo, &hi);
    c->st->rows++;
    for (size_t i = lo; i < hi; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue; /* subject IDs are skipped (:280) */
        c->st->edges++;
        res r = check_is_allowed(c, t->sns, t->sid, a->computed, d - 1, 0, vs); /* :281-286 */
        if (decisive(r)) return r;
    }
    return R_NOT;
}

/* OR computed-userset shortcut: rewrites.go:62-92 + TraverseSubjectSetRewrite (traverser.go:123-191) */
static res check_shortcut(qctx *c, uint32_t ns, uint32_t obj, const rs_ast *a, int d, vset *vs) {
    const rs_db *db = c->db;
    int any_probe = 0, found = 0;
    for (int k = 0; k < a->child_count; k++) {
        const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
        if (ch->type != RS_CSS) continue;
        int err;
        int ri = ast_relation_for(db, ns, ch->rel, &err); /* error ignored (:134) */
        if (db->strict && ri >= 0 && db->rels[ri].rewrite >= 0) continue; /* :137-139 */
        any_probe = 1;
        if (!found && exists(c, ns, obj, ch->rel)) found = 1; /* relation IN (...) LIMIT 1 */
    }
    (void)any_probe;
    if (found) return R_IS; /* :160-172, rewrites.go:81-86 */
    for (int k = 0; k < a->child_count; k++) {
        const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
        if (ch->type != RS_CSS) continue;
        res r = check_is_allowed(c, ns, obj, ch->rel, d - 1, 1, vs); /* rewrites.go:88-90 */
        if (decisive(r)) return r;
    }
    return R_NOT;
}

/* dispatch of one rewrite child (rewrites.go:100-125 / 153-178) */
static res check_child(qctx *c, uint32_t ns, uint32_t obj, int ci, int d, int nested_cost, vset *vs) {
    const rs_ast *ch = &c->db->ast[ci];
    switch (ch->type) {
    case RS_TTU:
        return check_ttu(c, ns, obj, ch, d, vs);
    case RS_CSS:
        return check_css(c, ns, obj, ch->rel, d, vs);
    case RS_REWRITE:
        return check_rewrite(c, ns, obj, ci, d - nested_cost, vs);
    case RS_INVERT:
        return check_inverted(c, ns, obj, ci, d, vs);
    default: {
        res r = {RS_UNKNOWN, RS_ERR_NOT_IMPLEMENTED};
        return r;
    }
    }
}

/* checkSubjectSetRewrite (rewrites.go:33-134) + or/and (binop.go:18-73) */
static res check_rewrite(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs) {
    if (d <= 0) { /* :39-42 */
        scope_trunc(vs);
        return R_UNK;
    }
    const rs_db *db = c->db;
    const rs_ast *a = &db->ast[ai];
    if (a->op == RS_OP_AND) scope_event(vs);
    if (a->op != RS_OP_OR && a->op != RS_OP_AND) {
        scope_event(vs);
        res r = {RS_UNKNOWN, RS_ERR_NOT_IMPLEMENTED}; /* :58-59 */
        return r;
    }
    if (++c->depth_guard > MAX_RECURSION) {
        c->depth_guard--;
        res r = {RS_UNKNOWN, RS_ERR_INTERNAL};
        return r;
    }
    int nchecks = 0;
    res out = R_NOT;
    if (a->op == RS_OP_OR) {
        int has_css = 0;
        for (int k = 0; k < a->child_count; k++)
            if (db->ast[db->children[a->child_begin + k]].type == RS_CSS) has_css = 1;
        if (has_css) {
            nchecks++;
            res r = check_shortcut(c, ns, obj, a, d, vs);
            if (decisive(r)) {
                out = r;
                goto done;
            }
        }
    }
    for (int k = 0; k < a->child_count; k++) {
        int ci = db->children[a->child_begin + k];
        if (a->op == RS_OP_OR && db->ast[ci].type == RS_CSS) continue; /* handled (:95-98) */
        nchecks++;
        res r = check_child(c, ns, obj, ci, d, 1, vs); /* nested rewrite: restDepth-1 (:118) */
        if (a->op == RS_OP_OR) {
            if (decisive(r)) { /* binop.go:23-26 */
                out = r;
                goto done;
            }
        } else if (r.err || r.m != RS_IS_MEMBER) { /* binop.go:52-54 */
            out.m = RS_NOT_MEMBER;
            out.err = r.err;
            goto done;
        }
    }
    if (a->op == RS_OP_AND) out = nchecks ? R_IS : R_NOT; /* binop.go:42-44, 62-65 */
    else out = R_NOT;                                     /* binop.go:19-21, 38 */
done:
    c->depth_guard--;
    return out;
}

/* checkInverted (rewrites.go:136-200) */
static res check_inverted(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs) {
    scope_event(vs);
    if (d < 0) return R_UNK; /* :142-145 */
    const rs_ast *a = &c->db->ast[ai];
    if (a->child_count != 1) {
        res r = {RS_UNKNOWN, RS_ERR_NOT_IMPLEMENTED};
        return r;
    }
    if (++c->depth_guard > MAX_RECURSION) {
        c->depth_guard--;
        res r = {RS_UNKNOWN, RS_ERR_INTERNAL};
        return r;
    }
    /* nested rewrite under NOT keeps restDepth (:171) */
    res r = check_child(c, ns, obj, c->db->children[a->child_begin], d, 0, vs);
    c->depth_guard--;
    if (r.m == RS_IS_MEMBER) r.m = RS_NOT_MEMBER; /* :189-194 */
    else if (r.m == RS_NOT_MEMBER) r.m = RS_IS_MEMBER;
    return r;
}

/* checkIsAllowed (engine.go:214-249) */
static res check_is_allowed(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip_direct,
                            vset *vs) {
    if (d <= 0) { /* :215-220 */
        scope_trunc(vs);
        return R_UNK;
    }
    const rs_db *db = c->db;
    if (++c->depth_guard > MAX_RECURSION) {
        c->depth_guard--;
        res r = {RS_UNKNOWN, RS_ERR_INTERNAL};
        return r;
    }
    int err;
    int ri = ast_relation_for(db, ns, rel, &err); /* :228-232 */
    res out = R_NOT;
    if (err) {
        scope_event(vs);
        out.m = RS_UNKNOWN;
        out.err = err;
        goto done;
    }
    int has_rewrite = ri >= 0 && db->rels[ri].rewrite >= 0;                 /* :233 */
    int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;        /* :235 */
    if (has_rewrite) {                                                      /* :236-238 */
        res r = check_rewrite(c, ns, obj, db->rels[ri].rewrite, d, vs);
        if (decisive(r)) {
            out = r;
            goto done;
        }
    }
    if ((!db->strict || !has_rewrite) && !skip_direct) { /* :239-243 */
        res r = check_direct(c, ns, obj, rel, d - 1, vs);
        if (decisive(r)) {
            out = r;
            goto done;
        }
    }
    if (can_ss) { /* :244-246 */
        res r = check_expand_subject(c, ns, obj, rel, d - 1, vs);
        if (decisive(r)) {
            out = r;
            goto done;
        }
    }
done:
    c->depth_guard--;
    return out;
}

/* Engine.CheckRelationTuple (engine.go:76-95) under schedule `sched` */
static int check_sched(rs_db *db, const rs_query *q, int32_t *err, rs_stats *st, int sched, uint32_t *flags) {
    rs_stats dummy = {0, 0, 0, 0};
    qctx c = {db, q->kind, q->sid, q->kind == 1 ? q->sns : 0, q->kind == 1 ? q->srel : 0,
              st ? st : &dummy, 0, sched, 0, 0};
    int d = q->depth;
    if (d <= 0 || db->max_depth < d) d = db->max_depth; /* :82-84 */
    res r = check_is_allowed(&c, q->ns, q->obj, q->rel, d, 0, NULL);
    if (err) *err = r.err;
    if (flags) *flags = c.flags;
    return r.m;
}

int rs_check(rs_db *db, const rs_query *q, int32_t *err, rs_stats *st) {
    return check_sched(db, q, err, st, SCHED_EAGER, NULL);
}

/* ------------------------------------------------------------------ */
/* Maximal exploration: every check some legal schedule of the reference can start.          */
/*
 * The two simulated schedules only explore what the recursion reads.  The reference starts
 * more, because its checks are built eagerly (oracle/refconc.py restates it goroutine by
 * goroutine):
 *   - building checkIsAllowed Adds its first sub-check at once (engine.go:226-246), so an
 *     expand-subject (engine.go:161), tuple-to-userset (rewrites.go:281-286) or OR-shortcut
 *     (rewrites.go:88-90) loop starts child k+1 while child k runs -- even when k decides;
 *   - checkSubjectSetRewrite builds its computed-subject-set, nested rewrite and NOT children
 *     when it is built (rewrites.go:94-125, 153-178), so an AND or NOT child runs even where
 *     binop.go's loop never reads it.
 * Those checks mark visited keys too.  So the flag looks at the tree of every check that can
 * be started: no visited pruning, no short-circuit, only the static cut-offs (depth, width,
 * a found-lookahead, a shortcut IN hit).  A scope whose key is reached twice in that tree,
 * together with an order-sensitive event (or a rest-depth difference plus depth truncation),
 * may answer differently under some interleaving.  Trees past MX_NODE_CAP checks, and
 * recursions that never end (an AND's computed subject set reaching its own relation keeps
 * restDepth: the reference overflows its stack), are flagged as they are. */
#define MX_NODE_CAP 2000000u

static void mx_ia(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip_direct, vset *vs);
static void mx_rewrite(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs);

static int mx_enter(qctx *c) {
    if (++c->mx_nodes > MX_NODE_CAP || c->depth_guard + 1 > MAX_RECURSION) {
        c->flags |= RS_F_SENSITIVE | RS_F_MAXEXP;
        return 0;
    }
    c->depth_guard++;
    return 1;
}

static void mx_es(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, vset *vs) {
    if (d <= 0) {
        scope_trunc(vs);
        return;
    }
    const rs_db *db = c->db;
    vset *own = NULL;
    if (!vs) vs = own = vset_new();
    size_t lo, hi;
    node_rows(db, ns, obj, rel, &lo, &hi);
    size_t nres = 0;
    for (size_t i = lo; i < hi; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue;
        nres++;
        if (exists(c, t->sns, t->sid, t->srel)) { /* found: no child is built (engine.go:133-138) */
            if (own && ((own->skips && own->events) || (own->dskips && own->trunc))) c->flags |= RS_F_MAXEXP;
            scope_close(&c->flags, own);
            return;
        }
    }
    size_t left = nres;
    if ((long)nres > (long)db->max_width) {
        left = db->max_width > 0 ? (size_t)(db->max_width - 1) : 0;
        scope_event(vs);
    }
    for (size_t i = lo; i < hi && left; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue;
        left--;
        int32_t prev = d;
        if (vset_add_d(vs, vkey(db, t->sns, t->sid, t->srel), d, &prev)) { /* reached again: explored anyway */
            vs->skips++;
            if (prev != d) vs->dskips++;
        }
        mx_ia(c, t->sns, t->sid, t->srel, d, 1, vs);
    }
    if (own && ((own->skips && own->events) || (own->dskips && own->trunc))) c->flags |= RS_F_MAXEXP;
    scope_close(&c->flags, own);
}

static void mx_child(qctx *c, uint32_t ns, uint32_t obj, int ci, int d, int nested_cost, vset *vs) {
    const rs_db *db = c->db;
    const rs_ast *ch = &db->ast[ci];
    switch (ch->type) {
    case RS_TTU: {
        if (d < 0) {
            scope_trunc(vs);
            return;
        }
        size_t lo, hi;
        node_rows(db, ns, obj, ch->rel, &lo, &hi);
        for (size_t i = lo; i < hi; i++) {
            const key7 *t = ROW(db, i);
            if (t->kind == 1) mx_ia(c, t->sns, t->sid, ch->computed, d - 1, 0, vs);
        }
        return;
    }
    case RS_CSS:
        if (d < 0) scope_trunc(vs);
        else mx_ia(c, ns, obj, ch->rel, d, 0, vs);
        return;
    case RS_REWRITE:
        mx_rewrite(c, ns, obj, ci, d - nested_cost, vs);
        return;
    case RS_INVERT:
        scope_event(vs);
        if (d >= 0 && ch->child_count == 1 && mx_enter(c)) {
            mx_child(c, ns, obj, db->children[ch->child_begin], d, 0, vs);
            c->depth_guard--;
        }
        return;
    default:
        scope_event(vs);
    }
}

static void mx_rewrite(qctx *c, uint32_t ns, uint32_t obj, int ai, int d, vset *vs) {
    if (d <= 0) {
        scope_trunc(vs);
        return;
    }
    const rs_db *db = c->db;
    const rs_ast *a = &db->ast[ai];
    if (a->op != RS_OP_OR) scope_event(vs); /* AND, and not-implemented operators: order-sensitive */
    if (a->op != RS_OP_OR && a->op != RS_OP_AND) return;
    if (!mx_enter(c)) return;
    if (a->op == RS_OP_OR) {
        int found = 0, has_css = 0;
        for (int k = 0; k < a->child_count; k++) {
            const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
            if (ch->type != RS_CSS) continue;
            has_css = 1;
            int err;
            int ri = ast_relation_for(db, ns, ch->rel, &err);
            if (db->strict && ri >= 0 && db->rels[ri].rewrite >= 0) continue;
            if (!found && exists(c, ns, obj, ch->rel)) found = 1;
        }
        if (has_css && !found)
            for (int k = 0; k < a->child_count; k++) {
                const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
                if (ch->type == RS_CSS) mx_ia(c, ns, obj, ch->rel, d - 1, 1, vs);
            }
    }
    for (int k = 0; k < a->child_count; k++) {
        int ci = db->children[a->child_begin + k];
        if (a->op == RS_OP_OR && db->ast[ci].type == RS_CSS) continue;
        mx_child(c, ns, obj, ci, d, 1, vs);
    }
    c->depth_guard--;
}

static void mx_ia(qctx *c, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip_direct, vset *vs) {
    if (d <= 0) {
        scope_trunc(vs);
        return;
    }
    const rs_db *db = c->db;
    if (!mx_enter(c)) return;
    int err;
    int ri = ast_relation_for(db, ns, rel, &err);
    if (err) {
        scope_event(vs);
    } else {
        int has_rewrite = ri >= 0 && db->rels[ri].rewrite >= 0;
        int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;
        if (has_rewrite) mx_rewrite(c, ns, obj, db->rels[ri].rewrite, d, vs);
        if ((!db->strict || !has_rewrite) && !skip_direct && d - 1 <= 0) scope_trunc(vs);
        if (can_ss) mx_es(c, ns, obj, rel, d - 1, vs);
    }
    c->depth_guard--;
}

static uint32_t max_exploration_flags(rs_db *db, const rs_query *q) {
    rs_stats dummy = {0, 0, 0, 0};
    qctx c = {db, q->kind, q->sid, q->kind == 1 ? q->sns : 0, q->kind == 1 ? q->srel : 0, &dummy, 0, SCHED_EAGER, 0, 0};
    int d = q->depth;
    if (d <= 0 || db->max_depth < d) d = db->max_depth;
    mx_ia(&c, q->ns, q->obj, q->rel, d, 0, NULL);
    return c.flags & (RS_F_SENSITIVE | RS_F_MAXEXP);
}

int rs_check_ex(rs_db *db, const rs_query *q, int32_t *err, rs_stats *st, uint32_t *flags) {
    uint32_t f0 = 0, f1 = 0;
    int32_t e0 = 0, e1 = 0;
    const int m0 = check_sched(db, q, &e0, st, SCHED_EAGER, &f0);
    const int m1 = check_sched(db, q, &e1, NULL, SCHED_SEQUENTIAL, &f1);
    const int a0 = e0 == 0 && m0 == RS_IS_MEMBER, a1 = e1 == 0 && m1 == RS_IS_MEMBER;
    uint32_t f = ((f0 | f1) & RS_F_SENSITIVE) | max_exploration_flags(db, q);
    if (a0 != a1 || e0 != e1) f |= RS_F_SEQ_DIFFERS;
    if (err) *err = e0;
    if (flags) *flags = f;
    return m0;
}

/* ------------------------------------------------------------------ */
/* Frontier semantics: the spec of the product's frontier engine (csrc/frontier.hip)         */
/*
 * U = the recursion above evaluated WITHOUT visited pruning.  Each check is a goal; a goal
 * spawns every sub-check of its group unless a result known when the goal is expanded
 * already decides it (a shortcut IN hit, a found-lookahead hit, a direct tuple) or a known
 * leaf result ends the group in add order.  Groups still reduce in add order (first Err /
 * IsMember; AND: first non-IsMember), so U is a pure function of the snapshot.
 *
 * Claim: if every key that a visited scope of U's goal tree receives more than once has
 * only non-decisive occurrences (U-value NotMember / Unknown), the eager DFS above
 * (rs_check) returns U's result.  Its explored tree is a subtree of U's with the same
 * scopes, and it only ever prunes an ES child whose key the scope already holds, i.e. an
 * occurrence of a repeated key.  By induction from the leaves every check it evaluates has
 * its U-value: a pruned child is non-decisive in U, and dropping a non-decisive child does
 * not change a first-decisive reduction (pruning happens only in ES loops, which reduce that
 * way).  Queries with a decisive occurrence of a repeated key, or with more than `budget`
 * goals, are "routed": the product runs them on the DFS interpreter instead.  Goal counting
 * and spawn rules here are the engine's exactly, so routing flags compare one to one.
 */
typedef struct {
    uint64_t vk;
    uint32_t scope, used; /* used: occurrences of (scope, key) */
    uint32_t decisive;    /* some occurrence evaluated to IsMember / an error */
    uint32_t pad;
} upair;

typedef struct {
    qctx *c;
    upair *set;
    size_t cap, cnt;
    uint32_t goals, budget, scopes, maxgen;
    int routed;
} uctx;

#define U_NONE 0xFFFFFFFFu

/* insert (scope, key) or count another occurrence; returns its slot */
static size_t u_insert(uctx *u, uint32_t scope, uint64_t vk) {
    if (2 * (u->cnt + 1) > u->cap) {
        size_t nc = u->cap ? u->cap * 2 : 64;
        upair *ns = calloc(nc, sizeof *ns);
        for (size_t i = 0; i < u->cap; i++) {
            if (!u->set[i].used) continue;
            size_t h = mix64(u->set[i].vk ^ ((uint64_t)u->set[i].scope << 17)) & (nc - 1);
            while (ns[h].used) h = (h + 1) & (nc - 1);
            ns[h] = u->set[i];
        }
        free(u->set);
        u->set = ns;
        u->cap = nc;
    }
    size_t h = mix64(vk ^ ((uint64_t)scope << 17)) & (u->cap - 1);
    while (u->set[h].used) {
        if (u->set[h].vk == vk && u->set[h].scope == scope) {
            u->set[h].used++;
            return h;
        }
        h = (h + 1) & (u->cap - 1);
    }
    u->set[h].vk = vk;
    u->set[h].scope = scope;
    u->set[h].used = 1;
    u->cnt++;
    return h;
}

static size_t u_insert_find(uctx *u, uint32_t scope, uint64_t vk) {
    size_t h = mix64(vk ^ ((uint64_t)scope << 17)) & (u->cap - 1);
    while (!(u->set[h].vk == vk && u->set[h].scope == scope)) h = (h + 1) & (u->cap - 1);
    return h;
}

/* one more goal for this query; 0 once the budget is exceeded (the query is routed) */
static int u_spawn(uctx *u, uint32_t gen) {
    if (u->routed) return 0;
    if (++u->goals > u->budget) {
        u->routed = 1;
        return 0;
    }
    if (gen > u->maxgen) u->maxgen = gen;
    return 1;
}

static res u_ia(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip, uint32_t scope, uint32_t gen);
static res u_rw(uctx *u, uint32_t ns, uint32_t obj, int ai, int d, uint32_t scope, uint32_t gen);
static res u_es(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, uint32_t scope, uint32_t gen, int chain);

static int u_reach_prunes(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel);

/* a relation whose rows can hold subject sets: some tuple of (ns, rel) has one (per snapshot) */
static int has_set_rows(const rs_db *db, uint32_t ns, uint32_t rel) {
    return ns < db->n_ns && rel < db->n_relnames && db->ssrel[(size_t)ns * db->n_relnames + rel];
}

/* a node with at least one subject-set tuple (what an expand-subject of it reads) */
static int node_has_set_rows(const rs_db *db, uint32_t ns, uint32_t obj, uint32_t rel) {
    size_t lo, hi;
    node_rows(db, ns, obj, rel, &lo, &hi);
    for (size_t i = lo; i < hi; i++)
        if (ROW(db, i)->kind == 1) return 1;
    return 0;
}

/* A sub-check checkIsAllowed(ns:obj#rel, d, skip) shaped when its parent spawns it: a relation
 * with a rewrite is an IA goal; one without is decided on the spot (d <= 0: Unknown; an error;
 * a direct tuple: IsMember) or is just its expand-subject, an ES(d-1) goal -- or NotMember when
 * that could find no subject set: no row of the relation holds one, or, with node_check (an
 * ES's children and an OR's shortcut candidates, whose rows the engine knows at spawn), the
 * node's own row holds none.  An ES's children (es_child) are goals also for an error, so every
 * decisive occurrence of a scope key is a goal.  Returns 1 when spawned, 0 for a leaf; *out =
 * the result either way. */
static int u_sub(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip, int es_child, uint32_t scope,
                 uint32_t gen, res *out, int node_check) {
    const rs_db *db = u->c->db;
    *out = R_UNK;
    if (d <= 0) return 0; /* engine.go:215-220 */
    int err;
    const int ri = ast_relation_for(db, ns, rel, &err);
    const int has_rewrite = !err && ri >= 0 && db->rels[ri].rewrite >= 0;
    if (has_rewrite && !es_child) {
        /* u_ia below with neither a direct check nor an expand-subject to run is its rewrite's
         * result: an OR / AND rewrite never yields a bare Unknown (u_rw), so the group's
         * Unknown -> NotMember changes nothing.  Its RW goal is spawned in the IA's place. */
        const int can_ss_rw = !db->strict || db->rels[ri].has_ss_type;
        const int direct = !db->strict && !skip && d - 1 > 0 && exists(u->c, ns, obj, rel);
        const int es = can_ss_rw && d - 1 > 0 && has_set_rows(db, ns, rel);
        if (!direct && !es) {
            if (!u_spawn(u, gen + 1)) return 0;
            *out = u_rw(u, ns, obj, db->rels[ri].rewrite, d, scope, gen + 1);
            return 1;
        }
    }
    if (has_rewrite || (err && es_child)) {
        if (!u_spawn(u, gen + 1)) return 0;
        *out = u_ia(u, ns, obj, rel, d, skip, scope, gen + 1);
        return 1;
    }
    if (err) {
        out->err = err;
        return 0;
    }
    const int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;
    if (!skip && d - 1 > 0 && exists(u->c, ns, obj, rel)) {
        *out = R_IS;
        return 0;
    }
    if (can_ss && d - 1 > 0 && has_set_rows(db, ns, rel) && (!node_check || node_has_set_rows(db, ns, obj, rel))) {
        if (!u_spawn(u, gen + 1)) return 0;
        *out = u_es(u, ns, obj, rel, d - 1, scope, gen + 1, 1);
        return 1;
    }
    *out = R_NOT;
    return 0;
}

/* Reachability pruning (csrc/reach.hip; the engine's REACH_CAP).  Reach(n) = n and every node
 * reachable from it over subject-set rows.  A node n is "tabled" when its relation slot is pure
 * (no rewrite, no ASTRelationFor error), holds subject-set rows and is some tuple's subject-set
 * relation, every node of Reach(n) is pure, and |Reach(n)| <= reach_cap -- and the snapshot has no
 * aliased visited keys.  Then checkExpandSubject(n, d >= 1) can only be IsMember through a node of
 * Reach(n) \ {n} whose own row holds the subject: with none, it is NotMember whatever the visited
 * set and depth do (a pure node yields IsMember or NotMember, never an error or a bare Unknown,
 * at d > 1), and no key below n can be a decisive occurrence for this subject anywhere in the
 * query (each such node's own reach is inside Reach(n)), so no routing decision depends on
 * them.  The engine's expand-subject goal on such a node decides NotMember at once: no scope, no
 * children (u_es). */
static int rel_pure(const rs_db *db, uint32_t ns, uint32_t rel) {
    int err;
    const int ri = ast_relation_for(db, ns, rel, &err);
    return !err && (ri < 0 || db->rels[ri].rewrite < 0);
}
void rs_set_reach(rs_db *db, int on) { db->no_reach = !on; }
static int u_reach_prunes(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel) {
    const rs_db *db = u->c->db;
    if (db->no_reach || db->aliased || ns >= db->n_ns || rel >= db->n_relnames) return 0;
    const size_t nr = (size_t)ns * db->n_relnames + rel;
    if (!db->ssrel[nr] || !db->sstarget[nr] || !rel_pure(db, ns, rel)) return 0;
    uint32_t lst[REACH_CAP_MAX][3];
    uint32_t cnt = 1, head = 0;
    lst[0][0] = ns;
    lst[0][1] = obj;
    lst[0][2] = rel;
    while (head < cnt) {
        const uint32_t a = lst[head][0], o = lst[head][1], r = lst[head][2];
        head++;
        if (!rel_pure(db, a, r)) return 0;
        size_t lo, hi;
        node_rows(db, a, o, r, &lo, &hi);
        for (size_t i = lo; i < hi; i++) {
            const key7 *t = ROW(db, i);
            if (t->kind != 1) continue;
            int dup = 0;
            for (uint32_t k = 0; k < cnt && !dup; k++) dup = lst[k][0] == t->sns && lst[k][1] == t->sid && lst[k][2] == t->srel;
            if (dup) continue;
            if (cnt == db->reach_cap) return 0;
            lst[cnt][0] = t->sns;
            lst[cnt][1] = t->sid;
            lst[cnt][2] = t->srel;
            cnt++;
        }
    }
    for (uint32_t k = 1; k < cnt; k++) /* (n's own row: the expand-subject never reads it) */
        if (exists(u->c, lst[k][0], lst[k][1], lst[k][2])) return 0;
    return 1;
}

/* u_sub's shaping decision without evaluating anything: 1 when it would spawn a goal */
static int u_sub_spawns(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip, int es_child) {
    const rs_db *db = u->c->db;
    if (d <= 0) return 0;
    int err;
    const int ri = ast_relation_for(db, ns, rel, &err);
    const int has_rewrite = !err && ri >= 0 && db->rels[ri].rewrite >= 0;
    if (has_rewrite || (err && es_child)) return 1;
    if (err) return 0;
    const int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;
    if (!skip && d - 1 > 0 && exists(u->c, ns, obj, rel)) return 0;
    return can_ss && d - 1 > 0 && has_set_rows(db, ns, rel);
}

/* A NOT whose operand is decided where it is spawned -- a malformed NOT, a computed userset
 * that is a leaf, a rewrite at rest depth 0 -- is folded into its parent: u_inv evaluates it
 * there and no goal is spawned for it or below it. */
static int u_inv_folds(uctx *u, uint32_t ns, uint32_t obj, int ai, int d) {
    const rs_db *db = u->c->db;
    const rs_ast *a = &db->ast[ai];
    if (a->child_count != 1) return 1;
    const rs_ast *ch = &db->ast[db->children[a->child_begin]];
    if (ch->type == RS_CSS) return !u_sub_spawns(u, ns, obj, ch->rel, d, 0, 0);
    if (ch->type == RS_REWRITE) return d <= 0;
    return 0;
}

/* a rewrite child (check_child): 1 = spawned as a goal (result in *out), 0 = a leaf result */
static int u_child(uctx *u, uint32_t ns, uint32_t obj, int ci, int d, int cost, uint32_t scope, uint32_t gen,
                   res *out);

static res u_ttu(uctx *u, uint32_t ns, uint32_t obj, const rs_ast *a, int d, uint32_t scope, uint32_t gen) {
    const rs_db *db = u->c->db;
    size_t lo, hi;
    node_rows(db, ns, obj, a->rel, &lo, &hi);
    res out = R_NOT;
    int have = 0;
    if (d - 1 <= 0) return R_NOT; /* every parent check is Unknown (engine.go:215-220) */
    for (size_t i = lo; i < hi; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue;
        res r;
        const int spawned = u_sub(u, t->sns, t->sid, a->computed, d - 1, 0, 0, scope, gen, &r, 0);
        if (u->routed) return R_NOT;
        if (!have && decisive(r)) {
            out = r;
            have = 1;
        }
        if (!spawned && decisive(r)) break; /* later parents are never spawned */
    }
    return out;
}

static res u_inv(uctx *u, uint32_t ns, uint32_t obj, int ai, int d, uint32_t scope, uint32_t gen) {
    const rs_ast *a = &u->c->db->ast[ai];
    if (a->child_count != 1) {
        res r = {RS_UNKNOWN, RS_ERR_NOT_IMPLEMENTED};
        return r;
    }
    res r;
    u_child(u, ns, obj, u->c->db->children[a->child_begin], d, 0, scope, gen, &r);
    if (r.m == RS_IS_MEMBER) r.m = RS_NOT_MEMBER;
    else if (r.m == RS_NOT_MEMBER) r.m = RS_IS_MEMBER;
    return r;
}

static int u_child(uctx *u, uint32_t ns, uint32_t obj, int ci, int d, int cost, uint32_t scope, uint32_t gen,
                   res *out) {
    const rs_ast *ch = &u->c->db->ast[ci];
    *out = R_UNK;
    switch (ch->type) {
    case RS_TTU:
        if (d < 0 || !u_spawn(u, gen + 1)) return 0;
        *out = u_ttu(u, ns, obj, ch, d, scope, gen + 1);
        return 1;
    case RS_CSS:
        if (d < 0) return 0;
        return u_sub(u, ns, obj, ch->rel, d, 0, 0, scope, gen, out, 0);
    case RS_REWRITE:
        if (d - cost <= 0 || !u_spawn(u, gen + 1)) return 0;
        *out = u_rw(u, ns, obj, ci, d - cost, scope, gen + 1);
        return 1;
    case RS_INVERT:
        if (d < 0) return 0;
        if (u_inv_folds(u, ns, obj, ci, d)) {
            *out = u_inv(u, ns, obj, ci, d, scope, gen);
            return 0;
        }
        if (!u_spawn(u, gen + 1)) return 0;
        *out = u_inv(u, ns, obj, ci, d, scope, gen + 1);
        return 1;
    default:
        out->err = RS_ERR_NOT_IMPLEMENTED;
        return 0;
    }
}

/* fold one item of a group into its first-decisive result; a deciding leaf stops the group */
static void u_fold(res r, int spawned, int is_or, res *out, int *have, int *stop) {
    const int dec = is_or ? decisive(r) : (r.err || r.m != RS_IS_MEMBER);
    if (!*have && dec) {
        *out = r;
        if (!is_or) out->m = RS_NOT_MEMBER;
        *have = 1;
    }
    if (!spawned && dec) *stop = 1;
}

/* The items of an OR rewrite in add order -- its IN shortcut, the shortcut candidates, its other
 * children (rewrites.go:62-129) -- with nested OR rewrites spliced in: a nested OR's result is
 * the first decisive of its own items (NotMember if none), so the concatenation decides the same
 * group; it only contributes when its rest depth d-1 > 0 (rewrites.go:39-42).  No goal is
 * spawned for the nested OR itself. */
static int u_and_merge(uctx *u, uint32_t ns, uint32_t obj, int ai, int d);
static int u_flatten_off = -1; /* RS_NO_FLATTEN=1: the spine off (the engine built without it) */

/* The spine (csrc/frontier_goal.inc "spine"): the last item of an OR's walk is a
 * tuple-to-userset whose row holds exactly one subject set, and that parent's check would be a
 * RW goal spawned in its IA's place (u_sub) whose rewrite is an OR, or an AND that u_and_merge
 * takes.  Then the parent's items run in this goal, in place of that RW goal: they are the
 * walk's own tail.  A nested group's result only matters when decisive (first decisive in add
 * order), and an and_merge keeps a decisive result decisive (IsMember stays, an error stays), so
 * the flat walk picks the same first decisive result; only an error's membership bit can differ,
 * which no output reads.  Returns the inner OR's index and sets *dn (its rest depth), else -1. */
static int u_spine(uctx *u, const key7 *t, int computed, int d, int *dn) {
    const rs_db *db = u->c->db;
    if (u_flatten_off < 0) {
        const char *e = getenv("RS_NO_FLATTEN");
        u_flatten_off = e && e[0] == '1';
    }
    if (u_flatten_off || d <= 0) return -1;
    int err;
    const int ri = ast_relation_for(db, t->sns, computed, &err);
    if (err || ri < 0 || db->rels[ri].rewrite < 0) return -1;
    /* u_sub's "RW goal in the IA's place" path: no direct check and no expand-subject */
    const int can_ss_rw = !db->strict || db->rels[ri].has_ss_type;
    const int direct = !db->strict && d - 1 > 0 && exists(u->c, t->sns, t->sid, computed);
    const int es = can_ss_rw && d - 1 > 0 && has_set_rows(db, t->sns, computed);
    if (direct || es) return -1;
    const int rw = db->rels[ri].rewrite;
    const rs_ast *a = &db->ast[rw];
    if (a->type != RS_REWRITE) return -1;
    if (a->op == RS_OP_OR) {
        *dn = d;
        return rw;
    }
    const int orc = u_and_merge(u, t->sns, t->sid, rw, d);
    if (orc < 0) return -1;
    *dn = d - 1;
    return orc;
}

static void u_or_items(uctx *u, uint32_t ns, uint32_t obj, int ai, int d, uint32_t scope, uint32_t gen, res *out,
                       int *have, int *stop, int last) {
    const rs_db *db = u->c->db;
    const rs_ast *a = &db->ast[ai];
    int lastnc = -1; /* the last non-CSS child: the walk's last item when `last` */
    for (int k = 0; k < a->child_count; k++)
        if (db->ast[db->children[a->child_begin + k]].type != RS_CSS) lastnc = k;
    int has_css = 0, found = 0;
    for (int k = 0; k < a->child_count; k++) {
        const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
        if (ch->type != RS_CSS) continue;
        has_css = 1;
        int err;
        int ri = ast_relation_for(db, ns, ch->rel, &err);
        if (db->strict && ri >= 0 && db->rels[ri].rewrite >= 0) continue;
        if (!found && exists(u->c, ns, obj, ch->rel)) found = 1;
    }
    if (found) {
        u_fold(R_IS, 0, 1, out, have, stop);
        return;
    }
    if (has_css && d - 1 > 0)
        for (int k = 0; k < a->child_count && !*stop; k++) {
            const rs_ast *ch = &db->ast[db->children[a->child_begin + k]];
            if (ch->type != RS_CSS) continue;
            res r;
            const int spawned = u_sub(u, ns, obj, ch->rel, d - 1, 1, 0, scope, gen, &r, 1);
            if (u->routed) return;
            u_fold(r, spawned, 1, out, have, stop);
        }
    for (int k = 0; k < a->child_count && !*stop; k++) {
        int ci = db->children[a->child_begin + k];
        const rs_ast *ch = &db->ast[ci];
        if (ch->type == RS_CSS) continue;
        if (ch->type == RS_REWRITE && ch->op == RS_OP_OR) { /* restDepth-1 (:118) */
            if (d - 1 > 0) u_or_items(u, ns, obj, ci, d - 1, scope, gen, out, have, stop, last && k == lastnc);
            if (u->routed) return;
            continue;
        }
        if (ch->type == RS_TTU) {
            /* spliced like a nested OR: a tuple-to-userset's result is the first decisive of
             * its parents' checks in row order (u_ttu), so the parents are this OR's own items;
             * with d - 1 <= 0 every parent check is Unknown and contributes nothing */
            if (d - 1 <= 0) continue;
            size_t lo, hi;
            node_rows(db, ns, obj, ch->rel, &lo, &hi);
            if (last && k == lastnc) {
                const key7 *one = NULL;
                int n1 = 0;
                for (size_t i = lo; i < hi; i++)
                    if (ROW(db, i)->kind == 1) {
                        one = ROW(db, i);
                        n1++;
                    }
                int dn = 0;
                const int inner = n1 == 1 ? u_spine(u, one, ch->computed, d - 1, &dn) : -1;
                if (inner >= 0) { /* the parent's items: this walk's tail (no goal for its RW) */
                    u_or_items(u, one->sns, one->sid, inner, dn, scope, gen, out, have, stop, 1);
                    continue;
                }
            }
            for (size_t i = lo; i < hi && !*stop; i++) {
                const key7 *t = ROW(db, i);
                if (t->kind != 1) continue;
                res r;
                const int spawned = u_sub(u, t->sns, t->sid, ch->computed, d - 1, 0, 0, scope, gen, &r, 0);
                if (u->routed) return;
                u_fold(r, spawned, 1, out, have, stop);
            }
            continue;
        }
        res r;
        const int spawned = u_child(u, ns, obj, ci, d, 1, scope, gen, &r);
        if (u->routed) return;
        u_fold(r, spawned, 1, out, have, stop);
    }
}

/* An AND at rest depth d > 1 whose children are one nested OR (a goal at d-1, rewrites.go:118)
 * and leaves that are all IsMember without an error: the OR's index, else -1.  Such an AND is
 * its OR mapped through AND -- a non-member (errors kept) becomes NotMember -- so its goal runs
 * the OR's items itself and no goal is spawned for the OR (csrc/frontier.hip and_merge). */
static int u_and_merge(uctx *u, uint32_t ns, uint32_t obj, int ai, int d) {
    const rs_db *db = u->c->db;
    const rs_ast *a = &db->ast[ai];
    if (a->op != RS_OP_AND || d <= 1) return -1;
    int orc = -1;
    for (int k = 0; k < a->child_count; k++) {
        const int ci = db->children[a->child_begin + k];
        const rs_ast *ch = &db->ast[ci];
        if (ch->type == RS_REWRITE) {
            if (orc >= 0 || ch->op != RS_OP_OR) return -1;
            orc = ci;
        } else if (ch->type == RS_CSS) {
            if (u_sub_spawns(u, ns, obj, ch->rel, d, 0, 0)) return -1;
            int err;
            (void)ast_relation_for(db, ns, ch->rel, &err);
            if (err || !(d - 1 > 0 && exists(u->c, ns, obj, ch->rel))) return -1; /* not a direct IsMember */
        } else if (ch->type == RS_INVERT) {
            if (!u_inv_folds(u, ns, obj, ci, d)) return -1;
            const res r = u_inv(u, ns, obj, ci, d, U_NONE, 0);
            if (r.err || r.m != RS_IS_MEMBER) return -1;
        } else {
            return -1; /* a tuple-to-userset is always a goal */
        }
    }
    return orc;
}

static res u_rw(uctx *u, uint32_t ns, uint32_t obj, int ai, int d, uint32_t scope, uint32_t gen) {
    const rs_db *db = u->c->db;
    const rs_ast *a = &db->ast[ai];
    if (a->op != RS_OP_OR && a->op != RS_OP_AND) {
        res r = {RS_UNKNOWN, RS_ERR_NOT_IMPLEMENTED};
        return r;
    }
    res out = R_NOT;
    int have = 0; /* the group's result is fixed (by a child in add order) */
    int stop = 0; /* a leaf decided it: later children are never spawned */
    const int orc = u_and_merge(u, ns, obj, ai, d);
    if (orc >= 0) {
        u_or_items(u, ns, obj, orc, d - 1, scope, gen, &out, &have, &stop, 1);
        if (u->routed) return R_NOT;
        res x = have ? out : R_NOT;
        if (x.err || x.m != RS_IS_MEMBER) x.m = RS_NOT_MEMBER;
        return x;
    }
    if (a->op == RS_OP_OR) {
        u_or_items(u, ns, obj, ai, d, scope, gen, &out, &have, &stop, 1);
        if (u->routed) return R_NOT;
        return have ? out : R_NOT;
    }
    for (int k = 0; k < a->child_count && !stop; k++) {
        int ci = db->children[a->child_begin + k];
        res r;
        const int spawned = u_child(u, ns, obj, ci, d, 1, scope, gen, &r);
        if (u->routed) return R_NOT;
        u_fold(r, spawned, 0, &out, &have, &stop);
    }
    if (!have) out = a->child_count > 0 ? R_IS : R_NOT;
    return out;
}

/* would u_sub(ns:obj#rel, d, skipDirect, es_child, node_check) spawn an ES goal (not an IA
 * goal, not a leaf)? */
static int u_es_child_is_es(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d) {
    const rs_db *db = u->c->db;
    if (d <= 0) return 0;
    int err;
    const int ri = ast_relation_for(db, ns, rel, &err);
    if (err || (ri >= 0 && db->rels[ri].rewrite >= 0)) return 0; /* an IA goal */
    const int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;
    return can_ss && d - 1 > 0 && has_set_rows(db, ns, rel) && node_has_set_rows(db, ns, obj, rel);
}

/* chain: an expand-subject whose row holds exactly one subject set, kept, that would be an ES
 * goal runs that child's expand-subject itself (one step; the child's own children are goals
 * as usual): the child's key is still an occurrence of the scope, its children are this goal's,
 * one generation earlier, and no goal is spawned for it.  Its result is the child's: the first
 * decisive of a one-child group is that child's result when decisive, else NotMember.
 * (csrc/frontier.hip G_ES "chain") */
static res u_es(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, uint32_t scope, uint32_t gen, int chain) {
    const rs_db *db = u->c->db;
    /* a goal of its own (chain: not the chained child run inside its parent's goal): the reach */
    if (chain && node_has_set_rows(db, ns, obj, rel) && u_reach_prunes(u, ns, obj, rel)) return R_NOT;
    size_t lo, hi;
    node_rows(db, ns, obj, rel, &lo, &hi);
    size_t nres = 0;
    const key7 *only = NULL;
    for (size_t i = lo; i < hi; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue;
        nres++;
        only = t;
        if (exists(u->c, t->sns, t->sid, t->srel)) return R_IS;
    }
    size_t keep = nres;
    if ((long)nres > (long)db->max_width) keep = db->max_width > 0 ? (size_t)(db->max_width - 1) : 0;
    if (scope == U_NONE) scope = u->scopes++;
    if (chain && nres == 1 && keep == 1 && u_es_child_is_es(u, only->sns, only->sid, only->srel, d)) {
        const uint64_t vk = vkey(db, only->sns, only->sid, only->srel);
        u_insert(u, scope, vk);
        const res r = u_es(u, only->sns, only->sid, only->srel, d - 1, scope, gen, 0);
        if (u->routed) return R_NOT;
        if (decisive(r)) u->set[u_insert_find(u, scope, vk)].decisive = 1;
        return decisive(r) ? r : R_NOT;
    }
    res out = R_NOT;
    int have = 0;
    for (size_t i = lo; i < hi && keep; i++) {
        const key7 *t = ROW(db, i);
        if (t->kind != 1) continue;
        keep--;
        const uint64_t vk = vkey(db, t->sns, t->sid, t->srel);
        u_insert(u, scope, vk);
        res r;
        /* checkIsAllowed(c, d, skipDirect) (engine.go:161); its leaves are never decisive */
        const int spawned = u_sub(u, t->sns, t->sid, t->srel, d, 1, 1, scope, gen, &r, 1);
        if (u->routed) return R_NOT;
        if (spawned && decisive(r)) u->set[u_insert_find(u, scope, vk)].decisive = 1; /* the table may have grown */
        if (!have && decisive(r)) {
            out = r;
            have = 1;
        }
    }
    return out;
}

static res u_ia(uctx *u, uint32_t ns, uint32_t obj, uint32_t rel, int d, int skip, uint32_t scope, uint32_t gen) {
    if (d <= 0) return R_UNK;
    const rs_db *db = u->c->db;
    int err;
    int ri = ast_relation_for(db, ns, rel, &err);
    if (err) {
        res r = {RS_UNKNOWN, err};
        return r;
    }
    const int has_rewrite = ri >= 0 && db->rels[ri].rewrite >= 0;
    const int can_ss = !db->strict || ri < 0 || db->rels[ri].has_ss_type;
    res rr = R_NOT, er = R_NOT;
    if (has_rewrite && u_spawn(u, gen + 1)) rr = u_rw(u, ns, obj, db->rels[ri].rewrite, d, scope, gen + 1);
    const int direct_is = (!db->strict || !has_rewrite) && !skip && d - 1 > 0 && exists(u->c, ns, obj, rel);
    if (can_ss && !direct_is && d - 1 > 0 && has_set_rows(db, ns, rel) && u_spawn(u, gen + 1))
        er = u_es(u, ns, obj, rel, d - 1, scope, gen + 1, 1);
    if (decisive(rr)) return rr;
    if (direct_is) return R_IS;
    if (decisive(er)) return er;
    return R_NOT;
}

static int rs_root_ia(void) { /* RS_IA_ROOT=1: roots as IA goals (an engine built with KETO_FR_IAROOT) */
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("RS_IA_ROOT");
        v = e && *e == '1';
    }
    return v;
}

int rs_check_u(rs_db *db, const rs_query *q, uint32_t budget, int32_t *err, uint32_t *routed, uint32_t *goals,
               uint32_t *gens) {
    rs_stats dummy = {0, 0, 0, 0};
    qctx c = {db, q->kind, q->sid, q->kind == 1 ? q->sns : 0, q->kind == 1 ? q->srel : 0, &dummy, 0, SCHED_EAGER, 0, 0};
    uctx u;
    memset(&u, 0, sizeof u);
    u.c = &c;
    u.budget = budget;
    int d = q->depth;
    if (d <= 0 || db->max_depth < d) d = db->max_depth; /* engine.go:82-84 */
    res r = R_NOT;
    if (u_spawn(&u, 0)) {
        /* the root shaped as u_sub shapes a sub-check (csrc/frontier_goal.inc root_word): a
         * rewrite with neither a direct check nor an expand-subject to run is its RW goal */
        int err;
        const int ri = ast_relation_for(db, q->ns, q->rel, &err);
        int rw_root = 0;
        if (!err && ri >= 0 && db->rels[ri].rewrite >= 0 && d >= 1 && !rs_root_ia()) {
            const int can_ss_rw = !db->strict || db->rels[ri].has_ss_type;
            const int direct = !db->strict && d - 1 > 0 && exists(&c, q->ns, q->obj, q->rel);
            const int es = can_ss_rw && d - 1 > 0 && has_set_rows(db, q->ns, q->rel);
            rw_root = !direct && !es;
        }
        r = rw_root ? u_rw(&u, q->ns, q->obj, db->rels[ri].rewrite, d, U_NONE, 0) : u_ia(&u, q->ns, q->obj, q->rel, d, 0, U_NONE, 0);
    }
    for (size_t i = 0; i < u.cap; i++)
        if (u.set[i].used > 1 && u.set[i].decisive) u.routed = 1;
    free(u.set);
    if (err) *err = r.err;
    if (routed) *routed = (uint32_t)u.routed;
    if (goals) *goals = u.goals;
    if (gens) *gens = u.maxgen + 1;
    return r.m;
}

typedef struct {
    rs_db *db;
    const rs_query *q;
    size_t n;
    uint32_t budget;
    uint8_t *decision;
    int32_t *err;
    uint32_t *routed, *goals, *gens;
    atomic_size_t next;
} ubatch_job;

static void *ubatch_worker(void *arg) {
    ubatch_job *j = arg;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 64);
        if (i >= j->n) break;
        size_t e = i + 64 < j->n ? i + 64 : j->n;
        for (; i < e; i++) {
            int32_t er = 0;
            int m = rs_check_u(j->db, &j->q[i], j->budget, &er, &j->routed[i], &j->goals[i], &j->gens[i]);
            j->decision[i] = (er == 0 && m == RS_IS_MEMBER);
            j->err[i] = er;
        }
    }
    return NULL;
}

void rs_check_u_batch(rs_db *db, const rs_query *q, size_t n, int threads, uint32_t budget, uint8_t *decision,
                      int32_t *err, uint32_t *routed, uint32_t *goals, uint32_t *gens) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    ubatch_job j;
    j.db = db;
    j.q = q;
    j.n = n;
    j.budget = budget;
    j.decision = decision;
    j.err = err;
    j.routed = routed;
    j.goals = goals;
    j.gens = gens;
    atomic_init(&j.next, 0);
    pthread_t th[256];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, ubatch_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
}

/* ------------------------------------------------------------------ */
/* batch (CPU baseline)                                                  */

typedef struct {
    rs_db *db;
    const rs_query *q;
    size_t n;
    uint8_t *decision;
    int32_t *err;
    uint32_t *flags; /* NULL: canonical schedule only */
    atomic_size_t next;
    pthread_mutex_t mu;
    rs_stats total;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = arg;
    rs_stats st = {0, 0, 0, 0};
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 64);
        if (i >= j->n) break;
        size_t e = i + 64 < j->n ? i + 64 : j->n;
        for (; i < e; i++) {
            int32_t er = 0;
            int m = j->flags ? rs_check_ex(j->db, &j->q[i], &er, &st, &j->flags[i]) : rs_check(j->db, &j->q[i], &er, &st);
            j->decision[i] = (er == 0 && m == RS_IS_MEMBER); /* engine.go:65-71 */
            j->err[i] = er;
        }
    }
    pthread_mutex_lock(&j->mu);
    j->total.rows += st.rows;
    j->total.edges += st.edges;
    j->total.probes += st.probes;
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

void rs_check_batch(rs_db *db, const rs_query *q, size_t n, int threads, uint8_t *decision,
                    int32_t *err, rs_stats *st) {
    rs_check_batch_ex(db, q, n, threads, decision, err, NULL, st);
}

void rs_check_batch_ex(rs_db *db, const rs_query *q, size_t n, int threads, uint8_t *decision,
                       int32_t *err, uint32_t *flags, rs_stats *st) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    batch_job j;
    j.db = db;
    j.q = q;
    j.n = n;
    j.decision = decision;
    j.err = err;
    j.flags = flags;
    atomic_init(&j.next, 0);
    pthread_mutex_init(&j.mu, NULL);
    memset(&j.total, 0, sizeof j.total);
    pthread_t th[256];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, batch_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j.mu);
    if (st) {
        st->rows += j.total.rows;
        st->edges += j.total.edges;
        st->probes += j.total.probes;
    }
}

/* ------------------------------------------------------------------ */
/* closure (bench helper for the SQL-mode baseline, oracle/refsql.py): every row of every    */
/* object within `levels` subject-set hops of the given objects, in index order (so rows of */
/* one (ns, obj, rel) keep their shard order; `pos` is the row's rank in it)                 */

static void obj_rows(const rs_db *db, uint32_t ns, uint32_t obj, size_t *lo, size_t *hi) {
    size_t a = 0, b = db->n;
    while (a < b) {
        size_t m = (a + b) / 2;
        const key7 *t = &db->rt[m];
        if (t->ns < ns || (t->ns == ns && t->obj < obj)) a = m + 1;
        else b = m;
    }
    *lo = a;
    b = db->n;
    while (a < b) {
        size_t m = (a + b) / 2;
        const key7 *t = &db->rt[m];
        if (t->ns < ns || (t->ns == ns && t->obj <= obj)) a = m + 1;
        else b = m;
    }
    *hi = a;
}

size_t rs_closure(rs_db *db, const uint32_t *ns, const uint32_t *obj, size_t n, int levels, rs_row *out, size_t cap) {
    vset *seen = vset_new();
    size_t fcap = n ? n : 1, fn = 0, total = 0;
    uint64_t *front = malloc(fcap * sizeof *front);
    for (size_t i = 0; i < n; i++) front[fn++] = ((uint64_t)ns[i] << 32) | obj[i];
    for (int level = 0; level < levels && fn; level++) {
        size_t ncap = 16, nn = 0;
        uint64_t *next = malloc(ncap * sizeof *next);
        for (size_t i = 0; i < fn; i++) {
            if (vset_add(seen, front[i])) continue;
            size_t lo, hi;
            obj_rows(db, (uint32_t)(front[i] >> 32), (uint32_t)front[i], &lo, &hi);
            for (size_t j = lo; j < hi; j++) {
                const key7 *t = &db->rt[j];
                if (total < cap) {
                    rs_row r = {t->ns, t->obj, t->rel, t->kind, t->sid, t->sns, t->srel, 0, (uint64_t)j};
                    out[total] = r;
                }
                total++;
                if (t->kind == 1) {
                    if (nn == ncap) next = realloc(next, (ncap *= 2) * sizeof *next);
                    next[nn++] = ((uint64_t)t->sns << 32) | t->sid;
                }
            }
        }
        free(front);
        front = next;
        fn = nn;
    }
    free(front);
    vset_free(seen);
    return total;
}

/* ------------------------------------------------------------------ */
/* Expand (internal/expand/engine.go:43-124)                            */

typedef struct {
    const rs_db *db;
    rs_tree_node *out;
    size_t cap, len;
    int overflow;
    vset *vs;
    rs_stats *st;
} xctx;

static void emit(xctx *x, uint32_t type, uint32_t kind, uint32_t sid, uint32_t sns, uint32_t srel) {
    if (x->len >= x->cap) {
        x->overflow = 1;
        x->len++;
        return;
    }
    rs_tree_node *n = &x->out[x->len++];
    n->type = type;
    n->kind = kind;
    n->sid = sid;
    n->sns = kind ? sns : 0;
    n->srel = kind ? srel : 0;
    n->n_children = 0;
}

/* returns 1 if a node was written, 0 for nil */
static int build_tree(xctx *x, uint32_t kind, uint32_t sid, uint32_t sns, uint32_t srel, int d) {
    const rs_db *db = x->db;
    if (d <= 0 || db->max_depth < d) d = db->max_depth; /* :56-58 */
    if (kind == 0) {                                     /* :60-67 */
        emit(x, 4, 0, sid, 0, 0);
        x->st->out_nodes++;
        return 1;
    }
    if (vset_add(x->vs, vkey(db, sns, sid, srel))) return 0; /* :69-72 (root included) */
    size_t lo, hi;
    node_rows(db, sns, sid, srel, &lo, &hi);
    x->st->rows++;
    if (lo == hi) return 0; /* :97-99 */
    size_t me = x->len;
    if (d <= 1) { /* :101-104 */
        emit(x, 4, 1, sid, sns, srel);
        x->st->out_nodes++;
        return 1;
    }
    emit(x, 1, 1, sid, sns, srel);
    x->st->out_nodes++;
    for (size_t i = lo; i < hi; i++) { /* :106-119 */
        const key7 *t = ROW(db, i);
        x->st->edges++;
        if (!build_tree(x, t->kind, t->sid, t->sns, t->srel, d - 1)) {
            emit(x, 4, t->kind, t->sid, t->sns, t->srel); /* nil child -> leaf (:112-117) */
            x->st->out_nodes++;
        }
        if (me < x->cap) x->out[me].n_children++;
    }
    return 1;
}

long rs_expand(rs_db *db, uint32_t kind, uint32_t sid, uint32_t sns, uint32_t srel, int32_t depth,
               rs_tree_node *out, size_t cap, rs_stats *st) {
    rs_stats dummy = {0, 0, 0, 0};
    xctx x = {db, out, cap, 0, 0, vset_new(), st ? st : &dummy};
    int wrote = build_tree(&x, kind, sid, sns, srel, depth);
    vset_free(x.vs);
    if (x.overflow) return -1;
    return wrote ? (long)x.len : 0;
}
