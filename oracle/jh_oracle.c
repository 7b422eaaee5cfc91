/*
 * jh_oracle.c -- TEST INFRASTRUCTURE ONLY (see jh_oracle.h).
 *
 * Plain-C restatement of the reference verification path. Every function
 * cites the reference file:line it follows. knossos 0.3.4 (the home of WGL,
 * cas-register and history/complete; jepsen/project.clj:13) is not vendored
 * in /root/reference: its semantics are restated from
 *   - the call sites  jepsen/src/jepsen/checker.clj:17-23,141-145,699
 *   - the in-tree copy of complete-fold-op  cassandra/src/cassandra/checker.clj:7-62
 *   - the CASRegister text  doc/tutorial/04-checker.md:58-72
 *   - the known answers in jepsen/test/jepsen/{perf,checker,independent,util}_test.clj
 * and from the published Wing-Gong / Lowe algorithm (G. Lowe, "Testing for
 * linearizability", CCPE 2017), which knossos.wgl implements.
 */
#define _GNU_SOURCE
#include "jh_oracle.h"
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

#define ORC_CRASHED INT64_MAX

/* ------------------------------------------------------------------------ */
/* int64 -> int64 open-addressing map (process -> open invocation).          */
typedef struct { int64_t *k, *v; uint8_t *used; int64_t cap, n; } imap;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}
static void imap_init(imap *m, int64_t cap) {
    int64_t c = 16; while (c < 2 * cap) c <<= 1;
    m->cap = c; m->n = 0;
    m->k = (int64_t *)malloc(sizeof(int64_t) * c);
    m->v = (int64_t *)malloc(sizeof(int64_t) * c);
    m->used = (uint8_t *)calloc(c, 1);
}
static void imap_free(imap *m) { free(m->k); free(m->v); free(m->used); }
/* Tombstone-free deletion by backward-shift keeps probe chains exact. */
static int64_t imap_find(const imap *m, int64_t key) {
    uint64_t i = mix64((uint64_t)key) & (m->cap - 1);
    while (m->used[i]) {
        if (m->k[i] == key) return (int64_t)i;
        i = (i + 1) & (m->cap - 1);
    }
    return -1;
}
static void imap_grow(imap *m);
static void imap_put(imap *m, int64_t key, int64_t val) {
    if (2 * (m->n + 1) > m->cap) imap_grow(m);
    uint64_t i = mix64((uint64_t)key) & (m->cap - 1);
    while (m->used[i]) {
        if (m->k[i] == key) { m->v[i] = val; return; }
        i = (i + 1) & (m->cap - 1);
    }
    m->used[i] = 1; m->k[i] = key; m->v[i] = val; m->n++;
}
static void imap_grow(imap *m) {
    imap o = *m; imap_init(m, o.cap);
    for (int64_t i = 0; i < o.cap; i++) if (o.used[i]) imap_put(m, o.k[i], o.v[i]);
    imap_free(&o);
}
static void imap_del(imap *m, int64_t slot) {
    uint64_t i = (uint64_t)slot, mask = (uint64_t)m->cap - 1;
    m->used[i] = 0; m->n--;
    uint64_t j = i;
    for (;;) {
        j = (j + 1) & mask;
        if (!m->used[j]) break;
        uint64_t h = mix64((uint64_t)m->k[j]) & mask;
        /* can the entry at j move to the hole at i? */
        if ((j > i && (h <= i || h > j)) || (j < i && (h <= i && h > j))) {
            m->k[i] = m->k[j]; m->v[i] = m->v[j]; m->used[i] = 1; m->used[j] = 0; i = j;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* knossos.model/cas-register step (doc/tutorial/04-checker.md:58-72):
 *   :write v      -> v
 *   :cas [cur new]-> new if cur = state, else inconsistent
 *   :read v       -> state if v is nil or v = state, else inconsistent     */
static inline int cas_step(int32_t f, int64_t v1, int64_t v2, int64_t s, int64_t *out) {
    switch (f) {
    case JH_F_WRITE: *out = v1; return 1;
    case JH_F_CAS:   if (s == v1) { *out = v2; return 1; } return 0;
    case JH_F_READ:  if (v1 == JH_NIL || v1 == s) { *out = s; return 1; } return 0;
    default: return 0;
    }
}

/* ------------------------------------------------------------------------ */
/* Key preparation = knossos.history/complete (complete-fold-op, restated from
 * cassandra/src/cassandra/checker.clj:7-62 and pinned by the :fails? effect
 * in jepsen/test/jepsen/checker_test.clj:107-116), then the op list the WGL
 * search walks.
 *   :invoke  while the process is open -> throws (checker.clj:77-88 makes
 *            that :unknown)                          cassandra/checker.clj:14-20
 *   :ok      invocation :value := (or inv-value ok-value); closes  :25-34
 *   :fail    invocation gets :fails? (dropped from the search); closes
 *   :info    no change; the process stays open (crashed op)     :52-54
 * Entries whose :process is not an integer (nemesis) are dropped: subhistory
 * keeps them in every key (independent.clj:243) and they are not ops.
 * Sound reductions shared with libjh.so (they change no verdict): a crashed
 * :read never changes the register so it is never linearized; an :ok :read
 * of nil is legal in every state (04-checker.md:66-67) and changes nothing,
 * so it can always be placed at its own return. Both are dropped.          */
static int cmp_ret(const void *a, const void *b, void *ctx) {
    const orc_op *ops = (const orc_op *)ctx;
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return ops[x].ret < ops[y].ret ? -1 : ops[x].ret > ops[y].ret;
}

int orc_key_prepare(const jh_history *h, const int64_t *sel, int64_t m, orc_key *k) {
    memset(k, 0, sizeof(*k));
    int64_t *pair = (int64_t *)malloc(sizeof(int64_t) * (m ? m : 1));
    for (int64_t j = 0; j < m; j++) pair[j] = -1;
    imap open; imap_init(&open, 64);
    int status = JH_CAUSE_NONE;
    for (int64_t j = 0; j < m && !status; j++) {
        int64_t r = sel[j], p = h->process[r];
        if (p < 0) continue;
        int64_t ty = h->type[r];
        int64_t slot = imap_find(&open, p);
        if (ty == JH_TYPE_INVOKE) {
            if (slot >= 0) status = JH_CAUSE_DOUBLE_INVOKE;
            else imap_put(&open, p, j);
        } else if (ty == JH_TYPE_OK || ty == JH_TYPE_FAIL) {
            if (slot < 0) { status = JH_CAUSE_ORPHAN; break; }
            int64_t i = open.v[slot];
            pair[i] = j; pair[j] = i;
            imap_del(&open, slot);
        }
    }
    imap_free(&open);
    if (status) { free(pair); k->status = status; return 0; }

    k->ops = (orc_op *)malloc(sizeof(orc_op) * (m ? m : 1));
    int32_t n = 0;
    for (int64_t j = 0; j < m; j++) {
        int64_t r = sel[j];
        if (h->process[r] < 0 || h->type[r] != JH_TYPE_INVOKE) continue;
        int64_t c = pair[j];
        if (c >= 0 && h->type[sel[c]] == JH_TYPE_FAIL) continue;      /* :fails? */
        int32_t f = (int32_t)h->f[r];
        int64_t v1 = h->value[r], v2 = h->value2[r], ret = ORC_CRASHED;
        if (c >= 0) {
            int64_t rc = sel[c];
            ret = rc;
            if (f == JH_F_CAS) {
                if (v1 == JH_NIL && v2 == JH_NIL) { v1 = h->value[rc]; v2 = h->value2[rc]; }
            } else if (v1 == JH_NIL) v1 = h->value[rc];
        }
        if (f != JH_F_READ && f != JH_F_WRITE && f != JH_F_CAS) { status = JH_CAUSE_BAD_F; break; }
        if (f == JH_F_READ && (ret == ORC_CRASHED || v1 == JH_NIL)) {
            if (!k->noop_call) {
                k->noop_call = (int64_t *)malloc(sizeof(int64_t) * (m ? m : 1));
                k->noop_ret = (int64_t *)malloc(sizeof(int64_t) * (m ? m : 1));
            }
            k->noop_call[k->n_noop] = r; k->noop_ret[k->n_noop++] = ret;
            continue;
        }
        orc_op *o = &k->ops[n++];
        o->call = r; o->ret = ret; o->f = f; o->v1 = v1; o->v2 = v2; o->rr = -1;
    }
    free(pair);
    k->n_ops = n;
    if (status) { k->status = status; return 0; }

    /* ok ops ordered by return row */
    int32_t n_ok = 0;
    k->ret_op = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; i++) if (k->ops[i].ret != ORC_CRASHED) k->ret_op[n_ok++] = i;
    qsort_r(k->ret_op, n_ok, sizeof(int32_t), cmp_ret, k->ops);
    for (int32_t t = 0; t < n_ok; t++) k->ops[k->ret_op[t]].rr = t;
    k->n_ok = n_ok;

    /* Windows. W(t) = ops called before the t-th ok return that are still
     * un-returned there (crashed ops stay forever), in call order. Every op
     * returning before it is linearized in any configuration with R = t, every
     * op called after it is not: (t, mask over W(t), state) is a bijective
     * image of knossos' (linearized BitSet, model) cache key.               */
    int64_t cap = 64, used = 0;
    k->w_off = (int32_t *)malloc(sizeof(int32_t) * (n_ok + 1));
    k->w_ops = (int32_t *)malloc(sizeof(int32_t) * cap);
    int32_t *act = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t na = 0, nxt = 0, maxw = 0;
    for (int32_t t = 0; t < n_ok; t++) {
        int64_t R = k->ops[k->ret_op[t]].ret;
        while (nxt < n && k->ops[nxt].call < R) act[na++] = nxt++;
        int32_t w = 0;
        for (int32_t i = 0; i < na; i++) {
            const orc_op *o = &k->ops[act[i]];
            if (o->rr >= 0 && o->rr < t) continue;
            act[w++] = act[i];
        }
        na = w;
        if (na > maxw) maxw = na;
        if (used + na > cap) {
            while (used + na > cap) cap *= 2;
            k->w_ops = (int32_t *)realloc(k->w_ops, sizeof(int32_t) * cap);
        }
        k->w_off[t] = (int32_t)used;
        memcpy(k->w_ops + used, act, sizeof(int32_t) * na);
        used += na;
    }
    k->w_off[n_ok] = (int32_t)used;
    free(act);
    k->max_window = maxw;
    if (orc_reduce_crashed) {
        k->pred = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
        for (int32_t i = 0; i < n; i++) {
            k->pred[i] = -1;
            if (k->ops[i].ret != ORC_CRASHED) continue;
            for (int32_t j = i - 1; j >= 0; j--)
                if (k->ops[j].ret == ORC_CRASHED && k->ops[j].f == k->ops[i].f && k->ops[j].v1 == k->ops[i].v1 &&
                    k->ops[j].v2 == k->ops[i].v2) { k->pred[i] = j; break; }
        }
    }
    if (maxw > JH_MAX_WINDOW) k->status = JH_CAUSE_WINDOW;
    return 0;
}

int orc_reduce_crashed = 0;

/* the crashed-op symmetry: window member i of W (mask over it) may be lifted
 * only if its class predecessor is linearized (it is in the window: crashed
 * ops never leave, and it was invoked earlier, so it sits at a lower position) */
static int sym_blocked(const orc_key *k, const int32_t *W, const uint64_t *mask, int i) {
    if (!k->pred) return 0;
    const int32_t p = k->pred[W[i]];
    if (p < 0) return 0;
    for (int j = i - 1; j >= 0; j--)
        if (W[j] == p) return !((mask[j >> 6] >> (j & 63)) & 1);
    return 0;
}

void orc_key_free(orc_key *k) {
    free(k->ops); free(k->ret_op); free(k->w_off); free(k->w_ops); free(k->pred);
    free(k->noop_call); free(k->noop_ret);
    memset(k, 0, sizeof(*k));
}

/* ------------------------------------------------------------------------ */
/* Memo set of canonical configurations (t, state, mask). The mask is over
 * the window W(t), at most JH_MAX_WINDOW = 256 members: MW 64-bit words.   */
#define MW (JH_MAX_WINDOW / 64)
typedef struct { uint32_t t; int64_t s; uint64_t m[MW]; } cfg;
typedef struct { cfg *e; uint8_t *used; int64_t cap, n; } cset;
static uint64_t cfg_hash(const cfg *c) {
    uint64_t h = mix64((uint64_t)c->s + ((uint64_t)c->t << 40));
    for (int w = 0; w < MW; w++) h = mix64(h ^ c->m[w] * 0x9E3779B97F4A7C15ULL) + (uint64_t)w;
    return h;
}
static int cfg_eq(const cfg *a, const cfg *b) {
    if (a->t != b->t || a->s != b->s) return 0;
    for (int w = 0; w < MW; w++) if (a->m[w] != b->m[w]) return 0;
    return 1;
}
static void cset_init(cset *s) {
    s->cap = 1024; s->n = 0;
    s->e = (cfg *)malloc(sizeof(cfg) * s->cap); s->used = (uint8_t *)calloc(s->cap, 1);
}
static void cset_free(cset *s) { free(s->e); free(s->used); }
static int cset_has(const cset *s, const cfg *c) {
    uint64_t i = cfg_hash(c) & (s->cap - 1);
    while (s->used[i]) {
        if (cfg_eq(&s->e[i], c)) return 1;
        i = (i + 1) & (s->cap - 1);
    }
    return 0;
}
static void cset_add(cset *s, const cfg *c);
static void cset_grow(cset *s) {
    cset o = *s; s->cap = o.cap * 2; s->n = 0;
    s->e = (cfg *)malloc(sizeof(cfg) * s->cap); s->used = (uint8_t *)calloc(s->cap, 1);
    for (int64_t i = 0; i < o.cap; i++) if (o.used[i]) cset_add(s, &o.e[i]);
    cset_free(&o);
}
static void cset_add(cset *s, const cfg *c) {
    if (2 * (s->n + 1) > s->cap) cset_grow(s);
    uint64_t i = cfg_hash(c) & (s->cap - 1);
    while (s->used[i]) i = (i + 1) & (s->cap - 1);
    s->used[i] = 1; s->e[i] = *c; s->n++;
}
static inline int bit_get(const uint64_t *m, int i) { return (int)((m[i >> 6] >> (i & 63)) & 1); }
static inline void bit_set(uint64_t *m, int i) { m[i >> 6] |= 1ULL << (i & 63); }

/* Lift window member i of configuration (t, mask): the op takes effect now.
 * If it is the op whose return defines R, R advances to the next ok return
 * whose op is not yet linearized, and the mask is compacted onto W(t'). */
static void cfg_lift(const orc_key *k, uint32_t t, const uint64_t *mask, int i,
                     uint32_t *t_out, uint64_t *mask_out) {
    const int32_t *W = k->w_ops + k->w_off[t];
    int w = k->w_off[t + 1] - k->w_off[t];
    uint64_t lin[MW];
    memcpy(lin, mask, sizeof lin);
    bit_set(lin, i);
    if (W[i] != k->ret_op[t]) { *t_out = t; memcpy(mask_out, lin, sizeof lin); return; }
    uint32_t u = t + 1;
    while (u < (uint32_t)k->n_ok) {
        int found = 0;
        for (int j = 0; j < w; j++)
            if (bit_get(lin, j) && k->ops[W[j]].rr == (int32_t)u) { found = 1; break; }
        if (!found) break;
        u++;
    }
    memset(mask_out, 0, sizeof(uint64_t) * MW);
    *t_out = u;
    if (u == (uint32_t)k->n_ok) return;
    int b = 0;
    for (int j = 0; j < w; j++) {
        const orc_op *o = &k->ops[W[j]];
        if (o->rr < 0 || o->rr >= (int32_t)u) {
            if (bit_get(lin, j)) bit_set(mask_out, b);
            b++;
        }
    }
}

/* The WGL depth-first search (Lowe 2017 Fig. 3, as knossos.wgl/analysis) in
 * canonical coordinates: at configuration C the candidates are the
 * un-linearized members of W(t) in call order (= the call entries before
 * the first return entry of the lifted linked list); a candidate is taken
 * if the model allows it and the child configuration is not in the cache,
 * which it is then added to; after a lift the scan restarts at the first
 * candidate, after a backtrack it resumes after the popped one. */
typedef struct { uint32_t t; int32_t i; int64_t s; uint64_t m[MW]; } frame;

int orc_wgl_canonical(const orc_key *k, int64_t init, int64_t budget,
                      int64_t *explored, int64_t *fail_entry) {
    *explored = 0; *fail_entry = -1;
    if (k->status) return JH_UNKNOWN;
    if (k->n_ok == 0) return JH_VALID;
    cset memo; cset_init(&memo);
    int64_t cap = 256, depth = 0;
    frame *st = (frame *)malloc(sizeof(frame) * cap);
    uint32_t t = 0, tmax = 0; int64_t s = init; int start = 0;
    uint64_t mask[MW] = {0};
    int verdict;
    for (;;) {
        const int32_t *W = k->w_ops + k->w_off[t];
        int w = k->w_off[t + 1] - k->w_off[t];
        int took = 0;
        for (int i = start; i < w; i++) {
            if (bit_get(mask, i) || sym_blocked(k, W, mask, i)) continue;
            const orc_op *o = &k->ops[W[i]];
            int64_t s2;
            if (!cas_step(o->f, o->v1, o->v2, s, &s2)) continue;
            cfg c; c.s = s2;
            cfg_lift(k, t, mask, i, &c.t, c.m);
            if (cset_has(&memo, &c)) continue;
            if (memo.n >= budget) { verdict = JH_UNKNOWN; goto done; }
            cset_add(&memo, &c);
            if (depth == cap) { cap *= 2; st = (frame *)realloc(st, sizeof(frame) * cap); }
            st[depth].t = t; st[depth].i = i; st[depth].s = s; memcpy(st[depth].m, mask, sizeof mask); depth++;
            t = c.t; s = c.s; memcpy(mask, c.m, sizeof mask); start = 0;
            if (t > tmax) tmax = t;
            if (t == (uint32_t)k->n_ok) { verdict = JH_VALID; goto done; }
            took = 1;
            break;
        }
        if (took) continue;
        if (depth == 0) {
            verdict = JH_INVALID;
            *fail_entry = k->ops[k->ret_op[tmax]].ret;
            goto done;
        }
        depth--;
        t = st[depth].t; s = st[depth].s; memcpy(mask, st[depth].m, sizeof mask); start = st[depth].i + 1;
    }
done:
    *explored = memo.n;
    cset_free(&memo); free(st);
    return verdict;
}

/* ------------------------------------------------------------------------ */
/* knossos.linear/analysis [K] (Lowe's JIT linearization, selected by
 * :algorithm :linear at jepsen/src/jepsen/checker.clj:141-145): the set of
 * configurations is carried forward through the history; at each :ok
 * completion every configuration must linearize the completing op (after
 * any pending ops, in every order), and the history is linearizable iff the
 * set survives the last completion. In canonical coordinates that is the
 * reachable configuration set enumerated layer by layer (layer t = the
 * configurations whose earliest un-linearized :ok return is the t-th; a
 * same-layer edge lifts a pending op, a cross-layer edge lifts RET[t]). Its
 * size -- every configuration it visits except the initial one and the
 * terminal ones -- is what this analysis explores (WGL's count is a subset).
 * Returns JH_VALID / JH_INVALID, or JH_UNKNOWN when more than `budget`
 * configurations are reachable (the analysis would not finish: the caller
 * falls back to WGL). *tmax = the deepest layer reached (the failing op of
 * an invalid key is RET[tmax], as for WGL). Configurations of layer tmax are
 * collected into `front` (sorted later) when it is not NULL. */
typedef struct { cfg *e; int64_t n, cap; } cvec;
static void cvec_push(cvec *v, const cfg *c) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 256; v->e = (cfg *)realloc(v->e, sizeof(cfg) * v->cap); }
    v->e[v->n++] = *c;
}
/* The final configurations of a valid key (libjh's jh_lin_configs, ABI 6):
 * what the JIT-linearization analysis holds after the last :ok completion.
 * Each terminal edge -- lifting RET[t] from a layer-t configuration with
 * every later :ok op already linearized -- ends one: the register value and
 * which crashed ops are linearized, as a mask over C = W(n_ok - 1) minus
 * RET[n_ok - 1] in call order (every crashed op called before the last :ok
 * return; crashed ops never leave a window). cpos[op] = the op's position in
 * C, -1 for an op not in C. */
static void final_cfg(const orc_key *k, const int32_t *cpos, uint32_t t, const uint64_t *mask, int i, int64_t s2,
                      cvec *fin) {
    const int32_t *W = k->w_ops + k->w_off[t];
    const int w = k->w_off[t + 1] - k->w_off[t];
    cfg d; memset(&d, 0, sizeof d);
    d.t = t; d.s = s2;                 /* t: the layer whose :ok op was linearized last */
    for (int j = 0; j < w; j++)
        if ((j == i || bit_get(mask, j)) && cpos[W[j]] >= 0) bit_set(d.m, cpos[W[j]]);
    cvec_push(fin, &d);
}
static int orc_linear_fin(const orc_key *k, int64_t init, int64_t budget, int64_t *explored, uint32_t *tmax_out,
                          cvec *front, cvec *fin);
static int orc_linear(const orc_key *k, int64_t init, int64_t budget, int64_t *explored, uint32_t *tmax_out,
               cvec *front) {
    return orc_linear_fin(k, init, budget, explored, tmax_out, front, NULL);
}
static int orc_linear_fin(const orc_key *k, int64_t init, int64_t budget, int64_t *explored, uint32_t *tmax_out,
                          cvec *front, cvec *fin) {
    *explored = 0; *tmax_out = 0;
    if (k->status) return JH_UNKNOWN;
    if (k->n_ok == 0) return JH_VALID;
    int32_t *cpos = NULL;
    if (fin) {
        cpos = (int32_t *)malloc(sizeof(int32_t) * (size_t)(k->n_ops > 0 ? k->n_ops : 1));
        for (int32_t i = 0; i < k->n_ops; i++) cpos[i] = -1;
        const uint32_t tl = (uint32_t)k->n_ok - 1;
        const int32_t *W = k->w_ops + k->w_off[tl];
        int c = 0;
        for (int j = 0; j < k->w_off[tl + 1] - k->w_off[tl]; j++)
            if (W[j] != k->ret_op[tl]) cpos[W[j]] = c++;
    }
    cset seen; cset_init(&seen);
    cvec q = {0, 0, 0};
    cfg root; memset(&root, 0, sizeof root); root.t = 0; root.s = init;
    cset_add(&seen, &root); cvec_push(&q, &root);
    int term = 0;
    uint32_t tmax = 0;
    int verdict = JH_INVALID;
    for (int64_t h = 0; h < q.n; h++) {
        const cfg c = q.e[h];
        if (c.t > tmax) tmax = c.t;
        const int32_t *W = k->w_ops + k->w_off[c.t];
        const int w = k->w_off[c.t + 1] - k->w_off[c.t];
        for (int i = 0; i < w; i++) {
            if (bit_get(c.m, i)) continue;
            const orc_op *o = &k->ops[W[i]];
            int64_t s2;
            if (!cas_step(o->f, o->v1, o->v2, c.s, &s2)) continue;
            cfg d; d.s = s2;
            cfg_lift(k, c.t, c.m, i, &d.t, d.m);
            if (d.t == (uint32_t)k->n_ok) {
                term = 1;
                if (fin) final_cfg(k, cpos, c.t, c.m, i, s2, fin);
                continue;
            }
            if (cset_has(&seen, &d)) continue;
            if (seen.n - 1 >= budget) { verdict = JH_UNKNOWN; goto done; }
            cset_add(&seen, &d);
            cvec_push(&q, &d);
        }
    }
    verdict = term ? JH_VALID : JH_INVALID;
    if (verdict == JH_INVALID && front)
        for (int64_t h = 0; h < q.n; h++) if (q.e[h].t == tmax) cvec_push(front, &q.e[h]);
done:
    *explored = seen.n - 1;
    *tmax_out = tmax;
    cset_free(&seen); free(q.e); free(cpos);
    return verdict;
}

/* The frontier of an invalid key (libjh's jh_lin_configs, knossos' :configs
 * kept to (take 10 ...) by checker.clj:146-158): the configurations of the
 * last layer the analysis reaches, ordered by register value (nil first;
 * then, with per-key value numbering, the initial value; then ascending) and
 * then by the linearized-members mask, the first per_key of them; each as
 * its value and the invocation rows of its linearized, then pending, window
 * members in call order. Returns the count, or -1 when the key is not
 * invalid or outside the analysis' domain. */
/* :algorithm :linear on libjh.so's terms: the JIT-linearization analysis
 * decides a key when its windows fit the reachable-set engine (at most 32
 * members, fewer than 4096 interned states) and its reachable set fits the
 * budget; any other key is decided by WGL and reported with :analyzer :wgl
 * (the choice knossos.competition makes when :linear cannot finish).
 * states_ok is the history-wide condition the device computes once. */
int orc_linear_states_ok = 1;
static int linear_domain(const orc_key *k) {
    return k->max_window <= 32 && orc_linear_states_ok && k->n_ok < (1 << 20) - 2;
}

/* the frontier's order: value bucket (nil, then with per-key value
 * numbering the initial value, then the rest), value, then the window mask
 * as a JH_MAX_WINDOW-bit number (high word first) */
typedef struct { int64_t bucket, v; uint64_t m[MW]; uint32_t t; } cfg_ord;
static int cmp_cfg_ord(const void *a, const void *b) {
    const cfg_ord *x = (const cfg_ord *)a, *y = (const cfg_ord *)b;
    if (x->bucket != y->bucket) return x->bucket < y->bucket ? -1 : 1;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    for (int w = MW - 1; w >= 0; w--)
        if (x->m[w] != y->m[w]) return x->m[w] < y->m[w] ? -1 : 1;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    return 0;
}
/* :configs are defined wherever the reachable set can be enumerated: any
 * window up to JH_MAX_WINDOW (libjh: the reachable-set engine up to 32
 * members, the 65-256-member search's table beyond) */
static int configs_domain(const orc_key *k) {
    return !k->status && k->max_window <= JH_MAX_WINDOW && k->n_ok < (1 << 20) - 2;
}
/* Round 6: the reads the search drops (a crashed :read, an :ok :read of nil:
 * they constrain nothing) are ops knossos holds all the same
 * (checker.clj:156-158 passes its analysis through). Each configuration
 * printed is the one knossos holds in which such a read is linearized exactly
 * when its own completion forces it and never otherwise: a read invoked before
 * the configuration's point p and not completed by then (a crashed read
 * always) is pending, merged into :pending in call order (the row list stays
 * within JH_MAX_WINDOW), and an :ok read of nil completing before p is the
 * last op an expansion linearized when it completes after the configuration's
 * own :last-op. */
static int cmp_rows(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}
static void add_noop_reads(const orc_key *k, int64_t p, jh_lin_config *c, int64_t *r) {
    for (int32_t q = 0; q < k->n_noop; q++) {
        if (k->noop_ret[q] != ORC_CRASHED && k->noop_ret[q] < p && k->noop_ret[q] > c->last_row)
            c->last_row = k->noop_ret[q];
        if (k->noop_call[q] < p && k->noop_ret[q] > p && c->n_linearized + c->n_pending < JH_MAX_WINDOW)
            r[c->n_linearized + c->n_pending++] = k->noop_call[q];
    }
    qsort(r + c->n_linearized, (size_t)c->n_pending, sizeof(int64_t), cmp_rows);
}
static int configs_one(const jh_history *h, const int64_t *sel, int64_t m, int64_t init, int64_t budget,
                       int per_key, int per_key_values, jh_lin_config *out, int64_t *rows) {
    orc_key k;
    orc_key_prepare(h, sel, m, &k);
    int n = -1;
    if (configs_domain(&k)) {
        cvec front = {0, 0, 0}, fin = {0, 0, 0};
        int64_t explored; uint32_t tmax;
        /* final configurations only where the analysis itself decides the key
         * (a valid key it cannot hold is WGL's, and WGL carries none) */
        const int want_fin = linear_domain(&k);
        const int verdict = orc_linear_fin(&k, init, budget, &explored, &tmax, &front, want_fin ? &fin : NULL);
        if (verdict == JH_VALID && want_fin && k.n_ok == 0) {
            /* no :ok op: the one configuration is the initial one, every
             * (crashed) op pending, no :last-op */
            n = 1;
            jh_lin_config *c = &out[0];
            c->key = 0; c->model_value = init; c->n_linearized = 0; c->n_pending = 0; c->rows_off = 0;
            c->last_row = -1;
            for (int32_t q = 0; q < k.n_ops && q < JH_MAX_WINDOW; q++) rows[c->n_pending++] = k.ops[q].call;
            add_noop_reads(&k, ORC_CRASHED - 1, c, rows);
        } else if (verdict == JH_INVALID || (verdict == JH_VALID && want_fin)) {
            const int final = verdict == JH_VALID;
            const cvec *src = final ? &fin : &front;
            cfg_ord *o = (cfg_ord *)malloc(sizeof(cfg_ord) * (src->n ? src->n : 1));
            for (int64_t i = 0; i < src->n; i++) {
                const int64_t v = src->e[i].s;
                o[i].bucket = v == JH_NIL ? 0 : (per_key_values && init != JH_NIL && v == init) ? 1 : 2;
                o[i].v = v; memcpy(o[i].m, src->e[i].m, sizeof o[i].m);
                o[i].t = final ? src->e[i].t : 0;
            }
            qsort(o, src->n, sizeof(cfg_ord), cmp_cfg_ord);
            int64_t nu = 0;                                   /* distinct configurations */
            for (int64_t i = 0; i < src->n; i++)
                if (nu == 0 || cmp_cfg_ord(&o[nu - 1], &o[i]) != 0) o[nu++] = o[i];
            const uint32_t tl = final ? (uint32_t)k.n_ok - 1 : tmax;
            const int32_t *W = k.w_ops + k.w_off[tl];
            const int w = k.w_off[tl + 1] - k.w_off[tl];
            /* the members the masks range over: W(tmax), or C = W(n_ok - 1) - RET[n_ok - 1] */
            int32_t *mem = (int32_t *)malloc(sizeof(int32_t) * (size_t)(w > 0 ? w : 1));
            int nm = 0;
            for (int j = 0; j < w; j++) if (!final || W[j] != k.ret_op[tl]) mem[nm++] = W[j];
            const int64_t last_ret = k.ops[k.ret_op[k.n_ok - 1]].ret;
            /* :last-op: the frontier's is RET[tmax - 1]'s completion, a final
             * configuration's the :ok op its terminal edge linearized last */
            const int64_t lfront = tmax == 0 ? -1 : k.ops[k.ret_op[tmax - 1]].ret;
            /* configurations that differ only in :last-op can coincide once the
             * reads of nil move it (add_noop_reads): adjacent in this order */
            n = 0;
            for (int64_t i = 0; i < nu && n < per_key; i++) {
                jh_lin_config *c = &out[n];
                c->key = 0; c->model_value = o[i].v; c->n_linearized = 0; c->n_pending = 0;
                c->rows_off = (int64_t)n * JH_MAX_WINDOW;
                c->last_row = final ? k.ops[k.ret_op[o[i].t]].ret : lfront;
                int64_t *r = rows + (int64_t)n * JH_MAX_WINDOW;
                for (int j = 0; j < nm; j++) if (bit_get(o[i].m, j)) r[c->n_linearized++] = k.ops[mem[j]].call;
                for (int j = 0; j < nm; j++) if (!bit_get(o[i].m, j)) r[c->n_linearized + c->n_pending++] = k.ops[mem[j]].call;
                if (final)      /* crashed ops called after the last :ok return: pending */
                    for (int32_t q = 0; q < k.n_ops; q++)
                        if (k.ops[q].ret == ORC_CRASHED && k.ops[q].call > last_ret &&
                            c->n_linearized + c->n_pending < JH_MAX_WINDOW)
                            r[c->n_linearized + c->n_pending++] = k.ops[q].call;
                add_noop_reads(&k, final ? ORC_CRASHED - 1 : k.ops[k.ret_op[tmax]].ret, c, r);
                const jh_lin_config *b = n ? &out[n - 1] : NULL;
                if (b && b->model_value == c->model_value && b->last_row == c->last_row &&
                    b->n_linearized == c->n_linearized && b->n_pending == c->n_pending &&
                    !memcmp(rows + b->rows_off, r, sizeof(int64_t) * (size_t)(c->n_linearized + c->n_pending)))
                    continue;
                n++;
            }
            free(mem);
            free(o);
        }
        free(front.e); free(fin.e);
    }
    orc_key_free(&k);
    return n;
}

int orc_lin_configs(const jh_history *h, int64_t init, int64_t budget, const int64_t *keys, int64_t nq,
                    int32_t per_key, int32_t per_key_values, jh_lin_config *out, int32_t *n_out, int64_t *rows) {
    if (budget <= 0) budget = JH_DEFAULT_BUDGET;
    int64_t *sel = (int64_t *)malloc(sizeof(int64_t) * (h->n ? h->n : 1));
    for (int64_t q = 0; q < nq; q++) {
        int64_t m = 0;
        for (int64_t r = 0; r < h->n; r++) {
            const int64_t kk = h->key ? h->key[r] : 0;
            if (kk == keys[q] || kk < 0) sel[m++] = r;
        }
        n_out[q] = configs_one(h, sel, m, init, budget, per_key, per_key_values, out + q * per_key,
                               rows + q * per_key * JH_MAX_WINDOW);
        for (int i = 0; i < per_key; i++) {
            out[q * per_key + i].key = keys[q];
            out[q * per_key + i].rows_off += q * per_key * JH_MAX_WINDOW;
        }
    }
    free(sel);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* knossos-style WGL: doubly linked list of call/return entries in history
 * order, lift/unlift, BitSet of linearized op ids, HashSet<(BitSet, model)>.
 * Crashed ops have a call entry and no return entry, so they may be lifted
 * at any point after their call or never; the search succeeds once no
 * return entry remains.                                                   */
typedef struct { int64_t pos; int32_t op; int32_t is_call; } lent;
static int cmp_lent(const void *a, const void *b) {
    const lent *x = (const lent *)a, *y = (const lent *)b;
    return x->pos < y->pos ? -1 : x->pos > y->pos;
}
typedef struct { uint64_t *bits; int64_t s; } bkey;
typedef struct { uint64_t *arena; int64_t *st; uint8_t *used; int64_t cap, n, words, acap; } bset;
static uint64_t bkey_hash(const uint64_t *b, int64_t w, int64_t s) {
    uint64_t h = mix64((uint64_t)s ^ 0x1234567ULL);
    for (int64_t i = 0; i < w; i++) h = mix64(h ^ b[i]) + i;
    return h;
}
static void bset_init(bset *s, int64_t words) {
    s->cap = 1024; s->n = 0; s->words = words; s->acap = 1024;
    s->arena = (uint64_t *)malloc(sizeof(uint64_t) * words * s->acap);
    s->st = (int64_t *)malloc(sizeof(int64_t) * s->cap);   /* slot -> entry id */
    s->used = (uint8_t *)calloc(s->cap, 1);
}
static void bset_free(bset *s) { free(s->arena); free(s->st); free(s->used); }
typedef struct { bset b; int64_t *states; } bcache;
static int bcache_has(const bcache *c, const uint64_t *bits, int64_t s) {
    uint64_t i = bkey_hash(bits, c->b.words, s) & (c->b.cap - 1);
    while (c->b.used[i]) {
        int64_t e = c->b.st[i];
        if (c->states[e] == s && !memcmp(c->b.arena + e * c->b.words, bits, 8 * c->b.words)) return 1;
        i = (i + 1) & (c->b.cap - 1);
    }
    return 0;
}
static void bcache_slot(bcache *c, int64_t e) {
    uint64_t i = bkey_hash(c->b.arena + e * c->b.words, c->b.words, c->states[e]) & (c->b.cap - 1);
    while (c->b.used[i]) i = (i + 1) & (c->b.cap - 1);
    c->b.used[i] = 1; c->b.st[i] = e;
}
static void bcache_add(bcache *c, const uint64_t *bits, int64_t s) {
    if (c->b.n == c->b.acap) {
        c->b.acap *= 2;
        c->b.arena = (uint64_t *)realloc(c->b.arena, sizeof(uint64_t) * c->b.words * c->b.acap);
        c->states = (int64_t *)realloc(c->states, sizeof(int64_t) * c->b.acap);
    }
    int64_t e = c->b.n++;
    memcpy(c->b.arena + e * c->b.words, bits, 8 * c->b.words);
    c->states[e] = s;
    if (2 * c->b.n > c->b.cap) {
        c->b.cap *= 2;
        free(c->b.st); free(c->b.used);
        c->b.st = (int64_t *)malloc(sizeof(int64_t) * c->b.cap);
        c->b.used = (uint8_t *)calloc(c->b.cap, 1);
        for (int64_t x = 0; x < c->b.n; x++) bcache_slot(c, x);
    } else bcache_slot(c, e);
}

int orc_wgl_list(const orc_key *k, int64_t init, int64_t budget, int64_t *explored) {
    *explored = 0;
    if (k->status) return JH_UNKNOWN;
    int32_t n = k->n_ops;
    int32_t E = n + k->n_ok;
    lent *ent = (lent *)malloc(sizeof(lent) * (E + 1));
    int32_t e = 0;
    for (int32_t i = 0; i < n; i++) {
        ent[e].pos = k->ops[i].call; ent[e].op = i; ent[e].is_call = 1; e++;
        if (k->ops[i].ret != ORC_CRASHED) { ent[e].pos = k->ops[i].ret; ent[e].op = i; ent[e].is_call = 0; e++; }
    }
    qsort(ent, E, sizeof(lent), cmp_lent);
    /* nodes 0..E-1, head = E; next[E] = first, END = -1 */
    int32_t *nx = (int32_t *)malloc(sizeof(int32_t) * (E + 1));
    int32_t *pv = (int32_t *)malloc(sizeof(int32_t) * (E + 1));
    int32_t *call_ent = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *ret_ent = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; i++) ret_ent[i] = -1;
    for (int32_t x = 0; x < E; x++) {
        nx[x] = x + 1 < E ? x + 1 : -1; pv[x] = x == 0 ? E : x - 1;
        if (ent[x].is_call) call_ent[ent[x].op] = x; else ret_ent[ent[x].op] = x;
    }
    nx[E] = E ? 0 : -1; pv[E] = -1;
    int64_t words = (n + 63) / 64; if (!words) words = 1;
    uint64_t *lin = (uint64_t *)calloc(words, 8);
    bcache cache; bset_init(&cache.b, words);
    cache.states = (int64_t *)malloc(sizeof(int64_t) * cache.b.acap);
    typedef struct { int32_t entry; int64_t s; } lfr;
    lfr *st = (lfr *)malloc(sizeof(lfr) * (n + 1));
    int32_t depth = 0, remaining = k->n_ok;
    int64_t s = init;
    int32_t cur = nx[E];
    int verdict;
#define UNLINK(x) do { nx[pv[x]] = nx[x]; if (nx[x] >= 0) pv[nx[x]] = pv[x]; } while (0)
#define RELINK(x) do { nx[pv[x]] = (x); if (nx[x] >= 0) pv[nx[x]] = (x); } while (0)
    for (;;) {
        if (remaining == 0) { verdict = JH_VALID; break; }
        if (cur < 0) { verdict = JH_INVALID; break; } /* unreachable: a return is ahead */
        if (ent[cur].is_call) {
            int32_t op = ent[cur].op;
            const orc_op *o = &k->ops[op];
            int64_t s2;
            int took = 0;
            if (cas_step(o->f, o->v1, o->v2, s, &s2)) {
                lin[op >> 6] |= 1ULL << (op & 63);
                if (!bcache_has(&cache, lin, s2)) {
                    if (cache.b.n >= budget) { verdict = JH_UNKNOWN; break; }
                    bcache_add(&cache, lin, s2);
                    st[depth].entry = cur; st[depth].s = s; depth++;
                    s = s2;
                    UNLINK(call_ent[op]);
                    if (ret_ent[op] >= 0) { UNLINK(ret_ent[op]); remaining--; }
                    cur = nx[E];
                    took = 1;
                } else lin[op >> 6] &= ~(1ULL << (op & 63));
            }
            if (!took) cur = nx[cur];
        } else {
            if (depth == 0) { verdict = JH_INVALID; break; }
            depth--;
            int32_t ce = st[depth].entry, op = ent[ce].op;
            s = st[depth].s;
            lin[op >> 6] &= ~(1ULL << (op & 63));
            if (ret_ent[op] >= 0) { RELINK(ret_ent[op]); remaining++; }
            RELINK(call_ent[op]);
            cur = nx[ce];
        }
    }
#undef UNLINK
#undef RELINK
    *explored = cache.b.n;
    bset_free(&cache.b); free(cache.states);
    free(st); free(lin); free(ent); free(nx); free(pv); free(call_ent); free(ret_ent);
    return verdict;
}

/* ------------------------------------------------------------------------ */
/* Brute force from the definition (Herlihy & Wing): some sequence of all ok
 * ops and any subset of crashed ops, respecting "a returned before b was
 * invoked => a before b", is legal for the model from init. No memo.     */
static int bf_rec(const orc_key *k, uint64_t lin, int64_t s, uint64_t okmask) {
    if ((lin & okmask) == okmask) return 1;
    for (int b = 0; b < k->n_ops; b++) {
        if ((lin >> b) & 1) continue;
        int allowed = 1;
        for (int a = 0; a < k->n_ops && allowed; a++) {
            if (a == b || ((lin >> a) & 1) || k->ops[a].ret == ORC_CRASHED) continue;
            if (k->ops[a].ret < k->ops[b].call) allowed = 0;
        }
        if (!allowed) continue;
        int64_t s2;
        if (!cas_step(k->ops[b].f, k->ops[b].v1, k->ops[b].v2, s, &s2)) continue;
        if (bf_rec(k, lin | (1ULL << b), s2, okmask)) return 1;
    }
    return 0;
}
int orc_lin_bruteforce(const orc_key *k, int64_t init) {
    if (k->status) return JH_UNKNOWN;
    if (k->n_ops > 16) return -1;
    uint64_t okm = 0;
    for (int i = 0; i < k->n_ops; i++) if (k->ops[i].ret != ORC_CRASHED) okm |= 1ULL << i;
    return bf_rec(k, 0, init, okm) ? JH_VALID : JH_INVALID;
}

/* ------------------------------------------------------------------------ */
static void check_one(const jh_history *h, const int64_t *sel, int64_t m,
                      int64_t init, int64_t budget, int list_algo, jh_key_verdict *out) {
    orc_key k;
    orc_key_prepare(h, sel, m, &k);
    out->fail_entry = -1; out->explored = 0;
    out->analyzer = list_algo == 2 ? JH_ANALYZER_LINEAR : JH_ANALYZER_WGL;
    out->reserved = 0;
    if (k.status) {
        out->valid = JH_UNKNOWN; out->cause = k.status;
    } else if (list_algo == 2 && linear_domain(&k) &&
               (out->valid = orc_linear(&k, init, budget, &out->explored, (uint32_t *)&out->reserved, NULL)) != JH_UNKNOWN) {
        out->cause = JH_CAUSE_NONE;
        if (out->valid == JH_INVALID) out->fail_entry = k.ops[k.ret_op[out->reserved]].ret;
        out->reserved = 0;
    } else if (list_algo == 2) {
        out->reserved = 0;
        out->analyzer = JH_ANALYZER_WGL;
        out->valid = orc_wgl_canonical(&k, init, budget, &out->explored, &out->fail_entry);
        out->cause = out->valid == JH_UNKNOWN ? JH_CAUSE_BUDGET : JH_CAUSE_NONE;
    } else if (list_algo) {
        out->valid = orc_wgl_list(&k, init, budget, &out->explored);
        out->cause = out->valid == JH_UNKNOWN ? JH_CAUSE_BUDGET : JH_CAUSE_NONE;
    } else {
        out->valid = orc_wgl_canonical(&k, init, budget, &out->explored, &out->fail_entry);
        out->cause = out->valid == JH_UNKNOWN ? JH_CAUSE_BUDGET : JH_CAUSE_NONE;
    }
    /* the search frontier of an invalid key (include/jh.h): last_op = the ok
     * completion of RET[tmax-1], previous_ok = the last client :ok before
     * the failing row in the key's subhistory */
    out->previous_ok = -1; out->last_op = -1;
    if (out->valid == JH_INVALID && out->fail_entry >= 0) {
        for (int t = 0; t < k.n_ok; t++)
            if (k.ops[k.ret_op[t]].ret == out->fail_entry) {
                if (t > 0) out->last_op = k.ops[k.ret_op[t - 1]].ret;
                break;
            }
        for (int64_t i = 0; i < m; i++) {
            const int64_t r = sel[i];
            if (r < out->fail_entry && h->process[r] >= 0 && h->type[r] == JH_TYPE_OK) out->previous_ok = r;
        }
    }
    orc_key_free(&k);
}

int orc_check_cas(const jh_history *h, int64_t init, int64_t budget, jh_key_verdict *out) {
    if (budget <= 0) budget = JH_DEFAULT_BUDGET;
    out->analyzer = JH_ANALYZER_WGL; out->reserved = 0;
    int64_t *sel = (int64_t *)malloc(sizeof(int64_t) * (h->n ? h->n : 1));
    for (int64_t i = 0; i < h->n; i++) sel[i] = i;
    check_one(h, sel, h->n, init, budget, 0, out);
    free(sel);
    return 0;
}

/* jepsen.independent/checker (independent.clj:247-298): history-keys
 * (:222-232), subhistory (:234-245) = every entry whose value is not a tuple
 * plus the entries of key k, in order; bounded-pmap over keys (:266-288).  */
typedef struct {
    const jh_history *h; int64_t init, budget; int mode;
    int64_t k0, k1; jh_key_verdict *out;
    const int64_t *koff, *krows, *unkeyed; int64_t n_unkeyed;
    int64_t next; pthread_mutex_t mu;
} indep_job;

static void *indep_worker(void *arg) {
    indep_job *J = (indep_job *)arg;
    const jh_history *h = J->h;
    int64_t *sel = (int64_t *)malloc(sizeof(int64_t) * (h->n ? h->n : 1));
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int64_t key = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (key >= J->k1) break;
        jh_key_verdict *o = &J->out[key - J->k0];
        int64_t m = 0, present = 0;
        if (J->mode & 1) {
            /* faithful: scan the whole history for this key, O(N) per key */
            for (int64_t r = 0; r < h->n; r++) {
                int64_t kk = h->key ? h->key[r] : -1;
                if (kk == key) { sel[m++] = r; present = 1; }
                else if (kk < 0) sel[m++] = r;
            }
        } else {
            const int64_t *a = J->krows + J->koff[key];
            int64_t na = J->koff[key + 1] - J->koff[key], ia = 0, iu = 0;
            present = na > 0;
            while (ia < na || iu < J->n_unkeyed) {
                if (iu >= J->n_unkeyed || (ia < na && a[ia] < J->unkeyed[iu])) sel[m++] = a[ia++];
                else sel[m++] = J->unkeyed[iu++];
            }
        }
        if (!present) {
            o->valid = JH_VALID; o->cause = 0; o->fail_entry = -1; o->explored = -1;
            o->previous_ok = -1; o->last_op = -1;
            o->analyzer = (J->mode & 4) ? JH_ANALYZER_LINEAR : JH_ANALYZER_WGL; o->reserved = 0;
            continue;
        }
        check_one(h, sel, m, J->init, J->budget, (J->mode & 4) ? 2 : (J->mode >> 1) & 1, o);
    }
    free(sel);
    return NULL;
}

int orc_check_cas_independent_range(const jh_history *h, int64_t init, int64_t budget,
                                    int mode, int threads, int64_t k0, int64_t k1,
                                    jh_key_verdict *out) {
    if (budget <= 0) budget = JH_DEFAULT_BUDGET;
    if (threads < 1) threads = 1;
    indep_job J; memset(&J, 0, sizeof(J));
    J.h = h; J.init = init; J.budget = budget; J.mode = mode; J.k0 = k0; J.k1 = k1;
    J.out = out; J.next = k0; pthread_mutex_init(&J.mu, NULL);
    int64_t *koff = NULL, *krows = NULL, *unk = NULL;
    if (!(mode & 1)) {
        int64_t K = h->n_keys;
        koff = (int64_t *)calloc(K + 1, sizeof(int64_t));
        int64_t nu = 0;
        for (int64_t r = 0; r < h->n; r++) {
            int64_t kk = h->key ? h->key[r] : -1;
            if (kk >= 0 && kk < K) koff[kk + 1]++; else nu++;
        }
        for (int64_t i = 0; i < K; i++) koff[i + 1] += koff[i];
        krows = (int64_t *)malloc(sizeof(int64_t) * (koff[K] ? koff[K] : 1));
        unk = (int64_t *)malloc(sizeof(int64_t) * (nu ? nu : 1));
        int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (K ? K : 1));
        memcpy(fill, koff, sizeof(int64_t) * K);
        nu = 0;
        for (int64_t r = 0; r < h->n; r++) {
            int64_t kk = h->key ? h->key[r] : -1;
            if (kk >= 0 && kk < K) krows[fill[kk]++] = r; else unk[nu++] = r;
        }
        free(fill);
        J.koff = koff; J.krows = krows; J.unkeyed = unk; J.n_unkeyed = nu;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, indep_worker, &J);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    free(th); free(koff); free(krows); free(unk);
    pthread_mutex_destroy(&J.mu);
    return 0;
}

int orc_check_cas_independent(const jh_history *h, int64_t init, int64_t budget,
                              int mode, int threads, jh_key_verdict *out, jh_summary *sum) {
    orc_check_cas_independent_range(h, init, budget, mode, threads, 0, h->n_keys, out);
    if (sum) {
        memset(sum, 0, sizeof(*sum));
        sum->first_fail_entry = -1;
        for (int64_t k = 0; k < h->n_keys; k++) {
            if (out[k].explored < 0) continue;
            sum->n_keys++;
            sum->explored += out[k].explored;
            if (out[k].valid > sum->valid) sum->valid = out[k].valid;
            if (out[k].valid == JH_INVALID) {
                sum->n_invalid++;
                if (sum->first_fail_entry < 0 || out[k].fail_entry < sum->first_fail_entry)
                    sum->first_fail_entry = out[k].fail_entry;
            }
            if (out[k].valid == JH_UNKNOWN) sum->n_unknown++;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* checker/counter, jepsen/src/jepsen/checker.clj:679-734: history/complete,
 * (remove :fails?), (remove op/fail?), then the lower/upper loop.
 * Clojure + throws on long overflow and <= on nil throws; both end in
 * check-safe's {:valid? :unknown} (checker.clj:77-88).                     */
int orc_check_counter(const jh_history *h, int64_t *reads_out, int64_t reads_cap,
                      int64_t *n_reads, int64_t *n_errors, int64_t *first_err_entry,
                      int32_t *valid, int32_t *cause) {
    int64_t n = h->n;
    *n_reads = 0; *n_errors = 0; *first_err_entry = -1; *valid = JH_VALID; *cause = 0;
    int64_t *pair = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    for (int64_t i = 0; i < n; i++) pair[i] = -1;
    imap open; imap_init(&open, 64);
    for (int64_t r = 0; r < n; r++) {
        int64_t p = h->process[r], ty = h->type[r];
        int64_t slot = imap_find(&open, p);
        if (ty == JH_TYPE_INVOKE) {
            if (slot >= 0) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_DOUBLE_INVOKE; break; }
            imap_put(&open, p, r);
        } else if (ty == JH_TYPE_OK || ty == JH_TYPE_FAIL) {
            if (slot < 0) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_ORPHAN; break; }
            pair[open.v[slot]] = r; pair[r] = open.v[slot];
            imap_del(&open, slot);
        }
    }
    imap_free(&open);
    if (*cause) { free(pair); return 0; }
    int64_t lower = 0, upper = 0, nr = 0;
    int64_t *rd = (int64_t *)malloc(sizeof(int64_t) * 3 * (n ? n : 1));  /* [inv-row v upper] */
    int64_t *rrow = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));    /* ok-read row */
    imap pend; imap_init(&pend, 64);            /* process -> invoke row */
    for (int64_t r = 0; r < n && !*cause; r++) {
        int64_t ty = h->type[r], f = h->f[r], c = pair[r];
        if (ty == JH_TYPE_FAIL) continue;                                    /* (remove op/fail?) */
        if (ty == JH_TYPE_INVOKE && c >= 0 && h->type[c] == JH_TYPE_FAIL) continue; /* (remove :fails?) */
        int64_t v = h->value[r];
        if (ty == JH_TYPE_INVOKE && v == JH_NIL && c >= 0) v = h->value[c];  /* (or inv ok) */
        if (ty == JH_TYPE_INVOKE && f == JH_F_READ) {
            imap_put(&pend, h->process[r], r);
        } else if (ty == JH_TYPE_OK && f == JH_F_READ) {
            int64_t slot = imap_find(&pend, h->process[r]);
            if (slot < 0) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_ORPHAN; break; }
            int64_t inv = pend.v[slot];
            imap_del(&pend, slot);
            int64_t rv = h->value[inv];
            if (rv == JH_NIL) rv = h->value[r];
            rd[3 * nr + 0] = inv; rd[3 * nr + 1] = rv; rd[3 * nr + 2] = upper;
            rrow[nr] = r;
            nr++;
        } else if (ty == JH_TYPE_INVOKE && f == JH_F_ADD) {
            if (v == JH_NIL) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_NIL_VALUE; break; }
            if (__builtin_add_overflow(upper, v, &upper)) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_OVERFLOW; break; }
        } else if (ty == JH_TYPE_OK && f == JH_F_ADD) {
            if (v == JH_NIL) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_NIL_VALUE; break; }
            if (__builtin_add_overflow(lower, v, &lower)) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_OVERFLOW; break; }
        }
    }
    imap_free(&pend);
    free(pair);
    if (*cause) { free(rd); free(rrow); return 0; }
    /* lower as stashed by [:invoke :read] (checker.clj:713-716) = sum of the
     * :ok :add values strictly before the invocation row */
    {
        int64_t nadd = 0, lo = 0;
        for (int64_t r = 0; r < n; r++) if (h->type[r] == JH_TYPE_OK && h->f[r] == JH_F_ADD) nadd++;
        int64_t *arow = (int64_t *)malloc(sizeof(int64_t) * (nadd + 1));
        int64_t *apre = (int64_t *)malloc(sizeof(int64_t) * (nadd + 1));
        nadd = 0; apre[0] = 0;
        for (int64_t r = 0; r < n; r++) if (h->type[r] == JH_TYPE_OK && h->f[r] == JH_F_ADD) {
            arow[nadd] = r; lo += h->value[r]; apre[nadd + 1] = lo; nadd++;
        }
        for (int64_t i = 0; i < nr; i++) {
            int64_t inv = rd[3 * i], a = 0, b = nadd;
            while (a < b) { int64_t mid = (a + b) / 2; if (arow[mid] < inv) a = mid + 1; else b = mid; }
            rd[3 * i] = apre[a];
        }
        free(arow); free(apre);
    }
    *n_reads = nr;
    /* errors = (remove (partial apply <=) reads) */
    int64_t ne = 0;
    for (int64_t i = 0; i < nr; i++) {
        int64_t lo = rd[3 * i], v = rd[3 * i + 1], hi = rd[3 * i + 2];
        if (v == JH_NIL) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_NIL_VALUE; break; }
        if (!(lo <= v && v <= hi)) {
            if (ne == 0) *first_err_entry = rrow[i];
            ne++;
        }
    }
    int64_t lim = nr < reads_cap ? nr : reads_cap;
    if (lim > 0) memcpy(reads_out, rd, sizeof(int64_t) * 3 * lim);
    free(rd); free(rrow);
    *n_errors = ne;
    if (!*cause) *valid = ne ? JH_INVALID : JH_VALID;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* checker/set, jepsen/src/jepsen/checker.clj:182-233.                       */
static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}
static int64_t sort_unique(int64_t *a, int64_t n) {
    if (!n) return 0;
    qsort(a, n, sizeof(int64_t), cmp_i64);
    int64_t m = 1;
    for (int64_t i = 1; i < n; i++) if (a[i] != a[m - 1]) a[m++] = a[i];
    return m;
}
static int64_t to_runs(const int64_t *a, int64_t n, int64_t *runs, int64_t cap) {
    int64_t nr = 0;
    for (int64_t i = 0; i < n; ) {
        int64_t j = i;
        while (j + 1 < n && a[j + 1] == a[j] + 1) j++;
        if (nr < cap) { runs[2 * nr] = a[i]; runs[2 * nr + 1] = a[j]; }
        nr++; i = j + 1;
    }
    return nr;
}
/* a minus b (both sorted unique) into out */
static int64_t set_diff(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int64_t *out) {
    int64_t i = 0, j = 0, m = 0;
    while (i < na) {
        while (j < nb && b[j] < a[i]) j++;
        if (j < nb && b[j] == a[i]) { i++; continue; }
        out[m++] = a[i++];
    }
    return m;
}
static int64_t set_inter(const int64_t *a, int64_t na, const int64_t *b, int64_t nb, int64_t *out) {
    int64_t i = 0, j = 0, m = 0;
    while (i < na && j < nb) {
        if (a[i] < b[j]) i++; else if (b[j] < a[i]) j++; else { out[m++] = a[i]; i++; j++; }
    }
    return m;
}

int orc_check_set(const jh_history *h, jh_set_result *res,
                  int64_t *runs_ok, int64_t *runs_lost, int64_t *runs_unexpected,
                  int64_t *runs_recovered, int64_t runs_cap) {
    memset(res, 0, sizeof(*res));
    res->first_fail_entry = -1; res->final_read_entry = -1;
    int64_t n = h->n, na = 0, nd = 0;
    int64_t *att = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    int64_t *add = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    int64_t fr = -1;
    for (int64_t r = 0; r < n; r++) {
        if (h->f[r] == JH_F_ADD && h->type[r] == JH_TYPE_INVOKE) att[na++] = h->value[r];
        if (h->f[r] == JH_F_ADD && h->type[r] == JH_TYPE_OK) add[nd++] = h->value[r];
        if (h->f[r] == JH_F_READ && h->type[r] == JH_TYPE_OK) fr = r;   /* (reduce (fn [_ x] x)) */
    }
    res->final_read_entry = fr;
    if (fr < 0 || h->value[fr] == JH_NIL) {
        /* {:valid? :unknown :error "Set was never read"} */
        res->valid = JH_UNKNOWN; res->cause = JH_CAUSE_NIL_VALUE;
        free(att); free(add); return 0;
    }
    for (int64_t i = 0; i < na; i++) if (att[i] == JH_NIL) { res->valid = JH_UNKNOWN; res->cause = JH_CAUSE_NIL_VALUE; }
    for (int64_t i = 0; i < nd; i++) if (add[i] == JH_NIL) { res->valid = JH_UNKNOWN; res->cause = JH_CAUSE_NIL_VALUE; }
    if (res->cause) { free(att); free(add); return 0; }
    na = sort_unique(att, na); nd = sort_unique(add, nd);
    int64_t off = h->value[fr], cnt = h->value2[fr];
    int64_t *rd = (int64_t *)malloc(sizeof(int64_t) * (cnt + 1));
    memcpy(rd, h->aux + off, sizeof(int64_t) * cnt);
    int64_t nrd = sort_unique(rd, cnt);
    int64_t big = na + nd + nrd + 1;
    int64_t *ok = (int64_t *)malloc(sizeof(int64_t) * big);
    int64_t *unexp = (int64_t *)malloc(sizeof(int64_t) * big);
    int64_t *lost = (int64_t *)malloc(sizeof(int64_t) * big);
    int64_t *rec = (int64_t *)malloc(sizeof(int64_t) * big);
    int64_t nok = set_inter(rd, nrd, att, na, ok);
    int64_t nun = set_diff(rd, nrd, att, na, unexp);
    int64_t nlo = set_diff(add, nd, rd, nrd, lost);
    int64_t nre = set_diff(ok, nok, add, nd, rec);
    res->attempt_count = na; res->acknowledged_count = nd; res->ok_count = nok;
    res->lost_count = nlo; res->recovered_count = nre; res->unexpected_count = nun;
    res->valid = (nlo == 0 && nun == 0) ? JH_VALID : JH_INVALID;
    if (nlo) {
        for (int64_t r = 0; r < n; r++) {
            if (h->f[r] == JH_F_ADD && h->type[r] == JH_TYPE_OK) {
                int64_t v = h->value[r], a = 0, b = nlo;
                while (a < b) { int64_t mid = (a + b) / 2; if (lost[mid] < v) a = mid + 1; else b = mid; }
                if (a < nlo && lost[a] == v) { res->first_fail_entry = r; break; }
            }
        }
    } else if (nun) res->first_fail_entry = fr;
    res->n_runs[0] = to_runs(ok, nok, runs_ok, runs_cap);
    res->n_runs[1] = to_runs(lost, nlo, runs_lost, runs_cap);
    res->n_runs[2] = to_runs(unexp, nun, runs_unexpected, runs_cap);
    res->n_runs[3] = to_runs(rec, nre, runs_recovered, runs_cap);
    free(att); free(add); free(rd); free(ok); free(unexp); free(lost); free(rec);
    return 0;
}

/* util/integer-interval-set-str, jepsen/src/jepsen/util.clj:536-575:
 * "#{1..3 5 7..9}" from a sorted set of integers. */
int64_t orc_interval_str(const int64_t *a, int64_t n, char *buf, int64_t cap) {
    int64_t len = 0;
    char tmp[64];
#define PUT(s) do { const char *_s = (s); while (*_s) { if (len + 1 < cap) buf[len] = *_s; len++; _s++; } } while (0)
    PUT("#{");
    int first = 1;
    for (int64_t i = 0; i < n; ) {
        int64_t j = i;
        while (j + 1 < n && a[j + 1] == a[j] + 1) j++;
        if (!first) PUT(" ");
        first = 0;
        if (i == j) snprintf(tmp, sizeof tmp, "%lld", (long long)a[i]);
        else snprintf(tmp, sizeof tmp, "%lld..%lld", (long long)a[i], (long long)a[j]);
        PUT(tmp);
        i = j + 1;
    }
    PUT("}");
#undef PUT
    if (cap > 0) buf[len < cap ? len : cap - 1] = 0;
    return len;
}

/* Self-test hook: the three formulations on one whole history.
 * res = {status, canonical, canonical_explored, list, list_explored,
 *        bruteforce (-1 if too large), n_ops, max_window}                  */
int orc_lin_selftest_key(const jh_history *h, int64_t init, int64_t budget, int64_t *res) {
    int64_t *sel = (int64_t *)malloc(sizeof(int64_t) * (h->n ? h->n : 1));
    for (int64_t i = 0; i < h->n; i++) sel[i] = i;
    orc_key k;
    orc_key_prepare(h, sel, h->n, &k);
    free(sel);
    int64_t ex = 0, fe = -1;
    res[0] = k.status;
    res[1] = orc_wgl_canonical(&k, init, budget, &ex, &fe); res[2] = ex;
    res[3] = orc_wgl_list(&k, init, budget, &ex); res[4] = ex;
    res[5] = k.n_ops <= 14 ? orc_lin_bruteforce(&k, init) : -1;
    res[6] = k.n_ops; res[7] = k.max_window;
    orc_key_free(&k);
    return 0;
}

/* Size of the full reachable configuration graph (excluding the initial
 * configuration), by a worklist over (t, mask, state), stopping past cap.
 * For an invalid key the WGL search inserts exactly this set into its
 * cache, so the two counts must agree; for a valid key the search stops at
 * the first terminal configuration. res = {verdict, reachable, terminal?} */
int orc_reachable(const orc_key *k, int64_t init, int64_t cap, int64_t *res) {
    res[0] = res[1] = res[2] = 0;
    if (k->status) { res[0] = JH_UNKNOWN; return 0; }
    if (k->n_ok == 0) { res[0] = JH_VALID; return 0; }
    cset seen; cset_init(&seen);
    int64_t qcap = 1024, qh = 0, qt = 0;
    cfg *q = (cfg *)malloc(sizeof(cfg) * qcap);
    cfg c0; memset(&c0, 0, sizeof c0); c0.s = init;
    q[qt++] = c0;
    int term = 0;
    while (qh < qt) {
        cfg c = q[qh++];
        if (c.t == (uint32_t)k->n_ok) { term = 1; continue; }
        const int32_t *W = k->w_ops + k->w_off[c.t];
        int w = k->w_off[c.t + 1] - k->w_off[c.t];
        for (int i = 0; i < w; i++) {
            if (bit_get(c.m, i)) continue;
            const orc_op *o = &k->ops[W[i]];
            int64_t s2;
            if (!cas_step(o->f, o->v1, o->v2, c.s, &s2)) continue;
            cfg d; d.s = s2;
            cfg_lift(k, c.t, c.m, i, &d.t, d.m);
            if (cset_has(&seen, &d)) continue;
            cset_add(&seen, &d);
            if (seen.n > cap) goto out;
            if (qt == qcap) { qcap *= 2; q = (cfg *)realloc(q, sizeof(cfg) * qcap); }
            q[qt++] = d;
        }
    }
out:
    res[0] = seen.n > cap ? JH_UNKNOWN : (term ? JH_VALID : JH_INVALID);
    res[1] = seen.n; res[2] = term;
    cset_free(&seen); free(q);
    return 0;
}

/* Per-key statistics for design work: res[k*6..] = {canonical verdict,
 * explored, reachable verdict, reachable, n_ops, max_window} */
int orc_key_stats(const jh_history *h, int64_t init, int64_t budget, int64_t cap,
                  int64_t k0, int64_t k1, int64_t *res) {
    int64_t *sel = (int64_t *)malloc(sizeof(int64_t) * (h->n ? h->n : 1));
    for (int64_t key = k0; key < k1; key++) {
        int64_t m = 0;
        for (int64_t r = 0; r < h->n; r++) if (h->key[r] == key || h->key[r] < 0) sel[m++] = r;
        orc_key k; orc_key_prepare(h, sel, m, &k);
        int64_t ex, fe, rr[3];
        int64_t *o = res + 6 * (key - k0);
        o[0] = orc_wgl_canonical(&k, init, budget, &ex, &fe); o[1] = ex;
        orc_reachable(&k, init, cap, rr); o[2] = rr[0]; o[3] = rr[1];
        o[4] = k.n_ops; o[5] = k.max_window;
        orc_key_free(&k);
    }
    free(sel);
    return 0;
}
