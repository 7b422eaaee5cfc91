/* Shape of one key's WGL search (a CPU analysis tool, not product code):
 * the canonical WGL DFS of oracle/jh_oracle.c (orc_wgl_canonical), with every
 * push and pop recorded, so that the inserts of a valid key split into the
 * final path and the dead subtrees hanging off it (their sizes, layer spans
 * and depths): what a multi-workgroup engine could run side by side.
 * Built and driven by tools/shape/wgl_shape.py. */
#include "../../oracle/jh_oracle.c"

typedef struct { int64_t parent, start, size, depth_max; uint32_t t0, t1; int popped; } node_rec;

int wgl_shape(const jh_history *h, const int64_t *sel, int64_t m, int64_t init, int64_t budget, int64_t *out,
              int64_t *dead_sizes, int64_t *dead_depths, int64_t *dead_par, int64_t *dead_span, int64_t cap) {
    orc_key kk; orc_key_prepare(h, sel, m, &kk); const orc_key *k = &kk;
    if (k->status || k->n_ok == 0) { orc_key_free(&kk); return -1; }
    cset memo; cset_init(&memo);
    int64_t scap = 256, depth = 0;
    frame *st = (frame *)malloc(sizeof(frame) * scap);
    int64_t *sid = (int64_t *)malloc(sizeof(int64_t) * scap);      /* node id at each depth (the child pushed) */
    int64_t ncap = 1 << 16, nn = 0;
    node_rec *nr = (node_rec *)malloc(sizeof(node_rec) * ncap);
    uint32_t t = 0; int64_t s = init; int start = 0;
    uint64_t mask[MW] = {0};
    int verdict = -1;
    int64_t cur = -1;     /* the current node's id (-1: root) */
    for (;;) {
        const int32_t *W = k->w_ops + k->w_off[t];
        int w = k->w_off[t + 1] - k->w_off[t];
        int took = 0;
        for (int i = start; i < w; i++) {
            if (bit_get(mask, i)) continue;
            const orc_op *o = &k->ops[W[i]];
            int64_t s2;
            if (!cas_step(o->f, o->v1, o->v2, s, &s2)) continue;
            cfg c; c.s = s2;
            cfg_lift(k, t, mask, i, &c.t, c.m);
            if (cset_has(&memo, &c)) continue;
            if (memo.n >= budget) { verdict = JH_UNKNOWN; goto done; }
            cset_add(&memo, &c);
            if (depth == scap) { scap *= 2; st = (frame *)realloc(st, sizeof(frame) * scap); sid = (int64_t *)realloc(sid, sizeof(int64_t) * scap); }
            if (nn == ncap) { ncap *= 2; nr = (node_rec *)realloc(nr, sizeof(node_rec) * ncap); }
            nr[nn].parent = cur; nr[nn].start = memo.n - 1; nr[nn].size = 0; nr[nn].t0 = c.t; nr[nn].t1 = c.t;
            nr[nn].popped = 0; nr[nn].depth_max = depth + 1;
            st[depth].t = t; st[depth].i = i; st[depth].s = s; memcpy(st[depth].m, mask, sizeof mask);
            sid[depth] = cur;
            depth++;
            cur = nn++;
            t = c.t; s = c.s; memcpy(mask, c.m, sizeof mask); start = 0;
            if (t == (uint32_t)k->n_ok) { verdict = JH_VALID; goto done; }
            took = 1;
            break;
        }
        if (took) continue;
        if (depth == 0) { verdict = JH_INVALID; goto done; }
        /* pop cur: its subtree is complete */
        nr[cur].size = memo.n - nr[cur].start;
        nr[cur].popped = 1;
        {
            const int64_t p = nr[cur].parent;
            if (p >= 0) {
                if (nr[cur].t1 > nr[p].t1) nr[p].t1 = nr[cur].t1;
                if (nr[cur].depth_max > nr[p].depth_max) nr[p].depth_max = nr[cur].depth_max;
            }
        }
        depth--;
        cur = sid[depth];
        t = st[depth].t; s = st[depth].s; memcpy(mask, st[depth].m, sizeof mask); start = st[depth].i + 1;
    }
done:
    out[0] = verdict; out[1] = memo.n; out[2] = depth; out[3] = nn;
    /* top-level dead subtrees: popped nodes whose parent is on the final path (never popped, or the root) */
    int64_t nd = 0;
    for (int64_t i = 0; i < nn; i++) {
        if (!nr[i].popped) continue;
        const int64_t p = nr[i].parent;
        if (p >= 0 && nr[p].popped) continue;
        if (nd < cap) {
            dead_sizes[nd] = nr[i].size;
            dead_depths[nd] = nr[i].depth_max - (p >= 0 ? 0 : 0);
            /* depth of the path node it hangs from */
            int64_t d = 0; for (int64_t q = p; q >= 0; q = nr[q].parent) d++;
            dead_par[nd] = d;
            dead_depths[nd] = nr[i].depth_max - d;
            dead_span[nd] = (int64_t)nr[i].t1 - nr[i].t0;
        }
        nd++;
    }
    out[4] = nd;
    out[5] = k->n_ok; out[6] = k->max_window; out[7] = k->n_ops;
    cset_free(&memo); free(st); free(sid); free(nr); orc_key_free(&kk);
    return 0;
}

/* For the heavy-key pass's order (round 6): the WGL DFS of one key up to `at`
 * inserts (phase 1's hand-over point) -- out: [0] total inserts (to the end,
 * capped by budget), [1] tmax at `at`, [2] inserts when tmax last rose before
 * `at`, [3] depth at `at`, [4] n_ok, [5] verdict. */
int wgl_at(const jh_history *h, const int64_t *sel, int64_t m, int64_t init, int64_t budget, int64_t at, int64_t *out) {
    orc_key kk; orc_key_prepare(h, sel, m, &kk); const orc_key *k = &kk;
    out[0] = out[1] = out[2] = out[3] = 0; out[4] = k->n_ok; out[5] = -1;
    if (k->status || k->n_ok == 0) { orc_key_free(&kk); return -1; }
    cset memo; cset_init(&memo);
    int64_t scap = 256, depth = 0;
    frame *st = (frame *)malloc(sizeof(frame) * scap);
    uint32_t t = 0, tmax = 0; int64_t s = init; int start = 0, snap = 0;
    int64_t last_rise = 0;
    uint64_t mask[MW] = {0};
    int verdict = -1;
    for (;;) {
        if (!snap && memo.n >= at) { out[1] = tmax; out[2] = last_rise; out[3] = depth; snap = 1; }
        const int32_t *W = k->w_ops + k->w_off[t];
        int w = k->w_off[t + 1] - k->w_off[t];
        int took = 0;
        for (int i = start; i < w; i++) {
            if (bit_get(mask, i)) continue;
            const orc_op *o = &k->ops[W[i]];
            int64_t s2;
            if (!cas_step(o->f, o->v1, o->v2, s, &s2)) continue;
            cfg c; c.s = s2;
            cfg_lift(k, t, mask, i, &c.t, c.m);
            if (cset_has(&memo, &c)) continue;
            if (memo.n >= budget) { verdict = JH_UNKNOWN; goto done; }
            cset_add(&memo, &c);
            if (depth == scap) { scap *= 2; st = (frame *)realloc(st, sizeof(frame) * scap); }
            st[depth].t = t; st[depth].i = i; st[depth].s = s; memcpy(st[depth].m, mask, sizeof mask); depth++;
            t = c.t; s = c.s; memcpy(mask, c.m, sizeof mask); start = 0;
            if (t > tmax) { tmax = t; last_rise = memo.n; }
            if (t == (uint32_t)k->n_ok) { verdict = JH_VALID; goto done; }
            took = 1;
            break;
        }
        if (took) continue;
        if (depth == 0) { verdict = JH_INVALID; goto done; }
        depth--;
        t = st[depth].t; s = st[depth].s; memcpy(mask, st[depth].m, sizeof mask); start = st[depth].i + 1;
    }
done:
    if (!snap) { out[1] = tmax; out[2] = last_rise; out[3] = depth; }
    out[0] = memo.n; out[5] = verdict;
    cset_free(&memo); free(st); orc_key_free(&kk);
    return 0;
}
