// gen.cpp -- seeded synthetic Jepsen histories.
//
// Workload and test-data generator: builds columnar histories (include/jh.h
// encoding) shaped like the reference workloads, by an event simulation of
// single-threaded client processes against a true linearizable object:
//   - cas-register per key: jepsen/src/jepsen/tests/linearizable_register.clj:18-53
//     (2n threads per key, n reserved readers, mix [w cas cas], values
//     (rand-int 5), per-key-limit x (0.9 + rand 0.1), process-limit 20),
//     independent/concurrent-generator key groups (independent.clj:130-220);
//   - counter: aerospike/src/aerospike/counter.clj:73-78 (add 1 : read = 100 : 1);
//   - set: adds of distinct integers then one final read (checker.clj:182-233).
// Each op gets a linearization point uniform in [invoke, complete]; the
// object is mutated at that point, so every key without an injected fault
// is linearizable by construction. :info completions (p_info) apply their
// effect with probability 1/2 and rename the process p -> p + concurrency
// (jepsen/src/jepsen/core.clj:349). Nemesis :info pairs with :process
// :nemesis are interleaved (core.clj:266-278).
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
#include <queue>
#include <algorithm>
#include <thread>
#include "../../include/jh.h"

namespace {

struct Rng {  // splitmix64 -> xoshiro256**
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        for (int i = 0; i < 4; i++) {
            seed += 0x9E3779B97F4A7C15ULL;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
            s[i] = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    int64_t below(int64_t n) { return (int64_t)(uni() * (double)n); }
    double expo(double mean) { return -mean * std::log(1.0 - uni()); }
};

struct Out {
    std::vector<int64_t> process, type, f, key, value, value2, aux, truth;
    void push(int64_t p, int64_t ty, int64_t ff, int64_t k, int64_t v, int64_t v2) {
        process.push_back(p); type.push_back(ty); f.push_back(ff); key.push_back(k);
        value.push_back(v); value2.push_back(v2);
    }
};

struct Ev {
    double t; int64_t seq; int32_t th;
    bool operator<(const Ev &o) const { return t > o.t || (t == o.t && seq > o.seq); }
};

}  // namespace

extern "C" {

typedef struct jhg_cas_params {
    int64_t n_keys;            // independent keys (C3: 10000)
    int64_t ops_per_key;       // :per-key-limit in ops (C3: 500 ops ~ 1000 entries)
    int32_t threads_per_key;   // 2n (C3: 10)
    int32_t readers;           // n reserved readers (C3: 5)
    int32_t n_values;          // (rand-int 5)
    int32_t process_limit;     // gen/process-limit (20)
    int32_t groups;            // keys checked concurrently = concurrency / threads_per_key
    int32_t init_nil;          // 1: (cas-register) ; 0: (cas-register 0)
    double p_info;             // :info completions
    double p_invalid;          // keys with one injected stale read
    int64_t nemesis_every;     // emit a nemesis :info pair every so many entries (0: none)
    uint64_t seed;
    int32_t keyed;             // 1: [k v] tuples; 0: single register, key column -1
    int32_t pad;
} jhg_cas_params;

typedef struct jhg_hist {
    int64_t n, n_aux, n_keys;
    int64_t *process, *type, *f, *key, *value, *value2, *aux;
    int64_t *truth;            // per key: 1 if a fault was injected
    void *impl;
} jhg_hist;

static void export_out(Out *o, jhg_hist *h, int64_t n_keys) {
    h->n = (int64_t)o->process.size(); h->n_aux = (int64_t)o->aux.size(); h->n_keys = n_keys;
    h->process = o->process.data(); h->type = o->type.data(); h->f = o->f.data();
    h->key = o->key.data(); h->value = o->value.data(); h->value2 = o->value2.data();
    h->aux = o->aux.data(); h->truth = o->truth.data(); h->impl = o;
}

void jhg_free(jhg_hist *h) {
    delete (Out *)h->impl;
    memset(h, 0, sizeof(*h));
}

int jhg_cas(const jhg_cas_params *P, jhg_hist *h) {
    Rng rng(P->seed);
    Out *o = new Out();
    const int T = P->threads_per_key;
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(P->groups, P->n_keys));
    const int64_t C = (int64_t)G * T;               // test :concurrency
    const double mean = 1.0, think = 0.05;
    const int64_t NIL = JH_NIL;
    o->truth.assign(P->n_keys, 0);
    o->process.reserve(P->n_keys * P->ops_per_key * 2 + 1024);

    struct Th { int64_t proc; int phase; bool stopped; int32_t f; int64_t v1, v2, res;
                bool info, applied, fail; double tc; };
    struct Gr { int64_t key = -1; int64_t issued = 0, limit = 0, done = 0, inject_at = -1;
                std::vector<int64_t> procs; int64_t reg = 0; int64_t prev = 0; int stopped = 0; };
    std::vector<Th> th(C);
    std::vector<Gr> gr(G);
    for (int64_t i = 0; i < C; i++) { th[i].proc = i; th[i].phase = 0; th[i].stopped = false; }
    std::priority_queue<Ev> pq;
    int64_t seq = 0, next_key = 0, emitted_since_nem = 0, nem_start = 1;

    auto start_key = [&](int g, double t) {
        Gr &G_ = gr[g];
        if (next_key >= P->n_keys) { G_.key = -1; return; }
        G_.key = next_key++;
        G_.issued = 0; G_.done = 0;
        G_.limit = (int64_t)std::floor(P->ops_per_key * (0.9 + 0.1 * rng.uni()));
        if (G_.limit < 1) G_.limit = 1;
        G_.procs.clear();
        G_.reg = P->init_nil ? NIL : 0; G_.prev = G_.reg;
        G_.inject_at = rng.uni() < P->p_invalid ? G_.limit / 2 : -1;
        if (G_.inject_at >= 0) o->truth[G_.key] = 1;
        G_.stopped = 0;
        for (int j = 0; j < T; j++) {
            int64_t id = (int64_t)g * T + j;
            th[id].stopped = false; th[id].phase = 0;
            pq.push({t + 0.01 * rng.uni(), seq++, (int32_t)id});
        }
    };
    for (int g = 0; g < G; g++) start_key(g, 0.5 * rng.uni() * g);

    auto emit_nemesis = [&]() {
        if (P->nemesis_every <= 0) return;
        if (++emitted_since_nem < P->nemesis_every) return;
        emitted_since_nem = 0;
        int64_t f = nem_start ? 16 : 17;           // :start / :stop, interned
        nem_start ^= 1;
        o->push(-1, JH_TYPE_INFO, f, -1, NIL, NIL);
        o->push(-1, JH_TYPE_INFO, f, -1, NIL, NIL);
    };
    auto keycol = [&](int64_t k) { return P->keyed ? k : (int64_t)-1; };

    while (!pq.empty()) {
        Ev e = pq.top(); pq.pop();
        Th &x = th[e.th];
        int g = e.th / T, j = e.th % T;
        Gr &G_ = gr[g];
        if (G_.key < 0) continue;
        if (x.phase == 0) {
            bool new_proc = std::find(G_.procs.begin(), G_.procs.end(), x.proc) == G_.procs.end();
            if (G_.issued >= G_.limit || (new_proc && (int64_t)G_.procs.size() >= P->process_limit)) {
                x.stopped = true;
                if (++G_.stopped == T) start_key(g, e.t + 0.1);   // group moves to the next key
                continue;
            }
            if (new_proc) G_.procs.push_back(x.proc);
            G_.issued++;
            if (j < P->readers) { x.f = JH_F_READ; x.v1 = NIL; x.v2 = NIL; }
            else {
                int64_t pick = rng.below(3);
                if (pick == 0) { x.f = JH_F_WRITE; x.v1 = rng.below(P->n_values); x.v2 = NIL; }
                else { x.f = JH_F_CAS; x.v1 = rng.below(P->n_values); x.v2 = rng.below(P->n_values); }
            }
            x.info = rng.uni() < P->p_info;
            x.applied = !x.info || rng.uni() < 0.5;
            double d = rng.expo(mean);
            double tl = e.t + rng.uni() * d;
            x.tc = e.t + d;
            o->push(x.proc, JH_TYPE_INVOKE, x.f, keycol(G_.key), x.v1, x.v2);
            emit_nemesis();
            x.phase = 1;
            pq.push({tl, seq++, e.th});
        } else if (x.phase == 1) {
            x.fail = false; x.res = NIL;
            if (x.applied) {
                if (x.f == JH_F_READ) x.res = G_.reg;
                else if (x.f == JH_F_WRITE) { if (G_.reg != x.v1) G_.prev = G_.reg; G_.reg = x.v1; }
                else {
                    if (G_.reg == x.v1) { if (G_.reg != x.v2) G_.prev = G_.reg; G_.reg = x.v2; }
                    else x.fail = true;
                }
            }
            x.phase = 2;
            pq.push({x.tc, seq++, e.th});
        } else {
            int64_t k = keycol(G_.key);
            if (x.info) {
                o->push(x.proc, JH_TYPE_INFO, x.f, k, x.v1, x.v2);
                x.proc += C;                                   // core.clj:349
            } else if (x.f == JH_F_READ) {
                int64_t v = x.res;
                if (G_.inject_at >= 0 && G_.done >= G_.inject_at) {
                    // one stale read: a value the register does not hold now
                    // half the faults read a value no op ever wrote (a corrupt
                    // read), half the register's previous value (a stale read,
                    // which concurrent writes can still explain)
                    int64_t nv = G_.prev;
                    if (rng.uni() < 0.5) nv = P->n_values;
                    else if (nv == v || nv == NIL) nv = (v == NIL ? 0 : (v + 1 + rng.below(P->n_values - 1)) % P->n_values);
                    v = nv; G_.inject_at = -1;
                }
                o->push(x.proc, JH_TYPE_OK, x.f, k, v, NIL);
            } else if (x.fail) {
                o->push(x.proc, JH_TYPE_FAIL, x.f, k, x.v1, x.v2);
            } else {
                o->push(x.proc, JH_TYPE_OK, x.f, k, x.v1, x.v2);
            }
            emit_nemesis();
            G_.done++;
            x.phase = 0;
            pq.push({x.tc + think * (0.5 + rng.uni()), seq++, e.th});
        }
    }
    export_out(o, h, P->keyed ? P->n_keys : 0);
    return 0;
}

typedef struct jhg_counter_params {
    int64_t n_ops;             // operations (entries ~ 2 x n_ops)
    int32_t n_procs;
    int32_t read_every;        // 1 read per read_every ops (101 -> 100:1)
    double p_fail, p_info;
    int64_t n_bad_reads;       // invalid variant: out-of-bounds reads
    uint64_t seed;
} jhg_counter_params;

int jhg_counter(const jhg_counter_params *P, jhg_hist *h) {
    Rng rng(P->seed);
    Out *o = new Out();
    const int64_t NIL = JH_NIL;
    const int N = P->n_procs;
    o->process.reserve(P->n_ops * 2 + 16); o->type.reserve(P->n_ops * 2 + 16);
    o->f.reserve(P->n_ops * 2 + 16); o->key.reserve(P->n_ops * 2 + 16);
    o->value.reserve(P->n_ops * 2 + 16); o->value2.reserve(P->n_ops * 2 + 16);
    struct Th { int64_t proc; int phase; int32_t f; int64_t v, res; bool info, applied, fail; double tc; };
    std::vector<Th> th(N);
    std::priority_queue<Ev> pq;
    int64_t seq = 0, issued = 0, counter = 0;
    for (int i = 0; i < N; i++) { th[i].proc = i; th[i].phase = 0; pq.push({rng.uni() * 0.1, seq++, i}); }
    // choose which reads are corrupted: every k-th read after the midpoint
    int64_t approx_reads = P->n_ops / std::max(1, P->read_every);
    int64_t bad_stride = P->n_bad_reads > 0 ? std::max<int64_t>(1, approx_reads / (4 * P->n_bad_reads)) : 0;
    int64_t reads_done = 0, bad_left = P->n_bad_reads;
    while (!pq.empty()) {
        Ev e = pq.top(); pq.pop();
        Th &x = th[e.th];
        if (x.phase == 0) {
            if (issued >= P->n_ops) continue;
            issued++;
            bool rd = rng.below(P->read_every) == 0;
            x.f = rd ? JH_F_READ : JH_F_ADD; x.v = rd ? NIL : 1;
            x.info = rng.uni() < P->p_info;
            x.fail = !x.info && !rd && rng.uni() < P->p_fail;
            x.applied = !x.fail && (!x.info || rng.uni() < 0.5);
            double d = rng.expo(1.0);
            x.tc = e.t + d;
            o->push(x.proc, JH_TYPE_INVOKE, x.f, -1, x.v, NIL);
            x.phase = 1;
            pq.push({e.t + rng.uni() * d, seq++, e.th});
        } else if (x.phase == 1) {
            if (x.applied) { if (x.f == JH_F_ADD) counter += x.v; else x.res = counter; }
            x.phase = 2;
            pq.push({x.tc, seq++, e.th});
        } else {
            if (x.info) { o->push(x.proc, JH_TYPE_INFO, x.f, -1, x.v, NIL); x.proc += N; }
            else if (x.fail) o->push(x.proc, JH_TYPE_FAIL, x.f, -1, x.v, NIL);
            else if (x.f == JH_F_READ) {
                int64_t v = x.res;
                reads_done++;
                if (bad_left > 0 && reads_done > approx_reads / 2 && bad_stride && reads_done % bad_stride == 0) {
                    // below every lower bound past the midpoint (the :info adds
                    // widen [lower, upper] without limit, so "v + k" need not be
                    // out of bounds in a long history)
                    v = -bad_left; bad_left--;
                }
                o->push(x.proc, JH_TYPE_OK, x.f, -1, v, NIL);
            } else o->push(x.proc, JH_TYPE_OK, x.f, -1, x.v, NIL);
            x.phase = 0;
            pq.push({x.tc + 0.05 * rng.uni(), seq++, e.th});
        }
    }
    export_out(o, h, 0);
    return 0;
}

typedef struct jhg_set_params {
    int64_t n_adds;
    int32_t n_procs;
    int32_t pad;
    double p_fail, p_info;
    int64_t n_lost, n_unexpected;   // invalid variant
    uint64_t seed;
} jhg_set_params;

int jhg_set(const jhg_set_params *P, jhg_hist *h) {
    Rng rng(P->seed);
    Out *o = new Out();
    const int64_t NIL = JH_NIL;
    const int N = P->n_procs;
    struct Th { int64_t proc; int phase; int64_t v; bool info, applied, fail; double tc; };
    std::vector<Th> th(N);
    std::priority_queue<Ev> pq;
    int64_t seq = 0, issued = 0;
    std::vector<uint8_t> in_set(P->n_adds, 0), acked(P->n_adds, 0);
    for (int i = 0; i < N; i++) { th[i].proc = i; th[i].phase = 0; pq.push({rng.uni() * 0.1, seq++, i}); }
    double tend = 0;
    while (!pq.empty()) {
        Ev e = pq.top(); pq.pop();
        Th &x = th[e.th];
        if (e.t > tend) tend = e.t;
        if (x.phase == 0) {
            if (issued >= P->n_adds) continue;
            x.v = issued++;
            x.info = rng.uni() < P->p_info;
            x.fail = !x.info && rng.uni() < P->p_fail;
            x.applied = !x.fail && (!x.info || rng.uni() < 0.5);
            double d = rng.expo(1.0);
            x.tc = e.t + d;
            o->push(x.proc, JH_TYPE_INVOKE, JH_F_ADD, -1, x.v, NIL);
            x.phase = 1;
            pq.push({e.t + rng.uni() * d, seq++, e.th});
        } else if (x.phase == 1) {
            if (x.applied) in_set[x.v] = 1;
            x.phase = 2;
            pq.push({x.tc, seq++, e.th});
        } else {
            if (x.info) { o->push(x.proc, JH_TYPE_INFO, JH_F_ADD, -1, x.v, NIL); x.proc += N; }
            else if (x.fail) o->push(x.proc, JH_TYPE_FAIL, JH_F_ADD, -1, x.v, NIL);
            else { o->push(x.proc, JH_TYPE_OK, JH_F_ADD, -1, x.v, NIL); acked[x.v] = 1; }
            x.phase = 0;
            pq.push({x.tc + 0.05 * rng.uni(), seq++, e.th});
        }
    }
    // drop n_lost acknowledged elements (spread out), add n_unexpected values
    int64_t lost_left = P->n_lost;
    int64_t stride = P->n_lost > 0 ? std::max<int64_t>(1, P->n_adds / (P->n_lost + 1)) : 0;
    for (int64_t v = stride; lost_left > 0 && v < P->n_adds; v += stride) {
        int64_t w = v;
        while (w < P->n_adds && !acked[w]) w++;
        if (w < P->n_adds && in_set[w]) { in_set[w] = 0; lost_left--; }
    }
    for (int64_t v = 0; v < P->n_adds; v++) if (in_set[v]) o->aux.push_back(v);
    for (int64_t i = 0; i < P->n_unexpected; i++) o->aux.push_back(P->n_adds + 7 + 3 * i);
    // shuffle the read's element order: the checker must not rely on it
    for (int64_t i = (int64_t)o->aux.size() - 1; i > 0; i--) std::swap(o->aux[i], o->aux[rng.below(i + 1)]);
    o->push(0, JH_TYPE_INVOKE, JH_F_READ, -1, NIL, NIL);
    o->push(0, JH_TYPE_OK, JH_F_READ, -1, 0, (int64_t)o->aux.size());
    // the final read's process 0 may still be open if its last add crashed:
    // use a fresh process id instead
    int64_t fresh = 0;
    for (auto &t : th) fresh = std::max(fresh, t.proc);
    o->process[o->process.size() - 1] = fresh + 1;
    o->process[o->process.size() - 2] = fresh + 1;
    export_out(o, h, 0);
    return 0;
}

/* A large independent history built from `parts` sub-histories generated in
 * parallel (one host thread each): part i holds keys [i*K/parts, (i+1)*K/parts)
 * and is simulated with seed P->seed * 1000003 + i, as if `parts` groups of
 * keys had run side by side; the parts are concatenated (each key's entries
 * stay in their own part's order, which is all the per-key checkers read).
 * For the 1M-key C4 history, whose single-threaded event simulation would take
 * minutes. truth[k] is per global key. */
int jhg_cas_par(const jhg_cas_params *P, int32_t parts, jhg_hist *h) {
    if (parts < 1) parts = 1;
    if (parts > P->n_keys) parts = (int32_t)std::max<int64_t>(1, P->n_keys);
    std::vector<jhg_hist> sub(parts);
    std::vector<jhg_cas_params> sp(parts, *P);
    std::vector<int64_t> k0(parts + 1);
    for (int i = 0; i <= parts; i++) k0[i] = P->n_keys * i / parts;
    std::vector<std::thread> ts;
    for (int i = 0; i < parts; i++) {
        sp[i].n_keys = k0[i + 1] - k0[i];
        sp[i].seed = P->seed * 1000003ULL + (uint64_t)i;
        memset(&sub[i], 0, sizeof sub[i]);
        ts.emplace_back([&, i] { jhg_cas(&sp[i], &sub[i]); });
    }
    for (auto &t : ts) t.join();
    Out *o = new Out();
    int64_t n = 0;
    for (auto &x : sub) n += x.n;
    for (auto *v : {&o->process, &o->type, &o->f, &o->key, &o->value, &o->value2}) v->resize(n);
    o->truth.assign(P->n_keys, 0);
    std::vector<int64_t> r0(parts + 1, 0);
    for (int i = 0; i < parts; i++) r0[i + 1] = r0[i] + sub[i].n;
    ts.clear();
    for (int i = 0; i < parts; i++) {
        ts.emplace_back([&, i] {
            const jhg_hist &x = sub[i];
            const int64_t b = r0[i];
            memcpy(o->process.data() + b, x.process, 8 * x.n);
            memcpy(o->type.data() + b, x.type, 8 * x.n);
            memcpy(o->f.data() + b, x.f, 8 * x.n);
            memcpy(o->value.data() + b, x.value, 8 * x.n);
            memcpy(o->value2.data() + b, x.value2, 8 * x.n);
            for (int64_t r = 0; r < x.n; r++) o->key[b + r] = x.key[r] >= 0 ? x.key[r] + k0[i] : x.key[r];
            // process ids repeat across parts: every op of a part completes
            // (or crashes and renames its process) before the next part starts
            if (P->keyed) memcpy(o->truth.data() + k0[i], x.truth, 8 * (k0[i + 1] - k0[i]));
            jhg_free(&sub[i]);
        });
    }
    for (auto &t : ts) t.join();
    export_out(o, h, P->keyed ? P->n_keys : 0);
    return 0;
}

}  // extern "C"
