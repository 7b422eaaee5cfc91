// jh_multi.hip -- several devices behind one jh_ctx (jh_open_multi), and the
// window-sum key cost model that splits keys between them (jh_key_costs).
//
// SURVEY 8(b) "Threading": the JVM opens one context and calls it from any
// thread; multi-GPU fan-out is internal. Keys are independent units
// (jepsen/src/jepsen/independent.clj:1-7, :247-298), so the history is cut by
// key into one sub-history per device -- its keys' rows plus every un-keyed
// row, which subhistory keeps in every key (independent.clj:234-245) -- and
// each device checks its part on its own host thread. The only exchange is the
// summary merge (merge-valid MAX, counts SUM, first failing row MIN), a few
// words, done on the host: no data-path collective.
#include "jh_internal.h"
#include <algorithm>
#include <queue>
#include <mutex>
#include <thread>

namespace {

int host_threads() {
    unsigned n = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(n, 16u));
}

// Per-key search-cost estimate: entries + the window sum, i.e. the sum over
// the key's client ops of the number of :ok returns that fall inside the op's
// window (invocation to completion; a crashed op stays open to the end, which
// is what makes crash-heavy keys expensive). It is the same quantity the
// device prep computes as KeyInfo::sumW (jh_lin.hip), restated on the host
// without pairing: for completed ops, sum of ok-counts at completions minus
// ok-counts at invocations; crashed ops add n_ok - ok-count at invocation.
// One ordered pass per key bucket: rows are bucketed by key % T in history
// order (two parallel passes), then each thread runs the recurrence over its
// own bucket.
void key_costs_host(const jh_history *h, int64_t *cost) {
    const int64_t N = h->n, K = h->n_keys;
    std::fill(cost, cost + K, 0);
    if (N == 0 || K == 0 || !h->key) return;
    const int T = host_threads();
    const int64_t chunk = (N + T - 1) / T;
    std::vector<int64_t> cnt((size_t)T * T, 0);   // [chunk][bucket]
    auto run = [&](auto &&fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(fn, t);
        for (auto &x : th) x.join();
    };
    run([&](int c) {
        const int64_t a = c * chunk, b = std::min(N, a + chunk);
        int64_t *my = &cnt[(size_t)c * T];
        for (int64_t i = a; i < b; ++i) {
            const int64_t k = h->key[i];
            if (k >= 0 && k < K && h->process[i] >= 0) my[k % T]++;
        }
    });
    std::vector<int64_t> off((size_t)T * T), bsize(T, 0);
    for (int bk = 0; bk < T; ++bk)
        for (int c = 0; c < T; ++c) { off[(size_t)c * T + bk] = bsize[bk]; bsize[bk] += cnt[(size_t)c * T + bk]; }
    std::vector<std::vector<int64_t>> rows(T);
    for (int bk = 0; bk < T; ++bk) rows[bk].resize(bsize[bk]);
    run([&](int c) {
        const int64_t a = c * chunk, b = std::min(N, a + chunk);
        std::vector<int64_t> pos(T);
        for (int bk = 0; bk < T; ++bk) pos[bk] = off[(size_t)c * T + bk];
        for (int64_t i = a; i < b; ++i) {
            const int64_t k = h->key[i];
            if (k >= 0 && k < K && h->process[i] >= 0) { const int bk = (int)(k % T); rows[bk][pos[bk]++] = i; }
        }
    });
    run([&](int bk) {
        // per-key state in a dense table indexed by k / T
        const int64_t KB = (K - bk + T - 1) / T;
        std::vector<int64_t> nok(KB, 0), ncrash(KB, 0), ent(KB, 0), acc(KB, 0);
        for (int64_t i : rows[bk]) {
            const int64_t j = h->key[i] / T;
            const int64_t t = h->type[i];
            ent[j]++;
            if (t == JH_TYPE_INVOKE) acc[j] -= nok[j];
            else if (t == JH_TYPE_OK) { nok[j]++; acc[j] += nok[j]; }
            else if (t == JH_TYPE_FAIL) acc[j] += nok[j];
            else if (t == JH_TYPE_INFO) ncrash[j]++;
        }
        for (int64_t j = 0; j < KB; ++j)
            cost[j * T + bk] = ent[j] + std::max<int64_t>(0, acc[j] + ncrash[j] * nok[j]);
    });
}

// LPT: heaviest key first, each to the least-loaded device.
std::vector<int32_t> assign_lpt(const int64_t *cost, int64_t K, int n) {
    std::vector<int64_t> order(K);
    for (int64_t k = 0; k < K; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return cost[a] > cost[b]; });
    using L = std::pair<int64_t, int>;   // (load, device): ties go to the lower device
    std::priority_queue<L, std::vector<L>, std::greater<L>> pq;
    for (int d = 0; d < n; ++d) pq.push({0, d});
    std::vector<int32_t> owner(K);
    for (int64_t k : order) {
        L l = pq.top();
        pq.pop();
        owner[k] = l.second;
        l.first += cost[k];
        pq.push(l);
    }
    return owner;
}

struct SubHist {
    std::vector<int64_t> process, type, f, key, value, value2, row;   // row: global row id
    std::vector<int64_t> keys;                                        // global key of each local key
};

// One sub-history per device, rows in history order. Two parallel passes over
// row chunks: count per (chunk, device), then gather into the offsets.
void split(const jh_history *h, const std::vector<int32_t> &owner, int n, std::vector<SubHist> &sub) {
    const int64_t N = h->n, K = h->n_keys;
    std::vector<int64_t> local(K);
    for (int d = 0; d < n; ++d) sub[d].keys.clear();
    for (int64_t k = 0; k < K; ++k) { local[k] = (int64_t)sub[owner[k]].keys.size(); sub[owner[k]].keys.push_back(k); }
    const int T = host_threads();
    const int64_t chunk = (N + T - 1) / T;
    std::vector<int64_t> cnt((size_t)T * n, 0);
    auto run = [&](auto &&fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(fn, t);
        for (auto &x : th) x.join();
    };
    auto dev_of = [&](int64_t k) { return (k >= 0 && k < K) ? owner[k] : -1; };   // -1: every device
    run([&](int c) {
        const int64_t a = c * chunk, b = std::min(N, a + chunk);
        int64_t *my = &cnt[(size_t)c * n];
        int64_t all = 0;
        for (int64_t i = a; i < b; ++i) {
            const int d = dev_of(h->key ? h->key[i] : -1);
            if (d < 0) all++; else my[d]++;
        }
        for (int d = 0; d < n; ++d) my[d] += all;
    });
    std::vector<int64_t> off((size_t)T * n);
    for (int d = 0; d < n; ++d) {
        int64_t s = 0;
        for (int c = 0; c < T; ++c) { off[(size_t)c * n + d] = s; s += cnt[(size_t)c * n + d]; }
        SubHist &S = sub[d];
        for (auto *v : {&S.process, &S.type, &S.f, &S.key, &S.value, &S.value2, &S.row}) v->resize(s);
    }
    run([&](int c) {
        const int64_t a = c * chunk, b = std::min(N, a + chunk);
        std::vector<int64_t> pos(n);
        for (int d = 0; d < n; ++d) pos[d] = off[(size_t)c * n + d];
        auto put = [&](int d, int64_t i, int64_t lk) {
            SubHist &S = sub[d];
            const int64_t p = pos[d]++;
            S.process[p] = h->process[i]; S.type[p] = h->type[i]; S.f[p] = h->f[i];
            S.key[p] = lk; S.value[p] = h->value[i]; S.value2[p] = h->value2[i]; S.row[p] = i;
        };
        for (int64_t i = a; i < b; ++i) {
            const int64_t k = h->key ? h->key[i] : -1;
            const int d = dev_of(k);
            if (d < 0) for (int e = 0; e < n; ++e) put(e, i, -1);
            else put(d, i, local[k]);
        }
    });
}

}  // namespace

extern "C" {

int jh_key_costs(const jh_history *h, int64_t *cost, char *err, size_t errlen) {
    if (!h || !cost || h->n < 0 || h->n_keys < 0 || h->on_device ||
        (h->n > 0 && (!h->process || !h->type))) {
        if (err && errlen) snprintf(err, errlen, "jh_key_costs: bad arguments (host history needed)");
        return JH_EINVAL;
    }
    try {
        key_costs_host(h, cost);
    } catch (const std::exception &e) {
        if (err && errlen) snprintf(err, errlen, "jh_key_costs: %s", e.what());
        return JH_ENOMEM;
    }
    if (err && errlen) err[0] = 0;
    return JH_OK;
}

int jh_open_devices(const int32_t *devices, int n, jh_ctx **out) {
    if (!out || !devices || n < 1) return JH_EINVAL;
    *out = nullptr;
    if (n == 1) return jh_open(devices[0], out);
    jh_ctx *g = new jh_ctx();
    g->device = -1;
    for (int d = 0; d < n; ++d) {
        jh_ctx *m = nullptr;
        const int rc = jh_open(devices[d], &m);
        if (rc != JH_OK) {
            for (jh_ctx *x : g->members) jh_close(x);
            delete g;
            return rc;
        }
        g->members.push_back(m);
    }
    // members on one device divide its free HBM between them (fit_units):
    // their checks run at once, one host thread each
    for (jh_ctx *m : g->members)
        for (jh_ctx *x : g->members) if (x != m && x->device == m->device) m->share++;
    *out = g;
    return JH_OK;
}

int jh_open_multi(int n_gpus, jh_ctx **out) {
    if (!out) return JH_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return JH_EDEVICE;
    const int n = n_gpus <= 0 ? ndev : n_gpus;
    if (n > ndev) return JH_EINVAL;
    std::vector<int32_t> devs(n);
    for (int d = 0; d < n; ++d) devs[d] = d;
    return jh_open_devices(devs.data(), n, out);
}

int jh_n_devices(const jh_ctx *ctx) {
    if (!ctx) return 0;
    return ctx->members.empty() ? 1 : (int)ctx->members.size();
}

}  // extern "C"

// Two stages (round 3; VERDICT r2: the window-sum cost model cannot see which
// keys are heavy, Spearman 0.04 against WGL's insert count):
//  1. the keys are split by that model (LPT) and every device runs phase 1 on
//     its part (JH_LIN_PHASE1_ONLY): most keys settle under the quick budget,
//     the rest come back deferred;
//  2. the deferred keys of every device are pooled, heaviest estimate first,
//     and the member threads pull batches from the pool (guided
//     self-scheduling: a batch is the pool's remainder over twice the device
//     count, at least one key) and check each batch's sub-history with every
//     key going straight to the heavy-key engines (JH_LIN_SKIP_PHASE1). A
//     device that drew light keys comes back for more, as bounded-pmap's
//     workers do (independent.clj:266-288).
// The verdicts are the single-device ones key by key (the engines are exact);
// the summary is recomputed from them.
namespace {
struct MultiStats {
    std::vector<double> ms;            // per device: device time, stage 1 + stage 2
    std::vector<int64_t> keys2;        // per device: deferred keys checked in stage 2
};

jh_history sub_view(const SubHist &S) {
    jh_history sh{};
    sh.n = (int64_t)S.row.size();
    sh.process = S.process.data(); sh.type = S.type.data(); sh.f = S.f.data();
    sh.key = S.key.data(); sh.value = S.value.data(); sh.value2 = S.value2.data();
    sh.n_keys = (int64_t)S.keys.size();
    return sh;
}
}  // namespace

int multi_check_cas_independent(jh_ctx *g, const jh_history *h, const jh_lin_opts *opts,
                                jh_key_verdict *out, jh_summary *sum, char *err, size_t errlen) {
    const int n = (int)g->members.size();
    if (h->on_device) {
        snprintf(err, errlen, "a multi-device context takes host columns (on_device=0)");
        return JH_EUNSUPPORTED;
    }
    const int64_t K = h->n_keys, N = h->n;
    std::vector<int64_t> cost(K);
    std::vector<SubHist> sub(n);
    try {
        key_costs_host(h, cost.data());
        split(h, assign_lpt(cost.data(), K, n), n, sub);
    } catch (const std::exception &e) {
        snprintf(err, errlen, "multi-device split: %s", e.what());
        return JH_ENOMEM;
    }
    jh_lin_opts o = opts ? *opts : jh_lin_opts{JH_NIL, 0, 0};
    o.stream = 0;                                   // each device runs on its own ctx stream
    const bool two_stage = o.algorithm != JH_ALGO_LINEAR && !(o.flags & (JH_LIN_PHASE1_ONLY | JH_LIN_SKIP_PHASE1));
    jh_lin_opts o1 = o;
    if (two_stage) o1.flags |= JH_LIN_PHASE1_ONLY;
    std::vector<std::vector<jh_key_verdict>> v(n);
    std::vector<jh_summary> s(n);
    std::vector<int> rc(n, JH_OK);
    std::vector<std::string> msg(n);
    MultiStats st{std::vector<double>(n, 0.0), std::vector<int64_t>(n, 0)};
    {
        std::vector<std::thread> th;
        for (int d = 0; d < n; ++d)
            th.emplace_back([&, d] {
                jh_history sh = sub_view(sub[d]);
                v[d].resize(std::max<int64_t>(1, sh.n_keys));
                char e[512];
                rc[d] = jh_check_cas_independent(g->members[d], &sh, &o1, v[d].data(), &s[d], e, sizeof e);
                msg[d] = e;
                st.ms[d] += s[d].device_ms;
            });
        for (auto &x : th) x.join();
    }
    for (int d = 0; d < n; ++d)
        if (rc[d] != JH_OK) {
            snprintf(err, errlen, "device %d: %s", d, msg[d].c_str());
            return rc[d];
        }
    auto place = [&](const SubHist &S, const std::vector<jh_key_verdict> &vv) {
        for (size_t j = 0; j < S.keys.size(); ++j) {
            jh_key_verdict x = vv[j];
            if (x.fail_entry >= 0) x.fail_entry = S.row[x.fail_entry];
            if (x.previous_ok >= 0) x.previous_ok = S.row[x.previous_ok];
            if (x.last_op >= 0) x.last_op = S.row[x.last_op];
            out[S.keys[j]] = x;
        }
    };
    for (int d = 0; d < n; ++d) place(sub[d], v[d]);

    // ---- stage 2: the pooled deferred keys ----
    std::vector<int64_t> pool;
    if (two_stage)
        for (int64_t k = 0; k < K; ++k)
            if (out[k].valid == JH_UNKNOWN && out[k].cause == JH_CAUSE_DEFERRED) pool.push_back(k);
    if (!pool.empty()) {
        // heaviest estimate first by phase 1's progress (stage 1 returns it as
        // `explored` of a deferred key): the window-sum cost ranks the heavy
        // keys no better than chance (Spearman 0.04 on C3)
        std::stable_sort(pool.begin(), pool.end(), [&](int64_t a, int64_t b) { return out[a].explored < out[b].explored; });
        // rows of the pooled keys (and the un-keyed rows every key's subhistory keeps)
        std::vector<int32_t> slot(K, -1);
        for (size_t i = 0; i < pool.size(); ++i) slot[pool[i]] = (int32_t)i;
        std::vector<std::vector<int64_t>> rows(pool.size());
        std::vector<int64_t> unkeyed;
        for (int64_t i = 0; i < N; ++i) {
            const int64_t k = h->key ? h->key[i] : -1;
            if (k < 0 || k >= K) unkeyed.push_back(i);
            else if (slot[k] >= 0) rows[slot[k]].push_back(i);
        }
        std::mutex mu;
        size_t next = 0;
        std::vector<std::thread> th;
        for (int d = 0; d < n; ++d)
            th.emplace_back([&, d] {
                jh_lin_opts o2 = o;
                o2.flags |= JH_LIN_SKIP_PHASE1;
                for (;;) {
                    size_t a, b;
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        if (next >= pool.size() || rc[d] != JH_OK) return;
                        const size_t rest = pool.size() - next;
                        const size_t take = std::max<size_t>(1, rest / (2 * (size_t)n));
                        a = next; b = next + take; next = b;
                    }
                    SubHist S;
                    std::vector<int64_t> rr(unkeyed);
                    std::vector<int64_t> local_of_row;
                    for (size_t i = a; i < b; ++i) {
                        S.keys.push_back(pool[i]);
                        rr.insert(rr.end(), rows[i].begin(), rows[i].end());
                    }
                    std::sort(rr.begin(), rr.end());
                    for (int64_t r : rr) {
                        const int64_t k = h->key ? h->key[r] : -1;
                        int64_t lk = -1;
                        if (k >= 0 && k < K && slot[k] >= 0) lk = (int64_t)slot[k] - (int64_t)a;
                        S.process.push_back(h->process[r]); S.type.push_back(h->type[r]); S.f.push_back(h->f[r]);
                        S.key.push_back(lk); S.value.push_back(h->value[r]); S.value2.push_back(h->value2[r]);
                        S.row.push_back(r);
                    }
                    jh_history sh = sub_view(S);
                    std::vector<jh_key_verdict> vv(std::max<int64_t>(1, sh.n_keys));
                    jh_summary ss;
                    char e[512];
                    const int r = jh_check_cas_independent(g->members[d], &sh, &o2, vv.data(), &ss, e, sizeof e);
                    std::lock_guard<std::mutex> lk(mu);
                    if (r != JH_OK) { rc[d] = r; msg[d] = e; return; }
                    place(S, vv);
                    st.ms[d] += ss.device_ms;
                    st.keys2[d] += (int64_t)(b - a);
                    s[d].seq_probes += ss.seq_probes; s[d].p3_probes += ss.p3_probes;
                    s[d].wide_probes += ss.wide_probes; s[d].helper_probes += ss.helper_probes;
                    s[d].seq_ms += ss.seq_ms; s[d].bfs_ms += ss.bfs_ms; s[d].wide_ms += ss.wide_ms;
                    s[d].p3_ms += ss.p3_ms; s[d].n_phase3 += ss.n_phase3; s[d].n_phase3_wide += ss.n_phase3_wide;
                }
            });
        for (auto &x : th) x.join();
        for (int d = 0; d < n; ++d)
            if (rc[d] != JH_OK) {
                snprintf(err, errlen, "device %d (stage 2): %s", d, msg[d].c_str());
                return rc[d];
            }
    }
    // the summary from the merged verdicts (merge-valid, counts, first failing row)
    jh_summary m{};
    m.first_fail_entry = -1;
    for (int64_t k = 0; k < K; ++k) {
        const jh_key_verdict &x = out[k];
        if (x.explored < 0) continue;                 // a key in no tuple
        m.n_keys++;
        m.explored += x.explored;
        m.valid = std::max<int64_t>(m.valid, x.valid);
        if (x.valid == JH_INVALID) {
            m.n_invalid++;
            if (x.fail_entry >= 0 && (m.first_fail_entry < 0 || x.fail_entry < m.first_fail_entry))
                m.first_fail_entry = x.fail_entry;
        }
        if (x.valid == JH_UNKNOWN) m.n_unknown++;
    }
    for (int d = 0; d < n; ++d) {
        const jh_summary &a = s[d];
        m.memo_probes += a.memo_probes;
        m.n_deferred += a.n_deferred; m.deferred_entries += a.deferred_entries; m.seq_probes += a.seq_probes;
        // devices run concurrently: the call's device time is the slowest device's
        m.device_ms = std::max(m.device_ms, st.ms[d]);
        m.dfs_ms = std::max(m.dfs_ms, a.dfs_ms);
        m.seq_ms = std::max(m.seq_ms, a.seq_ms);
        m.bfs_ms = std::max(m.bfs_ms, a.bfs_ms);
        m.p3_ms = std::max(m.p3_ms, a.p3_ms);
        m.wide_ms = std::max(m.wide_ms, a.wide_ms);
        m.xw_ms = std::max(m.xw_ms, a.xw_ms);
        m.p3_probes += a.p3_probes; m.wide_probes += a.wide_probes; m.xw_probes += a.xw_probes;
        m.helper_probes += a.helper_probes; m.n_deferred_wide += a.n_deferred_wide;
        m.n_phase3 += a.n_phase3; m.n_phase3_wide += a.n_phase3_wide; m.n_xw += a.n_xw;
        m.lean_entries += a.lean_entries; m.wide_entries += a.wide_entries; m.xw_entries += a.xw_entries;
        for (int i = 0; i < 4; i++) m.waves[i] = std::max(m.waves[i], a.waves[i]);
    }
    if (sum) *sum = m;
    if (err && errlen) err[0] = 0;
    return JH_OK;
}
