// jh_api.hip -- the C ABI of libjh.so (include/jh.h).
//
// Every entry point: validates arguments, takes the context mutex (the JVM
// side may call from compose's pmap and independent's bounded-pmap threads,
// jepsen/src/jepsen/checker.clj:98-101, independent.clj:266-275), stages host
// columns into HBM once, runs the device pipeline, and converts exceptions
// into a JH_* code plus a message (check-safe, checker.clj:77-88, turns the
// shim's ex-info into {:valid? :unknown :error ...}).
#include "jh_internal.h"
#include <algorithm>
#include <unordered_map>
#include <vector>

static void set_err(char *err, size_t errlen, const std::string &msg) {
    if (!err || errlen == 0) return;
    size_t k = std::min(errlen - 1, msg.size());
    memcpy(err, msg.data(), k);
    err[k] = 0;
}

template <class F>
static int guarded(char *err, size_t errlen, F &&f) {
    try {
        f();
        set_err(err, errlen, "");
        return JH_OK;
    } catch (const JhException &e) {
        set_err(err, errlen, e.msg);
        return e.code;
    } catch (const std::exception &e) {
        set_err(err, errlen, std::string("internal error: ") + e.what());
        return JH_EDEVICE;
    }
}

static const int64_t *stage_col(jh_ctx *ctx, int slot, const int64_t *src, int64_t n, hipStream_t st) {
    if (!src) return nullptr;
    int64_t *d = ctx->ws<int64_t>(slot, n);
    if (n > 0) HIP_TRY(hipMemcpyAsync(d, src, sizeof(int64_t) * n, hipMemcpyHostToDevice, st));
    return d;
}

jh_history stage_history(jh_ctx *ctx, const jh_history *h, bool need_key, bool need_aux) {
    if (h->on_device) return *h;
    jh_history d = *h;
    hipStream_t st = ctx->stream;
    if (h->n > 0) {
        // large histories: packed chunks, packing overlapped with the DMA (jh_ingest.hip)
        const int64_t *src[7] = {h->process, h->type, h->f, need_key ? h->key : nullptr, h->value, h->value2, nullptr};
        int64_t *dst[7] = {};
        const int slot[7] = {WS_COL_PROCESS, WS_COL_TYPE, WS_COL_F, WS_COL_KEY, WS_COL_VALUE, WS_COL_VALUE2, WS_COL_AUX};
        for (int c = 0; c < 6; c++)
            if (src[c]) dst[c] = ctx->ws<int64_t>(slot[c], h->n);
        if (ingest_columns(ctx, src, dst, h->n, st)) {
            d.process = dst[0]; d.type = dst[1]; d.f = dst[2]; d.key = dst[3];
            d.value = dst[4]; d.value2 = dst[5];
            d.aux = need_aux ? stage_col(ctx, WS_COL_AUX, h->aux, h->n_aux, st) : nullptr;
            d.on_device = 1;
            return d;
        }
    }
    d.process = stage_col(ctx, WS_COL_PROCESS, h->process, h->n, st);
    d.type = stage_col(ctx, WS_COL_TYPE, h->type, h->n, st);
    d.f = stage_col(ctx, WS_COL_F, h->f, h->n, st);
    d.key = need_key ? stage_col(ctx, WS_COL_KEY, h->key, h->n, st) : nullptr;
    d.value = stage_col(ctx, WS_COL_VALUE, h->value, h->n, st);
    d.value2 = stage_col(ctx, WS_COL_VALUE2, h->value2, h->n, st);
    d.aux = need_aux ? stage_col(ctx, WS_COL_AUX, h->aux, h->n_aux, st) : nullptr;
    d.on_device = 1;
    return d;
}

static void check_hist(const jh_history *h) {
    if (!h) throw_jh(JH_EINVAL, "null history");
    if (h->n < 0) throw_jh(JH_EINVAL, "negative entry count");
    if (h->n > 0 && (!h->process || !h->type || !h->f || !h->value || !h->value2))
        throw_jh(JH_EINVAL, "missing history column");
    if (h->n_keys < 0) throw_jh(JH_EINVAL, "negative key count");
}

// a multi-device context (jh_open_multi) shards the independent checks over
// its devices; the single-history checkers run on its first device
static jh_ctx *primary(jh_ctx *c) { return c->members.empty() ? c : c->members[0]; }

int multi_check_cas_independent(jh_ctx *g, const jh_history *h, const jh_lin_opts *opts,
                                jh_key_verdict *out, jh_summary *sum, char *err, size_t errlen);

static std::mutex g_open_mu;
static int g_open[256];              // open single-device contexts per device id
static void device_open_delta(int device, int d) {
    if (device < 0 || device >= 256) return;
    std::lock_guard<std::mutex> g(g_open_mu);
    g_open[device] += d;
}
int device_open_contexts(int device) {
    if (device < 0 || device >= 256) return 1;
    std::lock_guard<std::mutex> g(g_open_mu);
    return std::max(1, g_open[device]);
}

extern "C" {

int jh_version(void) { return JH_ABI_VERSION; }

int jh_open(int device, jh_ctx **out) {
    if (!out) return JH_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return JH_EDEVICE;
    if (device < 0 || device >= ndev) return JH_EINVAL;
    jh_ctx *c = new jh_ctx();
    c->device = device;
    try {
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->aux2, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->aux3, hipStreamNonBlocking));
        for (auto &e : c->ev) HIP_TRY(hipEventCreate(&e));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, device));
        c->n_cu = prop.multiProcessorCount;
    } catch (const JhException &e) {
        delete c;
        return e.code;
    }
    device_open_delta(device, 1);
    *out = c;
    return JH_OK;
}

void jh_close(jh_ctx *ctx) {
    if (!ctx) return;
    if (!ctx->members.empty()) {
        for (jh_ctx *m : ctx->members) jh_close(m);
        delete ctx;
        return;
    }
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        (void)hipSetDevice(ctx->device);
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        for (auto &b : ctx->bufs) if (b.p) (void)hipFree(b.p);
        if (ctx->hflag) (void)hipHostFree(ctx->hflag);
        if (ctx->ingest) ingest_free(ctx->ingest);
        for (auto &e : ctx->ev) if (e) (void)hipEventDestroy(e);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
        if (ctx->aux2) (void)hipStreamDestroy(ctx->aux2);
        if (ctx->aux3) (void)hipStreamDestroy(ctx->aux3);
    }
    device_open_delta(ctx->device, -1);
    delete ctx;
}

int jh_check_cas_independent(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts,
                             jh_key_verdict *out, jh_summary *sum, char *err, size_t errlen) {
    if (!ctx || !out) { set_err(err, errlen, "null context or output"); return JH_EINVAL; }
    if (!ctx->members.empty()) {
        char e[512] = "";
        int rc = guarded(e, sizeof e, [&] { check_hist(h); });
        if (rc == JH_OK) rc = multi_check_cas_independent(ctx, h, opts, out, sum, e, sizeof e);
        set_err(err, errlen, e);
        return rc;
    }
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        jh_history d = stage_history(ctx, h, true, false);
        const int64_t K = h->n_keys;
        jh_key_verdict *dv = ctx->ws<jh_key_verdict>(WS_VERDICT, std::max<int64_t>(K, 1));
        if (K == 0) {
            if (sum) { memset(sum, 0, sizeof *sum); sum->first_fail_entry = -1; }
            return;
        }
        lin_check_independent(ctx, &d, opts, true, dv, sum, st);
        HIP_TRY(hipMemcpyAsync(out, dv, sizeof(jh_key_verdict) * K, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    });
}

int jh_check_cas_independent_device(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts,
                                    jh_key_verdict *out_dev, jh_summary *sum, char *err,
                                    size_t errlen) {
    if (!ctx || !out_dev) { set_err(err, errlen, "null context or output"); return JH_EINVAL; }
    ctx = primary(ctx);   // device pointers live on one device: the first
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        if (!h->on_device) throw_jh(JH_EINVAL, "jh_check_cas_independent_device needs on_device=1");
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = opts && opts->stream ? (hipStream_t)(intptr_t)opts->stream : ctx->stream;
        if (h->n_keys == 0) {
            if (sum) { memset(sum, 0, sizeof *sum); sum->first_fail_entry = -1; }
            return;
        }
        lin_check_independent(ctx, h, opts, true, out_dev, sum, st);
    });
}

__global__ void k_cfg_slots(const int64_t *__restrict__ keys, int n, int64_t K, int32_t *slot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && keys[i] >= 0 && keys[i] < K) slot[keys[i]] = i;
}

// Round 6: the reads the search drops -- a crashed
// :read, an :ok :read of nil; they constrain nothing -- are ops knossos'
// analysis holds (checker.clj:156-158 passes it through). Each configuration
// printed is the one knossos holds in which such a read is linearized exactly
// when its own completion forces it, and never otherwise: a read invoked
// before the configuration's point (the failing op's completion for a
// frontier, the end of the history for final configurations) and not
// completed there -- a crashed read always -- is pending, in call order among
// the others (the row list stays within JH_MAX_WINDOW), and an :ok read of nil
// completing before the point and after the configuration's own :last-op is
// its :last-op. The oracle restates this (oracle/jh_oracle.c add_noop_reads);
// the pairing is knossos.history/complete's, as the device's key pass does it.
struct NoopRead { int64_t call, ret; };            // ret: :ok completion row, INT64_MAX crashed
static std::vector<std::vector<NoopRead>> noop_reads(const jh_history *h, bool keyed, const int64_t *keys, int nq) {
    const int64_t n = h->n;
    std::vector<int64_t> pr, ty, fc, va, ke;
    const int64_t *P = h->process, *T = h->type, *F = h->f, *V = h->value, *KC = keyed ? h->key : nullptr;
    if (h->on_device) {
        auto fetch = [&](std::vector<int64_t> &v, const int64_t *src) {
            v.resize((size_t)std::max<int64_t>(n, 1));
            if (n) HIP_TRY(hipMemcpy(v.data(), src, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
            return (const int64_t *)v.data();
        };
        P = fetch(pr, P); T = fetch(ty, T); F = fetch(fc, F); V = fetch(va, V);
        if (KC) KC = fetch(ke, KC);
    }
    std::unordered_map<int64_t, std::vector<int>> want;     // key -> queries
    for (int i = 0; i < nq; i++) want[keyed ? keys[i] : 0].push_back(i);
    std::vector<std::unordered_map<int64_t, int64_t>> open(nq);   // per query: process -> open invocation
    std::vector<std::vector<NoopRead>> out(nq);
    auto row = [&](int q, int64_t r) {
        const int64_t p = P[r];
        if (p < 0) return;
        auto it = open[q].find(p);
        if (T[r] == JH_TYPE_INVOKE) { open[q][p] = r; return; }
        if (T[r] != JH_TYPE_OK && T[r] != JH_TYPE_FAIL) return;          // :info leaves it open
        if (it == open[q].end()) return;
        const int64_t iv = it->second;
        open[q].erase(it);
        if (T[r] == JH_TYPE_OK && F[iv] == JH_F_READ && (V[iv] != JH_NIL ? V[iv] : V[r]) == JH_NIL)
            out[q].push_back({iv, r});
    };
    static const std::vector<int> none;
    for (int64_t r = 0; r < n; r++) {
        const int64_t k = KC ? KC[r] : 0;
        if (k < 0) { for (int q = 0; q < nq; q++) row(q, r); continue; }   // un-keyed rows: every key's
        auto w = want.find(k);
        if (w != want.end()) for (int q : w->second) row(q, r);
    }
    for (int q = 0; q < nq; q++) {
        for (auto &o : open[q]) if (F[o.second] == JH_F_READ) out[q].push_back({o.second, INT64_MAX});
        std::sort(out[q].begin(), out[q].end(), [](const NoopRead &a, const NoopRead &b) { return a.call < b.call; });
    }
    return out;
}

int jh_lin_configs(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts, const int64_t *keys,
                   int64_t n_keys_q, int32_t per_key, jh_lin_config *out, int32_t *n_out, int64_t *rows_out,
                   int64_t rows_cap, char *err, size_t errlen) {
    if (!ctx || !keys || !out || !n_out || !rows_out) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    if (per_key < 1 || per_key > 16) { set_err(err, errlen, "per_key must be in 1..16"); return JH_EINVAL; }
    if (n_keys_q < 0 || n_keys_q > (1 << 20)) { set_err(err, errlen, "bad number of keys"); return JH_EINVAL; }
    if (rows_cap < n_keys_q * per_key * JH_MAX_WINDOW) { set_err(err, errlen, "rows_cap < n_keys_q * per_key * JH_MAX_WINDOW"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        const bool keyed = h->key != nullptr && h->n_keys > 0;
        jh_history d = stage_history(ctx, h, keyed, false);
        if (!keyed) { d.key = nullptr; d.n_keys = 1; }
        const int64_t K = d.n_keys;
        for (int64_t i = 0; i < n_keys_q; i++) n_out[i] = -1;
        if (n_keys_q == 0 || K == 0) return;
        const int nq = (int)n_keys_q;
        int32_t *slot = ctx->ws<int32_t>(WS_CFG_SLOT, K);
        int64_t *kd = ctx->ws<int64_t>(WS_CFG_KEYS, nq);
        jh_lin_config *co = ctx->ws<jh_lin_config>(WS_CFG_OUT, (size_t)nq * per_key);
        int32_t *cn = ctx->ws<int32_t>(WS_CFG_N, nq);
        int64_t *cr = ctx->ws<int64_t>(WS_CFG_ROWS, (size_t)nq * per_key * JH_MAX_WINDOW);
        HIP_TRY(hipMemsetAsync(slot, 0xFF, sizeof(int32_t) * K, st));
        HIP_TRY(hipMemsetAsync(cn, 0xFF, sizeof(int32_t) * nq, st));
        HIP_TRY(hipMemcpyAsync(kd, keys, sizeof(int64_t) * nq, hipMemcpyHostToDevice, st));
        k_cfg_slots<<<(nq + 255) / 256, 256, 0, st>>>(kd, nq, K, slot);
        jh_key_verdict *dv = ctx->ws<jh_key_verdict>(WS_VERDICT, std::max<int64_t>(K, 1));
        LinCfgReq req{kd, nq, per_key, slot, co, cn, cr};
        lin_check_independent(ctx, &d, opts, keyed, dv, nullptr, st, &req);
        std::vector<jh_lin_config> hc((size_t)nq * per_key);
        std::vector<int64_t> hr((size_t)nq * per_key * JH_MAX_WINDOW);
        HIP_TRY(hipMemcpyAsync(n_out, cn, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hc.data(), co, sizeof(jh_lin_config) * hc.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hr.data(), cr, sizeof(int64_t) * hr.size(), hipMemcpyDeviceToHost, st));
        std::vector<jh_key_verdict> hv((size_t)K);
        HIP_TRY(hipMemcpyAsync(hv.data(), dv, sizeof(jh_key_verdict) * K, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const auto noop = noop_reads(h, keyed, keys, nq);
        // compact: configuration j of key i keeps slot i * per_key + j; its rows
        // move up, the dropped reads join :pending (noop_reads above)
        int64_t w = 0;
        for (int i = 0; i < nq; i++)
            for (int j = 0; j < per_key; j++) {
                jh_lin_config &c = out[(size_t)i * per_key + j];
                if (j >= n_out[i]) { memset(&c, 0, sizeof c); c.key = keys[i]; c.rows_off = w; continue; }
                c = hc[(size_t)i * per_key + j];
                const int64_t nl = c.n_linearized, np0 = c.n_pending;
                memcpy(rows_out + w, hr.data() + c.rows_off, sizeof(int64_t) * (nl + np0));
                const jh_key_verdict &v = hv[(size_t)(keyed ? keys[i] : 0)];
                const int64_t pt = v.valid == JH_INVALID ? v.fail_entry : INT64_MAX - 1;
                int64_t np = np0;
                for (const NoopRead &o : noop[i]) {
                    if (o.ret != INT64_MAX && o.ret < pt && o.ret > c.last_row) c.last_row = o.ret;
                    if (o.call < pt && o.ret > pt && nl + np < JH_MAX_WINDOW) rows_out[w + nl + np++] = o.call;
                }
                std::sort(rows_out + w + nl, rows_out + w + nl + np);
                c.n_pending = (int32_t)np;
                c.rows_off = w;
                w += nl + np;
            }
    });
}

int jh_stage_history(jh_ctx *ctx, const jh_history *h, int64_t *out, char *err, size_t errlen) {
    if (!ctx || !out) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        if (h->on_device) throw_jh(JH_EINVAL, "jh_stage_history takes a host history");
        HIP_TRY(hipSetDevice(ctx->device));
        const jh_history d = stage_history(ctx, h, h->key != nullptr, false);
        const int64_t *cols[6] = {d.process, d.type, d.f, d.key, d.value, d.value2};
        for (int c = 0; c < 6; c++)
            if (cols[c] && h->n > 0)
                HIP_TRY(hipMemcpyAsync(out + (size_t)c * h->n, cols[c], sizeof(int64_t) * h->n, hipMemcpyDeviceToHost,
                                       ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    });
}

int jh_key_index(jh_ctx *ctx, const jh_history *h, int64_t *key_off, int64_t *rows, char *err,
                 size_t errlen) {
    if (!ctx || !key_off || (!rows && h && h->n > 0)) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        if (!h || h->n < 0 || h->n_keys < 0) throw_jh(JH_EINVAL, "bad history");
        if (h->n > 0 && !h->key) throw_jh(JH_EINVAL, "jh_key_index needs the key column");
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = *h;
        if (!h->on_device) d.key = stage_col(ctx, WS_COL_KEY, h->key, h->n, ctx->stream);
        key_index(ctx, &d, key_off, rows, ctx->stream);
    });
}

int jh_check_cas(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts, jh_key_verdict *out,
                 char *err, size_t errlen) {
    if (!ctx || !out) { set_err(err, errlen, "null context or output"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        jh_history d = stage_history(ctx, h, false, false);
        d.key = nullptr;
        d.n_keys = 1;
        jh_key_verdict *dv = ctx->ws<jh_key_verdict>(WS_VERDICT, 1);
        jh_summary s;
        lin_check_independent(ctx, &d, opts, false, dv, &s, st);
        HIP_TRY(hipMemcpyAsync(out, dv, sizeof(jh_key_verdict), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        // a history with no client ops at all still has "a" key here; report
        // it like knossos does for an empty history: valid, nothing explored
        if (out->explored < 0) out->explored = 0;
    });
}

int jh_check_counter(jh_ctx *ctx, const jh_history *h, int64_t *reads_out, int64_t reads_cap,
                     int64_t *n_reads, int64_t *n_errors, int64_t *first_err_entry, int32_t *valid,
                     int32_t *cause, char *err, size_t errlen) {
    if (!ctx || !n_reads || !n_errors || !first_err_entry || !valid || !cause) {
        set_err(err, errlen, "null argument");
        return JH_EINVAL;
    }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, false);
        counter_check(ctx, &d, reads_out, reads_out ? reads_cap : 0, n_reads, n_errors,
                      first_err_entry, valid, cause, ctx->stream);
    });
}

int jh_check_set(jh_ctx *ctx, const jh_history *h, jh_set_result *res, int64_t *runs_ok,
                 int64_t *runs_lost, int64_t *runs_unexpected, int64_t *runs_recovered,
                 int64_t runs_cap, char *err, size_t errlen) {
    if (!ctx || !res) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, true);
        int64_t *runs[4] = {runs_ok, runs_lost, runs_unexpected, runs_recovered};
        set_check(ctx, &d, res, runs, runs_cap, ctx->stream);
    });
}

int jh_check_set_bitmaps(jh_ctx *ctx, const jh_history *h, jh_set_result *res, uint32_t *ok, uint32_t *lost,
                         uint32_t *unexpected, uint32_t *recovered, int64_t words_cap, int64_t *base,
                         int64_t *n_words, char *err, size_t errlen) {
    if (!ctx || !res || !base || !n_words) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, true);
        uint32_t *bits[4] = {ok, lost, unexpected, recovered};
        set_check_bitmaps(ctx, &d, res, bits, words_cap < 0 ? 0 : words_cap, base, n_words, ctx->stream);
    });
}

int jh_host_alloc(size_t bytes, void **out, char *err, size_t errlen) {
    if (!out) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    *out = nullptr;
    return guarded(err, errlen, [&] { HIP_TRY(hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault)); });
}

int jh_host_free(void *p) {
    if (!p) return JH_OK;
    return hipHostFree(p) == hipSuccess ? JH_OK : JH_EDEVICE;
}

int jh_check_set_full(jh_ctx *ctx, const jh_history *h, const int64_t *time, int32_t linearizable,
                      jh_set_full_result *res, int64_t *lost, int64_t *never_read, int64_t *stale,
                      int64_t list_cap, char *err, size_t errlen) {
    jh_set_full_opts o;
    memset(&o, 0, sizeof o);
    o.linearizable = linearizable;
    return jh_check_set_full_opts(ctx, h, time, &o, res, lost, never_read, stale, list_cap, err, errlen);
}

int jh_check_set_full_opts(jh_ctx *ctx, const jh_history *h, const int64_t *time, const jh_set_full_opts *opts,
                           jh_set_full_result *res, int64_t *lost, int64_t *never_read, int64_t *stale,
                           int64_t list_cap, char *err, size_t errlen) {
    if (!ctx || !res || !opts) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    if (opts->read_batch < 0) { set_err(err, errlen, "read_batch < 0"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        if (h->n > 0 && !time) throw_jh(JH_EINVAL, "set-full needs the :time column");
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, true);
        const int64_t *dt = h->on_device ? time : stage_col(ctx, WS_SF_TIME, time, h->n, ctx->stream);
        int64_t *lists[3] = {lost, never_read, stale};
        set_full_check(ctx, &d, dt, opts->linearizable != 0, opts->read_batch, res, lists, list_cap < 0 ? 0 : list_cap,
                       ctx->stream);
    });
}

int jh_check_total_queue(jh_ctx *ctx, const jh_history *h, jh_queue_result *res, int64_t *lost,
                         int64_t *unexpected, int64_t *duplicated, int64_t *recovered, int64_t pairs_cap,
                         char *err, size_t errlen) {
    if (!ctx || !res) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, true);
        int64_t *outs[4] = {lost, unexpected, duplicated, recovered};
        total_queue_check(ctx, &d, res, outs, pairs_cap < 0 ? 0 : pairs_cap, ctx->stream);
    });
}

int jh_check_queue(jh_ctx *ctx, const jh_history *h, jh_queue_result *res, int64_t *final_queue,
                   int64_t pairs_cap, char *err, size_t errlen) {
    if (!ctx || !res) { set_err(err, errlen, "null argument"); return JH_EINVAL; }
    ctx = primary(ctx);
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded(err, errlen, [&] {
        check_hist(h);
        HIP_TRY(hipSetDevice(ctx->device));
        jh_history d = stage_history(ctx, h, false, false);
        queue_check(ctx, &d, res, final_queue, pairs_cap < 0 ? 0 : pairs_cap, ctx->stream);
    });
}

}  // extern "C"
