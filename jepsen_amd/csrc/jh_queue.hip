// jh_queue.hip -- checker/total-queue and checker/queue (unordered-queue) on MI355X.
//
// total-queue, jepsen/src/jepsen/checker.clj:570-628: four multisets over the
// history after expand-queue-drain-ops (:536-568):
//   attempts = :invoke :enqueue values, enqueues = :ok :enqueue values,
//   dequeues = :ok :dequeue values + the elements of every :ok :drain;
//   ok = dequeues n attempts, unexpected = dequeues whose value was never
//   attempted, duplicated = dequeues - attempts - unexpected,
//   lost = enqueues - dequeues, recovered = ok - enqueues
// (metametadata/multiset: intersect = min of counts, minus floors at 0).
// Per value that is three counts a, e, d, so the check is three histograms
// over a dense value LUT (one streaming pass over the rows, one over the
// drains' elements) and a pass over the values.
//
// queue (checker.clj:160-180) reduces knossos' unordered-queue model over the
// :invoke :enqueue (+1) and :ok :dequeue (-1) ops in row order; it fails at
// the first dequeue whose value's running count goes negative. Here: the
// selected rows are radix-sorted by value id (stable, so row order within a
// value), one inclusive scan of the +-1 deltas, each value's running count is
// the scan minus the scan before the value's segment, and the failing row is
// the minimum row with a negative count.
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>
#include <algorithm>

namespace {
constexpr int T_INVOKE = 0, T_OK = 1, T_INFO = 3;

struct QMeta {
    long long vmin, vmax;
    long long n_drain;         // :ok :drain rows
    long long max_cnt;         // largest :ok :drain
    long long n_sel;           // queue: :invoke :enqueue + :ok :dequeue rows
    int nil_val;
    int crashed_drain;
    long long cnt[7];          // attempt, ack, ok, unexpected, duplicated, lost, recovered
    long long npairs[4];
    unsigned long long fail_row;
};

__device__ __forceinline__ bool q_row_value(int64_t ff, int64_t ty) {
    return (ff == JH_F_ENQUEUE && (ty == T_INVOKE || ty == T_OK)) || (ff == JH_F_DEQUEUE && ty == T_OK);
}

// value range over the enqueue / dequeue rows and (drains=1) the aux elements
__global__ void __launch_bounds__(256) k_q_scan(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                                                const int64_t *__restrict__ value, const int64_t *__restrict__ value2,
                                                int64_t n, const int64_t *__restrict__ aux, int64_t n_aux,
                                                int drains, long long *parts) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, nd = 0, mc = 0, ns = 0, nil = 0, crash = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += stride) {
        const int64_t ty = type[r], ff = f[r];
        if (q_row_value(ff, ty)) {
            const int64_t v = value[r];
            if (v == JH_NIL) nil = 1; else { lo = min(lo, (long long)v); hi = max(hi, (long long)v); }
            if ((ff == JH_F_ENQUEUE && ty == T_INVOKE) || ff == JH_F_DEQUEUE) ns++;
        } else if (drains && ff == JH_F_DRAIN) {
            if (ty == T_OK) {
                const int64_t c = (value[r] == JH_NIL || value2[r] == JH_NIL) ? 0 : value2[r];
                nd++; mc = max(mc, (long long)c);
            } else if (ty != T_INVOKE && ty != 2 /* fail */) crash = 1;
        }
    }
    if (drains)
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_aux; i += stride) {
            const int64_t v = aux[i];
            if (v == JH_NIL) nil = 1; else { lo = min(lo, (long long)v); hi = max(hi, (long long)v); }
        }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    nd = block_reduce256(nd, RedSum(), sh);
    mc = block_reduce256(mc, RedMax(), sh);
    ns = block_reduce256(ns, RedSum(), sh);
    nil = block_reduce256(nil, RedOr(), sh);
    crash = block_reduce256(crash, RedOr(), sh);
    if (threadIdx.x == 0) {
        long long *pp = parts + 8 * blockIdx.x;
        pp[0] = lo; pp[1] = hi; pp[2] = nd; pp[3] = mc; pp[4] = ns; pp[5] = nil; pp[6] = crash;
    }
}

__global__ void __launch_bounds__(256) k_q_scan_fin(const long long *__restrict__ parts, int np, QMeta *m) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, nd = 0, mc = 0, ns = 0, nil = 0, crash = 0;
    for (int i = threadIdx.x; i < np; i += 256) {
        const long long *pp = parts + 8 * i;
        lo = min(lo, pp[0]); hi = max(hi, pp[1]); nd += pp[2]; mc = max(mc, pp[3]); ns += pp[4];
        nil |= pp[5]; crash |= pp[6];
    }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    nd = block_reduce256(nd, RedSum(), sh);
    mc = block_reduce256(mc, RedMax(), sh);
    ns = block_reduce256(ns, RedSum(), sh);
    nil = block_reduce256(nil, RedOr(), sh);
    crash = block_reduce256(crash, RedOr(), sh);
    if (threadIdx.x == 0) {
        m->vmin = lo; m->vmax = hi; m->n_drain = nd; m->max_cnt = mc; m->n_sel = ns;
        m->nil_val = (int)nil; m->crashed_drain = (int)crash;
    }
}

// dense value id: v - vmin, and nil gets the last slot (span)
__device__ __forceinline__ int32_t q_id(int64_t v, long long vmin, int64_t span) {
    return v == JH_NIL ? (int32_t)span : (int32_t)(v - vmin);
}

// histograms a (attempts), e (enqueues), d (dequeues); flags :ok :drain rows
// (drains=1) or the queue model's rows (drains=0)
__global__ void __launch_bounds__(256) k_q_hist(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                                                const int64_t *__restrict__ value, int64_t n, long long vmin,
                                                int64_t span, int drains, unsigned long long *a,
                                                unsigned long long *e, unsigned long long *d, uint8_t *flag) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ty = type[r], ff = f[r];
        uint8_t fl = 0;
        if (q_row_value(ff, ty)) {
            const int32_t id = q_id(value[r], vmin, span);
            if (ff == JH_F_ENQUEUE) {
                if (ty == T_INVOKE) { atomicAdd(&a[id], 1ULL); fl = !drains; }
                else atomicAdd(&e[id], 1ULL);
            } else {
                atomicAdd(&d[id], 1ULL);
                fl = !drains;
            }
        } else if (drains && ff == JH_F_DRAIN && ty == T_OK) fl = 1;
        flag[r] = fl;
    }
}

constexpr int DRAIN_CHUNK = 4096;

// the elements of :ok :drain rows as :ok :dequeues (expand-queue-drain-ops)
__global__ void __launch_bounds__(256) k_q_drain(const int64_t *__restrict__ value, const int64_t *__restrict__ value2,
                                                 const int64_t *__restrict__ aux, const int64_t *__restrict__ drows,
                                                 long long vmin, int64_t span, unsigned long long *d) {
    const int64_t row = drows[blockIdx.y];
    const int64_t c = (value[row] == JH_NIL || value2[row] == JH_NIL) ? 0 : value2[row];
    const int64_t base = (int64_t)blockIdx.x * DRAIN_CHUNK;
    if (base >= c) return;
    const int64_t off = value[row], end = min(c, base + DRAIN_CHUNK);
    for (int64_t t = base + threadIdx.x; t < end; t += 256) atomicAdd(&d[q_id(aux[off + t], vmin, span)], 1ULL);
}

// total-queue per value: multiplicities of the four result multisets
__global__ void __launch_bounds__(256) k_q_total(int64_t S, const unsigned long long *__restrict__ a,
                                                 const unsigned long long *__restrict__ e,
                                                 const unsigned long long *__restrict__ d, long long *mult,
                                                 uint32_t *flag, long long *parts) {
    long long c[7] = {0, 0, 0, 0, 0, 0, 0}, np[4] = {0, 0, 0, 0};
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < S; v += (int64_t)gridDim.x * blockDim.x) {
        const long long av = (long long)a[v], ev = (long long)e[v], dv = (long long)d[v];
        const long long ok = min(dv, av);
        const long long un = av == 0 ? dv : 0;
        const long long dup = av > 0 ? max(dv - av, 0LL) : 0;
        const long long lost = max(ev - dv, 0LL);
        const long long rec = max(ok - ev, 0LL);
        c[0] += av; c[1] += ev; c[2] += ok; c[3] += un; c[4] += dup; c[5] += lost; c[6] += rec;
        const long long ms[4] = {lost, un, dup, rec};
        for (int s = 0; s < 4; s++) {
            mult[s * S + v] = ms[s];
            flag[s * S + v] = ms[s] > 0;
            np[s] += ms[s] > 0;
        }
    }
    __shared__ long long sh[4];
    long long *pp = parts + 16 * blockIdx.x;
    for (int q = 0; q < 7; q++) {
        const long long t = block_reduce256(c[q], RedSum(), sh);
        if (threadIdx.x == 0) pp[q] = t;
    }
    for (int q = 0; q < 4; q++) {
        const long long t = block_reduce256(np[q], RedSum(), sh);
        if (threadIdx.x == 0) pp[7 + q] = t;
    }
}

__global__ void __launch_bounds__(256) k_q_total_fin(const long long *__restrict__ parts, int np, QMeta *m) {
    __shared__ long long sh[4];
    for (int q = 0; q < 11; q++) {
        long long c = 0;
        for (int i = threadIdx.x; i < np; i += 256) c += parts[16 * i + q];
        const long long t = block_reduce256(c, RedSum(), sh);
        if (threadIdx.x == 0) { if (q < 7) m->cnt[q] = t; else m->npairs[q - 7] = t; }
    }
}

// (value, multiplicity) pairs of one multiset at their scanned positions
__global__ void __launch_bounds__(256) k_q_emit(int64_t S, int64_t span, long long vmin,
                                                const long long *__restrict__ mult, const uint32_t *__restrict__ flag,
                                                const uint32_t *__restrict__ pos, int64_t cap, int64_t *out) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < S; v += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[v]) continue;
        const int64_t p = pos[v];
        if (p >= cap) continue;
        out[2 * p] = v == span ? JH_NIL : vmin + v;
        out[2 * p + 1] = mult[v];
    }
}

// queue: sort keys of the selected rows
__global__ void __launch_bounds__(256) k_q_keys(const int64_t *__restrict__ value, const int64_t *__restrict__ rows,
                                                int64_t k, long long vmin, int64_t span, uint32_t *keys) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] = (uint32_t)q_id(value[rows[i]], vmin, span);
}

__global__ void __launch_bounds__(256) k_q_delta(const int64_t *__restrict__ f, const int64_t *__restrict__ rows,
                                                 int64_t k, long long *delta) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x)
        delta[i] = f[rows[i]] == JH_F_ENQUEUE ? 1 : -1;
}

// rows per value in the sorted order (the queue model's rows: a + d)
__global__ void __launch_bounds__(256) k_q_segcount(int64_t S, const unsigned long long *__restrict__ a,
                                                    const unsigned long long *__restrict__ d, uint32_t *cnt) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < S; v += (int64_t)gridDim.x * blockDim.x)
        cnt[v] = (uint32_t)(a[v] + d[v]);
}

// a dequeue whose value's running count drops below zero: the model is
// inconsistent there; keep the first such row
__global__ void __launch_bounds__(256) k_q_neg(const uint32_t *__restrict__ keys, const int64_t *__restrict__ rows,
                                               const long long *__restrict__ delta, const long long *__restrict__ scan,
                                               const uint32_t *__restrict__ seg_off, int64_t k, QMeta *m) {
    unsigned long long best = ~0ULL;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x) {
        if (delta[i] >= 0) continue;
        const int64_t st = seg_off[keys[i]];
        const long long base = st > 0 ? scan[st - 1] : 0;
        if (scan[i] - base < 0) best = min(best, (unsigned long long)rows[i]);
    }
    __shared__ unsigned long long sh[4];
    best = block_reduce256(best, RedMin(), sh);
    if (threadIdx.x == 0 && best != ~0ULL) atomicMin(&m->fail_row, best);
}

// queue: the final multiset (attempts - dequeues) per value
__global__ void __launch_bounds__(256) k_q_final(int64_t S, const unsigned long long *__restrict__ a,
                                                 const unsigned long long *__restrict__ d, long long *mult,
                                                 uint32_t *flag, long long *parts) {
    long long np = 0;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < S; v += (int64_t)gridDim.x * blockDim.x) {
        const long long r = (long long)a[v] - (long long)d[v];
        mult[v] = r;
        flag[v] = r > 0;
        np += r > 0;
    }
    __shared__ long long sh[4];
    np = block_reduce256(np, RedSum(), sh);
    if (threadIdx.x == 0) parts[16 * blockIdx.x + 7] = np;
}

__global__ void k_q_final_fin(const long long *__restrict__ parts, int np, QMeta *m) {
    __shared__ long long sh[4];
    long long c = 0;
    for (int i = threadIdx.x; i < np; i += 256) c += parts[16 * i + 7];
    c = block_reduce256(c, RedSum(), sh);
    if (threadIdx.x == 0) m->npairs[0] = c;
}

struct QState {
    QMeta mh;
    QMeta *m;
    long long *parts;
    int64_t span, S;
    unsigned long long *a, *e, *d;
    uint8_t *flag;
};

// range, LUT span and the three histograms (shared by both checkers)
QState q_prepare(jh_ctx *ctx, const jh_history *dh, bool drains, hipStream_t st) {
    QState q{};
    const int64_t n = dh->n;
    q.m = ctx->ws<QMeta>(WS_Q_META, 1);
    q.parts = ctx->ws<long long>(WS_Q_PART, 16 * 2048);
    const int64_t naux = (drains && dh->aux) ? dh->n_aux : 0;
    const int g = grid_for(std::max<int64_t>(n, naux), 256, 2048);
    k_q_scan<<<g, 256, 0, st>>>(dh->type, dh->f, dh->value, dh->value2, n, dh->aux, naux, drains ? 1 : 0, q.parts);
    k_q_scan_fin<<<1, 256, 0, st>>>(q.parts, g, q.m);
    HIP_TRY(hipMemcpyAsync(&q.mh, q.m, sizeof q.mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (q.mh.crashed_drain) throw_jh(JH_EINVAL, "Not sure how to handle a crashed drain operation");
    if (q.mh.n_drain > 0 && q.mh.max_cnt > 0 && !dh->aux) throw_jh(JH_EINVAL, "drain without an aux element array");
    const bool any = q.mh.vmin <= q.mh.vmax;
    const unsigned long long span = any ? (unsigned long long)(q.mh.vmax - q.mh.vmin) + 1 : 0;
    if (span >= (1ULL << 31) - 1) throw_jh(JH_EUNSUPPORTED, "queue values span 2^31 values or more");
    if (!any) q.mh.vmin = 0;
    q.span = (int64_t)span;
    q.S = q.span + 1;                                       // + nil
    unsigned long long *h = ctx->ws<unsigned long long>(WS_Q_HIST, 3 * q.S);
    q.a = h; q.e = h + q.S; q.d = h + 2 * q.S;
    HIP_TRY(hipMemsetAsync(h, 0, sizeof(unsigned long long) * 3 * q.S, st));
    QMeta init = q.mh;
    init.fail_row = ~0ULL;
    HIP_TRY(hipMemcpyAsync(q.m, &init, sizeof init, hipMemcpyHostToDevice, st));
    q.flag = ctx->ws<uint8_t>(WS_Q_FLAG, std::max<int64_t>(n, 1));
    if (n > 0)
        k_q_hist<<<grid_for(n, 256), 256, 0, st>>>(dh->type, dh->f, dh->value, n, q.mh.vmin, q.span, drains ? 1 : 0,
                                                   q.a, q.e, q.d, q.flag);
    return q;
}

// scan + emit the (value, multiplicity) pairs of multiset s
void q_pairs(jh_ctx *ctx, const QState &q, const long long *mult, const uint32_t *flag, int64_t npairs,
             int64_t cap, int64_t *out_host, hipStream_t st) {
    const int64_t k = std::min<int64_t>(npairs, cap);
    if (k <= 0 || !out_host) return;
    uint32_t *pos = ctx->ws<uint32_t>(WS_Q_POS, q.S);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, pos, (int)q.S, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ctx->ws<char>(WS_Q_TMP, tb), tb, flag, pos, (int)q.S, st));
    int64_t *out = ctx->ws<int64_t>(WS_Q_OUT, 2 * k);
    k_q_emit<<<grid_for(q.S, 256), 256, 0, st>>>(q.S, q.span, q.mh.vmin, mult, flag, pos, k, out);
    HIP_TRY(hipMemcpyAsync(out_host, out, sizeof(int64_t) * 2 * k, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
}

double q_elapsed(jh_ctx *ctx, hipStream_t st) {
    HIP_TRY(hipEventRecord(ctx->ev[1], st));
    HIP_TRY(hipEventSynchronize(ctx->ev[1]));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
    return ms;
}

}  // namespace

void total_queue_check(jh_ctx *ctx, const jh_history *dh, jh_queue_result *res, int64_t *outs[4],
                       int64_t cap, hipStream_t st) {
    memset(res, 0, sizeof *res);
    res->fail_entry = -1;
    HIP_TRY(hipEventRecord(ctx->ev[0], st));
    QState q = q_prepare(ctx, dh, true, st);
    const int64_t nd = q.mh.n_drain;
    if (nd > 0 && q.mh.max_cnt > 0) {
        int64_t *dr = ctx->ws<int64_t>(WS_Q_ROWS, nd + 1);
        hipcub::CountingInputIterator<int64_t> rows(0);
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, rows, q.flag, dr, dr + nd, dh->n, st));
        HIP_TRY(hipcub::DeviceSelect::Flagged(ctx->ws<char>(WS_Q_TMP, tb), tb, rows, q.flag, dr, dr + nd, dh->n, st));
        const unsigned gx = (unsigned)((q.mh.max_cnt + DRAIN_CHUNK - 1) / DRAIN_CHUNK);
        for (int64_t r0 = 0; r0 < nd; r0 += 65535)
            k_q_drain<<<dim3(gx, (unsigned)std::min<int64_t>(65535, nd - r0)), 256, 0, st>>>(
                dh->value, dh->value2, dh->aux, dr + r0, q.mh.vmin, q.span, q.d);
    }
    long long *mult = ctx->ws<long long>(WS_Q_MULT, 4 * q.S);
    uint32_t *flag = ctx->ws<uint32_t>(WS_Q_MFLAG, 4 * q.S);
    const int g = grid_for(q.S, 256, 2048);
    k_q_total<<<g, 256, 0, st>>>(q.S, q.a, q.e, q.d, mult, flag, q.parts);
    k_q_total_fin<<<1, 256, 0, st>>>(q.parts, g, q.m);
    HIP_TRY(hipMemcpyAsync(&q.mh, q.m, sizeof q.mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    res->attempt_count = q.mh.cnt[0]; res->acknowledged_count = q.mh.cnt[1]; res->ok_count = q.mh.cnt[2];
    res->unexpected_count = q.mh.cnt[3]; res->duplicated_count = q.mh.cnt[4];
    res->lost_count = q.mh.cnt[5]; res->recovered_count = q.mh.cnt[6];
    res->valid = (res->lost_count == 0 && res->unexpected_count == 0) ? JH_VALID : JH_INVALID;
    for (int s = 0; s < 4; s++) {
        res->n_pairs[s] = q.mh.npairs[s];
        q_pairs(ctx, q, mult + s * q.S, flag + s * q.S, q.mh.npairs[s], cap, outs[s], st);
    }
    res->device_ms = q_elapsed(ctx, st);
}

void queue_check(jh_ctx *ctx, const jh_history *dh, jh_queue_result *res, int64_t *final_out, int64_t cap,
                 hipStream_t st) {
    memset(res, 0, sizeof *res);
    res->fail_entry = -1;
    HIP_TRY(hipEventRecord(ctx->ev[0], st));
    QState q = q_prepare(ctx, dh, false, st);
    const int64_t k = q.mh.n_sel;
    if (k > 0) {
        int64_t *rb = ctx->ws<int64_t>(WS_Q_ROWS, 2 * k + 1);
        int64_t *rows_sel = rb, *rows_sorted = rb + k;
        hipcub::CountingInputIterator<int64_t> rows(0);
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, rows, q.flag, rows_sel, rb + 2 * k, dh->n, st));
        HIP_TRY(hipcub::DeviceSelect::Flagged(ctx->ws<char>(WS_Q_TMP, tb), tb, rows, q.flag, rows_sel, rb + 2 * k,
                                              dh->n, st));
        uint32_t *kb = ctx->ws<uint32_t>(WS_Q_KEYS, 2 * k + q.S);
        uint32_t *keys = kb, *keys_sorted = kb + k, *seg_off = kb + 2 * k;
        k_q_keys<<<grid_for(k, 256), 256, 0, st>>>(dh->value, rows_sel, k, q.mh.vmin, q.span, keys);
        int end_bit = 1;
        while (end_bit < 32 && (1LL << end_bit) < q.S) end_bit++;
        tb = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys_sorted, rows_sel, rows_sorted, k, 0,
                                                   end_bit, st));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(ctx->ws<char>(WS_Q_TMP, tb), tb, keys, keys_sorted, rows_sel,
                                                   rows_sorted, k, 0, end_bit, st));
        // segment start of each value = exclusive scan of its row count (a + d)
        long long *db = ctx->ws<long long>(WS_Q_MULT, 2 * k);
        long long *delta = db, *scan = db + k;
        k_q_delta<<<grid_for(k, 256), 256, 0, st>>>(dh->f, rows_sorted, k, delta);
        tb = 0;
        HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, delta, scan, k, st));
        HIP_TRY(hipcub::DeviceScan::InclusiveSum(ctx->ws<char>(WS_Q_TMP, tb), tb, delta, scan, k, st));
        uint32_t *cnt = ctx->ws<uint32_t>(WS_Q_POS, q.S);
        k_q_segcount<<<grid_for(q.S, 256), 256, 0, st>>>(q.S, q.a, q.d, cnt);
        tb = 0;
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, seg_off, (int)q.S, st));
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ctx->ws<char>(WS_Q_TMP, tb), tb, cnt, seg_off, (int)q.S, st));
        k_q_neg<<<grid_for(k, 256, 2048), 256, 0, st>>>(keys_sorted, rows_sorted, delta, scan, seg_off, k, q.m);
        HIP_TRY(hipMemcpyAsync(&q.mh, q.m, sizeof q.mh, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (k > 0 && q.mh.fail_row != ~0ULL) {
        res->valid = JH_INVALID;
        res->fail_entry = (int64_t)q.mh.fail_row;
        HIP_TRY(hipMemcpyAsync(&res->fail_value, dh->value + res->fail_entry, sizeof(int64_t),
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    } else {
        res->valid = JH_VALID;
        long long *mult = ctx->ws<long long>(WS_Q_MULT2, q.S);
        uint32_t *flag = ctx->ws<uint32_t>(WS_Q_MFLAG, q.S);
        const int g = grid_for(q.S, 256, 2048);
        k_q_final<<<g, 256, 0, st>>>(q.S, q.a, q.d, mult, flag, q.parts);
        k_q_final_fin<<<1, 256, 0, st>>>(q.parts, g, q.m);
        HIP_TRY(hipMemcpyAsync(&q.mh, q.m, sizeof q.mh, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        res->n_pairs[0] = q.mh.npairs[0];
        q_pairs(ctx, q, mult, flag, q.mh.npairs[0], cap, final_out, st);
    }
    res->device_ms = q_elapsed(ctx, st);
}
