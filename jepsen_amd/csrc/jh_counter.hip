// jh_counter.hip -- checker/counter on MI355X.
//
// Replaces (checker/counter), jepsen/src/jepsen/checker.clj:679-734:
//   history/complete, (remove :fails?), (remove op/fail?), then a sequential
//   loop carrying lower/upper bounds and pending reads.
// The loop is two exclusive prefix sums over the rows, in history order:
//   lower(row) = sum of :ok :add values before row        (checker.clj:725-726)
//   upper(row) = sum of non-failed :invoke :add values     (checker.clj:722-723)
// and each :ok :read emits [lower(its invocation) value upper(itself)]
// (checker.clj:713-720); errors are the triples with not (<= lower v upper).
//
//   k_cnt_last   last row of each process (LDS-privatised per chunk)
//   k_cnt_pair   complete pairing: next non-:info row of the same process,
//                stopping at the process' last row
//   k_cnt_orphan :ok/:fail with no open invocation
//   k_cnt_vals   per-row add contributions (+ :fails? / nil checks)
//   2 x hipcub ExclusiveSum (int64)
//   k_cnt_reads  compact the :ok :read triples in history order, count
//                errors, first failing row
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>

namespace {

constexpr int T_INVOKE = 0, T_OK = 1, T_FAIL = 2, T_INFO = 3;
constexpr int CHUNK = 4096, HSLOTS = 2048;

struct CntMeta {
    long long pmin, pmax;          // process range
    long long amax_abs;            // max |add value|
    long long n_add;
    unsigned long long viol1;      // complete: row << 4 | cause
    unsigned long long viol2;      // loop: row << 4 | cause
    unsigned long long viol3;      // read value nil: row << 4 | cause
    unsigned long long first_err;  // min row of an error read
    long long n_errors;
    long long n_reads;
};

__global__ void __launch_bounds__(256) k_cnt_range(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                            const int64_t *__restrict__ f, const int64_t *__restrict__ val,
                            int64_t n, CntMeta *m) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, am = 0, na = 0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        long long p = proc[r];
        lo = min(lo, p); hi = max(hi, p);
        if (f[r] == JH_F_ADD && (type[r] == T_INVOKE || type[r] == T_OK)) {
            long long v = val[r];
            if (v != JH_NIL) { am = max(am, v < 0 ? (v == LLONG_MIN ? LLONG_MAX : -v) : v); }
            na++;
        }
    }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    am = block_reduce256(am, RedMax(), sh);
    na = block_reduce256(na, RedSum(), sh);
    if (threadIdx.x == 0) {
        atomicMin(&m->pmin, lo); atomicMax(&m->pmax, hi);
        atomicMax(&m->amax_abs, am);
        if (na) atomicAdd((unsigned long long *)&m->n_add, (unsigned long long)na);
    }
}

// last row of every process: per-chunk LDS hash of (process -> max row),
// then one global atomicMax per distinct process of the chunk
__global__ void __launch_bounds__(256) k_cnt_last(const int64_t *__restrict__ proc,
                                                  const int64_t *__restrict__ type, int64_t n,
                                                  long long pmin, int32_t *__restrict__ last,
                                                  uint32_t *__restrict__ pt) {
    __shared__ long long hk[HSLOTS];
    __shared__ int hv[HSLOTS];
    const int64_t c0 = (int64_t)blockIdx.x * CHUNK;
    for (int i = threadIdx.x; i < HSLOTS; i += blockDim.x) { hk[i] = LLONG_MIN; hv[i] = -1; }
    __syncthreads();
    for (int i = threadIdx.x; i < CHUNK; i += blockDim.x) {
        const int64_t r = c0 + i;
        if (r >= n) break;
        const long long p = proc[r];
        pt[r] = ((uint32_t)(p - pmin) << 2) | (uint32_t)(type[r] & 3);   // span < 2^28
        uint32_t h = (uint32_t)jh_mix64((uint64_t)p) & (HSLOTS - 1);
        bool done = false;
        for (int probe = 0; probe < 64 && !done; probe++) {
            long long cur = hk[h];
            if (cur == LLONG_MIN) {
                cur = (long long)atomicCAS((unsigned long long *)&hk[h], (unsigned long long)LLONG_MIN,
                                           (unsigned long long)p);
                if (cur == LLONG_MIN) cur = p;
            }
            if (cur == p) { atomicMax(&hv[h], (int)r); done = true; }
            else h = (h + 1) & (HSLOTS - 1);
        }
        if (!done) atomicMax(&last[p - pmin], (int)r);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HSLOTS; i += blockDim.x)
        if (hk[i] != LLONG_MIN) atomicMax(&last[hk[i] - pmin], hv[i]);
}

// complete pairing: an invocation's completion is the next non-:info row of
// its process (util.clj:606-640). One wave per 64 consecutive rows: it reads
// the packed (process, type) words 64 rows at a time and, for each distinct
// process among its still-open invocations, one ballot over the window gives
// every candidate row; each open lane takes the first one after its own row.
// A lane gives up after its process' last row (no completion: stays open).
__global__ void __launch_bounds__(256) k_cnt_pair(const uint32_t *__restrict__ pt, int64_t n,
                                                  const int32_t *__restrict__ last,
                                                  int32_t *__restrict__ pair, CntMeta *m) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); wv * 64 < n; wv += nw) {
        const int64_t base = wv * 64, r = base + lane;
        const uint32_t x = r < n ? pt[r] : 3u;
        const uint32_t p = x >> 2;
        const bool inv = r < n && (x & 3) == T_INVOKE;
        const int64_t lr = inv ? (int64_t)last[p] : -1;
        bool open = inv && lr > r;
        int64_t got = -1;
        for (int64_t wb = base; wb < n; wb += 64) {
            if (!__ballot(open)) break;
            const int64_t j = wb + lane;
            const uint32_t y = j < n ? pt[j] : 3u;
            uint64_t todo = __ballot(open);
            while (todo) {
                const int l = __builtin_ctzll(todo);
                const uint32_t pl = (uint32_t)__builtin_amdgcn_readlane((int)p, l);
                const uint64_t mine = __ballot(open && p == pl);
                const uint64_t cand = __ballot((y >> 2) == pl && (y & 3) != T_INFO);
                todo &= ~mine;
                if ((mine >> lane) & 1) {
                    // candidates strictly after this lane's row
                    const int64_t rel = r - wb;          // in [-63.., 63]
                    const uint64_t after = rel < 0 ? ~0ULL : (rel >= 63 ? 0ULL : (~0ULL << (rel + 1)));
                    const uint64_t c = cand & after;
                    if (c) { got = wb + __builtin_ctzll(c); open = false; }
                }
            }
            // past the process' last row: no completion
            if (open && wb + 63 >= lr) open = false;
        }
        if (got >= 0) {
            if ((pt[got] & 3) == T_INVOKE)
                atomicMin(&m->viol1, ((unsigned long long)got << 4) | JH_CAUSE_DOUBLE_INVOKE);
            else { pair[r] = (int32_t)got; pair[got] = (int32_t)r; }
        }
    }
}

__global__ void k_cnt_orphan(const int64_t *__restrict__ type, int64_t n,
                             const int32_t *__restrict__ pair, CntMeta *m) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ty = type[r];
        if ((ty == T_OK || ty == T_FAIL) && pair[r] < 0)
            atomicMin(&m->viol1, ((unsigned long long)r << 4) | JH_CAUSE_ORPHAN);
    }
}

__global__ void k_cnt_vals(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                           const int64_t *__restrict__ val, int64_t n,
                           const int32_t *__restrict__ pair, int64_t *__restrict__ okadd,
                           int64_t *__restrict__ invadd, int32_t *__restrict__ isread, CntMeta *m) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ty = type[r], ff = f[r];
        const int32_t c = pair[r];
        int64_t lo = 0, hi = 0;
        int rd = 0;
        if (ty == T_INVOKE && ff == JH_F_ADD) {
            const bool failed = c >= 0 && type[c] == T_FAIL;
            if (!failed) {
                int64_t v = val[r];
                if (v == JH_NIL && c >= 0) v = val[c];          // (or inv ok)
                if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
                else hi = v;
            }
        } else if (ty == T_OK && ff == JH_F_ADD) {
            const int64_t v = val[r];
            if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
            else lo = v;
        } else if (ty == T_OK && ff == JH_F_READ) {
            // its pending read must come from an [:invoke :read] (checker.clj:713-716)
            if (c < 0 || f[c] != JH_F_READ)
                atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_ORPHAN);
            else rd = 1;
        }
        okadd[r] = lo; invadd[r] = hi; isread[r] = rd;
    }
}

__global__ void k_cnt_reads(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                            const int64_t *__restrict__ val, int64_t n,
                            const int32_t *__restrict__ pair, const int64_t *__restrict__ lo,
                            const int64_t *__restrict__ hi, const int32_t *__restrict__ isread,
                            const int32_t *__restrict__ ridx, int64_t *__restrict__ out,
                            int64_t cap, CntMeta *m) {
    long long nerr = 0;
    unsigned long long ferr = ~0ULL;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        if (!isread[r]) continue;
        const int32_t inv = pair[r];
        int64_t v = val[inv];
        if (v == JH_NIL) v = val[r];
        const int64_t l = lo[inv], u = hi[r];
        const int64_t i = ridx[r];
        if (i < cap) { out[3 * i] = l; out[3 * i + 1] = v; out[3 * i + 2] = u; }
        if (v == JH_NIL) {
            atomicMin(&m->viol3, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
        } else if (!(l <= v && v <= u)) {
            nerr++;
            ferr = min(ferr, (unsigned long long)r);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        nerr += __shfl_xor(nerr, o);
        ferr = min(ferr, __shfl_xor(ferr, o));
    }
    if ((threadIdx.x & 63) == 0) {
        if (nerr) atomicAdd((unsigned long long *)&m->n_errors, (unsigned long long)nerr);
        if (ferr != ~0ULL) atomicMin(&m->first_err, ferr);
    }
}

}  // namespace

void counter_check(jh_ctx *ctx, const jh_history *dh, int64_t *reads_out, int64_t reads_cap,
                   int64_t *n_reads, int64_t *n_errors, int64_t *first_err, int32_t *valid,
                   int32_t *cause, hipStream_t st) {
    const int64_t n = dh->n;
    *n_reads = 0; *n_errors = 0; *first_err = -1; *valid = JH_VALID; *cause = 0;
    if (n == 0) return;
    if (n >= (1LL << 31) - 1) throw_jh(JH_EUNSUPPORTED, "more than 2^31 entries");
    CntMeta *m = ctx->ws<CntMeta>(WS_C_TMP, 1);
    CntMeta mi{LLONG_MAX, LLONG_MIN, 0, 0, ~0ULL, ~0ULL, ~0ULL, ~0ULL, 0, 0};
    HIP_TRY(hipMemcpyAsync(m, &mi, sizeof mi, hipMemcpyHostToDevice, st));
    k_cnt_range<<<grid_for(n, 256, 4096), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n, m);
    CntMeta mh;
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const unsigned long long span = (unsigned long long)(mh.pmax - mh.pmin);
    if (span >= (1ULL << 28)) throw_jh(JH_EUNSUPPORTED, "process ids span more than 2^28");
    // Clojure + throws on long overflow; if no prefix can overflow we need no
    // ordered overflow check (else the shim falls back to the JVM checker).
    if (mh.amax_abs > 0 && (unsigned long long)mh.amax_abs > (unsigned long long)(LLONG_MAX / std::max(1LL, mh.n_add)))
        throw_jh(JH_EUNSUPPORTED, "add values large enough to overflow a long");

    int32_t *last = ctx->ws<int32_t>(WS_C_LAST, span + 1);
    int32_t *pair = ctx->ws<int32_t>(WS_C_PAIR, n);
    int64_t *lo = ctx->ws<int64_t>(WS_C_LO, n), *hi = ctx->ws<int64_t>(WS_C_HI, n);
    int32_t *isread = ctx->ws<int32_t>(WS_C_FLAG, n), *ridx = ctx->ws<int32_t>(WS_C_IDX, n);
    HIP_TRY(hipMemsetAsync(last, 0xFF, sizeof(int32_t) * (span + 1), st));
    HIP_TRY(hipMemsetAsync(pair, 0xFF, sizeof(int32_t) * n, st));
    uint32_t *pt = ctx->ws<uint32_t>(WS_C_PT, n);
    k_cnt_last<<<(int)((n + CHUNK - 1) / CHUNK), 256, 0, st>>>(dh->process, dh->type, n, mh.pmin, last, pt);
    k_cnt_pair<<<grid_for((n + 63) / 64, 4, 16384), 256, 0, st>>>(pt, n, last, pair, m);
    k_cnt_orphan<<<grid_for(n, 256), 256, 0, st>>>(dh->type, n, pair, m);
    k_cnt_vals<<<grid_for(n, 256), 256, 0, st>>>(dh->type, dh->f, dh->value, n, pair, lo, hi, isread, m);
    size_t tb = 0, tb2 = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lo, lo, (int)n, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, isread, ridx, (int)n, st));
    void *tmp = ctx->ws<char>(WS_S_TMP, std::max(tb, tb2));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, lo, lo, (int)n, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, hi, hi, (int)n, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, isread, ridx, (int)n, st));
    int32_t last_idx = 0, last_flag = 0;
    HIP_TRY(hipMemcpyAsync(&last_idx, ridx + n - 1, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&last_flag, isread + n - 1, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int64_t nr = (int64_t)last_idx + last_flag;
    const int64_t cap = std::min(nr, reads_cap);
    int64_t *out = ctx->ws<int64_t>(WS_C_OUT, 3 * std::max<int64_t>(cap, 1));
    k_cnt_reads<<<grid_for(n, 256), 256, 0, st>>>(dh->type, dh->f, dh->value, n, pair, lo, hi, isread,
                                                  ridx, out, cap, m);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    if (cap > 0 && reads_out)
        HIP_TRY(hipMemcpyAsync(reads_out, out, sizeof(int64_t) * 3 * cap, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *n_reads = nr;
    if (mh.viol1 != ~0ULL) { *valid = JH_UNKNOWN; *cause = (int)(mh.viol1 & 15); *n_reads = 0; return; }
    if (mh.viol2 != ~0ULL) { *valid = JH_UNKNOWN; *cause = (int)(mh.viol2 & 15); *n_reads = 0; return; }
    *n_errors = mh.n_errors;
    *first_err = mh.first_err == ~0ULL ? -1 : (int64_t)mh.first_err;
    if (mh.viol3 != ~0ULL) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_NIL_VALUE; return; }
    *valid = mh.n_errors ? JH_INVALID : JH_VALID;
}
