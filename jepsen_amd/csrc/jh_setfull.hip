// jh_setfull.hip -- checker/set-full on MI355X.
//
// Replaces (checker/set-full {:linearizable? b}), jepsen/src/jepsen/checker.clj:236-534.
// The reference folds the history once, and on every :ok :read walks EVERY
// tracked element (map-kv over `elements`, checker.clj:500-530): O(reads x
// elements) map updates. Per element e only four facts survive
// (SetFullElement, checker.clj:255-286), all counted from e's last
// :invoke :add (a re-invoke replaces the element's record, :483-487):
//   known        first :ok :add of e, or first :ok :read containing e (row order)
//   last-present read invocation of greatest :index whose :ok read contains e
//   last-absent  read invocation of greatest :index whose :ok read lacks e
// (set-full-read-present / -absent keep the invocation with the greater
// :index, :268-286). Here:
//   1. k_sf_scan        element range / counts over the add and read rows
//   2. k_sf_mark + scan dense element ids in sorted value order (a LUT over the span)
//   3. k_sf_addinv/okadd last :invoke :add per element, first :ok :add after it
//   4. select + k_sf_inv the :ok reads in row order, each with its invocation row
//   5. per batch of reads: k_sf_bits marks a read x element bitmap from the
//      reads' aux elements (the one streaming pass over the big input), then
//      k_sf_elem walks the reads per element (one wave = 64 elements = one
//      bitmap word per read) and updates known / last-present / last-absent
//   6. k_sf_final       set-full-element-results (:289-345) per element
//   7. selects and radix sorts: lost / never-read / stale lists (sorted), the
//      latency quantiles (frequency-distribution, :347-358) and worst-stale.
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>
#include <algorithm>

namespace {
constexpr int T_INVOKE = 0, T_OK = 1;

struct SfMeta {
    long long vmin, vmax;
    long long n_inv;           // :invoke :add rows of integer processes
    long long n_reads;         // :ok :read rows of integer processes
    long long max_cnt;         // largest element count of one :ok :read
    long long read_elems;      // sum of those counts
    long long n_elem;          // distinct elements
    long long cnt[4];          // stable, lost, never-read, stale
    int nil_elem;              // an :add of nil
    int bad_read;              // an :ok :read with no read invocation before it
};

__device__ __forceinline__ int64_t rd_count(const int64_t *value, const int64_t *value2, int64_t row) {
    const int64_t c = value2[row];
    return (c == JH_NIL || value[row] == JH_NIL || c < 0) ? 0 : c;
}

__global__ void __launch_bounds__(256) k_sf_scan(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                                                 const int64_t *__restrict__ f, const int64_t *__restrict__ value,
                                                 const int64_t *__restrict__ value2, int64_t n, long long *parts) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, ninv = 0, nrd = 0, mc = 0, re = 0;
    int nil = 0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        if (proc[r] < 0) continue;                       // (comp number? :process), checker.clj:480
        const int64_t ty = type[r], ff = f[r];
        if (ff == JH_F_ADD && ty == T_INVOKE) {
            const int64_t v = value[r];
            if (v == JH_NIL) nil = 1;
            else { lo = min(lo, (long long)v); hi = max(hi, (long long)v); ninv++; }
        } else if (ff == JH_F_READ && ty == T_OK) {
            const int64_t c = rd_count(value, value2, r);
            nrd++; re += c; mc = max(mc, (long long)c);
        }
    }
    __shared__ long long sh[4];
    __shared__ int shi[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    ninv = block_reduce256(ninv, RedSum(), sh);
    nrd = block_reduce256(nrd, RedSum(), sh);
    re = block_reduce256(re, RedSum(), sh);
    mc = block_reduce256(mc, RedMax(), sh);
    nil = block_reduce256(nil, RedOr(), shi);
    // per-block partials, reduced by k_sf_scan_fin: thousands of same-address
    // atomics serialise in one L2 channel (~5 ns each)
    if (threadIdx.x == 0) {
        long long *pp = parts + 8 * blockIdx.x;
        pp[0] = lo; pp[1] = hi; pp[2] = ninv; pp[3] = nrd; pp[4] = re; pp[5] = mc; pp[6] = nil;
    }
}

__global__ void __launch_bounds__(256) k_sf_scan_fin(const long long *__restrict__ parts, int np, SfMeta *m) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, ninv = 0, nrd = 0, re = 0, mc = 0, nil = 0;
    for (int i = threadIdx.x; i < np; i += 256) {
        const long long *pp = parts + 8 * i;
        lo = min(lo, pp[0]); hi = max(hi, pp[1]); ninv += pp[2]; nrd += pp[3]; re += pp[4];
        mc = max(mc, pp[5]); nil |= pp[6];
    }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    ninv = block_reduce256(ninv, RedSum(), sh);
    nrd = block_reduce256(nrd, RedSum(), sh);
    re = block_reduce256(re, RedSum(), sh);
    mc = block_reduce256(mc, RedMax(), sh);
    nil = block_reduce256(nil, RedOr(), sh);
    if (threadIdx.x == 0) {
        m->vmin = lo; m->vmax = hi; m->n_inv = ninv; m->n_reads = nrd; m->read_elems = re;
        m->max_cnt = mc; m->nil_elem = (int)nil;
    }
}

__device__ __forceinline__ bool add_invoke(const int64_t *proc, const int64_t *type, const int64_t *f, int64_t r) {
    return proc[r] >= 0 && f[r] == JH_F_ADD && type[r] == T_INVOKE;
}

// flag[v - vmin] = 1 for every added value
__global__ void __launch_bounds__(256) k_sf_mark(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                                                 const int64_t *__restrict__ f, const int64_t *__restrict__ value,
                                                 int64_t n, long long vmin, uint32_t *flag) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        if (add_invoke(proc, type, f, r)) flag[value[r] - vmin] = 1;
}

// ids (exclusive scan of flag) -> lut: dense id or -1; elem[id] = value
__global__ void __launch_bounds__(256) k_sf_lut(const uint32_t *__restrict__ flag, int32_t *ids, int64_t span,
                                                long long vmin, int64_t *elem, SfMeta *m) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < span; v += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t fl = flag[v];
        const int32_t id = ids[v];
        if (fl) elem[id] = vmin + v;
        ids[v] = fl ? id : -1;
        if (v == span - 1) m->n_elem = (long long)id + fl;
    }
}

__device__ __forceinline__ int32_t elem_id(const int32_t *lut, long long vmin, long long vmax, int64_t v) {
    return (v < vmin || v > vmax) ? -1 : lut[v - vmin];
}

// last :invoke :add row per element
__global__ void __launch_bounds__(256) k_sf_addinv(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                                                   const int64_t *__restrict__ f, const int64_t *__restrict__ value,
                                                   int64_t n, const int32_t *__restrict__ lut, long long vmin,
                                                   long long *last_inv) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        if (add_invoke(proc, type, f, r)) atomicMax(&last_inv[lut[value[r] - vmin]], (long long)r);
}

// set-full-add (checker.clj:262-266): the first :ok :add after the element's
// record was (re)created sets :known. Also flags the :ok :read rows.
__global__ void __launch_bounds__(256) k_sf_okadd(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                                                  const int64_t *__restrict__ f, const int64_t *__restrict__ value,
                                                  int64_t n, const int32_t *__restrict__ lut, long long vmin,
                                                  long long vmax, const long long *__restrict__ last_inv,
                                                  unsigned long long *known_add, uint8_t *read_flag) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = proc[r], ty = type[r], ff = f[r];
        uint8_t rf = 0;
        if (p >= 0 && ty == T_OK) {
            if (ff == JH_F_ADD) {
                const int32_t id = elem_id(lut, vmin, vmax, value[r]);
                if (id >= 0 && r > last_inv[id]) atomicMin(&known_add[id], (unsigned long long)r);
            } else if (ff == JH_F_READ) rf = 1;
        }
        read_flag[r] = rf;
    }
}

// The invocation of each :ok :read: the reads map holds, per process, its
// latest read invocation (checker.clj:489-493); a process is single-threaded,
// so that is the process' previous row, which must be a :read :invoke. One
// wave per read scans back 64 rows at a time.
__global__ void __launch_bounds__(256) k_sf_inv(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                                                const int64_t *__restrict__ f, const int64_t *__restrict__ rrow,
                                                int64_t nr, int64_t *rinv, SfMeta *m) {
    const int lane = threadIdx.x & 63;
    const int64_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= nr) return;
    const int64_t row = rrow[i];
    const int64_t p = proc[row];
    int64_t q = -1;
    for (int64_t hi = row - 1; hi >= 0; hi -= 64) {
        const int64_t r = hi - lane;
        const bool hit = r >= 0 && proc[r] == p;
        const unsigned long long b = __ballot(hit);
        if (b) { q = hi - (int64_t)__builtin_ctzll(b); break; }
    }
    if (lane == 0) {
        const bool ok = q >= 0 && f[q] == JH_F_READ && type[q] == T_INVOKE;
        rinv[i] = ok ? q : -1;
        if (!ok) atomicOr(&m->bad_read, 1);
    }
}

constexpr int BITS_CHUNK = 4096;    // aux entries per workgroup in k_sf_bits
constexpr int BITS_UNROLL = 4;      // 64-entry groups per wave in flight (8: no change, 246 -> 244 us)

// OR of `b` over each run of equal `w` in the wave (runs are contiguous lane
// ranges; heads = first lane of each run): a segmented Hillis-Steele suffix
// scan, after which every run head holds its run's OR.
__device__ __forceinline__ unsigned long long run_or(int64_t w, unsigned long long b, int lane,
                                                      unsigned long long &heads) {
    const int64_t wprev = __shfl_up(w, 1);
    heads = __ballot(lane == 0 || wprev != w);
    unsigned long long acc = b;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_down(acc, d);
        // same run iff no head in (lane, lane + d]
        const unsigned long long upto = (lane + d >= 63) ? ~0ULL : ((2ULL << (lane + d)) - 1);
        const unsigned long long span = upto & ~((2ULL << lane) - 1);
        if (lane + d < 64 && !(heads & span)) acc |= o;
    }
    return acc;
}

// Element-word-major bitmap for reads [r0, r0+nb): bit (e & 63) of
// bits[(e >> 6) * NB + j] is set iff read r0+j's :value contains element e,
// so k_sf_elem reads one element word for 64 consecutive reads as one
// coalesced 512-byte load. Lanes holding the same word are OR-combined
// before one atomicOr per run (reads are usually sorted, so 64 lanes touch
// one or two words). Each wave keeps BITS_UNROLL aux loads in flight.
__global__ void __launch_bounds__(256) k_sf_bits(const int64_t *__restrict__ value, const int64_t *__restrict__ value2,
                                                 const int64_t *__restrict__ aux, const int64_t *__restrict__ rrow,
                                                 int64_t r0, const int32_t *__restrict__ lut, long long vmin,
                                                 long long vmax, int64_t NB, unsigned long long *bits) {
    const int64_t j = blockIdx.y;
    const int64_t row = rrow[r0 + j];
    const int64_t cnt = rd_count(value, value2, row);
    const int64_t base = (int64_t)blockIdx.x * BITS_CHUNK;
    if (base >= cnt) return;
    const int64_t off = value[row];
    const int64_t end = min(cnt, base + BITS_CHUNK);
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    for (int64_t g = base + wv * 64 * BITS_UNROLL; g < end; g += 256 * BITS_UNROLL) {
        int64_t v[BITS_UNROLL];
#pragma unroll
        for (int u = 0; u < BITS_UNROLL; u++) {
            const int64_t t = g + u * 64 + lane;
            v[u] = t < end ? aux[off + t] : JH_NIL;
        }
        int32_t id[BITS_UNROLL];
#pragma unroll
        for (int u = 0; u < BITS_UNROLL; u++) id[u] = elem_id(lut, vmin, vmax, v[u]);
#pragma unroll
        for (int u = 0; u < BITS_UNROLL; u++) {
            const int64_t w = id[u] >= 0 ? (id[u] >> 6) : -1;
            const unsigned long long b = id[u] >= 0 ? (1ULL << (id[u] & 63)) : 0ULL;
            unsigned long long heads;
            const unsigned long long acc = run_or(w, b, lane, heads);
            if (((heads >> lane) & 1) && w >= 0 && acc) atomicOr(&bits[w * NB + j], acc);
        }
    }
}

__device__ __forceinline__ long long readlane64(long long v, int k) {
    const int lo = __builtin_amdgcn_readlane((int)v, k);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), k);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One thread per element, one wave per bitmap word: walks the batch's reads
// in row order (only reads completing after the element's last add
// invocation count) and applies set-full-read-present / -absent. Lane l
// loads the word, row and invocation of read j0+l (coalesced); the wave then
// steps through the 64 reads with scalar readlanes.
__global__ void __launch_bounds__(256) k_sf_elem(const int64_t *__restrict__ rrow, const int64_t *__restrict__ rinv,
                                                 int64_t r0, int64_t nb, const unsigned long long *__restrict__ bits,
                                                 int64_t NB, int64_t M, const long long *__restrict__ last_inv,
                                                 unsigned long long *known_read, long long *last_present,
                                                 long long *last_absent) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = e < M;
    const long long a = live ? last_inv[e] : LLONG_MAX;
    // first read of the batch completing after the wave's earliest add invocation
    long long amin = a;
    for (int o = 32; o > 0; o >>= 1) amin = min(amin, (long long)__shfl_xor(amin, o));
    int64_t lo = 0, hi = nb;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (rrow[r0 + mid] > amin) hi = mid; else lo = mid + 1;
    }
    if (lo >= nb) return;                                   // uniform over the wave
    unsigned long long kr = live ? known_read[e] : 0;
    long long lp = live ? last_present[e] : 0, la = live ? last_absent[e] : 0;
    const unsigned long long *col = bits + (e >> 6) * NB;
    const int sh = (int)(e & 63);
    for (int64_t j0 = lo; j0 < nb; j0 += 64) {
        const int64_t jj = j0 + lane;
        const bool in = jj < nb;
        const long long wv = in ? (long long)col[jj] : 0;
        const long long rr = in ? (long long)rrow[r0 + jj] : LLONG_MIN;
        const long long ri = in ? (long long)rinv[r0 + jj] : -1;
        const int kmax = (int)min((int64_t)64, nb - j0);
        for (int k = 0; k < kmax; k++) {
            const long long row = readlane64(rr, k);
            const long long inv = readlane64(ri, k);
            const unsigned long long word = (unsigned long long)readlane64(wv, k);
            if (row > a) {
                if ((word >> sh) & 1) {
                    if (kr == ~0ULL) kr = (unsigned long long)row;
                    lp = max(lp, inv);
                } else {
                    la = max(la, inv);
                }
            }
        }
    }
    if (live) {
        known_read[e] = kr;
        last_present[e] = lp;
        last_absent[e] = la;
    }
}

// set-full-element-results, checker.clj:289-345
__global__ void __launch_bounds__(256) k_sf_final(int64_t M, const int64_t *__restrict__ time,
                                                  const unsigned long long *__restrict__ known_add,
                                                  const unsigned long long *__restrict__ known_read,
                                                  const long long *__restrict__ last_present,
                                                  const long long *__restrict__ last_absent,
                                                  long long *known, long long *slat, long long *llat,
                                                  uint8_t *fl_stable, uint8_t *fl_lost, uint8_t *fl_never,
                                                  uint8_t *fl_stale, long long *parts) {
    long long cs = 0, cl = 0, cn = 0, cst = 0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = min(known_add[e], known_read[e]);
        const long long kn = k == ~0ULL ? -1 : (long long)k;
        const long long lp = last_present[e], la = last_absent[e];
        const bool stable = lp >= 0 && la < lp;
        const bool lost = kn >= 0 && la >= 0 && lp < la && kn < la;
        long long s = -1, l = -1;
        if (stable) {
            const long long st = la >= 0 ? time[la] + 1 : 0;
            s = max(st - (long long)time[kn], 0LL) / 1000000;      // util/nanos->ms, long
        }
        if (lost) {
            const long long lt = lp >= 0 ? time[lp] + 1 : 0;
            l = max(lt - (long long)time[kn], 0LL) / 1000000;
        }
        const bool stale = stable && s > 0;
        known[e] = kn; slat[e] = s; llat[e] = l;
        fl_stable[e] = stable; fl_lost[e] = lost && !stable; fl_never[e] = !stable && !lost; fl_stale[e] = stale;
        cs += stable; cl += (lost && !stable); cn += (!stable && !lost); cst += stale;
    }
    __shared__ long long sh[4];
    cs = block_reduce256(cs, RedSum(), sh);
    cl = block_reduce256(cl, RedSum(), sh);
    cn = block_reduce256(cn, RedSum(), sh);
    cst = block_reduce256(cst, RedSum(), sh);
    if (threadIdx.x == 0) {
        long long *pp = parts + 8 * blockIdx.x;
        pp[0] = cs; pp[1] = cl; pp[2] = cn; pp[3] = cst;
    }
}

__global__ void __launch_bounds__(256) k_sf_final_fin(const long long *__restrict__ parts, int np, SfMeta *m) {
    long long c[4] = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < np; i += 256)
        for (int q = 0; q < 4; q++) c[q] += parts[8 * i + q];
    __shared__ long long sh[4];
    for (int q = 0; q < 4; q++) {
        const long long t = block_reduce256(c[q], RedSum(), sh);
        if (threadIdx.x == 0) m->cnt[q] = t;
    }
}

struct SfOut {
    long long q[2][JH_SF_QUANTILES];          // stable / lost latency quantiles
    jh_set_full_elem worst[JH_SF_WORST];
};
struct Pick5 { long long idx[JH_SF_QUANTILES]; };

__global__ void k_sf_pick(const long long *__restrict__ sorted, Pick5 pk, long long *q) {
    if (threadIdx.x < JH_SF_QUANTILES) q[threadIdx.x] = sorted[pk.idx[threadIdx.x]];
}

// worst-stale: the last k of the (latency, id)-sorted stale pairs, reversed
__global__ void k_sf_worst(const long long *__restrict__ lat_sorted, const int32_t *__restrict__ id_sorted,
                           int64_t ns, int k, const int64_t *__restrict__ elem, const long long *__restrict__ known,
                           const long long *__restrict__ last_absent, jh_set_full_elem *out) {
    const int i = threadIdx.x;
    if (i >= k) return;
    const int64_t src = ns - 1 - i;
    const int32_t id = id_sorted[src];
    out[i].element = elem[id];
    out[i].stable_latency = lat_sorted[src];
    out[i].known_entry = known[id];
    out[i].last_absent_entry = last_absent[id];
}

}  // namespace

void set_full_check(jh_ctx *ctx, const jh_history *dh, const int64_t *time_dev, bool linearizable, int64_t read_batch,
                    jh_set_full_result *res, int64_t *lists_out[3], int64_t list_cap, hipStream_t st) {
    memset(res, 0, sizeof *res);
    const int64_t n = dh->n;
    hipEvent_t e0 = ctx->ev[0], e1 = ctx->ev[1];
    HIP_TRY(hipEventRecord(e0, st));
    SfMeta *m = ctx->ws<SfMeta>(WS_SF_META, 1);
    SfMeta mh{};
    mh.vmin = LLONG_MAX; mh.vmax = LLONG_MIN;
    HIP_TRY(hipMemcpyAsync(m, &mh, sizeof mh, hipMemcpyHostToDevice, st));
    long long *parts = ctx->ws<long long>(WS_SF_PART, 8 * 2048);
    if (n > 0) {
        const int g = grid_for(n, 256, 2048);
        k_sf_scan<<<g, 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, dh->value2, n, parts);
        k_sf_scan_fin<<<1, 256, 0, st>>>(parts, g, m);
    }
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (mh.nil_elem) throw_jh(JH_EUNSUPPORTED, "nil set-full element");
    if (mh.n_reads > 0 && mh.read_elems > 0 && !dh->aux) throw_jh(JH_EINVAL, "set read without an aux element array");
    res->n_reads = mh.n_reads;
    res->read_elements = mh.read_elems;
    auto finish = [&](int64_t M) {
        res->attempt_count = M;
        res->stable_count = mh.cnt[0]; res->lost_count = mh.cnt[1];
        res->never_read_count = mh.cnt[2]; res->stale_count = mh.cnt[3];
        // checker.clj:398-402
        if (res->lost_count > 0) res->valid = JH_INVALID;
        else if (res->stable_count == 0) res->valid = JH_UNKNOWN;
        else if (linearizable && res->stale_count > 0) res->valid = JH_INVALID;
        else res->valid = JH_VALID;
        HIP_TRY(hipEventRecord(e1, st));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        res->device_ms = ms;
    };
    if (mh.n_inv == 0) { finish(0); return; }
    const unsigned long long span = (unsigned long long)(mh.vmax - mh.vmin) + 1;
    if (mh.vmax < mh.vmin || span >= (1ULL << 31))
        throw_jh(JH_EUNSUPPORTED, "set-full elements span 2^31 values or more");
    const long long vmin = mh.vmin, vmax = mh.vmax;

    // 2. dense ids in sorted value order
    uint32_t *flag = ctx->ws<uint32_t>(WS_SF_FLAG, span);
    int32_t *lut = ctx->ws<int32_t>(WS_SF_LUT, span);
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(uint32_t) * span, st));
    k_sf_mark<<<grid_for(n, 256), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n, vmin, flag);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, (uint32_t *)lut, (int64_t)span, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ctx->ws<char>(WS_SF_TMP, tb), tb, flag, (uint32_t *)lut, (int64_t)span, st));
    const int64_t cap_elem = mh.n_inv;                      // >= distinct elements
    int64_t *elem = ctx->ws<int64_t>(WS_SF_ELEM, cap_elem);
    k_sf_lut<<<grid_for(span, 256), 256, 0, st>>>(flag, lut, span, vmin, elem, m);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int64_t M = mh.n_elem;

    // 3. per-element state; 0xff bytes = -1 (signed) / none (unsigned)
    long long *st8 = ctx->ws<long long>(WS_SF_STATE, 5 * M);
    long long *last_inv = st8, *lp = st8 + M, *la = st8 + 2 * M;
    unsigned long long *kadd = (unsigned long long *)(st8 + 3 * M), *kread = (unsigned long long *)(st8 + 4 * M);
    HIP_TRY(hipMemsetAsync(st8, 0xff, sizeof(long long) * 5 * M, st));
    uint8_t *rflag = ctx->ws<uint8_t>(WS_SF_RFLAG, n);
    k_sf_addinv<<<grid_for(n, 256), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n, lut, vmin, last_inv);
    k_sf_okadd<<<grid_for(n, 256), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n, lut, vmin, vmax,
                                                last_inv, kadd, rflag);

    // 4. :ok reads in row order and their invocations
    const int64_t R = mh.n_reads;
    if (R > 0) {
        int64_t *rr = ctx->ws<int64_t>(WS_SF_READS, 2 * R + 1);
        int64_t *rrow = rr, *rinv = rr + R, *nsel = rr + 2 * R;
        hipcub::CountingInputIterator<int64_t> rows(0);
        tb = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, rows, rflag, rrow, nsel, n, st));
        HIP_TRY(hipcub::DeviceSelect::Flagged(ctx->ws<char>(WS_SF_TMP, tb), tb, rows, rflag, rrow, nsel, n, st));
        k_sf_inv<<<(unsigned)((R + 3) / 4), 256, 0, st>>>(dh->process, dh->type, dh->f, rrow, R, rinv, m);
        // (a bad read is reported after the outcomes' sync: the kernels below tolerate rinv = -1)

        // 5. bitmap batches: at most 2 GiB of bitmap and 65535 reads per batch
        const int64_t W = (M + 63) / 64;
        int64_t batch = std::max<int64_t>(1, ((int64_t)2 << 30) / (W * 8));
        batch = std::min<int64_t>({batch, (int64_t)65535, R});
        if (read_batch > 0) batch = std::min(batch, read_batch);
        unsigned long long *bits = ctx->ws<unsigned long long>(WS_SF_BITS, batch * W);   // [W][batch]
        const unsigned gx = (unsigned)std::max<int64_t>(1, (mh.max_cnt + BITS_CHUNK - 1) / BITS_CHUNK);
        for (int64_t r0 = 0; r0 < R; r0 += batch) {
            const int64_t nb = std::min(batch, R - r0);
            HIP_TRY(hipMemsetAsync(bits, 0, sizeof(unsigned long long) * batch * W, st));
            if (mh.max_cnt > 0)
                k_sf_bits<<<dim3(gx, (unsigned)nb), 256, 0, st>>>(dh->value, dh->value2, dh->aux, rrow, r0, lut,
                                                                 vmin, vmax, batch, bits);
            k_sf_elem<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(rrow, rinv, r0, nb, bits, batch, M, last_inv,
                                                                  kread, lp, la);
        }
    }

    // 6. outcomes
    long long *o8 = ctx->ws<long long>(WS_SF_OUT, 3 * M);
    long long *known = o8, *slat = o8 + M, *llat = o8 + 2 * M;
    uint8_t *fl = ctx->ws<uint8_t>(WS_SF_FL, 4 * M);
    uint8_t *f_stable = fl, *f_lost = fl + M, *f_never = fl + 2 * M, *f_stale = fl + 3 * M;
    {
        const int g = grid_for(M, 256, 2048);
        k_sf_final<<<g, 256, 0, st>>>(M, time_dev, kadd, kread, lp, la, known, slat, llat,
                                      f_stable, f_lost, f_never, f_stale, parts);
        k_sf_final_fin<<<1, 256, 0, st>>>(parts, g, m);
    }
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));

    if (mh.bad_read) throw_jh(JH_EINVAL, "an :ok :read without a read invocation before it");

    // 7. lists (own regions), quantiles and worst-stale (scratch regions),
    // all stream-ordered; one wait for the copies at the end
    int64_t *sel = ctx->ws<int64_t>(WS_SF_SEL, 7 * M + 128);
    int64_t *lst[3] = {sel, sel + M, sel + 2 * M};
    int64_t *a0 = sel + 3 * M, *a1 = sel + 4 * M, *a2 = sel + 5 * M, *a3 = sel + 6 * M, *ns = sel + 7 * M;
    SfOut *dout = (SfOut *)(ns + 8);
    auto select = [&](auto in, const uint8_t *flg, auto *out) {
        size_t t = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, t, in, flg, out, ns, M, st));
        HIP_TRY(hipcub::DeviceSelect::Flagged(ctx->ws<char>(WS_SF_TMP, t), t, in, flg, out, ns, M, st));
    };
    const int64_t counts[3] = {mh.cnt[1], mh.cnt[2], mh.cnt[3]};
    const uint8_t *lflags[3] = {f_lost, f_never, f_stale};
    for (int s = 0; s < 3; s++)
        if (std::min<int64_t>(counts[s], list_cap) > 0 && lists_out[s]) select(elem, lflags[s], lst[s]);
    const double points[JH_SF_QUANTILES] = {0, 0.5, 0.95, 0.99, 1};
    auto quantiles = [&](const long long *lat, const uint8_t *flg, int64_t c, int which) {
        select(lat, flg, (long long *)a0);
        size_t t = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, t, (long long *)a0, (long long *)a1, c, 0, 64, st));
        HIP_TRY(hipcub::DeviceRadixSort::SortKeys(ctx->ws<char>(WS_SF_TMP, t), t, (long long *)a0, (long long *)a1,
                                                  c, 0, 64, st));
        Pick5 pk;
        for (int i = 0; i < JH_SF_QUANTILES; i++)            // frequency-distribution, checker.clj:347-358
            pk.idx[i] = std::min<int64_t>(c - 1, (int64_t)std::floor((double)c * points[i]));
        k_sf_pick<<<1, 64, 0, st>>>((long long *)a1, pk, dout->q[which]);
    };
    if (mh.cnt[0] > 0) { quantiles(slat, f_stable, mh.cnt[0], 0); res->has_stable_latencies = 1; }
    if (mh.cnt[1] > 0) { quantiles(llat, f_lost, mh.cnt[1], 1); res->has_lost_latencies = 1; }
    if (mh.cnt[3] > 0) {
        const int64_t S = mh.cnt[3];
        select(slat, f_stale, (long long *)a0);
        select(hipcub::CountingInputIterator<int32_t>(0), f_stale, (int32_t *)a1);
        size_t t = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t, (long long *)a0, (long long *)a2, (int32_t *)a1,
                                                   (int32_t *)a3, S, 0, 64, st));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(ctx->ws<char>(WS_SF_TMP, t), t, (long long *)a0, (long long *)a2,
                                                   (int32_t *)a1, (int32_t *)a3, S, 0, 64, st));
        res->n_worst = (int)std::min<int64_t>(S, JH_SF_WORST);
        k_sf_worst<<<1, 64, 0, st>>>((long long *)a2, (int32_t *)a3, S, (int)res->n_worst, elem, known, la,
                                     dout->worst);
    }
    SfOut ho;
    HIP_TRY(hipMemcpyAsync(&ho, dout, sizeof ho, hipMemcpyDeviceToHost, st));
    for (int s = 0; s < 3; s++) {
        const int64_t k = std::min<int64_t>(counts[s], list_cap);
        if (k > 0 && lists_out[s])
            HIP_TRY(hipMemcpyAsync(lists_out[s], lst[s], sizeof(int64_t) * k, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (res->has_stable_latencies) memcpy(res->stable_latencies, ho.q[0], sizeof ho.q[0]);
    if (res->has_lost_latencies) memcpy(res->lost_latencies, ho.q[1], sizeof ho.q[1]);
    memcpy(res->worst_stale, ho.worst, sizeof(jh_set_full_elem) * res->n_worst);
    finish(M);
}
