// jh_counter.hip -- checker/counter on MI355X.
//
// Replaces (checker/counter), jepsen/src/jepsen/checker.clj:679-734:
//   history/complete, (remove :fails?), (remove op/fail?), then a sequential
//   loop carrying lower/upper bounds and pending reads.
// The loop is two prefix sums over the rows, in history order:
//   lower(row) = sum of :ok :add values before row        (checker.clj:725-726)
//   upper(row) = sum of non-failed :invoke :add values     (checker.clj:722-723)
// and each :ok :read emits [lower(its invocation) value upper(itself)]
// (checker.clj:713-720); errors are the triples with not (<= lower v upper).
//
// HBM-bound streaming passes (bytes per row read / written):
//   k_cnt_prange  process range                                        8 / 0
//   k_cnt_pack    packed row code (process - pmin) << 4 | f2 << 2 | type,
//                 last row per process (LDS-privatised), add-value range,
//                 and the complete pairing of every invocation whose
//                 completion lies in its 2048-row chunk                     32 / 8
//   k_cnt_pair_spill  pairing of the few invocations the chunk could not
//                 pair (thread per spill, walks its process' rows)          ~0
//   k_cnt_tile_sums / hipcub scan / k_cnt_tile_scan
//                 reduce-then-scan of {lower, upper, reads} over 2048-row
//                 tiles, per-row :fails?, orphan and nil checks fused in;
//                 writes only at read rows (the ok read's row and upper,
//                 the invoke read's lower)                                2 x 16 / ~0
//   k_cnt_triples the triples, in history order, errors, first failing row
//                 (over the ~1% read rows only)
// (A single-pass decoupled look-back scan over the 49 K tiles was measured
// at 20.8 ms on MI355X: the tile-to-tile look-back chain is serial latency
// across XCDs. Reduce-then-scan costs one extra 16 B/row read and is ~1 ms.)
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>

namespace {

constexpr int T_INVOKE = 0, T_OK = 1, T_FAIL = 2, T_INFO = 3;
constexpr int CHUNK = 2048, HSLOTS = 1024;

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

constexpr uint32_t F2_OTHER = 0, F2_ADD = 1, F2_READ = 2;
constexpr int RF_OKREAD = 1, RF_INVREAD = 2;

__global__ void __launch_bounds__(256) k_cnt_prange(const int64_t *__restrict__ proc, int64_t n, CntMeta *m) {
    long long lo = LLONG_MAX, hi = LLONG_MIN;
    const int64_t n2 = n / 2;
    const longlong2 *p2 = (const longlong2 *)proc;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const longlong2 x = p2[i];
        lo = min(lo, min(x.x, x.y)); hi = max(hi, max(x.x, x.y));
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) { lo = min(lo, (long long)proc[n - 1]); hi = max(hi, (long long)proc[n - 1]); }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    if (threadIdx.x == 0) { atomicMin(&m->pmin, lo); atomicMax(&m->pmax, hi); }
}

// packed row codes + last row of every process (per-chunk LDS hash of
// (process -> max row), then one global atomicMax per distinct process) +
// the add-value range for the overflow check, and the complete pairing of
// every invocation whose completion lies in the same chunk.
//
// Pairing (util.clj:606-640: an invocation's completion is the next
// non-:info row of its process): the chunk's first PAIR_PROCS distinct
// processes get a compact index c, and each 64-row group g of the chunk a
// bit mask M[g][c] of its non-:info rows of process c (one LDS atomicOr per
// row). An invocation's completion is then the lowest set bit after its own
// lane in M[g][c], or in the next group with a non-zero M[g'][c]: O(1) LDS
// reads per row. Invocations with no completion in the chunk, or of a
// process beyond the first PAIR_PROCS, go to a spill list (k_cnt_pair_spill).
constexpr int PAIR_PROCS = 32, PAIR_GROUPS = CHUNK / 64;
__global__ void __launch_bounds__(256) k_cnt_pack(const int64_t *__restrict__ proc,
                                                  const int64_t *__restrict__ type,
                                                  const int64_t *__restrict__ f,
                                                  const int64_t *__restrict__ val, int64_t n,
                                                  long long pmin, int32_t *__restrict__ last,
                                                  uint32_t *__restrict__ code, int32_t *__restrict__ pair,
                                                  int32_t *__restrict__ spill, unsigned int *__restrict__ n_spill,
                                                  CntMeta *m) {
    __shared__ uint32_t hk[HSLOTS];                 // process - pmin + 1 (0: empty)
    __shared__ int hv[HSLOTS];                      // its last row
    __shared__ int8_t hc[HSLOTS];                   // its compact index, -1 beyond PAIR_PROCS
    __shared__ uint32_t sc[CHUNK];                  // the chunk's row codes
    __shared__ int8_t rc[CHUNK];                    // each row's compact process index (-1: none)
    __shared__ unsigned long long M[PAIR_GROUPS][PAIR_PROCS];
    __shared__ int nd, nls, gbase;
    __shared__ int32_t ls[CHUNK];                   // this chunk's spilled invocations
    __shared__ long long sh[4];
    const int64_t c0 = (int64_t)blockIdx.x * CHUNK;
    const int nc = (int)min<int64_t>(CHUNK, n - c0);
    for (int i = threadIdx.x; i < HSLOTS; i += blockDim.x) { hk[i] = 0; hv[i] = -1; hc[i] = -1; }
    for (int i = threadIdx.x; i < PAIR_GROUPS * PAIR_PROCS; i += blockDim.x) (&M[0][0])[i] = 0;
    if (threadIdx.x == 0) { nd = 0; nls = 0; }
    __syncthreads();
    long long am = 0, na = 0;
    // all of this thread's rows in flight at once (the loop below waits on LDS)
    constexpr int PER = CHUNK / 256;
    long long rp[PER], rt[PER], rf[PER], rv[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = k * 256 + threadIdx.x;
        if (i < nc) { rp[k] = proc[c0 + i]; rt[k] = type[c0 + i]; rf[k] = f[c0 + i]; rv[k] = val[c0 + i]; }
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = k * 256 + threadIdx.x;
        if (i >= nc) break;
        const int64_t r = c0 + i;
        const long long p = rp[k];
        const int64_t ty = rt[k] & 3, ff = rf[k];
        const uint32_t f2 = ff == JH_F_ADD ? F2_ADD : ff == JH_F_READ ? F2_READ : F2_OTHER;
        const uint32_t pk = (uint32_t)(p - pmin);                                  // span < 2^28
        const uint32_t x = (pk << 4) | (f2 << 2) | (uint32_t)ty;
        code[r] = x;
        sc[i] = x;
        if (f2 == F2_ADD && (ty == T_INVOKE || ty == T_OK)) {
            const long long v = rv[k];
            if (v != JH_NIL) am = max(am, v < 0 ? (v == LLONG_MIN ? LLONG_MAX : -v) : v);
            na++;
        }
        uint32_t h = (uint32_t)jh_mix64((uint64_t)p) & (HSLOTS - 1);
        int slot = -1;
        for (int probe = 0; probe < 64; probe++) {
            uint32_t cur = hk[h];
            if (cur == 0) {
                cur = atomicCAS(&hk[h], 0u, pk + 1);
                if (cur == 0) {
                    const int c = atomicAdd(&nd, 1);
                    hc[h] = (int8_t)(c < PAIR_PROCS ? c : -1);
                    cur = pk + 1;
                }
            }
            if (cur == pk + 1) { slot = (int)h; break; }
            h = (h + 1) & (HSLOTS - 1);
        }
        if (slot >= 0) atomicMax(&hv[slot], (int)r);
        else atomicMax(&last[pk], (int)r);
        rc[i] = slot >= 0 ? (int8_t)-2 : (int8_t)-1;   // -2: in the hash; its index is read below
    }
    am = block_reduce256(am, RedMax(), sh);
    na = block_reduce256(na, RedSum(), sh);
    if (threadIdx.x == 0) {
        if (am) atomicMax(&m->amax_abs, am);
        if (na) atomicAdd((unsigned long long *)&m->n_add, (unsigned long long)na);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HSLOTS; i += blockDim.x)
        if (hk[i]) atomicMax(&last[hk[i] - 1], hv[i]);
    // compact process index of every row (the hash is complete now), and the
    // group masks of non-:info rows
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        int c = -1;
        if (rc[i] == -2) {
            const uint32_t pk = sc[i] >> 4;
            uint32_t h = (uint32_t)jh_mix64((uint64_t)((long long)pk + pmin)) & (HSLOTS - 1);
            while (hk[h] != pk + 1) h = (h + 1) & (HSLOTS - 1);
            c = hc[h];
        }
        rc[i] = (int8_t)c;
        if (c >= 0 && (sc[i] & 3) != T_INFO) atomicOr(&M[i >> 6][c], 1ULL << (i & 63));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        const uint32_t x = sc[i];
        if ((x & 3) != T_INVOKE) continue;
        const int64_t r = c0 + i;
        const int c = rc[i];
        int got = -1;
        if (c >= 0) {
            const int g = i >> 6, l = i & 63;
            const unsigned long long after = l == 63 ? 0ULL : (M[g][c] & (~0ULL << (l + 1)));
            if (after) got = (g << 6) + __builtin_ctzll(after);
            else
                for (int g2 = g + 1; g2 < PAIR_GROUPS && (g2 << 6) < nc; g2++)
                    if (M[g2][c]) { got = (g2 << 6) + __builtin_ctzll(M[g2][c]); break; }
        }
        if (got < 0) {
            ls[atomicAdd(&nls, 1)] = (int32_t)r;       // spills gather in LDS: one global atomic per chunk
        } else if ((sc[got] & 3) == T_INVOKE) {
            atomicMin(&m->viol1, ((unsigned long long)(c0 + got) << 4) | JH_CAUSE_DOUBLE_INVOKE);
        } else {
            pair[r] = (int32_t)(c0 + got);
            pair[c0 + got] = (int32_t)r;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && nls) gbase = (int)atomicAdd(n_spill, (unsigned int)nls);
    __syncthreads();
    for (int k = threadIdx.x; k < nls; k += blockDim.x) spill[gbase + k] = ls[k];
}

// the spilled invocations: one thread each walks the codes forward to the
// completion, or past its process' last row (no completion: stays open)
__global__ void __launch_bounds__(256) k_cnt_pair_spill(const uint32_t *__restrict__ code, int64_t n,
                                                        const int32_t *__restrict__ last,
                                                        const int32_t *__restrict__ spill,
                                                        const unsigned int *__restrict__ n_spill,
                                                        int32_t *__restrict__ pair, CntMeta *m) {
    const unsigned int ns = *n_spill;
    for (unsigned int s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x) {
        const int64_t r = spill[s];
        const uint32_t p = code[r] >> 4;
        const int64_t lr = last[p];
        for (int64_t j = r + 1; j <= lr; j++) {
            const uint32_t y = code[j];
            if ((y >> 4) != p || (y & 3) == T_INFO) continue;
            if ((y & 3) == T_INVOKE) atomicMin(&m->viol1, ((unsigned long long)j << 4) | JH_CAUSE_DOUBLE_INVOKE);
            else { pair[r] = (int32_t)j; pair[j] = (int32_t)r; }
            break;
        }
    }
}

// per-row contributions and prefixes of lower / upper / ok reads; flags mark
// the read rows
struct CntAcc {
    long long lo, hi;
    int nr, flags;
};

// per-row contribution (checker.clj:709-727 after complete / remove :fails?);
// orphans, :fails? and nil checks fused in
__device__ __forceinline__ CntAcc cnt_row(const uint32_t *__restrict__ code, const int32_t *__restrict__ pair,
                                          const int64_t *__restrict__ val, CntMeta *m, int64_t r) {
    const uint32_t x = code[r];
    const uint32_t ty = x & 3, f2 = (x >> 2) & 3;
    const int32_t c = pair[r];
    CntAcc a{0, 0, 0, 0};
    if ((ty == T_OK || ty == T_FAIL) && c < 0)
        atomicMin(&m->viol1, ((unsigned long long)r << 4) | JH_CAUSE_ORPHAN);
    if (f2 == F2_ADD) {
        if (ty == T_INVOKE) {
            const bool failed = c >= 0 && (code[c] & 3) == T_FAIL;
            if (!failed) {
                long long v = val[r];
                if (v == JH_NIL && c >= 0) v = val[c];          // (or inv ok)
                if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
                else a.hi = v;
            }
        } else if (ty == T_OK) {
            const long long v = val[r];
            if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
            else a.lo = v;
        }
    } else if (f2 == F2_READ) {
        if (ty == T_OK) {
            // its pending read must come from an [:invoke :read] (checker.clj:713-716)
            if (c < 0 || ((code[c] >> 2) & 3) != F2_READ)
                atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_ORPHAN);
            else { a.nr = 1; a.flags = RF_OKREAD; }
        } else if (ty == T_INVOKE) {
            a.flags = RF_INVREAD;
        }
    }
    return a;
}

// Reduce-then-scan over tiles of CNT_TILE rows (the rows of a tile are read
// twice, 16 B each time: 32 B/row in all, coalesced).
constexpr int CNT_TILE = 2048, CNT_PER = CNT_TILE / 256;

__global__ void __launch_bounds__(256) k_cnt_tile_sums(const uint32_t *__restrict__ code,
                                                       const int32_t *__restrict__ pair,
                                                       const int64_t *__restrict__ val, int64_t n,
                                                       CntMeta *m, CntAcc *__restrict__ agg) {
    __shared__ long long sh[4];
    const int64_t base = (int64_t)blockIdx.x * CNT_TILE;
    long long lo = 0, hi = 0, nr = 0;
#pragma unroll
    for (int k = 0; k < CNT_PER; k++) {
        const int64_t r = base + k * 256 + threadIdx.x;
        if (r < n) { const CntAcc a = cnt_row(code, pair, val, m, r); lo += a.lo; hi += a.hi; nr += a.nr; }
    }
    lo = block_reduce256(lo, RedSum(), sh);
    hi = block_reduce256(hi, RedSum(), sh);
    nr = block_reduce256(nr, RedSum(), sh);
    if (threadIdx.x == 0) agg[blockIdx.x] = CntAcc{lo, hi, (int)nr, 0};
}

// rows in order within the tile (LDS transpose: thread t takes rows
// CNT_PER*t ..), from the tile's exclusive prefix; writes only at read rows
__global__ void __launch_bounds__(256) k_cnt_tile_scan(const uint32_t *__restrict__ code,
                                                       const int32_t *__restrict__ pair,
                                                       const int64_t *__restrict__ val, int64_t n,
                                                       CntMeta *m, const CntAcc *__restrict__ pre,
                                                       int32_t *__restrict__ rd_row, int64_t *__restrict__ rd_hi,
                                                       int64_t *__restrict__ lo_at, CntAcc *total) {
    // a row feeds at most one of lower / upper / reads: LDS holds its value
    // and a kind byte (20 KB per block: occupancy hides the HBM latency)
    constexpr int PAD = CNT_TILE + CNT_TILE / CNT_PER;
    __shared__ long long s_v[PAD];
    __shared__ uint8_t s_k[PAD];
    __shared__ long long sc[3][4];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * CNT_TILE;
#pragma unroll
    for (int k = 0; k < CNT_PER; k++) {
        const int j = k * 256 + tid;
        const int64_t r = base + j;
        CntAcc a{0, 0, 0, 0};
        if (r < n) a = cnt_row(code, pair, val, m, r);
        const int q = j + j / CNT_PER;
        s_v[q] = a.lo ? a.lo : a.hi;
        s_k[q] = (uint8_t)(a.lo ? 1 : a.hi ? 2 : a.flags == RF_OKREAD ? 3 : a.flags == RF_INVREAD ? 4 : 0);
    }
    __syncthreads();
    long long lo = 0, hi = 0, nr = 0;
    const int q0 = tid * (CNT_PER + 1);
#pragma unroll
    for (int j = 0; j < CNT_PER; j++) {
        const int kd = s_k[q0 + j];
        const long long v = s_v[q0 + j];
        lo += kd == 1 ? v : 0; hi += kd == 2 ? v : 0; nr += kd == 3;
    }
    // block exclusive scan of the per-thread sums: wave shuffles, then the
    // totals of the waves before
    long long il = lo, ih = hi, in = nr;
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long a0 = __shfl_up(il, o), a1 = __shfl_up(ih, o), a2 = __shfl_up(in, o);
        if (lane >= o) { il += a0; ih += a1; in += a2; }
    }
    if (lane == 63) { sc[0][wv] = il; sc[1][wv] = ih; sc[2][wv] = in; }
    __syncthreads();
    for (int w = 0; w < wv; w++) { il += sc[0][w]; ih += sc[1][w]; in += sc[2][w]; }
    const CntAcc p = pre[blockIdx.x];
    long long rl = p.lo + il - lo, rh = p.hi + ih - hi, rn = p.nr + in - nr;
#pragma unroll
    for (int j = 0; j < CNT_PER; j++) {
        const int kd = s_k[q0 + j];
        const long long v = s_v[q0 + j];
        rl += kd == 1 ? v : 0; rh += kd == 2 ? v : 0; rn += kd == 3;
        const int64_t r = base + (int64_t)tid * CNT_PER + j;
        if (kd == 3) { rd_row[rn - 1] = (int32_t)r; rd_hi[rn - 1] = rh; }
        else if (kd == 4) lo_at[r] = rl;
        if (r == n - 1) *total = CntAcc{rl, rh, (int)rn, 0};
    }
}

struct CntSumOp {
    __host__ __device__ CntAcc operator()(const CntAcc &a, const CntAcc &b) const {
        return CntAcc{a.lo + b.lo, a.hi + b.hi, a.nr + b.nr, 0};
    }
};

__global__ void k_cnt_triples(const int32_t *__restrict__ rd_row, const int64_t *__restrict__ rd_hi,
                              const int64_t *__restrict__ lo_at, const int32_t *__restrict__ pair,
                              const int64_t *__restrict__ val, int64_t nr, int64_t *__restrict__ out,
                              int64_t cap, CntMeta *m) {
    long long nerr = 0;
    unsigned long long ferr = ~0ULL;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nr;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = rd_row[i];
        const int32_t inv = pair[r];
        int64_t v = val[inv];
        if (v == JH_NIL) v = val[r];
        const int64_t l = lo_at[inv], u = rd_hi[i];
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
    k_cnt_prange<<<grid_for(n / 2 + 1, 256, 2048), 256, 0, st>>>(dh->process, n, m);
    CntMeta mh;
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const unsigned long long span = (unsigned long long)(mh.pmax - mh.pmin);
    if (span >= (1ULL << 28)) throw_jh(JH_EUNSUPPORTED, "process ids span more than 2^28");

    int32_t *last = ctx->ws<int32_t>(WS_C_LAST, span + 1);
    int32_t *pair = ctx->ws<int32_t>(WS_C_PAIR, n);
    uint32_t *code = ctx->ws<uint32_t>(WS_C_PT, n);
    HIP_TRY(hipMemsetAsync(last, 0xFF, sizeof(int32_t) * (span + 1), st));
    HIP_TRY(hipMemsetAsync(pair, 0xFF, sizeof(int32_t) * n, st));
    int32_t *spill = ctx->ws<int32_t>(WS_C_IDX, n);          // reused for the read rows below
    unsigned int *n_spill = (unsigned int *)ctx->ws<int32_t>(WS_C_FLAG, 4);
    HIP_TRY(hipMemsetAsync(n_spill, 0, sizeof(unsigned int), st));
    k_cnt_pack<<<(int)((n + CHUNK - 1) / CHUNK), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n,
                                                              mh.pmin, last, code, pair, spill, n_spill, m);
    k_cnt_pair_spill<<<grid_for(n / 64 + 1, 256, 4096), 256, 0, st>>>(code, n, last, spill, n_spill, pair, m);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // Clojure + throws on long overflow; if no prefix can overflow we need no
    // ordered overflow check (else the shim falls back to the JVM checker).
    if (mh.amax_abs > 0 && (unsigned long long)mh.amax_abs > (unsigned long long)(LLONG_MAX / std::max(1LL, mh.n_add)))
        throw_jh(JH_EUNSUPPORTED, "add values large enough to overflow a long");

    // reduce-then-scan over tiles of rows
    int32_t *rd_row = ctx->ws<int32_t>(WS_C_IDX, n);
    int64_t *rd_hi = ctx->ws<int64_t>(WS_C_HI, n);
    int64_t *lo_at = ctx->ws<int64_t>(WS_C_LO, n);
    const int64_t n_tiles = (n + CNT_TILE - 1) / CNT_TILE;
    CntAcc *agg = ctx->ws<CntAcc>(WS_C_OUT2, 2 * n_tiles + 1);
    CntAcc *pre = agg + n_tiles;
    CntAcc *total = pre + n_tiles;
    k_cnt_tile_sums<<<(unsigned)n_tiles, 256, 0, st>>>(code, pair, dh->value, n, m, agg);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tb, agg, pre, CntSumOp(), CntAcc{0, 0, 0, 0}, (int)n_tiles, st));
    void *tmp = ctx->ws<char>(WS_S_TMP, tb);
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(tmp, tb, agg, pre, CntSumOp(), CntAcc{0, 0, 0, 0}, (int)n_tiles, st));
    k_cnt_tile_scan<<<(unsigned)n_tiles, 256, 0, st>>>(code, pair, dh->value, n, m, pre, rd_row, rd_hi, lo_at, total);
    CntAcc th;
    HIP_TRY(hipMemcpyAsync(&th, total, sizeof th, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int64_t nr = th.nr;
    const int64_t cap = std::min(nr, reads_cap);
    int64_t *out = ctx->ws<int64_t>(WS_C_OUT, 3 * std::max<int64_t>(cap, 1));
    if (nr > 0)
        k_cnt_triples<<<grid_for(nr, 256, 4096), 256, 0, st>>>(rd_row, rd_hi, lo_at, pair, dh->value, nr,
                                                              out, cap, m);
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
