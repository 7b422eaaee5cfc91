// jh_set.hip -- checker/set on MI355X.
//
// Replaces (checker/set), jepsen/src/jepsen/checker.clj:182-233:
//   attempts = #{:value of every :invoke :add}     (:190-194)
//   adds     = #{:value of every :ok :add}         (:195-199)
//   final-read = :value of the LAST :ok :read      (:200-204)
//   ok = R n attempts, unexpected = R - attempts, lost = adds - R,
//   recovered = ok - adds                          (:210-223)
// plus counts and util/integer-interval-set-str strings (util.clj:536-575),
// which the library returns as sorted runs [lo hi] for the host to format.
//
// Elements live in [vmin, vmax]; each of the three sets is a bitmap over that
// span (atomicOr of 32-bit words), every set operation is a word-wise
// boolean, and runs fall out of the bit boundaries of each word.
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>

namespace {
constexpr int T_INVOKE = 0, T_OK = 1;

struct SetMeta {
    long long vmin, vmax;
    long long final_row;
    int nil_attempt, nil_add;
    long long cnt[10];         // attempt, ack, ok, lost, recovered, unexpected; runs of ok, lost, unexpected, recovered
    unsigned long long first_lost_row;
};

// Row pairs: both rows in one 16-byte load when the columns are 16-byte
// aligned (vec; workspace and torch allocations are), two 8-byte loads
// otherwise; a trailing odd row is the last pair's first half
__device__ __forceinline__ longlong2 ld_pair(const int64_t *__restrict__ c, int64_t i, int64_t n, bool vec) {
    if (2 * i + 1 < n) return vec ? ((const longlong2 *)c)[i] : make_longlong2(c[2 * i], c[2 * i + 1]);
    return make_longlong2(c[2 * i], 0);
}

#ifndef JH_SCAN_GRID
#define JH_SCAN_GRID 8192     // grid caps of the scan and the byte-map pass (profiles/r04/c2_spill/r4sgrid_*: scan 2048 / 4096 / 8192 / 16384 blocks 493 / 483-501 / 456-458 / 509-516 us)
#endif
#ifndef JH_BYTES_GRID
#define JH_BYTES_GRID 16384
#endif
#ifndef JH_SET_CODE_WIDE
#define JH_SET_CODE_WIDE 0   // eight lanes' codes in one 16-byte store (A/B)
#endif
#ifndef JH_SET_CODE
#define JH_SET_CODE 1        // the scan leaves a byte per row (1 :invoke :add, 2 :ok :add) for the byte-map pass
#endif
__global__ void __launch_bounds__(256) k_set_scan(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                           const int64_t *__restrict__ val, int64_t n, int vec, SetMeta *m,
                           uint16_t *__restrict__ code) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, fr = -1;
    int na = 0, nd = 0;
    const int64_t np = (n + 1) / 2;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    // software-pipelined: the next pair's loads are issued before this pair's
    // code store (stores and loads share one in-order counter on CDNA: a store
    // issued before a load would make the wait for that load wait for it too)
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    longlong2 t2 = make_longlong2(0, 0), f2 = t2, v2 = t2;
    if (i < np) { t2 = ld_pair(type, i, n, vec); f2 = ld_pair(f, i, n, vec); v2 = ld_pair(val, i, n, vec); }
#if JH_SET_CODE_WIDE
    // the loop runs while any lane of the wave has a pair (every lane takes
    // part in the shuffles that gather eight lanes' codes into one 16-byte
    // store; a lane past the end carries code 0)
    const int64_t i_lane0 = i - (threadIdx.x & 63);
    for (int64_t w0 = i_lane0; w0 < np; w0 += gs, i += gs) {
        const bool live = i < np;
#else
    for (; i < np; i += gs) {
        const bool live = true;
#endif
        const int64_t tt[2] = {t2.x, t2.y}, ffs[2] = {f2.x, f2.y}, vv[2] = {v2.x, v2.y};
        if (i + gs < np) { t2 = ld_pair(type, i + gs, n, vec); f2 = ld_pair(f, i + gs, n, vec); v2 = ld_pair(val, i + gs, n, vec); }
        uint32_t cc = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int64_t r = 2 * i + k;
            if (!live || r >= n) break;
            const int64_t ty = tt[k], ff = ffs[k];
            if (ff == JH_F_ADD && (ty == T_INVOKE || ty == T_OK)) {
                const int64_t v = vv[k];
                if (v == JH_NIL) { if (ty == T_INVOKE) na = 1; else nd = 1; }
                else { lo = min(lo, (long long)v); hi = max(hi, (long long)v); }
                cc |= (ty == T_INVOKE ? 1u : 2u) << (8 * k);
            } else if (ff == JH_F_READ && ty == T_OK) fr = max(fr, (long long)r);
        }
#if JH_SET_CODE_WIDE
        if (code) {
            const uint32_t x = cc | ((uint32_t)__shfl_down((int)cc, 1) << 16);     // lanes l, l + 1
            const uint32_t y1 = (uint32_t)__shfl_down((int)x, 2), y2 = (uint32_t)__shfl_down((int)x, 4),
                           y3 = (uint32_t)__shfl_down((int)x, 6);
            if ((threadIdx.x & 7) == 0 && live) ((uint4 *)code)[i >> 3] = make_uint4(x, y1, y2, y3);
        }
#else
        if (code) code[i] = (uint16_t)cc;
#endif
    }
    __shared__ long long sh[4];
    __shared__ int shi[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    fr = block_reduce256(fr, RedMax(), sh);
    na = block_reduce256(na, RedOr(), shi);
    nd = block_reduce256(nd, RedOr(), shi);
    if (threadIdx.x == 0) {
        if (lo != LLONG_MAX) atomicMin(&m->vmin, lo);
        if (hi != LLONG_MIN) atomicMax(&m->vmax, hi);
        if (fr >= 0) atomicMax(&m->final_row, fr);
        if (na) atomicOr(&m->nil_attempt, 1);
        if (nd) atomicOr(&m->nil_add, 1);
    }
}

// the final read's element range (its first element need not be 16-byte
// aligned: the aligned pairs inside it go four per thread per step, so four
// 16-byte loads are in flight; the odd elements at either end, thread 0).
// Round 4 (profiles/r04/c2_spill/r4unroll_*): 128 -> 119 us per 47 M
// elements; the same unrolling of k_cnt_prange and of k_set_scan (two row
// pairs per step) measured flat / slower, not kept.
#ifndef JH_RANGE_UNROLL
#define JH_RANGE_UNROLL 4
#endif
__global__ void __launch_bounds__(256) k_set_range(const int64_t *__restrict__ aux, int64_t off, int64_t cnt, int vec, SetMeta *m) {
    long long lo = LLONG_MAX, hi = LLONG_MIN;
    const int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
    if (vec) {
        const int64_t a0 = (off + 1) & ~1LL, a1 = (off + cnt) & ~1LL;
        const int64_t np = a1 > a0 ? (a1 - a0) / 2 : 0;
        const longlong2 *p2 = (const longlong2 *)(aux + a0);
        for (int64_t i = gt; i < np; i += JH_RANGE_UNROLL * gs) {
            longlong2 x[JH_RANGE_UNROLL];
#pragma unroll
            for (int u = 0; u < JH_RANGE_UNROLL; u++) x[u] = p2[i + u * gs < np ? i + u * gs : i];   // (a repeat is harmless)
#pragma unroll
            for (int u = 0; u < JH_RANGE_UNROLL; u++) { lo = min(lo, min(x[u].x, x[u].y)); hi = max(hi, max(x[u].x, x[u].y)); }
        }
        if (gt == 0) {
            if (a0 > off && cnt > 0) { const long long v = aux[off]; lo = min(lo, v); hi = max(hi, v); }
            if (a1 < off + cnt && a1 >= a0) { const long long v = aux[a1]; lo = min(lo, v); hi = max(hi, v); }
        }
    } else {
        for (int64_t j = off + gt; j < off + cnt; j += gs) { const long long v = aux[j]; lo = min(lo, v); hi = max(hi, v); }
    }
    __shared__ long long sh[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    if (threadIdx.x == 0) {
        if (lo != LLONG_MAX) atomicMin(&m->vmin, lo);
        if (hi != LLONG_MIN) atomicMax(&m->vmax, hi);
    }
}

// Marking: each workgroup takes a contiguous chunk of MARK_CH rows (or read
// elements) and merges its bits in LDS before touching HBM.
//  * Within a wave, lanes holding the same bitmap word are merged by a
//    segmented OR scan over lanes (shuffles); only the last lane of each run
//    writes. Jepsen's set elements are mostly written and read in ascending
//    order, so a wave's 64 elements fall into two or three words.
//  * Those few writes go to a direct-mapped LDS cache of words (tag + bits);
//    a word whose slot holds another word goes straight to HBM.
//  * At the end the cache is flushed: one global atomicOr per cached word.
// Any element order stays correct (unmerged lanes just write on their own).
constexpr int MARK_CH = 16384, MARK_SLOTS = 2048;
constexpr long long MARK_EMPTY = -1;

__device__ __forceinline__ void mark_bits(uint32_t *bm, long long *tag, uint32_t *lb, long long w, uint32_t bits) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long wn = __shfl_up(w, o);
        const uint32_t bn = (uint32_t)__shfl_up((int)bits, o);
        if (lane >= o && wn == w) bits |= bn;
    }
    const long long wnext = __shfl_down(w, 1);
    const bool tail = lane == 63 || wnext != w;
    if (w < 0 || !tail) return;
    const int sl = (int)(w & (MARK_SLOTS - 1));
    long long t = tag[sl];
    if (t == MARK_EMPTY)
        t = (long long)atomicCAS((unsigned long long *)&tag[sl], (unsigned long long)MARK_EMPTY, (unsigned long long)w);
    if (t == MARK_EMPTY || t == w) atomicOr(&lb[sl], bits);
    else atomicOr(&bm[w], bits);
}

__device__ __forceinline__ void mark_init(long long *tag, uint32_t *lb) {
    for (int i = threadIdx.x; i < MARK_SLOTS; i += blockDim.x) { tag[i] = MARK_EMPTY; lb[i] = 0; }
    __syncthreads();
}
__device__ __forceinline__ void mark_flush(uint32_t *bm, const long long *tag, const uint32_t *lb) {
    __syncthreads();
    for (int i = threadIdx.x; i < MARK_SLOTS; i += blockDim.x)
        if (tag[i] != MARK_EMPTY && lb[i]) atomicOr(&bm[tag[i]], lb[i]);
}

// one pass over the rows (24 B each): :invoke :add elements into A, :ok :add
// elements into D
__global__ void __launch_bounds__(256) k_set_mark_rows(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                                                       const int64_t *__restrict__ val, int64_t n, long long vmin,
                                                       uint32_t *__restrict__ A, uint32_t *__restrict__ D) {
    __shared__ long long ta[MARK_SLOTS], td[MARK_SLOTS];
    __shared__ uint32_t ba[MARK_SLOTS], bd[MARK_SLOTS];
    mark_init(ta, ba);
    mark_init(td, bd);
    const int64_t c0 = (int64_t)blockIdx.x * MARK_CH, c1 = min(n, c0 + MARK_CH);
    for (int64_t base = c0; base < c1; base += blockDim.x) {      // same trip count for every lane
        const int64_t r = base + threadIdx.x;
        long long wa = -1, wd = -1;
        uint32_t bit = 0;
        if (r < c1 && f[r] == JH_F_ADD) {
            const int64_t ty = type[r];
            if (ty == T_INVOKE || ty == T_OK) {
                const uint64_t b = (uint64_t)(val[r] - vmin);
                bit = 1u << (b & 31);
                if (ty == T_INVOKE) wa = (long long)(b >> 5); else wd = (long long)(b >> 5);
            }
        }
        mark_bits(A, ta, ba, wa, bit);
        mark_bits(D, td, bd, wd, bit);
    }
    mark_flush(A, ta, ba);
    mark_flush(D, td, bd);
}

// one pass over the final read's elements (8 B each) into R
__global__ void __launch_bounds__(256) k_set_mark_read(const int64_t *__restrict__ aux, int64_t off, int64_t cnt,
                                                       long long vmin, uint32_t *__restrict__ R) {
    __shared__ long long tr[MARK_SLOTS];
    __shared__ uint32_t br[MARK_SLOTS];
    mark_init(tr, br);
    const int64_t c0 = (int64_t)blockIdx.x * MARK_CH, c1 = min(cnt, c0 + MARK_CH);
    for (int64_t base = c0; base < c1; base += blockDim.x) {
        const int64_t i = base + threadIdx.x;
        long long w = -1;
        uint32_t bit = 0;
        if (i < c1) {
            const uint64_t b = (uint64_t)(aux[off + i] - vmin);
            w = (long long)(b >> 5);
            bit = 1u << (b & 31);
        }
        mark_bits(R, tr, br, w, bit);
    }
    mark_flush(R, tr, br);
}

// Dense spans (up to RB_SPAN_MAX elements): the attempts and acknowledged
// sets go through byte maps -- plain idempotent byte stores in row order (set
// elements are added in ascending order in Jepsen's set workloads, so the
// stores are nearly sequential), then one packing pass -- and the final read,
// whose elements come in any order (hash order on the JVM), is bucketed by
// element range before its bits are set in LDS (k_rb_*): round 2 stored one
// byte per read element straight into a byte map, and each random byte store
// cost a 32-byte write at the memory side (WRITE_SIZE 1.5 GB for 47 M
// elements).
constexpr unsigned long long RB_SPAN_MAX = 1ULL << 31;
constexpr int RB_CH = 8192;         // read elements per block of the histogram / scatter passes
constexpr int RB_MAXBINS = 4096;    // element-range buckets
constexpr int RB_MAXSB = 19;        // 2^19 elements per bucket at most: a 64 KB LDS bitmap

// runs of one value in consecutive lanes: each lane's run start lane and the
// run's length (one LDS atomic per run instead of per lane: sorted input puts
// a whole wave on one address, random input spreads it)
__device__ __forceinline__ void lane_runs(long long v, int &start, int &len) {
    const int lane = threadIdx.x & 63;
    const long long pv = __shfl_up(v, 1);
    const uint64_t hm = __ballot(lane == 0 || pv != v);
    const uint64_t upto = lane == 63 ? ~0ULL : ((2ULL << lane) - 1);
    start = 63 - __builtin_clzll(hm & upto);
    const uint64_t after = hm & ~upto;
    len = (after ? __builtin_ctzll(after) : 64) - start;
}

__global__ void __launch_bounds__(256) k_rb_hist(const int64_t *__restrict__ e, int64_t cnt, long long vmin, int sb,
                                                 int nbins, int nblk, uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t lh[];
    for (int i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t c0 = (int64_t)blockIdx.x * RB_CH, c1 = min(cnt, c0 + RB_CH);
    for (int64_t base = c0; base < c1; base += 1024) {       // same trip count for every lane
        long long v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { const int64_t i = base + k * 256 + threadIdx.x; v[k] = i < c1 ? e[i] : 0; }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t i = base + k * 256 + threadIdx.x;
            const long long b = i < c1 ? (long long)((uint64_t)(v[k] - vmin) >> sb) : -1;
            int s0, len;
            lane_runs(b, s0, len);
            if (b >= 0 && lane == s0) atomicAdd(&lh[b], (uint32_t)len);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += blockDim.x) hist[(size_t)i * nblk + blockIdx.x] = lh[i];
}

// each element's offset in its bucket, at the bucket's next free position
// (pos: the exclusive scan of hist, bucket-major). The block's elements are
// first sorted by bucket in LDS, then written out as one contiguous run per
// bucket: a 4-byte store per element to a random bucket cost a 32-byte write
// at the memory side.
__global__ void __launch_bounds__(256) k_rb_scatter(const int64_t *__restrict__ e, int64_t cnt, long long vmin, int sb,
                                                    int nbins, int nblk, const uint32_t *__restrict__ hist,
                                                    const uint32_t *__restrict__ pos, uint32_t *__restrict__ out) {
    extern __shared__ uint32_t lds_rb[];
    uint32_t *loff = lds_rb, *gb = loff + nbins, *cur = gb + nbins;
    uint32_t *st_low = cur + nbins;
    uint16_t *st_bin = (uint16_t *)(st_low + RB_CH);
    __shared__ uint32_t part[256];
    const int tid = threadIdx.x, lane = tid & 63;
    // the block's bucket counts -> local offsets (a block scan over the buckets)
    const int per = (nbins + 255) / 256;
    uint32_t acc = 0;
    for (int k = 0; k < per; k++) {
        const int bi = tid * per + k;
        if (bi < nbins) acc += hist[(size_t)bi * nblk + blockIdx.x];
    }
    part[tid] = acc;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t v = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    acc = part[tid] - acc;                          // exclusive prefix of this thread's first bucket
    for (int k = 0; k < per; k++) {
        const int bi = tid * per + k;
        if (bi < nbins) {
            loff[bi] = acc; cur[bi] = acc;
            gb[bi] = pos[(size_t)bi * nblk + blockIdx.x];
            acc += hist[(size_t)bi * nblk + blockIdx.x];
        }
    }
    __syncthreads();
    const uint64_t lowm = (1ULL << sb) - 1;
    const int64_t c0 = (int64_t)blockIdx.x * RB_CH, c1 = min(cnt, c0 + RB_CH);
    for (int64_t base = c0; base < c1; base += 1024) {
        long long v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { const int64_t i = base + k * 256 + tid; v[k] = i < c1 ? e[i] : 0; }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t i = base + k * 256 + tid;
            const uint64_t d = (uint64_t)(v[k] - vmin);
            const long long b = i < c1 ? (long long)(d >> sb) : -1;
            int s0, len;
            lane_runs(b, s0, len);
            uint32_t p0 = 0;
            if (b >= 0 && lane == s0) p0 = atomicAdd(&cur[b], (uint32_t)len);
            p0 = (uint32_t)__shfl((int)p0, s0);
            if (b >= 0) {
                const uint32_t lp = p0 + (uint32_t)(lane - s0);
                st_low[lp] = (uint32_t)(d & lowm);
                st_bin[lp] = (uint16_t)b;
            }
        }
    }
    __syncthreads();
    const int nb = (int)(c1 - c0);
    for (int i = tid; i < nb; i += 256) {
        const uint32_t bi = st_bin[i];
        out[gb[bi] + ((uint32_t)i - loff[bi])] = st_low[i];
    }
}

// one block per bucket: its elements' bits in an LDS bitmap, then every word
// of the bucket's range written out (so R needs no clearing)
__global__ void __launch_bounds__(1024) k_rb_build(const uint32_t *__restrict__ in, const uint32_t *__restrict__ pos,
                                                  int nblk, int nbins, int64_t cnt, int sb, int64_t nw,
                                                  uint32_t *__restrict__ R) {
    extern __shared__ uint32_t bits[];
    const int words = 1 << (sb - 5);
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < words; i += blockDim.x) bits[i] = 0;
    __syncthreads();
    const int b = blockIdx.x;
    const int64_t s0 = pos[(size_t)b * nblk];
    const int64_t s1 = b + 1 < nbins ? (int64_t)pos[(size_t)(b + 1) * nblk] : cnt;
    // eight elements per thread in flight; lanes holding one word are
    // OR-combined first (a segmented scan) only when neighbouring lanes share
    // words at all (sorted input), else each lane sets its bit directly
    for (int64_t base = s0; base < s1; base += 8 * (int64_t)blockDim.x) {
        uint32_t xs[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int64_t i = base + k * (int64_t)blockDim.x + threadIdx.x;
            xs[k] = i < s1 ? in[i] : ~0u;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const long long w = xs[k] != ~0u ? (long long)(xs[k] >> 5) : -1;
            uint32_t bit = xs[k] != ~0u ? 1u << (xs[k] & 31) : 0u;
            const long long pw = __shfl_up(w, 1);
            if (__ballot(lane > 0 && w >= 0 && pw == w)) {
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const long long wn = __shfl_up(w, o);
                    const uint32_t bn = (uint32_t)__shfl_up((int)bit, o);
                    if (lane >= o && wn == w) bit |= bn;
                }
                const long long wnext = __shfl_down(w, 1);
                if (w >= 0 && (lane == 63 || wnext != w)) atomicOr(&bits[w], bit);
            } else if (w >= 0) {
                atomicOr(&bits[w], bit);
            }
        }
    }
    __syncthreads();
    const int64_t w0 = (int64_t)b * words;
    for (int i = threadIdx.x; i < words; i += blockDim.x)
        if (w0 + i < nw) R[w0 + i] = bits[i];
}

// one pass over the rows (24 B each, row pairs): :invoke :add elements into the
// A byte map, :ok :add elements into D, and the first lost row -- the lowest
// :ok :add whose element the final read R lacks (lost = adds - R,
// checker.clj:214-215)
__global__ void __launch_bounds__(256) k_set_bytes_rows(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                                                        const int64_t *__restrict__ val, int64_t n, long long vmin,
                                                        uint8_t *__restrict__ Ab, uint8_t *__restrict__ Db,
                                                        const uint32_t *__restrict__ R, int vec, SetMeta *m) {
    unsigned long long best = ~0ULL;
    const int64_t np = (n + 1) / 2;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
        const longlong2 t2 = ld_pair(type, i, n, vec), f2 = ld_pair(f, i, n, vec), v2 = ld_pair(val, i, n, vec);
        const int64_t tt[2] = {t2.x, t2.y}, ffs[2] = {f2.x, f2.y}, vv[2] = {v2.x, v2.y};
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int64_t r = 2 * i + k;
            if (r >= n || ffs[k] != JH_F_ADD) continue;
            const int64_t b = vv[k] - vmin;
            if (tt[k] == T_INVOKE) Ab[b] = 1;
            else if (tt[k] == T_OK) {
                Db[b] = 1;
                if (!((R[b >> 5] >> (b & 31)) & 1)) best = min(best, (unsigned long long)r);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) best = min(best, __shfl_xor(best, o));
    if ((threadIdx.x & 63) == 0 && best != ~0ULL) atomicMin(&m->first_lost_row, best);
}

// the same from the scan's row codes: 2 + 16 bytes per row pair instead of 48
__global__ void __launch_bounds__(256) k_set_bytes_code(const uint16_t *__restrict__ code,
                                                        const int64_t *__restrict__ val, int64_t n, long long vmin,
                                                        uint8_t *__restrict__ Ab, uint8_t *__restrict__ Db,
                                                        const uint32_t *__restrict__ R, int vec, SetMeta *m) {
    unsigned long long best = ~0ULL;
    const int64_t np = (n + 1) / 2;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    // software-pipelined like k_set_scan: the next pair's code and values are
    // loaded before this pair's byte stores
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    uint32_t ccn = 0;
    longlong2 v2n = make_longlong2(0, 0);
    if (i < np) { ccn = code[i]; v2n = ld_pair(val, i, n, vec); }
    for (; i < np; i += gs) {
        const uint32_t cc = ccn;
        const int64_t vv[2] = {v2n.x, v2n.y};
        if (i + gs < np) { ccn = code[i + gs]; v2n = ld_pair(val, i + gs, n, vec); }
        if (!cc) continue;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t c = (cc >> (8 * k)) & 0xFF;       // rows past n carry code 0
            if (!c) continue;
            const int64_t r = 2 * i + k;
            const int64_t b = vv[k] - vmin;
            if (c == 1) Ab[b] = 1;
            else {
                Db[b] = 1;
                if (!((R[b >> 5] >> (b & 31)) & 1)) best = min(best, (unsigned long long)r);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) best = min(best, __shfl_xor(best, o));
    if ((threadIdx.x & 63) == 0 && best != ~0ULL) atomicMin(&m->first_lost_row, best);
}

// 32 bytes -> one bitmap word, for each of A and D
__global__ void __launch_bounds__(256) k_set_pack_bits(const uint8_t *__restrict__ bytes, int64_t span_pad, int64_t nw,
                                                       uint32_t *__restrict__ bits) {
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < 2 * nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = w / nw, ww = w - s * nw;
        const uint4 *src = (const uint4 *)(bytes + s * span_pad + ww * 32);
        const uint4 a = src[0], b = src[1];
        const uint32_t q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            // bytes are 0 or 1: gather bit 0 of each byte
            const uint32_t v = q[k];
            out |= ((v & 1u) | ((v >> 7) & 2u) | ((v >> 14) & 4u) | ((v >> 21) & 8u)) << (4 * k);
        }
        bits[w] = out;
    }
}

__device__ __forceinline__ void set_words(const uint32_t *A, const uint32_t *D, const uint32_t *R,
                                          int64_t w, int64_t nw, uint32_t out[4]) {
    const uint32_t a = A[w], d = D[w], r = R[w];
    const uint32_t ok = r & a;
    out[0] = ok;          // ok
    out[1] = d & ~r;      // lost
    out[2] = r & ~a;      // unexpected
    out[3] = ok & ~d;     // recovered
}

// per word: population counts and run-start counts of the four result sets;
// either the per-word run starts (starts != null: the runs output numbers
// them by a scan) or the four result bitmaps themselves (outb != null) and
// the run totals
__global__ void k_set_count(const uint32_t *__restrict__ A, const uint32_t *__restrict__ D,
                            const uint32_t *__restrict__ R, int64_t nw,
                            uint32_t *__restrict__ starts /* 4 x nw */, uint32_t *__restrict__ outb /* 4 x nw */,
                            SetMeta *m) {
    long long c[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw;
         w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x[4], px[4] = {0, 0, 0, 0};
        set_words(A, D, R, w, nw, x);
        if (w > 0) set_words(A, D, R, w - 1, nw, px);
        c[0] += __popc(A[w]); c[1] += __popc(D[w]);
        c[2] += __popc(x[0]); c[3] += __popc(x[1]); c[4] += __popc(x[3]); c[5] += __popc(x[2]);
        for (int s = 0; s < 4; s++) {
            const uint32_t st = x[s] & ~((x[s] << 1) | (px[s] >> 31));
            if (starts) starts[s * nw + w] = __popc(st);
            c[6 + s] += __popc(st);
            if (outb) outb[s * nw + w] = x[s];
        }
    }
    // one atomic per counter per workgroup (per wave, 48K waves would
    // serialise on six L2 lines)
    __shared__ long long sc[4][10];
    for (int i = 0; i < 10; i++) {
        long long v = c[i];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6][i] = v;
    }
    __syncthreads();
    if (threadIdx.x < 10) {
        long long v = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); k++) v += sc[k][threadIdx.x];
        if (v) atomicAdd((unsigned long long *)&m->cnt[threadIdx.x], (unsigned long long)v);
    }
}

__global__ void k_set_emit(const uint32_t *__restrict__ A, const uint32_t *__restrict__ D,
                           const uint32_t *__restrict__ R, int64_t nw, long long vmin,
                           const uint32_t *__restrict__ spos /* 4 x nw exclusive scans */,
                           int64_t *__restrict__ runs /* 4 x 2 x cap */, int64_t cap) {
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw;
         w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x[4], px[4] = {0, 0, 0, 0}, nx[4] = {0, 0, 0, 0};
        set_words(A, D, R, w, nw, x);
        if (w > 0) set_words(A, D, R, w - 1, nw, px);
        if (w + 1 < nw) set_words(A, D, R, w + 1, nw, nx);
        for (int s = 0; s < 4; s++) {
            // a run starting in this word is numbered by the scan; its end is
            // the next end bit at or after the start, possibly in later words
            uint32_t st = x[s] & ~((x[s] << 1) | (px[s] >> 31));
            int64_t k = spos[s * nw + w];
            while (st) {
                const int b = __ffs(st) - 1;
                st &= st - 1;
                if (k < cap) {
                    int64_t *o = runs + (int64_t)s * 2 * cap;
                    o[2 * k] = vmin + w * 32 + b;
                    // scan forward for the end of this run
                    int64_t ww = w;
                    uint32_t cur = x[s] >> b;
                    int bb = b;
                    for (;;) {
                        const uint32_t inv = ~cur;
                        const int len = inv ? __ffs(inv) - 1 : 32 - bb;
                        if (bb + len < 32 || ww + 1 >= nw) { o[2 * k + 1] = vmin + ww * 32 + bb + len - 1; break; }
                        // run reaches the word boundary: continue into the next word
                        ww++;
                        uint32_t y[4];
                        set_words(A, D, R, ww, nw, y);
                        cur = y[s]; bb = 0;
                        if (!(cur & 1)) { o[2 * k + 1] = vmin + ww * 32 - 1; break; }
                    }
                }
                k++;
            }
        }
    }
}

__global__ void k_set_first_lost(const int64_t *__restrict__ type, const int64_t *__restrict__ f,
                                 const int64_t *__restrict__ val, int64_t n, long long vmin,
                                 const uint32_t *__restrict__ D, const uint32_t *__restrict__ R,
                                 SetMeta *m) {
    unsigned long long best = ~0ULL;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        if (f[r] != JH_F_ADD || type[r] != T_OK) continue;
        const uint64_t b = (uint64_t)(val[r] - vmin);
        const uint32_t bit = 1u << (b & 31);
        if ((D[b >> 5] & bit) && !(R[b >> 5] & bit)) best = min(best, (unsigned long long)r);
    }
    for (int o = 32; o > 0; o >>= 1) best = min(best, __shfl_xor(best, o));
    if ((threadIdx.x & 63) == 0 && best != ~0ULL) atomicMin(&m->first_lost_row, best);
}
}  // namespace

// The front half of both outputs: the attempts / acknowledged / final-read
// bitmaps over [vmin, vmin + 32 nw), the counts and the first lost row.
// Returns false when the result is already final (no :ok :read, nil read).
static bool set_bitmaps(jh_ctx *ctx, const jh_history *dh, jh_set_result *res, SetMeta *m, SetMeta &mh,
                        uint32_t *&A, uint32_t *&D, uint32_t *&R, int64_t &nw, long long &vmin, hipStream_t st) {
    memset(res, 0, sizeof(*res));
    res->first_fail_entry = -1; res->final_read_entry = -1;
    const int64_t n = dh->n;
    SetMeta mi;
    memset(&mi, 0, sizeof mi);
    mi.vmin = LLONG_MAX; mi.vmax = LLONG_MIN; mi.final_row = -1; mi.first_lost_row = ~0ULL;
    HIP_TRY(hipMemcpyAsync(m, &mi, sizeof mi, hipMemcpyHostToDevice, st));
    const int vec = ((uintptr_t)dh->type | (uintptr_t)dh->f | (uintptr_t)dh->value) % 16 == 0;
    uint16_t *code = JH_SET_CODE ? ctx->ws<uint16_t>(WS_S_CODE, (size_t)(n + 1) / 2 + 16) : nullptr;   // + a 16-byte tail
    if (n > 0) k_set_scan<<<grid_for((n + 1) / 2, 256, JH_SCAN_GRID), 256, 0, st>>>(dh->type, dh->f, dh->value, n, vec, m, code);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    res->final_read_entry = mh.final_row;
    if (mh.final_row < 0) { res->valid = JH_UNKNOWN; res->cause = JH_CAUSE_NIL_VALUE; return false; }
    int64_t rd[2];
    HIP_TRY(hipMemcpyAsync(rd, dh->value + mh.final_row, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(rd + 1, dh->value2 + mh.final_row, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (rd[0] == JH_NIL) { res->valid = JH_UNKNOWN; res->cause = JH_CAUSE_NIL_VALUE; return false; }
    if (mh.nil_attempt || mh.nil_add)
        throw_jh(JH_EUNSUPPORTED, "nil set elements (integer-interval-set-str prints those in hash order)");
    if (!dh->aux && rd[1] > 0) throw_jh(JH_EINVAL, "set read without an aux element array");
    const int64_t off = rd[0], cnt = rd[1];
    if (cnt > 0)
        k_set_range<<<grid_for(cnt / 2 + 1, 256, 4096), 256, 0, st>>>(dh->aux, off, cnt, (uintptr_t)dh->aux % 16 == 0, m);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    vmin = mh.vmin;
    long long vmax = mh.vmax;
    if (vmin > vmax) { vmin = 0; vmax = 0; }
    const unsigned long long span = (unsigned long long)(vmax - vmin) + 1;
    if (span > (1ULL << 34)) throw_jh(JH_EUNSUPPORTED, "set elements span more than 2^34");
    nw = (int64_t)((span + 31) / 32);
    uint32_t *bits = ctx->ws<uint32_t>(WS_S_BITS, 3 * nw);
    A = bits; D = bits + nw; R = bits + 2 * nw;
    // dense spans: A / D byte maps, R bucketed (k_rb_*); sparse or huge spans
    // mark the bitmaps directly (a sparse set over a wide range does
    // not allocate a byte per element of span)
    int sb = 5;
    while (sb < RB_MAXSB && (span >> sb) > 256) sb++;
    const int nbins = (int)((span + (1ULL << sb) - 1) >> sb);
    if (span <= RB_SPAN_MAX && nbins <= RB_MAXBINS && span <= 8ULL * (unsigned long long)(n + cnt) + 4096) {
        if (cnt > 0) {
            const int nblk = (int)((cnt + RB_CH - 1) / RB_CH);
            const size_t nh = (size_t)nbins * nblk;
            uint32_t *hist = ctx->ws<uint32_t>(WS_S_RB_HIST, 2 * nh + 1);
            uint32_t *pos = hist + nh;
            uint32_t *rin = ctx->ws<uint32_t>(WS_S_RB_OUT, cnt);
            const int64_t *e = dh->aux + off;
            k_rb_hist<<<nblk, 256, nbins * 4, st>>>(e, cnt, vmin, sb, nbins, nblk, hist);
            size_t tb = 0;
            HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, hist, pos, (int)nh, st));
            HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ctx->ws<char>(WS_S_TMP, tb), tb, hist, pos, (int)nh, st));
            const int sc_lds = nbins * 12 + RB_CH * 6;
            HIP_TRY(hipFuncSetAttribute((const void *)k_rb_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, sc_lds));
            k_rb_scatter<<<nblk, 256, sc_lds, st>>>(e, cnt, vmin, sb, nbins, nblk, hist, pos, rin);
            k_rb_build<<<nbins, 1024, (1 << sb) / 8, st>>>(rin, pos, nblk, nbins, cnt, sb, nw, R);
        } else {
            HIP_TRY(hipMemsetAsync(R, 0, sizeof(uint32_t) * nw, st));
        }
        const int64_t span_pad = nw * 32;
        uint8_t *bytes = ctx->ws<uint8_t>(WS_S_BYTES, 2 * span_pad);
        HIP_TRY(hipMemsetAsync(bytes, 0, 2 * span_pad, st));
        if (n > 0 && code)
            k_set_bytes_code<<<grid_for((n + 1) / 2, 256, JH_BYTES_GRID), 256, 0, st>>>(code, dh->value, n, vmin, bytes,
                                                                               bytes + span_pad, R, vec, m);
        else if (n > 0)
            k_set_bytes_rows<<<grid_for((n + 1) / 2, 256, 16384), 256, 0, st>>>(dh->type, dh->f, dh->value, n, vmin, bytes,
                                                                               bytes + span_pad, R, vec, m);
        k_set_pack_bits<<<grid_for(2 * nw, 256, 16384), 256, 0, st>>>(bytes, span_pad, nw, bits);
    } else {
        HIP_TRY(hipMemsetAsync(bits, 0, sizeof(uint32_t) * 3 * nw, st));
        if (n > 0) k_set_mark_rows<<<(unsigned)((n + MARK_CH - 1) / MARK_CH), 256, 0, st>>>(dh->type, dh->f, dh->value, n, vmin, A, D);
        if (cnt > 0) k_set_mark_read<<<(unsigned)((cnt + MARK_CH - 1) / MARK_CH), 256, 0, st>>>(dh->aux, off, cnt, vmin, R);
        if (n > 0)
            k_set_first_lost<<<grid_for(n, 256), 256, 0, st>>>(dh->type, dh->f, dh->value, n, vmin, D, R, m);
    }
    return true;
}

static void set_finish(jh_set_result *res, const SetMeta &mh) {
    res->attempt_count = mh.cnt[0]; res->acknowledged_count = mh.cnt[1];
    res->ok_count = mh.cnt[2]; res->lost_count = mh.cnt[3];
    res->recovered_count = mh.cnt[4]; res->unexpected_count = mh.cnt[5];
    res->valid = (mh.cnt[3] == 0 && mh.cnt[5] == 0) ? JH_VALID : JH_INVALID;
    if (mh.cnt[3]) res->first_fail_entry = mh.first_lost_row == ~0ULL ? -1 : (int64_t)mh.first_lost_row;
    else if (mh.cnt[5]) res->first_fail_entry = mh.final_row;
    for (int s = 0; s < 4; s++) res->n_runs[s] = mh.cnt[6 + s];
}

void set_check(jh_ctx *ctx, const jh_history *dh, jh_set_result *res, int64_t *runs_out[4],
               int64_t runs_cap, hipStream_t st) {
    SetMeta *m = ctx->ws<SetMeta>(WS_S_CNT, 1);
    SetMeta mh;
    uint32_t *A, *D, *R;
    int64_t nw;
    long long vmin;
    if (!set_bitmaps(ctx, dh, res, m, mh, A, D, R, nw, vmin, st)) return;
    uint32_t *starts = ctx->ws<uint32_t>(WS_S_RUNS, 8 * nw + 8);
    uint32_t *spos = starts + 4 * nw;
    k_set_count<<<grid_for(nw, 256, 2048), 256, 0, st>>>(A, D, R, nw, starts, nullptr, m);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, starts, spos, (int)nw, st));
    void *tmp = ctx->ws<char>(WS_S_TMP, tb);
    for (int s = 0; s < 4; s++)   // per-set run numbering starts at 0
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, starts + s * nw, spos + s * nw, (int)nw, st));
    const int64_t cap = runs_cap;
    int64_t *runs = ctx->ws<int64_t>(WS_C_OUT, 8 * std::max<int64_t>(cap, 1));
    k_set_emit<<<grid_for(nw, 256), 256, 0, st>>>(A, D, R, nw, vmin, spos, runs, cap);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    set_finish(res, mh);
    for (int s = 0; s < 4; s++) {
        const int64_t k = std::min<int64_t>(res->n_runs[s], cap);
        if (k > 0 && runs_out[s])
            HIP_TRY(hipMemcpyAsync(runs_out[s], runs + (int64_t)s * 2 * cap, sizeof(int64_t) * 2 * k,
                                   hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
}

// The four result sets as bitmaps over [*base, *base + 32 * words): 4 bytes
// per 32 elements of span whatever the run structure (23 M runs of the C2
// workload are 370 MB as [lo hi] pairs, 25 MB as bitmaps)
void set_check_bitmaps(jh_ctx *ctx, const jh_history *dh, jh_set_result *res, uint32_t *bits_out[4],
                       int64_t words_cap, int64_t *base, int64_t *n_words, hipStream_t st) {
    SetMeta *m = ctx->ws<SetMeta>(WS_S_CNT, 1);
    SetMeta mh;
    uint32_t *A, *D, *R;
    int64_t nw;
    long long vmin;
    *base = 0; *n_words = 0;
    if (!set_bitmaps(ctx, dh, res, m, mh, A, D, R, nw, vmin, st)) return;
    uint32_t *outb = ctx->ws<uint32_t>(WS_S_RUNS, 4 * nw + 8);
    k_set_count<<<grid_for(nw, 256, 2048), 256, 0, st>>>(A, D, R, nw, nullptr, outb, m);
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    const int64_t k = std::min<int64_t>(nw, words_cap);
    for (int s = 0; s < 4; s++)
        if (k > 0 && bits_out[s])
            HIP_TRY(hipMemcpyAsync(bits_out[s], outb + (int64_t)s * nw, sizeof(uint32_t) * k, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    set_finish(res, mh);
    *base = vmin; *n_words = nw;
}
