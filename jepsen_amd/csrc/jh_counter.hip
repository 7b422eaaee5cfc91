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
//   k_cnt_pack    one pass over the four columns the checker reads: the
//                 complete pairing of every invocation whose completion lies
//                 in its 2048-row chunk, and each row's contribution word
//                 (kind | value) -- after (remove :fails?) / (remove op/fail?)
//                 and (or inv ok), with the nil checks -- plus the last row
//                 of every process (LDS-privatised) and the add-value range  32 / 4
//   k_cnt_pair_spill  the few invocations the chunk could not pair (thread
//                 per spill, walks its process' rows): completes their words ~0
//   hipcub scan / k_cnt_tile_scan
//                 reduce-then-scan of {lower, upper, reads} over 2048-row
//                 tiles of contribution words: each tile's sums come from the
//                 pack (a tile is a chunk) plus atomics of k_cnt_pair_spill,
//                 so one scan pass reads the words; writes only at read rows
//                 (the ok read's row and upper, the invoke read's lower)    4 / ~0
//   k_cnt_triples the triples, in history order, errors, first failing row
//                 (over the ~1% read rows only)
// Round 2 packed a 4-byte row code and re-read code, pair and value (16 B per
// row) in both scan passes; the contribution word carries what they need, and
// round 3 folds the reduce pass into the pack. (A single-pass decoupled
// look-back scan over the 49 K tiles was measured at 20.8 ms on MI355X: the
// tile-to-tile look-back chain is serial latency across XCDs.)
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>

namespace {

#ifndef JH_CNT_BALLOT
#define JH_CNT_BALLOT 0      // group masks by per-wave ballots instead of LDS atomics (A/B)
#endif
#ifndef JH_SPILL_VEC
#define JH_SPILL_VEC 8       // rows per step of the spill walk (0 or 1: one row per step)
#endif
constexpr int SPILL_VEC = JH_SPILL_VEC > 1 ? JH_SPILL_VEC : 1;
#ifndef JH_SPILL_LANES
#define JH_SPILL_LANES 32    // lanes per chunk in k_cnt_pair_spill (~20 spills per C2 chunk)
#endif
constexpr int SPILL_LANES = JH_SPILL_LANES;
static_assert(SPILL_LANES >= 1 && SPILL_LANES <= 256 && (SPILL_LANES & (SPILL_LANES - 1)) == 0, "power of two");
#ifndef JH_SPILL_TAB
#define JH_SPILL_TAB 2       // chunks publish their processes' first non-:info rows (2: built by ballots, 1: by wave 0; 0: walk only)
#endif
#ifndef JH_CNT_HASH32
#define JH_CNT_HASH32 0      // a 32-bit multiplicative slot hash instead of jh_mix64 (A/B)
#endif

// Round 6: k_cnt_pack's barriers order LDS only. Nothing the pack stores to
// global memory is read back inside a block (words, pairs, spills, tables and
// the counters' atomics are for later kernels), so a barrier need not wait
// for those stores -- __syncthreads() did (s_waitcnt vmcnt(0) before every
// s_barrier): the word pass's barrier waited on the block's word stores.
#ifndef JH_CNT_LDSBAR
#define JH_CNT_LDSBAR 1
#endif
#if JH_CNT_LDSBAR
#define PACK_BARRIER() do { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); \
                            __builtin_amdgcn_s_barrier(); \
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); } while (0)
#else
#define PACK_BARRIER() __syncthreads()
#endif

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

// A row's contribution word (checker.clj:709-727 after history/complete,
// (remove :fails?) and (remove op/fail?)):
//   bits 0-2  kind: what the row feeds
//   bit  3    U: a completion no invocation has claimed yet (an orphan unless
//             a spilled invocation of an earlier chunk claims it)
//   bit  4    X: the value does not fit the word: read it from the value
//             column (own row, or the completion's for (or inv ok))
//   bits 5-31 the value, 27-bit signed (adds of 1 in the C2 workload)
constexpr uint32_t CW_NONE = 0, CW_LO = 1, CW_HI = 2, CW_OKREAD = 3, CW_INVREAD = 4, CW_PEND = 5;
constexpr uint32_t CW_U = 8, CW_X = 16;
#ifndef JH_CNT_LUT
#define JH_CNT_LUT 1         // the word pass by a class LUT and selects (0: per-kind branches)
#endif
// The word pass's row classes by f2 << 2 | type (4 bits each): bits 0-2 the
// kind (HI for an :invoke :add, whose word depends on its completion; LO, the
// two reads), bit 3 the row may carry CW_U (:ok / :fail rows)
constexpr unsigned long long cnt_lut_entry(uint32_t q) {
    return (q & 3) == 0 ? ((q >> 2) == F2_ADD ? CW_HI : (q >> 2) == F2_READ ? CW_INVREAD : CW_NONE)
         : (q & 3) == 1 ? 8u | ((q >> 2) == F2_ADD ? CW_LO : (q >> 2) == F2_READ ? CW_OKREAD : CW_NONE)
         : (q & 3) == 2 ? 8u : 0u;
}
constexpr unsigned long long cnt_lut(uint32_t q) { return q == 12 ? 0ULL : (cnt_lut_entry(q) << (4 * q)) | cnt_lut(q + 1); }
constexpr unsigned long long CNT_KIND_LUT = cnt_lut(0);
constexpr long long CW_VMAX = (1LL << 26) - 1, CW_VMIN = -(1LL << 26);
__device__ __forceinline__ uint32_t cw_make(uint32_t kind, long long v) {
    if (v < CW_VMIN || v > CW_VMAX) return kind | CW_X;
    return kind | ((uint32_t)(int32_t)v << 5);
}
__device__ __forceinline__ long long cw_val(uint32_t w, const int64_t *__restrict__ val,
                                            const int32_t *__restrict__ pair, int64_t r) {
    if (!(w & CW_X)) return (long long)((int32_t)w >> 5);
    long long v = val[r];
    if (v == JH_NIL) v = val[pair[r]];        // (or inv ok): pair[r] is written for these rows
    return v;
}

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

// One chunk of CHUNK rows per block: contribution words, the last row of
// every process (per-chunk LDS hash of (process -> max row), then one global
// atomicMax per distinct process), the add-value range for the overflow
// check, and the complete pairing of every invocation whose completion lies
// in the same chunk.
//
// Pairing (util.clj:606-640: an invocation's completion is the next
// non-:info row of its process): the chunk's first PAIR_PROCS distinct
// processes get a compact index c, and each 64-row group g of the chunk a
// bit mask M[g][c] of its non-:info rows of process c (one LDS atomicOr per
// row). An invocation's completion is then the lowest set bit after its own
// lane in M[g][c], or in the next group with a non-zero M[g'][c]: O(1) LDS
// reads per row. Invocations with no completion in the chunk, or of a
// process beyond the first PAIR_PROCS, go to a spill list (k_cnt_pair_spill)
// and their words stay CW_PEND until it completes them.
// per-row contributions and prefixes of lower / upper / ok reads (an :ok
// :read still marked U has no invocation: an orphan, never a read row, so
// pair is only ever read where it was written)
struct CntAcc {
    long long lo, hi;
    int nr, flags;
};

// Reduce-then-scan over tiles of CNT_TILE rows. A tile is a pack chunk: the
// pack writes each tile's sums {lower, upper, ok reads} (k_cnt_pair_spill adds
// what the spilled invocations complete), then one scan pass reads the
// contribution words (4 B per row).
constexpr int CNT_TILE = 2048, CNT_PER = CNT_TILE / 256;
static_assert(CNT_TILE == CHUNK, "a counter tile is a pack chunk");
constexpr int PAIR_PROCS = 32, PAIR_GROUPS = CHUNK / 64;
constexpr int PACK_THREADS = 512;
constexpr int PER = CHUNK / PACK_THREADS;   // rows per thread per chunk (row k * PACK_THREADS + tid)
// One chunk per 512-thread block (four rows per thread), 32 KB of LDS (round
// 2: 256 threads and 50 KB: 1.59 ms per 100 M rows). Measured against it:
// 256-thread blocks at four and six per CU (1.34 / 1.44 ms) and a chunk per
// wave with the pairing done by ballots instead of LDS (1.61 ms: ~200 VALU
// instructions per row).
// A spilled invocation is stored as its row when its walk must start right
// after it (a process beyond the chunk's first PAIR_PROCS), as ~row when the
// chunk already showed every later row of its process in the chunk to be
// :info, so the walk starts at the chunk's end (a crashed op's walk then ends
// at once: its process' last row lies inside the chunk).
__global__ void __launch_bounds__(PACK_THREADS) k_cnt_pack(const int64_t *__restrict__ proc,
                                                  const int64_t *__restrict__ type,
                                                  const int64_t *__restrict__ f,
                                                  const int64_t *__restrict__ val, int64_t n,
                                                  long long pmin, int32_t *__restrict__ last,
                                                  uint32_t *__restrict__ cw, int32_t *__restrict__ pair,
                                                  uint2 *__restrict__ spill, int32_t *__restrict__ spill_n,
                                                  uint2 *__restrict__ tab, int32_t *__restrict__ tab_n,
                                                  CntMeta *m, CntAcc *__restrict__ agg) {
    __shared__ uint32_t hk[HSLOTS];                 // process - pmin + 1 (0: empty)
    __shared__ int hv[HSLOTS];                      // its last row
    __shared__ int8_t hc[HSLOTS];                   // its compact index, -1 beyond PAIR_PROCS
    __shared__ uint8_t sc[CHUNK];                   // the chunk's rows: f2 << 2 | type
    __shared__ int16_t sp[CHUNK];                   // each row's partner in the chunk (-1: none)
    __shared__ unsigned long long M[PAIR_GROUPS][PAIR_PROCS];
    __shared__ int nd, nls;
    __shared__ uint32_t cproc[PAIR_PROCS];            // compact index -> process offset
    __shared__ long long sh[5][PACK_THREADS / 64];
    const int tid = threadIdx.x;
    long long am = 0, na = 0;
    long long t_lo = 0, t_hi = 0, t_nr = 0;          // this tile's sums
    {
        const int64_t c0 = (int64_t)blockIdx.x * CHUNK;
        const int nc = (int)min<int64_t>(CHUNK, n - c0);
        // every row of the thread in flight at once, then compacted
        // (process offset, f2 << 2 | type, value)
        long long rp[PER], rt[PER], rf[PER], cv[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int64_t r = c0 + k * PACK_THREADS + tid;
            if (r < n) { rp[k] = proc[r]; rt[k] = type[r]; rf[k] = f[r]; cv[k] = val[r]; }
            else { rp[k] = pmin; rt[k] = T_INFO; rf[k] = 0; cv[k] = 0; }
        }
        uint32_t cp[PER], cx[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            cp[k] = (uint32_t)(rp[k] - pmin);                                      // span < 2^28
            const uint32_t f2 = rf[k] == JH_F_ADD ? F2_ADD : rf[k] == JH_F_READ ? F2_READ : F2_OTHER;
            cx[k] = (f2 << 2) | (uint32_t)(rt[k] & 3);
        }
        for (int i = tid; i < HSLOTS; i += PACK_THREADS) { hk[i] = 0; hv[i] = -1; hc[i] = -1; }
        for (int i = tid; i < PAIR_GROUPS * PAIR_PROCS; i += PACK_THREADS) (&M[0][0])[i] = 0;
        if (tid == 0) { nd = 0; nls = 0; }
        PACK_BARRIER();
        // each row's hash slot (-1: none) and kind stay in this thread's
        // registers: only the pairing reads other rows' (round 4)
        int rsl[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) rsl[k] = -1;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = k * PACK_THREADS + tid;
            if (i >= nc) break;
            const int64_t r = c0 + i;
            const uint32_t pk = cp[k];
            const uint32_t ty = cx[k] & 3, f2 = cx[k] >> 2;
            sc[i] = (uint8_t)cx[k];
            if (ty != T_INVOKE) sp[i] = -1;            // an invocation's partner stays in registers
            if (f2 == F2_ADD && (ty == T_INVOKE || ty == T_OK)) {
                const long long v = cv[k];
                if (v != JH_NIL) am = max(am, v < 0 ? (v == LLONG_MIN ? LLONG_MAX : -v) : v);
                na++;
            }
#if JH_CNT_HASH32
            uint32_t h = (pk * 0x9E3779B1u) >> (32 - 10);               // HSLOTS = 2^10
#else
            uint32_t h = (uint32_t)jh_mix64((uint64_t)pk) & (HSLOTS - 1);
#endif
            int slot = -1;
            for (int probe = 0; probe < 64; probe++) {
                uint32_t cur = hk[h];
                if (cur == 0) {
                    cur = atomicCAS(&hk[h], 0u, pk + 1);
                    if (cur == 0) {
                        const int c = atomicAdd(&nd, 1);
                        hc[h] = (int8_t)(c < PAIR_PROCS ? c : -1);
                        if (c < PAIR_PROCS) cproc[c] = pk;
                        cur = pk + 1;
                    }
                }
                if (cur == pk + 1) { slot = (int)h; break; }
                h = (h + 1) & (HSLOTS - 1);
            }
            // the process' last row: the wave's last lane of each slot only
            // (one LDS atomic per process per wave, not per row)
            const int nxt = __shfl_down(slot, 1);
            // (lane + 1 holds row i + 1: past the chunk's end it is inactive)
            if (slot >= 0) { if ((tid & 63) == 63 || i + 1 >= nc || nxt != slot) atomicMax(&hv[slot], (int)r); }
            else atomicMax(&last[pk], (int)r);
            rsl[k] = slot;
        }
        PACK_BARRIER();
        // compact process index of every row (the hash is complete now), and the
        // group masks of non-:info rows
        int8_t rc[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = k * PACK_THREADS + tid;
            rc[k] = -1;
#if JH_CNT_BALLOT
            // a wave's 64 lanes are the 64 rows of group i >> 6 (PACK_THREADS
            // is a multiple of 64), and no other wave writes that group's
            // masks: one ballot per distinct process, one plain LDS store
            int c = -1;
            if (i < nc) { const int slot = rsl[k]; c = slot >= 0 ? hc[slot] : -1; }
            rc[k] = (int8_t)c;
            const bool on = c >= 0 && (cx[k] & 3) != T_INFO;
            unsigned long long todo = __ballot(on);
            while (todo) {
                const int l0 = __builtin_ctzll(todo);
                const int cc = __shfl(c, l0);
                const unsigned long long mm = __ballot(on && c == cc);
                if ((tid & 63) == l0) M[i >> 6][cc] = mm;
                todo &= ~mm;
            }
#else
            if (i >= nc) continue;
            const int slot = rsl[k];
            const int c = slot >= 0 ? hc[slot] : -1;
            rc[k] = (int8_t)c;
            if (c >= 0 && (cx[k] & 3) != T_INFO) atomicOr(&M[i >> 6][c], 1ULL << (i & 63));
#endif
        }
        PACK_BARRIER();
#if JH_SPILL_TAB
        // the chunk's table for k_cnt_pair_spill: per tracked process its
        // first non-:info row here (flag << 31 | sc << 16 | row in chunk), so a
        // walk from an earlier chunk reads one table instead of these rows
#if JH_SPILL_TAB == 2
        // every wave takes four processes, two per step (a half-wave per
        // process, a lane per 64-row group): the first group with a set bit by
        // one ballot, no lane walks the groups
        {
            const int lane = tid & 63, wv = tid >> 6, half = lane >> 5, g = lane & 31;
            const int ndc = min(nd, PAIR_PROCS);
            static_assert(PAIR_GROUPS == 32 && PAIR_PROCS == 32 && PACK_THREADS == 512, "table layout");
#pragma unroll
            for (int st = 0; st < 2; st++) {
                const int c = (st * 8 + wv) * 2 + half;
                const unsigned long long mg = (c < ndc && (g << 6) < nc) ? M[g][c] : 0ULL;
                const unsigned long long b = __ballot(mg != 0ULL);
                const uint32_t bh = half ? (uint32_t)(b >> 32) : (uint32_t)b;
                if (g == 0) {
                    uint2 e = make_uint2(0u, 0u);
                    if (c < ndc) {
                        e.x = cproc[c] + 1;
                        if (bh) {
                            const int g0 = __builtin_ctz(bh);
                            const int first = (g0 << 6) + __builtin_ctzll(M[g0][c]);
                            e.y = (1u << 31) | ((uint32_t)sc[first] << 16) | (uint32_t)first;
                        }
                    }
                    tab[(int64_t)blockIdx.x * PAIR_PROCS + c] = e;
                }
            }
            if (tid == 0) tab_n[blockIdx.x] = nd;
        }
#else
        if (tid < PAIR_PROCS) {
            uint2 e = make_uint2(0u, 0u);
            if (tid < min(nd, PAIR_PROCS)) {
                int first = -1;
                for (int g = 0; g < PAIR_GROUPS && (g << 6) < nc; g++) {
                    const unsigned long long mg = M[g][tid];
                    if (mg) { first = (g << 6) + __builtin_ctzll(mg); break; }
                }
                e.x = cproc[tid] + 1;
                e.y = first < 0 ? 0u : (1u << 31) | ((uint32_t)sc[first] << 16) | (uint32_t)first;
            }
            tab[(int64_t)blockIdx.x * PAIR_PROCS + tid] = e;
            if (tid == 0) tab_n[blockIdx.x] = nd;
        }
#endif
#endif
        bool walk_from_end[PER];
        int gotk[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = k * PACK_THREADS + tid;
            walk_from_end[k] = false;
            gotk[k] = -1;
            if (i >= nc) continue;
            const uint32_t x = cx[k];
            if ((x & 3) != T_INVOKE) continue;
            const int c = rc[k];
            int got = -1;
            if (c >= 0) {
                const int g = i >> 6, l = i & 63;
                const unsigned long long after = l == 63 ? 0ULL : (M[g][c] & (~0ULL << (l + 1)));
                if (after) got = (g << 6) + __builtin_ctzll(after);
                else
                    for (int g2 = g + 1; g2 < PAIR_GROUPS && (g2 << 6) < nc; g2++)
                        if (M[g2][c]) { got = (g2 << 6) + __builtin_ctzll(M[g2][c]); break; }
                walk_from_end[k] = got < 0;      // every later row of its process in the chunk is :info
            }
            if (got >= 0 && (sc[got] & 3) == T_INVOKE) {
                atomicMin(&m->viol1, ((unsigned long long)(c0 + got) << 4) | JH_CAUSE_DOUBLE_INVOKE);
                got = -2;
            }
            gotk[k] = got;                             // -1: spill (no completion in the chunk)
            if (got >= 0) sp[got] = (int16_t)i;
        }
        PACK_BARRIER();
        // the contribution words
#if JH_CNT_LUT
        // Round 6: the (type, f) class from a LUT and the
        // word by selects; only the rare rows branch (a spill's store, a nil
        // value, an orphan read, a partner's value)
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = k * PACK_THREADS + tid;
            if (i >= nc) continue;
            const uint32_t x = cx[k];
            const uint32_t ty = x & 3;
            const int64_t r = c0 + i;
            const uint32_t e = (uint32_t)(CNT_KIND_LUT >> (4 * x)) & 15u;
            const uint32_t kd = e & 7u;
            const int c = ty == T_INVOKE ? gotk[k] : (int)sp[i];
            const bool spl = ty == T_INVOKE && c == -1;
            if (spl)
                spill[c0 + atomicAdd(&nls, 1)] = make_uint2((uint32_t)(walk_from_end[k] ? ~(int32_t)r : (int32_t)r),
                                                            cp[k] | ((x >> 2) << 28));
            const uint32_t psc = sc[c > 0 ? c : 0];
            long long v = cv[k];
            const bool hi = kd == CW_HI && c >= 0 && (psc & 3) != T_FAIL;
            const bool lo = kd == CW_LO;
            const bool okr = kd == CW_OKREAD;
            const bool own = !(hi && v == JH_NIL);
            if (!own) v = val[c0 + c];
            const bool isv = hi || lo;
            const bool nil = isv && v == JH_NIL;
            const bool orphan = okr && c >= 0 && (psc >> 2) != F2_READ;
            if (nil || orphan)
                atomicMin(&m->viol2, ((unsigned long long)r << 4) | (nil ? JH_CAUSE_NIL_VALUE : JH_CAUSE_ORPHAN));
            const bool fits = v >= CW_VMIN && v <= CW_VMAX;
            const uint32_t vw = fits ? ((uint32_t)(int32_t)v << 5) : CW_X;
            const bool good = isv && !nil;
            uint32_t w = good ? (kd | vw) : kd == CW_HI ? (spl ? CW_PEND : CW_NONE) : lo || orphan ? CW_NONE : kd;
            w |= (e >> 3) && c < 0 ? CW_U : 0u;
            const long long vz = good ? v : 0;
            t_hi += hi ? vz : 0;
            t_lo += lo ? vz : 0;
            const bool rd = okr && !orphan && c >= 0;
            t_nr += rd ? 1 : 0;
            if (rd || (hi && !own && !fits)) pair[r] = (int32_t)(c0 + c);
            cw[r] = w;
        }
#else
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = k * PACK_THREADS + tid;
            if (i >= nc) continue;
            const uint32_t x = cx[k];
            const uint32_t ty = x & 3, f2 = x >> 2;
            const int64_t r = c0 + i;
            const int c = ty == T_INVOKE ? gotk[k] : (int)sp[i];
            uint32_t w = CW_NONE;
            if (ty == T_INVOKE) {
                if (c == -1) {
                    // spills gather in LDS: one global atomic per chunk
                    // the chunk's own spill region: no global atomic
                    spill[c0 + atomicAdd(&nls, 1)] = make_uint2((uint32_t)(walk_from_end[k] ? ~(int32_t)r : (int32_t)r),
                                                                cp[k] | (f2 << 28));
                    w = f2 == F2_READ ? CW_INVREAD : f2 == F2_ADD ? CW_PEND : CW_NONE;
                } else if (f2 == F2_READ) {
                    w = CW_INVREAD;
                } else if (f2 == F2_ADD && c >= 0 && (sc[c] & 3) != T_FAIL) {
                    // (remove :fails?) keeps it: upper += (or inv ok)
                    long long v = cv[k];
                    bool own = true;
                    if (v == JH_NIL) { v = val[c0 + c]; own = false; }
                    if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
                    else {
                        w = cw_make(CW_HI, v);
                        if ((w & CW_X) && !own) pair[r] = (int32_t)(c0 + c);
                        t_hi += v;
                    }
                }
            } else if (ty == T_OK || ty == T_FAIL) {
                const uint32_t u = c < 0 ? CW_U : 0u;      // no invocation in the chunk (yet)
                if (ty == T_OK && f2 == F2_ADD) {
                    const long long v = cv[k];
                    if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
                    else { w = cw_make(CW_LO, v); t_lo += v; }
                } else if (ty == T_OK && f2 == F2_READ) {
                    // its pending read must come from an [:invoke :read] (checker.clj:713-716)
                    if (c >= 0 && (sc[c] >> 2) != F2_READ)
                        atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_ORPHAN);
                    else {
                        w = CW_OKREAD;
                        if (c >= 0) { pair[r] = (int32_t)(c0 + c); t_nr++; }   // U-marked: counted when claimed
                    }
                }
                w |= u;
            }
            cw[r] = w;
        }
#endif
    }
    for (int o = 32; o > 0; o >>= 1) {
        am = max(am, (long long)__shfl_xor(am, o)); na += (long long)__shfl_xor(na, o);
        t_lo += (long long)__shfl_xor(t_lo, o); t_hi += (long long)__shfl_xor(t_hi, o); t_nr += (long long)__shfl_xor(t_nr, o);
    }
    if ((tid & 63) == 0) {
        sh[0][tid >> 6] = am; sh[1][tid >> 6] = na; sh[2][tid >> 6] = t_lo; sh[3][tid >> 6] = t_hi; sh[4][tid >> 6] = t_nr;
    }
    PACK_BARRIER();                                  // (also orders every nls increment)
    if (tid == 0) {
        for (int w = 1; w < PACK_THREADS / 64; w++) {
            am = max(am, sh[0][w]); na += sh[1][w]; t_lo += sh[2][w]; t_hi += sh[3][w]; t_nr += sh[4][w];
        }
        agg[blockIdx.x] = CntAcc{t_lo, t_hi, (int)t_nr, 0};
        spill_n[blockIdx.x] = nls;
        if (am) atomicMax(&m->amax_abs, am);
        if (na) atomicAdd((unsigned long long *)&m->n_add, (unsigned long long)na);
    }
    // the last row of each of the chunk's processes, after the last barrier
    // (these few atomics hit the same addresses from every block: no barrier
    // waits on them)
    for (int i = tid; i < HSLOTS; i += PACK_THREADS)
        if (hk[i]) atomicMax(&last[hk[i] - 1], hv[i]);
}

// the spilled invocations: one thread each walks its process' rows forward
// to the completion, or past the process' last row (no completion: a crashed
// op, which stays in), and completes the invocation's word (and claims the
// completion's). A spill carries its row and its process offset | f2 << 28
// (span < 2^28), so the walk starts after one dependent load (last[]).
__global__ void __launch_bounds__(256) k_cnt_pair_spill(const int64_t *__restrict__ proc,
                                                        const int64_t *__restrict__ type,
                                                        const int64_t *__restrict__ f,
                                                        const int64_t *__restrict__ val, int64_t n,
                                                        long long pmin, const int32_t *__restrict__ last,
                                                        const uint2 *__restrict__ spill,
                                                        const int32_t *__restrict__ spill_n, int64_t n_chunks,
                                                        const uint2 *__restrict__ tab, const int32_t *__restrict__ tab_n,
                                                        uint32_t *__restrict__ cw, int32_t *__restrict__ pair,
                                                        CntMeta *m, CntAcc *__restrict__ agg) {
    // SPILL_LANES lanes per chunk: its spills are spill[chunk * CHUNK ..][0 .. spill_n[chunk])
    const int sl = threadIdx.x & (SPILL_LANES - 1);
    const int cpb = 256 / SPILL_LANES;
    for (int64_t ch = (int64_t)blockIdx.x * cpb + threadIdx.x / SPILL_LANES; ch < n_chunks;
         ch += (int64_t)gridDim.x * cpb)
    for (int s = sl; s < spill_n[ch]; s += SPILL_LANES) {
        const uint2 e = spill[ch * CHUNK + s];
        const int32_t se = (int32_t)e.x;
        const int64_t r = se >= 0 ? se : ~se;
        const uint32_t pk = e.y & ((1u << 28) - 1), f2 = e.y >> 28;
        const long long p = pmin + (long long)pk;
        const int64_t lr = last[pk];
        const long long vr = f2 == F2_ADD ? (long long)val[r] : 0;    // issued with last[]
        int64_t got = -1;
        int gty = -1;                                                  // the completion's type
        // from the chunk's end when the chunk held only :info rows of p after r
        const int64_t j0 = se >= 0 ? r + 1 : (r / CHUNK + 1) * CHUNK;
#if JH_SPILL_TAB
        // at each chunk boundary the chunk's table gives p's first non-:info
        // row there (or says it has none); inside a chunk (r's own, or one
        // with more than PAIR_PROCS processes) SPILL_VEC rows per step, their
        // process and type loads issued together
        for (int64_t j = j0; got == -1 && j <= lr;) {
            const int64_t cj = j / CHUNK;
            if (j == cj * CHUNK && tab_n[cj] <= PAIR_PROCS) {
                const uint4 *t4 = (const uint4 *)(tab + cj * PAIR_PROCS);
                uint32_t ey = 0;
#pragma unroll
                for (int q0 = 0; q0 < PAIR_PROCS / 2; q0 += 4) {
                    uint4 x[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) x[u] = t4[q0 + u];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (x[u].x == pk + 1) ey = x[u].y;
                        if (x[u].z == pk + 1) ey = x[u].w;
                    }
                }
                if (!(ey >> 31)) { j = (cj + 1) * CHUNK; continue; }     // no non-:info row of p in chunk cj
                const int64_t jq = cj * CHUNK + (ey & 0xFFFF);
                const int ty = (int)((ey >> 16) & 3);
                if (ty == T_INVOKE) { atomicMin(&m->viol1, ((unsigned long long)jq << 4) | JH_CAUSE_DOUBLE_INVOKE); got = -2; }
                else { got = jq; gty = ty; }
                break;
            }
            const int64_t jend = min(lr, (cj + 1) * CHUNK - 1);
            long long pv[SPILL_VEC], tv[SPILL_VEC];
#pragma unroll
            for (int q = 0; q < SPILL_VEC; q++) {
                const int64_t jq = min(j + q, jend);
                pv[q] = proc[jq]; tv[q] = type[jq];
            }
#pragma unroll
            for (int q = 0; q < SPILL_VEC; q++) {
                const int64_t jq = j + q;
                if (got != -1 || jq > jend || pv[q] != p) continue;
                const int64_t ty = tv[q] & 3;
                if (ty == T_INFO) continue;
                if (ty == T_INVOKE) { atomicMin(&m->viol1, ((unsigned long long)jq << 4) | JH_CAUSE_DOUBLE_INVOKE); got = -2; }
                else { got = jq; gty = (int)ty; }
            }
            j = min(j + SPILL_VEC, jend + 1);
        }
#elif JH_SPILL_VEC > 1
        // SPILL_VEC rows per step: their process and type loads are issued
        // together, so a long walk waits on one memory latency per step, not
        // per row (lr < n: every load is in bounds)
        for (int64_t j = j0; j <= lr && got == -1; j += SPILL_VEC) {
            long long pv[SPILL_VEC], tv[SPILL_VEC];
#pragma unroll
            for (int q = 0; q < SPILL_VEC; q++) {
                const int64_t jq = min(j + q, lr);
                pv[q] = proc[jq]; tv[q] = type[jq];
            }
#pragma unroll
            for (int q = 0; q < SPILL_VEC; q++) {
                const int64_t jq = j + q;
                if (got != -1 || jq > lr || pv[q] != p) continue;
                const int64_t ty = tv[q] & 3;
                if (ty == T_INFO) continue;
                if (ty == T_INVOKE) { atomicMin(&m->viol1, ((unsigned long long)jq << 4) | JH_CAUSE_DOUBLE_INVOKE); got = -2; }
                else { got = jq; gty = (int)ty; }
            }
        }
#else
        for (int64_t j = j0; j <= lr; j++) {
            if (proc[j] != p) continue;
            const int64_t ty = type[j] & 3;
            if (ty == T_INFO) continue;
            if (ty == T_INVOKE) { atomicMin(&m->viol1, ((unsigned long long)j << 4) | JH_CAUSE_DOUBLE_INVOKE); got = -2; }
            else { got = j; gty = (int)ty; }
            break;
        }
#endif
        if (got >= 0) atomicAnd(&cw[got], ~CW_U);
        const bool got_okread = got >= 0 && gty == T_OK && f[got] == JH_F_READ;
        if (got_okread) {
            // an :ok :read counts in its tile as a read row only when it
            // completes an [:invoke :read] (checker.clj:713-716); completing
            // anything else it has no pending read: an orphan, stripped of its
            // kind as the in-chunk pairing does (k_cnt_pack), so no later pass
            // reads its pair[] (never written for it)
            if (f2 == F2_READ) atomicAdd(&agg[got / CNT_TILE].nr, 1);
            else {
                atomicMin(&m->viol2, ((unsigned long long)got << 4) | JH_CAUSE_ORPHAN);
                atomicAnd(&cw[got], ~7u);
            }
        }
        if (f2 == F2_ADD) {
            uint32_t w = CW_NONE;
            const bool failed = got >= 0 && gty == T_FAIL;
            if (got != -2 && !failed) {
                long long v = vr;
                bool own = true;
                if (v == JH_NIL && got >= 0) { v = val[got]; own = false; }
                if (v == JH_NIL) atomicMin(&m->viol2, ((unsigned long long)r << 4) | JH_CAUSE_NIL_VALUE);
                else {
                    w = cw_make(CW_HI, v);
                    if ((w & CW_X) && !own) pair[r] = (int32_t)got;
                    atomicAdd((unsigned long long *)&agg[r / CNT_TILE].hi, (unsigned long long)v);
                }
            }
            cw[r] = w;
        } else if (f2 == F2_READ && got_okread) {
            pair[got] = (int32_t)r;
        }
    }
}


// thread t takes rows CNT_PER*t .. of each of the block's TS_TILES tiles in
// order, from the tile's exclusive prefix; writes only at read rows. Every
// tile's words are loaded before any is scanned, and one barrier serves them
// all. Measured (profiles/r04/c2_spill/): 1 tile 207 us per 100 M rows, 2
// tiles (122 VGPRs) 263, 4 tiles 458; one tile per block stays.
#ifndef JH_TS_TILES
#define JH_TS_TILES 1
#endif
constexpr int TS_TILES = JH_TS_TILES;
#ifdef JH_TS_WPE
#define TS_ATTR __attribute__((amdgpu_waves_per_eu(JH_TS_WPE, JH_TS_WPE)))
#else
#define TS_ATTR
#endif
__global__ void TS_ATTR __launch_bounds__(256) k_cnt_tile_scan(const uint32_t *__restrict__ cw,
                                                       const int32_t *__restrict__ pair,
                                                       const int64_t *__restrict__ val, int64_t n,
                                                       int64_t n_tiles, const CntAcc *__restrict__ pre,
                                                       int32_t *__restrict__ rd_row, int64_t *__restrict__ rd_hi,
                                                       int64_t *__restrict__ lo_at, CntAcc *total, CntMeta *m) {
    __shared__ long long sc[TS_TILES][3][4];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * TS_TILES;
    CntAcc p[TS_TILES];
    uint32_t w[TS_TILES][CNT_PER];
#pragma unroll
    for (int t = 0; t < TS_TILES; t++) {
        const int64_t r0 = (t0 + t) * CNT_TILE + (int64_t)tid * CNT_PER;
        p[t] = t0 + t < n_tiles ? pre[t0 + t] : CntAcc{0, 0, 0, 0};
        if (r0 + CNT_PER <= n) {
            const uint4 a = *(const uint4 *)(cw + r0), b = *(const uint4 *)(cw + r0 + 4);
            w[t][0] = a.x; w[t][1] = a.y; w[t][2] = a.z; w[t][3] = a.w;
            w[t][4] = b.x; w[t][5] = b.y; w[t][6] = b.z; w[t][7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < CNT_PER; j++) w[t][j] = r0 + j < n ? cw[r0 + j] : 0u;
        }
    }
    long long lo[TS_TILES], hi[TS_TILES], il[TS_TILES], ih[TS_TILES];
    int nr[TS_TILES], in[TS_TILES];
    unsigned long long orphan = ~0ULL;        // a completion no invocation claimed
#pragma unroll
    for (int t = 0; t < TS_TILES; t++) {
        const int64_t r0 = (t0 + t) * CNT_TILE + (int64_t)tid * CNT_PER;
        lo[t] = 0; hi[t] = 0; nr[t] = 0;
#pragma unroll
        for (int j = 0; j < CNT_PER; j++) {
            const uint32_t k = w[t][j] & 7;
            if (w[t][j] & CW_U) orphan = min(orphan, (unsigned long long)(r0 + j));
            if (k == CW_LO) lo[t] += cw_val(w[t][j], val, pair, r0 + j);
            else if (k == CW_HI) hi[t] += cw_val(w[t][j], val, pair, r0 + j);
            else if (k == CW_OKREAD && !(w[t][j] & CW_U)) nr[t]++;
        }
        il[t] = lo[t]; ih[t] = hi[t]; in[t] = nr[t];
    }
    if (__any(orphan != ~0ULL)) {
        for (int o = 32; o > 0; o >>= 1) orphan = min(orphan, (unsigned long long)__shfl_xor(orphan, o));
        if (lane == 0) atomicMin(&m->viol1, (orphan << 4) | JH_CAUSE_ORPHAN);
    }
    // block exclusive scans of the per-thread sums: wave shuffles, then the
    // totals of the waves before (one barrier for every tile)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int t = 0; t < TS_TILES; t++) {
            const long long a0 = __shfl_up(il[t], o), a1 = __shfl_up(ih[t], o);
            const int a2 = __shfl_up(in[t], o);
            if (lane >= o) { il[t] += a0; ih[t] += a1; in[t] += a2; }
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int t = 0; t < TS_TILES; t++) { sc[t][0][wv] = il[t]; sc[t][1][wv] = ih[t]; sc[t][2][wv] = in[t]; }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TS_TILES; t++) {
        const int64_t r0 = (t0 + t) * CNT_TILE + (int64_t)tid * CNT_PER;
        long long el = il[t], eh = ih[t], en = in[t];
        for (int v = 0; v < wv; v++) { el += sc[t][0][v]; eh += sc[t][1][v]; en += sc[t][2][v]; }
        long long rl = p[t].lo + el - lo[t], rh = p[t].hi + eh - hi[t], rn = p[t].nr + en - nr[t];
#pragma unroll
        for (int j = 0; j < CNT_PER; j++) {
            const uint32_t k = w[t][j] & 7;
            const int64_t r = r0 + j;
            if (k == CW_LO) rl += cw_val(w[t][j], val, pair, r);
            else if (k == CW_HI) rh += cw_val(w[t][j], val, pair, r);
            else if (k == CW_OKREAD && !(w[t][j] & CW_U)) { rn++; rd_row[rn - 1] = (int32_t)r; rd_hi[rn - 1] = rh; }
            else if (k == CW_INVREAD) lo_at[r] = rl;
            if (r == n - 1) *total = CntAcc{rl, rh, (int)rn, 0};
        }
    }
}

struct CntSumOp {
    __host__ __device__ CntAcc operator()(const CntAcc &a, const CntAcc &b) const {
        return CntAcc{a.lo + b.lo, a.hi + b.hi, a.nr + b.nr, 0};
    }
};

__global__ void k_cnt_triples(const int32_t *__restrict__ rd_row, const int64_t *__restrict__ rd_hi,
                              const int64_t *__restrict__ lo_at, const int32_t *__restrict__ pair,
                              const int64_t *__restrict__ val, const CntAcc *__restrict__ total,
                              int64_t *__restrict__ out, int64_t cap, CntMeta *m) {
    const int64_t nr = total->nr;
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
    // pair: written (and read) only at :ok :read rows and at the rare rows
    // whose value word escapes to the column
    int32_t *pair = ctx->ws<int32_t>(WS_C_PAIR, n);
    uint32_t *cw = ctx->ws<uint32_t>(WS_C_PT, n + 8);
    HIP_TRY(hipMemsetAsync(last, 0xFF, sizeof(int32_t) * (span + 1), st));
    uint2 *spill = ctx->ws<uint2>(WS_C_IDX, n);              // reused for the read rows below
    const int64_t n_tiles = (n + CNT_TILE - 1) / CNT_TILE;
    CntAcc *agg = ctx->ws<CntAcc>(WS_C_OUT2, 2 * n_tiles + 1);     // written by every pack block
    int32_t *spill_n = ctx->ws<int32_t>(WS_C_FLAG, n_tiles);       // likewise
    CntAcc *pre = agg + n_tiles;
    uint2 *tab = ctx->ws<uint2>(WS_C_TAB, (size_t)n_tiles * (PAIR_PROCS + 1));   // + tab_n
    int32_t *tab_n = (int32_t *)(tab + (size_t)n_tiles * PAIR_PROCS);
    CntAcc *total = pre + n_tiles;
    k_cnt_pack<<<(int)n_tiles, PACK_THREADS, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n,
                                                     mh.pmin, last, cw, pair, spill, spill_n, tab, tab_n, m, agg);
    k_cnt_pair_spill<<<grid_for(n_tiles * SPILL_LANES, 256, 16384), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, n,
                                                                      mh.pmin, last, spill, spill_n, n_tiles, tab, tab_n, cw, pair, m, agg);

    // reduce-then-scan over tiles of contribution words
    int32_t *rd_row = ctx->ws<int32_t>(WS_C_IDX, n);
    int64_t *rd_hi = ctx->ws<int64_t>(WS_C_HI, n);
    int64_t *lo_at = ctx->ws<int64_t>(WS_C_LO, n);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tb, agg, pre, CntSumOp(), CntAcc{0, 0, 0, 0}, (int)n_tiles, st));
    void *tmp = ctx->ws<char>(WS_S_TMP, tb);
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(tmp, tb, agg, pre, CntSumOp(), CntAcc{0, 0, 0, 0}, (int)n_tiles, st));
    k_cnt_tile_scan<<<(unsigned)((n_tiles + TS_TILES - 1) / TS_TILES), 256, 0, st>>>(cw, pair, dh->value, n, n_tiles, pre,
                                                                                      rd_row, rd_hi, lo_at, total, m);
    // the triples of every :ok :read (their count stays on the device: the
    // kernel reads it), then one host round trip for the verdict
    const int64_t cap = std::min(n, reads_cap);
    int64_t *out = ctx->ws<int64_t>(WS_C_OUT, 3 * std::max<int64_t>(cap, 1));
    k_cnt_triples<<<grid_for(n / 64 + 1, 256, 4096), 256, 0, st>>>(rd_row, rd_hi, lo_at, pair, dh->value, total,
                                                                  out, cap, m);
    CntAcc th;
    HIP_TRY(hipMemcpyAsync(&th, total, sizeof th, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&mh, m, sizeof mh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // Clojure + throws on long overflow; if no prefix can overflow we need no
    // ordered overflow check (else the shim falls back to the JVM checker).
    if (mh.amax_abs > 0 && (unsigned long long)mh.amax_abs > (unsigned long long)(LLONG_MAX / std::max(1LL, mh.n_add)))
        throw_jh(JH_EUNSUPPORTED, "add values large enough to overflow a long");
    const int64_t nr = th.nr;
    const int64_t got = std::min(nr, cap);
    if (got > 0 && reads_out) {
        HIP_TRY(hipMemcpyAsync(reads_out, out, sizeof(int64_t) * 3 * got, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    *n_reads = nr;
    if (mh.viol1 != ~0ULL) { *valid = JH_UNKNOWN; *cause = (int)(mh.viol1 & 15); *n_reads = 0; return; }
    if (mh.viol2 != ~0ULL) { *valid = JH_UNKNOWN; *cause = (int)(mh.viol2 & 15); *n_reads = 0; return; }
    *n_errors = mh.n_errors;
    *first_err = mh.first_err == ~0ULL ? -1 : (int64_t)mh.first_err;
    if (mh.viol3 != ~0ULL) { *valid = JH_UNKNOWN; *cause = JH_CAUSE_NIL_VALUE; return; }
    *valid = mh.n_errors ? JH_INVALID : JH_VALID;
}
