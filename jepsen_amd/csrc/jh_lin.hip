// jh_lin.hip -- independent cas-register linearizability on MI355X.
//
// Replaces (independent/checker (checker/linearizable {:model (model/cas-register)}))
//   jepsen/src/jepsen/independent.clj:247-298, jepsen/src/jepsen/checker.clj:127-158
// with one batched device pass over the whole columnar history:
//
//   k_range      value/process ranges (values are interned to dense state ids)
//   k_keys       (key, row) pairs; nemesis/unkeyed rows go to a sentinel key
//   radix sort   stable partition by key = history-keys + subhistory for every
//                key at once (independent.clj:222-245), O(N) not O(K*N)
//   k_seg_off    CSR segment offsets per key
//   k_gather     16-byte records per sorted position
//   k_pair       knossos.history/complete pairing inside each key segment
//   k_orphan     completions with no open invocation
//   k_lin_dfs    persistent waves, one key at a time per wave: build the op
//                table and the window table W(t) in LDS, then the WGL search
//                in canonical coordinates (t, mask, state) with a wave-ballot
//                over the window and an HBM-resident open-addressed memo
//   k_summary    merge-valid / failures / first failing row
//
// The search order and the memo semantics are exactly those of the CPU
// oracle's orc_wgl_canonical (oracle/jh_oracle.c), so verdicts AND explored
// counts (= knossos' WGL cache size) are bit-identical.
#include "jh_internal.h"
#include <hipcub/hipcub.hpp>
#include <algorithm>

namespace {

constexpr int F_READ = 0, F_WRITE = 1, F_CAS = 2, F_OTHER = 4;
constexpr int T_INVOKE = 0, T_OK = 1, T_FAIL = 2, T_INFO = 3;
constexpr uint64_t VIOL_NONE = ~0ULL;
#ifndef JH_LDS_TBL
#define JH_LDS_TBL 0
#endif
constexpr int LDS_TBL = JH_LDS_TBL;       // per-wave op + layer tables in LDS (0: global, L2-resident)
#ifdef JH_STEP_PROF
#define PROF_MARK(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(acc, a, b) acc += (b) - (a)
#else
#define PROF_MARK(v)
#define PROF_ADD(acc, a, b)
#endif
#ifdef JH_DFS_STATS
#define DFS_STAT(x) x
#else
#define DFS_STAT(x)
#endif
// Per-wave LDS of the DFS: [tables LDS_TBL][memo BKT x 4 x 8 B][Bloom][bucket fill bytes]
template <int LG_BKT, int LG_BLOOM>
struct MemoCfg {
    static constexpr int LG = LG_BKT;
    static constexpr int BKT = 1 << LG_BKT;           // 4-slot buckets (hot layers t >= theta)
    static constexpr int SLOTS = BKT * 4;
    static constexpr int EVICT = SLOTS * 5 / 8;        // evict at load factor 5/8
    static constexpr int BLOOM = 1 << LG_BLOOM;       // bits, over the HBM-resident entries
    static constexpr int OFF_MEMO = LDS_TBL;
    static constexpr int OFF_BLOOM = OFF_MEMO + SLOTS * 8;
    static constexpr int OFF_CNT = OFF_BLOOM + BLOOM / 8;
    static constexpr int LDS = OFF_CNT + BKT;
};
// phase 1: 4 KB memo + 2 KB Bloom = 6.1 KB -> 26 waves/CU. Measured against the
// 8 KB memo (15 waves/CU): C3 40.8 -> 40.2 ms, C4 shard 283 -> 268 ms (phase 1
// 108 -> 93 ms), C5 flat (tools/gpu_ab_workloads.sh); 2 KB memos lose again
#ifndef JH_MEMOQ_LG
#define JH_MEMOQ_LG 7
#define JH_MEMOQ_BLOOM 14
#endif
using MemoQ = MemoCfg<JH_MEMOQ_LG, JH_MEMOQ_BLOOM>;
#ifndef JH_MEMOH_BLOOM
#define JH_MEMOH_BLOOM 17
#endif
using MemoH = MemoCfg<12, JH_MEMOH_BLOOM>;   // heavy keys: 128 KB memo + 16 KB Bloom = 152 KB -> 1 wave/CU
                                              // (16 KB Bloom vs 8 KB: -4..7% on the heaviest C3 keys)
using MemoM = MemoCfg<10, 15>;   // very heavy keys: 32 KB memo + 4 KB Bloom = 37 KB -> 4 waves/CU
// phase 2's LEAN role (k_lin_seq_lw) when no WIDE keys share its grid: the
// 32 KB memo with a 16 KB Bloom filter over its HBM-resident layers, three
// waves per CU, tables for the phase-2 budget (phase 3 takes the keys past
// it). Round 5, profiles/r05/ab_p2_bloom/: the heavy keys of the slow ranks
// keep ~30 K configurations in HBM, where MemoM's 4 KB filter answers "maybe"
// for most probes (each then an HBM round trip): C3 rank 4 53.4 -> 50.4 ms,
// rank 7 43.7 -> 41.5 ms, ranks 0 / 3 and C4 flat
#ifndef JH_P2_LG
#define JH_P2_LG 10
#define JH_P2_BLOOM 17
#endif
#ifndef JH_P2_PER_CU
#define JH_P2_PER_CU 3
#endif
using MemoP2 = MemoCfg<JH_P2_LG, JH_P2_BLOOM>;
constexpr int STATE_BITS = 20, T_BITS = 20, GEN_BITS = 24;
constexpr uint32_t STATE_MASK = (1u << STATE_BITS) - 1, T_MASK = (1u << T_BITS) - 1;

// 16-byte record per sorted position
struct Rec {
    int32_t proc;
    uint8_t type, f;
    uint16_t pad;
    int32_t v1, v2;   // interned state ids: 0 = nil, value - vmin + 1 otherwise
};

// one op of a key, in call order
struct Op {
    int32_t v1, v2;
    int32_t rr;       // return rank among ok ops; -1 crashed
    int32_t fa;       // f | (a << 2); a = ok returns before the invocation
};

struct Frame {        // DFS stack frame: the parent configuration + taken candidate
    uint64_t mask;
    uint64_t rest;    // candidates after i whose child was not known present at the push
    uint32_t t_i;     // t << 6 | i
    int32_t s;
    uint32_t pad[2];
};

struct RangeOut {
    long long vmin, vmax;
    long long pmax;
    int unkeyed_client;
    int bad_value;
    int smax;
    int pad;
};

__device__ __forceinline__ int f_code(int64_t f) {
    return f == JH_F_READ ? F_READ : f == JH_F_WRITE ? F_WRITE : f == JH_F_CAS ? F_CAS : F_OTHER;
}

__global__ void __launch_bounds__(256) k_range(const int64_t *__restrict__ proc, const int64_t *__restrict__ f,
                        const int64_t *__restrict__ key, const int64_t *__restrict__ v1,
                        const int64_t *__restrict__ v2, int64_t n, int keyed, RangeOut *out) {
    long long lo = LLONG_MAX, hi = LLONG_MIN, pm = -1;
    int unk = 0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int64_t p = proc[r];
        if (p < 0) continue;
        pm = max(pm, (long long)p);
        if (keyed && key && key[r] < 0) unk = 1;
        const int fc = f_code(f[r]);
        if (fc <= F_CAS) {
            int64_t a = v1[r];
            if (a != JH_NIL) { lo = min(lo, (long long)a); hi = max(hi, (long long)a); }
            if (fc == F_CAS) {
                int64_t b = v2[r];
                if (b != JH_NIL) { lo = min(lo, (long long)b); hi = max(hi, (long long)b); }
            }
        }
    }
    __shared__ long long sh[4];
    __shared__ int shi[4];
    lo = block_reduce256(lo, RedMin(), sh);
    hi = block_reduce256(hi, RedMax(), sh);
    pm = block_reduce256(pm, RedMax(), sh);
    unk = block_reduce256(unk, RedOr(), shi);
    if (threadIdx.x == 0) {
        if (lo != LLONG_MAX) atomicMin(&out->vmin, lo);
        if (hi != LLONG_MIN) atomicMax(&out->vmax, hi);
        if (pm >= 0) atomicMax(&out->pmax, pm);
        if (unk) atomicOr(&out->unkeyed_client, 1);
    }
}

// Sort keys: client keyed rows -> key; everything else -> K (sentinel).
// Keyed rows of a non-client process stay in their key's segment (the key
// exists for history-keys, independent.clj:222-232) and are skipped later.
__global__ void k_keys(const int64_t *__restrict__ key, int64_t n, int64_t K, int keyed,
                       uint32_t *__restrict__ k32, uint32_t *__restrict__ r32) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        int64_t k = keyed ? (key ? key[r] : -1) : 0;
        k32[r] = (k >= 0 && k < K) ? (uint32_t)k : (uint32_t)K;
        r32[r] = (uint32_t)r;
    }
}

__global__ void k_seg_off(const uint32_t *__restrict__ sk, int64_t n, int64_t K,
                          uint32_t *__restrict__ off, RangeOut *ro) {
    int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k > K) return;
    // lower_bound(sk, k)
    int64_t a = 0, b = n;
    while (a < b) {
        int64_t m = (a + b) >> 1;
        if (sk[m] < (uint32_t)k) a = m + 1; else b = m;
    }
    off[k] = (uint32_t)a;
    if (k < K) {
        // segment size needs off[k+1]; recompute the upper bound locally
        int64_t a2 = a, b2 = n;
        while (a2 < b2) {
            int64_t m = (a2 + b2) >> 1;
            if (sk[m] <= (uint32_t)k) a2 = m + 1; else b2 = m;
        }
        atomicMax(&ro->smax, (int)(a2 - a));
    }
}

__global__ void k_gather(const int64_t *__restrict__ proc, const int64_t *__restrict__ type,
                         const int64_t *__restrict__ f, const int64_t *__restrict__ v1,
                         const int64_t *__restrict__ v2, const uint32_t *__restrict__ rows,
                         int64_t m, long long vmin, Rec *__restrict__ rec) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m;
         p += (int64_t)gridDim.x * blockDim.x) {
        uint32_t r = rows[p];
        Rec x;
        int64_t pr = proc[r];
        x.proc = pr < 0 ? -1 : (int32_t)pr;
        x.type = (uint8_t)type[r];
        x.f = (uint8_t)f_code(f[r]);
        x.pad = 0;
        int64_t a = v1[r], b = v2[r];
        x.v1 = a == JH_NIL ? 0 : (int32_t)(a - vmin + 1);
        x.v2 = b == JH_NIL ? 0 : (int32_t)(b - vmin + 1);
        if (x.f > F_CAS) { x.v1 = 0; x.v2 = 0; }
        rec[p] = x;
    }
}

// knossos.history/complete pairing (cassandra/src/cassandra/checker.clj:7-62):
// the completion of an invocation is the next entry of the same process
// that is not :info; an :invoke there is a double invocation. One wave per
// 64 consecutive sorted positions walks 64-row windows of the records: for
// each distinct (key, process) among its still-open invocations one ballot
// gives every candidate row, and each open lane takes the first one after
// its own position; a lane stops at its key segment's end.
__global__ void __launch_bounds__(256) k_pair(const Rec *__restrict__ rec, const uint32_t *__restrict__ sk,
                                              const uint32_t *__restrict__ off, int64_t m,
                                              int32_t *__restrict__ pair,
                                              unsigned long long *__restrict__ viol) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); wv * 64 < m; wv += nw) {
        const int64_t base = wv * 64, p = base + lane;
        int32_t xp = -1, xt = T_INFO;
        uint32_t k = 0;
        if (p < m) { const Rec x = rec[p]; xp = x.proc; xt = x.type; k = sk[p]; }
        const bool inv = p < m && xp >= 0 && xt == T_INVOKE;
        const int64_t end = inv ? (int64_t)off[k + 1] : 0;
        bool open = inv && end > p + 1;
        int64_t got = -1;
        int gtype = 0;
        for (int64_t wb = base; wb < m; wb += 64) {
            if (!__ballot(open)) break;
            const int64_t j = wb + lane;
            int32_t yp = -1, yt = T_INFO;
            uint32_t yk = 0xFFFFFFFFu;
            if (j < m) { const Rec y = rec[j]; yp = y.proc; yt = y.type; yk = sk[j]; }
            uint64_t todo = __ballot(open);
            while (todo) {
                const int l = __builtin_ctzll(todo);
                const int32_t pl = __builtin_amdgcn_readlane(xp, l);
                const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)k, l);
                const uint64_t mine = __ballot(open && xp == pl && k == kl);
                const uint64_t cand = __ballot(yp == pl && yk == kl && yt != T_INFO);
                const uint64_t cinv = __ballot(yt == T_INVOKE);
                todo &= ~mine;
                if ((mine >> lane) & 1) {
                    const int64_t rel = p - wb;
                    const uint64_t after = rel < 0 ? ~0ULL : (rel >= 63 ? 0ULL : (~0ULL << (rel + 1)));
                    const uint64_t c = cand & after;
                    if (c) {
                        const int b = __builtin_ctzll(c);
                        got = wb + b; gtype = (int)((cinv >> b) & 1); open = false;
                    }
                }
            }
            if (open && wb + 64 >= end) open = false;
        }
        if (got >= 0) {
            if (gtype) atomicMin(&viol[k], ((unsigned long long)got << 4) | JH_CAUSE_DOUBLE_INVOKE);
            else { pair[p] = (int32_t)got; pair[got] = (int32_t)p; }
        }
    }
}

__global__ void k_orphan(const Rec *__restrict__ rec, const uint32_t *__restrict__ sk,
                         int64_t m, const int32_t *__restrict__ pair,
                         unsigned long long *__restrict__ viol) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m;
         p += (int64_t)gridDim.x * blockDim.x) {
        Rec x = rec[p];
        if (x.proc < 0 || (x.type != T_OK && x.type != T_FAIL)) continue;
        if (pair[p] < 0) atomicMin(&viol[sk[p]], ((unsigned long long)p << 4) | JH_CAUSE_ORPHAN);
    }
}

// ---------------------------------------------------------------------------
struct DfsArgs {
    const Rec *rec;
    const int32_t *pair;
    const uint32_t *off;
    const uint32_t *rows;
    const unsigned long long *viol;
    int32_t *rank;              // per sorted position scratch
    const int32_t *list;        // keys to process
    int32_t n_list;
    int32_t *queue;             // work counter
    jh_key_verdict *out;
    int32_t *defer_list;        // phase 2: keys over its budget (to phase 3)
    int32_t *defer_count;
    // phase 1: keys over the quick budget as (progress << 32 | key), progress =
    // deepest layer / layers (k_sort_defer orders the heavy pass by it): every
    // deferred key in defer64, and this kernel's mode (LEAN / WIDE) in defer_kind
    uint64_t *defer64;
    uint64_t *defer_kind;
    int32_t *defer_kind_count;
    uint64_t *memo;             // per wave: memo_cap entries x 2 words
    uint32_t memo_cap;          // power of two
    Frame *stack;               // per wave: stack_cap frames
    uint32_t stack_cap;
    char *scratch;              // per wave: the LDS memo eviction stage
    uint64_t scratch_bytes;
    int64_t budget;             // memo inserts before giving up
    int32_t defer;              // 1: over budget -> defer list; 0: -> :unknown
    int32_t init_state;
    uint32_t gen_base;
    int32_t *flags;             // [0] |= 1: key too large for this build
    unsigned long long *probes; // total memo probes (roofline accounting)
    int32_t states8;            // every interned state < 256 (LDS memo packing)
    unsigned long long *dbg;    // JH_DEBUG=2: per-wave cycle accounting (8 words)
    int32_t *claim;             // race with k_lin_bfs: per-key first-writer flag (or null)
    const struct KeyMeta *meta; // per key: tables offset and sizes (k_key_tables)
    const char *tables;         // the tables arena
    const int32_t *n_list_dev;  // if set: the list length, on the device
    int64_t budget_full;        // defer mode: past `budget` a search keeps going up to this
                                // budget once the queue has no key left for its wave
    // phase 2 with late helpers (k_lin_wg in helper mode): per key, the
    // s_memrealtime at which a wave took it (0 not yet, SEQ_HANDED: gone to
    // phase 3), and the number of waves that have left the queue
    unsigned long long *seq_start;
    int32_t *exit_count;
    // round 6 (JH_LIN_HELP_STALL): the sequential search re-stamps seq_start
    // whenever its deepest layer advances, so the late helpers pick the keys
    // stuck longest (a big dead subtree) rather than the ones running longest
    int32_t stamp_progress;
    // JH_DEFER_TIMES=1 (timeline study): [0] first wave start, [1] last wave
    // end (s_memrealtime), [2 + key] the time the key was handed on
    unsigned long long *defer_time;
    // run only when the list length (read on the device) is in [n_min, n_max]
    // (n_max 0: no upper bound): phase 3 picks one of two launched kernels
    int32_t n_min, n_max;
    int32_t cause_or;           // :linear mode: CAUSE_BY_WGL on the verdicts (k_frontier)
    // k_lin_seq_lw runs two roles in one grid: this role's waves are blocks
    // wave_off.. (their per-wave tables are indexed from 0)
    int32_t wave_off;
    // [0] first wave start, [1] last wave end (s_memrealtime, 100 MHz): the
    // role's time when it shares a launch with another role (or null)
    unsigned long long *t_span;
    // phase 1: once its queue is empty, a search past handover_min inserts
    // stops and goes to the heavy-key pass (which restarts it with its own
    // budget, so verdicts and counts do not change) instead of holding the
    // phase open while every other wave idles; 0: never
    int32_t handover_min;
    // phase 1: a search raises its wave's issue priority (s_setprio 1..3) at
    // prio_ins, 2 x and 4 x prio_ins inserts, so the few long searches of a
    // crowded CU (26 waves) run near a lone wave's speed while the many short
    // ones fill the gaps; 0: off
    int32_t prio_ins;
    // The streaming heavy-key pass (round 4: the heavy keys start when phase 1
    // defers them, not when phase 1 ends). Phase 1 also appends each deferred
    // key (int32) to s_all and to its kind's s_kind (lists filled with -1
    // first; their lengths are defer_count / defer_kind_count), counts every
    // key it finishes in p1_count, and the wave that first finds the last
    // phase-1 kernel's queue empty raises *drained (host-mapped memory) so the
    // host launches the consumers then, into CUs that phase 1 is leaving.
    // Consumers: `list` is live, *live_n long, and complete once *p1_done ==
    // p1_tot[0] + p1_tot[1] (phase 1's LEAN and WIDE list lengths).
    int32_t *s_all, *s_kind;
    int32_t *p1_count;          // phase 1 (producer): incremented per finished key
    const int32_t *p1_done;     // consumers: the same counter, read
    const int32_t *p1_tot;
    int32_t *drained;
    const int32_t *live_n;
    unsigned long long *tl;     // -DJH_TUNING timeline (JH_DEFER_TIMES): per key [2] search start, [3] end
    // Resume (round 5): phase 1 (rs_mode 1) saves a deferred LEAN key's search
    // -- its configuration, stack and every configuration in its memo (WGL's
    // cache) -- as a record in rs_arena (bump-allocated by rs_used, rs_off[key]
    // = its byte offset, -1 none); phase 2's sequential search (rs_mode 2)
    // continues that key from its record instead of restarting it. The DFS is
    // the same from there on, so verdicts and explored counts do not change.
    uint8_t *rs_arena;
    unsigned long long *rs_used;
    uint64_t rs_cap;
    int64_t *rs_off;
    int32_t rs_mode;
    // phase 1 with resume: per wave, the HBM-table slot of every configuration
    // the search writes there (hlog_cap each), so a save gathers the key's
    // entries instead of scanning the wave's whole table
    uint32_t *hlog;
    uint32_t hlog_cap;
    // JH_DEFER_TIMES (tuning builds): per deferred key {inserts, tmax | n_ok << 32}
    unsigned long long *defer_info;
    // Round 6, the takeover: per key, a late helper that takes a key phase 2's
    // sequential search is running asks it for its state (HO_ASK); the search
    // saves its record at its next check (HO_SAVING, then HO_DONE with
    // rs_off[key] set, or HO_REFUSED) and leaves the key, and the helper's
    // dfs_acc continues it instead of restarting it. null: off.
    int32_t *handoff;
};
constexpr int V_HANDED = -9;            // dfs_lean: saved for a takeover, continue from the record
constexpr int32_t HO_NONE = 0, HO_ASK = 1, HO_DONE = 2, HO_REFUSED = 3, HO_WITHDRAWN = 4, HO_SAVING = 5;
constexpr int TL_W = 6;         // timeline words per key: BFS, sequential, helper (start, end)
#ifdef JH_TUNING
#define TL_REC(tl, key, w) \
    do { if ((tl) && (threadIdx.x & 63) == 0) (tl)[TL_W * (size_t)(key) + (w)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TL_REC(tl, key, w) do { } while (0)
#endif
constexpr unsigned long long SEQ_HANDED = ~0ULL;

__device__ __forceinline__ int ld_agent(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
// every key of phase 1 finished: no more deferrals (p1_done is raised after
// the key's list entries are written, with release order)
__device__ __forceinline__ bool p1_finished(const int32_t *done, const int32_t *tot) {
    return ld_agent(done) >= ld_agent(tot) + ld_agent(tot + 1);
}
// One lane: the key at index idx of a live list, waiting until phase 1 has
// appended it; -1 once phase 1 has finished without reaching idx. A wait
// past STREAM_WATCHDOG (a bug, not a slow search: phase 1's longest search
// is bounded by its quick budget) sets flag 512 and gives up, so the grid
// always drains.
constexpr unsigned long long STREAM_WATCHDOG = 3000000000ULL;   // 30 s of s_memrealtime (100 MHz)
__device__ int stream_key(const int32_t *list, const int32_t *live_n, const int32_t *done, const int32_t *tot,
                          int idx, int32_t *flags) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (idx < ld_agent(live_n)) {
            for (;;) {
                const int k = ld_agent(&list[idx]);
                if (k >= 0) return k;
                if (__builtin_amdgcn_s_memrealtime() - t0 > STREAM_WATCHDOG) { atomicOr(flags, 512); return -1; }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (p1_finished(done, tot) && idx >= ld_agent(live_n)) return -1;
        if (__builtin_amdgcn_s_memrealtime() - t0 > STREAM_WATCHDOG) { atomicOr(flags, 512); return -1; }
        __builtin_amdgcn_s_sleep(20);
    }
}
// verdict cause bits naming the engine in :linear mode (k_frontier turns them into jh_key_verdict.analyzer)
constexpr int32_t CAUSE_BY_LINEAR = 0x100, CAUSE_BY_WGL = 0x200;

constexpr int JH_CANCELLED = 3; // internal: the other search settled the key first

// Phase 2 hands a key that reaches its budget to phase 3, which restarts it
// with the full budget, so that one long search does not hold back the keys
// queued behind it. Once every key of the list has been taken, and no key
// has gone to phase 3 yet, there is nothing to hold back: the search raises
// its budget to the full one and carries on (same DFS, same insert count)
// instead of starting over.
__device__ __forceinline__ bool extend_budget(const DfsArgs &A, uint32_t &budget) {
    if (A.budget_full <= (int64_t)budget) return false;
    int q = 0, d = 0, n = 0;
    if ((threadIdx.x & 63) == 0) {
        q = __hip_atomic_load(A.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        d = __hip_atomic_load(A.defer_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // a live list is only known to be exhausted once phase 1 has finished
        if (A.live_n) n = p1_finished(A.p1_done, A.p1_tot) ? ld_agent(A.live_n) : 0x7FFFFFFF;
        else n = A.n_list_dev ? *A.n_list_dev : A.n_list;
    }
    q = __builtin_amdgcn_readlane(q, 0);
    d = __builtin_amdgcn_readlane(d, 0);
    n = __builtin_amdgcn_readlane(n, 0);
    // with keys already handed to phase 3 it runs anyway (4 waves per CU for
    // many deep searches): join it rather than delay its start
    if (q < n || d > 0) return false;
    budget = (uint32_t)min<int64_t>(A.budget_full, 0x7FFFFFFF);
    return true;
}
// phase 1's hand-over check (every 1 024 inserts): the queue has run dry
__device__ __forceinline__ bool handover(const DfsArgs &A, uint32_t ins) {
    if (A.handover_min <= 0 || ins < (uint32_t)A.handover_min) return false;
    int q = 0;
    if ((threadIdx.x & 63) == 0) q = __hip_atomic_load(A.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    q = __builtin_amdgcn_readlane(q, 0);
    return q >= (A.n_list_dev ? *A.n_list_dev : A.n_list);
}
constexpr int64_t P2_BUDGET = 1 << 16;  // phase-2 inserts before a key moves to phase 3
constexpr int64_t QUICK_BUDGET = 8192;  // phase-1 inserts before a key is deferred
// phase-1 inserts after which a search may be handed over once the queue is
// empty. Round 1 measured it at 1 024 (phase 1 12.4 -> 8.0 ms but 3x the keys
// restart in phase 2: C3 59.5 -> 69.9 ms), rounds 3-4 kept it off for the same
// reason. Round 5: a handed-over search continues from its saved state (the
// resume records), so the hand-over costs nothing: 1 024 is the default when
// resuming (C3 rank 0 41.4 -> 39.2 ms, ranks 4 / 6 / 7 and C4 down too:
// profiles/r05/ab/); without resume it stays off. The checks run every 1 024
// inserts (at 1 023, 2 047, ...), so 1 024 hands searches over at 2 047.
// 1 023 (the first check) ends phase 1 at 6.3 ms instead of 7.6 and helps
// ranks 3 / 4 / 7 by 0.6-1.6 ms, but rank 0 -- the one-GPU line -- turns
// heavy-tailed: 2 of 10 runs at 46-49 ms, mean 40.1 vs 39.4 ms over 12 runs at
// 1 024 (profiles/r05/ab_handover/); finer checks (every 256 / 512 inserts)
// are worse still. 1 024 stays.
constexpr int32_t HANDOVER_MIN = 1024;
// phase-1 issue priority by insert count (DfsArgs.prio_ins): 0 = off until measured
constexpr int32_t P1_PRIO_INS = 0;
// phase-2 late helpers (workgroups, one per CU) and how long a key must have run
// in the sequential search before one takes it: 32 and 250 us measured against
// 16 and 2 000 us (C3 rank 0 43.2 -> 40.9 ms, ranks 3 / 6 unchanged; the sweep
// of tools/gpu_env_sweep.sh is flat from 24 to 48 helpers and 0 to 250 us).
// Round 6, with the spec board (idle helpers enumerate the mains' dead
// subtrees): 64 (a quarter of the CUs), measured against 32 and 96
// (profiles/r06/ab_helpers64/: C3 rank 0 39.5 -> 39.2 ms, rank 4 47.7 ->
// 45.3, the strong-scaling shards' max at N = 2 / 4 / 8 35.9 / 29.1 / 24.7 ->
// 32.6 / 24.9 / 21.1 ms; 96 leaves the sequential search too few CUs)
constexpr int HELPERS = 64;
constexpr uint64_t HELPER_LATE_US = 250;

// write a key's verdict; in a race only the first finisher writes
__device__ __forceinline__ bool emit_verdict(jh_key_verdict *out, int32_t *claim, int key,
                                             const jh_key_verdict &v) {
    if (claim && atomicCAS(&claim[key], 0, 1) != 0) return false;
    out[key] = v;
    return true;
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __ballot(b); }
__device__ __forceinline__ int mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t rflu(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int readlane(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}
// whole-wave lane shifts on the VALU (DPP), no LDS round trip:
// lane i <- lane i+1 (lane 63 keeps its value) / lane i <- lane i-1 (lane 0 keeps)
__device__ __forceinline__ int wave_shl1(int x) { return __builtin_amdgcn_update_dpp(x, x, 0x130, 0xF, 0xF, false); }
__device__ __forceinline__ int wave_shr1(int x) { return __builtin_amdgcn_update_dpp(x, x, 0x138, 0xF, 0xF, false); }

__device__ __forceinline__ uint64_t memo_hash(uint32_t t, uint32_t s, uint64_t m) {
    return jh_mix64(m * 0x9E3779B97F4A7C15ULL ^ jh_mix64(((uint64_t)t << 32) | s));
}

// cas-register step (doc/tutorial/04-checker.md:58-72) on interned states
__device__ __forceinline__ bool cas_step(int f, int v1, int v2, int s, int *o) {
    if (f == F_WRITE) { *o = v1; return true; }
    if (f == F_CAS) { if (s == v1) { *o = v2; return true; } return false; }
    if (v1 == 0 || v1 == s) { *o = s; return true; }
    return false;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Per-key tables, built by ONE wave (lanes 0..63) into LDS when they fit,
// else into the wave's global scratch. Everything that touches them is
// templated on the location so LDS tables compile to ds_* and scratch to
// global_* instructions (a runtime-chosen pointer would be a flat access,
// which waits for every outstanding global store of the wave).
//   ops[j]   the key's ops in call order: completed values, return rank rr
//            (-1 crashed) and a = # ok returns before the invocation
//   W, woff  the window table: W(t) = ops called before the t-th ok return
//            and not yet returned there, in call order (<= 64 per t)
// knossos.history/complete is applied here from the pairing (k_pair):
// failed ops and crashed/nil reads are dropped (sound; see jh_oracle.c).
extern __shared__ __attribute__((aligned(16))) char jh_lds[];

struct KeySrc {
    const Rec *rec;
    const int32_t *pair;
    const uint32_t *off;
    const uint32_t *rows;
    const unsigned long long *viol;
    int32_t *rank;
    int32_t *flags;
};
struct KeyInfo {
    int n_ops, n_ok;
    long long sumW;
    uint32_t s0, s1;
};

__device__ __forceinline__ uint64_t tbl_ops_bytes(const KeyInfo &K) { return (uint64_t)K.n_ops * sizeof(Op); }
__device__ __forceinline__ uint64_t tbl_off_bytes(const KeyInfo &K) { return ((uint64_t)(K.n_ok + 1) * 4 + 15) & ~15ULL; }
__device__ __forceinline__ uint64_t tbl_w_bytes(const KeyInfo &K) { return ((uint64_t)K.sumW * 2 + 128 + 15) & ~15ULL; }
__device__ __forceinline__ uint64_t tbl_bytes(const KeyInfo &K) {
    return tbl_ops_bytes(K) + tbl_off_bytes(K) + tbl_w_bytes(K);
}

// table base: the dynamic LDS region at lds_off, or the global scratch
template <bool L>
__device__ __forceinline__ char *tbl_base(uint32_t lds_off, char *gscr) {
    if constexpr (L) return jh_lds + lds_off;
    else return gscr;
}

// Pass 1: ranks of kept invocations and of ok returns (into S.rank), op and
// window sizes. Returns true if the key needs a search; otherwise v is final.
__device__ bool key_pass1(const KeySrc &S, int key, int lane, KeyInfo &K, jh_key_verdict &v) {
    v.valid = JH_VALID; v.cause = 0; v.fail_entry = -1; v.explored = 0;
    const uint32_t s0 = S.off[key], s1 = S.off[key + 1];
    K.s0 = s0; K.s1 = s1;
    if (s0 == s1) {                          // key absent: no :results entry
        v.explored = -1;
        return false;
    }
    const unsigned long long vi = S.viol[key];
    if (vi != VIOL_NONE) {
        v.valid = JH_UNKNOWN; v.cause = (int)(vi & 15);
        return false;
    }
    int n_ops = 0, n_ok = 0, n_crash = 0, badf = 0;
    long long sum_a_ok = 0, sum_a_crash = 0;
    for (uint32_t base = s0; base < s1; base += 64) {
        const uint32_t p = base + lane;
        const bool valid = p < s1;
        Rec x = valid ? S.rec[p] : Rec{-1, 0, 0, 0, 0, 0};
        const int q = valid ? S.pair[p] : -1;
        Rec y = q >= 0 ? S.rec[q] : Rec{-1, 0, 0, 0, 0, 0};
        // as an invocation
        const bool inv = x.proc >= 0 && x.type == T_INVOKE;
        const bool c_ok = inv && q >= 0 && y.type == T_OK;
        const bool c_fail = inv && q >= 0 && y.type == T_FAIL;
        int v1c = x.v1;
        if (c_ok && x.v1 == 0 && (x.f != F_CAS || x.v2 == 0)) v1c = y.v1;
        const bool kept = inv && !c_fail && !(x.f == F_READ && (!c_ok || v1c == 0));
        // as an ok return whose invocation is kept
        bool ret = false;
        if (x.proc >= 0 && x.type == T_OK && q >= 0) {
            int iv1 = y.v1;
            if (iv1 == 0 && (y.f != F_CAS || y.v2 == 0)) iv1 = x.v1;
            ret = !(y.f == F_READ && iv1 == 0);
        }
        const uint64_t bi = ballot(kept), br = ballot(ret);
        const int my_op = n_ops + mbcnt(bi);
        const int a = n_ok + mbcnt(br);
        if (valid) S.rank[p] = kept ? my_op : (ret ? -(a + 2) : -1);
        badf |= (int)(ballot(kept && x.f > F_CAS) != 0);
        const bool crash = kept && !c_ok;
        n_crash += __popcll(ballot(crash));
        long long sa_ok = (kept && c_ok) ? a : 0, sa_cr = crash ? a : 0;
        for (int o = 32; o > 0; o >>= 1) {
            sa_ok += __shfl_xor(sa_ok, o);
            sa_cr += __shfl_xor(sa_cr, o);
        }
        sum_a_ok += sa_ok; sum_a_crash += sa_cr;
        n_ops += __popcll(bi);
        n_ok += __popcll(br);
    }
    K.n_ops = n_ops; K.n_ok = n_ok;
    if (badf) {
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_BAD_F;
        return false;
    }
    if (n_ok == 0) return false;
    K.sumW = (long long)n_ok * (n_ok + 1) / 2 - sum_a_ok + (long long)n_crash * n_ok - sum_a_crash;
    if (K.sumW > (long long)JH_MAX_WINDOW * n_ok) {   // the average window is wider than the widest
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }
    if (n_ok >= (int)T_MASK) {   // beyond every table's t field: this key alone is :unknown
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }
    return true;
}

// Pass 2 + window sweep into the table at `tb`. Returns the widest window
// (> 64: the key is :unknown with cause window, as in the oracle).
template <bool L>
__device__ int key_fill(const KeySrc &S, const KeyInfo &K, int lane, char *tb) {
    Op *ops = (Op *)tb;
    int32_t *woff = (int32_t *)(tb + tbl_ops_bytes(K));
    uint16_t *W = (uint16_t *)(tb + tbl_ops_bytes(K) + tbl_off_bytes(K));
    const int n_ops = K.n_ops, n_ok = K.n_ok;
    {
        int nok = 0;
        for (uint32_t base = K.s0; base < K.s1; base += 64) {
            const uint32_t p = base + lane;
            const bool valid = p < K.s1;
            const int rk = valid ? S.rank[p] : -1;
            const bool kept = rk >= 0, ret = rk <= -2;
            const uint64_t br = ballot(ret);
            if (kept) {
                Rec x = S.rec[p];
                const int q = S.pair[p];
                int rr = -1, v1c = x.v1, v2c = x.v2;
                if (q >= 0) {
                    Rec y = S.rec[q];
                    if (y.type == T_OK) {
                        rr = -(S.rank[q] + 2);
                        if (x.f == F_CAS) { if (x.v1 == 0 && x.v2 == 0) { v1c = y.v1; v2c = y.v2; } }
                        else if (x.v1 == 0) v1c = y.v1;
                    }
                }
                const int a = nok + mbcnt(br);
                Op o; o.v1 = v1c; o.v2 = v2c; o.rr = rr; o.fa = x.f | (a << 2);
                ops[rk] = o;
            }
            nok += __popcll(br);
        }
    }
    wave_sync();
    // W(t) = W(t-1) - {RET[t-1]} + {ops with a == t}
    int maxw = 0;
    int w = 0, nxt = 0, offt = 0;
    for (int t = 0; t < n_ok; t++) {
        int prev = 0;
        bool keep = false;
        if (t > 0 && lane < w) {
            prev = W[offt - w + lane];
            keep = ops[prev].rr != t - 1;
        }
        const uint64_t bk = ballot(keep);
        const int nk = __popcll(bk);
        if (keep) W[offt + mbcnt(bk)] = (uint16_t)prev;
        // append ops whose invocation precedes the t-th ok return
        int added = 0;
        for (;;) {
            const int j = nxt + lane;
            const bool in = j < n_ops && (ops[j].fa >> 2) <= t;
            const uint64_t ba = ballot(in);
            const int c = __popcll(ba);     // a is non-decreasing: a prefix
            if (in && nk + added + lane < 64) W[offt + nk + added + lane] = (uint16_t)j;
            added += c; nxt += c;
            if (c < 64) break;
        }
        w = nk + added;
        maxw = max(maxw, w);
        if (w > 64) break;
        if (lane == 0) woff[t] = offt;
        offt += w;
        wave_sync();
    }
    if (lane == 0) woff[n_ok] = offt;
    wave_sync();
    return maxw;
}

// history row of the ok completion of RET[t] (the first op no configuration
// gets past, for an invalid key)
__device__ long long ret_row(const KeySrc &S, const KeyInfo &K, uint32_t t, int lane) {
    const int want = -((int)t + 2);
    for (uint32_t base = K.s0; base < K.s1; base += 64) {
        const uint32_t p = base + lane;
        const bool hit = p < K.s1 && S.rank[p] == want;
        const uint64_t b = ballot(hit);
        if (b) {
            const int l = __builtin_ctzll(b);
            return (long long)S.rows[readlane((int)p, l)];
        }
    }
    return -1;
}

// ---------------------------------------------------------------------------
// The WGL depth-first search, one key per wave.
//
// One wave alone issues roughly one instruction every 4 cycles, so a DFS
// step costs what its instruction count says; everything below is shaped to
// keep the common step short (no per-step divergence, scalar bookkeeping,
// one LDS round trip).
//
// Compact per-key tables, both read only in 64-entry windows:
//   OpC ops[j]   rq = req | nv << 16 (req: the state the op needs, RQ_ANY for
//                a write; nv: the state after it), fa = f | a << 2 | (rr+1) << 16
//   Lay lay[t]   rq of RET[t] ; r_t | c_t << 6
// where RET[t] is the op whose ok return defines layer t, r_t its position
// in the window W(t), and c_t the number of ops appended to the window on
// entering layer t (c_0 = |W(0)|). W(t+1) = W(t) - {RET[t]} + the next
// c_{t+1} ops in call order, so the window lives in lane registers (lane i =
// member i) and moves between layers with DPP lane shifts plus lane writes
// from two register-resident prefetch windows: the next ops in call order
// (ops[pb + lane]) and the layer table (lay[tb0 + lane]). Lifting RET[t]
// removes bit r_t from the mask and keeps removing while the next layer's RET
// op is already linearized: the canonical compaction of orc_wgl_canonical
// (oracle/jh_oracle.c) done on the mask directly. The DFS stack's top 64
// frames live in VGPRs (lane = depth mod 64) and spill to HBM in halves.
//
// Memo, LEAN mode (window <= 40, states < 256): 8-byte keys
// 1:1|t:15|state:8|mask:40 in an LDS table of 4-slot buckets, each key in
// either of its two buckets (a byte per bucket counts its filled slots).
// Every configuration with t >= theta lives there; when the table reaches
// MEMO_EVICT entries the layers farthest below the current one move to the
// wave's gen-tagged HBM table and theta rises. A child below theta that is not
// in LDS is looked up in a Bloom filter of the HBM-resident entries and then
// in HBM. WIDE mode (any window <= 64, states < 0xFFFE): every configuration
// in the HBM table, behind a Bloom filter of all inserts.
struct OpC {
    uint32_t rq;      // req | nv << 16
    uint32_t fa;      // f | a << 2 | (rr + 1) << 16   (a < 2^14, rr + 1 < 2^16)
};
struct Lay {
    uint32_t rq;      // RET[t]'s req | nv << 16
    uint32_t hi;      // r_t | c_t << 6
};
constexpr uint32_t RQ_ANY = 0xFFFF, RQ_EMPTY = 0xFFFE;
constexpr int COMPACT_MAX_OK = 16000;

__device__ __forceinline__ uint64_t tblc_ops_bytes(const KeyInfo &K) { return ((uint64_t)K.n_ops * 8 + 15) & ~15ULL; }
__device__ __forceinline__ uint64_t tblc_bytes(const KeyInfo &K) {
    return tblc_ops_bytes(K) + (((uint64_t)K.n_ok * 8 + 15) & ~15ULL);
}

// Pass 2 + layer sweep. Returns the widest window (> 64: :unknown, window).
template <bool L>
__device__ int key_fill_c(const KeySrc &S, const KeyInfo &K, int lane, char *tb) {
    OpC *ops = (OpC *)tb;
    Lay *lay = (Lay *)(tb + tblc_ops_bytes(K));
    const int n_ops = K.n_ops, n_ok = K.n_ok;
    {
        int nok = 0;
        for (uint32_t base = K.s0; base < K.s1; base += 64) {
            const uint32_t p = base + lane;
            const bool valid = p < K.s1;
            const int rk = valid ? S.rank[p] : -1;
            const bool kept = rk >= 0, ret = rk <= -2;
            const uint64_t br = ballot(ret);
            if (kept) {
                Rec x = S.rec[p];
                const int q = S.pair[p];
                int rr = -1, v1c = x.v1, v2c = x.v2;
                if (q >= 0) {
                    Rec y = S.rec[q];
                    if (y.type == T_OK) {
                        rr = -(S.rank[q] + 2);
                        if (x.f == F_CAS) { if (x.v1 == 0 && x.v2 == 0) { v1c = y.v1; v2c = y.v2; } }
                        else if (x.v1 == 0) v1c = y.v1;
                    }
                }
                const int a = nok + mbcnt(br);
                OpC o;
                // cas-register step (doc/tutorial/04-checker.md:58-72) as (needs, becomes)
                o.rq = x.f == F_READ ? ((uint32_t)v1c | ((uint32_t)v1c << 16))
                     : x.f == F_WRITE ? (RQ_ANY | ((uint32_t)v1c << 16))
                     : ((uint32_t)v1c | ((uint32_t)v2c << 16));
                o.fa = (uint32_t)x.f | ((uint32_t)a << 2) | ((uint32_t)(rr + 1) << 16);
                ops[rk] = o;
            }
            nok += __popcll(br);
        }
    }
    wave_sync();
    // Sweep the layers with the window as lane-resident ops (fa, rq).
    int maxw = 0, w = 0, nxt = 0, r_prev = 0;
    uint32_t mfa = 0, mrq = 0;
    for (int t = 0; t < n_ok; t++) {
        if (t > 0) {                               // drop RET[t-1]
            const int src = (lane + (lane >= r_prev ? 1 : 0)) & 63;
            mfa = (uint32_t)__shfl((int)mfa, src); mrq = (uint32_t)__shfl((int)mrq, src);
            w--;
        }
        int c = 0;
        for (;;) {                                 // append ops invoked before R_t
            const int j = nxt + lane;
            OpC oj = {0, 0xFFFFFFFCu};
            if (j < n_ops) oj = ops[j];
            const bool in = j < n_ops && (int)((oj.fa >> 2) & 0x3FFF) <= t;
            const int k = __popcll(ballot(in));    // a is non-decreasing: a prefix
            const int src = (lane - (w + c)) & 63;
            const uint32_t fam = (uint32_t)__shfl((int)oj.fa, src), rqm = (uint32_t)__shfl((int)oj.rq, src);
            const int dst = lane - (w + c);
            if (dst >= 0 && dst < k) { mfa = fam; mrq = rqm; }
            c += k; nxt += k;
            if (k < 64) break;
        }
        w += c;
        maxw = max(maxw, w);
        if (w > 64) { maxw = max(maxw, 65); break; }
        const bool is_ret = lane < w && (int)(mfa >> 16) == t + 1;
        const uint64_t br = ballot(is_ret);
        const int r = br ? __builtin_ctzll(br) : 0;
        if (lane == r) {
            Lay e;
            e.rq = mrq;
            e.hi = (uint32_t)r | ((uint32_t)c << 6);
            lay[t] = e;
        }
        r_prev = r;
    }
    wave_sync();
    return maxw;
}

// Bloom filter (positions from the HBM table's own 64-bit hash): a false
// positive only costs an HBM probe, never a wrong answer
template <class M>
__device__ __forceinline__ bool bloom_test2(const uint32_t *bloom, uint32_t p1, uint32_t p2) {
    p1 &= M::BLOOM - 1; p2 &= M::BLOOM - 1;
    return ((bloom[p1 >> 5] >> (p1 & 31)) & (bloom[p2 >> 5] >> (p2 & 31)) & 1u) != 0;
}
template <class M>
__device__ __forceinline__ void bloom_set2(uint32_t *bloom, uint32_t p1, uint32_t p2) {
    p1 &= M::BLOOM - 1; p2 &= M::BLOOM - 1;
    atomicOr(&bloom[p1 >> 5], 1u << (p1 & 31));
    atomicOr(&bloom[p2 >> 5], 1u << (p2 & 31));
}
// WIDE mode: positions from the HBM table's own 64-bit hash
template <class M>
__device__ __forceinline__ bool bloom_test(const uint32_t *bloom, uint64_t h) {
    return bloom_test2<M>(bloom, (uint32_t)(h >> 20), (uint32_t)(h >> 44));
}
template <class M>
__device__ __forceinline__ void bloom_set(uint32_t *bloom, uint64_t h) {
    bloom_set2<M>(bloom, (uint32_t)(h >> 20), (uint32_t)(h >> 44));
}

// insert a configuration absent from this wave's HBM table (CAS on the first
// slot of its chain whose generation tag is stale)
// The wave's HBM table: entries {mask, gen:24 | t:20 | state:20} of 16 B in
// buckets of 4 (one 64-byte line). A key hashes to a bucket; within the
// current generation a bucket fills front to back and a full bucket chains
// to the next one, so a probe reads one line per bucket (four 16-byte loads
// in flight at once) and stops at the first slot of another generation:
// one HBM round trip for nearly every probe, hit or miss (at load <= 1/2 a
// bucket is full ~14% of the time), where a linear probe over single
// entries took ~2.5 dependent round trips per miss.
constexpr uint32_t HB = 4;

#ifdef JH_DUP_WRITE
// tuning builds (round 5, the cost of phase 1's memo writes): every HBM memo
// insert is written a second time, 16 B scattered into a 1 GB mirror no one reads
__device__ ulonglong2 *g_dup_base;
#endif
__device__ __forceinline__ uint32_t hbm_insert(uint64_t *memo, uint32_t cap_mask, uint32_t gen,
                                               uint32_t ct, uint32_t cs, uint64_t cm) {
    uint32_t b = (uint32_t)memo_hash(ct, cs, cm) & cap_mask & ~(HB - 1);
    const uint64_t w1 = ((uint64_t)gen << 40) | ((uint64_t)ct << 20) | cs;
    for (;;) {
        const ulonglong2 *B = (const ulonglong2 *)(memo + 2 * (size_t)b);
        ulonglong2 e[HB];
#pragma unroll
        for (uint32_t j = 0; j < HB; j++) e[j] = B[j];
        // the first slot of another generation and its tag word, selected
        // with static indices (e[j0] put the bucket through scratch memory:
        // a store and a reload per insert)
        int j0 = -1;
        unsigned long long exp = 0;
#pragma unroll
        for (int j = HB - 1; j >= 0; j--)
            if ((e[j].y >> 40) != gen) { j0 = j; exp = e[j].y; }
        if (j0 < 0) { b = (b + HB) & cap_mask; continue; }
        // lanes of one wave may race for a slot (evictions insert from all
        // lanes at once): claim it with a CAS on the tag word
        if (__hip_atomic_compare_exchange_strong((unsigned long long *)&memo[2 * (size_t)(b + j0) + 1],
                                                 &exp, (unsigned long long)w1,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
            __hip_atomic_store(&memo[2 * (size_t)(b + j0)], cm, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef JH_DUP_WRITE
            if (g_dup_base)
                g_dup_base[((uintptr_t)&memo[2 * (size_t)(b + j0)] >> 4) & ((1u << 26) - 1)] = make_ulonglong2(cm, w1);
#endif
            return b + (uint32_t)j0;
        }
    }
}

// Probe this wave's HBM table. Returns slot | absent << 32 (absent: the slot
// an insert of this key would take).
__device__ __forceinline__ uint64_t hbm_probe(const uint64_t *memo, uint32_t cap_mask, uint32_t gen,
                                              uint32_t ct, uint32_t cs, uint64_t cm,
                                              unsigned long long &probes) {
    const uint64_t w1want = ((uint64_t)gen << 40) | ((uint64_t)ct << 20) | cs;
    uint32_t b = (uint32_t)memo_hash(ct, cs, cm) & cap_mask & ~(HB - 1);
    for (;;) {
        const ulonglong2 *B = (const ulonglong2 *)(memo + 2 * (size_t)b);
        ulonglong2 e[HB];
#pragma unroll
        for (uint32_t j = 0; j < HB; j++) e[j] = B[j];
        probes++;
        int empty = -1, hit = -1;
#pragma unroll
        for (int j = HB - 1; j >= 0; j--) {
            if ((e[j].y >> 40) != gen) empty = j;
            if (e[j].y == w1want && e[j].x == cm) hit = j;
        }
        // current-generation entries form a prefix of the bucket
        if (hit >= 0 && (empty < 0 || hit < empty)) return b + (uint32_t)hit;
        if (empty >= 0) return (1ULL << 32) | (b + (uint32_t)empty);
        b = (b + HB) & cap_mask;
    }
}

// LEAN key fields
__device__ __forceinline__ uint32_t lk_t(uint64_t k) { return (uint32_t)(k >> 48) & 0x3FFF; }   // t < COMPACT_MAX_OK < 2^14
__device__ __forceinline__ uint32_t lk_s(uint64_t k) { return (uint32_t)(k >> 40) & 0xFF; }
__device__ __forceinline__ uint64_t lk_m(uint64_t k) { return k & ((1ULL << 40) - 1); }
// two independent 32-bit hashes of a LEAN key: the top bits pick its two
// buckets, folded low bits its two Bloom positions (one multiply each: the
// fold is on the critical path of every DFS step)
__device__ __forceinline__ void lk_hash(uint32_t klo, uint32_t khi, uint32_t &h1, uint32_t &h2) {
    h1 = (klo ^ __builtin_rotateleft32(khi, 16)) * 0x9E3779B1u;
    h2 = (klo + __builtin_rotateleft32(khi, 5)) * 0x85EBCA77u;
}
template <class M>
__device__ __forceinline__ void lk_bkts(uint32_t h1, uint32_t h2, uint32_t &b1, uint32_t &b2) {
    b1 = h1 >> (32 - M::LG);
    b2 = h2 >> (32 - M::LG);
}
__device__ __forceinline__ uint32_t lk_bl(uint32_t h) { return h ^ (h >> 15); }

// Evict LDS memo layers into this wave's HBM table (out of line: it runs
// once per MEMO_EVICT inserts). theta is chosen so that the layers kept in
// LDS (t >= theta, at most a few below the current layer t_cur) fill at most
// half of what triggered the eviction; 0xFFFFFFFF = the current layer alone
// is too wide: HBM for everything below it from now on. Entries are staged
// through global scratch and the LDS table is rebuilt; an entry that finds
// both of its buckets full goes to HBM too and theta rises above its layer.
// Every entry written to HBM enters the Bloom filter, and its slot the
// wave's log when there is one (hlog: nlog entries so far). Returns
// theta << 32 | min(nlog', 0xFFFF) << 16 | kept.
template <class M>
__device__ __noinline__ uint64_t memo_evict(uint64_t *lmemo, uint32_t *bcnt, uint32_t *bloom,
                                            uint64_t *memo, uint64_t *stage,
                                            uint32_t cap_mask, uint32_t gen, uint32_t t_cur,
                                            uint32_t theta_old, int lane,
                                            uint32_t *hlog = nullptr, uint32_t hlog_cap = 0, uint32_t nlog = 0) {
    static_assert(M::SLOTS < 65536, "kept fits 16 bits");
    // histogram of entries by distance below t_cur (entries at or above it: bin 0)
    int bins = 0;                                  // lane b < 16 holds bin b
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) {
        const uint64_t x = lmemo[lane + 64 * r];
        stage[lane + 64 * r] = x;
        const uint32_t xt = lk_t(x);
        const int d = x == 0 ? 99 : (xt >= t_cur ? 0 : (int)min(t_cur - xt, 15u));
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const int cnt = __popcll(ballot(d == b));
            if (lane == b) bins += cnt;
        }
    }
    // theta = t_cur - d*, d* the largest distance keeping <= MEMO_EVICT/2
    int acc = 0, dstar = -1;
#pragma unroll 1
    for (int b = 0; b < 16; b++) {
        acc += readlane(bins, b);
        if (acc > M::EVICT / 2) break;
        dstar = b;
    }
    uint32_t th2;
    if (dstar < 0) th2 = t_cur + 1;              // the current layer alone is too wide
    else {
        th2 = t_cur > (uint32_t)dstar ? t_cur - (uint32_t)dstar : 0u;
        if (dstar == 15) th2 = t_cur - min(t_cur, 15u);
    }
    // theta never moves down: layers below the old theta may sit in HBM
    th2 = max(th2, theta_old);
    wave_sync();
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) lmemo[lane + 64 * r] = 0;
    for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    wave_sync();
    int kept = 0;
    uint32_t th_min = 0;
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) {
        const uint64_t x = stage[lane + 64 * r];
        const uint32_t xt = lk_t(x);
        bool to_hbm = x != 0 && xt < th2;
        if (x != 0 && !to_hbm) {
            uint32_t h1, h2, b1, b2;
            lk_hash((uint32_t)x, (uint32_t)(x >> 32), h1, h2);
            lk_bkts<M>(h1, h2, b1, b2);
            bool placed = false;
            for (int j = 0; j < 2 && !placed; j++) {
                const uint32_t b = j ? b2 : b1;
                const uint32_t sh = 8 * (b & 3);
                const uint32_t old = (atomicAdd(&bcnt[b >> 2], 1u << sh) >> sh) & 0xFF;
                if (old < 4) { lmemo[4 * b + old] = x; placed = true; }
                else atomicSub(&bcnt[b >> 2], 1u << sh);
            }
            if (placed) kept++;
            else { to_hbm = true; th_min = max(th_min, xt + 1); }
        }
        uint32_t slot = 0;
        if (to_hbm) {
            const uint32_t cs = lk_s(x);
            const uint64_t cm = lk_m(x);
            slot = hbm_insert(memo, cap_mask, gen, xt, cs, cm);
            uint32_t h1, h2;
            lk_hash((uint32_t)x, (uint32_t)(x >> 32), h1, h2);
            bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
        }
        if (hlog) {
            const uint64_t hm = ballot(to_hbm);
            const uint32_t at = nlog + (uint32_t)mbcnt(hm);
            if (to_hbm && at < hlog_cap) hlog[at] = slot;
            nlog += (uint32_t)__popcll(hm);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        kept += __shfl_xor(kept, o);
        th_min = max(th_min, (uint32_t)__shfl_xor((int)th_min, o));
    }
    th2 = max(th2, th_min);
    // every HBM write of this wave is visible to its later probes (the
    // table is private to the wave: workgroup scope, served by this CU's
    // caches, no L2 write-back)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    wave_sync();
    return ((uint64_t)th2 << 32) | ((uint64_t)min(nlog, 0xFFFFu) << 16) | (uint32_t)kept;
}


__device__ __forceinline__ uint64_t drop_bit(uint64_t m, uint32_t r) {
    const uint64_t lo = (1ULL << r) - 1;
    return (m & lo) | ((m >> 1) & ~lo);
}

template <bool L, bool LEAN, class M>
__device__ int dfs_search(const DfsArgs &A, const KeyInfo &K, char *tb, int key, int lane,
                          uint64_t *memo, Frame *stack, uint64_t *stage,
                          long long &inserts, uint32_t &tmax_out, unsigned long long &my_probes) {
    const OpC *ops = (const OpC *)tb;
    const Lay *lay = (const Lay *)(tb + tblc_ops_bytes(K));
    const uint32_t n_ok = (uint32_t)K.n_ok;
    const int n_ops = K.n_ops;
    const uint32_t cap_mask = A.memo_cap - 1;
    const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
    const uint64_t gen_hi = (uint64_t)gen << 40;
    uint64_t *lmemo = (uint64_t *)(jh_lds + M::OFF_MEMO);
    uint32_t *bloom = (uint32_t *)(jh_lds + M::OFF_BLOOM);
    uint32_t *bcnt = (uint32_t *)(jh_lds + M::OFF_CNT);
    const uint8_t *bcnt8 = (const uint8_t *)bcnt;
    if constexpr (LEAN) {
        for (int i = lane; i < M::SLOTS; i += 64) lmemo[i] = 0;
        for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    }
    for (int i = lane; i < M::BLOOM / 32; i += 64) bloom[i] = 0;
    const uint32_t lb_lo = lane < 32 ? 1u << lane : 0u, lb_hi = lane >= 32 ? 1u << (lane - 32) : 0u;
    uint32_t theta = 0;
    int lcount = 0;

    // layer-table window: lane j holds lay[tb0 + j]
    uint32_t tb0 = 0, drq = 0, dhi = 0;
    auto load_lay = [&](uint32_t base) {
        tb0 = base;
        const uint32_t u = base + (uint32_t)lane;
        if (u < n_ok) { const Lay e = lay[u]; drq = e.rq; dhi = e.hi; }
    };
    auto lay_hi = [&](uint32_t u) -> uint32_t {
        if (u - tb0 >= 64u) load_lay(u >= 32 ? u - 32 : 0);
        return (uint32_t)readlane((int)dhi, (int)(u - tb0));
    };
    // next-ops window: lane j holds ops[pb + j]
    int pb = 0;
    uint32_t urq = RQ_EMPTY;
    auto load_up = [&](int base) {
        pb = base;
        const int j = base + lane;
        urq = j < n_ops ? ops[j].rq : RQ_EMPTY;
    };
    // DFS stack: frames [ring_lo, depth) in lane registers, lane = index mod 64
    uint32_t fm_lo = 0, fm_hi = 0, f_ti = 0, f_s = 0, fr_lo = 0, fr_hi = 0;

    load_lay(0);
    uint32_t t = 0, tmax = 0, depth = 0, ring_lo = 0;
    uint64_t mask = 0;
    uint32_t s = (uint32_t)A.init_state;
    uint64_t cand = 0;
    bool fresh = true;
    unsigned long long pc_lift = 0, pc_probe = 0, pc_ins = 0, pc_fwd = 0, pc_pop = 0, pc_cand = 0, pc_key = 0, pc_lds = 0;          // cand = the legal un-linearized members (else: a popped frame's rest)
    int verdict = -1;
    uint32_t ins = 0;
    uint32_t budget = (uint32_t)min<int64_t>(A.budget, 0x7FFFFFFF);
    uint32_t n_steps = 0, n_evict = 0, n_reload = 0, n_slow = 0;
    // the window of layer t in lane registers
    int w = (int)(lay_hi(0) >> 6), P = w;
    uint32_t r = lay_hi(0) & 63;                    // position of RET[t]
    uint32_t wrq = lane < w ? ops[lane].rq : RQ_EMPTY;
    load_up(P);
    wave_sync();
    while (true) {
        DFS_STAT(n_steps++);
        PROF_MARK(q0);
        // candidates: un-linearized members the model allows; after a pop,
        // the frame's rest (children seen absent after the taken one: the
        // memo only grows, so nothing else can be absent now)
        const uint32_t req = wrq & 0xFFFF, nv = wrq >> 16;
        if (fresh) cand = (ballot(req == s) | ballot(req == RQ_ANY)) & ~mask;
        PROF_MARK(qa); PROF_ADD(pc_cand, q0, qa);
        fresh = true;
        uint64_t absent = 0;
        // the RET child (lane r), computed on the scalar unit
        uint32_t u_r = t;
        uint64_t nm_r = 0;
        uint32_t klo = 0, khi = 0, b1 = 0, b2 = 0, n1 = 0, n2 = 0, h1 = 0, h2 = 0;
        uint32_t ct = t;
        uint64_t cm = 0;
        bool probed = false;
        uint32_t hslot = 0;
        if (cand) {
            if ((cand >> r) & 1) {
                uint64_t nm = mask | (1ULL << r);
                uint32_t u = t, ru = r;
                for (;;) {
                    nm = drop_bit(nm, ru);
                    u++;
                    if (u >= n_ok) { nm = 0; break; }
                    ru = lay_hi(u) & 63;
                    if (!((nm >> ru) & 1)) break;
                }
                u_r = u; nm_r = nm;
            }
            PROF_MARK(q1a); PROF_ADD(pc_lift, q0, q1a);
            const bool is_r = lane == (int)r;
            if constexpr (LEAN) {
                // 8-byte child keys, all lanes at once, then one LDS round trip
                klo = is_r ? (uint32_t)nm_r : ((uint32_t)mask | lb_lo);
                khi = (is_r ? ((uint32_t)(nm_r >> 32) | (u_r << 16))
                            : ((uint32_t)(mask >> 32) | lb_hi | (t << 16))) | (nv << 8) | 0x80000000u;
                lk_hash(klo, khi, h1, h2);
                lk_bkts<M>(h1, h2, b1, b2);
                PROF_MARK(qc); PROF_ADD(pc_key, q1a, qc);
                const uint64_t k = ((uint64_t)khi << 32) | klo;
                bool hit = false;
                if ((cand >> lane) & 1) {          // candidate lanes only: fewer bank conflicts
                    const ulonglong2 *B = (const ulonglong2 *)lmemo;
                    const ulonglong2 x0 = B[2 * b1], x1 = B[2 * b1 + 1];
                    const ulonglong2 y0 = B[2 * b2], y1 = B[2 * b2 + 1];
                    n1 = bcnt8[b1]; n2 = bcnt8[b2];
                    // bitwise, not short-circuit: no branches between the four reads
                    hit = (x0.x == k) | (x0.y == k) | (x1.x == k) | (x1.y == k) |
                          (y0.x == k) | (y0.y == k) | (y1.x == k) | (y1.y == k);
                }
                absent = cand & ~ballot(hit);
                PROF_MARK(qd); PROF_ADD(pc_lds, qc, qd);
                if (t < theta && absent) {
                    DFS_STAT(n_slow++);
                    // children below theta may sit in HBM: Bloom, then HBM for
                    // the lanes before the first surely-absent one
                    uint64_t low = absent;
                    if (u_r >= theta) low &= ~(1ULL << r);
                    const uint32_t kt = khi >> 16 & 0x7FFF, ks = (khi >> 8) & 0xFF;
                    const uint64_t km = k & ((1ULL << 40) - 1);
                    const bool maybe = ((low >> lane) & 1) && bloom_test2<M>(bloom, lk_bl(h1), lk_bl(h2));
                    const uint64_t bm = ballot(maybe);
                    const uint64_t sure = absent & ~bm;
                    const uint64_t lim = sure ? ((1ULL << __builtin_ctzll(sure)) - 1) : ~0ULL;
                    bool found = false;
                    if (((bm & lim) >> lane) & 1) {
                        found = (hbm_probe(memo, cap_mask, gen, kt, ks, km, my_probes) >> 32) == 0;
                    }
                    absent &= ~ballot(found);
                }
            } else {
                ct = is_r ? u_r : t;
                cm = is_r ? nm_r : (mask | (1ULL << lane));
                const bool c_l = (cand >> lane) & 1;
                const uint64_t hh = memo_hash(ct, nv, cm);
                const bool maybe = c_l && bloom_test<M>(bloom, hh);
                const uint64_t bm = ballot(maybe);
                const uint64_t sure = cand & ~bm;
                const uint64_t lim = sure ? ((1ULL << __builtin_ctzll(sure)) - 1) : ~0ULL;
                bool found = false;
                if (((bm & lim) >> lane) & 1) {
                    const uint64_t rr = hbm_probe(memo, cap_mask, gen, ct, nv, cm, my_probes);
                    hslot = (uint32_t)rr;
                    found = (rr >> 32) == 0;
                    probed = true;
                }
                absent = cand & ~ballot(found);
            }
        }
        PROF_MARK(q2); PROF_ADD(pc_probe, q0, q2);
        if (absent) {
            if (ins >= budget && !extend_budget(A, budget)) { verdict = JH_UNKNOWN; break; }
            if ((ins & 1023) == 1023 && handover(A, ins)) { ins = budget; verdict = JH_UNKNOWN; break; }
            if (A.claim && (ins & 1023) == 1023) {
                // racing k_lin_bfs: stop if it settled this key first
                int c = 0;
                if (lane == 0) c = __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (readlane(c, 0)) { verdict = JH_CANCELLED; break; }
            }
            const int i = __builtin_ctzll(absent);
            ins++;
            const bool to_r = (uint32_t)i == r;
            const uint32_t nt = to_r ? u_r : t;
            const uint64_t nmask = to_r ? nm_r : (mask | (1ULL << i));
            const uint32_t ns = (uint32_t)readlane((int)nv, i);
            if constexpr (LEAN) {
                const bool pick1 = n1 <= n2;
                const uint32_t bs = pick1 ? b1 : b2, nsl = pick1 ? n1 : n2;
                const bool full = nsl >= 4;
                if (lane == i && !full) {
                    lmemo[4 * bs + nsl] = ((uint64_t)khi << 32) | klo;
                    ((uint8_t *)bcnt)[bs] = (uint8_t)(nsl + 1);
                }
                if ((ballot(full) >> i) & 1) {
                    // both buckets full: HBM, and theta rises above the layer
                    if (lane == i) {
                        hbm_insert(memo, cap_mask, gen, nt, ns, nmask);
                        bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
                    }
                    theta = max(theta, nt + 1);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                } else if (++lcount >= M::EVICT) {
                    DFS_STAT(n_evict++);
                    const uint64_t er = memo_evict<M>(lmemo, bcnt, bloom, memo, stage, cap_mask, gen, nt, theta, lane);
                    // a call's result is divergent to the compiler: make it scalar again
                    lcount = rfl((int)(uint32_t)er);
                    theta = rflu((uint32_t)(er >> 32));
                }
            } else {
                if (lane == i) {
                    bloom_set<M>(bloom, memo_hash(ct, nv, cm));
                    if (!probed) hbm_insert(memo, cap_mask, gen, ct, nv, cm);
                    else {
                        __hip_atomic_store(&memo[2 * (size_t)hslot], cm, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&memo[2 * (size_t)hslot + 1],
                                           gen_hi | ((uint64_t)ct << 20) | nv,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            // push the parent; a full ring spills its oldest half to HBM
            if (depth - ring_lo == 64) {
                const uint32_t k = ((uint32_t)lane - ring_lo) & 63;
                if (k < 32) {
                    Frame fr;
                    fr.mask = ((uint64_t)fm_hi << 32) | fm_lo; fr.t_i = f_ti; fr.s = (int32_t)f_s;
                    fr.rest = ((uint64_t)fr_hi << 32) | fr_lo; fr.pad[0] = fr.pad[1] = 0;
                    stack[ring_lo + k] = fr;
                }
                ring_lo += 32;
            }
            {
                const uint64_t rest = absent & (~1ULL << i);
                if (lane == (int)(depth & 63)) {
                    fm_lo = (uint32_t)mask; fm_hi = (uint32_t)(mask >> 32);
                    f_ti = (t << 6) | (uint32_t)i; f_s = s;
                    fr_lo = (uint32_t)rest; fr_hi = (uint32_t)(rest >> 32);
                }
            }
            depth++;
            mask = nmask;
            s = ns;
            PROF_MARK(q3); PROF_ADD(pc_ins, q2, q3);
            if (nt != t) {
                if (nt >= n_ok) { t = nt; tmax = max(tmax, t); verdict = JH_VALID; break; }
                // move the window forward layer by layer
                for (uint32_t u = t; u < nt; u++) {
                    const uint32_t ru = u == t ? r : (lay_hi(u) & 63);
                    const uint32_t sh = (uint32_t)wave_shl1((int)wrq);
                    if (lane >= (int)ru) wrq = sh;
                    w--;
                    if (lane == w) wrq = RQ_EMPTY;
                    const int c = (int)(lay_hi(u + 1) >> 6);
                    if (c > 0) {
                        if (P < pb || P + c > pb + 64) load_up(P);
                        for (int k = 0; k < c; k++) {
                            const uint32_t x = (uint32_t)readlane((int)urq, P - pb + k);
                            if (lane == w + k) wrq = x;
                        }
                        w += c; P += c;
                    }
                }
                t = nt;
                tmax = max(tmax, t);
                r = lay_hi(t) & 63;
                DFS_STAT(n_reload++);
            }
            PROF_MARK(q4); PROF_ADD(pc_fwd, q3, q4);
        } else {
            if (depth == 0) { verdict = JH_INVALID; break; }
            depth--;
            if (depth < ring_lo) {
                // ring empty: refill up to 32 frames below from the HBM stack
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint32_t lo = depth + 1 >= 32 ? depth + 1 - 32 : 0;
                const uint32_t k = ((uint32_t)lane - lo) & 63;
                if (k <= depth - lo) {
                    const Frame fr = stack[lo + k];
                    fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i; f_s = (uint32_t)fr.s;
                    fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32);
                }
                ring_lo = lo;
            }
            const int ln = (int)(depth & 63);
            const uint32_t ti = (uint32_t)readlane((int)f_ti, ln);
            const uint32_t pt = ti >> 6;
            mask = ((uint64_t)(uint32_t)readlane((int)fm_hi, ln) << 32) | (uint32_t)readlane((int)fm_lo, ln);
            s = (uint32_t)readlane((int)f_s, ln);
            cand = ((uint64_t)(uint32_t)readlane((int)fr_hi, ln) << 32) | (uint32_t)readlane((int)fr_lo, ln);
            fresh = false;
            if (pt != t) {
                // move the window back: drop appended ops, re-insert RETs
                for (uint32_t u = t; u > pt; u--) {
                    const int c = (int)(lay_hi(u) >> 6);
                    w -= c; P -= c;
                    if (lane >= w) wrq = RQ_EMPTY;
                    const uint32_t h = lay_hi(u - 1);
                    const int ru = (int)(h & 63);
                    const uint32_t sh = (uint32_t)wave_shr1((int)wrq);
                    if (lane > ru) wrq = sh;
                    const uint32_t x = (uint32_t)readlane((int)drq, (int)(u - 1 - tb0));
                    if (lane == ru) wrq = x;
                    w++;
                }
                t = pt;
                r = lay_hi(t) & 63;
                DFS_STAT(n_reload++);
            }
            PROF_MARK(q5); PROF_ADD(pc_pop, q2, q5);
        }
        if (depth >= A.stack_cap) { verdict = JH_UNKNOWN; if (lane == 0) atomicOr(A.flags, 4); break; }
    }
    inserts = ins;
    tmax_out = tmax;
#ifdef JH_STEP_PROF
    if (A.dbg && lane == 0) {
        unsigned long long *d = A.dbg + 16 * (size_t)blockIdx.x;
        d[10] += pc_lift; d[11] += pc_probe; d[12] += pc_ins; d[13] += pc_fwd; d[14] += pc_pop;
        d[0] += pc_cand; d[1] += pc_key; d[8] += pc_lds;
    }
#endif
#ifdef JH_DFS_STATS
    if (A.dbg && lane == 0) {
        unsigned long long *d = A.dbg + 16 * (size_t)blockIdx.x;
        d[4] += n_steps; d[5] += (unsigned long long)ins; d[6] += n_evict; d[7] += n_reload; d[9] += n_slow;
    }
#endif
    return verdict;
}

// The LEAN-mode search (window <= 40, states < 256). A lone wave issues at
// most one instruction per 4 cycles whatever its kind (VALU, SALU, branch,
// LDS), so a step costs ~4 cycles per instruction plus its LDS round trips:
// this loop is shaped to issue few instructions and few round trips.
//   - no divergent control flow on the common path: non-candidate lanes
//     probe bucket 0 (one broadcast LDS address) and are masked out of the
//     ballots afterwards; lane selects are v_cndmask;
//   - the RET child's lift is one scalar bit test in the common case (the
//     next layer's RET position rn is kept with the layer);
//   - a frame is (mask, t<<6|i, state, rest) in lane depth mod 64, where rest
//     are the candidates after i found absent when the parent was expanded;
//   - after a pop the memo is NOT probed again: a remaining child P+j holds
//     the linearized set L(P)+{j}, while everything explored in between lies
//     below P+i and holds L(P)+{i} (the canonical coordinates are a bijective
//     image of (linearized set, state), and linearized sets only grow along
//     edges), so every child in rest is still absent. The next child is
//     inserted with one read of its bucket fill counts;
//   - budget, race-cancel and ring spill/refill checks are one compare each.
// Search order and memo contents are exactly WGL's (orc_wgl_canonical,
// oracle/jh_oracle.c, which does probe after a backtrack and never finds the
// child present): explored counts stay identical.
template <class M, bool HO = false>    // HO: phase 2's takeover code (A.handoff) compiled in
__device__ __forceinline__ int dfs_lean(const DfsArgs &A, const KeyInfo &K, const char *tb, int key, int lane,
                        uint64_t *memo, Frame *stack, uint64_t *stage,
                        long long &inserts, uint32_t &tmax_out, unsigned long long &my_probes,
                        uint32_t &ins_real, uint32_t *hlog) {
    const OpC *ops = (const OpC *)tb;
    const Lay *lay = (const Lay *)(tb + tblc_ops_bytes(K));
    const uint32_t n_ok = (uint32_t)K.n_ok;
    const int n_ops = K.n_ops;
    const uint32_t cap_mask = A.memo_cap - 1;
    const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
    uint64_t *lmemo = (uint64_t *)(jh_lds + M::OFF_MEMO);
    uint32_t *bloom = (uint32_t *)(jh_lds + M::OFF_BLOOM);
    uint32_t *bcnt = (uint32_t *)(jh_lds + M::OFF_CNT);
    uint8_t *bcnt8 = (uint8_t *)bcnt;
    for (int i = lane; i < M::SLOTS; i += 64) lmemo[i] = 0;
    for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    for (int i = lane; i < M::BLOOM / 32; i += 64) bloom[i] = 0;
    const uint32_t lb_lo = lane < 32 ? 1u << lane : 0u, lb_hi = lane >= 32 ? 1u << (lane - 32) : 0u;
    uint32_t theta = 0;
    int lcount = 0;
    uint32_t n_steps = 0, n_lay = 0, n_up = 0, n_spill = 0, n_refill = 0, n_slow = 0, n_evict = 0, n_hbm = 0;
    const unsigned long long probes0 = my_probes;

    // layer-table window: lane j holds lay[tb0 + j]
    uint32_t tb0 = 0, drq = 0, dhi = 0;
    auto load_lay = [&](uint32_t base) {
        DFS_STAT(n_lay++);
        tb0 = base;
        const uint32_t u = base + (uint32_t)lane;
        if (u < n_ok) { const Lay e = lay[u]; drq = e.rq; dhi = e.hi; }
    };
    auto lay_hi = [&](uint32_t u) -> uint32_t {
        if (u - tb0 >= 64u) load_lay(u >= 32 ? u - 32 : 0);
        return (uint32_t)readlane((int)dhi, (int)(u - tb0));
    };
    // next-ops window: lane j holds ops[pb + j]
    int pb = 0;
    uint32_t urq = RQ_EMPTY;
    auto load_up = [&](int base) {
        DFS_STAT(n_up++);
        pb = base;
        const int j = base + lane;
        urq = j < n_ops ? ops[j].rq : RQ_EMPTY;
    };
    // DFS stack: frames [ring_lo, depth) in lane registers, lane = index mod 64
    uint32_t fm_lo = 0, fm_hi = 0, f_ti = 0, f_s = 0, fr_lo = 0, fr_hi = 0;

    load_lay(0);
    uint32_t t = 0, tmax = 0, depth = 0, ring_lo = 0;
    uint64_t mask = 0;
    uint32_t s = (uint32_t)A.init_state;
    int verdict = -1;
    uint32_t ins = 0;
    uint32_t budget = (uint32_t)min<int64_t>(A.budget, 0x7FFFFFFF);
    uint32_t chk = min(budget, 1023u);               // next insert count that needs a check
    int w = (int)(lay_hi(0) >> 6), P = w;
    uint32_t r = lay_hi(0) & 63;                       // position of RET[t] in W(t)
    uint32_t rn = n_ok > 1 ? (lay_hi(1) & 63) : 0;     // position of RET[t+1] in W(t+1)
    uint32_t wrq = lane < w ? ops[lane].rq : RQ_EMPTY;
    load_up(P);
    wave_sync();
    uint32_t ins_saved = 0xFFFFFFFFu;     // a handed-over search's real insert count
    uint32_t nlog = 0;                    // hlog entries (saturating at 0xFFFF)
    bool ho = false;                      // a late helper takes this search over (A.handoff)
    unsigned long long ho_off = 0;        // its record's place, reserved when the request is accepted
    // move the window forward from layer t to layer nt (a lift, or a resume)
    auto advance = [&](uint32_t nt) {
        for (uint32_t u = t; u < nt; u++) {
            const uint32_t ru = u == t ? r : (lay_hi(u) & 63);
            const uint32_t sh = (uint32_t)wave_shl1((int)wrq);
            if (lane >= (int)ru) wrq = sh;
            w--;
            if (lane == w) wrq = RQ_EMPTY;
            const int c = (int)(lay_hi(u + 1) >> 6);
            if (c > 0) {
                if (P < pb || P + c > pb + 64) load_up(c <= 32 && P >= 32 ? P - 32 : P);
                for (int kk = 0; kk < c; kk++) {
                    const uint32_t x = (uint32_t)readlane((int)urq, P - pb + kk);
                    if (lane == w + kk) wrq = x;
                }
                w += c; P += c;
            }
        }
    };
    if (A.rs_mode == 2 && A.rs_off) {
        // Resume a search phase 1 deferred (round 5): its memo into this wave's
        // HBM table behind the Bloom filter (theta above every restored layer,
        // so each probe there is exact), its stack into the ring and the HBM
        // stack, then expand its current configuration again: the children it
        // had inserted are present, the others absent -- the DFS goes on
        // exactly where phase 1 stopped it.
        const int64_t ro = A.rs_off[key];
        if (ro >= 0) {
            const uint64_t *hd = (const uint64_t *)(A.rs_arena + ro);
            const uint64_t h_mask = hd[0], h_ts = hd[1], h_dt = hd[2], h_ins = hd[3], h_n = hd[4];
            const uint32_t d = (uint32_t)h_dt;
            if (d <= A.stack_cap && h_n <= (uint64_t)A.memo_cap / 4) {
                const Frame *fsrc = (const Frame *)(hd + 8);
                const ulonglong2 *ent = (const ulonglong2 *)(fsrc + d);
                uint32_t tmx = 0;
                for (uint32_t j = (uint32_t)lane; j < (uint32_t)h_n; j += 64) {
                    const ulonglong2 e = ent[j];
                    const uint32_t et = (uint32_t)(e.y >> 20) & T_MASK, es = (uint32_t)e.y & STATE_MASK;
                    const uint32_t sl = hbm_insert(memo, cap_mask, gen, et, es, e.x);
                    // (a takeover's save gathers the restored entries too)
                    if constexpr (HO) { if (hlog && j < A.hlog_cap) hlog[j] = sl; } else (void)sl;
                    uint32_t g1, g2;
                    lk_hash((uint32_t)e.x, (uint32_t)(e.x >> 32) | (et << 16) | (es << 8) | 0x80000000u, g1, g2);
                    bloom_set2<M>(bloom, lk_bl(g1), lk_bl(g2));
                    tmx = max(tmx, et + 1);
                }
                for (int o = 32; o > 0; o >>= 1) tmx = max(tmx, (uint32_t)__shfl_xor((int)tmx, o));
                theta = rflu(tmx);
                if constexpr (HO) nlog = (uint32_t)min<uint64_t>(h_n, 0xFFFFu);
                ring_lo = d > 32 ? d - 32 : 0;
                for (uint32_t j = (uint32_t)lane; j < ring_lo; j += 64) stack[j] = fsrc[j];
                {
                    const uint32_t idx = ring_lo + (((uint32_t)lane - ring_lo) & 63);
                    if (idx < d) {
                        const Frame fr = fsrc[idx];
                        fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i;
                        f_s = (uint32_t)fr.s; fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                wave_sync();
                depth = d;
                mask = h_mask;
                s = (uint32_t)(h_ts >> 32);
                ins = (uint32_t)h_ins;
                chk = min(budget, ins);                  // the next insert runs the checks
                const uint32_t nt = (uint32_t)h_ts;
                advance(nt);
                t = nt;
                tmax = max((uint32_t)(h_dt >> 32), t);
                r = lay_hi(t) & 63;
                rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
            }
        }
    }
    const ulonglong2 *B = (const ulonglong2 *)lmemo;
    // per-step values shared by the two ways into an insert
    uint64_t absent = 0, nm_r = 0;
    uint32_t u_r = 0, klo = 0, khi = 0, b1 = 0, b2 = 0, n1 = 0, n2 = 0, h1 = 0, h2 = 0, nvl = 0;
    // the RET child of the current configuration (lifted) and the child keys of all lanes
    auto child_keys = [&]() {
        u_r = t; nm_r = 0;
        if ((absent >> r) & 1) {
            // lift RET[t]: drop its bit, then keep lifting while the next
            // layer's RET op is already linearized (rarely more than once)
            uint64_t nm = drop_bit(mask, r);
            uint32_t u = t + 1;
            if (u >= n_ok) nm = 0;
            else if ((nm >> rn) & 1) {
                uint32_t ru = rn;
                for (;;) {
                    nm = drop_bit(nm, ru);
                    u++;
                    if (u >= n_ok) { nm = 0; break; }
                    ru = lay_hi(u) & 63;
                    if (!((nm >> ru) & 1)) break;
                }
            }
            u_r = u; nm_r = nm;
        }
        // child keys 1:1|t:15|state:8|mask:40, all lanes at once
        nvl = wrq >> 16;
        const bool is_r = lane == (int)r;
        const uint32_t hi_a = (uint32_t)(mask >> 32) | (t << 16) | 0x80000000u;
        const uint32_t hi_r = (uint32_t)(nm_r >> 32) | (u_r << 16) | 0x80000000u;
        klo = is_r ? (uint32_t)nm_r : ((uint32_t)mask | lb_lo);
        khi = (is_r ? hi_r : (hi_a | lb_hi)) | (nvl << 8);
        lk_hash(klo, khi, h1, h2);
        lk_bkts<M>(h1, h2, b1, b2);
    };

expand:
    // a configuration entered by a push: probe every candidate child
    DFS_STAT(n_steps++);
    {
        const uint32_t req = wrq & 0xFFFF;
        absent = (ballot(req == s) | ballot(req == RQ_ANY)) & ~mask;
    }
    if (!absent) goto pop;
    child_keys();
    {
        // one LDS round trip; non-candidate lanes all read bucket 0 (broadcast)
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        const uint64_t k = ((uint64_t)khi << 32) | klo;
        // the fill counts first, in the same LDS round trip as the slots
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
        __builtin_amdgcn_sched_barrier(0);
        const ulonglong2 x0 = B[2 * a1], x1 = B[2 * a1 + 1];
        const ulonglong2 y0 = B[2 * a2], y1 = B[2 * a2 + 1];
        const uint64_t hit = ballot(x0.x == k) | ballot(x0.y == k) | ballot(x1.x == k) | ballot(x1.y == k) |
                             ballot(y0.x == k) | ballot(y0.y == k) | ballot(y1.x == k) | ballot(y1.y == k);
        absent &= ~hit;
        if (t < theta && absent) {
            DFS_STAT(n_slow++);
            // children below theta may sit in HBM: Bloom, then HBM for every
            // Bloom-positive lane (all at once), so that absent is exact: the
            // frame's rest relies on it
            uint64_t low = absent;
            if (u_r >= theta) low &= ~(1ULL << r);
            const uint32_t kt = khi >> 16 & 0x7FFF, ks = (khi >> 8) & 0xFF;
            const uint64_t km = k & ((1ULL << 40) - 1);
            const bool maybe = ((low >> lane) & 1) && bloom_test2<M>(bloom, lk_bl(h1), lk_bl(h2));
            bool found = false;
            if (maybe) found = (hbm_probe(memo, cap_mask, gen, kt, ks, km, my_probes) >> 32) == 0;
            absent &= ~ballot(found);
        }
    }
    if (!absent) goto pop;

insert:
    {
        if (ins >= chk) {
            if (ins >= budget && !extend_budget(A, budget)) { verdict = JH_UNKNOWN; goto done; }
            if (handover(A, ins)) { ins_saved = ins; ins = budget; verdict = JH_UNKNOWN; goto done; }
            if (A.claim) {
                // racing k_lin_bfs: stop if it settled this key first
                int c = 0;
                if (lane == 0) c = __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (readlane(c, 0)) { verdict = JH_CANCELLED; goto done; }
            }
            if (A.prio_ins > 0 && ins >= (uint32_t)A.prio_ins) {
                if (ins >= 4u * (uint32_t)A.prio_ins) __builtin_amdgcn_s_setprio(3);
                else if (ins >= 2u * (uint32_t)A.prio_ins) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(1);
            }
            if (HO && A.handoff) {
                // round 6: a late helper asks for this search (the takeover);
                // saved only if the slot log holds every HBM entry of the key
                int h = 0;
                if (lane == 0) h = __hip_atomic_load(&A.handoff[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (readlane(h, 0) == HO_ASK) {
                    // accepted only if the save cannot fail: the slot log holds
                    // every HBM entry, the record fits this wave's table when the
                    // search continues from it, and its arena space is reserved
                    // now (a failed save would leave the table holding entries
                    // the record lacks)
                    bool ok = hlog && nlog <= A.hlog_cap && ins <= A.memo_cap / 4;
                    if (ok) {
                        const uint64_t bytes = 64 + (uint64_t)depth * sizeof(Frame) + (uint64_t)ins * 16;
                        unsigned long long off = 0;
                        if (lane == 0) off = atomicAdd(A.rs_used, (unsigned long long)((bytes + 255) & ~255ULL));
                        ho_off = readlane64(off, 0);
                        ok = ho_off + bytes <= A.rs_cap;
                    }
                    int won = 0;
                    if (lane == 0) {
                        int exp = HO_ASK;
                        won = __hip_atomic_compare_exchange_strong(&A.handoff[key], &exp, ok ? HO_SAVING : HO_REFUSED,
                                                                   __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT) ? 1 : 0;
                    }
                    // saved in done:, then the caller continues this search from
                    // the same record (V_HANDED): it races the helper that
                    // continues its copy (measured: leaving the key to the
                    // helper was slower). A restart from the record rather than a
                    // jump back here keeps the search loop's registers its own.
                    if (readlane(won, 0) && ok) { ho = true; goto done; }
                }
            }
            chk = min(budget, ins + (HO && A.handoff ? 256u : 1024u));
        }
        const int i = __builtin_ctzll(absent);
        ins++;
        const uint32_t ns = (uint32_t)readlane((int)nvl, i);
        const bool to_r = (uint32_t)i == r;
        const uint32_t nt = to_r ? u_r : t;
        {
            // into the emptier of the child's two buckets
            const bool pick1 = n1 <= n2;
            const uint32_t bs = pick1 ? b1 : b2, nsl = pick1 ? n1 : n2;
            const uint64_t full_m = ballot(nsl >= 4);
            if (!((full_m >> i) & 1)) {
                if (lane == i) {
                    lmemo[4 * bs + nsl] = ((uint64_t)khi << 32) | klo;
                    bcnt8[bs] = (uint8_t)(nsl + 1);
                }
                if (++lcount >= M::EVICT) {
                    DFS_STAT(n_evict++);
                    const uint64_t er = memo_evict<M>(lmemo, bcnt, bloom, memo, stage, cap_mask, gen, nt, theta, lane,
                                                      hlog, A.hlog_cap, nlog);
                    DFS_STAT(n_hbm += (uint32_t)lcount - ((uint32_t)er & 0xFFFF));
                    lcount = rfl((int)((uint32_t)er & 0xFFFF));
                    nlog = rflu(((uint32_t)er >> 16) & 0xFFFF);
                    theta = rflu((uint32_t)(er >> 32));
                }
            } else {
                // both buckets full: HBM, and theta rises above the layer
                const uint64_t nmask = to_r ? nm_r : (mask | (1ULL << i));
                if (lane == i) {
                    const uint32_t sl = hbm_insert(memo, cap_mask, gen, nt, ns, nmask);
                    bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
                    if (hlog && nlog < A.hlog_cap) hlog[nlog] = sl;
                }
                nlog = min(nlog + 1, 0xFFFFu);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                theta = max(theta, nt + 1);
                DFS_STAT(n_hbm++);
            }
        }
        // push the parent; a full ring spills its oldest half to HBM
        if (depth - ring_lo == 64) {
            DFS_STAT(n_spill++);
            const uint32_t kk = ((uint32_t)lane - ring_lo) & 63;
            if (kk < 32) {
                Frame fr;
                fr.mask = ((uint64_t)fm_hi << 32) | fm_lo; fr.t_i = f_ti; fr.s = (int32_t)f_s;
                fr.rest = ((uint64_t)fr_hi << 32) | fr_lo; fr.pad[0] = fr.pad[1] = 0;
                stack[ring_lo + kk] = fr;
            }
            ring_lo += 32;
        }
        {
            const uint64_t nrest = absent & (absent - 1);
            const bool me = lane == (int)(depth & 63);
            fm_lo = me ? (uint32_t)mask : fm_lo;
            fm_hi = me ? (uint32_t)(mask >> 32) : fm_hi;
            f_ti = me ? ((t << 6) | (uint32_t)i) : f_ti;
            f_s = me ? s : f_s;
            fr_lo = me ? (uint32_t)nrest : fr_lo;
            fr_hi = me ? (uint32_t)(nrest >> 32) : fr_hi;
        }
        depth++;
        s = ns;
        if (!to_r) {
            mask |= 1ULL << i;
            goto expand;
        }
        mask = nm_r;
        if (nt >= n_ok) { t = nt; tmax = max(tmax, t); verdict = JH_VALID; goto done; }
        // move the window forward layer by layer
        advance(nt);
        t = nt;
        if (t > tmax) {
            tmax = t;
            if (A.stamp_progress && A.seq_start && lane == 0)
                __hip_atomic_store(&A.seq_start[key], __builtin_amdgcn_s_memrealtime() | 1ULL, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        r = lay_hi(t) & 63;
        rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        goto expand;
    }

pop:
    DFS_STAT(n_steps++);
    if (depth == ring_lo) {
        if (depth == 0) { verdict = JH_INVALID; goto done; }
        // ring empty: refill up to 32 frames below from the HBM stack
        DFS_STAT(n_refill++);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t lo = depth >= 32 ? depth - 32 : 0;
        const uint32_t kk = ((uint32_t)lane - lo) & 63;
        if (kk < depth - lo) {
            const Frame fr = stack[lo + kk];
            fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i; f_s = (uint32_t)fr.s;
            fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32);
        }
        ring_lo = lo;
    }
    depth--;
    {
        const int ln = (int)(depth & 63);
        absent = ((uint64_t)(uint32_t)readlane((int)fr_hi, ln) << 32) | (uint32_t)readlane((int)fr_lo, ln);
        const uint32_t pt = (uint32_t)readlane((int)f_ti, ln) >> 6;
        mask = ((uint64_t)(uint32_t)readlane((int)fm_hi, ln) << 32) | (uint32_t)readlane((int)fm_lo, ln);
        s = (uint32_t)readlane((int)f_s, ln);
        if (pt != t) {
            // move the window back: drop appended ops, re-insert RETs
            for (uint32_t u = t; u > pt; u--) {
                const int c = (int)(lay_hi(u) >> 6);
                w -= c; P -= c;
                if (lane >= w) wrq = RQ_EMPTY;
                const uint32_t h = lay_hi(u - 1);
                const int ru = (int)(h & 63);
                const uint32_t sh = (uint32_t)wave_shr1((int)wrq);
                if (lane > ru) wrq = sh;
                const uint32_t x = (uint32_t)readlane((int)drq, (int)(u - 1 - tb0));
                if (lane == ru) wrq = x;
                w++;
            }
            t = pt;
            r = lay_hi(t) & 63;
            rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        }
    }
    // every child in rest is absent (see above): only its bucket fill counts are needed
    if (!absent) goto pop;
    child_keys();
    {
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
    }
    goto insert;

done:
    if ((A.rs_mode == 1 && A.rs_off && verdict == JH_UNKNOWN && A.defer) || (HO && ho)) {
        // Save the deferred search for phase 2 (round 5): header {mask, t | s << 32,
        // depth | tmax << 32, inserts, entries}, the stack frames, then every
        // configuration in the memo as {mask, t << 20 | s}: the LDS ones and this
        // key's generation in the wave's HBM table (scanned whole, 16 entries in
        // flight per lane). Published only if the count is the insert count.
        const uint32_t nmem = ins_saved != 0xFFFFFFFFu ? ins_saved : ins;
        const uint64_t bytes = 64 + (uint64_t)depth * sizeof(Frame) + (uint64_t)nmem * 16;
        unsigned long long off = 0;
        if (HO && ho) off = ho_off;
        else {
            if (lane == 0) off = atomicAdd(A.rs_used, (unsigned long long)((bytes + 255) & ~255ULL));
            off = readlane64(off, 0);
        }
        if (off + bytes <= A.rs_cap) {
            uint64_t *hd = (uint64_t *)(A.rs_arena + off);
            Frame *fdst = (Frame *)(hd + 8);
            ulonglong2 *ent = (ulonglong2 *)(fdst + depth);
            for (uint32_t j = (uint32_t)lane; j < ring_lo; j += 64) fdst[j] = stack[j];
            {
                const uint32_t idx = ring_lo + (((uint32_t)lane - ring_lo) & 63);
                if (idx < depth) {
                    Frame fr;
                    fr.mask = ((uint64_t)fm_hi << 32) | fm_lo; fr.t_i = f_ti; fr.s = (int32_t)f_s;
                    fr.rest = ((uint64_t)fr_hi << 32) | fr_lo; fr.pad[0] = fr.pad[1] = 0;
                    fdst[idx] = fr;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint32_t n = 0;
            for (int base = 0; base < M::SLOTS; base += 64) {
                const uint64_t x = lmemo[base + lane];
                const uint64_t bm = ballot(x != 0);
                const uint32_t at = n + (uint32_t)mbcnt(bm);
                if (x != 0 && at < nmem) ent[at] = make_ulonglong2(lk_m(x), ((uint64_t)lk_t(x) << 20) | lk_s(x));
                n += (uint32_t)__popcll(bm);
            }
            const ulonglong2 *tab = (const ulonglong2 *)memo;
            if (hlog && nlog <= A.hlog_cap) {
                // the logged slots: this key's entries only (8 gathers in flight per lane)
                for (uint32_t base = 0; base < nlog; base += 64 * 8) {
                    ulonglong2 e[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const uint32_t j = base + 64 * q + (uint32_t)lane;
                        e[q] = j < nlog ? tab[hlog[j]] : make_ulonglong2(0ULL, 0ULL);
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const bool mine = base + 64 * q + (uint32_t)lane < nlog && (uint32_t)(e[q].y >> 40) == gen;
                        const uint64_t bm = ballot(mine);
                        const uint32_t at = n + (uint32_t)mbcnt(bm);
                        if (mine && at < nmem) ent[at] = make_ulonglong2(e[q].x, e[q].y & ((1ULL << 40) - 1));
                        n += (uint32_t)__popcll(bm);
                    }
                }
            } else
            for (uint32_t base = 0; base < A.memo_cap; base += 64 * 16) {
                ulonglong2 e[16];
#pragma unroll
                for (int q = 0; q < 16; q++) e[q] = tab[base + 64 * q + lane];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    const bool mine = (uint32_t)(e[q].y >> 40) == gen;
                    const uint64_t bm = ballot(mine);
                    const uint32_t at = n + (uint32_t)mbcnt(bm);
                    if (mine && at < nmem) ent[at] = make_ulonglong2(e[q].x, e[q].y & ((1ULL << 40) - 1));
                    n += (uint32_t)__popcll(bm);
                }
            }
            if (lane == 0) {
                hd[0] = mask; hd[1] = (uint64_t)t | ((uint64_t)s << 32); hd[2] = (uint64_t)depth | ((uint64_t)tmax << 32);
                hd[3] = nmem; hd[4] = n;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (lane == 0 && n == nmem) {
                A.rs_off[key] = (int64_t)off;
                // Q_RS_N: records published; [91]: takeovers (round 6)
                atomicAdd((int32_t *)A.rs_used + (ho ? 3 : 2), 1);
            }
            if (ho && lane == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_store(&A.handoff[key], n == nmem ? HO_DONE : HO_REFUSED, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            // (never expected: a save whose gather missed an entry leaves the
            // key to the helper, which restarts it -- this wave's table would
            // hold entries the record lacks)
            if (HO && ho && n != nmem) { ins = 0; verdict = JH_CANCELLED; ho = false; }
        } else if (ho) {
            // (not reached: the space was reserved at the request) the helper
            // restarts the key and this wave leaves it
            if (lane == 0) __hip_atomic_store(&A.handoff[key], HO_REFUSED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            verdict = JH_CANCELLED; ho = false;
        }
    }
    if (HO && ho) return V_HANDED;      // (published: HO_DONE, or HO_REFUSED)
    inserts = ins;
    ins_real = ins_saved != 0xFFFFFFFFu ? ins_saved : ins;    // a handed-over search's own count
    tmax_out = tmax;
#ifdef JH_DFS_STATS
    if (A.dbg && lane == 0) {
        unsigned long long *d = A.dbg + 16 * (size_t)blockIdx.x;
        d[4] += n_steps; d[5] += ins; d[6] += n_evict; d[7] += n_lay; d[10] += n_up;
        d[11] += n_spill; d[12] += n_refill; d[13] += n_slow; d[14] += my_probes - probes0; d[8] += n_hbm;
    }
#endif
    return verdict;
}

// ---------------------------------------------------------------------------
// WIDE keys (windows of 41-64 members, or >= 256 states) with an LDS memo:
// dfs_lean's search with 16-byte LDS entries {mask:64, 1|t:15|state:16}.
// Round 2 searched these keys with every configuration in the HBM table
// behind a Bloom filter (dfs_search), one HBM round trip per step once the
// filter saturates (C5's deep searches); the layered LDS memo keeps the
// layers near the current one on chip exactly as for LEAN keys (theta: below
// it, entries may sit in HBM; at or above it, the LDS is exact), so most
// steps of a deep search probe LDS only.
__device__ __forceinline__ uint32_t w_t(uint64_t y) { return (uint32_t)(y >> 16) & 0x7FFF; }
__device__ __forceinline__ uint32_t w_s(uint64_t y) { return (uint32_t)y & 0xFFFF; }
__device__ __forceinline__ void w_hash(uint64_t m, uint32_t y, uint32_t &h1, uint32_t &h2) {
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    h1 = (lo ^ __builtin_rotateleft32(hi, 16) ^ __builtin_rotateleft32(y, 8)) * 0x9E3779B1u;
    h2 = (lo + __builtin_rotateleft32(hi, 5) + __builtin_rotateleft32(y, 11)) * 0x85EBCA77u;
}

// dfs_lean's eviction for 16-byte entries (stage: SLOTS x 16 B of global scratch)
template <class M>
__device__ __noinline__ uint64_t memo_evict_w(ulonglong2 *lmemo, uint32_t *bcnt, uint32_t *bloom, uint64_t *memo,
                                              ulonglong2 *stage, uint32_t cap_mask, uint32_t gen, uint32_t t_cur,
                                              uint32_t theta_old, int lane) {
    int bins = 0;
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) {
        const ulonglong2 x = lmemo[lane + 64 * r];
        stage[lane + 64 * r] = x;
        const uint32_t xt = w_t(x.y);
        const int d = x.y == 0 ? 99 : (xt >= t_cur ? 0 : (int)min(t_cur - xt, 15u));
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const int cnt = __popcll(ballot(d == b));
            if (lane == b) bins += cnt;
        }
    }
    int acc = 0, dstar = -1;
#pragma unroll 1
    for (int b = 0; b < 16; b++) {
        acc += readlane(bins, b);
        if (acc > M::EVICT / 2) break;
        dstar = b;
    }
    uint32_t th2;
    if (dstar < 0) th2 = t_cur + 1;
    else {
        th2 = t_cur > (uint32_t)dstar ? t_cur - (uint32_t)dstar : 0u;
        if (dstar == 15) th2 = t_cur - min(t_cur, 15u);
    }
    th2 = max(th2, theta_old);
    wave_sync();
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) lmemo[lane + 64 * r] = make_ulonglong2(0, 0);
    for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    wave_sync();
    int kept = 0;
    uint32_t th_min = 0;
#pragma unroll 1
    for (int r = 0; r < M::SLOTS / 64; r++) {
        const ulonglong2 x = stage[lane + 64 * r];
        if (x.y == 0) continue;
        const uint32_t xt = w_t(x.y);
        bool to_hbm = xt < th2;
        uint32_t h1, h2;
        w_hash(x.x, (uint32_t)x.y, h1, h2);
        if (!to_hbm) {
            const uint32_t b1 = h1 >> (32 - M::LG), b2 = h2 >> (32 - M::LG);
            bool placed = false;
            for (int j = 0; j < 2 && !placed; j++) {
                const uint32_t b = j ? b2 : b1;
                const uint32_t sh = 8 * (b & 3);
                const uint32_t old = (atomicAdd(&bcnt[b >> 2], 1u << sh) >> sh) & 0xFF;
                if (old < 4) { lmemo[4 * b + old] = x; placed = true; }
                else atomicSub(&bcnt[b >> 2], 1u << sh);
            }
            if (placed) kept++;
            else { to_hbm = true; th_min = max(th_min, xt + 1); }
        }
        if (to_hbm) {
            hbm_insert(memo, cap_mask, gen, xt, w_s(x.y), x.x);
            bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        kept += __shfl_xor(kept, o);
        th_min = max(th_min, (uint32_t)__shfl_xor((int)th_min, o));
    }
    th2 = max(th2, th_min);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    wave_sync();
    return ((uint64_t)th2 << 32) | (uint32_t)kept;
}

// dfs_lean for WIDE keys: the same state machine (expand / insert / pop), the
// same search order and memo contents (explored counts equal WGL's), 16-byte
// LDS keys. M::SLOTS 16-byte slots; M::LDS counts them as 8 bytes, so the
// kernels pass MemoW16<M>::LDS.
template <class M>
__device__ __forceinline__ int dfs_lean_w(const DfsArgs &A, const KeyInfo &K, const char *tb, int key, int lane,
                                          uint64_t *memo, Frame *stack, uint64_t *stage64,
                                          long long &inserts, uint32_t &tmax_out, unsigned long long &my_probes) {
    const OpC *ops = (const OpC *)tb;
    const Lay *lay = (const Lay *)(tb + tblc_ops_bytes(K));
    const uint32_t n_ok = (uint32_t)K.n_ok;
    const int n_ops = K.n_ops;
    const uint32_t cap_mask = A.memo_cap - 1;
    const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
    constexpr int OFF_BLOOM = LDS_TBL + M::SLOTS * 16, OFF_CNT = OFF_BLOOM + M::BLOOM / 8;
    ulonglong2 *lmemo = (ulonglong2 *)(jh_lds + LDS_TBL);
    uint32_t *bloom = (uint32_t *)(jh_lds + OFF_BLOOM);
    uint32_t *bcnt = (uint32_t *)(jh_lds + OFF_CNT);
    uint8_t *bcnt8 = (uint8_t *)bcnt;
    ulonglong2 *stage = (ulonglong2 *)stage64;
    for (int i = lane; i < M::SLOTS; i += 64) lmemo[i] = make_ulonglong2(0, 0);
    for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    for (int i = lane; i < M::BLOOM / 32; i += 64) bloom[i] = 0;
    uint32_t theta = 0;
    int lcount = 0;

    uint32_t tb0 = 0, drq = 0, dhi = 0;
    auto load_lay = [&](uint32_t base) {
        tb0 = base;
        const uint32_t u = base + (uint32_t)lane;
        if (u < n_ok) { const Lay e = lay[u]; drq = e.rq; dhi = e.hi; }
    };
    auto lay_hi = [&](uint32_t u) -> uint32_t {
        if (u - tb0 >= 64u) load_lay(u >= 32 ? u - 32 : 0);
        return (uint32_t)readlane((int)dhi, (int)(u - tb0));
    };
    int pb = 0;
    uint32_t urq = RQ_EMPTY;
    auto load_up = [&](int base) {
        pb = base;
        const int j = base + lane;
        urq = j < n_ops ? ops[j].rq : RQ_EMPTY;
    };
    uint32_t fm_lo = 0, fm_hi = 0, f_ti = 0, f_s = 0, fr_lo = 0, fr_hi = 0;

    load_lay(0);
    uint32_t t = 0, tmax = 0, depth = 0, ring_lo = 0;
    uint64_t mask = 0;
    uint32_t s = (uint32_t)A.init_state;
    int verdict = -1;
    uint32_t ins = 0;
    uint32_t budget = (uint32_t)min<int64_t>(A.budget, 0x7FFFFFFF);
    uint32_t chk = min(budget, 1023u);
    int w = (int)(lay_hi(0) >> 6), P = w;
    uint32_t r = lay_hi(0) & 63;
    uint32_t rn = n_ok > 1 ? (lay_hi(1) & 63) : 0;
    uint32_t wrq = lane < w ? ops[lane].rq : RQ_EMPTY;
    load_up(P);
    wave_sync();
    uint64_t absent = 0, nm_r = 0, km = 0;
    uint32_t u_r = 0, ky = 0, b1 = 0, b2 = 0, n1 = 0, n2 = 0, h1 = 0, h2 = 0, nvl = 0;
    auto child_keys = [&]() {
        u_r = t; nm_r = 0;
        if ((absent >> r) & 1) {
            uint64_t nm = drop_bit(mask, r);
            uint32_t u = t + 1;
            if (u >= n_ok) nm = 0;
            else if ((nm >> rn) & 1) {
                uint32_t ru = rn;
                for (;;) {
                    nm = drop_bit(nm, ru);
                    u++;
                    if (u >= n_ok) { nm = 0; break; }
                    ru = lay_hi(u) & 63;
                    if (!((nm >> ru) & 1)) break;
                }
            }
            u_r = u; nm_r = nm;
        }
        nvl = wrq >> 16;
        const bool is_r = lane == (int)r;
        km = is_r ? nm_r : (mask | (1ULL << lane));
        ky = 0x80000000u | ((is_r ? u_r : t) << 16) | nvl;
        w_hash(km, ky, h1, h2);
        b1 = h1 >> (32 - M::LG);
        b2 = h2 >> (32 - M::LG);
    };

expand:
    {
        const uint32_t req = wrq & 0xFFFF;
        absent = (ballot(req == s) | ballot(req == RQ_ANY)) & ~mask;
    }
    if (!absent) goto pop;
    child_keys();
    {
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
        __builtin_amdgcn_sched_barrier(0);
        const ulonglong2 x0 = lmemo[4 * a1], x1 = lmemo[4 * a1 + 1], x2 = lmemo[4 * a1 + 2], x3 = lmemo[4 * a1 + 3];
        const ulonglong2 y0 = lmemo[4 * a2], y1 = lmemo[4 * a2 + 1], y2 = lmemo[4 * a2 + 2], y3 = lmemo[4 * a2 + 3];
        const uint64_t kyy = ky;
        const bool hit = (x0.x == km && x0.y == kyy) | (x1.x == km && x1.y == kyy) | (x2.x == km && x2.y == kyy) |
                         (x3.x == km && x3.y == kyy) | (y0.x == km && y0.y == kyy) | (y1.x == km && y1.y == kyy) |
                         (y2.x == km && y2.y == kyy) | (y3.x == km && y3.y == kyy);
        absent &= ~ballot(hit);
        if (t < theta && absent) {
            uint64_t low = absent;
            if (u_r >= theta) low &= ~(1ULL << r);
            const bool maybe = ((low >> lane) & 1) && bloom_test2<M>(bloom, lk_bl(h1), lk_bl(h2));
            bool found = false;
            if (maybe) found = (hbm_probe(memo, cap_mask, gen, w_t(ky), w_s(ky), km, my_probes) >> 32) == 0;
            absent &= ~ballot(found);
        }
    }
    if (!absent) goto pop;

insert:
    {
        if (ins >= chk) {
            if (ins >= budget && !extend_budget(A, budget)) { verdict = JH_UNKNOWN; goto done; }
            if (handover(A, ins)) { ins = budget; verdict = JH_UNKNOWN; goto done; }
            if (A.claim) {
                int c = 0;
                if (lane == 0) c = __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (readlane(c, 0)) { verdict = JH_CANCELLED; goto done; }
            }
            chk = min(budget, ins + 1024);
        }
        const int i = __builtin_ctzll(absent);
        ins++;
        const uint32_t ns = (uint32_t)readlane((int)nvl, i);
        const bool to_r = (uint32_t)i == r;
        const uint32_t nt = to_r ? u_r : t;
        {
            const bool pick1 = n1 <= n2;
            const uint32_t bs = pick1 ? b1 : b2, nsl = pick1 ? n1 : n2;
            const uint64_t full_m = ballot(nsl >= 4);
            if (!((full_m >> i) & 1)) {
                if (lane == i) {
                    lmemo[4 * bs + nsl] = make_ulonglong2(km, (uint64_t)ky);
                    bcnt8[bs] = (uint8_t)(nsl + 1);
                }
                if (++lcount >= M::EVICT) {
                    const uint64_t er = memo_evict_w<M>(lmemo, bcnt, bloom, memo, stage, cap_mask, gen, nt, theta, lane);
                    lcount = rfl((int)(uint32_t)er);
                    theta = rflu((uint32_t)(er >> 32));
                }
            } else {
                const uint64_t nmask = to_r ? nm_r : (mask | (1ULL << i));
                if (lane == i) {
                    hbm_insert(memo, cap_mask, gen, nt, ns, nmask);
                    bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
                }
                theta = max(theta, nt + 1);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
        }
        if (depth - ring_lo == 64) {
            const uint32_t kk = ((uint32_t)lane - ring_lo) & 63;
            if (kk < 32) {
                Frame fr;
                fr.mask = ((uint64_t)fm_hi << 32) | fm_lo; fr.t_i = f_ti; fr.s = (int32_t)f_s;
                fr.rest = ((uint64_t)fr_hi << 32) | fr_lo; fr.pad[0] = fr.pad[1] = 0;
                stack[ring_lo + kk] = fr;
            }
            ring_lo += 32;
        }
        {
            const uint64_t nrest = absent & (absent - 1);
            const bool me = lane == (int)(depth & 63);
            fm_lo = me ? (uint32_t)mask : fm_lo;
            fm_hi = me ? (uint32_t)(mask >> 32) : fm_hi;
            f_ti = me ? ((t << 6) | (uint32_t)i) : f_ti;
            f_s = me ? s : f_s;
            fr_lo = me ? (uint32_t)nrest : fr_lo;
            fr_hi = me ? (uint32_t)(nrest >> 32) : fr_hi;
        }
        depth++;
        s = ns;
        if (!to_r) {
            mask |= 1ULL << i;
            goto expand;
        }
        mask = nm_r;
        if (nt >= n_ok) { t = nt; tmax = max(tmax, t); verdict = JH_VALID; goto done; }
        for (uint32_t u = t; u < nt; u++) {
            const uint32_t ru = u == t ? r : (lay_hi(u) & 63);
            const uint32_t sh = (uint32_t)wave_shl1((int)wrq);
            if (lane >= (int)ru) wrq = sh;
            w--;
            if (lane == w) wrq = RQ_EMPTY;
            const int c = (int)(lay_hi(u + 1) >> 6);
            if (c > 0) {
                if (P < pb || P + c > pb + 64) load_up(c <= 32 && P >= 32 ? P - 32 : P);
                for (int kk = 0; kk < c; kk++) {
                    const uint32_t x = (uint32_t)readlane((int)urq, P - pb + kk);
                    if (lane == w + kk) wrq = x;
                }
                w += c; P += c;
            }
        }
        t = nt;
        tmax = max(tmax, t);
        r = lay_hi(t) & 63;
        rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        goto expand;
    }

pop:
    if (depth == ring_lo) {
        if (depth == 0) { verdict = JH_INVALID; goto done; }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t lo = depth >= 32 ? depth - 32 : 0;
        const uint32_t kk = ((uint32_t)lane - lo) & 63;
        if (kk < depth - lo) {
            const Frame fr = stack[lo + kk];
            fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i; f_s = (uint32_t)fr.s;
            fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32);
        }
        ring_lo = lo;
    }
    depth--;
    {
        const int ln = (int)(depth & 63);
        absent = ((uint64_t)(uint32_t)readlane((int)fr_hi, ln) << 32) | (uint32_t)readlane((int)fr_lo, ln);
        const uint32_t pt = (uint32_t)readlane((int)f_ti, ln) >> 6;
        mask = ((uint64_t)(uint32_t)readlane((int)fm_hi, ln) << 32) | (uint32_t)readlane((int)fm_lo, ln);
        s = (uint32_t)readlane((int)f_s, ln);
        if (pt != t) {
            for (uint32_t u = t; u > pt; u--) {
                const int c = (int)(lay_hi(u) >> 6);
                w -= c; P -= c;
                if (lane >= w) wrq = RQ_EMPTY;
                const uint32_t h = lay_hi(u - 1);
                const int ru = (int)(h & 63);
                const uint32_t sh = (uint32_t)wave_shr1((int)wrq);
                if (lane > ru) wrq = sh;
                const uint32_t x = (uint32_t)readlane((int)drq, (int)(u - 1 - tb0));
                if (lane == ru) wrq = x;
                w++;
            }
            t = pt;
            r = lay_hi(t) & 63;
            rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        }
    }
    if (!absent) goto pop;
    child_keys();
    {
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
    }
    goto insert;

done:
    inserts = ins;
    tmax_out = tmax;
    return verdict;
}
// LDS bytes of a dfs_lean_w wave: 16-byte slots + Bloom + fill counts
template <class M>
constexpr int lds_w() { return LDS_TBL + M::SLOTS * 16 + M::BLOOM / 8 + M::BKT; }

// Per-key search tables, built once per call for every key by one wave per
// key (pass 1, then pass 2 + layer sweep into a bump-allocated slot of the
// tables arena). The search kernels then only search: their hot loop does not
// share registers with table building. Keys settled here (no search needed,
// window wider than 64, beyond the compact encoding) get their verdict now.
// bytes of a k_lin_xw key's tables (ops, windows per layer)
__device__ __forceinline__ uint64_t a16(uint64_t x) { return (x + 15) & ~15ULL; }
__device__ __forceinline__ uint64_t xw_bytes(int n_ops, int n_ok, long long sumW) {
    return 3 * a16((uint64_t)n_ops * 4) + a16((uint64_t)(n_ok + 1) * 4) + a16((uint64_t)sumW * 4 + 1024) +
           a16((uint64_t)sumW * 8 + 2048);
}

struct KeyMeta {
    uint64_t off;      // byte offset of the key's tables in the arena
    int32_t n_ops, n_ok;
    int32_t maxw;      // widest window
    int32_t pad;
};

struct TblArgs {
    KeySrc src;
    int64_t K;
    KeyMeta *meta;
    char *arena;
    unsigned long long *bump;   // arena bytes used
    jh_key_verdict *out;
    int32_t *list;              // keys that need a search: LEAN mode
    int32_t *n_list;
    int32_t *list_w;            // keys that need a search: WIDE mode
    int32_t *n_list_w;
    int32_t *list_x;            // keys that need a search: windows wider than 64 (k_lin_xw)
    int32_t *n_list_x;
    unsigned long long *xw_max; // the largest k_lin_xw table (bytes)
    int32_t states8;            // every interned state < 256
};

__global__ void __launch_bounds__(256) k_key_tables(TblArgs A) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t key = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); key < A.K; key += nw) {
        KeyInfo K;
        jh_key_verdict v;
        bool need = key_pass1(A.src, (int)key, lane, K, v);
        // long keys (beyond the compact encoding: a < 2^14, op ids < 2^16) take
        // the k_lin_xw path, whose tables are 32-bit
        const bool long_key = K.n_ok >= COMPACT_MAX_OK || K.n_ops > 65535;
        if (need) {
            int maxw = 65;
            if (!long_key && K.sumW <= 64LL * K.n_ok) {
                unsigned long long off = 0;
                if (lane == 0) off = atomicAdd(A.bump, (unsigned long long)tblc_bytes(K));
                off = (unsigned long long)rfl64(__shfl(off, 0));
                maxw = key_fill_c<false>(A.src, K, lane, A.arena + off);
                if (maxw <= 64 && lane == 0) {
                    KeyMeta m;
                    // pad: the window sum, the phase-1 ordering's cost estimate (k_list_cost)
                    m.off = off; m.n_ops = K.n_ops; m.n_ok = K.n_ok; m.maxw = maxw;
                    m.pad = (int32_t)min(K.sumW, (long long)0x7FFFFFFE);
                    A.meta[key] = m;
                    if (A.states8 && maxw <= 40) A.list[atomicAdd(A.n_list, 1)] = (int32_t)key;
                    else A.list_w[atomicAdd(A.n_list_w, 1)] = (int32_t)key;
                }
            }
            if (maxw > 64 && lane == 0) {
                // wider than 64 (up to JH_MAX_WINDOW): k_lin_xw builds its own tables
                KeyMeta m;
                m.off = 0; m.n_ops = K.n_ops; m.n_ok = K.n_ok; m.maxw = -1; m.pad = (int32_t)K.sumW;
                A.meta[key] = m;
                A.list_x[atomicAdd(A.n_list_x, 1)] = (int32_t)key;
                atomicMax(A.xw_max, (unsigned long long)xw_bytes(K.n_ops, K.n_ok, K.sumW));
            }
        }
        if (!need && lane == 0) A.out[key] = v;
    }
}

// LEAN: dfs_lean (8-byte LDS keys); else WL: dfs_lean_w (16-byte LDS keys),
// else dfs_search (every configuration in the HBM table)
// STREAM: the kernel takes part in the streaming heavy-key pass (phase 1 as
// the producer of the live lists, or a consumer of them); without it the
// streaming code is compiled out (it costs phase 1 registers and occupancy).
template <class M, bool LEAN, bool WL = false, bool STREAM = false, bool HO = false>
__device__ __forceinline__ void lin_dfs_waves(const DfsArgs &A) {
    const int lane = threadIdx.x;
    const size_t wv = (size_t)(blockIdx.x - A.wave_off);
    uint64_t *memo = A.memo + wv * A.memo_cap * 2;
    Frame *stack = A.stack + wv * A.stack_cap;
    uint64_t *stage = (uint64_t *)(A.scratch + wv * A.scratch_bytes);
    unsigned long long my_probes = 0;
    const int n_list = A.n_list_dev ? *A.n_list_dev : A.n_list;
    if (n_list < A.n_min || (A.n_max > 0 && n_list > A.n_max)) return;
    const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
    bool spanned = false;       // t_span[0]: the first key any wave of the role took
    if (A.defer_time && lane == 0) atomicMin(&A.defer_time[0], __builtin_amdgcn_s_memrealtime());
    // phase 1 (streaming): this key is finished -- after its list entries
    auto p1_key_done = [&]() {
        if constexpr (STREAM)
            if (A.p1_count && lane == 0) __hip_atomic_fetch_add(A.p1_count, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    };
    for (;;) {
        int idx = 0;
        if (lane == 0) idx = atomicAdd(A.queue, 1);
        idx = readlane(idx, 0);
        int key;
        if (STREAM && A.live_n) {
            int k = -1;
            if (lane == 0) k = stream_key(A.list, A.live_n, A.p1_done, A.p1_tot, idx, A.flags);
            key = readlane(k, 0);
            if (key < 0) break;
        } else {
            if (idx >= n_list) {
                // the first wave to find the queue empty: the host may launch
                // the streaming consumers now (system scope: host-mapped)
                if (STREAM && A.drained && idx == n_list && lane == 0)
                    __hip_atomic_store(A.drained, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            key = A.list[idx];
        }
        if (A.t_span && !spanned && lane == 0) atomicMin(&A.t_span[0], __builtin_amdgcn_s_memrealtime());
        spanned = true;
        TL_REC(A.tl, key, 2);
        const KeyMeta mt = A.meta[key];
        KeyInfo K;
        K.n_ops = mt.n_ops; K.n_ok = mt.n_ok; K.sumW = 0;
        K.s0 = 0; K.s1 = 0;
        const char *tb = A.tables + mt.off;
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        long long inserts = 0;
        uint32_t tmax = 0;
        // the LDS memo packs states in 8 bits and masks in 40 (LEAN); else
        // the HBM table only (WIDE). One mode per kernel: the two searches do
        // not share a register allocation.
        if ((A.states8 && mt.maxw <= 40) != LEAN) { p1_key_done(); continue; }
        if (A.prio_ins > 0) __builtin_amdgcn_s_setprio(0);
        if (A.seq_start && lane == 0)
            __hip_atomic_store(&A.seq_start[key], __builtin_amdgcn_s_memrealtime() | 1ULL, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        int verdict;
        uint32_t ins_real = 0;
        if constexpr (LEAN) {
            // (a takeover's save returns V_HANDED: the search goes on from the
            // record it just published, rs_off[key], as phase 2 resumes phase 1's)
            do {
                verdict = dfs_lean<M, HO>(A, K, tb, key, lane, memo, stack, stage, inserts, tmax, my_probes, ins_real,
                                          (A.rs_mode == 1 || (HO && A.handoff)) && A.hlog ? A.hlog + wv * A.hlog_cap
                                                                                     : nullptr);
            } while (verdict == V_HANDED);
        }
        else if constexpr (WL) verdict = dfs_lean_w<M>(A, K, tb, key, lane, memo, stack, stage, inserts, tmax, my_probes);
        else verdict = dfs_search<false, false, M>(A, K, (char *)tb, key, lane, memo, stack, stage, inserts, tmax, my_probes);
        if (A.dbg && lane == 0) { A.dbg[16 * wv + 2] += __builtin_amdgcn_s_memtime() - c1; A.dbg[16 * wv + 3] += 1; }
        if (verdict == JH_CANCELLED) {
            TL_REC(A.tl, key, 3);
            p1_key_done();
            continue;
        }
        if (verdict == JH_UNKNOWN && A.defer && inserts >= A.budget &&
            (A.budget_full == 0 || inserts < A.budget_full)) {
            if (lane == 0) {
                const int d = atomicAdd(A.defer_count, 1);
                if (A.defer_list) A.defer_list[d] = key;
                // the heavy-key pass starts with the keys of most estimated work:
                // the quick search's inserts over its progress (deepest layer /
                // layers). Round 5: with the hand-over most deferred keys are
                // short searches handed over at 1 024 inserts; ordered by progress
                // alone (rounds 3-4) they went first and the genuinely heavy keys
                // waited ~12 ms for a sequential wave (profiles/r05/timeline/).
                // Sort key: 2^31 - 1 - estimate, ascending (the pool's rank too)
                const uint64_t prog = max<uint64_t>(1, (uint64_t)tmax * 1000000u / (uint64_t)max(1, K.n_ok));
                const uint64_t real = LEAN ? (uint64_t)ins_real : (uint64_t)inserts;
                const uint64_t est = min<uint64_t>(0x7FFFFFFFull, real * 1000000ull / prog);
#ifdef JH_ORDER_PROGRESS
                // rounds 3-4: least phase-1 progress first (A/B builds)
                const uint64_t pk = ((prog < 0x7FFFFFFFull ? prog : 0x7FFFFFFFull) << 32) | (uint32_t)key;
                (void)est;
#else
                const uint64_t pk = ((0x7FFFFFFFull - est) << 32) | (uint32_t)key;
#endif
                if (A.defer64) A.defer64[d] = pk;
                if (A.defer_kind) {
                    const int dk = atomicAdd(A.defer_kind_count, 1);
                    A.defer_kind[dk] = pk;
                    if (STREAM && A.s_kind) __hip_atomic_store(&A.s_kind[dk], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (STREAM && A.s_all) __hip_atomic_store(&A.s_all[d], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (A.defer_time) A.defer_time[2 + key] = __builtin_amdgcn_s_memrealtime();
                if (A.defer_info) {
                    A.defer_info[2 * (size_t)key] = real;
                    A.defer_info[2 * (size_t)key + 1] = (uint64_t)tmax | ((uint64_t)K.n_ok << 32);
                }
                if (A.seq_start)
                    __hip_atomic_store(&A.seq_start[key], SEQ_HANDED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            p1_key_done();
            continue;
        }
        jh_key_verdict v;
        v.valid = verdict;
        v.cause = (verdict == JH_UNKNOWN ? JH_CAUSE_BUDGET : 0) | A.cause_or;
        v.explored = inserts;
        v.fail_entry = -1;
        // an invalid key's failing row is resolved by k_fail_rows from tmax
        if (verdict == JH_INVALID) v.fail_entry = -(int64_t)tmax - 2;
        if (lane == 0) emit_verdict(A.out, A.claim, key, v);
        TL_REC(A.tl, key, 3);
        p1_key_done();
    }
    if (A.dbg && lane == 0) A.dbg[16 * wv + 9] = __builtin_amdgcn_s_memtime() - t_begin;
    if (A.t_span && lane == 0) atomicMax(&A.t_span[1], __builtin_amdgcn_s_memrealtime());
    for (int o = 32; o > 0; o >>= 1) my_probes += __shfl_xor(my_probes, o);
    if (A.dbg && lane == 0) A.dbg[16 * wv + 15] = my_probes;
    if (lane == 0 && A.probes) atomicAdd(A.probes, my_probes);
    if (lane == 0 && A.exit_count) atomicAdd(A.exit_count, 1);
    if (A.defer_time && lane == 0) atomicMax(&A.defer_time[1], __builtin_amdgcn_s_memrealtime());
}

// Phase 1 hands keys out in list order and ends when its slowest wave ends;
// a wave that takes a costly key late leaves a tail. Largest estimated cost
// first (LPT): the cost is the key's window sum (sum over ok returns of the
// open calls, which bounds each layer's branching). Slots past the list's
// length get cost 0 and sort last. Only the order changes: every key is
// still searched by the same DFS.
__global__ void __launch_bounds__(256) k_list_cost(const int32_t *__restrict__ list, const int32_t *__restrict__ n_list,
                                                   const KeyMeta *__restrict__ meta, int64_t K, uint32_t *cost,
                                                   int32_t *val) {
    const int n = *n_list;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < n) {
            const int32_t k = list[i];
            cost[i] = (uint32_t)meta[k].pad + 1u;
            val[i] = k;
        } else {
            cost[i] = 0;
            val[i] = -1;
        }
    }
}

// phase 1: every key under the quick budget (STREAM: the producer of the
// streaming heavy-key pass's live lists)
// six waves per SIMD (<= 80 VGPRs, 24 per CU; LDS allows 26): phase 1
// 16.5 -> 15.7 ms on C3 (round 4, profiles/r04); JH_P1_WPE=0: no cap
#ifndef JH_P1_WPE
#define JH_P1_WPE 6
#endif
#if JH_P1_WPE > 0
#define JH_P1_ATTR __attribute__((amdgpu_waves_per_eu(JH_P1_WPE)))
#else
#define JH_P1_ATTR
#endif
template <bool LEAN, bool STREAM>
__global__ void __launch_bounds__(64) JH_P1_ATTR k_lin_dfs(DfsArgs A) {
    lin_dfs_waves<MemoQ, LEAN, false, STREAM>(A);
}
// heavy keys: the full-budget sequential search racing k_lin_bfs, one wave
// per CU with a 128 KB LDS memo
template <bool LEAN>
__global__ void __launch_bounds__(64) k_lin_seq(DfsArgs A) { lin_dfs_waves<MemoH, LEAN>(A); }
// very heavy keys (over the phase-2 budget, mostly on their way to the full
// budget, i.e. :unknown): their memo lives in HBM whatever the LDS holds, so
// a step waits on an HBM round trip; four waves per CU (one per SIMD) keep
// four times as many of those searches in flight
template <bool LEAN>
__global__ void __launch_bounds__(64) k_lin_seq3(DfsArgs A) { lin_dfs_waves<MemoM, LEAN>(A); }
// the deferred WIDE keys (phases 2 and 3): their own list, stream and waves,
// as many as there are keys (up to 4 per CU, bounded by free HBM), beside the
// LEAN pipeline instead of behind it; 2 048 16-byte LDS memo slots + 4 KB
// Bloom per wave (37 KB: four waves per CU)
using MemoWL = MemoCfg<9, 15>;
constexpr int SEQW_LDS = lds_w<MemoWL>();
constexpr uint64_t SEQW_SCR = MemoWL::SLOTS * 16;   // per wave: the eviction stage
__global__ void __launch_bounds__(64) k_lin_seqw(DfsArgs A) { lin_dfs_waves<MemoWL, false, true>(A); }
// phase 2 of LEAN and WIDE keys in one grid (blocks 0..n_l-1 LEAN, the rest
// WIDE; both 37 KB of LDS): one stream for both, so the heavy-key pass needs
// no more streams than the hardware has queues
struct DfsPair { DfsArgs l, w; int32_t n_l; };
// (two roles: the LEAN role keeps MemoM, four waves per CU with the WIDE ones;
// LEAN keys alone: MemoP2)
constexpr int SEQLW_LDS = MemoM::LDS > SEQW_LDS ? MemoM::LDS : SEQW_LDS;
template <bool STREAM, class ML = MemoM>
__global__ void __launch_bounds__(64) k_lin_seq_lw(DfsPair P) {
    if ((int)blockIdx.x < P.n_l) lin_dfs_waves<ML, true, false, STREAM, !STREAM>(P.l);
    else lin_dfs_waves<MemoWL, false, true, STREAM>(P.w);
}

// Deferred keys, heaviest estimate first (phase 1's progress, ties by key: the
// likely longest searches start first), then the key ids alone: one workgroup
// per list, a bitonic sort of (progress << 32 | key) in LDS. Lists longer than
// SORT_SMALL are sorted by hipcub on the host side of the call.
constexpr int SORT_SMALL = 4096;
struct SortLists {
    const uint64_t *in[3];
    int32_t *out[3];
    int n[3];
};
__global__ void __launch_bounds__(1024) k_sort_defer(SortLists L) {
    __shared__ uint64_t s[SORT_SMALL];
    const int n = L.n[blockIdx.x];
    if (n <= 0 || n > SORT_SMALL) return;
    const uint64_t *in = L.in[blockIdx.x];
    int32_t *out = L.out[blockIdx.x];
    int P = 2;
    while (P < n) P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x) s[i] = i < n ? in[i] : ~0ULL;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    if ((a > b) == ((i & k) == 0)) { s[i] = b; s[ixj] = a; }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = (int32_t)(uint32_t)s[i];
}
__global__ void k_unpack_keys(const uint64_t *__restrict__ in, int n, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (int32_t)(uint32_t)in[i];
}

// :linear mode has no WGL phase: every key that needs a search goes to the
// reachable-set analysis, as if phase 1 had handed it on (q[1] all, q[29]
// LEAN, q[30] WIDE, as phase 1's deferral counters)
__global__ void __launch_bounds__(1024) k_linear_lists(const int32_t *__restrict__ list, const int32_t *n_list,
                                                      const int32_t *__restrict__ list_w, const int32_t *n_list_w,
                                                      int32_t *defer, int32_t *defer_l, int32_t *defer_w, int32_t *q) {
    const int nl = *n_list, nw = *n_list_w;
    for (int i = threadIdx.x; i < nl; i += blockDim.x) { defer[i] = list[i]; defer_l[i] = list[i]; }
    for (int i = threadIdx.x; i < nw; i += blockDim.x) { defer[nl + i] = list_w[i]; defer_w[i] = list_w[i]; }
    if (threadIdx.x == 0) { q[1] = nl + nw; q[29] = nl; q[30] = nw; }
}

// ---------------------------------------------------------------------------
// Phase 2 (deferred LEAN keys): one workgroup per key. Wave 0 runs the WGL
// DFS (dfs_acc: dfs_lean's search plus the hooks below); every wave of the
// workgroup joins an exhaustive parallel enumeration (wg_enum_work) when the
// DFS spends many inserts below one stack node.
//
// Why the count stays exactly WGL's. Let X be an open node of the DFS stack
// and M_X the memo when X was inserted. If no terminal configuration is
// reachable from X ("X is dead"), the sequential DFS inserts exactly
// Reach(X) \ M_X before it pops X: it visits every node reachable from X that
// is not in the memo, and a node already there is closed and dead (a child of
// an expanded node can only be an ancestor on the stack in a cycle, and the
// graph is a DAG: linearized sets grow along edges), so its reach is in the
// memo too. The nodes inserted below X so far belong to that set, and the
// still-open ones (the stack from X to the current node) are its only members
// whose children may not all be in the memo. So an enumeration from the roots
// {open nodes from X down}, pruned at the current memo, yields
// N = Reach(X) \ memo_now; if it meets no terminal configuration, X is dead
// and memo_now + N is exactly the memo the sequential DFS holds when it pops
// X: the search merges N, adds |N| to its insert count and pops X. If the
// enumeration meets a terminal configuration, X is live (the DFS never pops a
// live node: it ends below it), N is dropped and the DFS goes on untouched.
// The frames' "rest" sets stay exact: a sibling P+j of X holds L(P)+{j}, while
// every node of N contains L(P)+{i} (i = X's member), so no sibling is in N.
// Verdict, explored count (WGL's cache size) and the deepest layer reached
// (the failing row of an invalid key) are the sequential search's; the tests
// compare them with oracle/jh_oracle.c's orc_wgl_canonical key by key.
//
// Policy (simulated on every deferred key of the C3 histories, all exact):
// every ACC_T inserts, accelerate the deepest open node with >= ACC_T/2
// inserts below it that is not known to be live (and, after an inconclusive
// try, has twice as many); after a success, try its parent at once (climb)
// until a live node is met. An enumeration gives up (inconclusive) past
// max(ACC_CAPMIN, ACC_CAPF x the inserts below X) new nodes.
#ifndef JH_WG_THREADS
#define JH_WG_THREADS 512
#endif
constexpr int WG_THREADS = JH_WG_THREADS;
// One workgroup per CU: a 64 KB LDS memo and a 64 KB Bloom filter (the merged
// dead regions live in HBM: a small filter would send most DFS steps there)
using MemoW = MemoCfg<11, 19>;
constexpr uint32_t ACC_T = 1024, ACC_CAPF = 4, ACC_CAPMIN = 2048;
constexpr int ACC_MAXROOTS = 65;    // X lies in the register ring: <= 64 frames + the current node
constexpr int CMD_ENUM = 1, CMD_DONE = 2, CMD_MERGE = 3;

// Round 6: speculative dead-subtree enumeration across workgroups (VERDICT r5
// item 2). On a heavy valid key WGL's time is nearly all one dead subtree:
// C3 rank 0's key 1086 spends 44 700 of its 46 490 inserts below one node at
// depth 128 (28 layers, 38 levels deep), rank 4's key 1631 25 790 + 7 696
// below two (tools/shape/wgl_shape.py) -- a few ms for a parallel
// enumeration, tens of ms for the one-wave DFS, which cannot tell that
// node's subtree is dead until it has walked all of it. A late helper that
// runs a key's exact search (the main, dfs_acc) posts the open nodes of its
// stack near the current one that have many inserts below them to this
// board; late helpers with no key of their own take them and enumerate each
// posted node's whole reachable set, with no memo (so nothing the main's
// open nodes have not finished is pruned), up to a cap. A node whose
// enumeration meets no terminal configuration is dead: the main, if the node
// is still on its stack (same depth, same insert index), merges the set into
// its memo -- the nodes not there yet are exactly what WGL inserts before
// popping it (the argument of wg_enum_work: memo_X + Reach(X) is WGL's memo at
// the pop, and everything inserted since X is in Reach(X)) -- adds their
// number to its count and pops the node. A live result marks the node (and so
// its ancestors) live. Verdicts, counts and failing rows stay WGL's.
constexpr int SPEC_SLOTS = 64;         // one per lane of the main's wave
constexpr int SPEC_PER_CHECK = 4;      // new posts per poll of the main
constexpr uint32_t SPEC_CHK = 128;     // inserts between polls
constexpr uint32_t SPEC_RES_CAP = 1u << 18;    // nodes per helper result buffer (2 MB)
constexpr int SPEC_FREE = 0, SPEC_POSTED = 1, SPEC_CLAIMED = 2, SPEC_DEAD = 3, SPEC_LIVE = 4, SPEC_INC = 5,
              SPEC_STALE = 6, SPEC_BUSY = 7;
struct SpecSlot {
    int32_t state, key;
    uint32_t depth, seq;       // the node on the main's stack: depth and insert index
    uint64_t cfg;              // its configuration (lk_make)
    uint32_t cap, n;           // the enumeration's cap; a dead result's node count
    int32_t helper, pad;       // the helper whose result buffer holds the nodes
    uint64_t pad2;
};
constexpr int ENUM_LIVE = 1, ENUM_CAP = 2;

struct WgShared {
    int cmd, key, merge, status;
    uint32_t n_roots, n_ok, theta, acc_lo, acc_hi, gen;
    uint32_t cap_total;       // work positions this call may fill (roots + new nodes)
    uint32_t head, tail, active;   // the current layer's queue: work[head, tail)
    uint32_t tmin_new, tmax_new;
    uint32_t t_cur, t_next;   // the layer being closed / the lowest pending layer
    uint32_t npend, npend2, pend_sel, gset_used;
    uint32_t w_cur, r_cur;    // the current layer's window size and RET position
    uint32_t nchild;          // children of the staged chunk
    unsigned long long pick;  // helper mode: (longest running, lowest list index) candidate
    int n_live;               // helper mode: the list's length at this scan (live in streaming)
    uint32_t win[64];         // the current layer's window: need | becomes << 16 per member
    const uint32_t *woff;     // the key's window table (wtab_build)
    const uint32_t *wrq;
    const uint8_t *rpos;
    // round 6, the spec board (see SpecSlot): an enumeration a helper runs for
    // another workgroup's search keeps its new nodes (keep), ignores its own
    // memo (nomemo) and stops when the slot goes stale (abort_state); a merge
    // (CMD_MERGE) folds such a result into this workgroup's memo
    uint64_t *keep;
    uint32_t keep_n;
    int nomemo;
    const int32_t *abort_state;
    const uint64_t *m_src;
    uint32_t m_n, m_new, m_tmin, m_tmax;
    int spec_slot, res_slot, wtab_key;
};
constexpr int WG_SH_OFF = (MemoW::LDS + 255) & ~255;
constexpr int ESET = 2048;          // LDS set of the current layer's configurations (8-byte keys)
constexpr int ESET_PROBES = 16;     // a key whose first 16 slots are taken goes to the HBM set
constexpr int WG_ESET_OFF = WG_SH_OFF + (int)((sizeof(WgShared) + 255) & ~255);
// a round's configurations are expanded child by child across all worker
// lanes: FL_CHUNK of them at a time are staged (key, candidate bits, prefix)
constexpr int FL_CHUNK = 512;
constexpr int WG_STAGE_OFF = WG_ESET_OFF + ESET * 8;
constexpr int WG_LDS = WG_STAGE_OFF + FL_CHUNK * 20;

struct WgArgs {
    DfsArgs d;                 // the search: per-workgroup memo / stack / stage, budget, gen, tables
    uint64_t *gset;            // per workgroup: gset_cap slots, all zero between enumerations
    uint32_t gset_cap;         // power of two
    uint64_t *work;            // per workgroup: work_cap keys, all zero between enumerations
    uint32_t work_cap;
    char *wtab;                // per workgroup: the current key's window table
    uint64_t wtab_bytes;
    uint64_t *pend;            // per workgroup: 2 x pend_cap configurations waiting for a later layer
    uint32_t pend_cap;
    unsigned long long *key_prof;    // JH_DEBUG=4: per key {cycles, inserts, verdict | workgroup << 8}
    uint32_t acc_t;            // inserts between acceleration attempts (ACC_T; 0: plain DFS)
    unsigned long long *acc_stats;   // [0] enumerations [1] their new nodes [2] dead [3] live [4] inconclusive
    // helper mode (late helpers of phase 2, see wg_helper_pick): the
    // sequential search's per-key start times and exit count, a per-key
    // taken flag, and how long (s_memrealtime ticks) a key must have run
    const unsigned long long *seq_start;
    const int32_t *seq_exit;
    int32_t seq_waves;
    int32_t *taken;
    uint64_t late_ticks;
    // streaming heavy-key pass: the sequential search's wave count on the
    // device (its early and late grids); d.live_n etc. make d.list live
    const int32_t *seq_waves_dev;
    // round 6: the spec board (late helpers only; null: off), each helper's
    // result buffer (spec_res_cap nodes), and the posting policy: nodes with
    // at least spec_min inserts below them, within spec_dist levels of the
    // current node, enumerated up to spec_mult x their inserts so far
    SpecSlot *spec;
    uint64_t *spec_res;
    uint32_t spec_res_cap, spec_min, spec_mult, spec_dist;
    int32_t *spec_q;           // the counters (q + Q_SPEC)
    int32_t spec_first;        // helpers serve the board before taking keys (JH_LIN_SPEC_FIRST)
    int32_t n_mains;           // helpers [n_mains, grid) only serve the board (never take a key)
    int32_t *mains_live;       // helpers running a key now (the board's servers stay while any does)
};

__device__ __forceinline__ uint64_t lk_make(uint32_t t, uint32_t s, uint64_t m) {
    return (1ULL << 63) | ((uint64_t)t << 48) | ((uint64_t)s << 40) | m;
}
// enumeration roots are marked with bit 62 (t < 2^14 leaves it clear in every key)
constexpr uint64_t LK_ROOT = 1ULL << 62;

// Random-access window table of a key for the enumeration, from the compact
// tables (dfs_lean's lane-resident window moved layer by layer): W(t) is
// wrq[woff[t] .. woff[t+1]) (need | becomes << 16 per member, call order) and
// rpos[t] the position of RET[t] in W(t).
__device__ void wtab_build(const KeyInfo &K, const char *tb, int lane, uint32_t *woff, uint32_t *wrq,
                           uint8_t *rpos) {
    const OpC *ops = (const OpC *)tb;
    const Lay *lay = (const Lay *)(tb + tblc_ops_bytes(K));
    const int n_ok = K.n_ok;
    int w = (int)(lay[0].hi >> 6), P = w;
    uint32_t wr = lane < w ? ops[lane].rq : RQ_EMPTY;
    uint32_t off = 0;
    for (int t = 0; t < n_ok; t++) {
        const uint32_t r = lay[t].hi & 63;
        if (lane == 0) { woff[t] = off; rpos[t] = (uint8_t)r; }
        if (lane < w) wrq[off + lane] = wr;
        off += (uint32_t)w;
        if (t + 1 < n_ok) {
            const uint32_t sh = (uint32_t)wave_shl1((int)wr);
            if (lane >= (int)r) wr = sh;
            w--;
            if (lane == w) wr = RQ_EMPTY;
            const int c = (int)(lay[t + 1].hi >> 6);
            if (lane >= w && lane < w + c) wr = ops[P + (lane - w)].rq;
            w += c; P += c;
        }
    }
    if (lane == 0) woff[n_ok] = off;
}

__device__ __forceinline__ uint32_t wtab_bytes_for(uint32_t max_ok) {
    return (((max_ok + 1) * 4 + 255) & ~255u) + ((max_ok * 40 * 4 + 255) & ~255u) + ((max_ok + 255) & ~255u);
}

// Is the configuration in the DFS memo? The LDS table always; the HBM table
// (behind the Bloom filter) for layers below theta and in the merged range.
__device__ unsigned int g_prof_hbm, g_prof_gset, g_prof_rounds, g_prof_layers;
__device__ unsigned long long g_prof_form, g_prof_close, g_prof_merge;
__device__ __forceinline__ bool wg_memo_has(uint64_t k, const WgShared &sh, const uint64_t *memo,
                                            uint32_t cap_mask, unsigned long long &probes) {
    if (sh.nomemo) return false;        // a spec enumeration: the whole reachable set
    const ulonglong2 *B = (const ulonglong2 *)(jh_lds + MemoW::OFF_MEMO);
    const uint32_t *bloom = (const uint32_t *)(jh_lds + MemoW::OFF_BLOOM);
    uint32_t h1, h2, b1, b2;
    lk_hash((uint32_t)k, (uint32_t)(k >> 32), h1, h2);
    lk_bkts<MemoW>(h1, h2, b1, b2);
    const ulonglong2 x0 = B[2 * b1], x1 = B[2 * b1 + 1], y0 = B[2 * b2], y1 = B[2 * b2 + 1];
    if ((x0.x == k) | (x0.y == k) | (x1.x == k) | (x1.y == k) | (y0.x == k) | (y0.y == k) | (y1.x == k) |
        (y1.y == k))
        return true;
    const uint32_t t = lk_t(k);
    if ((t < sh.theta || (t >= sh.acc_lo && t <= sh.acc_hi)) && bloom_test2<MemoW>(bloom, lk_bl(h1), lk_bl(h2))) {
#ifdef JH_ENUM_PROF
        atomicAdd(&g_prof_hbm, 1u);
#endif
        return (hbm_probe(memo, cap_mask, sh.gen, t, lk_s(k), lk_m(k), probes) >> 32) == 0;
    }
    return false;
}

// the enumeration's own set of new nodes (HBM, open addressing, CAS claim)
__device__ __forceinline__ bool gset_insert(uint64_t *g, uint32_t gmask, uint64_t k, uint32_t &slot,
                                            int32_t *flags) {
    uint32_t h = (uint32_t)jh_mix64(k) & gmask;
    for (uint32_t n = 0;; n++) {
        if (n > gmask) { atomicOr(flags, 64); return false; }
        const unsigned long long prev = atomicCAS((unsigned long long *)&g[h], 0ULL, (unsigned long long)k);
        if (prev == 0) { slot = h; return true; }
        if (prev == k) return false;
        h = (h + 1) & gmask;
    }
}
// the slot holding k (every key looked up here was inserted), or ~0u
__device__ __forceinline__ uint32_t gset_find(const uint64_t *g, uint32_t gmask, uint64_t k) {
    uint32_t h = (uint32_t)jh_mix64(k) & gmask;
    for (uint32_t n = 0; n <= gmask; n++) {
        const uint64_t x = __hip_atomic_load(&g[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (x == k) return h;
        if (x == 0) return ~0u;
        h = (h + 1) & gmask;
    }
    return ~0u;
}

// The current layer's set: an LDS table, with the HBM set behind it for a key
// whose first ESET_PROBES slots are taken. Slots are never freed during a
// layer, so every inserter of one key sees the same slots and makes the same
// choice (LDS or HBM): a key is counted once. Returns true if k is new.
__device__ __forceinline__ bool layer_insert(WgShared &sh, uint64_t *gset, uint32_t gmask, uint64_t k,
                                             int32_t *flags) {
    uint64_t *es = (uint64_t *)(jh_lds + WG_ESET_OFF);
    uint32_t h = (uint32_t)jh_mix64(k) & (ESET - 1);
    for (int n = 0; n < ESET_PROBES; n++) {
        const unsigned long long prev = atomicCAS((unsigned long long *)&es[h], 0ULL, (unsigned long long)k);
        if (prev == 0) return true;
        if (prev == k) return false;
        h = (h + 1) & (ESET - 1);
    }
    if (!sh.gset_used) sh.gset_used = 1;
#ifdef JH_ENUM_PROF
    atomicAdd(&g_prof_gset, 1u);
#endif
    uint32_t slot;
    return gset_insert(gset, gmask, k, slot, flags);
}

// Append a configuration to the work array (the current layer's queue and the
// list of new nodes). Past the cap it is still recorded, in the slack that is
// never claimed, so that the clean-up finds every HBM-set entry.
__device__ __forceinline__ void wg_append(WgShared &sh, uint64_t *work, uint32_t work_cap, uint64_t e,
                                          int32_t *flags) {
    const uint32_t pos = atomicAdd(&sh.tail, 1u);
    if (pos < work_cap) __hip_atomic_store(&work[pos], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else atomicOr(flags, 64);
    if (pos >= sh.cap_total) atomicOr(&sh.status, ENUM_CAP);
}

// The children of a configuration of the current layer the model allows,
// as window-member bits (the lane-parallel expansion takes them one by one).
__device__ __forceinline__ uint64_t wg_cands(uint64_t k, const WgShared &sh) {
    const uint32_t s = lk_s(k);
    const uint64_t mask = lk_m(k);
    const uint32_t w = sh.w_cur;
    uint64_t c = 0;
    for (uint32_t j = 0; j < w; j++) {
        const uint32_t need = sh.win[j] & 0xFFFF;
        c |= (uint64_t)(need == s || need == RQ_ANY) << j;
    }
    return c & ~mask;
}

// One child (member j) of configuration k of the current layer: a same-layer
// child that is neither in the memo nor in the layer's set joins the layer's
// queue; the RET child (a later layer) waits in the pending list; a terminal
// child ends the enumeration (the node is live).
__device__ __forceinline__ void wg_child(uint64_t k, uint32_t j, WgShared &sh, uint64_t *gset, uint32_t gmask,
                                         uint64_t *work, uint32_t work_cap, uint64_t *pcur, uint32_t pend_cap,
                                         const uint64_t *memo, uint32_t cap_mask, unsigned long long &probes,
                                         int32_t *flags) {
    const uint32_t t = lk_t(k);
    const uint64_t mask = lk_m(k);
    const uint32_t nv = sh.win[j] >> 16;
    if (j == sh.r_cur) {
        // lift RET[t], then every next RET op already linearized
        const uint32_t n_ok = sh.n_ok;
        uint64_t nm = drop_bit(mask, j);
        uint32_t u = t + 1;
        for (;;) {
            if (u >= n_ok) break;
            const uint32_t ru = sh.rpos[u];
            if (!((nm >> ru) & 1)) break;
            nm = drop_bit(nm, ru);
            u++;
        }
        if (u >= n_ok) { atomicOr(&sh.status, ENUM_LIVE); return; }   // a terminal configuration
        const uint32_t q = atomicAdd(&sh.npend, 1u);
        if (q < pend_cap) {
            __hip_atomic_store(&pcur[q], lk_make(u, nv, nm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            atomicMin(&sh.t_next, u);
        } else {
            atomicOr(&sh.status, ENUM_CAP);
        }
        return;
    }
    const uint64_t ck = lk_make(t, nv, mask | (1ULL << j));
    if (wg_memo_has(ck, sh, memo, cap_mask, probes)) return;
    if (!layer_insert(sh, gset, gmask, ck, flags)) return;
    wg_append(sh, work, work_cap, ck, flags);
}

// All waves: the enumeration wave 0 set up in sh (its roots in the pending
// list, marked LK_ROOT), layer by layer: form the lowest pending layer from its
// pending entries (deduplicated in the layer set, pruned at the memo), close
// it under same-layer lifts with every worker taking queued configurations,
// go on with the next pending layer. Then, if it met neither a terminal
// configuration nor the cap and sh.merge is set, merge the new nodes into the
// DFS memo (HBM table + Bloom), and clean up (HBM set and work array all zero).
__device__ __forceinline__ void wg_enum_work(const WgArgs &W, WgShared &sh, int tid, uint64_t *gset, uint64_t *work,
                                          uint64_t *memo, uint64_t *pend, unsigned long long &probes) {
    const int lane = tid & 63;
    // Waves 1.. do the work; wave 0 (the DFS, which calls in from deep inside
    // its loop) only takes part in the barriers.
    const bool worker = tid >= 64;
    const int wid = tid >> 6;
    const uint32_t wt = (uint32_t)tid - 64, WN = WG_THREADS - 64;
    const uint32_t gmask = W.gset_cap - 1, cap_mask = W.d.memo_cap - 1;
    uint64_t *es = (uint64_t *)(jh_lds + WG_ESET_OFF);
    int32_t *flags = W.d.flags;
    const unsigned long long cw0 = __builtin_amdgcn_s_memtime();
    if (worker)
        for (uint32_t i = wt; i < (uint32_t)ESET; i += WN) es[i] = 0;
    for (;;) {
        // ---- form the lowest pending layer ------------------------------------
        __syncthreads();
#ifdef JH_ENUM_PROF
        const unsigned long long pf0 = __builtin_amdgcn_s_memtime();
        if (tid == 64) atomicAdd(&g_prof_layers, 1u);
#endif
        if (tid == 64) {
            sh.t_cur = sh.t_next; sh.t_next = 0xFFFFFFFFu; sh.npend2 = 0;
            sh.head = sh.tail; sh.active = 0;
            // racing k_lin_bfs: a key it settled ends the enumeration as incomplete
            if (W.d.claim && __hip_atomic_load(&W.d.claim[sh.key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                sh.status |= ENUM_CAP;
            // a spec enumeration whose main no longer needs it
            if (sh.abort_state &&
                __hip_atomic_load(sh.abort_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == SPEC_STALE)
                sh.status |= ENUM_CAP;
        }
        __syncthreads();
        const uint32_t tc = sh.t_cur, np = sh.npend, sel = sh.pend_sel;
        uint64_t *pin = pend + (size_t)sel * W.pend_cap, *pout = pend + (size_t)(sel ^ 1) * W.pend_cap;
        if (worker && wt < 64) {
            // the layer's window into LDS (the closure reads it for every configuration)
            const uint32_t base = sh.woff[tc], w = sh.woff[tc + 1] - base;
            if (wt < w) sh.win[wt] = sh.wrq[base + wt];
            if (wt == 0) { sh.w_cur = w; sh.r_cur = sh.rpos[tc]; }
        }
        if (worker) {
            for (uint32_t i = wt; i < np; i += WN) {
                const uint64_t e = __hip_atomic_load(&pin[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t u = lk_t(e);
                if (u == tc) {
                    const bool root = (e & LK_ROOT) != 0;
                    const uint64_t key = e & ~LK_ROOT;
                    if (!root && wg_memo_has(key, sh, memo, cap_mask, probes)) continue;
                    if (!layer_insert(sh, gset, gmask, key, flags)) continue;
                    wg_append(sh, work, W.work_cap, e, flags);
                } else {
                    const uint32_t q = atomicAdd(&sh.npend2, 1u);
                    __hip_atomic_store(&pout[q], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    atomicMin(&sh.t_next, u);
                }
            }
        }
        __syncthreads();
        if (tid == 64) { sh.pend_sel = sel ^ 1; sh.npend = sh.npend2; }
        __syncthreads();
        uint64_t *pcur = pout;
#ifdef JH_ENUM_PROF
        const unsigned long long pf1 = __builtin_amdgcn_s_memtime();
        if (tid == 64) atomicAdd(&g_prof_form, pf1 - pf0);
#endif
        // ---- close it, round by round (what a round appends is the next one):
        // stage the round's configurations with their candidate children, then
        // every worker lane takes one child at a time, so that the memo probes
        // and set inserts of a round are all in flight together
        uint64_t *st_key = (uint64_t *)(jh_lds + WG_STAGE_OFF);
        uint64_t *st_cand = st_key + FL_CHUNK;
        uint32_t *st_pre = (uint32_t *)(st_cand + FL_CHUNK);
        for (;;) {
            const uint32_t ra = sh.head, rb = min(sh.tail, sh.cap_total);
            __syncthreads();
            if (tid == 64) sh.head = rb;
            for (uint32_t c0 = ra; c0 < rb; c0 += FL_CHUNK) {
                const uint32_t nI = min((uint32_t)FL_CHUNK, rb - c0);
                if (worker)
                    for (uint32_t q = wt; q < nI; q += WN) {
                        const uint64_t k = __hip_atomic_load(&work[c0 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~LK_ROOT;
                        const uint64_t c = wg_cands(k, sh);
                        st_key[q] = k; st_cand[q] = c; st_pre[q] = (uint32_t)__popcll(c);
                    }
                __syncthreads();
                if (wid == 1) {
                    // exclusive prefix of the children counts (one wave)
                    uint32_t carry = 0;
                    for (uint32_t b0 = 0; b0 < nI; b0 += 64) {
                        const uint32_t v = b0 + lane < nI ? st_pre[b0 + lane] : 0u;
                        uint32_t x = v;
                        for (int o = 1; o < 64; o <<= 1) {
                            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
                            if (lane >= o) x += y;
                        }
                        if (b0 + lane < nI) st_pre[b0 + lane] = carry + x - v;
                        carry += (uint32_t)readlane((int)x, 63);
                    }
                    if (lane == 0) sh.nchild = carry;
                }
                __syncthreads();
                const uint32_t C = sh.nchild;
                if (worker && !sh.status)
                    for (uint32_t ci = wt; ci < C; ci += WN) {
                        // the staged configuration holding child ci, then its (ci - pre)-th candidate bit
                        uint32_t lo = 0, hi = nI;
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (st_pre[mid] <= ci) lo = mid; else hi = mid;
                        }
                        uint64_t c = st_cand[lo];
                        for (uint32_t n = ci - st_pre[lo]; n > 0; n--) c &= c - 1;
                        wg_child(st_key[lo], (uint32_t)__builtin_ctzll(c), sh, gset, gmask, work, W.work_cap, pcur,
                                 W.pend_cap, memo, cap_mask, probes, flags);
                    }
                __syncthreads();
            }
#ifdef JH_ENUM_PROF
            if (tid == 64) atomicAdd(&g_prof_rounds, 1u);
#endif
            if (sh.status || sh.tail == rb) break;
        }
        __syncthreads();
#ifdef JH_ENUM_PROF
        if (tid == 64) atomicAdd(&g_prof_close, __builtin_amdgcn_s_memtime() - pf1);
#endif
        if (worker)
            for (uint32_t i = wt; i < (uint32_t)ESET; i += WN) es[i] = 0;
        if (sh.status || sh.npend == 0) break;
    }
    if (tid == 64 && W.acc_stats) atomicAdd(&W.acc_stats[6], __builtin_amdgcn_s_memtime() - cw0);
    __syncthreads();
    // new nodes: the work entries without the root mark
    const uint32_t end = worker ? min(sh.tail, sh.cap_total) : 0;
    const uint32_t rec_end = worker ? min(sh.tail, W.work_cap) : 0;     // recorded keys, slack included
    if (worker) {
        uint32_t tmin = 0xFFFFFFFFu, tmax = 0;
        for (uint32_t i = wt; i < end; i += WN) {
            const uint64_t k = __hip_atomic_load(&work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!(k & LK_ROOT)) { tmin = min(tmin, lk_t(k)); tmax = max(tmax, lk_t(k)); }
        }
        for (int o = 32; o > 0; o >>= 1) {
            tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, o));
            tmax = max(tmax, (uint32_t)__shfl_xor((int)tmax, o));
        }
        if (lane == 0) { atomicMin(&sh.tmin_new, tmin); atomicMax(&sh.tmax_new, tmax); }
        if (sh.keep && sh.status == 0) {
            // a spec enumeration's result: its new nodes, for the main to merge
            for (uint32_t i = wt; i < end; i += WN) {
                const uint64_t k = __hip_atomic_load(&work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (k & LK_ROOT) continue;
                sh.keep[atomicAdd(&sh.keep_n, 1u)] = k;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        }
        if (sh.merge && sh.status == 0) {
            uint32_t *bloom = (uint32_t *)(jh_lds + MemoW::OFF_BLOOM);
            for (uint32_t i = wt; i < end; i += WN) {
                const uint64_t k = __hip_atomic_load(&work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (k & LK_ROOT) continue;
                hbm_insert(memo, cap_mask, sh.gen, lk_t(k), lk_s(k), lk_m(k));
                uint32_t h1, h2;
                lk_hash((uint32_t)k, (uint32_t)(k >> 32), h1, h2);
                bloom_set2<MemoW>(bloom, lk_bl(h1), lk_bl(h2));
            }
        }
    }
    // clean-up in two passes: locate every HBM-set slot first (zeroing as we
    // went would cut the probe chains of keys placed after a zeroed slot)
    const bool gu = sh.gset_used != 0;
    if (gu)
        for (uint32_t i = wt; i < rec_end; i += WN) {
            const uint64_t k = __hip_atomic_load(&work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t slot = (k & LK_ROOT) ? ~0u : gset_find(gset, gmask, k);
            __hip_atomic_store(&work[i], (uint64_t)slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    __syncthreads();
    for (uint32_t i = wt; i < rec_end; i += WN) {
        if (gu) {
            const uint32_t slot = (uint32_t)__hip_atomic_load(&work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (slot != ~0u) __hip_atomic_store(&gset[slot], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __hip_atomic_store(&work[i], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (tid == 64 && W.acc_stats) {
        atomicAdd(&W.acc_stats[0], 1ULL);
        atomicAdd(&W.acc_stats[1], (unsigned long long)(end - min(end, sh.n_roots)));
        atomicAdd(&W.acc_stats[sh.status == 0 ? 2 : (sh.status & ENUM_LIVE) ? 3 : 4], 1ULL);
    }
    // every store of this call (merged memo entries, zeroed set and work
    // slots) is complete before any wave goes on: the next call's atomics and
    // the DFS's memo probes must not race a late store (workgroup scope: the
    // waves of a workgroup share this CU's L1)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// All waves (CMD_MERGE): fold a spec result -- the reachable set of a node of
// this workgroup's stack that a helper found dead -- into the DFS memo (HBM
// table + Bloom filter): the nodes not there yet are counted (sh.m_new) with
// their layer range (sh.m_tmin / m_tmax: the merged range the DFS probes).
__device__ void wg_merge(const WgArgs &W, WgShared &sh, int tid, uint64_t *memo, unsigned long long &probes) {
    // the helper published the buffer at agent scope; drop any stale L1 copy
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t cap_mask = W.d.memo_cap - 1;
    uint32_t *bloom = (uint32_t *)(jh_lds + MemoW::OFF_BLOOM);
    const uint32_t n = sh.m_n;
    const uint64_t *src = sh.m_src;
    uint32_t nnew = 0, tmin = 0xFFFFFFFFu, tmax = 0;
    for (uint32_t i = (uint32_t)tid; i < n; i += WG_THREADS) {
        const uint64_t k = src[i];
        if (wg_memo_has(k, sh, memo, cap_mask, probes)) continue;
        hbm_insert(memo, cap_mask, sh.gen, lk_t(k), lk_s(k), lk_m(k));
        uint32_t h1, h2;
        lk_hash((uint32_t)k, (uint32_t)(k >> 32), h1, h2);
        bloom_set2<MemoW>(bloom, lk_bl(h1), lk_bl(h2));
        nnew++;
        tmin = min(tmin, lk_t(k));
        tmax = max(tmax, lk_t(k));
    }
    for (int o = 32; o > 0; o >>= 1) {
        nnew += (uint32_t)__shfl_xor((int)nnew, o);
        tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, o));
        tmax = max(tmax, (uint32_t)__shfl_xor((int)tmax, o));
    }
    if ((tid & 63) == 0) {
        atomicAdd(&sh.m_new, nnew);
        atomicMin(&sh.m_tmin, tmin);
        atomicMax(&sh.m_tmax, tmax);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The takeover's restore, out of line (dfs_acc's registers stay its own):
// the record's configurations into the HBM table and Bloom filter, its frames
// below the ring into the HBM stack (insert index hseq). Returns one past the
// highest restored layer (the theta above which no probe needs HBM).
template <class M>
__device__ __noinline__ uint32_t acc_restore(const uint64_t *hd, uint32_t d, uint32_t h_n, uint32_t ring_lo,
                                             uint32_t hseq, uint64_t *memo, uint32_t cap_mask, uint32_t gen,
                                             uint32_t *bloom, Frame *stack, int lane) {
    const Frame *fsrc = (const Frame *)(hd + 8);
    const ulonglong2 *ent = (const ulonglong2 *)(fsrc + d);
    uint32_t tmx = 0;
    for (uint32_t j = (uint32_t)lane; j < h_n; j += 64) {
        const ulonglong2 e = ent[j];
        const uint32_t et = (uint32_t)(e.y >> 20) & T_MASK, es = (uint32_t)e.y & STATE_MASK;
        hbm_insert(memo, cap_mask, gen, et, es, e.x);
        uint32_t g1, g2;
        lk_hash((uint32_t)e.x, (uint32_t)(e.x >> 32) | (et << 16) | (es << 8) | 0x80000000u, g1, g2);
        bloom_set2<M>(bloom, lk_bl(g1), lk_bl(g2));
        tmx = max(tmx, et + 1);
    }
    for (int o = 32; o > 0; o >>= 1) tmx = max(tmx, (uint32_t)__shfl_xor((int)tmx, o));
    for (uint32_t j = (uint32_t)lane; j < ring_lo; j += 64) {
        Frame fr = fsrc[j];
        fr.pad[0] = hseq; fr.pad[1] = 0;
        stack[j] = fr;
    }
    return tmx;
}

// dfs_lean with the acceleration hooks (see above). Only wave 0 runs it; the
// other waves wait at the workgroup barrier for wg_enum_work.
template <class M>
__device__ int dfs_acc(const WgArgs &W, WgShared &sh, const KeyInfo &K, const char *tb, int key, int lane,
                       uint64_t *memo, Frame *stack, uint64_t *stage, uint64_t *gset, uint64_t *work, char *wtab,
                       uint64_t *pend, long long &inserts, uint32_t &tmax_out, unsigned long long &my_probes,
                       const bool resume) {
    const DfsArgs &A = W.d;
    const OpC *ops = (const OpC *)tb;
    const Lay *lay = (const Lay *)(tb + tblc_ops_bytes(K));
    const uint32_t n_ok = (uint32_t)K.n_ok;
    const int n_ops = K.n_ops;
    const uint32_t cap_mask = A.memo_cap - 1;
    const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
    uint64_t *lmemo = (uint64_t *)(jh_lds + M::OFF_MEMO);
    uint32_t *bloom = (uint32_t *)(jh_lds + M::OFF_BLOOM);
    uint32_t *bcnt = (uint32_t *)(jh_lds + M::OFF_CNT);
    uint8_t *bcnt8 = (uint8_t *)bcnt;
    for (int i = lane; i < M::SLOTS; i += 64) lmemo[i] = 0;
    for (int i = lane; i < M::BKT / 4; i += 64) bcnt[i] = 0;
    for (int i = lane; i < M::BLOOM / 32; i += 64) bloom[i] = 0;
    const uint32_t lb_lo = lane < 32 ? 1u << lane : 0u, lb_hi = lane >= 32 ? 1u << (lane - 32) : 0u;
    uint32_t theta = 0;
    int lcount = 0;

    uint32_t tb0 = 0, drq = 0, dhi = 0;
    auto load_lay = [&](uint32_t base) {
        tb0 = base;
        const uint32_t u = base + (uint32_t)lane;
        if (u < n_ok) { const Lay e = lay[u]; drq = e.rq; dhi = e.hi; }
    };
    auto lay_hi = [&](uint32_t u) -> uint32_t {
        if (u - tb0 >= 64u) load_lay(u >= 32 ? u - 32 : 0);
        return (uint32_t)readlane((int)dhi, (int)(u - tb0));
    };
    int pb = 0;
    uint32_t urq = RQ_EMPTY;
    auto load_up = [&](int base) {
        pb = base;
        const int j = base + lane;
        urq = j < n_ops ? ops[j].rq : RQ_EMPTY;
    };
    // DFS stack ring: frames [ring_lo, depth) in lane registers (lane = depth mod 64);
    // f_seq / f_inc: the frame node's insert index and its last inconclusive size
    uint32_t fm_lo = 0, fm_hi = 0, f_ti = 0, f_s = 0, fr_lo = 0, fr_hi = 0, f_seq = 0, f_inc = 0;

    load_lay(0);
    uint32_t t = 0, tmax = 0, depth = 0, ring_lo = 0;
    uint64_t mask = 0;
    uint32_t s = (uint32_t)A.init_state;
    int verdict = -1;
    uint32_t ins = 0;
    const uint32_t budget = (uint32_t)min<int64_t>(A.budget, 0x7FFFFFFF);
    const uint32_t acc_t = W.acc_t ? W.acc_t : 0x7FFFFFFFu;
    uint32_t next_acc = acc_t;
    uint32_t spec_chk = 0;                             // the next spec-board poll (round 6)
    // a late helper checks its key more often: it races a search that may be about to finish
    const uint32_t chk_step = W.seq_start ? 128u : 1024u;
    uint32_t chk = min(budget, min(acc_t, chk_step));
    uint32_t cur_seq = 0xFFFFFFFFu, cur_inc = 0;      // the root: seq -1
    int l_live = -1;                                   // deepest node known to be live
    uint32_t acc_lo = 1, acc_hi = 0;                   // layers holding merged (HBM) entries
    bool wtab_ready = false, climb = false;
    uint32_t climb_jump = 1;                           // levels the next climb test goes up
    uint32_t n_steps = 0, n_acc = 0;
    int w = (int)(lay_hi(0) >> 6), P = w;
    uint32_t r = lay_hi(0) & 63;
    uint32_t rn = n_ok > 1 ? (lay_hi(1) & 63) : 0;
    uint32_t wrq = lane < w ? ops[lane].rq : RQ_EMPTY;
    load_up(P);
    wave_sync();
    uint32_t ins_saved = 0xFFFFFFFFu;     // a handed-over search's real insert count
    if (resume) {
        // Round 6, the takeover: continue the record phase 2's sequential
        // search saved for this helper (dfs_lean's save: header, frames, every
        // configuration of its memo). As dfs_lean's resume: the memo into the
        // HBM table behind the Bloom filter with theta above every restored
        // layer, the stack into the ring and the HBM stack, then the current
        // configuration is expanded again. The restored frames' insert index is
        // the record's insert count (a node pushed later has a larger one, so a
        // spec result still names one stack node).
        const uint64_t *hd = (const uint64_t *)(A.rs_arena + A.rs_off[key]);
        const uint64_t h_mask = hd[0], h_ts = hd[1], h_dt = hd[2], h_ins = hd[3], h_n = hd[4];
        const uint32_t d = (uint32_t)h_dt;
        if (d <= A.stack_cap && h_n <= (uint64_t)A.memo_cap / 4) {
            const Frame *fsrc = (const Frame *)(hd + 8);
            const uint32_t hseq = (uint32_t)h_ins;
            ring_lo = d > 32 ? d - 32 : 0;
            theta = rflu(acc_restore<M>(hd, d, (uint32_t)h_n, ring_lo, hseq, memo, cap_mask, gen, bloom, stack, lane));
            {
                const uint32_t idx = ring_lo + (((uint32_t)lane - ring_lo) & 63);
                if (idx < d) {
                    const Frame fr = fsrc[idx];
                    fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i;
                    f_s = (uint32_t)fr.s; fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32);
                    f_seq = hseq; f_inc = 0;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            wave_sync();
            depth = d;
            mask = h_mask;
            s = (uint32_t)(h_ts >> 32);
            ins = hseq;
            cur_seq = hseq;
            chk = min(budget, ins);                  // the next insert runs the checks
            next_acc = ins + acc_t;
            spec_chk = ins;
            // the window forward from layer 0 to the record's layer
            const uint32_t nt = (uint32_t)h_ts;
            for (uint32_t u = t; u < nt; u++) {
                const uint32_t ru = u == t ? r : (lay_hi(u) & 63);
                const uint32_t shv = (uint32_t)wave_shl1((int)wrq);
                if (lane >= (int)ru) wrq = shv;
                w--;
                if (lane == w) wrq = RQ_EMPTY;
                const int c = (int)(lay_hi(u + 1) >> 6);
                if (c > 0) {
                    if (P < pb || P + c > pb + 64) load_up(c <= 32 && P >= 32 ? P - 32 : P);
                    for (int kk = 0; kk < c; kk++) {
                        const uint32_t x = (uint32_t)readlane((int)urq, P - pb + kk);
                        if (lane == w + kk) wrq = x;
                    }
                    w += c; P += c;
                }
            }
            t = nt;
            tmax = max((uint32_t)(h_dt >> 32), t);
            r = lay_hi(t) & 63;
            rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        }
    }
    const ulonglong2 *B = (const ulonglong2 *)lmemo;
    uint64_t absent = 0, nm_r = 0;
    uint32_t u_r = 0, klo = 0, khi = 0, b1 = 0, b2 = 0, n1 = 0, n2 = 0, h1 = 0, h2 = 0, nvl = 0;
    auto child_keys = [&]() {
        u_r = t; nm_r = 0;
        if ((absent >> r) & 1) {
            uint64_t nm = drop_bit(mask, r);
            uint32_t u = t + 1;
            if (u >= n_ok) nm = 0;
            else if ((nm >> rn) & 1) {
                uint32_t ru = rn;
                for (;;) {
                    nm = drop_bit(nm, ru);
                    u++;
                    if (u >= n_ok) { nm = 0; break; }
                    ru = lay_hi(u) & 63;
                    if (!((nm >> ru) & 1)) break;
                }
            }
            u_r = u; nm_r = nm;
        }
        nvl = wrq >> 16;
        const bool is_r = lane == (int)r;
        const uint32_t hi_a = (uint32_t)(mask >> 32) | (t << 16) | 0x80000000u;
        const uint32_t hi_r = (uint32_t)(nm_r >> 32) | (u_r << 16) | 0x80000000u;
        klo = is_r ? (uint32_t)nm_r : ((uint32_t)mask | lb_lo);
        khi = (is_r ? hi_r : (hi_a | lb_hi)) | (nvl << 8);
        lk_hash(klo, khi, h1, h2);
        lk_bkts<M>(h1, h2, b1, b2);
    };
    // Accelerate the open node at depth d (ring_lo <= d <= depth, or d == depth):
    // 0 dead (merged unless d == 0), 1 live, 2 inconclusive.
    uint32_t acc_new = 0, acc_tmax = 0, acc_tmin = 0;
    auto accel = [&](uint32_t d) -> int {
        const uint32_t seq_d = d == depth ? cur_seq : (uint32_t)readlane((int)f_seq, (int)(d & 63));
        const uint32_t below = ins - seq_d;
        int64_t cap = max<int64_t>(ACC_CAPMIN, (int64_t)ACC_CAPF * below);
        cap = min<int64_t>(cap, (int64_t)budget - ins + 1);
        const uint32_t n_roots = depth - d + 1;
        cap = min<int64_t>(cap, (int64_t)W.work_cap - 16384 - n_roots);
        if (n_roots > W.pend_cap) return 2;
        if (cap <= 0) return 2;
        if (!wtab_ready) {
            if (lane == 0) sh.wtab_key = -1;        // (a spec job's cached table is gone)
            uint32_t *woff = (uint32_t *)wtab;
            uint32_t *wrqt = (uint32_t *)(wtab + (((n_ok + 1) * 4 + 255) & ~255u));
            uint8_t *rp = (uint8_t *)((char *)wrqt + ((n_ok * 40 * 4 + 255) & ~255u));
            wtab_build(K, tb, lane, woff, wrqt, rp);
            if (lane == 0) { sh.woff = woff; sh.wrq = wrqt; sh.rpos = rp; }
            wtab_ready = true;
        }
        // roots: the frames' nodes at depths [d, depth) and the current node,
        // as pending entries marked LK_ROOT (expanded, not counted)
        {
            const uint32_t fd = ring_lo + (((uint32_t)lane - ring_lo) & 63);
            if (fd >= d && fd < depth)
                __hip_atomic_store(&pend[fd - d], lk_make(f_ti >> 6, f_s, ((uint64_t)fm_hi << 32) | fm_lo) | LK_ROOT,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lane == 0)
                __hip_atomic_store(&pend[depth - d], lk_make(t, s, mask) | LK_ROOT, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const uint32_t t_x = d == depth ? t : ((uint32_t)readlane((int)f_ti, (int)(d & 63)) >> 6);
        if (lane == 0) {
            sh.cmd = CMD_ENUM; sh.merge = d > 0 ? 1 : 0; sh.status = 0;
            sh.n_roots = n_roots; sh.n_ok = n_ok; sh.theta = theta; sh.acc_lo = acc_lo; sh.acc_hi = acc_hi;
            sh.gen = gen; sh.cap_total = n_roots + (uint32_t)cap;
            sh.head = 0; sh.tail = 0; sh.active = 0; sh.tmin_new = 0xFFFFFFFFu; sh.tmax_new = 0;
            sh.t_next = t_x; sh.npend = n_roots; sh.pend_sel = 0; sh.gset_used = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();                    // the helpers wait here (k_lin_wg)
        const unsigned long long c0 = __builtin_amdgcn_s_memtime();
        unsigned long long *d8 = A.dbg && n_acc < 31 ? A.dbg + 256 * (size_t)blockIdx.x + 8 * n_acc : nullptr;
        if (d8 && lane == 0) {
            // JH_DEBUG=3 trace: one record per enumeration (the workgroup's first 31)
            d8[0] = key; d8[1] = d; d8[2] = depth; d8[3] = n_roots; d8[4] = (unsigned long long)cap;
            d8[5] = 99; d8[6] = 0; d8[7] = ins;
        }
        wg_enum_work(W, sh, lane, gset, work, memo, pend, my_probes);
        const int st = sh.status;
        if (d8 && lane == 0) { d8[5] = st; d8[6] = sh.tail; }
        if (W.acc_stats && lane == 0) atomicAdd(&W.acc_stats[5], __builtin_amdgcn_s_memtime() - c0);
        n_acc++;
        if (st & ENUM_LIVE) return 1;
        if (st) return 2;
        acc_new = sh.tail - n_roots;
        acc_tmax = sh.tmax_new; acc_tmin = sh.tmin_new;
        return 0;
    };

expand:
    if (W.spec && ins >= spec_chk) {
        // Round 6, the spec board (SpecSlot), every SPEC_CHK inserts, here where
        // the children's keys are not live yet: this search's results first.
        spec_chk = ins + SPEC_CHK;
        SpecSlot *SB = W.spec;
        const int st = __hip_atomic_load(&SB[lane].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const bool mine = st >= SPEC_DEAD && st <= SPEC_INC && SB[lane].key == key;
        const uint32_t sd = mine ? SB[lane].depth : 0u, sq = mine ? SB[lane].seq : 0u;
        const uint32_t fsq = (uint32_t)__shfl((int)f_seq, (int)(sd & 63));
        // a node below the register ring: its frame in the HBM stack
        const uint32_t hsq = mine && sd >= 1 && sd < ring_lo ? stack[sd].pad[0] : 0xFFFFFFFFu;
        // still on the stack: same depth, same insert index
        const bool on = mine && sd >= 1 && sd <= depth &&
                        (sd == depth ? cur_seq : sd >= ring_lo ? fsq : hsq) == sq;
        int lmax = on && st == SPEC_LIVE ? (int)sd : -1;          // live: it and its ancestors
        for (int o = 32; o > 0; o >>= 1) lmax = max(lmax, __shfl_xor(lmax, o));
        if (lmax > l_live) l_live = lmax;
        const bool dd = on && st == SPEC_DEAD && (int)sd > l_live;
        uint32_t dmin = dd ? sd : 0xFFFFFFFFu;                      // the shallowest dead one
        for (int o = 32; o > 0; o >>= 1) dmin = min(dmin, (uint32_t)__shfl_xor((int)dmin, o));
        const uint64_t pm = ballot(dd && sd == dmin);
        const int pk = pm ? __builtin_ctzll(pm) : -1;
        if (mine && lane != pk)
            __hip_atomic_store(&SB[lane].state, SPEC_FREE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (pk >= 0) {
            // merge the dead node's reachable set (every wave: wg_merge) and pop it
            const uint32_t rn = (uint32_t)readlane((int)(lane == pk ? SB[lane].n : 0u), pk);
            const int rh = readlane(lane == pk ? SB[lane].helper : 0, pk);
            if (lane == 0) {
                sh.cmd = CMD_MERGE; sh.m_src = W.spec_res + (size_t)rh * W.spec_res_cap; sh.m_n = rn;
                sh.m_new = 0; sh.m_tmin = 0xFFFFFFFFu; sh.m_tmax = 0;
                sh.theta = theta; sh.acc_lo = acc_lo; sh.acc_hi = acc_hi; sh.gen = gen; sh.nomemo = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            wg_merge(W, sh, lane, memo, my_probes);
            if (lane == pk)
                __hip_atomic_store(&SB[pk].state, SPEC_FREE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t mnew = sh.m_new;
            if (lane == 0) {
                atomicAdd((unsigned long long *)W.spec_q, (unsigned long long)mnew);
                atomicAdd(&W.spec_q[2], 1);
            }
            ins += mnew;
            if (ins > budget) { ins = budget; verdict = JH_UNKNOWN; goto done; }
            if (mnew) {
                tmax = max(tmax, sh.m_tmax);
                acc_lo = acc_lo > acc_hi ? sh.m_tmin : min(acc_lo, sh.m_tmin);
                acc_hi = max(acc_hi, sh.m_tmax);
            }
            next_acc = ins + acc_t;
            chk = min(budget, min(ins + chk_step, next_acc));
            depth = dmin;
            // a node below the register ring: the ring is empty down to it, the
            // pop refills it from the HBM stack (whose frames below ring_lo are
            // the current ones)
            if (dmin < ring_lo) ring_lo = dmin;
            goto pop;                  // pops node dmin
        }
        // New posts: the open nodes within spec_dist levels of the current
        // one (the register ring), below the deepest known live node, with
        // spec_min inserts below them and never posted (or 4x as many since),
        // deepest first, into free slots; posting counts as an attempt (inc)
        uint64_t freem = ballot(st == SPEC_FREE || mine);
        const uint32_t dlo_all = max(max(1u, (uint32_t)(l_live + 1)), depth > W.spec_dist ? depth - W.spec_dist : 0u);
        const uint32_t dlo = max(ring_lo, dlo_all);
        auto elig = [&](uint32_t sqv, uint32_t inc) {
            const uint32_t b = ins - sqv;
            return b >= W.spec_min && (inc == 0 || b >= 4 * inc);
        };
        auto post = [&](uint32_t d, uint64_t cfgk, uint32_t sqv) -> bool {
            while (freem) {
                const int sl = __builtin_ctzll(freem);
                freem &= freem - 1;
                int ok = 0;
                if (lane == 0) {
                    int exp = SPEC_FREE;
                    ok = __hip_atomic_compare_exchange_strong(&SB[sl].state, &exp, SPEC_BUSY, __ATOMIC_ACQUIRE,
                                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (ok) {
                        SB[sl].key = key; SB[sl].depth = d; SB[sl].seq = sqv; SB[sl].cfg = cfgk;
                        SB[sl].cap = min(W.spec_res_cap - 1, max(8192u, W.spec_mult * (ins - sqv)));
                        SB[sl].n = 0; SB[sl].helper = -1;
                        __hip_atomic_store(&SB[sl].state, SPEC_POSTED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                if (readlane(ok, 0)) return true;
            }
            return false;
        };
        int nposted = 0;
        if (depth >= dlo && depth >= 1 && elig(cur_seq, cur_inc) && post(depth, lk_make(t, s, mask), cur_seq)) {
            cur_inc = ins - cur_seq;
            nposted++;
        }
        {
            const uint32_t fd = ring_lo + (((uint32_t)lane - ring_lo) & 63);
            const uint64_t cm = ballot(fd < depth && fd >= dlo && elig(f_seq, f_inc));
            const uint32_t rs = ring_lo & 63;
            uint64_t rot = rs ? ((cm >> rs) | (cm << (64 - rs))) : cm;
            while (rot && freem && nposted < SPEC_PER_CHECK) {
                const int q = 63 - __builtin_clzll(rot);
                rot &= ~(1ULL << q);
                const uint32_t d = ring_lo + (uint32_t)q;
                const int ln = (int)(d & 63);
                const uint32_t qs = (uint32_t)readlane((int)f_seq, ln);
                const uint64_t ck = lk_make((uint32_t)readlane((int)f_ti, ln) >> 6, (uint32_t)readlane((int)f_s, ln),
                                            ((uint64_t)(uint32_t)readlane((int)fm_hi, ln) << 32) |
                                            (uint32_t)readlane((int)fm_lo, ln));
                if (!post(d, ck, qs)) break;
                if (lane == ln) f_inc = ins - qs;
                nposted++;
            }
        }
        if (freem && nposted < SPEC_PER_CHECK && ring_lo > dlo_all) {
            // the nodes below the ring (a dead subtree deeper than 64 levels:
            // rank 4's key 1631 has one of 95), from the HBM stack, deepest first
            const uint32_t nh = min(64u, ring_lo - dlo_all);
            const uint32_t hd = ring_lo - 1 - (uint32_t)lane;
            Frame fr{};
            if ((uint32_t)lane < nh) fr = stack[hd];
            const uint64_t hm = ballot((uint32_t)lane < nh && elig(fr.pad[0], fr.pad[1]));
            uint64_t hr = hm;
            while (hr && freem && nposted < SPEC_PER_CHECK) {
                const int q = __builtin_ctzll(hr);
                hr &= hr - 1;
                const uint32_t d = ring_lo - 1 - (uint32_t)q;
                const uint32_t qs = (uint32_t)readlane((int)fr.pad[0], q);
                const uint64_t fm = ((uint64_t)(uint32_t)readlane((int)(uint32_t)(fr.mask >> 32), q) << 32) |
                                    (uint32_t)readlane((int)(uint32_t)fr.mask, q);
                const uint64_t ck = lk_make((uint32_t)readlane((int)fr.t_i, q) >> 6, (uint32_t)readlane(fr.s, q), fm);
                if (!post(d, ck, qs)) break;
                if (lane == q) stack[d].pad[1] = ins - qs;
                nposted++;
            }
        }
    }
    if (++n_steps > (1u << 28)) {       // watchdog: far beyond any budget's step count
        if (lane == 0) atomicOr(A.flags, 128);
        verdict = JH_UNKNOWN;
        goto done;
    }
    {
        const uint32_t req = wrq & 0xFFFF;
        absent = (ballot(req == s) | ballot(req == RQ_ANY)) & ~mask;
    }
    if (!absent) goto pop;
    child_keys();
    {
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        const uint64_t k = ((uint64_t)khi << 32) | klo;
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
        __builtin_amdgcn_sched_barrier(0);
        const ulonglong2 x0 = B[2 * a1], x1 = B[2 * a1 + 1];
        const ulonglong2 y0 = B[2 * a2], y1 = B[2 * a2 + 1];
        const uint64_t hit = ballot(x0.x == k) | ballot(x0.y == k) | ballot(x1.x == k) | ballot(x1.y == k) |
                             ballot(y0.x == k) | ballot(y0.y == k) | ballot(y1.x == k) | ballot(y1.y == k);
        absent &= ~hit;
        // children that may sit in HBM: below theta, or in a merged layer range
        const bool t_slow = t < theta || (t >= acc_lo && t <= acc_hi);
        const bool r_slow = u_r < theta || (u_r >= acc_lo && u_r <= acc_hi);
        if ((t_slow || r_slow) && absent) {
            uint64_t low = t_slow ? absent : 0ULL;
            low = r_slow ? (low | (absent & (1ULL << r))) : (low & ~(1ULL << r));
            const uint32_t kt = khi >> 16 & 0x7FFF, ks = (khi >> 8) & 0xFF;
            const uint64_t km = k & ((1ULL << 40) - 1);
            const bool maybe = ((low >> lane) & 1) && bloom_test2<M>(bloom, lk_bl(h1), lk_bl(h2));
            bool found = false;
            if (maybe) found = (hbm_probe(memo, cap_mask, gen, kt, ks, km, my_probes) >> 32) == 0;
            absent &= ~ballot(found);
        }
    }
    if (!absent) goto pop;

insert:
    {
        if (ins >= chk) {
            if (ins >= budget) { verdict = JH_UNKNOWN; goto done; }
            if (A.claim) {
                // racing k_lin_bfs: stop if it settled this key first; a late
                // helper also stops once the sequential search has handed the
                // key to phase 3 (which settles it)
                int c = 0;
                if (lane == 0) {
                    c = __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (W.seq_start && __hip_atomic_load(&W.seq_start[key], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) == SEQ_HANDED)
                        c = 1;
                }
                if (readlane(c, 0)) { verdict = JH_CANCELLED; goto done; }
            }
            if (ins >= next_acc) {
                next_acc = ins + acc_t;
                // the deepest open node with >= ACC_T/2 inserts below it, not known live
                auto ok_node = [&](uint32_t sq, uint32_t inc) {
                    const uint32_t b = ins - sq;
                    return b >= acc_t / 2 && (inc == 0 || b >= 2 * inc);
                };
                int64_t d = -1;
                if ((int)depth > l_live && ok_node(cur_seq, cur_inc)) d = depth;
                else {
                    const uint32_t q = ((uint32_t)lane - ring_lo) & 63, fd = ring_lo + q;
                    const uint64_t bm = ballot(fd < depth && (int)fd > l_live && ok_node(f_seq, f_inc));
                    if (bm) {
                        // rotate so bit q = frame ring_lo + q; take the highest
                        const uint32_t rs = ring_lo & 63;
                        const uint64_t rot = rs ? ((bm >> rs) | (bm << (64 - rs))) : bm;
                        d = (int64_t)ring_lo + (63 - __builtin_clzll(rot));
                    }
                }
                if (d >= 0) {
                    const int res = accel((uint32_t)d);
                    if (res == 0) {
                        ins += acc_new;
                        tmax = max(tmax, acc_tmax);
                        if (ins > budget) { ins = budget; verdict = JH_UNKNOWN; goto done; }
                        if (d == 0) { verdict = JH_INVALID; goto done; }
                        if (acc_new) {
                            acc_lo = acc_lo > acc_hi ? acc_tmin : min(acc_lo, acc_tmin);
                            acc_hi = max(acc_hi, acc_tmax);
                        }
                        next_acc = ins + acc_t;
                        depth = (uint32_t)d;
                        climb = true; climb_jump = 1;
                        goto pop;
                    }
                    if (res == 1) l_live = (int)d;
                    else {
                        const uint32_t b = ins - (d == depth ? cur_seq : (uint32_t)readlane((int)f_seq, (int)(d & 63)));
                        if ((uint32_t)d == depth) cur_inc = b;
                        else if (lane == (int)(d & 63)) f_inc = b;
                    }
                }
            }
            chk = min(budget, min(ins + chk_step, next_acc));
        }
        const int i = __builtin_ctzll(absent);
        const uint32_t myseq = ins;
        ins++;
        const uint32_t ns = (uint32_t)readlane((int)nvl, i);
        const bool to_r = (uint32_t)i == r;
        const uint32_t nt = to_r ? u_r : t;
        {
            const bool pick1 = n1 <= n2;
            const uint32_t bs = pick1 ? b1 : b2, nsl = pick1 ? n1 : n2;
            const uint64_t full_m = ballot(nsl >= 4);
            if (!((full_m >> i) & 1)) {
                if (lane == i) {
                    lmemo[4 * bs + nsl] = ((uint64_t)khi << 32) | klo;
                    bcnt8[bs] = (uint8_t)(nsl + 1);
                }
                if (++lcount >= M::EVICT) {
                    const uint64_t er = memo_evict<M>(lmemo, bcnt, bloom, memo, stage, cap_mask, gen, nt, theta, lane);
                    lcount = rfl((int)(uint32_t)er);
                    theta = rflu((uint32_t)(er >> 32));
                }
            } else {
                const uint64_t nmask = to_r ? nm_r : (mask | (1ULL << i));
                if (lane == i) {
                    hbm_insert(memo, cap_mask, gen, nt, ns, nmask);
                    bloom_set2<M>(bloom, lk_bl(h1), lk_bl(h2));
                }
                theta = max(theta, nt + 1);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
        }
        if (depth - ring_lo == 64) {
            const uint32_t kk = ((uint32_t)lane - ring_lo) & 63;
            if (kk < 32) {
                Frame fr;
                fr.mask = ((uint64_t)fm_hi << 32) | fm_lo; fr.t_i = f_ti; fr.s = (int32_t)f_s;
                fr.rest = ((uint64_t)fr_hi << 32) | fr_lo; fr.pad[0] = f_seq; fr.pad[1] = f_inc;
                stack[ring_lo + kk] = fr;
            }
            ring_lo += 32;
        }
        {
            const uint64_t nrest = absent & (absent - 1);
            const bool me = lane == (int)(depth & 63);
            fm_lo = me ? (uint32_t)mask : fm_lo;
            fm_hi = me ? (uint32_t)(mask >> 32) : fm_hi;
            f_ti = me ? ((t << 6) | (uint32_t)i) : f_ti;
            f_s = me ? s : f_s;
            fr_lo = me ? (uint32_t)nrest : fr_lo;
            fr_hi = me ? (uint32_t)(nrest >> 32) : fr_hi;
            f_seq = me ? cur_seq : f_seq;
            f_inc = me ? cur_inc : f_inc;
        }
        depth++;
        s = ns;
        cur_seq = myseq; cur_inc = 0;
        if (!to_r) {
            mask |= 1ULL << i;
            goto expand;
        }
        mask = nm_r;
        if (nt >= n_ok) { t = nt; tmax = max(tmax, t); verdict = JH_VALID; goto done; }
        for (uint32_t u = t; u < nt; u++) {
            const uint32_t ru = u == t ? r : (lay_hi(u) & 63);
            const uint32_t sh2 = (uint32_t)wave_shl1((int)wrq);
            if (lane >= (int)ru) wrq = sh2;
            w--;
            if (lane == w) wrq = RQ_EMPTY;
            const int c = (int)(lay_hi(u + 1) >> 6);
            if (c > 0) {
                if (P < pb || P + c > pb + 64) load_up(c <= 32 && P >= 32 ? P - 32 : P);
                for (int kk = 0; kk < c; kk++) {
                    const uint32_t x = (uint32_t)readlane((int)urq, P - pb + kk);
                    if (lane == w + kk) wrq = x;
                }
                w += c; P += c;
            }
        }
        t = nt;
        tmax = max(tmax, t);
        r = lay_hi(t) & 63;
        rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        goto expand;
    }

pop:
    if (depth == ring_lo) {
        if (depth == 0) { verdict = JH_INVALID; goto done; }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t lo = depth >= 32 ? depth - 32 : 0;
        const uint32_t kk = ((uint32_t)lane - lo) & 63;
        if (kk < depth - lo) {
            const Frame fr = stack[lo + kk];
            fm_lo = (uint32_t)fr.mask; fm_hi = (uint32_t)(fr.mask >> 32); f_ti = fr.t_i; f_s = (uint32_t)fr.s;
            fr_lo = (uint32_t)fr.rest; fr_hi = (uint32_t)(fr.rest >> 32); f_seq = fr.pad[0]; f_inc = fr.pad[1];
        }
        ring_lo = lo;
    }
    depth--;
    {
        const int ln = (int)(depth & 63);
        absent = ((uint64_t)(uint32_t)readlane((int)fr_hi, ln) << 32) | (uint32_t)readlane((int)fr_lo, ln);
        const uint32_t pt = (uint32_t)readlane((int)f_ti, ln) >> 6;
        mask = ((uint64_t)(uint32_t)readlane((int)fm_hi, ln) << 32) | (uint32_t)readlane((int)fm_lo, ln);
        s = (uint32_t)readlane((int)f_s, ln);
        cur_seq = (uint32_t)readlane((int)f_seq, ln);
        cur_inc = (uint32_t)readlane((int)f_inc, ln);
        if (pt != t) {
            for (uint32_t u = t; u > pt; u--) {
                const int c = (int)(lay_hi(u) >> 6);
                w -= c; P -= c;
                if (lane >= w) wrq = RQ_EMPTY;
                const uint32_t h = lay_hi(u - 1);
                const int ru = (int)(h & 63);
                const uint32_t sh2 = (uint32_t)wave_shr1((int)wrq);
                if (lane > ru) wrq = sh2;
                const uint32_t x = (uint32_t)readlane((int)drq, (int)(u - 1 - tb0));
                if (lane == ru) wrq = x;
                w++;
            }
            t = pt;
            r = lay_hi(t) & 63;
            rn = t + 1 < n_ok ? (lay_hi(t + 1) & 63) : 0;
        }
    }
    if (climb) {
        // After a dead node, test its ancestors at once, climbing 1, 2, 4, ...
        // levels per success (an invalid key reaches its root in a few
        // steps); a live node ends the climb, after a live far ancestor the
        // climb restarts one level at a time from the current node.
        climb = false;
        for (;;) {
            uint32_t dt = depth >= climb_jump - 1 ? depth - (climb_jump - 1) : 0;
            dt = max(dt, max(ring_lo, (uint32_t)(l_live + 1)));
            if ((int)dt <= l_live || dt > depth) break;
            const int res = accel(dt);
            if (res == 0) {
                ins += acc_new;
                tmax = max(tmax, acc_tmax);
                if (ins > budget) { ins = budget; verdict = JH_UNKNOWN; goto done; }
                if (dt == 0) { verdict = JH_INVALID; goto done; }
                if (acc_new) {
                    acc_lo = acc_lo > acc_hi ? acc_tmin : min(acc_lo, acc_tmin);
                    acc_hi = max(acc_hi, acc_tmax);
                }
                next_acc = ins + acc_t;
                chk = min(budget, min(ins + chk_step, next_acc));
                climb = true;
                climb_jump = min(climb_jump * 2, 64u);
                depth = dt;
                goto pop;          // pops node dt (pop decrements depth)
            }
            if (res == 1) {
                l_live = (int)dt;
                if (dt < depth && climb_jump > 1) { climb_jump = 1; continue; }
            } else {
                const uint32_t b = ins - (dt == depth ? cur_seq : (uint32_t)readlane((int)f_seq, (int)(dt & 63)));
                if (dt == depth) cur_inc = b;
                else if (lane == (int)(dt & 63)) f_inc = b;
            }
            climb_jump = 1;
            break;
        }
        chk = min(budget, min(ins + chk_step, next_acc));
    }
    if (!absent) goto pop;
    child_keys();
    {
        const bool cl = (absent >> lane) & 1;
        const uint32_t a1 = cl ? b1 : 0u, a2 = cl ? b2 : 0u;
        n1 = bcnt8[a1]; n2 = bcnt8[a2];
    }
    goto insert;

done:
    inserts = ins;
    tmax_out = tmax;
    return verdict;
}

// Late helpers of phase 2 (k_lin_wg in helper mode, a few CUs beside the
// sequential search and the BFS): a workgroup takes the unclaimed LEAN key the
// sequential search has been on longest, once that is more than late_ticks,
// and races it with the workgroup engine (exact, so whoever settles first
// writes the same verdict). That is the valid key with a huge reachable set
// (too large for the BFS) and a long backtracking DFS, which otherwise holds
// the whole step on one wave. Sets sh.key (-1: the sequential search has
// left its queue, or the helper has waited HELPER_MAX_TICKS: done).
constexpr unsigned long long HELPER_MAX_TICKS = 500000000ULL;   // 5 s of s_memrealtime (100 MHz)
#ifndef JH_HELP_BY_ORDER
#define JH_HELP_BY_ORDER 0
#endif
// Round 6: a late helper claims a posted spec job (wave 0): the smallest cap
// first, once the main has released this helper's last dead result (its
// buffer). Sets sh.key = -4 (a job) or -3 (lost a race: scan again).
__device__ void spec_try_claim(const WgArgs &W, WgShared &sh, int tid) {
    const DfsArgs &A = W.d;
    if (!(W.spec && sh.key == -2 && tid < 64)) return;
    SpecSlot *SB = W.spec;
    const int lane = tid;
    bool busy = false;
    const int rs = sh.res_slot;
    if (rs >= 0)
        busy = __hip_atomic_load(&SB[rs].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == SPEC_DEAD &&
               SB[rs].helper == (int)blockIdx.x;
    if (busy) return;
    const int st = __hip_atomic_load(&SB[lane].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const int k = SB[lane].key;
    const bool cand = st == SPEC_POSTED && k >= 0 &&
                      !__hip_atomic_load(&A.claim[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long c = cand ? ((unsigned long long)SB[lane].cap << 8) | (unsigned)lane : ~0ULL;
    for (int o = 32; o > 0; o >>= 1) c = min(c, (unsigned long long)__shfl_xor(c, o));
    if (c != ~0ULL && lane == 0) {
        const int sl = (int)(c & 255);
        int exp = SPEC_POSTED;
        if (__hip_atomic_compare_exchange_strong(&SB[sl].state, &exp, SPEC_CLAIMED, __ATOMIC_ACQUIRE,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            sh.res_slot = -1;
            sh.spec_slot = sl;
            sh.key = -4;
        } else {
            sh.key = -3;
        }
    }
}

__device__ void wg_helper_pick(const WgArgs &W, WgShared &sh, int tid, unsigned long long t_enter) {
    const DfsArgs &A = W.d;
    for (;;) {
        if (tid == 0) {
            sh.pick = ~0ULL;
            sh.cmd = 0;
            const int waves = W.seq_waves_dev ? ld_agent(W.seq_waves_dev) : W.seq_waves;
            // streaming: the sequential search's waves may all be idle
            // (left the queue) before phase 1 has finished deferring
            const bool more = A.live_n && !p1_finished(A.p1_done, A.p1_tot);
            // (round 6: while a helper still runs a key -- one it took over from
            // a sequential wave that has left -- the others stay to serve its board)
            const bool over = (!more && __hip_atomic_load(W.seq_exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= waves &&
                               !(W.mains_live && __hip_atomic_load(W.mains_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0)) ||
                              __builtin_amdgcn_s_memrealtime() - t_enter > HELPER_MAX_TICKS;
            sh.key = over ? -1 : -2;
            sh.n_live = A.live_n ? ld_agent(A.live_n) : A.n_list;
        }
        __syncthreads();
        if (sh.key == -1) return;
        // a server (JH_SPEC_SERVERS, tuning builds) takes spec jobs only
        const bool server = W.spec && (int)blockIdx.x >= W.n_mains;
        if (W.spec_first || server) {
            // spec jobs before keys of its own (JH_LIN_SPEC_FIRST)
            spec_try_claim(W, sh, tid);
            __syncthreads();
            if (sh.key == -4) return;
            if (sh.key == -3) continue;
        }
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        const int n_list = server ? 0 : sh.n_live;
        for (int i = tid; i < n_list; i += WG_THREADS) {
            const int key = A.live_n ? ld_agent(&A.list[i]) : A.list[i];
            if (key < 0) continue;
            const unsigned long long s = __hip_atomic_load(&W.seq_start[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (s == 0 || s == SEQ_HANDED || s > now || now - s < W.late_ticks) continue;
            if (__hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                __hip_atomic_load(&W.taken[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                continue;
            const unsigned long long run = min(now - s, (1ULL << 40) - 1);
            // JH_HELP_BY_ORDER: the first key in the list's order (least
            // phase-1 progress first) among those past the delay; else the
            // key the sequential search has been on longest
            atomicMin(&sh.pick, JH_HELP_BY_ORDER ? (unsigned long long)i
                                                 : (((1ULL << 40) - 1 - run) << 24) | (unsigned long long)i);
        }
        __syncthreads();
        if (tid == 0 && sh.pick != ~0ULL) {
            const int i = (int)(sh.pick & ((1u << 24) - 1));
            const int key = A.live_n ? ld_agent(&A.list[i]) : A.list[i];
            sh.key = atomicCAS(&W.taken[key], 0, 1) == 0 ? key : -3;
        }
        __syncthreads();
        if (sh.key >= 0) return;
        if (!(W.spec_first || server)) spec_try_claim(W, sh, tid);
        __syncthreads();
        if (sh.key == -4) return;
        if (sh.key == -2)
            for (int k = 0; k < 16; k++) __builtin_amdgcn_s_sleep(127);   // ~50 us between scans
        __syncthreads();
    }
}

// Round 6: a late helper's spec job (wave 0 with the other waves in
// wg_enum_work): the posted node's whole reachable set, no memo, up to the
// slot's cap; the result goes to the slot (dead: the new nodes in this
// helper's buffer, which stays the main's until it frees the slot).
__device__ void spec_enum(const WgArgs &W, WgShared &sh, int lane, char *wtab, uint64_t *gset, uint64_t *work,
                          uint64_t *memo, uint64_t *pend, unsigned long long &probes) {
    const DfsArgs &A = W.d;
    SpecSlot *S = W.spec + sh.spec_slot;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int key = S->key;
    const uint64_t cfg = S->cfg;
    const uint32_t cap = S->cap;
    if (sh.wtab_key != key) {
        const KeyMeta mt = A.meta[key];
        KeyInfo K;
        K.n_ops = mt.n_ops; K.n_ok = mt.n_ok; K.sumW = mt.pad; K.s0 = 0; K.s1 = 0;
        const uint32_t n_ok = (uint32_t)K.n_ok;
        uint32_t *woff = (uint32_t *)wtab;
        uint32_t *wrqt = (uint32_t *)(wtab + (((n_ok + 1) * 4 + 255) & ~255u));
        uint8_t *rp = (uint8_t *)((char *)wrqt + ((n_ok * 40 * 4 + 255) & ~255u));
        wtab_build(K, A.tables + mt.off, lane, woff, wrqt, rp);
        if (lane == 0) { sh.woff = woff; sh.wrq = wrqt; sh.rpos = rp; sh.wtab_key = key; sh.n_ok = n_ok; }
    }
    uint32_t c = min(cap, W.spec_res_cap - 1);
    c = min(c, W.work_cap - 16384u - 2u);
    if (lane == 0) {
        __hip_atomic_store(&pend[0], cfg | LK_ROOT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        sh.n_ok = (uint32_t)A.meta[key].n_ok;
        sh.cmd = CMD_ENUM; sh.merge = 0; sh.status = 0; sh.key = key;
        sh.n_roots = 1; sh.theta = 0; sh.acc_lo = 1; sh.acc_hi = 0; sh.gen = 0;
        sh.cap_total = 1 + c;
        sh.head = 0; sh.tail = 0; sh.active = 0; sh.tmin_new = 0xFFFFFFFFu; sh.tmax_new = 0;
        sh.t_next = lk_t(cfg); sh.npend = 1; sh.pend_sel = 0; sh.gset_used = 0;
        sh.keep = W.spec_res + (size_t)blockIdx.x * W.spec_res_cap; sh.keep_n = 0;
        sh.nomemo = 1; sh.abort_state = &S->state;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();                        // the other waves join wg_enum_work
    wg_enum_work(W, sh, lane, gset, work, memo, pend, probes);
    const int st = sh.status;
    const int res = st == 0 ? SPEC_DEAD : (st & ENUM_LIVE) ? SPEC_LIVE : SPEC_INC;
    if (lane == 0) {
        atomicAdd(&W.spec_q[3], 1);
        if (res == SPEC_DEAD) { S->n = sh.keep_n; S->helper = (int)blockIdx.x; atomicAdd(&W.spec_q[4], 1); }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        int exp = SPEC_CLAIMED;
        if (__hip_atomic_compare_exchange_strong(&S->state, &exp, res, __ATOMIC_RELEASE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            if (res == SPEC_DEAD) sh.res_slot = sh.spec_slot;
        } else {
            // stale: the main has left (or moved on); the slot is free again
            __hip_atomic_store(&S->state, SPEC_FREE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        sh.keep = nullptr; sh.nomemo = 0; sh.abort_state = nullptr;
        sh.cmd = CMD_DONE;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();                        // releases the other waves
}

// Round 6: a main leaving its key gives back every slot of it: posted ones
// freed, claimed ones marked stale (their helper stops and frees them),
// results freed.
__device__ void spec_release(const WgArgs &W, int key, int lane) {
    SpecSlot *SB = W.spec;
    for (;;) {
        const int st = __hip_atomic_load(&SB[lane].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const bool mine = st != SPEC_FREE && st != SPEC_STALE && st != SPEC_BUSY && SB[lane].key == key;
        bool retry = false;
        if (mine) {
            int exp = st;
            retry = !__hip_atomic_compare_exchange_strong(&SB[lane].state, &exp,
                                                          st == SPEC_CLAIMED ? SPEC_STALE : SPEC_FREE,
                                                          __ATOMIC_RELEASE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!ballot(retry)) break;
    }
}

__global__ void __launch_bounds__(WG_THREADS) k_lin_wg(WgArgs W) {
    WgShared &sh = *(WgShared *)(jh_lds + WG_SH_OFF);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const DfsArgs &A = W.d;
    uint64_t *memo = A.memo + (size_t)blockIdx.x * A.memo_cap * 2;
    Frame *stack = A.stack + (size_t)blockIdx.x * A.stack_cap;
    uint64_t *stage = (uint64_t *)(A.scratch + (size_t)blockIdx.x * A.scratch_bytes);
    uint64_t *gset = W.gset + (size_t)blockIdx.x * W.gset_cap;
    uint64_t *work = W.work + (size_t)blockIdx.x * W.work_cap;
    char *wtab = W.wtab + (size_t)blockIdx.x * W.wtab_bytes;
    uint64_t *pend = W.pend + (size_t)blockIdx.x * 2 * W.pend_cap;
    unsigned long long my_probes = 0;
    const unsigned long long t_enter = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        sh.keep = nullptr; sh.keep_n = 0; sh.nomemo = 0; sh.abort_state = nullptr;
        sh.spec_slot = -1; sh.res_slot = -1; sh.wtab_key = -1;
    }
    __syncthreads();
    for (;;) {
        if (W.seq_start) {
            wg_helper_pick(W, sh, tid, t_enter);
        } else if (tid == 0) {
            const int idx = atomicAdd(A.queue, 1);
            sh.key = idx < A.n_list ? A.list[idx] : -1;
            sh.cmd = 0;
        }
        __syncthreads();
        const int key = sh.key;
        if (key == -4) {
            // round 6: a spec job for another helper's search
            if (wid == 0) {
                spec_enum(W, sh, lane, wtab, gset, work, memo, pend, my_probes);
            } else {
                for (;;) {
                    __syncthreads();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    if (sh.cmd == CMD_DONE) break;
                    wg_enum_work(W, sh, tid, gset, work, memo, pend, my_probes);
                }
            }
            __syncthreads();
            continue;
        }
        if (key < 0) break;
        const KeyMeta mt = A.meta[key];
        if (!(A.states8 && mt.maxw <= 40)) {      // WIDE keys: k_lin_seq3<false>
            __syncthreads();
            continue;
        }
        if (wid == 0) {
            KeyInfo K;
            K.n_ops = mt.n_ops; K.n_ok = mt.n_ok; K.sumW = mt.pad; K.s0 = 0; K.s1 = 0;
            long long inserts = 0;
            uint32_t tmax = 0;
            const unsigned long long ck0 = __builtin_amdgcn_s_memtime();
            TL_REC(A.tl, key, 4);
            // Round 6, the takeover: ask the sequential search for its state
            // (it answers at its next check, every 256 inserts); a search that
            // does not answer within ~3 ms (not running this key) is withdrawn
            // from, and a refused or unsaved one restarts here from the root
            int ho_st = HO_NONE;
            if (W.mains_live && lane == 0) atomicAdd(W.mains_live, 1);
            if (A.handoff && lane == 0) {
                __hip_atomic_store(&A.handoff[key], HO_ASK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long h0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    ho_st = __hip_atomic_load(&A.handoff[key], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    if (ho_st == HO_DONE || ho_st == HO_REFUSED) break;
                    if (__hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                    const unsigned long long el = __builtin_amdgcn_s_memrealtime() - h0;
                    if (ho_st == HO_ASK && el > 300000ULL) {
                        int exp = HO_ASK;
                        if (__hip_atomic_compare_exchange_strong(&A.handoff[key], &exp, HO_WITHDRAWN, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            ho_st = HO_WITHDRAWN;
                            break;
                        }
                        continue;
                    }
                    if (el > HELPER_MAX_TICKS) break;      // (a save never takes this long)
                    __builtin_amdgcn_s_sleep(16);
                }
            }
            ho_st = readlane(ho_st, 0);
            const int verdict = dfs_acc<MemoW>(W, sh, K, A.tables + mt.off, key, lane, memo, stack, stage, gset,
                                               work, wtab, pend, inserts, tmax, my_probes, ho_st == HO_DONE);
            TL_REC(A.tl, key, 5);
            if (W.spec) spec_release(W, key, lane);
            if (W.mains_live && lane == 0) atomicSub(W.mains_live, 1);
            jh_key_verdict v;
            v.valid = verdict;
            v.cause = verdict == JH_UNKNOWN ? JH_CAUSE_BUDGET : 0;
            v.explored = inserts;
            v.fail_entry = verdict == JH_INVALID ? -(int64_t)tmax - 2 : -1;
            bool won = false;
            if (lane == 0) {
                if (verdict != JH_CANCELLED) won = emit_verdict(A.out, A.claim, key, v);
                sh.cmd = CMD_DONE;
            }
            if (lane == 0 && W.acc_stats) atomicAdd(&W.acc_stats[7], __builtin_amdgcn_s_memtime() - ck0);
            if (lane == 0 && W.key_prof) {
                // JH_DEBUG=4: per-key cycles / inserts / verdict | workgroup << 8 | won << 20 |
                // start (us after the kernel's start) << 32, for the tail analysis
                const unsigned long long t_us = (__builtin_amdgcn_s_memrealtime() - t_enter) / 100;
                W.key_prof[3 * (size_t)key] = __builtin_amdgcn_s_memtime() - ck0;
                W.key_prof[3 * (size_t)key + 1] = (unsigned long long)inserts;
                W.key_prof[3 * (size_t)key + 2] = (unsigned long long)verdict | ((unsigned long long)blockIdx.x << 8) |
                                                  ((unsigned long long)won << 20) | (t_us << 32);
            }
            __syncthreads();                    // releases the helpers
        } else {
            for (;;) {
                __syncthreads();                // wave 0's enumeration / merge request, or the end of the key
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (sh.cmd == CMD_DONE) break;
                if (sh.cmd == CMD_MERGE) wg_merge(W, sh, tid, memo, my_probes);
                else wg_enum_work(W, sh, tid, gset, work, memo, pend, my_probes);
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) my_probes += __shfl_xor(my_probes, o);
    if (lane == 0 && A.probes) atomicAdd(A.probes, my_probes);
}

// ---------------------------------------------------------------------------
// Heavy keys: parallel breadth-first enumeration of the reachable
// configuration graph by a whole workgroup. For a key with no terminal
// configuration (invalid) WGL's cache ends up holding exactly this set, so
// verdict, explored count and the furthest return rank (fail_entry) are
// identical to the sequential search (over the budget: :unknown with the
// budget as count, where the search stops).
//
// A key where a terminal configuration is reachable (valid, or :unknown if
// WGL runs out of budget first) gets WGL's exact count from the stored set
// (bfs_wgl_count): a node is live iff a terminal configuration is reachable
// from it; WGL's DFS goes from the root to the first live child at every
// step (in candidate order), and before taking it exhausts every earlier
// (dead) child's whole reachable set. So WGL's cache at the terminal is the
// path (root excluded, terminal included) plus the closure of those dead
// children -- computed here in parallel: liveness layer by layer backwards,
// the path by one wave, the closure by a multi-source BFS. Sets beyond the
// storage cap are left to the sequential search.
// 1024 threads (16 waves on the BFS's CU): the closure rounds and the count
// pass are latency-bound, and twice the waves in flight took the heavy valid
// keys of C3 ranks 3 / 6 from 104 / 111 to 82 / 88 ms per step (512 before)
#ifndef JH_BFS_THREADS
#define JH_BFS_THREADS 1024
#endif
constexpr int BFS_THREADS = JH_BFS_THREADS;
constexpr int BFS_HDR = 1024;                      // shared scalars + the layer's window
constexpr int BFS_TBL = 28672;                     // W-format tables (ops, woff, W) + r[]
constexpr int LSET = 16384;                        // layer set slots (8 B keys)
constexpr int BFS_LDS_BYTES = BFS_HDR + BFS_TBL + LSET * 8;   // 157 KB: one workgroup per CU
// the count pass's LDS-resident liveness of one layer (over the free layer set):
// keys, global slots, a key -> local index hash, live flags
constexpr int LV_CAP = 4096, LV_H = 8192;
static_assert(LV_CAP * 8 + LV_CAP * 4 + LV_H * 4 + LV_CAP + LV_CAP * 2 + 512 <= LSET * 8, "liveness LDS");
__device__ __forceinline__ uint32_t lv_hash(uint64_t k) { return (uint32_t)jh_mix64(k) & (LV_H - 1); }
// the count pass's per-bucket live sets of layers past LV_CAP: two LDS sets
// of GL_H keys (not a power of two: both fit beside the bucket histogram),
// at most half full; GL_XLIVE marks a node whose cross-layer child is live
constexpr uint32_t GL_H = 8064, GL_CAP = GL_H / 2;
constexpr uint32_t GL_XLIVE = 0x80000000u;
static_assert(512 + 2 * GL_H * 8 <= LSET * 8, "count-pass live sets");
__device__ __forceinline__ uint32_t gl_hash(uint64_t k) {
    return (uint32_t)(((uint64_t)(uint32_t)jh_mix64(k) * GL_H) >> 32);
}
constexpr uint64_t BFS_EMPTY = ~0ULL;
// JH_DEBUG=2: where a BFS closure round's time goes (tid 0's s_memtime, summed
// over workgroups): [0] claim + first barrier, [1] tid 0's items, [2] the
// barrier after the items, [3] swap + counters + last barrier, [4] rounds,
// [5] layer formation (clear, window, pending scan), [6] layers
#ifdef JH_BFS_PROF
#define BFS_PROF(x) x
#else
#define BFS_PROF(x)
#endif
__device__ unsigned long long g_bfs_prof[8];
__device__ unsigned long long g_bfs_prof_x[4];   // [0] insert8, [1] record8, [2] tid 0's items ([7] above: load + children)
// A valid key is settled by the BFS (instead of waiting for the sequential
// search) when its whole reachable set is complete and smaller than the
// budget; only for sets this large, which the DFS takes milliseconds over.
constexpr long long BFS_VALID_MIN = 1 << 16;

struct BfsArgs {
    unsigned long long *dbg;  // JH_DEBUG=2: per-workgroup accounting (16 words)
    KeySrc src;
    const int32_t *list;
    int32_t n_list;
    int32_t *queue;
    jh_key_verdict *out;
    int32_t *unres_list;
    int32_t *unres_count;
    uint64_t *gset;         // per workgroup: gset_cap slots, layers too wide for LDS
    uint32_t gset_cap;      // power of two
    uint64_t *pend;         // per workgroup: 2 x q_cap pending cross-layer configurations
    uint64_t *front;        // per workgroup: 2 x q_cap frontier configurations
    uint32_t q_cap;
    char *scratch;          // per workgroup table space
    uint64_t scratch_bytes;
    int64_t budget;
    int32_t init_state;
    int32_t states_ok;      // every interned state < 2^12
    int32_t *claim;         // race with the sequential search (see emit_verdict)
    int64_t reach_cap;      // reachable configurations enumerated at most (>= budget + 1)
    int32_t dbg_plen;       // JH_BFS_ONLY=1 (debugging): the BFS alone settles, fail_entry = path length
    int32_t exact_count;    // JH_LIN_EXACT_COUNT: WGL's count for the valid keys it settles (else uncounted)
    // per workgroup, for bfs_wgl_count (valid keys): every node of the set in
    // layer order, its layer offsets, a node -> id hash, liveness / closure marks
    uint64_t *nodes;        // ncap
    uint32_t ncap;
    uint32_t *lstart;       // n_ok + 2 (sized by the longest key)
    uint32_t lcap;
    ulonglong2 *ent;        // hcap (power of two) hash entries {configuration, id | LIVE}
    uint32_t hcap;
    uint32_t *slot;         // ncap: each node's hash slot
    uint32_t *vis;          // ncap / 32 + 1
    uint32_t *tmp;          // ncap
    uint64_t *tmpk;         // ncap: the liveness pass's node keys, beside their slots in tmp
    // :linear mode (knossos.linear, checker.clj:141-145): this search is the
    // analysis -- a key is valid iff a terminal configuration is reachable,
    // explored = the reachable configurations (initial and terminal ones
    // excluded), no WGL count; keys past reach_cap (= budget + 1) go to the
    // unresolved list, which WGL then decides
    int32_t linear;
    // frontier configurations of invalid keys (jh_lin_configs, knossos'
    // :configs): per key its output slot (-1: none); per slot up to cfg_per
    // configurations of the last layer reached and their window rows
    const int32_t *cfg_slot;
    jh_lin_config *cfg_out;
    int32_t *cfg_n;
    int64_t *cfg_rows;
    int32_t cfg_per;
    const int64_t *col_val, *col_val2;   // the raw value columns (model values)
    int64_t vmin, init_value;
    int32_t per_key_values;
    // the streaming heavy-key pass (DfsArgs): `list` is live, *live_n long,
    // complete once phase 1 has finished; t_span = [first key taken, last
    // workgroup end] (s_memrealtime), the BFS's own time
    const int32_t *live_n;
    const int32_t *p1_done, *p1_tot;
    unsigned long long *t_span;
    unsigned long long *tl;     // -DJH_TUNING timeline: per key [0] BFS start, [1] end
};

struct BfsShared {
    KeyInfo K;
    jh_key_verdict v;
    int key, need, maxw, status, mode, gclear, ovf, term;
    unsigned npend, npend2, nfront, nnext, tmax, lcount, r;
    unsigned nnodes, nostore, dlen, clen, cnext, ok;
    unsigned fbase;          // nnodes when the frontier being built started (its slot 0)
    unsigned long long count, ccount, plen;
    alignas(16) uint32_t win_vv[64];    // the current layer's window: v1 | v2 << 16
    uint32_t win_f[64];     // f, or 3 for no member
    unsigned long long cfg_min;
    unsigned gl_cnt[2], gl_ovf[2];   // the count pass's per-bucket LDS live sets (two in turn)
};

static_assert(sizeof(BfsShared) <= BFS_HDR, "BFS header");

// a configuration of the pending list / global set: t:20 | s:12 | mask:32
__device__ __forceinline__ uint64_t bfs_pack(uint32_t t, uint32_t s, uint32_t m) {
    return ((uint64_t)t << 44) | ((uint64_t)s << 32) | m;
}
__device__ __forceinline__ uint32_t lset_hash(uint64_t k) {
    uint32_t h = (uint32_t)k * 0x9E3779B1u ^ (uint32_t)(k >> 32) * 0x85EBCA77u;
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    return (h >> 11) & (LSET - 1);
}

// child j of configuration (t, s, mask) in the canonical coordinates of the
// BFS: 0 none (member linearized or the model refuses it), 1 same layer,
// 2 a later layer, 3 a terminal configuration; *ck = the child's packed key
__device__ __forceinline__ int bfs_child(const Op *ops, const int32_t *woff, const uint16_t *W, const uint8_t *rpos,
                                         uint32_t n_ok, uint32_t t, uint32_t s, uint32_t mask, int j,
                                         uint64_t *ck) {
    const int wo = woff[t], w = woff[t + 1] - wo;
    if (j >= w || ((mask >> j) & 1)) return 0;
    const Op o = ops[W[wo + j]];
    int s2;
    if (!cas_step(o.fa & 3, o.v1, o.v2, (int)s, &s2)) return 0;
    const uint32_t r = rpos[t];
    if ((uint32_t)j != r) { *ck = bfs_pack(t, (uint32_t)s2, mask | (1u << j)); return 1; }
    uint64_t nm = mask | (1u << j);
    uint32_t u = t, ru = r;
    for (;;) {
        nm = drop_bit(nm, ru);
        u++;
        if (u >= n_ok) return 3;
        ru = rpos[u];
        if (!((nm >> ru) & 1)) break;
    }
    *ck = bfs_pack(u, (uint32_t)s2, (uint32_t)nm);
    return 2;
}

// The stored set's hash: 16-byte entries {packed configuration, id | LIVE},
// so that one load answers "which node, and is it live" for a child.
constexpr uint64_t BFS_LIVE = 1ULL << 40;

// The LIVE bit is set with a global atomic, which is performed in L2 and does
// not update the CU's L1 copy of the line: its readers load the info word with
// an L1-bypassing (agent-scope) atomic load, never a plain load.
__device__ __forceinline__ uint64_t bfs_info(const ulonglong2 *ent, uint32_t h) {
    return __hip_atomic_load(&ent[h].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the keys are placed with a global CAS as well: read the same way
__device__ __forceinline__ uint64_t bfs_keyat(const ulonglong2 *ent, uint32_t h) {
    return __hip_atomic_load(&ent[h].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// slot of key k, or -1 (the table is at most half full)
__device__ __forceinline__ int64_t bfs_slot(const ulonglong2 *ent, uint32_t hmask, uint64_t k) {
    uint32_t h = (uint32_t)jh_mix64(k) & hmask;
    for (;;) {
        const uint64_t e = bfs_keyat(ent, h);
        if (e == k) return h;
        if (e == BFS_EMPTY) return -1;
        h = (h + 1) & hmask;
    }
}

// a batch of child keys (k[i] = 0: none): slot and info word of each, the
// first probes all in flight together; slot -1 for a key not in the set
template <int B>
__device__ __forceinline__ void bfs_lookup_batch(const ulonglong2 *ent, uint32_t hmask, const uint64_t (&k)[B],
                                                 int64_t (&slot)[B], uint64_t (&info)[B]) {
    uint32_t h[B];
    uint64_t e[B], y[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
        h[i] = (uint32_t)jh_mix64(k[i]) & hmask;
        e[i] = k[i] ? bfs_keyat(ent, h[i]) : BFS_EMPTY;
        y[i] = k[i] ? bfs_info(ent, h[i]) : 0;
    }
#pragma unroll
    for (int i = 0; i < B; i++) {
        slot[i] = -1; info[i] = 0;
        if (!k[i]) continue;
        if (e[i] == k[i]) { slot[i] = h[i]; info[i] = y[i]; }
        else if (e[i] != BFS_EMPTY) {
            slot[i] = bfs_slot(ent, hmask, k[i]);
            if (slot[i] >= 0) info[i] = bfs_info(ent, (uint32_t)slot[i]);
        }
    }
}

// the count pass's same-layer liveness: one item per (node, 8 members) (1,
// kept) or one node per thread with its members in series (0: measured in
// round 4, ranks 3 / 4 / 6 1.5-2.7 ms slower, profiles/r04/bfs_lv/)
#ifndef JH_BFS_LV_ITEMS
#define JH_BFS_LV_ITEMS 1
#endif
// the window's operations of members j0 .. j0+7 (j0 a multiple of 8 below
// 64): four 16-byte LDS reads issued together, instead of one dependent LDS
// round trip per member inside the children's branches
struct Win8 { uint32_t f[8], vv[8]; };
__device__ __forceinline__ void win8(const BfsShared &sh, int j0, Win8 &x) {
    const uint4 *pf = (const uint4 *)&sh.win_f[j0 & 56], *pv = (const uint4 *)&sh.win_vv[j0 & 56];
    const uint4 a = pf[0], b = pf[1], c = pv[0], d = pv[1];
    x.f[0] = a.x; x.f[1] = a.y; x.f[2] = a.z; x.f[3] = a.w; x.f[4] = b.x; x.f[5] = b.y; x.f[6] = b.z; x.f[7] = b.w;
    x.vv[0] = c.x; x.vv[1] = c.y; x.vv[2] = c.z; x.vv[3] = c.w; x.vv[4] = d.x; x.vv[5] = d.y; x.vv[6] = d.z; x.vv[7] = d.w;
}

// bfs_child for layer t with member j's operation given (f, vv = v1 | v2 << 16; r = RET's position)
__device__ __forceinline__ int bfs_child_fv(uint32_t f, uint32_t vv, const uint8_t *rpos, uint32_t n_ok, uint32_t t,
                                            uint32_t r, int w, uint32_t s, uint32_t mask, int j, uint64_t *ck) {
    if (j >= w || ((mask >> j) & 1)) return 0;
    int s2;
    if (!cas_step((int)f, (int)(vv & 0xFFFF), (int)(vv >> 16), (int)s, &s2)) return 0;
    if ((uint32_t)j != r) { *ck = bfs_pack(t, (uint32_t)s2, mask | (1u << j)); return 1; }
    uint64_t nm = mask | (1u << j);
    uint32_t u = t, ru = r;
    for (;;) {
        nm = drop_bit(nm, ru);
        u++;
        if (u >= n_ok) return 3;
        ru = rpos[u];
        if (!((nm >> ru) & 1)) break;
    }
    *ck = bfs_pack(u, (uint32_t)s2, (uint32_t)nm);
    return 2;
}

// bfs_child for layer t with its window in LDS (sh.win_vv / sh.win_f, r = RET's position)
__device__ __forceinline__ int bfs_child_w(const BfsShared &sh, const uint8_t *rpos, uint32_t n_ok, uint32_t t,
                                           uint32_t r, int w, uint32_t s, uint32_t mask, int j, uint64_t *ck) {
    if (j >= w || ((mask >> j) & 1)) return 0;
    return bfs_child_fv(sh.win_f[j], sh.win_vv[j], rpos, n_ok, t, r, w, s, mask, j, ck);
}

// live if any child among members j0 .. j0+7 is terminal or live
__device__ __forceinline__ bool bfs_any_live8(const ulonglong2 *ent, uint32_t hmask, const BfsShared &sh,
                                              const uint8_t *rpos, uint32_t n_ok, uint32_t t, uint32_t r, int w,
                                              uint32_t s0, uint32_t m0, int j0) {
    uint64_t k[8];
    int64_t sl[8];
    uint64_t inf[8];
    bool term = false;
    Win8 wn;
    win8(sh, j0, wn);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t ck = 0;
        const int c = bfs_child_fv(wn.f[i], wn.vv[i], rpos, n_ok, t, r, w, s0, m0, j0 + i, &ck);
        term |= c == 3;
        k[i] = (c == 1 || c == 2) ? ck : 0;
    }
    if (term) return true;
    bfs_lookup_batch<8>(ent, hmask, k, sl, inf);
    bool any = false;
#pragma unroll
    for (int i = 0; i < 8; i++) any |= (inf[i] & BFS_LIVE) != 0;
    return any;
}

// WGL's cache size for a key whose whole reachable set the BFS has stored
// (see above). Sets sh.ok, sh.plen (path: root excluded, terminal included)
// and sh.ccount (closure of the dead children left of the path).
__device__ void bfs_wgl_count(const BfsArgs &A, BfsShared &sh, int tid, int key, const Op *ops,
                              const int32_t *woff, const uint16_t *W, const uint8_t *rpos, uint32_t n_ok) {
    const int lane = tid & 63;
    if (sh.nostore) return;
    const uint32_t N = sh.nnodes;
    if ((uint64_t)N * 2 > A.hcap) return;
    // the hash sized to this key: load <= 1/4 where it fits (short probe
    // chains: every liveness / closure lookup is an HBM round trip)
    uint32_t hc = 1u << 12;
    while (hc < A.hcap && (uint64_t)hc < 4ull * N) hc <<= 1;
    const uint32_t hmask = hc - 1;
    ulonglong2 *ent = A.ent;
    uint32_t *slot_of = A.slot;
    unsigned long long *dq = A.dbg ? A.dbg + 16 * (size_t)blockIdx.x : nullptr;   // JH_DEBUG=2 phase cycles
    unsigned long long tq = __builtin_amdgcn_s_memtime();
    auto stamp = [&](int idx) {
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        if (dq && tid == 0) dq[idx] += n - tq;
        tq = n;
    };
    // ---- node -> slot hash ----------------------------------------------------
    for (uint32_t i = tid; i < hc; i += BFS_THREADS) ent[i] = make_ulonglong2(BFS_EMPTY, 0);
    for (uint32_t i = tid; i < N / 32 + 1; i += BFS_THREADS) A.vis[i] = 0;
    __syncthreads();
    // four nodes per thread per pass, their first CAS in flight together
    constexpr int HBN = 4;
    for (uint32_t i0 = tid; i0 < N; i0 += HBN * BFS_THREADS) {
        uint64_t k[HBN];
        uint32_t h[HBN];
        unsigned long long pv[HBN];
#pragma unroll
        for (int u = 0; u < HBN; u++) {
            const uint32_t i = i0 + (uint32_t)u * BFS_THREADS;
            k[u] = i < N ? A.nodes[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < HBN; u++) {
            const uint32_t i = i0 + (uint32_t)u * BFS_THREADS;
            h[u] = (uint32_t)jh_mix64(k[u]) & hmask;
            pv[u] = i < N ? atomicCAS((unsigned long long *)&ent[h[u]].x, BFS_EMPTY, k[u]) : BFS_EMPTY;
        }
#pragma unroll
        for (int u = 0; u < HBN; u++) {
            const uint32_t i = i0 + (uint32_t)u * BFS_THREADS;
            if (i >= N) continue;
            uint32_t hh = h[u];
            while (pv[u] != BFS_EMPTY) {
                hh = (hh + 1) & hmask;
                pv[u] = atomicCAS((unsigned long long *)&ent[hh].x, BFS_EMPTY, k[u]);
            }
            ent[hh].y = i;
            slot_of[i] = hh;
        }
    }
    __syncthreads();
    stamp(5);
    // ---- liveness, layer by layer backwards; within a layer by mask size
    // descending (same-layer edges add one member) ------------------------------
    uint32_t *hist = (uint32_t *)(jh_lds + BFS_HDR + BFS_TBL);     // the layer set's LDS, free now
    for (int t = (int)n_ok - 1; t >= 0; t--) {
        const unsigned long long lt0 = __builtin_amdgcn_s_memtime();
        if (A.claim && tid == 0 &&
            __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            sh.status |= 4;
        const uint32_t a = A.lstart[t], b = A.lstart[t + 1];
        __syncthreads();
        if (sh.status) return;
        if (a == b) continue;
        if (dq && tid == 0) { dq[14] += 1; dq[15] += __builtin_amdgcn_s_memtime() - lt0; }
        if (tid < 66) hist[tid] = 0;
        const int w = woff[t + 1] - woff[t];
        if (tid < 64) {       // the layer's window into LDS, as in the forward pass
            if (tid < w) {
                const Op o = ops[W[woff[t] + tid]];
                sh.win_vv[tid] = (uint32_t)o.v1 | ((uint32_t)o.v2 << 16);
                sh.win_f[tid] = (uint32_t)(o.fa & 3);
            } else sh.win_f[tid] = 3;
        }
        const uint32_t rt = rpos[t];
        __syncthreads();
        if (b - a <= (uint32_t)LV_CAP) {
            // The layer in LDS. A node's children are one cross-layer child
            // (member RET[t], into a later layer whose liveness is final) and
            // same-layer children (one member more, so one popcount higher):
            // the cross-layer lookups of the whole layer go out together (one
            // HBM round trip), then the same-layer liveness runs by popcount
            // descending on LDS only, and the live marks go back in one pass.
            const uint32_t n = b - a;
            uint64_t *lk = (uint64_t *)(jh_lds + BFS_HDR + BFS_TBL + 512);
            uint32_t *ls = (uint32_t *)(lk + LV_CAP);
            uint32_t *lh = ls + LV_CAP;
            uint8_t *lv = (uint8_t *)(lh + LV_H);
            uint16_t *ord = (uint16_t *)(lv + LV_CAP);            // nodes by popcount, descending
            for (uint32_t i = tid; i < LV_H; i += BFS_THREADS) lh[i] = 0;
            if (tid < 2) hist[tid] = tid ? 0u : 32u;               // [0] min popcount, [1] max
            if (tid >= 2 && tid < 2 + 2 * 33) hist[tid] = 0;      // [2+p] count, [35+p] fill
            __syncthreads();
            for (uint32_t i0 = tid - lane; i0 < n; i0 += BFS_THREADS) {
                const uint32_t i = i0 + lane;
                const uint64_t x = i < n ? A.nodes[a + i] : 0;
                const uint32_t pc = (uint32_t)__popc((uint32_t)x);
                {
                    // popcount range: one LDS atomic per wave
                    uint32_t pmn = i < n ? pc : 32u, pmx = pc;
                    for (int o = 32; o > 0; o >>= 1) {
                        pmn = min(pmn, (uint32_t)__shfl_xor((int)pmn, o));
                        pmx = max(pmx, (uint32_t)__shfl_xor((int)pmx, o));
                    }
                    if (lane == 0) { atomicMin(&hist[0], pmn); atomicMax(&hist[1], pmx); }
                }
                if (i >= n) continue;
                const uint32_t sl = slot_of[a + i];
                lk[i] = x;
                ls[i] = sl;
                atomicAdd(&hist[2 + pc], 1u);
                uint32_t h = lv_hash(x);
                while (atomicCAS(&lh[h], 0u, i + 1) != 0u) h = (h + 1) & (LV_H - 1);
                // the cross-layer child (or a terminal one)
                uint64_t ck = 0;
                const int c = bfs_child_w(sh, rpos, n_ok, (uint32_t)t, rt, w, (uint32_t)(x >> 32) & 0xFFF, (uint32_t)x,
                                          (int)rt, &ck);
                bool live = c == 3;
                if (c == 2) {
                    const int64_t cs = bfs_slot(ent, hmask, ck);
                    live = cs >= 0 && (bfs_info(ent, (uint32_t)cs) & BFS_LIVE);
                }
                lv[i] = live ? 1 : 0;
            }
            __syncthreads();
            if (tid == 0) {                                         // bucket starts, largest first
                uint32_t acc = 0;
                for (int p = 32; p >= 0; p--) { hist[35 + p] = acc; acc += hist[2 + p]; }
            }
            __syncthreads();
            for (uint32_t i = tid; i < n; i += BFS_THREADS)
                ord[atomicAdd(&hist[35 + __popc((uint32_t)lk[i])], 1u)] = (uint16_t)i;
            __syncthreads();
            const int pmin = (int)hist[0], pmax = (int)hist[1];
            // JH_BFS_LV_ITEMS: one item per (node, 8 members) (round 3); else
            // one node per thread, its members eight at a time until a live
            // child is found (round 4)
            const uint32_t nb = JH_BFS_LV_ITEMS ? (uint32_t)(w + 7) / 8 : 1u;
            for (int p = pmax; p >= pmin; p--) {
                // the 8 children's LDS probes issue together
                const uint32_t cnt = hist[2 + p], b0 = hist[35 + p] - cnt;
                for (uint32_t q = tid; q < cnt * nb; q += BFS_THREADS) {
                    const uint32_t i = ord[b0 + q / nb];
                    if (lv[i]) continue;
                    const uint64_t x = lk[i];
                    const uint32_t s0 = (uint32_t)(x >> 32) & 0xFFF, m0 = (uint32_t)x;
                    const int jb = JH_BFS_LV_ITEMS ? (int)(q % nb) * 8 : 0;
                    const int je = JH_BFS_LV_ITEMS ? jb + 8 : w;
                    bool live = false;
                    for (int j0 = jb; j0 < je && !live; j0 += 8) {
                    uint64_t ck[8];
                    uint32_t h[8], e[8];
                    Win8 wn;
                    win8(sh, j0, wn);
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        ck[u] = 0;
                        const int j = j0 + u;
                        if ((uint32_t)j != rt &&
                            bfs_child_fv(wn.f[u], wn.vv[u], rpos, n_ok, (uint32_t)t, rt, w, s0, m0, j, &ck[u]) != 1)
                            ck[u] = 0;
                        if ((uint32_t)j == rt) ck[u] = 0;
                        h[u] = lv_hash(ck[u]);
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++) e[u] = ck[u] ? lh[h[u]] : 0u;
                    uint64_t kk[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) kk[u] = e[u] ? lk[e[u] - 1] : 0;
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        if (!ck[u] || !e[u]) continue;
                        uint32_t idx = 0;
                        if (kk[u] == ck[u]) idx = e[u];
                        else
                            for (uint32_t hh = (h[u] + 1) & (LV_H - 1);; hh = (hh + 1) & (LV_H - 1)) {
                                const uint32_t ee = lh[hh];
                                if (ee == 0) break;
                                if (lk[ee - 1] == ck[u]) { idx = ee; break; }
                            }
                        if (idx && lv[idx - 1]) live = true;
                    }
                    }
                    if (live) lv[i] = 1;
                }
                __syncthreads();
            }
            for (uint32_t i = tid; i < n; i += BFS_THREADS)
                if (lv[i]) atomicOr((unsigned long long *)&ent[ls[i]].y, BFS_LIVE);
            if (dq && tid == 0) { dq[2] += __builtin_amdgcn_s_memtime() - lt0; dq[14] += 1ULL << 32; }
            continue;                                              // (the loop head syncs)
        }
        for (uint32_t i = a + tid; i < b; i += BFS_THREADS)
            atomicAdd(&hist[__popc((uint32_t)A.nodes[i])], 1u);
        __syncthreads();
        if (tid == 0) {   // bucket starts, largest masks first
            uint32_t acc = 0;
            for (int p = 32; p >= 0; p--) { const uint32_t c = hist[p]; hist[33 + p] = acc; hist[p] = acc; acc += c; }
        }
        __syncthreads();
        for (uint32_t i = a + tid; i < b; i += BFS_THREADS) {
            const uint64_t x = A.nodes[i];
            const uint32_t pos = atomicAdd(&hist[__popc((uint32_t)x)], 1u);
            A.tmp[pos] = slot_of[i];
            A.tmpk[pos] = x;
        }
        __syncthreads();
        // Bucket by bucket, largest masks first. A node's same-layer children
        // hold one member more, so they are the previous bucket's nodes: that
        // bucket's LIVE keys are kept in an LDS set and the children become
        // LDS lookups. The cross-layer child (member RET[t], a later layer
        // whose marks are final) is looked up in HBM once per node, the whole
        // layer's lookups in flight together, before the buckets. A bucket
        // whose live keys overflow its LDS set sends the next bucket to HBM
        // lookups of every child (bfs_any_live8).
        const uint32_t n = b - a;
        uint64_t *gl_base = (uint64_t *)(jh_lds + BFS_HDR + BFS_TBL + 512);
        for (uint32_t i0 = tid; i0 < n; i0 += 4 * BFS_THREADS) {
            uint64_t k4[4];
            int c4[4];
            int64_t sl4[4];
            uint64_t in4[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + (uint32_t)u * BFS_THREADS;
                uint64_t ck = 0;
                c4[u] = 0;
                if (i < n) {
                    const uint64_t x = A.tmpk[i];
                    c4[u] = bfs_child_w(sh, rpos, n_ok, (uint32_t)t, rt, w, (uint32_t)(x >> 32) & 0xFFF, (uint32_t)x,
                                        (int)rt, &ck);
                }
                k4[u] = c4[u] == 2 ? ck : 0;
            }
            bfs_lookup_batch<4>(ent, hmask, k4, sl4, in4);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + (uint32_t)u * BFS_THREADS;
                if (i < n && (c4[u] == 3 || (in4[u] & BFS_LIVE))) A.tmp[i] |= GL_XLIVE;
            }
        }
        int prev_state = 0;          // the previous bucket's live set: 0 empty, 1 in LDS, 2 overflowed
        int cur = 0, par = 0;
        for (int p = 32; p >= 0; p--) {
            const uint32_t bs = hist[33 + p], be = p > 0 ? hist[33 + p - 1] : n;
            if (bs == be) { prev_state = 0; continue; }
            uint64_t *cs = gl_base + (cur ? GL_H : 0);
            const uint64_t *ps = gl_base + (cur ? 0 : GL_H);
            for (uint32_t i = tid; i < GL_H; i += BFS_THREADS) cs[i] = 0;
            if (tid == 0) { sh.gl_cnt[par] = 0; sh.gl_ovf[par] = 0; }
            __syncthreads();
            for (uint32_t i0 = bs + tid - lane; i0 < be; i0 += BFS_THREADS) {
                const uint32_t i = i0 + lane;
                const bool act = i < be;
                const uint32_t sw = act ? A.tmp[i] : 0;
                const uint64_t x = act ? A.tmpk[i] : 0;
                const uint32_t s0 = (uint32_t)(x >> 32) & 0xFFF, m0 = (uint32_t)x;
                bool live = (sw & GL_XLIVE) != 0;
                if (act && !live && prev_state == 1) {
                    for (int j0 = 0; j0 < w && !live; j0 += 8) {
                        uint64_t kk[8];
                        uint32_t h[8];
                        uint64_t e[8];
                        Win8 wn;
                        win8(sh, j0, wn);
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            uint64_t ck = 0;
                            const int j = j0 + u;
                            kk[u] = ((uint32_t)j != rt &&
                                     bfs_child_fv(wn.f[u], wn.vv[u], rpos, n_ok, (uint32_t)t, rt, w, s0, m0, j, &ck) == 1)
                                    ? ck + 1 : 0;
                            h[u] = gl_hash(kk[u]);
                        }
#pragma unroll
                        for (int u = 0; u < 8; u++) e[u] = kk[u] ? ps[h[u]] : 0;
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            if (!kk[u] || !e[u]) continue;
                            if (e[u] == kk[u]) { live = true; continue; }
                            for (uint32_t hh = h[u] + 1 == GL_H ? 0 : h[u] + 1;; hh = hh + 1 == GL_H ? 0 : hh + 1) {
                                const uint64_t y = ps[hh];
                                if (y == 0) break;
                                if (y == kk[u]) { live = true; break; }
                            }
                        }
                    }
                } else if (act && !live && prev_state == 2) {
                    for (int j0 = 0; j0 < w && !live; j0 += 8)
                        live = bfs_any_live8(ent, hmask, sh, rpos, n_ok, (uint32_t)t, rt, w, s0, m0, j0);
                }
                if (act && live) atomicOr((unsigned long long *)&ent[sw & ~GL_XLIVE].y, BFS_LIVE);
                // this bucket's live keys into its LDS set: room reserved per wave
                const uint64_t lm = ballot(act && live);
                if (!lm) continue;
                int room = 1;
                if (lane == 0) {
                    const uint32_t c = (uint32_t)__popcll(lm);
                    const uint32_t old = atomicAdd(&sh.gl_cnt[par], c);
                    if (old + c > GL_CAP) { sh.gl_ovf[par] = 1; room = 0; }
                }
                if (readlane(room, 0) && act && live) {
                    const uint64_t k = x + 1;
                    for (uint32_t hh = gl_hash(k);; hh = hh + 1 == GL_H ? 0 : hh + 1)
                        if (atomicCAS((unsigned long long *)&cs[hh], 0ULL, k) == 0ULL) break;
                }
            }
            __syncthreads();
            prev_state = sh.gl_ovf[par] ? 2 : 1;
            cur ^= 1;
            par ^= 1;
        }
    }
    stamp(6);
    // ---- the path: from the root, the first live child each step; the dead
    // children before it seed the closure (one wave) -------------------------------
    uint32_t *dl = A.tmp;                                    // dead children (slots), then closure frontiers
    if (tid < 64) {
        uint64_t x = A.nodes[0];                             // the root (layer 0's first entry)
        unsigned long long plen = 0;
        uint32_t dn = 0;
        bool done = false;
        while (!done && dn + 64 < A.ncap / 2) {
            const uint32_t t = (uint32_t)(x >> 44), s0 = (uint32_t)(x >> 32) & 0xFFF, m0 = (uint32_t)x;
            uint64_t ck = 0;
            const int c = bfs_child(ops, woff, W, rpos, n_ok, t, s0, m0, lane, &ck);
            int64_t sl = -1;
            uint64_t inf = 0;
            if (c == 1 || c == 2) { sl = bfs_slot(ent, hmask, ck); if (sl >= 0) inf = bfs_info(ent, (uint32_t)sl); }
            const bool lv = c == 3 || (inf & BFS_LIVE);
            const uint64_t lm = ballot(lv);
            if (!lm) break;                                   // cannot happen on a live node
            const int jl = __builtin_ctzll(lm);
            const bool dead = sl >= 0 && lane < jl;
            const uint64_t dm = ballot(dead);
            if (dead) dl[dn + mbcnt(dm)] = (uint32_t)sl;
            dn += (uint32_t)__popcll(dm);
            plen++;
            if (readlane(c, jl) == 3) done = true;
            else x = readlane64(ck, jl);
        }
        if (lane == 0) { sh.plen = plen; sh.dlen = dn; sh.ok = done ? 1u : 0u; }
    }
    __syncthreads();
    stamp(7);
    if (!sh.ok) return;
    // ---- closure of the dead children: a multi-source BFS over stored slots ----
    if (tid == 0) { sh.ccount = 0; sh.clen = 0; }
    __syncthreads();
    uint32_t *fa = dl, *fb = dl + A.ncap / 2;
    uint32_t nf = 0;
    auto visit = [&](uint32_t sl, uint64_t info) -> bool {
        const uint32_t id = (uint32_t)info & 0xFFFFFFFFu;
        const uint32_t old = atomicOr(&A.vis[id >> 5], 1u << (id & 31));
        return !(old & (1u << (id & 31)));
    };
    for (uint32_t i = tid; i < sh.dlen; i += BFS_THREADS) {
        const uint32_t sl = dl[i];
        if (visit(sl, ent[sl].y)) fb[atomicAdd(&sh.clen, 1u)] = sl;
    }
    __syncthreads();
    for (;;) {
        nf = sh.clen;
        if (tid == 0) { sh.ccount += nf; sh.cnext = 0; }
        if (nf == 0 || nf > A.ncap / 2) break;
        { uint32_t *tp = fa; fa = fb; fb = tp; }
        __syncthreads();
        // one work item per (node, 8 members), as in the liveness pass
        // (wave-uniform loop: the new nodes are counted with one LDS atomic per
        // wave and child, not one per node on a single address)
        const uint32_t nbc = (uint32_t)(sh.maxw + 7) / 8;
        for (uint32_t q0 = tid - lane; q0 < nf * nbc; q0 += BFS_THREADS) {
            const uint32_t qq = q0 + lane;
            const bool act = qq < nf * nbc;
            uint64_t k[8];
            int64_t sl[8];
            uint64_t inf[8];
            {
                const uint64_t x = act ? bfs_keyat(ent, fa[qq / nbc]) : 0;
                const uint32_t t = (uint32_t)(x >> 44), s0 = (uint32_t)(x >> 32) & 0xFFF, m0 = (uint32_t)x;
                const int j0 = (int)(qq % nbc) * 8;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    uint64_t ck = 0;
                    const int c = act ? bfs_child(ops, woff, W, rpos, n_ok, t, s0, m0, j0 + i, &ck) : 0;
                    k[i] = (c == 1 || c == 2) ? ck : 0;
                }
            }
            bfs_lookup_batch<8>(ent, hmask, k, sl, inf);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const bool nw = sl[i] >= 0 && visit((uint32_t)sl[i], inf[i]);
                const uint64_t m = ballot(nw);
                if (!m) continue;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&sh.cnext, (uint32_t)__popcll(m));
                base = readlane(base, 0);
                const uint32_t pos = base + mbcnt(m);
                if (nw && pos < A.ncap / 2) fb[pos] = (uint32_t)sl[i];
            }
        }
        __syncthreads();
        if (tid == 0) sh.clen = sh.cnext;
        __syncthreads();
    }
    __syncthreads();
    stamp(8);
    if (tid == 0 && nf > A.ncap / 2) sh.ok = 0;
    __syncthreads();
}

// Heavy keys, one workgroup each: the reachable configuration set layer by
// layer. Layer t = configurations whose earliest un-linearized ok return is
// the t-th; every edge either stays in the layer (lift a non-returning
// member) or goes to a later layer (lift the returning member RET[t]). So
// layer t is the closure, under same-layer lifts, of the configurations the
// earlier layers sent to it: processed in t order, each layer's set is
// exact and lives in an LDS hash (LDS atomics), and only cross-layer edges
// go through HBM (a pending list, deduplicated when their layer is formed).
// For a key with no terminal configuration (invalid) WGL's cache ends up
// holding exactly this set, so verdict, explored count and the furthest
// layer (fail_entry) equal the sequential search's. A key where a terminal
// configuration is reachable (valid) or the set outgrows the budget is left
// to the sequential search, which alone defines :unknown for those.
// The frontier of an invalid key (knossos' :configs, of which
// checker.clj:146-158 keeps (take 10 ...)): the configurations of the last
// layer reached, tmax -- every way of linearizing the ops before RET[tmax]
// from which RET[tmax] itself cannot be -- in a canonical order (model
// state, then the linearized members of W(tmax) as a bit mask in call
// order; nil first, then values ascending), the first cfg_per of them, each
// as its register value, the window's linearized ops and its pending ops
// (invocation rows, call order). Selection by cfg_per rounds of a workgroup
// minimum over the layer (the configurations are distinct); knossos itself
// is not vendored, so this order and cut are this library's (oracle:
// orc_lin_configs).
constexpr int CFG_MAX = 16;
constexpr int CFG_ROWS = JH_MAX_WINDOW;     // row slots per configuration (the widest window)
// A configuration's register value from its interned state id (one wave):
// 0 is nil; one global range: vmin + id - 1; per-key ids (k_iassign): 1 the
// initial value, the others the raw value of a record of the key carrying it
__device__ long long cfg_state_value(uint32_t st, int per_key_values, long long vmin, long long init_value,
                                     const KeySrc &S, uint32_t s0, uint32_t s1, const int64_t *col_val,
                                     const int64_t *col_val2, int lane) {
    if (st == 0) return JH_NIL;
    if (!per_key_values) return vmin + (long long)st - 1;
    if (st == 1 && init_value != JH_NIL) return init_value;
    for (uint32_t base = s0; base < s1; base += 64) {
        const uint32_t p = base + lane;
        long long v = JH_NIL;
        if (p < s1) {
            const Rec x = S.rec[p];
            const long long row = (long long)S.rows[p];
            if (x.proc >= 0 && x.v1 == (int32_t)st) v = col_val[row];
            else if (x.proc >= 0 && x.f == F_CAS && x.v2 == (int32_t)st) v = col_val2[row];
        }
        const uint64_t hit = ballot(v != JH_NIL);
        if (hit) return (long long)readlane64((uint64_t)v, __builtin_ctzll(hit));
    }
    return JH_NIL;
}
// fin = false: the frontier of an invalid key (above). fin = true (ABI 6):
// the final configurations of a valid key under :linear -- what the
// JIT-linearization analysis holds after the key's last :ok completion. Each
// terminal edge of the reachable set ends one: lifting RET[t] from a layer-t
// configuration whose cross-layer cascade reaches n_ok. What remains of W(t)
// then is crashed ops only (every op returning at or after t was dropped on
// the way), and W(t)'s crashed ops are the first members, in call order, of
// C = W(n_ok - 1) - {RET[n_ok - 1]} (crashed ops never leave a window): a final
// configuration is (value, mask over C), ordered like the frontier's. Kept
// crashed ops invoked after the last :ok return enter no window; they are
// pending in every final configuration.
__device__ void bfs_dump_configs(const BfsArgs &A, BfsShared &sh, int tid, int key, const Op *ops,
                                 const int32_t *woff, const uint16_t *W, const uint8_t *rpos, uint32_t n_ok,
                                 bool fin) {
    const int slot = A.cfg_slot[key];
    const int lane = tid & 63, wid = tid >> 6;
    const uint32_t tm = fin ? n_ok - 1 : sh.tmax;
    const uint32_t a = fin ? 0 : A.lstart[tm], b = (!fin && tm + 1 < n_ok) ? A.lstart[tm + 1] : sh.nnodes;
    __shared__ unsigned long long sel[CFG_MAX];
    __shared__ long long wrow[64];
    __shared__ int nsel;
    const int per = min(A.cfg_per, CFG_MAX);
    unsigned long long prev = 0;
    if (tid == 0) nsel = 0;
    // Round 6: an :ok read of nil, which the search drops, is an op knossos
    // holds; in the configuration printed for each of ours it is linearized
    // when its completion forces it, so that completion becomes the :last-op
    // of every final configuration whose own last op returned before it (the
    // host moves last_row: jh_api.hip add_noop_reads). Configurations that then
    // differ in nothing print alike: the selection takes every layer whose
    // RET returns before the last such read as one, tf = the last of them.
    __shared__ uint32_t tf;
    if (fin) {
        if (wid == 0) {
            long long y = -1;
            for (uint32_t base = sh.K.s0; base < sh.K.s1; base += 64) {
                const uint32_t p = base + lane;
                if (p < sh.K.s1) {
                    const Rec x = A.src.rec[p];
                    const int q = A.src.pair[p];
                    if (x.proc >= 0 && x.type == T_OK && q >= 0) {
                        const Rec iv = A.src.rec[q];
                        if (iv.f == F_READ && (iv.v1 != 0 ? iv.v1 : x.v1) == 0) y = max(y, (long long)A.src.rows[p]);
                    }
                }
            }
            for (int o = 32; o > 0; o >>= 1) y = max(y, (long long)__shfl_xor(y, o));
            int before = 0;
            for (uint32_t base = sh.K.s0; base < sh.K.s1; base += 64) {
                const uint32_t p = base + lane;
                before += __popcll(ballot(p < sh.K.s1 && A.src.rank[p] <= -2 && (long long)A.src.rows[p] < y));
            }
            if (lane == 0) tf = before > 0 ? (uint32_t)before - 1 : 0;
        }
        __syncthreads();
    }
    for (int i = 0; i < per; i++) {
        if (tid == 0) sh.cfg_min = ~0ULL;
        __syncthreads();
        unsigned long long m = ~0ULL;
        for (uint32_t j = a + tid; j < b; j += BFS_THREADS) {
            const uint64_t e = A.nodes[j];
            unsigned long long kk = e & ((1ULL << 44) - 1);   // s:12 | mask:32
            if (fin) {
                const uint32_t t = (uint32_t)(e >> 44), r = rpos[t];
                const Op o = ops[W[woff[t] + r]];
                int s2;
                if (!cas_step(o.fa & 3, o.v1, o.v2, (int)((e >> 32) & 0xFFF), &s2)) continue;
                uint64_t nm = (uint32_t)e | (1ULL << r);
                uint32_t u = t, ru = r;
                for (;;) {
                    nm = drop_bit(nm, ru);
                    u++;
                    if (u >= n_ok) break;
                    ru = rpos[u];
                    if (!((nm >> ru) & 1)) break;
                }
                if (u < n_ok) continue;                          // not a terminal edge
                // s:12 | mask over C:32 | t:20 (the layer whose RET was lifted last)
                kk = ((unsigned long long)(uint32_t)s2 << 52) | ((unsigned long long)(uint32_t)nm << 20) | max(t, tf);
            }
            if ((i == 0 || kk > prev) && kk < m) m = kk;
        }
        for (int o = 32; o > 0; o >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, o));
        if (lane == 0 && m != ~0ULL) atomicMin(&sh.cfg_min, m);
        __syncthreads();
        prev = sh.cfg_min;
        if (prev == ~0ULL) break;
        if (tid == 0) { sel[i] = prev; nsel = i + 1; }
        __syncthreads();
    }
    __syncthreads();
    if (wid != 0) return;
    // the invocation row of every member of W(tm)
    const int wo = woff[tm], w = woff[tm + 1] - wo;
    for (uint32_t base = sh.K.s0; base < sh.K.s1; base += 64) {
        const uint32_t p = base + lane;
        const int rk = p < sh.K.s1 ? A.src.rank[p] : -1;
        if (rk >= 0)
            for (int j = 0; j < w; j++)
                if ((int)W[wo + j] == rk) wrow[j] = (long long)A.src.rows[p];
    }
    wave_sync();
    // final configurations: C is W(tm) without RET[tm] (member rl)
    const int rl = fin ? (int)rpos[tm] : 64;
    const int wc = fin ? w - 1 : w;
    const long long crow = lane < wc ? wrow[lane + (lane >= rl ? 1 : 0)] : -1;
    // :last-op: a frontier's is the last :ok op before the failing one
    // (RET[tmax - 1]); a final configuration's the :ok op its terminal edge
    // linearized last -- JIT linearization ends each expansion in the op that
    // completes, and a configuration that already holds a later op keeps it
    const long long lfront = fin || tm == 0 ? -1 : ret_row(A.src, sh.K, tm - 1, lane);
    for (int i = 0; i < nsel; i++) {
        const uint32_t st = fin ? (uint32_t)(sel[i] >> 52) : (uint32_t)(sel[i] >> 32) & 0xFFF;
        const uint32_t mask = fin ? (uint32_t)(sel[i] >> 20) : (uint32_t)sel[i];
        const long long lrow = fin ? ret_row(A.src, sh.K, (uint32_t)(sel[i] & 0xFFFFF), lane) : lfront;
        const long long val = cfg_state_value(st, A.per_key_values, A.vmin, A.init_value, A.src, sh.K.s0, sh.K.s1,
                                              A.col_val, A.col_val2, lane);
        const int64_t o = ((int64_t)slot * A.cfg_per + i) * CFG_ROWS;
        const bool in = lane < wc, lin = in && ((mask >> lane) & 1);
        const uint64_t bl = ballot(lin), bp = ballot(in && !lin);
        const int nl = __popcll(bl);
        int np = __popcll(bp);
        if (lin) A.cfg_rows[o + mbcnt(bl)] = crow;
        if (in && !lin) A.cfg_rows[o + nl + mbcnt(bp)] = crow;
        if (fin) {
            // kept crashed ops invoked after the last :ok return (call order)
            for (uint32_t base = sh.K.s0; base < sh.K.s1; base += 64) {
                const uint32_t p = base + lane;
                const int rk = p < sh.K.s1 ? A.src.rank[p] : -1;
                const bool late = rk >= 0 && ops[rk].rr < 0 && (uint32_t)(ops[rk].fa >> 2) >= n_ok;
                const uint64_t bm = ballot(late);
                const int at = nl + np + (int)mbcnt(bm);
                if (late && at < CFG_ROWS) A.cfg_rows[o + at] = (int64_t)A.src.rows[p];
                np = min(np + __popcll(bm), CFG_ROWS - nl);
            }
        }
        if (lane == 0) {
            jh_lin_config c;
            c.key = key; c.model_value = val; c.n_linearized = nl; c.n_pending = np; c.rows_off = o;
            c.last_row = lrow;
            A.cfg_out[(int64_t)slot * A.cfg_per + i] = c;
        }
    }
    if (lane == 0) A.cfg_n[slot] = nsel;
}

// the configuration of a valid key with no :ok op (one wave)
__device__ void bfs_dump_initial(const BfsArgs &A, BfsShared &sh, int lane, int key) {
    const int slot = A.cfg_slot[key];
    const long long val = cfg_state_value((uint32_t)A.init_state, A.per_key_values, A.vmin, A.init_value, A.src,
                                          sh.K.s0, sh.K.s1, A.col_val, A.col_val2, lane);
    const int64_t o = (int64_t)slot * A.cfg_per * CFG_ROWS;
    int np = 0;
    for (uint32_t base = sh.K.s0; base < sh.K.s1; base += 64) {
        const uint32_t p = base + lane;
        const bool kept = p < sh.K.s1 && A.src.rank[p] >= 0;
        const uint64_t bm = ballot(kept);
        const int at = np + (int)mbcnt(bm);
        if (kept && at < CFG_ROWS) A.cfg_rows[o + at] = (int64_t)A.src.rows[p];
        np = min(np + __popcll(bm), CFG_ROWS);
    }
    if (lane == 0) {
        jh_lin_config c;
        c.key = key; c.model_value = val; c.n_linearized = 0; c.n_pending = np; c.rows_off = o; c.last_row = -1;
        A.cfg_out[(int64_t)slot * A.cfg_per] = c;
        A.cfg_n[slot] = 1;
    }
}

#ifndef JH_BFS_ITEMS
#define JH_BFS_ITEMS 0
#endif
// JH_BFS_ROOM_EXACT=1: a refused batch reservation (it counts duplicates and
// other waves' batches) retries per new configuration before the layer moves
// to the global set. Measured in round 4 (profiles/r04/bfs_room/): slower --
// C4 222 vs 215 ms, C3 ranks 0 / 3 / 6 42.5 / 71.3 / 78.1 vs 40.4 / 70.3 /
// 77.3 ms -- so off.
#ifndef JH_BFS_ROOM_EXACT
#define JH_BFS_ROOM_EXACT 0
#endif
template <bool L>
__device__ void bfs_key(const BfsArgs &A, BfsShared &sh, char *gscr, int tid, uint64_t *gset,
                        uint64_t *pend, uint64_t *front) {
    const int lane = tid & 63, wid = tid >> 6;
    char *tb = tbl_base<L>(BFS_HDR, gscr);
    const KeyInfo K = sh.K;
    const int key = sh.key;
    if (wid == 0) {
        const int mw = key_fill<L>(A.src, K, lane, tb);
        if (lane == 0) sh.maxw = mw;
    }
    __syncthreads();
    const Op *ops = (const Op *)tb;
    const int32_t *woff = (const int32_t *)(tb + tbl_ops_bytes(K));
    const uint16_t *W = (const uint16_t *)(tb + tbl_ops_bytes(K) + tbl_off_bytes(K));
    uint8_t *rpos = (uint8_t *)(tb + tbl_bytes(K));           // r[t], after the tables
    const uint32_t n_ok = (uint32_t)K.n_ok;
    uint64_t *lset = (uint64_t *)(jh_lds + BFS_HDR + BFS_TBL);
    const uint32_t gmask = A.gset_cap - 1;
    if (sh.maxw > 64 && !A.cfg_slot) {
        // (a configurations request hands such a key to the 65-256-member
        // search below, with the other keys this engine cannot hold)
        if (tid == 0) {
            jh_key_verdict v;
            v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW; v.fail_entry = -1; v.explored = 0;
            emit_verdict(A.out, A.claim, key, v);
        }
        __syncthreads();
        return;
    }
    if (sh.maxw > 32 || !A.states_ok || n_ok >= (1u << 20) - 2) {
        if (tid == 0) A.unres_list[atomicAdd(A.unres_count, 1)] = key;
        __syncthreads();
        return;
    }
    // position of RET[t] in W(t), for every layer
    for (uint32_t t = tid; t < n_ok; t += BFS_THREADS) {
        const int wo = woff[t], w = woff[t + 1] - wo;
        int r = 0;
        for (int m = 0; m < w; m++)
            if (ops[W[wo + m]].rr == (int)t) { r = m; break; }
        rpos[t] = (uint8_t)r;
    }
    if (tid == 0) {
        pend[0] = bfs_pack(0, (uint32_t)A.init_state, 0);
        sh.npend = 1; sh.tmax = 0; sh.count = 0; sh.status = 0; sh.gclear = 0; sh.term = 0;
        sh.nnodes = 0; sh.nostore = n_ok + 2 > A.lcap ? 1u : 0u;
    }
    __syncthreads();
    const unsigned long long b0 = __builtin_amdgcn_s_memtime();
    unsigned long long rounds = 0;
    uint64_t *pcur = pend, *pnxt = pend + A.q_cap;
    uint64_t *fcur = front, *fnxt = front + A.q_cap;
    for (uint32_t t = 0; t < n_ok; t++) {
        BFS_PROF(const unsigned long long lf0 = __builtin_amdgcn_s_memtime();)
        // ---- form layer t: dedupe its entries from the pending list ---------
        for (int i = tid; i < LSET; i += BFS_THREADS) lset[i] = 0;
        const int wo = woff[t], w = woff[t + 1] - wo;
        if (tid < 64) {
            if (tid < w) {
                const Op o = ops[W[wo + tid]];
                sh.win_vv[tid] = (uint32_t)o.v1 | ((uint32_t)o.v2 << 16);
                sh.win_f[tid] = (uint32_t)(o.fa & 3);
            } else sh.win_f[tid] = 3;
        }
        if (tid == 0) {
            if (t < A.lcap) A.lstart[t] = sh.nnodes;
            sh.fbase = sh.nnodes; sh.nfront = 0; sh.lcount = 0; sh.mode = 0; sh.ovf = 0; sh.r = rpos[t];
            // the sequential search settled this key first
            if (A.claim && __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                sh.status |= 4;
        }
        __syncthreads();
        const unsigned np = sh.npend;
        // a layer too wide for the LDS set moves to the global set (t-tagged keys)
        auto migrate = [&]() {
            if (!sh.gclear) {
                for (uint32_t i = tid; i < A.gset_cap; i += BFS_THREADS) gset[i] = BFS_EMPTY;
                __syncthreads();
                if (tid == 0) sh.gclear = 1;
            }
            for (int i = tid; i < LSET; i += BFS_THREADS) {
                const uint64_t k = lset[i];
                if (!k) continue;
                const uint64_t g = bfs_pack(t, (uint32_t)((k - 1) >> 32) & 0xFFF, (uint32_t)(k - 1));
                uint32_t h = (uint32_t)jh_mix64(g) & gmask;
                while (atomicCAS((unsigned long long *)&gset[h], BFS_EMPTY, g) != BFS_EMPTY)
                    h = (h + 1) & gmask;
            }
            __syncthreads();
            if (tid == 0) { sh.mode = 1; sh.ovf = 0; }
            __syncthreads();
        };
        // the global set's inserts of up to 8 children, their first probes all
        // in flight together (a lone CAS per child was one HBM round trip each,
        // serial per thread: the forward pass's bound once a layer is global)
        auto insert8 = [&](const uint64_t (&ck)[8], bool (&nw)[8]) {
            if (sh.mode == 0) {
                // the LDS set: room for the wave's candidates reserved with one
                // LDS atomic (a per-insert count on one address serialises lane
                // by lane), the eight CAS issued together, collisions resolved
                // after, the duplicates' reservation given back
#pragma unroll
                for (int q = 0; q < 8; q++) nw[q] = false;
                if (sh.status & 2) return;
                uint32_t cand = 0;
#pragma unroll
                for (int q = 0; q < 8; q++) cand += (uint32_t)__popcll(ballot(ck[q] != 0));
                if (cand == 0) return;
                int room = 1;
                if (lane == 0) {
                    const uint32_t old = atomicAdd(&sh.lcount, cand);
                    if (old + cand > (uint32_t)(LSET * 3 / 4)) { atomicSub(&sh.lcount, cand); room = 0; }
                }
                if (!readlane(room, 0)) {
                    if (!JH_BFS_ROOM_EXACT) { if (lane == 0) sh.ovf = 1; return; }
                    // the batch's reservation counts its duplicates too (and the
                    // other waves' batches in flight): near the limit, room is
                    // taken per new configuration instead, so a layer moves to
                    // the global set only when the set is really 3/4 full
                    // (round 3's batched reservation alone moved C4's layers
                    // early: C4 222.7 -> 245 ms, round 4)
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        if (!ck[q]) continue;
                        const uint64_t kq = ck[q] + 1;
                        for (uint32_t hh = lset_hash(kq);; hh = (hh + 1) & (LSET - 1)) {
                            const unsigned long long x = lset[hh];
                            if (x == kq) break;                          // present
                            if (x != 0) continue;
                            const uint32_t old = atomicAdd(&sh.lcount, 1u);
                            if (old + 1 > (uint32_t)(LSET * 3 / 4)) { atomicSub(&sh.lcount, 1u); sh.ovf = 1; break; }
                            const unsigned long long y = atomicCAS((unsigned long long *)&lset[hh], 0ULL, kq);
                            if (y == 0) { nw[q] = true; break; }
                            atomicSub(&sh.lcount, 1u);                   // lost the slot
                            if (y == kq) break;
                        }
                    }
                    return;
                }
                uint64_t k[8];
                uint32_t h[8];
                unsigned long long pv[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    k[q] = ck[q] ? ck[q] + 1 : 0;
                    h[q] = lset_hash(k[q]);
                    pv[q] = k[q] ? atomicCAS((unsigned long long *)&lset[h[q]], 0ULL, k[q]) : 0ULL;
                }
                uint32_t dups = 0;
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    if (!k[q]) continue;
                    if (pv[q] == 0) { nw[q] = true; continue; }
                    if (pv[q] == k[q]) { dups++; continue; }
                    for (uint32_t hh = (h[q] + 1) & (LSET - 1);; hh = (hh + 1) & (LSET - 1)) {
                        const unsigned long long x = atomicCAS((unsigned long long *)&lset[hh], 0ULL, k[q]);
                        if (x == 0) { nw[q] = true; break; }
                        if (x == k[q]) { dups++; break; }
                    }
                }
                for (int o = 32; o > 0; o >>= 1) dups += (uint32_t)__shfl_xor((int)dups, o);
                if (lane == 0 && dups) atomicSub(&sh.lcount, dups);
                return;
            }
            uint64_t g[8];
            uint32_t h[8];
            unsigned long long prev[8];
            const bool off = (sh.status & 2) != 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                nw[q] = false;
                g[q] = bfs_pack(t, (uint32_t)(ck[q] >> 32), (uint32_t)ck[q]);
                h[q] = (uint32_t)jh_mix64(g[q]) & gmask;
                prev[q] = (ck[q] && !off) ? atomicCAS((unsigned long long *)&gset[h[q]], BFS_EMPTY, g[q]) : (unsigned long long)g[q];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if (!ck[q] || off) continue;
                if (prev[q] == g[q]) continue;
                if (prev[q] != BFS_EMPTY) {
                    uint32_t hh = h[q];
                    bool dup = false;
                    for (uint32_t probe = 1;; probe++) {
                        if (probe > gmask) { atomicOr(&sh.status, 2); dup = true; break; }
                        hh = (hh + 1) & gmask;
                        const unsigned long long pv = atomicCAS((unsigned long long *)&gset[hh], BFS_EMPTY, g[q]);
                        if (pv == BFS_EMPTY) break;
                        if (pv == g[q]) { dup = true; break; }
                    }
                    if (dup) continue;
                }
                nw[q] = true;
            }
        };
        // the new children of a batch, counted once per wave: one LDS atomic
        // per counter per wave instead of three per configuration (same-address
        // LDS atomics serialise lane by lane); wave-uniform control flow
        auto record8 = [&](const uint64_t (&ck)[8], const bool (&nw)[8]) {
            uint32_t below[8], tot = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint64_t bq = ballot(nw[q]);
                below[q] = tot + mbcnt(bq);
                tot += (uint32_t)__popcll(bq);
            }
            if (tot == 0) return;
            // one LDS atomic per wave (round 5): a new configuration's node id
            // and its frontier slot differ by the round's base (the node list
            // and the frontier grow together), and the reachable count is the
            // node count
            unsigned nb0 = 0;
            if (lane == 0) {
                nb0 = atomicAdd(&sh.nnodes, tot);
                if ((long long)nb0 + tot > A.reach_cap) atomicOr(&sh.status, 2);
            }
            nb0 = readlane(nb0, 0);
            const unsigned fb0 = nb0 - sh.fbase;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if (!nw[q]) continue;
                const unsigned id = nb0 + below[q];
                if (id < A.ncap) A.nodes[id] = bfs_pack(t, (uint32_t)(ck[q] >> 32), (uint32_t)ck[q]);
                else sh.nostore = 1;
                const unsigned pos = fb0 + below[q];
                if (pos < A.q_cap) fnxt[pos] = ck[q];
                else atomicOr(&sh.status, 2);
            }
        };
        // An insert refused for LDS load (ovf) re-runs the pass against the
        // global set: configurations already inserted stay (and are already on
        // the frontier), the rest are inserted now.
        for (;;) {
        if (tid == 0) sh.npend2 = 0;
        __syncthreads();
        // per wave: the later layers' entries carried over and the new
        // configurations counted with one LDS atomic per counter (same-address
        // atomics serialise lane by lane); LDS-set room reserved per wave
        for (unsigned i0 = tid - lane; i0 < np; i0 += BFS_THREADS) {
            const unsigned i = i0 + lane;
            const uint64_t e = i < np ? pcur[i] : 0;
            const bool here = i < np && (uint32_t)(e >> 44) == t;
            const uint64_t lm = ballot(i < np && !here);
            unsigned pb = 0;
            if (lane == 0 && lm) pb = atomicAdd(&sh.npend2, (unsigned)__popcll(lm));
            pb = readlane(pb, 0);
            if (i < np && !here) pnxt[pb + mbcnt(lm)] = e;
            const uint64_t hm = ballot(here);
            if (!hm || (sh.status & 2)) continue;
            const uint32_t cs = (uint32_t)(e >> 32) & 0xFFF, cm = (uint32_t)e;
            bool nw = false;
            if (sh.mode == 0) {
                int room = 1;
                if (lane == 0) {
                    const uint32_t cand = (uint32_t)__popcll(hm);
                    const uint32_t old = atomicAdd(&sh.lcount, cand);
                    if (old + cand > (uint32_t)(LSET * 3 / 4)) { atomicSub(&sh.lcount, cand); sh.ovf = 1; room = 0; }
                }
                if (!readlane(room, 0)) continue;
                if (here) {
                    const uint64_t k = (((uint64_t)cs << 32) | cm) + 1;
                    for (uint32_t h = lset_hash(k);; h = (h + 1) & (LSET - 1)) {
                        const unsigned long long x = atomicCAS((unsigned long long *)&lset[h], 0ULL, k);
                        if (x == 0) { nw = true; break; }
                        if (x == k) break;
                    }
                }
                const uint32_t dups = (uint32_t)__popcll(hm & ~ballot(nw));
                if (lane == 0 && dups) atomicSub(&sh.lcount, dups);
            } else if (here) {
                const uint64_t g = bfs_pack(t, cs, cm);
                uint32_t h = (uint32_t)jh_mix64(g) & gmask;
                for (uint32_t probe = 0;; probe++) {
                    if (probe > gmask) { atomicOr(&sh.status, 2); break; }
                    const unsigned long long x = atomicCAS((unsigned long long *)&gset[h], BFS_EMPTY, g);
                    if (x == BFS_EMPTY) { nw = true; break; }
                    if (x == g) break;
                    h = (h + 1) & gmask;
                }
            }
            const uint64_t nm = ballot(nw);
            if (!nm) continue;
            const uint32_t tot = (uint32_t)__popcll(nm);
            unsigned nb0 = 0;
            if (lane == 0) {
                nb0 = atomicAdd(&sh.nnodes, tot);
                if ((long long)nb0 + tot > A.reach_cap) atomicOr(&sh.status, 2);
            }
            nb0 = readlane(nb0, 0);
            const unsigned fb0 = nb0 - sh.fbase;
            if (nw) {
                const unsigned below = mbcnt(nm);
                if (nb0 + below < A.ncap) A.nodes[nb0 + below] = bfs_pack(t, cs, cm);
                else sh.nostore = 1;
                if (fb0 + below < A.q_cap) fcur[fb0 + below] = ((uint64_t)cs << 32) | cm;
                else atomicOr(&sh.status, 2);
            }
        }
        __syncthreads();
        if (!sh.ovf) break;
        migrate();
        }
        { uint64_t *tp = pcur; pcur = pnxt; pnxt = tp; }
        if (tid == 0) { sh.npend = sh.npend2; sh.nfront = sh.nnodes - sh.fbase; if (sh.nfront) sh.tmax = t; }
        __syncthreads();
        // ---- close layer t under same-layer lifts ---------------------------
        if (sh.status) break;
        const uint32_t r = sh.r;
        BFS_PROF(if (A.dbg && tid == 0) { atomicAdd(&g_bfs_prof[5], __builtin_amdgcn_s_memtime() - lf0); atomicAdd(&g_bfs_prof[6], 1ULL); })
        while (sh.nfront > 0 && !sh.status) {
            rounds++;
            const unsigned nf = sh.nfront;
            const unsigned long long rt0 = __builtin_amdgcn_s_memtime();
            const int mode_at = sh.mode;
            if (tid == 0) {
                sh.fbase = sh.nnodes;
                // the sequential search settled this key: stop at the next round
                if (A.claim && __hip_atomic_load(&A.claim[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                    sh.status |= 4;
            }
            __syncthreads();
            BFS_PROF(unsigned long long pt = 0;
            if (A.dbg && tid == 0) { pt = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof[0], pt - rt0); atomicAdd(&g_bfs_prof[4], 1ULL); })
            if (sh.status & 4) break;
            for (;;) {
            // one configuration per lane, its members eight at a time in series
            // (round 2's layout; round 3 split a round into (configuration, 8
            // members) items over every wave, JH_BFS_ITEMS=1: measured in round
            // 4 on one box, C4 250 -> 222 ms, C3 ranks 0 / 3 / 6 43.3 / 72.7 /
            // 82.6 -> 41.3 / 70.8 / 78.3 ms with this layout; the bisect of
            // round 3's C4 regression pointed at that change, profiles/r04/)
            const unsigned ng = JH_BFS_ITEMS ? (unsigned)(w + 7) >> 3 : 1u;
            const unsigned items = nf * ng;
            for (unsigned i0 = tid - lane; i0 < items; i0 += BFS_THREADS) {
                const unsigned it = i0 + lane;
                BFS_PROF(unsigned long long pq0 = A.dbg && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;)
                const unsigned i = it < items ? it / ng : 0;
                const uint64_t c = it < items ? fcur[i] : 0xFFFFFFFFull;    // past the end: every member taken
                const uint32_t s = (uint32_t)(c >> 32), mask = (uint32_t)c;
                const int jb = JH_BFS_ITEMS && it < items ? (int)(it - i * ng) * 8 : 0;
                const int je = JH_BFS_ITEMS ? jb + 8 : w;
                for (int j0 = jb; j0 < je; j0 += 8) {
                    uint64_t ck[8];       // same-layer children of members j0..j0+7: s2 << 32 | mask'
                    uint64_t pe = 0;      // the cross-layer child (member r), appended per wave
                    bool hp = false;
                    Win8 wn;
                    win8(sh, j0, wn);
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        ck[q] = 0;
                        const int j = j0 + q;
                        if (j >= w || ((mask >> j) & 1)) continue;
                        const uint32_t f = wn.f[q], vv = wn.vv[q];
                        const int v1 = (int)(vv & 0xFFFF), v2 = (int)(vv >> 16);
                        int s2;
                        if (!cas_step((int)f, v1, v2, (int)s, &s2)) continue;
                        if ((uint32_t)j == r) {
                            // cross-layer edge: drop RET members until one is not linearized
                            uint64_t nm = mask | (1u << j);
                            uint32_t u = t, ru = r;
                            for (;;) {
                                nm = drop_bit(nm, ru);
                                u++;
                                if (u >= n_ok) break;
                                ru = rpos[u];
                                if (!((nm >> ru) & 1)) break;
                            }
                            if (u >= n_ok) { sh.term = 1; continue; }   // a terminal configuration
                            pe = bfs_pack(u, (uint32_t)s2, (uint32_t)nm);
                            hp = true;
                        } else {
                            ck[q] = ((uint64_t)(uint32_t)s2 << 32) | (mask | (1u << j));
                        }
                    }
                    if (const uint64_t pm = ballot(hp)) {
                        unsigned pb = 0;
                        if (lane == 0) pb = atomicAdd(&sh.npend, (unsigned)__popcll(pm));
                        pb = readlane(pb, 0);
                        if (hp) {
                            const unsigned pos = pb + mbcnt(pm);
                            if (pos < A.q_cap) pcur[pos] = pe;
                            else atomicOr(&sh.status, 2);
                        }
                    }
                    BFS_PROF(if (A.dbg && tid == 0) { const unsigned long long q = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof[7], q - pq0); pq0 = q; })
                    bool nw[8];
                    insert8(ck, nw);
                    BFS_PROF(if (A.dbg && tid == 0) { const unsigned long long q = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof_x[0], q - pq0); pq0 = q; })
                    record8(ck, nw);
                    BFS_PROF(if (A.dbg && tid == 0) { const unsigned long long q = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof_x[1], q - pq0); atomicAdd(&g_bfs_prof_x[2], 1ULL); })
                }
            }
            BFS_PROF(if (A.dbg && tid == 0) { const unsigned long long q = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof[1], q - pt); pt = q; })
            __syncthreads();
            BFS_PROF(if (A.dbg && tid == 0) { const unsigned long long q = __builtin_amdgcn_s_memtime(); atomicAdd(&g_bfs_prof[2], q - pt); pt = q; })
            if (sh.ovf) { migrate(); continue; }
            break;
            }
            { uint64_t *tp = fcur; fcur = fnxt; fnxt = tp; }
            if (sh.mode == 0 && sh.lcount > LSET / 2 && !sh.status) migrate();
            if (tid == 0) sh.nfront = sh.nnodes - sh.fbase;
            if (A.dbg && tid == 0) {
                // JH_DEBUG=2: rounds and cycles with the layer in the global set (mode 1)
                unsigned long long *d = A.dbg + 16 * (size_t)blockIdx.x;
                if (mode_at) { d[9] += __builtin_amdgcn_s_memtime() - rt0; d[10] += 1; d[11] += nf; }
                else { d[12] += __builtin_amdgcn_s_memtime() - rt0; d[13] += nf; }
            }
            __syncthreads();
            BFS_PROF(if (A.dbg && tid == 0) atomicAdd(&g_bfs_prof[3], __builtin_amdgcn_s_memtime() - pt);)
        }
        if (sh.status) break;
    }
    if (tid == 0) sh.count = sh.nnodes;                  // initial included, terminals not
    __syncthreads();
    if (A.dbg && tid == 0) {
        unsigned long long *d = A.dbg + 16 * (size_t)blockIdx.x;
        d[0] += __builtin_amdgcn_s_memtime() - b0; d[1] += rounds; d[3] += sh.count; d[4] += 1;
    }
    if (sh.status) {
        if (tid == 0 && !(sh.status & 4)) A.unres_list[atomicAdd(A.unres_count, 1)] = key;
    } else if (A.linear) {
        // JIT linearization's verdict: the configuration set survives the last return or not
        if (A.cfg_slot && A.cfg_slot[key] >= 0 && !sh.nostore)
            bfs_dump_configs(A, sh, tid, key, ops, woff, W, rpos, n_ok, sh.term != 0);
        __syncthreads();
        if (wid == 0) {
            jh_key_verdict v;
            v.valid = sh.term ? JH_VALID : JH_INVALID;
            v.cause = CAUSE_BY_LINEAR;
            v.explored = (int64_t)sh.count - 1;
            v.fail_entry = sh.term ? -1 : ret_row(A.src, K, sh.tmax, lane);
            if (lane == 0) emit_verdict(A.out, A.claim, key, v);
        }
    } else if (sh.term && !A.exact_count && (long long)sh.count <= A.budget) {
        // valid for certain (round 5): WGL's cache -- the path's configurations
        // and the dead ones left of it, one terminal included -- is a subset of
        // the reachable set (sh.count, initial included, terminals not), so WGL
        // cannot have run out of budget; no count pass unless asked for
        if (tid == 0) {
            jh_key_verdict v;
            v.valid = JH_VALID; v.cause = 0; v.fail_entry = -1; v.explored = JH_EXPLORED_UNCOUNTED;
            emit_verdict(A.out, A.claim, key, v);
        }
    } else if (sh.term) {
        // valid, or :unknown if WGL's count passes the budget: WGL's exact count
        if (tid == 0) { if (n_ok < A.lcap) A.lstart[n_ok] = sh.nnodes; sh.ok = 0; }
        __syncthreads();
        bfs_wgl_count(A, sh, tid, key, ops, woff, W, rpos, n_ok);
        if (tid == 0) {
            if (!sh.ok) {
                A.unres_list[atomicAdd(A.unres_count, 1)] = key;
            } else {
                jh_key_verdict v;
                v.cause = 0; v.fail_entry = -1;
                const unsigned long long cnt = sh.plen + sh.ccount;
                if ((long long)cnt <= A.budget) { v.valid = JH_VALID; v.explored = (int64_t)cnt; }
                else { v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_BUDGET; v.explored = A.budget; }
                if (A.dbg_plen) { v.fail_entry = (int64_t)sh.plen; v.cause = (int32_t)sh.nnodes; v.explored = (int64_t)cnt; }   // debugging
                emit_verdict(A.out, A.claim, key, v);
            }
        }
    } else if ((long long)sh.count - 1 > A.budget) {
        // no terminal, more reachable configurations than the budget: WGL stops at it
        if (tid == 0) {
            jh_key_verdict v;
            v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_BUDGET; v.fail_entry = -1; v.explored = A.budget;
            emit_verdict(A.out, A.claim, key, v);
        }
    } else if (wid == 0) {
        jh_key_verdict v;
        v.valid = JH_INVALID; v.cause = 0;
        v.explored = (int64_t)sh.count - 1;           // the initial configuration is not cached
        v.fail_entry = ret_row(A.src, K, sh.tmax, lane);
        if (lane == 0) emit_verdict(A.out, A.claim, key, v);
    }
    __syncthreads();
}

__global__ void __launch_bounds__(BFS_THREADS) k_lin_bfs(BfsArgs A0) {
    BfsShared &sh = *(BfsShared *)jh_lds;
    BfsArgs A = A0;                      // this workgroup's slices of the count buffers
    A.nodes += (size_t)blockIdx.x * A.ncap;
    A.lstart += (size_t)blockIdx.x * A.lcap;
    A.ent += (size_t)blockIdx.x * A.hcap;
    A.slot += (size_t)blockIdx.x * A.ncap;
    A.vis += (size_t)blockIdx.x * (A.ncap / 32 + 1);
    A.tmp += (size_t)blockIdx.x * A.ncap;
    A.tmpk += (size_t)blockIdx.x * A.ncap;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint64_t *gset = A.gset + (size_t)blockIdx.x * A.gset_cap;
    uint64_t *pend = A.pend + (size_t)blockIdx.x * 2 * A.q_cap;
    uint64_t *front = A.front + (size_t)blockIdx.x * 2 * A.q_cap;
    char *gscr = A.scratch + (size_t)blockIdx.x * A.scratch_bytes;
    bool spanned = false;
    for (;;) {
        if (tid == 0) {
            const int idx = atomicAdd(A.queue, 1);
            if (A.live_n) sh.key = stream_key(A.list, A.live_n, A.p1_done, A.p1_tot, idx, A.src.flags);
            else sh.key = idx < A.n_list ? A.list[idx] : -1;
        }
        __syncthreads();
        const int key = sh.key;
        if (key < 0) break;
        if (A.t_span && !spanned && tid == 0) atomicMin(&A.t_span[0], __builtin_amdgcn_s_memrealtime());
        spanned = true;
        TL_REC(A.tl, key, 0);
        if (wid == 0) {
            KeyInfo K;
            jh_key_verdict v;
            const bool need = key_pass1(A.src, key, lane, K, v);
            if (lane == 0) { sh.K = K; sh.v = v; sh.need = need; }
        }
        __syncthreads();
        if (!sh.need) {
            if (tid == 0) emit_verdict(A.out, A.claim, key, sh.v);
            // jh_lin_configs on a key with no :ok op (valid, no search): its one
            // configuration is the initial one, every crashed op pending
            if (wid == 0 && A.cfg_slot && A.cfg_slot[key] >= 0 && sh.v.valid == JH_VALID && sh.v.explored == 0 &&
                sh.K.n_ok == 0)
                bfs_dump_initial(A, sh, lane, key);
            __syncthreads();
            continue;
        }
        const uint64_t need = tbl_bytes(sh.K) + (uint64_t)sh.K.n_ok + 16;
        if (need <= (uint64_t)BFS_TBL) bfs_key<true>(A, sh, gscr, tid, gset, pend, front);
        else if (need <= A.scratch_bytes) bfs_key<false>(A, sh, gscr, tid, gset, pend, front);
        else {
            if (tid == 0) A.unres_list[atomicAdd(A.unres_count, 1)] = key;
            __syncthreads();
        }
        TL_REC(A.tl, key, 1);
    }
    if (A.t_span && tid == 0) atomicMax(&A.t_span[1], __builtin_amdgcn_s_memrealtime());
}

// Invalid keys settled by the DFS carry -(tmax + 2): the failing row is the
// ok completion of RET[tmax] (the first op no configuration gets past).
// ---------------------------------------------------------------------------
// Windows wider than 64 (up to JH_MAX_WINDOW = 256 members): the same WGL
// search in the same canonical coordinates (orc_wgl_canonical with its
// 4-word masks, oracle/jh_oracle.c), one wave per key, member j of W(t) in
// lane j mod 64 of slice j / 64. Such keys are rare (C5's 50-thread keys
// with many crashed ops) and almost all of them are deep searches, so this
// path is kept simple: tables in global scratch (ops, windows W(t) listed
// per layer), every configuration in the wave's HBM table (48-byte entries
// {mask[4], gen|t|state}, buckets of 4), the stack in HBM with its top
// XW_RING frames mirrored in LDS. A step is one HBM round trip per probed
// slice, plus one to load the next layer's members when t moves (a pop reads
// its frame from LDS; the frame carries the layer's window offset and width).
constexpr int XW_SL = JH_MAX_WINDOW / 64;        // mask words / member slices
constexpr uint32_t XW_HB = 4;                    // entries per bucket
constexpr int XW_EW = 6;                         // words per entry (the four-slice layout; the buffer's stride)
// Entries per search instantiation: SL mask words, then gen|t|state; the
// two-slice search (windows of 65-128 members, round 4) packs 4 words (32 B:
// a bucket is one 128-byte line), the four-slice one 6
template <int SL> struct XwL { static constexpr int EW = SL == 2 ? 4 : 6; };
constexpr int XW_FW = 8;                         // words per stack frame
// LDS ring of the top stack frames: 1.5 KB, under what k_lin_bfs's 157 KB
// leaves of a CU (the two share CUs in C5)
constexpr int XW_RING = 24;
// JH_XW_PROF builds: where a step's time goes (s_memtime, summed over waves)
#ifdef JH_XW_PROF
#define XW_PROF(x) x
#define XW_PROFA(x) , x
#else
#define XW_PROF(x)
#define XW_PROFA(x)
#endif
__device__ unsigned long long g_xw_prof[12];

struct XwArgs {
    KeySrc src;
    const int32_t *list;
    int32_t n_list;
    int32_t *queue;
    const KeyMeta *meta;
    jh_key_verdict *out;
    char *scratch;              // per wave: the key's tables
    uint64_t scratch_bytes;
    uint64_t *memo;             // per wave: memo_cap entries x XW_EW words
    uint32_t memo_cap;          // power of two
    uint64_t *stack;            // per wave: stack_cap frames x XW_FW words
    uint32_t stack_cap;
    int64_t budget;
    int32_t init_state;
    uint32_t gen_base;
    int32_t *flags;
    unsigned long long *probes;
    int32_t cause_or;           // :linear mode: CAUSE_BY_WGL on the verdicts (k_frontier)
    unsigned long long *t_span; // [first key taken, last wave end] (s_memrealtime), or null
    // jh_lin_configs for the keys the reachable-set engine cannot hold: the
    // frontier of each requested invalid key, from this search's table
    const int32_t *cfg_slot;
    jh_lin_config *cfg_out;
    int32_t *cfg_n;
    int64_t *cfg_rows;
    int32_t cfg_per;
    const int64_t *col_val, *col_val2;
    int64_t vmin, init_value;
    int32_t per_key_values;
};

struct XwTbl {
    uint32_t *rq;     // need | becomes << 16 (cas-register step, 04-checker.md:58-72)
    int32_t *rr;      // ok-return rank, -1 crashed
    int32_t *a;       // ok returns before the invocation (the op joins W(a))
    int32_t *woff;    // W(t) = W[woff[t] .. woff[t+1])
    uint32_t *W;      // op ids: 32-bit, long keys come here
    uint2 *P;         // {rq, rr} of W's ops, in W's order: a layer is one load
};
__device__ __forceinline__ XwTbl xw_tbl(char *tb, int n_ops, int n_ok, long long sumW) {
    XwTbl T;
    uint64_t o = 0;
    T.rq = (uint32_t *)(tb + o); o += a16((uint64_t)n_ops * 4);
    T.rr = (int32_t *)(tb + o); o += a16((uint64_t)n_ops * 4);
    T.a = (int32_t *)(tb + o); o += a16((uint64_t)n_ops * 4);
    T.woff = (int32_t *)(tb + o); o += a16((uint64_t)(n_ok + 1) * 4);
    T.W = (uint32_t *)(tb + o); o += a16((uint64_t)sumW * 4 + 1024);
    T.P = (uint2 *)(tb + o);
    return T;
}

// ops in call order and the windows of every layer; returns the widest
// window (JH_MAX_WINDOW + 1 if wider: the key is :unknown, cause window)
__device__ int xw_fill(const KeySrc &S, uint32_t s0, uint32_t s1, int n_ops, int n_ok,
                       long long sumW, int lane, const XwTbl &T) {
    {
        int nok = 0;
        for (uint32_t base = s0; base < s1; base += 64) {
            const uint32_t p = base + lane;
            const bool valid = p < s1;
            const int rk = valid ? S.rank[p] : -1;
            const bool kept = rk >= 0, ret = rk <= -2;
            const uint64_t br = ballot(ret);
            if (kept) {
                Rec x = S.rec[p];
                const int q = S.pair[p];
                int rr = -1, v1c = x.v1, v2c = x.v2;
                if (q >= 0) {
                    Rec y = S.rec[q];
                    if (y.type == T_OK) {
                        rr = -(S.rank[q] + 2);
                        if (x.f == F_CAS) { if (x.v1 == 0 && x.v2 == 0) { v1c = y.v1; v2c = y.v2; } }
                        else if (x.v1 == 0) v1c = y.v1;
                    }
                }
                T.rq[rk] = x.f == F_READ ? ((uint32_t)v1c | ((uint32_t)v1c << 16))
                         : x.f == F_WRITE ? (RQ_ANY | ((uint32_t)v1c << 16))
                         : ((uint32_t)v1c | ((uint32_t)v2c << 16));
                T.rr[rk] = rr;
                T.a[rk] = nok + mbcnt(br);
            }
            nok += __popcll(br);
        }
    }
    wave_sync();
    // W(t) = W(t-1) - {RET[t-1]} + the ops with a == t, in call order
    int maxw = 0, w = 0, nxt = 0;
    long long offt = 0, offp = 0;
    for (int t = 0; t < n_ok; t++) {
        int nk = 0;
        if (t > 0) {
            for (int k = 0; k < XW_SL; k++) {
                const int idx = 64 * k + lane;
                int prev = 0;
                bool keep = false;
                if (idx < w) { prev = T.W[offp + idx]; keep = T.rr[prev] != t - 1; }
                const uint64_t bk = ballot(keep);
                if (keep) {
                    T.W[offt + nk + mbcnt(bk)] = (uint32_t)prev;
                    T.P[offt + nk + mbcnt(bk)] = make_uint2(T.rq[prev], (uint32_t)T.rr[prev]);
                }
                nk += __popcll(bk);
            }
        }
        int added = 0;
        for (;;) {
            const int j = nxt + lane;
            const bool in = j < n_ops && T.a[j] <= t;
            const uint64_t ba = ballot(in);
            const int c = __popcll(ba);             // a is non-decreasing: a prefix
            if (in && nk + added + lane < JH_MAX_WINDOW) {
                T.W[offt + nk + added + lane] = (uint32_t)j;
                T.P[offt + nk + added + lane] = make_uint2(T.rq[j], (uint32_t)T.rr[j]);
            }
            added += c; nxt += c;
            if (c < 64) break;
        }
        w = nk + added;
        maxw = max(maxw, w);
        if (w > JH_MAX_WINDOW || offt + w > sumW) { maxw = max(maxw, JH_MAX_WINDOW + 1); break; }
        if (lane == 0) T.woff[t] = (int32_t)offt;
        offp = offt;
        offt += w;
        wave_sync();
    }
    if (lane == 0) T.woff[n_ok] = (int32_t)offt;
    wave_sync();
    return maxw;
}

// a configuration's hash: the XOR of one Zobrist word per linearized member
// (a child's is its parent's ^ its member's word; the RET child's, whose
// mask is re-indexed onto the next window, is a wave reduction), mixed once
// with (t, state) -- one 64-bit mix per probe instead of one per mask word
__device__ __forceinline__ uint64_t xw_zw(int b) { return jh_mix64(0x9E3779B97F4A7C15ULL * (uint64_t)(b + 1)); }
__device__ __forceinline__ uint64_t xw_hash(uint32_t t, uint32_t s, uint64_t hm) {
    return jh_mix64(hm ^ (((uint64_t)t << 32) | s));
}
template <int SL>
__device__ __forceinline__ uint64_t xw_zsum(const uint64_t *m, const uint64_t *zk, int lane) {
    uint64_t x = 0;
#pragma unroll
    for (int q = 0; q < SL; q++) x ^= ((m[q] >> lane) & 1) ? zk[q] : 0ULL;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
    return rfl64(x);
}

// probe: slot | absent << 32 (absent: the slot an insert of this key takes)
template <int SL>
__device__ uint64_t xw_probe(const uint64_t *memo, uint32_t cap_mask, uint32_t gen, uint32_t t,
                             uint32_t s, const uint64_t *m, uint64_t hm, unsigned long long &probes) {
    constexpr int EW = XwL<SL>::EW, E2 = EW / 2;           // 16-byte pairs per entry
    const uint64_t want = ((uint64_t)gen << 40) | ((uint64_t)t << 20) | s;
    uint32_t b = (uint32_t)xw_hash(t, s, hm) & cap_mask & ~(XW_HB - 1);
    for (;;) {
        const ulonglong2 *B = (const ulonglong2 *)(memo + (size_t)b * EW);
        ulonglong2 e[XW_HB * E2];
#pragma unroll
        for (uint32_t j = 0; j < XW_HB * E2; j++) e[j] = B[j];
        probes++;
        int empty = -1, hit = -1;
#pragma unroll
        for (int j = XW_HB - 1; j >= 0; j--) {
            const ulonglong2 *x = e + E2 * j;
            const uint64_t w1 = SL == 2 ? x[1].x : x[2].x;
            if ((w1 >> 40) != gen) empty = j;
            bool eq = w1 == want && x[0].x == m[0] && x[0].y == m[1];
            if constexpr (SL == 4) eq = eq && x[1].x == m[2] && x[1].y == m[3];
            if (eq) hit = j;
        }
        if (hit >= 0 && (empty < 0 || hit < empty)) return b + (uint32_t)hit;
        if (empty >= 0) return (1ULL << 32) | (b + (uint32_t)empty);
        b = (b + XW_HB) & cap_mask;
    }
}

template <int SL>
__device__ __forceinline__ void xw_store(uint64_t *memo, uint32_t slot, uint32_t gen, uint32_t t,
                                         uint32_t s, const uint64_t *m) {
    uint64_t *e = memo + (size_t)slot * XwL<SL>::EW;
    for (int w = 0; w < SL; w++)
        __hip_atomic_store(&e[w], m[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&e[SL], ((uint64_t)gen << 40) | ((uint64_t)t << 20) | s, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}

// jh_lin_configs beyond the reachable-set engine (windows over 32 members,
// >= 4096 states): for an invalid key this search's table holds every
// configuration it reached (WGL's cache is the whole reachable set), so the
// frontier is the table's entries of the key's generation at layer tmax (and
// the root when tmax is 0, which is never inserted). The first cfg_per of them
// in the canonical order -- state id (= register value order), then the
// window mask as a 256-bit number -- by repeated wave minima, each written as
// bfs_dump_configs writes its own: value, then the invocation rows of the
// linearized and the pending members of W(tmax) in call order.
struct Cfg5 { uint32_t s; uint64_t m3, m2, m1, m0; };
__device__ __forceinline__ bool cfg_less(const Cfg5 &a, const Cfg5 &b) {
    if (a.s != b.s) return a.s < b.s;
    if (a.m3 != b.m3) return a.m3 < b.m3;
    if (a.m2 != b.m2) return a.m2 < b.m2;
    if (a.m1 != b.m1) return a.m1 < b.m1;
    return a.m0 < b.m0;
}
template <int SL>
__device__ void xw_dump_configs(const XwArgs &A, const uint64_t *memo, uint32_t gen, uint32_t tmax, int key,
                                const XwTbl &T, int lane) {
    const int slot = A.cfg_slot[key];
    if (slot < 0) return;
    const uint32_t s0 = A.src.off[key], s1 = A.src.off[key + 1];
    const int wo = T.woff[tmax], w = T.woff[tmax + 1] - wo;
    // the invocation row of every member of W(tmax): member 64 c + lane in wrow[c]
    long long wrow[XW_SL];
#pragma unroll
    for (int c = 0; c < XW_SL; c++) {
        wrow[c] = -1;
        const int j = 64 * c + lane;
        if (j < w) {
            const int32_t id = (int32_t)T.W[wo + j];
            for (uint32_t p = s0; p < s1; p++)
                if (A.src.rank[p] == id) { wrow[c] = (long long)A.src.rows[p]; break; }
        }
    }
    const int per = min(A.cfg_per, CFG_MAX);
    KeyInfo Ki{};
    Ki.s0 = s0; Ki.s1 = s1;
    const long long lrow = tmax == 0 ? -1 : ret_row(A.src, Ki, tmax - 1, lane);   // :last-op, RET[tmax - 1]
    Cfg5 prev{0, 0, 0, 0, 0};
    int n = 0;
    for (int i = 0; i < per; i++) {
        Cfg5 best{0xFFFFFFFFu, ~0ULL, ~0ULL, ~0ULL, ~0ULL};
        bool have = false;
        auto offer = [&](const Cfg5 &c) {
            if ((i == 0 || cfg_less(prev, c)) && (!have || cfg_less(c, best))) { best = c; have = true; }
        };
        if (tmax == 0 && lane == 0) offer(Cfg5{(uint32_t)A.init_state, 0, 0, 0, 0});
        for (uint32_t j = (uint32_t)lane; j < A.memo_cap; j += 64) {
            const uint64_t *e = memo + (size_t)j * XwL<SL>::EW;
            const uint64_t e4 = e[SL];
            if ((uint32_t)(e4 >> 40) != gen || ((uint32_t)(e4 >> 20) & T_MASK) != tmax) continue;
            offer(Cfg5{(uint32_t)e4 & STATE_MASK, SL == 4 ? e[3] : 0ULL, SL == 4 ? e[2] : 0ULL, e[1], e[0]});
        }
        // wave minimum of the lanes' best
        for (int o = 32; o > 0; o >>= 1) {
            Cfg5 x;
            x.s = (uint32_t)__shfl_xor((int)best.s, o);
            x.m3 = (uint64_t)__shfl_xor((long long)best.m3, o); x.m2 = (uint64_t)__shfl_xor((long long)best.m2, o);
            x.m1 = (uint64_t)__shfl_xor((long long)best.m1, o); x.m0 = (uint64_t)__shfl_xor((long long)best.m0, o);
            const bool xh = __shfl_xor((int)have, o) != 0;
            if (xh && (!have || cfg_less(x, best))) { best = x; have = true; }
        }
        if (!have) break;
        prev = best;
        n = i + 1;
        const long long val = cfg_state_value(best.s, A.per_key_values, A.vmin, A.init_value, A.src, s0, s1,
                                              A.col_val, A.col_val2, lane);
        const int64_t o = ((int64_t)slot * A.cfg_per + i) * CFG_ROWS;
        const uint64_t mw[XW_SL] = {best.m0, best.m1, best.m2, best.m3};
        int nl = 0, np = 0;
#pragma unroll
        for (int c = 0; c < XW_SL; c++) nl += __popcll(ballot(64 * c + lane < w && ((mw[c] >> lane) & 1)));
#pragma unroll
        for (int c = 0; c < XW_SL; c++) {
            const bool in = 64 * c + lane < w, lin = in && ((mw[c] >> lane) & 1);
            const uint64_t bl = ballot(lin), bp = ballot(in && !lin);
            int lo = 0, po = 0;
            for (int c2 = 0; c2 < c; c2++) {
                const bool in2 = 64 * c2 + lane < w, lin2 = in2 && ((mw[c2] >> lane) & 1);
                lo += __popcll(ballot(lin2));
                po += __popcll(ballot(in2 && !lin2));
            }
            if (lin) A.cfg_rows[o + lo + mbcnt(bl)] = wrow[c];
            if (in && !lin) A.cfg_rows[o + nl + po + mbcnt(bp)] = wrow[c];
            np += __popcll(bp);
        }
        if (lane == 0) {
            jh_lin_config cf;
            cf.key = key; cf.model_value = val; cf.n_linearized = nl; cf.n_pending = np; cf.rows_off = o;
            cf.last_row = lrow;
            A.cfg_out[(int64_t)slot * A.cfg_per + i] = cf;
        }
    }
    if (lane == 0) A.cfg_n[slot] = n;
}

// one wave of the 65-256-member search: wave wv's tables, nm_sh / ring in LDS
// (k_lin_xw's own, or the dynamic LDS of k_lin_seq_lwx's xw role)
// One key's search once its tables are built (xw_fill): SL mask words, the
// two-slice instantiation for windows of 65-128 members, the four-slice one
// for 129-256. Same search order and memo contents either way.
template <int SL>
__device__ __forceinline__ void xw_search(const XwArgs &A, int key, const XwTbl &T, int n_ok, uint64_t *memo,
                                          uint64_t *stk, const uint64_t *zk, unsigned long long *nm_sh,
                                          uint64_t *ring, unsigned long long &my_probes
                                          XW_PROFA(unsigned long long *pf)) {
    const int lane = threadIdx.x;
    const uint32_t cap_mask = A.memo_cap - 1;
    jh_key_verdict v;
    {
        const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
        const uint32_t budget = (uint32_t)min<int64_t>(A.budget, 0x7FFFFFFF);

        // the current layer's members: member 64k + lane in slice k
        uint32_t t = 0, tmax = 0, s = (uint32_t)A.init_state, ins = 0, depth = 0;
        uint64_t mask[SL];
#pragma unroll
        for (int q = 0; q < SL; q++) mask[q] = 0;
        uint32_t mrq[SL];
        int32_t mrr[SL];
        int w = 0, r = 0, start = 0, lo = 0;
        // after a pop: the popped member's slice and which of its children
        // were absent when the parent took that member. The table never
        // drops an entry, so the others are still present: only these are
        // probed again (none left: no round trip for the slice)
        int k_known = -1;
        uint64_t abs_known = 0;
        // layer t's members: W(t) = P[o .. o + w)
        auto load_layer = [&](int o, int wt) {
            XW_PROF(const unsigned long long l0 = __builtin_amdgcn_s_memtime();)
            lo = o; w = wt;
            r = 0;
#pragma unroll
            for (int k = 0; k < SL; k++) {
                const int j = 64 * k + lane;
                mrq[k] = RQ_EMPTY; mrr[k] = -2;
                if (j < w) { const uint2 pr = T.P[o + j]; mrq[k] = pr.x; mrr[k] = (int32_t)pr.y; }
                const uint64_t b = ballot(j < w && mrr[k] == (int32_t)t);
                if (b) r = 64 * k + __builtin_ctzll(b);
            }
            XW_PROF(pf[2] += __builtin_amdgcn_s_memtime() - l0; pf[7]++;)
        };
        load_layer(T.woff[0], T.woff[1] - T.woff[0]);
        uint32_t rlo = 0;      // the LDS ring holds frames [rlo, depth)
        uint64_t hm = 0;       // Zobrist sum of the configuration's mask
        XW_PROF(const unsigned long long k0 = __builtin_amdgcn_s_memtime();)
        int verdict = -1;
        for (;;) {
            // expand: candidates from `start` on, in call order, slice by slice
            bool took = false;
            uint32_t u_r = t;
            uint64_t nm_r[SL], hr = 0;
#pragma unroll
            for (int q = 0; q < SL; q++) nm_r[q] = 0;
            bool lifted = false;
            int wo0 = 0, wo1 = 0;          // woff[u_r], woff[u_r + 1]: loaded beside the probes
            // unrolled: static slice indices (no register-array selects, no
            // SGPR spills: 4.02 -> 3.37 s of C5's k_lin_xw)
#pragma unroll
            for (int k = 0; k < SL && !took; k++) {
                if (64 * k >= w) break;
                const int j = 64 * k + lane;
                const uint32_t req = mrq[k] & 0xFFFF;
                const bool cl = j < w && j >= start && !((mask[k] >> lane) & 1) && (req == s || req == RQ_ANY) &&
                                (k != k_known || ((abs_known >> lane) & 1));
                const uint64_t cand = ballot(cl);
                if (!cand) continue;
                if (!lifted && (r >> 6) == k && ((cand >> (r & 63)) & 1)) {
                    // the RET child: lift RET[t], keep lifting while the next
                    // layer's RET op is already linearized, compact onto W(u)
                    XW_PROF(const unsigned long long f0 = __builtin_amdgcn_s_memtime();)
                    lifted = true;
                    uint64_t lin[SL];
#pragma unroll
                    for (int q = 0; q < SL; q++) lin[q] = mask[q];
                    lin[r >> 6] |= 1ULL << (r & 63);
                    uint32_t u = t + 1;
                    while (u < (uint32_t)n_ok) {
                        bool hit = false;
#pragma unroll
                        for (int q = 0; q < SL; q++) hit |= ((lin[q] >> lane) & 1) && mrr[q] == (int32_t)u;
                        if (!ballot(hit)) break;
                        u++;
                    }
                    u_r = u;
                    if (u < (uint32_t)n_ok) {
                        wo0 = T.woff[u]; wo1 = T.woff[u + 1];
                        if (lane < SL) nm_sh[lane] = 0;
                        wave_sync();
                        int base = 0;
#pragma unroll
                        for (int q = 0; q < SL; q++) {
                            const bool kept = 64 * q + lane < w && (mrr[q] < 0 || mrr[q] >= (int32_t)u);
                            const uint64_t bk = ballot(kept);
                            const int pos = base + mbcnt(bk);
                            if (kept && ((lin[q] >> lane) & 1)) atomicOr(&nm_sh[pos >> 6], 1ULL << (pos & 63));
                            base += __popcll(bk);
                        }
                        wave_sync();
#pragma unroll
                        for (int q = 0; q < SL; q++) nm_r[q] = rfl64(nm_sh[q]);
                        wave_sync();
                        hr = xw_zsum<SL>(nm_r, zk, lane);
                    }
                    XW_PROF(pf[9] += __builtin_amdgcn_s_memtime() - f0;)
                }
                // every candidate lane probes its child
                const bool is_r = j == r;
                uint64_t cm[SL];
#pragma unroll
                for (int q = 0; q < SL; q++) cm[q] = is_r ? nm_r[q] : (mask[q] | (q == k ? (1ULL << lane) : 0ULL));
                const uint32_t ct = is_r ? u_r : t, cs = mrq[k] >> 16;
                const uint64_t chm = is_r ? hr : (hm ^ zk[k]);
                bool found = false;
                uint32_t slot = 0;
                XW_PROF(const unsigned long long q0 = __builtin_amdgcn_s_memtime();)
                if (cl) {
                    const uint64_t pr = xw_probe<SL>(memo, cap_mask, gen, ct, cs, cm, chm, my_probes);
                    found = (pr >> 32) == 0;
                    slot = (uint32_t)pr;
                }
                const uint64_t absent = cand & ~ballot(found);
                XW_PROF(pf[1] += __builtin_amdgcn_s_memtime() - q0; pf[6]++;)
                if (!absent) continue;
                const int i = __builtin_ctzll(absent);
                if (ins >= budget) { verdict = JH_UNKNOWN; break; }
                ins++;
                XW_PROF(const unsigned long long h0 = __builtin_amdgcn_s_memtime();)
                if (lane == i) xw_store<SL>(memo, slot, gen, ct, cs, cm);
                // push the parent (t, its window, member, s, mask): HBM, and
                // the LDS ring slot a pop reads while the frame stays in it
                if (lane == 0) {
                    uint64_t *f = stk + (size_t)depth * XW_FW;
                    uint64_t *g = ring + (depth % XW_RING) * XW_FW;
                    const uint64_t f4 = ((uint64_t)t << 32) | ((uint32_t)w << 16) | (uint32_t)(64 * k + i);
                    const uint64_t f5 = ((uint64_t)(uint32_t)lo << 32) | s;
#pragma unroll
                    for (int q = 0; q < SL; q++) { f[q] = mask[q]; g[q] = mask[q]; }
                    f[4] = f4; f[5] = f5; f[6] = hm; f[7] = absent;
                    g[4] = f4; g[5] = f5; g[6] = hm; g[7] = absent;
                }
                depth++;
                if (depth - rlo > (uint32_t)XW_RING) rlo = depth - XW_RING;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                XW_PROF(pf[4] += __builtin_amdgcn_s_memtime() - h0; pf[5]++;)
                s = (uint32_t)readlane((int)cs, i);
                hm = readlane64(chm, i);
                const uint32_t nt = (uint32_t)readlane((int)ct, i);
#pragma unroll
                for (int q = 0; q < SL; q++) mask[q] = readlane64(cm[q], i);
                took = true;
                start = 0;
                k_known = -1;
                if (nt != t) {
                    t = nt;
                    tmax = max(tmax, t);
                    if (t >= (uint32_t)n_ok) { verdict = JH_VALID; break; }
                    load_layer(wo0, wo1 - wo0);     // nt != t only for the RET child: t == u_r
                }
            }
            if (verdict >= 0) break;
            if (took) continue;
            // pop
            if (depth == 0) { verdict = JH_INVALID; break; }
            XW_PROF(const unsigned long long o0 = __builtin_amdgcn_s_memtime();)
            depth--;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint64_t ti, f5;
            if (depth >= rlo) {
                const uint64_t *g = ring + (depth % XW_RING) * XW_FW;
#pragma unroll
                for (int q = 0; q < SL; q++) mask[q] = rfl64(g[q]);
                ti = rfl64(g[4]); f5 = rfl64(g[5]); hm = rfl64(g[6]); abs_known = rfl64(g[7]);
            } else {
                const uint64_t *f = stk + (size_t)depth * XW_FW;
#pragma unroll
                for (int q = 0; q < SL; q++) mask[q] = rfl64(f[q]);
                ti = rfl64(f[4]); f5 = rfl64(f[5]); hm = rfl64(f[6]); abs_known = rfl64(f[7]);
                rlo = depth;
                XW_PROF(pf[10]++;)
            }
            s = (uint32_t)f5;
            start = (int)(ti & 0xFFFF) + 1;
            k_known = (int)(ti & 0xFFFF) >> 6;
            const uint32_t pt = (uint32_t)(ti >> 32);
            XW_PROF(pf[3] += __builtin_amdgcn_s_memtime() - o0; pf[8]++;)
            if (pt != t) { t = pt; load_layer((int)(f5 >> 32), (int)((ti >> 16) & 0xFFFF)); }
        }
        XW_PROF(pf[0] += __builtin_amdgcn_s_memtime() - k0; pf[11]++;)
        v.valid = verdict;
        v.cause = (verdict == JH_UNKNOWN ? JH_CAUSE_BUDGET : 0) | A.cause_or;
        v.explored = ins;
        v.fail_entry = verdict == JH_INVALID ? -(int64_t)tmax - 2 : -1;
        if (lane == 0) A.out[key] = v;
        if (A.cfg_slot && verdict == JH_INVALID) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            xw_dump_configs<SL>(A, memo, gen, tmax, key, T, lane);
        }
    }
}

#ifndef JH_XW_SL2
#define JH_XW_SL2 1     // the two-slice search for windows of 65-128 members (0: four slices for all)
#endif
__device__ __forceinline__ void xw_waves(const XwArgs &A, size_t wv, unsigned long long *nm_sh, uint64_t *ring) {
    const int lane = threadIdx.x;
    XW_PROF(unsigned long long pf[12] = {0};)
    char *tb = A.scratch + wv * A.scratch_bytes;
    uint64_t *memo = A.memo + wv * A.memo_cap * XW_EW;
    uint64_t *stk = A.stack + wv * A.stack_cap * XW_FW;
    uint64_t zk[XW_SL];          // this lane's members' Zobrist words
#pragma unroll
    for (int k = 0; k < XW_SL; k++) zk[k] = xw_zw(64 * k + lane);
    unsigned long long my_probes = 0;
    for (;;) {
        int idx = 0;
        if (lane == 0) idx = atomicAdd(A.queue, 1);
        idx = readlane(idx, 0);
        if (idx >= A.n_list) break;
        const int key = A.list[idx];
        if (A.t_span && idx < 64 && lane == 0) atomicMin(&A.t_span[0], __builtin_amdgcn_s_memrealtime());
        const KeyMeta mt = A.meta[key];
        const int n_ops = mt.n_ops, n_ok = mt.n_ok;
        const long long sumW = (long long)(uint32_t)mt.pad;
        jh_key_verdict v;
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW; v.fail_entry = -1; v.explored = 0;
        if (xw_bytes(n_ops, n_ok, sumW) > A.scratch_bytes || (uint32_t)n_ops + 2 > A.stack_cap) {
            if (lane == 0) { atomicOr(A.flags, 2); A.out[key] = v; }
            continue;
        }
        const XwTbl T = xw_tbl(tb, n_ops, n_ok, sumW);
        const int maxw = xw_fill(A.src, A.src.off[key], A.src.off[key + 1], n_ops, n_ok, sumW, lane, T);
        if (maxw > JH_MAX_WINDOW) {
            if (lane == 0) A.out[key] = v;
            continue;
        }
        if (JH_XW_SL2 && maxw <= 128) xw_search<2>(A, key, T, n_ok, memo, stk, zk, nm_sh, ring, my_probes XW_PROFA(pf));
        else xw_search<4>(A, key, T, n_ok, memo, stk, zk, nm_sh, ring, my_probes XW_PROFA(pf));
    }
    for (int o = 32; o > 0; o >>= 1) my_probes += __shfl_xor(my_probes, o);
    if (lane == 0 && A.probes) atomicAdd(A.probes, my_probes);
    if (A.t_span && lane == 0) atomicMax(&A.t_span[1], __builtin_amdgcn_s_memrealtime());
    XW_PROF(if (lane == 0) for (int k = 0; k < 12; k++) atomicAdd(&g_xw_prof[k], pf[k]);)
}
__global__ void __launch_bounds__(64) k_lin_xw(XwArgs A) {
    __shared__ unsigned long long nm_sh[XW_SL];
    __shared__ uint64_t ring[XW_RING * XW_FW];
    xw_waves(A, blockIdx.x, nm_sh, ring);
}
// The streaming heavy-key pass's grid behind phase 1 (one stream): the
// 65-256-member search (blocks 0..n_x-1: first, they are the longest), the
// deferred WIDE keys, then LEAN waves beyond the early grid's -- three roles
// so that the pass needs no more streams than the hardware has queues
struct DfsTriple { XwArgs x; DfsArgs w, l; int32_t n_x, n_w; };
constexpr int XW_LDS = (int)(XW_SL * 8 + XW_RING * XW_FW * 8);
__global__ void __launch_bounds__(64) k_lin_seq_lwx(DfsTriple P) {
    const int b = (int)blockIdx.x;
    if (b < P.n_x) xw_waves(P.x, (size_t)b, (unsigned long long *)jh_lds, (uint64_t *)(jh_lds + XW_SL * 8));
    else if (b < P.n_x + P.n_w) lin_dfs_waves<MemoWL, false, true, true>(P.w);
    else lin_dfs_waves<MemoM, true, false, true>(P.l);
}

__global__ void __launch_bounds__(256) k_fail_rows(KeySrc S, jh_key_verdict *out, int64_t K) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t key = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); key < K; key += nw) {
        const int64_t fe = out[key].fail_entry;
        if (fe > -2) continue;
        KeyInfo Ki;
        Ki.s0 = S.off[key]; Ki.s1 = S.off[key + 1];
        const long long row = ret_row(S, Ki, (uint32_t)(-fe - 2), lane);
        if (lane == 0) out[key].fail_entry = row;
    }
}

// The search frontier of every invalid key (include/jh.h): the failing row is
// the ok completion of RET[t]; last_op = that of RET[t-1], previous_ok = the
// last client :ok row before it in the key's segment. -1 for other keys.
// The analysis that decided a key (knossos' :analyzer, include/jh.h): in
// :linear mode the engines mark the cause word while searching (CAUSE_BY_LINEAR
// for the reachable-set analysis, CAUSE_BY_WGL for a WGL search standing in
// for it); an unmarked key took no search and gets the mode's own analyzer.
__global__ void __launch_bounds__(256) k_frontier(KeySrc S, jh_key_verdict *out, int64_t K, int linear_mode) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t key = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); key < K; key += nw) {
        const jh_key_verdict v = out[key];
        if (lane == 0) {
            out[key].analyzer = (v.cause & CAUSE_BY_LINEAR) ? JH_ANALYZER_LINEAR
                                : (v.cause & CAUSE_BY_WGL) ? JH_ANALYZER_WGL
                                : linear_mode ? JH_ANALYZER_LINEAR : JH_ANALYZER_WGL;
            out[key].cause = v.cause & 0xFF;
            out[key].reserved = 0;
        }
        long long prev = -1, last = -1;
        if (v.valid == JH_INVALID && v.fail_entry >= 0) {
            const uint32_t s0 = S.off[key], s1 = S.off[key + 1];
            int want = 0;     // rank code of RET[t] = -(t + 2); 0 = not found yet
            for (uint32_t base = s0; base < s1; base += 64) {
                const uint32_t p = base + lane;
                const bool in = p < s1;
                const long long row = in ? (long long)S.rows[p] : -1;
                const Rec x = in ? S.rec[p] : Rec{-1, 0, 0, 0, 0, 0};
                if (in && row == v.fail_entry) want = S.rank[p];
                if (in && row < v.fail_entry && x.proc >= 0 && x.type == T_OK) prev = max(prev, row);
            }
            for (int o = 32; o > 0; o >>= 1) {
                prev = max(prev, (long long)__shfl_xor(prev, o));
                want = min(want, __shfl_xor(want, o));
            }
            const int t = -want - 2;
            if (want <= -3) {   // t >= 1
                KeyInfo Ki;
                Ki.s0 = s0; Ki.s1 = s1;
                last = ret_row(S, Ki, (uint32_t)(t - 1), lane);
            }
        }
        if (lane == 0) { out[key].previous_ok = prev; out[key].last_op = last; }
    }
}

__global__ void k_summary(const jh_key_verdict *__restrict__ v, int64_t K, long long *sum) {
    // sum: [0] valid max [1] n_invalid [2] n_unknown [3] first_fail [4] n_keys [5] explored
    long long vmax = 0, ninv = 0, nunk = 0, ff = LLONG_MAX, nk = 0, ex = 0;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < K;
         k += (int64_t)gridDim.x * blockDim.x) {
        jh_key_verdict x = v[k];
        if (x.explored == -1) continue;                 // a key in no tuple
        // explored sums WGL insert counts only: not JH_EXPLORED_UNCOUNTED, and
        // not a stage-1 deferred key's progress (another unit)
        nk++; ex += (x.explored > 0 && x.cause != JH_CAUSE_DEFERRED) ? x.explored : 0;
        vmax = max(vmax, (long long)x.valid);
        if (x.valid == JH_INVALID) { ninv++; ff = min(ff, (long long)x.fail_entry); }
        if (x.valid == JH_UNKNOWN) nunk++;
    }
    for (int o = 32; o > 0; o >>= 1) {
        vmax = max(vmax, __shfl_xor(vmax, o));
        ninv += __shfl_xor(ninv, o); nunk += __shfl_xor(nunk, o);
        ff = min(ff, __shfl_xor(ff, o));
        nk += __shfl_xor(nk, o); ex += __shfl_xor(ex, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&sum[0], vmax);
        atomicAdd((unsigned long long *)&sum[1], (unsigned long long)ninv);
        atomicAdd((unsigned long long *)&sum[2], (unsigned long long)nunk);
        atomicMin(&sum[3], ff);
        atomicAdd((unsigned long long *)&sum[4], (unsigned long long)nk);
        atomicAdd((unsigned long long *)&sum[5], (unsigned long long)ex);
    }
}

// history entries of the keys in each of four lists (the deferred keys, LEAN,
// WIDE, the k_lin_xw keys): each phase's roofline bytes
struct EntryLists {
    const int32_t *list[5];
    int n[5];
    const int32_t *n_dev[5];       // if set: the list's length, on the device
    unsigned long long *sum[5];
    const uint32_t *off;
};
__global__ void __launch_bounds__(256) k_list_entries(EntryLists L) {
    const int y = blockIdx.y, n = L.n_dev[y] ? *L.n_dev[y] : L.n[y];
    const int32_t *list = L.list[y];
    unsigned long long x = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int k = list[i];
        x += L.off[k + 1] - L.off[k];
    }
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd(L.sum[y], x);
}

__global__ void k_iota(int32_t *a, int64_t n) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}

// Per-key dense interning of register values, for histories whose values
// span more than one 16-bit state range (unique values, wide ids). Every key
// numbers its own distinct values: 0 = nil, 1 = the initial value (when not
// nil), then the key's other values in order. The search compares states
// only for equality, so any per-key bijection leaves every configuration
// set, search order and count unchanged. Items are (record, v1|v2) pairs:
// radix-sorted by value, then stably by key, ranked by a scan of "new
// distinct value" flags within each key's item range [2*off[k], 2*off[k+1]).
__global__ void k_ival(const int64_t *__restrict__ v1, const int64_t *__restrict__ v2,
                       const int64_t *__restrict__ f, const uint32_t *__restrict__ rows, int64_t m,
                       uint64_t *__restrict__ u, uint32_t *__restrict__ idx) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 2 * m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t r = rows[i >> 1];
        int64_t raw = (i & 1) ? v2[r] : v1[r];
        if (f_code(f[r]) > F_CAS) raw = JH_NIL;
        u[i] = (uint64_t)raw ^ (1ULL << 63);           // signed order; nil -> 0
        idx[i] = (uint32_t)i;
    }
}
__global__ void k_ikey(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ rkey, int64_t n2,
                       uint32_t *__restrict__ key_of) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n2; j += (int64_t)gridDim.x * blockDim.x)
        key_of[j] = rkey[idx[j] >> 1];
}
__global__ void k_iflag(const uint32_t *__restrict__ idx, const uint64_t *__restrict__ u,
                        const uint32_t *__restrict__ rkey, const uint32_t *__restrict__ off, int64_t n2,
                        uint32_t *__restrict__ flag) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n2; j += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = idx[j];
        const uint64_t x = u[i];
        const uint32_t k = rkey[i >> 1];
        const bool first = j == 2 * (int64_t)off[k];
        flag[j] = (x != 0 && (first || u[idx[j - (first ? 0 : 1)]] != x)) ? 1u : 0u;
    }
}
// rank within the key: 1..n_distinct (0 for nil)
__device__ __forceinline__ uint32_t ival_rank(const uint32_t *P, const uint32_t *off, uint32_t k, int64_t j) {
    const int64_t s = 2 * (int64_t)off[k];
    return P[j] - (s > 0 ? P[s - 1] : 0u);
}
__global__ void k_iinit(const uint32_t *__restrict__ idx, const uint64_t *__restrict__ u,
                        const uint32_t *__restrict__ rkey, const uint32_t *__restrict__ off,
                        const uint32_t *__restrict__ P, int64_t n2, uint64_t init_u, uint32_t *__restrict__ r_init) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n2; j += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = idx[j];
        if (u[i] == init_u) { const uint32_t k = rkey[i >> 1]; r_init[k] = ival_rank(P, off, k, j); }
    }
}
__global__ void k_iassign(const uint32_t *__restrict__ idx, const uint64_t *__restrict__ u,
                          const uint32_t *__restrict__ rkey, const uint32_t *__restrict__ off,
                          const uint32_t *__restrict__ P, int64_t n2, int has_init, uint64_t init_u,
                          const uint32_t *__restrict__ r_init, Rec *__restrict__ rec,
                          unsigned long long *__restrict__ viol, unsigned int *__restrict__ maxid) {
    unsigned int mx = 0;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n2; j += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = idx[j];
        const uint64_t x = u[i];
        const uint32_t p = i >> 1, k = rkey[p];
        uint32_t id = 0;
        if (x != 0) {
            const uint32_t r = ival_rank(P, off, k, j);
            if (!has_init) id = r;
            else if (x == init_u) id = 1;
            else id = 1 + r - ((r_init[k] > 0 && r > r_init[k]) ? 1u : 0u);
        }
        if (id >= RQ_EMPTY - 1) {      // beyond the 16-bit state encoding: this key alone is :unknown
            atomicMin(&viol[k], ((unsigned long long)p << 4) | JH_CAUSE_STATES);
            id = 0;
        }
        if (i & 1) rec[p].v2 = (int32_t)id; else rec[p].v1 = (int32_t)id;
        mx = max(mx, id);
    }
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned int)__shfl_xor((int)mx, o));
    if ((threadIdx.x & 63) == 0) atomicMax(maxid, mx);
}

// widens the sorted row ids / segment offsets for the jh_key_index CSR
__global__ void k_widen(const uint32_t *__restrict__ a, int64_t n, int64_t *__restrict__ b) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

inline int bits_for(uint64_t x) {
    int b = 1;
    while ((1ULL << b) <= x) b++;
    return b;
}

}  // namespace

// ---------------------------------------------------------------------------
// Tuning and diagnostics knobs (JH_* environment variables) are read only by a
// build with -DJH_TUNING (tools/build_variants.sh): the release library ignores
// the environment. Options that change what a call does are jh_lin_opts fields.
static inline const char *tune_env(const char *name) {
#ifdef JH_TUNING
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Units (waves or workgroups) of per_unit bytes each that fit in HBM: at most
// `want`, at least 1. The buffers of `slots` count as free (they are what the
// units' tables replace); a reserve stays free, and no one kind of search
// table takes more than a quarter of the device. No query in the steady state
// (the slots already hold `want` units).
static int fit_units(jh_ctx *ctx, int want, uint64_t per_unit, std::initializer_list<int> slots) {
    if (want <= 1 || per_unit == 0) return std::max(want, 1);
    uint64_t held = 0;
    for (int sl : slots)
        if ((int)ctx->bufs.size() > sl) held += ctx->bufs[sl].bytes;
    if ((uint64_t)want * per_unit <= held) return want;
    size_t fr = 0, tot = 0;
    HIP_TRY(hipMemGetInfo(&fr, &tot));
    // (round 6: 1/16, was 1/32 -- the buffers sized outside fit_units grew with
    // the helpers, the spec board and the takeover's logs, and a second context
    // opened beside a first that holds ~140 GB ran out at budget 2^24)
    const uint64_t reserve = std::max<uint64_t>(4ULL << 30, tot / 16);
    // contexts sharing the device (jh_open_devices with a device listed more
    // than once; round 6: or opened one by one, device_open_contexts) may run
    // at once: each takes its share of what is free
    const uint64_t share = (uint64_t)std::max(ctx->share, device_open_contexts(ctx->device));
    uint64_t room = fr / share + held;
    room = room > reserve ? room - reserve : 0;
    room = std::min<uint64_t>(room, tot / (4 * share));
    const uint64_t fit = room / (per_unit + per_unit / 8);    // ws() allocates 1/8 over
    return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)want, fit));
}

// words of the per-call counter block q (device): queues, list lengths, probe
// and entry counters of the phases
constexpr int Q_WORDS = 104;
constexpr int Q_ENT_ALL = 24, Q_DEFER_L = 29, Q_DEFER_W = 30, Q_DEFER3W = 31;
constexpr int Q_PROBES_HELP = 32, Q_PROBES_P3 = 34, Q_PROBES_WIDE = 36;
constexpr int Q_ENT_LEAN = 40, Q_ENT_WIDE = 42, Q_ENT_XW = 44;
constexpr int Q_T_WIDE = 46;        // [46..47] first WIDE wave start, [48..49] last end (s_memrealtime)
// the streaming heavy-key pass (round 4): phase 1's finished keys, the LEAN
// sequential waves of both grids, the BFS's queue, and spans (first key taken,
// last wave end; s_memrealtime) of the BFS, the LEAN role, the xw role and phase 1
constexpr int Q_P1_DONE = 64, Q_SEQ_WAVES = 65, Q_BFS_QUEUE = 66;
constexpr int Q_T_BFS = 68, Q_T_LEAN = 72, Q_T_XW = 76, Q_T_P1 = 80;
constexpr int Q_ENT_P3 = 84;        // entries of the LEAN keys restarted in phase 3
constexpr int Q_RS_USED = 88;       // [88..89] resume records' bytes, [90] records published (round 5), [91] takeovers (round 6)
constexpr int Q_MAINS = 92;         // round 6: late helpers running a key now
constexpr int Q_SPEC = 96;          // round 6: [96..97] merged nodes, [98] merges, [99] spec jobs, [100] dead results
// LEAN sequential waves launched with the BFS while phase 1 still runs (the
// rest start behind phase 1): enough for the keys deferred before it ends
constexpr int EARLY_LEAN_WAVES = 128;
static inline int64_t q64(const int32_t *qh, int i) {
    return (int64_t)(((uint64_t)(uint32_t)qh[i + 1] << 32) | (uint32_t)qh[i]);
}

// stage 1 of a two-stage check: each deferred key comes back with its quick
// search's progress (deepest layer / layers, in millionths) as `explored`,
// the order the stage-2 pool takes them in (heaviest estimate first: the likely
// longest searches start first, as k_sort_defer orders a device's own pass)
__global__ void k_mark_deferred(const uint64_t *__restrict__ d64, int n, jh_key_verdict *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t pk = d64[i];
        jh_key_verdict v;
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_DEFERRED; v.fail_entry = -1; v.explored = (int64_t)(pk >> 32);
        v.previous_ok = -1; v.last_op = -1; v.analyzer = JH_ANALYZER_WGL; v.reserved = 0;
        out[(uint32_t)pk] = v;
    }
}

// stage 1 of a two-stage check: keys of a list (the 65-256-member keys) come
// back deferred with progress 0
__global__ void k_mark_list_deferred(const int32_t *__restrict__ list, int n, jh_key_verdict *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        jh_key_verdict v;
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_DEFERRED; v.fail_entry = -1; v.explored = 0;
        v.previous_ok = -1; v.last_op = -1; v.analyzer = JH_ANALYZER_WGL; v.reserved = 0;
        out[list[i]] = v;
    }
}

// jh_lin_configs: the k_lin_xw table bytes of the keys the reachable-set
// engine gave up (their configurations come from that search)
__global__ void k_xw_need(const int32_t *__restrict__ list, const int32_t *n, const KeyMeta *__restrict__ meta,
                          unsigned long long *need) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < *n) {
        const KeyMeta m = meta[list[i]];
        atomicMax(need, (unsigned long long)xw_bytes(m.n_ops, m.n_ok, (long long)(uint32_t)m.pad));
    }
}

// jh_lin_configs: the requested keys are the whole heavy list, all LEAN
__global__ void k_req_lists(const int64_t *__restrict__ keys, int n, int64_t K, int32_t *defer, int32_t *defer_l,
                            int32_t *q) {
    int m = 0;
    for (int i = 0; i < n; i++) {           // one thread: a handful of keys
        const int64_t k = keys[i];
        if (k < 0 || k >= K) continue;
        defer[m] = (int32_t)k; defer_l[m] = (int32_t)k; m++;
    }
    q[1] = m; q[29] = m; q[30] = 0;
}

void lin_check_independent(jh_ctx *ctx, const jh_history *dh, const jh_lin_opts *opts,
                           bool keyed, jh_key_verdict *out_dev, jh_summary *sum,
                           hipStream_t st, const LinCfgReq *cfgreq) {
    const int64_t n = dh->n;
    const int64_t K = keyed ? dh->n_keys : 1;
    if (K >= (1LL << 23)) throw_jh(JH_EUNSUPPORTED, "more than 2^23 keys in one call");
    if (n >= (1LL << 31)) throw_jh(JH_EUNSUPPORTED, "more than 2^31 entries in one call");
    const int64_t budget = opts && opts->budget > 0 ? opts->budget : JH_DEFAULT_BUDGET;
    const int64_t init = opts ? opts->init_value : JH_NIL;
    const int32_t lflags = opts ? opts->flags : 0;
    const bool linear_mode = (opts && opts->algorithm == JH_ALGO_LINEAR) || cfgreq;
    HIP_TRY(hipEventRecord(ctx->ev[0], st));

    // ranges
    RangeOut *ro = ctx->ws<RangeOut>(WS_MISC, 1);
    RangeOut ro_init{LLONG_MAX, LLONG_MIN, -1, 0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(ro, &ro_init, sizeof ro_init, hipMemcpyHostToDevice, st));
    if (n > 0)
        k_range<<<grid_for(n, 256, 4096), 256, 0, st>>>(dh->process, dh->f, keyed ? dh->key : nullptr,
                                                        dh->value, dh->value2, n, keyed ? 1 : 0, ro);
    RangeOut rh;
    HIP_TRY(hipMemcpyAsync(&rh, ro, sizeof rh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (keyed && rh.unkeyed_client)
        throw_jh(JH_EUNSUPPORTED, "client ops whose :value is not an independent tuple");
    if (rh.pmax > INT32_MAX) throw_jh(JH_EUNSUPPORTED, "process ids beyond int32");
    long long vmin = rh.vmin, vmax = rh.vmax;
    if (init != JH_NIL) { vmin = std::min<long long>(vmin, init); vmax = std::max<long long>(vmax, init); }
    if (vmin > vmax) { vmin = 0; vmax = 0; }
    // values spanning more than one 16-bit state range are interned per key
    // (k_ival..k_iassign) instead of as one global offset
    const bool per_key_values = (unsigned long long)(vmax - vmin) >= (unsigned long long)(RQ_EMPTY - 3) ||
                                (lflags & JH_LIN_INTERN_PER_KEY) != 0;
    const int init_state = init == JH_NIL ? 0 : per_key_values ? 1 : (int)(init - vmin + 1);
    long long n_states = vmax - vmin + 2;      // state ids 0 (nil) .. vmax - vmin + 1

    // partition by key
    uint32_t *kA = ctx->ws<uint32_t>(WS_KEYS_A, n), *kB = ctx->ws<uint32_t>(WS_KEYS_B, n);
    uint32_t *rA = ctx->ws<uint32_t>(WS_ROWS_A, n), *rB = ctx->ws<uint32_t>(WS_ROWS_B, n);
    if (n > 0)
        k_keys<<<grid_for(n, 256), 256, 0, st>>>(keyed ? dh->key : nullptr, n, K, keyed ? 1 : 0, kA, rA);
    const int endbit = bits_for((uint64_t)K);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kA, kB, rA, rB, (int)n, 0, endbit, st));
    void *tmp = ctx->ws<char>(WS_SORT_TMP, tb);
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kA, kB, rA, rB, (int)n, 0, endbit, st));
    uint32_t *off = ctx->ws<uint32_t>(WS_SEG_OFF, K + 2);
    k_seg_off<<<grid_for(K + 1, 256), 256, 0, st>>>(kB, n, K, off, ro);
    uint32_t m_keyed = 0;
    HIP_TRY(hipMemcpyAsync(&m_keyed, off + K, sizeof m_keyed, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&rh, ro, sizeof rh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int64_t m = m_keyed;
    const int smax = std::max(rh.smax, 1);

    Rec *rec = ctx->ws<Rec>(WS_REC, m);
    int32_t *pair = ctx->ws<int32_t>(WS_PAIR, m);
    unsigned long long *viol = ctx->ws<unsigned long long>(WS_VIOL, K);
    int32_t *rank = ctx->ws<int32_t>(WS_RANK, m);
    HIP_TRY(hipMemsetAsync(viol, 0xFF, sizeof(unsigned long long) * K, st));
    if (m > 0) {
        HIP_TRY(hipMemsetAsync(pair, 0xFF, sizeof(int32_t) * m, st));
        k_gather<<<grid_for(m, 256), 256, 0, st>>>(dh->process, dh->type, dh->f, dh->value, dh->value2,
                                                   rB, m, vmin, rec);
        k_pair<<<grid_for((m + 63) / 64, 4, 16384), 256, 0, st>>>(rec, kB, off, m, pair, viol);
        k_orphan<<<grid_for(m, 256), 256, 0, st>>>(rec, kB, m, pair, viol);
    }
    if (per_key_values && m > 0) {
        const int64_t n2 = 2 * m;
        if (n2 >= (1LL << 32) - 1) throw_jh(JH_EUNSUPPORTED, "too many entries for per-key value interning");
        uint64_t *iu = ctx->ws<uint64_t>(WS_IV_U, 2 * n2);
        uint32_t *ix = ctx->ws<uint32_t>(WS_IV_IDX, 3 * n2);
        uint32_t *ik = ctx->ws<uint32_t>(WS_IV_KEY, 2 * n2);
        uint32_t *rinit = ctx->ws<uint32_t>(WS_IV_RINIT, K + 1);
        unsigned int *maxid = (unsigned int *)ctx->ws<uint32_t>(WS_IV_MAX, 4);
        uint32_t *flag = ik + n2;                   // reuses the key buffer's second half
        k_ival<<<grid_for(n2, 256), 256, 0, st>>>(dh->value, dh->value2, dh->f, rB, m, iu, ix);
        size_t tb1 = 0, tb2 = 0, tb3 = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb1, iu, iu + n2, ix, ix + n2, (int)n2, 0, 64, st));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, ik, ik + n2, ix + n2, ix + 2 * n2, (int)n2, 0, endbit, st));
        HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb3, flag, flag, (int)n2, st));
        char *itmp = ctx->ws<char>(WS_IV_TMP, std::max(tb1, std::max(tb2, tb3)));
        // by value (iu keeps the original values, iu + n2 the sorted ones) ...
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(itmp, tb1, iu, iu + n2, ix, ix + n2, (int)n2, 0, 64, st));
        // ... then stably by key: each key's items in value order
        k_ikey<<<grid_for(n2, 256), 256, 0, st>>>(ix + n2, kB, n2, ik);
        uint32_t *ik2 = (uint32_t *)(iu + n2);      // sorted values no longer needed: key output
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(itmp, tb2, ik, ik2, ix + n2, ix + 2 * n2, (int)n2, 0, endbit, st));
        const uint32_t *idx2 = ix + 2 * n2;
        k_iflag<<<grid_for(n2, 256), 256, 0, st>>>(idx2, iu, kB, off, n2, flag);
        HIP_TRY(hipcub::DeviceScan::InclusiveSum(itmp, tb3, flag, flag, (int)n2, st));
        const uint64_t init_u = (uint64_t)init ^ (1ULL << 63);
        HIP_TRY(hipMemsetAsync(rinit, 0, sizeof(uint32_t) * (K + 1), st));
        HIP_TRY(hipMemsetAsync(maxid, 0, sizeof(unsigned int), st));
        if (init != JH_NIL) k_iinit<<<grid_for(n2, 256), 256, 0, st>>>(idx2, iu, kB, off, flag, n2, init_u, rinit);
        k_iassign<<<grid_for(n2, 256), 256, 0, st>>>(idx2, iu, kB, off, flag, n2, init != JH_NIL ? 1 : 0, init_u,
                                                     rinit, rec, viol, maxid);
        unsigned int mh = 0;
        HIP_TRY(hipMemcpyAsync(&mh, maxid, sizeof mh, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n_states = (long long)std::max<unsigned int>(mh, init != JH_NIL ? 1u : 0u) + 1;
    }

    // memo generation tags: distinct per (call, key, pass); wrap -> clear
    const uint32_t gen_span = (uint32_t)(3 * K + 3);
    bool clear_memo = false;
    // JH_LIN_GEN_JUMP (tests): start this call at the top of the generation range,
    // so it wraps and must clear every memo table before its searches read them
    if (lflags & JH_LIN_GEN_JUMP) ctx->gen_base = (1u << GEN_BITS) - 2;
    if ((uint64_t)ctx->gen_base + gen_span >= (1u << GEN_BITS) - 1) {
        ctx->gen_base = 0;
#ifndef JH_NO_WRAP_CLEAR          // (a test build that leaves the tables stale: the wrap test must fail)
        clear_memo = true;
#endif
    }

    // phase 1: every key, quick budget, persistent grid
    const uint32_t memo_cap1 = 1u << 16;
    // 8192: measured against 4096 (C3 rank 0 50.7 -> 42.4 ms, C4 635 -> 430 ms, C5 and ranks 3/4/6
    // unchanged): phase 1 runs 15 waves per CU, phase 2 one, and phase 2 restarts a deferred
    // key from scratch, so every key phase 1 can finish is cheaper there
    int64_t quick = std::min<int64_t>(budget, QUICK_BUDGET);
    if (opts && opts->quick_budget > 0)
        quick = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(budget, memo_cap1 / 2), opts->quick_budget));
    int p1_per_cu = 163840 / MemoQ::LDS;
    if (opts && opts->p1_waves_per_cu > 0) p1_per_cu = std::min(p1_per_cu, (int)opts->p1_waves_per_cu);
    const int waves1 = (int)std::min<int64_t>(K, (int64_t)ctx->n_cu * p1_per_cu);
    uint64_t *memo = ctx->ws<uint64_t>(WS_MEMO, (size_t)waves1 * memo_cap1 * 2, /*zero=*/true);
    if (clear_memo) HIP_TRY(hipMemsetAsync(memo, 0, ctx->bufs[WS_MEMO].bytes, st));
    const uint32_t stack_cap = (uint32_t)smax + 2;
    Frame *stack = ctx->ws<Frame>(WS_STACK, (size_t)waves1 * stack_cap);
    const uint64_t scr_bytes = MemoQ::SLOTS * 8;          // per wave: the memo eviction stage
    const uint64_t scr_bytes_h = MemoH::SLOTS * 8;
    const uint64_t scr_bytes_bfs = (((uint64_t)smax * 84 + 4096) + 255) & ~255ULL;
    char *scr = ctx->ws<char>(WS_SCRATCH, (size_t)waves1 * scr_bytes);
    int32_t *q = ctx->ws<int32_t>(WS_QUEUE, Q_WORDS);
    int32_t *list = ctx->ws<int32_t>(WS_STATS, K);
    // the deferred keys, ordered for the heavy pass (k_sort_defer): every one
    // (the BFS's list), the LEAN ones and the WIDE ones (each mode's own searches)
    int32_t *defer = ctx->ws<int32_t>(WS_DEFER, 3 * (size_t)(K + 1));
    int32_t *defer_l = defer + (K + 1), *defer_w = defer + 2 * (K + 1);
    uint64_t *d64 = ctx->ws<uint64_t>(WS_DEFER64, 3 * (size_t)(K + 1));
    unsigned long long *probes = (unsigned long long *)(q + 4);
    HIP_TRY(hipMemsetAsync(q, 0, Q_WORDS * sizeof(int32_t), st));
    HIP_TRY(hipMemsetAsync(q + Q_T_WIDE, 0xFF, 2 * sizeof(int32_t), st));
    for (int w : {Q_T_BFS, Q_T_LEAN, Q_T_XW, Q_T_P1}) HIP_TRY(hipMemsetAsync(q + w, 0xFF, 2 * sizeof(int32_t), st));

    // per-key search tables for every key (<= 8 B per entry + 32 B per key)
    KeyMeta *meta = ctx->ws<KeyMeta>(WS_META, K);
    char *arena = ctx->ws<char>(WS_ARENA, (size_t)m * 8 + (size_t)K * 32 + 256);
    TblArgs ta{};
    ta.src = KeySrc{rec, pair, off, rB, viol, rank, q + 2};
    ta.K = K; ta.meta = meta; ta.arena = arena; ta.bump = (unsigned long long *)(q + 10);
    int32_t *list_w = ctx->ws<int32_t>(WS_LIST_W, K);
    ta.out = out_dev; ta.list = list; ta.n_list = q + 12; ta.list_w = list_w; ta.n_list_w = q + 13;
    int32_t *list_x = ctx->ws<int32_t>(WS_LIST_X, K);
    ta.list_x = list_x; ta.n_list_x = q + 19; ta.xw_max = (unsigned long long *)(q + 26);
    ta.states8 = n_states <= 256 ? 1 : 0;
    k_key_tables<<<(unsigned)std::min<int64_t>((K + 3) / 4, 8192), 256, 0, st>>>(ta);

    int32_t *list1 = list;
    if (!tune_env("JH_NO_LPT") && K > 1) {
        uint32_t *cost = ctx->ws<uint32_t>(WS_LCOST, 2 * K);
        int32_t *lv = ctx->ws<int32_t>(WS_LSORT, 2 * K);
        k_list_cost<<<grid_for(K, 256, 4096), 256, 0, st>>>(list, q + 12, meta, K, cost, lv);
        size_t tbl = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tbl, cost, cost + K, lv, lv + K, (int)K, 0, 32, st));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(ctx->ws<char>(WS_LTMP, tbl), tbl, cost, cost + K, lv,
                                                             lv + K, (int)K, 0, 32, st));
        list1 = lv + K;
    }

    DfsArgs a{};
    a.rec = rec; a.pair = pair; a.off = off; a.rows = rB; a.viol = viol; a.rank = rank;
    a.list = list1; a.n_list = 0; a.n_list_dev = q + 12; a.queue = q; a.out = out_dev;
    a.meta = meta; a.tables = arena;
    a.defer_list = nullptr; a.defer_count = q + 1;
    a.defer64 = d64; a.defer_kind = d64 + (K + 1); a.defer_kind_count = q + Q_DEFER_L;
    a.memo = memo; a.memo_cap = memo_cap1; a.stack = stack; a.stack_cap = stack_cap;
    a.scratch = scr; a.scratch_bytes = scr_bytes; a.budget = quick; a.defer = quick < budget ? 1 : 0;
    a.init_state = init_state; a.gen_base = ctx->gen_base; a.flags = q + 2; a.probes = probes;
    a.states8 = n_states <= 256 ? 1 : 0;
    // (the default, HANDOVER_MIN, only once resume is known to be on: below)
    a.handover_min = 0;
    if (a.defer && !(lflags & JH_LIN_NO_HANDOVER) && opts && opts->handover_min)
        a.handover_min = std::max(0, opts->handover_min);
    if (const char *e = tune_env("JH_HANDOVER_MIN")) a.handover_min = a.defer ? std::max(0, atoi(e)) : 0;
    a.prio_ins = P1_PRIO_INS;
    if (const char *e = tune_env("JH_P1_PRIO")) a.prio_ins = std::max(0, atoi(e));
    const char *dbgenv = tune_env("JH_DEBUG");
    const bool dbg2 = dbgenv && atoi(dbgenv) >= 2;
    unsigned long long *dbg = nullptr;
    if (dbg2) {
        dbg = ctx->ws<unsigned long long>(WS_DEBUG, (size_t)(waves1 + 512) * 16);
        HIP_TRY(hipMemsetAsync(dbg, 0, sizeof(unsigned long long) * (waves1 + 512) * 16, st));
        a.dbg = dbg;
    }
    const bool defer_times = tune_env("JH_DEFER_TIMES") && atoi(tune_env("JH_DEFER_TIMES"));
    if (defer_times) {
        a.defer_time = ctx->ws<unsigned long long>(WS_DEFER_TIME, (size_t)K + 2);
        HIP_TRY(hipMemsetAsync(a.defer_time, 0, sizeof(unsigned long long) * (K + 2), st));
        HIP_TRY(hipMemsetAsync(a.defer_time, 0xFF, sizeof(unsigned long long), st));
        a.defer_info = ctx->ws<unsigned long long>(WS_DEFER_INFO, 2 * (size_t)K);
        HIP_TRY(hipMemsetAsync(a.defer_info, 0, sizeof(unsigned long long) * 2 * K, st));
    }
    const bool skip_p1 = (lflags & JH_LIN_SKIP_PHASE1) != 0 && !linear_mode;
    const bool p1_only = (lflags & JH_LIN_PHASE1_ONLY) != 0 && !linear_mode && !skip_p1;
    // resume (round 5): phase 1's deferred LEAN searches saved for the heavy-key
    // pass (a record is <= 64 B + a frame per stack level + 16 B per insert)
    // (not for the workgroup engine's tuning modes, JH_WG: its
    // searches start at the root, so records would only be written)
    const bool wg_mode = tune_env("JH_WG") && atoi(tune_env("JH_WG")) != 0;
    const bool resume = a.defer && !linear_mode && !skip_p1 && !p1_only && !(lflags & JH_LIN_NO_RESUME) &&
                        !(lflags & JH_LIN_STREAM) && !wg_mode &&
                        !tune_env("JH_NO_RESUME");
    if (resume) {
        if (!ctx->hbm_total) {
            size_t fr = 0, tot = 0;
            HIP_TRY(hipMemGetInfo(&fr, &tot));
            ctx->hbm_total = tot;
        }
        // ADVICE r5 / VERDICT r5 item 7: the record arena and the slot log are
        // bounded by the device's HBM over the contexts sharing it (1/64 each:
        // 4.5 GB for one context on an MI355X, so the 256 MB cap rules there).
        // A smaller log only fails saves (those searches restart: same results)
        const uint64_t rs_lim = (uint64_t)ctx->hbm_total /
                                (64 * (uint64_t)std::max(ctx->share, device_open_contexts(ctx->device)));
        const uint64_t per_key = 64 + (uint64_t)stack_cap * sizeof(Frame) + (uint64_t)quick * 16;
        // (+ 64 MB for the takeovers' records, round 6)
        const uint64_t cap = std::min<uint64_t>(std::min<uint64_t>((uint64_t)320 << 20, rs_lim),
                                                (uint64_t)K * per_key + ((uint64_t)64 << 20));
        a.rs_arena = ctx->ws<uint8_t>(WS_RS_ARENA, cap);
        a.rs_cap = cap;
        a.rs_off = ctx->ws<int64_t>(WS_RS_OFF, K);
        a.rs_used = (unsigned long long *)(q + Q_RS_USED);
        HIP_TRY(hipMemsetAsync(a.rs_off, 0xFF, (size_t)K * sizeof(int64_t), st));
        a.rs_mode = 1;
#ifdef JH_DUP_WRITE
        {
            ulonglong2 *mirror = ctx->ws<ulonglong2>(WS_DEFER_INFO + 1, (size_t)1 << 26);
            HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_dup_base), &mirror, sizeof mirror));
        }
#endif
        if (!tune_env("JH_RS_SCAN")) {
            a.hlog_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(quick, 1024), 32768);
            a.hlog_cap = (uint32_t)std::max<uint64_t>(256, std::min<uint64_t>(a.hlog_cap, rs_lim / (4 * (uint64_t)std::max(1, waves1))));
            a.hlog = ctx->ws<uint32_t>(WS_RS_LOG, (size_t)waves1 * a.hlog_cap);
        }
        // a handed-over search continues where it stopped: the hand-over is free
        if (!(lflags & JH_LIN_NO_HANDOVER) && !(opts && opts->handover_min) && !tune_env("JH_HANDOVER_MIN"))
            a.handover_min = HANDOVER_MIN;
    }
    int32_t qh[Q_WORDS];
    int n_defer = 0, n_def_l = 0, n_def_w = 0, n_x = 0;
    int waves_x = 0;
    XwArgs xa{};
    // windows wider than 64 (k_lin_xw): one wave per key, up to four per CU
    // (round 2 capped this at 128 waves); qw: the queue words after k_key_tables
    auto prep_xw = [&](const int32_t *qw) {
        if (n_x <= 0) return;
        uint32_t capx = 1u << 12;
        while ((int64_t)capx < 2 * budget && capx < (1u << 30)) capx <<= 1;
        const uint64_t scr_x = (((uint64_t)(uint32_t)qw[26] | ((uint64_t)(uint32_t)qw[27] << 32)) + 255) & ~255ULL;
        int want_x = std::min(n_x, 4 * ctx->n_cu);
        if (opts && opts->xw_waves > 0) want_x = std::min(n_x, opts->xw_waves);
        const uint64_t per_x = (uint64_t)capx * XW_EW * 8 + (uint64_t)stack_cap * XW_FW * 8 + scr_x;
        waves_x = fit_units(ctx, want_x, per_x, {WS_MEMO_X, WS_STACK_X, WS_SCRATCH_X});
        const bool freshx = ctx->ws_fresh(WS_MEMO_X) || ctx->bufs[WS_MEMO_X].bytes < (size_t)waves_x * capx * XW_EW * 8;
        uint64_t *memox = ctx->ws<uint64_t>(WS_MEMO_X, (size_t)waves_x * capx * XW_EW, /*zero=*/true);
        if (clear_memo && !freshx) HIP_TRY(hipMemsetAsync(memox, 0, ctx->bufs[WS_MEMO_X].bytes, st));
        xa = XwArgs{};
        xa.src = KeySrc{rec, pair, off, rB, viol, rank, q + 2};
        xa.list = list_x; xa.n_list = n_x; xa.queue = q + 21; xa.meta = meta; xa.out = out_dev;
        xa.scratch = ctx->ws<char>(WS_SCRATCH_X, (size_t)waves_x * scr_x); xa.scratch_bytes = scr_x;
        xa.memo = memox; xa.memo_cap = capx;
        xa.stack = ctx->ws<uint64_t>(WS_STACK_X, (size_t)waves_x * stack_cap * XW_FW); xa.stack_cap = stack_cap;
        xa.budget = budget; xa.init_state = init_state;
        xa.gen_base = ctx->gen_base + 2 * (uint32_t)K + 1;   // its own table: any gen range works
        xa.flags = q + 2; xa.probes = (unsigned long long *)(q + 22);
        xa.cause_or = linear_mode ? CAUSE_BY_WGL : 0;
        xa.t_span = (unsigned long long *)(q + Q_T_XW);
    };

    // phase 2 hands a key that reaches P2_BUDGET inserts to phase 3 (when the
    // phase has fewer waves than keys)
    int64_t p2 = P2_BUDGET;
    if (opts && opts->phase2_budget > 0) p2 = std::max<int64_t>(quick + 1, opts->phase2_budget);
    uint32_t cap2 = 1u << 16;
    while ((int64_t)cap2 < 2 * budget && cap2 < (1u << 30)) cap2 <<= 1;
    if (const char *e = tune_env("JH_MEMO_CAP_SHIFT")) cap2 <<= std::max(0, std::min(3, atoi(e)));   // experiments
    int32_t *defer3 = ctx->ws<int32_t>(WS_DEFER3, 2 * (size_t)(K + 1));
    int32_t *defer3w = defer3 + (K + 1);
    int32_t *claim = nullptr;
    int waves_w = 0, waves2 = 0;
    int waves3 = 0;                  // phase 3's LEAN waves (full tables; waves2 unless p2_small)
    uint32_t cap2l = cap2;           // phase 2's LEAN tables (entries per wave)
    bool p2_small_ok = true;         // (the streaming pass keeps round 4's sizing)
    bool split3 = false, split3w = false;

    // ---- the deferred WIDE keys (windows of 41-64 members or >= 256 states):
    // their own pipeline on the fourth stream, beside the LEAN one. As many
    // waves as keys, up to four per CU and bounded by free HBM (round 2: 32
    // waves in phase 2 and 128 in phase 3, queued behind the LEAN kernels on
    // one stream). With a wave per key there is one pass at the full budget;
    // with fewer, phase 2 stops a key at P2_BUDGET and phase 3 restarts it
    // (same waves and tables, a fresh generation range), the count of phase
    // 3's keys read on the device: no host round trip.
    DfsArgs bw{};
    auto prep_wide = [&]() {
        if (n_def_w == 0) return;
        const uint64_t per_w = (uint64_t)cap2 * 16 + (uint64_t)stack_cap * sizeof(Frame) + SEQW_SCR;
        int want_w = std::min(n_def_w, 4 * ctx->n_cu);
        if (opts && opts->wide_waves > 0) want_w = std::min(want_w, opts->wide_waves);
        waves_w = fit_units(ctx, want_w, per_w, {WS_MEMO_WIDE, WS_STACK_WIDE, WS_SCRATCH_WIDE});
        const bool freshw = ctx->ws_fresh(WS_MEMO_WIDE) || ctx->bufs[WS_MEMO_WIDE].bytes < (size_t)waves_w * cap2 * 16;
        uint64_t *memow = ctx->ws<uint64_t>(WS_MEMO_WIDE, (size_t)waves_w * cap2 * 2, /*zero=*/true);
        if (clear_memo && !freshw) HIP_TRY(hipMemsetAsync(memow, 0, ctx->bufs[WS_MEMO_WIDE].bytes, st));
        bw = a;
        bw.handover_min = 0;
        bw.rs_mode = 0;
        bw.list = defer_w; bw.n_list = n_def_w; bw.n_list_dev = nullptr; bw.queue = q + 7;
        bw.defer64 = nullptr; bw.defer_kind = nullptr; bw.defer_kind_count = nullptr;
        split3w = waves_w < n_def_w && budget > p2;
        bw.defer = split3w ? 1 : 0; bw.defer_list = defer3w; bw.defer_count = q + Q_DEFER3W;
        bw.budget = split3w ? p2 : budget; bw.budget_full = split3w ? budget : 0;
        bw.memo = memow; bw.memo_cap = cap2;
        bw.stack = ctx->ws<Frame>(WS_STACK_WIDE, (size_t)waves_w * stack_cap);
        bw.scratch = ctx->ws<char>(WS_SCRATCH_WIDE, (size_t)waves_w * SEQW_SCR);
        bw.scratch_bytes = SEQW_SCR;
        bw.gen_base = ctx->gen_base + (uint32_t)K + 1;
        bw.claim = claim;                    // the BFS may settle a WIDE key with a narrow window
        bw.probes = (unsigned long long *)(q + Q_PROBES_WIDE);
        bw.seq_start = nullptr; bw.exit_count = nullptr; bw.dbg = nullptr; bw.defer_time = nullptr;
        bw.t_span = (unsigned long long *)(q + Q_T_WIDE);
    };
    // phase 2 of the WIDE keys alone (paths without the two-role grid), then phase 3
    auto launch_wide = [&](hipStream_t sw, bool p2) {
        if (waves_w == 0) return;
        if (p2) k_lin_seqw<<<waves_w, 64, SEQW_LDS, sw>>>(bw);
        HIP_TRY(hipGetLastError());
        if (split3w) {
            DfsArgs c3 = bw;
            c3.list = defer3w; c3.n_list = 0; c3.n_list_dev = q + Q_DEFER3W; c3.queue = q + 20; c3.defer = 0;
            c3.defer_list = nullptr; c3.defer_count = nullptr;
            c3.budget = budget; c3.budget_full = 0; c3.wave_off = 0;
            c3.gen_base = ctx->gen_base + 2 * (uint32_t)K + 1;
            k_lin_seqw<<<waves_w, 64, SEQW_LDS, sw>>>(c3);
            HIP_TRY(hipGetLastError());
        }
    };

    unsigned long long *acc_stats = nullptr;
    int n_wg = 0;
    // the workgroup engine (k_lin_wg): exact WGL, dead subtrees enumerated by
    // the workgroup's helper waves; built for wg_cus CUs, racing the BFS when
    // wg_claim is set
    auto build_wg = [&](int wg_cus, int32_t *wg_claim, int32_t *wg_queue, bool all_cus = false) -> WgArgs {
        acc_stats = ctx->ws<unsigned long long>(WS_ACC_STATS, 8);
        HIP_TRY(hipMemsetAsync(acc_stats, 0, 8 * sizeof(unsigned long long), st));
        // + slack: keys claimed in the set after the cap is hit are still recorded
        const uint64_t work_cap = (uint64_t)std::min<int64_t>(budget, (int64_t)1 << 30) + ACC_MAXROOTS + 16384;
        uint64_t gcap = 1024;
        while (gcap < 2 * work_cap) gcap <<= 1;
        const uint32_t mo = (uint32_t)smax;   // >= n_ok of any key
        const uint64_t wtab_b = (((uint64_t)(mo + 1) * 4 + 255) & ~255ULL) + (((uint64_t)mo * 40 * 4 + 255) & ~255ULL) +
                                (((uint64_t)mo + 255) & ~255ULL);
        const uint64_t per_wg = (uint64_t)cap2 * 16 + gcap * 8 + 3 * work_cap * 8 + (uint64_t)stack_cap * sizeof(Frame) +
                                MemoW::SLOTS * 8 + wtab_b;
        uint64_t mem_limit = 48ULL << 30;
        if (const char *e = tune_env("JH_WG_MEM_GB")) mem_limit = (uint64_t)std::max(1, atoi(e)) << 30;
        // (with the spec board every helper is useful, a key of its own or not)
        n_wg = all_cus ? wg_cus : (int)std::min<int64_t>(n_def_l, (int64_t)wg_cus);
        n_wg = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)n_wg, mem_limit / per_wg));
        n_wg = fit_units(ctx, n_wg, per_wg, {WS_WG_MEMO, WS_WG_GSET, WS_WG_WORK, WS_WG_PEND});
        const bool fresh2 = ctx->ws_fresh(WS_WG_MEMO) || ctx->bufs[WS_WG_MEMO].bytes < (size_t)n_wg * cap2 * 16;
        uint64_t *memo2 = ctx->ws<uint64_t>(WS_WG_MEMO, (size_t)n_wg * cap2 * 2, /*zero=*/true);
        if (clear_memo && !fresh2) HIP_TRY(hipMemsetAsync(memo2, 0, ctx->bufs[WS_WG_MEMO].bytes, st));
        // kept all zero between calls by the enumeration's clean-up
        uint64_t *gset = ctx->ws<uint64_t>(WS_WG_GSET, (size_t)n_wg * gcap, /*zero=*/true);
        uint64_t *work = ctx->ws<uint64_t>(WS_WG_WORK, (size_t)n_wg * work_cap, /*zero=*/true);
        WgArgs wa{};
        wa.d = a;
        wa.d.rs_mode = 0;
        wa.d.handover_min = 0;
        wa.d.list = defer_l; wa.d.n_list = n_def_l; wa.d.n_list_dev = nullptr; wa.d.queue = wg_queue; wa.d.defer = 0;
        wa.d.defer_list = nullptr; wa.d.defer_count = nullptr;
        wa.d.defer64 = nullptr; wa.d.defer_kind = nullptr; wa.d.defer_kind_count = nullptr;
        wa.d.memo = memo2; wa.d.memo_cap = cap2;
        wa.d.stack = ctx->ws<Frame>(WS_WG_STACK, (size_t)n_wg * stack_cap);
        wa.d.scratch = ctx->ws<char>(WS_WG_SCR, (size_t)n_wg * MemoW::SLOTS * 8);
        wa.d.scratch_bytes = MemoW::SLOTS * 8;
        wa.d.budget = budget; wa.d.budget_full = 0; wa.d.claim = wg_claim;
        wa.d.gen_base = ctx->gen_base + (uint32_t)K + 1;
        wa.d.dbg = nullptr; wa.d.probes = (unsigned long long *)(q + Q_PROBES_HELP);
        wa.gset = gset; wa.gset_cap = (uint32_t)gcap; wa.work = work; wa.work_cap = (uint32_t)work_cap;
        wa.wtab = ctx->ws<char>(WS_WG_WTAB, (size_t)n_wg * wtab_b); wa.wtab_bytes = wtab_b;
        if (dbgenv && atoi(dbgenv) >= 3) {
            // its own slot: the BFS's JH_DEBUG words live in WS_DEBUG (a shared slot
            // grown here would leave their pointer dangling)
            wa.d.dbg = ctx->ws<unsigned long long>(WS_DEBUG_WG, (size_t)n_wg * 256 + 16 * 1024);
            HIP_TRY(hipMemsetAsync(wa.d.dbg, 0, sizeof(unsigned long long) * n_wg * 256, st));
        }
        wa.acc_stats = acc_stats;
        wa.pend_cap = (uint32_t)work_cap;
        wa.acc_t = ACC_T;
        if (const char *e = tune_env("JH_ACC_T")) wa.acc_t = (uint32_t)std::max(0, atoi(e));
        if (dbgenv && atoi(dbgenv) >= 4) {
            wa.key_prof = ctx->ws<unsigned long long>(WS_STATS_KEYS, 3 * (size_t)K);
            HIP_TRY(hipMemsetAsync(wa.key_prof, 0, 3 * sizeof(unsigned long long) * K, st));
        }
        wa.pend = ctx->ws<uint64_t>(WS_WG_PEND, (size_t)n_wg * 2 * work_cap);
        if (!ctx->lds_attr_wg) {
            HIP_TRY(hipFuncSetAttribute((const void *)k_lin_wg, hipFuncAttributeMaxDynamicSharedMemorySize, WG_LDS));
            ctx->lds_attr_wg = true;
        }
        return wa;
    };
    int n_unres = 0;
    const char *wg_env = tune_env("JH_WG");
    // JH_WG=1 (tuning builds): the workgroup engine (k_lin_wg, exact DFS with
    // accelerated dead subtrees) for deferred LEAN keys; default: the BFS /
    // sequential race
    const bool use_wg = wg_env && atoi(wg_env) == 1;
    // JH_WG=2: the workgroup engine races the BFS in place of the sequential search
    const bool wg_race = wg_env && atoi(wg_env) == 2;
    int wg2 = 0, n_help = 0;
    // the heavy-key race's engines for at most nd_all deferred keys (nd_l of
    // them LEAN): the BFS (c), the sequential search of the LEAN keys (b),
    // the late helpers (wh) or the workgroup race (wr); allocations only
    BfsArgs c{};
    DfsArgs b{};
    WgArgs wr{}, wh{};
    unsigned long long *seq_start = nullptr;
    bool p2_m = true, bfs_only = false;
    auto prep_race = [&](int nd_all, int nd_l) {
        claim = ctx->ws<int32_t>(WS_CLAIM, K);
        HIP_TRY(hipMemsetAsync(claim, 0, (size_t)K * sizeof(int32_t), st));
        // q[0] (phase 1's queue) becomes the BFS's; q[3] its give-up count; q[6] phase 2's queue
        HIP_TRY(hipMemsetAsync(q, 0, sizeof(int32_t), st));
        HIP_TRY(hipMemsetAsync(q + 3, 0, sizeof(int32_t), st));
        HIP_TRY(hipMemsetAsync(q + 6, 0, sizeof(int32_t), st));

        // the BFS enumerates up to reach_cap configurations and keeps up to
        // ncap of them for WGL's exact count of valid keys (bfs_wgl_count)
        uint32_t ncap = 1u << 22;
        if (const char *e = tune_env("JH_BFS_NODES")) ncap = (uint32_t)std::max(1 << 16, std::min(1 << 26, atoi(e)));
        const int64_t reach_cap = std::max<int64_t>(budget + 1, ncap);
        uint32_t set_cap = 1u << 12;
        while ((int64_t)set_cap < 2 * reach_cap && set_cap < (1u << 30)) set_cap <<= 1;
        const uint32_t q_cap = (uint32_t)std::min<int64_t>(reach_cap + 64, (int64_t)1 << 30);
        uint32_t hcap = 1u << 16;
        while (hcap < 2 * (uint64_t)ncap) hcap <<= 1;
        const uint32_t lcap = (uint32_t)smax + 2;
        // CU split of the heavy-key pass (one BFS workgroup or one sequential
        // wave per CU, by LDS): invalid keys are few, the sequential searches
        // many (every valid deferred key), so most CUs go to the latter
        // 96 of 256 (round 2, with phase 2 at four waves per CU): C4 shard
        // 230 -> 223 ms, C3 ranks 0 / 3 / 6 flat (32: C4 +9 %, 128: no better)
        // Round 6, with 64 helpers: 64 when 2 000-4 000 keys are deferred
        // (the sequential search keeps 128 CUs for its queue; C3 ranks 0-4,
        // 3 550-3 750 deferred keys: 39.0 / 36.0 / 35.2 / 39.6 / 45.4 -> 38.1 /
        // 34.0 / 31.3 / 40.5 / 43.7 ms), 96 for fewer (the strong-scaling
        // shards' 1 335 / 694 deferred keys: 27.1 / 21.0 -> 24.5 / 19.4 ms) and
        // for more (C4's shard, 4 258 deferred keys, 812 of them invalid ones
        // the BFS settles: 209.7 -> 202.0 ms); profiles/r06/ab_bfs_helpers/,
        // ab_c4_split/. A measured band, not a model of the race.
        const int bfs_cus = std::max(1, nd_all > 2000 && nd_all <= 4000 ? ctx->n_cu / 4
                                                                          : std::min(96, ctx->n_cu * 3 / 8));
        wg2 = std::min(nd_all, tune_env("JH_BFS_CUS") ? std::max(1, atoi(tune_env("JH_BFS_CUS"))) :
                               opts && opts->bfs_wgs > 0 ? std::min(opts->bfs_wgs, ctx->n_cu - 16) : bfs_cus);
        const uint64_t per_bfs = (uint64_t)set_cap * 8 + 4ULL * q_cap * 8 + scr_bytes_bfs + (uint64_t)ncap * 8 +
                                 (uint64_t)lcap * 4 + (uint64_t)hcap * 16 + (uint64_t)ncap * 4 + ((uint64_t)ncap / 32 + 1) * 4 +
                                 (uint64_t)ncap * 4 + (uint64_t)ncap * 8;
        wg2 = fit_units(ctx, wg2, per_bfs, {WS_BFS_SET, WS_BFS_Q, WS_BFS_NODES, WS_BFS_HKEY, WS_BFS_TMPK});
        uint64_t *bset = ctx->ws<uint64_t>(WS_BFS_SET, (size_t)wg2 * set_cap);
        uint64_t *bq = ctx->ws<uint64_t>(WS_BFS_Q, (size_t)wg2 * 4 * q_cap);
        char *bscr = ctx->ws<char>(WS_SCRATCH_BFS, (size_t)wg2 * scr_bytes_bfs);
        int32_t *unres = ctx->ws<int32_t>(WS_BFS_META, nd_all + 1);
        c = BfsArgs{};
        c.src = KeySrc{rec, pair, off, rB, viol, rank, q + 2};
        c.list = defer; c.n_list = nd_all; c.queue = q; c.out = out_dev;
        c.unres_list = unres; c.unres_count = q + 3;
        c.gset = bset; c.gset_cap = set_cap; c.pend = bq; c.front = bq + (size_t)wg2 * 2 * q_cap;
        c.q_cap = q_cap;
        c.scratch = bscr; c.scratch_bytes = scr_bytes_bfs; c.budget = budget;
        c.init_state = init_state; c.states_ok = n_states < 4096 ? 1 : 0;
        c.dbg = dbg; c.claim = claim;
        // every key the BFS settles carries WGL's exact count (the whole set for
        // an invalid key; path + dead closure for a valid one, bfs_wgl_count)
        c.reach_cap = reach_cap;
        // JH_LIN_BFS_ONLY (tests): no sequential search, the BFS settles every
        // key it can (the others stay unsettled); JH_BFS_DBGV=1 (tuning builds):
        // its valid verdicts carry fail_entry = path length, cause = stored
        // configurations, explored = count
        bfs_only = (lflags & JH_LIN_BFS_ONLY) != 0;
        c.dbg_plen = tune_env("JH_BFS_DBGV") && atoi(tune_env("JH_BFS_DBGV")) ? 1 : 0;
        c.exact_count = (lflags & JH_LIN_EXACT_COUNT) || c.dbg_plen ? 1 : 0;
        c.ncap = ncap; c.hcap = hcap; c.lcap = lcap;
        c.nodes = ctx->ws<uint64_t>(WS_BFS_NODES, (size_t)wg2 * ncap);
        c.lstart = ctx->ws<uint32_t>(WS_BFS_LSTART, (size_t)wg2 * lcap);
        c.ent = ctx->ws<ulonglong2>(WS_BFS_HKEY, (size_t)wg2 * hcap);
        c.slot = ctx->ws<uint32_t>(WS_BFS_LIVE, (size_t)wg2 * ncap);
        c.vis = ctx->ws<uint32_t>(WS_BFS_VIS, (size_t)wg2 * (ncap / 32 + 1));
        c.tmp = ctx->ws<uint32_t>(WS_BFS_TMP, (size_t)wg2 * ncap);
        c.tmpk = ctx->ws<uint64_t>(WS_BFS_TMPK, (size_t)wg2 * ncap);
        // per context (= per device; calls on one context are serialised by its mutex)
        if (!ctx->lds_attr) {
            HIP_TRY(hipFuncSetAttribute((const void *)k_lin_bfs, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        BFS_LDS_BYTES));
            HIP_TRY(hipFuncSetAttribute((const void *)k_lin_seq<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        MemoH::LDS));
            HIP_TRY(hipFuncSetAttribute((const void *)k_lin_seq<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        MemoH::LDS));
            ctx->lds_attr = true;
        }

        // late helpers (k_lin_wg in helper mode, wg_helper_pick): a few CUs
        // taken from the sequential search of the LEAN keys
        n_help = bfs_only || wg_race || nd_l == 0 ? 0 : std::min(HELPERS, std::max(0, ctx->n_cu / 4));
        if (opts && opts->helpers > 0) n_help = std::min(ctx->n_cu / 2, opts->helpers);
        if (const char *e = tune_env("JH_HELPERS")) n_help = std::max(0, std::min(ctx->n_cu, atoi(e)));
        if (lflags & JH_LIN_NO_HELPERS) n_help = 0;
        // JH_HELP_CUS (tuning builds): CUs the sizing of phase 2's sequential
        // search leaves to the helpers (default: one per helper); helpers
        // beyond it start when CUs free up
        int help_cus = n_help;
        if (const char *e = tune_env("JH_HELP_CUS")) help_cus = std::max(0, std::min(n_help, atoi(e)));
        if (n_help > 0 && ctx->n_cu - wg2 - help_cus < 16) n_help = help_cus = 0;
        // phase 2's sequential search with four waves per CU and the 32 KB memo
        // (k_lin_seq3), p2_waves_per_cu = 1 for one wave per CU and the 128 KB
        // memo (k_lin_seq): measured C4 shard 268 -> 228 ms, C3 / ranks 3, 6 / C5 flat
        p2_m = !(opts && opts->p2_waves_per_cu == 1);
        cap2l = cap2;
        if (nd_l > 0) {
            const int cus2 = std::max(1, ctx->n_cu - wg2 - help_cus);
            // LEAN keys alone in the grid: MemoP2's waves per CU
            const int lean_per_cu = n_def_w > 0 || !p2_small_ok ? 4 : JH_P2_PER_CU;
            int want2 = std::min(nd_l, cus2 * (p2_m ? lean_per_cu : 1));
            if (opts && opts->lean_waves > 0) want2 = std::min(want2, opts->lean_waves);
            const uint64_t fixed = (uint64_t)stack_cap * sizeof(Frame) + scr_bytes_h;
            const uint64_t per2 = (uint64_t)cap2 * 16 + fixed;
            waves2 = fit_units(ctx, want2, per2, {WS_MEMO_DEEP, WS_STACK_DEEP, WS_SCRATCH_DEEP});
            waves3 = waves2;
            // more keys than waves: phase 2 stops at p2 inserts and phase 3
            // takes the rest on full tables, so phase 2's LEAN role can run
            // JH_P2_PER_CU waves per CU on tables for 2 x p2 entries
            if (p2_m && p2_small_ok && n_def_w == 0 && !(opts && opts->lean_waves > 0) && budget > p2) {
                uint32_t cs = 1u << 16;
                while ((int64_t)cs < 2 * p2 && cs < cap2) cs <<= 1;
                const int want_s = std::min(nd_l, cus2 * JH_P2_PER_CU);
                const int ws = fit_units(ctx, want_s, (uint64_t)cs * 16 + fixed, {WS_MEMO_DEEP, WS_STACK_DEEP, WS_SCRATCH_DEEP});
                if (ws < nd_l) {
                    cap2l = cs;
                    waves2 = ws;
                }
            }
        }
        // generation-tagged: zeroed once when allocated (and on wrap), not per
        // call; phases 2 and 3 share it at their own strides (their generation
        // ranges differ, so one phase's entries are empty slots to the other's)
        uint64_t *memo2 = nullptr;
        const size_t m2 = std::max((size_t)waves2 * cap2l, (size_t)waves3 * cap2);
        if (waves2 > 0) {
            const bool fresh2 = ctx->ws_fresh(WS_MEMO_DEEP) || ctx->bufs[WS_MEMO_DEEP].bytes < m2 * 16;
            memo2 = ctx->ws<uint64_t>(WS_MEMO_DEEP, m2 * 2, /*zero=*/true);
            if (clear_memo && !fresh2) HIP_TRY(hipMemsetAsync(memo2, 0, ctx->bufs[WS_MEMO_DEEP].bytes, st));
        }
        wr = WgArgs{};
        if (wg_race && nd_l > 0) wr = build_wg(std::max(1, ctx->n_cu - wg2), claim, q + 6);
        wh = WgArgs{};
        seq_start = nullptr;
        if (n_help > 0) {
            const bool spec_on = !(lflags & JH_LIN_NO_SPEC) && !(tune_env("JH_SPEC") && !atoi(tune_env("JH_SPEC")));
            wh = build_wg(n_help, claim, nullptr, spec_on);
            seq_start = ctx->ws<unsigned long long>(WS_HELP_START, K);
            int32_t *taken = ctx->ws<int32_t>(WS_HELP_TAKEN, K);
            HIP_TRY(hipMemsetAsync(seq_start, 0, (size_t)K * sizeof(unsigned long long), st));
            HIP_TRY(hipMemsetAsync(taken, 0, (size_t)K * sizeof(int32_t), st));
            wh.seq_start = seq_start; wh.seq_exit = q + 28; wh.seq_waves = waves2; wh.taken = taken;
            wh.mains_live = q + Q_MAINS;
            uint64_t late_us = HELPER_LATE_US;
            if (opts && opts->helper_late_us > 0) late_us = (uint64_t)opts->helper_late_us;
            if (lflags & JH_LIN_HELPERS_NOW) late_us = 0;
            wh.late_ticks = late_us * 100;     // s_memrealtime: 100 MHz
            // round 6: the spec board (SpecSlot), unless JH_LIN_NO_SPEC
            if (spec_on) {
                wh.spec = ctx->ws<SpecSlot>(WS_SPEC, SPEC_SLOTS);
                HIP_TRY(hipMemsetAsync(wh.spec, 0, sizeof(SpecSlot) * SPEC_SLOTS, st));
                wh.spec_res_cap = SPEC_RES_CAP;
                wh.spec_res = ctx->ws<uint64_t>(WS_SPEC_RES, (size_t)n_wg * SPEC_RES_CAP);
                wh.spec_min = 512; wh.spec_mult = 32; wh.spec_dist = 128;
                wh.spec_q = q + Q_SPEC;
                wh.spec_first = (lflags & JH_LIN_SPEC_FIRST) ? 1 : 0;
                wh.n_mains = n_wg;
                if (const char *e = tune_env("JH_SPEC_SERVERS")) wh.n_mains = std::max(1, n_wg - std::max(0, atoi(e)));
                if (const char *e = tune_env("JH_SPEC_MIN")) wh.spec_min = (uint32_t)std::max(1, atoi(e));
                if (const char *e = tune_env("JH_SPEC_MULT")) wh.spec_mult = (uint32_t)std::max(1, atoi(e));
                if (const char *e = tune_env("JH_SPEC_DIST")) wh.spec_dist = (uint32_t)std::max(1, atoi(e));
            }
        }
        const int wmax = std::max(waves2, waves3);
        Frame *stack2 = waves2 > 0 ? ctx->ws<Frame>(WS_STACK_DEEP, (size_t)wmax * stack_cap) : nullptr;
        char *scr2 = waves2 > 0 ? ctx->ws<char>(WS_SCRATCH_DEEP, (size_t)wmax * scr_bytes_h) : nullptr;
        // a wave per key: one pass at the full budget; fewer waves than keys:
        // phase 2 stops at p2 inserts and phase 3 restarts those keys
        split3 = waves2 < nd_l && budget > p2;
        b = a;
        b.rs_mode = 0;                  // the default race below continues phase 1's records
        b.handover_min = 0;
        b.list = defer_l; b.n_list = nd_l; b.n_list_dev = nullptr; b.queue = q + 6; b.defer = split3 ? 1 : 0;
        b.defer_list = defer3; b.defer_count = q + 16;
        b.defer64 = nullptr; b.defer_kind = nullptr; b.defer_kind_count = nullptr;
        b.memo = memo2; b.memo_cap = cap2l; b.stack = stack2; b.scratch = scr2; b.scratch_bytes = scr_bytes_h;
        b.budget = split3 ? p2 : budget;
        // (past p2 a search goes on while the queue is empty, on full tables only)
        b.budget_full = split3 && cap2l == cap2 ? budget : 0;
        b.gen_base = ctx->gen_base + (uint32_t)K + 1;
        b.dbg = dbg ? dbg + 16 * 256 : nullptr; b.claim = claim;
        b.probes = (unsigned long long *)(q + 8);
        b.seq_start = seq_start; b.exit_count = seq_start ? q + 28 : nullptr;
        b.stamp_progress = seq_start && (lflags & JH_LIN_HELP_STALL) ? 1 : 0;
        b.defer_time = nullptr;
        // round 6, the takeover: a late helper continues the sequential
        // search's record (phase 2's own slot log, 32 K entries per wave)
        // instead of restarting the key
        b.handoff = nullptr;
        // (opt-in, JH_LIN_TAKEOVER: one exact-count call of sixteen final
        // lines disagreed with the oracle with it on, unexplained)
        if (n_help > 0 && a.rs_off && waves2 > 0 && (lflags & JH_LIN_TAKEOVER) && !(lflags & JH_LIN_NO_TAKEOVER)) {
            int32_t *ho = ctx->ws<int32_t>(WS_HANDOFF, K);
            HIP_TRY(hipMemsetAsync(ho, 0, (size_t)K * sizeof(int32_t), st));
            b.handoff = ho;
            b.hlog_cap = 32768;
            b.hlog = ctx->ws<uint32_t>(WS_RS_LOG2, (size_t)wmax * b.hlog_cap);
            wh.d.handoff = ho;
        }
    };
    // the streaming heavy-key pass (round 4) whenever the default race runs
    const bool stream_p2 = !linear_mode && !skip_p1 && !p1_only && !use_wg && !wg_race && !dbg2 &&
                           (lflags & JH_LIN_STREAM) && !(lflags & JH_LIN_BFS_ONLY);
    if (stream_p2) {
        // ---- the streaming heavy-key pass (round 4) --------------------------
        // Round 3 started the heavy keys when phase 1 ended (~17 ms into C3),
        // though most were deferred at 9-13 ms. Here phase 1 appends every key
        // it defers to live lists; once its last kernel's queue is drained (each
        // of its waves then finishes the key it holds and leaves) the host
        // launches the consumers -- the BFS (aux2), the late helpers (aux3) and
        // an early grid of LEAN sequential waves (aux) -- which take CUs as
        // phase 1 frees them and take keys as they are deferred. A grid behind
        // phase 1 on st runs the 65-256-member keys, the WIDE keys and more LEAN
        // waves; phase 3 follows on st. Four streams: the hardware's queues.
        // Every search is the one the round-3 schedule runs (same verdicts and
        // counts); only when each starts changes.
        // (round 4's CU-masked variant, JH_CU_SPLIT, is gone: slower at every
        // split, and at R = 48 the late helpers -- which spin until the
        // sequential grid has left its queue -- held the 48 consumer CUs the
        // sequential waves needed to become resident, so each step waited out
        // HELPER_MAX_TICKS, 5 s: DESIGN.md section 5)
        hipStream_t p1s = st, cs1 = ctx->aux, cs2 = ctx->aux2, cs3 = ctx->aux3;
        int32_t qt[Q_WORDS];
        HIP_TRY(hipMemcpyAsync(qt, q, sizeof qt, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const int n_l1 = qt[12], n_w1 = qt[13];
        n_x = qt[19];
        prep_xw(qt);
        // bounds: phase 1 defers at most the keys it searches
        n_def_l = n_l1; n_def_w = n_w1; n_defer = n_l1 + n_w1;
        int w_early = 0;
        const bool any = n_defer > 0;
        if (any) {
            HIP_TRY(hipMemsetAsync(defer, 0xFF, 3 * sizeof(int32_t) * (size_t)(K + 1), st));   // live lists: -1 = not yet
            p2_small_ok = false;
            prep_race(n_defer, n_def_l);
            prep_wide();
            c.list = defer; c.n_list = 0; c.queue = q + Q_BFS_QUEUE;
            c.live_n = q + 1; c.p1_done = q + Q_P1_DONE; c.p1_tot = q + 12;
            c.t_span = (unsigned long long *)(q + Q_T_BFS);
            b.list = defer_l; b.n_list = 0; b.live_n = q + Q_DEFER_L; b.p1_done = q + Q_P1_DONE; b.p1_tot = q + 12;
            b.s_all = nullptr; b.s_kind = nullptr; b.drained = nullptr; b.wave_off = 0;
            b.t_span = (unsigned long long *)(q + Q_T_LEAN);
            if (waves_w > 0) {
                bw.list = defer_w; bw.n_list = 0; bw.live_n = q + Q_DEFER_W; bw.p1_done = q + Q_P1_DONE; bw.p1_tot = q + 12;
                bw.s_all = nullptr; bw.s_kind = nullptr; bw.drained = nullptr;
            }
            if (n_help > 0) {
                wh.d.list = defer_l; wh.d.n_list = 0; wh.d.live_n = q + Q_DEFER_L;
                wh.d.p1_done = q + Q_P1_DONE; wh.d.p1_tot = q + 12;
                wh.d.s_all = nullptr; wh.d.s_kind = nullptr; wh.d.drained = nullptr;
                wh.seq_waves_dev = q + Q_SEQ_WAVES;
            }
            // the early LEAN grid: enough waves for the keys deferred while
            // phase 1 runs (C3: ~120), few enough to leave the BFS whole CUs
            w_early = std::min(waves2, EARLY_LEAN_WAVES);
            if (const char *e = tune_env("JH_EARLY_LEAN")) w_early = std::min(waves2, std::max(0, atoi(e)));
            const int32_t sw = waves2;
            HIP_TRY(hipMemcpyAsync(q + Q_SEQ_WAVES, &sw, sizeof sw, hipMemcpyHostToDevice, st));
            if (defer_times) {
                // tuning builds: per key [BFS start, BFS end, sequential start, end]
                unsigned long long *tl = ctx->ws<unsigned long long>(WS_TL, TL_W * (size_t)K);
                HIP_TRY(hipMemsetAsync(tl, 0, TL_W * sizeof(unsigned long long) * K, st));
                c.tl = tl; b.tl = tl;
                if (n_help > 0) wh.d.tl = tl;
            }
        }
        // phase-1 producer side: live lists, finished-key count, drain flag
        if (!ctx->hflag) {
            HIP_TRY(hipHostMalloc((void **)&ctx->hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void **)&ctx->hflag_dev, ctx->hflag, 0));
        }
        *(volatile int32_t *)ctx->hflag = 0;
        a.p1_count = q + Q_P1_DONE;
        if (any) { a.s_all = defer; a.s_kind = defer_l; }
        DfsArgs aw = a;
        aw.list = list_w; aw.n_list_dev = q + 13; aw.queue = q + 14;
        aw.defer_kind = d64 + 2 * (K + 1); aw.defer_kind_count = q + Q_DEFER_W;
        if (any) aw.s_kind = defer_w;
        // the last phase-1 kernel with keys raises the flag (WIDE keys run
        // after the LEAN kernel: then consumers start at the WIDE drain)
        a.drained = n_w1 == 0 ? ctx->hflag_dev : nullptr;
        aw.drained = n_w1 > 0 ? ctx->hflag_dev : nullptr;
        a.t_span = (unsigned long long *)(q + Q_T_P1);
        HIP_TRY(hipEventRecord(ctx->ev[6], st));     // fork: tables, lists and counters are ready
        HIP_TRY(hipEventRecord(ctx->ev[1], st));
        if (p1s != st) HIP_TRY(hipStreamWaitEvent(p1s, ctx->ev[6], 0));
        k_lin_dfs<true, true><<<waves1, 64, MemoQ::LDS, p1s>>>(a);
        HIP_TRY(hipGetLastError());
        k_lin_dfs<false, true><<<std::min(waves1, 1024), 64, MemoQ::LDS, p1s>>>(aw);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->ev[4], p1s));
        if (p1s != st) HIP_TRY(hipStreamWaitEvent(st, ctx->ev[4], 0));
        a.prio_ins = 0;
        // behind phase 1 on st: xw keys, WIDE keys, LEAN waves past the early grid's
        const int late_l = any ? waves2 - w_early : 0;
        const int n_late = waves_x + waves_w + late_l;
        if (n_late > 0) {
            DfsTriple tr{};
            tr.x = xa; tr.n_x = waves_x;
            tr.w = bw; tr.w.wave_off = waves_x; tr.n_w = waves_w;
            tr.l = b; tr.l.wave_off = waves_x + waves_w - w_early;   // its waves use tables w_early..waves2-1
            const int lds = std::max(SEQLW_LDS, XW_LDS);
            k_lin_seq_lwx<<<n_late, 64, lds, st>>>(tr);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(ctx->ev[10], st));
        if (any) {
            // the consumers, once phase 1's queue is drained: until then phase
            // 1 holds every CU, and a consumer launched earlier could take CUs
            // from it while it still has keys to hand out
            volatile int32_t *hf = (volatile int32_t *)ctx->hflag;
            while (!*hf) {
                const hipError_t e = hipEventQuery(ctx->ev[4]);
                if (e == hipSuccess) break;
                if (e != hipErrorNotReady) HIP_TRY(e);
                std::this_thread::yield();
            }
            HIP_TRY(hipStreamWaitEvent(cs2, ctx->ev[6], 0));
            k_lin_bfs<<<wg2, BFS_THREADS, BFS_LDS_BYTES, cs2>>>(c);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ctx->ev[5], cs2));
            if (n_help > 0) {
                HIP_TRY(hipStreamWaitEvent(cs3, ctx->ev[6], 0));
                k_lin_wg<<<n_wg, WG_THREADS, WG_LDS, cs3>>>(wh);
                HIP_TRY(hipGetLastError());
                HIP_TRY(hipEventRecord(ctx->ev[12], cs3));
            }
            HIP_TRY(hipStreamWaitEvent(cs1, ctx->ev[6], 0));
            if (w_early > 0) {
                DfsPair pr{};
                pr.l = b; pr.n_l = w_early;
                k_lin_seq_lw<true><<<w_early, 64, SEQLW_LDS, cs1>>>(pr);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipEventRecord(ctx->ev[11], cs1));
            // phase 3 after every phase-2 wave (both grids hand keys to it)
            HIP_TRY(hipStreamWaitEvent(st, ctx->ev[11], 0));
            HIP_TRY(hipEventRecord(ctx->ev[13], st));
            if (split3) {
                DfsArgs c3 = b;
                c3.list = defer3; c3.n_list = 0; c3.n_list_dev = q + 16; c3.defer = 0; c3.live_n = nullptr;
                c3.defer_list = nullptr; c3.defer_count = nullptr;
                c3.seq_start = nullptr; c3.exit_count = nullptr; c3.t_span = nullptr; c3.wave_off = 0;
                c3.budget = budget; c3.budget_full = 0; c3.handoff = nullptr;
                c3.gen_base = ctx->gen_base + 2 * (uint32_t)K + 1;
                c3.dbg = nullptr;
                c3.probes = (unsigned long long *)(q + Q_PROBES_P3);
                const int few = std::max(1, ctx->n_cu - wg2);
                DfsArgs c3a = c3;
                c3a.queue = q + 17; c3a.n_max = few;
                k_lin_seq<true><<<std::min(waves2, few), 64, MemoH::LDS, st>>>(c3a);
                HIP_TRY(hipGetLastError());
                DfsArgs c3b = c3;
                c3b.queue = q + 18; c3b.n_min = few + 1;
                k_lin_seq3<true><<<waves2, 64, MemoM::LDS, st>>>(c3b);
                HIP_TRY(hipGetLastError());
            }
            if (split3w) {
                DfsArgs c3 = bw;
                c3.list = defer3w; c3.n_list = 0; c3.n_list_dev = q + Q_DEFER3W; c3.queue = q + 20; c3.defer = 0;
                c3.live_n = nullptr; c3.t_span = nullptr;
                c3.defer_list = nullptr; c3.defer_count = nullptr;
                c3.budget = budget; c3.budget_full = 0; c3.wave_off = 0;
                c3.gen_base = ctx->gen_base + 2 * (uint32_t)K + 1;
                k_lin_seqw<<<waves_w, 64, SEQW_LDS, st>>>(c3);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipEventRecord(ctx->ev[7], st));
            HIP_TRY(hipStreamWaitEvent(st, ctx->ev[5], 0));
            if (n_help > 0) HIP_TRY(hipStreamWaitEvent(st, ctx->ev[12], 0));
        } else {
            HIP_TRY(hipEventRecord(ctx->ev[13], st));
            HIP_TRY(hipEventRecord(ctx->ev[7], st));
        }
        // entries per list (the phases' rooflines), the lists' lengths on the device
        EntryLists el{};
        el.list[0] = defer; el.n_dev[0] = q + 1; el.sum[0] = (unsigned long long *)(q + Q_ENT_ALL);
        el.list[1] = defer_l; el.n_dev[1] = q + Q_DEFER_L; el.sum[1] = (unsigned long long *)(q + Q_ENT_LEAN);
        el.list[2] = defer_w; el.n_dev[2] = q + Q_DEFER_W; el.sum[2] = (unsigned long long *)(q + Q_ENT_WIDE);
        el.list[3] = list_x; el.n[3] = n_x; el.sum[3] = (unsigned long long *)(q + Q_ENT_XW);
        el.list[4] = defer3; el.n_dev[4] = q + 16; el.sum[4] = (unsigned long long *)(q + Q_ENT_P3);
        el.off = off;
        k_list_entries<<<dim3(16, 5), 256, 0, st>>>(el);
    } else {
        HIP_TRY(hipEventRecord(ctx->ev[1], st));
        if (!linear_mode && !skip_p1) {
            k_lin_dfs<true, false><<<waves1, 64, MemoQ::LDS, st>>>(a);
            HIP_TRY(hipGetLastError());
            DfsArgs aw = a;
            aw.list = list_w; aw.n_list_dev = q + 13; aw.queue = q + 14;
            aw.defer_kind = d64 + 2 * (K + 1); aw.defer_kind_count = q + Q_DEFER_W;
            k_lin_dfs<false, false><<<std::min(waves1, 1024), 64, MemoQ::LDS, st>>>(aw);
            a.prio_ins = 0;                       // the heavy-key passes inherit a: no priorities there
        } else if (cfgreq) {
            k_req_lists<<<1, 1, 0, st>>>(cfgreq->keys_dev, cfgreq->n_q, K, defer, defer_l, q);
        } else {
            // :linear, or stage 2 of a two-stage check: every key that needs a
            // search is a heavy key
            k_linear_lists<<<1, 1024, 0, st>>>(list, q + 12, list_w, q + 13, defer, defer_l, defer_w, q);
        }
        a.prio_ins = 0;
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->ev[4], st));
        HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n_defer = qh[1]; n_def_l = qh[Q_DEFER_L]; n_def_w = qh[Q_DEFER_W];
        n_x = cfgreq ? 0 : qh[19];
        if (n_def_l + n_def_w != n_defer) throw_jh(JH_EDEVICE, "deferred-key lists disagree");
        if (n_defer > 0 && !linear_mode && !skip_p1) {
            // heavy keys, heaviest estimate first (the likely longest searches start
            // first), sorted on the device: no host round trip between the phases
            // (stage 1 of a two-stage check reads the list too: k_mark_deferred)
            SortLists sl{};
            const int nn[3] = {n_defer, n_def_l, n_def_w};
            int32_t *outs[3] = {defer, defer_l, defer_w};
            for (int i = 0; i < 3; i++) { sl.in[i] = d64 + (size_t)i * (K + 1); sl.out[i] = outs[i]; sl.n[i] = nn[i]; }
            k_sort_defer<<<3, 1024, 0, st>>>(sl);
            for (int i = 0; i < 3; i++) {
                if (nn[i] <= SORT_SMALL) continue;
                uint64_t *tk = ctx->ws<uint64_t>(WS_DEFER64_T, (size_t)K + 1);
                size_t tbs = 0;
                HIP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tbs, sl.in[i], tk, nn[i], 0, 64, st));
                HIP_TRY(hipcub::DeviceRadixSort::SortKeys(ctx->ws<char>(WS_LTMP, tbs), tbs, sl.in[i], tk, nn[i], 0, 64, st));
                k_unpack_keys<<<grid_for(nn[i], 256), 256, 0, st>>>(tk, nn[i], outs[i]);
            }
        }
        if (n_defer > 0 || n_x > 0) {
            // entries per list: the phases' rooflines (56 B per entry of the keys they search)
            EntryLists el{};
            el.list[0] = defer; el.n[0] = n_defer; el.sum[0] = (unsigned long long *)(q + Q_ENT_ALL);
            el.list[1] = defer_l; el.n[1] = n_def_l; el.sum[1] = (unsigned long long *)(q + Q_ENT_LEAN);
            el.list[2] = defer_w; el.n[2] = n_def_w; el.sum[2] = (unsigned long long *)(q + Q_ENT_WIDE);
            el.list[3] = list_x; el.n[3] = n_x; el.sum[3] = (unsigned long long *)(q + Q_ENT_XW);
        el.list[4] = nullptr; el.n[4] = 0;
            el.off = off;
            k_list_entries<<<dim3(16, 4), 256, 0, st>>>(el);
        }
        if (dbg2) {
            std::vector<unsigned long long> h((size_t)waves1 * 16);
            HIP_TRY(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long tot[16] = {0}, mx9 = 0;
            for (int w = 0; w < waves1; w++) { for (int k = 0; k < 16; k++) tot[k] += h[16 * w + k]; mx9 = std::max(mx9, h[16 * w + 9]); }
            fprintf(stderr, "[jh-dfs] waves=%d keys=%llu search=%.0f cyc/key | steps=%llu inserts=%llu evict=%llu lay-loads=%llu op-loads=%llu spills=%llu refills=%llu slow=%llu hbm-probes=%llu hbm-inserts=%llu | cyc/step=%.0f | wave-busy avg=%.0f max=%llu cyc\n",
                    waves1, tot[3], (double)tot[2] / std::max(1ULL, tot[3]), tot[4], tot[5], tot[6], tot[7], tot[10],
                    tot[11], tot[12], tot[13], tot[14], tot[8], (double)tot[2] / std::max(1ULL, tot[4]), (double)tot[9] / waves1, mx9);
            HIP_TRY(hipMemsetAsync(dbg, 0, sizeof(unsigned long long) * (waves1 + 512) * 16, st));
        }
        // stage 1 of a two-stage check: the 65-256-member keys are heavy keys
        // too -- they come back deferred (progress 0) for the pool, unsearched
        if (n_x > 0 && p1_only) {
            k_mark_list_deferred<<<grid_for(n_x, 256), 256, 0, st>>>(list_x, n_x, out_dev);
            HIP_TRY(hipGetLastError());
            n_x = 0;
        }
        // windows wider than 64: k_lin_xw on the third stream, alongside phases 2 and 3
        if (n_x > 0) {
            prep_xw(qh);
            xa.t_span = nullptr;
            HIP_TRY(hipEventRecord(ctx->ev[8], st));
            HIP_TRY(hipStreamWaitEvent(ctx->aux2, ctx->ev[8], 0));
            k_lin_xw<<<waves_x, 64, 0, ctx->aux2>>>(xa);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ctx->ev[9], ctx->aux2));
        }
        if (n_defer > 0 && p1_only) {
            // stage 1 of a two-stage check: the deferred keys come back unsearched
            k_mark_deferred<<<grid_for(n_defer, 256), 256, 0, st>>>(d64, n_defer, out_dev);
            HIP_TRY(hipEventRecord(ctx->ev[6], st));
            HIP_TRY(hipEventRecord(ctx->ev[5], st));
            HIP_TRY(hipEventRecord(ctx->ev[10], st));
            HIP_TRY(hipEventRecord(ctx->ev[7], st));
        } else if (n_defer > 0 && use_wg) {
            // Deferred LEAN keys on k_lin_wg (one workgroup per key, stream st),
            // WIDE keys on the aux stream
            HIP_TRY(hipMemsetAsync(q, 0, sizeof(int32_t), st));
            WgArgs wa{};
            if (n_def_l > 0) wa = build_wg(ctx->n_cu, nullptr, q);
            prep_wide();
            HIP_TRY(hipEventRecord(ctx->ev[6], st));
            HIP_TRY(hipEventRecord(ctx->ev[11], st));
            if (n_def_l > 0) {
                k_lin_wg<<<n_wg, WG_THREADS, WG_LDS, st>>>(wa);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipEventRecord(ctx->ev[5], st));
            HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev[6], 0));
            HIP_TRY(hipEventRecord(ctx->ev[10], ctx->aux));
            launch_wide(ctx->aux, true);
            HIP_TRY(hipEventRecord(ctx->ev[7], ctx->aux));
        } else if (n_defer > 0 && linear_mode) {
            // :algorithm :linear (checker.clj:141-145): the reachable-set search
            // (k_lin_bfs in linear mode) is the analysis for every key it can hold
            // -- JIT linearization's configuration sets, layer by layer -- on every
            // CU; the keys it cannot (windows over 32 members, >= 4096 states, more
            // than budget + 1 configurations) are decided by WGL afterwards on the
            // same stream, and k_frontier reports each key's analyzer.
            claim = ctx->ws<int32_t>(WS_CLAIM, K);
            HIP_TRY(hipMemsetAsync(claim, 0, (size_t)K * sizeof(int32_t), st));
            HIP_TRY(hipMemsetAsync(q, 0, sizeof(int32_t), st));
            HIP_TRY(hipMemsetAsync(q + 3, 0, sizeof(int32_t), st));
            HIP_TRY(hipMemsetAsync(q + 6, 0, 2 * sizeof(int32_t), st));
            const int64_t reach_cap = budget + 1;
            // no WGL count, nothing to store -- except for a configurations request,
            // which needs the last layer reached: every node
            const uint32_t ncap = cfgreq ? (uint32_t)std::min<int64_t>(reach_cap + 64, (int64_t)1 << 30) : 1u << 16;
            uint32_t set_cap = 1u << 12;
            while ((int64_t)set_cap < 2 * reach_cap && set_cap < (1u << 30)) set_cap <<= 1;
            const uint32_t q_cap = (uint32_t)std::min<int64_t>(reach_cap + 64, (int64_t)1 << 30);
            const uint32_t lcap = (uint32_t)smax + 2;
            const uint64_t per_bfs = (uint64_t)set_cap * 8 + 4ULL * q_cap * 8 + scr_bytes_bfs + (uint64_t)ncap * 8 +
                                     (uint64_t)lcap * 4;
            wg2 = fit_units(ctx, std::min(n_defer, ctx->n_cu), per_bfs, {WS_BFS_SET, WS_BFS_Q, WS_BFS_NODES});
            BfsArgs c{};
            c.src = KeySrc{rec, pair, off, rB, viol, rank, q + 2};
            c.list = defer; c.n_list = n_defer; c.queue = q; c.out = out_dev;
            c.unres_list = ctx->ws<int32_t>(WS_BFS_META, n_defer + 1); c.unres_count = q + 3;
            c.gset = ctx->ws<uint64_t>(WS_BFS_SET, (size_t)wg2 * set_cap); c.gset_cap = set_cap;
            uint64_t *bq = ctx->ws<uint64_t>(WS_BFS_Q, (size_t)wg2 * 4 * q_cap);
            c.pend = bq; c.front = bq + (size_t)wg2 * 2 * q_cap; c.q_cap = q_cap;
            c.scratch = ctx->ws<char>(WS_SCRATCH_BFS, (size_t)wg2 * scr_bytes_bfs); c.scratch_bytes = scr_bytes_bfs;
            c.budget = budget; c.init_state = init_state; c.states_ok = n_states < 4096 ? 1 : 0;
            c.claim = claim; c.reach_cap = reach_cap; c.linear = 1;
            c.ncap = ncap; c.hcap = 1u << 17; c.lcap = lcap;
            if (cfgreq) {
                c.cfg_slot = cfgreq->slot_dev; c.cfg_out = cfgreq->out_dev; c.cfg_n = cfgreq->n_dev;
                c.cfg_rows = cfgreq->rows_dev; c.cfg_per = cfgreq->per_key;
                c.col_val = dh->value; c.col_val2 = dh->value2;
                c.vmin = vmin; c.init_value = init; c.per_key_values = per_key_values ? 1 : 0;
            }
            c.nodes = ctx->ws<uint64_t>(WS_BFS_NODES, (size_t)wg2 * ncap);
            c.lstart = ctx->ws<uint32_t>(WS_BFS_LSTART, (size_t)wg2 * lcap);
            if (!ctx->lds_attr) {
                HIP_TRY(hipFuncSetAttribute((const void *)k_lin_bfs, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            BFS_LDS_BYTES));
                HIP_TRY(hipFuncSetAttribute((const void *)k_lin_seq<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            MemoH::LDS));
                HIP_TRY(hipFuncSetAttribute((const void *)k_lin_seq<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            MemoH::LDS));
                ctx->lds_attr = true;
            }
            // WGL for what the analysis cannot hold: LEAN and WIDE kernels over the
            // unresolved list (each takes its own kind), after the BFS
            const int want_f = std::min(n_defer, 4 * ctx->n_cu);
            const uint64_t per_f = (uint64_t)cap2 * 16 + (uint64_t)stack_cap * sizeof(Frame) + scr_bytes_h;
            waves2 = fit_units(ctx, want_f, per_f, {WS_MEMO_DEEP, WS_STACK_DEEP, WS_SCRATCH_DEEP});
            const bool fresh2 = ctx->ws_fresh(WS_MEMO_DEEP) || ctx->bufs[WS_MEMO_DEEP].bytes < (size_t)waves2 * cap2 * 16;
            uint64_t *memo2 = ctx->ws<uint64_t>(WS_MEMO_DEEP, (size_t)waves2 * cap2 * 2, /*zero=*/true);
            if (clear_memo && !fresh2) HIP_TRY(hipMemsetAsync(memo2, 0, ctx->bufs[WS_MEMO_DEEP].bytes, st));
            DfsArgs f = a;
            f.handover_min = 0;
            f.rs_mode = 0;
            f.list = c.unres_list; f.n_list = 0; f.n_list_dev = q + 3; f.queue = q + 6; f.defer = 0;
            f.defer_list = nullptr; f.defer_count = nullptr;
            f.defer64 = nullptr; f.defer_kind = nullptr; f.defer_kind_count = nullptr;
            f.memo = memo2; f.memo_cap = cap2;
            f.stack = ctx->ws<Frame>(WS_STACK_DEEP, (size_t)waves2 * stack_cap);
            f.scratch = ctx->ws<char>(WS_SCRATCH_DEEP, (size_t)waves2 * scr_bytes_h); f.scratch_bytes = scr_bytes_h;
            f.budget = budget; f.budget_full = 0; f.claim = nullptr;
            f.gen_base = ctx->gen_base + (uint32_t)K + 1;
            f.probes = (unsigned long long *)(q + 8); f.dbg = nullptr; f.defer_time = nullptr;
            f.seq_start = nullptr; f.exit_count = nullptr; f.cause_or = CAUSE_BY_WGL;
            HIP_TRY(hipEventRecord(ctx->ev[6], st));
            k_lin_bfs<<<wg2, BFS_THREADS, BFS_LDS_BYTES, st>>>(c);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ctx->ev[5], st));
            if (!cfgreq) {
                k_lin_seq3<true><<<waves2, 64, MemoM::LDS, st>>>(f);
                HIP_TRY(hipGetLastError());
                DfsArgs fw = f;
                fw.queue = q + 7;
                k_lin_seqw<<<waves2, 64, SEQW_LDS, st>>>(fw);
                HIP_TRY(hipGetLastError());
            } else {
                // configurations of the requested keys the reachable-set
                // engine cannot hold (windows over 32 members, >= 4096 states):
                // the 65-256-member search (4-word masks, every configuration
                // in its table, any window up to JH_MAX_WINDOW) and the
                // frontier from its table (xw_dump_configs)
                HIP_TRY(hipMemsetAsync(q + 26, 0, 2 * sizeof(int32_t), st));
                k_xw_need<<<grid_for(n_defer, 256), 256, 0, st>>>(c.unres_list, q + 3, meta,
                                                                 (unsigned long long *)(q + 26));
                int32_t qx[Q_WORDS];
                HIP_TRY(hipMemcpyAsync(qx, q, sizeof qx, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                n_x = qx[3];
                if (n_x > 0) {
                    prep_xw(qx);
                    xa.list = c.unres_list; xa.n_list = n_x; xa.t_span = nullptr;
                    xa.cfg_slot = cfgreq->slot_dev; xa.cfg_out = cfgreq->out_dev; xa.cfg_n = cfgreq->n_dev;
                    xa.cfg_rows = cfgreq->rows_dev; xa.cfg_per = cfgreq->per_key;
                    xa.col_val = dh->value; xa.col_val2 = dh->value2;
                    xa.vmin = vmin; xa.init_value = init; xa.per_key_values = per_key_values ? 1 : 0;
                    k_lin_xw<<<waves_x, 64, 0, st>>>(xa);
                    HIP_TRY(hipGetLastError());
                }
                n_x = 0;
            }
            HIP_TRY(hipEventRecord(ctx->ev[10], st));
            HIP_TRY(hipEventRecord(ctx->ev[7], st));
        } else if (n_defer > 0) {
            // Heavy keys: two exact searches race per key and the first to settle
            // it writes its verdict (emit_verdict), the other abandons it.
            //  - the workgroup BFS (stream st) settles keys with no reachable
            //    terminal configuration (invalid) within the budget, and valid
            //    keys whose reachable set it can store (WGL's exact count);
            //  - the sequential search with the full budget (aux stream: LEAN
            //    and WIDE keys in one grid) settles every key.
            prep_race(n_defer, n_def_l);
            if (resume) b.rs_mode = 2;      // (and phase 3, c3 = b: a record is replaced only by a takeover's newer one)
            if (!resume) { b.handoff = nullptr; wh.d.handoff = nullptr; }   // (a takeover continues from records)
            if (defer_times) {
                // tuning builds: per key [BFS start, end, sequential start, end, helper start, end]
                unsigned long long *tl = ctx->ws<unsigned long long>(WS_TL, TL_W * (size_t)K);
                HIP_TRY(hipMemsetAsync(tl, 0, TL_W * sizeof(unsigned long long) * K, st));
                c.tl = tl; b.tl = tl; bw.tl = tl;
                if (n_help > 0) wh.d.tl = tl;
            }

            // the fork point: everything the phase-2 searches read (claims, queue
            // counters, sorted lists, the cleared memo on a generation wrap) is
            // ordered before it; every table of phases 2 and 3 is allocated above
            // (an allocation after the fork would synchronise the device)
            prep_wide();
            HIP_TRY(hipEventRecord(ctx->ev[6], st));
            // fork: the BFS on st, the LEAN and WIDE sequential searches on aux
            // (one grid), helpers on aux3
            HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev[6], 0));
            k_lin_bfs<<<wg2, BFS_THREADS, BFS_LDS_BYTES, st>>>(c);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ctx->ev[5], st));
            bool wide_done = bfs_only;
            if (bfs_only || (waves2 == 0 && waves_w == 0)) {}
            else if (wg_race) { if (waves2) k_lin_wg<<<n_wg, WG_THREADS, WG_LDS, ctx->aux>>>(wr); }
            else if (p2_m) {
                DfsPair pr;
                pr.l = b; pr.w = bw; pr.n_l = waves2;
                pr.w.wave_off = waves2;
                if (n_def_w > 0) k_lin_seq_lw<false, MemoM><<<waves2 + waves_w, 64, SEQLW_LDS, ctx->aux>>>(pr);
                else k_lin_seq_lw<false, MemoP2><<<waves2, 64, MemoP2::LDS, ctx->aux>>>(pr);
                wide_done = true;
            } else if (waves2) k_lin_seq<true><<<waves2, 64, MemoH::LDS, ctx->aux>>>(b);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ctx->ev[10], ctx->aux));
            if (!bfs_only) launch_wide(ctx->aux, !wide_done);
            if (n_help > 0) {
                // every helper leaves once the sequential search has left its
                // queue (or after HELPER_MAX_TICKS): joined before the verdicts are read
                HIP_TRY(hipStreamWaitEvent(ctx->aux3, ctx->ev[6], 0));
                k_lin_wg<<<n_wg, WG_THREADS, WG_LDS, ctx->aux3>>>(wh);
                HIP_TRY(hipGetLastError());
                HIP_TRY(hipEventRecord(ctx->ev[12], ctx->aux3));
            }
            if (split3 && !bfs_only && !wg_race) {
                // phase 3: the LEAN keys phase 2 handed over, full budget, on phase 2's
                // tables (same stream, phase 2 has ended; a fresh generation range).
                // Few of them (no more than phase 2's CUs): a lone wave and the 128 KB
                // LDS memo each, as in phase 2; more: four waves per CU. Both kernels
                // are launched and the count phase 2 left on the device picks one.
                DfsArgs c3 = b;
                c3.list = defer3; c3.n_list = 0; c3.n_list_dev = q + 16; c3.defer = 0;
                c3.defer_list = nullptr; c3.defer_count = nullptr;
                c3.seq_start = nullptr; c3.exit_count = nullptr;
                c3.budget = budget; c3.budget_full = 0; c3.handoff = nullptr;
                c3.memo_cap = cap2;
                c3.gen_base = ctx->gen_base + 2 * (uint32_t)K + 1;
                c3.dbg = nullptr;
                c3.probes = (unsigned long long *)(q + Q_PROBES_P3);
                const int few = std::max(1, ctx->n_cu - wg2);
                DfsArgs c3a = c3;
                c3a.queue = q + 17; c3a.n_max = few;
                k_lin_seq<true><<<std::min(waves3, few), 64, MemoH::LDS, ctx->aux>>>(c3a);
                HIP_TRY(hipGetLastError());
                DfsArgs c3b = c3;
                c3b.queue = q + 18; c3b.n_min = few + 1;
                k_lin_seq3<true><<<waves3, 64, MemoM::LDS, ctx->aux>>>(c3b);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipEventRecord(ctx->ev[7], ctx->aux));
            HIP_TRY(hipStreamWaitEvent(st, ctx->ev[7], 0));
            if (n_help > 0) HIP_TRY(hipStreamWaitEvent(st, ctx->ev[12], 0));
            if (n_help > 0 && wh.key_prof) {
                // JH_DEBUG=4: what the late helpers took (end time in us after their start)
                HIP_TRY(hipStreamSynchronize(st));
                std::vector<unsigned long long> kp(3 * (size_t)K);
                HIP_TRY(hipMemcpy(kp.data(), wh.key_prof, kp.size() * 8, hipMemcpyDeviceToHost));
                for (int64_t k = 0; k < K; k++)
                    if (kp[3 * k])
                        fprintf(stderr, "[jh-help] key %lld wg %llu verdict %llu won %llu inserts %llu cycles %llu end_us %llu\n",
                                (long long)k, (kp[3 * k + 2] >> 8) & 0xFFF, kp[3 * k + 2] & 0xFF, (kp[3 * k + 2] >> 20) & 1,
                                kp[3 * k + 1], kp[3 * k], kp[3 * k + 2] >> 32);
            }
            if (const char *dp = tune_env("JH_BFS_DUMP")) {
                // debugging: workgroup 0's stored configurations (t:20 | s:12 | mask:32)
                HIP_TRY(hipStreamSynchronize(st));
                std::vector<uint64_t> nd(c.ncap);
                HIP_TRY(hipMemcpy(nd.data(), c.nodes, nd.size() * 8, hipMemcpyDeviceToHost));
                if (FILE *fp = fopen(dp, "wb")) { fwrite(nd.data(), 8, nd.size(), fp); fclose(fp); }
            }
            if (dbg2) {
                HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                n_unres = qh[3];
                std::vector<unsigned long long> h((size_t)wg2 * 16);
                HIP_TRY(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
                for (int w = 0; w < wg2; w++)
                    if (h[16 * w + 4])
                        fprintf(stderr, "[jh-bfs] wg %d keys=%llu cycles=%llu rounds=%llu configs=%llu cyc/round=%.0f | "
                                "count: hash=%llu live=%llu path=%llu closure=%llu cyc | global-set rounds=%llu cyc=%llu "
                                "configs=%llu, LDS-set rounds cyc=%llu configs=%llu | live: layers=%llu (LDS %llu) head-cyc=%llu LDS-layers-cyc=%llu\n",
                                w, h[16 * w + 4], h[16 * w], h[16 * w + 1], h[16 * w + 3],
                                (double)h[16 * w] / std::max(1ULL, h[16 * w + 1]), h[16 * w + 5], h[16 * w + 6],
                                h[16 * w + 7], h[16 * w + 8], h[16 * w + 10], h[16 * w + 9], h[16 * w + 11],
                                h[16 * w + 12], h[16 * w + 13], h[16 * w + 14] & 0xFFFFFFFF, h[16 * w + 14] >> 32, h[16 * w + 15], h[16 * w + 2]);
    #ifdef JH_BFS_PROF
                {
                    unsigned long long bp[8];
                    HIP_TRY(hipMemcpyFromSymbol(bp, HIP_SYMBOL(g_bfs_prof), sizeof bp));
                    const double nr = (double)std::max(1ULL, bp[4]), nl = (double)std::max(1ULL, bp[6]);
                    unsigned long long bx[4];
                    HIP_TRY(hipMemcpyFromSymbol(bx, HIP_SYMBOL(g_bfs_prof_x), sizeof bx));
                    const double ni = (double)std::max(1ULL, bx[2]);
                    fprintf(stderr, "[jh-bfs-prof] rounds=%llu cyc/round: claim+barrier %.0f items %.0f barrier %.0f tail %.0f | "
                            "layers=%llu formation cyc/layer %.0f | tid0 items=%llu cyc/item: load+children %.0f insert8 %.0f record8 %.0f\n",
                            bp[4], bp[0] / nr, bp[1] / nr, bp[2] / nr, bp[3] / nr, bp[6], bp[5] / nl, bx[2], bp[7] / ni, bx[0] / ni, bx[1] / ni);
                    memset(bx, 0, sizeof bx);
                    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_bfs_prof_x), bx, sizeof bx));
                    memset(bp, 0, sizeof bp);
                    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_bfs_prof), bp, sizeof bp));
                }
    #endif
                std::vector<unsigned long long> g((size_t)waves2 * 16);
                HIP_TRY(hipMemcpy(g.data(), dbg + 16 * 256, g.size() * 8, hipMemcpyDeviceToHost));
                for (int w = 0; w < waves2; w++)
                    if (g[16 * w + 4] > 0)
                        fprintf(stderr, "[jh-seq] wave %d keys=%llu search=%llu cyc busy=%llu | steps=%llu inserts=%llu evict=%llu lay-loads=%llu op-loads=%llu spills=%llu refills=%llu slow=%llu hbm-probes=%llu | cyc/step=%.0f\n",
                                w, g[16 * w + 3], g[16 * w + 2], g[16 * w + 9], g[16 * w + 4], g[16 * w + 5], g[16 * w + 6],
                                g[16 * w + 7], g[16 * w + 10], g[16 * w + 11], g[16 * w + 12], g[16 * w + 13], g[16 * w + 14],
                                (double)g[16 * w + 2] / std::max(1ULL, g[16 * w + 4]));
            }
        } else {
            HIP_TRY(hipEventRecord(ctx->ev[6], st));
            HIP_TRY(hipEventRecord(ctx->ev[5], st));
            HIP_TRY(hipEventRecord(ctx->ev[10], st));
            HIP_TRY(hipEventRecord(ctx->ev[7], st));
        }
        if (n_x > 0) HIP_TRY(hipStreamWaitEvent(st, ctx->ev[9], 0));
    }
    HIP_TRY(hipEventRecord(ctx->ev[2], st));
    if (defer_times && n_defer > 0) {
        // timeline: when each deferred key was handed on (us after phase 1's
        // first wave), when phase 1 ended, when the sequential search took the
        // key (if helpers ran), and the key's final insert count
        HIP_TRY(hipStreamSynchronize(st));
        if (stream_p2) {
            int32_t nd = 0;
            HIP_TRY(hipMemcpy(&nd, q + 1, sizeof nd, hipMemcpyDeviceToHost));
            n_defer = nd;
        }
        std::vector<unsigned long long> dt((size_t)K + 2);
        HIP_TRY(hipMemcpy(dt.data(), a.defer_time, dt.size() * 8, hipMemcpyDeviceToHost));
        std::vector<int32_t> dk(n_defer);
        HIP_TRY(hipMemcpy(dk.data(), defer, sizeof(int32_t) * n_defer, hipMemcpyDeviceToHost));
        std::vector<jh_key_verdict> vv(K);
        HIP_TRY(hipMemcpy(vv.data(), out_dev, sizeof(jh_key_verdict) * K, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> ss;
        if (ctx->bufs.size() > WS_HELP_START && ctx->bufs[WS_HELP_START].p) {
            ss.resize(K);
            HIP_TRY(hipMemcpy(ss.data(), ctx->bufs[WS_HELP_START].p, 8 * K, hipMemcpyDeviceToHost));
        }
        fprintf(stderr, "[jh-defer] phase 1: %.1f us (first wave start to last wave end)\n", (dt[1] - dt[0]) / 100.0);
        std::vector<std::pair<double, int>> ev;
        for (int d = 0; d < n_defer; d++) ev.push_back({(dt[2 + dk[d]] - dt[0]) / 100.0, dk[d]});
        std::vector<std::pair<long long, int>> heavy;
        for (int d = 0; d < n_defer; d++) heavy.push_back({vv[dk[d]].explored, dk[d]});
        std::sort(heavy.rbegin(), heavy.rend());
        std::vector<unsigned long long> tl;
        if (ctx->bufs.size() > WS_TL && ctx->bufs[WS_TL].p) {
            tl.resize(TL_W * (size_t)K);
            HIP_TRY(hipMemcpy(tl.data(), ctx->bufs[WS_TL].p, 8 * tl.size(), hipMemcpyDeviceToHost));
        }
        auto us = [&](unsigned long long t) { return t ? (double)(t - dt[0]) / 100.0 : -1.0; };
        for (int i = 0; i < std::min(n_defer, 12); i++) {
            const int k = heavy[i].second;
            double st_us = -1;
            if (!ss.empty() && ss[k] && ss[k] != SEQ_HANDED) st_us = ((ss[k] & ~1ULL) - dt[0]) / 100.0;
            fprintf(stderr, "[jh-defer] key %d explored %lld valid %d deferred %.1f us seq-start %.1f us", k,
                    heavy[i].first, vv[k].valid, (dt[2 + k] - dt[0]) / 100.0, st_us);
            if (!tl.empty())
                fprintf(stderr, " | bfs %.1f-%.1f us seq %.1f-%.1f us", us(tl[TL_W * k]), us(tl[TL_W * k + 1]),
                        us(tl[TL_W * k + 2]), us(tl[TL_W * k + 3]));
            fprintf(stderr, "\n");
        }
        if (!tl.empty()) {
            // the keys that ended last (the step's critical path)
            std::vector<std::pair<unsigned long long, int>> last;
            for (int d = 0; d < n_defer; d++) {
                const int k = dk[d];
                unsigned long long e = 0;
                for (int w = 1; w < TL_W; w += 2) e = std::max(e, tl[TL_W * k + w]);
                last.push_back({e, k});
            }
            std::sort(last.rbegin(), last.rend());
            for (int i = 0; i < std::min(n_defer, 8); i++) {
                const int k = last[i].second;
                fprintf(stderr, "[jh-last] key %d explored %lld valid %d deferred %.1f | bfs %.1f-%.1f seq %.1f-%.1f help %.1f-%.1f us\n",
                        k, (long long)vv[k].explored, vv[k].valid, (dt[2 + k] - dt[0]) / 100.0, us(tl[TL_W * k]),
                        us(tl[TL_W * k + 1]), us(tl[TL_W * k + 2]), us(tl[TL_W * k + 3]), us(tl[TL_W * k + 4]),
                        us(tl[TL_W * k + 5]));
            }
        }
        if (const char *csv = tune_env("JH_TL_CSV")) {
            // every deferred key: its quick search, its engines' times, its verdict
            std::vector<unsigned long long> di(2 * (size_t)K);
            HIP_TRY(hipMemcpy(di.data(), a.defer_info, 8 * di.size(), hipMemcpyDeviceToHost));
            if (FILE *fo = fopen(csv, "a")) {
                fprintf(fo, "key,explored,valid,deferred_us,p1_inserts,p1_tmax,n_ok,bfs0,bfs1,seq0,seq1,help0,help1\n");
                for (int d = 0; d < n_defer; d++) {
                    const int k = dk[d];
                    fprintf(fo, "%d,%lld,%d,%.1f,%llu,%llu,%llu", k, (long long)vv[k].explored, vv[k].valid,
                            (dt[2 + k] - dt[0]) / 100.0, di[2 * k], di[2 * k + 1] & 0xFFFFFFFFull, di[2 * k + 1] >> 32);
                    for (int w = 0; w < TL_W; w++) fprintf(fo, ",%.1f", tl.empty() ? -1.0 : us(tl[TL_W * k + w]));
                    fprintf(fo, "\n");
                }
                fclose(fo);
            }
        }
        int q5[5] = {0, 0, 0, 0, 0};
        for (auto &e2 : ev) q5[std::min(4, (int)(e2.first / (std::max(1.0, (dt[1] - dt[0]) / 100.0) / 5)))]++;
        fprintf(stderr, "[jh-defer] deferrals by fifth of phase 1: %d %d %d %d %d\n", q5[0], q5[1], q5[2], q5[3], q5[4]);
    }
    ctx->gen_base += gen_span;

    k_fail_rows<<<(unsigned)std::min<int64_t>((K + 3) / 4, 4096), 256, 0, st>>>(
        KeySrc{rec, pair, off, rB, viol, rank, q + 2}, out_dev, K);
    k_frontier<<<(unsigned)std::min<int64_t>((K + 3) / 4, 4096), 256, 0, st>>>(
        KeySrc{rec, pair, off, rB, viol, rank, q + 2}, out_dev, K, linear_mode ? 1 : 0);
    long long *sd = ctx->ws<long long>(WS_SUMMARY, 8);
    long long s_init[8] = {0, 0, 0, LLONG_MAX, 0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(sd, s_init, sizeof s_init, hipMemcpyHostToDevice, st));
    k_summary<<<grid_for(K, 256, 1024), 256, 0, st>>>(out_dev, K, sd);
    long long sh[8];
    HIP_TRY(hipMemcpyAsync(sh, sd, sizeof sh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ctx->ev[3], st));
    HIP_TRY(hipStreamSynchronize(st));
    if (qh[2] & 2) throw_jh(JH_EDEVICE, "per-key table exceeded the scratch reservation");
    if (qh[2] & 4) throw_jh(JH_EDEVICE, "DFS stack overflow");
    if ((qh[2] & 0x1F0) && acc_stats && ctx->bufs.size() > WS_DEBUG_WG && ctx->bufs[WS_DEBUG_WG].p && n_wg > 0 &&
        dbgenv && atoi(dbgenv) >= 3) {
        std::vector<unsigned long long> tr((size_t)n_wg * 256);
        HIP_TRY(hipMemcpy(tr.data(), ctx->bufs[WS_DEBUG_WG].p, tr.size() * 8, hipMemcpyDeviceToHost));
        for (int g = 0; g < n_wg; g++) {
            for (int e = 0; e < 31; e++) {
                const unsigned long long *d8 = &tr[(size_t)g * 256 + 8 * e];
                if (!d8[3]) break;
                fprintf(stderr, "[jh-acc] wg %d key %llu d %llu depth %llu roots %llu cap %llu status %llu tail %llu ins %llu\n",
                        g, d8[0], d8[1], d8[2], d8[3], d8[4], d8[5], d8[6], d8[7]);
            }
            const unsigned long long *w8 = &tr[(size_t)g * 256 + 248];
            if (w8[6] == 0xDEAD)
                fprintf(stderr, "[jh-acc] wg %d WATCHDOG head %llu tail %llu active %llu cap_total %llu roots %llu wave %llu\n",
                        g, w8[0], w8[1], w8[2], w8[3], w8[4], w8[5]);
            const unsigned long long *l8 = &tr[(size_t)g * 256 + 240];
            if (l8[3] == 0xBEEF)
                fprintf(stderr, "[jh-acc] wg %d LOST ITEM pos %llu tail %llu cap_total %llu\n", g, l8[0], l8[1], l8[2]);
        }
    }
    if (qh[2] & 0x3F0) {
        char m[192];
        snprintf(m, sizeof m, "search watchdog tripped (flags 0x%x: 16 lost work item, 32 idle enumeration, "
                 "64 full set, 128 step limit, 256 bad window, 512 stream wait)", qh[2]);
        throw_jh(JH_EDEVICE, m);
    }
    if (stream_p2) {
        // the live lists' final lengths (the bounds used to size the pass above)
        n_defer = qh[1]; n_def_l = qh[Q_DEFER_L]; n_def_w = qh[Q_DEFER_W];
        if (n_def_l + n_def_w != n_defer) throw_jh(JH_EDEVICE, "deferred-key lists disagree");
    }
    if (tune_env("JH_WS_REPORT")) {
        // tuning builds: the context's workspace, largest buffers first
        std::vector<std::pair<size_t, int>> b;
        size_t tot = 0;
        for (int i = 0; i < (int)ctx->bufs.size(); i++) { b.push_back({ctx->bufs[i].bytes, i}); tot += ctx->bufs[i].bytes; }
        std::sort(b.rbegin(), b.rend());
        fprintf(stderr, "[jh-ws] total %.2f GB:", tot / 1073741824.0);
        for (size_t i = 0; i < b.size() && i < 12; i++) fprintf(stderr, " slot %d %.2f GB;", b[i].second, b[i].first / 1073741824.0);
        fprintf(stderr, "\n");
    }
    if (sum) {
        sum->valid = sh[0]; sum->n_invalid = sh[1]; sum->n_unknown = sh[2];
        sum->first_fail_entry = sh[3] == LLONG_MAX ? -1 : sh[3];
        sum->n_keys = sh[4]; sum->explored = sh[5];
        sum->memo_probes = q64(qh, 4);
        float ms = 0, ms_dfs = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[3]));
        HIP_TRY(hipEventElapsedTime(&ms_dfs, ctx->ev[1], ctx->ev[4]));
        sum->device_ms = ms; sum->dfs_ms = ms_dfs;
        sum->n_deferred = n_defer;
        sum->deferred_entries = q64(qh, Q_ENT_ALL);
        sum->seq_probes = q64(qh, 8);
        sum->seq_ms = 0; sum->bfs_ms = 0; sum->p3_ms = 0; sum->wide_ms = 0; sum->xw_ms = 0;
        sum->streamed = stream_p2 ? 1 : 0;
        sum->p3_entries = q64(qh, Q_ENT_P3);
        sum->p2_start_ms = -1; sum->p1_span_ms = 0;
        sum->resumed = resume ? qh[Q_RS_USED + 2] : 0;
        sum->takeovers = resume ? qh[Q_RS_USED + 3] : 0;
        sum->spec_nodes = q64(qh, Q_SPEC); sum->spec_merges = qh[Q_SPEC + 2];
        sum->spec_jobs = qh[Q_SPEC + 3]; sum->spec_dead = qh[Q_SPEC + 4];
        sum->resume_bytes = resume ? q64(qh, Q_RS_USED) : 0;
        // an engine's own span from its s_memrealtime words (100 MHz): [first key, last wave end]
        auto span_ms = [&](int w) {
            const int64_t t0 = q64(qh, w), t1 = q64(qh, w + 2);
            return (t0 != -1 && t1 > t0) ? (t1 - t0) / 1e5 : 0.0;
        };
        if (stream_p2) {
            sum->p1_span_ms = span_ms(Q_T_P1);
            sum->seq_ms = span_ms(Q_T_LEAN);
            sum->bfs_ms = span_ms(Q_T_BFS);
            sum->xw_ms = span_ms(Q_T_XW);
            if (waves_w > 0) sum->wide_ms = span_ms(Q_T_WIDE);
            if (split3) { float c2 = 0; HIP_TRY(hipEventElapsedTime(&c2, ctx->ev[13], ctx->ev[7])); sum->p3_ms = c2; }
            const int64_t p1s = q64(qh, Q_T_P1);
            int64_t first = -1;
            for (int w : {Q_T_BFS, Q_T_LEAN}) {
                const int64_t t = q64(qh, w);
                if (t != -1 && (first == -1 || t < first)) first = t;
            }
            if (first != -1 && p1s != -1) sum->p2_start_ms = (first - p1s) / 1e5;
        } else if (n_defer > 0) {
            float a2 = 0, b2 = 0;
            if (use_wg) HIP_TRY(hipEventElapsedTime(&a2, ctx->ev[11], ctx->ev[5]));
            else HIP_TRY(hipEventElapsedTime(&a2, ctx->ev[6], ctx->ev[10]));
            sum->seq_ms = a2;
            if (!use_wg) { HIP_TRY(hipEventElapsedTime(&b2, ctx->ev[6], ctx->ev[5])); sum->bfs_ms = b2; }
            if (split3) { float c2 = 0; HIP_TRY(hipEventElapsedTime(&c2, ctx->ev[10], ctx->ev[7])); sum->p3_ms = c2; }
            // the heavy-key pass's start (the fork), after phase 1's start
            if (!use_wg && !p1_only) { float g2 = 0; HIP_TRY(hipEventElapsedTime(&g2, ctx->ev[1], ctx->ev[6])); sum->p2_start_ms = g2; }
            // the WIDE waves' own span (they share a grid with the LEAN ones)
            if (waves_w > 0 && q64(qh, Q_T_WIDE + 2) > q64(qh, Q_T_WIDE)) sum->wide_ms = (q64(qh, Q_T_WIDE + 2) - q64(qh, Q_T_WIDE)) / 1e5;
        }
        if (n_x > 0 && !stream_p2) { float e2 = 0; HIP_TRY(hipEventElapsedTime(&e2, ctx->ev[8], ctx->ev[9])); sum->xw_ms = e2; }
#ifdef JH_XW_PROF
        if (n_x > 0) {
            unsigned long long x[12];
            HIP_TRY(hipMemcpyFromSymbol(x, HIP_SYMBOL(g_xw_prof), sizeof x));
            const double ni = (double)std::max(1ULL, x[5]);
            fprintf(stderr, "[jh-xw-prof] keys=%llu inserts=%llu cyc/insert: search %.0f | probe %.0f (%.2f slice probes) "
                    "push %.0f lift %.0f | layer loads %.2f x %.0f cyc | pops %.2f x %.0f cyc (HBM frames %llu)\n",
                    x[11], x[5], x[0] / ni, x[1] / ni, x[6] / ni, x[4] / ni, x[9] / ni, x[7] / ni,
                    x[2] / (double)std::max(1ULL, x[7]), x[8] / ni, x[3] / (double)std::max(1ULL, x[8]), x[10]);
            memset(x, 0, sizeof x);
            HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_xw_prof), x, sizeof x));
        }
#endif
        sum->p3_probes = q64(qh, Q_PROBES_P3);
        sum->wide_probes = q64(qh, Q_PROBES_WIDE);
        sum->xw_probes = q64(qh, 22);
        sum->helper_probes = q64(qh, Q_PROBES_HELP);
        sum->n_deferred_wide = n_def_w;
        sum->n_phase3 = split3 ? qh[16] : 0;
        sum->n_phase3_wide = split3w ? qh[Q_DEFER3W] : 0;
        sum->n_xw = n_x;
        sum->lean_entries = q64(qh, Q_ENT_LEAN);
        sum->wide_entries = q64(qh, Q_ENT_WIDE);
        sum->xw_entries = q64(qh, Q_ENT_XW);
        sum->waves[0] = waves2; sum->waves[1] = waves_w; sum->waves[2] = split3 ? waves3 : 0; sum->waves[3] = waves_x;
        if (dbgenv) {
            float a = 0, b = 0, c = 0;
            HIP_TRY(hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]));
            HIP_TRY(hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[4]));
            float d = 0;
            HIP_TRY(hipEventElapsedTime(&d, ctx->ev[4], ctx->ev[7]));
            HIP_TRY(hipEventElapsedTime(&c, ctx->ev[4], ctx->ev[5]));
            fprintf(stderr, "[jh] keys=%lld prep=%.3f ms phase1=%.3f ms (waves %d) deferred=%d (wide %d) bfs=%.3f ms (gave up %d) "
                    "seq=%.3f ms (phase 2 %.3f ms, phase 3 %lld keys %.3f ms) wide %.3f ms (%d waves, phase 3 %lld keys) "
                    "xw %d keys %.3f ms (%d waves)\n",
                    (long long)K, a, b, waves1, n_defer, n_def_w, c, n_unres, d, sum->seq_ms, (long long)sum->n_phase3,
                    sum->p3_ms, sum->wide_ms, waves_w, (long long)sum->n_phase3_wide, n_x, sum->xw_ms, waves_x);
            if (acc_stats && dbgenv && atoi(dbgenv) >= 3 && n_wg > 0) {
                std::vector<unsigned long long> tr((size_t)n_wg * 256);
                HIP_TRY(hipMemcpy(tr.data(), ctx->bufs[WS_DEBUG_WG].p, tr.size() * 8, hipMemcpyDeviceToHost));
                for (int g = 0; g < std::min(n_wg, 8); g++)
                    for (int e = 0; e < 32; e++) {
                        const unsigned long long *d8 = &tr[(size_t)g * 256 + 8 * e];
                        if (!d8[3]) break;
                        fprintf(stderr, "[jh-acc] wg %d key %llu d %llu depth %llu roots %llu cap %llu status %llu tail %llu ins %llu\n",
                                g, d8[0], d8[1], d8[2], d8[3], d8[4], d8[5], d8[6], d8[7]);
                    }
            }
            if (acc_stats && dbgenv && atoi(dbgenv) >= 4) {
                std::vector<unsigned long long> kp(3 * (size_t)K);
                HIP_TRY(hipMemcpy(kp.data(), ctx->bufs[WS_STATS_KEYS].p, kp.size() * 8, hipMemcpyDeviceToHost));
                std::vector<int> ix;
                for (int64_t k = 0; k < K; k++) if (kp[3 * k]) ix.push_back((int)k);
                std::sort(ix.begin(), ix.end(), [&](int x, int y) { return kp[3 * x] > kp[3 * y]; });
                for (size_t i = 0; i < std::min<size_t>(12, ix.size()); i++)
                    fprintf(stderr, "[jh-key] key %d memtime %.3g inserts %llu verdict %llu wg %llu\n", ix[i],
                            (double)kp[3 * ix[i]], kp[3 * ix[i] + 1], kp[3 * ix[i] + 2] & 255, kp[3 * ix[i] + 2] >> 8);
            }
#ifdef JH_ENUM_PROF
            {
                unsigned int a4[4]; unsigned long long b3[3];
                HIP_TRY(hipMemcpyFromSymbol(a4, HIP_SYMBOL(g_prof_hbm), 4));
                HIP_TRY(hipMemcpyFromSymbol(a4 + 1, HIP_SYMBOL(g_prof_gset), 4));
                HIP_TRY(hipMemcpyFromSymbol(a4 + 2, HIP_SYMBOL(g_prof_rounds), 4));
                HIP_TRY(hipMemcpyFromSymbol(a4 + 3, HIP_SYMBOL(g_prof_layers), 4));
                HIP_TRY(hipMemcpyFromSymbol(b3, HIP_SYMBOL(g_prof_form), 8));
                HIP_TRY(hipMemcpyFromSymbol(b3 + 1, HIP_SYMBOL(g_prof_close), 8));
                fprintf(stderr, "[jh-prof] hbm-probes %u gset-inserts %u rounds %u layers %u | memtime formation %.3g closure %.3g\n",
                        a4[0], a4[1], a4[2], a4[3], (double)b3[0], (double)b3[1]);
                unsigned int z4[4] = {0, 0, 0, 0}; unsigned long long zb[3] = {0, 0, 0};
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_hbm), z4, 4));
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_gset), z4, 4));
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_rounds), z4, 4));
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_layers), z4, 4));
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_form), zb, 8));
                HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_close), zb, 8));
            }
#endif
            if (acc_stats) {
                unsigned long long st8[8];
                HIP_TRY(hipMemcpy(st8, acc_stats, sizeof st8, hipMemcpyDeviceToHost));
                fprintf(stderr, "[jh-wg] workgroups=%d enumerations=%llu new-nodes=%llu dead=%llu live=%llu inconclusive=%llu | "
                        "memtime: keys %.3g, in enumerations %.3g (work loops %.3g)\n",
                        n_wg, st8[0], st8[1], st8[2], st8[3], st8[4], (double)st8[7], (double)st8[5], (double)st8[6]);
            }
        }
    }
}

// The per-key row index (CSR) of an independent history: the same stable
// radix partition the check starts with, handed back so a caller can write
// every key's subhistory (independent.clj:234-245, :277-284) in one O(N) pass
// instead of K scans of the whole history.
void key_index(jh_ctx *ctx, const jh_history *dh, int64_t *key_off, int64_t *rows, hipStream_t st) {
    const int64_t n = dh->n, K = dh->n_keys;
    if (K >= (1LL << 31) - 2) throw_jh(JH_EUNSUPPORTED, "more than 2^31 keys");
    if (n >= (1LL << 32) - 1) throw_jh(JH_EUNSUPPORTED, "more than 2^32 entries");
    uint32_t *kA = ctx->ws<uint32_t>(WS_KEYS_A, n), *kB = ctx->ws<uint32_t>(WS_KEYS_B, n);
    uint32_t *rA = ctx->ws<uint32_t>(WS_ROWS_A, n), *rB = ctx->ws<uint32_t>(WS_ROWS_B, n);
    uint32_t *off = ctx->ws<uint32_t>(WS_SEG_OFF, K + 2);
    RangeOut *ro = ctx->ws<RangeOut>(WS_MISC, 1);
    int64_t *wide = ctx->ws<int64_t>(WS_C_TMP, std::max<int64_t>(n, K + 1));
    if (n > 0) {
        k_keys<<<grid_for(n, 256), 256, 0, st>>>(dh->key, n, K, 1, kA, rA);
        const int endbit = bits_for((uint64_t)K);
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kA, kB, rA, rB, (int)n, 0, endbit, st));
        void *tmp = ctx->ws<char>(WS_SORT_TMP, tb);
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kA, kB, rA, rB, (int)n, 0, endbit, st));
        k_seg_off<<<grid_for(K + 1, 256), 256, 0, st>>>(kB, n, K, off, ro);
        k_widen<<<grid_for(n, 256), 256, 0, st>>>(rB, n, wide);
        HIP_TRY(hipMemcpyAsync(rows, wide, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
        k_widen<<<grid_for(K + 1, 256), 256, 0, st>>>(off, K + 1, wide);
        HIP_TRY(hipMemcpyAsync(key_off, wide, sizeof(int64_t) * (K + 1), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    } else {
        for (int64_t k = 0; k <= K; ++k) key_off[k] = 0;
    }
}

