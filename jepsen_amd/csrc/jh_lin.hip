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
constexpr int LDS_BYTES = 20480;          // per-wave table budget (8 waves/CU)
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
    uint32_t t_i;     // t << 6 | i
    int32_t s;
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

__global__ void k_range(const int64_t *__restrict__ proc, const int64_t *__restrict__ f,
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
    // wave reduce
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
        pm = max(pm, __shfl_xor(pm, o));
        unk |= __shfl_xor(unk, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&out->vmin, lo);
        atomicMax(&out->vmax, hi);
        atomicMax(&out->pmax, pm);
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
// that is not :info; an :invoke there is a double invocation.
__global__ void k_pair(const Rec *__restrict__ rec, const uint32_t *__restrict__ sk,
                       const uint32_t *__restrict__ off, int64_t m, int32_t *__restrict__ pair,
                       unsigned long long *__restrict__ viol) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m;
         p += (int64_t)gridDim.x * blockDim.x) {
        Rec x = rec[p];
        if (x.proc < 0 || x.type != T_INVOKE) continue;
        uint32_t k = sk[p];
        uint32_t end = off[k + 1];
        for (uint32_t j = (uint32_t)p + 1; j < end; j++) {
            Rec y = rec[j];
            if (y.proc != x.proc || y.type == T_INFO) continue;
            if (y.type == T_INVOKE) {
                atomicMin(&viol[k], ((unsigned long long)j << 4) | JH_CAUSE_DOUBLE_INVOKE);
            } else {
                pair[p] = (int32_t)j;
                pair[j] = (int32_t)p;
            }
            break;
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
    int32_t *defer_list;        // phase 1: keys over the quick budget
    int32_t *defer_count;
    uint64_t *memo;             // per wave: memo_cap entries x 2 words
    uint32_t memo_cap;          // power of two
    Frame *stack;               // per wave: stack_cap frames
    uint32_t stack_cap;
    char *scratch;              // per wave global table space (keys too big for LDS)
    uint64_t scratch_bytes;
    int64_t budget;             // memo inserts before giving up
    int32_t defer;              // 1: over budget -> defer list; 0: -> :unknown
    int32_t init_state;
    uint32_t gen_base;
    int32_t *flags;             // [0] |= 1: key too large for this build
    unsigned long long *probes; // total memo probes (roofline accounting)
};

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

// Per-key tables, built by ONE wave (lanes 0..63) into LDS (or this wave's
// global scratch when they do not fit):
//   ops[j]   the key's ops in call order: completed values, return rank rr
//            (-1 crashed) and a = # ok returns before the invocation
//   W, woff  the window table: W(t) = ops called before the t-th ok return
//            and not yet returned there, in call order (<= 64 per t)
// knossos.history/complete is applied here from the pairing (k_pair):
// failed ops and crashed/nil reads are dropped (sound; see jh_oracle.c).
// Returns true if a search is needed; otherwise v is the key's verdict.
struct KeySrc {
    const Rec *rec;
    const int32_t *pair;
    const uint32_t *off;
    const uint32_t *rows;
    const unsigned long long *viol;
    int32_t *rank;
    int32_t *flags;
};
struct KeyTables {
    Op *ops;
    int32_t *woff;
    uint16_t *W;
    int n_ops, n_ok;
    uint32_t s0, s1;
};

__device__ bool build_key_tables(const KeySrc &S, int key, int lane, char *lds, int lds_bytes,
                                 char *gscr, uint64_t scr_bytes, KeyTables &T, jh_key_verdict &v) {
    const uint32_t s0 = S.off[key], s1 = S.off[key + 1];
    v.valid = JH_VALID; v.cause = 0; v.fail_entry = -1; v.explored = 0;
    if (s0 == s1) {                          // key absent: no :results entry
        v.explored = -1;
        return false;
    }
    const unsigned long long vi = S.viol[key];
    if (vi != VIOL_NONE) {
        v.valid = JH_UNKNOWN; v.cause = (int)(vi & 15);
        return false;
    }

    // ---- pass 1: ranks of kept invocations and of ok returns -----------
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
    if (badf) {
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_BAD_F;
        return false;
    }
    if (n_ok == 0) {
        return false;
    }
    const long long sumW = (long long)n_ok * (n_ok + 1) / 2 - sum_a_ok +
                           (long long)n_crash * n_ok - sum_a_crash;
    if (sumW > 64LL * n_ok) {                // the average window is wider than 64
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }
    if (n_ops > 65535 || n_ok >= (int)T_MASK) {
        if (lane == 0) atomicOr(S.flags, 1);
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }
    // ---- table placement: LDS if it fits, else this wave's global scratch
    const uint64_t b_ops = (uint64_t)n_ops * sizeof(Op);
    const uint64_t b_off = ((uint64_t)(n_ok + 1) * 4 + 15) & ~15ULL;
    const uint64_t b_w = ((uint64_t)sumW * 2 + 128 + 15) & ~15ULL;   // +64 entries slack
    const uint64_t total = b_ops + b_off + b_w;
    char *tb;
    if (total <= (uint64_t)lds_bytes) tb = lds;
    else if (total <= scr_bytes) tb = gscr;
    else {
        if (lane == 0) atomicOr(S.flags, 2);
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }
    Op *ops = (Op *)tb;
    int32_t *woff = (int32_t *)(tb + b_ops);
    uint16_t *W = (uint16_t *)(tb + b_ops + b_off);

    // ---- pass 2: op records in call order --------------------------------
    {
        int nops = 0, nok = 0;
        for (uint32_t base = s0; base < s1; base += 64) {
            const uint32_t p = base + lane;
            const bool valid = p < s1;
            const int rk = valid ? S.rank[p] : -1;
            const bool kept = rk >= 0, ret = rk <= -2;
            const uint64_t bi = ballot(kept), br = ballot(ret);
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
            nops += __popcll(bi);
            nok += __popcll(br);
        }
    }
    wave_sync();

    // ---- window table W(t): W(t) = W(t-1) - {RET[t-1]} + {ops with a == t}
    int too_wide = 0;
    {
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
            if (w > 64) { too_wide = 1; break; }
            if (lane == 0) woff[t] = offt;
            offt += w;
            wave_sync();
        }
        if (lane == 0) woff[n_ok] = offt;
    }
    wave_sync();
    if (too_wide) {
        v.valid = JH_UNKNOWN; v.cause = JH_CAUSE_WINDOW;
        return false;
    }

    T.ops = ops; T.woff = woff; T.W = W; T.n_ops = n_ops; T.n_ok = n_ok; T.s0 = s0; T.s1 = s1;
    return true;
}

// history row of the ok completion of RET[t] (the first op no configuration
// gets past, for an invalid key)
__device__ long long ret_row(const KeySrc &S, const KeyTables &T, uint32_t t, int lane) {
    const int want = -((int)t + 2);
    for (uint32_t base = T.s0; base < T.s1; base += 64) {
        const uint32_t p = base + lane;
        const bool hit = p < T.s1 && S.rank[p] == want;
        const uint64_t b = ballot(hit);
        if (b) {
            const int l = __builtin_ctzll(b);
            return (long long)S.rows[readlane((int)p, l)];
        }
    }
    return -1;
}

__global__ void __launch_bounds__(64) k_lin_dfs(DfsArgs A) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x;
    const uint64_t lane_bit = 1ULL << lane;
    uint64_t *memo = A.memo + (size_t)blockIdx.x * A.memo_cap * 2;
    Frame *stack = A.stack + (size_t)blockIdx.x * A.stack_cap;
    char *gscr = A.scratch + (size_t)blockIdx.x * A.scratch_bytes;
    const uint32_t cap_mask = A.memo_cap - 1;
    unsigned long long my_probes = 0;
    const KeySrc src{A.rec, A.pair, A.off, A.rows, A.viol, A.rank, A.flags};

    for (;;) {
        int idx = 0;
        if (lane == 0) idx = atomicAdd(A.queue, 1);
        idx = readlane(idx, 0);
        if (idx >= A.n_list) break;
        const int key = A.list[idx];
        jh_key_verdict v;
        KeyTables T;
        if (!build_key_tables(src, key, lane, lds, LDS_BYTES, gscr, A.scratch_bytes, T, v)) {
            if (lane == 0) A.out[key] = v;
            continue;
        }
        const int n_ok = T.n_ok;
        const Op *ops = T.ops;
        const int32_t *woff = T.woff;
        const uint16_t *W = T.W;
        // ---- WGL search in canonical coordinates ------------------------------
        const uint32_t gen = (A.gen_base + (uint32_t)key + 1) & ((1u << GEN_BITS) - 1);
        const uint64_t gen_hi = (uint64_t)gen << 40;
        uint32_t t = 0, tmax = 0, depth = 0;
        uint64_t mask = 0;
        int s = A.init_state, start = 0;
        long long inserts = 0;
        int verdict = -1;
        // lane-resident window member
        int w = 0, o_f = 0, o_v1 = 0, o_v2 = 0, o_rr = -1;
        auto load_window = [&](uint32_t tt) {
            const int wo = woff[tt];
            w = woff[tt + 1] - wo;
            if (lane < w) {
                const Op o = ops[W[wo + lane]];
                o_f = o.fa & 3; o_v1 = o.v1; o_v2 = o.v2; o_rr = o.rr;
            } else { o_f = 0; o_v1 = 0; o_v2 = 0; o_rr = -1; }
        };
        load_window(0);
        while (verdict < 0) {
            // candidates: un-linearized members at or after `start` the model allows
            int s2 = 0;
            const bool cand = lane < w && lane >= start && !((mask >> lane) & 1) &&
                              cas_step(o_f, o_v1, o_v2, s, &s2);
            const uint64_t bc = ballot(cand);
            uint32_t ct = t;
            uint64_t cm = mask | lane_bit;
            // the member whose return defines R advances t and compacts the mask
            const uint64_t bret = ballot(cand && o_rr == (int)t);
            if (bret) {
                const uint64_t lin = mask | bret;
                uint32_t u = t + 1;
                while (u < (uint32_t)n_ok && ballot(((lin >> lane) & 1) && o_rr == (int)u)) u++;
                uint64_t nm = 0;
                if (u < (uint32_t)n_ok) {
                    const uint64_t keep = ballot(lane < w && (o_rr < 0 || o_rr >= (int)u));
                    uint64_t bits = lin & keep;
                    while (bits) {
                        const int b = __builtin_ctzll(bits);
                        bits &= bits - 1;
                        nm |= 1ULL << __popcll(keep & ((1ULL << b) - 1));
                    }
                }
                if (o_rr == (int)t) { ct = u; cm = nm; }
            }
            // memo probes, all candidates at once (= the sequential scan, since
            // nothing is inserted until the first new child is chosen)
            bool absent = false;
            uint32_t slot = 0;
            if (cand) {
                uint32_t h = (uint32_t)memo_hash(ct, (uint32_t)s2, cm) & cap_mask;
                const uint64_t w1want = gen_hi | ((uint64_t)ct << 20) | (uint32_t)s2;
                for (;;) {
                    const uint64_t e1 = __hip_atomic_load(&memo[2 * (size_t)h + 1], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                    my_probes++;
                    if ((e1 >> 40) != gen) { absent = true; slot = h; break; }
                    if (e1 == w1want) {
                        const uint64_t e0 = __hip_atomic_load(&memo[2 * (size_t)h], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (e0 == cm) break;
                    }
                    h = (h + 1) & cap_mask;
                }
            }
            const uint64_t bn = ballot(absent);
            if (bn) {
                if (inserts >= A.budget) { verdict = JH_UNKNOWN; break; }
                const int i = __builtin_ctzll(bn);
                if (lane == i) {
                    __hip_atomic_store(&memo[2 * (size_t)slot], cm, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&memo[2 * (size_t)slot + 1],
                                       gen_hi | ((uint64_t)ct << 20) | (uint32_t)s2,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                inserts++;
                if (lane == 0) {
                    Frame fr; fr.mask = mask; fr.t_i = (t << 6) | (uint32_t)i; fr.s = s;
                    stack[depth] = fr;
                }
                depth++;
                const uint32_t nt = (uint32_t)readlane((int)ct, i);
                const uint64_t nm = ((uint64_t)(uint32_t)readlane((int)(uint32_t)(cm >> 32), i) << 32) |
                                    (uint32_t)readlane((int)(uint32_t)cm, i);
                s = readlane(s2, i);
                mask = nm;
                start = 0;
                if (nt != t) {
                    t = nt;
                    if (t > tmax) tmax = t;
                    if (t == (uint32_t)n_ok) { verdict = JH_VALID; break; }
                    load_window(t);
                }
                // make the insert visible to this wave's next probes
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            } else {
                if (depth == 0) { verdict = JH_INVALID; break; }
                depth--;
                const Frame fr = stack[depth];
                const uint32_t pt = fr.t_i >> 6;
                mask = fr.mask; s = fr.s; start = (int)(fr.t_i & 63) + 1;
                if (pt != t) { t = pt; load_window(t); }
            }
            if (depth >= A.stack_cap) { verdict = JH_UNKNOWN; if (lane == 0) atomicOr(A.flags, 4); break; }
        }
        if (verdict == JH_UNKNOWN && A.defer && inserts >= A.budget) {
            if (lane == 0) {
                const int d = atomicAdd(A.defer_count, 1);
                A.defer_list[d] = key;
            }
            continue;
        }
        v.valid = verdict;
        v.cause = verdict == JH_UNKNOWN ? JH_CAUSE_BUDGET : 0;
        v.explored = inserts;
        if (verdict == JH_INVALID) v.fail_entry = ret_row(src, T, tmax, lane);
        if (lane == 0) A.out[key] = v;
    }
    for (int o = 32; o > 0; o >>= 1) my_probes += __shfl_xor(my_probes, o);
    if (lane == 0 && A.probes) atomicAdd(A.probes, my_probes);
}

// ---------------------------------------------------------------------------
// Heavy keys: parallel breadth-first enumeration of the reachable
// configuration graph by a whole workgroup. For a key with no terminal
// configuration (invalid) WGL's cache ends up holding exactly this set, so
// verdict, explored count and the furthest return rank (fail_entry) are
// identical to the sequential search. A key where a terminal configuration
// is reachable (valid) or the set outgrows the budget is handed to the
// sequential search (only it defines where :unknown starts for those).
constexpr int BFS_THREADS = 512;
constexpr int BFS_LDS_BYTES = 49152;
constexpr uint64_t BFS_EMPTY = ~0ULL;

struct BfsArgs {
    KeySrc src;
    const int32_t *list;
    int32_t n_list;
    int32_t *queue;
    jh_key_verdict *out;
    int32_t *unres_list;
    int32_t *unres_count;
    uint64_t *set;          // per workgroup: set_cap slots
    uint32_t set_cap;       // power of two
    uint64_t *q;            // per workgroup: 2 x q_cap configurations
    uint32_t q_cap;
    char *scratch;          // per workgroup table space
    uint64_t scratch_bytes;
    int64_t budget;
    int32_t init_state;
    int32_t states_ok;      // every interned state < 2^12
};

__device__ __forceinline__ uint64_t bfs_pack(uint32_t t, uint32_t s, uint32_t m) {
    return ((uint64_t)t << 44) | ((uint64_t)s << 32) | m;
}

__global__ void __launch_bounds__(BFS_THREADS) k_lin_bfs(BfsArgs A) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    __shared__ KeyTables sT;
    __shared__ jh_key_verdict sv;
    __shared__ int s_key, s_need, s_maxw, s_status;
    __shared__ unsigned s_ncur, s_nnext, s_tmax;
    __shared__ unsigned long long s_count;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint64_t *set = A.set + (size_t)blockIdx.x * A.set_cap;
    uint64_t *qa = A.q + (size_t)blockIdx.x * 2 * A.q_cap;
    char *gscr = A.scratch + (size_t)blockIdx.x * A.scratch_bytes;
    const uint32_t cmask = A.set_cap - 1;
    for (;;) {
        if (tid == 0) {
            const int idx = atomicAdd(A.queue, 1);
            s_key = idx < A.n_list ? A.list[idx] : -1;
        }
        __syncthreads();
        const int key = s_key;
        if (key < 0) break;
        if (wid == 0) {
            KeyTables T;
            jh_key_verdict v;
            const bool need = build_key_tables(A.src, key, lane, lds, BFS_LDS_BYTES, gscr,
                                               A.scratch_bytes, T, v);
            if (lane == 0) { sT = T; sv = v; s_need = need; s_maxw = 0; s_status = 0; }
        }
        __syncthreads();
        if (!s_need) {
            if (tid == 0) A.out[key] = sv;
            __syncthreads();
            continue;
        }
        const KeyTables T = sT;
        for (int t = tid; t < T.n_ok; t += BFS_THREADS) atomicMax(&s_maxw, T.woff[t + 1] - T.woff[t]);
        __syncthreads();
        if (s_maxw > 32 || !A.states_ok || T.n_ok >= (1 << 20) - 2) {
            if (tid == 0) A.unres_list[atomicAdd(A.unres_count, 1)] = key;
            __syncthreads();
            continue;
        }
        for (uint32_t i = tid; i < A.set_cap; i += BFS_THREADS) set[i] = BFS_EMPTY;
        if (tid == 0) {
            qa[0] = bfs_pack(0, (uint32_t)A.init_state, 0);
            s_ncur = 1; s_nnext = 0; s_tmax = 0; s_count = 0;
        }
        __syncthreads();
        uint64_t *cur = qa, *nxt = qa + A.q_cap;
        for (;;) {
            const unsigned ncur = s_ncur;
            for (unsigned i = tid; i < ncur; i += BFS_THREADS) {
                const uint64_t c = cur[i];
                const uint32_t t = (uint32_t)(c >> 44), s = (uint32_t)(c >> 32) & 0xFFF;
                const uint32_t mask = (uint32_t)c;
                const int wo = T.woff[t], w = T.woff[t + 1] - wo;
                for (int j = 0; j < w; j++) {
                    if ((mask >> j) & 1) continue;
                    const Op o = T.ops[T.W[wo + j]];
                    int s2;
                    if (!cas_step(o.fa & 3, o.v1, o.v2, (int)s, &s2)) continue;
                    uint32_t u = t, nm = mask | (1u << j);
                    if (o.rr == (int)t) {
                        const uint32_t lin = nm;
                        u = t + 1;
                        while (u < (uint32_t)T.n_ok) {
                            bool hit = false;
                            for (int m = 0; m < w && !hit; m++)
                                hit = ((lin >> m) & 1) && T.ops[T.W[wo + m]].rr == (int)u;
                            if (!hit) break;
                            u++;
                        }
                        nm = 0;
                        if (u < (uint32_t)T.n_ok) {
                            int b = 0;
                            for (int m = 0; m < w; m++) {
                                const int rr = T.ops[T.W[wo + m]].rr;
                                if (rr < 0 || rr >= (int)u) {
                                    if ((lin >> m) & 1) nm |= 1u << b;
                                    b++;
                                }
                            }
                        }
                    }
                    const uint64_t ck = bfs_pack(u, (uint32_t)s2, nm);
                    uint32_t h = (uint32_t)jh_mix64(ck) & cmask;
                    bool ins = false;
                    for (uint32_t probe = 0; probe <= cmask; probe++) {
                        const unsigned long long prev =
                            atomicCAS((unsigned long long *)&set[h], BFS_EMPTY, ck);
                        if (prev == BFS_EMPTY) { ins = true; break; }
                        if (prev == ck) break;
                        h = (h + 1) & cmask;
                    }
                    if (!ins) continue;
                    const unsigned long long n = atomicAdd(&s_count, 1ULL);
                    if ((long long)n >= A.budget) atomicOr(&s_status, 2);
                    if (u == (uint32_t)T.n_ok) atomicOr(&s_status, 1);
                    atomicMax(&s_tmax, u);
                    const unsigned pos = atomicAdd(&s_nnext, 1u);
                    if (pos < A.q_cap) nxt[pos] = ck; else atomicOr(&s_status, 2);
                }
            }
            __syncthreads();
            const int st = s_status;
            const unsigned nn = s_nnext;
            __syncthreads();
            if (st || nn == 0) break;
            if (tid == 0) { s_ncur = nn; s_nnext = 0; }
            uint64_t *tmp = cur; cur = nxt; nxt = tmp;
            __syncthreads();
        }
        if (s_status) {
            if (tid == 0) A.unres_list[atomicAdd(A.unres_count, 1)] = key;
        } else if (wid == 0) {
            jh_key_verdict v;
            v.valid = JH_INVALID; v.cause = 0; v.explored = (int64_t)s_count;
            v.fail_entry = ret_row(A.src, T, s_tmax, lane);
            if (lane == 0) A.out[key] = v;
        }
        __syncthreads();
    }
}

__global__ void k_summary(const jh_key_verdict *__restrict__ v, int64_t K, long long *sum) {
    // sum: [0] valid max [1] n_invalid [2] n_unknown [3] first_fail [4] n_keys [5] explored
    long long vmax = 0, ninv = 0, nunk = 0, ff = LLONG_MAX, nk = 0, ex = 0;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < K;
         k += (int64_t)gridDim.x * blockDim.x) {
        jh_key_verdict x = v[k];
        if (x.explored < 0) continue;
        nk++; ex += x.explored;
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

__global__ void k_iota(int32_t *a, int64_t n) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}

inline int bits_for(uint64_t x) {
    int b = 1;
    while ((1ULL << b) <= x) b++;
    return b;
}

}  // namespace

// ---------------------------------------------------------------------------
void lin_check_independent(jh_ctx *ctx, const jh_history *dh, const jh_lin_opts *opts,
                           bool keyed, jh_key_verdict *out_dev, jh_summary *sum,
                           hipStream_t st) {
    const int64_t n = dh->n;
    const int64_t K = keyed ? dh->n_keys : 1;
    if (K >= (1LL << 23)) throw_jh(JH_EUNSUPPORTED, "more than 2^23 keys in one call");
    if (n >= (1LL << 31)) throw_jh(JH_EUNSUPPORTED, "more than 2^31 entries in one call");
    const int64_t budget = opts && opts->budget > 0 ? opts->budget : JH_DEFAULT_BUDGET;
    const int64_t init = opts ? opts->init_value : JH_NIL;
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
    if ((unsigned long long)(vmax - vmin) >= (unsigned long long)(STATE_MASK - 2))
        throw_jh(JH_EUNSUPPORTED, "register values span more than 2^20 distinct states");
    const int init_state = init == JH_NIL ? 0 : (int)(init - vmin + 1);

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
        k_pair<<<grid_for(m, 256), 256, 0, st>>>(rec, kB, off, m, pair, viol);
        k_orphan<<<grid_for(m, 256), 256, 0, st>>>(rec, kB, m, pair, viol);
    }

    // memo generation tags: distinct per (call, key, pass); wrap -> clear
    const uint32_t gen_span = (uint32_t)(2 * K + 2);
    bool clear_memo = false;
    if ((uint64_t)ctx->gen_base + gen_span >= (1u << GEN_BITS) - 1) { ctx->gen_base = 0; clear_memo = true; }

    // phase 1: every key, quick budget, persistent grid
    const uint32_t memo_cap1 = 1u << 16;
    int64_t quick = std::min<int64_t>(budget, memo_cap1 / 4);
    if (const char *e = getenv("JH_QUICK_BUDGET")) quick = std::max<int64_t>(1, std::min<int64_t>(quick, atoll(e)));
    const int waves1 = (int)std::min<int64_t>(K, (int64_t)ctx->n_cu * 8);
    uint64_t *memo = ctx->ws<uint64_t>(WS_MEMO, (size_t)waves1 * memo_cap1 * 2, /*zero=*/true);
    if (clear_memo) HIP_TRY(hipMemsetAsync(memo, 0, ctx->bufs[WS_MEMO].bytes, st));
    const uint32_t stack_cap = (uint32_t)smax + 2;
    Frame *stack = ctx->ws<Frame>(WS_STACK, (size_t)waves1 * stack_cap);
    const uint64_t scr_bytes = (((uint64_t)smax * 84 + 4096) + 255) & ~255ULL;
    char *scr = ctx->ws<char>(WS_SCRATCH, (size_t)waves1 * scr_bytes);
    int32_t *q = ctx->ws<int32_t>(WS_QUEUE, 8);
    int32_t *list = ctx->ws<int32_t>(WS_STATS, K);
    int32_t *defer = ctx->ws<int32_t>(WS_DEFER, K + 1);
    unsigned long long *probes = (unsigned long long *)(q + 4);
    HIP_TRY(hipMemsetAsync(q, 0, 8 * sizeof(int32_t), st));
    k_iota<<<grid_for(K, 256), 256, 0, st>>>(list, K);

    DfsArgs a{};
    a.rec = rec; a.pair = pair; a.off = off; a.rows = rB; a.viol = viol; a.rank = rank;
    a.list = list; a.n_list = (int32_t)K; a.queue = q; a.out = out_dev;
    a.defer_list = defer; a.defer_count = q + 1;
    a.memo = memo; a.memo_cap = memo_cap1; a.stack = stack; a.stack_cap = stack_cap;
    a.scratch = scr; a.scratch_bytes = scr_bytes; a.budget = quick; a.defer = quick < budget ? 1 : 0;
    a.init_state = init_state; a.gen_base = ctx->gen_base; a.flags = q + 2; a.probes = probes;
    HIP_TRY(hipEventRecord(ctx->ev[1], st));
    k_lin_dfs<<<waves1, 64, LDS_BYTES, st>>>(a);
    HIP_TRY(hipGetLastError());
    int32_t qh[8];
    HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int n_defer = qh[1];
    HIP_TRY(hipEventRecord(ctx->ev[4], st));
    int n_unres = 0;
    if (n_defer > 0) {
        // phase 2: heavy keys, one workgroup each, parallel reachable-set BFS
        uint32_t set_cap = 1u << 12;
        while ((int64_t)set_cap < 2 * budget && set_cap < (1u << 30)) set_cap <<= 1;
        const uint32_t q_cap = (uint32_t)std::min<int64_t>(budget + 64, (int64_t)1 << 30);
        const int wg2 = std::min(n_defer, 128);
        uint64_t *bset = ctx->ws<uint64_t>(WS_BFS_SET, (size_t)wg2 * set_cap);
        uint64_t *bq = ctx->ws<uint64_t>(WS_BFS_Q, (size_t)wg2 * 2 * q_cap);
        char *bscr = ctx->ws<char>(WS_SCRATCH_DEEP, (size_t)wg2 * scr_bytes);
        int32_t *unres = ctx->ws<int32_t>(WS_BFS_META, n_defer + 1);
        HIP_TRY(hipMemsetAsync(q, 0, sizeof(int32_t), st));
        HIP_TRY(hipMemsetAsync(q + 3, 0, sizeof(int32_t), st));
        BfsArgs c{};
        c.src = KeySrc{rec, pair, off, rB, viol, rank, q + 2};
        c.list = defer; c.n_list = n_defer; c.queue = q; c.out = out_dev;
        c.unres_list = unres; c.unres_count = q + 3;
        c.set = bset; c.set_cap = set_cap; c.q = bq; c.q_cap = q_cap;
        c.scratch = bscr; c.scratch_bytes = scr_bytes; c.budget = budget;
        c.init_state = init_state; c.states_ok = (vmax - vmin + 2) < 4096 ? 1 : 0;
        k_lin_bfs<<<wg2, BFS_THREADS, BFS_LDS_BYTES, st>>>(c);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n_unres = qh[3];
    }
    HIP_TRY(hipEventRecord(ctx->ev[5], st));
    if (n_unres > 0) {
        // phase 3: keys BFS could not settle (a terminal configuration is
        // reachable, or the set outgrew the budget): the sequential search
        // with the full budget defines their verdict and explored count
        uint32_t cap2 = 1u << 16;
        while ((int64_t)cap2 < 2 * budget && cap2 < (1u << 30)) cap2 <<= 1;
        const int waves2 = std::min(n_unres, 64);
        uint64_t *memo2 = ctx->ws<uint64_t>(WS_MEMO_DEEP, (size_t)waves2 * cap2 * 2);
        Frame *stack2 = ctx->ws<Frame>(WS_STACK_DEEP, (size_t)waves2 * stack_cap);
        char *scr2 = ctx->ws<char>(WS_SCRATCH_DEEP, (size_t)std::max(waves2, 1) * scr_bytes);
        HIP_TRY(hipMemsetAsync(memo2, 0, (size_t)waves2 * cap2 * 16, st));
        HIP_TRY(hipMemsetAsync(q, 0, sizeof(int32_t), st));
        DfsArgs b = a;
        b.list = ctx->ws<int32_t>(WS_BFS_META, 1); b.n_list = n_unres; b.memo = memo2; b.memo_cap = cap2;
        b.stack = stack2; b.scratch = scr2; b.budget = budget; b.defer = 0;
        b.gen_base = ctx->gen_base + (uint32_t)K + 1;
        k_lin_dfs<<<waves2, 64, LDS_BYTES, st>>>(b);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(ctx->ev[2], st));
    ctx->gen_base += gen_span;

    long long *sd = ctx->ws<long long>(WS_SUMMARY, 8);
    long long s_init[8] = {0, 0, 0, LLONG_MAX, 0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(sd, s_init, sizeof s_init, hipMemcpyHostToDevice, st));
    k_summary<<<grid_for(K, 256, 1024), 256, 0, st>>>(out_dev, K, sd);
    long long sh[8];
    HIP_TRY(hipMemcpyAsync(sh, sd, sizeof sh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(qh, q, sizeof qh, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ctx->ev[3], st));
    HIP_TRY(hipStreamSynchronize(st));
    if (qh[2] & 1) throw_jh(JH_EUNSUPPORTED, "a key with more than 65535 ops or 2^20 ok returns");
    if (qh[2] & 2) throw_jh(JH_EDEVICE, "per-key table exceeded the scratch reservation");
    if (qh[2] & 4) throw_jh(JH_EDEVICE, "DFS stack overflow");
    if (sum) {
        sum->valid = sh[0]; sum->n_invalid = sh[1]; sum->n_unknown = sh[2];
        sum->first_fail_entry = sh[3] == LLONG_MAX ? -1 : sh[3];
        sum->n_keys = sh[4]; sum->explored = sh[5];
        sum->memo_probes = (int64_t)(((uint64_t)(uint32_t)qh[5] << 32) | (uint32_t)qh[4]);
        float ms = 0, ms_dfs = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[3]));
        HIP_TRY(hipEventElapsedTime(&ms_dfs, ctx->ev[1], ctx->ev[2]));
        sum->device_ms = ms; sum->dfs_ms = ms_dfs;
        if (getenv("JH_DEBUG")) {
            float a = 0, b = 0, c = 0;
            HIP_TRY(hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]));
            HIP_TRY(hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[4]));
            HIP_TRY(hipEventElapsedTime(&c, ctx->ev[4], ctx->ev[2]));
            float d = 0;
            HIP_TRY(hipEventElapsedTime(&d, ctx->ev[5], ctx->ev[2]));
            HIP_TRY(hipEventElapsedTime(&c, ctx->ev[4], ctx->ev[5]));
            fprintf(stderr, "[jh] keys=%lld prep=%.3f ms phase1=%.3f ms (waves %d) deferred=%d bfs=%.3f ms unresolved=%d deep=%.3f ms\n",
                    (long long)K, a, b, waves1, n_defer, c, n_unres, d);
        }
    }
}
