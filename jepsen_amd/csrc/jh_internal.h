// jh_internal.h -- shared internals of libjh.so (HIP, gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>
#include <string>
#include "../../include/jh.h"

#define JH_WAVE 64

// ---------------------------------------------------------------------------
// error plumbing: every entry point returns a JH_* code and fills err.
struct JhError {
    int code = JH_OK;
    std::string msg;
};

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess) {                                                       \
            throw_hip(_e, #expr, __FILE__, __LINE__);                                 \
        }                                                                             \
    } while (0)

struct JhException {
    int code;
    std::string msg;
};

[[noreturn]] inline void throw_hip(hipError_t e, const char *expr, const char *file, int line) {
    char buf[512];
    snprintf(buf, sizeof buf, "HIP error %s (%d) at %s:%d: %s", hipGetErrorString(e), (int)e,
             file, line, expr);
    throw JhException{e == hipErrorOutOfMemory ? JH_ENOMEM : JH_EDEVICE, buf};
}
[[noreturn]] inline void throw_jh(int code, const std::string &msg) { throw JhException{code, msg}; }

// ---------------------------------------------------------------------------
// Device workspace: named, grow-only buffers owned by the context. Entry
// points never allocate in the steady state (same-size calls reuse).
struct Buf {
    void *p = nullptr;
    size_t bytes = 0;
};

struct jh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t aux = nullptr;     // second stream for racing searches (jh_lin.hip)
    hipStream_t aux2 = nullptr;    // third stream: windows wider than 64 (jh_lin.hip)
    hipStream_t aux3 = nullptr;    // fourth stream: phase-2 late helpers (jh_lin.hip)
    std::mutex mu;
    std::vector<Buf> bufs;
    hipEvent_t ev[24] = {};
    uint32_t gen_base = 0;        // memo generation tags (see jh_lin.hip)
    bool lds_attr = false;        // >64 KB dynamic-LDS attributes set for this device's kernels
    bool lds_attr_wg = false;
    int n_cu = 256;
    int share = 1;                // contexts of one jh_open_devices call on this device (fit_units divides by it)
    size_t hbm_total = 0;         // the device's HBM (hipMemGetInfo, once): bounds the resume buffers
    int32_t *hflag = nullptr;     // host-mapped flag: phase 1's queue drained (jh_lin.hip)
    int32_t *hflag_dev = nullptr;
    void *pinned = nullptr;       // small pinned staging for scalars
    size_t pinned_bytes = 0;
    std::vector<jh_ctx *> members;  // jh_open_multi: one context per device (jh_multi.hip); empty otherwise
    struct Ingest *ingest = nullptr;  // host-buffer staging: packing threads, pinned chunks (jh_ingest.hip)

    template <class T>
    T *ws(int slot, size_t count, bool zero = false) {
        if ((int)bufs.size() <= slot) bufs.resize(slot + 1);
        size_t need = count * sizeof(T);
        if (need == 0) need = 16;
        Buf &b = bufs[slot];
        if (b.bytes < need) {
            if (b.p) HIP_TRY(hipFree(b.p));
            b.p = nullptr;
            size_t alloc = need + need / 8;
            HIP_TRY(hipMalloc(&b.p, alloc));
            b.bytes = alloc;
            if (zero) {
                HIP_TRY(hipMemsetAsync(b.p, 0, alloc, stream));
                HIP_TRY(hipStreamSynchronize(stream));   // callers may run on another stream
            }
        }
        return (T *)b.p;
    }
    bool ws_fresh(int slot) const { return (int)bufs.size() <= slot || bufs[slot].p == nullptr; }
};

// Round 6: contexts open on each device in this process (jh_open / jh_close):
// fit_units and the resume buffers divide a device by max(share, this), so a
// second context opened with its own jh_open does not size its tables as if
// it had the device to itself
int device_open_contexts(int device);

// workspace slot ids (one namespace for the whole library)
enum WsSlot {
    WS_COL_PROCESS = 0, WS_COL_TYPE, WS_COL_F, WS_COL_KEY, WS_COL_VALUE, WS_COL_VALUE2, WS_COL_AUX,
    WS_KEYS_A, WS_KEYS_B, WS_ROWS_A, WS_ROWS_B, WS_SORT_TMP, WS_SEG_OFF, WS_REC, WS_PAIR,
    WS_VIOL, WS_RANK, WS_MISC, WS_VERDICT, WS_QUEUE, WS_DEFER, WS_MEMO, WS_STACK, WS_SCRATCH,
    WS_MEMO_DEEP, WS_STACK_DEEP, WS_SCRATCH_DEEP, WS_SUMMARY, WS_STATS,
    WS_C_PAIR, WS_C_LAST, WS_C_LO, WS_C_HI, WS_C_OUT, WS_C_FLAG, WS_C_TMP, WS_C_IDX,
    WS_S_BITS, WS_S_RUNS, WS_S_TMP, WS_S_CNT,
    WS_BFS_SET, WS_BFS_Q, WS_BFS_META, WS_CLAIM, WS_SCRATCH_BFS, WS_DEBUG, WS_META, WS_ARENA, WS_DEFER_PROG, WS_LIST_W, WS_C_PT,
    WS_DEFER3, WS_MEMO_P3, WS_STACK_P3, WS_SCRATCH_P3,
    WS_LIST_X, WS_MEMO_X, WS_STACK_X, WS_SCRATCH_X, WS_C_OUT2, WS_C_TAB, WS_S_CODE,
    WS_SF_META, WS_SF_FLAG, WS_SF_LUT, WS_SF_TMP, WS_SF_ELEM, WS_SF_STATE, WS_SF_RFLAG, WS_SF_READS,
    WS_SF_BITS, WS_SF_OUT, WS_SF_FL, WS_SF_SEL, WS_SF_TIME, WS_SF_PART,
    WS_Q_META, WS_Q_PART, WS_Q_HIST, WS_Q_FLAG, WS_Q_ROWS, WS_Q_TMP, WS_Q_MULT, WS_Q_MFLAG, WS_Q_POS,
    WS_Q_OUT, WS_Q_KEYS, WS_Q_MULT2, WS_LCOST, WS_LSORT, WS_LTMP, WS_ACC_STATS, WS_WG_GSET, WS_WG_WORK, WS_WG_WTAB, WS_WG_PEND, WS_STATS_KEYS,
    WS_BFS_NODES, WS_BFS_LSTART, WS_BFS_HKEY, WS_BFS_HID, WS_BFS_LIVE, WS_BFS_VIS, WS_BFS_TMP,
    WS_WG_MEMO, WS_WG_STACK, WS_WG_SCR, WS_S_BYTES, WS_IV_U, WS_IV_IDX, WS_IV_KEY, WS_IV_RINIT, WS_IV_MAX, WS_IV_TMP,
    WS_HELP_START, WS_HELP_TAKEN, WS_DEFER_TIME, WS_BFS_TMPK,
    WS_DEFER64, WS_DEFER64_T, WS_MEMO_WIDE, WS_STACK_WIDE, WS_SCRATCH_WIDE,
    WS_CFG_SLOT, WS_CFG_OUT, WS_CFG_N, WS_CFG_ROWS, WS_CFG_KEYS,
    WS_S_RB_HIST, WS_S_RB_OUT, WS_TL, WS_RS_ARENA, WS_RS_OFF, WS_RS_LOG, WS_DEFER_INFO,
    WS_SPEC, WS_SPEC_RES, WS_DEBUG_WG, WS_HANDOFF, WS_RS_LOG2,
    WS_COUNT
};

// row-level helpers shared by kernels
__device__ __forceinline__ uint64_t jh_mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

// Block-wide reduction for 256-thread blocks (4 waves): one value per block,
// so a reduction kernel issues one global atomic per block, not per wave
// (per-wave atomics on a few addresses serialise in L2).
template <class T, class Op>
__device__ __forceinline__ T block_reduce256(T v, Op op, T *sh /* [4] shared */) {
    for (int o = 32; o > 0; o >>= 1) v = op(v, (T)__shfl_xor(v, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return op(op(sh[0], sh[1]), op(sh[2], sh[3]));
}
struct RedMin { template <class T> __device__ T operator()(T a, T b) const { return a < b ? a : b; } };
struct RedMax { template <class T> __device__ T operator()(T a, T b) const { return a > b ? a : b; } };
struct RedSum { template <class T> __device__ T operator()(T a, T b) const { return a + b; } };
struct RedOr { template <class T> __device__ T operator()(T a, T b) const { return a | b; } };

inline int grid_for(int64_t n, int block, int cap = 65536) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// Copies a host jh_history to device workspace columns (or passes device
// pointers through). Returns a device-pointer view.
jh_history stage_history(jh_ctx *ctx, const jh_history *h, bool need_key, bool need_aux);
// jh_ingest.hip: packed, pipelined staging of large host histories (false: too small)
bool ingest_columns(jh_ctx *ctx, const int64_t *const src[7], int64_t *const dst[7], int64_t n, hipStream_t st);
void ingest_free(struct Ingest *g);

// linearizability (jh_lin.hip). cfg: a jh_lin_configs request (the frontier
// configurations of the listed keys, device buffers; null for a check)
struct LinCfgReq {
    const int64_t *keys_dev;      // n_q requested keys
    int32_t n_q, per_key;
    const int32_t *slot_dev;      // per key: its index in keys_dev, or -1
    jh_lin_config *out_dev;       // n_q * per_key
    int32_t *n_dev;               // n_q, -1 on entry
    int64_t *rows_dev;            // n_q * per_key * 64
};
void lin_check_independent(jh_ctx *ctx, const jh_history *dh, const jh_lin_opts *opts,
                           bool keyed, jh_key_verdict *out_dev, jh_summary *sum,
                           hipStream_t stream, const LinCfgReq *cfg = nullptr);
// per-key row CSR of an independent history (jh_lin.hip)
void key_index(jh_ctx *ctx, const jh_history *dh, int64_t *key_off, int64_t *rows, hipStream_t stream);
// counter (jh_counter.hip)
void counter_check(jh_ctx *ctx, const jh_history *dh, int64_t *reads_out, int64_t reads_cap,
                   int64_t *n_reads, int64_t *n_errors, int64_t *first_err, int32_t *valid,
                   int32_t *cause, hipStream_t stream);
// set (jh_set.hip)
void set_check(jh_ctx *ctx, const jh_history *dh, jh_set_result *res, int64_t *runs[4],
               int64_t runs_cap, hipStream_t stream);
void set_check_bitmaps(jh_ctx *ctx, const jh_history *dh, jh_set_result *res, uint32_t *bits_out[4],
                       int64_t words_cap, int64_t *base, int64_t *n_words, hipStream_t stream);
// set-full (jh_setfull.hip); lists_out = {lost, never-read, stale}
void set_full_check(jh_ctx *ctx, const jh_history *dh, const int64_t *time_dev, bool linearizable, int64_t read_batch,
                    jh_set_full_result *res, int64_t *lists_out[3], int64_t list_cap, hipStream_t stream);
// queues (jh_queue.hip); outs = {lost, unexpected, duplicated, recovered}
void total_queue_check(jh_ctx *ctx, const jh_history *dh, jh_queue_result *res, int64_t *outs[4],
                       int64_t cap, hipStream_t stream);
void queue_check(jh_ctx *ctx, const jh_history *dh, jh_queue_result *res, int64_t *final_out, int64_t cap,
                 hipStream_t stream);
