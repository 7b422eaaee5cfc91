// jh_ingest.hip -- host-buffer histories into HBM (the boundary's host entry
// points: jh_check_cas_independent, jh_check_counter, ... with on_device = 0).
//
// A host history is int64 columns (include/jh.h); most hold small numbers
// (types and :f codes, process ids, keys, register values), so a large one
// crosses PCIe packed: in chunks of ING_CHUNK rows, a column is narrowed to
// 1 byte (type, f) or 4 bytes (the others; nil <-> INT32_MIN) when every
// value of the chunk fits, else sent whole. A pool of host threads packs
// chunk c + 1 into one pinned buffer while chunk c's DMA and the kernel that
// widens it back to int64 (k_widen_cols) run from the other, all on the
// context's stream: the pipeline after it reads the same int64 columns in HBM
// as before. The C3 history (9.49 M rows, six columns): 455 MB -> 171 MB.
// Histories under ING_MIN rows (and, in -DJH_TUNING builds, every call when
// JH_INGEST_PLAIN=1 is set: the A/B) take one plain hipMemcpyAsync per column.
#include "jh_internal.h"
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <chrono>
#include <memory>

namespace {

constexpr int64_t ING_CHUNK = 1 << 20;       // rows per chunk
constexpr int64_t ING_MIN = 1 << 21;         // smaller histories: plain copies
constexpr int ING_COLS = 7;                  // process type f key value value2 aux
constexpr int ING_MAX_THREADS = 16;          // the GPU box's CPU share

// a fixed pool of packing threads (run(f) calls f(i) on each, then returns)
struct Pool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done;
    std::function<void(int)> job;
    int gen = 0, pending = 0, n = 0;
    bool stop = false;
    explicit Pool(int k) : n(k) {
        for (int i = 0; i < k; i++) th.emplace_back([this, i] { loop(i); });
    }
    void loop(int i) {
        int seen = 0;
        for (;;) {
            std::function<void(int)> j;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                j = job;
            }
            j(i);
            std::lock_guard<std::mutex> lk(m);
            if (--pending == 0) done.notify_all();
        }
    }
    std::mutex serial;              // one job at a time: contexts share the pool (jh_open_multi's threads)
    void run(const std::function<void(int)> &f) {
        std::lock_guard<std::mutex> one(serial);
        {
            std::lock_guard<std::mutex> lk(m);
            job = f;
            pending = n;
            gen++;
        }
        cv.notify_all();
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return pending == 0; });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
};

// per column of a chunk: its bytes per row in the packed buffer (1, 4 or 8;
// 0: the column is absent)
struct WidenArgs {
    const char *src[ING_COLS];
    int64_t *dst[ING_COLS];
    int width[ING_COLS];
    int64_t n;
};

__global__ void __launch_bounds__(256) k_widen_cols(WidenArgs A) {
    const int c = blockIdx.y;
    const int w = A.width[c];
    if (w == 0) return;
    const int64_t n = A.n;
    int64_t *__restrict__ d = A.dst[c];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < n; i0 += stride) {
        long long v[4];
        if (w == 1) {
            const int8_t *s = (const int8_t *)A.src[c];
            if (i0 + 4 <= n) {
                const char4 x = *(const char4 *)(s + i0);
                v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
            } else
                for (int k = 0; k < 4; k++) v[k] = i0 + k < n ? s[i0 + k] : 0;
        } else if (w == 4) {
            const int32_t *s = (const int32_t *)A.src[c];
            int32_t x[4];
            if (i0 + 4 <= n) {
                const int4 y = *(const int4 *)(s + i0);
                x[0] = y.x; x[1] = y.y; x[2] = y.z; x[3] = y.w;
            } else
                for (int k = 0; k < 4; k++) x[k] = i0 + k < n ? s[i0 + k] : 0;
            for (int k = 0; k < 4; k++) v[k] = x[k] == INT32_MIN ? (long long)JH_NIL : (long long)x[k];
        } else {
            const int64_t *s = (const int64_t *)A.src[c];
            for (int k = 0; k < 4; k++) v[k] = i0 + k < n ? s[i0 + k] : 0;
        }
        if (i0 + 4 <= n) {
            *(longlong2 *)(d + i0) = make_longlong2(v[0], v[1]);
            *(longlong2 *)(d + i0 + 2) = make_longlong2(v[2], v[3]);
        } else
            for (int k = 0; k < 4 && i0 + k < n; k++) d[i0 + k] = v[k];
    }
}

// Round 6: ONE packing pool per process, shared by every
// context (a JVM may open many), created on first use and kept to the end.
Pool &packing_pool() {
    static Pool *p = new Pool((int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()),
                                                      ING_MAX_THREADS));
    return *p;
}

}  // namespace

// Per context: two pinned chunk buffers and their device twins (7 columns x
// ING_CHUNK rows x 8 B = 56 MB each, 112 MB pinned host + 112 MB HBM), made on
// the first packed call; INTEGRATION.md lists them.
struct Ingest {
    void *pin[2] = {nullptr, nullptr};      // packed chunk, host side (pinned)
    void *dev[2] = {nullptr, nullptr};      // packed chunk, device side
    hipEvent_t ev[2] = {nullptr, nullptr};  // chunk's DMA out of pin[b] done
    bool rec[2] = {false, false};           // ev[b] recorded (by this call or an earlier one)
    ~Ingest() {
        for (int b = 0; b < 2; b++) {
            if (pin[b]) (void)hipHostFree(pin[b]);
            if (dev[b]) (void)hipFree(dev[b]);
            if (ev[b]) (void)hipEventDestroy(ev[b]);
        }
    }
};

void ingest_free(Ingest *g) { delete g; }

static bool ingest_plain() {
#ifdef JH_TUNING
    static const bool plain = [] {
        const char *e = getenv("JH_INGEST_PLAIN");
        return e && atoi(e) != 0;
    }();
    return plain;
#else
    return false;
#endif
}

// Stages the given host columns (null: absent) into the device columns dst
// (each n int64). Returns false when the history is too small for packing
// (the caller copies plainly).
bool ingest_columns(jh_ctx *ctx, const int64_t *const src[ING_COLS], int64_t *const dst[ING_COLS], int64_t n,
                    hipStream_t st) {
    if (n < ING_MIN || ingest_plain()) return false;
    const size_t region = (size_t)ING_CHUNK * 8;              // one column's room in a chunk buffer
    if (!ctx->ingest) {
        // every buffer first, then the context's: a failed allocation leaves
        // nothing half made -- the Ingest destructor frees what was
        std::unique_ptr<Ingest> fresh(new Ingest());
        for (int b = 0; b < 2; b++) {
            HIP_TRY(hipHostMalloc(&fresh->pin[b], region * ING_COLS, hipHostMallocNonCoherent));   // CPU-cached: the packers write it byte by byte
            HIP_TRY(hipMalloc(&fresh->dev[b], region * ING_COLS));
            HIP_TRY(hipEventCreateWithFlags(&fresh->ev[b], hipEventDisableTiming));
        }
        ctx->ingest = fresh.release();
    }
    Ingest &g = *ctx->ingest;
    Pool &pool = packing_pool();
    const int nt = pool.n;
    const int64_t n_chunks = (n + ING_CHUNK - 1) / ING_CHUNK;
#ifdef JH_TUNING
    // JH_INGEST_TRACE=1: where the host time goes (event waits, packing, enqueue)
    static const bool trace = getenv("JH_INGEST_TRACE") && atoi(getenv("JH_INGEST_TRACE"));
    double t_wait = 0, t_pack = 0, t_enq = 0;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_all = now();
#define ING_T(acc, stmt) do { const double t0_ = trace ? now() : 0; stmt; if (trace) acc += now() - t0_; } while (0)
#else
#define ING_T(acc, stmt) do { stmt; } while (0)
#endif
    for (int64_t ch = 0; ch < n_chunks; ch++) {
        const int b = (int)(ch & 1);
        const int64_t r0 = ch * ING_CHUNK, cn = std::min<int64_t>(ING_CHUNK, n - r0);
        // the DMA that last read pin[b] (chunk ch - 2) has finished
        if (g.rec[b]) ING_T(t_wait, HIP_TRY(hipEventSynchronize(g.ev[b])));
        char *pb = (char *)g.pin[b];
        std::atomic<int> wide[ING_COLS];
        for (auto &x : wide) x.store(0, std::memory_order_relaxed);
        // narrow every column of the chunk; a value that does not fit marks
        // the column wide (then it is copied whole, below)
        ING_T(t_pack, pool.run([&](int i) {
            const int64_t a = cn * i / nt, e = cn * (i + 1) / nt;
            for (int c = 0; c < ING_COLS; c++) {
                if (!src[c]) continue;
                const int64_t *s = src[c] + r0;
                bool bad = false;
                if (c == 1 || c == 2) {                         // type, f: 1 byte
                    int8_t *d = (int8_t *)(pb + region * c);
                    for (int64_t r = a; r < e; r++) {
                        const int64_t v = s[r];
                        bad |= v < -128 || v > 127;
                        d[r] = (int8_t)v;
                    }
                } else {                                        // 4 bytes, nil <-> INT32_MIN
                    int32_t *d = (int32_t *)(pb + region * c);
                    for (int64_t r = a; r < e; r++) {
                        const int64_t v = s[r];
                        const bool nil = v == JH_NIL;
                        bad |= !nil && (v <= INT32_MIN || v > INT32_MAX);
                        d[r] = nil ? INT32_MIN : (int32_t)v;
                    }
                }
                if (bad) wide[c].store(1, std::memory_order_relaxed);
            }
        }));
        // a column some value of the chunk did not fit: copied whole
        WidenArgs wa{};
        wa.n = cn;
        bool any_wide = false;
        for (int c = 0; c < ING_COLS; c++) any_wide |= src[c] && wide[c].load();
        if (any_wide)
            pool.run([&](int i) {
                const int64_t a = cn * i / nt, e = cn * (i + 1) / nt;
                for (int c = 0; c < ING_COLS; c++)
                    if (src[c] && wide[c].load(std::memory_order_relaxed))
                        memcpy(pb + region * c + a * 8, src[c] + r0 + a, (size_t)(e - a) * 8);
            });
        for (int c = 0; c < ING_COLS; c++) {
            if (!src[c]) continue;
            const int w = wide[c].load() ? 8 : (c == 1 || c == 2) ? 1 : 4;
            char *dv = (char *)g.dev[b] + region * c;
            HIP_TRY(hipMemcpyAsync(dv, pb + region * c, (size_t)cn * w, hipMemcpyHostToDevice, st));
            wa.src[c] = dv;
            wa.dst[c] = dst[c] + r0;
            wa.width[c] = w;
        }
        HIP_TRY(hipEventRecord(g.ev[b], st));
        g.rec[b] = true;
        const unsigned gx = (unsigned)std::min<int64_t>((cn + 1023) / 1024, 1024);
        k_widen_cols<<<dim3(gx, ING_COLS), 256, 0, st>>>(wa);
        HIP_TRY(hipGetLastError());
    }
#ifdef JH_TUNING
    if (trace)
        fprintf(stderr, "[jh-ingest] %lld rows, %lld chunks, %d threads: %.2f ms (event waits %.2f, packing %.2f)\n",
                (long long)n, (long long)n_chunks, nt, now() - t_all, t_wait, t_pack);
    (void)t_enq;
#endif
#undef ING_T
    return true;
}
