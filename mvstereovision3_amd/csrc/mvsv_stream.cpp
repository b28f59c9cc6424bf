// mvsv_stream.cpp — double-buffered frame stream for a camera loop.
//
// Replaces the reference's worker-thread pattern (trgt/mean_test.cpp:61-70: one
// thread waits on a condition variable, runs Disparity::sgbm on the shared
// Stereopair, flags newDisparityMap; the main loop then runs
// MeanDisparityDetection::build on an ROI of the map, :258-318).  Here every
// pushed frame owns a slot (pinned host staging + device buffers + events); the
// upload of frame i+1 (copy stream), the compute of frame i (context stream:
// SGBM + the 9x9 mean grid of the ROI) and the download of frame i-1 (second
// copy stream) overlap, and frames come back in push order.
// With mvsv_stream_set_batch(b), pushed frames are computed b at a time: the
// slots' device buffers are one contiguous [depth][frame] array, so a group of
// consecutive slots is one frame-batch launch (sustained rate of the batch
// kernels instead of the single-frame ones, at b frames of extra latency);
// pop and set_params launch a partial group when they need to.
// With mvsv_stream_set_inflight(n), consecutive launches go round-robin to n
// compute lanes: the caller's context and n-1 contexts the stream owns (each
// its own HIP stream and scratch buffers), so up to n frame-batch launches run
// concurrently and one fills the chip's gaps left by another's
// latency-bound kernels.
// The host copies of a frame (caller rows -> pinned slot on push, pinned map ->
// caller rows on pop) are split over a small pool of copy threads that the
// stream owns (MVSV_STREAM_COPY_THREADS, default 4 including the caller), so a
// host whose single-core memcpy is slow still feeds the GPU at its rate.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "mvsv_internal.hpp"
#include "mvsv_ring.hpp"

using namespace mvsv;

static constexpr int kStreamMaxInflight = 4;
static constexpr size_t kPoolMinBytes = (size_t)1 << 20;  // smaller copies stay on the caller's thread

// Persistent row-copy pool: run(fn) calls fn(p, parts) once for every part
// p < parts = size(), the calling thread taking parts too, and returns when
// every worker has checked out of the run (so none touches fn or the part
// counter after run returns).
class CopyPool {
  public:
    // A worker that cannot be created (std::system_error, bad_alloc) leaves the
    // pool with the workers made so far: nothing escapes into the C ABI.
    explicit CopyPool(int threads)
    {
        try {
            workers_.reserve((size_t)std::max(threads - 1, 0));
            for (int i = 1; i < threads; i++) workers_.emplace_back([this] { loop(); });
        } catch (...) {
        }
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return (int)workers_.size() + 1; }
    void run(const std::function<void(int, int)>& fn)
    {
        const int parts = size();
        if (parts == 1) {
            fn(0, 1);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            next_.store(0, std::memory_order_relaxed);
            active_ = parts - 1;
            gen_++;
        }
        cv_.notify_all();
        for (int p; (p = next_.fetch_add(1, std::memory_order_relaxed)) < parts;) fn(p, parts);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return active_ == 0; });
        fn_ = nullptr;
    }

  private:
    void loop()
    {
        long seen = 0;
        for (;;) {
            const std::function<void(int, int)>* fn;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
            }
            const int parts = size();
            for (int p; (p = next_.fetch_add(1, std::memory_order_relaxed)) < parts;) (*fn)(p, parts);
            std::lock_guard<std::mutex> g(m_);
            if (--active_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int, int)>* fn_ = nullptr;
    std::atomic<int> next_{0};
    int active_ = 0;
    long gen_ = 0;
    bool stop_ = false;
};

// rows [0, H) of W-byte rows: src (stride ss) -> dst (stride ds), split by part
static void copy_rows(uint8_t* dst, size_t ds, const uint8_t* src, size_t ss, size_t W, int H, int part,
                      int parts)
{
    const int y0 = (int)((long)H * part / parts), y1 = (int)((long)H * (part + 1) / parts);
    if (ds == W && ss == W) {
        std::memcpy(dst + (size_t)y0 * W, src + (size_t)y0 * W, (size_t)(y1 - y0) * W);
        return;
    }
    for (int y = y0; y < y1; y++) std::memcpy(dst + (size_t)y * ds, src + (size_t)y * ss, W);
}

struct mvsv_stream {
    mvsv_ctx* ctx = nullptr;
    std::vector<mvsv_ctx*> lanes;  // [0] = ctx; the rest are owned by the stream
    long runs = 0;                 // launches enqueued (lane = runs % lanes)
    int W = 0, H = 0;
    mvsv_sgbm_params params{};
    SgbmEff eff{};
    bool grid = false;
    mvsv_rect roi{};
    hipStream_t up = nullptr, down = nullptr;
    struct Slot {
        uint8_t *hL = nullptr, *hR = nullptr;  // pinned
        int16_t* hOut = nullptr;
        float* hMeans = nullptr;
        uint8_t *dL = nullptr, *dR = nullptr;
        int16_t* dOut = nullptr;
        float* dMeans = nullptr;
        hipEvent_t uploaded = nullptr, computed = nullptr, done = nullptr;
        int status = MVSV_OK;
        int run_len = 0;     // > 0: this slot starts a frame-batch launch of run_len slots
        bool gave_up = false;  // the launch of this frame gave up a strip wait
    };
    std::vector<Slot> slots;
    uint8_t *dL_all = nullptr, *dR_all = nullptr;  // [depth][H][W]
    int16_t* dOut_all = nullptr;
    float* dMeans_all = nullptr;  // [depth][81]
    // per-slot report words (host-mapped): a launch starting at slot i reports
    // a given-up strip wait into rep[i], read when slot i is popped
    int* rep = nullptr;
    int* rep_dev = nullptr;
    long head = 0, tail = 0;      // pushed / popped frame counters
    long launched = 0;            // frames whose compute is enqueued
    int batch = 1;
    CopyPool* pool = nullptr;     // host copies of push / pop (nullptr: caller's thread only)
};

static void stream_free(mvsv_stream* st)
{
    for (size_t i = 1; i < st->lanes.size(); i++) mvsv_destroy(st->lanes[i]);
    for (auto& s : st->slots) {
        if (s.hL) (void)hipHostFree(s.hL);
        if (s.hR) (void)hipHostFree(s.hR);
        if (s.hOut) (void)hipHostFree(s.hOut);
        if (s.hMeans) (void)hipHostFree(s.hMeans);
        for (hipEvent_t e : {s.uploaded, s.computed, s.done})
            if (e) (void)hipEventDestroy(e);
    }
    if (st->dL_all) (void)hipFree(st->dL_all);
    if (st->dR_all) (void)hipFree(st->dR_all);
    if (st->dOut_all) (void)hipFree(st->dOut_all);
    if (st->dMeans_all) (void)hipFree(st->dMeans_all);
    if (st->rep) (void)hipHostFree(st->rep);
    if (st->up) (void)hipStreamDestroy(st->up);
    if (st->down) (void)hipStreamDestroy(st->down);
    delete st->pool;
    delete st;
}

int mvsv_stream_create(mvsv_ctx* ctx, int W, int H, const mvsv_sgbm_params* p, int depth,
                       const mvsv_rect* grid_roi, mvsv_stream** out)
{
    if (!ctx || !out) return MVSV_E_INVALID_ARG;
    *out = nullptr;
    if (depth < 1 || depth > 64) return set_error(ctx, MVSV_E_INVALID_ARG, "stream depth must be 1..64");
    SgbmEff e;
    std::string why;
    int rc = resolve_sgbm(p, W, H, &e, &why);
    if (rc) return set_error(ctx, rc, why);
    if (grid_roi && (grid_roi->x0 < 0 || grid_roi->y0 < 0 || grid_roi->x1 > W || grid_roi->y1 > H ||
                     grid_roi->x1 - grid_roi->x0 < 9 || grid_roi->y1 - grid_roi->y0 < 9))
        return set_error(ctx, MVSV_E_INVALID_ARG, "grid ROI outside the image or smaller than 9x9");
    DeviceGuard dev_guard(ctx->device);
    mvsv_stream* st = new (std::nothrow) mvsv_stream();
    if (!st) return MVSV_E_OOM;
    st->ctx = ctx;
    st->lanes.push_back(ctx);
    st->W = W;
    st->H = H;
    st->params = *p;
    st->eff = e;
    st->grid = grid_roi != nullptr;
    if (grid_roi) st->roi = *grid_roi;
    const size_t px = (size_t)W * H;
    bool ok = hipStreamCreateWithFlags(&st->up, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&st->down, hipStreamNonBlocking) == hipSuccess;
    st->slots.resize(depth);
    ok = ok && hipMalloc((void**)&st->dL_all, px * depth) == hipSuccess &&
         hipMalloc((void**)&st->dR_all, px * depth) == hipSuccess &&
         hipMalloc((void**)&st->dOut_all, px * 2 * depth) == hipSuccess &&
         hipMalloc((void**)&st->dMeans_all, 81 * sizeof(float) * depth) == hipSuccess;
    for (size_t i = 0; i < st->slots.size(); i++) {
        auto& s = st->slots[i];
        if (!ok) break;
        s.dL = st->dL_all + i * px;
        s.dR = st->dR_all + i * px;
        s.dOut = st->dOut_all + i * px;
        s.dMeans = st->dMeans_all + i * 81;
        ok = hipHostMalloc((void**)&s.hL, px, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hR, px, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hOut, px * 2, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hMeans, 81 * sizeof(float), hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.computed, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
    }
    ok = ok && alloc_report(ctx, depth, &st->rep, &st->rep_dev) == MVSV_OK;
    if (ok && px * 2 >= kPoolMinBytes) {
        int threads = 4;
        if (const char* v = std::getenv("MVSV_STREAM_COPY_THREADS")) threads = std::max(1, std::min(16, std::atoi(v)));
        if (threads > 1) {
            try {
                st->pool = new CopyPool(threads);
            } catch (...) {
                st->pool = nullptr;  // copies on the caller's thread
            }
        }
    }
    if (!ok) {
        (void)hipGetLastError();
        stream_free(st);
        return set_error(ctx, MVSV_E_OOM, "stream slot allocation failed");
    }
    *out = st;
    return MVSV_OK;
}

// Enqueue compute + download for the pushed frames [launched, head): one
// frame-batch launch per run of consecutive slots (a run ends at the ring's end).
static int stream_launch(mvsv_stream* st)
{
    const int W = st->W, H = st->H;
    const size_t px = (size_t)W * H;
    const long depth = (long)st->slots.size();
    int rc;
    RingRun run;
    while (ring_next_run(st->launched, st->head, depth, &run)) {
        const long i0 = run.i0;
        const int n = run.n;
        auto& first = st->slots[i0];
        auto& last = st->slots[i0 + n - 1];
        mvsv_ctx* ctx = st->lanes[st->runs % (long)st->lanes.size()];
        // the upload stream is in order: the last slot's upload covers the run
        if ((rc = check_hip(ctx, hipStreamWaitEvent(ctx->stream, last.uploaded, 0), "stream wait")))
            return rc;
        // slot i0 was popped (or never used): nothing reads rep[i0] any more
        __atomic_store_n(&st->rep[i0], 0, __ATOMIC_RELEASE);
        first.run_len = n;
        int* prev_target = ctx->report_target;
        ctx->report_target = st->rep_dev + i0;
        int status = sgbm_device(ctx, n, first.dL, W, px, first.dR, W, px, W, H, st->eff, first.dOut, W, px);
        ctx->report_target = prev_target;
        if (status == MVSV_OK && st->grid) {
            const mvsv_rect& q = st->roi;
            status = mean_grid_device(ctx, n, first.dOut + (size_t)q.y0 * W + q.x0, W, px, q.x1 - q.x0,
                                      q.y1 - q.y0, first.dMeans);
        }
        if (status != MVSV_OK && ctx != st->ctx) st->ctx->err = ctx->err;  // reported by pop
        st->runs++;
        if ((rc = mark_last_use(ctx, MVSV_OK)) ||
            (rc = check_hip(ctx, hipEventRecord(last.computed, ctx->stream), "stream event")) ||
            (rc = check_hip(ctx, hipStreamWaitEvent(st->down, last.computed, 0), "stream wait"))) {
            if (ctx != st->ctx) st->ctx->err = ctx->err;
            return rc;
        }
        for (int k = 0; k < n; k++) {
            auto& s = st->slots[i0 + k];
            s.status = status;
            mvsv_ctx* c = st->ctx;
            if ((rc = check_hip(c, hipMemcpyAsync(s.hOut, s.dOut, px * 2, hipMemcpyDeviceToHost, st->down),
                                "stream D2H")))
                return rc;
            if (st->grid &&
                (rc = check_hip(c, hipMemcpyAsync(s.hMeans, s.dMeans, 81 * sizeof(float),
                                                  hipMemcpyDeviceToHost, st->down), "stream D2H")))
                return rc;
            if ((rc = check_hip(c, hipEventRecord(s.done, st->down), "stream event"))) return rc;
        }
        st->launched += n;
    }
    return MVSV_OK;
}

int mvsv_stream_set_batch(mvsv_stream* st, int batch)
{
    if (!st) return MVSV_E_INVALID_ARG;
    if (batch < 1 || batch > (int)st->slots.size())
        return set_error(st->ctx, MVSV_E_INVALID_ARG, "stream batch must be 1..depth");
    DeviceGuard dev_guard(st->ctx->device);
    int rc = stream_launch(st);  // frames already pushed keep the old grouping
    if (rc) return rc;
    st->batch = batch;
    return MVSV_OK;
}

// The stream's own lanes follow the caller context's kernel options.
static void copy_options(mvsv_ctx* d, const mvsv_ctx* s)
{
    d->spin_limit = s->spin_limit;
    d->path16 = s->path16;
    d->cost2 = s->cost2;
    d->cost_fixed_pp = s->cost_fixed_pp;
    d->cost_ty = s->cost_ty;
    d->tri = s->tri;
    d->path_sched = s->path_sched;
    d->strip_waves = s->strip_waves;
    d->cost_res = s->cost_res;
    d->lines_aux = s->lines_aux;
    d->strip_tickets = s->strip_tickets;
    d->bm2 = s->bm2;
    d->bm_ty = s->bm_ty;
    d->bitslice = s->bitslice;
    d->bs_groups = s->bs_groups;
    d->bs_serial = s->bs_serial;
    d->cost_xcd = s->cost_xcd;
    d->bs_fuse = s->bs_fuse;
}

int mvsv_stream_set_inflight(mvsv_stream* st, int n)
{
    if (!st) return MVSV_E_INVALID_ARG;
    mvsv_ctx* ctx = st->ctx;
    if (n < 1 || n > kStreamMaxInflight)
        return set_error(ctx, MVSV_E_INVALID_ARG, "stream launches in flight must be 1..4");
    DeviceGuard dev_guard(ctx->device);
    int rc = stream_launch(st);  // frames already pushed keep the old lanes
    if (rc) return rc;
    while ((int)st->lanes.size() < n) {
        mvsv_ctx* c = nullptr;
        if ((rc = mvsv_create(&c, ctx->device))) return set_error(ctx, rc, "stream lane context creation failed");
        copy_options(c, ctx);
        st->lanes.push_back(c);
    }
    while ((int)st->lanes.size() > n) {  // mvsv_destroy waits for the lane's work
        mvsv_destroy(st->lanes.back());
        st->lanes.pop_back();
    }
    st->runs = 0;
    return MVSV_OK;
}

int mvsv_stream_set_params(mvsv_stream* st, const mvsv_sgbm_params* p)
{
    if (!st) return MVSV_E_INVALID_ARG;
    SgbmEff e;
    std::string why;
    int rc = resolve_sgbm(p, st->W, st->H, &e, &why);
    if (rc) return set_error(st->ctx, rc, why);
    DeviceGuard dev_guard(st->ctx->device);
    if ((rc = stream_launch(st))) return rc;  // pending frames keep the old parameters
    st->params = *p;  // applies to frames pushed from now on (trgt/mean_test.cpp:348 setters)
    st->eff = e;
    return MVSV_OK;
}

int mvsv_stream_pending(const mvsv_stream* st) { return st ? (int)(st->head - st->tail) : 0; }

int mvsv_stream_push(mvsv_stream* st, const uint8_t* L, size_t ls, const uint8_t* R, size_t rs)
{
    if (!st) return MVSV_E_INVALID_ARG;
    mvsv_ctx* ctx = st->ctx;
    if (!L || !R || ls < (size_t)st->W || rs < (size_t)st->W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "null frame or stride smaller than width");
    if (ring_full(st->head, st->tail, (long)st->slots.size()))
        return set_error(ctx, MVSV_E_INVALID_ARG, "stream full: pop a frame first");
    DeviceGuard dev_guard(ctx->device);
    auto& s = st->slots[st->head % st->slots.size()];
    const int W = st->W, H = st->H;
    // the slot's previous frame was popped, so its copies are complete
    auto copy_in = [&](int part, int parts) {
        copy_rows(s.hL, W, L, ls, W, H, part, parts);
        copy_rows(s.hR, W, R, rs, W, H, part, parts);
    };
    if (st->pool)
        st->pool->run(copy_in);
    else
        copy_in(0, 1);
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(s.dL, s.hL, px, hipMemcpyHostToDevice, st->up), "stream H2D")) ||
        (rc = check_hip(ctx, hipMemcpyAsync(s.dR, s.hR, px, hipMemcpyHostToDevice, st->up), "stream H2D")) ||
        (rc = check_hip(ctx, hipEventRecord(s.uploaded, st->up), "stream event")))
        return rc;
    st->head++;
    // a full group, or a group that would otherwise wrap past the ring's end
    if (ring_launch_after_push(st->head, st->launched, st->batch, (long)st->slots.size()))
        return stream_launch(st);
    return MVSV_OK;
}

// Wait for the oldest pending frame and release its slot: its status, and the
// slot whose pinned map / means hold the result (valid until the slot's reuse).
static int stream_pop_slot(mvsv_stream* st, mvsv_stream::Slot** slot)
{
    mvsv_ctx* ctx = st->ctx;
    if (st->head == st->tail) return set_error(ctx, MVSV_E_INVALID_ARG, "stream empty");
    auto& s = st->slots[st->tail % st->slots.size()];
    *slot = &s;
    int rc = MVSV_OK;
    if (st->tail >= st->launched && (rc = stream_launch(st))) return rc;  // partial group
    rc = check_hip(ctx, hipEventSynchronize(s.done), "stream sync");
    const long idx = st->tail % (long)st->slots.size();
    st->tail++;
    if (rc) return rc;
    if (s.run_len > 0) {  // first frame of its launch: that launch has completed
        const bool gave_up = __atomic_exchange_n(&st->rep[idx], 0, __ATOMIC_ACQ_REL) != 0;
        for (int k = 0; k < s.run_len; k++) st->slots[idx + k].gave_up = gave_up;
        s.run_len = 0;
    }
    if (s.status) return s.status;
    if (s.gave_up) {
        s.gave_up = false;
        return set_error(ctx, MVSV_E_TIMEOUT,
                         "stream frame: a strip-boundary wait of its SGBM launch gave up");
    }
    return MVSV_OK;
}

static void stream_means(const mvsv_stream* st, const mvsv_stream::Slot& s, float* means)
{
    if (!means) return;
    if (st->grid)
        std::memcpy(means, s.hMeans, 81 * sizeof(float));
    else
        std::memset(means, 0, 81 * sizeof(float));
}

int mvsv_stream_pop(mvsv_stream* st, int16_t* out, size_t os, float* means)
{
    if (!st) return MVSV_E_INVALID_ARG;
    if (out && os < (size_t)st->W) return set_error(st->ctx, MVSV_E_INVALID_ARG, "stride smaller than width");
    DeviceGuard dev_guard(st->ctx->device);
    mvsv_stream::Slot* sp = nullptr;
    int rc = stream_pop_slot(st, &sp);
    if (rc) return rc;
    const auto& s = *sp;
    if (out) {
        auto copy_out = [&](int part, int parts) {
            copy_rows((uint8_t*)out, os * 2, (const uint8_t*)s.hOut, (size_t)st->W * 2, (size_t)st->W * 2, st->H,
                      part, parts);
        };
        if (st->pool)
            st->pool->run(copy_out);
        else
            copy_out(0, 1);
    }
    stream_means(st, s, means);
    return MVSV_OK;
}

int mvsv_stream_pop_view(mvsv_stream* st, const int16_t** map, float* means)
{
    if (!st || !map) return MVSV_E_INVALID_ARG;
    *map = nullptr;
    DeviceGuard dev_guard(st->ctx->device);
    mvsv_stream::Slot* sp = nullptr;
    int rc = stream_pop_slot(st, &sp);
    if (rc) return rc;
    *map = sp->hOut;
    stream_means(st, *sp, means);
    return MVSV_OK;
}

void mvsv_stream_destroy(mvsv_stream* st)
{
    if (!st) return;
    DeviceGuard dev_guard(st->ctx->device);
    (void)hipStreamSynchronize(st->up);
    for (mvsv_ctx* c : st->lanes) (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(st->down);
    stream_free(st);
}

int mvsv_mean_disparity_grid(mvsv_ctx* ctx, const int16_t* dmap, size_t st, int W, int H,
                             float* means)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!dmap || !means || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad mean-grid arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, [&]() -> int {  // every exit after an enqueue
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = ensure(ctx, ctx->h_out, px * 2 + 4 + 81 * sizeof(float), "grid staging"))) return rc;
    int16_t* d = (int16_t*)ctx->h_out.ptr;
    float* m = (float*)(d + px + (px & 1));
    hipStream_t s = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(d, (size_t)W * 2, dmap, st * 2, (size_t)W * 2, H,
                                              hipMemcpyHostToDevice, s), "H2D map")) ||
        (rc = mean_grid_device(ctx, 1, d, W, px, W, H, m)) ||
        (rc = check_hip(ctx, hipMemcpyAsync(means, m, 81 * sizeof(float), hipMemcpyDeviceToHost, s),
                        "D2H means")))
        return rc;
    return check_hip(ctx, hipStreamSynchronize(s), "hipStreamSynchronize");
    }());
}
