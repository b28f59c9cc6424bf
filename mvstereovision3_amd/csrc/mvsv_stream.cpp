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
#include <cstring>
#include <vector>

#include "mvsv_internal.hpp"

using namespace mvsv;

struct mvsv_stream {
    mvsv_ctx* ctx = nullptr;
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
    };
    std::vector<Slot> slots;
    long head = 0, tail = 0;  // pushed / popped frame counters
};

static void stream_free(mvsv_stream* st)
{
    for (auto& s : st->slots) {
        if (s.hL) (void)hipHostFree(s.hL);
        if (s.hR) (void)hipHostFree(s.hR);
        if (s.hOut) (void)hipHostFree(s.hOut);
        if (s.hMeans) (void)hipHostFree(s.hMeans);
        if (s.dL) (void)hipFree(s.dL);
        if (s.dR) (void)hipFree(s.dR);
        if (s.dOut) (void)hipFree(s.dOut);
        if (s.dMeans) (void)hipFree(s.dMeans);
        for (hipEvent_t e : {s.uploaded, s.computed, s.done})
            if (e) (void)hipEventDestroy(e);
    }
    if (st->up) (void)hipStreamDestroy(st->up);
    if (st->down) (void)hipStreamDestroy(st->down);
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
    (void)hipSetDevice(ctx->device);
    mvsv_stream* st = new (std::nothrow) mvsv_stream();
    if (!st) return MVSV_E_OOM;
    st->ctx = ctx;
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
    for (auto& s : st->slots) {
        if (!ok) break;
        ok = hipHostMalloc((void**)&s.hL, px, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hR, px, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hOut, px * 2, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.hMeans, 81 * sizeof(float), hipHostMallocDefault) == hipSuccess &&
             hipMalloc((void**)&s.dL, px) == hipSuccess && hipMalloc((void**)&s.dR, px) == hipSuccess &&
             hipMalloc((void**)&s.dOut, px * 2) == hipSuccess &&
             hipMalloc((void**)&s.dMeans, 81 * sizeof(float)) == hipSuccess &&
             hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.computed, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) {
        (void)hipGetLastError();
        stream_free(st);
        return set_error(ctx, MVSV_E_OOM, "stream slot allocation failed");
    }
    *out = st;
    return MVSV_OK;
}

int mvsv_stream_set_params(mvsv_stream* st, const mvsv_sgbm_params* p)
{
    if (!st) return MVSV_E_INVALID_ARG;
    SgbmEff e;
    std::string why;
    int rc = resolve_sgbm(p, st->W, st->H, &e, &why);
    if (rc) return set_error(st->ctx, rc, why);
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
    if (st->head - st->tail >= (long)st->slots.size())
        return set_error(ctx, MVSV_E_INVALID_ARG, "stream full: pop a frame first");
    (void)hipSetDevice(ctx->device);
    auto& s = st->slots[st->head % st->slots.size()];
    const int W = st->W, H = st->H;
    // the slot's previous frame was popped, so its copies are complete
    for (int y = 0; y < H; y++) {
        std::memcpy(s.hL + (size_t)y * W, L + (size_t)y * ls, W);
        std::memcpy(s.hR + (size_t)y * W, R + (size_t)y * rs, W);
    }
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(s.dL, s.hL, px, hipMemcpyHostToDevice, st->up), "stream H2D")) ||
        (rc = check_hip(ctx, hipMemcpyAsync(s.dR, s.hR, px, hipMemcpyHostToDevice, st->up), "stream H2D")) ||
        (rc = check_hip(ctx, hipEventRecord(s.uploaded, st->up), "stream event")) ||
        (rc = check_hip(ctx, hipStreamWaitEvent(ctx->stream, s.uploaded, 0), "stream wait")))
        return rc;
    s.status = sgbm_device(ctx, 1, s.dL, W, px, s.dR, W, px, W, H, st->eff, s.dOut, W, px);
    if (s.status == MVSV_OK && st->grid) {
        const mvsv_rect& q = st->roi;
        s.status = mean_grid_device(ctx, 1, s.dOut + (size_t)q.y0 * W + q.x0, W, px, q.x1 - q.x0,
                                    q.y1 - q.y0, s.dMeans);
    }
    if ((rc = check_hip(ctx, hipEventRecord(s.computed, ctx->stream), "stream event")) ||
        (rc = check_hip(ctx, hipStreamWaitEvent(st->down, s.computed, 0), "stream wait")) ||
        (rc = check_hip(ctx, hipMemcpyAsync(s.hOut, s.dOut, px * 2, hipMemcpyDeviceToHost, st->down),
                        "stream D2H")))
        return rc;
    if (st->grid &&
        (rc = check_hip(ctx, hipMemcpyAsync(s.hMeans, s.dMeans, 81 * sizeof(float),
                                            hipMemcpyDeviceToHost, st->down), "stream D2H")))
        return rc;
    if ((rc = check_hip(ctx, hipEventRecord(s.done, st->down), "stream event"))) return rc;
    st->head++;
    return MVSV_OK;
}

int mvsv_stream_pop(mvsv_stream* st, int16_t* out, size_t os, float* means)
{
    if (!st) return MVSV_E_INVALID_ARG;
    mvsv_ctx* ctx = st->ctx;
    if (st->head == st->tail) return set_error(ctx, MVSV_E_INVALID_ARG, "stream empty");
    if (out && os < (size_t)st->W) return set_error(ctx, MVSV_E_INVALID_ARG, "stride smaller than width");
    auto& s = st->slots[st->tail % st->slots.size()];
    (void)hipSetDevice(ctx->device);
    int rc = check_hip(ctx, hipEventSynchronize(s.done), "stream sync");
    st->tail++;
    if (rc) return rc;
    if (s.status) return s.status;
    if (out)
        for (int y = 0; y < st->H; y++)
            std::memcpy(out + (size_t)y * os, s.hOut + (size_t)y * st->W, (size_t)st->W * 2);
    if (means) {
        if (st->grid)
            std::memcpy(means, s.hMeans, 81 * sizeof(float));
        else
            std::memset(means, 0, 81 * sizeof(float));
    }
    return MVSV_OK;
}

void mvsv_stream_destroy(mvsv_stream* st)
{
    if (!st) return;
    (void)hipSetDevice(st->ctx->device);
    (void)hipStreamSynchronize(st->up);
    (void)hipStreamSynchronize(st->ctx->stream);
    (void)hipStreamSynchronize(st->down);
    stream_free(st);
}

int mvsv_mean_disparity_grid(mvsv_ctx* ctx, const int16_t* dmap, size_t st, int W, int H,
                             float* means)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!dmap || !means || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad mean-grid arguments");
    (void)hipSetDevice(ctx->device);
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
}
