// mvsv_host.cpp — host side of libmvsv: parameter resolution (OpenCV's
// defaulting + assert rules), context / stream / buffer management, the
// host-pointer entry points, the YAML loaders and the synthetic generator.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

#include "mvsv_internal.hpp"

namespace mvsv {

int set_error(mvsv_ctx* ctx, int code, const std::string& msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

int check_hip(mvsv_ctx* ctx, hipError_t e, const char* what)
{
    if (e == hipSuccess) return MVSV_OK;
    return set_error(ctx, e == hipErrorOutOfMemory ? MVSV_E_OOM : MVSV_E_HIP,
                     std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(mvsv_ctx* ctx, DevBuf& b, size_t bytes, const char* what)
{
    if (bytes <= b.bytes && b.ptr) return MVSV_OK;
    if (b.ptr) {
        // the stream may still use the old buffer
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(b.ptr);
        b.ptr = nullptr;
        b.bytes = 0;
    }
    if (bytes == 0) return MVSV_OK;
    hipError_t e = hipMalloc(&b.ptr, bytes);
    if (e != hipSuccess) {
        b.ptr = nullptr;
        (void)hipGetLastError();
        return set_error(ctx, MVSV_E_OOM,
                         std::string("device allocation of ") + std::to_string(bytes) +
                             " bytes for " + what + " failed");
    }
    b.bytes = bytes;
    return MVSV_OK;
}

int check_report(mvsv_ctx* ctx)
{
    if (!ctx->report) return MVSV_OK;
    const int v = __atomic_load_n(ctx->report, __ATOMIC_ACQUIRE);
    if (v == 0) return MVSV_OK;
    __atomic_store_n(ctx->report, 0, __ATOMIC_RELEASE);
    return set_error(ctx, MVSV_E_TIMEOUT,
                     "sgbm path kernel: a strip-boundary wait gave up (that launch's maps are all "
                     "INVALID)");
}

int alloc_report(mvsv_ctx* ctx, int count, int** host, int** dev)
{
    *host = nullptr;
    *dev = nullptr;
    void* h = nullptr;
    // fine-grained, coherent: kernels store into it with system scope and the
    // host reads it without a copy
    hipError_t e = hipHostMalloc(&h, sizeof(int) * (size_t)count,
                                 hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return check_hip(ctx, e, "report word allocation");
    std::memset(h, 0, sizeof(int) * (size_t)count);
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return check_hip(ctx, e, "report word mapping");
    }
    *host = (int*)h;
    *dev = (int*)d;
    return MVSV_OK;
}

static hipEvent_t pool_get(mvsv_ctx* ctx)
{
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return e;
}

StageTimer::StageTimer(mvsv_ctx* c, int s, hipStream_t on) : ctx(c), stage(s), st(on ? on : c->stream)
{
    if (!ctx->prof) return;
    a = pool_get(ctx);
    b = pool_get(ctx);
    if (a) (void)hipEventRecord(a, st);
}

StageTimer::~StageTimer()
{
    if (!ctx->prof || !a || !b) return;
    (void)hipEventRecord(b, st);
    ctx->marks.push_back({stage, a, b});
}

// [OpenCV] StereoSGBMImpl::compute asserts + computeDisparitySGBM prologue.
int resolve_sgbm(const mvsv_sgbm_params* p, int W, int H, SgbmEff* e, std::string* why)
{
    if (!p) { *why = "null parameters"; return MVSV_E_INVALID_ARG; }
    if (W <= 0 || H <= 0) { *why = "empty image"; return MVSV_E_INVALID_ARG; }
    if (p->num_disparities <= 0 || p->num_disparities % 16 != 0) {
        *why = "numDisparities must be positive and divisible by 16";
        return MVSV_E_INVALID_ARG;
    }
    if (p->mode != MVSV_MODE_SGBM && p->mode != MVSV_MODE_HH) {
        *why = "mode must be MODE_SGBM (0) or MODE_HH (1)";
        return MVSV_E_INVALID_ARG;
    }
    int bs = p->block_size > 0 ? p->block_size : 5;
    e->minD = p->min_disparity;
    e->D = p->num_disparities;
    e->maxD = e->minD + e->D;
    e->SW2 = bs / 2;
    e->SH2 = bs / 2;
    e->ftzero = std::max(p->pre_filter_cap, 15) | 1;
    e->uniq = p->uniqueness_ratio >= 0 ? p->uniqueness_ratio : 10;
    e->disp12 = p->disp12_max_diff > 0 ? p->disp12_max_diff : 1;
    e->P1 = p->p1 > 0 ? p->p1 : 2;
    e->P2 = std::max(p->p2 > 0 ? p->p2 : 5, e->P1 + 1);
    e->minX1 = std::max(e->maxD, 0);
    e->maxX1 = W + std::min(e->minD, 0);
    e->W1 = e->maxX1 - e->minX1;
    e->invalid = (e->minD - 1) * kDispScale;
    e->fullDP = p->mode == MVSV_MODE_HH;
    e->variant = p->variant;
    e->speckle_window = p->speckle_window_size;
    e->speckle_diff = kDispScale * p->speckle_range;
    if (e->W1 > 0 && e->W1 <= e->SW2) {
        *why = "image narrower than the SGBM block half-width (OpenCV reads uninitialised memory)";
        return MVSV_E_INVALID_ARG;
    }
    return MVSV_OK;
}

// [OpenCV] StereoBMImpl::compute checks + findStereoCorrespondenceBM setup.
int resolve_bm(const mvsv_bm_params* p, int W, int H, BmEff* e, std::string* why)
{
    if (!p) { *why = "null parameters"; return MVSV_E_INVALID_ARG; }
    if (W <= 0 || H <= 0) { *why = "empty image"; return MVSV_E_INVALID_ARG; }
    if (p->pre_filter_type != MVSV_PREFILTER_NORMALIZED_RESPONSE &&
        p->pre_filter_type != MVSV_PREFILTER_XSOBEL) {
        *why = "preFilterType must be = CV_STEREO_BM_NORMALIZED_RESPONSE";
        return MVSV_E_INVALID_ARG;
    }
    if (p->pre_filter_size < 5 || p->pre_filter_size > 255 || p->pre_filter_size % 2 == 0) {
        *why = "preFilterSize must be odd and be within 5..255";
        return MVSV_E_INVALID_ARG;
    }
    if (p->pre_filter_cap < 1 || p->pre_filter_cap > 63) {
        *why = "preFilterCap must be within 1..63";
        return MVSV_E_INVALID_ARG;
    }
    if (p->block_size < 5 || p->block_size > 255 || p->block_size % 2 == 0 ||
        p->block_size >= std::min(W, H)) {
        *why = "SADWindowSize must be odd, be within 5..255 and be not larger than image width or height";
        return MVSV_E_INVALID_ARG;
    }
    if (p->num_disparities <= 0 || p->num_disparities % 16 != 0) {
        *why = "numDisparities must be positive and divisible by 16";
        return MVSV_E_INVALID_ARG;
    }
    if (p->texture_threshold < 0) { *why = "texture threshold must be non-negative"; return MVSV_E_INVALID_ARG; }
    if (p->uniqueness_ratio < 0) { *why = "uniqueness ratio must be non-negative"; return MVSV_E_INVALID_ARG; }
    e->ndisp = p->num_disparities;
    e->mindisp = p->min_disparity;
    e->wsz2 = p->block_size / 2;
    e->cap = p->pre_filter_cap;
    e->tex = p->texture_threshold;
    e->uniq = p->uniqueness_ratio;
    e->lofs = std::max(e->ndisp - 1 + e->mindisp, 0);
    e->rofs = -std::min(e->ndisp - 1 + e->mindisp, 0);
    e->width1 = W - e->rofs - e->ndisp + 1;
    e->ncol = std::min(e->width1, W - e->lofs);
    e->filtered = (e->mindisp - 1) * kDispScale;
    int maxDm1 = e->mindisp + e->ndisp - 1;
    e->xmin = std::max(0, maxDm1) + e->wsz2;
    e->xmax = W - e->wsz2;
    e->ymin = e->wsz2;
    e->ymax = H - e->wsz2;
    e->disp12 = p->disp12_max_diff;
    e->speckle_window = p->speckle_window_size;
    e->speckle_range = p->speckle_range;
    e->prefilter_type = p->pre_filter_type;
    e->prefilter_size = p->pre_filter_size;
    return MVSV_OK;
}

}  // namespace mvsv

using namespace mvsv;

extern "C" {

int mvsv_version(void) { return MVSV_VERSION; }

void mvsv_sgbm_params_create(mvsv_sgbm_params* p, int min_disparity, int num_disparities,
                             int block_size, int p1, int p2, int disp12_max_diff,
                             int pre_filter_cap, int uniqueness_ratio, int speckle_window_size,
                             int speckle_range, int mode)
{
    if (!p) return;
    p->min_disparity = min_disparity;
    p->num_disparities = num_disparities;
    p->block_size = block_size;
    p->p1 = p1;
    p->p2 = p2;
    p->disp12_max_diff = disp12_max_diff;
    p->pre_filter_cap = pre_filter_cap;
    p->uniqueness_ratio = uniqueness_ratio;
    p->speckle_window_size = speckle_window_size;
    p->speckle_range = speckle_range;
    p->mode = mode;
    p->variant = 0;
}

void mvsv_sgbm_params_default(mvsv_sgbm_params* p)
{
    mvsv_sgbm_params_create(p, 0, 16, 3, 0, 0, 0, 0, 0, 0, 0, MVSV_MODE_SGBM);
}

void mvsv_bm_params_default(mvsv_bm_params* p, int num_disparities, int block_size)
{
    if (!p) return;
    p->pre_filter_type = MVSV_PREFILTER_XSOBEL;
    p->pre_filter_size = 9;
    p->pre_filter_cap = 31;
    p->block_size = block_size;
    p->min_disparity = 0;
    p->num_disparities = num_disparities > 0 ? num_disparities : 64;
    p->texture_threshold = 10;
    p->uniqueness_ratio = 15;
    p->speckle_window_size = 0;
    p->speckle_range = 0;
    p->disp12_max_diff = -1;
}

int mvsv_sgbm_validate(const mvsv_sgbm_params* p, int W, int H)
{
    SgbmEff e;
    std::string why;
    return resolve_sgbm(p, W, H, &e, &why);
}

int mvsv_bm_validate(const mvsv_bm_params* p, int W, int H)
{
    BmEff e;
    std::string why;
    return resolve_bm(p, W, H, &e, &why);
}

int mvsv_create(mvsv_ctx** out, int hip_device)
{
    if (!out) return MVSV_E_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        return MVSV_E_NODEV;
    }
    if (hip_device < 0 || hip_device >= count) return MVSV_E_INVALID_ARG;
    mvsv_ctx* c = new (std::nothrow) mvsv_ctx();
    if (!c) return MVSV_E_OOM;
    c->device = hip_device;
    DeviceGuard dev_guard(hip_device);
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_switch, hipEventDisableTiming) != hipSuccess ||
        alloc_report(c, 1, &c->report, &c->report_dev) != MVSV_OK) {
        (void)hipGetLastError();
        if (c->ev_switch) (void)hipEventDestroy(c->ev_switch);
        if (c->own) (void)hipStreamDestroy(c->own);
        delete c;
        return MVSV_E_HIP;
    }
    c->report_target = c->report_dev;
    c->stream = c->own;
    if (const char* v = std::getenv("MVSV_STRIP_SPIN_LIMIT"))
        c->spin_limit = (unsigned)std::strtoul(v, nullptr, 0);
    // kernel-variant switches for A/B measurement and for testing the
    // general-shape kernels on shapes the specialised ones also cover
    if (const char* v = std::getenv("MVSV_KERNELS")) {
        if (std::strstr(v, "cost-lds")) c->cost2 = 0;
        if (std::strstr(v, "path-wave")) c->path16 = 0;
        if (std::strstr(v, "path-lines")) c->tri = 0;
    }
    if (const char* v = std::getenv("MVSV_COST_TY")) c->cost_ty = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("MVSV_LINES_AUX")) c->lines_aux = std::max(0, std::min(2, std::atoi(v)));
    *out = c;
    return MVSV_OK;
}

static void free_buf(DevBuf& b)
{
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
}

int mvsv_trim(mvsv_ctx* ctx)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    DeviceGuard dev_guard(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    DevBuf* all[] = {&ctx->pre, &ctx->cost, &ctx->agg, &ctx->raw, &ctx->uf_parent, &ctx->uf_size,
                     &ctx->uf_tile, &ctx->tri_bnd, &ctx->status,
                     &ctx->dummy, &ctx->keys,
                     &ctx->bm_lf, &ctx->bm_rf, &ctx->bm_cost, &ctx->h_left, &ctx->h_right,
                     &ctx->h_out};
    for (DevBuf* b : all) free_buf(*b);
    return MVSV_OK;
}

static const char* kStageNames[MVSV_NUM_STAGES] = {
    "prefilter", "cost_volume", "cost_fixup", "path_aggregation", "final_wta_lr", "post_filters",
    "bm_match", "path_strips", "path_lines"};

const char* mvsv_profile_stage_name(int s)
{
    return (s >= 0 && s < MVSV_NUM_STAGES) ? kStageNames[s] : "";
}

int mvsv_profile_enable(mvsv_ctx* ctx, int on)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    ctx->prof = on ? 1 : 0;
    return MVSV_OK;
}

int mvsv_profile_reset(mvsv_ctx* ctx)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& m : ctx->marks) {
        ctx->event_pool.push_back(m.a);
        ctx->event_pool.push_back(m.b);
    }
    ctx->marks.clear();
    return MVSV_OK;
}

int mvsv_profile_read(mvsv_ctx* ctx, double* ms, int* launches, int n)
{
    if (!ctx || n < 0) return MVSV_E_INVALID_ARG;
    DeviceGuard dev_guard(ctx->device);
    int rc = check_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (rc) return rc;
    for (int i = 0; i < n; i++) {
        if (ms) ms[i] = 0.0;
        if (launches) launches[i] = 0;
    }
    for (auto& m : ctx->marks) {
        if (m.stage >= n) continue;
        float t = 0.f;
        if (hipEventElapsedTime(&t, m.a, m.b) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        if (ms) ms[m.stage] += t;
        if (launches) launches[m.stage] += 1;
    }
    return MVSV_OK;
}

void mvsv_destroy(mvsv_ctx* ctx)
{
    if (!ctx) return;
    mvsv_trim(ctx);
    mvsv_profile_reset(ctx);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_switch) (void)hipEventDestroy(ctx->ev_switch);
    if (ctx->report) (void)hipHostFree(ctx->report);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    delete ctx;
}

const char* mvsv_last_error(const mvsv_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// Every launch of a context shares its cached buffers, so work enqueued on a
// new stream must not start before the work already on the previous one: the
// new stream waits on an event recorded on the old (no host synchronisation).
static int switch_stream(mvsv_ctx* ctx, hipStream_t s)
{
    if (s == ctx->stream) return MVSV_OK;
    DeviceGuard dev_guard(ctx->device);
    int rc;
    if ((rc = check_hip(ctx, hipEventRecord(ctx->ev_switch, ctx->stream), "stream switch record")) ||
        (rc = check_hip(ctx, hipStreamWaitEvent(s, ctx->ev_switch, 0), "stream switch wait")))
        return rc;
    ctx->stream = s;
    return MVSV_OK;
}

int mvsv_set_stream(mvsv_ctx* ctx, void* s)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    return switch_stream(ctx, (hipStream_t)s);  // NULL = the HIP null stream
}

int mvsv_use_own_stream(mvsv_ctx* ctx)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    return switch_stream(ctx, ctx->own);
}

int mvsv_set_option(mvsv_ctx* ctx, int option, long long value)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    switch (option) {
    case MVSV_OPT_STRIP_SPIN_LIMIT:
        if (value < 0 || value > 0xffffffffLL)
            return set_error(ctx, MVSV_E_INVALID_ARG, "spin limit must be 0..2^32-1");
        ctx->spin_limit = (unsigned)value;
        return MVSV_OK;
    default:
        return set_error(ctx, MVSV_E_INVALID_ARG, "unknown option");
    }
}

void* mvsv_get_stream(mvsv_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int mvsv_synchronize(mvsv_ctx* ctx)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    DeviceGuard dev_guard(ctx->device);
    int rc = check_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    return rc ? rc : check_report(ctx);
}

size_t mvsv_sgbm_workspace_bytes(int n, int W, int H, const mvsv_sgbm_params* p)
{
    SgbmEff e;
    std::string why;
    if (n <= 0 || resolve_sgbm(p, W, H, &e, &why) != MVSV_OK) return 0;
    size_t frame = (size_t)W * H;
    size_t vol = e.W1 > 0 ? (size_t)e.W1 * H * e.D * 2 : 0;
    size_t b = (size_t)n * (frame * 4 + 2 * vol + frame * 2);
    if (e.speckle_window > 0) b += (size_t)n * frame * 8;
    return b;
}

int mvsv_sgbm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs,
                     const uint8_t* R, size_t rs, size_t rfs, int W, int H,
                     const mvsv_sgbm_params* p, int16_t* out, size_t os, size_t ofs)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !L || !R || !out) return set_error(ctx, MVSV_E_INVALID_ARG, "null buffer or n <= 0");
    if (ls < (size_t)W || rs < (size_t)W || os < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "stride smaller than width");
    SgbmEff e;
    std::string why;
    int rc = resolve_sgbm(p, W, H, &e, &why);
    if (rc) return set_error(ctx, rc, why);
    // an earlier launch that has finished by now gave up a strip wait: its
    // maps are INVALID; say so before anything else runs on this context
    if ((rc = check_report(ctx))) return rc;
    DeviceGuard dev_guard(ctx->device);
    return sgbm_device(ctx, n, L, ls, lfs, R, rs, rfs, W, H, e, out, os, ofs);
}

int mvsv_bm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs,
                   const uint8_t* R, size_t rs, size_t rfs, int W, int H,
                   const mvsv_bm_params* p, int16_t* out, size_t os, size_t ofs)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !L || !R || !out) return set_error(ctx, MVSV_E_INVALID_ARG, "null buffer or n <= 0");
    if (ls < (size_t)W || rs < (size_t)W || os < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "stride smaller than width");
    BmEff e;
    std::string why;
    int rc = resolve_bm(p, W, H, &e, &why);
    if (rc) return set_error(ctx, rc, why);
    DeviceGuard dev_guard(ctx->device);
    return bm_device(ctx, n, L, ls, lfs, R, rs, rfs, W, H, e, out, os, ofs);
}

int mvsv_mean_disparity_grid_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st,
                                    size_t fs, int W, int H, float* means)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !dmap || !means || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad mean-grid arguments");
    DeviceGuard dev_guard(ctx->device);
    return mean_grid_device(ctx, n, dmap, st, fs, W, H, means);
}

// Host-pointer path: stage through cached device buffers, run, copy back, sync.
static int host_call(mvsv_ctx* ctx, const uint8_t* L, size_t ls, const uint8_t* R, size_t rs,
                     int W, int H, int16_t* out, size_t os, bool sgbm, const void* params)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!L || !R || !out || W <= 0 || H <= 0)
        return set_error(ctx, MVSV_E_INVALID_ARG, "null buffer or empty image");
    if (ls < (size_t)W || rs < (size_t)W || os < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "stride smaller than width");
    int rc;
    SgbmEff se;
    BmEff be;
    std::string why;
    rc = sgbm ? resolve_sgbm((const mvsv_sgbm_params*)params, W, H, &se, &why)
              : resolve_bm((const mvsv_bm_params*)params, W, H, &be, &why);
    if (rc) return set_error(ctx, rc, why);
    if (sgbm && (rc = check_report(ctx))) return rc;  // an earlier device call's give-up
    DeviceGuard dev_guard(ctx->device);
    size_t fb = (size_t)W * H;
    if ((rc = ensure(ctx, ctx->h_left, fb, "left staging"))) return rc;
    if ((rc = ensure(ctx, ctx->h_right, fb, "right staging"))) return rc;
    if ((rc = ensure(ctx, ctx->h_out, fb * 2, "output staging"))) return rc;
    hipStream_t s = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(ctx->h_left.ptr, W, L, ls, W, H, hipMemcpyHostToDevice, s), "H2D left"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(ctx->h_right.ptr, W, R, rs, W, H, hipMemcpyHostToDevice, s), "H2D right"))) return rc;
    int16_t* dout = (int16_t*)ctx->h_out.ptr;
    rc = sgbm ? sgbm_device(ctx, 1, (const uint8_t*)ctx->h_left.ptr, W, fb,
                            (const uint8_t*)ctx->h_right.ptr, W, fb, W, H, se, dout, W, fb)
              : bm_device(ctx, 1, (const uint8_t*)ctx->h_left.ptr, W, fb,
                          (const uint8_t*)ctx->h_right.ptr, W, fb, W, H, be, dout, W, fb);
    if (rc) return rc;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(out, os * 2, dout, (size_t)W * 2, (size_t)W * 2, H, hipMemcpyDeviceToHost, s), "D2H out"))) return rc;
    if ((rc = check_hip(ctx, hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    return check_report(ctx);
}

int mvsv_sgbm(mvsv_ctx* ctx, const uint8_t* L, size_t ls, const uint8_t* R, size_t rs, int W,
              int H, const mvsv_sgbm_params* p, int16_t* out, size_t os)
{
    return host_call(ctx, L, ls, R, rs, W, H, out, os, true, p);
}

int mvsv_bm(mvsv_ctx* ctx, const uint8_t* L, size_t ls, const uint8_t* R, size_t rs, int W,
            int H, const mvsv_bm_params* p, int16_t* out, size_t os)
{
    return host_call(ctx, L, ls, R, rs, W, H, out, os, false, p);
}

// ---------------------------------------------------------------------------
// Flat %YAML:1.0 "key: number" reader (the subset cv::FileStorage writes for
// configs/sgbm.yml and configs/bm.yml). Numbers are rounded like cvRound.
// ---------------------------------------------------------------------------
static int read_flat_yaml(const char* path, std::map<std::string, double>* kv)
{
    if (!path) return MVSV_E_INVALID_ARG;
    std::ifstream f(path);
    if (!f.is_open()) return MVSV_E_IO;
    std::string line;
    bool first = true;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (first) {
            first = false;
            if (line.rfind("%YAML", 0) == 0) continue;
        }
        size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (line.find_first_not_of(" \t") == std::string::npos) continue;
        if (line == "---" || line == "...") continue;
        size_t colon = line.find(':');
        if (colon == std::string::npos) continue;
        std::string key = line.substr(0, colon);
        std::string val = line.substr(colon + 1);
        auto trim = [](std::string& s) {
            size_t a = s.find_first_not_of(" \t\"'");
            size_t b = s.find_last_not_of(" \t\"'");
            s = a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
        };
        trim(key);
        trim(val);
        if (key.empty() || val.empty()) continue;  // nested map / empty node
        char* end = nullptr;
        errno = 0;
        double d = std::strtod(val.c_str(), &end);
        if (end == val.c_str() || errno) continue;  // non-numeric: not an int node
        (*kv)[key] = d;
    }
    return MVSV_OK;
}

static int kv_int(const std::map<std::string, double>& kv, const char* key, int dflt)
{
    auto it = kv.find(key);
    return it == kv.end() ? dflt : (int)std::lrint(it->second);
}

int mvsv_load_sgbm_yaml(const char* path, mvsv_sgbm_params* p, mvsv_sgbm_yaml_values* v)
{
    std::map<std::string, double> kv;
    int rc = read_flat_yaml(path, &kv);
    if (rc) return rc;  // reference: LOG(ERROR) "Unable to open disparity parameters"
    // src/disparity.cpp:67 — required nodes
    for (const char* k : {"numDisp", "blockSize", "speckleWindowSize", "speckleWindowRange"})
        if (!kv.count(k)) return MVSV_E_PARSE;
    mvsv_sgbm_yaml_values tmp;
    tmp.minDisp = kv_int(kv, "minDisp", 0);
    tmp.numDisp = kv_int(kv, "numDisp", 0);
    tmp.blockSize = kv_int(kv, "blockSize", 0);
    tmp.disp12MaxDiff = kv_int(kv, "disp12MaxDiff", 0);
    tmp.preFilterCap = kv_int(kv, "preFilterCap", 0);
    tmp.uniquenessRatio = kv_int(kv, "uniquenessRatio", 0);
    tmp.speckleWindowSize = kv_int(kv, "speckleWindowSize", 0);
    tmp.speckleRange = kv_int(kv, "speckleWindowRange", 0);
    tmp.disparityMode = kv_int(kv, "mode", 0);
    if (v) *v = tmp;
    if (p) {  // src/disparity.cpp:83-95 — eight setters + mode, P1/P2 untouched
        p->min_disparity = tmp.minDisp;
        p->num_disparities = tmp.numDisp;
        p->block_size = tmp.blockSize;
        p->pre_filter_cap = tmp.preFilterCap;
        p->uniqueness_ratio = tmp.uniquenessRatio;
        p->disp12_max_diff = tmp.disp12MaxDiff;
        p->speckle_window_size = tmp.speckleWindowSize;
        p->speckle_range = tmp.speckleRange;
        p->mode = tmp.disparityMode == 1 ? MVSV_MODE_HH : MVSV_MODE_SGBM;
    }
    return MVSV_OK;
}

int mvsv_load_bm_yaml(const char* path, mvsv_bm_params* p)
{
    std::map<std::string, double> kv;
    int rc = read_flat_yaml(path, &kv);
    if (rc) return rc;
    for (const char* k : {"numDisp", "blockSize"})
        if (!kv.count(k)) return MVSV_E_PARSE;
    if (p) {
        p->num_disparities = kv_int(kv, "numDisp", p->num_disparities);
        p->block_size = kv_int(kv, "blockSize", p->block_size);
        p->pre_filter_cap = kv_int(kv, "preFilterCap", p->pre_filter_cap);
        p->pre_filter_size = kv_int(kv, "preFilterSize", p->pre_filter_size);
        p->uniqueness_ratio = kv_int(kv, "uniquenessRatio", p->uniqueness_ratio);
        p->texture_threshold = kv_int(kv, "textureThreshold", p->texture_threshold);
        p->min_disparity = kv_int(kv, "minDisp", p->min_disparity);
        p->speckle_window_size = kv_int(kv, "speckleWindowSize", p->speckle_window_size);
        p->speckle_range = kv_int(kv, "speckleWindowRange", p->speckle_range);
        p->disp12_max_diff = kv_int(kv, "disp12MaxDiff", p->disp12_max_diff);
        p->pre_filter_type = kv_int(kv, "preFilterType", p->pre_filter_type);
    }
    return MVSV_OK;
}

// ---------------------------------------------------------------------------
// Synthetic rectified pair.
// ---------------------------------------------------------------------------
namespace {
struct Pcg32 {
    uint64_t state;
    static constexpr uint64_t inc = 0xda3e39cb94b95bdbULL;
    explicit Pcg32(uint32_t seed) : state((uint64_t)seed * 2u + 1u) {}
    uint32_t next()
    {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
};
}  // namespace

int mvsv_synth_pair(uint32_t seed, int W, int H, int minD, int D, uint8_t* Lout, uint8_t* Rout)
{
    if (W <= 0 || H <= 0 || D <= 0 || !Lout || !Rout) return MVSV_E_INVALID_ARG;
    Pcg32 rng(seed);
    size_t np = (size_t)W * H;
    uint8_t* noise = (uint8_t*)std::malloc(np);
    if (!noise) return MVSV_E_OOM;
    for (size_t i = 0; i < np; i++) noise[i] = (uint8_t)(rng.next() >> 24);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int s = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = std::min(std::max(y + dy, 0), H - 1);
                    int xx = std::min(std::max(x + dx, 0), W - 1);
                    s += noise[(size_t)yy * W + xx];
                }
            Lout[(size_t)y * W + x] = (uint8_t)((2 * s + 9) / 18);  // round half up of s/9
        }
    std::free(noise);
    const int rect = (int)std::floor(0.6 * D + 0.5);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            bool in = x >= W / 3 && x < 2 * W / 3 && y >= H / 3 && y < 2 * H / 3;
            int d = in ? rect : (int)std::floor(D / 8.0 + (D / 4.0) * y / H + 0.5);
            d = std::min(std::max(d, minD), minD + D - 1);
            int xs = std::min(std::max(x + d, 0), W - 1);
            int v = Lout[(size_t)y * W + xs] + (int)(rng.next() % 3u) - 1;
            Rout[(size_t)y * W + x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    return MVSV_OK;
}

}  // extern "C"

// ---- reprojection and PLY output -------------------------

int mvsv_reproject_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W,
                          int H, const float* Q, float* xyzw, size_t xs, size_t xfs)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !dmap || !Q || !xyzw || W <= 0 || H <= 0 || st < (size_t)W || xs < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad reprojection arguments");
    DeviceGuard dev_guard(ctx->device);
    return reproject_device(ctx, n, dmap, st, fs, W, H, Q, xyzw, xs, xfs);
}

// [Utility::calcCoordinate] src/utility.cpp:176-198 with OpenCV's float matrix
// product (double accumulation, one rounding) and Mat /= w (float scale).
void mvsv_calc_coordinate(float image_x, float image_y, float d_value, const float* Q, float* out)
{
    const float c[4] = {image_x, image_y, d_value / 16, 1.0f};
    float r[4];
    for (int i = 0; i < 4; i++) {
        double acc = 0.0;
        for (int k = 0; k < 4; k++) acc += (double)Q[4 * i + k] * (double)c[k];
        r[i] = (float)acc;
    }
    const float alpha = (float)(1.0 / (double)r[3]);
    for (int i = 0; i < 4; i++) out[i] = r[i] * alpha;
    if (std::isinf(out[2] / 1000)) out[2] = 0.0f;
}

// [Utility::calcDistance] src/utility.cpp:200-222
float mvsv_calc_distance(float image_x, float image_y, float d_value, const float* Q)
{
    const float c[4] = {image_x, image_y, d_value / 16, 1.0f};
    float r[4];
    for (int i = 0; i < 4; i++) {
        double acc = 0.0;
        for (int k = 0; k < 4; k++) acc += (double)Q[4 * i + k] * (double)c[k];
        r[i] = (float)acc;
    }
    const float alpha = (float)(1.0 / (double)r[3]);
    const float distance = (r[2] * alpha) / 1000;
    return std::isinf(distance) ? 0.0f : distance;
}

// [Utility::calcDMapValues] src/utility.cpp:224-240
void mvsv_calc_dmap_values(const float* c, const float* Q, float* image_x, float* image_y,
                           float* d_value)
{
    const float numerator = Q[2 * 4 + 3] - c[2] * Q[3 * 4 + 3];
    const float denominator = c[2] * Q[3 * 4 + 2];
    const float disparity_value = numerator / denominator;
    *image_x = c[0] * (disparity_value * Q[3 * 4 + 2] * Q[3 * 4 + 3]) + Q[0 * 4 + 3];
    *image_y = c[1] * (disparity_value * Q[3 * 4 + 2] * Q[3 * 4 + 3]) + Q[1 * 4 + 3];
    *d_value = disparity_value * 16;
}

// [Utility::calcMinMaxDisparity] src/utility.cpp:286-303 (positive values only)
static bool min_max_positive(const int16_t* d, size_t st, int W, int H, short* mn, short* mx)
{
    bool any = false;
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++) {
            const short v = d[(size_t)r * st + c];
            if (v > 0) {
                if (!any || v < *mn) *mn = v;
                if (!any || v > *mx) *mx = v;
                any = true;
            }
        }
    return any;
}

// [ply::write] src/ply.cpp:37-133: std::ofstream with default float formatting
int mvsv_write_ply(const char* path, const char* author, const char* object_name,
                   const float* xyz, size_t count, size_t vstride, int mode, const int16_t* dmap,
                   size_t dst, int W, int H)
{
    if (!path || (!xyz && count) || vstride < 3 || mode < MVSV_PLY_PLAIN ||
        mode > MVSV_PLY_WITH_COLOR_SHADING)
        return MVSV_E_INVALID_ARG;
    short mn = 0, mx = 0;
    if (mode != MVSV_PLY_PLAIN) {
        if (!dmap || W <= 0 || H <= 0) return MVSV_E_INVALID_ARG;  // "mDMap.rows == 0" -> false
        if (!min_max_positive(dmap, dst, W, H, &mn, &mx)) return MVSV_E_INVALID_ARG;
    }
    std::ofstream out(path);
    if (!out) return MVSV_E_IO;
    out << "ply\nformat ascii 1.0\ncomment author: " << (author ? author : "")
        << "\ncomment object:" << (object_name ? object_name : "") << "\n";
    out << "element vertex " << std::to_string(count) << "\n";
    out << "property float x\nproperty float y\nproperty float z\n";
    if (mode != MVSV_PLY_PLAIN) out << "property uchar red\nproperty uchar green\nproperty uchar blue\n";
    out << "end_header\n";
    for (size_t i = 0; i < count; i++) {
        const float* t = xyz + i * vstride;
        if (mode == MVSV_PLY_WITH_COLOR) {
            out << t[0] << " " << t[1] << " " << t[2] << " ";
            const int g = int((t[2] - mn) / (mx - mn) * 255.0);
            out << g << " " << g << " " << g << "\n";
        } else {
            out << t[0] << " " << t[1] << " " << t[2] << "\n";
        }
    }
    return out ? MVSV_OK : MVSV_E_IO;
}

// [Utility::dmap2pcl] src/utility.cpp:242-262
int mvsv_dmap2pcl(mvsv_ctx* ctx, const char* path, const int16_t* dmap, size_t st, int W, int H,
                  const float* Q)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!path || !dmap || !Q || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad dmap2pcl arguments");
    DeviceGuard dev_guard(ctx->device);
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = ensure(ctx, ctx->h_out, px * 2, "dmap staging"))) return rc;
    if ((rc = ensure(ctx, ctx->h_left, px * 16, "point staging"))) return rc;
    hipStream_t s = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(ctx->h_out.ptr, (size_t)W * 2, dmap, st * 2,
                                              (size_t)W * 2, H, hipMemcpyHostToDevice, s),
                        "H2D dmap")))
        return rc;
    if ((rc = reproject_device(ctx, 1, (const int16_t*)ctx->h_out.ptr, W, px, W, H, Q,
                               (float*)ctx->h_left.ptr, W, px)))
        return rc;
    std::vector<float> pts(px * 4);
    if ((rc = check_hip(ctx, hipMemcpyAsync(pts.data(), ctx->h_left.ptr, px * 16,
                                            hipMemcpyDeviceToHost, s),
                        "D2H points")) ||
        (rc = check_hip(ctx, hipStreamSynchronize(s), "hipStreamSynchronize")))
        return rc;
    size_t k = 0;
    for (size_t i = 0; i < px; i++)  // raster order, v > 0 (flag in the 4th float)
        if (pts[4 * i + 3] != 0.0f) {
            for (int j = 0; j < 4; j++) pts[4 * k + j] = pts[4 * i + j];
            k++;
        }
    rc = mvsv_write_ply(path, "Hagen Hiller", "disparity pointcloud", pts.data(), k, 4,
                        MVSV_PLY_WITH_COLOR, dmap, st, W, H);
    if (rc == MVSV_E_IO) return set_error(ctx, rc, std::string("cannot write ") + path);
    if (rc) return set_error(ctx, rc, "dmap2pcl: map has no positive disparity");
    return MVSV_OK;
}

// ---- rectification ------------------------------------------

int mvsv_remap_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw,
                      int sh, const float* mx, const float* my, size_t ms, uint8_t* dst, size_t ds,
                      size_t dfs, int dw, int dh)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !src || !mx || !my || !dst || sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 ||
        ss < (size_t)sw || ds < (size_t)dw || ms < (size_t)dw)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad remap arguments");
    DeviceGuard dev_guard(ctx->device);
    return remap_device(ctx, n, src, ss, sfs, sw, sh, mx, my, ms, dst, ds, dfs, dw, dh);
}

// [Stereosystem::getRectifiedImagepair] src/Stereosystem.cpp:243-262
int mvsv_rectify_pair(mvsv_ctx* ctx, const uint8_t* L, size_t ls, const uint8_t* R, size_t rs,
                      int W, int H, const float* const* maps, const mvsv_rect* roi, uint8_t* oL,
                      size_t ols, uint8_t* oR, size_t ors)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!L || !R || !maps || !roi || !oL || !oR || W <= 0 || H <= 0 || ls < (size_t)W ||
        rs < (size_t)W || roi->x0 < 0 || roi->y0 < 0 || roi->x1 > W || roi->y1 > H ||
        roi->x1 <= roi->x0 || roi->y1 <= roi->y0 || ols < (size_t)(roi->x1 - roi->x0) ||
        ors < (size_t)(roi->x1 - roi->x0))
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad rectification arguments");
    for (int i = 0; i < 4; i++)
        if (!maps[i]) return set_error(ctx, MVSV_E_INVALID_ARG, "null map");
    DeviceGuard dev_guard(ctx->device);
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = ensure(ctx, ctx->h_left, 2 * px, "rectify staging")) ||
        (rc = ensure(ctx, ctx->h_right, 2 * px, "rectify staging")) ||
        (rc = ensure(ctx, ctx->h_out, 4 * px * sizeof(float), "rectify maps")))
        return rc;
    uint8_t* dsrc = (uint8_t*)ctx->h_left.ptr;   // [2][H][W] inputs
    uint8_t* ddst = (uint8_t*)ctx->h_right.ptr;  // [2][H][W] outputs
    float* dmap = (float*)ctx->h_out.ptr;         // [4][H][W]
    hipStream_t s = ctx->stream;
    const uint8_t* ins[2] = {L, R};
    const size_t istr[2] = {ls, rs};
    for (int i = 0; i < 2; i++)
        if ((rc = check_hip(ctx, hipMemcpy2DAsync(dsrc + i * px, W, ins[i], istr[i], W, H,
                                                  hipMemcpyHostToDevice, s), "H2D image")))
            return rc;
    for (int i = 0; i < 4; i++)
        if ((rc = check_hip(ctx, hipMemcpyAsync(dmap + i * px, maps[i], px * sizeof(float),
                                                hipMemcpyHostToDevice, s), "H2D map")))
            return rc;
    for (int i = 0; i < 2; i++)
        if ((rc = remap_device(ctx, 1, dsrc + i * px, W, px, W, H, dmap + (2 * i) * px,
                               dmap + (2 * i + 1) * px, W, ddst + i * px, W, px, W, H)))
            return rc;
    const int cw = roi->x1 - roi->x0, ch = roi->y1 - roi->y0;
    uint8_t* outs[2] = {oL, oR};
    const size_t ostr[2] = {ols, ors};
    for (int i = 0; i < 2; i++)
        if ((rc = check_hip(ctx, hipMemcpy2DAsync(outs[i], ostr[i],
                                                  ddst + i * px + (size_t)roi->y0 * W + roi->x0, W, cw,
                                                  ch, hipMemcpyDeviceToHost, s), "D2H image")))
            return rc;
    return check_hip(ctx, hipStreamSynchronize(s), "hipStreamSynchronize");
}

// [cv::initUndistortRectifyMap] (OpenCV 3.4 undistort.cpp), CV_32FC1 output
int mvsv_init_undistort_rectify_map(const double* K, const double* dist, int ndist,
                                    const double* Rm, const double* P, int W, int H, float* mx,
                                    float* my, size_t ms)
{
    if (!K || !P || !mx || !my || W <= 0 || H <= 0 || ms < (size_t)W ||
        !(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8) || (ndist && !dist))
        return MVSV_E_INVALID_ARG;
    const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double* R = Rm ? Rm : I3;
    // A = P[:, :3] * R; iR = A^-1
    double A[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) acc += P[i * 3 + k] * R[k * 3 + j];
            A[i * 3 + j] = acc;
        }
    const double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                       A[2] * (A[3] * A[7] - A[4] * A[6]);
    if (det == 0) return MVSV_E_INVALID_ARG;
    double ir[9] = {(A[4] * A[8] - A[5] * A[7]) / det, (A[2] * A[7] - A[1] * A[8]) / det,
                    (A[1] * A[5] - A[2] * A[4]) / det, (A[5] * A[6] - A[3] * A[8]) / det,
                    (A[0] * A[8] - A[2] * A[6]) / det, (A[2] * A[3] - A[0] * A[5]) / det,
                    (A[3] * A[7] - A[4] * A[6]) / det, (A[1] * A[6] - A[0] * A[7]) / det,
                    (A[0] * A[4] - A[1] * A[3]) / det};
    double k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < ndist; i++) k[i] = dist[i];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
    const double u0 = K[2], v0 = K[5], fx = K[0], fy = K[4];
    for (int i = 0; i < H; i++) {
        float* m1 = mx + (size_t)i * ms;
        float* m2 = my + (size_t)i * ms;
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double u = fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2)) + u0;
            const double v = fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy) + v0;
            m1[j] = (float)u;
            m2[j] = (float)v;
        }
    }
    return MVSV_OK;
}
