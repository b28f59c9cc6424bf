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
#include <functional>
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
    ++ctx->alloc_epoch;  // captured graphs hold the old addresses
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
    // one read-and-clear: a give-up stored by a launch still in flight between a
    // separate load and store would be erased unreported
    const int v = __atomic_exchange_n(ctx->report, 0, __ATOMIC_ACQ_REL);
    if (v == 0) return MVSV_OK;
    return set_error(ctx, MVSV_E_TIMEOUT,
                     "sgbm path kernel: a strip-boundary wait gave up (that launch's maps are all "
                     "INVALID)");
}

int mark_last_use(mvsv_ctx* ctx, int rc)
{
    if (hipEventRecord(ctx->ev_last, ctx->stream) != hipSuccess) {
        (void)hipGetLastError();
        return rc ? rc : set_error(ctx, MVSV_E_HIP, "last-use event record failed");
    }
    ctx->last_valid = true;
    return rc;
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

static void drop_graphs(mvsv_ctx* ctx)
{
    for (auto& g : ctx->graph_cache)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    ctx->graph_cache.clear();
    ctx->graph_seen.clear();
}

// Replay of repeated small launches as HIP graphs.  `key` holds every argument
// of the call; the first call with a key runs eagerly, an immediate repeat is
// captured (on the context's capture stream, so a caller on the legacy null
// stream is served too) and every later one launches the instantiated graph on
// the context stream.  Any failure of the capture path turns graphs off for the
// context and runs the call eagerly.
constexpr size_t kGraphCache = 4;
static int graph_run(mvsv_ctx* ctx, const std::vector<unsigned char>& key, const std::function<int()>& body)
{
    for (auto& g : ctx->graph_cache) {
        if (g.key != key) continue;
        if (g.epoch == ctx->alloc_epoch) {
            g.used = ++ctx->graph_clock;
            return check_hip(ctx, hipGraphLaunch(g.exec, ctx->stream), "graph launch");
        }
        (void)hipGraphExecDestroy(g.exec);  // its buffers were reallocated
        g.exec = nullptr;
        g.key.clear();
    }
    if (ctx->graph_seen != key) {
        ctx->graph_seen = key;
        return body();
    }
    static const bool dbg = std::getenv("MVSV_GRAPH_DEBUG") != nullptr;
    auto fail = [&]() {
        const hipError_t le = hipGetLastError();
        if (dbg) std::fprintf(stderr, "[mvsv graph] capture failed (%s); graphs off for this context\n",
                              hipGetErrorString(le));
        ctx->graphs = 0;
        ctx->graph_seen.clear();
        return body();
    };
    if (!ctx->cap && hipStreamCreateWithFlags(&ctx->cap, hipStreamNonBlocking) != hipSuccess) return fail();
    const unsigned ep = ctx->alloc_epoch;
    if (hipStreamBeginCapture(ctx->cap, hipStreamCaptureModeRelaxed) != hipSuccess) return fail();
    hipStream_t keep = ctx->stream;
    ctx->stream = ctx->cap;
    const int rc = body();
    ctx->stream = keep;
    hipGraph_t graph = nullptr;
    const hipError_t ce = hipStreamEndCapture(ctx->cap, &graph);
    hipGraphExec_t exec = nullptr;
    const bool ok = rc == MVSV_OK && ce == hipSuccess && graph && ctx->alloc_epoch == ep &&
                    hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
    if (graph) (void)hipGraphDestroy(graph);
    if (!ok) return fail();
    // keep the kGraphCache most recently used graphs
    auto slot = ctx->graph_cache.end();
    for (auto it = ctx->graph_cache.begin(); it != ctx->graph_cache.end(); ++it)
        if (!it->exec) slot = it;
    if (slot == ctx->graph_cache.end() && ctx->graph_cache.size() >= kGraphCache) {
        slot = std::min_element(ctx->graph_cache.begin(), ctx->graph_cache.end(),
                                [](const mvsv_ctx::GraphEntry& a, const mvsv_ctx::GraphEntry& b) {
                                    return a.used < b.used;
                                });
        (void)hipGraphExecDestroy(slot->exec);
    }
    if (slot == ctx->graph_cache.end()) {
        ctx->graph_cache.emplace_back();
        slot = ctx->graph_cache.end() - 1;
    }
    slot->key = key;
    slot->exec = exec;
    slot->epoch = ep;
    slot->used = ++ctx->graph_clock;
    ctx->graph_seen.clear();
    if (dbg)
        std::fprintf(stderr, "[mvsv graph] captured a %zu-byte key, %zu cached\n", key.size(),
                     ctx->graph_cache.size());
    return check_hip(ctx, hipGraphLaunch(exec, ctx->stream), "graph launch");
}

template <typename T>
static void key_put(std::vector<unsigned char>& k, const T& v)
{
    const unsigned char* p = reinterpret_cast<const unsigned char*>(&v);
    k.insert(k.end(), p, p + sizeof(T));
}

extern "C" {

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
        hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming) != hipSuccess ||
        alloc_report(c, 1, &c->report, &c->report_dev) != MVSV_OK) {
        (void)hipGetLastError();
        if (c->ev_last) (void)hipEventDestroy(c->ev_last);
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
        if (std::strstr(v, "bm-tile")) c->bm2 = 0;
        if (std::strstr(v, "cost-generic")) c->cost_fixed_pp = 0;
    }
    if (const char* v = std::getenv("MVSV_COST_TY")) c->cost_ty = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("MVSV_PATH_SCHEDULE")) c->path_sched = std::max(0, std::min(2, std::atoi(v)));
    if (const char* v = std::getenv("MVSV_STRIP_WAVES")) c->strip_waves = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("MVSV_TRI32")) c->tri32 = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_FINAL_SPLIT")) c->final_split = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_COST_RESIDUAL")) c->cost_res = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_BM_TY")) c->bm_ty = std::max(0, std::min(128, std::atoi(v)));
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, hip_device) != hipSuccess) {
        (void)hipGetLastError();
        c->cus = 256;
    }
    if (const char* v = std::getenv("MVSV_STRIP_ORDER")) c->strip_tickets = std::strcmp(v, "blockidx") != 0;
    if (const char* v = std::getenv("MVSV_LINES_AUX")) c->lines_aux = std::max(-1, std::min(2, std::atoi(v)));
    if (const char* v = std::getenv("MVSV_BITSLICE")) c->bitslice = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_GRAPHS")) c->graphs = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_BS_SERIAL")) c->bs_serial = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_COST_XCD")) c->cost_xcd = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_BS_FUSE")) c->bs_fuse = std::atoi(v) != 0;
    if (const char* v = std::getenv("MVSV_BS_GROUPS")) {
        const int g = std::atoi(v);
        c->bs_groups = (g >= 1 && g <= 5) ? g : 0;
    }
    *out = c;
    return MVSV_OK;
}

static void free_buf(DevBuf& b)
{
    if (b.ptr) (void)hipFree(b.ptr);  // (the caller bumps alloc_epoch)
    b.ptr = nullptr;
    b.bytes = 0;
}

int mvsv_trim(mvsv_ctx* ctx)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    ++ctx->alloc_epoch;
    DeviceGuard dev_guard(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    DevBuf* all[] = {&ctx->pre, &ctx->cost, &ctx->cres, &ctx->agg, &ctx->raw, &ctx->uf_parent, &ctx->uf_size, &ctx->uf_lroot, &ctx->uf_list,
                     &ctx->uf_tile, &ctx->tri_bnd, &ctx->bs_bnd, &ctx->status,
                     &ctx->dummy, &ctx->keys,
                     &ctx->bm_lf, &ctx->bm_rf, &ctx->bm_cost, &ctx->bm_sad, &ctx->h_left, &ctx->h_right,
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
    drop_graphs(ctx);
    mvsv_trim(ctx);
    if (ctx->cap) (void)hipStreamDestroy(ctx->cap);
    mvsv_profile_reset(ctx);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_last) (void)hipEventDestroy(ctx->ev_last);
    if (ctx->report) (void)hipHostFree(ctx->report);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    delete ctx;
}

const char* mvsv_last_error(const mvsv_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// Every launch of a context shares its cached buffers, so work enqueued on a
// new stream must not start before the context's work already enqueued: the
// new stream waits on the context's last-use event (recorded by the entry
// points themselves, so neither the previous stream handle -- possibly
// destroyed by its owner since -- nor unrelated work queued on it is touched).
static int switch_stream(mvsv_ctx* ctx, hipStream_t s)
{
    if (s == ctx->stream) return MVSV_OK;
    DeviceGuard dev_guard(ctx->device);
    if (ctx->last_valid) {
        int rc = check_hip(ctx, hipStreamWaitEvent(s, ctx->ev_last, 0), "stream switch wait");
        if (rc) return rc;
    }
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
    case MVSV_OPT_BM_TILE_ROWS:
        if (value < 0 || value > 128) return set_error(ctx, MVSV_E_INVALID_ARG, "BM tile rows must be 0..128");
        ctx->bm_ty = (int)value;
        return MVSV_OK;
    case MVSV_OPT_PATH_SCHEDULE:
        if (value < 0 || value > 2) return set_error(ctx, MVSV_E_INVALID_ARG, "path schedule must be 0..2");
        ctx->path_sched = (int)value;
        return MVSV_OK;
    case MVSV_OPT_STRIP_WAVES:
        if (value < 0 || value > 64) return set_error(ctx, MVSV_E_INVALID_ARG, "strip waves must be 0..64");
        ctx->strip_waves = (int)value;
        return MVSV_OK;
    case MVSV_OPT_STRIP_TICKETS:
        if (value < 0 || value > 1) return set_error(ctx, MVSV_E_INVALID_ARG, "strip tickets must be 0 or 1");
        ctx->strip_tickets = (int)value;
        return MVSV_OK;
    case MVSV_OPT_COST_RESIDUAL:
        if (value < 0 || value > 1) return set_error(ctx, MVSV_E_INVALID_ARG, "cost residual must be 0 or 1");
        ctx->cost_res = (int)value;
        return MVSV_OK;
    case MVSV_OPT_BITSLICE:
        if (value < 0 || value > 1) return set_error(ctx, MVSV_E_INVALID_ARG, "bitslice must be 0 or 1");
        ctx->bitslice = (int)value;
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
    // speckle filter (speckle_buffers, mvsv_post.hip): parent, size and tile
    // words, u16 local roots and the compact root list (+ its count)
    if (e.speckle_window > 0) b += (size_t)n * frame * (4 + 4 + 4 + 2 + 4) + 4;
    // cost residual plane + per-pixel minimum (MVSV_OPT_COST_RESIDUAL, where exact)
    if (3 * e.P2 <= 15 && e.D <= 128 && e.W1 > 0) b += (size_t)n * e.W1 * H * (e.D / 2 + 2);
    // the BT interval planes of both views (u64 per pixel each)
    b += (size_t)n * frame * 16;
    // the bit-sliced pipeline (MVSV_OPT_BITSLICE, default on):
    // rows padded to 4 pixels, delta planes beyond the accumulator budget above
    // (eight 48-byte planes side by side for small launches), strip boundary
    // granules (2 passes x strips of 64 U-columns x H rows x 36 u64)
    const long bsz = 2L * e.SW2 + 1;
    const bool bs_regime = e.D == 128 && e.P1 == 2 && e.P2 == 5 && e.uniq == 0 && e.W1 > 0 &&
                           (long)e.P2 + bsz * bsz * (2L * e.ftzero + 63) + e.P2 <= 32767;
    if (bs_regime) {
        const size_t W1q = (size_t)(e.W1 + 3) & ~(size_t)3;
        b += (size_t)n * H * (W1q - e.W1) * (e.D * 2 + 64);               // padded C and C'
        const size_t side = (size_t)n * H * W1q * 8 * 48, acc = (size_t)n * vol;
        if (side > acc) b += side - acc;
        const size_t nstrips = ((size_t)e.W1 + H - 1 + 63) / 64;
        b += 2 * (size_t)n * nstrips * H * 36 * 8;
    } else if (e.P2 > 15 && e.W1 > 0) {
        // directions side by side on byte / u16 planes (round 6: the reference's
        // liveDisparity / captureDisparity shapes), one plane per direction
        // (D <= 32: R->L included), beyond the one-volume accumulator budget above
        const size_t planes = (e.fullDP ? 7 : 4) + (e.D <= 32 ? 1 : 0), ebytes = (e.fullDP ? 8 : 5) * e.P2 <= 255 ? 1 : 2;
        const size_t side = (size_t)n * e.W1 * H * e.D * planes * ebytes, acc = (size_t)n * vol;
        if (side > acc) b += side - acc;
    }
    return b;
}

int mvsv_sgbm_plan(mvsv_ctx* ctx, int n, int W, int H, const mvsv_sgbm_params* p, int* plan)
{
    if (!ctx || !plan || n <= 0) return MVSV_E_INVALID_ARG;
    SgbmEff e;
    std::string why;
    const int rc = resolve_sgbm(p, W, H, &e, &why);
    if (rc) return set_error(ctx, rc, why);
    *plan = sgbm_plan(ctx, e, n, H);
    return MVSV_OK;
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
    auto body = [&]() { return sgbm_device(ctx, n, L, ls, lfs, R, rs, rfs, W, H, e, out, os, ofs); };
    // small launches (one camera frame): one graph launch instead of ~8 kernel
    // launches (config 3, one 640x480 frame: ~5 us of launch gap per kernel)
    if (ctx->graphs && !ctx->prof && sgbm_graphable(ctx, e, n, H)) {
        std::vector<unsigned char> key;
        key_put(key, 'S');
        key_put(key, n);
        key_put(key, L);
        key_put(key, ls);
        key_put(key, lfs);
        key_put(key, R);
        key_put(key, rs);
        key_put(key, rfs);
        key_put(key, W);
        key_put(key, H);
        key_put(key, e);
        key_put(key, out);
        key_put(key, os);
        key_put(key, ofs);
        return mark_last_use(ctx, graph_run(ctx, key, body));
    }
    return mark_last_use(ctx, body());
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
    auto body = [&]() { return bm_device(ctx, n, L, ls, lfs, R, rs, rfs, W, H, e, out, os, ofs); };
    // StereoBM launches carry no per-launch state: repeats replay as a graph
    // (config 2, one 640x480 frame: 0.045 ms per call, ~6 kernel launches)
    if (ctx->graphs && !ctx->prof) {
        std::vector<unsigned char> key;
        key_put(key, 'B');
        key_put(key, n);
        key_put(key, L);
        key_put(key, ls);
        key_put(key, lfs);
        key_put(key, R);
        key_put(key, rs);
        key_put(key, rfs);
        key_put(key, W);
        key_put(key, H);
        key_put(key, e);
        key_put(key, out);
        key_put(key, os);
        key_put(key, ofs);
        return mark_last_use(ctx, graph_run(ctx, key, body));
    }
    return mark_last_use(ctx, body());
}

int mvsv_mean_disparity_grid_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st,
                                    size_t fs, int W, int H, float* means)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !dmap || !means || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad mean-grid arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, mean_grid_device(ctx, n, dmap, st, fs, W, H, means));
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
    // every exit after the first enqueue records the context's last-use event,
    // so a later stream switch waits for whatever this call left queued
    return mark_last_use(ctx, [&]() -> int {
    int rc;
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
    // only an SGBM call reads the sticky give-up word: a BM call's valid map is
    // returned and the word waits for the next SGBM call or mvsv_synchronize
    return sgbm ? check_report(ctx) : MVSV_OK;
    }());
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

}  // extern "C"

// ---- reprojection and PLY output -------------------------

int mvsv_reproject_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W,
                          int H, const float* Q, float* xyzw, size_t xs, size_t xfs)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (n <= 0 || !dmap || !Q || !xyzw || W <= 0 || H <= 0 || st < (size_t)W || xs < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad reprojection arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, reproject_device(ctx, n, dmap, st, fs, W, H, Q, xyzw, xs, xfs));
}

// [Utility::dmap2pcl] src/utility.cpp:242-262
int mvsv_dmap2pcl(mvsv_ctx* ctx, const char* path, const int16_t* dmap, size_t st, int W, int H,
                  const float* Q)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    if (!path || !dmap || !Q || W <= 0 || H <= 0 || st < (size_t)W)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad dmap2pcl arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, [&]() -> int {
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
    }());
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
    return mark_last_use(ctx, remap_device(ctx, n, src, ss, sfs, sw, sh, mx, my, ms, dst, ds, dfs, dw, dh));
}

int mvsv_resize_size(int sw, int sh, double fx, double fy, int* dw, int* dh)
{
    if (!dw || !dh) return MVSV_E_INVALID_ARG;
    return resize_size(sw, sh, fx, fy, dw, dh);
}

// [cv::resize in Stereosystem::getRectifiedImagepair(Stereopair&, float)] src/Stereosystem.cpp:279-315
int mvsv_resize_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw, int sh,
                       double fx, double fy, uint8_t* dst, size_t ds, size_t dfs)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    int dw, dh;
    if (n <= 0 || !src || !dst || ss < (size_t)std::max(sw, 0) || resize_size(sw, sh, fx, fy, &dw, &dh))
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad resize arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, resize_device(ctx, n, src, ss, sfs, sw, sh, fx, fy, dst, ds, dfs));
}

int mvsv_resize(mvsv_ctx* ctx, const uint8_t* src, size_t ss, int sw, int sh, double fx, double fy,
                uint8_t* dst, size_t ds)
{
    if (!ctx) return MVSV_E_INVALID_ARG;
    int dw, dh;
    if (!src || !dst || ss < (size_t)std::max(sw, 0) || resize_size(sw, sh, fx, fy, &dw, &dh) ||
        ds < (size_t)dw)
        return set_error(ctx, MVSV_E_INVALID_ARG, "bad resize arguments");
    DeviceGuard dev_guard(ctx->device);
    return mark_last_use(ctx, [&]() -> int {
    const size_t in = (size_t)sw * sh, outb = (size_t)dw * dh;
    int rc;
    if ((rc = ensure(ctx, ctx->h_left, in, "resize staging")) ||
        (rc = ensure(ctx, ctx->h_right, outb, "resize staging")))
        return rc;
    hipStream_t s = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpy2DAsync(ctx->h_left.ptr, sw, src, ss, sw, sh, hipMemcpyHostToDevice, s),
                        "H2D image")) ||
        (rc = resize_device(ctx, 1, (const uint8_t*)ctx->h_left.ptr, sw, in, sw, sh, fx, fy,
                            (uint8_t*)ctx->h_right.ptr, dw, outb)) ||
        (rc = check_hip(ctx, hipMemcpy2DAsync(dst, ds, ctx->h_right.ptr, dw, dw, dh, hipMemcpyDeviceToHost, s),
                        "D2H image")))
        return rc;
    return check_hip(ctx, hipStreamSynchronize(s), "hipStreamSynchronize");
    }());
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
    return mark_last_use(ctx, [&]() -> int {
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
    }());
}

