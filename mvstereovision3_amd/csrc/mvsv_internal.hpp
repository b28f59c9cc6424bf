// mvsv_internal.hpp — shared declarations of libmvsv (host + HIP kernels).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mvsv.h"

namespace mvsv {

constexpr int kMaxCost = 32767;    // OpenCV StereoSGBM MAX_COST (SHRT_MAX)
constexpr int kDispShift = 4;      // StereoMatcher::DISP_SHIFT
constexpr int kDispScale = 16;

// Effective StereoSGBM parameters after OpenCV's defaulting rules
// ([OpenCV] computeDisparitySGBM prologue).
struct SgbmEff {
    int minD, maxD, D;
    int SW2, SH2;
    int ftzero;
    int uniq, disp12;
    int P1, P2;
    int minX1, maxX1, W1;
    int invalid;  // (minD - 1) * 16
    int fullDP;   // MODE_HH
    int variant;
    int speckle_window, speckle_diff;  // speckle_diff = 16 * speckleRange
};

struct BmEff {
    int ndisp, mindisp, wsz2, cap, tex, uniq;
    int lofs, rofs, width1, ncol;
    int xmin, xmax, ymin, ymax;  // validDisparityRect (half-open)
    int filtered;                // (minD - 1) << 4
    int disp12;                  // < 0: off
    int speckle_window, speckle_range;
    int prefilter_type, prefilter_size;
};

// Resolve + validate (OpenCV's asserts). Return MVSV_OK or MVSV_E_INVALID_ARG
// and an explanation in *why.
int resolve_sgbm(const mvsv_sgbm_params* p, int W, int H, SgbmEff* e, std::string* why);
int resolve_bm(const mvsv_bm_params* p, int W, int H, BmEff* e, std::string* why);

// Grow-only cached device buffer.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
};

// Entry points switch to the context's device and give the caller's current
// device back on return (a compute on cuda:1 must not change the thread's
// device under the torch code that runs next).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Default number of polls a strip-boundary wait of the sheared-strip kernel
// makes before it gives up (each poll = one s_sleep + one L2 load of the
// producer's granule, ~1 us): ~1 s, far beyond any producer delay of a
// healthy launch; the wait only exists to turn a lost hand-off into an error
// instead of a hang.  mvsv_set_option(MVSV_OPT_STRIP_SPIN_LIMIT) overrides it.
constexpr unsigned kStripSpinLimitDefault = 1u << 20;

}  // namespace mvsv

struct mvsv_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // SGBM
    mvsv::DevBuf pre, cost, cres, agg, raw, uf_parent, uf_size, uf_tile, uf_lroot, uf_list, dummy, keys, tri_bnd, bs_bnd, status;
    bool uf_list_dirty = false;  // a speckle run launched its first stage but not its last
    // launch number of the last sheared-strip launch: its low 16 bits tag the
    // boundary granules (tri_bnd is re-zeroed whenever they wrap), all 32 bits
    // go into status[0] when that launch gives up a wait (no per-call reset)
    unsigned tri_epoch = 0;
    // strip blocks draw their strip as a ticket (status[2]) unless strip_tickets
    // is 0 (blockIdx order, MVSV_STRIP_ORDER=blockidx); tri_tickets = the first
    // ticket of the next launch (the counter is zeroed with the status word)
    int strip_tickets = 1;
    unsigned tri_tickets = 0;
    unsigned spin_limit = mvsv::kStripSpinLimitDefault;
    // given-up strip waits are reported into host-mapped ints: `report` is the
    // context's sticky word (device calls; read and cleared by the next call,
    // mvsv_synchronize and the host-pointer calls), report_target is where the
    // next launches report (a frame stream points it at its run's own word)
    int* report = nullptr;      // host view
    int* report_dev = nullptr;  // device view of report
    int* report_target = nullptr;
    // context-owned "last use" event: recorded on ctx->stream at the end of every
    // enqueueing entry point; a stream switch makes the new stream wait on it
    // (never records on the previous stream handle, which the caller may have
    // destroyed since)
    hipEvent_t ev_last = nullptr;
    bool last_valid = false;
    hipStream_t aux = nullptr;  // second stream for concurrent direction passes
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int path16 = 1;  // 16-lanes-per-scanline path kernels where D allows
    int cost2 = 1;   // register-ring cost kernel where blockSize <= 15
    int cost_fixed_pp = 1;  // fixed-pair-count cost kernels for D = 128 / 256 (MVSV_KERNELS=cost-generic: off)
    int cost_ty = 0;  // cost-volume tile height (0 = by image height); MVSV_COST_TY for A/B runs
    int tri = 1;     // sheared-strip kernels: three directions per sweep
    int path_sched = 0;   // 16-lane path schedule: 0 = by launch size, 1 = strips, 2 = directions side by side
    int tri32 = 1;
    int final_split = 1;  // side by side on byte / u16 planes: R->L as a chain set + per-pixel WTA (MVSV_FINAL_SPLIT)
    int tri_xseg = 0;     // A/B: one strip chain's neighbours on one XCD (MVSV_TRI_XSEG)        // D = 256 narrow strips on 32 lanes per column (MVSV_TRI32)
    int strip_waves = 0;  // compute waves per strip (0 = by launch size; 4 or the wide count forces)
    int cost_res = 1;     // direction passes read the cost residual plane where exact (MVSV_OPT_COST_RESIDUAL)
    int lines_aux = -1;  // L->R line kernel beside the strip kernel: -1 = small launches only, 0 / 1 / 2 force
    int bitslice = 1;    // bit-sliced MODE_HH paths where they apply (MVSV_OPT_BITSLICE, env MVSV_BITSLICE)
    int bs_groups = 0;   // column groups (3 direction waves each) per bit-sliced strip: 1-5 (MVSV_BS_GROUPS), 0 = by mode
    int cost_xcd = 1;    // cost kernel: whole row bands per XCD (MVSV_COST_XCD=0: blockIdx order, A/B)
    int bs_fuse = 1;     // bit-sliced batches: R->L lines fused with the WTA (MVSV_BS_FUSE=0: separate, A/B)
    int bs_serial = 0;   // 1: bit-sliced line kernel after the strips on the context stream (MVSV_BS_SERIAL, A/B)
    int bm2 = 1;     // StereoBM: disparities-on-lanes match kernel where blockSize <= 21, D <= 128
    int bm_ty = 0;   // its tile height (0 = chosen per launch); MVSV_BM_TY for A/B runs
    int cus = 256;   // compute units of the device (launch-shape choices)
    // HIP graphs (round 6): a small SGBM launch (no strip chain, whose launches
    // carry per-launch epochs) repeated with the same arguments is captured once
    // on the capture stream and then replayed as one graph launch; every cached
    // buffer (re)allocation or free bumps alloc_epoch and retires the graphs
    // measured slower than eager launches on ROCm 7.2 / MI355X (config 3 one
    // frame 0.259 vs 0.250 ms, config 2 0.041 vs 0.033 ms; profiles/r06/graphs),
    // so opt-in: MVSV_GRAPHS=1
    int graphs = 0;
    unsigned alloc_epoch = 0;
    struct GraphEntry {
        std::vector<unsigned char> key;
        hipGraphExec_t exec = nullptr;
        unsigned epoch = 0;
        unsigned long long used = 0;
    };
    std::vector<GraphEntry> graph_cache;
    std::vector<unsigned char> graph_seen;  // arguments of the last eager launch
    unsigned long long graph_clock = 0;
    hipStream_t cap = nullptr;  // capture stream
    // BM
    mvsv::DevBuf bm_lf, bm_rf, bm_cost, bm_sad;
    // host-pointer staging
    mvsv::DevBuf h_left, h_right, h_out;
    // stage profiling (HIP events on the context stream)
    int prof = 0;
    struct Mark {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Mark> marks;
    std::vector<hipEvent_t> event_pool;
};

namespace mvsv {

int set_error(mvsv_ctx* ctx, int code, const std::string& msg);
int ensure(mvsv_ctx* ctx, DevBuf& b, size_t bytes, const char* what);
int check_hip(mvsv_ctx* ctx, hipError_t e, const char* what);
// Reads and clears the context's sticky report word: MVSV_E_TIMEOUT if a
// strip-boundary wait of an earlier launch gave up.  No synchronisation.
int check_report(mvsv_ctx* ctx);
// Host-mapped int (host and device views), zeroed.
int alloc_report(mvsv_ctx* ctx, int count, int** host, int** dev);
// Records the context's last-use event on ctx->stream after an entry point
// enqueued work (keeps rc: an error code passes through unchanged).
int mark_last_use(mvsv_ctx* ctx, int rc);

enum Stage {
    kStagePre = 0,
    kStageCost,
    kStageFixup,
    kStagePath,
    kStageFinal,
    kStagePost,
    kStageBm,
    kStageStrips,
    kStageLines
};
// RAII: records a start / stop event pair around the launches in its scope
// when profiling is enabled (no-op otherwise).
struct StageTimer {
    mvsv_ctx* ctx;
    int stage;
    hipStream_t st;  // stream the events are recorded on (default: the context stream)
    hipEvent_t a = nullptr, b = nullptr;
    StageTimer(mvsv_ctx* c, int s, hipStream_t on = nullptr);
    ~StageTimer();
};

// Device pipelines (defined in the .hip translation units). All enqueue on
// ctx->stream. Strides are in elements.
int sgbm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R,
                size_t rs, size_t rfs, int W, int H, const SgbmEff& e, int16_t* out, size_t os,
                size_t ofs);
// the launch runs no strip chain (path schedule 2): its kernels and arguments are
// the same on every call with the same arguments, so it may be replayed as a graph
bool sgbm_graphable(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H);
// MVSV_PLAN_* bits of the pipeline sgbm_device runs for these arguments
int sgbm_plan(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H);
// the register-ring cost kernel runs (and can write the bit-sliced planes)
bool cost2_runs(const mvsv_ctx* ctx, const SgbmEff& e);
int bm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R,
              size_t rs, size_t rfs, int W, int H, const BmEff& e, int16_t* out, size_t os,
              size_t ofs);
// SGBM stages 1-3 (mvsv_cost.hip): BT interval planes, the cost volume (the
// register-ring kernel also writes the residual plane *Rv or the bit-sliced C'
// planes *Bv where given and possible -- each is set to nullptr otherwise), and
// OpenCV 3.4's cost-row quirks on the int16 volume.
int launch_prefilter(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R, size_t rs,
                     size_t rfs, int W, int H, int ftzero, uint64_t* pre);
int launch_cost(mvsv_ctx* ctx, int n, int W, int H, const SgbmEff& e, int TY, const uint64_t* pre, int16_t* Cv,
                uint8_t** Rv, uint16_t* Mv, bool* pinned_hh, uint32_t** Bv);
int launch_cost_fixup(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, int16_t* Cv, uint8_t* Rv, uint16_t* Mv);
// Post filters shared by both matchers.
// poison != nullptr: when *poison == epoch (the launch `epoch` gave up a strip
// wait) every output pixel is `invalid` instead of the median -- no map computed
// from stale hand-off data leaves the pipeline.
// Bit-sliced path aggregation + WTA, MODE_HH and MODE_SGBM (mvsv_bsgm.hip).  bsgm_eligible:
// the parameters admit it; the cost kernel then writes the C' planes Bv
// (bsgm_plane_bytes) and bsgm_paths computes raw disparities from them.
bool bsgm_eligible(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H);
size_t bsgm_plane_bytes(int n, int H, int W1);
int bsgm_paths(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, const int16_t* Cv, const uint32_t* Bv,
               const uint16_t* Mv, int16_t* raw, bool side);
// MODE_SGBM's never-recomputed rows and column 0 on the bit-sliced layouts (C'
// planes, pixel-quad C, m); no-op for MODE_HH, whose cost kernel pins them
int bsgm_cost_fixup(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, int16_t* Cv, uint32_t* Bv, uint16_t* Mv);
int median3x3_device(mvsv_ctx* ctx, int n, const int16_t* src, size_t ss, size_t sfs,
                     int16_t* dst, size_t ds, size_t dfs, int W, int H,
                     const int* poison = nullptr, unsigned epoch = 0, int invalid = 0);
int speckle_device(mvsv_ctx* ctx, int n, int16_t* img, size_t st, size_t fs, int W, int H,
                   int new_val, int max_size, int max_diff);

int remap_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw, int sh,
                 const float* mx, const float* my, size_t ms, uint8_t* dst, size_t ds, size_t dfs,
                 int dw, int dh);
// cv::resize INTER_LINEAR (CV_8UC1) output size / launch (mvsv_post.hip)
int resize_size(int sw, int sh, double fx, double fy, int* dw, int* dh);
int resize_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw, int sh, double fx,
                  double fy, uint8_t* dst, size_t ds, size_t dfs);
int reproject_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W, int H,
                     const float* Q, float* out, size_t os, size_t ofs);
int mean_grid_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W,
                     int H, float* means);

}  // namespace mvsv
