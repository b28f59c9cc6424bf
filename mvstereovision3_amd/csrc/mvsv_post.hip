// mvsv_post.hip — post-filters of the disparity path on MI355X:
//   * 3x3 median, replicate border  ([OpenCV] medianBlur(disp, disp, 3), applied
//     by StereoSGBM::compute after the core)
//   * speckle filter                ([OpenCV] filterSpeckles, CV_16S): 4-connected
//     components of pixels != newVal whose neighbours differ by <= maxDiff;
//     components of size <= maxSpeckleSize become newVal.  Computed with a
//     lock-free union-find (atomicMin linking towards the smaller index), which
//     yields exactly the same components as OpenCV's raster-order flood fill.
//   * MeanDisparityDetection grid   (src/MeanDisparityDetection.cpp:159-206,
//     Utility::calcMeanDisparity src/utility.cpp:265-285)
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "mvsv_device.hpp"
#include "mvsv_internal.hpp"

namespace mvsv {
namespace {

using namespace dev;

__device__ __forceinline__ void sort2(int& a, int& b)
{
    int lo = min(a, b), hi = max(a, b);
    a = lo;
    b = hi;
}

// median of 9 with the 19-exchange network (Paeth / Devillard opt_med9)
__device__ __forceinline__ int med9(int p0, int p1, int p2, int p3, int p4, int p5, int p6, int p7,
                                    int p8)
{
    sort2(p1, p2); sort2(p4, p5); sort2(p7, p8);
    sort2(p0, p1); sort2(p3, p4); sort2(p6, p7);
    sort2(p1, p2); sort2(p4, p5); sort2(p7, p8);
    sort2(p0, p3); sort2(p5, p8); sort2(p4, p7);
    sort2(p3, p6); sort2(p1, p4); sort2(p2, p5);
    sort2(p4, p7); sort2(p4, p2); sort2(p6, p4);
    sort2(p4, p2);
    return p4;
}

__global__ __launch_bounds__(256) void median3x3_kernel(const int16_t* __restrict__ src, size_t ss,
                                                        size_t sfs, int16_t* __restrict__ dst,
                                                        size_t ds, size_t dfs, int W, int H,
                                                        const int* __restrict__ poison,
                                                        unsigned epoch, int invalid)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (x >= W || y >= H) return;
    if (poison && __builtin_expect(*poison == (int)epoch, 0)) {
        dst[f * dfs + (size_t)y * ds + x] = (int16_t)invalid;
        return;
    }
    const int16_t* s = src + f * sfs;
    const int xm = max(x - 1, 0), xp = min(x + 1, W - 1);
    const int16_t* r0 = s + (size_t)max(y - 1, 0) * ss;
    const int16_t* r1 = s + (size_t)y * ss;
    const int16_t* r2 = s + (size_t)min(y + 1, H - 1) * ss;
    int m = med9(r0[xm], r0[x], r0[xp], r1[xm], r1[x], r1[xp], r2[xm], r2[x], r2[xp]);
    dst[f * dfs + (size_t)y * ds + x] = (int16_t)m;
}

// Two horizontally adjacent pixels per thread on packed int16 pairs
// (v_pk_min_i16 / v_pk_max_i16): the three taps of a row are the dwords
// (p[x-1], p[x]), (p[x], p[x+1]), (p[x+1], p[x+2]) made by v_alignbit from the
// aligned words at x - 2, x, x + 2 (replicate border).  Needs an even width,
// even strides and 4-byte-aligned rows (median3x3_device checks).
__device__ __forceinline__ void sort2p(uint32_t& a, uint32_t& b)
{
    const uint32_t lo = pk_min(a, b), hi = as_u(__builtin_elementwise_max(as_s2(a), as_s2(b)));
    a = lo;
    b = hi;
}

__global__ __launch_bounds__(256) void median3x3_pk_kernel(const int16_t* __restrict__ src, size_t ss,
                                                           size_t sfs, int16_t* __restrict__ dst,
                                                           size_t ds, size_t dfs, int W, int H,
                                                           const int* __restrict__ poison,
                                                           unsigned epoch, int invalid)
{
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);  // pixel pair (2i, 2i + 1)
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (2 * i >= W || y >= H) return;
    uint32_t* o = (uint32_t*)(dst + f * dfs + (size_t)y * ds) + i;
    if (poison && __builtin_expect(*poison == (int)epoch, 0)) {
        *o = (uint32_t)(invalid & 0xffff) * 0x10001u;
        return;
    }
    const int16_t* s = src + f * sfs;
    uint32_t t[9];
    const int rows[3] = {max(y - 1, 0), y, min(y + 1, H - 1)};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t* q = (const uint32_t*)(s + (size_t)rows[k] * ss);
        const uint32_t M = q[i];
        const uint32_t P = i > 0 ? q[i - 1] : M << 16;             // hi half = p[x - 1] (p[0] at x = 0)
        const uint32_t N = 2 * i + 2 < W ? q[i + 1] : M >> 16;     // lo half = p[x + 2] (p[W - 1] at the end)
        t[3 * k] = __builtin_amdgcn_alignbit(M, P, 16);
        t[3 * k + 1] = M;
        t[3 * k + 2] = __builtin_amdgcn_alignbit(N, M, 16);
    }
    // the 19-exchange network of med9 on both pixels at once
    sort2p(t[1], t[2]); sort2p(t[4], t[5]); sort2p(t[7], t[8]);
    sort2p(t[0], t[1]); sort2p(t[3], t[4]); sort2p(t[6], t[7]);
    sort2p(t[1], t[2]); sort2p(t[4], t[5]); sort2p(t[7], t[8]);
    sort2p(t[0], t[3]); sort2p(t[5], t[8]); sort2p(t[4], t[7]);
    sort2p(t[3], t[6]); sort2p(t[1], t[4]); sort2p(t[2], t[5]);
    sort2p(t[4], t[7]); sort2p(t[4], t[2]); sort2p(t[6], t[4]);
    sort2p(t[4], t[2]);
    *o = t[4];
}

// ---- speckle filter: union-find ----------------------------------------------
// Stage 1: union-find inside a 32x32 tile in LDS (one 256-thread block per
// tile, 4 pixels per thread).  Outputs: per pixel its tile-local root (u16, lroot; row-major
// local order is monotone in the global index, so a root is the smallest
// global index of its tile component); per tile component (at its root's
// global index gi): parent[gi] = gi, tilew[gi] = the component's pixel count,
// size[gi] = 0, and gi + frame * W * H appended to the compact root list.
constexpr int kSpTile = 32;

__device__ __forceinline__ int lds_load(const int* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ int lfind(int* par, int i)
{
    int p = lds_load(par + i);
    while (p != i) {
        int gp = lds_load(par + p);
        if (gp != p) atomicMin(par + i, gp);
        i = p;
        p = gp;
    }
    return i;
}

// the root without path compression: the lanes of a wave mostly walk the same
// chains, and the compressing atomicMin of lfind serialised them on one LDS
// address (0.51 of the kernel's LDS cycles were bank conflicts, round 5)
__device__ __forceinline__ int lroot_ro(const int* par, int i)
{
    int p = lds_load(par + i);
    for (;;) {
        const int q = lds_load(par + p);
        if (q == p) return p;
        p = q;
    }
}

__device__ void lunite(int* par, int a, int b)
{
    for (;;) {
        a = lfind(par, a);
        b = lfind(par, b);
        if (a == b) return;
        if (a > b) {
            int t = a;
            a = b;
            b = t;
        }
        int old = atomicMin(par + b, a);
        if (old == b) return;
        b = old;
    }
}

__global__ __launch_bounds__(256) void speckle_local_kernel(int16_t* __restrict__ img, size_t st, size_t fs,
                                                            int W, int H, int new_val, int max_diff,
                                                            int* __restrict__ parent,
                                                            int* __restrict__ tilew,
                                                            int* __restrict__ size,
                                                            uint16_t* __restrict__ lroot,
                                                            unsigned* __restrict__ list)
{
    __shared__ int lpar[kSpTile * kSpTile];
    __shared__ int lval[kSpTile * kSpTile];
    __shared__ int lcnt[kSpTile * kSpTile];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int lane = threadIdx.x & 63;
    const int x0 = blockIdx.x * kSpTile, y0 = blockIdx.y * kSpTile;
    const int f = blockIdx.z;
    const int kInvalid = 0x7fffffff;
    const int16_t* s = img + f * fs;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ly = ty + 8 * k, li = ly * kSpTile + tx;
        const int gx = x0 + tx, gy = y0 + ly;
        int v = kInvalid;
        if (gx < W && gy < H) {
            int t = s[(size_t)gy * st + gx];
            if (t != new_val) v = t;
        }
        lval[li] = v;
        lpar[li] = li;
        lcnt[li] = 0;
    }
    __syncthreads();
    // Horizontal runs without atomics: a wave holds two whole tile rows, so the
    // ballot of "connected to the right neighbour" gives each lane its run's
    // first pixel (the smallest index, so roots stay minimal), and every pixel
    // links straight to it.
    __shared__ unsigned hrow[kSpTile];  // bit x: (x, ly) -- (x + 1, ly) connected
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ly = ty + 8 * k, li = ly * kSpTile + tx;
        const int v = lval[li];
        const int u = tx + 1 < kSpTile ? lval[li + 1] : kInvalid;
        const bool h = v != kInvalid && u != kInvalid && abs(v - u) <= max_diff;
        const unsigned hm = (unsigned)(__ballot(h) >> (lane & 32));
        const unsigned starts = ~(hm << 1) & ((2u << tx) - 1u);  // run starts at or left of tx
        lpar[li] = ly * kSpTile + 31 - __clz(starts);
        if (tx == 0) hrow[ly] = hm;
    }
    __syncthreads();
    // Vertical links join runs; of a stretch of vertical links between the same
    // two runs only the leftmost one unites
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ly = ty + 8 * k, li = ly * kSpTile + tx;
        if (ly + 1 >= kSpTile) continue;
        const int v = lval[li], u = lval[li + kSpTile];
        if (v == kInvalid || u == kInvalid || abs(v - u) > max_diff) continue;
        if (tx > 0 && ((hrow[ly] & hrow[ly + 1]) >> (tx - 1) & 1u)) {
            const int vl = lval[li - 1], ul = lval[li + kSpTile - 1];
            if (abs(vl - ul) <= max_diff) continue;  // both valid: h bits set
        }
        lunite(lpar, li, li + kSpTile);
    }
    __syncthreads();
    int root[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ly = ty + 8 * k, li = ly * kSpTile + tx;
        root[k] = lval[li] != kInvalid ? lroot_ro(lpar, li) : -1;
        // component sizes by horizontal runs: a run (one root) adds its length
        // once, from its first pixel -- one LDS atomic per run instead of one
        // per pixel (same-address atomics of a smooth region serialise) or a
        // ballot loop over the wave's distinct roots (many in a noisy region)
        const unsigned hm = hrow[ly];
        const bool start = tx == 0 || !((hm >> (tx - 1)) & 1u);
        if (root[k] >= 0 && start) {
            const unsigned rest = ~(hm >> tx);  // bit j: (tx + j) not joined to its right neighbour
            atomicAdd(lcnt + root[k], __builtin_ctz(rest) + 1);
        }
    }
    __shared__ unsigned s_roots, s_base;
    if (threadIdx.x == 0) s_roots = 0u;
    __syncthreads();
    const size_t npix = (size_t)W * H;
    int* par = parent + f * npix;
    int* tl = tilew + f * npix;
    int* sz = size + f * npix;
    uint16_t* lr = lroot + f * npix;
    // the tile's components go to the compact root list (list[0] = count) with
    // ONE global atomic per block: every block appending per wave and row group
    // put 16 same-address L2 atomics per tile on list[0], serialised across the
    // whole launch (9 600 tiles per 8-frame step)
    unsigned long long rm[4];
    unsigned roff[4];
    int rgi[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ly = ty + 8 * k, li = ly * kSpTile + tx;
        const int gx = x0 + tx, gy = y0 + ly;
        const bool in = gx < W && gy < H;
        const int gi = gy * W + gx;
        if (in) lr[gi] = (uint16_t)(root[k] >= 0 ? root[k] : 0xffff);
        const int c = lcnt[li];
        const bool isroot = in && c > 0;
        if (isroot) {
            par[gi] = gi;
            tl[gi] = c;
            sz[gi] = 0;
        }
        rgi[k] = isroot ? gi : -1;
        rm[k] = __ballot(isroot);
        roff[k] = 0;
        if (rm[k]) {
            const int leader = __ffsll((long long)rm[k]) - 1;
            unsigned o = 0;
            if (lane == leader) o = atomicAdd(&s_roots, (unsigned)__popcll(rm[k]));  // LDS
            roff[k] = (unsigned)__builtin_amdgcn_readlane((int)o, leader);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_roots ? atomicAdd(list, s_roots) : 0u;
    __syncthreads();
    const unsigned base = s_base;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (rgi[k] >= 0)
            list[1 + base + roff[k] + (unsigned)__popcll(rm[k] & ((1ull << lane) - 1ull))] =
                (unsigned)(f * npix + rgi[k]);
}

// Union-find over tile components (the global parent words of tile roots).
// Parent words are read with agent-scope relaxed atomics (L1-bypassing):
// other workgroups rewrite them inside the same launch.  Roots are linked
// towards the smaller index with atomicMin (ECL-CC style): parents only ever
// decrease and stay inside their component, so concurrent unions never lose a
// link.
__device__ __forceinline__ int uf_load(const int* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int uf_find(int* parent, int i)
{
    int p = uf_load(parent + i);
    while (p != i) {
        int gp = uf_load(parent + p);
        if (gp != p) atomicMin(parent + i, gp);  // path halving, never increases
        i = p;
        p = gp;
    }
    return i;
}

__device__ void uf_unite(int* parent, int a, int b)
{
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a > b) {
            int t = a;
            a = b;
            b = t;
        }
        int old = atomicMin(parent + b, a);  // link root b under a (a < b)
        if (old == b) return;
        b = old;  // b was re-linked concurrently: continue with its new parent
    }
}

// the tile root (global index) of pixel (x, y) from its local root
__device__ __forceinline__ int tile_root(const uint16_t* lr, int W, int x, int y)
{
    const int l = lr[y * W + x];
    return (y & ~(kSpTile - 1)) * W + (x & ~(kSpTile - 1)) + (l / kSpTile) * W + (l % kSpTile);
}

// Stage 2: unions across tile borders (right and bottom edge of each tile),
// one wave per tile, four tiles per block.  A pair joins the two pixels' tile
// components; lanes whose (component, component) pair repeats a lower lane's
// skip it, so a tile edge inside one smooth region costs one union instead of
// 32.
__global__ __launch_bounds__(256) void speckle_border_kernel(const int16_t* __restrict__ img,
                                                             size_t st, size_t fs, int W, int H,
                                                             int new_val, int max_diff,
                                                             int* __restrict__ parent,
                                                             const uint16_t* __restrict__ lroot,
                                                             int tiles_x)
{
    const int t = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tyi = tile / tiles_x;
    const int x0 = (tile - tyi * tiles_x) * kSpTile, y0 = tyi * kSpTile;
    const int f = blockIdx.y;
    int x, y, nx, ny;
    if (t < kSpTile) {  // right edge: (x0+31, y0+t) -- (x0+32, y0+t)
        x = x0 + kSpTile - 1;
        y = y0 + t;
        nx = x + 1;
        ny = y;
    } else {  // bottom edge: (x0+t', y0+31) -- (x0+t', y0+32)
        x = x0 + (t - kSpTile);
        y = y0 + kSpTile - 1;
        nx = x;
        ny = y + 1;
    }
    const size_t npix = (size_t)W * H;
    int* par = parent + f * npix;
    const uint16_t* lr = lroot + f * npix;
    int a = -1, b = -1;
    if (y0 < H && x < W && y < H && nx < W && ny < H) {
        const int16_t* s = img + f * fs;
        const int v = s[(size_t)y * st + x], u = s[(size_t)ny * st + nx];
        if (v != new_val && u != new_val && abs(v - u) <= max_diff) {
            a = tile_root(lr, W, x, y);
            b = tile_root(lr, W, nx, ny);
        }
    }
    bool pending = a >= 0;
    for (;;) {
        unsigned long long m = __ballot(pending);
        if (m == 0ull) break;
        const int leader = __ffsll((long long)m) - 1;
        const int a0 = __builtin_amdgcn_readlane(a, leader);
        const int b0 = __builtin_amdgcn_readlane(b, leader);
        if (t == leader) uf_unite(par, a0, b0);
        if (a == a0 && b == b0) pending = false;
    }
}

// Stage 3: per tile component (the compact root list, grid-stride): its
// global root, the component sizes, and the tile word becomes ~root
// (negative: "resolved").
__global__ __launch_bounds__(256) void speckle_count_kernel(int W, int H, int* __restrict__ parent,
                                                            int* __restrict__ tilew,
                                                            int* __restrict__ size,
                                                            const unsigned* __restrict__ list)
{
    const unsigned cnt = list[0];
    const size_t npix = (size_t)W * H;
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const unsigned e = list[1 + i];
        const size_t f = e / npix;
        const int gi = (int)(e - f * npix);
        int* par = parent + f * npix;
        const int g = uf_find(par, gi);
        atomicAdd(size + f * npix + g, tilew[f * npix + gi]);
        tilew[f * npix + gi] = ~g;
    }
}

// Stage 4: pixel -> tile root -> global root -> size.  Block (0, 0, 0) also
// rewinds the root list for the next call (stage 3 has finished with it).
__global__ __launch_bounds__(256) void speckle_apply_kernel(int16_t* __restrict__ img, size_t st,
                                                            size_t fs, int W, int H, int new_val,
                                                            int max_size,
                                                            const int* __restrict__ tilew,
                                                            const int* __restrict__ size,
                                                            const uint16_t* __restrict__ lroot,
                                                            unsigned* __restrict__ list)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (blockIdx.x == 0 && blockIdx.y == 0 && f == 0 && threadIdx.x == 0) list[0] = 0u;
    if (x >= W || y >= H) return;
    int16_t* p = img + f * fs + (size_t)y * st + x;
    if (*p == new_val) return;
    const size_t base = (size_t)f * W * H;
    const int g = ~tilew[base + tile_root(lroot + base, W, x, y)];
    if (size[base + g] <= max_size) *p = (int16_t)new_val;
}

// ---- MeanDisparityDetection::build(MEAN_VALUE) --------------------------------
__global__ __launch_bounds__(256) void mean_grid_kernel(const int16_t* __restrict__ dmap,
                                                        size_t st, size_t fs, int W, int H,
                                                        float* __restrict__ means)
{
    __shared__ int s_tot[4], s_cnt[4];
    const int tile = blockIdx.x;  // 0..80, row-major 9x9
    const int f = blockIdx.y;
    const int r = tile / 9, c = tile % 9;
    const int dx = W / 9, dy = H / 9;
    const int16_t* m = dmap + f * fs;
    int tot = 0, cnt = 0;
    for (int i = threadIdx.x; i < dx * dy; i += 256) {
        int yy = r * dy + i / dx, xx = c * dx + i % dx;
        int v = m[(size_t)yy * st + xx];
        if (v > 1) {
            tot += v;
            cnt++;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o);
        cnt += __shfl_xor(cnt, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_tot[w] = tot;
        s_cnt[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int T = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
        int N = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        means[(size_t)f * 81 + tile] = (T == 0 || N == 0) ? 0.0f : (float)(T / abs(N));
    }
}

// ---- cv::remap(INTER_LINEAR, BORDER_CONSTANT 0), CV_8UC1, CV_32FC1 maps ----------
// The rectification step of Stereosystem::getRectifiedImagepair
// (src/Stereosystem.cpp:243-262).  [OpenCV 3.4 RemapInvoker + remapBilinear]:
// X = cvRound(mapx * 32), Y = cvRound(mapy * 32) (round half to even);
// (sx, sy) = (X >> 5, Y >> 5) saturated to short, (ax, ay) = the low 5 bits;
// weights (32-ay)(32-ax)*32, (32-ay)ax*32, ay(32-ax)*32, ay*ax*32 (sum 2^15,
// exact for bilinear); out = (sum + 2^14) >> 15.  A 2x2 footprint entirely
// outside the source gives 0; partially outside, the outside taps read 0.
__device__ __forceinline__ int remap_tap(const uint8_t* s, size_t ss, int W, int H, int x, int y)
{
    return (x >= 0 && x < W && y >= 0 && y < H) ? (int)s[(size_t)y * ss + x] : 0;
}

__global__ __launch_bounds__(256) void remap_linear_kernel(
    const uint8_t* __restrict__ src, size_t ss, size_t sfs, int sw, int sh,
    const float* __restrict__ mx, const float* __restrict__ my, size_t ms,
    uint8_t* __restrict__ dst, size_t ds, size_t dfs, int dw, int dh)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (x >= dw || y >= dh) return;
    const int X = __float2int_rn(mx[(size_t)y * ms + x] * 32.0f);
    const int Y = __float2int_rn(my[(size_t)y * ms + x] * 32.0f);
    const int sx = clampi(X >> 5, -32768, 32767), sy = clampi(Y >> 5, -32768, 32767);
    const int ax = X & 31, ay = Y & 31;
    const uint8_t* s = src + f * sfs;
    int v;
    if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        v = 0;
    } else {
        const int w00 = (32 - ay) * (32 - ax) * 32, w01 = (32 - ay) * ax * 32;
        const int w10 = ay * (32 - ax) * 32, w11 = ay * ax * 32;
        const int acc = remap_tap(s, ss, sw, sh, sx, sy) * w00 + remap_tap(s, ss, sw, sh, sx + 1, sy) * w01 +
                        remap_tap(s, ss, sw, sh, sx, sy + 1) * w10 +
                        remap_tap(s, ss, sw, sh, sx + 1, sy + 1) * w11;
        v = clampi((acc + (1 << 14)) >> 15, 0, 255);
    }
    dst[f * dfs + (size_t)y * ds + x] = (uint8_t)v;
}

// ---- cv::resize(src, dst, Size(0, 0), fx, fy, INTER_LINEAR), CV_8UC1 ----------
// The resize of Stereosystem::getRectifiedImagepair(Stereopair&, float)
// (src/Stereosystem.cpp:279-315).  [OpenCV 3.4 resize.cpp, x86 build] (oracle:
// orc_resize_linear): x / y source taps and 11-bit coefficients per output
// column / row in float (fx = (float)((dx + 0.5) * scale - 0.5), sx = floor,
// coefficients cvRound((1 - f) * 2048), cvRound(f * 2048); x clamped with
// f = 0, rows clamped); horizontal taps exact in int32; vertical combine as
// the SIMD op for columns x < simd_end ((S >> 4) x beta >> 16 per row, int16
// saturating add, (+2) >> 2) and (sum + 2^21) >> 22 past it.  A 2 x 2
// reduction (scale exactly 2) is INTER_AREA's fast path: (a+b+c+d+2) >> 2 on
// whole blocks, a float mean rounded half to even on clipped edge blocks.
__device__ __forceinline__ int sat16(int v) { return clampi(v, -32768, 32767); }

__global__ __launch_bounds__(256) void resize_linear_kernel(const uint8_t* __restrict__ src, size_t ss,
                                                            size_t sfs, int sw, int sh, double scale_x,
                                                            double scale_y, int area2, int simd_end,
                                                            uint8_t* __restrict__ dst, size_t ds, size_t dfs,
                                                            int dw, int dh)
{
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (dx >= dw || dy >= dh) return;
    const uint8_t* S = src + f * sfs;
    int v;
    if (area2) {
        const int sy0 = 2 * dy, sx0 = 2 * dx;
        const int w1 = sw / 2;
        const int w = sy0 + 2 <= sh ? w1 : 0;
        if (sy0 >= sh || sx0 >= sw) {
            v = 0;
        } else if (dx < w) {
            const uint8_t* r = S + (size_t)sy0 * ss + sx0;
            v = (r[0] + r[1] + r[ss] + r[ss + 1] + 2) >> 2;
        } else {
            int sum = 0, cnt = 0;
            for (int yy = 0; yy < 2 && sy0 + yy < sh; yy++)
                for (int xx = 0; xx < 2 && sx0 + xx < sw; xx++) {
                    sum += S[(size_t)(sy0 + yy) * ss + sx0 + xx];
                    cnt++;
                }
            v = clampi(__float2int_rn((float)sum / (float)cnt), 0, 255);
        }
    } else {
        float fxv = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fxv);
        fxv -= (float)sx;
        if (sx < 0) fxv = 0.f, sx = 0;
        if (sx >= sw - 1) fxv = 0.f, sx = sw - 1;
        const int a0 = __float2int_rn((1.f - fxv) * 2048.f), a1 = __float2int_rn(fxv * 2048.f);
        float fyv = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)floorf(fyv);
        fyv -= (float)sy;
        const int b0 = (int)(short)__float2int_rn((1.f - fyv) * 2048.f);
        const int b1 = (int)(short)__float2int_rn(fyv * 2048.f);
        const int r0 = clampi(sy, 0, sh - 1), r1 = clampi(sy + 1, 0, sh - 1);
        const uint8_t* p0 = S + (size_t)r0 * ss + sx;
        const uint8_t* p1 = S + (size_t)r1 * ss + sx;
        const int s0 = p0[0] * a0 + (a1 ? p0[1] * a1 : 0);
        const int s1 = p1[0] * a0 + (a1 ? p1[1] * a1 : 0);
        if (dx < simd_end) {
            const int h0 = sat16(s0 >> 4), h1 = sat16(s1 >> 4);
            const int r = sat16(((h0 * b0) >> 16) + ((h1 * b1) >> 16));
            v = sat16(r + 2) >> 2;
        } else {
            v = (s0 * b0 + s1 * b1 + (1 << 21)) >> 22;
        }
        v = clampi(v, 0, 255);
    }
    dst[f * dfs + (size_t)dy * ds + dx] = (uint8_t)v;
}

// ---- Utility::calcCoordinate per pixel (src/utility.cpp:176-198) -------------
// (X, Y, Z, W) = Q * (x, y, v / 16, 1) with OpenCV's float GEMM (products and
// sums in double, one rounding to float per element), then Mat /= W as
// convertTo(alpha = (float)(1 / W)) (float multiply); Z = 0 when Z / 1000 is
// infinite.  The 4th output is 1 for v > 0 (the pixels Utility::dmap2pcl keeps).
struct QMat {
    float q[16];
};

__global__ __launch_bounds__(256) void reproject_kernel(const int16_t* __restrict__ dmap, size_t st,
                                                        size_t fs, int W, int H, QMat Q,
                                                        float4* __restrict__ out, size_t os,
                                                        size_t ofs)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (x >= W || y >= H) return;
    const float v = (float)dmap[f * fs + (size_t)y * st + x];
    const float c[4] = {(float)x, (float)y, v / 16.0f, 1.0f};
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) acc = __dadd_rn(acc, __dmul_rn((double)Q.q[4 * i + k], (double)c[k]));
        r[i] = (float)acc;
    }
    const float alpha = (float)(1.0 / (double)r[3]);
    float X = __fmul_rn(r[0], alpha), Y = __fmul_rn(r[1], alpha), Z = __fmul_rn(r[2], alpha);
    if (isinf(__fdiv_rn(Z, 1000.0f))) Z = 0.0f;
    out[f * ofs + (size_t)y * os + x] = make_float4(X, Y, Z, v > 0.0f ? 1.0f : 0.0f);
}

}  // namespace

int median3x3_device(mvsv_ctx* ctx, int n, const int16_t* src, size_t ss, size_t sfs, int16_t* dst,
                     size_t ds, size_t dfs, int W, int H, const int* poison, unsigned epoch,
                     int invalid)
{
    const bool packed = (W % 2) == 0 && (ss % 2) == 0 && (sfs % 2) == 0 && (ds % 2) == 0 && (dfs % 2) == 0 &&
                        ((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 3) == 0;
    if (packed) {
        dim3 grid((W / 2 + 63) / 64, (H + 3) / 4, n);
        hipLaunchKernelGGL(median3x3_pk_kernel, grid, dim3(256), 0, ctx->stream, src, ss, sfs, dst, ds, dfs, W, H,
                           poison, epoch, invalid);
    } else {
        dim3 grid((W + 63) / 64, (H + 3) / 4, n);
        hipLaunchKernelGGL(median3x3_kernel, grid, dim3(256), 0, ctx->stream, src, ss, sfs, dst, ds, dfs, W, H,
                           poison, epoch, invalid);
    }
    return check_hip(ctx, hipGetLastError(), "median3x3");
}

// The speckle filter's buffers: parent / tile words / sizes (int per pixel,
// only tile-component roots used), the tile-local root of every pixel (u16)
// and the compact root list (count + entries).
static int speckle_buffers(mvsv_ctx* ctx, int n, int W, int H, int** parent, int** tilew, int** size,
                           uint16_t** lroot, unsigned** list)
{
    int rc;
    const size_t npix = (size_t)n * W * H;
    // the list count is rewound by the apply kernel of every run; a fresh
    // (re)allocation, or a run that did not reach its apply launch, rewinds here
    const bool fresh_list = ctx->uf_list.bytes < (npix + 1) * 4 || ctx->uf_list_dirty;
    if ((rc = ensure(ctx, ctx->uf_parent, npix * 4, "speckle labels"))) return rc;
    if ((rc = ensure(ctx, ctx->uf_size, npix * 4, "speckle sizes"))) return rc;
    if ((rc = ensure(ctx, ctx->uf_tile, npix * 4, "speckle tile components"))) return rc;
    if ((rc = ensure(ctx, ctx->uf_lroot, npix * 2, "speckle local roots"))) return rc;
    if ((rc = ensure(ctx, ctx->uf_list, (npix + 1) * 4, "speckle root list"))) return rc;
    if (fresh_list && (rc = check_hip(ctx, hipMemsetAsync(ctx->uf_list.ptr, 0, 4, ctx->stream), "root list reset")))
        return rc;
    ctx->uf_list_dirty = true;  // until this run's apply kernel is launched
    *parent = (int*)ctx->uf_parent.ptr;
    *size = (int*)ctx->uf_size.ptr;
    *tilew = (int*)ctx->uf_tile.ptr;
    *lroot = (uint16_t*)ctx->uf_lroot.ptr;
    *list = (unsigned*)ctx->uf_list.ptr;
    return MVSV_OK;
}

// stages 2-4 (stage 1 launched by the caller)
static int speckle_tail(mvsv_ctx* ctx, int n, int16_t* img, size_t st, size_t fs, int W, int H, int new_val,
                        int max_size, int max_diff, int* parent, int* tilew, int* size, uint16_t* lroot,
                        unsigned* list)
{
    hipStream_t s = ctx->stream;
    const int tx = (W + kSpTile - 1) / kSpTile, tyn = (H + kSpTile - 1) / kSpTile;
    hipLaunchKernelGGL(speckle_border_kernel, dim3((unsigned)((tx * tyn + 3) / 4), n), dim3(256), 0, s, img, st, fs,
                       W, H, new_val, max_diff, parent, lroot, tx);
    hipLaunchKernelGGL(speckle_count_kernel, dim3((unsigned)std::max(1, ctx->cus * 4)), dim3(256), 0, s, W, H, parent,
                       tilew, size, list);
    dim3 grid((W + 63) / 64, (H + 3) / 4, n);
    hipLaunchKernelGGL(speckle_apply_kernel, grid, dim3(256), 0, s, img, st, fs, W, H, new_val, max_size, tilew,
                       size, lroot, list);
    const int rc = check_hip(ctx, hipGetLastError(), "speckle filter");
    if (rc == MVSV_OK) ctx->uf_list_dirty = false;
    return rc;
}

int speckle_device(mvsv_ctx* ctx, int n, int16_t* img, size_t st, size_t fs, int W, int H,
                   int new_val, int max_size, int max_diff)
{
    int rc, *parent, *tilew, *size;
    uint16_t* lroot;
    unsigned* list;
    if ((rc = speckle_buffers(ctx, n, W, H, &parent, &tilew, &size, &lroot, &list))) return rc;
    dim3 tiles((W + kSpTile - 1) / kSpTile, (H + kSpTile - 1) / kSpTile, n);
    hipLaunchKernelGGL(speckle_local_kernel, tiles, dim3(256), 0, ctx->stream, img, st, fs, W, H, new_val, max_diff,
                       parent, tilew, size, lroot, list);
    return speckle_tail(ctx, n, img, st, fs, W, H, new_val, max_size, max_diff, parent, tilew, size, lroot, list);
}

int mean_grid_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W, int H,
                     float* means)
{
    hipLaunchKernelGGL(mean_grid_kernel, dim3(81, n), dim3(256), 0, ctx->stream, dmap, st, fs, W,
                       H, means);
    return check_hip(ctx, hipGetLastError(), "mean disparity grid");
}

int remap_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw, int sh,
                 const float* mx, const float* my, size_t ms, uint8_t* dst, size_t ds, size_t dfs,
                 int dw, int dh)
{
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, n);
    hipLaunchKernelGGL(remap_linear_kernel, grid, dim3(256), 0, ctx->stream, src, ss, sfs, sw, sh,
                       mx, my, ms, dst, ds, dfs, dw, dh);
    return check_hip(ctx, hipGetLastError(), "remap");
}

int resize_size(int sw, int sh, double fx, double fy, int* dw, int* dh)
{
    if (sw <= 0 || sh <= 0 || !(fx > 0) || !(fy > 0)) return MVSV_E_INVALID_ARG;
    const double w = std::nearbyint(sw * fx), h = std::nearbyint(sh * fy);  // cvRound (half to even)
    if (!(w >= 1 && h >= 1 && w <= 1 << 20 && h <= 1 << 20)) return MVSV_E_INVALID_ARG;
    *dw = (int)w;
    *dh = (int)h;
    return MVSV_OK;
}

int resize_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t ss, size_t sfs, int sw, int sh, double fx,
                  double fy, uint8_t* dst, size_t ds, size_t dfs)
{
    int dw, dh;
    if (resize_size(sw, sh, fx, fy, &dw, &dh)) return set_error(ctx, MVSV_E_INVALID_ARG, "bad resize factors");
    if (ds < (size_t)dw) return set_error(ctx, MVSV_E_INVALID_ARG, "resize destination stride smaller than width");
    if (dw == sw && dh == sh) {
        // [OpenCV 3.4 resize] dsize == ssize: src.copyTo(dst), whatever fx, fy
        for (int f = 0; f < n; f++) {
            const int rc = check_hip(ctx, hipMemcpy2DAsync(dst + (size_t)f * dfs, ds, src + (size_t)f * sfs, ss, sw, sh,
                                                           hipMemcpyDeviceToDevice, ctx->stream),
                                     "resize copy");
            if (rc) return rc;
        }
        return MVSV_OK;
    }
    const double scale_x = 1.0 / fx, scale_y = 1.0 / fy;
    const double isx = std::nearbyint(scale_x), isy = std::nearbyint(scale_y);
    const bool area2 = std::fabs(scale_x - isx) < DBL_EPSILON && std::fabs(scale_y - isy) < DBL_EPSILON &&
                       isx == 2.0 && isy == 2.0;
    // columns the SIMD vertical op covers: its 16-wide loop, then its 8-wide one
    int simd_end = 0;
    while (simd_end <= dw - 16) simd_end += 16;
    while (simd_end < dw - 8) simd_end += 8;
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, n);
    hipLaunchKernelGGL(resize_linear_kernel, grid, dim3(256), 0, ctx->stream, src, ss, sfs, sw, sh, scale_x,
                       scale_y, area2 ? 1 : 0, simd_end, dst, ds, dfs, dw, dh);
    return check_hip(ctx, hipGetLastError(), "resize");
}

int reproject_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t st, size_t fs, int W, int H,
                     const float* Q, float* out, size_t os, size_t ofs)
{
    QMat q;
    for (int i = 0; i < 16; i++) q.q[i] = Q[i];
    dim3 grid((W + 63) / 64, (H + 3) / 4, n);
    hipLaunchKernelGGL(reproject_kernel, grid, dim3(256), 0, ctx->stream, dmap, st, fs, W, H, q,
                       (float4*)out, os, ofs);
    return check_hip(ctx, hipGetLastError(), "reprojection");
}

}  // namespace mvsv
