// bs_chain.hip — latency of the bit-sliced direction step (mvsv_bsgm.hip's
// bs_dir_step) as a dependent chain: every lane pair runs ILP independent
// pixels' recurrences for STEPS steps from registers (no memory), with W waves
// per SIMD.  Prints shader cycles per step (s_memtime, all waves of a block
// bracketed by a barrier) -- the floor the line / strip kernels' step time
// sits on when they run one wave per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../mvstereovision3_amd/csrc bs_chain.hip -o bs_chain
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "mvsv_bitslice.hpp"

using namespace mvsv::bs;

constexpr int STEPS = 2048;

__device__ __forceinline__ uint32_t xswap(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true);
}

template <int P1, int P2>
__device__ __forceinline__ void step(uint32_t (&sE)[3], uint32_t (&sO)[3], const uint32_t (&cE)[4],
                                     const uint32_t (&cO)[4], uint32_t fill0, uint32_t fill1, uint32_t (&acc)[3])
{
    uint32_t slE[3], srO[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t prevO = xswap(sO[k]) | fill0;
        const uint32_t nextE = xswap(sE[k]) | fill1;
        slE[k] = fshr(sO[k], prevO, 31);
        srO[k] = fshr(nextE, sE[k], 1);
    }
    uint32_t dE[3], dO[3];
    delta3<P1, P2>(sE, slE, sO, dE);
    delta3<P1, P2>(sO, sE, srO, dO);
    uint32_t vE[4], vO[4];
    add43(cE, dE, vE);
    add43(cO, dO, vO);
    uint32_t kE = ~vE[3], kO = ~vO[3], M[3];
#pragma unroll
    for (int b = 2; b >= 0; b--) {
        const uint32_t zE = lop3<kAndNotAB>(vE[b], kE, kE);
        const uint32_t zO = lop3<kAndNotAB>(vO[b], kO, kO);
        uint32_t any = zE | zO;
        any |= xswap(any);
        const bool f = any != 0u;
        if (b > 0) {
            kE = f ? zE : kE;
            kO = f ? zO : kO;
        }
        M[b] = f ? 0u : 0xffffffffu;
    }
    subclamp<P2>(vE, M[0], M[1], M[2], sE);
    subclamp<P2>(vO, M[0], M[1], M[2], sO);
#pragma unroll
    for (int k = 0; k < 3; k++) acc[k] ^= dE[k] ^ dO[k];
}

// the lane-quad form (mvsv_bsgm.hip bs_quad_step)
template <int P1, int P2>
__device__ __forceinline__ void qstep(uint32_t (&s)[3], const uint32_t (&c)[4], uint32_t fill_hi, uint32_t fill_lo,
                                      bool odd, uint32_t sh, uint32_t (&acc)[3])
{
    uint32_t nb[3], pt[3], d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)s[k], 0xF9, 0xf, 0xf, true) | fill_hi;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)s[k], 0x90, 0xf, 0xf, true) | fill_lo;
        nb[k] = __builtin_amdgcn_alignbit(hi, lo, sh);
        pt[k] = odd ? lo : hi;
    }
    delta3<P1, P2>(s, nb, pt, d);
    uint32_t v[4];
    add43(c, d, v);
    uint32_t kk = ~v[3], M[3];
#pragma unroll
    for (int b = 2; b >= 0; b--) {
        const uint32_t z = lop3<kAndNotAB>(v[b], kk, kk);
        uint32_t any = z | xswap(z);
        any |= (uint32_t)__builtin_amdgcn_mov_dpp((int)any, 0x4E, 0xf, 0xf, true);
        const bool f = any != 0u;
        if (b > 0) kk = f ? z : kk;
        M[b] = f ? 0u : 0xffffffffu;
    }
    subclamp<P2>(v, M[0], M[1], M[2], s);
#pragma unroll
    for (int k = 0; k < 3; k++) acc[k] ^= d[k];
}

template <int ILP>
__global__ void qchain(const uint32_t* seed, uint32_t* out, unsigned long long* clk)
{
    const int lane = threadIdx.x & 63, q = lane & 3;
    const bool odd = q & 1;
    const uint32_t fill_hi = q == 3 ? 0xffffffffu : 0u, fill_lo = q == 0 ? 0xffffffffu : 0u, sh = odd ? 1u : 31u;
    uint32_t s[ILP][3], c[ILP][4], acc[ILP][3];
    for (int i = 0; i < ILP; i++) {
        for (int k = 0; k < 3; k++) s[i][k] = acc[i][k] = 0;
        for (int k = 0; k < 4; k++) c[i][k] = seed[(lane * 8 + k + i) & 255];
        c[i][3] = 0;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < STEPS; t++) {
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            qstep<2, 5>(s[i], c[i], fill_hi, fill_lo, odd, sh, acc[i]);
#pragma unroll
            for (int k = 0; k < 3; k++) c[i][k] = __builtin_amdgcn_alignbit(c[i][k], c[i][k], 7);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < ILP; i++)
        for (int k = 0; k < 3; k++) r ^= acc[i][k] ^ s[i][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) clk[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int ILP>
__global__ void chain(const uint32_t* seed, uint32_t* out, unsigned long long* clk)
{
    const int lane = threadIdx.x & 63, h = lane & 1;
    const uint32_t fill0 = h == 0 ? 0xffffffffu : 0u, fill1 = h == 1 ? 0xffffffffu : 0u;
    uint32_t sE[ILP][3], sO[ILP][3], cE[ILP][4], cO[ILP][4], acc[ILP][3];
    for (int i = 0; i < ILP; i++) {
        for (int k = 0; k < 3; k++) sE[i][k] = sO[i][k] = acc[i][k] = 0;
        for (int k = 0; k < 4; k++) {
            cE[i][k] = seed[(lane * 8 + k + i) & 255];
            cO[i][k] = seed[(lane * 8 + 4 + k + i) & 255];
        }
        cE[i][3] = 0;  // C' <= 7 here (some d small enough: the row minimum stays <= P2)
        cO[i][3] = 0;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < STEPS; t++) {
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            step<2, 5>(sE[i], sO[i], cE[i], cO[i], fill0, fill1, acc[i]);
            // new costs per step without memory: rotate the words (1 op each)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                cE[i][k] = __builtin_amdgcn_alignbit(cE[i][k], cE[i][k], 7);
                cO[i][k] = __builtin_amdgcn_alignbit(cO[i][k], cO[i][k], 11);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < ILP; i++)
        for (int k = 0; k < 3; k++) r ^= acc[i][k] ^ sE[i][k] ^ sO[i][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) clk[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int ILP, bool Q = false>
static void run(int waves_per_simd)
{
    const int threads = 256 * waves_per_simd;  // 4 SIMDs per CU
    const int blocks = 256;                    // one block per CU
    uint32_t *seed, *out;
    unsigned long long* clk;
    hipMalloc(&seed, 256 * 4);
    std::vector<uint32_t> hs(256);
    uint32_t x = 12345;
    for (auto& v : hs) v = (x = x * 1664525u + 1013904223u);
    hipMemcpy(seed, hs.data(), 256 * 4, hipMemcpyHostToDevice);
    hipMalloc(&out, (size_t)blocks * threads * 4);
    hipMalloc(&clk, (size_t)blocks * threads / 64 * 8);
    auto kern = Q ? qchain<ILP> : chain<ILP>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, seed, out, clk);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, seed, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> c((size_t)blocks * threads / 64);
    hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : c) mean += (double)v;
    mean /= c.size();
    std::printf("%s ILP %d, %d waves/SIMD: %.1f shader cycles per step per wave (%.1f per pixel-step per SIMD), "
                "kernel %.3f ms\n",
                Q ? "quad" : "pair", ILP, waves_per_simd, mean / STEPS, mean / STEPS / (ILP * waves_per_simd), ms);
    hipFree(seed);
    hipFree(out);
    hipFree(clk);
}

int main()
{
    for (int w : {1, 2, 4}) {
        run<1>(w);
        run<2>(w);
        run<1, true>(w);
        run<2, true>(w);
    }
    return 0;
}
