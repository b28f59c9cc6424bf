// valu_rate.hip — issue rate of the VALU instructions the SGM kernels live on
// (gfx950): cycles per wave-instruction per SIMD with W waves per SIMD, each
// wave running 8 independent chains (no dependency stalls).
//
// Two clocks, reconciled:
//   * in-kernel: every wave stamps s_memtime (shader clock) and s_memrealtime
//     (constant 100 MHz) after a block barrier and again at its end; a block's
//     span is max(end) - min(start) over ALL its waves (the oldest wave gets
//     VALU priority and finishes first, so wave 0's own interval understates
//     the SIMD's work); the shader clock is Δmemtime / Δmemrealtime x 100 MHz;
//   * hipEvents around the launch, converted with that measured clock (not the
//     nominal 2.4 GHz): includes launch overhead, so it reads slightly higher.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int ITER = 4096;
constexpr int CHAINS = 8;

#define OPS(X)                                                                                  \
    X(0, "v_add_u32", "v_add_u32 %0, %0, %1")                                                  \
    X(1, "v_sub_u32", "v_sub_u32 %0, %0, %1")                                                  \
    X(2, "v_and_b32", "v_and_b32 %0, %0, %1")                                                  \
    X(3, "v_or_b32", "v_or_b32 %0, %0, %1")                                                    \
    X(4, "v_xor_b32", "v_xor_b32 %0, %0, %1")                                                  \
    X(5, "v_lshlrev_b32", "v_lshlrev_b32 %0, 3, %0")                                           \
    X(6, "v_min_i32", "v_min_i32 %0, %0, %1")                                                  \
    X(7, "v_min_u32", "v_min_u32 %0, %0, %1")                                                  \
    X(8, "v_max_i32", "v_max_i32 %0, %0, %1")                                                  \
    X(9, "v_add_f32", "v_add_f32 %0, %0, %1")                                                  \
    X(10, "v_fma_f32", "v_fma_f32 %0, %0, %1, %1")                                             \
    X(11, "v_min_f32", "v_min_f32 %0, %0, %1")                                                 \
    X(12, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1")                                         \
    X(13, "v_add3_u32", "v_add3_u32 %0, %0, %1, %1")                                           \
    X(14, "v_min3_i32", "v_min3_i32 %0, %0, %1, %1")                                           \
    X(15, "v_med3_i32", "v_med3_i32 %0, %0, %1, %1")                                           \
    X(16, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 4, %1")                                      \
    X(17, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %1")                                             \
    X(18, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 16")                                   \
    X(19, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1")                                           \
    X(20, "v_cndmask_b32_e64", "v_cndmask_b32_e64 %0, %0, %1, s[8:9]")                         \
    X(21, "v_pk_min_i16", "v_pk_min_i16 %0, %0, %1")                                           \
    X(22, "v_pk_min_u16", "v_pk_min_u16 %0, %0, %1")                                           \
    X(23, "v_pk_max_u16", "v_pk_max_u16 %0, %0, %1")                                           \
    X(24, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1")                                           \
    X(25, "v_pk_add_i16 clamp", "v_pk_add_i16 %0, %0, %1 clamp")                               \
    X(26, "v_pk_sub_u16 clamp", "v_pk_sub_u16 %0, %0, %1 clamp")                               \
    X(27, "v_pk_sub_i16 clamp", "v_pk_sub_i16 %0, %0, %1 clamp")                               \
    X(28, "v_pk_mad_u16", "v_pk_mad_u16 %0, %0, %1, %1")                                       \
    X(29, "v_pk_add_f16", "v_pk_add_f16 %0, %0, %1")                                           \
    X(30, "v_pk_min_f16", "v_pk_min_f16 %0, %0, %1")                                           \
    X(31, "v_pk_max_i16", "v_pk_max_i16 %0, %0, %1")                                              \
    X(32, "v_min_u16 (VOP2)", "v_min_u16 %0, %0, %1")                                          \
    X(33, "v_add_u16 (VOP2)", "v_add_u16 %0, %0, %1")                                          \
    X(34, "v_min3_u16", "v_min3_u16 %0, %0, %1, %1")                                           \
    X(35, "v_min_u16_sdwa", "v_min_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1") \
    X(36, "v_sad_u8", "v_sad_u8 %0, %0, %1, %1")                                               \
    X(37, "v_msad_u8", "v_msad_u8 %0, %0, %1, %1")                                             \
    X(38, "v_sad_u16", "v_sad_u16 %0, %0, %1, %1")                                             \
    X(39, "v_min_i32_dpp row_shr", "v_min_i32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1") \
    X(40, "v_mov_b32_dpp row_shr", "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")  \
    X(41, "v_or_b32_dpp row_shr", "v_or_b32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1") \
    X(42, "v_bitop3_b32", "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")                           \
    X(43, "v_max_u16 (VOP2)", "v_max_u16 %0, %0, %1")

constexpr int NOPS = 44;

template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t b);
#define DEF_OP(N, NAME, ASM)                                                                    \
    template <>                                                                                 \
    __device__ __forceinline__ void op<N>(uint32_t & a, uint32_t b)                             \
    {                                                                                           \
        asm volatile(ASM : "+v"(a) : "v"(b));                                                   \
    }
OPS(DEF_OP)

static const char* kNames[NOPS] = {
#define NAME_OP(N, NAME, ASM) NAME,
    OPS(NAME_OP)};

struct Stamp {
    unsigned long long t0, t1, r0, r1;
};

template <int OP>
__global__ __launch_bounds__(1024) void kern(uint32_t* out, Stamp* st, uint32_t seed)
{
    uint32_t a[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; i++) a[i] = seed * (threadIdx.x + i + 1);
    const uint32_t b = seed ^ threadIdx.x;
    if constexpr (OP == 20) asm volatile("s_mov_b64 s[8:9], exec" ::: "s8", "s9");
    __syncthreads();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < CHAINS; i++) op<OP>(a[i], b);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) s ^= a[i];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {  // one stamp per wave, vector stores
        Stamp v{t0, t1, r0, r1};
        st[(size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = v;
    }
}

template <int OP>
void run(int waves_per_simd, int cus)
{
    const int blocks_per_cu = waves_per_simd > 4 ? waves_per_simd / 4 : 1;
    const int wps_block = waves_per_simd / blocks_per_cu;
    const int threads = 64 * 4 * wps_block;
    const int nblk = cus * blocks_per_cu;
    const int nw = threads / 64;
    uint32_t* d;
    Stamp* st;
    hipMalloc(&d, 4096 * 4);
    hipMalloc(&st, sizeof(Stamp) * (size_t)nblk * nw);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(threads), 0, 0, d, st, 7u);  // warm
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(threads), 0, 0, d, st, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<Stamp> h((size_t)nblk * nw);
    hipMemcpy(h.data(), st, sizeof(Stamp) * h.size(), hipMemcpyDeviceToHost);
    // per block: span over all its waves; clock from the same waves
    std::vector<double> span, clk, w0;
    for (int b = 0; b < nblk; b++) {
        unsigned long long t0 = ~0ull, t1 = 0, r0 = ~0ull, r1 = 0;
        for (int w = 0; w < nw; w++) {
            const Stamp& s = h[(size_t)b * nw + w];
            t0 = std::min(t0, s.t0);
            t1 = std::max(t1, s.t1);
            r0 = std::min(r0, s.r0);
            r1 = std::max(r1, s.r1);
        }
        span.push_back((double)(t1 - t0));
        clk.push_back((double)(t1 - t0) / (double)(r1 - r0) * 100e6);
        w0.push_back((double)(h[(size_t)b * nw].t1 - h[(size_t)b * nw].t0));
    }
    std::sort(span.begin(), span.end());
    std::sort(clk.begin(), clk.end());
    std::sort(w0.begin(), w0.end());
    const double med_span = span[span.size() / 2], med_clk = clk[clk.size() / 2];
    // waves_per_simd waves of one SIMD share it: instructions issued per SIMD
    // over the span of the CU's blocks (blocks of one CU run concurrently)
    const double instr = (double)waves_per_simd * ITER * CHAINS;
    const double cyc = med_span / instr;
    const double cyc_ev = ms * 1e-3 * med_clk / instr;
    std::printf("%-24s w/SIMD %d: %5.2f cyc/wave-instr/SIMD (all-wave span; clock %.2f GHz), "
                "%5.2f by hipEvents at that clock, wave-0 alone %5.2f cyc per own instr\n",
                kNames[OP], waves_per_simd, cyc, med_clk / 1e9, cyc_ev, w0[w0.size() / 2] / (ITER * CHAINS));
    hipFree(d);
    hipFree(st);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int... I>
void run_all(int w, int cus, std::integer_sequence<int, I...>)
{
    (run<I>(w, cus), ...);
}

int main(int argc, char** argv)
{
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, dev);
    std::printf("device %s, %d CUs, nominal clock %.2f GHz\n", pr.gcnArchName, pr.multiProcessorCount,
                pr.clockRate / 1e6);
    // optional argument: one waves-per-SIMD count (the counter-calibration run)
    const int only = argc > 1 ? std::atoi(argv[1]) : 0;
    for (int w : {1, 2, 4, 8})
        if (!only || w == only) run_all(w, pr.multiProcessorCount, std::make_integer_sequence<int, NOPS>{});
    return 0;
}
