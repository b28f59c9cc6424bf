// valu_rate.hip — issue rate of the VALU instructions the SGM kernels live on
// (gfx950): cycles per wave-instruction per SIMD with W waves per SIMD, each
// wave running 8 independent chains (no dependency stalls).
// Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pkmin(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ uint32_t pkadds(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}

constexpr int ITER = 4096;
// inline asm: exactly one instruction of the measured kind per chain step
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t b)
{
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 1) asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 2) asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a) : "v"(b));
    if constexpr (OP == 3) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 4) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(a) : "v"(b));
    if constexpr (OP == 5) asm volatile("v_min_i32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a) : "v"(b));
    if constexpr (OP == 6) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 7) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 8) asm volatile("v_pk_sub_i16 %0, %0, %1 clamp" : "+v"(a) : "v"(b));
    if constexpr (OP == 9) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
}
template <int OP>
__global__ __launch_bounds__(1024) void kern(uint32_t* out, uint32_t seed)
{
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (threadIdx.x + i + 1);
    const uint32_t b = seed ^ threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) op<OP>(a[i], b);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= a[i];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1000] = (uint32_t)(t1 - t0);  // shader ticks, wave 0
}

template <int OP>
float run(int waves_per_simd, const char* name)
{
    uint32_t* d;
    hipMalloc(&d, 4096);
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, dev);
    const int cus = pr.multiProcessorCount;
    const int threads = 64 * 4 * waves_per_simd;  // one block per CU, waves spread over 4 SIMDs
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<OP>, dim3(cus), dim3(threads), 0, 0, d, 7u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<OP>, dim3(cus), dim3(threads), 0, 0, d, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr_per_simd = (double)waves_per_simd * ITER * 8;
    const double cyc = ms * 1e-3 * pr.clockRate * 1e3 / instr_per_simd;
    uint32_t ticks = 0;
    hipMemcpy(&ticks, d + 1000, 4, hipMemcpyDeviceToHost);
    std::printf("%-22s waves/SIMD %d: %.2f cycles/instr/SIMD at the nominal clock, %.2f in s_memtime ticks\n",
                name, waves_per_simd, cyc, ticks / instr_per_simd);
    hipFree(d);
    return (float)cyc;
}

int main()
{
    for (int w : {1, 2, 4}) {
        run<0>(w, "v_add_u32");
        run<1>(w, "v_pk_min_i16");
        run<2>(w, "v_pk_add_i16 clamp");
        run<3>(w, "v_pk_add_u16");
        run<4>(w, "v_alignbit_b32");
        run<5>(w, "v_min_i32_dpp row_shr");
        run<6>(w, "v_perm_b32");
        run<7>(w, "v_min_i32");
        run<8>(w, "v_pk_sub_i16 clamp");
        run<9>(w, "v_cndmask_b32");
    }
    return 0;
}
