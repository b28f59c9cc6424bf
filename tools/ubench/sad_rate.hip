// sad_rate.hip — issue rate of the SAD family with 64-/128-bit results on gfx950
// (candidates for StereoBM's column sums: v_mqsad_pk_u16_u8 gives four
// disparities' |L - R| as u16 halves in one instruction) next to v_msad_u8 and
// the adds that would go with them.  8 independent chains per wave, W waves
// per SIMD; cycles per wave-instruction per SIMD from s_memtime over the
// block's waves (same method as valu_rate.hip).
// Build: hipcc --offload-arch=gfx950 -O3 sad_rate.hip -o /tmp/sad_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int ITER = 2048;
constexpr int CHAINS = 8;

template <int OP>
__device__ __forceinline__ void op(uint64_t& a, uint64_t b, uint32_t c)
{
    if constexpr (OP == 0) asm volatile("v_msad_u8 %0, %1, %2, %0" : "+v"(*(uint32_t*)&a) : "v"((uint32_t)b), "v"(c));
    if constexpr (OP == 1) asm volatile("v_mqsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == 2) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == 3) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(*(uint32_t*)&a) : "v"(c));
    if constexpr (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 5) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(*(uint32_t*)&a) : "v"(c));
}

static const char* kNames[] = {"v_msad_u8", "v_mqsad_pk_u16_u8", "v_qsad_pk_u16_u8", "v_pk_sub_u16",
                               "v_lshl_add_u64", "v_sub_u32"};
constexpr int NOPS = 6;

template <int OP>
__global__ __launch_bounds__(1024) void kern(uint32_t* out, unsigned long long* st, uint32_t seed)
{
    uint64_t a[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; i++) a[i] = (uint64_t)seed * (threadIdx.x + i + 1) * 0x9e3779b97f4a7c15ull;
    const uint64_t b = (uint64_t)(seed ^ threadIdx.x) * 0x2545f4914f6cdd1dull;
    const uint32_t c = 0x01u * (seed + threadIdx.x);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < CHAINS; i++) op<OP>(a[i], b, c);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) s ^= a[i];
    if (s == 0x12345678ull) out[threadIdx.x] = (uint32_t)s;
    if ((threadIdx.x & 63) == 0) {
        st[2 * ((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = t0;
        st[2 * ((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = t1;
    }
}

template <int OP>
void run(int wps, int cus)
{
    const int threads = 64 * 4 * wps, nw = threads / 64;
    uint32_t* d;
    unsigned long long* st;
    (void)hipMalloc(&d, 4096 * 4);
    (void)hipMalloc(&st, 16 * (size_t)cus * nw);
    hipLaunchKernelGGL(kern<OP>, dim3(cus), dim3(threads), 0, 0, d, st, 7u);
    hipLaunchKernelGGL(kern<OP>, dim3(cus), dim3(threads), 0, 0, d, st, 7u);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * (size_t)cus * nw);
    (void)hipMemcpy(h.data(), st, 16 * h.size() / 2, hipMemcpyDeviceToHost);
    std::vector<double> span;
    for (int b = 0; b < cus; b++) {
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int w = 0; w < nw; w++) {
            t0 = std::min(t0, h[2 * ((size_t)b * nw + w)]);
            t1 = std::max(t1, h[2 * ((size_t)b * nw + w) + 1]);
        }
        span.push_back((double)(t1 - t0));
    }
    std::sort(span.begin(), span.end());
    // s_memtime is the shader clock (valu_rate.hip checks it against s_memrealtime)
    const double cyc = span[span.size() / 2] / ((double)wps * ITER * CHAINS);
    std::printf("%-20s w/SIMD %d: %5.2f cyc/wave-instr/SIMD\n", kNames[OP], wps, cyc);
    (void)hipFree(d);
    (void)hipFree(st);
}

template <int... I>
void run_all(int w, int cus, std::integer_sequence<int, I...>)
{
    (run<I>(w, cus), ...);
}

// semantics check: R bytes 1..8 against L = 5 in byte 0 only (masked: the
// zero bytes of the reference do not count) -> |R[i] - 5| for i = 0..3
__global__ void semantics(uint64_t* out)
{
    uint64_t a = 0x0000000100020003ull;
    asm volatile("v_mqsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(a) : "v"(0x0807060504030201ull), "v"(5u));
    out[0] = a;
    uint64_t q = 0;
    asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(q) : "v"(0x0807060504030201ull), "v"(5u));
    out[1] = q;
}

int main()
{
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    uint64_t* o;
    (void)hipMalloc(&o, 16);
    hipLaunchKernelGGL(semantics, dim3(1), dim3(64), 0, 0, o);
    uint64_t h[2];
    (void)hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
    std::printf("mqsad(R=01..08, L=05 byte0, acc=(3,2,1,0)) = %016llx  qsad(no mask, acc 0) = %016llx\n",
                (unsigned long long)h[0], (unsigned long long)h[1]);
    for (int w : {2, 4})
        run_all(w, pr.multiProcessorCount, std::make_integer_sequence<int, NOPS>{});
    return 0;
}
