// Workgroup dispatch placement probe: which XCC each block of a strip-kernel
// shaped launch (1024 threads, 78 KB LDS, one block per CU) starts on, and when.
// Usage: ./xcc_map [blocks] [busy_us]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(1024) void probe(unsigned long long* out, unsigned spin)
{
    extern __shared__ unsigned char smem[];
    if (threadIdx.x == 0) {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        out[blockIdx.x * 3 + 0] = __builtin_amdgcn_s_memrealtime();
        out[blockIdx.x * 3 + 1] = xcc;
        out[blockIdx.x * 3 + 2] = hw;
        smem[0] = 1;
    }
    // hold the CU a while (variable per block, like strips of different lengths)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long len = spin * (1 + (blockIdx.x % 7));
    while (__builtin_amdgcn_s_memrealtime() - t0 < len) __builtin_amdgcn_s_sleep(10);
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 576;
    const unsigned spin = (unsigned)(argc > 2 ? atoi(argv[2]) : 20) * 100;  // us -> 100 MHz ticks
    unsigned long long* d;
    hipMalloc(&d, n * 24);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    probe<<<n, 1024, 78 * 1024>>>(d, spin);
    std::vector<unsigned long long> h(n * 3);
    hipMemcpy(h.data(), d, n * 24, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < n; b++) t0 = std::min(t0, h[b * 3]);
    int same = 0;
    for (int b = 0; b < n; b++) {
        if (b < 40 || b % 37 == 0)
            printf("blk %4d xcc %llu start_us %8.2f hw_id %08llx\n", b, h[b * 3 + 1], (h[b * 3] - t0) / 100.0, h[b * 3 + 2]);
        same += (int)((h[b * 3 + 1] & 7) == (unsigned long long)(b % 8));
    }
    // does block b start before block b+1 (dispatch in blockIdx order)?
    int inorder = 0;
    for (int b = 0; b + 1 < n; b++) inorder += h[b * 3] <= h[(b + 1) * 3];
    printf("blocks %d: xcc == b%%8 for %d, start(b) <= start(b+1) for %d of %d\n", n, same, inorder, n - 1);
    return 0;
}
