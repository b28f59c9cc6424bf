// FETCH_SIZE / WRITE_SIZE calibration for the access widths the SGBM kernels use
// (MI355X_MICROARCH.md: "other access widths are uncalibrated").  Each kernel
// streams exactly `bytes` (1 GiB, past the 256 MiB Infinity Cache) through
// coalesced per-lane loads or stores of W bytes; rocprofv3 --pmc FETCH_SIZE /
// WRITE_SIZE in separate passes then gives counter bytes / true bytes per width.
// Usage: ./fetch_cal  (prints the true byte count per kernel)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W>
struct VecT;
template <> struct VecT<2> { using T = unsigned short; };
template <> struct VecT<4> { using T = unsigned; };
template <> struct VecT<8> { using T = unsigned long long; };
template <> struct VecT<16> { using T = uint4; };

__device__ __forceinline__ unsigned fold(unsigned short v) { return v; }
__device__ __forceinline__ unsigned fold(unsigned v) { return v; }
__device__ __forceinline__ unsigned fold(unsigned long long v) { return (unsigned)v ^ (unsigned)(v >> 32); }
__device__ __forceinline__ unsigned fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int W>
__global__ __launch_bounds__(256) void read_w(const typename VecT<W>::T* __restrict__ p, size_t n, unsigned* sink)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= fold(p[i]);
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // never true for the zeroed buffer: keeps the loads
}

template <int W>
__global__ __launch_bounds__(256) void write_w(typename VecT<W>::T* __restrict__ p, size_t n)
{
    typename VecT<W>::T v{};
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = v;
}

int main()
{
    const size_t bytes = 1ull << 30;
    void* buf;
    unsigned* sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 1024) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    const int grid = 256 * 16;
    read_w<2><<<grid, 256>>>((const unsigned short*)buf, bytes / 2, sink);
    read_w<4><<<grid, 256>>>((const unsigned*)buf, bytes / 4, sink);
    read_w<8><<<grid, 256>>>((const unsigned long long*)buf, bytes / 8, sink);
    read_w<16><<<grid, 256>>>((const uint4*)buf, bytes / 16, sink);
    write_w<2><<<grid, 256>>>((unsigned short*)buf, bytes / 2);
    write_w<4><<<grid, 256>>>((unsigned*)buf, bytes / 4);
    write_w<8><<<grid, 256>>>((unsigned long long*)buf, bytes / 8);
    write_w<16><<<grid, 256>>>((uint4*)buf, bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("bytes per kernel %zu\n", bytes);
    return 0;
}
