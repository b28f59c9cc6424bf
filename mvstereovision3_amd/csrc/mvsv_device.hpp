// mvsv_device.hpp — CDNA4 (gfx950) device helpers shared by the kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mvsv {
namespace dev {

// Two int16 disparity costs packed in one VGPR: v_pk_{add,sub}_i16 clamp,
// v_pk_min_i16 do the whole SGM update for two disparities per instruction.
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_s2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ uint32_t pk_add_sat(uint32_t a, uint32_t b)
{
    return as_u(__builtin_elementwise_add_sat(as_s2(a), as_s2(b)));
}
__device__ __forceinline__ uint32_t pk_sub_sat(uint32_t a, uint32_t b)
{
    return as_u(__builtin_elementwise_sub_sat(as_s2(a), as_s2(b)));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b)
{
    return as_u(__builtin_elementwise_min(as_s2(a), as_s2(b)));
}
// Two u16 halves added / subtracted as one 32-bit word: exact only where no
// half carries or borrows (each call site states why).  v_add_u32 / v_sub_u32
// issue at twice the rate of the VOP3P packed ops (2.5 vs 4.2 cycles per
// wave-instruction, tools/ubench/valu_rate.hip).
__device__ __forceinline__ uint32_t add2_nc(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t sub2_nb(uint32_t a, uint32_t b) { return a - b; }
__device__ __forceinline__ int lo16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ int hi16(uint32_t v) { return (int)(int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t pk2(int lo, int hi)
{
    return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xffffu);
}

// Whole-wave (64-lane) shifts by one lane; the lane that has no source keeps
// `edge` (DPP wave_shr:1 / wave_shl:1, bound_ctrl off).
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t edge)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v, uint32_t edge)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x130, 0xf, 0xf, false);
}

// Shifts by one lane inside each 16-lane DPP row (row_shr:1 / row_shl:1); the
// lane of a row that has no source keeps `edge`.
__device__ __forceinline__ uint32_t row_shr1(uint32_t v, uint32_t edge)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x111, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t row_shl1(uint32_t v, uint32_t edge)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x101, 0xf, 0xf, false);
}

// Minimum / maximum over each 16-lane row; every lane of the row gets the result.
// bound_ctrl is set: these patterns never read outside the row, and with it
// the compiler folds each DPP move into the min/max (v_min_i32_dpp).
__device__ __forceinline__ int row_min_i32(int v)
{
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true));  // row_half_mirror
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true));  // row_mirror
    return v;
}
__device__ __forceinline__ int row_max_i32(int v)
{
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true));
    return v;
}

// Minimum over the 64 lanes, returned wave-uniform (scalar).  DPP butterfly
// inside each 16-lane row, then the four row results through readlane.
__device__ __forceinline__ int wave_min_i32(int v)
{
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true));  // row_half_mirror
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true));  // row_mirror
    int a = __builtin_amdgcn_readlane(v, 0);
    int b = __builtin_amdgcn_readlane(v, 16);
    int c = __builtin_amdgcn_readlane(v, 32);
    int d = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, d));
}

template <typename T>
__device__ __forceinline__ T clampi(T v, T lo, T hi)
{
    return v < lo ? lo : (v > hi ? hi : v);
}

}  // namespace dev
}  // namespace mvsv
