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

// packed unsigned 16-bit pairs (VOP3P v_pk_*_u16)
__device__ __forceinline__ uint32_t pk_subsat_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a),
                                                                      __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}

// Two independent u16 minima over each 16-lane row (packed in one dword).
__device__ __forceinline__ uint32_t row_min_u16x2(uint32_t v)
{
    v = pk_min_u16(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false));
    v = pk_min_u16(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false));
    v = pk_min_u16(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));
    v = pk_min_u16(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false));
    return v;
}

// ... over aligned segments of `lanes` = 16, 32 or 64 lanes (wave-uniform):
// the row butterfly, then rows (0,1) / (2,3) joined by v_permlane16_swap and the
// two halves by v_permlane32_swap; every lane of a segment gets its minima.
__device__ __forceinline__ uint32_t seg_min_u16x2(uint32_t v, int lanes)
{
    v = row_min_u16x2(v);
    if (lanes >= 32) {
        const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = pk_min_u16(sw[0], sw[1]);
    }
    if (lanes >= 64) {
        const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = pk_min_u16(sw[0], sw[1]);
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T clampi(T v, T lo, T hi)
{
    return v < lo ? lo : (v > hi ? hi : v);
}

}  // namespace dev
}  // namespace mvsv
