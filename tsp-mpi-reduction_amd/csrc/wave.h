// Wavefront-wide minimum on gfx950 through DPP (north_star: "a wavefront-level
// min via DPP/ballot"): four DPP steps reduce each row of 16 lanes (swap
// neighbours, swap pairs, half-row mirror, row mirror: after them every lane
// of a row holds the row's minimum), then the four row minima are read with
// v_readlane into scalars and combined.  No LDS traffic (the previous
// __shfl_xor ladder was ds_bpermute / ds_swizzle through the LDS crossbar).
// Callers run it with all 64 lanes active; the minimum is wave-uniform.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tspgpu {

namespace wave_detail {
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // row_half_mirror: lane i <-> 7 - i within 8
constexpr int kDppMirror = 0x140;      // row_mirror: lane i <-> 15 - i within 16

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v)
{
    const uint32_t lo = dpp32<CTRL>((uint32_t)v), hi = dpp32<CTRL>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// bit-level carriers of the supported types
template <typename T> struct Bits;
template <> struct Bits<double> {
    using U = uint64_t;
    __device__ static U to(double v) { return (U)__double_as_longlong(v); }
    __device__ static double from(U u) { return __longlong_as_double((long long)u); }
};
template <> struct Bits<int32_t> {
    using U = uint32_t;
    __device__ static U to(int32_t v) { return (U)v; }
    __device__ static int32_t from(U u) { return (int32_t)u; }
};
template <> struct Bits<unsigned long long> {
    using U = uint64_t;
    __device__ static U to(unsigned long long v) { return (U)v; }
    __device__ static unsigned long long from(U u) { return (unsigned long long)u; }
};

template <int CTRL, typename T>
__device__ __forceinline__ T dpp(T v)
{
    using B = Bits<T>;
    if constexpr (sizeof(typename B::U) == 8)
        return B::from(dpp64<CTRL>(B::to(v)));
    else
        return B::from(dpp32<CTRL>(B::to(v)));
}
template <typename T>
__device__ __forceinline__ T readlane(T v, int lane)
{
    using B = Bits<T>;
    if constexpr (sizeof(typename B::U) == 8)
        return B::from(readlane64(B::to(v), lane));
    else
        return B::from((typename B::U)__builtin_amdgcn_readlane((int)B::to(v), lane));
}
template <typename T>
__device__ __forceinline__ T tmin(T a, T b)
{
    if constexpr (sizeof(T) == 8 && !__is_same(T, unsigned long long))
        return __builtin_fmin(a, b);  // v_min_f64
    else
        return b < a ? b : a;
}
}  // namespace wave_detail

// minimum over the 64 lanes of the wave (every lane active), wave-uniform
template <typename T>
__device__ __forceinline__ T wave_min_dpp(T v)
{
    using namespace wave_detail;
    v = tmin(v, dpp<kDppXor1>(v));
    v = tmin(v, dpp<kDppXor2>(v));
    v = tmin(v, dpp<kDppHalfMirror>(v));
    v = tmin(v, dpp<kDppMirror>(v));
    return tmin(tmin(readlane(v, 0), readlane(v, 16)), tmin(readlane(v, 32), readlane(v, 48)));
}

}  // namespace tspgpu
