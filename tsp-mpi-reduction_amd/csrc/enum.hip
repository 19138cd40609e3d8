// K2e — exhaustive enumeration of ONE instance on gfx950 (BASELINE config 2,
// "14-city exhaustive enumeration on 1 MI355X").
//
// Every one of the (n-1)! tours of the reference's tsp() problem
// (tsp.cpp:405-509) is folded in the reference's left-to-right order
// ((d[0][t1] + d[t1][t2]) + ...) + d[tN][0], so the minimum
// and the recorded optimal tours are bit-exact; the tour tsp() returns is then
// picked from the records by the DP's own tie rule (search_abi.cpp,
// select_tour), exactly as for the branch-and-bound kernels in search.hip.
//
// Shape: one lane per depth-G prefix (0, t1..tG) with G = N - 6, N = n - 1.
//   * the prefix index is decoded in registers (mixed radix N, N-1, ..,
//     divisions by compile-time constants; the unused cities kept as a nibble
//     list, so picking and removing a city is two shifts and a mask),
//   * the prefix cost is folded from the distance matrix in LDS (G reads),
//   * the six cities left are loaded once as a 6x6 sub-matrix (+ the edges
//     from the prefix end and to city 0: 42 LDS reads) into VGPRs, and all
//     6! = 720 completions are folded by fully unrolled code: 1,956 partial
//     paths (the "search nodes", one add each) + 720 closing adds + 720
//     v_min_f64 — about 3,400 VALU lane-ops per lane and no memory traffic,
//     so the kernel is bound by VALU issue (2 ops per node).
//   * a lane whose best completion is within the incumbent (rare: the host
//     seeds the incumbent with a 2-opt tour) re-walks its 720 tours with
//     rolled loops and records every tour within the incumbent (atomicMin on
//     the 64-bit cost word, then a record slot), like search.hip.
// No bound, no queue, no rounds: the enumeration is uniform, a grid-stride
// loop over the prefixes balances it.
#include <hip/hip_runtime.h>

#include <utility>

#include "search.h"

namespace tspgpu {
namespace {

constexpr int kTail = 6;     // cities enumerated in registers
constexpr int kERow = 16;    // LDS row stride (n <= 16)
constexpr int kTailNodes = 6 + 30 + 120 + 360 + 720 + 720;  // partial paths below a depth-G prefix

template <typename V>
struct ENum;
template <>
struct ENum<double> {
    __device__ static uint64_t bits(double v) { return (uint64_t)__double_as_longlong(v); }
    __device__ static double val(uint64_t b) { return __longlong_as_double((long long)b); }
    __device__ static double vmin(double x, double y) { return __builtin_fmin(x, y); }
    __device__ static double big() { return 1.0e300; }  // above every tour cost
};
template <>
struct ENum<int32_t> {
    __device__ static uint64_t bits(int32_t v) { return (uint64_t)(uint32_t)v; }
    __device__ static int32_t val(uint64_t b) { return (int32_t)(uint32_t)b; }
    __device__ static int32_t vmin(int32_t x, int32_t y) { return x < y ? x : y; }
    __device__ static int32_t big() { return 2147483647; }
};

template <typename F, int... I>
__device__ __forceinline__ void static_for(F &&f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}

// All completions of the path ending at tail city LAST (cost p) through the
// tail cities in LEFT (bit mask over 0..5), then back to city 0.  The
// recursion is resolved at compile time: straight-line adds and mins.
template <typename V, int LEFT, int LAST>
__device__ __forceinline__ void complete(const V (&s)[kTail][kTail], const V (&d0)[kTail], V p, V &best)
{
    if constexpr ((LEFT & (LEFT - 1)) == 0) {
        constexpr int r = __builtin_ctz(LEFT);
        best = ENum<V>::vmin(best, (p + s[LAST][r]) + d0[r]);
    } else {
        static_for(
            [&](auto q) {
                constexpr int Q = decltype(q)::value;
                if constexpr ((LEFT >> Q) & 1) complete<V, (LEFT & ~(1 << Q)), Q>(s, d0, p + s[LAST][Q], best);
            },
            std::make_integer_sequence<int, kTail>{});
    }
}

template <typename V, int NN>
__global__ __launch_bounds__(256) void enum_kernel(SearchArgs a)
{
    constexpr int N = NN - 1;  // inner cities 1..N
    constexpr int G = N - kTail;
    static_assert(G >= 0 && NN <= 16, "enum_kernel: 7 <= n <= 16");
    __shared__ V dl[NN * kERow];
    const V *gd = static_cast<const V *>(a.dist);
    for (int i = threadIdx.x; i < NN * NN; i += blockDim.x) dl[(i / NN) * kERow + i % NN] = gd[i];
    __syncthreads();

    unsigned long long lanes = 0;  // wave-uniform
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < a.items; base += stride) {
        const uint32_t idx = base + threadIdx.x;
        const bool act = idx < a.items;
        lanes += (unsigned long long)__popcll(__ballot(act));
        // ---- decode the prefix: digit l picks the dig[l]-th unused city
        int dig[G > 0 ? G : 1];
        uint32_t x = act ? idx : 0u;
#pragma unroll
        for (int l = G - 1; l >= 0; --l) {
            const uint32_t r = (uint32_t)(N - l);
            dig[l] = (int)(x % r);
            x /= r;
        }
        uint64_t list = 0;  // unused cities 1..N, ascending, one per nibble
#pragma unroll
        for (int c = 1; c <= N; ++c) list |= (uint64_t)c << (4 * (c - 1));
        int pc[G > 0 ? G : 1];
        int prev = 0;
        V cp = 0;
#pragma unroll
        for (int l = 0; l < G; ++l) {
            const int sh = 4 * dig[l];
            const int c = (int)((list >> sh) & 15u);
            list = (list & ((1ull << sh) - 1ull)) | ((list >> (sh + 4)) << sh);
            cp = cp + dl[prev * kERow + c];  // the reference's left fold
            prev = c;
            pc[l] = c;
        }
        const uint32_t rest = (uint32_t)list;  // the six cities left, ascending
        int t[kTail];
#pragma unroll
        for (int i = 0; i < kTail; ++i) t[i] = (int)((rest >> (4 * i)) & 15u);
        V s[kTail][kTail], d0[kTail], dk[kTail];
#pragma unroll
        for (int i = 0; i < kTail; ++i) {
            dk[i] = dl[prev * kERow + t[i]];
            d0[i] = dl[t[i] * kERow];
#pragma unroll
            for (int j = 0; j < kTail; ++j)
                if (j != i) s[i][j] = dl[t[i] * kERow + t[j]];
        }
        // ---- all 720 completions in registers
        V best = ENum<V>::big();
        static_for(
            [&](auto i) {
                constexpr int I = decltype(i)::value;
                complete<V, (((1 << kTail) - 1) & ~(1 << I)), I>(s, d0, cp + dk[I], best);
            },
            std::make_integer_sequence<int, kTail>{});
        V inc = ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (act && best <= inc) {
            // rare: record every tour within the incumbent (rolled loops, same fold)
            for (int p = 0; p < 720; ++p) {
                uint32_t lst = rest;
                int ord[kTail];
                int q = p;
#pragma unroll
                for (int l = 0; l < kTail; ++l) {
                    const int r = kTail - l;
                    int fact = 1;  // (r-1)!: the l-th city is digit q / (r-1)! of the r left
                    for (int z = 2; z < r; ++z) fact *= z;
                    const int dgt = q / fact;
                    q -= dgt * fact;
                    const int sh = 4 * dgt;
                    ord[l] = (int)((lst >> sh) & 15u);
                    lst = (lst & ((1u << sh) - 1u)) | ((lst >> (sh + 4)) << sh);
                }
                V c = cp;
                int k = prev;
#pragma unroll
                for (int l = 0; l < kTail; ++l) {
                    c = c + dl[k * kERow + ord[l]];
                    k = ord[l];
                }
                const V total = c + dl[k * kERow];
                if (total <= inc) {
                    const uint64_t tb = ENum<V>::bits(total);
                    const unsigned long long old = atomicMin(a.inc, (unsigned long long)tb);
                    if (tb <= old) {
                        const unsigned int slot = atomicAdd(a.rec_count, 1u);
                        if (slot < a.rec_cap) {
                            SearchRecord *R = a.rec + slot;
                            R->cost = tb;
                            for (int l = 0; l < G; ++l) R->city[l] = (uint8_t)pc[l];
#pragma unroll
                            for (int l = 0; l < kTail; ++l) R->city[G + l] = (uint8_t)ord[l];
                        }
                    }
                    const V o = ENum<V>::val(old);
                    inc = o < total ? o : total;
                }
            }
        }
    }
    if (__lane_id() == 0) atomicAdd(a.nodes, lanes * (unsigned long long)kTailNodes);
}

template <typename V, int NN>
hipError_t launch_n(const SearchArgs &a, int grid)
{
    hipLaunchKernelGGL((enum_kernel<V, NN>), dim3(grid), dim3(256), 0, a.stream, a);
    return hipGetLastError();
}

template <typename V>
hipError_t launch_v(const SearchArgs &a, int grid)
{
    switch (a.n) {
    case 7: return launch_n<V, 7>(a, grid);
    case 8: return launch_n<V, 8>(a, grid);
    case 9: return launch_n<V, 9>(a, grid);
    case 10: return launch_n<V, 10>(a, grid);
    case 11: return launch_n<V, 11>(a, grid);
    case 12: return launch_n<V, 12>(a, grid);
    case 13: return launch_n<V, 13>(a, grid);
    case 14: return launch_n<V, 14>(a, grid);
    case 15: return launch_n<V, 15>(a, grid);
    case 16: return launch_n<V, 16>(a, grid);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_enum(const SearchArgs &a, bool f64, int grid)
{
    return f64 ? launch_v<double>(a, grid) : launch_v<int32_t>(a, grid);
}

}  // namespace tspgpu
