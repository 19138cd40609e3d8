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

#include <algorithm>
#include <utility>

#include "search.h"
#include "wave.h"

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
// tail cities in LEFT (bit mask over 0..TL-1), then back to city 0.  The
// recursion is resolved at compile time: straight-line adds and mins.
template <typename V, int TL, int LEFT, int LAST>
__device__ __forceinline__ void complete(const V (&s)[TL][TL], const V (&d0)[TL], V p, V &best)
{
    if constexpr ((LEFT & (LEFT - 1)) == 0) {
        constexpr int r = __builtin_ctz(LEFT);
        best = ENum<V>::vmin(best, (p + s[LAST][r]) + d0[r]);
    } else {
        static_for(
            [&](auto q) {
                constexpr int Q = decltype(q)::value;
                if constexpr ((LEFT >> Q) & 1) complete<V, TL, (LEFT & ~(1 << Q)), Q>(s, d0, p + s[LAST][Q], best);
            },
            std::make_integer_sequence<int, TL>{});
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
    TieCache tcache;
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
                complete<V, kTail, (((1 << kTail) - 1) & ~(1 << I)), I>(s, d0, cp + dk[I], best);
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
                        tie_offer(a, tcache, tb, [&](int q) {
                            int v = 0;  // (static indices: the arrays stay in registers)
#pragma unroll
                            for (int l = 0; l < G; ++l) v = q == l + 1 ? pc[l] : v;
#pragma unroll
                            for (int l = 0; l < kTail; ++l) v = q == G + 1 + l ? ord[l] : v;
                            return v;
                        });
                    }
                    const V o = ENum<V>::val(old);
                    inc = o < total ? o : total;
                }
            }
        }
    }
    if (__lane_id() == 0) atomicAdd(stat_line(a), lanes * (unsigned long long)kTailNodes);
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

// ---------------------------------------------------------------------------
// Register tails of the frontier search: every prefix in a.ftail (written
// by expand_kernel) has exactly TL cities left; a lane refolds
// the prefix (the same left fold, from LDS), tests it against the current
// incumbent with the search's bound (cheapest incoming edge of every city
// still to be entered, 2^-20 grid values, exact sums), and folds all TL!
// completions with the straight-line code above.  Tours within the incumbent
// are recorded exactly like the DFS records them, so the optimal set — and
// the tie rule's answer — is unchanged; pruning inside the tail is dropped
// because a DFS step costs ~1000x a register add.
constexpr int kTRow = 32;  // LDS row stride (n <= 32)

template <typename V>
struct EThr;  // prune iff bound > thr (the round kernel's margin)
template <>
struct EThr<double> {
    __device__ static double of(double inc) { return inc * (1.0 + 0x1p-39); }
};
template <>
struct EThr<int32_t> {
    __device__ static int32_t of(int32_t inc) { return inc; }
};

__host__ __device__ constexpr unsigned long long tail_nodes(int tl)
{
    unsigned long long sum = 0, f = 1;
    for (int l = 1; l <= tl; ++l) {
        f *= (unsigned long long)(tl - l + 1);
        sum += f;
    }
    return sum;
}

// A frontier path in registers: two dwordx4 loads.
// path i of a frontier step's input (up to four segments, SearchArgs::fseg)
__device__ __forceinline__ const PathItem *fin_at(const SearchArgs &a, uint32_t i)
{
    const PathItem *p = a.fseg[0];
    uint32_t st = 0;
    if (a.nseg > 1 && i >= a.fseg_start[1]) p = a.fseg[1], st = a.fseg_start[1];
    if (a.nseg > 2 && i >= a.fseg_start[2]) p = a.fseg[2], st = a.fseg_start[2];
    if (a.nseg > 3 && i >= a.fseg_start[3]) p = a.fseg[3], st = a.fseg_start[3];
    return p + (i - st);
}

__device__ __forceinline__ void load_path(const PathItem *p, bool act, uint32_t (&w)[8])
{
    if (act) {
        const uint4 lo = reinterpret_cast<const uint4 *>(p)[0];
        const uint4 hi = reinterpret_cast<const uint4 *>(p)[1];
        w[0] = lo.x, w[1] = lo.y, w[2] = lo.z, w[3] = lo.w;
        w[4] = hi.x, w[5] = hi.y, w[6] = hi.z, w[7] = hi.w;
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b) w[b] = 0u;
    }
}

// The left fold ((d[0][t1] + d[t1][t2]) + ...) of the path in w (len cities),
// its end city and its members, from the matrix in LDS.
// The distances of eight positions are read before any of them is added (the
// addresses come from the path bytes alone, and every byte indexes inside the
// 32 x 32 table): one LDS round trip per eight cities instead of one per city;
// the adds stay in path order.
template <typename V>
__device__ __forceinline__ void fold_path(const V *dl, const uint32_t (&w)[8], int len, V &c, int &k, uint32_t &mem)
{
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        if (8 * g >= len) break;
        V v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int lv = 8 * g + q;
            const int t = (int)((w[lv >> 2] >> (8 * (lv & 3))) & 31u);
            const int pl = lv - 1;
            const int p = pl <= 0 ? 0 : (int)((w[pl >> 2] >> (8 * (pl & 3))) & 31u);
            v[q] = lv >= 1 ? dl[p * kTRow + t] : V(0);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int lv = 8 * g + q;
            if (lv >= 1 && lv < len) {
                const int t = (int)((w[lv >> 2] >> (8 * (lv & 3))) & 255u);
                c = c + v[q];
                mem |= 1u << t;
                k = t;
            }
        }
    }
}

// byte l of a path's words (a select chain: no dynamically indexed registers)
__device__ __forceinline__ int path_byte(const uint32_t (&w)[8], int l)
{
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) v = (l >> 2) == b ? w[b] : v;
    return (int)((v >> (8 * (l & 3))) & 255u);
}

// One handed-over prefix (slot idx of a.ftail): refold, bound test, all
// TL! completions; `act` false = a lane with nothing to do (wave-uniform code).
// (A wave with only a few prefixes takes tail_wide below instead.)
template <typename V, int TL>
__device__ __forceinline__ void tail_one(const SearchArgs &a, const V *dl, const V *am, uint32_t full,
                                         const uint32_t (&w)[8], bool act, unsigned long long &lanes,
                                         TieCache &tcache)
{
    const int len = act ? (int)(w[0] & 255u) : 1;
    // ---- the prefix 0, t1..t(len-1): the reference's left fold
    V cp = 0;
    int prev = 0;
    uint32_t mem = 0;
    fold_path<V>(dl, w, len, cp, prev, mem);
    const uint32_t rest = full & ~mem;  // the TL cities left
    int t[TL];
    uint32_t tpack = 0;  // t[i] in bits 5i..5i+4 (record path)
    V ra = am[0];
    uint32_t x = rest;
#pragma unroll
    for (int i = 0; i < TL; ++i) {
        t[i] = x ? __builtin_ctz(x) : 0;
        x &= x - 1u;
        ra += am[t[i]];
        tpack |= (uint32_t)t[i] << (5 * i);
    }
    V inc = ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (!a.noprune && cp + ra > EThr<V>::of(inc)) act = false;
    const unsigned long long am_ = __ballot(act);
    if (am_ == 0) return;
    lanes += (unsigned long long)__popcll(am_);
    V s[TL][TL], d0[TL], dk[TL];
#pragma unroll
    for (int i = 0; i < TL; ++i) {
        dk[i] = dl[prev * kTRow + t[i]];
        d0[i] = dl[t[i] * kTRow];
#pragma unroll
        for (int j = 0; j < TL; ++j)
            if (j != i) s[i][j] = dl[t[i] * kTRow + t[j]];
    }
    // per first tail city g the best of its (TL-1)! completions
    V bg[TL];
    static_for(
        [&](auto i) {
            constexpr int I = decltype(i)::value;
            bg[I] = ENum<V>::big();
            complete<V, TL, (((1 << TL) - 1) & ~(1 << I)), I>(s, d0, cp + dk[I], bg[I]);
        },
        std::make_integer_sequence<int, TL>{});
    V best = bg[0];
#pragma unroll
    for (int i = 1; i < TL; ++i) best = ENum<V>::vmin(best, bg[i]);
    // rare: record every tour within the incumbent (same fold, enumeration
    // order), only in the first-city groups whose best is within it.  The
    // lanes that have such groups are served one at a time by the whole wave,
    // each lane folding every 64th of the group's (TL-1)! orders.
    (void)best;
    constexpr int kGroup = TL == 6 ? 120 : 24;  // (TL-1)!
    uint32_t gm = 0;  // groups of this lane within the incumbent
#pragma unroll
    for (int g = 0; g < TL; ++g) gm |= (act && bg[g] <= inc) ? (1u << g) : 0u;
    for (unsigned long long owners = __ballot(gm != 0); owners; owners &= owners - 1ull) {
        const int o = __ffsll((long long)owners) - 1;
        const uint32_t ogm = (uint32_t)__shfl((int)gm, o);
        const uint32_t otp = (uint32_t)__shfl((int)tpack, o);
        const int oprev = __shfl(prev, o), olen = __shfl(len, o);
        uint32_t ow[8];  // the owner's path words (its record's and tie key's first cities)
#pragma unroll
        for (int b = 0; b < 8; ++b) ow[b] = (uint32_t)__shfl((int)w[b], o);
        V ocp;
        if constexpr (sizeof(V) == 8)
            ocp = __longlong_as_double(__shfl((long long)__double_as_longlong(cp), o));
        else
            ocp = (V)__shfl((int)cp, o);
        // ONE atomicMin per owner, with its best completion (round 5): the
        // incumbent it returns, lowered by that best, is the bound every order
        // below is recorded against — the optimal tours still all pass (a
        // lane's best is never below the optimum), and no order waits on an
        // atomicMin of its own (before: one dependent atomicMin per improving
        // order, the tail's critical path)
        V obest;
        if constexpr (sizeof(V) == 8)
            obest = __longlong_as_double(__shfl((long long)__double_as_longlong(best), o));
        else
            obest = (V)__shfl((int)best, o);
        unsigned long long oinc = 0;
        if (__lane_id() == 0) oinc = atomicMin(a.inc, (unsigned long long)ENum<V>::bits(obest));
        oinc = (unsigned long long)__shfl((long long)oinc, 0);
        const V cur = ENum<V>::vmin(ENum<V>::val(oinc), obest);
        for (uint32_t gg = ogm; gg; gg &= gg - 1u) {
            const int g = __builtin_ctz(gg);
            for (int p = g * kGroup + __lane_id(); p < (g + 1) * kGroup; p += 64) {
                uint32_t lst = 0;  // indices 0..TL-1 not used yet, one per nibble
#pragma unroll
                for (int i = 0; i < TL; ++i) lst |= (uint32_t)i << (4 * i);
                int ord[TL];
                int q = p;
#pragma unroll
                for (int l = 0; l < TL; ++l) {
                    const int r = TL - l;
                    int fact = 1;  // (r-1)!: the l-th city is digit q / (r-1)! of the r left
                    for (int z = 2; z < r; ++z) fact *= z;
                    const int dgt = q / fact;
                    q -= dgt * fact;
                    const int sh = 4 * dgt;
                    const int ix = (int)((lst >> sh) & 15u);
                    lst = (lst & ((1u << sh) - 1u)) | ((lst >> (sh + 4)) << sh);
                    ord[l] = (int)((otp >> (5 * ix)) & 31u);
                }
                V c = ocp;
                int k = oprev;
#pragma unroll
                for (int l = 0; l < TL; ++l) {
                    c = c + dl[k * kTRow + ord[l]];
                    k = ord[l];
                }
                const V total = c + dl[k * kTRow];
                if (total <= cur) {
                    // (total <= cur <= the incumbent the atomicMin returned: a
                    // record slot only for such tours — rec_count decides the
                    // -EOVERFLOW / second-phase fallback)
                    const uint64_t tb = ENum<V>::bits(total);
                    const unsigned int slot = atomicAdd(a.rec_count, 1u);
                    if (slot < a.rec_cap) {
                        SearchRecord *R = a.rec + slot;
                        R->cost = tb;
                        for (int l = 1; l < olen; ++l) R->city[l - 1] = (uint8_t)path_byte(ow, l);
#pragma unroll
                        for (int l = 0; l < TL; ++l) R->city[olen - 1 + l] = (uint8_t)ord[l];
                    }
                    tie_offer(a, tcache, tb, [&](int q) {
                        int v = 0;
#pragma unroll
                        for (int l = 0; l < TL; ++l) v = q == olen + l ? ord[l] : v;
                        return q < olen ? path_byte(ow, q) : v;
                    });
                }
            }
        }
    }
}

// permutation idx (0..23, lexicographic) of {0,1,2,3}: element at position pos
__host__ __device__ constexpr int perm4(int idx, int pos)
{
    int avail[4] = {0, 1, 2, 3};
    const int f[4] = {6, 2, 1, 1};
    int n = 4, res = 0;
    for (int p = 0; p <= pos; ++p) {
        const int d = idx / f[p];
        idx %= f[p];
        res = avail[d];
        for (int k = d; k < n - 1; ++k) avail[k] = avail[k + 1];
        --n;
    }
    return res;
}
// v[i] / m[i][j] for a runtime i, j by selects (no dynamically indexed registers)
template <typename T>
__device__ __forceinline__ T sel4(const T (&v)[4], int i)
{
    return i == 0 ? v[0] : (i == 1 ? v[1] : (i == 2 ? v[2] : v[3]));
}
template <typename T>
__device__ __forceinline__ T sel44(const T (&m)[4][4], int i, int j)
{
    const T r[4] = {sel4(m[0], j), sel4(m[1], j), sel4(m[2], j), sel4(m[3], j)};
    return sel4(r, i);
}

// A wave with only a few prefixes (<= kTailWide; e.g. the two tails of the
// reference's 16-city instance): tail_one's per-lane TL! chain would leave 63
// lanes idle for ~20 us, so the prefixes' completions are split over the
// lanes instead — one lane per (prefix, first tail city, second tail city),
// each folding the (TL-2)! = 24 orders of the other four by the same
// straight-line `complete` — and the tours within the incumbent are recorded
// and offered to the tie rule exactly as in tail_one (TL = 6 only).
template <typename V, int TL>
__device__ __forceinline__ void tail_wide(const SearchArgs &a, const V *dl, const V *am, uint32_t full,
                                          const uint32_t (&w)[8], bool act, unsigned long long &lanes,
                                          TieCache &tcache)
{
    static_assert(TL == 6, "tail_wide: six tail cities");
    const int len = act ? (int)(w[0] & 255u) : 1;
    V cp = 0;
    int prev = 0;
    uint32_t mem = 0;
    fold_path<V>(dl, w, len, cp, prev, mem);
    const uint32_t rest = full & ~mem;
    uint32_t tpack = 0;
    V ra = am[0];
    uint32_t x = rest;
#pragma unroll
    for (int i = 0; i < TL; ++i) {
        const int t = x ? __builtin_ctz(x) : 0;
        x &= x - 1u;
        ra += am[t];
        tpack |= (uint32_t)t << (5 * i);
    }
    V cur = ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (!a.noprune && cp + ra > EThr<V>::of(cur)) act = false;
    const unsigned long long owners = __ballot(act);
    if (owners == 0) return;
    const int nown = __popcll(owners);
    lanes += (unsigned long long)nown;
    constexpr int kPairs = TL * (TL - 1);
    for (int base = 0; base < nown * kPairs; base += 64) {  // (wave-uniform)
        const int combo = base + __lane_id();
        const bool on = combo < nown * kPairs;
        const int oi = on ? combo / kPairs : 0, pr = on ? combo % kPairs : 0;
        int o = 0;  // the oi-th owner lane
        {
            unsigned long long m = owners;
            for (int k = 0; k < oi; ++k) m &= m - 1ull;
            o = __ffsll((long long)m) - 1;
        }
        const uint32_t otp = (uint32_t)__shfl((int)tpack, o);
        const int oprev = __shfl(prev, o), olen = __shfl(len, o);
        V ocp;
        if constexpr (sizeof(V) == 8)
            ocp = __longlong_as_double(__shfl((long long)__double_as_longlong(cp), o));
        else
            ocp = (V)__shfl((int)cp, o);
        uint32_t ow[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) ow[b] = (uint32_t)__shfl((int)w[b], o);
        const int i = pr / (TL - 1), jj = pr % (TL - 1), j = jj < i ? jj : jj + 1;
        const int ti = (int)((otp >> (5 * i)) & 31u), tj = (int)((otp >> (5 * j)) & 31u);
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        int r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int p = k;
            p += p >= lo ? 1 : 0;
            p += p >= hi ? 1 : 0;
            r[k] = (int)((otp >> (5 * p)) & 31u);
        }
        V s4[4][4], d04[4], dk4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            d04[u] = dl[r[u] * kTRow];
            dk4[u] = dl[tj * kTRow + r[u]];
#pragma unroll
            for (int v = 0; v < 4; ++v) s4[u][v] = u == v ? (V)0 : dl[r[u] * kTRow + r[v]];
        }
        const V pj = (ocp + dl[oprev * kTRow + ti]) + dl[ti * kTRow + tj];
        V best = ENum<V>::big();
        static_for(
            [&](auto q) {
                constexpr int Q = decltype(q)::value;
                complete<V, 4, (15 & ~(1 << Q)), Q>(s4, d04, pj + dk4[Q], best);
            },
            std::make_integer_sequence<int, 4>{});
        // rare: this lane's orders within the incumbent.  ONE atomicMin with
        // the lane's best, ONE record-slot range for the orders within the
        // bound it returns (all at the lane's best) and ONE tie offer, of the
        // least key among them (the slot keeps the least key anyway): the
        // 24-step loop below only stores.  Per-order atomics in that loop,
        // taken by a different lane at every step, cost ~21 us of the 16-city
        // chain's ~98 (round-5 ablation builds, profiles/r05/k2_tail_ablation.txt).
        if (!(on && best <= cur)) continue;
        const unsigned long long linc = atomicMin(a.inc, (unsigned long long)ENum<V>::bits(best));
        cur = ENum<V>::vmin(ENum<V>::val(linc), best);
        // order pi of the four: lexicographic permutation pi of {0,1,2,3},
        // decoded arithmetically (a __constant__ table read per step was a
        // dependent memory round trip per order: ~18 us of the 16-city chain)
        auto total_of = [&](int pi, int (&ax)[4]) {
            uint32_t lst = 0x3210u;  // indices not used yet, one per nibble
            int q = pi;
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const int fact = l == 0 ? 6 : (l == 1 ? 2 : 1);
                const int dgt = q / fact;
                q -= dgt * fact;
                const int sh = 4 * dgt;
                ax[l] = (int)((lst >> sh) & 15u);
                lst = (lst & ((1u << sh) - 1u)) | ((lst >> (sh + 4)) << sh);
            }
            V c = pj + sel4(dk4, ax[0]);
            c = c + sel44(s4, ax[0], ax[1]);
            c = c + sel44(s4, ax[1], ax[2]);
            c = c + sel44(s4, ax[2], ax[3]);
            return c + sel4(d04, ax[3]);
        };
        // the mask pass: the 24 orders at compile time (constant indices, no selects)
        uint32_t pass = 0;
        static_for(
            [&](auto i) {
                constexpr int PI = decltype(i)::value;
                constexpr int A0 = perm4(PI, 0), A1 = perm4(PI, 1), A2 = perm4(PI, 2), A3 = perm4(PI, 3);
                V c = pj + dk4[A0];
                c = c + s4[A0][A1];
                c = c + s4[A1][A2];
                c = c + s4[A2][A3];
                if (c + d04[A3] <= cur) pass |= 1u << PI;
            },
            std::make_integer_sequence<int, 24>{});
        if (!pass) continue;
        // keys first (VALU only), then the slot range and the tie offer issued
        // back to back (the offer's wait covers both round trips), then the
        // record stores (no later wait on them)
        const int N = a.n - 1;
        int kpi = -1;
        unsigned long long kw0 = ~0ull, kw1 = ~0ull;
        if (a.tie) {
#pragma unroll 1
            for (uint32_t pp = pass; pp; pp &= pp - 1u) {
                const int pi = __builtin_ctz(pp);
                int ax[4];
                (void)total_of(pi, ax);
                const int ord[TL] = {ti, tj, sel4(r, ax[0]), sel4(r, ax[1]), sel4(r, ax[2]), sel4(r, ax[3])};
                unsigned long long w0, w1;
                tie_key(N, [&](int q) {
                    int v = 0;
#pragma unroll
                    for (int l = 0; l < TL; ++l) v = q == olen + l ? ord[l] : v;
                    return q < olen ? path_byte(ow, q) : v;
                }, w0, w1);
                if (w0 < kw0 || (w0 == kw0 && w1 < kw1)) {
                    kw0 = w0;
                    kw1 = w1;
                    kpi = pi;
                }
            }
        }
        unsigned int slot = atomicAdd(a.rec_count, (unsigned int)__builtin_popcount(pass));  // (as tail_one)
        if (kpi >= 0) {
            int ax[4];
            const V total = total_of(kpi, ax);
            const int ord[TL] = {ti, tj, sel4(r, ax[0]), sel4(r, ax[1]), sel4(r, ax[2]), sel4(r, ax[3])};
            tie_offer(a, tcache, ENum<V>::bits(total), [&](int q) {
                int v = 0;
#pragma unroll
                for (int l = 0; l < TL; ++l) v = q == olen + l ? ord[l] : v;
                return q < olen ? path_byte(ow, q) : v;
            });
        }
#pragma unroll 1
        for (uint32_t pp = pass; pp; pp &= pp - 1u, ++slot) {
            if (slot >= a.rec_cap) break;
            const int pi = __builtin_ctz(pp);
            int ax[4];
            const V total = total_of(pi, ax);
            const int ord[TL] = {ti, tj, sel4(r, ax[0]), sel4(r, ax[1]), sel4(r, ax[2]), sel4(r, ax[3])};
            SearchRecord *R = a.rec + slot;
            R->cost = ENum<V>::bits(total);
            for (int l = 1; l < olen; ++l) R->city[l - 1] = (uint8_t)path_byte(ow, l);
#pragma unroll
            for (int l = 0; l < TL; ++l) R->city[olen - 1 + l] = (uint8_t)ord[l];
        }
    }
}

// Every wave reads 64 slots at a time, queues the non-empty ones (len > 0) in
// LDS and folds them 64 at a time, so a producer may leave holes without
// idling lanes here.  A batch of at most kTailWide prefixes is folded wide
// (tail_wide: the lanes over each prefix's first two tail cities).
constexpr uint32_t kTailWide = 4;
template <typename V, int TL>
__global__ __launch_bounds__(256) void tail_kernel(SearchArgs a)
{
    __shared__ V dl[kSearchMaxN * kTRow];
    __shared__ V am[kSearchMaxN];
    __shared__ uint4 wq[4][128][2];  // queued prefixes' words (read once, in the queue pass)
    const int n = a.n;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    // a chained search whose level overflowed is abandoned: its tail slots may
    // hold paths nobody wrote (stale or uninitialised memory), so none is read;
    // and a block beyond the waiting tails leaves before staging its tables
    __shared__ uint32_t dead;
    const unsigned int claimed = __hip_atomic_load(a.tail_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t count = claimed < a.tail_cap ? claimed : a.tail_cap;
    if (threadIdx.x == 0) dead = a.overflow ? __hip_atomic_load(a.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    __syncthreads();
    if (dead || blockIdx.x * 256u >= count) return;  // (block-uniform: count is one load of one word)
    for (int i = threadIdx.x; i < n * n; i += blockDim.x) dl[(i / n) * kTRow + i % n] = gd[i];
    for (int i = threadIdx.x; i < n; i += blockDim.x) am[i] = ga[i];
    __syncthreads();

    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    const int lane = __lane_id();
    uint4 (*q)[2] = wq[threadIdx.x >> 6];
    uint32_t qn = 0;               // wave-uniform: live slots queued
    unsigned long long lanes = 0;  // wave-uniform
    TieCache tcache;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), waves = gridDim.x * 4;
    for (uint32_t base = wave * 64u;; base += waves * 64u) {
        const bool more = base < count;
        if (more) {
            const uint32_t idx = base + lane;
            const bool in = idx < count;
            const uint4 lo = in ? reinterpret_cast<const uint4 *>(a.ftail + idx)[0] : make_uint4(0, 0, 0, 0);
            const uint4 hi = in ? reinterpret_cast<const uint4 *>(a.ftail + idx)[1] : make_uint4(0, 0, 0, 0);
            const bool live = in && (lo.x & 255u) != 0;
            const unsigned long long m = __ballot(live);
            if (live) {
                const uint32_t pos = qn + __popcll(m & ((1ull << lane) - 1ull));
                q[pos][0] = lo;
                q[pos][1] = hi;
            }
            qn += (uint32_t)__popcll(m);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        while (qn >= 64u || (!more && qn > 0u)) {
            const uint32_t take = qn < 64u ? qn : 64u;
            const bool act = (uint32_t)lane < take;
            uint32_t w[8];
            {
                const uint4 lo = act ? q[qn - take + lane][0] : make_uint4(0, 0, 0, 0);
                const uint4 hi = act ? q[qn - take + lane][1] : make_uint4(0, 0, 0, 0);
                w[0] = lo.x, w[1] = lo.y, w[2] = lo.z, w[3] = lo.w;
                w[4] = hi.x, w[5] = hi.y, w[6] = hi.z, w[7] = hi.w;
            }
            __builtin_amdgcn_wave_barrier();
            qn -= take;
            if constexpr (TL == 6) {
                if (take <= kTailWide) {
                    tail_wide<V, TL>(a, dl, am, full, w, act, lanes, tcache);
                    continue;
                }
            }
            tail_one<V, TL>(a, dl, am, full, w, act, lanes, tcache);
        }
        if (!more) break;
    }
    if (lane == 0) atomicAdd(stat_line(a), lanes * tail_nodes(TL));
}

// Frontier expansion, one level: a lane per path of a.fin (0, t1..t(len-1),
// refolded from LDS); every child j (ascending) whose bound passes becomes a
// path of a.ftail when it has tail_level inner cities, else of a.fout.  The
// host sizes both outputs for (N - depth) children per input path.
//
// Slots: device-scope atomics on one address serialise at ~20 ns each, so a
// block owns a contiguous run of a.fin_per_block paths and takes ONE range
// per output: pass 1 counts its live children, one atomicAdd per output,
// pass 2 re-evaluates (cheap: LDS + registers) and writes the children at
// block-scanned offsets.
// ---------------------------------------------------------------------------
// Stronger bounds of the frontier search (SearchArgs::bnd2, ::hsuf).
//
// Colex rank of a set of inner-city places c_0 < c_1 < ... (place = city - 1):
// sum_i C(c_i, i + 1); bn[m][k] = C(m, k) in LDS.
__device__ __forceinline__ void load_binom(uint32_t (*bn)[8])
{
    stage_search_binom(bn, threadIdx.x, blockDim.x);
}

// Suffix table of size TL = a.hs_len, one thread per set U of TL inner cities
// (colex rank r): H[U][x] for every x in U = the cheapest path from x over U
// to city 0, all (TL-1)! orders folded by the same straight-line code as the
// register tails (`complete`) — a bound only, compared with the incumbent's
// 2^-39 margin, so its rounding order does not matter.
// ---------------------------------------------------------------------------
// Seeds of the search (both modes) and the frontier prologue.
constexpr double kSeedShrink = 1.0 - 0x1p-40;
template <typename V>
struct SeedNum;
template <>
struct SeedNum<double> {
    using Wide = double;
    __device__ static double val(uint64_t b) { return __longlong_as_double((long long)b); }
    __device__ static bool pruned(double lb, double inc) { return lb * kSeedShrink > inc; }
};
template <>
struct SeedNum<int32_t> {
    using Wide = long long;
    __device__ static int32_t val(uint64_t b) { return (int32_t)(uint32_t)b; }
    __device__ static bool pruned(long long lb, int32_t inc) { return lb > (long long)inc; }
};

// Seed: every depth-D prefix of this shard that survives the bound becomes an item.
template <typename V>
__device__ __forceinline__ void seed_body(const SearchArgs &a, uint32_t block, uint32_t nblocks)
{
    using W = typename SeedNum<V>::Wide;
    __shared__ uint32_t pv[33];
    __shared__ V dl[kSearchMaxN * kSearchMaxN];
    __shared__ V al[kSearchMaxN];
    const int n = a.n, N = n - 1, D = a.depth;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    for (int i = threadIdx.x; i < n * n; i += kSearchThreads) dl[i] = gd[i];
    for (int i = threadIdx.x; i < n; i += kSearchThreads) al[i] = ga[i];
    if (threadIdx.x == 0) {
        uint32_t p = 1;
        pv[D] = 1;
        for (int l = D; l >= 2; --l) {
            p *= (uint32_t)(N - l + 1);
            pv[l - 1] = p;
        }
    }
    __syncthreads();
    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    W aall = 0;
    for (int x = 0; x < n; ++x) aall += (W)al[x];
    const V inc = SeedNum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t local = a.items / a.nshards + (a.items % a.nshards > a.shard ? 1u : 0u);
    const int lane = __lane_id();
    // the loop runs the same trip count on every lane of a wave (ballots inside)
    const uint32_t stride = nblocks * kSearchThreads;
    for (uint32_t i0 = block * kSearchThreads + (threadIdx.x & ~63u); i0 < local; i0 += stride) {
        const uint32_t i = i0 + (uint32_t)lane;
        uint32_t p = i * a.nshards + a.shard;
        uint32_t rr = full;
        W ra = aall;
        V c = 0;
        int prev = 0;
        bool live = i < local;
        uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // city bytes, statically indexed below
        for (int l = 1; l <= D && live; ++l) {
            const uint32_t q = p / pv[l];
            p -= q * pv[l];
            uint32_t x = rr;
            for (uint32_t s = 0; s < q; ++s) x &= x - 1u;
            const int t = __builtin_ctz(x);
            c = c + dl[prev * n + t];
            rr &= ~(1u << t);
            ra -= (W)al[t];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if ((l >> 2) == b) w[b] |= (uint32_t)t << (8 * (l & 3));
            prev = t;
            if (!a.noprune && SeedNum<V>::pruned((W)c + ra, inc)) live = false;
        }
        // one atomic per wave for its live prefixes
        const unsigned long long lm = __ballot(live);
        if (!lm) continue;
        const int leader = __ffsll((long long)lm) - 1;
        unsigned int base = 0;
        if (lane == leader) base = atomicAdd(a.out_count, (unsigned int)__popcll(lm));
        base = __shfl(base, leader);
        if (!live) continue;
        const uint32_t slot = base + __popcll(lm & ((1ull << lane) - 1ull));
        if (a.fout) {  // frontier search: the prefix as a path (byte 0 = len), two dwordx4
            uint4 *dp = reinterpret_cast<uint4 *>(a.fout + slot);
            dp[0] = make_uint4(w[0] | (uint32_t)(D + 1), w[1], w[2], w[3]);
            dp[1] = make_uint4(w[4], w[5], w[6], w[7]);
            continue;
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.out + slot);
#pragma unroll
        for (int b = 0; b < 8; ++b) dst[b] = w[b];
        dst[8] = (uint32_t)(D + 1) | (1u << 8);  // len, from = 1
    }
}

template <typename V>
__global__ __launch_bounds__(kSearchThreads) void seed_kernel(SearchArgs a)
{
    // (a chain without the suffix table starts here: its clock, as the prologue's)
    if (a.t_start && blockIdx.x == 0 && threadIdx.x == 0) *a.t_start = wall_clock64();
    seed_body<V>(a, blockIdx.x, gridDim.x);
}

// The cheapest completion from tail city I over the other TL - 1 (straight
// through them, then to city 0) as a left-fold DP over subsets, layer by
// layer: f[S][y] = the cheapest path from I over S ending at y, each path's
// cost summed from I forward like `complete` does.  fl(a + d) is monotone in
// a, so fl(min_P fl(P) + d) = min_P fl(fl(P) + d): every f[S][y] — and the
// result — is bit-identical to the minimum over all (TL-1)! orders that
// `complete` folds, at 165 adds instead of 445 for TL = 6.
template <typename V, int TL, int I>
__device__ __forceinline__ V suffix_dp(const V (&s)[TL][TL], const V (&d0)[TL])
{
    constexpr int R = ((1 << TL) - 1) & ~(1 << I);
    V f[1 << TL][TL];
    static_for(
        [&](auto kk) {
            constexpr int K = decltype(kk)::value + 1;  // |S|
            static_for(
                [&](auto ss) {
                    constexpr int S = decltype(ss)::value;
                    if constexpr ((S & ~R) == 0 && __builtin_popcount(S) == K) {
                        static_for(
                            [&](auto yy) {
                                constexpr int Y = decltype(yy)::value;
                                if constexpr ((S >> Y) & 1) {
                                    if constexpr (K == 1) {
                                        f[S][Y] = V(0) + s[I][Y];
                                    } else {
                                        constexpr int P = S & ~(1 << Y), Z0 = __builtin_ctz(P);
                                        V m = f[P][Z0] + s[Z0][Y];
                                        static_for(
                                            [&](auto zz) {
                                                constexpr int Z = decltype(zz)::value;
                                                if constexpr (Z > Z0 && ((P >> Z) & 1)) m = ENum<V>::vmin(m, f[P][Z] + s[Z][Y]);
                                            },
                                            std::make_integer_sequence<int, TL>{});
                                        f[S][Y] = m;
                                    }
                                }
                            },
                            std::make_integer_sequence<int, TL>{});
                    }
                },
                std::make_integer_sequence<int, 1 << TL>{});
        },
        std::make_integer_sequence<int, TL - 1>{});
    V best = ENum<V>::big();
    static_for(
        [&](auto yy) {
            constexpr int Y = decltype(yy)::value;
            if constexpr ((R >> Y) & 1) best = ENum<V>::vmin(best, f[R][Y] + d0[Y]);
        },
        std::make_integer_sequence<int, TL>{});
    return best;
}

template <typename V, int TL>
__device__ __forceinline__ void suffix_body(const SearchArgs &a, uint32_t sets, uint32_t block, uint32_t nblocks)
{
    __shared__ uint32_t bn[32][8];
    __shared__ double dl[kSearchMaxN * kTRow];
    const int n = a.n;
    const V *gd = static_cast<const V *>(a.dist);
    for (int i = threadIdx.x; i < n * n; i += blockDim.x) dl[(i / n) * kTRow + i % n] = (double)gd[i];
    load_binom(bn);
    __syncthreads();
    double *H = const_cast<double *>(a.hsuf) + a.hs_off[TL];
    // one thread per (set, place x): wave w serves place I = w % TL of 64
    // sets (I wave-uniform: one straight-line `complete` per wave), so the
    // table's (TL-1)!-order chains spread over TL times the waves (the
    // prologue's critical path: 14 us at 16 cities with a thread per set)
    for (uint32_t g0 = block * 256u + (threadIdx.x & ~63u);; g0 += nblocks * 256u) {
        const uint32_t wv = g0 >> 6;
        const int I = (int)(wv % (uint32_t)TL);
        const uint32_t r0 = (wv / (uint32_t)TL) * 64u + (uint32_t)__lane_id();
        if ((wv / (uint32_t)TL) * 64u >= sets) break;  // (wave-uniform)
        if (r0 >= sets) continue;
        // unrank U (colex): the largest place c with C(c, i) <= r, i = TL .. 1
        int c[TL];
        uint32_t r = r0;
        int hi = n - 2;  // places 0 .. N-1 (inner city = place + 1)
#pragma unroll
        for (int i = TL; i >= 1; --i) {
            int m = hi;
            while (bn[m][i] > r) --m;
            c[i - 1] = m + 1;
            r -= bn[m][i];
            hi = m - 1;
        }
        double sm[TL][TL], d0[TL];
#pragma unroll
        for (int i = 0; i < TL; ++i) {
            d0[i] = dl[c[i] * kTRow];
#pragma unroll
            for (int j = 0; j < TL; ++j) sm[i][j] = i == j ? 0.0 : dl[c[i] * kTRow + c[j]];
        }
        static_for(
            [&](auto i) {
                constexpr int J = decltype(i)::value;
                if (J != I) return;
                H[(size_t)r0 * TL + J] = suffix_dp<double, TL, J>(sm, d0);
            },
            std::make_integer_sequence<int, TL>{});
    }
}

template <typename V, int TL>
__global__ __launch_bounds__(256) void suffix_kernel(SearchArgs a, uint32_t sets)
{
    suffix_body<V, TL>(a, sets, blockIdx.x, gridDim.x);
}

// Frontier prologue: the seeds (blocks [0, seed_blocks)) and the suffix table
// (the other blocks) are independent — one launch runs both side by side.
template <typename V, int TL>
__global__ __launch_bounds__(256) void prologue_kernel(SearchArgs a, uint32_t sets, uint32_t seed_blocks)
{
    if (a.t_start && blockIdx.x == 0 && threadIdx.x == 0) *a.t_start = wall_clock64();
    if (blockIdx.x < seed_blocks)
        seed_body<V>(a, blockIdx.x, seed_blocks);
    else
        suffix_body<V, TL>(a, sets, blockIdx.x - seed_blocks, gridDim.x - seed_blocks);
}

template <typename V>
struct Expand {
    uint32_t w[8];
    int len;
    uint32_t rem, live;
    uint32_t hnodes;  // suffix-table candidates evaluated (nodes one level down)
    double ub;        // the best completion a suffix test saw, as an upper bound on the optimum
};

// Children of a path with exactly TL + 1 cities left (the suffix level):
// every bound of expand_eval, with the suffix test's (TL + 1) x TL table reads
// and distance reads unrolled and independent of the tests, so they are all
// in flight together instead of one child after another.  Returns the live
// mask; ub = the smallest completion seen (an upper bound on the optimum).
template <typename V, int TL>
__device__ __forceinline__ uint32_t hlevel_live(const SearchArgs &a, const V *dl, const V *am, const V *b2,
                                                const uint32_t (*bn)[8], V c, int k, uint32_t rem, V remA, V remB,
                                                V thr, double &ub)
{
    int m[TL + 1];
    uint32_t x = rem;
#pragma unroll
    for (int i = 0; i <= TL; ++i) {
        m[i] = __builtin_ctz(x | 0x80000000u);
        x &= x - 1u;
    }
    // rank(rem \ m[i]) = sum_{q<i} C(m[q]-1, q+1) + sum_{q>i} C(m[q]-1, q)
    uint32_t up[TL + 1], dn[TL + 1];
#pragma unroll
    for (int q = 0; q <= TL; ++q) {
        up[q] = bn[m[q] - 1][q + 1];
        dn[q] = bn[m[q] - 1][q];
    }
    const double *H0 = a.hsuf + a.hs_off[TL];
    const double dthr = (double)thr;
    uint32_t live = 0;
#pragma unroll
    for (int i = 0; i <= TL; ++i) {
        uint32_t rk = 0;
#pragma unroll
        for (int q = 0; q <= TL; ++q) rk += q < i ? up[q] : (q > i ? dn[q] : 0u);
        const double *Hs = H0 + (size_t)rk * TL;
        const int j = m[i];
        const V cj = c + dl[k * kTRow + j];
        double best = 1.0e300;
#pragma unroll
        for (int r = 0; r <= TL; ++r) {
            if (r == i) continue;
            const double v = (double)dl[j * kTRow + m[r]] + Hs[r < i ? r : r - 1];
            best = v < best ? v : best;
        }
        bool ok = !(cj + (remA - am[j]) > thr);
        if (a.sym) ok = ok && !(cj + (((remB - b2[2 * j]) + b2[2 * j + 1]) + b2[1]) > thr);
        ok = ok && !((double)cj + best > dthr);
        if (ok) {
            live |= 1u << j;
            const double u = ((double)cj + best) * (1.0 + 0x1p-30);
            ub = u < ub ? u : ub;
        }
    }
    return live;
}

// Held-Karp tree bound of the rest of a path (SearchArgs::mst): the path from
// tail city k over the cities rem back to 0, on d' = d + pi_x + pi_y, is a
// first edge k -> x, a Hamiltonian path over rem (a spanning tree of rem)
// and a last edge y -> 0, and its d'-cost is its d-cost + pi_k + pi_0 +
// 2 sum_rem pi; so its d-cost is at least MST'(rem) + min_x d'[k][x] +
// min_y d'[y][0] - pi_k - pi_0 - 2 sum_rem pi (k = 0 at the root: the same
// for the whole tour).  Prim's algorithm per lane, the keys of the (at most
// 31) cities in registers, indexed by city; rem non-empty.
__device__ __forceinline__ double tree_bound(const double *dm, const double *pim, int k, uint32_t rem)
{
    double ek = 1.0e300, e0 = 1.0e300, ps = pim[k] + pim[0];
    for (uint32_t x = rem; x; x &= x - 1u) {
        const int t = __builtin_ctz(x);
        ps += 2.0 * pim[t];
        const double a = dm[k * kTRow + t], b = dm[t];
        ek = a < ek ? a : ek;
        e0 = b < e0 ? b : e0;
    }
    double key[kSearchMaxN];
#pragma unroll
    for (int v = 0; v < kSearchMaxN; ++v) key[v] = 1.0e300;
    uint32_t todo = rem & (rem - 1u);
    int u = __builtin_ctz(rem);
    double tot = 0.0;
    while (todo) {
        double best = 1.0e300;
        int bi = 0;
#pragma unroll
        for (int v = 1; v < kSearchMaxN; ++v) {  // (city 0 is never in rem)
            if ((todo >> v) & 1u) {
                const double w = dm[u * kTRow + v];
                const double kv = w < key[v] ? w : key[v];
                key[v] = kv;
                if (kv < best) best = kv, bi = v;
            }
        }
        tot += best;
        todo &= ~(1u << bi);
        u = bi;
    }
    return tot + ek + e0 - ps;
}

// The bound of child j of path (c, k, rem) (rem includes j), any of:
//   B0: every city still to be entered pays its cheapest incoming edge;
//   B1 (symmetric matrices): e[j] + sum over rem \ j of b + e[0];
//   H  (the child has a.hs_len cities left): min over x in rem \ j of
//       d[j][x] + H[rem \ j][x], the exact cheapest completion up to rounding.
#ifndef TSPGPU_REM_GROUP
#define TSPGPU_REM_GROUP 4
#endif
#ifndef TSPGPU_CHILD_GROUP
#define TSPGPU_CHILD_GROUP 2
#endif
constexpr int kRemGroup = TSPGPU_REM_GROUP;      // remaining cities whose table reads are in flight together
constexpr int kChildGroup = TSPGPU_CHILD_GROUP;  // children likewise
template <typename V, int TL>
__device__ __forceinline__ Expand<V> expand_eval(const SearchArgs &a, const V *dl, const V *am, const V *b2,
                                                 const uint32_t (*bn)[8], const double *dm, uint32_t full,
                                                 uint32_t idx, uint32_t end, V thr, const uint32_t *pre = nullptr)
{
    Expand<V> e;
    const bool act = idx < end;
    if (pre) {  // (read before the count was known: only an active lane's words count)
#pragma unroll
        for (int b = 0; b < 8; ++b) e.w[b] = act ? pre[b] : 0u;
    } else {
        load_path(fin_at(a, idx), act, e.w);
    }
    e.len = act ? (int)(e.w[0] & 255u) : 0;
    V c = 0;  // the reference's left fold of the path
    int k = 0;
    uint32_t mem = 0;
    fold_path<V>(dl, e.w, e.len, c, k, mem);
    e.rem = act ? (full & ~mem) : 0u;
    V remA = am[0];  // every city still to be entered: its cheapest incoming edge (exact sums)
    V remB = 0;      // B1: the rem cities' half sums (exact sums)
    // kRemGroup cities' table reads in flight before their adds (ascending order kept)
    for (uint32_t x = e.rem; x;) {
        V va[kRemGroup], vb[kRemGroup];
        uint32_t y = x;
#pragma unroll
        for (int q = 0; q < kRemGroup; ++q) {
            const int t = __builtin_ctz(y | 0x80000000u) & 31;
            va[q] = am[t];
            vb[q] = a.sym ? b2[2 * t] : V(0);
            y &= y - 1u;
        }
#pragma unroll
        for (int q = 0; q < kRemGroup; ++q) {
            if (x) {
                remA += va[q];
                if (a.sym) remB += vb[q];
                x &= x - 1u;
            }
        }
    }
    const bool htest = a.hs_len == TL && a.tail_len == TL && e.len == a.tail_level && !a.noprune;
    e.live = 0;
    e.hnodes = 0;
    e.ub = 1.0e300;
    if (htest) {  // wave-divergent only when a tile mixes levels
        e.live = act ? hlevel_live<V, TL>(a, dl, am, b2, bn, c, k, e.rem, remA, remB, thr, e.ub) : 0u;
        e.hnodes = act ? (uint32_t)((TL + 1) * TL) : 0u;
        return e;
    }
    // children kChildGroup at a time, their table reads in flight together
    for (uint32_t x = e.rem; x;) {
        V vd[kChildGroup], va[kChildGroup], vb0[kChildGroup], vb1[kChildGroup];
        int jj[kChildGroup];
        uint32_t y = x;
#pragma unroll
        for (int q = 0; q < kChildGroup; ++q) {
            const int j = __builtin_ctz(y | 0x80000000u) & 31;
            jj[q] = j;
            vd[q] = dl[k * kTRow + j];
            va[q] = am[j];
            vb0[q] = a.sym ? b2[2 * j] : V(0);
            vb1[q] = a.sym ? b2[2 * j + 1] : V(0);
            y &= y - 1u;
        }
#pragma unroll
        for (int q = 0; q < kChildGroup; ++q) {
            if (x) {
                const V cj = c + vd[q];
                bool ok = a.noprune || !(cj + (remA - va[q]) > thr);
                if (ok && a.sym && !a.noprune) ok = !(cj + (((remB - vb0[q]) + vb1[q]) + b2[1]) > thr);
                if (ok) e.live |= 1u << jj[q];
                x &= x - 1u;
            }
        }
    }
    // the tree bound of the whole rest (all children at once), only for paths
    // the cheaper bounds left children of; its margin
    // dm[kSearchMaxN * kTRow + kSearchMaxN] covers the device's rounding
    if (e.live && a.mst && !a.noprune && __builtin_popcount(e.rem) >= a.mst_min_rem) {
        const double lb = (double)c + tree_bound(dm, dm + kSearchMaxN * kTRow, k, e.rem) -
                          dm[kSearchMaxN * kTRow + kSearchMaxN];
        if (lb > (double)thr) e.live = 0;  // no child survives
    }
    return e;
}

constexpr int kExpandTiles = 4;  // tiles of 256 paths per expand_kernel block (a.fin_per_block <= 1024)

// One atomicMin per wave with the smallest suffix-test upper bound (f64
// incumbents only: the integer search's incumbent stays a tour cost).
template <typename V>
__device__ __forceinline__ void publish_ub(const SearchArgs &a, double ub)
{
    if constexpr (sizeof(V) == 8) {
        ub = wave_min_dpp(ub);
        if (__lane_id() == 0 && ub < 1.0e300)
            atomicMin(a.inc, (unsigned long long)__double_as_longlong(ub));
    }
}

template <typename V, int TL>
__global__ __launch_bounds__(256) void expand_kernel(SearchArgs a)
{
    __shared__ V dl[kSearchMaxN * kTRow];
    __shared__ V am[kSearchMaxN];
    __shared__ V b2[2 * kSearchMaxN];
    __shared__ uint32_t bn[32][8];
    __shared__ uint32_t wtot[2][4];
    __shared__ uint32_t bbase[2];
    const int n = a.n;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    // chained levels: once a level has overflowed, the later ones return at
    // once — the input slots an overflowing block reserved were never written
    // (they hold stale or uninitialised paths) and must not be read
    // every device read of the launch's set-up in flight together (the
    // level's count, the overflow flag, the incumbent, the tables): one
    // memory round trip and one barrier before the work, not three of each —
    // a chained level is a latency chain of such round trips (~2 us each)
    // the next step counts its children into the other counter word (no host memset per step)
    if (a.out_next && blockIdx.x == 0 && threadIdx.x == 0) *a.out_next = 0u;
    uint32_t fin_count = a.fin_count;
    if (a.fin_count_dev) {  // chained level: the previous level's child count, at most its buffer
        const uint32_t c = __hip_atomic_load(a.fin_count_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fin_count = c < a.fout_cap ? c : a.fout_cap;
    }
    const V thr = EThr<V>::of(ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    // the tables into registers first (a thread per (row, column) with
    // column = lane & 31: no division), the count and overflow checked while
    // they are in flight, and only a block with a run of this level writes
    // them to LDS — at 16 cities most of the grid has no run (24-157 runs of
    // 512 blocks per level) and leaves before doing any of it
    __shared__ double dm[kSearchMaxN * kTRow + kSearchMaxN + 1];
    const int tcol = (int)(threadIdx.x & 31u), trow = (int)(threadIdx.x >> 5);
    constexpr int kRowsPer = 256 / 32;
    V dv[kSearchMaxN / kRowsPer];
    double mv[kSearchMaxN / kRowsPer];
#pragma unroll
    for (int k = 0; k < kSearchMaxN / kRowsPer; ++k) {
        const int row = trow + kRowsPer * k;
        const bool in = row < n && tcol < n;
        dv[k] = in ? gd[row * n + tcol] : V(0);
        mv[k] = in && a.mst ? a.mst[row * n + tcol] : 0.0;
    }
    const int t = (int)threadIdx.x;
    const V av = t < n ? ga[t] : V(0);
    const V bv = a.sym && t < 2 * n ? static_cast<const V *>(a.bnd2)[t] : V(0);
    const double pv = a.mst && t <= n ? a.mst[n * n + t] : 0.0;
    const uint32_t ovf = a.overflow ? __hip_atomic_load(a.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if (ovf || blockIdx.x * a.fin_per_block >= fin_count) return;  // (block-uniform)
#pragma unroll
    for (int k = 0; k < kSearchMaxN / kRowsPer; ++k) {
        const int row = trow + kRowsPer * k;
        if (row < n && tcol < n) {
            dl[row * kTRow + tcol] = dv[k];
            if (a.mst) dm[row * kTRow + tcol] = mv[k];
        }
    }
    if (t < n) am[t] = av;
    if (a.sym && t < 2 * n) b2[t] = bv;
    if (a.mst && t < n) dm[kSearchMaxN * kTRow + t] = pv;
    if (a.mst && t == n) dm[kSearchMaxN * kTRow + kSearchMaxN] = pv;
    load_binom(bn);
    __syncthreads();

    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    __shared__ uint32_t bskip;
    // every run of fin_per_block input paths (one per block, or a fixed grid looping)
    for (uint32_t runi = blockIdx.x; runi * a.fin_per_block < fin_count; runi += gridDim.x) {
    __syncthreads();  // the previous run's wtot / bbase reads are done
    const uint32_t b0 = runi * a.fin_per_block;
    const uint32_t b1 = b0 + a.fin_per_block < fin_count ? b0 + a.fin_per_block : fin_count;

    // ---- pass 1: this block's live children per output, nodes evaluated; the
    // live masks stay in registers for pass 2 (at most kExpandTiles tiles of
    // 256 paths per block: the bounds are evaluated once)
    uint32_t cT = 0, cF = 0;
    unsigned long long nodes = 0;
    uint32_t lv[kExpandTiles];
    uint32_t w0[8];  // the first tile's path, kept for pass 2 (no reload)
#pragma unroll
    for (int t = 0; t < kExpandTiles; ++t) {
        const uint32_t base = b0 + 256u * t;
        lv[t] = 0;
        if (base >= b1) continue;
        const Expand<V> e = expand_eval<V, TL>(a, dl, am, b2, bn, dm, full, base + threadIdx.x, b1, thr);
        if (t == 0) {
#pragma unroll
            for (int b = 0; b < 8; ++b) w0[b] = e.w[b];
        }
        lv[t] = e.live;
        const uint32_t cnt = (uint32_t)__builtin_popcount(e.live);
        if (e.len == a.tail_level) cT += cnt; else cF += cnt;  // children have len inner cities
        nodes += (unsigned long long)__builtin_popcount(e.rem) + e.hnodes;
        publish_ub<V>(a, e.ub);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        cT += __shfl_xor(cT, off);
        cF += __shfl_xor(cF, off);
        nodes += __shfl_xor(nodes, off);
    }
    if (lane == 0) {
        wtot[0][wv] = cT;
        wtot[1][wv] = cF;
        if (nodes) atomicAdd(stat_line(a), nodes);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t tt = wtot[0][0] + wtot[0][1] + wtot[0][2] + wtot[0][3];
        const uint32_t tf = wtot[1][0] + wtot[1][1] + wtot[1][2] + wtot[1][3];
        bbase[0] = tt ? atomicAdd(a.tail_count, tt) : 0u;
        bbase[1] = tf ? atomicAdd(a.out_count, tf) : 0u;
        bskip = 0u;
        if (a.overflow && ((tt && (uint64_t)bbase[0] + tt > a.tail_cap) || (tf && (uint64_t)bbase[1] + tf > a.fout_cap))) {
            *a.overflow = 1u;  // the chained search is abandoned (the host reruns it step by step)
            bskip = 1u;
        }
    }
    __syncthreads();
    if (bskip) continue;  // (block-uniform)
    uint32_t run[2] = {bbase[0], bbase[1]};

    // ---- pass 2: the children, at block-scanned offsets
#pragma unroll
    for (int t = 0; t < kExpandTiles; ++t) {
        const uint32_t base = b0 + 256u * t;
        if (base >= b1) break;  // block-uniform
        Expand<V> e;
        const bool act = base + threadIdx.x < b1;
        if (t == 0) {
#pragma unroll
            for (int b = 0; b < 8; ++b) e.w[b] = act ? w0[b] : 0u;
        } else {
            load_path(fin_at(a, base + threadIdx.x), act, e.w);
        }
        e.len = act ? (int)(e.w[0] & 255u) : 0;
        e.live = lv[t];
        const bool tail = e.len == a.tail_level;
        const uint32_t cnt = (uint32_t)__builtin_popcount(e.live);
        const uint32_t v[2] = {tail ? cnt : 0u, tail ? 0u : cnt};
        uint32_t incl[2] = {v[0], v[1]};
#pragma unroll
        for (int off = 1; off < 64; off <<= 1)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t y = __shfl_up(incl[i], off);
                if (lane >= off) incl[i] += y;
            }
        __syncthreads();  // wtot of the previous tile has been read
        if (lane == 63) {
            wtot[0][wv] = incl[0];
            wtot[1][wv] = incl[1];
        }
        __syncthreads();
        uint32_t wofs[2] = {0u, 0u}, ttot[2] = {0u, 0u};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            wofs[0] += u < wv ? wtot[0][u] : 0u;
            wofs[1] += u < wv ? wtot[1][u] : 0u;
            ttot[0] += wtot[0][u];
            ttot[1] += wtot[1][u];
        }
        uint32_t slot = tail ? run[0] + wofs[0] + incl[0] - v[0] : run[1] + wofs[1] + incl[1] - v[1];
        run[0] += ttot[0];
        run[1] += ttot[1];
        PathItem *dstb = tail ? a.ftail : a.fout;
        // parent path + j, len + 1 (two dwordx4 stores each)
        const int cb = e.len >> 2, cs = 8 * (e.len & 3);
        uint32_t cw[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) cw[b] = b == 0 ? ((e.w[0] & ~255u) | (uint32_t)(e.len + 1)) : e.w[b];
        for (uint32_t x = e.live; x; x &= x - 1u, ++slot) {
            const uint32_t j = (uint32_t)__builtin_ctz(x);
            uint32_t o[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) o[b] = b == cb ? ((cw[b] & ~(255u << cs)) | (j << cs)) : cw[b];
            uint4 *dst = reinterpret_cast<uint4 *>(dstb + slot);
            dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
            dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
        }
    }
    }  // runs
}

// The chain's first level fused into the prologue's seed blocks (chained
// searches with at least two levels: the seeds' children are not tail paths
// and take no suffix test, so the suffix table the other blocks of the same
// launch are building is not read).  A seed block builds 256 seeds at a time
// in registers — the same prefixes and the same B0 pruning as seed_body — and
// expands the survivors at once with expand_kernel's bounds, writing the
// children at block-scanned offsets of a.fout (a.out_count): one launch and
// one round of set-up reads fewer than seeds + level 0.  Same children, same
// node counts.
// children of one evaluated path at slots [slot, slot + |live|) of out
template <typename V>
__device__ __forceinline__ void seed_emit(PathItem *out, uint32_t slot, const Expand<V> &e)
{
    const int cb = e.len >> 2, cs = 8 * (e.len & 3);
    uint32_t cw[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) cw[b] = b == 0 ? ((e.w[0] & ~255u) | (uint32_t)(e.len + 1)) : e.w[b];
    for (uint32_t x = e.live; x; x &= x - 1u, ++slot) {
        const uint32_t j = (uint32_t)__builtin_ctz(x);
        uint32_t o[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) o[b] = b == cb ? ((cw[b] & ~(255u << cs)) | (j << cs)) : cw[b];
        uint4 *dst = reinterpret_cast<uint4 *>(out + slot);
        dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
        dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
}

template <typename V, int TL>
__device__ __forceinline__ void seed_expand_body(const SearchArgs &a, uint32_t block, uint32_t nblocks)
{
    using W = typename SeedNum<V>::Wide;
    __shared__ V dl[kSearchMaxN * kTRow];
    __shared__ V am[kSearchMaxN];
    __shared__ V b2[2 * kSearchMaxN];
    __shared__ uint32_t bn[32][8];
    __shared__ double dm[kSearchMaxN * kTRow + kSearchMaxN + 1];
    __shared__ uint32_t pv[33];
    __shared__ uint32_t wtot[4];
    __shared__ uint32_t bbase, bskip;
    __shared__ typename SeedNum<V>::Wide aall_s;
    __shared__ uint4 sq[256][2];  // the round's live seeds, compacted
    __shared__ uint32_t nlive_s;
    const int n = a.n, N = n - 1, D = a.depth;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    const int t = (int)threadIdx.x, tcol = t & 31;
    for (int row = t >> 5; row < n; row += 8)
        if (tcol < n) {
            dl[row * kTRow + tcol] = gd[row * n + tcol];
            if (a.mst) dm[row * kTRow + tcol] = a.mst[row * n + tcol];
        }
    if (t < n) am[t] = ga[t];
    if (a.sym && t < 2 * n) b2[t] = static_cast<const V *>(a.bnd2)[t];
    if (a.mst && t < n) dm[kSearchMaxN * kTRow + t] = a.mst[n * n + t];
    if (a.mst && t == n) dm[kSearchMaxN * kTRow + kSearchMaxN] = a.mst[n * n + n];
    load_binom(bn);
    if (t == 0) {
        uint32_t p = 1;
        pv[D] = 1;
        for (int l = D; l >= 2; --l) {
            p *= (uint32_t)(N - l + 1);
            pv[l - 1] = p;
        }
        // seed_body's sum, in its order, once per block
        W s0 = 0;
        for (int x = 0; x < n; ++x) s0 += (W)ga[x];
        aall_s = s0;
    }
    __syncthreads();
    const uint64_t incw = __hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const V inc = SeedNum<V>::val(incw);
    const V thr = EThr<V>::of(ENum<V>::val(incw));
    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    const W aall = aall_s;
    const uint32_t local = a.items / a.nshards + (a.items % a.nshards > a.shard ? 1u : 0u);
    const int lane = __lane_id(), wv = t >> 6;
    unsigned long long nodes = 0;
    for (uint32_t base = block * 256u; base < local; base += nblocks * 256u) {  // (block-uniform)
        // the seed of this thread (seed_body's prefix order and bound)
        const uint32_t i = base + (uint32_t)t;
        uint32_t p = i * a.nshards + a.shard;
        uint32_t rr = full;
        W ra = aall;
        V c = 0;
        int prev = 0;
        bool live = i < local;
        uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int l = 1; l <= D && live; ++l) {
            const uint32_t q = p / pv[l];
            p -= q * pv[l];
            uint32_t x = rr;
            for (uint32_t u = 0; u < q; ++u) x &= x - 1u;
            const int tc = __builtin_ctz(x);
            c = c + dl[prev * kTRow + tc];
            rr &= ~(1u << tc);
            ra -= (W)am[tc];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if ((l >> 2) == b) w[b] |= (uint32_t)tc << (8 * (l & 3));
            prev = tc;
            if (!a.noprune && SeedNum<V>::pruned((W)c + ra, inc)) live = false;
        }
        w[0] |= (uint32_t)(D + 1);
        // the round's live seeds compacted to the first threads (most seeds
        // fail their bound: the evaluation below then runs on full waves only)
        {
            const unsigned long long lm = __ballot(live);
            if (lane == 0) wtot[wv] = (uint32_t)__popcll(lm);
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) off += u < wv ? wtot[u] : 0u;
            if (live) {
                const uint32_t pos = off + (uint32_t)__popcll(lm & ((1ull << lane) - 1ull));
                sq[pos][0] = make_uint4(w[0], w[1], w[2], w[3]);
                sq[pos][1] = make_uint4(w[4], w[5], w[6], w[7]);
            }
            if (t == 0) nlive_s = wtot[0] + wtot[1] + wtot[2] + wtot[3];
            __syncthreads();
        }
        const uint32_t nlive = nlive_s;
        const bool mine = (uint32_t)t < nlive;
        {
            const uint4 lo = mine ? sq[t][0] : make_uint4(0, 0, 0, 0);
            const uint4 hi = mine ? sq[t][1] : make_uint4(0, 0, 0, 0);
            w[0] = lo.x, w[1] = lo.y, w[2] = lo.z, w[3] = lo.w;
            w[4] = hi.x, w[5] = hi.y, w[6] = hi.z, w[7] = hi.w;
        }
        // its children (expand_kernel's bounds; no tail children at this level)
        Expand<V> e;
        e.len = 0;
        e.rem = 0;
        e.live = 0;
        e.hnodes = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) e.w[b] = 0u;
        if ((uint32_t)(wv * 64) < nlive)  // (wave-uniform: a wave without seeds skips the evaluation)
            e = expand_eval<V, TL>(a, dl, am, b2, bn, dm, full, mine ? 0u : 1u, 1u, thr, w);
        nodes += (unsigned long long)__builtin_popcount(e.rem) + e.hnodes;
        const uint32_t cnt = (uint32_t)__builtin_popcount(e.live);
        uint32_t incl = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wtot[wv] = incl;
        __syncthreads();
        uint32_t wofs = 0, tot = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            wofs += u < wv ? wtot[u] : 0u;
            tot += wtot[u];
        }
        if (t == 0) {
            bbase = tot ? atomicAdd(a.out_count, tot) : 0u;
            bskip = 0u;
            if (a.overflow && tot && (uint64_t)bbase + tot > a.fout_cap) {
                *a.overflow = 1u;  // the chained search is abandoned (the host reruns it step by step)
                bskip = 1u;
            }
        }
        __syncthreads();
        if (!bskip) seed_emit(a.fout, bbase + wofs + incl - cnt, e);
        __syncthreads();  // (wtot, bbase and bskip are rewritten by the next round)
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nodes += __shfl_xor(nodes, off);
    if (lane == 0 && nodes) atomicAdd(stat_line(a), nodes);
}

template <typename V, int TL>
__global__ __launch_bounds__(256) void prologue1_kernel(SearchArgs a, uint32_t sets, uint32_t seed_blocks)
{
    if (a.t_start && blockIdx.x == 0 && threadIdx.x == 0) *a.t_start = wall_clock64();
    if (blockIdx.x < seed_blocks)
        seed_expand_body<V, TL>(a, blockIdx.x, seed_blocks);
    else
        suffix_body<V, TL>(a, sets, blockIdx.x - seed_blocks, gridDim.x - seed_blocks);
}

// Chained frontier levels, block-local (SearchArgs::local_levels): a block
// takes a run of fin_per_block input paths and expands its subtree level after
// level inside the launch — the paths between two levels stay in an LDS queue
// (kLocalCap per level), with the block's own barriers between levels instead
// of a launch per level.  The chain's level launches cost ~11 us each at 16
// cities whatever their size, nearly all of it latency (set-up reads, the
// path reads, the slot atomics: profiles/r04/k2_chain_costs.log), and a grid
// barrier costs more than a launch (5-21 us), so the levels are folded per
// block instead.  Children that reach the tail level go to ftail as before;
// children the queue cannot hold (or those of the last local level) go to
// fout, which the chain's next launch expands: every launch still advances
// every path at least one level, so the chain's launch count bounds the depth
// as before (the later launches mostly find nothing and leave).
constexpr uint32_t kLocalCap = 512;

template <typename V, int TL>
__global__ __launch_bounds__(256) void expand_local_kernel(SearchArgs a)
{
    __shared__ V dl[kSearchMaxN * kTRow];
    __shared__ V am[kSearchMaxN];
    __shared__ V b2[2 * kSearchMaxN];
    __shared__ uint32_t bn[32][8];
    __shared__ double dm[kSearchMaxN * kTRow + kSearchMaxN + 1];
    __shared__ uint4 q[2][kLocalCap][2];  // the level queues (32-byte paths)
    __shared__ uint32_t wtot[2][4];
    __shared__ uint32_t bbase[2];
    __shared__ uint32_t dead, bskip;
    const int n = a.n;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    if (threadIdx.x == 0) dead = a.overflow ? __hip_atomic_load(a.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if (a.out_next && blockIdx.x == 0 && threadIdx.x == 0) *a.out_next = 0u;
    uint32_t fin_count = a.fin_count;
    if (a.fin_count_dev) {
        const uint32_t c = __hip_atomic_load(a.fin_count_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fin_count = c < a.fout_cap ? c : a.fout_cap;
    }
    V thr = EThr<V>::of(ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    const uint32_t fpb = a.fin_per_block;
    uint32_t pre[8];  // the first run's paths, read beside the set-up (see expand_kernel)
    const bool spec = a.fin_cap && a.nseg == 1 && threadIdx.x < fpb && blockIdx.x * fpb + threadIdx.x < a.fin_cap;
    load_path(a.fseg[0] + blockIdx.x * fpb + threadIdx.x, spec, pre);
    for (int i = threadIdx.x; i < n * n; i += blockDim.x) dl[(i / n) * kTRow + i % n] = gd[i];
    for (int i = threadIdx.x; i < n; i += blockDim.x) am[i] = ga[i];
    if (a.sym)
        for (int i = threadIdx.x; i < 2 * n; i += blockDim.x) b2[i] = static_cast<const V *>(a.bnd2)[i];
    load_binom(bn);
    if (a.mst) {
        for (int i = threadIdx.x; i < n * n; i += blockDim.x) dm[(i / n) * kTRow + i % n] = a.mst[i];
        for (int i = threadIdx.x; i < n; i += blockDim.x) dm[kSearchMaxN * kTRow + i] = a.mst[n * n + i];
        if (threadIdx.x == 0) dm[kSearchMaxN * kTRow + kSearchMaxN] = a.mst[n * n + n];
    }
    __syncthreads();
    if (dead || blockIdx.x * fpb >= fin_count) return;  // (block-uniform)

    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    unsigned long long nodes = 0;
    for (uint32_t runi = blockIdx.x; runi * fpb < fin_count; runi += gridDim.x) {
        const uint32_t b0 = runi * fpb;
        uint32_t qn = fin_count - b0 < fpb ? fin_count - b0 : fpb;  // this level's paths (block-uniform)
        int cur = 0;
        for (int L = 0; L < a.local_levels && qn > 0; ++L) {
            // the incumbent for the next level, read now (its latency under this level's work)
            const V thr_next = EThr<V>::of(ENum<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
            const bool last = L + 1 >= a.local_levels;
            uint32_t qnext = 0;  // block-uniform
            for (uint32_t t0 = 0; t0 < qn; t0 += 256u) {
                const uint32_t i = t0 + threadIdx.x;
                const bool act = i < qn;
                uint32_t w[8];
                if (L == 0 && t0 == 0 && runi == blockIdx.x && spec) {
#pragma unroll
                    for (int b = 0; b < 8; ++b) w[b] = pre[b];
                } else if (L == 0) {
                    load_path(fin_at(a, b0 + i), act, w);
                } else if (act) {
                    const uint4 lo = q[cur][i][0], hi = q[cur][i][1];
                    w[0] = lo.x, w[1] = lo.y, w[2] = lo.z, w[3] = lo.w;
                    w[4] = hi.x, w[5] = hi.y, w[6] = hi.z, w[7] = hi.w;
                } else {
#pragma unroll
                    for (int b = 0; b < 8; ++b) w[b] = 0u;
                }
                const Expand<V> e = expand_eval<V, TL>(a, dl, am, b2, bn, dm, full, i, qn, thr, w);
                nodes += (unsigned long long)__builtin_popcount(e.rem) + e.hnodes;
                publish_ub<V>(a, e.ub);
                const uint32_t cnt = (uint32_t)__builtin_popcount(e.live);
                const bool tail = e.len == a.tail_level;  // children with tail_level inner cities
                const uint32_t v[2] = {tail ? cnt : 0u, tail ? 0u : cnt};
                uint32_t incl[2] = {v[0], v[1]};
#pragma unroll
                for (int off = 1; off < 64; off <<= 1)
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const uint32_t y = __shfl_up(incl[k], off);
                        if (lane >= off) incl[k] += y;
                    }
                if (lane == 63) {
                    wtot[0][wv] = incl[0];
                    wtot[1][wv] = incl[1];
                }
                __syncthreads();
                uint32_t wofs[2] = {0u, 0u}, ttot[2] = {0u, 0u};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    wofs[0] += u < wv ? wtot[0][u] : 0u;
                    wofs[1] += u < wv ? wtot[1][u] : 0u;
                    ttot[0] += wtot[0][u];
                    ttot[1] += wtot[1][u];
                }
                // the non-tail children stay in the block unless this is the
                // last local level or the queue cannot take the tile's
                const bool local = !last && qnext + ttot[1] <= kLocalCap;  // (block-uniform)
                if (threadIdx.x == 0) {
                    bbase[0] = ttot[0] ? atomicAdd(a.tail_count, ttot[0]) : 0u;
                    bbase[1] = !local && ttot[1] ? atomicAdd(a.out_count, ttot[1]) : 0u;
                    bskip = 0u;
                    if (a.overflow && ((ttot[0] && (uint64_t)bbase[0] + ttot[0] > a.tail_cap) ||
                                       (!local && ttot[1] && (uint64_t)bbase[1] + ttot[1] > a.fout_cap))) {
                        *a.overflow = 1u;  // the chain is abandoned (the host reruns it step by step)
                        bskip = 1u;
                    }
                }
                __syncthreads();
                if (bskip) return;  // (block-uniform; nothing this block reserved is read: see expand_kernel)
                uint32_t slot = tail ? bbase[0] + wofs[0] + incl[0] - v[0]
                                     : (local ? qnext : bbase[1]) + wofs[1] + incl[1] - v[1];
                const int cb = e.len >> 2, cs = 8 * (e.len & 3);
                uint32_t cw[8];
#pragma unroll
                for (int b = 0; b < 8; ++b) cw[b] = b == 0 ? ((e.w[0] & ~255u) | (uint32_t)(e.len + 1)) : e.w[b];
                for (uint32_t x = e.live; x; x &= x - 1u, ++slot) {
                    const uint32_t j = (uint32_t)__builtin_ctz(x);
                    uint32_t o[8];
#pragma unroll
                    for (int b = 0; b < 8; ++b) o[b] = b == cb ? ((cw[b] & ~(255u << cs)) | (j << cs)) : cw[b];
                    const uint4 lo = make_uint4(o[0], o[1], o[2], o[3]), hi = make_uint4(o[4], o[5], o[6], o[7]);
                    if (!tail && local) {
                        q[cur ^ 1][slot][0] = lo;
                        q[cur ^ 1][slot][1] = hi;
                    } else {
                        uint4 *dst = reinterpret_cast<uint4 *>((tail ? a.ftail : a.fout) + slot);
                        dst[0] = lo;
                        dst[1] = hi;
                    }
                }
                if (local) qnext += ttot[1];
                __syncthreads();  // (wtot reused; the queue's writes before the next level reads them)
            }
            cur ^= 1;
            qn = qnext;
            thr = thr_next < thr ? thr_next : thr;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nodes += __shfl_xor(nodes, off);
    if (lane == 0 && nodes) atomicAdd(stat_line(a), nodes);
}

// Seeds (SearchItem, from seed_kernel) -> frontier paths.
__global__ __launch_bounds__(256) void to_paths_kernel(SearchArgs a)
{
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    if (idx >= a.in_count) return;
    const SearchItem &it = a.in[idx];
    uint32_t o[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) o[b] = 0u;
    const int len = it.len;
    for (int l = 0; l < len; ++l) o[l >> 2] |= (uint32_t)(l == 0 ? len : it.city[l]) << (8 * (l & 3));
    uint4 *dst = reinterpret_cast<uint4 *>(a.fout + idx);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

template <typename V>
hipError_t launch_tail_v(const SearchArgs &a, int grid)
{
    if (a.n > kSearchMaxN || a.tail_level < 1 || a.tail_level + a.tail_len != a.n - 1) return hipErrorInvalidValue;
    switch (a.tail_len) {
    case 5: hipLaunchKernelGGL((tail_kernel<V, 5>), dim3(grid), dim3(256), 0, a.stream, a); break;
    case 6: hipLaunchKernelGGL((tail_kernel<V, 6>), dim3(grid), dim3(256), 0, a.stream, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_enum(const SearchArgs &a, bool f64, int grid)
{
    return f64 ? launch_v<double>(a, grid) : launch_v<int32_t>(a, grid);
}

hipError_t launch_to_paths(const SearchArgs &a)
{
    if (a.in_count == 0) return hipSuccess;
    hipLaunchKernelGGL(to_paths_kernel, dim3((a.in_count + 255u) / 256u), dim3(256), 0, a.stream, a);
    return hipGetLastError();
}

hipError_t launch_expand(const SearchArgs &a, bool f64)
{
    if (a.n > kSearchMaxN || a.fin_count == 0) return a.fin_count ? hipErrorInvalidValue : hipSuccess;
    if (a.fin_per_block == 0 || (a.local_levels <= 0 && (a.fin_per_block % 256u || a.fin_per_block > 256u * kExpandTiles)))
        return hipErrorInvalidValue;
    int grid = (int)((a.fin_count + a.fin_per_block - 1u) / a.fin_per_block);
    if (a.max_grid > 0 && grid > a.max_grid) grid = a.max_grid;  // chained: the blocks loop over the runs
    if (a.local_levels > 0) {
        if (a.fin_per_block > 256u) return hipErrorInvalidValue;
#define TSPGPU_LOC(VT, TLV) hipLaunchKernelGGL((expand_local_kernel<VT, TLV>), dim3(grid), dim3(256), 0, a.stream, a)
        if (a.tail_len == 5) {
            if (f64) TSPGPU_LOC(double, 5); else TSPGPU_LOC(int32_t, 5);
        } else {
            if (f64) TSPGPU_LOC(double, 6); else TSPGPU_LOC(int32_t, 6);
        }
#undef TSPGPU_LOC
        return hipGetLastError();
    }
    if (a.tail_len == 5) {
        if (f64)
            hipLaunchKernelGGL((expand_kernel<double, 5>), dim3(grid), dim3(256), 0, a.stream, a);
        else
            hipLaunchKernelGGL((expand_kernel<int32_t, 5>), dim3(grid), dim3(256), 0, a.stream, a);
    } else {
        if (f64)
            hipLaunchKernelGGL((expand_kernel<double, 6>), dim3(grid), dim3(256), 0, a.stream, a);
        else
            hipLaunchKernelGGL((expand_kernel<int32_t, 6>), dim3(grid), dim3(256), 0, a.stream, a);
    }
    return hipGetLastError();
}

hipError_t launch_seed(const SearchArgs &a, bool f64, int grid)
{
    if (f64)
        hipLaunchKernelGGL(seed_kernel<double>, dim3(grid), dim3(kSearchThreads), 0, a.stream, a);
    else
        hipLaunchKernelGGL(seed_kernel<int32_t>, dim3(grid), dim3(kSearchThreads), 0, a.stream, a);
    return hipGetLastError();
}

hipError_t launch_prologue1(const SearchArgs &a, bool f64, int seed_grid, uint32_t sets)
{
    if (a.n > kSearchMaxN || !a.hsuf || (a.hs_len != 5 && a.hs_len != 6) || !a.fout) return hipErrorInvalidValue;
    const int grid = seed_grid + (int)std::min<uint32_t>((sets * (uint32_t)a.hs_len + 255u) / 256u, 4096u);
    const uint32_t sb = (uint32_t)seed_grid;
#define TSPGPU_PRO(VT, TLV) hipLaunchKernelGGL((prologue1_kernel<VT, TLV>), dim3(grid), dim3(256), 0, a.stream, a, sets, sb)
    if (a.hs_len == 5) {
        if (f64) TSPGPU_PRO(double, 5); else TSPGPU_PRO(int32_t, 5);
    } else {
        if (f64) TSPGPU_PRO(double, 6); else TSPGPU_PRO(int32_t, 6);
    }
#undef TSPGPU_PRO
    return hipGetLastError();
}

hipError_t launch_prologue(const SearchArgs &a, bool f64, int seed_grid, uint32_t sets)
{
    if (a.n > kSearchMaxN || !a.hsuf || (a.hs_len != 5 && a.hs_len != 6)) return hipErrorInvalidValue;
    const int grid = seed_grid + (int)std::min<uint32_t>((sets * (uint32_t)a.hs_len + 255u) / 256u, 4096u);
    const uint32_t sb = (uint32_t)seed_grid;
#define TSPGPU_PRO(VT, TLV) hipLaunchKernelGGL((prologue_kernel<VT, TLV>), dim3(grid), dim3(256), 0, a.stream, a, sets, sb)
    if (a.hs_len == 5) {
        if (f64) TSPGPU_PRO(double, 5); else TSPGPU_PRO(int32_t, 5);
    } else {
        if (f64) TSPGPU_PRO(double, 6); else TSPGPU_PRO(int32_t, 6);
    }
#undef TSPGPU_PRO
    return hipGetLastError();
}

hipError_t launch_suffix(const SearchArgs &a, bool f64, uint32_t sets)
{
    if (a.n > kSearchMaxN || !a.hsuf || (a.hs_len != 5 && a.hs_len != 6)) return hipErrorInvalidValue;
    if (sets == 0) return hipSuccess;
    const int grid = (int)std::min<uint32_t>((sets * (uint32_t)a.hs_len + 255u) / 256u, 4096u);
    if (a.hs_len == 5) {
        if (f64)
            hipLaunchKernelGGL((suffix_kernel<double, 5>), dim3(grid), dim3(256), 0, a.stream, a, sets);
        else
            hipLaunchKernelGGL((suffix_kernel<int32_t, 5>), dim3(grid), dim3(256), 0, a.stream, a, sets);
    } else {
        if (f64)
            hipLaunchKernelGGL((suffix_kernel<double, 6>), dim3(grid), dim3(256), 0, a.stream, a, sets);
        else
            hipLaunchKernelGGL((suffix_kernel<int32_t, 6>), dim3(grid), dim3(256), 0, a.stream, a, sets);
    }
    return hipGetLastError();
}

hipError_t launch_tail(const SearchArgs &a, bool f64, int grid)
{
    return f64 ? launch_tail_v<double>(a, grid) : launch_tail_v<int32_t>(a, grid);
}

}  // namespace tspgpu
