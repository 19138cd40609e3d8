// K2 — prefix-parallel exact search of ONE instance on gfx950 (MI355X).
//
// The north_star's search shape for the reference's per-block problem
// (tsp.cpp:405-509): the tour space is cut into fixed-depth prefixes
// (0, t1..tD); every lane of every wave takes prefixes from a device-wide
// queue (one atomic per fetch round: the lanes that need work share it), so a
// lane that finishes a small subtree immediately takes the next prefix — the
// intra-GPU work distribution.  Below its prefix a lane runs an iterative
// depth-first search with
//   * the distance matrix staged in LDS (one coalesced read per workgroup),
//   * the path cost carried as the reference's left fold
//     ((d[0][t1] + d[t1][t2]) + ...) so that complete tours have bit-exactly
//     the cost tsp() reports,
//   * a consistent lower bound: every city still to be entered (the unvisited
//     ones and city 0) costs at least its cheapest incoming edge a[x]; the
//     a[x] are rounded down to a 2^-20 grid so their running sums are exact,
//   * pruning only when the bound, shrunk by 2^-40 (far more than the
//     <= 32 roundings of a fold), is strictly above the incumbent, so every
//     tour whose cost equals the optimum survives,
//   * a device-wide incumbent held as a 64-bit atomicMin word (IEEE bits of
//     the f64 cost, or the integer cost) and re-read every 64 iterations.
// Load balance ("work stealing" without locks): the search runs in rounds.
// A seed kernel writes every live depth-D prefix as an item; a round kernel
// gives each lane items from a device queue and lets it spend at most
// `budget` DFS iterations per item.  A lane whose budget runs out hands the
// untried siblings of every level of its stack back as new items, which the
// next round spreads over all lanes — deep subtrees are split until they fit.
// Every complete tour whose cost is <= the incumbent at the moment it is found
// is recorded.  After the search the records with cost == optimum are exactly
// the set O of optimal tours, from which the host picks the tour tsp()
// returns with the DP's own tie rule (search_abi.cpp, tspgpu_select_tour).
#include <hip/hip_runtime.h>

#include "search.h"

namespace tspgpu {
namespace {

constexpr double kShrink = 1.0 - 0x1p-40;
constexpr unsigned kChunk = 64;  // items a wave takes from the device queue per atomic (= lanes)

template <typename V>
struct Num;
template <>
struct Num<double> {
    using Wide = double;
    __device__ static uint64_t bits(double v) { return (uint64_t)__double_as_longlong(v); }
    __device__ static double val(uint64_t b) { return __longlong_as_double((long long)b); }
    __device__ static bool pruned(double lb, double inc) { return lb * kShrink > inc; }
};
template <>
struct Num<int32_t> {
    using Wide = long long;
    __device__ static uint64_t bits(int32_t v) { return (uint64_t)(uint32_t)v; }
    __device__ static int32_t val(uint64_t b) { return (int32_t)(uint32_t)b; }
    __device__ static bool pruned(long long lb, int32_t inc) { return lb > (long long)inc; }
};

__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS: place values pv[0..32] (u32, seed only) | d (n*n) | a (n) | cost stack [level][lane] | city stack [level][lane]
template <typename V>
__host__ __device__ constexpr size_t head_bytes(int n)
{
    return 33 * 8 + align16((size_t)(n * n + n) * sizeof(V));
}
template <typename V>
__host__ __device__ constexpr size_t stack_end(int n)
{
    return align16(head_bytes<V>(n) + (size_t)n * kSearchThreads * sizeof(V) + (size_t)n * kSearchThreads);
}
// + per wave a staging buffer of kChunk items (one coalesced load per chunk)
template <typename V>
__host__ __device__ constexpr size_t lds_bytes(int n)
{
    return stack_end<V>(n) + (size_t)(kSearchThreads / 64) * kChunk * sizeof(SearchItem);
}

// Seed: every depth-D prefix of this shard that survives the bound becomes an item.
template <typename V>
__global__ __launch_bounds__(kSearchThreads) void seed_kernel(SearchArgs a)
{
    using W = typename Num<V>::Wide;
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
    const V inc = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t local = a.items / a.nshards + (a.items % a.nshards > a.shard ? 1u : 0u);
    const int lane = __lane_id();
    // the loop runs the same trip count on every lane of a wave (ballots inside)
    const uint32_t stride = gridDim.x * kSearchThreads;
    for (uint32_t i0 = blockIdx.x * kSearchThreads + (threadIdx.x & ~63u); i0 < local; i0 += stride) {
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
            if (Num<V>::pruned((W)c + ra, inc)) live = false;
        }
        // one atomic per wave for its live prefixes
        const unsigned long long lm = __ballot(live);
        if (!lm) continue;
        const int leader = __ffsll((long long)lm) - 1;
        unsigned int base = 0;
        if (lane == leader) base = atomicAdd(a.out_count, (unsigned int)__popcll(lm));
        base = __shfl(base, leader);
        if (!live) continue;
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.out + base + __popcll(lm & ((1ull << lane) - 1ull)));
#pragma unroll
        for (int b = 0; b < 8; ++b) dst[b] = w[b];
        dst[8] = (uint32_t)(D + 1) | (1u << 8);  // len, from = 1
    }
}

// One round over the items a.in[0 .. in_count).
template <typename V>
__global__ __launch_bounds__(kSearchThreads) void round_kernel(SearchArgs a)
{
    using W = typename Num<V>::Wide;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n = a.n;
    const int tid = threadIdx.x;
    V *dl = reinterpret_cast<V *>(smem + 33 * 8);
    V *al = dl + n * n;
    V *cst = reinterpret_cast<V *>(smem + head_bytes<V>(n));
    uint8_t *cty = reinterpret_cast<uint8_t *>(cst + (size_t)n * kSearchThreads);
#define COST(l) cst[(l) * kSearchThreads + tid]
#define CITY(l) cty[(l) * kSearchThreads + tid]

    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    for (int i = tid; i < n * n; i += kSearchThreads) dl[i] = gd[i];
    for (int i = tid; i < n; i += kSearchThreads) al[i] = ga[i];
    __syncthreads();

    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;  // cities 1..N
    W aall = 0;
    for (int x = 0; x < n; ++x) aall += (W)al[x];                // exact: grid values
    V inc = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    unsigned long long nodes = 0;
    int L = -1;          // current depth; < root: the lane needs an item
    int root = 0;        // depth of the item's last fixed city
    int k = 0;           // city at depth L
    uint32_t rem = 0;    // unvisited cities
    uint32_t from = 1;   // next child of k to try: lowest city >= from in rem
    W remA = 0;          // sum of a[x] over rem and city 0
    V ck = 0;            // fold cost of the path to depth L
    uint32_t spent = 0;  // iterations spent on the current item
    bool done = false;   // the queue is drained for this lane
    uint32_t tick = 0;
    // wave-private slice of the queue [pnext, pend) staged in LDS at wbuf[0..kChunk):
    // one atomic and one coalesced load per kChunk items
    const int lane = __lane_id();
    SearchItem *wbuf = reinterpret_cast<SearchItem *>(smem + stack_end<V>(n)) + (tid / 64) * kChunk;
    uint32_t pbase = 0, pnext = 0, pend = 0;

    // rebuild an item's stack: the same left fold as when it was cut
    auto load_item = [&](const SearchItem &it) {
        const int len = it.len;
        uint32_t rr = full;
        W ra = aall;
        V c = 0;
        int prev = 0;
        CITY(0) = 0;
        COST(0) = 0;
        for (int l = 1; l < len; ++l) {
            const int t = it.city[l];
            c = c + dl[prev * n + t];
            rr &= ~(1u << t);
            ra -= (W)al[t];
            CITY(l) = (uint8_t)t;
            COST(l) = c;
            prev = t;
        }
        if (!Num<V>::pruned((W)c + ra, inc)) {
            root = len - 1;
            L = root;
            k = prev;
            ck = c;
            rem = rr;
            remA = ra;
            from = it.from;
            spent = 0;
        }
    };

    for (;;) {
        if ((++tick & 255u) == 0) {
            const V g = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            inc = g < inc ? g : inc;
        }
        const bool need = !done && L < root;
        const unsigned long long nm = __ballot(need);
        if (nm) {
            // hand the lanes that need an item consecutive queue entries
            const uint32_t cnt = (uint32_t)__popcll(nm);
            const uint32_t r = (uint32_t)__popcll(nm & ((1ull << lane) - 1ull));
            const uint32_t left = pend - pnext;
            if (need && r < left) {
                if (pnext + r >= a.in_count)
                    done = true;
                else
                    load_item(wbuf[pnext - pbase + r]);
            }
            if (cnt > left) {
                const int leader = __ffsll((long long)nm) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(a.queue, kChunk);
                base = __shfl(base, leader);
                __builtin_amdgcn_wave_barrier();
                if (base + lane < a.in_count) wbuf[lane] = a.in[base + lane];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (need && r >= left) {
                    if (base + (r - left) >= a.in_count)
                        done = true;
                    else
                        load_item(wbuf[r - left]);
                }
                pbase = base;
                pnext = base + (cnt - left);
                pend = base + kChunk;
            } else {
                pnext += cnt;
            }
        }
        if (__ballot(!done) == 0) break;
        if (done || L < root) continue;
        if (++spent > a.budget) {
            // budget spent: hand back, level by level, the children not tried yet
            uint32_t rl = rem, fl = from;
            unsigned int cnt = 0;
            for (int l = L; l >= root; --l) {
                if (rl & (uint32_t)(0xFFFFFFFFull << fl)) ++cnt;
                if (l > root) {
                    const int c1 = CITY(l);
                    rl |= 1u << c1;
                    fl = (uint32_t)c1 + 1u;
                }
            }
            // the host sizes the output for (N-1) items per input item: always room
            unsigned int slot = cnt ? atomicAdd(a.out_count, cnt) : 0u;
            rl = rem;
            fl = from;
            for (int l = L; l >= root; --l) {
                if (rl & (uint32_t)(0xFFFFFFFFull << fl)) {
                    uint32_t *dst = reinterpret_cast<uint32_t *>(a.out + slot);
                    for (int b = 0; b < 8; ++b) {
                        uint32_t word = 0;
                        for (int q = 0; q < 4; ++q) {
                            const int lv = 4 * b + q;
                            if (lv <= l) word |= (uint32_t)CITY(lv) << (8 * q);
                        }
                        dst[b] = word;
                    }
                    dst[8] = (uint32_t)(l + 1) | (fl << 8);
                    ++slot;
                }
                if (l > root) {
                    const int c1 = CITY(l);
                    rl |= 1u << c1;
                    fl = (uint32_t)c1 + 1u;
                }
            }
            L = -1;
            continue;
        }
        const uint32_t cand = rem & (uint32_t)(0xFFFFFFFFull << from);
        if (cand == 0) {  // all children of k tried: back up
            if (L == root) {
                L = -1;
                continue;
            }
            rem |= 1u << k;
            remA += (W)al[k];
            from = (uint32_t)k + 1u;
            --L;
            k = CITY(L);
            ck = COST(L);
            continue;
        }
        const int j = __builtin_ctz(cand);
        from = (uint32_t)j + 1u;
        ++nodes;
        const V c = ck + dl[k * n + j];
        if (L + 2 == n) {  // j is the last inner city: close the tour (tsp.cpp:483-499)
            const V total = c + dl[j * n];
            if (total <= inc) {
                const uint64_t tb = Num<V>::bits(total);
                const unsigned long long old = atomicMin(a.inc, (unsigned long long)tb);
                if (tb <= old) {
                    const unsigned int s = atomicAdd(a.rec_count, 1u);
                    if (s < a.rec_cap) {
                        SearchRecord *R = a.rec + s;
                        R->cost = tb;
                        for (int l = 1; l <= L; ++l) R->city[l - 1] = CITY(l);
                        R->city[L] = (uint8_t)j;
                    }
                }
                const V o = Num<V>::val(old);
                inc = o < total ? o : total;
            }
            continue;
        }
        const W rest = remA - (W)al[j];
        if (Num<V>::pruned((W)c + rest, inc)) continue;
        ++L;
        CITY(L) = (uint8_t)j;
        COST(L) = c;
        rem &= ~(1u << j);
        remA = rest;
        k = j;
        ck = c;
        from = 1;
    }
#undef COST
#undef CITY
    atomicAdd(a.nodes, nodes);
}

}  // namespace

size_t search_lds_bytes(int n, bool f64) { return f64 ? lds_bytes<double>(n) : lds_bytes<int32_t>(n); }

hipError_t launch_seed(const SearchArgs &a, bool f64, int grid)
{
    if (f64)
        hipLaunchKernelGGL(seed_kernel<double>, dim3(grid), dim3(kSearchThreads), 0, a.stream, a);
    else
        hipLaunchKernelGGL(seed_kernel<int32_t>, dim3(grid), dim3(kSearchThreads), 0, a.stream, a);
    return hipGetLastError();
}

hipError_t launch_round(const SearchArgs &a, bool f64, int grid)
{
    const size_t lds = search_lds_bytes(a.n, f64);
    const void *fn = f64 ? reinterpret_cast<const void *>(&round_kernel<double>)
                         : reinterpret_cast<const void *>(&round_kernel<int32_t>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (f64)
        hipLaunchKernelGGL(round_kernel<double>, dim3(grid), dim3(kSearchThreads), lds, a.stream, a);
    else
        hipLaunchKernelGGL(round_kernel<int32_t>, dim3(grid), dim3(kSearchThreads), lds, a.stream, a);
    return hipGetLastError();
}

}  // namespace tspgpu
