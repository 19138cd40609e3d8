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
#include "wave.h"

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

// One round over the items a.in[0 .. in_count) (v1: one DFS iteration per
// loop trip with a branch per case; kept for A/B measurements).
template <typename V>
__global__ __launch_bounds__(kSearchThreads) void round_kernel_v1(SearchArgs a)
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
    TieCache tcache;
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
                    tie_offer(a, tcache, tb, [&](int i) { return i <= L ? (int)CITY(i) : j; });
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
    atomicAdd(stat_line(a), nodes);
}


// ---------------------------------------------------------------------------
// v2 round kernel: the same search, but every lane of a wave advances its DFS
// by exactly one step per trip of a branch-free inner loop.  A step evaluates
// the next untried child j of the path's last city k — one search node: the
// fold cost c = ck + d[k][j] and the bound c + (remA - a[j]) — and then
// descends (push j), moves to the next sibling, or backs up one level (pop),
// all as selects.  At the third-to-last level the child's completion is
// forced (one city r left), so the step closes the tour directly,
// ((c + d[j][r]) + d[r][0]), instead of descending twice and popping twice.
// Only the rare record (a complete tour within the incumbent), the refill of
// lanes whose item is finished and the budget hand-back leave the loop.  v1
// ran each case as its own branch, so a wave executed all of them every
// iteration (5.1 wave instructions per node, 9% of the lane slots useful).
//
// Per-lane state in VGPRs: level L, path end k, unvisited set rem, the
// untried-children mask fm of level L, fold cost ck, sum remA of the cheapest
// incoming edges still to be paid.  Stack in LDS, [level][lane] (conflict
// free): the fold cost and the city of every level, written one level above
// the current one on every step (dead unless the step descends) and read one
// level below (used only by a pop).  remA is restored exactly on a pop
// (remA + a[k]: a[] lies on a grid), so it needs no stack.
//
// LDS: d (n rows of stride 32) | {a[x], d[x][0]} pairs | cost stack [n][T] |
//      city stack [n][T] | wave item buffers.
template <typename V>
struct ValT2;  // a value above every tour cost
template <>
struct ValT2<double> {
    __device__ static double big() { return 1.0e300; }
};
template <>
struct ValT2<int32_t> {
    __device__ static int32_t big() { return 2147483647; }
};

template <typename V>
struct Thr;  // prune threshold from the incumbent: prune iff bound > thr
template <>
struct Thr<double> {
    // bound > inc*(1+2^-39) implies bound*(1-2^-40) > inc: v1's margin
    __device__ static double of(double inc) { return inc * (1.0 + 0x1p-39); }
};
template <>
struct Thr<int32_t> {
    __device__ static int32_t of(int32_t inc) { return inc; }
};

template <typename V>
struct alignas(2 * sizeof(V)) APair {
    V a;   // cheapest edge into x (bound)
    V d0;  // d[x][0] (closing edge)
};

constexpr int kRow = 32;  // LDS row stride of d (row offset k << 5)
template <typename V>
__host__ __device__ constexpr size_t v2_ad(int n) { return align16((size_t)n * kRow * sizeof(V)); }
template <typename V>
__host__ __device__ constexpr size_t v2_cost(int n) { return v2_ad<V>(n) + align16((size_t)n * sizeof(APair<V>)); }
template <typename V>
__host__ __device__ constexpr size_t v2_city(int n) { return v2_cost<V>(n) + (size_t)n * kSearchThreads * sizeof(V); }
template <typename V>
__host__ __device__ constexpr size_t v2_wbuf(int n) { return align16(v2_city<V>(n) + (size_t)n * kSearchThreads); }
template <typename V>
__host__ __device__ constexpr size_t v2_lds(int n)
{
    return v2_wbuf<V>(n) + (size_t)(kSearchThreads / 64) * kChunk * sizeof(SearchItem);
}

// The last four cities of a path, all in registers: the 4 + 12 + 24 + 24
// partial paths below the path end k (fold cost ck) are folded in the
// reference's order ((ck + d[k][a]) + d[a][b]) + d[b][c]) + d[c][e]) + d[e][0]
// from 20 LDS reads and 88 adds of static code — no stack, no per-node
// select — and every tour within the incumbent is recorded.  First cities
// outside fm (already tried) are skipped.  No bound inside: pruning is only an
// optimisation, so the outcome (records, incumbent) is that of the DFS.
// Returns the mask of first-city slots evaluated (16 nodes each).
template <typename V>
__device__ __forceinline__ uint32_t tail4(const V *dl, const APair<V> *ad, const uint8_t *myk, int T, int krow, V ck,
                                          uint32_t rem, uint32_t fm, int L, V &inc, V &thr, const SearchArgs &a,
                                          TieCache &tcache)
{
    int c[4];
    uint32_t x = rem;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c[i] = __builtin_ctz(x);
        x &= x - 1u;
    }
    V dk[4], d0[4], dd[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dk[i] = dl[krow + c[i]];
        d0[i] = ad[c[i]].d0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j != i) dd[i][j] = dl[c[i] * kRow + c[j]];
    }
    uint32_t valid = 0;
    V tot[24];
    int e = 0;
    V best = ValT2<V>::big();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool vi = (fm >> c[i]) & 1u;
        valid |= vi ? (1u << i) : 0u;
        const V p1 = ck + dk[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j == i) continue;
            const V p2 = p1 + dd[i][j];
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                if (l == i || l == j) continue;
                const int m = 6 - i - j - l;
                const V t = ((p2 + dd[j][l]) + dd[l][m]) + d0[m];
                tot[e] = vi ? t : ValT2<V>::big();
                best = tot[e] < best ? tot[e] : best;
                ++e;
            }
        }
    }
    if (best <= inc) {
        // rare: record every tour within the incumbent, in enumeration order
        e = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j == i) continue;
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    if (l == i || l == j) continue;
                    const int m = 6 - i - j - l;
                    const V total = tot[e++];
                    if (total <= inc) {
                        const uint64_t tb = Num<V>::bits(total);
                        const unsigned long long old = atomicMin(a.inc, (unsigned long long)tb);
                        if (tb <= old) {
                            const unsigned int s = atomicAdd(a.rec_count, 1u);
                            if (s < a.rec_cap) {
                                SearchRecord *R = a.rec + s;
                                R->cost = tb;
                                for (int q = 1; q <= L; ++q) R->city[q - 1] = myk[q * T];
                                R->city[L] = (uint8_t)c[i];
                                R->city[L + 1] = (uint8_t)c[j];
                                R->city[L + 2] = (uint8_t)c[l];
                                R->city[L + 3] = (uint8_t)c[m];
                            }
                            tie_offer(a, tcache, tb, [&](int q) {
                                return q <= L ? (int)myk[q * T] : (q == L + 1 ? c[i] : q == L + 2 ? c[j] : q == L + 3 ? c[l] : c[m]);
                            });
                        }
                        const V o = Num<V>::val(old);
                        inc = o < total ? o : total;
                        thr = Thr<V>::of(inc);
                    }
                }
            }
    }
    return valid;
}

template <typename V>
__global__ __launch_bounds__(kSearchThreads) void round_kernel(SearchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int T = kSearchThreads;
    const int n = a.n;
    const int tid = threadIdx.x;
    V *dl = reinterpret_cast<V *>(smem);
    APair<V> *ad = reinterpret_cast<APair<V> *>(smem + v2_ad<V>(n));
    V *myc = reinterpret_cast<V *>(smem + v2_cost<V>(n)) + tid;              // cost of level l: myc[l*T]
    uint8_t *myk = reinterpret_cast<uint8_t *>(smem + v2_city<V>(n)) + tid;  // city of level l: myk[l*T]
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    // the frontier search's stronger bounds (SearchArgs::bnd2, ::hsuf), when given
    __shared__ V b2s[2 * kSearchMaxN];
    __shared__ uint32_t bn[32][8];
    for (int i = tid; i < n * n; i += T) dl[(i / n) * kRow + i % n] = gd[i];
    for (int i = tid; i < n; i += T) {
        ad[i].a = ga[i];
        ad[i].d0 = gd[i * n];
    }
    const bool sym = a.sym && !a.noprune, hsuf = a.hs_len > 0 && !a.noprune;
    for (int i = tid; i < 2 * n; i += T) b2s[i] = sym ? static_cast<const V *>(a.bnd2)[i] : V(0);
    stage_search_binom(bn, tid, T);
    __syncthreads();

    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;  // cities 1..N
    V aall = 0, ball = 0;
    for (int x = 0; x < n; ++x) aall += ad[x].a;                 // exact: grid values
    for (int x = 1; x < n; ++x) ball += b2s[2 * x];             // exact: grid values
    V inc = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    V thr = Thr<V>::of(inc);
    unsigned long long nodes = 0;  // wave-uniform counts
    TieCache tcache;
    unsigned long long wsteps = 0, wactive = 0, wloads = 0;
    int L = -1, root = 1;          // L < root: the lane needs an item
    int k = 0, krow = 0;           // path end and its row offset in d
    uint32_t rem = 0, fm = 0, t0 = 0;
    V ck = 0, remA = 0, remB = 0;  // remB: sum of b over rem (two-edge bound)
    bool done = false;
    uint32_t tick = 0;
    const int lane = __lane_id();
    SearchItem *wbuf = reinterpret_cast<SearchItem *>(smem + v2_wbuf<V>(n)) + (tid / 64) * kChunk;
    uint32_t pbase = 0, pnext = 0, pend = 0;

    // rebuild an item's stack: the same left fold as when it was cut
    auto load_item = [&](const SearchItem &it) {
        const int len = it.len;
        uint32_t rr = full;
        V ra = aall, rb = ball, c = 0;
        int prev = 0;
        myk[0] = 0;
        myc[0] = 0;
        for (int l = 1; l < len; ++l) {
            const int t = it.city[l];
            c = c + dl[prev * kRow + t];
            rr &= ~(1u << t);
            ra -= ad[t].a;
            rb -= b2s[2 * t];
            myk[l * T] = (uint8_t)t;
            myc[l * T] = c;
            prev = t;
        }
        if (a.noprune || !(c + ra > thr)) {
            root = len - 1;
            L = root;
            k = prev;
            krow = prev * kRow;
            ck = c;
            rem = rr;
            remA = ra;
            remB = rb;
            fm = 0xFFFFFFFEu << (it.from - 1);
            t0 = tick;
        }
    };

    auto step = [&]() {
        const bool act = L >= root;
        wsteps += 64;
        wactive += (unsigned long long)__popcll(__ballot(act));
        // Four cities left: the whole subtree in registers (see tail4), then pop.
        // (Exhaustive mode; with the bound on, the DFS's pruning inside the last
        // four levels is worth more than the tail's static code: k2_tail_time.log.)
        const bool tail = a.tails && act && __builtin_popcount(rem) == 4;
        if (__ballot(tail)) {
            uint32_t valid = 0;
            if (tail) valid = tail4<V>(dl, ad, myk, T, krow, ck, rem, fm, L, inc, thr, a, tcache);
            nodes += 16ull * (unsigned long long)(__popcll(__ballot(valid & 1u)) + __popcll(__ballot(valid & 2u)) +
                                                  __popcll(__ballot(valid & 4u)) + __popcll(__ballot(valid & 8u)));
        }
        const uint32_t cand = act && !tail ? (rem & fm) : 0u;
        const bool has = cand != 0u;
        const int j = has ? __builtin_ctz(cand) : 0;
        const uint32_t others = rem & ~(1u << j);
        const int r = others ? __builtin_ctz(others) : 0;  // the forced last city when L == n-3
        const bool sc = L == n - 3;
        const bool lf = L == n - 2;  // only for items seeded at depth n-2 (tiny n)
        const int lm1 = L > 0 ? L - 1 : 0;
        const V dkj = dl[krow + j];
        const APair<V> pr = ad[sc ? r : j];
        const V djr = dl[j * kRow + r];
        const V ak = ad[k].a;
        const V cprev = myc[lm1 * T];
        const int kprev = myk[lm1 * T];
        const V c = ck + dkj;
        const V total = (sc ? c + djr : c) + pr.d0;
        const V rest = remA - pr.a;
        const bool close = has && (sc || lf);
        nodes += (unsigned long long)__popcll(__ballot(has)) + (unsigned long long)__popcll(__ballot(has && sc));
        if (close && total <= inc) {
            // a complete tour within the incumbent (tsp.cpp:483-499): record it
            const uint64_t tb = Num<V>::bits(total);
            const unsigned long long old = atomicMin(a.inc, (unsigned long long)tb);
            if (tb <= old) {
                const unsigned int s = atomicAdd(a.rec_count, 1u);
                if (s < a.rec_cap) {
                    SearchRecord *R = a.rec + s;
                    R->cost = tb;
                    for (int l = 1; l <= L; ++l) R->city[l - 1] = myk[l * T];
                    R->city[L] = (uint8_t)j;
                    if (sc) R->city[L + 1] = (uint8_t)r;
                }
                tie_offer(a, tcache, tb, [&](int q) { return q <= L ? (int)myk[q * T] : (q == L + 1 ? j : r); });
            }
            const V o = Num<V>::val(old);
            inc = o < total ? o : total;
            thr = Thr<V>::of(inc);
        }
        bool desc = has && !close && (a.noprune || !(c + rest > thr));
        // two-edge bound: e[j] + sum over rem \ j of b + e[0] (exact grid sums)
        const V bj = b2s[2 * j], bk = b2s[2 * k];
        if (sym) desc = desc && !(c + (((remB - bj) + b2s[2 * j + 1]) + b2s[1]) > thr);
        // exact-suffix bound when j leaves hs_len cities: the cheapest completion
        if (hsuf && desc && __builtin_popcount(rem) == a.hs_len + 1) {
            const uint32_t R = rem & ~(1u << j);
            uint32_t rk = 0;
            int i = 0;
            for (uint32_t y = R; y; y &= y - 1u) rk += bn[__builtin_ctz(y) - 1][++i];
            const double *Hs = a.hsuf + a.hs_off[a.hs_len] + (size_t)rk * (uint32_t)a.hs_len;
            double best = 1.0e300;
            i = 0;
            for (uint32_t y = R; y; y &= y - 1u) {
                const double v = (double)dl[j * kRow + __builtin_ctz(y)] + Hs[i++];
                best = v < best ? v : best;
            }
            desc = !((double)c + best > (double)thr);
            if constexpr (sizeof(V) == 8) {
                // a real tour's cost up to a few roundings: scaled up, an upper bound on the optimum
                const double u = ((double)c + best) * (1.0 + 0x1p-30);
                if (desc && u < (double)inc) {
                    atomicMin(a.inc, (unsigned long long)__double_as_longlong(u));
                    inc = (V)u;
                    thr = Thr<V>::of(inc);
                }
            }
        }
        const bool pop = act && !has;
        myc[(L + 1) * T] = c;  // dead unless desc (L + 1 <= n - 2)
        myk[(L + 1) * T] = (uint8_t)j;
        rem = (rem & ~(desc ? (1u << j) : 0u)) | (pop ? (1u << k) : 0u);
        fm = desc ? 0xFFFFFFFEu : (0xFFFFFFFEu << (has ? j : k));
        remA = desc ? rest : (pop ? remA + ak : remA);
        remB = desc ? remB - bj : (pop ? remB + bk : remB);
        ck = desc ? c : (pop ? cprev : ck);
        k = desc ? j : (pop ? kprev : k);
        krow = k * kRow;
        L = (pop && L == root) ? -1 : L + (desc ? 1 : 0) - (pop ? 1 : 0);
    };

    for (;;) {
        // ---- refill: lanes without an item take consecutive queue entries
        const bool need = !done && L < root;
        const unsigned long long nm = __ballot(need);
        if (nm) {
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
        wloads += (unsigned long long)__popcll(nm) - (unsigned long long)__popcll(__ballot(done) & nm);
        const unsigned long long live = __ballot(!done);
        if (live == 0) break;
        if (__ballot(L >= root) == 0) continue;  // every loaded item was pruned: refill again

        // ---- lock-step DFS, two steps per exit test
        for (;;) {
            tick += 2;
            if ((tick & 255u) == 0) {
                const V g = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (g < inc) {
                    inc = g;
                    thr = Thr<V>::of(g);
                }
            }
            step();
            step();
            const unsigned long long needm = __ballot(L < root) & live;
            const unsigned long long over = __ballot(L >= root && tick - t0 > a.budget);
            if (needm == live || (uint32_t)__popcll(needm) >= a.refill || over) break;
        }

        // ---- budget spent: hand back, level by level, the children not tried yet
        if (L >= root && tick - t0 > a.budget) {
            uint32_t rl = rem, fl = fm ? (uint32_t)__builtin_ctz(fm) : 32u;
            unsigned int cnt = 0;
            for (int l = L; l >= root; --l) {
                if (rl & (uint32_t)(0xFFFFFFFFull << fl)) ++cnt;
                if (l > root) {
                    const int c1 = myk[l * T];
                    rl |= 1u << c1;
                    fl = (uint32_t)c1 + 1u;
                }
            }
            // the host sizes the output for (N-1) items per input item: always room
            unsigned int slot = cnt ? atomicAdd(a.out_count, cnt) : 0u;
            rl = rem;
            fl = fm ? (uint32_t)__builtin_ctz(fm) : 32u;
            for (int l = L; l >= root; --l) {
                if (rl & (uint32_t)(0xFFFFFFFFull << fl)) {
                    uint32_t *dst = reinterpret_cast<uint32_t *>(a.out + slot);
                    for (int b = 0; b < 8; ++b) {
                        uint32_t word = 0;
                        for (int q = 0; q < 4; ++q) {
                            const int lv = 4 * b + q;
                            if (lv <= l) word |= (uint32_t)myk[lv * T] << (8 * q);
                        }
                        dst[b] = word;
                    }
                    dst[8] = (uint32_t)(l + 1) | (fl << 8);
                    ++slot;
                }
                if (l > root) {
                    const int c1 = myk[l * T];
                    rl |= 1u << c1;
                    fl = (uint32_t)c1 + 1u;
                }
            }
            L = -1;
        }
    }
    if (lane == 0) {
        unsigned long long *st = stat_line(a);
        atomicAdd(st, nodes);
        atomicAdd(st + 1, wsteps);
        atomicAdd(st + 2, wactive);
        atomicAdd(st + 3, wloads);
    }
}

// ---------------------------------------------------------------------------
// Persistent search (kernel 3): ONE launch runs the whole search.  Lanes take
// this shard's seed prefixes from a cursor (decoded on the fly, no seed
// array), then items from a device ring; a busy lane donates work only when
// the ring runs low ("hungry"): its root level's untried children become one
// ring item and its own root moves one level down (the largest untried piece
// goes, the lane keeps its current path).  No rounds, no host round trips, no
// budget splitting while every lane is busy.  Termination: `work` counts
// items created and not finished (a donor adds before publishing, a lane
// subtracts when its item is done); a wave whose lanes all wait for ring
// items exits when work == 0.  A watchdog (wall clock) and a ring-lap check
// end every wave with an abort code instead of hanging.
//
// Hand-off (cross-XCD, MI355X L2s are per XCD): the donor writes the item's
// four payload words with agent-scope atomic stores (write-through), drains
// them (s_waitcnt vmcnt(0)), then stores the tag word (ticket+1 in the high
// half); the claimer polls the tag relaxed, then one agent-scope acquire, then
// agent-scope loads of the payload.
using gu64 = unsigned long long;

__device__ __forceinline__ gu64 ld_agent(const gu64 *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(gu64 *p, gu64 v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename V>
__global__ __launch_bounds__(kSearchThreads) void persist_kernel(SearchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ uint32_t pv[33];
    constexpr int T = kSearchThreads;
    const int n = a.n, N = n - 1, D = a.depth;
    const int tid = threadIdx.x;
    V *dl = reinterpret_cast<V *>(smem);
    APair<V> *ad = reinterpret_cast<APair<V> *>(smem + v2_ad<V>(n));
    V *myc = reinterpret_cast<V *>(smem + v2_cost<V>(n)) + tid;
    uint8_t *myk = reinterpret_cast<uint8_t *>(smem + v2_city<V>(n)) + tid;
    const V *gd = static_cast<const V *>(a.dist);
    const V *ga = static_cast<const V *>(a.amin);
    for (int i = tid; i < n * n; i += T) dl[(i / n) * kRow + i % n] = gd[i];
    for (int i = tid; i < n; i += T) {
        ad[i].a = ga[i];
        ad[i].d0 = gd[i * n];
    }
    if (tid == 0) {
        uint32_t p = 1;
        pv[D] = 1;
        for (int l = D; l >= 2; --l) {
            p *= (uint32_t)(N - l + 1);
            pv[l - 1] = p;
        }
    }
    __syncthreads();
    const long long t_start = wall_clock64();
    PersistState *ps = a.ps;
    const uint32_t full = (uint32_t)((1ull << n) - 1ull) & ~1u;
    V aall = 0;
    for (int x = 0; x < n; ++x) aall += ad[x].a;
    V inc = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    V thr = Thr<V>::of(inc);
    const unsigned long long local = a.items / a.nshards + (a.items % a.nshards > a.shard ? 1u : 0u);
    const int lane = __lane_id();

    // lane state (as the v2 round kernel) + ring claim
    int L = -1, root = 1, k = 0, krow = 0;
    uint32_t rem = 0, fm = 0, t0 = 0;
    V ck = 0, remA = 0;
    bool owned = false, done = false;
    long long slot = -1;
    // wave-uniform state
    uint32_t tick = 0, idle = 0;
    bool seeds_left = true, hungry = false;
    unsigned long long nodes = 0, wsteps = 0, wactive = 0, wloads = 0, wfin = 0;
    TieCache tcache;

    auto start = [&](int len, int prev, V c, uint32_t rr, V ra, uint32_t from) {
        root = len - 1;
        L = root;
        k = prev;
        krow = prev * kRow;
        ck = c;
        rem = rr;
        remA = ra;
        fm = 0xFFFFFFFEu << (from - 1);
        t0 = tick;
    };
    // seed prefix `idx` of this shard: decode (as seed_kernel), fold, bound
    auto load_seed = [&](unsigned long long idx) -> bool {
        uint32_t p = (uint32_t)(idx * a.nshards + a.shard);
        uint32_t rr = full;
        V ra = aall, c = 0;
        int prev = 0;
        myk[0] = 0;
        myc[0] = 0;
        for (int l = 1; l <= D; ++l) {
            const uint32_t q = p / pv[l];
            p -= q * pv[l];
            uint32_t x = rr;
            for (uint32_t s2 = 0; s2 < q; ++s2) x &= x - 1u;
            const int t = __builtin_ctz(x);
            c = c + dl[prev * kRow + t];
            rr &= ~(1u << t);
            ra -= ad[t].a;
            myk[l * T] = (uint8_t)t;
            myc[l * T] = c;
            prev = t;
            if (c + ra > thr) return false;
        }
        start(D + 1, prev, c, rr, ra, 1u);
        return true;
    };
    // ring item: refold the prefix (the same left fold as when it was cut)
    auto load_ring = [&](const gu64 *w, uint32_t meta) -> bool {
        const int len = (int)(meta & 0xFFu);
        const uint32_t from = (meta >> 8) & 0xFFu;
        uint32_t rr = full;
        V ra = aall, c = 0;
        int prev = 0;
        myk[0] = 0;
        myc[0] = 0;
        gu64 word = 0;
        for (int l = 1; l < len; ++l) {
            if ((l & 7) == 0 || l == 1) word = ld_agent(w + (l >> 3));
            const int t = (int)((word >> (8 * (l & 7))) & 0xFFu);
            c = c + dl[prev * kRow + t];
            rr &= ~(1u << t);
            ra -= ad[t].a;
            myk[l * T] = (uint8_t)t;
            myc[l * T] = c;
            prev = t;
        }
        if (c + ra > thr) return false;
        start(len, prev, c, rr, ra, from);
        return true;
    };

    auto step = [&]() {
        const bool act = L >= root;
        wsteps += 64;
        wactive += (unsigned long long)__popcll(__ballot(act));
        const uint32_t cand = act ? (rem & fm) : 0u;
        const bool has = cand != 0u;
        const int j = has ? __builtin_ctz(cand) : 0;
        const uint32_t others = rem & ~(1u << j);
        const int r = others ? __builtin_ctz(others) : 0;
        const bool sc = L == n - 3;
        const bool lf = L == n - 2;
        const int lm1 = L > 0 ? L - 1 : 0;
        const V dkj = dl[krow + j];
        const APair<V> pr = ad[sc ? r : j];
        const V djr = dl[j * kRow + r];
        const V ak = ad[k].a;
        const V cprev = myc[lm1 * T];
        const int kprev = myk[lm1 * T];
        const V c = ck + dkj;
        const V total = (sc ? c + djr : c) + pr.d0;
        const V rest = remA - pr.a;
        const bool close = has && (sc || lf);
        nodes += (unsigned long long)__popcll(__ballot(has)) + (unsigned long long)__popcll(__ballot(has && sc));
        if (close && total <= inc) {
            const uint64_t tb = Num<V>::bits(total);
            const unsigned long long old = atomicMin(a.inc, (unsigned long long)tb);
            if (tb <= old) {
                const unsigned int s2 = atomicAdd(a.rec_count, 1u);
                if (s2 < a.rec_cap) {
                    SearchRecord *R = a.rec + s2;
                    R->cost = tb;
                    for (int l = 1; l <= L; ++l) R->city[l - 1] = myk[l * T];
                    R->city[L] = (uint8_t)j;
                    if (sc) R->city[L + 1] = (uint8_t)r;
                }
                tie_offer(a, tcache, tb, [&](int q) { return q <= L ? (int)myk[q * T] : (q == L + 1 ? j : r); });
            }
            const V o = Num<V>::val(old);
            inc = o < total ? o : total;
            thr = Thr<V>::of(inc);
        }
        const bool desc = has && !close && !(c + rest > thr);
        const bool pop = act && !has;
        myc[(L + 1) * T] = c;
        myk[(L + 1) * T] = (uint8_t)j;
        rem = (rem & ~(desc ? (1u << j) : 0u)) | (pop ? (1u << k) : 0u);
        fm = desc ? 0xFFFFFFFEu : (0xFFFFFFFEu << (has ? j : k));
        remA = desc ? rest : (pop ? remA + ak : remA);
        ck = desc ? c : (pop ? cprev : ck);
        k = desc ? j : (pop ? kprev : k);
        krow = k * kRow;
        L = (pop && L == root) ? -1 : L + (desc ? 1 : 0) - (pop ? 1 : 0);
    };

    for (;;) {
        // ---- finished items leave `work` (before this wave can wait on it)
        const bool fin = owned && L < root;
        if (fin) owned = false;
        wfin += (unsigned long long)__popcll(__ballot(fin));
        if (wfin) {
            if (lane == 0) atomicAdd(&ps->work.v, (unsigned long long)0 - wfin);
            wfin = 0;
        }
        // ---- lanes without an item: seeds first, then ring tickets
        bool need = !done && L < root && slot < 0;
        unsigned long long nm = __ballot(need);
        if (nm && seeds_left) {
            const uint32_t cnt = (uint32_t)__popcll(nm);
            const uint32_t r = (uint32_t)__popcll(nm & ((1ull << lane) - 1ull));
            const int leader = __ffsll((long long)nm) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(&ps->seed_cursor.v, (unsigned long long)cnt);
            base = __shfl(base, leader);
            if (base + cnt >= local) seeds_left = false;
            const bool got = need && base + r < local;
            bool live = false;
            if (got) {
                live = load_seed(base + r);
                owned = live;
            }
            wloads += (unsigned long long)__popcll(__ballot(got));
            wfin += (unsigned long long)__popcll(__ballot(got && !live));
            need = need && !got;
            nm = __ballot(need);
        }
        if (nm && !seeds_left) {
            const uint32_t cnt = (uint32_t)__popcll(nm);
            const uint32_t r = (uint32_t)__popcll(nm & ((1ull << lane) - 1ull));
            const int leader = __ffsll((long long)nm) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(&ps->head.v, (unsigned long long)cnt);
            base = __shfl(base, leader);
            if (need) slot = (long long)(base + r);
        }
        // ---- claimed tickets: take the item once its tag shows up
        const bool wt = slot >= 0;
        if (__ballot(wt)) {
            bool ready = false, live = false;
            if (wt) {
                const gu64 *w = a.ring + (size_t)((uint64_t)slot & a.ring_mask) * kRingWords;
                const gu64 meta = ld_agent(w + 4);
                const uint32_t tag = (uint32_t)(meta >> 32), want = (uint32_t)(slot + 1);
                if (tag == want) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    ready = true;
                    slot = -1;
                    live = load_ring(w, (uint32_t)meta);
                    owned = live;
                } else if ((int32_t)(tag - want) > 0) {
                    atomicOr((unsigned int *)&ps->abort.v, 2u);  // lapped: never expected (capacity check)
                }
            }
            const unsigned long long rm = __ballot(ready);
            if (rm) {
                if (lane == __ffsll((long long)rm) - 1) atomicAdd(&ps->consumed.v, (unsigned long long)__popcll(rm));
                wloads += (unsigned long long)__popcll(rm);
                wfin += (unsigned long long)__popcll(__ballot(ready && !live));
            }
        }
        // ---- nothing to step: flush, then wait for tickets or the end
        if (__ballot(L >= root) == 0) {
            if (wfin) {
                if (lane == 0) atomicAdd(&ps->work.v, (unsigned long long)0 - wfin);
                wfin = 0;
            }
            if (__ballot(!done) == 0) break;
            if (seeds_left) continue;  // seeds were pruned at once: take more
            // every wave polls its own ring tags each pass; the shared words only every 16th
            if ((++idle & 15u) == 0) {
                const gu64 w = ld_agent(&ps->work.v);
                const unsigned ab = (unsigned)ld_agent(&ps->abort.v);
                if (w == 0 || ab) break;
                if (wall_clock64() - t_start > (long long)a.wall_limit) {
                    if (lane == 0) atomicOr((unsigned int *)&ps->abort.v, 1u);
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(8);
            continue;
        }
        const unsigned long long live = __ballot(!done);

        // ---- lock-step DFS, two steps per exit test
        for (;;) {
            tick += 2;
            if ((tick & 255u) == 0) {
                const V g = Num<V>::val(__hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (g < inc) {
                    inc = g;
                    thr = Thr<V>::of(g);
                }
                const gu64 sc = ld_agent(&ps->seed_cursor.v), h = ld_agent(&ps->head.v), t = ld_agent(&ps->tail.v);
                // hungry: lanes hold tickets no donor has reserved yet
                hungry = sc >= local && (long long)(h - t) > (long long)a.hungry;
                if ((tick & 65535u) == 0) {
                    const unsigned ab = (unsigned)ld_agent(&ps->abort.v);
                    if (ab || wall_clock64() - t_start > (long long)a.wall_limit) {
                        if (lane == 0) atomicOr((unsigned int *)&ps->abort.v, 1u);
                        done = true;
                        L = -1;
                        owned = false;
                        break;
                    }
                }
            }
            step();
            step();
            // lanes holding a ticket are already served: they count for the
            // refill only as idle lanes, and their tags are polled every 128 ticks
            const unsigned long long idlem = __ballot(L < root) & live;
            const unsigned long long needm = idlem & ~__ballot(slot >= 0);
            const bool don = hungry && L > root && tick - t0 > a.min_split;
            if (idlem == live || (uint32_t)__popcll(needm) >= a.refill || __ballot(don) ||
                ((tick & 255u) == 0 && idlem != needm))
                break;
        }
        if (__ballot(done)) break;  // watchdog

        // ---- donate: the root level's untried children become one ring item
        if (hungry) {
            bool don = L > root && tick - t0 > a.min_split;
            int c1 = 0;
            if (don) {
                // unvisited set at the root level; a root level with nothing
                // left untried moves the root down (the same remaining work)
                uint32_t rr = rem;
                for (int l = root + 1; l <= L; ++l) rr |= 1u << myk[l * T];
                don = false;
                while (root < L) {
                    c1 = myk[(root + 1) * T];
                    rr &= ~(1u << c1);
                    if ((rr & (0xFFFFFFFEu << c1)) != 0u) {
                        don = true;
                        break;
                    }
                    root += 1;
                }
                if (!don) t0 = tick;
            }
            const unsigned long long dm = __ballot(don);
            if (dm) {
                const uint32_t cnt = (uint32_t)__popcll(dm);
                const uint32_t r = (uint32_t)__popcll(dm & ((1ull << lane) - 1ull));
                const int leader = __ffsll((long long)dm) - 1;
                unsigned long long base = ~0ull;
                if (lane == leader) {
                    const gu64 t = ld_agent(&ps->tail.v), cns = ld_agent(&ps->consumed.v);
                    if (t + cnt - cns <= (gu64)a.ring_mask + 1 - a.ring_margin) {
                        atomicAdd(&ps->work.v, (unsigned long long)cnt);  // before anything is published
                        base = atomicAdd(&ps->tail.v, (unsigned long long)cnt);
                    }
                }
                base = __shfl(base, leader);
                if (base != ~0ull && don) {
                    const unsigned long long tk = base + r;
                    gu64 *w = a.ring + (size_t)(tk & a.ring_mask) * kRingWords;
                    for (int b = 0; b < 4; ++b) {
                        gu64 word = 0;
                        for (int q = 0; q < 8; ++q) {
                            const int lv = 8 * b + q;
                            if (lv <= root) word |= (gu64)myk[lv * T] << (8 * q);
                        }
                        st_agent(w + b, word);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    st_agent(w + 4, ((gu64)(uint32_t)(tk + 1) << 32) | ((gu64)(c1 + 1) << 8) | (gu64)(root + 1));
                    root += 1;
                    t0 = tick;
                }
            }
        }
    }
    if (lane == 0) {
        unsigned long long *st = stat_line(a);
        atomicAdd(st, nodes);
        atomicAdd(st + 1, wsteps);
        atomicAdd(st + 2, wactive);
        atomicAdd(st + 3, wloads);
    }
}

// The optimum's tie slot: out[0] = 1 if a slot holds cost *a.inc, out[1] =
// its least w0, out[2..3] = (w0, least w1) of that w0's sub-slot (two-word
// keys), out[4] = the overflow flag.  One wave.
__global__ __launch_bounds__(64) void tie_lookup_kernel(SearchArgs a, unsigned long long *out, int at_inc,
                                                        unsigned long long cost)
{
    const unsigned long long opt =
        at_inc ? __hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : cost;
    const int lane = (int)threadIdx.x;
    if (lane == 0) {
        out[0] = 0;
        out[4] = *a.tie_overflow;
    }
    __syncthreads();
    for (uint32_t i = (uint32_t)lane; i <= a.tie_mask; i += 64) {
        const TieSlot &e = a.tie[i];
        if (e.cost == opt) {
            out[0] = 1;
            out[1] = e.w0;
            out[2] = kTieEmpty;
            out[3] = kTieEmpty;
            for (int k = 0; k < kTieSub; ++k)
                if (e.sub[k][0] == e.w0) {
                    out[2] = e.sub[k][0];
                    out[3] = e.sub[k][1];
                }
        }
    }
}

// search_solve's readbacks in ONE launch, written straight into pinned host
// memory (no copy commands): out[0..3] the summed statistics lines, out[4..19]
// the 16 counter words, out[20..24] the optimum's tie slot (as
// tie_lookup_kernel), out[25] the device wall clock at its start, out[32..]
// the first min(records, spec_cap) records.
__global__ __launch_bounds__(256) void fetch_kernel(SearchArgs a, const unsigned long long *words,
                                                    unsigned long long *out, uint32_t spec_cap)
{
    const int t = (int)threadIdx.x;
    if (t == 0) out[25] = wall_clock64();  // (the chain's end: see SearchArgs::t_start)
    __shared__ unsigned long long part[4][kStatLines];
    __shared__ unsigned long long tie[4];
    part[t & 3][t >> 2] = a.nodes[(t >> 2) * kStatStride + (t & 3)];  // 256 threads = 64 lines x 4
    if (t == 0) tie[0] = 0;
    __syncthreads();
    const unsigned long long opt = __hip_atomic_load(a.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.tie)
        for (uint32_t i = (uint32_t)t; i <= a.tie_mask; i += 256) {
            const TieSlot &e = a.tie[i];
            if (e.cost == opt) {  // (at most one slot holds a cost)
                tie[0] = 1;
                tie[1] = e.w0;
                tie[2] = kTieEmpty;
                tie[3] = kTieEmpty;
                for (int k = 0; k < kTieSub; ++k)
                    if (e.sub[k][0] == e.w0) {
                        tie[2] = e.sub[k][0];
                        tie[3] = e.sub[k][1];
                    }
            }
        }
    __syncthreads();
    if (t < 4) {
        unsigned long long sum = 0;
        for (int l = 0; l < kStatLines; ++l) sum += part[t][l];
        out[t] = sum;
    }
    if (t < 16) out[4 + t] = words[t];
    if (t < 4) out[20 + t] = tie[t];
    if (t == 0) out[24] = a.tie_overflow ? *a.tie_overflow : 0u;
    const uint32_t claimed = *a.rec_count;
    const uint32_t cnt = claimed < spec_cap ? claimed : spec_cap;
    const unsigned long long *src = reinterpret_cast<const unsigned long long *>(a.rec);
    constexpr uint32_t kW = sizeof(SearchRecord) / 8;
    for (uint32_t i = (uint32_t)t; i < cnt * kW; i += 256) out[32 + i] = src[i];
}

// The search's upper bound computed on the device, in the init launch (block
// 0, sixteen waves), instead of by the host before the search: the host
// heuristic's construction (search_host.cpp: nearest neighbour from four
// spread start cities, local search, the smaller exact left fold of either
// direction) with one wave per start city.  Nearest neighbour (ties: the lowest city),
// then best-improvement 2-opt over all position pairs at once (up to three
// per lane): on symmetric matrices the four-edge delta is exact; otherwise the
// chosen move's reversed edges are priced and a move that does not gain ends
// the descent.  The distances are read from the host staging (pinned) into
// LDS once.  Any tour's cost is a valid incumbent, so a tour that is not a
// permutation (never expected) is dropped rather than published.
__device__ __forceinline__ double wave_sum(double x)
{
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

__device__ __forceinline__ void init_heuristic(const SearchInit &in)
{
    // 1024 threads (heur_starts of them work); heur_n <= kSearchMaxN: <= 465 pairs (8 per lane)
    constexpr int kWaves = 16, kPairs = ((kSearchMaxN - 1) * (kSearchMaxN - 2) / 2 + 63) / 64;
    __shared__ double hd[kSearchMaxN * kSearchMaxN];
    __shared__ int ht[kWaves][kSearchMaxN];
    __shared__ double hbest[kWaves];
    const int n = in.heur_n;
    for (int i = threadIdx.x; i < n * n; i += blockDim.x)
        hd[i] = in.heur_f64 ? static_cast<const double *>(in.heur_dist)[i]
                            : (double)static_cast<const int32_t *>(in.heur_dist)[i];
    __syncthreads();
    const int lane = __lane_id(), wv = (int)(threadIdx.x >> 6);
    int *t = ht[wv];
    // this lane's moves: reverse positions i..j, 1 <= i < j <= n-1 (pair lane + 64 r)
    int mi[kPairs], mj[kPairs];
#pragma unroll
    for (int r = 0; r < kPairs; ++r) {
        int rem = lane + 64 * r;
        mi[r] = 0;
        mj[r] = 0;
        for (int i = 1; i <= n - 2; ++i) {
            const int c = n - 1 - i;
            if (rem < c) {
                mi[r] = i;
                mj[r] = i + 1 + rem;
                break;
            }
            rem -= c;
        }
    }
    double wbest = 1.0e300;
    // start cities spread over the tour like the host's (search_host.cpp
    // heuristic: 0, n/4, n/2, 3n/4 for four), one wave each on its own SIMD
    const int ns = in.heur_starts < n ? in.heur_starts : n;
    for (int w = wv; w < ns; w += kWaves) {  // (wave-uniform)
        const int s0 = w * n / ns;
        if (lane == 0) t[0] = s0;
        uint32_t used = 1u << s0;
        int cur = s0;
        for (int k = 1; k < n; ++k) {
            const bool cand = lane < n && !((used >> (lane & 31)) & 1u);
            const double v = cand ? hd[cur * n + lane] : 1.0e300;
            const double m = wave_min_dpp(v);
            const int j = __builtin_ctzll(__ballot(cand && v == m));
            if (lane == 0) t[k] = j;
            used |= 1u << j;
            cur = j;
        }
        double total = wave_sum(lane < n ? hd[t[lane] * n + t[lane + 1 < n ? lane + 1 : 0]] : 0.0);
        for (int it = 0; it < in.heur_iters; ++it) {
            double best = 0.0;
            int bi = 0, bj = 0;
#pragma unroll
            for (int r = 0; r < kPairs; ++r) {
                if (!mi[r]) continue;
                const int i = mi[r], j = mj[r];
                const int a = t[i - 1], b = t[i], c = t[j], e = t[j + 1 < n ? j + 1 : 0];
                const double dlt = (hd[a * n + c] + hd[b * n + e]) - (hd[a * n + b] + hd[c * n + e]);
                if (dlt < best) best = dlt, bi = i, bj = j;
            }
            const double m = wave_min_dpp(best);
            const double tol = -1e-9 * (1.0 + total);
            if (!(m < tol)) break;  // (wave-uniform)
            const int wl = __builtin_ctzll(__ballot(bi > 0 && best == m));
            const int i = __builtin_amdgcn_readlane(bi, wl), j = __builtin_amdgcn_readlane(bj, wl);
            double gain = m;
            if (!in.heur_sym) {  // the segment's own edges, reversed
                const double x = lane >= i && lane < j ? hd[t[lane + 1] * n + t[lane]] - hd[t[lane] * n + t[lane + 1]] : 0.0;
                gain += wave_sum(x);
                if (!(gain < tol)) break;
            }
            const bool in_seg = lane >= i && lane <= j;
            const int v = in_seg ? t[i + j - lane] : 0;
            if (in_seg) t[lane] = v;
            total += gain;
        }
        // the left fold from city 0: lane 0 forward, lane 1 backward
        const int p0 = __builtin_ctzll(__ballot(lane < n && t[lane] == 0));
        const int dir = lane == 1 ? n - 1 : 1;
        double c = 0.0;
        int prev = 0;
        for (int q = 1; q < n; ++q) {
            const int x = t[(p0 + q * dir) % n];
            c = c + hd[prev * n + x];
            prev = x;
        }
        c = c + hd[prev * n];
        const uint32_t bit = lane < n ? 1u << (t[lane] & 31) : 0u;
        uint32_t seen = bit;
        for (int off = 32; off >= 1; off >>= 1) seen |= (uint32_t)__shfl_xor((int)seen, off);
        const bool perm = seen == (uint32_t)((1ull << n) - 1ull);
        const double c0 = __shfl(c, 0), c1 = __shfl(c, 1);
        if (perm) wbest = fmin(wbest, fmin(c0, c1));
    }
    if (lane == 0) hbest[wv] = wbest;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = hbest[0];
        for (int w = 1; w < kWaves; ++w) b = fmin(b, hbest[w]);
        unsigned long long u = in.inc_init;
        if (b < 1.0e300) {
            const unsigned long long hb = in.heur_f64 ? (unsigned long long)__double_as_longlong(b)
                                                      : (unsigned long long)(uint32_t)(int32_t)b;
            u = hb < u ? hb : u;  // (non-negative costs: the encodings order like the values)
        }
        *in.inc_word[0] = u;
        *in.inc_word[1] = u;
    }
}

__global__ __launch_bounds__(1024) void init_kernel(SearchInit in)
{
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
    // every table's first word of this thread loaded before any store: the
    // sources are pinned host memory, one PCIe round trip instead of one per
    // table (the tables are far below one stride; the loops below are the rest)
    uint32_t v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < in.ncopy && t0 < in.words[c] ? in.src[c][t0] : 0u;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        if (c < in.ncopy && t0 < in.words[c]) in.dst[c][t0] = v[c];
    for (int c = 0; c < in.ncopy; ++c)
        for (uint32_t i = t0 + stride; i < in.words[c]; i += stride) in.dst[c][i] = in.src[c][i];
    for (uint32_t i = t0; i < in.n_ff; i += stride) in.fill_ff[i] = 0xFFFFFFFFu;
    for (int z = 0; z < 2; ++z)
        for (uint32_t i = t0; i < in.n_zero[z]; i += stride) in.zero[z][i] = 0u;
    if (blockIdx.x != 0) return;  // (block-uniform)
    if (in.heur_n > 0) {
        init_heuristic(in);
    } else if (threadIdx.x == 0) {
        *in.inc_word[0] = in.inc_init;
        *in.inc_word[1] = in.inc_init;
    }
}

}  // namespace

hipError_t launch_init(const SearchInit &init, hipStream_t stream)
{
    if (init.ncopy < 0 || init.ncopy > 8 || init.heur_n < 0 || init.heur_n > kSearchMaxN ||
        (init.heur_n && (init.heur_n < 4 || init.heur_starts < 1 || init.heur_starts > 16)))
        return hipErrorInvalidValue;
    // 16 blocks of 1024 (block 0's sixteen waves: the heuristic's start cities)
    hipLaunchKernelGGL(init_kernel, dim3(16), dim3(1024), 0, stream, init);
    return hipGetLastError();
}

hipError_t launch_fetch(const SearchArgs &a, const unsigned long long *words, unsigned long long *out,
                        uint32_t spec_cap)
{
    static_assert(sizeof(SearchRecord) % 8 == 0 && kStatLines * 4 == 256, "fetch layout");
    hipLaunchKernelGGL(fetch_kernel, dim3(1), dim3(256), 0, a.stream, a, words, out, spec_cap);
    return hipGetLastError();
}

hipError_t launch_tie_lookup(const SearchArgs &a, unsigned long long *out, const unsigned long long *cost)
{
    hipLaunchKernelGGL(tie_lookup_kernel, dim3(1), dim3(64), 0, a.stream, a, out, cost ? 0 : 1, cost ? *cost : 0ull);
    return hipGetLastError();
}

size_t search_lds_bytes(int n, bool f64, int kernel)
{
    if (kernel == 1) return f64 ? lds_bytes<double>(n) : lds_bytes<int32_t>(n);
    if (kernel == 3) return f64 ? v2_wbuf<double>(n) : v2_wbuf<int32_t>(n);  // no item buffers
    return f64 ? v2_lds<double>(n) : v2_lds<int32_t>(n);
}

hipError_t launch_persist(const SearchArgs &a, bool f64, int grid)
{
    const size_t lds = search_lds_bytes(a.n, f64, 3);
    void (*fn)(SearchArgs) = f64 ? persist_kernel<double> : persist_kernel<int32_t>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kSearchThreads), lds, a.stream, a);
    return hipGetLastError();
}

hipError_t launch_round(const SearchArgs &a, bool f64, int grid)
{
    const size_t lds = search_lds_bytes(a.n, f64, a.kernel);
    void (*fn)(SearchArgs) = a.kernel == 1 ? (f64 ? round_kernel_v1<double> : round_kernel_v1<int32_t>)
                                           : (f64 ? round_kernel<double> : round_kernel<int32_t>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kSearchThreads), lds, a.stream, a);
    return hipGetLastError();
}

}  // namespace tspgpu
