// Internal launch interface of K2, the prefix-parallel exact search
// (search.hip).  Public entry points: include/tspgpu.h, "K2".
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tspgpu {

constexpr int kSearchMaxN = 32;     // cities, city 0 included (tour bits 1..31 of a u32)
constexpr int kSearchThreads = 256; // workgroup size of the search kernels

// One recorded complete tour: cost (IEEE bits of the f64 fold, or the integer
// cost) and the inner cities t1..tN in visiting order (tsp.cpp's path minus
// the two 0s).
struct SearchRecord {
    uint64_t cost;
    uint8_t city[kSearchMaxN];
};

// One unit of search work: the subtrees below the path city[0..len-1]
// (city[0] = 0) whose next city is >= `from`.  Seeds are whole prefixes
// (from = 1); a lane that spends its budget on an item hands back, per level
// of its stack, the siblings it has not tried yet as new items.
struct SearchItem {
    uint8_t city[kSearchMaxN];
    uint8_t len;
    uint8_t from;
    uint8_t pad[2];
};

// A frontier path (frontier search: expand_kernel, tail_kernel): byte 0 =
// len (cities on the path, city 0 included), bytes 1..len-1 = t1..t(len-1).
// 32 bytes, 16-byte aligned: two dwordx4 per item.
struct alignas(16) PathItem {
    uint8_t b[32];
};

// Device words of the persistent search (search_persist_kernel), zeroed by
// the host before every launch except work = this shard's seed count.  Each
// word has a 256-byte line of its own: the counters take atomics from every
// wave and idle waves poll `work`, so sharing a line would serialise them.
struct alignas(256) PersistWord {
    unsigned long long v;
    unsigned long long pad[31];
};
struct PersistState {
    PersistWord seed_cursor;  // next seed (index into this shard's prefixes)
    PersistWord head;         // ring tickets claimed by lanes
    PersistWord tail;         // ring tickets reserved by donors
    PersistWord consumed;     // ring items read
    PersistWord work;         // items created (seeds + donations) and not finished
    PersistWord abort;        // 1: watchdog, 2: ring lapped (never expected)
};
constexpr int kRingWords = 5;  // ring item: 4 words of city bytes + (ticket+1) << 32 | from << 8 | len

struct SearchArgs {
    const void *dist;          // n*n row-major, f64 or i32 (device)
    const void *amin;          // n: cheapest edge entering each city (device), f64 on a 2^-20 grid or i32
    int n;
    int depth;                 // seed prefix depth D (1 <= D <= n-2)
    uint32_t items;            // global prefix count N!/(N-D)!
    uint32_t shard, nshards;   // this shard seeds prefixes p = i*nshards + shard
    uint32_t budget;           // DFS iterations per item before its rest is handed back
    const SearchItem *in;      // round input
    uint32_t in_count;
    SearchItem *out;           // seed output / round spill output
    unsigned int *out_count;
    unsigned int *queue;       // next input item (device counter, zeroed by the host)
    unsigned long long *inc;   // incumbent: f64 bits or integer cost (device, atomicMin)
    SearchRecord *rec;         // record buffer (device)
    unsigned int *rec_count;   // records claimed (may exceed rec_cap: overflow)
    unsigned int rec_cap;
    // statistics: kStatLines lines of kStatStride u64, a block adds to line
    // blockIdx % kStatLines (one hot address serialises device atomics):
    // [0] search nodes evaluated, v2: [1] lane slots, [2] active lane steps, [3] item loads
    unsigned long long *nodes;
    uint32_t refill;           // v2: a wave refills once this many lanes wait for an item
    // persistent search (kernel 3)
    PersistState *ps;
    unsigned long long *ring;  // kRingWords u64 per item
    uint32_t ring_mask;        // capacity - 1 (power of two)
    uint32_t ring_margin;      // reservations stop this far below capacity
    int32_t hungry;            // donate while more than this many lanes wait for unreserved tickets
    uint32_t min_split;        // steps on an item before it may donate
    unsigned long long wall_limit;  // watchdog, wall_clock64 ticks
    int kernel;                // round kernel: 2 (lock-step DFS, default) or 1 (branching DFS); 3 = persistent
    int noprune;               // exhaustive enumeration: no bound test (kernels 2 and seed only)
    int tails;                 // kernel 2: last four cities enumerated in registers (tail4)
    // frontier search (expand_kernel + tail_kernel): fin is expanded one
    // level; children with tail_level inner cities (tail_len = N - tail_level
    // cities left) go to ftail, the others to fout.
    int tail_level;
    int tail_len;              // 5 or 6
    const PathItem *fin;       // (the first input segment)
    uint32_t fin_count;        // paths of the step, over all its input segments
    // a step's input may span up to kFinSegs frontier segments (the top of the
    // LIFO stack): path i is fseg[k][i - fseg_start[k]] for the last k < nseg
    // with fseg_start[k] <= i
    const PathItem *fseg[4];
    uint32_t fseg_start[4];
    int nseg;
    uint32_t fin_per_block;    // expand_kernel: paths per block (multiple of 256; expand_local_kernel: of 64)
    // chained levels expanded block-locally (expand_local_kernel, > 0): up to
    // this many levels of a run's subtree inside one launch, the levels between
    // kept in LDS; children that reach the tail level, that the LDS queue
    // cannot hold or that the last local level makes go to ftail / fout
    int local_levels;
    PathItem *fout;
    PathItem *ftail;
    unsigned int *tail_count;  // items in ftail (tail_kernel reads it on the device)
    unsigned int *out_next;    // expand_kernel: zeroes the next step's out_count (double-buffered counters)
    unsigned int tail_cap;
    // chained frontier levels (search_abi.cpp run_chain): the step's input
    // count read on the device (fin_count is then only the grid's bound),
    // a fixed grid of at most max_grid blocks looping over the input runs,
    // and outputs checked against fout_cap / tail_cap (*overflow = 1, the
    // block's children dropped) instead of sized on the host
    const unsigned int *fin_count_dev;
    unsigned int fin_cap;      // chained: paths the input buffer holds (its first tile is read before the count; 0: not)
    unsigned int fout_cap;
    unsigned int *overflow;
    int max_grid;
    // stronger bounds of the frontier search (expand_kernel):
    //  * bnd2 (sym != 0, symmetric matrices only): per city x the pair
    //    {b[x], e[x]} = half the sum of its two cheapest incident edges and
    //    half its cheapest one (2^-20 grid / integer, rounded down), so a path
    //    from j over R to 0 costs at least e[j] + sum_R b + e[0];
    //  * hsuf (hs_len > 0): the suffix table H[U][x] = cheapest path from x
    //    over the inner-city set U to city 0, for |U| <= hs_len (f64, any
    //    rounding: it is only compared with the incumbent's 2^-39 margin);
    //    size hs_len only, at hs_off[hs_len] + colex_rank(U) * hs_len +
    //    (place of x in U).
    const void *bnd2;
    int sym;
    //  * mst (symmetric matrices, may be null): the Held-Karp (1-tree)
    //    city weights pi and d'[x][y] = d[x][y] + pi_x + pi_y, as doubles:
    //    mst[0 .. n*n) = d', mst[n*n .. n*n+n) = pi, mst[n*n+n] = a margin for
    //    the rounding of the device's sums.  A path from k over R to 0 costs
    //    at least MST'(R) + min_{x in R} d'[k][x] + min_{y in R} d'[y][0]
    //    - pi_k - pi_0 - 2 sum_R pi (expand_kernel: the tree bound).
    const double *mst;
    int mst_min_rem;  // the tree bound only for paths with at least this many cities left
    const double *hsuf;
    int hs_len;
    uint32_t hs_off[8];
    // device tie rule (TieSlot below; null: records only)
    struct TieSlot *tie;
    uint32_t tie_mask;         // slots - 1 (power of two)
    unsigned int *tie_overflow;
    // chained searches: the prologue's block 0 stores the device wall clock
    // (wall_clock64) here at its start, the fetch kernel its own beside it, so
    // the chain is timed without events (an event costs ~5 us of the GPU's
    // timeline between two launches); null: not stored
    unsigned long long *t_start;
    hipStream_t stream;
};

// ---------------------------------------------------------------------------
// Device tie rule.  tsp() returns, among the optimal tours, the one its
// backward argmin chain picks (tsp.cpp:457-470 first strict minimum over the
// members ascending, tsp.cpp:484-499 the same at the closing step).  Every
// tour that chain can pick has all its prefix folds minimal ("DP-consistent"),
// and among those it is the least in reverse-lexicographic order (t_N first,
// then t_(N-1), ...).  The kernels therefore keep, per recorded cost, the
// reverse-lex least tour offered at that cost — a two-level MIN: the slot of
// the cost (claimed by CAS), then the key (atomicMin); a two-word key's second
// word goes to a sub-slot of its first word (CAS, then atomicMin).  The host certifies the
// winner of the optimum's slot as DP-consistent (exact for integer costs; for
// f64 a per-step rounding test, search_host.cpp tie_certify) and otherwise
// falls back to the record set.
//
// Key: digit p (p = 0..N-1) = rank of t_(N-p) among the cities not placed
// yet, radix N - p; for N <= 20 all digits fit one word (N! < 2^64), else
// digits 0..12 go to w0 and 13..N-1 to w1 (31!/18! and 18! < 2^64).
constexpr int kTieSub = 8;  // second-word sub-slots per cost slot
struct TieSlot {
    unsigned long long cost;  // kTieEmpty: free
    unsigned long long w0;    // least first word offered at this cost
    // (two-word keys) per first word that was ever the least at this cost:
    // sub[i][0] = that w0 (claimed by CAS), sub[i][1] = the least w1 offered with it
    unsigned long long sub[kTieSub][2];
};
constexpr unsigned long long kTieEmpty = ~0ull;  // (never a cost: f64 NaN bits / > any u32 cost)
constexpr int kTieSplit = 13;  // digits in w0 when N > 20
constexpr uint32_t kTieSlots = 1024;
constexpr int kTieProbe = 32;

__host__ __device__ constexpr int tie_split(int N) { return N <= 20 ? N : kTieSplit; }

// the key of the tour t_1..t_N, city(i) = t_i
template <typename F>
__device__ __forceinline__ void tie_key(int N, F city, unsigned long long &w0, unsigned long long &w1)
{
    const int split = tie_split(N);
    uint32_t unused = (uint32_t)(((1ull << N) - 1ull) << 1);  // cities 1..N
    w0 = 0;
    w1 = 0;
    for (int p = 0; p < N; ++p) {
        const int c = city(N - p);
        const unsigned long long dig = (unsigned long long)__builtin_popcount(unused & ((1u << c) - 1u));
        unused &= ~(1u << c);
        if (p < split)
            w0 = w0 * (unsigned long long)(N - p) + dig;
        else
            w1 = w1 * (unsigned long long)(N - p) + dig;
    }
}

// Per-lane filter of repeated offers at one cost: the last slot minimum seen.
struct TieCache {
    unsigned long long cost = kTieEmpty, w0 = kTieEmpty;
};

// Offer a recorded tour (cost bits tb, tb <= the incumbent when it was found).
template <typename F>
__device__ __forceinline__ void tie_offer(const SearchArgs &a, TieCache &tc, unsigned long long tb, F city)
{
    if (!a.tie) return;
    const int N = a.n - 1;
    unsigned long long w0, w1;
    tie_key(N, city, w0, w1);
    const bool two = N > 20;
    if (tb == tc.cost && (two ? w0 > tc.w0 : w0 >= tc.w0)) return;  // a better key holds this slot already
    const uint32_t h = (uint32_t)((tb ^ (tb >> 31)) * 0x9E3779B97F4A7C15ull >> 40);
    TieSlot *e = nullptr;
    for (int i = 0; i < kTieProbe; ++i) {
        TieSlot *s = a.tie + ((h + (uint32_t)i) & a.tie_mask);
        const unsigned long long old = atomicCAS(&s->cost, kTieEmpty, tb);
        if (old == kTieEmpty || old == tb) {
            e = s;
            break;
        }
    }
    if (!e) {
        atomicOr(a.tie_overflow, 1u);
        return;
    }
    tc.cost = tb;
    if (!two) {  // (the old key is not waited for: the cache keeps our own, an upper bound of the slot's)
        atomicMin(&e->w0, w0);
        tc.w0 = w0;
        return;
    }
    const unsigned long long o0 = atomicMin(&e->w0, w0);
    tc.w0 = o0 < w0 ? o0 : w0;
    if (w0 > o0) return;
    // second word: the sub-slot of this w0 (lock-free: CAS claim, atomicMin)
    for (int i = 0; i < kTieSub; ++i) {
        const unsigned long long old = atomicCAS(&e->sub[i][0], kTieEmpty, w0);
        if (old == kTieEmpty || old == w0) {
            atomicMin(&e->sub[i][1], w1);
            return;
        }
    }
    atomicOr(a.tie_overflow, 1u);
}

constexpr int kStatLines = 64, kStatStride = 16;
__device__ __forceinline__ unsigned long long *stat_line(const SearchArgs &a)
{
    return a.nodes + (blockIdx.x & (kStatLines - 1)) * kStatStride;
}

size_t search_lds_bytes(int n, bool f64, int kernel = 2);
hipError_t launch_seed(const SearchArgs &a, bool f64, int grid);
hipError_t launch_round(const SearchArgs &a, bool f64, int grid);
// exhaustive enumeration (enum.hip), 7 <= n <= 16: a.items = depth-(n-7) prefixes
hipError_t launch_enum(const SearchArgs &a, bool f64, int grid);
// frontier search (enum.hip): one level of a.in -> a.out / a.tail_out, and
// the register tails of a.tail_out (a.tail_len in {5, 6})
hipError_t launch_to_paths(const SearchArgs &a);  // a.in (seeds) -> a.fout
hipError_t launch_expand(const SearchArgs &a, bool f64);
hipError_t launch_tail(const SearchArgs &a, bool f64, int grid);
hipError_t launch_persist(const SearchArgs &a, bool f64, int grid);
// the tie slot of *cost (null: of the incumbent) -> out[0..4] (search.hip
// tie_lookup_kernel): found, w0, the sub-slot's (w0, w1), overflow
hipError_t launch_tie_lookup(const SearchArgs &a, unsigned long long *out, const unsigned long long *cost = nullptr);
// statistics sums, counter words, tie slot and the first records -> pinned
// host memory in one launch (search.hip fetch_kernel; layout there)
hipError_t launch_fetch(const SearchArgs &a, const unsigned long long *words, unsigned long long *out,
                        uint32_t spec_cap);
constexpr int kFetchWords = 32;  // fetch_kernel's words before the records
// search_create's device state in ONE launch (search.hip init_kernel): the
// host tables copied from pinned host memory (read by the kernel directly),
// the tie table filled with 0xFF, its trailing words and the statistics
// lines zeroed — instead of a dozen memsets and copies of a few KB each
struct SearchInit {
    const uint32_t *src[8];
    uint32_t *dst[8];
    uint32_t words[8];  // 4-byte words per copy
    int ncopy;
    uint32_t *fill_ff;  // 0xFF words (the tie slots)
    uint32_t n_ff;
    uint32_t *zero[2];  // zero words (tie words, statistics)
    uint32_t n_zero[2];
    // the incumbent words (counter words 1 and 14; the copies above leave them
    // out): block 0 stores inc_init there or, with heur_n > 0, the smaller of
    // it and the device heuristic's tour cost (search.hip init_heuristic)
    unsigned long long *inc_word[2];
    unsigned long long inc_init;  // f64 bits or a non-negative int32 cost
    const void *heur_dist;        // heur_n x heur_n, f64 or i32 (host staging, read by the kernel)
    int heur_n;                   // 0: no device heuristic; else 4 <= heur_n <= kSearchMaxN
    int heur_f64;
    int heur_sym;                 // the matrix is symmetric (2-opt deltas are then exact)
    int heur_starts;              // start cities, spread over 0..n-1 (at most 16)
    int heur_iters;               // 2-opt moves at most per start (0: nearest neighbour only)
};
hipError_t launch_init(const SearchInit &init, hipStream_t stream);
// suffix table (enum.hip): size a.hs_len of a.hsuf, one thread per set
hipError_t launch_suffix(const SearchArgs &a, bool f64, uint32_t sets);
// seeds (seed_grid blocks) and the suffix table in one launch (enum.hip)
hipError_t launch_prologue(const SearchArgs &a, bool f64, int seed_grid, uint32_t sets);
// the same with the chain's first level fused into the seed blocks (children to a.fout / a.out_count)
hipError_t launch_prologue1(const SearchArgs &a, bool f64, int seed_grid, uint32_t sets);
// colex rank helpers shared by host and device: C(n, k) for n < 32, k <= 7
__host__ __device__ constexpr uint32_t search_binom(int nn, int k)
{
    if (k < 0 || k > nn) return 0;
    uint64_t r = 1;
    for (int i = 1; i <= k; ++i) r = r * (uint64_t)(nn - k + i) / (uint64_t)i;
    return (uint32_t)r;
}
// the same values as a compile-time table (kernels stage it into LDS: no
// 64-bit divisions on the device)
struct SearchBinom {
    uint32_t v[32][8];
};
constexpr SearchBinom make_search_binom()
{
    SearchBinom t{};
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 8; ++k) t.v[i][k] = search_binom(i, k);
    return t;
}
__device__ __forceinline__ void stage_search_binom(uint32_t (*bn)[8], int tid, int nthreads)
{
    constexpr SearchBinom kT = make_search_binom();
    for (int i = tid; i < 32 * 8; i += nthreads) bn[i >> 3][i & 7] = kT.v[i >> 3][i & 7];
}

}  // namespace tspgpu
