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
    uint32_t fin_per_block;    // expand_kernel: paths per block (multiple of 256)
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
    hipStream_t stream;
};

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
// suffix table (enum.hip): size a.hs_len of a.hsuf, one thread per set
hipError_t launch_suffix(const SearchArgs &a, bool f64, uint32_t sets);
// seeds (seed_grid blocks) and the suffix table in one launch (enum.hip)
hipError_t launch_prologue(const SearchArgs &a, bool f64, int seed_grid, uint32_t sets);
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
