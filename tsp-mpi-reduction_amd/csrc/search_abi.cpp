// C-ABI of K2 (include/tspgpu.h, "K2"): one instance searched by the
// prefix-parallel kernel (search.hip), optionally as one shard of several
// GPUs, plus the host steps around it: the initial bound (a 2-opt tour), the
// cheapest-incoming-edge bound table, and the selection of tsp()'s own tour
// from the set O of optimal tours the search records.
//
// Why the selection reproduces the reference exactly:
// tsp() returns the tour it reaches by backtracking from the closing min,
// each step taking the SMALLEST predecessor m with G[S\k][m] + d[m][k] ==
// G[S][k] (tsp.cpp:457-470, 483-499; K1 does the same on the device).  Let
// F_j(tau) be the left fold of tau up to its j-th city.  Rounding is monotone,
// so (i) a DP-optimal path to a state extended by the suffix of an optimal
// tour is again an optimal tour, hence (ii) G[S_j][t_j] = min F_j over the
// tours of O that share the suffix (t_j..t_N), and (iii) a predecessor m
// satisfies the DP test iff some tour of O ends in (m, t_j..t_N) and
// fl(min F_{j-1} over those + d[m][t_j]) == G[S_j][t_j].  So walking j = N..1
// over O with that test picks the same cities as the DP, including when a
// non-DP-optimal prefix is absorbed by rounding into the optimal cost.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"
#include <cstdio>

#include "search.h"
#include "search_host.h"
#include "tspgpu.h"
#include "tuning.h"

using namespace tspgpu;
using tspgpu::host::held_karp_pi;
using tspgpu::host::lagrange_pi;
using tspgpu::host::validate_search;
using tspgpu::tuned;
using tspgpu::tuned_int;
using tspgpu::tuned_or;

static_assert(sizeof(SearchRecord) == sizeof(tspgpu_tour_record), "record layout");
constexpr int kWords = 16;  // device counter words of a search (see tspgpu_search::d_words)
constexpr size_t kStatBytes = sizeof(unsigned long long) * kStatLines * kStatStride;
constexpr size_t kStageSpec = 24 * 1024;  // h_stage: tables below, speculative records above
constexpr unsigned kSpecRecs = 512;
constexpr size_t kStageBytes = kStageSpec + 8 * kFetchWords + sizeof(SearchRecord) * kSpecRecs;

struct tspgpu_search {
    tspgpu_ctx *ctx = nullptr;
    int n = 0;
    int dtype = TSPGPU_F64;
    int depth = 0;
    uint64_t items = 0;        // global prefixes
    uint64_t local_items = 0;  // prefixes of this shard
    uint32_t shard = 0, nshards = 1;
    int grid = 0;
    std::vector<double> hd;    // host copy (f64 view) for the selection
    std::vector<int32_t> hi;
    void *d_dist = nullptr, *d_amin = nullptr;
    // [0] queue (u32), [1] incumbent, [2] nodes, [3] record count (u32), [4] items out / seed
    // count (u32), [5..7] utilisation counters, [8] tail items (u32), [9] odd frontier steps'
    // child count (u32), [10..12] chained level counters (u32, in rotation), [13] chained
    // overflow flag (u32), [14] the incumbent a chain started from (its rerun restores it),
    // [15] a chain's start: the device wall clock (SearchArgs::t_start)
    unsigned long long *d_words = nullptr;
    unsigned long long *d_stats = nullptr;  // kStatLines x kStatStride: [0] nodes, [1..3] lane-step counters
    SearchRecord *d_rec = nullptr;
    unsigned int rec_cap = 0;    // records the kernels may write
    unsigned int rec_alloc = 0;  // records d_rec holds
    SearchItem *d_items[2] = {nullptr, nullptr};  // round input / output (ping-pong)
    size_t item_cap[2] = {0, 0};
    int cur = 0;                 // d_items[cur] holds the pending items
    uint64_t pending = 0;        // items waiting for the next round
    uint32_t budget = 256;       // DFS iterations per item per round
    uint32_t refill = 16;        // v2/persistent: refill a wave once this many lanes wait
    // round kernel (knob SEARCH_KERNEL): 2 lock-step DFS (default), 1 branching DFS;
    // 3 = run_all as ONE persistent launch with a device work ring (measured
    // 1.3-2x slower than rounds at n = 18: profiles/r01/k2_persistent.log)
    int kernel = 2;
    // persistent search
    PersistState *d_ps = nullptr;
    unsigned long long *d_ring = nullptr;
    uint32_t ring_cap = 1u << 20;
    int32_t hungry = 0;
    uint32_t min_split = 64;
    double wall_s = 300.0;
    int noprune = 0;             // exhaustive enumeration (tspgpu_search_enumerate)
    int enum_kernel = 0;         // enumeration by enum.hip (6-city register tails, 7 <= n <= 16)
    // Frontier search (default for the bounded search when n - 1 - tail_len >
    // the seed depth; knob SEARCH_TAIL = 0 selects the DFS rounds, 5 or 6 the
    // tail length): each step expands up to kExpandMax items of the frontier
    // (LIFO) by one level with the bound; prefixes with tail_len cities left
    // collect in d_tail and are folded by tail_kernel, all tail_len!
    // completions in registers, once tail_cap / 2 of them wait or the
    // frontier is empty.
    int tail_len = 6;
    bool frontier = false;
    bool chain = true;  // run_all: small searches as chained levels (knob SEARCH_CHAIN=0: step by step)
    // stronger frontier bounds (SearchArgs::bnd2 / ::hsuf): the two-edge bound
    // for symmetric matrices and the suffix table for the last tail_len cities
    int sym = 0;
    void *d_bnd2 = nullptr;
    double *d_mst = nullptr;
    double *d_hsuf = nullptr;
    size_t hsuf_alloc = 0;      // bytes
    int hs_len = 0;             // sizes 1..hs_len built (0: none)
    uint32_t hs_off[8] = {};
    int suffix_len = 6;         // knob SEARCH_SUFFIX=0/5/6: table size (0: B0/B1 only)
    bool use_two_edge = true;   // knob SEARCH_TWO_EDGE=0: no B1
    bool use_lagrange = true;   // knob SEARCH_LAGRANGE=0: B1 without the Lagrangian city weights
    bool use_mst = true;        // knob SEARCH_MST=0: no Held-Karp tree bound in the expand kernel
    bool mst_on = false;        // (symmetric matrices only)
    int mst_min_rem = 12;       // knob SEARCH_MST_MINREM: paths with fewer cities left skip it (measured: profiles/r02/k2_tree_minrem.log)
    // The frontier is a LIFO stack of segments, each a run of paths in its own
    // buffer (fb): a step expands the top T items of the top segment and its
    // children become a new segment on top, written straight into a spare
    // buffer (no device copy of the children behind the items left below:
    // those copies were 11 ms of a 61 ms 30-city search).
    std::vector<PathItem *> fb;       // frontier buffers (kept in the context's pool between searches)
    std::vector<size_t> fb_cap;
    std::vector<int> seg_buf;         // buffer index of each segment, bottom first
    std::vector<uint64_t> seg_n;      // paths in each segment
    PathItem *d_tail = nullptr;
    // one frontier step expands at most min(expand_max, free tail slots / branch)
    // items; bigger steps mean fewer host round trips (n = 30 random, seed 2:
    // 2^23 tails / 2^21 items 2903 steps, 192 ms; 2^26 / 2^24 373 steps, 58 ms;
    // profiles/r02/k2_knobs.log).  Buffers grow on demand.
    unsigned int tail_cap = 1u << 26;
    unsigned int tail_alloc = 0;
    // 2^21: the output buffer of a step holds T x branch paths, and a step's
    // children can become a segment of their own: at 2^24 a cold 32-city
    // search spent 1.3 s in hipMalloc (1714 vs 524 ms warm), at 2^21 564 vs
    // 545 ms (profiles/r02/k2_expand_cap.log)
    uint64_t expand_max = (uint64_t)1 << 21;
    uint64_t expand_steps = 0;  // frontier expansions so far (parity of the double-buffered child counter)  // frontier items one step expands, at most (knob SEARCH_EXPAND_LOG2)
    uint64_t tails = 0;          // items waiting in d_tail
    int rounds = 0;
    double ms = 0.0;             // device time of all seed/round launches
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    unsigned long long *h_cnt = nullptr;  // pinned host words: the frontier step's counter readback
    // pinned host copy of the statistics lines + 8 counter words (one DMA
    // pair and one synchronisation per counters read)
    unsigned long long *h_stats = nullptr;
    // device tie rule (search.h): kTieSlots slots, then 8 words: [0..4] the
    // optimum's slot (tie_lookup_kernel), [5] the overflow flag
    TieSlot *d_tie = nullptr;
    bool tie_on = true;  // knob SEARCH_TIE=0: records and the host rule only
    // pinned staging: the host tables of create (so their copies need no
    // synchronisation) and, at kStageSpec, the speculative records readback
    char *h_stage = nullptr;
    // search_solve: the chained run enqueues the solve's readbacks (counters,
    // statistics, records, tie slot) before its one synchronisation
    bool fetch = false, fetched = false;
    // the fetch buffer still reflects the device state (a finished chain and
    // nothing run or written since): counters, tie slot and records read from it
    bool fresh = false;
    // straight from create's init launch: the counter words 0, 4 and 8..13 are
    // zero, so the first start / chain skips its memsets of them
    bool pristine = false;
    bool inc_shared = false;  // tspgpu_search_incumbent_device handed word 1 out
    bool stamp = false;       // the next prologue stores the chain's start clock in word 15
    int dev_heur = 0;  // create's init launch computed the initial bound on the device (its n)
};

namespace {

int herr(hipError_t e)
{
    if (e == hipSuccess) return 0;
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    return -EIO;
}

uint64_t falling(int N, int D)
{
    uint64_t p = 1;
    for (int l = 0; l < D; ++l) p *= (uint64_t)(N - l);
    return p;
}

}  // namespace

// Device buffers a context keeps between searches (hipMalloc of the tail
// and frontier buffers cost more than a 16-city search itself).  One set per
// context: the next search takes it, its destroy gives it back.
namespace {
struct SearchPool {
    void *d_dist = nullptr, *d_amin = nullptr;
    unsigned long long *d_words = nullptr, *d_stats = nullptr;
    SearchRecord *d_rec = nullptr;
    unsigned int rec_alloc = 0;
    SearchItem *d_items[2] = {nullptr, nullptr};
    size_t item_cap[2] = {0, 0};
    std::vector<PathItem *> fb;
    std::vector<size_t> fb_cap;
    PathItem *d_tail = nullptr;
    unsigned int tail_alloc = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    unsigned long long *h_cnt = nullptr;
    unsigned long long *h_stats = nullptr;
    void *d_bnd2 = nullptr;
    double *d_mst = nullptr;
    double *d_hsuf = nullptr;
    size_t hsuf_alloc = 0;
    TieSlot *d_tie = nullptr;
    char *h_stage = nullptr;
};

template <typename A, typename B>
void move_buffers(A &to, B &from)
{
    to.d_dist = from.d_dist, from.d_dist = nullptr;
    to.d_amin = from.d_amin, from.d_amin = nullptr;
    to.d_words = from.d_words, from.d_words = nullptr;
    to.d_stats = from.d_stats, from.d_stats = nullptr;
    to.d_rec = from.d_rec, from.d_rec = nullptr;
    to.rec_alloc = from.rec_alloc, from.rec_alloc = 0;
    for (int i = 0; i < 2; ++i) {
        to.d_items[i] = from.d_items[i], from.d_items[i] = nullptr;
        to.item_cap[i] = from.item_cap[i], from.item_cap[i] = 0;
    }
    for (PathItem *p : to.fb)  // (never non-empty at the call sites; freed rather than leaked)
        if (p) (void)hipFree(p);
    to.fb = std::move(from.fb);
    to.fb_cap = std::move(from.fb_cap);
    from.fb.clear();
    from.fb_cap.clear();
    to.d_tail = from.d_tail, from.d_tail = nullptr;
    to.tail_alloc = from.tail_alloc, from.tail_alloc = 0;
    to.e0 = from.e0, from.e0 = nullptr;
    to.e1 = from.e1, from.e1 = nullptr;
    to.e2 = from.e2, from.e2 = nullptr;
    to.h_cnt = from.h_cnt, from.h_cnt = nullptr;
    to.h_stats = from.h_stats, from.h_stats = nullptr;
    to.d_bnd2 = from.d_bnd2, from.d_bnd2 = nullptr;
    to.d_mst = from.d_mst, from.d_mst = nullptr;
    to.d_hsuf = from.d_hsuf, from.d_hsuf = nullptr;
    to.hsuf_alloc = from.hsuf_alloc, from.hsuf_alloc = 0;
    to.d_tie = from.d_tie, from.d_tie = nullptr;
    to.h_stage = from.h_stage, from.h_stage = nullptr;
}

template <typename A>
void free_buffers(A &b)
{
    if (b.d_dist) (void)hipFree(b.d_dist);
    if (b.d_amin) (void)hipFree(b.d_amin);
    if (b.d_words) (void)hipFree(b.d_words);
    if (b.d_stats) (void)hipFree(b.d_stats);
    if (b.d_rec) (void)hipFree(b.d_rec);
    for (int i = 0; i < 2; ++i) {
        if (b.d_items[i]) (void)hipFree(b.d_items[i]);
    }
    for (PathItem *p : b.fb)
        if (p) (void)hipFree(p);
    b.fb.clear();
    b.fb_cap.clear();
    if (b.d_tail) (void)hipFree(b.d_tail);
    if (b.e0) (void)hipEventDestroy(b.e0);
    if (b.e1) (void)hipEventDestroy(b.e1);
    if (b.e2) (void)hipEventDestroy(b.e2);
    if (b.h_cnt) (void)hipHostFree(b.h_cnt);
    if (b.h_stats) (void)hipHostFree(b.h_stats);
    if (b.d_bnd2) (void)hipFree(b.d_bnd2);
    if (b.d_mst) (void)hipFree(b.d_mst);
    if (b.d_hsuf) (void)hipFree(b.d_hsuf);
    if (b.d_tie) (void)hipFree(b.d_tie);
    if (b.h_stage) (void)hipHostFree(b.h_stage);
    SearchPool z;
    move_buffers(b, z);
}

void pool_free(void *p)
{
    auto *pool = static_cast<SearchPool *>(p);
    free_buffers(*pool);
    delete pool;
}

void take_pool(tspgpu_search *s)
{
    SearchPool *pool = nullptr;
    {
        std::lock_guard<std::mutex> g(s->ctx->mu);
        pool = static_cast<SearchPool *>(s->ctx->search_pool);
        s->ctx->search_pool = nullptr;
    }
    if (!pool) return;
    move_buffers(*s, *pool);
    delete pool;
}

void give_pool(tspgpu_search *s)
{
    if (s->d_words == nullptr) return;  // a failed create: nothing worth keeping
    auto *pool = new (std::nothrow) SearchPool();
    if (!pool) return;
    move_buffers(*pool, *s);
    std::lock_guard<std::mutex> g(s->ctx->mu);
    if (!s->ctx->search_pool) {
        s->ctx->search_pool = pool;
        s->ctx->search_pool_free = pool_free;
        pool = nullptr;
    }
    if (pool) move_buffers(*s, *pool), delete pool;  // the context has one already: free ours
}
}  // namespace

static void front_release(tspgpu_search *s);

extern "C" {

// (bound: the initial incumbent, written with the counter words; null: none)
// (dev_bound: the init launch computes the bound on the device, search.hip
// init_heuristic; s->dev_heur says whether it did)
static int search_create(tspgpu_ctx *c, const void *dist, int dtype, int n, int shard, int nshards, int depth,
                         const double *bound, tspgpu_search **out, bool dev_bound = false)
{
    if (!c || !out) return -EINVAL;
    *out = nullptr;
    int rc = validate_search(dist, dtype, n);
    if (rc) return rc;
    if (nshards < 1 || shard < 0 || shard >= nshards) return -EINVAL;
    const int N = n - 1;
    const bool f64 = dtype == TSPGPU_F64;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    auto *s = new (std::nothrow) tspgpu_search();
    if (!s) return -ENOMEM;
    {
        // the search's reference on its context (ctx.h "Lifetime"); dropped by
        // tspgpu_search_destroy, also on the failure path below
        std::lock_guard<std::mutex> g(c->mu);
        if (c->closing) {
            delete s;
            return -EINVAL;
        }
        ++c->live_searches;
    }
    s->ctx = c;
    s->n = n;
    s->dtype = dtype;
    s->shard = (uint32_t)shard;
    s->nshards = (uint32_t)nshards;
    // tuning knobs (tuning.h; tests and A/B runs only, the defaults above are the product)
    double kv = 0.0;
    if (tuned("SEARCH_KERNEL", &kv)) s->kernel = (int)kv == 1 ? 1 : ((int)kv == 3 ? 3 : 2);
    if (tuned("SEARCH_HUNGRY", &kv)) s->hungry = (int32_t)kv;
    if (tuned("SEARCH_MIN_SPLIT", &kv)) s->min_split = (uint32_t)std::max(0.0, kv);
    if (tuned("SEARCH_WALL_S", &kv)) s->wall_s = std::max(0.1, kv);
    if (tuned("SEARCH_RING_LOG2", &kv) && kv >= 6 && kv <= 24) s->ring_cap = 1u << (int)kv;  // tests: a small ring
    if (tuned("SEARCH_REFILL", &kv) && kv > 0) s->refill = (uint32_t)std::min(kv, 64.0);
    if (tuned("SEARCH_TAIL", &kv)) s->tail_len = ((int)kv == 5 || (int)kv == 6) ? (int)kv : 0;
    if (tuned("SEARCH_SUFFIX", &kv)) s->suffix_len = ((int)kv == 5 || (int)kv == 6) ? (int)kv : 0;
    if (tuned("SEARCH_TWO_EDGE", &kv)) s->use_two_edge = kv != 0;
    if (tuned("SEARCH_CHAIN", &kv)) s->chain = kv != 0;
    if (tuned("SEARCH_LAGRANGE", &kv)) s->use_lagrange = kv != 0;
    if (tuned("SEARCH_MST", &kv)) s->use_mst = kv != 0;
    if (tuned("SEARCH_MST_MINREM", &kv)) s->mst_min_rem = (int)kv;
    if (tuned("SEARCH_TAIL_CAP_LOG2", &kv) && kv >= 8 && kv <= 27) s->tail_cap = 1u << (int)kv;  // tests: many flushes
    if (tuned("SEARCH_EXPAND_LOG2", &kv) && kv >= 8 && kv <= 26) s->expand_max = (uint64_t)1 << (int)kv;
    const size_t lds = search_lds_bytes(n, f64, s->kernel == 1 ? 1 : 2);
    const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / lds)));
    s->grid = c->cu_count * per_cu;
    // seed depth: the smallest D with at least one prefix per lane of the
    // whole grid (the rounds split whatever is still too coarse), at most
    // N-1, at least 1, and < 2^31 prefixes
    const uint64_t lanes = (uint64_t)s->grid * kSearchThreads * (uint64_t)nshards;
    const bool auto_depth = depth <= 0;
    if (depth <= 0) {
        depth = 1;
        while (depth < N - 1 && falling(N, depth + 1) < (1ull << 31) && falling(N, depth) < lanes) ++depth;
    }
    if (depth > N - 1) depth = N - 1;
    while (depth > 1 && falling(N, depth) >= (1ull << 31)) --depth;
    if (tuned("SEARCH_BUDGET", &kv) && kv > 0) s->budget = (uint32_t)kv;
    s->frontier = s->tail_len && s->kernel == 2 && N - s->tail_len > depth;
    // the frontier search expands level by level with its own bounds: a
    // smaller seed set (~64 prefixes per CU) costs less than the round
    // kernels' one-per-lane (measured at n = 16: depth 4 vs 5, 0.14 vs 0.16 ms)
    if (s->frontier && auto_depth) {
        const uint64_t want = (uint64_t)c->cu_count * 64 * nshards;
        int d = 1;
        while (d < depth && falling(N, d) < want) ++d;
        // several shards: one level deeper, so that the heavy subtrees near
        // the optimum spread over the shards (n = 30 random, 8 shards: node
        // imbalance max/mean 1.91 at depth 4, 1.20 at depth 5;
        // profiles/r02/k2_shard_balance_depth.log)
        // Not with the tree bound (symmetric matrices): it leaves no heavy
        // subtree to spread, and the deeper seed level, bounded only by B0/B1,
        // costs more than it balances (n = 32 seed 35, 2 shards: 5.0e7 nodes
        // per shard vs 7.1e5 for one GPU; profiles/r02/k2_shard_depth_tree.log)
        bool tree = s->use_mst && s->use_two_edge;
        for (int i = 0; i < n && tree; ++i)
            for (int j = 0; j < i && tree; ++j)
                tree = f64 ? static_cast<const double *>(dist)[i * n + j] == static_cast<const double *>(dist)[j * n + i]
                           : static_cast<const int32_t *>(dist)[i * n + j] == static_cast<const int32_t *>(dist)[j * n + i];
        if (nshards > 1 && !tree && d + 1 < N - s->tail_len && falling(N, d + 1) < (1ull << 31)) ++d;
        depth = d;
    }
    s->depth = depth;
    s->items = falling(N, depth);
    s->local_items = s->items / nshards + (s->items % nshards > (uint64_t)shard ? 1 : 0);
    const size_t vb = f64 ? sizeof(double) : sizeof(int32_t);
    // cheapest incoming edge per city; f64 rounded DOWN to a 2^-20 grid
    std::vector<double> ad(n);
    std::vector<int32_t> ai(n);
    if (f64) {
        const double *d = static_cast<const double *>(dist);
        s->hd.assign(d, d + n * n);
        for (int x = 0; x < n; ++x) {
            double m = INFINITY;
            for (int i = 0; i < n; ++i)
                if (i != x) m = std::min(m, d[i * n + x]);
            ad[x] = std::ldexp(std::floor(std::ldexp(m, 20)), -20);
        }
    } else {
        const int32_t *d = static_cast<const int32_t *>(dist);
        s->hi.assign(d, d + n * n);
        for (int x = 0; x < n; ++x) {
            int32_t m = INT32_MAX;
            for (int i = 0; i < n; ++i)
                if (i != x) m = std::min(m, d[i * n + x]);
            ai[x] = m;
        }
    }
    // two-edge bound (symmetric matrices): per city x, b[x] = half the sum of
    // its two cheapest incident edges, e[x] = half its cheapest, rounded down
    // to the bound's grid (f64: 2^-20, exact sums; i32: integers)
    std::vector<double> bd(2 * n, 0.0);
    std::vector<int32_t> bi(2 * n, 0);
    std::vector<double> hk_pi;  // Held-Karp weights of the tree bound (symmetric matrices)
    {
        bool sym = s->use_two_edge;
        for (int i = 0; i < n && sym; ++i)
            for (int j = 0; j < i && sym; ++j)
                sym = f64 ? static_cast<const double *>(dist)[i * n + j] == static_cast<const double *>(dist)[j * n + i]
                          : static_cast<const int32_t *>(dist)[i * n + j] == static_cast<const int32_t *>(dist)[j * n + i];
        s->sym = sym ? 1 : 0;
        if (sym) {
            std::vector<double> D((size_t)n * n);
            for (int i = 0; i < n * n; ++i)
                D[i] = f64 ? static_cast<const double *>(dist)[i] : (double)static_cast<const int32_t *>(dist)[i];
            std::vector<double> pi(n, 0.0);
            // the tree bound's weights on a second thread meanwhile (host time
            // at n = 32: 1.3 ms beside lagrange_pi's 0.45 ms)
            // (only if some path can reach it: the expand kernel applies the
            // tree bound to paths with >= mst_min_rem cities left, and the
            // frontier starts at the seed depth — at n = 16 none does, and
            // the weights cost 0.22 ms of host time, profiles/r03/k2_variants.log)
            const bool want_tree = s->use_mst && n >= 4 && s->frontier && N - depth >= s->mst_min_rem;
            std::thread ht;
            bool threaded = false;
            if (want_tree && n >= 20) {  // (smaller: a thread costs more than it saves)
                try {
                    ht = std::thread([&] { held_karp_pi(D, n, hk_pi); });
                    threaded = true;
                } catch (...) {
                }
            }
            if (s->use_lagrange) lagrange_pi(D, n, pi);
            if (threaded)
                ht.join();
            else if (want_tree)
                held_karp_pi(D, n, hk_pi);
            for (int x = 0; x < n; ++x) {
                double m1 = INFINITY, m2 = INFINITY;  // the two cheapest d'[x][y] = d + pi_x + pi_y
                for (int y = 0; y < n; ++y) {
                    if (y == x) continue;
                    const double v = D[(size_t)x * n + y] + pi[x] + pi[y];
                    if (v < m1) {
                        m2 = m1;
                        m1 = v;
                    } else if (v < m2) {
                        m2 = v;
                    }
                }
                // b = (m1 + m2)/2 - 2 pi_x, e = m1/2 - pi_x: lower bounds, so
                // a margin for the double rounding of d + pi + pi, then DOWN
                // to the grid
                const double bx = (m1 + m2) * 0.5 - 2.0 * pi[x], ex = m1 * 0.5 - pi[x];
                const double mg = 1e-9 * (std::fabs(m1) + std::fabs(m2) + 4.0 * std::fabs(pi[x]) + 1.0);
                if (f64) {
                    bd[2 * x] = std::ldexp(std::floor(std::ldexp(bx - mg, 20)), -20);
                    bd[2 * x + 1] = std::ldexp(std::floor(std::ldexp(ex - mg, 20)), -20);
                } else {
                    bi[2 * x] = (int32_t)std::floor(bx - mg);
                    bi[2 * x + 1] = (int32_t)std::floor(ex - mg);
                }
            }
        }
    }
    // tree bound (symmetric matrices): d' and pi as doubles, and a margin far
    // above the rounding of the device's sums of <= 2n + 2 such terms
    std::vector<double> mt;
    s->mst_on = s->sym && s->use_mst && !s->noprune && n >= 4 && (int)hk_pi.size() == n;
    if (s->mst_on) {
        std::vector<double> D((size_t)n * n);
        const std::vector<double> &pi = hk_pi;
        for (int i = 0; i < n * n; ++i)
            D[i] = f64 ? static_cast<const double *>(dist)[i] : (double)static_cast<const int32_t *>(dist)[i];
        mt.assign((size_t)n * n + n + 1, 0.0);
        double mx = 0.0, ps = 0.0;
        for (int x = 0; x < n; ++x)
            for (int y = 0; y < n; ++y) {
                mt[(size_t)x * n + y] = D[(size_t)x * n + y] + pi[x] + pi[y];
                mx = std::max(mx, std::fabs(mt[(size_t)x * n + y]));
            }
        for (int x = 0; x < n; ++x) mt[(size_t)n * n + x] = pi[x], ps += std::fabs(pi[x]);
        mt[(size_t)n * n + n] = 1e-9 * ((n + 2) * mx + 2.0 * ps + 1.0);
    }
    s->rec_cap = 1u << 16;
    take_pool(s);  // device buffers of the context's previous search, if any
    hipStream_t st = c->stream;
    hipError_t e = hipSuccess;
    if (!s->d_dist) e = hipMalloc(&s->d_dist, sizeof(double) * kSearchMaxN * kSearchMaxN);
    if (e == hipSuccess && !s->d_amin) e = hipMalloc(&s->d_amin, sizeof(double) * kSearchMaxN);
    if (e == hipSuccess && !s->d_bnd2) e = hipMalloc(&s->d_bnd2, sizeof(double) * 2 * kSearchMaxN);
    if (e == hipSuccess && s->mst_on && !s->d_mst)
        e = hipMalloc((void **)&s->d_mst, sizeof(double) * (kSearchMaxN * kSearchMaxN + kSearchMaxN + 1));
    if (e == hipSuccess && !s->d_words) e = hipMalloc((void **)&s->d_words, kWords * sizeof(unsigned long long));
    if (e == hipSuccess && !s->d_stats) e = hipMalloc((void **)&s->d_stats, kStatBytes);
    if (e == hipSuccess && s->frontier && s->d_tail && s->tail_alloc != s->tail_cap) {
        (void)hipFree(s->d_tail);
        s->d_tail = nullptr;
    }
    if (e == hipSuccess && s->frontier && !s->d_tail) {
        e = hipMalloc((void **)&s->d_tail, sizeof(PathItem) * s->tail_cap);
        if (e == hipSuccess) s->tail_alloc = s->tail_cap;
    }
    if (e == hipSuccess && s->rec_alloc < s->rec_cap) {
        if (s->d_rec) (void)hipFree(s->d_rec);
        s->d_rec = nullptr;
        e = hipMalloc((void **)&s->d_rec, sizeof(SearchRecord) * s->rec_cap);
        if (e == hipSuccess) s->rec_alloc = s->rec_cap;
    }
    if (double v; tuned("SEARCH_TIE", &v)) s->tie_on = v != 0;
    constexpr size_t kTieBytes = sizeof(TieSlot) * kTieSlots;
    if (e == hipSuccess && !s->d_tie) e = hipMalloc((void **)&s->d_tie, kTieBytes + 8 * sizeof(unsigned long long));
    const bool pinned = tuned_or("SEARCH_PAGEABLE", 0) == 0;
    if (e == hipSuccess && pinned && !s->h_cnt)
        e = hipHostMalloc((void **)&s->h_cnt, 16 * sizeof(unsigned long long), hipHostMallocDefault);
    if (e == hipSuccess && pinned && !s->h_stats)
        e = hipHostMalloc((void **)&s->h_stats, kStatBytes + 8 * sizeof(unsigned long long), hipHostMallocDefault);
    if (e == hipSuccess && pinned && !s->h_stage) e = hipHostMalloc((void **)&s->h_stage, kStageBytes, hipHostMallocDefault);
    unsigned long long w[kWords] = {};
    if (f64) {
        const double inf = INFINITY;
        std::memcpy(&w[1], bound ? bound : &inf, 8);
    } else {
        w[1] = bound ? (unsigned long long)std::min<double>(*bound, (double)INT32_MAX) : (unsigned long long)INT32_MAX;
    }
    w[14] = w[1];  // the incumbent a chain starts from (run_chain copies it only after a run)
    // the host tables and the counter words, with the sizes
    struct Part {
        void *dst;
        const void *src;
        size_t bytes;
    };
    Part parts[5];
    int np = 0;
    parts[np++] = {s->d_dist, dist, vb * n * n};
    parts[np++] = {s->d_amin, f64 ? (const void *)ad.data() : (const void *)ai.data(), vb * n};
    if (s->sym) parts[np++] = {s->d_bnd2, f64 ? (const void *)bd.data() : (const void *)bi.data(), vb * 2 * n};
    if (s->mst_on) parts[np++] = {s->d_mst, mt.data(), sizeof(double) * mt.size()};
    parts[np++] = {s->d_words, w, sizeof w};
    size_t need = 0;
    for (int i = 0; i < np; ++i) need += (parts[i].bytes + 15) & ~(size_t)15;
    if (e == hipSuccess && s->h_stage && need <= kStageSpec) {
        // ONE launch: the tables staged in pinned host memory, read by the
        // kernel directly (no copy commands), the tie slots filled and the
        // statistics zeroed beside them (a dozen memsets and copies took
        // ~70 us of the 16-city search's timeline, profiles/r04)
        // (the counter words without 1 and 14, the incumbent: block 0 stores those)
        Part ip[8];
        int ni = 0;
        for (int i = 0; i + 1 < np; ++i) ip[ni++] = parts[i];
        ip[ni++] = {s->d_words, w, 8};
        ip[ni++] = {s->d_words + 2, w + 2, 12 * 8};
        ip[ni++] = {s->d_words + 15, w + 15, 8};
        SearchInit in{};
        size_t soff = 0;
        for (int i = 0; i < ni; ++i) {
            std::memcpy(s->h_stage + soff, ip[i].src, ip[i].bytes);
            in.src[i] = reinterpret_cast<const uint32_t *>(s->h_stage + soff);
            in.dst[i] = static_cast<uint32_t *>(ip[i].dst);
            in.words[i] = (uint32_t)(ip[i].bytes / 4);
            soff += (ip[i].bytes + 15) & ~(size_t)15;
        }
        in.ncopy = ni;
        in.inc_word[0] = s->d_words + 1;
        in.inc_word[1] = s->d_words + 14;
        in.inc_init = w[1];
        if (dev_bound && n >= 4 && n <= kSearchMaxN) {
            bool msym = true;
            for (int i = 0; i < n && msym; ++i)
                for (int j = 0; j < i && msym; ++j)
                    msym = f64 ? static_cast<const double *>(dist)[i * n + j] == static_cast<const double *>(dist)[j * n + i]
                               : static_cast<const int32_t *>(dist)[i * n + j] == static_cast<const int32_t *>(dist)[j * n + i];
            in.heur_dist = in.src[0];  // (the distances, staged first)
            in.heur_n = n;
            in.heur_f64 = f64 ? 1 : 0;
            in.heur_sym = msym ? 1 : 0;
            // four spread starts, as the host's (search_host.cpp heuristic): at
            // 14/16/19 cities the same bound and nodes as 8 or 16 starts, and
            // each wave has a SIMD to itself (profiles/r04/k2_device_bound.log);
            // from 20 cities sixteen (the host multi-start takes ~2 ms there)
            in.heur_starts = n >= 20 ? 16 : 4;
            in.heur_iters = tuned_int("SEARCH_HEUR_ITERS", 8 * n);
        }
        in.fill_ff = reinterpret_cast<uint32_t *>(s->d_tie);
        in.n_ff = (uint32_t)(kTieBytes / 4);
        in.zero[0] = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(s->d_tie) + kTieBytes);
        in.n_zero[0] = 16;
        in.zero[1] = reinterpret_cast<uint32_t *>(s->d_stats);
        in.n_zero[1] = (uint32_t)(kStatBytes / 4);
        e = launch_init(in, st);
        s->pristine = e == hipSuccess;  // (words 0, 4, 8..13 are zero: the first run skips its memsets)
        s->dev_heur = e == hipSuccess ? in.heur_n : 0;
    } else if (e == hipSuccess) {
        // pageable staging (knob SEARCH_PAGEABLE): memsets, copies and a synchronisation
        e = hipMemsetAsync(s->d_tie, 0xFF, kTieBytes, st);
        if (e == hipSuccess)
            e = hipMemsetAsync(reinterpret_cast<char *>(s->d_tie) + kTieBytes, 0, 8 * sizeof(unsigned long long), st);
        if (e == hipSuccess) e = hipMemsetAsync(s->d_stats, 0, kStatBytes, st);
        for (int i = 0; i < np && e == hipSuccess; ++i)
            e = hipMemcpyAsync(parts[i].dst, parts[i].src, parts[i].bytes, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    if (e == hipSuccess && !s->e0) e = hipEventCreate(&s->e0);
    if (e == hipSuccess && !s->e1) e = hipEventCreate(&s->e1);
    if (e == hipSuccess && !s->e2) e = hipEventCreate(&s->e2);
    if (e != hipSuccess) {
        tspgpu_search_destroy(s);
        return herr(e);
    }
    *out = s;
    return 0;
}

int tspgpu_search_create(tspgpu_ctx *c, const void *dist, int dtype, int n, int shard, int nshards, int depth,
                         tspgpu_search **out)
{
    return search_create(c, dist, dtype, n, shard, nshards, depth, nullptr, out);
}

int tspgpu_search_create_ex(tspgpu_ctx *c, const void *dist, int dtype, int n, int shard, int nshards, int depth,
                            int flags, tspgpu_search **out)
{
    if (flags & ~TSPGPU_SEARCH_DEVICE_BOUND) return -EINVAL;
    const bool dev = (flags & TSPGPU_SEARCH_DEVICE_BOUND) != 0;
    int rc = search_create(c, dist, dtype, n, shard, nshards, depth, nullptr, out, dev);
    if (rc || !dev || (*out)->dev_heur) return rc;
    // (pageable staging knob: no create launch, so the host's bound)
    double ub = 0.0;
    rc = tspgpu_heuristic_tour(dist, dtype, n, &ub, nullptr);
    if (!rc) rc = tspgpu_search_set_bound(*out, ub);
    if (rc) {
        tspgpu_search_destroy(*out);
        *out = nullptr;
    }
    return rc;
}

int tspgpu_search_destroy(tspgpu_search *s)
{
    if (!s) return 0;
    (void)hipSetDevice(s->ctx->device);
    (void)hipStreamSynchronize(s->ctx->stream);
    front_release(s);
    give_pool(s);  // the buffers stay with the context for its next search
    free_buffers(*s);
    if (s->d_ps) (void)hipFree(s->d_ps);
    if (s->d_ring) (void)hipFree(s->d_ring);
    tspgpu_ctx *c = s->ctx;
    delete s;
    // dropping the reference is the last use of the context: when
    // tspgpu_ctx_destroy came first, the last search releases it (with the
    // pool just given back)
    bool last = false;
    {
        std::lock_guard<std::mutex> g(c->mu);
        last = --c->live_searches == 0 && c->closing;
    }
    if (last) tspgpu_ctx_release(c);
    return 0;
}

int tspgpu_search_info(const tspgpu_search *s, int *depth, uint64_t *items, uint64_t *local_items)
{
    if (!s) return -EINVAL;
    if (depth) *depth = s->depth;
    if (items) *items = s->items;
    if (local_items) *local_items = s->local_items;
    return 0;
}

int tspgpu_search_set_bound(tspgpu_search *s, double bound)
{
    if (!s) return -EINVAL;
    s->fresh = false;
    unsigned long long w;
    if (s->dtype == TSPGPU_F64) {
        if (!(bound >= 0.0)) return -EINVAL;
        std::memcpy(&w, &bound, 8);
    } else {
        if (!(bound >= 0.0)) return -EINVAL;
        w = (unsigned long long)std::min<double>(bound, (double)INT32_MAX);
    }
    (void)hipSetDevice(s->ctx->device);
    // on the search's stream: ordered after create's (asynchronous) counter words
    hipError_t e = hipMemcpyAsync(s->d_words + 1, &w, 8, hipMemcpyHostToDevice, s->ctx->stream);
    if (e == hipSuccess)  // word 14: a chain's starting incumbent (read by its overflow rerun)
        e = hipMemcpyAsync(s->d_words + 14, &w, 8, hipMemcpyHostToDevice, s->ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->ctx->stream);
    return herr(e);
}

static unsigned long long *tie_words(tspgpu_search *s)
{
    return reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(s->d_tie) + sizeof(TieSlot) * kTieSlots);
}

static SearchArgs args_of(tspgpu_search *s)
{
    SearchArgs a{};
    a.dist = s->d_dist;
    a.amin = s->d_amin;
    a.n = s->n;
    a.depth = s->depth;
    a.items = (uint32_t)s->items;
    a.shard = s->shard;
    a.nshards = s->nshards;
    a.budget = s->budget;
    a.refill = s->refill;
    a.kernel = s->kernel == 1 && !s->noprune ? 1 : 2;  // the round kernels (2 for enumeration)
    a.noprune = s->noprune;
    a.tails = s->noprune;  // knob SEARCH_TAILS=0/1 overrides
    if (double v; tuned("SEARCH_TAILS", &v)) a.tails = v != 0;
    a.queue = reinterpret_cast<unsigned int *>(s->d_words);
    a.inc = s->d_words + 1;
    a.nodes = s->d_stats;
    a.rec_count = reinterpret_cast<unsigned int *>(s->d_words + 3);
    a.out_count = reinterpret_cast<unsigned int *>(s->d_words + 4);
    a.tail_count = reinterpret_cast<unsigned int *>(s->d_words + 8);
    if (s->frontier) {
        a.tail_len = s->tail_len;
        a.tail_level = s->n - 1 - s->tail_len;
        a.ftail = s->d_tail;
        a.tail_cap = s->tail_cap;
    }
    a.rec = s->d_rec;
    a.rec_cap = s->rec_cap;
    a.bnd2 = s->d_bnd2;
    a.sym = s->sym;
    a.mst = s->mst_on ? s->d_mst : nullptr;
    a.mst_min_rem = s->mst_min_rem;
    a.hsuf = s->d_hsuf;
    a.hs_len = s->hs_len;
    for (int i = 0; i < 8; ++i) a.hs_off[i] = s->hs_off[i];
    if (s->tie_on) {
        a.tie = s->d_tie;
        a.tie_mask = kTieSlots - 1;
        a.tie_overflow = reinterpret_cast<unsigned int *>(tie_words(s) + 5);
    }
    a.t_start = s->stamp ? s->d_words + 15 : nullptr;
    a.stream = s->ctx->stream;
    return a;
}

// the device wall clock's rate (wall_clock64 ticks per ms), per device
static double wall_clock_khz(int device)
{
    static std::mutex mu;
    static std::map<int, double> rate;
    std::lock_guard<std::mutex> g(mu);
    auto it = rate.find(device);
    if (it != rate.end()) return it->second;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
        khz = 100000;  // (gfx9: 100 MHz)
    rate[device] = (double)khz;
    return (double)khz;
}

static int ensure_items(tspgpu_search *s, int which, size_t count)
{
    if (s->item_cap[which] >= count && s->d_items[which]) return 0;
    // grow geometrically (up to 2^27 items) so that rounds rarely reallocate
    const size_t cap = std::max<size_t>(std::max<size_t>(count, 1024),
                                        std::min<size_t>(2 * s->item_cap[which], (size_t)1 << 27));
    if (s->d_items[which]) (void)hipFree(s->d_items[which]);
    s->d_items[which] = nullptr;
    s->item_cap[which] = 0;
    hipError_t e = hipMalloc((void **)&s->d_items[which], cap * sizeof(SearchItem));
    if (e != hipSuccess) return herr(e);
    s->item_cap[which] = cap;
    return 0;
}

// the statistics lines, summed: [0] nodes, [1] lane slots, [2] active lane steps, [3] item loads
// The counter words [0..4] and the summed statistics lines in one
// synchronisation (both copies into the pinned h_stats when it exists).
static int read_words_stats(tspgpu_search *s, unsigned long long (&w)[5], uint64_t (&out)[4])
{
    std::vector<unsigned long long> tmp;
    unsigned long long *h = s->h_stats;
    if (!h) {
        tmp.resize(kStatLines * kStatStride + 8);
        h = tmp.data();
    }
    unsigned long long *hw = h + kStatLines * kStatStride;
    hipError_t e = hipMemcpyAsync(h, s->d_stats, kStatBytes, hipMemcpyDeviceToHost, s->ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(hw, s->d_words, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->ctx->stream);
    if (e != hipSuccess) return herr(e);
    for (int i = 0; i < 4; ++i) {
        out[i] = 0;
        for (int l = 0; l < kStatLines; ++l) out[i] += h[l * kStatStride + i];
    }
    for (int i = 0; i < 5; ++i) w[i] = hw[i];
    return 0;
}

// A frontier buffer that no segment uses, holding at least `count` paths:
// the smallest spare one that is big enough, else a new allocation (rounded up
// to 2^20 paths); buffers are only freed when the search ends.
// -> index into s->fb, or < 0 (*rc set).
static int front_spare(tspgpu_search *s, size_t count, int *rc)
{
    int best = -1;
    for (int i = 0; i < (int)s->fb.size(); ++i) {
        bool used = false;
        for (int b : s->seg_buf) used = used || b == i;
        if (used || !s->fb[i] || s->fb_cap[i] < count) continue;
        if (best < 0 || s->fb_cap[i] < s->fb_cap[best]) best = i;
    }
    if (best >= 0) return best;
    const size_t gran = (size_t)1 << 20;
    const size_t cap = std::max<size_t>(4096, count <= 4096 ? 4096 : (count + gran - 1) / gran * gran);
    PathItem *p = nullptr;
    hipError_t e = hipMalloc((void **)&p, cap * sizeof(PathItem));
    if (e != hipSuccess) {
        *rc = herr(e);
        return -1;
    }
    s->fb.push_back(p);
    s->fb_cap.push_back(cap);
    return (int)s->fb.size() - 1;
}

// the search ends: its segments go, its frontier buffers stay for the pool
static void front_release(tspgpu_search *s)
{
    s->seg_buf.clear();
    s->seg_n.clear();
}

// launch + wait + read the item count the launch produced (sync = false: the
// count stays in word 4 for a chained search to read on the device; the
// launch's time is then the chain's)
static int launch_and_count(tspgpu_search *s, bool seed, int grid, SearchArgs &a, uint32_t suffix_sets = 0,
                            bool sync = true)
{
    hipStream_t st = s->ctx->stream;
    hipError_t e = hipSuccess;
    if (!s->pristine) {
        e = hipMemsetAsync(s->d_words, 0, 8, st);  // queue
        if (e == hipSuccess) e = hipMemsetAsync(s->d_words + 4, 0, 8, st);  // items out
    }
    s->pristine = false;
    if (e != hipSuccess) return herr(e);
    if (sync) (void)hipEventRecord(s->e0, st);  // (a chain times itself: SearchArgs::t_start)
    if (seed && suffix_sets)  // the frontier's seeds and its suffix table, side by side in one launch
        e = launch_prologue(a, s->dtype == TSPGPU_F64, grid, suffix_sets);
    else
        e = seed ? launch_seed(a, s->dtype == TSPGPU_F64, grid) : launch_round(a, s->dtype == TSPGPU_F64, grid);
    if (sync) (void)hipEventRecord(s->e1, st);
    if (e != hipSuccess) return herr(e);
    if (!sync) return 0;
    unsigned long long out = 0;
    e = hipMemcpyAsync(&out, s->d_words + 4, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
    s->pending = (uint32_t)out;
    return 0;
}

// The suffix table of the frontier search (sizes 1..tail_len, one launch
// each, device time counted in the search's kernel time): built once per
// search, when the bounded frontier search will use it.
static int build_suffix(tspgpu_search *s, bool launch, uint32_t *sets_out)
{
    s->hs_len = 0;
    *sets_out = 0;
    // the frontier's expansion tests children with tail_len cities left: the
    // table has that size there; the lock-step DFS tests at suffix_len
    const int N = s->n - 1, L = s->frontier ? s->tail_len : s->suffix_len;
    if (s->noprune || s->suffix_len == 0 || L < 1 || N < L + 2 || s->kernel == 1 || s->kernel == 3) return 0;
    for (int k = 0; k < 8; ++k) s->hs_off[k] = 0;  // one size stored: L, at offset 0
    const uint32_t sets = search_binom(N, L), off = sets * (uint32_t)L;
    const size_t bytes = (size_t)off * sizeof(double);
    hipStream_t st = s->ctx->stream;
    if (s->hsuf_alloc < bytes) {
        if (s->d_hsuf) (void)hipFree(s->d_hsuf);
        s->d_hsuf = nullptr;
        s->hsuf_alloc = 0;
        hipError_t e = hipMalloc((void **)&s->d_hsuf, bytes);
        if (e != hipSuccess) return herr(e);
        s->hsuf_alloc = bytes;
    }
    s->hs_len = L;
    *sets_out = sets;
    if (!launch) return 0;  // the caller launches it (with the seeds)
    SearchArgs a = args_of(s);
    (void)hipEventRecord(s->e0, st);
    if (hipError_t e = launch_suffix(a, s->dtype == TSPGPU_F64, sets); e != hipSuccess) return herr(e);
    (void)hipEventRecord(s->e1, st);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
    return 0;
}

static int search_start(tspgpu_search *s, bool sync);
int tspgpu_search_start(tspgpu_search *s) { return s ? search_start(s, true) : -EINVAL; }

// sync = false (chained searches): the seeds' launch is only enqueued, their
// count stays on the device (word 4), s->pending is the upper bound
// local_items and the seed segment is left to the caller
static int search_start(tspgpu_search *s, bool sync)
{
    (void)hipSetDevice(s->ctx->device);
    s->fresh = false;
    if (int rc = ensure_items(s, 0, s->local_items + 1)) return rc;
    SearchArgs a = args_of(s);
    a.out = s->d_items[0];
    s->cur = 0;
    s->rounds = 0;
    s->tails = 0;
    if (s->frontier) {  // tails (word 8) and the odd steps' child counter (word 9)
        hipError_t e = s->pristine ? hipSuccess : hipMemsetAsync(s->d_words + 8, 0, 16, s->ctx->stream);
        if (e != hipSuccess) return herr(e);
        s->expand_steps = 0;
    }
    uint32_t sets = 0;  // the frontier builds its suffix table in the seed launch
    if (int rc = build_suffix(s, !s->frontier, &sets)) return rc;
    a = args_of(s);
    a.out = s->d_items[0];
    int seed_buf = -1;
    if (s->frontier) {  // the live seeds are written as the first frontier segment (32-byte paths)
        s->seg_buf.clear();
        s->seg_n.clear();
        int rc = 0;
        seed_buf = front_spare(s, (size_t)s->local_items + 1, &rc);
        if (seed_buf < 0) return rc;
        a.fout = s->fb[seed_buf];
    }
    const uint64_t blocks = (s->local_items + kSearchThreads - 1) / kSearchThreads;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)s->ctx->cu_count * 8));
    int rc = launch_and_count(s, true, grid, a, s->frontier ? sets : 0u, sync);
    if (!rc && !sync) {
        s->pending = s->local_items;
        s->seg_buf.push_back(seed_buf);
        s->seg_n.push_back(0);
        return 0;
    }
    if (!rc && s->frontier && s->pending) {
        s->seg_buf.push_back(seed_buf);
        s->seg_n.push_back(s->pending);
    }
    return rc;
}

// Chained searches of at least two levels: the seeds and the first level in
// one launch (launch_prologue1): the seed segment is allocated as in
// search_start (unused), then the chain's two level buffers ob[0..1]; the
// first level's children go to ob[0] and their count to word 11 (the word the
// chain's level 1 reads).
static bool fusable(const tspgpu_search *s)
{
    // build_suffix's conditions for a frontier table, and a size prologue1 has
    const int N = s->n - 1, L = s->tail_len;
    return s->frontier && !s->noprune && s->suffix_len != 0 && (L == 5 || L == 6) && N >= L + 2 && s->kernel != 1 &&
           s->kernel != 3;
}
static int search_start_fused(tspgpu_search *s, uint64_t cap, int ob[2])
{
    (void)hipSetDevice(s->ctx->device);
    s->fresh = false;
    if (int rc = ensure_items(s, 0, s->local_items + 1)) return rc;
    s->cur = 0;
    s->rounds = 0;
    s->tails = 0;
    hipStream_t st = s->ctx->stream;
    hipError_t e = s->pristine ? hipSuccess : hipMemsetAsync(s->d_words + 8, 0, 16, st);
    if (e != hipSuccess) return herr(e);
    s->expand_steps = 0;
    uint32_t sets = 0;
    if (int rc = build_suffix(s, false, &sets)) return rc;
    if (!sets) return -EIO;  // (run_chain fuses only when the table is built: fusable())
    s->seg_buf.clear();
    s->seg_n.clear();
    int rc = 0;
    const int seed_buf = front_spare(s, (size_t)s->local_items + 1, &rc);
    if (seed_buf < 0) return rc;
    s->seg_buf.push_back(seed_buf);
    s->seg_n.push_back(0);
    for (int k = 0; k < 2; ++k) {
        ob[k] = front_spare(s, (size_t)cap, &rc);
        if (ob[k] < 0) return rc;
        s->seg_buf.push_back(ob[k]);  // (marked used so the second front_spare picks another)
        s->seg_n.push_back(0);
    }
    if (tuned_or("SEARCH_CHAIN_POISON", 0) != 0) {  // tests: no slot may be read that was not written
        for (int k = 0; k < 2 && e == hipSuccess; ++k)
            e = hipMemsetAsync(s->fb[ob[k]], 0xFF, sizeof(PathItem) * cap, st);
        if (e == hipSuccess) e = hipMemsetAsync(s->d_tail, 0xFF, sizeof(PathItem) * s->tail_cap, st);
    }
    if (!s->pristine && e == hipSuccess) {
        e = hipMemsetAsync(s->d_words, 0, 8, st);  // queue
        if (e == hipSuccess) e = hipMemsetAsync(s->d_words + 4, 0, 8, st);  // items out
    }
    s->pristine = false;
    if (e != hipSuccess) return herr(e);
    SearchArgs a = args_of(s);
    a.fout = s->fb[ob[0]];
    a.fout_cap = (uint32_t)cap;
    a.out_count = reinterpret_cast<unsigned int *>(s->d_words + 11);
    a.overflow = reinterpret_cast<unsigned int *>(s->d_words + 13);
    const uint64_t blocks = (s->local_items + kSearchThreads - 1) / kSearchThreads;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)s->ctx->cu_count * 8));
    e = launch_prologue1(a, s->dtype == TSPGPU_F64, grid, sets);
    if (e != hipSuccess) return herr(e);
    s->pending = s->local_items;
    return 0;
}

// Frontier search, one step: either fold the waiting tails, or expand the
// last T frontier items (LIFO keeps the frontier small) by one level.
static int frontier_step(tspgpu_search *s, uint64_t *pending)
{
    (void)hipSetDevice(s->ctx->device);
    hipStream_t st = s->ctx->stream;
    const bool f64 = s->dtype == TSPGPU_F64;
    const uint64_t branch = (uint64_t)(s->n - 1 - s->depth);  // children per item, at most
    SearchArgs a = args_of(s);
    hipError_t e = hipSuccess;
    if (s->pending == 0 || s->tails >= s->tail_cap / 2) {
        if (s->tails) {
            (void)hipEventRecord(s->e0, st);
            // a wave folds 64 tails at a time: no more blocks than that needs
            const uint64_t tb = (s->tails + 255) / 256;
            e = launch_tail(a, f64, (int)std::max<uint64_t>(1, std::min<uint64_t>(tb, (uint64_t)s->ctx->cu_count * 8)));
            (void)hipEventRecord(s->e1, st);
            if (e == hipSuccess) e = hipMemsetAsync(s->d_words + 8, 0, 8, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return herr(e);
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
            s->tails = 0;
            ++s->rounds;
        }
        if (pending) *pending = s->pending;
        return 0;
    }
    // the step's input: the top `want` paths of the stack, over at most four segments
    const uint64_t want = std::min<uint64_t>({s->pending, s->expand_max, (s->tail_cap - s->tails) / branch});
    uint64_t T = 0, take[4] = {};
    int used = 0;
    for (int k = (int)s->seg_n.size() - 1; k >= 0 && T < want && used < 4; --k, ++used) {
        const uint64_t c = std::min<uint64_t>(s->seg_n[k], want - T);
        a.fseg[used] = s->fb[s->seg_buf[k]] + (s->seg_n[k] - c);
        a.fseg_start[used] = (uint32_t)T;
        take[used] = c;
        T += c;
    }
    a.nseg = used;
    int rc = 0;
    const int ob = front_spare(s, (size_t)(T * branch + 64), &rc);
    if (ob < 0) return rc;
    a.fin = a.fseg[0];
    a.fin_count = (uint32_t)T;
    // a few blocks per CU, each over a contiguous run (one slot atomic per block and output)
    // (at most 1024 paths per block: expand_kernel keeps their live masks in registers)
    const uint64_t blocks = std::max<uint64_t>(
        (T + 1023) / 1024, std::max<uint64_t>(1, std::min<uint64_t>((T + 255) / 256, (uint64_t)s->ctx->cu_count * 4)));
    a.fin_per_block = (uint32_t)(((T + blocks - 1) / blocks + 255) / 256 * 256);
    a.fout = s->fb[ob];
    // children counted in word 9 or 4 by step parity; the kernel zeroes the
    // other one for the next step (word 9 is zeroed when the frontier starts,
    // word 4 still holds the seed count then)
    const int cw = (s->expand_steps & 1) ? 4 : 9;
    a.out_count = reinterpret_cast<unsigned int *>(s->d_words + cw);
    a.out_next = reinterpret_cast<unsigned int *>(s->d_words + (13 - cw));
    (void)hipEventRecord(s->e0, st);
    e = launch_expand(a, f64);
    (void)hipEventRecord(s->e1, st);
    // words 4..9: children (even steps), ..., tails (8), children (odd steps);
    // read into pinned host memory (a direct DMA, no staging copy)
    unsigned long long local[6] = {};
    unsigned long long *cnt = s->h_cnt ? s->h_cnt : local;
    if (e == hipSuccess) e = hipMemcpyAsync(cnt, s->d_words + 4, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
    ++s->rounds;
    ++s->expand_steps;
    const uint64_t kids = (uint32_t)cnt[cw - 4];
    s->tails = (uint32_t)cnt[4];
    // the expanded paths leave the top segments (all but the deepest one used
    // are now empty); their children go on top: appended to the top segment
    // when few (a small copy), as a segment of their own (no copy) when many
    for (int u = 0; u < used; ++u) s->seg_n[s->seg_n.size() - 1 - u] -= take[u];
    while (!s->seg_n.empty() && s->seg_n.back() == 0) {
        s->seg_buf.pop_back();
        s->seg_n.pop_back();
    }
    constexpr uint64_t kAppendMax = (uint64_t)1 << 20;
    if (kids && !s->seg_n.empty() && kids <= kAppendMax && s->fb_cap[s->seg_buf.back()] >= s->seg_n.back() + kids) {
        e = hipMemcpyAsync(s->fb[s->seg_buf.back()] + s->seg_n.back(), s->fb[ob], kids * sizeof(PathItem),
                           hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return herr(e);
        s->seg_n.back() += kids;  // stream-ordered before the next step's launch
    } else if (kids) {
        s->seg_buf.push_back(ob);
        s->seg_n.push_back(kids);
    }
    s->pending = s->pending - T + kids;
    if (pending) *pending = s->pending + s->tails;
    return 0;
}

int tspgpu_search_step(tspgpu_search *s, uint64_t *pending)
{
    if (!s) return -EINVAL;
    s->fresh = false;
    if (s->frontier) return frontier_step(s, pending);
    if (s->pending == 0) {
        if (pending) *pending = 0;
        return 0;
    }
    (void)hipSetDevice(s->ctx->device);
    const int in = s->cur, out = 1 - s->cur;
    // A round takes at most kMaxRound input items; every item hands back at
    // most one item per level of its stack (N-1), so the output always has
    // room for them plus the inputs carried over to the next round.
    constexpr uint64_t kMaxRound = (uint64_t)1 << 22;
    const uint64_t take = std::min<uint64_t>(s->pending, kMaxRound);
    const uint64_t carry = s->pending - take;
    int rc = ensure_items(s, out, (size_t)(take * (uint64_t)(s->n - 1) + carry + 64));
    if (rc) return rc;
    SearchArgs a = args_of(s);
    a.in = s->d_items[in];
    a.in_count = (uint32_t)take;
    a.out = s->d_items[out];
    const uint64_t blocks = (take + kSearchThreads - 1) / kSearchThreads;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)s->grid));
    rc = launch_and_count(s, false, grid, a);
    if (rc) return rc;
    if (carry) {  // inputs this round did not take: behind the spilled items
        hipError_t e = hipMemcpyAsync(s->d_items[out] + s->pending, s->d_items[in] + take, carry * sizeof(SearchItem),
                                      hipMemcpyDeviceToDevice, s->ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->ctx->stream);
        if (e != hipSuccess) return herr(e);
        s->pending += carry;
    }
    s->cur = out;
    ++s->rounds;
    if (pending) *pending = s->pending;
    return 0;
}

// Small searches, chained (one shard, n <= kChainMaxN): after the seeds, every
// frontier level is enqueued back to back — each expand launch reads its input
// count from the counter the previous level wrote (three counter words in
// rotation: read one, write the next, zero the third), loops a fixed grid
// over its input runs and writes its children into one of two ping-pong
// buffers of kChainCap paths — then the tail fold, and ONE synchronisation.
// No host round trip per level (the stepwise search pays ~30 us each: 0.2 of
// the 16-city search's 0.45 ms, profiles/r03/k2_variants.log).  A level whose
// children or tails would not fit sets an overflow word (13); every later
// chained kernel then returns at once (the slots an overflowing block
// reserved were never written and are not read), and the search reruns step
// by step from the chain's starting state: records, tails, tie slots and
// statistics reset, the incumbent restored from word 14.  Breadth first
// instead of the stepwise LIFO: the same bounds, the same optimal set, a
// different node count.
// search_solve's readbacks, enqueued behind the search: one kernel writes
// the statistics, counter words, tie slot and first records straight into
// the pinned h_stage + kStageSpec (fetch_kernel's layout)
static unsigned long long *fetch_buf(tspgpu_search *s)
{
    return reinterpret_cast<unsigned long long *>(s->h_stage + kStageSpec);
}
static hipError_t enqueue_fetch(tspgpu_search *s)
{
    SearchArgs a = args_of(s);
    return launch_fetch(a, s->d_words, fetch_buf(s), std::min(kSpecRecs, s->rec_cap));
}

// (up to 32 cities: at 20-32 cities the chained search takes 0.70-1.73 ms in
// process against 0.95-2.8 ms step by step, same nodes and answers,
// profiles/r03/k2_chain_maxn.log)
constexpr int kChainMaxN = 32;
// The tie certificate's prefix DP on the GPU (K1-wide): G[{t1..tj}][tj] is
// the closing min of the sub-instance over the cities 0, t1..tj whose closing
// edges are 0 from tj and BIG from every other city (BIG above any path:
// the min is G + 0, exact).  Up to kTieGpuMax cities (K1-wide's table: 1 GB
// at 26 cities, 2.4 ms); host Held-Karp below kTieHostMax (it grows as
// j^2 2^j: 0.6 M steps at 12 cities, 17 M at 16).
constexpr int kTieGpuMax = 26, kTieHostMax = 12;
static int gpu_prefix(void *user, const double *d, int n, const int32_t *t, int j, double *g)
{
    const int m = j + 1;
    if (m < 3 || m > kTieGpuMax) return -ERANGE;
    double mx = 0.0;
    for (int i = 0; i < n * n; ++i) mx = std::max(mx, d[i]);
    const double big = mx * (m + 1) + 1.0;
    if ((double)m * big >= (double)INT_MAX) return -ERANGE;
    std::vector<double> sub((size_t)m * m);
    auto city = [&](int a) { return a == 0 ? 0 : t[a]; };
    for (int a = 0; a < m; ++a)
        for (int b = 0; b < m; ++b)
            sub[(size_t)a * m + b] = a == b ? 0.0 : (b == 0 ? (a == j ? 0.0 : big) : d[city(a) * n + city(b)]);
    std::vector<int32_t> tour(m + 1);
    return tspgpu_solve_instance(static_cast<tspgpu_ctx *>(user), sub.data(), m, g, tour.data(), nullptr);
}

int tspgpu_tie_tour_gpu(tspgpu_ctx *ctx, const void *dist, int dtype, int n, uint64_t w0, uint64_t w1,
                        uint64_t cost_bits, int32_t *tour_out)
{
    if (!ctx) return -EINVAL;
    return tspgpu::host::tie_tour(dist, dtype, n, w0, w1, cost_bits, tour_out, true, gpu_prefix, ctx, kTieHostMax);
}

int tspgpu_tie_tour_records(tspgpu_ctx *ctx, const void *dist, int dtype, int n, uint64_t w0, uint64_t w1,
                            uint64_t cost_bits, const tspgpu_tour_record *records, int count, int32_t *tour_out)
{
    if (count < 0 || (count > 0 && !records)) return -EINVAL;
    tspgpu::host::RecordsPrefix rp{records, count, cost_bits, ctx ? gpu_prefix : nullptr, ctx};
    // (host_max 0: every prefix check from the records first)
    return tspgpu::host::tie_tour(dist, dtype, n, w0, w1, cost_bits, tour_out, true, tspgpu::host::records_prefix,
                                  &rp, 0);
}

static bool chainable(const tspgpu_search *s)
{
    // above 18 cities only with the tree bound (its frontiers are small; without
    // it a 32-city chain overflows its level buffers and reruns step by step)
    return s->frontier && !s->noprune && s->chain && s->kernel != 3 && s->n <= (s->mst_on ? kChainMaxN : 18);
}

// every `every` levels (0: never) hook(user, stream, incumbent word) enqueues
// an exchange of the incumbent on the search's stream (e.g. an RCCL
// all-reduce MIN): the same number of calls on every shard of one instance
static int run_chain(tspgpu_search *s, bool *done, int every = 0, tspgpu_level_hook hook = nullptr,
                     void *user = nullptr)
{
    *done = false;
    // ping-pong buffer capacity (knob SEARCH_CHAIN_CAP_LOG2: tests force the overflow fallback)
    uint64_t kChainCap = (uint64_t)1 << 22;
    if (double v; tuned("SEARCH_CHAIN_CAP_LOG2", &v) && v >= 8 && v <= 24) kChainCap = (uint64_t)1 << (int)v;
    SearchArgs a0 = args_of(s);
    const int levels = a0.tail_level - s->depth;
    // a run of 256 paths per block (one per lane) and two blocks per CU:
    // the reference's 16-city instance 0.30 -> 0.22 ms in process against
    // 1024-path runs on one block per CU (profiles/r03/k2_chain_sweep.log)
    uint32_t chain_fpb = 256;
    // (at <= 16 cities a level has at most ~160 runs of 256 paths: one block
    // per CU covers them, and the blocks without a run cost VALU for nothing)
    int chain_grid = s->n <= 16 ? 1 : 2;
    chain_fpb = (uint32_t)tuned_int("CHAIN_FPB", (int)chain_fpb);  // (sweeps)
    chain_grid = std::max(1, tuned_int("CHAIN_GRID", chain_grid));
    // the tail's count is only known on the device, so its grid is sized for
    // the buffer and the blocks beyond the count leave at once
    // (<= 16 cities: one block per CU — the waves beyond the count only read
    // it and leave, 4 VALU lane-instructions per node at 8 per CU)
    const int tail_grid = std::max(1, tuned_int("CHAIN_TAIL_GRID", s->n <= 16 ? 1 : 8));
    // the levels expanded block-locally (expand_local_kernel; knob
    // CHAIN_LOCAL), runs of 64 input paths per block
    // (from 20 cities: 7-11% fewer kernel-us at 20-32 cities; at 14-16 cities
    // the per-level launches win, profiles/r04/k2_local_sweep.log)
    const bool chain_local = tuned_or("CHAIN_LOCAL", s->n >= 20 ? 1 : 0) != 0;
    const uint32_t chain_local_fpb = (uint32_t)std::max(1, std::min(256, tuned_int("CHAIN_LOCAL_FPB", 64)));
    hipStream_t st = s->ctx->stream;
    const int hooks = hook && every > 0 && levels > 1 ? (levels - 1) / every : 0;
    // Every return enqueues all `hooks` exchanges, also after a failure
    // halfway (the other shards block in theirs otherwise): the guard
    // enqueues whatever the level loop did not.
    struct HookGuard {
        tspgpu_level_hook hook;
        void *user;
        hipStream_t st;
        void *word;
        int want, done = 0;
        ~HookGuard()
        {
            for (; done < want; ++done) hook(user, st, word);
        }
    } guard{hook, user, st, s->d_words + 1, hooks};
    if (levels < 1 || s->local_items + 1 > kChainCap) return 0;  // (not chained: the guard's exchanges pair up)
    const bool f64 = s->dtype == TSPGPU_F64;
    // words 10..13 zeroed before the seeds (10..12: level counters, 13:
    // overflow); word 14 keeps the incumbent the chain starts from
    // (pristine: create wrote them, word 14 = word 1; set_bound keeps that)
    hipError_t e = s->pristine ? hipSuccess : hipMemsetAsync(s->d_words + 10, 0, 4 * sizeof(unsigned long long), st);
    if (e == hipSuccess && (!s->pristine || s->inc_shared))
        e = hipMemcpyAsync(s->d_words + 14, s->d_words + 1, sizeof(unsigned long long), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return herr(e);
    // timed by the device clock when the fetch carries it (prologue start to
    // fetch start), else by events around the chain
    const bool fetch = s->fetch && s->h_stage;
    if (!fetch) (void)hipEventRecord(s->e2, st);
    s->stamp = fetch;
    // the first level fused into the seeds' launch (knob CHAIN_FUSE_SEEDS, on
    // with per-level launches and >= 2 levels: then no seed's child is a
    // tail; 16 cities: 0.081 -> 0.072 ms, profiles/r06/k2_16/fuse/; a second
    // fused level inside the seed blocks took as long as its own launch)
    const bool fuse = !chain_local && levels >= 2 && fusable(s) && tuned_or("CHAIN_FUSE_SEEDS", 1) != 0;
    int ob[2] = {-1, -1};
    int rc = fuse ? search_start_fused(s, kChainCap, ob) : search_start(s, false);  // (unfused: the seeds' count stays in word 4)
    s->stamp = false;
    if (rc) return rc;
    if (!fuse) {
        for (int k = 0; k < 2; ++k) {
            ob[k] = front_spare(s, (size_t)kChainCap, &rc);
            if (ob[k] < 0) return rc;
            s->seg_buf.push_back(ob[k]);  // (marked used so the second front_spare picks another)
            s->seg_n.push_back(0);
        }
    }
    if (!fuse && tuned_or("SEARCH_CHAIN_POISON", 0) != 0) {  // tests: no slot may be read that was not written
        for (int k = 0; k < 2 && e == hipSuccess; ++k)
            e = hipMemsetAsync(s->fb[ob[k]], 0xFF, sizeof(PathItem) * kChainCap, st);
        if (e == hipSuccess) e = hipMemsetAsync(s->d_tail, 0xFF, sizeof(PathItem) * s->tail_cap, st);
        if (e != hipSuccess) return herr(e);
    }
    // level l reads its input count from word 4 (the seeds, l = 0) or
    // 10 + l%3, writes 10 + (l+1)%3 and zeroes 10 + (l+2)%3
    if (fuse && hooks && 1 % every == 0) {  // (level 0 ran in the seeds' launch)
        hook(user, st, s->d_words + 1);
        ++guard.done;
    }
    for (int l = fuse ? 1 : 0; l < levels && e == hipSuccess; ++l) {
        SearchArgs a = args_of(s);
        a.fseg[0] = l == 0 ? s->fb[s->seg_buf[0]] : s->fb[ob[(l - 1) & 1]];
        a.fseg_start[0] = 0;
        a.nseg = 1;
        a.fin = a.fseg[0];
        a.fin_count = l == 0 ? (uint32_t)s->local_items : (uint32_t)kChainCap;  // (the grid's bound)
        a.fin_count_dev = reinterpret_cast<const unsigned int *>(s->d_words + (l == 0 ? 4 : 10 + l % 3));
        a.fin_cap = (uint32_t)std::min<size_t>(l == 0 ? s->fb_cap[s->seg_buf[0]] : s->fb_cap[ob[(l - 1) & 1]],
                                               UINT32_MAX);
        a.out_count = reinterpret_cast<unsigned int *>(s->d_words + 10 + (l + 1) % 3);
        a.out_next = reinterpret_cast<unsigned int *>(s->d_words + 10 + (l + 2) % 3);
        a.fout = s->fb[ob[l & 1]];
        a.fout_cap = (uint32_t)kChainCap;
        a.overflow = reinterpret_cast<unsigned int *>(s->d_words + 13);
        a.fin_per_block = chain_local ? chain_local_fpb : chain_fpb;
        a.local_levels = chain_local ? levels - l : 0;  // (block-local: every level left, in LDS where it fits)
        a.max_grid = s->ctx->cu_count * chain_grid;  // (blocks beyond the level's runs only stage tables and leave)
        e = launch_expand(a, f64);
        if (e == hipSuccess && hooks && (l + 1) % every == 0 && (l + 1) / every <= hooks) {
            hook(user, st, s->d_words + 1);  // (enqueued between two levels)
            ++guard.done;
        }
    }
    if (e == hipSuccess) {
        SearchArgs a = args_of(s);
        a.overflow = reinterpret_cast<unsigned int *>(s->d_words + 13);  // (an abandoned chain folds no tails)
        e = launch_tail(a, f64, s->ctx->cu_count * tail_grid);
    }
    if (!fetch) (void)hipEventRecord(s->e1, st);
    unsigned long long local[8] = {};
    unsigned long long *h = s->h_cnt ? s->h_cnt : local;
    // (search_solve: its readbacks ride on this synchronisation, words 8..13 among them)
    if (e == hipSuccess && fetch) {
        e = enqueue_fetch(s);
        h = fetch_buf(s) + 4 + 8;
    } else if (e == hipSuccess) {
        e = hipMemcpyAsync(h, s->d_words + 8, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    if (fetch) {  // seeds through the tail fold: device wall clock, prologue start to fetch start
        const unsigned long long *f = fetch_buf(s);
        const unsigned long long t0 = f[4 + 15], t1 = f[25];
        if (t0 != 0 && t1 > t0) s->ms += (double)(t1 - t0) / wall_clock_khz(s->ctx->device);
    } else {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, s->e2, s->e1) == hipSuccess) s->ms += ms;
    }
    s->rounds += levels + 1;
    front_release(s);
    s->pending = 0;
    s->tails = 0;
    if ((uint32_t)h[5] == 0) {  // word 13: no overflow
        *done = true;
        s->fetched = fetch;
        return 0;
    }
    // overflow: the search reruns step by step from the state before the
    // chain — records, tails, tie slots and the incumbent reset.  (A block
    // that overflowed reserved output slots it never wrote; later levels and
    // the tail fold read whatever those slots held before, paths of an
    // earlier search, possibly of more cities: their "tours" must not leave
    // an incumbent, record or tie key behind.)
    e = hipMemsetAsync(s->d_words + 3, 0, 8, st);
    if (e == hipSuccess) e = hipMemsetAsync(s->d_words + 8, 0, 8, st);
    if (e == hipSuccess) e = hipMemsetAsync(s->d_words + 13, 0, 8, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(s->d_words + 1, s->d_words + 14, sizeof(unsigned long long), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && s->d_tie) {
        constexpr size_t kTieBytes = sizeof(TieSlot) * kTieSlots;
        e = hipMemsetAsync(s->d_tie, 0xFF, kTieBytes, st);
        if (e == hipSuccess) e = hipMemsetAsync(tie_words(s), 0, 8 * sizeof(unsigned long long), st);
    }
    if (e == hipSuccess) e = hipMemsetAsync(s->d_stats, 0, kStatBytes, st);
    return herr(e);
}

// The whole search in ONE persistent launch (kernel 3): seeds decoded on the
// fly, work handed between lanes through a device ring, no rounds.
static int run_persist(tspgpu_search *s)
{
    (void)hipSetDevice(s->ctx->device);
    hipStream_t st = s->ctx->stream;
    hipError_t e = hipSuccess;
    if (!s->d_ps) e = hipMalloc((void **)&s->d_ps, sizeof(PersistState));
    if (e == hipSuccess && !s->d_ring)
        e = hipMalloc((void **)&s->d_ring, (size_t)s->ring_cap * kRingWords * sizeof(unsigned long long));
    if (e != hipSuccess) return herr(e);
    const bool f64 = s->dtype == TSPGPU_F64;
    const size_t lds = search_lds_bytes(s->n, f64, 3);
    const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / lds)));
    const int grid = s->ctx->cu_count * per_cu;
    PersistState h{};
    h.work.v = s->local_items;
    int wall_khz = 0;
    if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, s->ctx->device) != hipSuccess || wall_khz <= 0)
        wall_khz = 100000;
    SearchArgs a = args_of(s);
    a.kernel = 3;
    a.ps = s->d_ps;
    a.ring = s->d_ring;
    a.ring_mask = s->ring_cap - 1;
    // every resident wave may reserve up to 64 tickets between two capacity checks
    a.ring_margin = (uint32_t)std::min<uint64_t>((uint64_t)grid * (kSearchThreads / 64) * 64, s->ring_cap / 2);
    a.hungry = s->hungry;
    a.min_split = s->min_split;
    a.wall_limit = (unsigned long long)(s->wall_s * wall_khz * 1000.0);
    // tags of a previous launch would match this launch's tickets: clear the ring
    e = hipMemcpyAsync(s->d_ps, &h, sizeof h, hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemsetAsync(s->d_ring, 0, (size_t)s->ring_cap * kRingWords * sizeof(unsigned long long), st);
    if (e == hipSuccess) e = hipMemsetAsync(s->d_words, 0, 8, st);
    if (e != hipSuccess) return herr(e);
    (void)hipEventRecord(s->e0, st);
    e = launch_persist(a, f64, grid);
    (void)hipEventRecord(s->e1, st);
    if (e != hipSuccess) return herr(e);
    e = hipMemcpyAsync(&h, s->d_ps, sizeof h, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
    s->pending = 0;
    s->rounds = 1;
    if (tuned("SEARCH_DEBUG", nullptr))
        std::fprintf(stderr, "persist: grid %d seeds %llu/%llu head %llu tail %llu consumed %llu work %llu abort %llu ms %.3f\n",
                     grid, h.seed_cursor.v, (unsigned long long)s->local_items, h.head.v, h.tail.v, h.consumed.v,
                     h.work.v, h.abort.v, ms);
    if (h.abort.v & 1u) return -ETIMEDOUT;
    if (h.abort.v) return -EIO;
    if (h.work.v != 0) return -EIO;  // every item must have finished
    return 0;
}

// Exhaustive enumeration in ONE launch (enum.hip): a lane per depth-(N-6)
// prefix, its 720 completions in registers.  nodes = the prefix levels (host,
// exact) + 1,956 per lane (device).
static int run_enum(tspgpu_search *s)
{
    (void)hipSetDevice(s->ctx->device);
    hipStream_t st = s->ctx->stream;
    const int N = s->n - 1, G = N - 6;
    unsigned long long upper = 0;
    for (int l = 1; l <= G; ++l) upper += falling(N, l);
    SearchArgs a = args_of(s);
    a.depth = G;
    a.items = (uint32_t)falling(N, G);
    const uint64_t blocks = (a.items + kSearchThreads - 1) / kSearchThreads;
    int per_cu = 8;
    per_cu = std::max(1, tuned_int("ENUM_WG_PER_CU", per_cu));
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)s->ctx->cu_count * per_cu));
    hipError_t e = hipMemcpyAsync(s->d_stats, &upper, 8, hipMemcpyHostToDevice, st);  // line 0, nodes
    if (e != hipSuccess) return herr(e);
    (void)hipEventRecord(s->e0, st);
    e = launch_enum(a, s->dtype == TSPGPU_F64, grid);
    (void)hipEventRecord(s->e1, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return herr(e);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->e0, s->e1) == hipSuccess) s->ms += ms;
    s->depth = G;
    s->items = a.items;
    s->pending = 0;
    ++s->rounds;
    return 0;
}

int tspgpu_search_run_all(tspgpu_search *s)
{
    if (!s) return -EINVAL;
    if (s->noprune && s->enum_kernel) return run_enum(s);
    if (s->kernel == 3 && !s->noprune) return run_persist(s);
    s->fresh = false;
    if (s->nshards == 1 && chainable(s)) {
        bool done = false;
        int rc = run_chain(s, &done);
        if (rc || done) return rc;
    }
    int rc = tspgpu_search_start(s);
    uint64_t pending = 1;
    const bool trace = tuned_or("SEARCH_DEBUG", 0) >= 2;
    while (!rc && pending) {
        rc = tspgpu_search_step(s, &pending);
        if (trace)
            std::fprintf(stderr, "step %d: pending %llu tails %llu kernel %.3f ms\n", s->rounds,
                         (unsigned long long)pending, (unsigned long long)s->tails, s->ms);
    }
    return rc;
}

int tspgpu_search_chain(tspgpu_search *s, int exchange_every, tspgpu_level_hook hook, void *user, int *done)
{
    if (!s || !done || exchange_every < 0) return -EINVAL;
    *done = 0;
    (void)hipSetDevice(s->ctx->device);
    s->fresh = false;
    if (!chainable(s)) {
        // the same number of exchanges as a chained shard would enqueue
        const int levels = s->frontier ? s->n - 1 - s->tail_len - s->depth : 0;
        const int hooks = hook && exchange_every > 0 && levels > 1 ? (levels - 1) / exchange_every : 0;
        for (int k = 0; k < hooks; ++k) hook(user, s->ctx->stream, s->d_words + 1);
        return 0;
    }
    s->fetch = true;
    bool ok = false;
    const int rc = run_chain(s, &ok, exchange_every, hook, user);
    s->fetch = false;
    if (rc) return rc;
    *done = ok ? 1 : 0;
    s->fresh = ok && s->fetched;
    return 0;
}

int tspgpu_search_tie_slot(tspgpu_search *s, uint64_t cost_bits, tspgpu_tie_slot *out)
{
    if (!s || !out) return -EINVAL;
    std::memset(out, 0, sizeof *out);
    if (!s->tie_on) {
        out->overflow = 1;  // (no device tie rule: the records decide)
        return 0;
    }
    (void)hipSetDevice(s->ctx->device);
    unsigned long long local[5] = {};
    const unsigned long long *t = local;
    if (s->fresh && fetch_buf(s)[4 + 1] == cost_bits) {
        t = fetch_buf(s) + 20;  // read with the chain's synchronisation
    } else {
        SearchArgs a = args_of(s);
        const unsigned long long c = cost_bits;
        unsigned long long *h = s->h_cnt ? s->h_cnt + 8 : local;
        hipError_t e = launch_tie_lookup(a, tie_words(s), &c);
        if (e == hipSuccess)
            e = hipMemcpyAsync(h, tie_words(s), 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->ctx->stream);
        if (e != hipSuccess) return herr(e);
        t = h;
    }
    const bool two = s->n - 1 > 20;
    out->found = t[0] == 1 ? 1 : 0;
    out->overflow = t[4] != 0 ? 1 : 0;
    out->w0 = out->found ? t[1] : ~0ull;
    out->w1 = out->found && two ? t[3] : 0ull;
    // two-word keys: the least w0's own sub-slot must hold its w1
    if (out->found && two && t[2] != t[1]) out->overflow = 1;
    return 0;
}

int tspgpu_search_timing(const tspgpu_search *s, double *kernel_ms, int *rounds)
{
    if (!s) return -EINVAL;
    if (kernel_ms) *kernel_ms = s->ms;
    if (rounds) *rounds = s->rounds;
    return 0;
}

void *tspgpu_search_incumbent_device(tspgpu_search *s)
{
    if (!s) return nullptr;
    s->inc_shared = true;  // (the caller may write word 1: a chain then saves it itself)
    // ... and the last chain's readback may no longer hold it: counters and
    // tie_slot read the device from now on (an all-reduce after the chain
    // lowers word 1 below the shard's own incumbent)
    s->fresh = false;
    return (void *)(s->d_words + 1);
}

int tspgpu_search_counters(tspgpu_search *s, uint64_t *incumbent_bits, uint64_t *nodes, uint64_t *records)
{
    if (!s) return -EINVAL;
    (void)hipSetDevice(s->ctx->device);
    unsigned long long w[5];
    uint64_t st[4];
    if (s->fresh) {  // (the chain's readback)
        const unsigned long long *f = fetch_buf(s);
        for (int i = 0; i < 4; ++i) st[i] = f[i];
        for (int i = 0; i < 5; ++i) w[i] = f[4 + i];
    } else if (int rc = read_words_stats(s, w, st)) {
        return rc;
    }
    if (incumbent_bits) *incumbent_bits = w[1];
    if (records) *records = (uint32_t)w[3];
    if (nodes) *nodes = st[0];
    return 0;
}

int tspgpu_search_reset_records(tspgpu_search *s, unsigned int capacity)
{
    if (!s) return -EINVAL;
    s->fresh = false;
    (void)hipSetDevice(s->ctx->device);
    hipError_t e = hipStreamSynchronize(s->ctx->stream);
    if (e == hipSuccess && capacity > s->rec_cap) {
        if (capacity > s->rec_alloc) {
            (void)hipFree(s->d_rec);
            s->d_rec = nullptr;
            s->rec_alloc = 0;
            e = hipMalloc((void **)&s->d_rec, sizeof(SearchRecord) * (size_t)capacity);
            if (e == hipSuccess) s->rec_alloc = capacity;
        }
        if (e == hipSuccess) s->rec_cap = capacity;
    }
    if (e == hipSuccess) e = hipMemset(s->d_words + 3, 0, 8);
    return herr(e);
}

// the records of cost cost_bits among the `claimed` the kernels wrote
static int records_of(tspgpu_search *s, uint64_t claimed, uint64_t cost_bits, tspgpu_tour_record *out, int cap,
                      int *count)
{
    if (claimed > s->rec_cap) return -EOVERFLOW;
    std::vector<SearchRecord> h(claimed);
    if (claimed && s->fresh && claimed <= std::min(kSpecRecs, s->rec_cap)) {  // (the chain's readback)
        std::memcpy(h.data(), fetch_buf(s) + kFetchWords, sizeof(SearchRecord) * claimed);
    } else if (claimed) {
        hipError_t e = hipMemcpy(h.data(), s->d_rec, sizeof(SearchRecord) * claimed, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return herr(e);
    }
    int k = 0;
    for (const auto &r : h) {
        if (r.cost != cost_bits) continue;
        if (k < cap) std::memcpy(&out[k], &r, sizeof r);
        ++k;
    }
    *count = k;
    return k > cap ? -ENOSPC : 0;
}

int tspgpu_search_records(tspgpu_search *s, uint64_t cost_bits, tspgpu_tour_record *out, int cap, int *count)
{
    if (!s || !count || (cap > 0 && !out)) return -EINVAL;
    uint64_t claimed = 0;
    int rc = tspgpu_search_counters(s, nullptr, nullptr, &claimed);
    if (rc) return rc;
    return records_of(s, claimed, cost_bits, out, cap, count);
}

static int search_solve(tspgpu_ctx *c, const void *dist, int dtype, int n, double *cost_out, int32_t *tour_out,
                        tspgpu_search_stats *stats, int noprune)
{
    if (!c || !cost_out || !tour_out) return -EINVAL;
    // knob SEARCH_DEBUG: host phase times on stderr (development aid)
    const bool dbg = tuned("SEARCH_DEBUG", nullptr);
    using clk = std::chrono::steady_clock;
    const clk::time_point T0 = clk::now();
    clk::time_point T1 = T0, T2 = T0, T3 = T0, T4 = T0;
    auto ms_of = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    tspgpu_search *s = nullptr;
    int depth = 0;  // automatic; knob SEARCH_DEPTH (tests): a shallow seed, a deep frontier
    depth = std::max(0, tuned_int("SEARCH_DEPTH", depth));
    // the multi-start bound (host) while the search is created (host tables,
    // device buffers): both take ~1 ms at 32 cities
    double ub = 0.0;
    int hrc = 0;
    std::thread ht;
    bool threaded = false;
    // 13..19 cities: the bound computed on the device by the search's init
    // launch (search.hip init_heuristic, one wave per start city) instead of
    // by the host before the search (~35 us of the ~0.2 ms at 16 cities);
    // knob SEARCH_DEVICE_BOUND=0: the host
    const bool dev_bound = !noprune && n >= 13 && n < tuned_int("SEARCH_DEVICE_BOUND_MAXN", 20) &&
                           tuned_or("SEARCH_DEVICE_BOUND", 1) != 0;
    if (n >= 20) {  // (smaller: a thread costs more than it saves)
        try {
            ht = std::thread([&] { hrc = tspgpu_heuristic_tour(dist, dtype, n, &ub, nullptr); });
            threaded = true;
        } catch (...) {
        }
    }
    // (n < 20: the bound first, then written with the counter words at create)
    if (!threaded && !dev_bound) hrc = tspgpu_heuristic_tour(dist, dtype, n, &ub, nullptr);
    int rc = search_create(c, dist, dtype, n, 0, 1, depth, threaded || hrc || dev_bound ? nullptr : &ub, &s,
                           dev_bound);
    if (threaded) ht.join();
    if (rc) return rc;
    s->noprune = noprune;
    if (dev_bound && !s->dev_heur) {  // (pageable staging: no init launch, the host's bound)
        hrc = tspgpu_heuristic_tour(dist, dtype, n, &ub, nullptr);
        if (!hrc) hrc = tspgpu_search_set_bound(s, ub);
    }
    // enumeration work is uniform and every lane reaches the register tails:
    // long budgets (fewer, fuller rounds) win (profiles/r01/k2_exhaustive_budget.log)
    if (noprune && !tuned("SEARCH_BUDGET", nullptr)) s->budget = 16384;
    // 7 <= n <= 16, one shard: the register-tail enumeration kernel (enum.hip);
    // knob ENUM_KERNEL=0 keeps the round kernels (tests compare both)
    s->enum_kernel = noprune && n >= 7 && n <= 16 && tuned_or("ENUM_KERNEL", 1) != 0;
    if (double v; tuned("SEARCH_RECORD_CAP", &v) && v > 0)  // tests: force the second phase
        s->rec_cap = (unsigned int)std::min<double>(v, s->rec_cap);
    rc = hrc;
    if (dbg) T1 = clk::now();
    if (!rc && threaded) rc = tspgpu_search_set_bound(s, ub);
    int phases = 1, fallback = 0;
    uint64_t inc = 0, nodes = 0, nodes_total = 0, recs = 0;
    uint64_t u[4] = {0, 0, 0, 0};  // statistics of the last read (lane-step counters)
    unsigned long long w[5] = {};
    // counter words and statistics in one readback
    auto counters = [&]() {
        int r = read_words_stats(s, w, u);
        inc = w[1];
        recs = (uint32_t)w[3];
        nodes = u[0];
        return r;
    };
    // counters, statistics and (speculatively) the first kSpecRecs records in
    // one synchronisation
    std::vector<SearchRecord> spec;
    const SearchRecord *specp = nullptr;
    bool spec_ok = false;
    if (dbg) T2 = clk::now();
    s->fetch = true;  // (the chained search reads everything below in its one synchronisation)
    if (!rc) rc = tspgpu_search_run_all(s);
    if (dbg) T3 = clk::now();
    // the device tie rule's answer: the optimum's slot, read with the counters
    unsigned long long tie_local[5] = {};
    unsigned long long *tie_h = s->h_cnt ? s->h_cnt + 8 : tie_local;
    if (!rc && s->fetched) {
        const unsigned long long *f = fetch_buf(s);
        for (int i = 0; i < 4; ++i) u[i] = f[i];
        for (int i = 0; i < 5; ++i) w[i] = f[4 + i];
        tie_h = const_cast<unsigned long long *>(f + 20);
        inc = w[1];
        recs = (uint32_t)w[3];
        nodes = u[0];
        specp = reinterpret_cast<const SearchRecord *>(f + kFetchWords);
        spec_ok = recs <= std::min(kSpecRecs, s->rec_cap);
    } else if (!rc && s->tie_on) {
        SearchArgs a = args_of(s);
        hipError_t e = launch_tie_lookup(a, tie_words(s));
        if (e == hipSuccess)
            e = hipMemcpyAsync(tie_h, tie_words(s), 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               s->ctx->stream);
        rc = herr(e);
    }
    if (!rc && !s->fetched) {
        const unsigned k = std::min<unsigned>(kSpecRecs, s->rec_cap);
        spec.resize(k);
        hipError_t e = hipMemcpyAsync(spec.data(), s->d_rec, sizeof(SearchRecord) * k, hipMemcpyDeviceToHost,
                                      s->ctx->stream);
        rc = herr(e);
        if (!rc) rc = counters();  // (its synchronisation covers the record copy)
        spec_ok = !rc && recs <= k;
        specp = spec.data();
    }
    nodes_total = nodes;
    if (dbg) T4 = clk::now();
    // device tie rule: the optimum's slot decoded and certified on the host
    // (tspgpu_tie_tour); then neither the records nor a second search are needed
    bool tie_done = false;
    int tie_checked = 0;
    std::vector<int32_t> tie_tour(n + 1, 0);
    if (!rc && s->tie_on && tie_h[0] == 1 && tie_h[4] == 0) {
        const bool two = n - 1 > 20;
        // every record on the host already (the fetch's speculative read):
        // the certificate's prefix minima come from the optimal set itself
        // (search_host.h records_prefix), no prefix DP on the GPU
        tspgpu::host::RecordsPrefix rp{specp, (int)recs, inc, gpu_prefix, c};
        if (!two || tie_h[2] == tie_h[1])
            tie_done = (spec_ok ? tspgpu::host::tie_tour(dist, dtype, n, two ? tie_h[2] : tie_h[1],
                                                         two ? tie_h[3] : 0ull, inc, tie_tour.data(), true,
                                                         tspgpu::host::records_prefix, &rp, 0)
                                : tspgpu::host::tie_tour(dist, dtype, n, two ? tie_h[2] : tie_h[1],
                                                         two ? tie_h[3] : 0ull, inc, tie_tour.data(),
                                                         recs > s->rec_cap, gpu_prefix, c, kTieHostMax)) == 0;
    }
    // the record buffer overflowed: search again with the optimum as the bound,
    // so only optimal tours are recorded, into a buffer of the size now known
    constexpr uint64_t kPhase2Cap = 1u << 22;
    if (!rc && !tie_done && recs > s->rec_cap && recs <= kPhase2Cap) {
        phases = 2;
        unsigned long long w = inc;
        rc = tspgpu_search_reset_records(s, (unsigned int)recs);
        if (!rc) rc = herr(hipMemcpy(s->d_words + 1, &w, 8, hipMemcpyHostToDevice));
        if (!rc) rc = herr(hipMemset(s->d_stats, 0, kStatBytes));
        if (!rc) rc = tspgpu_search_run_all(s);
        if (!rc) rc = counters();
        spec_ok = false;
        nodes_total += nodes;
    }
    std::vector<tspgpu_tour_record> opt;
    int count = 0;
    if (!rc && tie_done) {
        std::memcpy(tour_out, tie_tour.data(), sizeof(int32_t) * (n + 1));
        if (dtype == TSPGPU_F64)
            std::memcpy(cost_out, &inc, 8);
        else
            *cost_out = (double)(int32_t)(uint32_t)inc;
        // the records came back with the counters: the host rule over them
        // must give the same tour (a self-check; the records then decide)
        if (spec_ok) {
            for (uint64_t i = 0; i < recs; ++i)
                if (specp[i].cost == inc) opt.push_back(reinterpret_cast<const tspgpu_tour_record &>(specp[i]));
            count = (int)opt.size();
            std::vector<int32_t> ht(n + 1, 0);
            if (count > 0 && tspgpu_select_tour(dist, dtype, n, opt.data(), count, inc, ht.data()) == 0) {
                tie_checked = ht == tie_tour ? 1 : -1;
                if (tie_checked < 0) std::memcpy(tour_out, ht.data(), sizeof(int32_t) * (n + 1));
            }
        }
    } else if (!rc && recs > s->rec_cap) {
        // |O| too large to enumerate (e.g. coincident cities): the DP itself
        // (K1-wide, also on the GPU) gives tsp()'s tour directly for n <= 31
        if (n <= TSPGPU_WIDE_MAX_CITIES) {
            fallback = 1;
            std::vector<double> dd(n * n);
            if (dtype == TSPGPU_F64)
                std::memcpy(dd.data(), dist, sizeof(double) * n * n);
            else
                for (int i = 0; i < n * n; ++i) dd[i] = static_cast<const int32_t *>(dist)[i];
            rc = tspgpu_solve_instance(c, dd.data(), n, cost_out, tour_out, nullptr);
        } else {
            rc = -EOVERFLOW;
        }
    } else if (!rc) {
        opt.resize(recs);
        if (spec_ok) {
            for (uint64_t i = 0; i < recs; ++i)
                if (specp[i].cost == inc) std::memcpy(&opt[count++], &specp[i], sizeof(SearchRecord));
        } else {
            rc = records_of(s, recs, inc, opt.data(), (int)recs, &count);
        }
        if (!rc) rc = tspgpu_select_tour(dist, dtype, n, opt.data(), count, inc, tour_out);
        if (!rc) {
            if (dtype == TSPGPU_F64)
                std::memcpy(cost_out, &inc, 8);
            else
                *cost_out = (double)(int32_t)(uint32_t)inc;
        }
    }
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->nodes = nodes_total;
        stats->records = recs;
        stats->optimal_tours = fallback ? 0 : (uint64_t)count;
        stats->depth = s->depth;
        stats->phases = phases;
        stats->fallback = fallback;
        stats->kernel_ms = s->ms;
        stats->items = s->items;
        stats->rounds = s->rounds;
        stats->lane_steps = u[1];
        stats->active_steps = u[2];
        stats->item_loads = u[3];
        stats->tie = tie_done && tie_checked >= 0 ? 1 : 0;
        stats->tie_checked = tie_checked;
    }
    const double dev_ms = s->ms;
    tspgpu_search_destroy(s);
    if (dbg)
        std::fprintf(stderr,
                     "search_solve n=%d: create+bound %.3f ms, set_bound %.3f, run %.3f (device %.3f), read %.3f, "
                     "select+destroy %.3f, total %.3f; tie %d checked %d phases %d\n",
                     n, ms_of(T0, T1), ms_of(T1, T2), ms_of(T2, T3), dev_ms, ms_of(T3, T4), ms_of(T4, clk::now()),
                     ms_of(T0, clk::now()), stats ? stats->tie : -1, stats ? stats->tie_checked : -1, phases);
    return rc;
}

int tspgpu_search_solve(tspgpu_ctx *c, const void *dist, int dtype, int n, double *cost_out, int32_t *tour_out,
                        tspgpu_search_stats *stats)
{
    return search_solve(c, dist, dtype, n, cost_out, tour_out, stats, 0);
}

int tspgpu_search_enumerate(tspgpu_ctx *c, const void *dist, int dtype, int n, double *cost_out, int32_t *tour_out,
                            tspgpu_search_stats *stats)
{
    return search_solve(c, dist, dtype, n, cost_out, tour_out, stats, 1);
}

}  // extern "C"
