// K3 — the reference's mergeBlocks (tsp.cpp:197-269) and its reduction tree
// (tsp.cpp:52-134, 348-352) with the paths resident on the GPU.
//
// mergeBlocks looks for the pair of edges (A,B) of path 1 and (C,D) of path 2
// (cyclic successors, the closing duplicate city included) with the smallest
//     swapPairCost = ((d(A,D) + d(B,C)) - d(A,B)) - d(C,D)        (tsp.cpp:197-200)
// first strict minimum in row-major (i, j) order from INT_MAX (tsp.cpp:204-227),
// then splices path 2 (closing city dropped, rotated to start after C,
// reversed) behind the first city of path 1 that is A or B (tsp.cpp:229-259).
// The reference is O(L1 * L2^2) (it rotates a vector per step); the search is
// an L1 x L2 argmin, i.e. GPU work once the running path grows (a rank folds
// all its blocks into one path, so at ./tsp 16 16384 the fold alone is ~4e10
// pair evaluations).
//
// Exactness.  d() is sqrt(pow(dx,2) + pow(dy,2)) with glibc pow, which differs
// from dx*dx in ~0.08% of inputs, so the device cannot reproduce d() bit for
// bit.  It computes every swap cost with dx*dx (a few ulp from the glibc
// value) and keeps as candidates all pairs within 2*eps of its minimum, eps =
// 2^-36 * 4 * Dmax (Dmax: the diagonal of the cities' bounding box) — about
// 10^4 times the largest possible discrepancy.  The host re-evaluates the
// candidates with glibc pow, in row-major order, with the reference's strict
// <: the exact minimum and every pair tied with it are always among them.
// If there are more candidates than the buffer holds, the host scans all
// pairs itself.  The splice is a gather kernel; the first-occurrence searches
// it needs are atomicMin reductions.  One host round trip per merge.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "xfer.h"
#include "tuning.h"
#include "wave.h"
#include "tspgpu.h"

using tspgpu::xcopy_async;

namespace {

constexpr int kMergeThreads = 256;
constexpr unsigned kCandCap = 1u << 16;
constexpr int kChunk = 1024;       // path-2 cities staged in LDS per block column
constexpr int kBatch = 2048;       // merges in flight between two host synchronisations
constexpr int kMaxBlocks = 4096;   // argmin / candidate grid (per-block minima kept)

struct Cand {
    int i, j;
    tspgpu_city a, b, c, d;
};

// Device control words of the merge stream.
struct Ctl {
    unsigned long long count;     // candidates of the current merge
    unsigned long long minkey;    // min order key of its swap costs
    unsigned long long done;      // candidate blocks finished (last block decides)
    unsigned long long stall;     // 0 ok; 1 the host must pick (several candidates); 2 EDEADLK; 3 EIO
    unsigned long long stall_at;  // batch index of the merge that stalled
    unsigned long long fw[2];     // first index of A|B in path 1, of C in path 2
    unsigned long long pad;
};

// What each merge leaves for the host: the chosen pair (the exact swap cost
// is recomputed with glibc pow on the host, tsp.cpp:263).
struct Pick {
    Cand c;
};

__device__ __forceinline__ double ddist(double ax, double ay, double bx, double by)
{
    const double dx = ax - bx;
    const double dy = ay - by;
    return sqrt(dx * dx + dy * dy);
}

__device__ __forceinline__ unsigned long long order_key(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__host__ __device__ __forceinline__ double key_value(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __builtin_bit_cast(double, b);
}

// Stage path-2 cities [j0, j0 + J] (successor included, cyclic) and the path-2
// edge lengths d(C_j, D_j) in LDS.
struct Stage {
    double x[kChunk + 1], y[kChunk + 1], e[kChunk];
};
__device__ __forceinline__ int stage_chunk(Stage &sm, const tspgpu_city *c2, int L2, int j0, int cw = kChunk)
{
    const int J = min(cw, L2 - j0);
    for (int t = threadIdx.x; t <= J; t += kMergeThreads) {
        const int j = j0 + t;
        const tspgpu_city c = c2[j < L2 ? j : j - L2];
        sm.x[t] = c.x;
        sm.y[t] = c.y;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < J; t += kMergeThreads) sm.e[t] = ddist(sm.x[t], sm.y[t], sm.x[t + 1], sm.y[t + 1]);
    __syncthreads();
    return J;
}

// Approximate swap costs (dx*dx, IEEE sqrt; tsp.cpp:197-200 order of operations)
// of path-1 edge i against the staged path-2 edges; calls f(j, cost).
template <typename F>
__device__ __forceinline__ void sweep_row(const Stage &sm, int J, const tspgpu_city *c1, int L1, int i, F &&f)
{
    const tspgpu_city A = c1[i], B = c1[i + 1 == L1 ? 0 : i + 1];
    const double eab = ddist(A.x, A.y, B.x, B.y);
    for (int t = 0; t < J; ++t) {
        const double sc = ((ddist(A.x, A.y, sm.x[t + 1], sm.y[t + 1]) + ddist(B.x, B.y, sm.x[t], sm.y[t])) - eab) -
                          sm.e[t];
        f(t, sc);
    }
}

// Pass 1: min swap key over all L1 x L2 pairs; blockIdx.y = path-2 chunk.
// Also resets this merge's first-occurrence words for find_kernel.
__global__ __launch_bounds__(kMergeThreads) void argmin_kernel(const tspgpu_city *c1, int L1, const tspgpu_city *c2,
                                                               int L2, int cw, Ctl *ctl, unsigned long long *blockmin)
{
    if (ctl->stall) return;
    __shared__ Stage sm;
    __shared__ unsigned long long wmin[kMergeThreads / 64];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        ctl->fw[0] = ~0ull;
        ctl->fw[1] = ~0ull;
    }
    unsigned long long best = ~0ull;
    for (int j0 = blockIdx.y * cw; j0 < L2; j0 += gridDim.y * cw) {
        const int J = stage_chunk(sm, c2, L2, j0, cw);
        for (int i = blockIdx.x * kMergeThreads + threadIdx.x; i < L1; i += gridDim.x * kMergeThreads)
            sweep_row(sm, J, c1, L1, i, [&](int, double sc) {
                const unsigned long long k = order_key(sc);
                best = k < best ? k : best;
            });
        __syncthreads();  // before the next chunk overwrites the stage
    }
    best = tspgpu::wave_min_dpp(best);
    if (__lane_id() == 0) wmin[threadIdx.x / 64] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = wmin[0];
        for (int w = 1; w < kMergeThreads / 64; ++w) b = wmin[w] < b ? wmin[w] : b;
        blockmin[blockIdx.y * gridDim.x + blockIdx.x] = b;
        if (b != ~0ull) atomicMin(&ctl->minkey, b);
    }
}

// Fold merges (path 2 is one block tour, L2 <= kChunk; path 1 holds each
// city once plus the closing copy of its first city): ONE kernel does both
// passes and the decision.  Every block computes its minimum; the last block
// to finish rescans the blocks within eps2 of the global minimum, and with
// exactly one candidate it logs the pick and the splice positions directly:
// the first city of path 1 that is A or B is index i (0 when A or B is the
// start city), C's first index in path 2 is j (0 for the closing copy).
// Otherwise the stream stalls for the host.
__global__ __launch_bounds__(kMergeThreads) void fold_pick_kernel(const tspgpu_city *c1, int L1, const tspgpu_city *c2,
                                                                  int L2, double eps2, Ctl *ctl,
                                                                  unsigned long long *blockmin, Cand *cand,
                                                                  Pick *picks, int idx)
{
    if (ctl->stall) return;
    __shared__ Stage sm;
    __shared__ unsigned long long wmin[kMergeThreads / 64];
    __shared__ bool last;
    __shared__ unsigned nc;
    const int J = stage_chunk(sm, c2, L2, 0);
    unsigned long long best = ~0ull;
    for (int i = blockIdx.x * kMergeThreads + threadIdx.x; i < L1; i += gridDim.x * kMergeThreads)
        sweep_row(sm, J, c1, L1, i, [&](int, double sc) {
            const unsigned long long k = order_key(sc);
            best = k < best ? k : best;
        });
    best = tspgpu::wave_min_dpp(best);
    if (__lane_id() == 0) wmin[threadIdx.x / 64] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = wmin[0];
        for (int w = 1; w < kMergeThreads / 64; ++w) b = wmin[w] < b ? wmin[w] : b;
        blockmin[blockIdx.x] = b;
        if (b != ~0ull) atomicMin(&ctl->minkey, b);
        __threadfence();
        last = atomicAdd(&ctl->done, 1ull) == (unsigned long long)gridDim.x - 1;
        nc = 0;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    const double thr = key_value(__hip_atomic_load(&ctl->minkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + eps2;
    // the blocks within eps2 of the minimum (usually one), gathered in parallel
    __shared__ int close[64];
    __shared__ unsigned nclose;
    if (threadIdx.x == 0) nclose = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < (int)gridDim.x; b += kMergeThreads) {
        const unsigned long long bm = __hip_atomic_load(&blockmin[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (key_value(bm) <= thr) {
            const unsigned q = atomicAdd(&nclose, 1u);
            if (q < 64) close[q] = b;
        }
    }
    __syncthreads();
    const bool all = nclose > 64;  // (many near-ties: rescan every block)
    const int nb = all ? (int)gridDim.x : (int)nclose;
    for (int q = 0; q < nb; ++q) {
        const int b = all ? q : close[q];
        for (int i = b * kMergeThreads + threadIdx.x; i < L1; i += gridDim.x * kMergeThreads)
            sweep_row(sm, J, c1, L1, i, [&](int t, double sc) {
                if (sc <= thr) {
                    const unsigned s2 = atomicAdd(&nc, 1u);
                    if (s2 < kCandCap) {
                        Cand c;
                        c.i = i;
                        c.j = t;
                        c.a = c1[i];
                        c.b = c1[i + 1 == L1 ? 0 : i + 1];
                        c.c = c2[t];
                        c.d = c2[t + 1 == L2 ? 0 : t + 1];
                        cand[s2] = c;
                    }
                }
            });
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    __threadfence();
    ctl->count = nc;
    if (nc != 1) {
        ctl->stall_at = (unsigned long long)idx;
        ctl->stall = 1;
        return;
    }
    const Cand k = cand[0];
    picks[idx].c = k;
    const int first = c1[0].id;
    ctl->fw[0] = (k.a.id == first || k.b.id == first) ? 0ull : (unsigned long long)k.i;
    ctl->fw[1] = k.j == L2 - 1 ? 0ull : (unsigned long long)k.j;
}

// Pass 2: every pair within eps2 of the minimum is a candidate (only blocks
// whose own minimum is that close rescan; the others return at once).
__global__ __launch_bounds__(kMergeThreads) void cand_kernel(const tspgpu_city *c1, int L1, const tspgpu_city *c2,
                                                             int L2, int cw, double eps2, Ctl *ctl,
                                                             const unsigned long long *blockmin, Cand *cand)
{
    if (ctl->stall) return;
    __shared__ Stage sm;
    const double thr = key_value(ctl->minkey) + eps2;
    if (!(key_value(blockmin[blockIdx.y * gridDim.x + blockIdx.x]) <= thr)) return;
    for (int j0 = blockIdx.y * cw; j0 < L2; j0 += gridDim.y * cw) {
        const int J = stage_chunk(sm, c2, L2, j0, cw);
        for (int i = blockIdx.x * kMergeThreads + threadIdx.x; i < L1; i += gridDim.x * kMergeThreads)
            sweep_row(sm, J, c1, L1, i, [&](int t, double sc) {
                if (sc <= thr) {
                    const unsigned s2 = (unsigned)atomicAdd(&ctl->count, 1ull);
                    if (s2 < kCandCap) {
                        const int j = j0 + t;
                        Cand c;
                        c.i = i;
                        c.j = j;
                        c.a = c1[i];
                        c.b = c1[i + 1 == L1 ? 0 : i + 1];
                        c.c = c2[j];
                        c.d = c2[j + 1 == L2 ? 0 : j + 1];
                        cand[s2] = c;
                    }
                }
            });
        __syncthreads();
    }
}

// first index of path 1 whose id is A or B -> fw[0], first index of path 2
// [0, M) whose id is C -> fw[1] (tsp.cpp:229-239); ids from the pick unless given
// Unforced: exactly one candidate -> it is the reference's pair (the exact
// minimum and all its ties are always inside the window): log it as the
// merge's pick; else stall the stream for the host's exact re-evaluation.
__global__ __launch_bounds__(kMergeThreads) void find_kernel(const tspgpu_city *c1, int L1, const tspgpu_city *c2,
                                                             int M, Ctl *ctl, const Cand *cand, Pick *picks, int idx,
                                                             int idA, int idB, int idC, int forced)
{
    if (ctl->stall && !forced) return;
    if (!forced) {
        __shared__ int ids[4];
        if (threadIdx.x == 0) {
            const bool one = ctl->count == 1;
            ids[3] = one;
            if (one) {
                const Cand k = cand[0];
                ids[0] = k.a.id;
                ids[1] = k.b.id;
                ids[2] = k.c.id;
                if (blockIdx.x == 0) picks[idx].c = k;
            } else if (blockIdx.x == 0) {
                ctl->stall_at = (unsigned long long)idx;
                ctl->stall = 1;
            }
        }
        __syncthreads();
        if (!ids[3]) return;
        idA = ids[0];
        idB = ids[1];
        idC = ids[2];
    }
    const int t = blockIdx.x * kMergeThreads + threadIdx.x;
    const int stride = gridDim.x * kMergeThreads;
    for (int i = t; i < L1; i += stride)
        if (c1[i].id == idA || c1[i].id == idB) atomicMin(&ctl->fw[0], (unsigned long long)i);
    for (int j = t; j < M; j += stride)
        if (c2[j].id == idC) atomicMin(&ctl->fw[1], (unsigned long long)j);
}

// out = c1[0..p] ++ reverse(c2 rotated to start after C, closing city dropped) ++ c1[p+1..]
// (tsp.cpp:240-259), copied as 8-byte words (3 per city); then clears the
// words of the next merge.
__global__ __launch_bounds__(kMergeThreads) void splice_kernel(const tspgpu_city *c1, int L1, const tspgpu_city *c2,
                                                               int M, Ctl *ctl, tspgpu_city *out, int idx, int forced)
{
    static_assert(sizeof(tspgpu_city) == 24, "City layout");
    if (ctl->stall && !forced) return;
    const unsigned long long pw = ctl->fw[0], sw = ctl->fw[1];
    if (pw >= (unsigned long long)L1 || sw >= (unsigned long long)M) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctl->stall_at = (unsigned long long)idx;
            ctl->stall = sw >= (unsigned long long)M ? 2 : 3;  // C not in path 2: tsp.cpp:236-239 never ends
        }
        return;
    }
    const int p = (int)pw, start = (int)((sw + 1) % (unsigned)M);
    const unsigned long long *w1 = reinterpret_cast<const unsigned long long *>(c1);
    const unsigned long long *w2 = reinterpret_cast<const unsigned long long *>(c2);
    unsigned long long *wo = reinterpret_cast<unsigned long long *>(out);
    const int total = 3 * (L1 + M);
    for (int w = blockIdx.x * kMergeThreads + threadIdx.x; w < total; w += gridDim.x * kMergeThreads) {
        const int k = w / 3, f = w - 3 * k;
        int src;
        const unsigned long long *base;
        if (k <= p) {
            base = w1;
            src = k;
        } else if (k <= p + M) {
            const int q = start + (M - 1 - (k - p - 1));
            base = w2;
            src = q >= M ? q - M : q;
        } else {
            base = w1;
            src = k - M;
        }
        wo[w] = base[3 * src + f];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->count = 0;
        ctl->minkey = ~0ull;
        ctl->done = 0;
        if (forced) ctl->stall = 0;
    }
}

// ---- persistent per-rank fold (tsp.cpp:348-352) --------------------------------
//
// The local fold s = ((b0 ⊕ b1) ⊕ b2) ... of every logical rank's contiguous
// blocks is a chain of small dependent merges (path 1 grows by one block tour
// of M = L2 - 1 cities per merge).  As separate launches it was 2 kernels per
// merge in strict sequence (./tsp 8 1024 at P = 8: 1,016 fold_pick + 1,023
// splice launches, ~10 us each, profiles/r04/k3_kernel_stats.csv).  Here ONE
// launch runs every rank's whole fold: a workgroup per rank keeps its path in
// LDS (structure of arrays), and each merge is three phases between workgroup
// barriers — the swap-cost minimum (dx*dx, IEEE sqrt, the reference's order of
// operations), the candidates within eps2 of it, and, with exactly one
// candidate (then it is the reference's pair, as for fold_pick_kernel), the
// splice in LDS.  The pick (A, B, C, D) of every merge is logged for the
// host's exact cost fold (glibc pow, tsp.cpp:263).  A merge with several
// candidates, or one whose result would not fit the LDS path, stops the rank:
// its path goes to global memory with the index of the merge, for the host
// (exact pick, then the remaining merges by the general path or a relaunch).
constexpr int kFoldThreads = 1024;
constexpr int kFoldCap = 4096;   // cities of a rank's path held in LDS (20 B each)
constexpr int kFoldL2 = 33;      // block tours up to 32 cities + the closing copy

struct FoldJob {
    int first;     // block of the rank's running path when the kernel starts (path = that block's tour if k0 == 0)
    int count;     // blocks of the rank: merges k0 .. count-2 fold blocks first + 1 + k
    int k0;        // next merge (0: start from the block; > 0: from path/len, a relaunch)
    int len;       // running path length when k0 > 0 (in `path`)
    tspgpu_city *path;  // the rank's running path (global; capacity >= all cities)
    Pick *picks;        // one per merge of this rank (count - 1)
};
struct FoldOut {
    int status;  // 0 done, 1 stalled (several candidates) at merge `at`, 2 path cap reached before merge `at`
    int at;
    int len;     // running path length written to path (status != 0: before merge `at`)
    int count;   // candidates of the stalled merge
};

// (key, pair) of the smallest swap cost and the second-smallest key of a set
// of pairs: exactly one pair is within eps2 of the minimum iff the second key
// lies above min + eps2 — one pass over the pairs decides what fold_pick's
// two passes did
struct Top2 {
    unsigned long long k1, k2;
    unsigned i1;
};
__device__ __forceinline__ void top2_add(Top2 &a, unsigned long long k, unsigned i)
{
    if (k < a.k1) {
        a.k2 = a.k1;
        a.k1 = k;
        a.i1 = i;
    } else if (k < a.k2) {
        a.k2 = k;
    }
}
__device__ __forceinline__ Top2 top2_merge(const Top2 &a, const Top2 &b)
{
    Top2 r;
    const bool lo = a.k1 < b.k1 || (a.k1 == b.k1 && a.i1 < b.i1);
    r.k1 = lo ? a.k1 : b.k1;
    r.i1 = lo ? a.i1 : b.i1;
    const unsigned long long hi = lo ? b.k1 : a.k1;
    r.k2 = min(hi, min(a.k2, b.k2));
    return r;
}
__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int m)
{
    const int lo = __shfl_xor((int)(unsigned)v, m), hi = __shfl_xor((int)(unsigned)(v >> 32), m);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

__global__ __launch_bounds__(kFoldThreads) void fold_persist_kernel(const tspgpu_city *blocks, int L2, double eps2,
                                                                    const FoldJob *jobs, FoldOut *outs)
{
    __shared__ double px[kFoldCap], py[kFoldCap];
    __shared__ int pid[kFoldCap];
    __shared__ double cx[kFoldL2], cy[kFoldL2], ce[kFoldL2];
    __shared__ int cid[kFoldL2];
    __shared__ Top2 wtop[kFoldThreads / 64];
    const FoldJob J = jobs[blockIdx.x];
    const int t = threadIdx.x;
    const int M = L2 - 1;
    int len;
    if (J.k0 == 0) {
        len = L2;
        const tspgpu_city *b = blocks + (size_t)J.first * L2;
        for (int k = t; k < L2; k += kFoldThreads) {
            const tspgpu_city c = b[k];
            px[k] = c.x, py[k] = c.y, pid[k] = c.id;
        }
    } else {
        len = J.len;
        for (int k = t; k < len; k += kFoldThreads) {
            const tspgpu_city c = J.path[k];
            px[k] = c.x, py[k] = c.y, pid[k] = c.id;
        }
    }
    int status = 0, at = J.count - 1, nc = 1;
    for (int m = J.k0; m < J.count - 1; ++m) {
        if (len + M > kFoldCap) {
            status = 2, at = m;
            break;
        }
        // stage the block (cities and edge lengths, read straight from memory:
        // one barrier, which also orders the previous splice's LDS writes)
        const tspgpu_city *c2 = blocks + (size_t)(J.first + 1 + m) * L2;
        if (t < L2) {
            const tspgpu_city c = c2[t], d = c2[t + 1 == L2 ? 0 : t + 1];
            cx[t] = c.x, cy[t] = c.y, cid[t] = c.id;
            ce[t] = ddist(c.x, c.y, d.x, d.y);
        }
        __syncthreads();
        // one pass: the two smallest order keys of every swap cost (i over path
        // edges, j over block edges, pair index i * L2 + j = row-major order)
        Top2 tp{~0ull, ~0ull, ~0u};
        for (int i = t; i < len; i += kFoldThreads) {
            const int i1 = i + 1 == len ? 0 : i + 1;
            const double ax = px[i], ay = py[i], bx = px[i1], by = py[i1];
            const double eab = ddist(ax, ay, bx, by);
            for (int j = 0; j < L2; ++j) {
                const int j1 = j + 1 == L2 ? 0 : j + 1;
                const double sc = ((ddist(ax, ay, cx[j1], cy[j1]) + ddist(bx, by, cx[j], cy[j])) - eab) - ce[j];
                top2_add(tp, order_key(sc), (unsigned)(i * L2 + j));
            }
        }
#pragma unroll
        for (int o = 1; o < 64; o *= 2) {
            Top2 q;
            q.k1 = shfl_u64(tp.k1, o);
            q.k2 = shfl_u64(tp.k2, o);
            q.i1 = (unsigned)__shfl_xor((int)tp.i1, o);
            tp = top2_merge(tp, q);
        }
        if (__lane_id() == 0) wtop[t / 64] = tp;
        __syncthreads();
        Top2 g = wtop[0];
#pragma unroll
        for (int w = 1; w < kFoldThreads / 64; ++w) g = top2_merge(g, wtop[w]);
        // exactly one pair within eps2 of the minimum (then it is the
        // reference's pair, as in fold_pick_kernel), else the host decides
        const double thr = key_value(g.k1) + eps2;
        if (!(g.k2 == ~0ull || g.k2 > order_key(thr))) {
            status = 1, at = m, nc = 2;
            break;
        }
        const int pi = (int)(g.i1 / (unsigned)L2), pj = (int)(g.i1 % (unsigned)L2);
        const int pi1 = pi + 1 == len ? 0 : pi + 1, pj1 = pj + 1 == L2 ? 0 : pj + 1;
        if (t == 0) {
            Cand k;
            k.i = pi, k.j = pj;
            k.a = tspgpu_city{pid[pi], px[pi], py[pi]};
            k.b = tspgpu_city{pid[pi1], px[pi1], py[pi1]};
            k.c = tspgpu_city{cid[pj], cx[pj], cy[pj]};
            k.d = tspgpu_city{cid[pj1], cx[pj1], cy[pj1]};
            J.picks[m].c = k;
        }
        // splice (tsp.cpp:240-259): p = first index of A or B in path 1 (0 when
        // either is its first city: the path closes on it), C's first index in
        // path 2 (0 for the closing copy); out = path[0..p] ++ reversed rotation
        // of the block after C ++ path[p+1..]
        const int first = pid[0];
        const int p = (pid[pi] == first || pid[pi1] == first) ? 0 : pi;
        const int sw = pj == L2 - 1 ? 0 : pj;
        const int start = (sw + 1) % M;
        // shift path[p+1 .. len) up by M: through registers (4 per thread at the cap)
        constexpr int kPer = kFoldCap / kFoldThreads;
        double sx[kPer], sy[kPer];
        int sid[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int k = p + 1 + t + q * kFoldThreads;
            if (k < len) sx[q] = px[k], sy[q] = py[k], sid[q] = pid[k];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int k = p + 1 + t + q * kFoldThreads;
            if (k < len) px[k + M] = sx[q], py[k + M] = sy[q], pid[k + M] = sid[q];
        }
        if (t < M) {
            const int k = p + 1 + t;
            const int q = start + (M - 1 - t);
            const int src = q >= M ? q - M : q;
            px[k] = cx[src], py[k] = cy[src], pid[k] = cid[src];
        }
        len += M;
    }
    __syncthreads();
    for (int k = t; k < len; k += kFoldThreads) J.path[k] = tspgpu_city{pid[k], px[k], py[k]};
    if (t == 0) {
        FoldOut o;
        o.status = status, o.at = at, o.len = len, o.count = nc;
        outs[blockIdx.x] = o;
    }
}

// ---- host side ---------------------------------------------------------------

double (*volatile g_pow)(double, double) = ::pow;
double (*volatile g_sqrt)(double) = ::sqrt;

double hdist(const tspgpu_city &a, const tspgpu_city &b)
{
    return g_sqrt(g_pow(a.x - b.x, 2) + g_pow(a.y - b.y, 2));  // assignment2.h:141-144
}

double hswap(const tspgpu_city &A, const tspgpu_city &B, const tspgpu_city &C, const tspgpu_city &D)
{
    return ((hdist(A, D) + hdist(B, C)) - hdist(A, B)) - hdist(C, D);  // tsp.cpp:197-200
}

int herr(hipError_t e)
{
    if (e == hipSuccess) return 0;
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    return -EIO;
}

struct DVec {
    tspgpu_city *p = nullptr;
    size_t len = 0, cap = 0;
    // grows only when nothing in flight references it (callers reserve up front)
    int reserve(size_t n, hipStream_t st)
    {
        if (n <= cap) return 0;
        size_t c = std::max<size_t>(n, cap * 2 + 64);
        tspgpu_city *q = nullptr;
        hipError_t e = hipMalloc((void **)&q, c * sizeof(tspgpu_city));
        if (e != hipSuccess) return herr(e);
        if (len) e = xcopy_async(q, p, len * sizeof(tspgpu_city), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (p) (void)hipFree(p);
        p = q;
        cap = c;
        return herr(e);
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        len = cap = 0;
    }
};

// The merge stream.  merge() only enqueues: argmin, candidates, find, splice,
// all on the context's stream, no host round trip.  When exactly one pair is
// within eps2 of the device minimum it is the reference's pair (the exact
// minimum and all its ties are always inside the window) and the device
// splices at once; otherwise the stream stalls (later kernels return at once)
// and sync() lets the host pick with glibc pow, re-runs the stalled merge with
// the host's pair and re-enqueues the rest.  Costs, which need the exact swap
// cost (glibc pow) of every chosen pair, are folded on the host in merge order
// at sync(): cost_target = (cost_target + cost2) + best (tsp.cpp:263).
struct Merger {
    hipStream_t st = nullptr;
    int cus = 256;
    double eps2 = 0.0;
    Ctl *ctl = nullptr;
    Cand *cand = nullptr;
    Pick *picks = nullptr;
    unsigned long long *blockmin = nullptr;
    Ctl *hctl = nullptr;    // pinned mirror
    Pick *hpicks = nullptr; // pinned mirror
    struct Op {
        const tspgpu_city *src;
        tspgpu_city *dst;
        int L1;
        const tspgpu_city *c2;
        int L2;
        double *target;
        const double *cost2;
        bool fold;  // path 1 holds each city once + closing copy, path 2 is one block tour
    };
    std::vector<Op> ops;
    int init(tspgpu_ctx *c, double dmax)
    {
        st = c->stream;
        cus = c->cu_count;
        eps2 = 2.0 * std::ldexp(4.0 * dmax, -36);
        hipError_t e = hipMalloc((void **)&ctl, sizeof(Ctl));
        if (e == hipSuccess) e = hipMalloc((void **)&cand, kCandCap * sizeof(Cand));
        if (e == hipSuccess) e = hipMalloc((void **)&picks, kBatch * sizeof(Pick));
        if (e == hipSuccess) e = hipMalloc((void **)&blockmin, kMaxBlocks * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipHostMalloc((void **)&hctl, sizeof(Ctl), 0);
        if (e == hipSuccess) e = hipHostMalloc((void **)&hpicks, kBatch * sizeof(Pick), 0);
        if (e == hipSuccess) {
            Ctl z{};
            z.minkey = ~0ull;
            e = xcopy_async(ctl, &z, sizeof z, hipMemcpyHostToDevice, st);
        }
        ops.reserve(kBatch);
        return herr(e);
    }
    ~Merger()
    {
        if (ctl) (void)hipFree(ctl);
        if (cand) (void)hipFree(cand);
        if (picks) (void)hipFree(picks);
        if (blockmin) (void)hipFree(blockmin);
        if (hctl) (void)hipHostFree(hctl);
        if (hpicks) (void)hipHostFree(hpicks);
    }
    int grid_for(unsigned long long work) const
    {
        const unsigned long long b = (work + kMergeThreads - 1) / kMergeThreads;
        return (int)std::max<unsigned long long>(1, std::min<unsigned long long>(b, (unsigned long long)cus * 8));
    }
    // blockIdx.x strides path-1 edges, blockIdx.y path-2 chunks of *cw cities;
    // gx * gy <= kMaxBlocks.  The chunks narrow (down to 8 cities) until the
    // grid has about two blocks per CU: a tree merge of two ~1000-city paths
    // was 4 blocks on 4 CUs (argmin + candidates ~380 us, profiles/r05)
    dim3 pair_grid(int L1, int L2, int *cw) const
    {
        const int cap = std::min(cus * 8, kMaxBlocks);
        const int gx0 = std::max(1, std::min((L1 + kMergeThreads - 1) / kMergeThreads, cap));
        int w = kChunk;
        while (w > 8 && (long long)gx0 * ((L2 + w - 1) / w) < 2LL * cus) w /= 2;
        const int gy = std::min((L2 + w - 1) / w, cap);
        const int gx = std::max(1, std::min(gx0, cap / gy));
        *cw = w;
        return dim3(gx, gy);
    }
    void enqueue(const Op &o, int idx)
    {
        const int M = o.L2 - 1;
        if (o.fold && o.L2 <= kChunk) {
            const int gx = std::max(1, std::min((o.L1 + kMergeThreads - 1) / kMergeThreads, std::min(cus * 8, kMaxBlocks)));
            hipLaunchKernelGGL(fold_pick_kernel, dim3(gx), dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, o.L2, eps2,
                               ctl, blockmin, cand, picks, idx);
            hipLaunchKernelGGL(splice_kernel, dim3(grid_for(3ull * ((unsigned long long)o.L1 + M))),
                               dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, M, ctl, o.dst, idx, 0);
            return;
        }
        int cw = kChunk;
        const dim3 g = pair_grid(o.L1, o.L2, &cw);
        hipLaunchKernelGGL(argmin_kernel, g, dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, o.L2, cw, ctl, blockmin);
        hipLaunchKernelGGL(cand_kernel, g, dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, o.L2, cw, eps2, ctl, blockmin,
                           cand);
        hipLaunchKernelGGL(find_kernel, dim3(grid_for((unsigned long long)std::max(o.L1, M))), dim3(kMergeThreads), 0,
                           st, o.src, o.L1, o.c2, M, ctl, cand, picks, idx, 0, 0, 0, 0);
        hipLaunchKernelGGL(splice_kernel, dim3(grid_for(3ull * ((unsigned long long)o.L1 + M))), dim3(kMergeThreads),
                           0, st, o.src, o.L1, o.c2, M, ctl, o.dst, idx, 0);
    }
    // s1 <- mergeBlocks(s1, c2); *cost1 = (*cost1 + *cost2) + best once sync() ran.
    // tmp: a buffer of capacity >= s1.len + L2 - 1 (swapped with s1).
    int merge(DVec &s1, DVec &tmp, double *cost1, const tspgpu_city *c2, int L2, const double *cost2,
              bool fold = false)
    {
        const int L1 = (int)s1.len;
        if (L1 < 1 || L2 < 2) return -EINVAL;
        const int M = L2 - 1;
        if ((int)ops.size() == kBatch || tmp.cap < (size_t)L1 + M) {
            // (the reference's stale received lists can grow a path past all
            // cities: grow the spare buffer once nothing in flight uses it)
            int rc = sync();
            if (!rc) rc = tmp.reserve((size_t)L1 + M, st);
            if (rc) return rc;
        }
        Op o{s1.p, tmp.p, L1, c2, L2, cost1, cost2, fold};
        ops.push_back(o);
        enqueue(o, (int)ops.size() - 1);
        if (hipPeekAtLastError() != hipSuccess) return herr(hipGetLastError());
        std::swap(s1, tmp);
        s1.len = (size_t)L1 + M;
        tmp.len = 0;
        return 0;
    }
    // the host's pick for a stalled merge: exact (glibc) re-evaluation of the
    // candidates in row-major order with the reference's strict < from INT_MAX
    int host_pick(const Op &o, Cand &pick, double &best)
    {
        hipError_t e = hipSuccess;
        const unsigned long long nc = hctl->count;
        best = (double)INT_MAX;  // tsp.cpp:204
        bool found = false;
        if (nc > 0 && nc <= kCandCap) {
            std::vector<Cand> hc(nc);
            e = xcopy_async(hc.data(), cand, nc * sizeof(Cand), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return herr(e);
            std::sort(hc.begin(), hc.end(),
                      [](const Cand &x, const Cand &y) { return x.i != y.i ? x.i < y.i : x.j < y.j; });
            for (const Cand &k : hc) {
                const double sc = hswap(k.a, k.b, k.c, k.d);
                if (sc < best) {
                    best = sc;
                    pick = k;
                    found = true;
                }
            }
        } else {
            // too many near-ties for the buffer: exact scan on the host
            std::vector<tspgpu_city> h1(o.L1), h2(o.L2);
            e = xcopy_async(h1.data(), o.src, o.L1 * sizeof(tspgpu_city), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess)
                e = xcopy_async(h2.data(), o.c2, o.L2 * sizeof(tspgpu_city), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return herr(e);
            for (int i = 0; i < o.L1; ++i)
                for (int j = 0; j < o.L2; ++j) {
                    const tspgpu_city &a = h1[i], &b = h1[(i + 1) % o.L1], &c = h2[j], &d = h2[(j + 1) % o.L2];
                    const double sc = hswap(a, b, c, d);
                    if (sc < best) {
                        best = sc;
                        pick = Cand{i, j, a, b, c, d};
                        found = true;
                    }
                }
        }
        return found ? 0 : -EIO;  // no swap below INT_MAX (distances are validated far below)
    }
    // run every enqueued merge to completion, resolving stalls on the host,
    // and fold their costs in order
    int sync()
    {
        size_t first = 0;  // ops[first..] not yet folded
        for (;;) {
            hipError_t e = xcopy_async(hctl, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return herr(e);
            const size_t upto = hctl->stall ? (size_t)hctl->stall_at : ops.size();
            if (upto > first) {
                e = xcopy_async(hpicks + first, picks + first, (upto - first) * sizeof(Pick), hipMemcpyDeviceToHost, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) return herr(e);
                for (size_t m = first; m < upto; ++m) {
                    const Cand &k = hpicks[m].c;
                    *ops[m].target = (*ops[m].target + *ops[m].cost2) + hswap(k.a, k.b, k.c, k.d);
                }
                first = upto;
            }
            if (!hctl->stall) break;
            if (hctl->stall == 2) return -EDEADLK;
            if (hctl->stall != 1) return -EIO;
            // the host picks merge `first`, then the device splices it and the rest resumes
            const Op &o = ops[first];
            Cand pk{};
            double best = 0.0;
            int rc = host_pick(o, pk, best);
            if (rc) return rc;
            const int M = o.L2 - 1;
            Ctl reset = *hctl;
            reset.fw[0] = reset.fw[1] = ~0ull;
            e = xcopy_async(ctl, &reset, sizeof reset, hipMemcpyHostToDevice, st);
            if (e != hipSuccess) return herr(e);
            hipLaunchKernelGGL(find_kernel, dim3(grid_for((unsigned long long)std::max(o.L1, M))),
                               dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, M, ctl, cand, picks, (int)first,
                               pk.a.id, pk.b.id, pk.c.id, 1);
            hipLaunchKernelGGL(splice_kernel, dim3(grid_for(3ull * ((unsigned long long)o.L1 + M))),
                               dim3(kMergeThreads), 0, st, o.src, o.L1, o.c2, M, ctl, o.dst, (int)first, 1);
            e = xcopy_async(hctl, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return herr(e);
            if (hctl->stall == 2) return -EDEADLK;
            if (hctl->stall) return -EIO;
            *o.target = (*o.target + *o.cost2) + best;
            ++first;
            for (size_t m = first; m < ops.size(); ++m) enqueue(ops[m], (int)m);
            if (hipPeekAtLastError() != hipSuccess) return herr(hipGetLastError());
        }
        ops.clear();
        return 0;
    }
};

// mergeBlocks (tsp.cpp:202-269) on the host, exactly: glibc distances, first
// strict minimum in row-major order from INT_MAX, then the splice; for a fold
// merge that stalled the persistent kernel (several near-tied candidates).
// -> the pick (for the cost fold) and the new path in `path`.
int host_fold_merge(std::vector<tspgpu_city> &path, const tspgpu_city *c2, int L2, Cand &pick)
{
    const int L1 = (int)path.size(), M = L2 - 1;
    double best = (double)INT_MAX;  // tsp.cpp:204
    bool found = false;
    for (int i = 0; i < L1; ++i)
        for (int j = 0; j < L2; ++j) {
            const tspgpu_city &a = path[i], &b = path[(i + 1) % L1], &c = c2[j], &d = c2[(j + 1) % L2];
            const double sc = hswap(a, b, c, d);
            if (sc < best) {
                best = sc;
                pick = Cand{i, j, a, b, c, d};
                found = true;
            }
        }
    if (!found) return -EIO;
    // tsp.cpp:229-239: first index of A or B in path 1, of C in path 2 (without its closing copy)
    int p = -1, sw = -1;
    for (int k = 0; k < L1 && p < 0; ++k)
        if (path[k].id == pick.a.id || path[k].id == pick.b.id) p = k;
    for (int k = 0; k < M && sw < 0; ++k)
        if (c2[k].id == pick.c.id) sw = k;
    if (p < 0) return -EIO;
    if (sw < 0) return -EDEADLK;
    std::vector<tspgpu_city> out;
    out.reserve((size_t)L1 + M);
    const int start = (sw + 1) % M;
    for (int k = 0; k <= p; ++k) out.push_back(path[k]);
    for (int t = 0; t < M; ++t) {
        const int q = start + (M - 1 - t);
        out.push_back(c2[q >= M ? q - M : q]);
    }
    for (int k = p + 1; k < L1; ++k) out.push_back(path[k]);
    path.swap(out);
    return 0;
}

// The fold of every logical rank (tsp.cpp:348-352) by fold_persist_kernel.
// Ranks that stall (several near-tied candidates) get the merge exactly on the
// host and are relaunched from the next one; ranks whose path outgrows LDS
// finish through the Merger's per-merge kernels.  rank[r] holds the path and
// rcost[r] the cost on return (costs folded in merge order, tsp.cpp:263, with
// glibc swap costs of the logged picks).
int persist_folds(Merger &m, const tspgpu_city *blocks, int L, const double *costs, const std::vector<int> &cnt,
                  std::vector<DVec> &rank, DVec &tmp, std::vector<double> &rcost)
{
    const int P = (int)cnt.size();
    int nb = 0;
    for (int c : cnt) nb += c;
    const size_t ncity = (size_t)nb * L;
    FoldJob *djobs = nullptr;
    FoldOut *douts = nullptr;
    Pick *dpicks = nullptr;
    hipError_t e = hipMalloc((void **)&djobs, P * sizeof(FoldJob));
    if (e == hipSuccess) e = hipMalloc((void **)&douts, P * sizeof(FoldOut));
    if (e == hipSuccess) e = hipMalloc((void **)&dpicks, (size_t)std::max(nb, 1) * sizeof(Pick));
    auto release = [&] {
        if (djobs) (void)hipFree(djobs);
        if (douts) (void)hipFree(douts);
        if (dpicks) (void)hipFree(dpicks);
    };
    if (e != hipSuccess) {
        release();
        return herr(e);
    }
    std::vector<FoldJob> jobs(P);
    std::vector<int> firstb(P), cap_at(P, -1);
    std::vector<Pick> hpick((size_t)nb);
    std::vector<char> host_picked((size_t)nb, 0);
    int rc = 0;
    for (int r = 0, b = 0; r < P && !rc; b += cnt[r], ++r) {
        rc = rank[r].reserve(ncity, m.st);
        firstb[r] = b;
        jobs[r] = FoldJob{b, cnt[r], 0, 0, rank[r].p, dpicks + b};
    }
    std::vector<int> active(P);
    for (int r = 0; r < P; ++r) active[r] = r;
    std::vector<FoldOut> outs(P);
    while (!rc && !active.empty()) {
        std::vector<FoldJob> aj;
        for (int r : active) aj.push_back(jobs[r]);
        e = xcopy_async(djobs, aj.data(), aj.size() * sizeof(FoldJob), hipMemcpyHostToDevice, m.st);
        if (e == hipSuccess)
            hipLaunchKernelGGL(fold_persist_kernel, dim3((unsigned)aj.size()), dim3(kFoldThreads), 0, m.st, blocks, L,
                               m.eps2, djobs, douts);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = xcopy_async(outs.data(), douts, aj.size() * sizeof(FoldOut), hipMemcpyDeviceToHost, m.st);
        if (e == hipSuccess) e = hipStreamSynchronize(m.st);
        if (e != hipSuccess) {
            rc = herr(e);
            break;
        }
        std::vector<int> again;
        for (size_t q = 0; q < active.size() && !rc; ++q) {
            const int r = active[q];
            const FoldOut &o = outs[q];
            rank[r].len = (size_t)o.len;
            if (o.status == 0) continue;
            if (o.status == 2) {  // the path outgrew LDS: the per-merge kernels take over at merge o.at
                cap_at[r] = o.at;
                continue;
            }
            // several candidates: merge o.at exactly on the host, then relaunch
            std::vector<tspgpu_city> path((size_t)o.len), blk((size_t)L);
            e = xcopy_async(path.data(), rank[r].p, path.size() * sizeof(tspgpu_city), hipMemcpyDeviceToHost, m.st);
            if (e == hipSuccess)
                e = xcopy_async(blk.data(), blocks + (size_t)(firstb[r] + 1 + o.at) * L, L * sizeof(tspgpu_city),
                                   hipMemcpyDeviceToHost, m.st);
            if (e == hipSuccess) e = hipStreamSynchronize(m.st);
            if (e != hipSuccess) {
                rc = herr(e);
                break;
            }
            Cand pk{};
            rc = host_fold_merge(path, blk.data(), L, pk);
            if (rc) break;
            hpick[(size_t)firstb[r] + o.at].c = pk;
            host_picked[(size_t)firstb[r] + o.at] = 1;
            e = xcopy_async(rank[r].p, path.data(), path.size() * sizeof(tspgpu_city), hipMemcpyHostToDevice, m.st);
            if (e != hipSuccess) {
                rc = herr(e);
                break;
            }
            rank[r].len = path.size();
            jobs[r].k0 = o.at + 1;
            jobs[r].len = (int)path.size();
            if (jobs[r].k0 < cnt[r] - 1) again.push_back(r);
        }
        active.swap(again);
    }
    if (!rc) {
        // the logged picks -> exact costs in merge order (tsp.cpp:263)
        std::vector<Pick> dp((size_t)nb);
        e = xcopy_async(dp.data(), dpicks, dp.size() * sizeof(Pick), hipMemcpyDeviceToHost, m.st);
        if (e == hipSuccess) e = hipStreamSynchronize(m.st);
        rc = herr(e);
        for (int r = 0; r < P && !rc; ++r) {
            const int b0 = firstb[r];
            rcost[r] = costs[b0];
            const int done = cap_at[r] >= 0 ? cap_at[r] : cnt[r] - 1;
            for (int k = 0; k < done; ++k) {
                const size_t idx = (size_t)b0 + k;
                const Cand &c = host_picked[idx] ? hpick[idx].c : dp[idx].c;
                rcost[r] = (rcost[r] + costs[b0 + 1 + k]) + hswap(c.a, c.b, c.c, c.d);
            }
        }
        // the rest of an outgrown rank through the per-merge kernels
        for (int r = 0; r < P && !rc; ++r)
            for (int k = cap_at[r]; k >= 0 && k < cnt[r] - 1 && !rc; ++k)
                rc = m.merge(rank[r], tmp, &rcost[r], blocks + (size_t)(firstb[r] + 1 + k) * L, L,
                             &costs[firstb[r] + 1 + k], true);
    }
    if (!rc) rc = m.sync();  // (the picks buffer is freed below: nothing in flight may use it)
    (void)hipStreamSynchronize(m.st);
    release();
    return rc;
}

double bbox_diagonal(const tspgpu_city *c, size_t n)
{
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    for (size_t i = 0; i < n; ++i) {
        x0 = std::min(x0, c[i].x);
        x1 = std::max(x1, c[i].x);
        y0 = std::min(y0, c[i].y);
        y1 = std::max(y1, c[i].y);
    }
    if (!(x1 >= x0) || !(y1 >= y0)) return 0.0;
    return std::sqrt((x1 - x0) * (x1 - x0) + (y1 - y0) * (y1 - y0)) * (1.0 + 1e-9) + 1e-300;
}

bool finite_cities(const tspgpu_city *c, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        if (!std::isfinite(c[i].x) || !std::isfinite(c[i].y)) return false;
    return true;
}

}  // namespace

extern "C" {

int tspgpu_merge(tspgpu_ctx *ctx, const tspgpu_city *p1, int L1, double c1, const tspgpu_city *p2, int L2, double c2,
                 tspgpu_city *out, double *cost_out)
{
    if (!ctx || !p1 || !p2 || !out || !cost_out || L1 < 1 || L2 < 2) return -EINVAL;
    if (!finite_cities(p1, L1) || !finite_cities(p2, L2)) return -EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return -ENODEV;
    std::vector<tspgpu_city> all(p1, p1 + L1);
    all.insert(all.end(), p2, p2 + L2);
    Merger m;
    int rc = m.init(ctx, bbox_diagonal(all.data(), all.size()));
    DVec s, t, b;
    if (!rc) rc = s.reserve(L1, m.st);
    if (!rc) rc = t.reserve((size_t)L1 + L2, m.st);
    if (!rc) rc = b.reserve(L2, m.st);
    hipError_t e = hipSuccess;
    if (!rc) e = xcopy_async(s.p, p1, L1 * sizeof(tspgpu_city), hipMemcpyHostToDevice, m.st);
    if (!rc && e == hipSuccess) e = xcopy_async(b.p, p2, L2 * sizeof(tspgpu_city), hipMemcpyHostToDevice, m.st);
    if (!rc) rc = herr(e);
    s.len = L1;
    double cost = c1;
    if (!rc) rc = m.merge(s, t, &cost, b.p, L2, &c2);
    if (!rc) rc = m.sync();
    if (!rc) rc = herr(xcopy_async(out, s.p, s.len * sizeof(tspgpu_city), hipMemcpyDeviceToHost, m.st));
    if (!rc) rc = herr(hipStreamSynchronize(m.st));
    const int len = (int)s.len;
    s.release();
    t.release();
    b.release();
    if (rc) return rc;
    *cost_out = cost;
    return len;
}

int tspgpu_reduce(tspgpu_ctx *ctx, const tspgpu_city *paths, int L, const double *costs, int nblocks, int nprocs,
                  double *final_cost, char *log, int logcap)
{
    if (log && logcap > 0) log[0] = 0;
    if (!ctx || !paths || !costs || !final_cost) return -EINVAL;
    if (nblocks < 1 || nprocs < 1 || nblocks < nprocs || L < 2) return -EINVAL;
    const size_t ncity = (size_t)nblocks * L;
    if (!finite_cities(paths, ncity)) return -EINVAL;
    if (nblocks == 1) {  // one rank, one block: no fold, no tree (nothing to launch or load)
        *final_cost = costs[0];
        return 0;
    }
    std::lock_guard<std::mutex> g(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return -ENODEV;
    Merger m;
    int rc = m.init(ctx, bbox_diagonal(paths, ncity));
    if (rc) return rc;
    DVec blocks;
    rc = blocks.reserve(ncity, m.st);
    if (!rc) rc = herr(xcopy_async(blocks.p, paths, ncity * sizeof(tspgpu_city), hipMemcpyHostToDevice, m.st));
    if (!rc) rc = herr(hipStreamSynchronize(m.st));
    blocks.len = ncity;
    // distributeBlocks' counts (tsp.cpp:167-192): rank r gets #{b in [1,B] : b mod P == r}
    std::vector<int> cnt(nprocs, 0);
    for (int b = nblocks; b > 0; --b) cnt[b % nprocs]++;
    // one-kernel fold merges need block tours that close on their first city
    // and ids unique across blocks (the reference's generator numbers cities
    // globally); anything else takes the general path
    bool fold_ok = L >= 3;
    if (fold_ok) {
        std::vector<int> ids;
        ids.reserve((size_t)nblocks * (L - 1));
        for (int b = 0; b < nblocks && fold_ok; ++b) {
            const tspgpu_city *pb = paths + (size_t)b * L;
            if (pb[0].id != pb[L - 1].id) fold_ok = false;
            for (int k = 0; k < L - 1; ++k) ids.push_back(pb[k].id);
        }
        std::sort(ids.begin(), ids.end());
        if (fold_ok && std::adjacent_find(ids.begin(), ids.end()) != ids.end()) fold_ok = false;
    }
    // Every buffer a queued merge may touch is sized up front (a merged path
    // never exceeds all cities; a received list never exceeds all cities), so
    // nothing is reallocated while merges are in flight.
    std::vector<DVec> rank(nprocs), received(nprocs);
    DVec tmp;
    std::vector<double> rcost(nprocs, 0.0);
    if (!rc) rc = tmp.reserve(ncity, m.st);
    int next = 0;
    if (!rc && fold_ok && L <= kFoldL2 && tspgpu::tuned_or("K3_PERSIST", 1) != 0) {
        // (tuning knob K3_PERSIST = 0: the per-merge launches instead; tests compare both)
        // every rank's fold in one persistent launch (fold_persist_kernel)
        rc = persist_folds(m, blocks.p, L, costs, cnt, rank, tmp, rcost);
        next = nblocks;
    }
    for (int r = 0; r < nprocs && !rc && next < nblocks; ++r) {
        rc = rank[r].reserve(ncity, m.st);
        if (rc) break;
        rc = herr(xcopy_async(rank[r].p, blocks.p + (size_t)next * L, L * sizeof(tspgpu_city),
                                 hipMemcpyDeviceToDevice, m.st));
        rank[r].len = L;
        rcost[r] = costs[next];
        ++next;
        // each logical rank folds its contiguous block range left (tsp.cpp:348-352)
        for (int j = 1; j < cnt[r] && !rc; ++j, ++next)
            rc = m.merge(rank[r], tmp, &rcost[r], blocks.p + (size_t)next * L, L, &costs[next], fold_ok);
    }
    // MPI_ManualReduce (tsp.cpp:52-134): the receiver appends every received
    // path to one function-local list and merges with the WHOLE list
    // (tsp.cpp:67,93-98,115-120)
    std::string text;
    auto receive = [&](int to, int from) -> int {
        // the copy below reads rank[from]'s final path: every queued merge
        // (and any stall) must be resolved first
        int r2 = m.sync();
        if (r2) return r2;
        DVec &acc = received[to];
        const size_t add = rank[from].len;
        r2 = acc.reserve(std::max(acc.len + add, ncity), m.st);
        if (r2) return r2;
        r2 = herr(xcopy_async(acc.p + acc.len, rank[from].p, add * sizeof(tspgpu_city), hipMemcpyDeviceToDevice,
                                 m.st));
        if (r2) return r2;
        acc.len += add;
        return m.merge(rank[to], tmp, &rcost[to], acc.p, (int)acc.len, &rcost[from]);
    };
    const int lastpower = 1 << (int)std::log2((double)nprocs);
    for (int i = 0; i < nprocs - lastpower && !rc; ++i) {
        char line[128];
        std::snprintf(line, sizeof line, "process %i is about to receive %i cities from process %i\n", i,
                      (int)rank[i + lastpower].len, i + lastpower);  // tsp.cpp:88
        text += line;
        rc = receive(i, i + lastpower);
    }
    for (int d = 0; d < (int)std::log2((double)lastpower) && !rc; ++d)
        for (int k = 0; k < lastpower && !rc; k += 1 << (d + 1)) rc = receive(k, k + (1 << d));
    if (!rc) rc = m.sync();
    (void)hipStreamSynchronize(m.st);
    for (auto &v : rank) v.release();
    for (auto &v : received) v.release();
    tmp.release();
    blocks.release();
    if (rc) return rc;
    *final_cost = rcost[0];
    if (log && logcap > 0) {
        const size_t k = std::min(text.size(), (size_t)logcap - 1);
        std::memcpy(log, text.data(), k);
        log[k] = 0;
    }
    return 0;
}

}  // extern "C"
