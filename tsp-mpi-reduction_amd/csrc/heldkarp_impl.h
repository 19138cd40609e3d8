// Templates of the K1 Held-Karp kernels; instantiated per N in hk_n*.hip so the
// instantiations compile in parallel (see heldkarp.hip for the dispatch).
#pragma once
// K1 — batched exact Held-Karp for gfx950 (MI355X): kernel templates.
//
// Replaces the hot loop of the reference's per-block solver
// `BlockSolution tsp(vector<City>)` (tsp.cpp:405-509): the std::map subset DP
// with per-state path vectors becomes a dense, colex-ranked FP64 table that one
// workgroup sweeps layer by layer.
//
// Semantics kept bit-exact:
//   layer 1   G[{i}][i]  = d[0][i]
//   layer s   G[S][k]    = min_{m in S\k} G[S\k][m] + d[m][k]      (s >= 2)
//             layer 2 = d[0][i] + d[i][k], the reference's init (tsp.cpp:435;
//             IEEE add commutes); layers >= 3 start from INT_MAX like
//             tsp.cpp:453 (the host guarantees every candidate < INT_MAX).
//   closing   OPT = first strict min over m ascending of G[full][m] + d[m][0]
//   tour      backtracking with the SMALLEST m whose candidate equals the
//             state value == the reference's first strict-< argmin path.
// Only IEEE adds and min/compare touch the values: no FMA, no reassociation,
// distances come from the host (glibc pow), never recomputed here.
//
// Table layout per block, position-major ("SoA") inside each layer:
//   G[S][k], |S| = t, at  off(t) + pos(k in S) * C(N,t) + colexrank(S)
// so a wave that sweeps 64 consecutive source rows reads each position as one
// contiguous 512-B segment, and its scattered destination writes land ~4x
// denser in 64-B sectors than with row-major rows (tools/layout_sim.py).
// Every entry is written once and read once: 2*8*N*2^(N-1) bytes per block.
//
// Work split: layer t -> t+1 is one pass over the C(N,t) SOURCE rows T,
// compiled separately for every t (offsets, counts, row length are constants).
// A thread issues the t loads of its next row early (software pipelining into
// VGPRs), parks the current row in a thread-private LDS slot, sweeps the
// members m of T (d-row of m from LDS, N running minima acc[k] in VGPRs) and
// stores acc[k] for every k not in T to G[T+k][k] (its unique writer).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "heldkarp.h"
#include "wave.h"

namespace tspgpu {

constexpr int kBinomStride = kBinomCols;   // ints per binomial row, C(a,b) a<=20, b<=23
constexpr int kBinomBytesPadded = 2048;    // 21*24*4 = 2016 rounded to 16
constexpr double kIntMax = 2147483647.0;   // the reference's sentinel (tsp.cpp:411,453)

// Value type of the DP: f64 (the reference's distances) or i32 (the integer
// matrix extension; exact, half the table bytes, integer VALU ops).
template <typename V>
struct ValT;
template <>
struct ValT<double> {
    static constexpr double inf = 2147483647.0;  // INT_MAX, tsp.cpp:411,453
    static constexpr double invalid = 1.0e300;
    static constexpr int bytes = 8;
    __device__ static double vmin(double a, double b) { return fmin(a, b); }
};
template <>
struct ValT<int32_t> {
    static constexpr int32_t inf = 2147483647;
    static constexpr int32_t invalid = 2147483647;
    static constexpr int bytes = 4;
    __device__ static int32_t vmin(int32_t a, int32_t b) { return a < b ? a : b; }
};

__host__ __device__ constexpr int cbinom(int a, int b)
{
    if (b < 0 || b > a) return 0;
    long long r = 1;
    for (int i = 1; i <= b; ++i) r = r * (a - b + i) / i;
    return (int)r;
}
__host__ __device__ constexpr int layer_off(int N, int t)
{
    int o = 0;
    for (int u = 1; u < t; ++u) o += cbinom(N, u) * u;
    return o;
}
__host__ __device__ constexpr int mask_off(int N, int t)
{
    int o = 0;
    for (int u = 0; u < t; ++u) o += cbinom(N, u);
    return o;
}
// d row stride in doubles: >= N+1, even (16-B rows), and 2 mod 4 in 8-B units
// so distinct rows start on distinct 16-B bank groups (ds_read_b128).
__host__ __device__ constexpr int dist_stride(int N) { return ((N + 2) & ~1) + 2; }
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t dl_bytes(int N, int vb = 8) { return align16((size_t)(N + 1) * dist_stride(N) * vb); }
// only the digit groups N needs are staged in LDS
__host__ __device__ constexpr int rank_lut_ints(int N)
{
    return N <= 7 ? kRankR1 : (N <= 14 ? kRankR1 + kRankR2 : kRankLutInts);
}
__host__ __device__ constexpr int rank_lut_bytes(int N) { return (rank_lut_ints(N) * 4 + 15) & ~15; }
__host__ __device__ constexpr size_t layer_bytes(int N, int t, int vb = 8) { return (size_t)cbinom(N, t) * t * vb; }
__host__ __device__ constexpr size_t low_bytes(int N, int a, int vb = 8)
{
    size_t b = 0;
    for (int t = 1; t <= a; ++t) b += layer_bytes(N, t, vb);
    return b;
}
__host__ __device__ constexpr size_t high_bytes(int N, int a, int vb = 8)
{
    size_t b = 0;
    for (int t = N - a + 1; t <= N; ++t) b += layer_bytes(N, t, vb);
    return b;
}
__host__ __device__ constexpr size_t lds_base_bytes(int N, int vb = 8)
{
    return kBinomBytesPadded + dl_bytes(N, vb) + rank_lut_bytes(N);
}
// Compact global-table kernels keep the a smallest-index and the a
// largest-index layers (the smallest layers, e.g. 1-4 and 12-15 of N = 15) in
// LDS: a workgroup of THREADS threads gets THREADS/1024 of a CU's 160 KiB
// (the launch places 1024/THREADS workgroups per CU at most).  Those passes
// then neither touch HBM nor wait on global round trips.
__host__ __device__ constexpr int lds_end_layers(int N, int threads, int vb = 8)
{
    const size_t budget = (size_t)160 * 1024 * (size_t)threads / 1024;
    const size_t base = lds_base_bytes(N, vb) + 1024;
    if (budget <= base) return 0;
    int a = 0;
    while (2 * (a + 1) < N && low_bytes(N, a + 1, vb) + high_bytes(N, a + 1, vb) <= budget - base) ++a;
    return a;
}
// LDS: binomials | distance rows | rank LUT | table (LDS_TABLE) | end layers
// (compact global kernels) | per-thread row slots (member-sweep global kernels)
__host__ __device__ constexpr size_t lds_bytes(int N, bool lds_table, int threads, bool compact, int vb = 8)
{
    return lds_base_bytes(N, vb) +
           (lds_table ? ((size_t)N << (N - 1)) * vb
                      : (compact ? low_bytes(N, lds_end_layers(N, threads, vb), vb) +
                                       high_bytes(N, lds_end_layers(N, threads, vb), vb)
                                 : (size_t)(N - 1) * threads * 8));
}

// colex rank through the three-digit LUT (heldkarp.h)
template <int N>
__device__ __forceinline__ uint32_t lut_rank(uint32_t mask, const int *rl)
{
    const uint32_t lo = mask & 127u;
    int r = rl[lo];
    if constexpr (N > 7) r += rl[kRankR1 + ((mask >> 7) & 127u) * 8 + __builtin_popcount(lo)];
    if constexpr (N > 14) r += rl[kRankR1 + kRankR2 + (mask >> 14) * 15 + __builtin_popcount(mask & 0x3fffu)];
    return (uint32_t)r;
}

__device__ __forceinline__ int colex_rank(uint32_t mask, const int *binom)
{
    int rank = 0, j = 0;
    while (mask) {
        const int b = __builtin_ctz(mask);
        rank += binom[b * kBinomStride + j + 1];
        ++j;
        mask &= mask - 1u;
    }
    return rank;
}

// minimum over the wave (all 64 lanes active): DPP row reduction + readlane (wave.h)
template <typename V>
__device__ __forceinline__ V wave_min(V v)
{
    return wave_min_dpp(v);
}

// dl row m holds d[m][1..N] at [0, N) and d[m][0] at N: the N values a row
// sweep needs start 16-B aligned.
template <int N, typename V>
__device__ __forceinline__ V dget(const V *dl, int m, int k)
{
    return dl[m * dist_stride(N) + (k == 0 ? N : k - 1)];
}

// Global table access through a buffer resource (SRSRC): 32-bit offsets in
// one VGPR instead of 64-bit pointers, and the hardware range check turns
// any out-of-slot index into a dropped access instead of a fault.
template <typename V>
struct GlobalTableT;
template <>
struct GlobalTableT<int32_t> {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ int32_t load(uint32_t idx) const
    {
        return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(idx * 4u), 0, 0);
    }
    __device__ __forceinline__ void store(uint32_t idx, int32_t v) const
    {
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, rs, (int)(idx * 4u), 0, 0);
    }
};
// cache-policy bits of the table value loads (development knob)
#ifndef TSPGPU_VAL_LOAD_AUX
#define TSPGPU_VAL_LOAD_AUX 0
#endif
template <>
struct GlobalTableT<double> {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ double load(uint32_t idx) const
    {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(idx * 8u), 0,
                                                                               TSPGPU_VAL_LOAD_AUX));
    }
    // a store at an offset past num_records is dropped by the buffer range
    // check: predication without a branch
    __device__ __forceinline__ void store_if(bool pred, uint32_t idx, double v) const
    {
        using u2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
        const int off = pred ? (int)(idx * 8u) : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rs, off, 0, 0);
    }
    __device__ __forceinline__ void store(uint32_t idx, double v) const
    {
        using u2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rs, (int)(idx * 8u), 0, 0);
    }
};
using GlobalTable = GlobalTableT<double>;
template <typename V>
struct LdsTableT {
    V *p;
    uint32_t base = 0;  // table index of p[0]
    __device__ __forceinline__ V load(uint32_t idx) const { return p[idx - base]; }
    __device__ __forceinline__ void store_if(bool pred, uint32_t idx, V v) const
    {
        if (pred) p[idx - base] = v;
    }
    __device__ __forceinline__ void store(uint32_t idx, V v) const { p[idx - base] = v; }
};
using LdsTable = LdsTableT<double>;

// Ping-pong value layout (VAR 4): a middle layer t lives in buffer t & 1 at
// the start of the slot instead of its own span, so the two live layers of
// all resident workgroups stay in the Infinity Cache and are rewritten there
// (1.4x at n = 16, profiles/r01/k1_pingpong_experiment.log); the backtracking
// then follows the parent bytes stored by the forward pass instead of the
// values.  Logical indices stay those of the compact layout.
template <typename V, long SHIFT>
struct ShiftTable {
    GlobalTableT<V> g;
    __device__ __forceinline__ V load(uint32_t idx) const { return g.load((uint32_t)((long)idx - SHIFT)); }
    __device__ __forceinline__ void store(uint32_t idx, V v) const { g.store((uint32_t)((long)idx - SHIFT), v); }
};
// largest layer of one parity (odd layers share buffer 0, even ones buffer 1)
__host__ __device__ constexpr uint32_t max_layer_elems(int N, int parity)
{
    uint32_t m = 0;
    for (int t = 1; t <= N; ++t)
        if ((t & 1) == parity) m = m > cbinom(N, t) * t ? m : cbinom(N, t) * t;
    return m;
}
// byte offset of the parent bytes in a VAR-4 slot (behind the two buffers,
// each sized for its own parity: 0.77 MB instead of 0.82 MB live at n = 16)
template <typename V>
__host__ __device__ constexpr uint32_t parent_base(int N)
{
    return (max_layer_elems(N, 1) + max_layer_elems(N, 0)) * (uint32_t)sizeof(V);
}
// Parents (N <= 15): for every SOURCE row T of layer t, one 64-bit word
// holding, per non-member k of T (q-th non-member, 4 bits at 4q), m - 1 for
// the city m of the first strict minimum over m ascending (tsp.cpp:457-471)
// of destination (T+k, k).  One coalesced 8-byte store per row (consecutive
// threads own consecutive rows) instead of N - t scattered bytes; word index
// = the row's place in the colex mask list (mask_off(N, t) + rank).
// Cache-policy bits of the parent-word stores (aux: 2 = nt, 16 = sc1).  The
// words are read back only by the backtracking (N - 1 loads per block), so
// they are stored non-temporal: the ping-pong values keep the Infinity Cache.
// n = 16, 16384 blocks, 3 interleaved runs each: nt 12.39-12.40 ms, default
// policy 13.3-14.3 ms, sc1 13.6 ms (profiles/r01/k1_parent_policy_n16.log).
#ifndef TSPGPU_PAR_AUX
#define TSPGPU_PAR_AUX 2
#endif
struct ParentTable {
    static constexpr bool on = true;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t base;
    __device__ __forceinline__ void store(uint32_t widx, uint64_t w) const
    {
        using u2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, w), rs, (int)(base + widx * 8u), 0,
                                              TSPGPU_PAR_AUX);
    }
    __device__ __forceinline__ uint64_t load(uint32_t widx) const
    {
        return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(base + widx * 8u), 0, 0));
    }
};
struct NoParents {
    static constexpr bool on = false;
    __device__ __forceinline__ void store(uint32_t, uint64_t) const {}
};

// The table of a compact global kernel: layers 1..A and N-A+1..N in LDS, the
// rest in the workgroup's HBM slot (same indices everywhere).
template <typename V, int N, int A, bool PP = false>
struct SplitTable {
    GlobalTableT<V> g;
    V *lo, *hi;
    template <int t>
    __device__ __forceinline__ auto layer() const
    {
        if constexpr (A > 0 && t <= A)
            return LdsTableT<V>{lo, 0u};
        else if constexpr (A > 0 && t >= N - A + 1)
            return LdsTableT<V>{hi, (uint32_t)layer_off(N, N - A + 1)};
        else if constexpr (PP)
            return ShiftTable<V, (long)layer_off(N, t) - ((t & 1) ? 0L : (long)max_layer_elems(N, 1))>{g};
        else
            return g;
    }
    __device__ __forceinline__ V get(int t, uint32_t idx) const
    {
        if (A > 0 && t <= A) return lo[idx];
        if (A > 0 && t >= N - A + 1) return hi[idx - layer_off(N, N - A + 1)];
        return g.load(idx);
    }
};

// acc[k] = min(acc[k], g + d[m][k+1]) for all k: one member of the source row.
template <int N>
__device__ __forceinline__ void relax_member(double (&acc)[N], const double *dl, int m, double g)
{
    const double2 *drow = reinterpret_cast<const double2 *>(__builtin_assume_aligned(dl + m * dist_stride(N), 16));
#pragma unroll
    for (int q = 0; q < N / 2; ++q) {
        const double2 v = drow[q];
        acc[2 * q] = fmin(acc[2 * q], g + v.x);
        acc[2 * q + 1] = fmin(acc[2 * q + 1], g + v.y);
    }
    if constexpr (N & 1) acc[N - 1] = fmin(acc[N - 1], g + dl[m * dist_stride(N) + N - 1]);
}

// Store acc[k] for every k not in Tm at G[Tm+k][k] of layer S = T+1.
// colex rank of T+{k} (e_i = members ascending, p = #members below k):
//   sum_{i<p} C(e_i,i+1) + C(k,p+1) + sum_{i>=p} C(e_i,i+2)
//   = r - s1 + C(k,p+1) + s2, with s1/s2 the suffix sums of C(e_i,i+1) /
// C(e_i,i+2) over the members above k, built while k runs downwards.
// Branch-free: two binomial lookups per k and a predicated store.
template <int N, int S, typename Tab>
__device__ __forceinline__ void scatter_row(const Tab &tab, const double (&acc)[N], uint32_t Tm, uint32_t r,
                                            const int *binom)
{
    constexpr int T = S - 1;
    constexpr uint32_t ROWS_S = cbinom(N, S);
    constexpr uint32_t DST = layer_off(N, S);
    int q = 0, s1 = 0, s2 = 0;
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
        const int in = (Tm >> k) & 1u;
        const int p = T - q - in;
        const int c1 = binom[k * kBinomStride + p + 1];
        const int c2 = binom[k * kBinomStride + p + 2];
        const uint32_t rank = r - (uint32_t)s1 + (uint32_t)c1 + (uint32_t)s2;
        tab.store_if(!in, DST + (uint32_t)p * ROWS_S + rank, acc[k]);
        s1 += in ? c1 : 0;
        s2 += in ? c2 : 0;
        q += in;
    }
}

// Global table: layer T -> T+1, rows r = tid, tid+THREADS, ...; the next row's
// t loads are in flight while the current row is swept.
template <int N, int T, int THREADS>
__device__ __forceinline__ void layer_pass_global(const GlobalTable &tab, const double *__restrict__ dl,
                                                  const int *__restrict__ binom, double *__restrict__ slot,
                                                  const uint32_t *__restrict__ masks, uint32_t tid)
{
    constexpr int S = T + 1;
    constexpr uint32_t ROWS = cbinom(N, T);
    constexpr uint32_t SRC = layer_off(N, T);
    const uint32_t *mt = masks + mask_off(N, T);
    uint32_t r = tid;
    if (r >= ROWS) return;
    double nxt[T];
    uint32_t nmask = mt[r];
#pragma unroll
    for (int j = 0; j < T; ++j) nxt[j] = tab.load(SRC + j * ROWS + r);
    for (; r < ROWS; r += THREADS) {
        const uint32_t Tm = nmask;
#pragma unroll
        for (int j = 0; j < T; ++j) slot[j * THREADS] = nxt[j];
        const uint32_t rn = r + THREADS;
        if (rn < ROWS) {
            nmask = mt[rn];
#pragma unroll
            for (int j = 0; j < T; ++j) nxt[j] = tab.load(SRC + j * ROWS + rn);
        }
        double acc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k] = kIntMax;
        uint32_t bits = Tm;
#pragma unroll 2
        for (int j = 0; j < T; ++j) {
            const int m = __builtin_ctz(bits) + 1;
            bits &= bits - 1u;
            relax_member<N>(acc, dl, m, slot[j * THREADS]);
        }
        scatter_row<N, S>(tab, acc, Tm, r, binom);
    }
}

// LDS table: the source row is read straight from the table.
template <int N, int T, int THREADS>
__device__ __forceinline__ void layer_pass_lds(const LdsTable &tab, const double *__restrict__ dl,
                                               const int *__restrict__ binom, const uint32_t *__restrict__ masks,
                                               uint32_t tid)
{
    constexpr int S = T + 1;
    constexpr uint32_t ROWS = cbinom(N, T);
    constexpr uint32_t SRC = layer_off(N, T);
    const uint32_t *mt = masks + mask_off(N, T);
    for (uint32_t r = tid; r < ROWS; r += THREADS) {
        const uint32_t Tm = mt[r];
        double acc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k] = kIntMax;
        uint32_t bits = Tm;
#pragma unroll 2
        for (int j = 0; j < T; ++j) {
            const int m = __builtin_ctz(bits) + 1;
            bits &= bits - 1u;
            relax_member<N>(acc, dl, m, tab.load(SRC + j * ROWS + r));
        }
        scatter_row<N, S>(tab, acc, Tm, r, binom);
    }
}

// Compact pass, layer T -> T+1: a thread owns source rows r = tid, tid+THREADS,
// ... and relaxes ONLY the Q = N-T destinations k not in T (every row of a
// layer has exactly Q of them, so the loops have static trip counts):
//   acc[q] = min_j g[j] + d[m_j][k_q]           (m_j: j-th member, k_q: q-th non-member)
//   G[T+k_q][k_q] = acc[q]  at  DST + (k_q - q) * C(N,T+1) + colexrank(T + k_q)
// (k_q - q = number of members below k_q = position of k_q in T+k_q).
// t*(N-t) relaxations per row instead of t*N for the member sweep: no lane
// computes a value that is thrown away.  Registers: t + 2(N-t) + O(1) per
// thread, so the kernel runs at 8 waves/SIMD without spilling.
// PF (prefetch depth): the masks and t values of the next PF rows are in
// flight while the current row is relaxed (software pipelining, 2t VGPRs per row).
#ifndef TSPGPU_K1_SELMIN
#define TSPGPU_K1_SELMIN 0  // development knob: argmin pass keeps the minimum by select, not v_min_f64
#endif
template <typename V, int N, int T, int THREADS, int PF, typename SrcTab, typename DstTab, typename PTab = NoParents>
__device__ __forceinline__ void layer_pass_compact(const SrcTab &src, const DstTab &dst, const V *__restrict__ dl,
                                                   const int *__restrict__ rl, const uint32_t *__restrict__ masks,
                                                   uint32_t tid, const PTab &par = PTab{})
{
    constexpr int S = T + 1;
    constexpr int Q = N - T;
    constexpr int DS = dist_stride(N);
    constexpr uint32_t ROWS = cbinom(N, T);
    constexpr uint32_t ROWS_S = cbinom(N, S);
    constexpr uint32_t SRC = layer_off(N, T);
    constexpr uint32_t DST = layer_off(N, S);
    constexpr uint32_t FULL = (1u << N) - 1u;
    const uint32_t *mt = masks + mask_off(N, T);
    uint32_t m1 = 0, m2 = 0;
    V g1[T], g2[T];
    if constexpr (PF >= 1) {
        if (tid < ROWS) {
            m1 = mt[tid];
#pragma unroll
            for (int j = 0; j < T; ++j) g1[j] = src.load(SRC + j * ROWS + tid);
        }
    }
    if constexpr (PF >= 2) {
        if (tid + THREADS < ROWS) {
            m2 = mt[tid + THREADS];
#pragma unroll
            for (int j = 0; j < T; ++j) g2[j] = src.load(SRC + j * ROWS + tid + THREADS);
        }
    }
    for (uint32_t r = tid; r < ROWS; r += THREADS) {
        uint32_t Tm;
        V g[T];
        if constexpr (PF == 0) {
            Tm = mt[r];
#pragma unroll
            for (int j = 0; j < T; ++j) g[j] = src.load(SRC + j * ROWS + r);
        } else {
            Tm = m1;
#pragma unroll
            for (int j = 0; j < T; ++j) g[j] = g1[j];
            if constexpr (PF >= 2) {
                m1 = m2;
#pragma unroll
                for (int j = 0; j < T; ++j) g1[j] = g2[j];
            }
            const uint32_t rn = r + PF * THREADS;
            if (rn < ROWS) {
                if constexpr (PF >= 2) {
                    m2 = mt[rn];
#pragma unroll
                    for (int j = 0; j < T; ++j) g2[j] = src.load(SRC + j * ROWS + rn);
                } else {
                    m1 = mt[rn];
#pragma unroll
                    for (int j = 0; j < T; ++j) g1[j] = src.load(SRC + j * ROWS + rn);
                }
            }
        }
        uint32_t kb[Q];
        uint32_t nb = ~Tm & FULL;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            kb[q] = __builtin_ctz(nb);
            nb &= nb - 1u;
        }
        V acc[Q];
        uint32_t arg[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            acc[q] = ValT<V>::inf;
            arg[q] = 0;
        }
        uint32_t bits = Tm;
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int m = __builtin_ctz(bits) + 1;
            bits &= bits - 1u;
            const V *drow = dl + m * DS;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const V cnd = g[j] + drow[kb[q]];
                if constexpr (PTab::on) {
                    // first strict minimum over m ascending (tsp.cpp:465): the parent
#if TSPGPU_K1_SELMIN
                    const bool lt = cnd < acc[q];
                    arg[q] = lt ? (uint32_t)m : arg[q];
                    acc[q] = lt ? cnd : acc[q];
#else
                    arg[q] = cnd < acc[q] ? (uint32_t)m : arg[q];
                    acc[q] = ValT<V>::vmin(acc[q], cnd);
#endif
                } else {
                    acc[q] = ValT<V>::vmin(acc[q], cnd);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t k = kb[q];
            const uint32_t rank = lut_rank<N>(Tm | (1u << k), rl);
            dst.store(DST + (k - (uint32_t)q) * ROWS_S + rank, acc[q]);
        }
        if constexpr (PTab::on) {
            uint64_t w = 0;
#pragma unroll
            for (int q = 0; q < Q; ++q) w |= (uint64_t)((arg[q] - 1u) & 15u) << (4 * q);  // no argmin -> 15
            par.store(mask_off(N, T) + r, w);
        }
    }
}

template <typename V, int N, int T, int THREADS, int PF, typename Tab>
__device__ __forceinline__ void all_layers_compact(const Tab &tab, const V *dl, const int *rl,
                                                   const uint32_t *masks, uint32_t tid)
{
    if constexpr (T < N) {
        layer_pass_compact<V, N, T, THREADS, PF>(tab, tab, dl, rl, masks, tid);
        __syncthreads();
        all_layers_compact<V, N, T + 1, THREADS, PF>(tab, dl, rl, masks, tid);
    }
}
template <typename V, int N, int A, int T, int THREADS, int PF, bool PP, typename PTab>
__device__ __forceinline__ void all_layers_split(const SplitTable<V, N, A, PP> &tb, const V *dl, const int *rl,
                                                 const uint32_t *masks, uint32_t tid, const PTab &par)
{
    if constexpr (T < N) {
        layer_pass_compact<V, N, T, THREADS, PF>(tb.template layer<T>(), tb.template layer<T + 1>(), dl, rl, masks,
                                                 tid, par);
        __syncthreads();
        all_layers_split<V, N, A, T + 1, THREADS, PF>(tb, dl, rl, masks, tid, par);
    }
}

template <int N, int T, int THREADS, typename Tab>
__device__ __forceinline__ void all_layers(const Tab &tab, const double *dl, const int *binom, double *slot,
                                           const uint32_t *masks, uint32_t tid)
{
    if constexpr (T < N) {
        if constexpr (std::is_same<Tab, LdsTable>::value)
            layer_pass_lds<N, T, THREADS>(tab, dl, binom, masks, tid);
        else
            layer_pass_global<N, T, THREADS>(tab, dl, binom, slot, masks, tid);
        __syncthreads();
        all_layers<N, T + 1, THREADS>(tab, dl, binom, slot, masks, tid);
    }
}

// One workgroup solves blocks blockIdx.x, blockIdx.x + gridDim.x, ...
// LDS_TABLE: the whole compact table lives in LDS (N <= 11), else in the
// workgroup's global slot.  COMPACT selects the layer pass (see above).
// Occupancy target (waves per SIMD): the member sweep holds N running minima
// plus a prefetched row (<= 128 VGPRs, 4 waves); the compact pass needs about
// half of that (<= 64 VGPRs, 8 waves) at the reference's sizes.
// VAR: 0 member sweep, 1 compact, 2 compact + next-row prefetch, 3 compact + two rows prefetched,
// 4 = 2 + ping-pong values + parent bytes
#ifndef TSPGPU_K1_V4_PF
#define TSPGPU_K1_V4_PF 1  // rows prefetched by the variant-4 pass
#endif
__host__ __device__ constexpr int var_pf(int var) { return var == 4 ? TSPGPU_K1_V4_PF : var - 1; }
// The 512-thread variant-4 kernels (the n = 16 default: one workgroup per CU)
// target 2 waves/SIMD, i.e. up to 256 VGPRs: 171 used, the LDS reads of a row
// overlap instead of one round trip per relaxation, and SGPR spills fall from
// 207 to 69; 11.85 ms vs 12.44 ms for 1024 threads at 4 waves/SIMD
// (profiles/r01/k1_512x2_n16.log).
#ifndef TSPGPU_K1_WAVES_512V4
#define TSPGPU_K1_WAVES_512V4 2
#endif
__host__ __device__ constexpr int min_waves(int N, int var, int threads = 0)
{
    return (TSPGPU_K1_WAVES_512V4 > 0 && threads == 512 && var == 4) ? TSPGPU_K1_WAVES_512V4
           : var == 1                                               ? (N <= 15 ? 8 : 4)
                                                                    : (N <= 15 ? 4 : 2);
}
template <typename V, int N, bool LDS_TABLE, int THREADS, int VAR>
__global__ __launch_bounds__(THREADS, min_waves(N, VAR, THREADS)) void heldkarp_kernel(
    const V *__restrict__ dist, int nblocks, V *__restrict__ slots, size_t slot_doubles,
    const uint32_t *__restrict__ masks, const LayerInfo *__restrict__ info, V *__restrict__ cost_out,
    int32_t *__restrict__ tour_out)
{
    constexpr int n = N + 1;
    constexpr int DS = dist_stride(N);
    constexpr int VB = ValT<V>::bytes;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int *binom = reinterpret_cast<int *>(smem);
    V *dl = reinterpret_cast<V *>(smem + kBinomBytesPadded);
    int *rl = reinterpret_cast<int *>(smem + kBinomBytesPadded + dl_bytes(N, VB));
    V *lds_rest = reinterpret_cast<V *>(smem + kBinomBytesPadded + dl_bytes(N, VB) + rank_lut_bytes(N));
    const int tid = threadIdx.x;

    for (int i = tid; i < kBinomRows * kBinomStride; i += THREADS) binom[i] = info->binom[i];
    for (int i = tid; i < rank_lut_ints(N); i += THREADS) rl[i] = info->rlut[i];

    V *tab;
    if constexpr (LDS_TABLE)
        tab = lds_rest;
    else
        tab = slots + (size_t)blockIdx.x * slot_doubles;
    using Tab = typename std::conditional<LDS_TABLE, LdsTableT<V>, GlobalTableT<V>>::type;
    // compact global kernels: the end layers live in LDS behind the LUT
    constexpr int A = (!LDS_TABLE && VAR >= 1) ? lds_end_layers(N, THREADS, VB) : 0;
    constexpr bool PP = VAR == 4 && !LDS_TABLE;
    SplitTable<V, N, A, PP> tb;
    tb.lo = lds_rest;
    tb.hi = lds_rest + low_bytes(N, A, VB) / VB;
    Tab th;
    if constexpr (LDS_TABLE) {
        th.p = tab;
    } else {
        // descriptor inputs made provably wave-uniform (readfirstlane), else
        // hipcc wraps every buffer op in a waterfall loop (guide T20)
        const uint64_t base = reinterpret_cast<uint64_t>(tab);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
        const int bytes = __builtin_amdgcn_readfirstlane((int)(slot_doubles * VB));
        th.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, bytes,
                                                  0x00020000);
        tb.g = th;
    }
    ParentTable par{};
    if constexpr (PP) {
        par.rs = th.rs;
        par.base = parent_base<V>(N);
    }
    // table entry (layer t, index idx) wherever it lives
    auto tget = [&](int t, uint32_t idx) -> V {
        if constexpr (LDS_TABLE)
            return tab[idx];
        else if constexpr (A > 0)
            return tb.get(t, idx);
        else
            return tab[idx];
    };

    for (int blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
        const V *dsrc = dist + (size_t)blk * n * n;
        for (int i = tid; i < n * n; i += THREADS) {
            const int row = i / n, col = i % n;
            dl[row * DS + (col == 0 ? N : col - 1)] = dsrc[i];
        }
        __syncthreads();

        // layer 1: G[{i}][i] = d[0][i]; colex rank of {i} is i-1, position 0
        if (tid < N) {
            if constexpr (A > 0)
                tb.lo[tid] = dget<N>(dl, 0, tid + 1);
            else
                tab[tid] = dget<N>(dl, 0, tid + 1);
        }
        __syncthreads();

        // Opaque per-block copies: keeps the compiler from hoisting every
        // layer's per-thread addresses out of the block loop (that LICM alone
        // costs ~200 VGPRs of 64-bit pointers).
        int tid_b = tid;
        asm volatile("" : "+v"(tid_b));
        if constexpr (PP)
            all_layers_split<V, N, A, 1, THREADS, var_pf(VAR)>(tb, dl, rl, masks, (uint32_t)tid_b, par);
        else if constexpr (!LDS_TABLE && VAR >= 1)
            all_layers_split<V, N, A, 1, THREADS, var_pf(VAR)>(tb, dl, rl, masks, (uint32_t)tid_b, NoParents{});
        else if constexpr (VAR >= 1)
            all_layers_compact<V, N, 1, THREADS, var_pf(VAR)>(th, dl, rl, masks, (uint32_t)tid_b);
        else if constexpr (std::is_same<V, double>::value)
            all_layers<N, 1, THREADS>(th, dl, binom, lds_rest + tid_b, masks, (uint32_t)tid_b);

        // closing min (tsp.cpp:483-499) and backtracking, one wave: lane m-1
        // holds candidate m.  The state value of the next step is the g value
        // the picked lane loaded, so each step costs one dependent load.
        if (PP && tid < 64) {
            // closing min as below; the tour follows the parent bytes
            const int lane = tid;
            const int m = lane + 1;
            const bool valid = m <= N;
            const V glast = valid ? tb.template layer<N>().load(layer_off(N, N) + (uint32_t)(m - 1)) : V(0);
            const V cand = valid ? glast + dget<N>(dl, m, 0) : ValT<V>::invalid;
            const V best = ValT<V>::vmin(wave_min(cand), ValT<V>::inf);
            const unsigned long long hit = __ballot(valid && cand == best && cand < ValT<V>::inf);
            const int bestM = hit ? __ffsll(hit) : 0;
            if (lane == 0) {
                int32_t *tour = tour_out + (size_t)blk * (n + 1);
                uint32_t S = (1u << N) - 1u;
                int k = bestM;
                bool ok = true;
                for (int pos = n - 2; bestM && ok && pos >= 1; --pos) {
                    // parent word of the source row T = S \ k (layer |S| - 1), nibble of k
                    const uint32_t T = S & ~(1u << (k - 1));
                    const int tt = __builtin_popcount(T);
                    const int q = (k - 1) - __builtin_popcount(T & ((1u << (k - 1)) - 1u));
                    const uint64_t w = par.load((uint32_t)info->moff[tt] + lut_rank<N>(T, rl));
                    const int pm = (int)((w >> (4 * q)) & 15u) + 1;
                    // a parent outside T (only from unvalidated input whose every
                    // candidate reached INT_MAX) ends the walk with cost -1, like variant 2
                    ok = pm <= N && ((T >> (pm - 1)) & 1u);
                    tour[pos] = ok ? pm : 0;
                    S &= ~(1u << (k - 1));
                    k = pm;
                }
                tour[0] = 0;
                tour[n - 1] = bestM;
                tour[n] = 0;
                cost_out[blk] = (bestM && ok) ? best : V(-1);
            }
        } else if (tid < 64) {
            const int lane = tid;
            const int m = lane + 1;
            const uint32_t full = (1u << N) - 1u;
            const bool valid = m <= N;
            // the last layer is one row: position m-1 at m-1
            const V glast = valid ? tget(N, layer_off(N, N) + (uint32_t)(m - 1)) : V(0);
            const V cand = valid ? glast + dget<N>(dl, m, 0) : ValT<V>::invalid;
            const V best = ValT<V>::vmin(wave_min(cand), ValT<V>::inf);
            const unsigned long long hit = __ballot(valid && cand == best && cand < ValT<V>::inf);
            const int bestM = hit ? __ffsll(hit) : 0;
            int32_t *tour = tour_out + (size_t)blk * (n + 1);
            uint32_t S = full;
            int k = bestM;
            int pos = n - 2;
            bool ok = bestM != 0;
            V target = __shfl(glast, ok ? bestM - 1 : 0);
            while (ok && __builtin_popcount(S) >= 2) {
                const uint32_t T = S & ~(1u << (k - 1));
                const int tt = __builtin_popcount(T);
                const uint32_t rT = lut_rank<N>(T, rl);
                const bool inT = valid && ((T >> (m - 1)) & 1u);
                V gv = V(0), c = V(0);
                if (inT) {
                    gv = tget(tt, info->off[tt] + __builtin_popcount(T & ((1u << (m - 1)) - 1u)) * info->count[tt] + rT);
                    c = gv + dget<N>(dl, m, k);
                }
                const unsigned long long bb = __ballot(inT && c == target);
                const int pick = bb ? __ffsll(bb) : 0;
                ok = pick != 0;
                if (lane == 0) tour[pos] = pick;
                target = __shfl(gv, ok ? pick - 1 : 0);
                --pos;
                S = T;
                k = pick;
            }
            if (lane == 0) {
                tour[0] = 0;
                tour[n - 1] = bestM;
                tour[n] = 0;
                cost_out[blk] = ok ? best : V(-1);  // -1: no predecessor matched (never expected)
            }
        }
        __syncthreads();
    }
}

template <typename V, int N, bool LDS, int THREADS, int VAR>
hipError_t launch_n(const LaunchArgs &a, int grid)
{
    const size_t lds = lds_bytes(N, LDS, THREADS, VAR >= 1, ValT<V>::bytes);
    if (lds > 64 * 1024) {
        static bool raised = false;  // once per instantiation
        if (!raised) {
            hipError_t e = hipFuncSetAttribute(
                reinterpret_cast<const void *>(&heldkarp_kernel<V, N, LDS, THREADS, VAR>),
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            raised = true;
        }
    }
    hipLaunchKernelGGL((heldkarp_kernel<V, N, LDS, THREADS, VAR>), dim3(grid), dim3(THREADS), lds, a.stream,
                       static_cast<const V *>(a.dist), a.nblocks, static_cast<V *>(a.slots), a.slot_doubles, a.masks,
                       a.info, static_cast<V *>(a.cost), a.tour);
    return hipGetLastError();
}

// Workgroup size of the LDS-table kernels: the whole table of N=11 (88 KiB)
// admits one workgroup per CU, so it gets 1024 threads (4 waves per SIMD).
__host__ __device__ constexpr int lds_table_threads(int N) { return N >= 11 ? 1024 : 256; }

template <typename V, int N, int VAR>
hipError_t launch_threads_v(const LaunchArgs &a, int grid)
{
    if constexpr (N <= kLdsTableMaxN) {
        if (a.use_lds) return launch_n<V, N, true, lds_table_threads(N), VAR >= 2 ? 1 : VAR>(a, grid);
    }
    if constexpr (VAR == 4 && (N < 11 || N > 15)) {
        // ping-pong + parent words: 12..16 cities (4-bit parents, <= 14 per row)
        return launch_n<V, N, false, 256, 2>(a, grid);
    } else {  // (else: no unreachable variant-4 kernel is instantiated)
        if constexpr (N >= 12 && N <= 15) {
            if (a.threads == 512) return launch_n<V, N, false, 512, VAR>(a, grid);
            if (a.threads == 1024) return launch_n<V, N, false, 1024, VAR>(a, grid);
        }
        return launch_n<V, N, false, 256, VAR>(a, grid);
    }
}

template <int N>
hipError_t launch_threads(const LaunchArgs &a, int grid)
{
    // integer matrices: the default (compact + prefetch) pass only
    if (a.vbytes == 4)
        return a.variant >= 4 ? launch_threads_v<int32_t, N, 4>(a, grid) : launch_threads_v<int32_t, N, 2>(a, grid);
    // (VAR 3, two rows in flight, measured no faster than one: not instantiated)
    if (a.variant >= 4) return launch_threads_v<double, N, 4>(a, grid);
    if (a.variant >= 2) return launch_threads_v<double, N, 2>(a, grid);
    return a.variant == 1 ? launch_threads_v<double, N, 1>(a, grid) : launch_threads_v<double, N, 0>(a, grid);
}

}  // namespace tspgpu
