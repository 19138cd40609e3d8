// K1 variant 5 — "sub-cube" tiled Held-Karp for gfx950 (MI355X).
//
// Same recurrence, same IEEE operations and the same first-strict-minimum
// argmin as heldkarp_impl.h (tsp.cpp:424-499), so the same cost and tour bits;
// only the order in which DP entries are produced and where they live change.
//
// Split the N inner cities into L "low" ones (bits 0..L-1) and H = N-L "high"
// ones.  A state mask S = h<<L | l has a high part h (H bits) and a low part l.
// The transition G[S\k][m] -> G[S][k] adds ONE city k:
//   * k low:  S\k has the same high part h          -> stays in sub-cube h
//   * k high: S\k has high part h\k (a smaller one) -> crosses sub-cubes
// So the DP can run sub-cube by sub-cube (h = 0, 1, ..., 2^H-1: every h\k is
// done before h), and inside a sub-cube layer by layer over |l| = j.  The
// entries G[S][m] with m LOW never leave the workgroup's LDS (only the two
// live low layers of the current sub-cube are kept: 20 KB at L = 10); only
// the entries with m HIGH go through memory, written once by sub-cube h\m
// ("push", coalesced: same row index l on both sides) and read once by
// sub-cube h.  At n = 16 with the default L = 10 (N = 15, H = 5) that is
// 81,920 of the block's 245,760 entries: 1.31 MB of table traffic per block
// instead of 3.93 MB (SURVEY.md §8(d)'s compulsory bytes of the
// layer-by-layer form).
//
// Row-owner pass (h, j): a thread owns a source row T = h<<L | l, |l| = j,
// t = |h|+j members, Q = N-t non-members; for every non-member k it computes
//   acc[k] = min over members m of G[T][m] + d[m][k]
// (the values of tsp.cpp:457-470) and stores acc[k] to the next LDS layer (k
// low) or to the push area of sub-cube h|k (k high).  The argmin (the
// reference's first strict minimum over members ascending) is kept only for
// the top rows (>= N - TSPGPU_TILED_TA_OFF members: one 64-bit word of 4-bit
// parents per row); everywhere else the pass is min-only — two VALU
// instructions per relaxation instead of four.  The backtracking kernel
// (hk_tiled_backtrack, one wave per block, all blocks at once) follows the
// parent words down to that size, then recomputes the few rows the path still
// needs from the block's pushed values (only subsets of the path's row, 2-8%
// of the forward relaxations) and takes the same first strict minimum of the
// same candidates — so the same tour bits.  At n = 16: 7.4 ms forward + 0.7 ms
// backtracking per 16384 blocks, against 9.6 ms with the argmin everywhere
// (profiles/r02/k1_argmin_threshold.txt).
//
// Distances: the N x N inner matrix in LDS with an odd row stride
// (kTiledDS = 19 entries), optionally replicated R times (element e of copy c
// at 8*(e*R + c), lane uses copy lane % R).  The product configurations use
// R = 1: replication R = 2..32 measured within +-1% (k1_cfg.h,
// profiles/r02/k1_tiled_v*.log).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "heldkarp_impl.h"

namespace tspgpu {

constexpr int kTiledMaxL = 12;
// distance row stride (entries): the per-lane gathers d[m][k] of a half-wave
// fall on bank pair (m * stride + k) mod 32.  16 made every pair m, m+2
// collide (94% bank-conflict cycles); a bank model over every pass's
// (member, destination) positions gives 0.44 extra cycles per low-low gather
// at 17, 0.065 at 19; measured at n = 16 (cfg 14, 4096 blocks,
// profiles/r02/lds_conflicts_stride.txt): conflict cycles 29.7 K -> 20.2 K
// per block (0.575 -> 0.391 of LDS-active cycles), time equal or 0.5% less.
// The rest are the scattered next-layer stores and rank lookups.
#ifndef TSPGPU_TILED_DS
#define TSPGPU_TILED_DS 19
#endif
constexpr int kTiledDS = TSPGPU_TILED_DS;
// Rows with at least N - TSPGPU_TILED_TA_OFF members keep the argmin (a
// 64-bit parent word each); every smaller row is relaxed without it and the
// backtracking recomputes the few rows it needs (see tiled_backtrack).
#ifndef TSPGPU_TILED_TA_OFF
#define TSPGPU_TILED_TA_OFF 4
#endif
#ifndef TSPGPU_TILED_QC
#define TSPGPU_TILED_QC 7  // destinations relaxed together (register budget of a chunk)
#endif
#ifndef TSPGPU_TILED_AHEAD
#define TSPGPU_TILED_AHEAD 6  // d loads in flight per lane in the relaxation loop
#endif
// Measured and not kept (profiles/r02; the switches were removed in round
// 6): the high distance rows/columns permuted into sub-cube order between
// sub-cubes (the passes 3% faster, the permutation on wave 0's path 6% slower
// — variant 6 does it on idle threads instead, hk_sub.h) and
// destination-parallel edge passes (spills; variant 6 has them in a form that
// does not spill).

// host-built tables of one L (device copy, staged into LDS per workgroup)
struct TiledInfo {
    uint16_t mask[1 << kTiledMaxL];  // L-bit masks sorted by (popcount, colex rank)
    uint16_t rank[1 << kTiledMaxL];  // colex rank of a mask among the masks of its popcount
    uint16_t rankb8[1 << kTiledMaxL];  // rank x 8, rank x 4: byte offsets inside a push / layer column
    uint16_t rankb4[1 << kTiledMaxL];
    int moff[kTiledMaxL + 2];        // first index of popcount class j in mask[]
    int cnt[kTiledMaxL + 2];         // C(L, j)
};

__host__ __device__ constexpr int tiled_layer_vals(int L, int j) { return cbinom(L, j) * j; }
// one LDS region holds the two live low layers: layer j at the bottom when j
// is even, at the top when odd (adjacent layers never overlap)
__host__ __device__ constexpr int tiled_region_vals(int L)
{
    int m = 0;
    for (int j = 0; j < L; ++j) {
        const int s = tiled_layer_vals(L, j) + tiled_layer_vals(L, j + 1);
        m = s > m ? s : m;
    }
    return m;
}
__host__ __device__ constexpr size_t tiled_lds_bytes(int N, int L, int R, int vb, bool tables = true)
{
    return (size_t)N * kTiledDS * R * vb     // replicated inner distances, rows of kTiledDS
           + (size_t)2 * 16 * vb             // d[0][k], d[m][0]
           + (size_t)tiled_region_vals(L) * vb  // live low layers
           + (tables ? (size_t)2 * 2 * (1 << L) : 0);  // mask + rank (u16), unless read from global
}
// the mask/rank tables stay in global memory (L1/L2-resident) when staging
// them in LDS would keep WG workgroups from fitting a CU's 160 KB
__host__ __device__ constexpr bool tiled_global_tables(int N, int L, int R, int vb, int wg)
{
    return tiled_lds_bytes(N, L, R, vb, true) * wg > 160 * 1024;
}
// push area of one slot: [h][c][idx] values (c = high city index 0..H-1,
// idx = the row's place in the sorted L-bit mask list)
__host__ __device__ constexpr size_t tiled_push_bytes(int N, int L, int vb)
{
    return (size_t)(1 << (N - L)) * (N - L) * (1 << L) * vb;
}
// parent words of the workgroup's current block: [h][idx] u64 (only rows
// with >= N - TSPGPU_TILED_TA_OFF members are written)
__host__ __device__ constexpr size_t tiled_parent_bytes(int N, int L)
{
    return TSPGPU_TILED_TA_OFF > 0 ? (size_t)8 << N : 0;
}
// backtracking recompute area: G[h<<L | l][m] of one sub-cube h, [l][m], m low
__host__ __device__ constexpr size_t tiled_recomp_bytes(int L, int vb) { return (size_t)(1 << L) * L * vb; }
// one block's global slot: push area, parent words, recompute area (kept
// until the backtracking kernel has run: one slot per block of a launch)
__host__ __device__ constexpr size_t tiled_slot_bytes(int N, int L, int vb)
{
    return tiled_push_bytes(N, L, vb) + tiled_parent_bytes(N, L) + ((tiled_recomp_bytes(L, vb) + 255) & ~(size_t)255);
}

// f(std::integral_constant<int, 0>), ..., f(std::integral_constant<int, C-1>)
template <int I, int C, typename F>
__device__ __forceinline__ void static_for_impl(F &&f)
{
    if constexpr (I < C) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, C>(f);
    }
}
template <int C, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    static_for_impl<0, C>(f);
}

__host__ __device__ constexpr int tiled_moff(int L, int J)
{
    int o = 0;
    for (int i = 0; i < J; ++i) o += cbinom(L, i);
    return o;
}

// Buffer-resource access with the uniform part of the offset in soffset (an
// SGPR) and the per-lane part in voffset: no VALU address arithmetic.
// (cache-policy bits of the pushes' loads and stores: A/B builds only)
#ifndef TSPGPU_RS_LOAD_AUX
#define TSPGPU_RS_LOAD_AUX 0
#endif
#ifndef TSPGPU_RS_STORE_AUX
#define TSPGPU_RS_STORE_AUX 0
#endif
template <typename V>
struct Rsrc {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ V load(uint32_t voff, uint32_t soff) const
    {
        if constexpr (sizeof(V) == 8)
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)voff, (int)soff,
                                                                                  TSPGPU_RS_LOAD_AUX));
        else
            return (V)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)voff, (int)soff, TSPGPU_RS_LOAD_AUX);
    }
    __device__ __forceinline__ void store(uint32_t voff, uint32_t soff, V v) const
    {
        if constexpr (sizeof(V) == 8) {
            using u2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rs, (int)voff, (int)soff,
                                                  TSPGPU_RS_STORE_AUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, rs, (int)voff, (int)soff, TSPGPU_RS_STORE_AUX);
        }
    }
    // non-temporal 8-byte store (parent words: read back only by the backtracking)
    __device__ __forceinline__ void store_nt(uint32_t voff, uint32_t soff, uint64_t w) const
    {
        using u2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, w), rs, (int)voff, (int)soff, 2);
    }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *p, uint32_t bytes)
{
    const uint64_t base = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, (int)nb,
                                             0x00020000);
}

// LDS barrier: the passes inside a sub-cube hand data over through LDS only
// (their pushes are read by later sub-cubes, behind a full __syncthreads), so
// they wait for their own LDS operations, not for their global stores.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// acc = min(acc, g + d) with arg = m where g + d < acc (the first strict
// minimum over members ascending, tsp.cpp:465): exactly four VALU
// instructions with the compare in VCC (compiler-scheduled compares landed in
// SGPR pairs that were spilled, round-1 K1 counters).
__device__ __forceinline__ void relax_argmin(double &acc, uint32_t &arg, double g, double d, uint32_t m)
{
    double t;
    asm volatile(
        "v_add_f64 %[t], %[g], %[d]\n\t"
        "v_cmp_lt_f64 vcc, %[t], %[acc]\n\t"
        "v_cndmask_b32 %[arg], %[arg], %[m], vcc\n\t"
        "v_min_f64 %[acc], %[acc], %[t]"
        : [acc] "+v"(acc), [arg] "+v"(arg), [t] "=&v"(t)
        : [g] "v"(g), [d] "v"(d), [m] "v"(m)
        : "vcc");
}
__device__ __forceinline__ void relax_argmin(int32_t &acc, uint32_t &arg, int32_t g, int32_t d, uint32_t m)
{
    int32_t t;
    asm volatile(
        "v_add_u32 %[t], %[g], %[d]\n\t"
        "v_cmp_lt_i32 vcc, %[t], %[acc]\n\t"
        "v_cndmask_b32 %[arg], %[arg], %[m], vcc\n\t"
        "v_min_i32 %[acc], %[acc], %[t]"
        : [acc] "+v"(acc), [arg] "+v"(arg), [t] "=&v"(t)
        : [g] "v"(g), [d] "v"(d), [m] "v"(m)
        : "vcc");
}

// acc = min(acc, g + d), no argmin (ablation 8 / argmin-free passes)
__device__ __forceinline__ void relax_min(double &acc, double g, double d)
{
    double t;
    asm volatile("v_add_f64 %[t], %[g], %[d]\n\tv_min_f64 %[acc], %[acc], %[t]"
                 : [acc] "+v"(acc), [t] "=&v"(t)
                 : [g] "v"(g), [d] "v"(d));
}
__device__ __forceinline__ void relax_min(int32_t &acc, int32_t g, int32_t d)
{
    int32_t t;
    asm volatile("v_add_u32 %[t], %[g], %[d]\n\tv_min_i32 %[acc], %[acc], %[t]"
                 : [acc] "+v"(acc), [t] "=&v"(t)
                 : [g] "v"(g), [d] "v"(d));
}

template <typename V, int N, int L, int R>
struct TiledCtx {
    const V *dr;               // LDS replicated distances
    const uint16_t *lmask;     // sorted L-bit masks (LDS, or global: tiled_global_tables)
    const uint16_t *lrankb;    // colex rank x sizeof(V) (byte offset inside a position column)
    V *region;                 // LDS live low layers
    Rsrc<V> push;              // this slot's push area
    Rsrc<uint64_t> par;        // this slot's parent words (the current block's)
    Rsrc<V> rec;               // this slot's backtracking recompute area
    const int *moff;           // first index of each popcount class (backtracking)
};

// One pass (h, J) of a sub-cube: T = |h| + J members per source row, all
// counts static (one instantiation per (T, J)), so the split of members and
// non-members into low (per lane) and high (uniform) parts costs no branch.
template <typename V, int N, int L, int T, int J, int THREADS, int R>
__device__ __forceinline__ void tiled_pass(const TiledCtx<V, N, L, R> &c, uint32_t h, uint32_t tid)
{
    constexpr int H = N - L;
    constexpr int Q = N - T;
    constexpr int HC = T - J;   // high members (uniform)
    constexpr int QL = L - J;   // low non-members (per lane), listed first
    constexpr int QH = Q - QL;  // high non-members (uniform)
    static_assert(HC >= 0 && HC <= H && QL >= 0 && QH >= 0 && T >= 1 && T < N, "bad pass");
    constexpr int NL = 1 << L;
    constexpr int VB = sizeof(V);
    constexpr int ROWS = cbinom(L, J);
    constexpr int BASE = tiled_moff(L, J);
    constexpr int ROWS_N = J < L ? cbinom(L, J + 1) : 0;
    constexpr int REGV = tiled_region_vals(L);
    constexpr int CUR = (J & 1) ? REGV - ROWS * J : 0;
    constexpr int NXT = ((J + 1) & 1) ? REGV - ROWS_N * (J + 1) : 0;
    // argmin and parent word only for the top rows (tiled_backtrack recomputes
    // the rest)
    constexpr bool ARG = T >= N - TSPGPU_TILED_TA_OFF;
    // distance rows of kTiledDS entries (R copies each): a member's row
    // offset is bit * DROW, a non-member's column offset bit << SK; the argmin
    // is kept as the member's row offset (one register less per member) and
    // turned back into the bit by a division by the constant DROW
    constexpr int SK = __builtin_ctz((unsigned)(R * VB));
    constexpr uint32_t DROW = (uint32_t)(kTiledDS * R * VB);
    static_assert((R & (R - 1)) == 0 && N < kTiledDS, "R must be a power of two");
    // uniform: the high members and high non-members of h, ascending
    uint32_t hm[HC > 0 ? HC : 1], hn[QH > 0 ? QH : 1];
    {
        uint32_t hb = h;
#pragma unroll
        for (int i = 0; i < HC; ++i) {
            hm[i] = __builtin_ctz(hb);
            hb &= hb - 1u;
        }
        uint32_t nb = ~h & ((1u << H) - 1u);
#pragma unroll
        for (int i = 0; i < QH; ++i) {
            hn[i] = __builtin_ctz(nb);
            nb &= nb - 1u;
        }
    }
    const uint32_t lane_off = (tid & (uint32_t)(R - 1)) * VB;
    const char *drb = reinterpret_cast<const char *>(c.dr);
    char *lds_nxt = reinterpret_cast<char *>(c.region + NXT);
    for (uint32_t r = tid; r < (uint32_t)ROWS; r += THREADS) {
        const uint32_t l = c.lmask[BASE + r];
        const uint32_t voff = (BASE + r) * VB;   // row offset in a push column
        // the row's T values: low members from LDS, high members from the pushes
        V g[T];
#pragma unroll
        for (int p = 0; p < J; ++p) g[p] = c.region[CUR + p * ROWS + r];
#pragma unroll
        for (int i = 0; i < HC; ++i) g[J + i] = c.push.load(voff, (h * H + hm[i]) * (uint32_t)(NL * VB));
        // members ascending (low bits of l, then the high members of h)
        uint32_t mrow[T];
        uint32_t lb = l;
#pragma unroll
        for (int p = 0; p < J; ++p) {
            mrow[p] = (uint32_t)__builtin_ctz(lb) * DROW + lane_off;
            lb &= lb - 1u;
        }
#pragma unroll
        for (int i = 0; i < HC; ++i) mrow[J + i] = (L + hm[i]) * DROW + lane_off;
        // Destinations in chunks of at most TSPGPU_TILED_QC (registers: acc,
        // arg and the column offsets of one chunk only); the non-members come
        // ascending (low non-members of l, then those of h).  Per chunk: the
        // T*QC relaxations, member-major (members ascending for every
        // destination), each d value loaded TSPGPU_TILED_AHEAD relaxations
        // ahead; a scheduling barrier per relaxation keeps the compiler from
        // hoisting all loads (and their registers) up front.  The first
        // member initialises acc/arg: with validated inputs every candidate is
        // below the reference's INT_MAX start value (tsp.cpp:453), so its
        // first comparison always succeeds.
        uint32_t nb = ~l & (uint32_t)(NL - 1);
        uint32_t wlo = 0, whi = 0;
        constexpr int QC = TSPGPU_TILED_QC;
        static_for<(Q + QC - 1) / QC>([&](auto ci) {
            constexpr int C0 = decltype(ci)::value * QC;
            constexpr int QN = Q - C0 < QC ? Q - C0 : QC;
            uint32_t kof[QN];
#pragma unroll
            for (int qq = 0; qq < QN; ++qq) {
                const int q = C0 + qq;
                if (q < QL) {
                    kof[qq] = (uint32_t)__builtin_ctz(nb) << SK;
                    nb &= nb - 1u;
                } else {  // high non-member q - QL
                    kof[qq] = (L + hn[q - QL]) << SK;
                }
            }
            V acc[QN];
            uint32_t arg[ARG ? QN : 1];
            {
                constexpr int TQ = T * QN;
                constexpr int AH = TSPGPU_TILED_AHEAD < TQ ? TSPGPU_TILED_AHEAD : TQ;
                V dv[AH];
#pragma unroll
                for (int i = 0; i < AH; ++i) dv[i] = *reinterpret_cast<const V *>(drb + mrow[i / QN] + kof[i % QN]);
#pragma unroll
                for (int i = 0; i < TQ; ++i) {
                    const V d = dv[i % AH];
                    if (i + AH < TQ)
                        dv[i % AH] = *reinterpret_cast<const V *>(drb + mrow[(i + AH) / QN] + kof[(i + AH) % QN]);
                    if (i < QN) {
                        acc[i] = g[0] + d;
                        if constexpr (ARG) arg[i] = mrow[0];
                    } else {
                        if constexpr (ARG)
                            relax_argmin(acc[i % QN], arg[i % QN], g[i / QN], d, mrow[i / QN]);
                        else
                            relax_min(acc[i % QN], g[i / QN], d);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int qq = 0; qq < QN; ++qq) {
                const int q = C0 + qq;
                if (q < QL) {
                    // low k -> next LDS layer (position k - q, colex rank of l + k)
                    const uint32_t k = kof[qq] >> SK;
                    const uint32_t rb = c.lrankb[l | (1u << k)];
                    *reinterpret_cast<V *>(lds_nxt + (k - (uint32_t)q) * (uint32_t)(ROWS_N * VB) + rb) = acc[qq];
                } else {
                    // high k -> the push column (h | k, k) of sub-cube h | k, same row index
                    const uint32_t cb = hn[q - QL];
                    c.push.store(voff, ((h | (1u << cb)) * H + cb) * (uint32_t)(NL * VB), acc[qq]);
                }
                // the row's parent word: nibble q = bit index of the argmin member
                if constexpr (ARG) {
                    const uint32_t pos = arg[qq] / DROW;  // table row of the argmin member = its city bit
                    if (q < 8)
                        wlo |= pos << (4 * q);
                    else
                        whi |= pos << (4 * (q - 8));
                }
            }
        });
        if constexpr (ARG) c.par.store((BASE + r) * 8u, h * (uint32_t)(NL * 8), ((uint64_t)whi << 32) | wlo);
    }
}

__host__ __device__ constexpr int pow2_at_least(int q)
{
    int p = 1;
    while (p < q) p *= 2;
    return p;
}

// Parallel bit deposit: the i-th set bit of m receives bit i of x.
__device__ __forceinline__ uint32_t pdep_u32(uint32_t x, uint32_t m)
{
    uint32_t r = 0;
    for (uint32_t b = 1; m; b <<= 1) {
        const uint32_t low = m & (0u - m);
        if (x & b) r |= low;
        m ^= low;
    }
    return r;
}

// G[h<<L | l][m] after the forward pass: a high m from the push area, a low m
// from the recompute area (valid for the sub-cube and the subsets the last
// tiled_recompute covered).  Any m < N gives a valid address (the value of a
// non-member is garbage): callers load unconditionally, then select.
template <typename V, int N, int L, int R>
__device__ __forceinline__ V tiled_g(const TiledCtx<V, N, L, R> &c, uint32_t h, uint32_t l, uint32_t pidx, int m)
{
    constexpr int H = N - L, NL = 1 << L, VB = sizeof(V);
    if (m < L) return c.rec.load((l * L + (uint32_t)m) * VB, 0);
    return c.push.load(pidx, (h * H + (uint32_t)(m - L)) * (uint32_t)(NL * VB));
}
// byte offset of row l inside a push column
template <typename V, int N, int L, int R>
__device__ __forceinline__ uint32_t tiled_pidx(const TiledCtx<V, N, L, R> &c, uint32_t l)
{
    return (uint32_t)c.moff[__builtin_popcount(l)] * (uint32_t)sizeof(V) + c.lrankb[l];
}

// Backtracking recompute (one wave): G[h<<L | l'][m] for every l' within lT and
// every low member m, layer by layer from the pushed high-member values — the
// forward pass's own relaxations restricted to those rows, the minimum only
// (IEEE min is order-free, so the values are the forward pass's bits).
// Round 6: a lane per (row, destination) pair — a layer of C(nl, j) rows has
// (nl - j) destinations per row, so a wave's lanes are busy where the
// row-per-lane form left most idle in the small layers, and each lane relaxes
// only its own destination over the row's members only (not N predicated
// relaxations per possible destination): hk_tiled_backtrack per 65536 16-city
// blocks 1.76 ms (row per lane) -> 1.44 ms (pairs) -> ~1.33 ms (members
// only; profiles/r06/bt_ab.txt).
template <typename V, int N, int L, int R>
__device__ void tiled_recompute(const TiledCtx<V, N, L, R> &c, const V *d0, uint32_t h, uint32_t lT,
                                uint32_t lane)
{
    constexpr int VB = sizeof(V);
    const int nl = __builtin_popcount(lT);
    const int hcnt = __builtin_popcount(h);
    int j0 = 0;
    if (h == 0) {  // no high member: layer 1 is G[{k}][k] = d[0][k] (tsp.cpp:435)
        if (lane < (uint32_t)L && ((lT >> lane) & 1u)) c.rec.store(((1u << lane) * L + lane) * VB, 0, d0[lane]);
        j0 = 1;
    }
    for (int j = j0; j < nl; ++j) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int q = nl - j, pairs = cbinom(nl, j) * q, mo = c.moff[j];
        for (int e = (int)lane; e < pairs; e += 64) {
            const int r = e / q, qi = e - r * q;
            // the r-th j-subset of lT in colex order = the r-th j-subset of
            // the low bits, deposited on lT's cities; its qi-th destination
            const uint32_t lp = pdep_u32(c.lmask[mo + r], lT);
            const uint32_t s = (uint32_t)__builtin_ctz(pdep_u32(1u << qi, lT & ~lp));
            const uint32_t Tm = (h << L) | lp;
            const uint32_t pidx = tiled_pidx(c, lp);
            // members only: the row's T = j + |h| members (T wave-uniform, so
            // every "q < T" is a scalar branch), their loads all in flight
            // (round 6: -7.5% against N predicated relaxations per pair)
            const int T = j + hcnt;
            V acc = ValT<V>::inf;
            // (every value in flight at once: 9 VGPRs of spills at six
            // workgroups per CU, and still faster than loading the member
            // list in two halves without spills, 0.41 vs 0.51 ms per 16384
            // blocks: profiles/r06/bt_ab.txt)
            V gv[N - 1];
            uint32_t x = Tm;
#pragma unroll
            for (int q = 0; q < N - 1; ++q) {
                if (q < T) gv[q] = tiled_g(c, h, lp, pidx, __builtin_ctz(x));
                x &= x - 1u;
            }
            x = Tm;
#pragma unroll
            for (int q = 0; q < N - 1; ++q) {
                if (q < T) acc = ValT<V>::vmin(acc, gv[q] + c.dr[((uint32_t)__builtin_ctz(x) * kTiledDS + s) * R]);
                x &= x - 1u;
            }
            c.rec.store(((lp | (1u << s)) * L + s) * VB, 0, acc);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Backtracking of the block just solved (one wave, tsp.cpp:473-481's parent
// walk): from the last inner city k_last back to the start.  A row with
// >= N - TSPGPU_TILED_TA_OFF members has its parent word; below that the row's
// values are recomputed (tiled_recompute, once per sub-cube the path enters)
// and the parent is the first strict minimum over its members ascending of
// G[T][m] + d[m][k] — the forward pass's candidates, so its argmin.
template <typename V, int N, int L, int R>
__device__ bool tiled_backtrack(const TiledCtx<V, N, L, R> &c, const V *d0, int bestM,
                                int32_t *tour, uint32_t lane)
{
    constexpr int NL = 1 << L, VB = sizeof(V), n = N + 1;
    uint32_t S = (1u << N) - 1u;
    int k = bestM - 1;
    bool ok = bestM >= 1 && bestM <= N;
    uint32_t hcur = ~0u, lcur = 0;
    for (int pos = n - 2; ok && pos >= 1; --pos) {
        const uint32_t T = S & ~(1u << k);
        const uint32_t hT = T >> L, lT = T & (uint32_t)(NL - 1);
        int pm;
        if (__builtin_popcount(T) >= N - TSPGPU_TILED_TA_OFF) {
            const uint32_t idx = (uint32_t)c.moff[__builtin_popcount(lT)] + c.lrankb[lT] / VB;
            const uint64_t w = c.par.load(idx * 8u, hT * (uint32_t)(NL * 8));
            const int q = k - __builtin_popcount(T & ((1u << k) - 1u));  // k's place among T's non-members
            pm = (int)((w >> (4 * q)) & 15u);
        } else {
            if (hT != hcur || (lT & ~lcur)) {
                tiled_recompute(c, d0, hT, lT, lane);
                hcur = hT;
                lcur = lT;
            }
            const bool mem = lane < (uint32_t)N && ((T >> lane) & 1u);
            V cand = ValT<V>::invalid;
            const V g = tiled_g(c, hT, lT, tiled_pidx(c, lT), lane < (uint32_t)N ? (int)lane : 0);
            if (mem) cand = g + c.dr[(lane * kTiledDS + (uint32_t)k) * R];
            const V best = wave_min(cand);
            const unsigned long long hit = __ballot(mem && cand == best);
            pm = hit ? __ffsll(hit) - 1 : N;
        }
        ok = pm < N && ((T >> pm) & 1u);
        if (lane == 0) tour[pos] = ok ? pm + 1 : 0;
        S = T;
        k = pm;
    }
    return ok;
}

template <typename V, int N, int L, int J, int THREADS, int R>
__device__ __forceinline__ void tiled_dispatch_h(const TiledCtx<V, N, L, R> &c, uint32_t h, int hc, uint32_t tid)
{
    constexpr int H = N - L;
#define TSPGPU_TP(HC)                                                                      \
    case HC:                                                                               \
        if constexpr (HC <= H && J + HC >= 1 && J + HC < N)                                \
            tiled_pass<V, N, L, J + HC, J, THREADS, R>(c, h, tid);                         \
        break;
    switch (hc) {
        TSPGPU_TP(0) TSPGPU_TP(1) TSPGPU_TP(2) TSPGPU_TP(3) TSPGPU_TP(4) TSPGPU_TP(5) TSPGPU_TP(6)
        TSPGPU_TP(7)
    default: break;
    }
#undef TSPGPU_TP
}

template <typename V, int N, int L, int THREADS, int R>
__device__ __forceinline__ void tiled_dispatch(const TiledCtx<V, N, L, R> &c, uint32_t h, int hc, int j, uint32_t tid)
{
#define TSPGPU_TJ(JJ)                                                                      \
    case JJ:                                                                               \
        if constexpr (JJ <= L) tiled_dispatch_h<V, N, L, JJ, THREADS, R>(c, h, hc, tid);   \
        break;
    switch (j) {
        TSPGPU_TJ(0) TSPGPU_TJ(1) TSPGPU_TJ(2) TSPGPU_TJ(3) TSPGPU_TJ(4) TSPGPU_TJ(5) TSPGPU_TJ(6)
        TSPGPU_TJ(7) TSPGPU_TJ(8) TSPGPU_TJ(9) TSPGPU_TJ(10) TSPGPU_TJ(11) TSPGPU_TJ(12)
    default: break;
    }
#undef TSPGPU_TJ
}

__host__ __device__ constexpr int tiled_waves(int threads, int wg_per_cu) { return threads * wg_per_cu / 256; }

// Forward pass + closing min of blocks blk0 + blockIdx.x, +gridDim.x, ...;
// writes cost_out[blk] and the tour's last inner city (tour[n-1]).  Every
// block has its own global slot, kept for hk_tiled_backtrack.
template <typename V, int N, int L, int THREADS, int R, int WG>
__global__ __launch_bounds__(THREADS, tiled_waves(THREADS, WG)) void hk_tiled_kernel(
    const V *__restrict__ dist, int nblocks, int blk0, char *__restrict__ slots, uint32_t slot_bytes,
    const TiledInfo *__restrict__ info, V *__restrict__ cost_out, int32_t *__restrict__ tour_out)
{
    constexpr int H = N - L;
    constexpr int NH = 1 << H;
    constexpr int NL = 1 << L;
    constexpr int n = N + 1;
    constexpr int VB = sizeof(V);
    static_assert(H <= 7, "tiled_dispatch_h covers at most 7 high cities");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    V *dr = reinterpret_cast<V *>(smem);
    V *d0 = dr + N * kTiledDS * R;  // d[0][k], k = 1..N at [k-1]
    V *dc = d0 + 16;                // d[m][0], m = 1..N at [m-1]
    V *region = dc + 16;
    constexpr bool GT = tiled_global_tables(N, L, R, VB, WG);
    uint16_t *lmask = reinterpret_cast<uint16_t *>(region + tiled_region_vals(L));
    uint16_t *lrankb = lmask + NL;
    const uint32_t tid = threadIdx.x;

    if constexpr (!GT) {
        for (int i = tid; i < NL; i += THREADS) {
            lmask[i] = info->mask[i];
            lrankb[i] = VB == 8 ? info->rankb8[i] : info->rankb4[i];
        }
    }
    TiledCtx<V, N, L, R> c;
    c.dr = dr;
    c.lmask = GT ? info->mask : lmask;
    c.lrankb = GT ? (VB == 8 ? info->rankb8 : info->rankb4) : lrankb;
    c.region = region;
    c.moff = nullptr;  // (backtracking only)

    for (int blk = blk0 + blockIdx.x; blk < nblocks; blk += gridDim.x) {
        char *slot = slots + (size_t)(blk - blk0) * slot_bytes;
        c.push.rs = uniform_rsrc(slot, (uint32_t)tiled_push_bytes(N, L, VB));
        c.par.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB), (uint32_t)tiled_parent_bytes(N, L));
        const V *dsrc = dist + (size_t)blk * n * n;
        for (int i = tid; i < N * kTiledDS * R; i += THREADS) {
            const int e = i / R, m = e / kTiledDS, k = e % kTiledDS;  // columns >= N unused
            dr[i] = k < N ? dsrc[(m + 1) * n + (k + 1)] : V(0);
        }
        if (tid < N) {
            d0[tid] = dsrc[tid + 1];
            dc[tid] = dsrc[(tid + 1) * n];
        }
        __syncthreads();
        // layer 1: G[{i}][i] = d[0][i] (tsp.cpp:435's d[0][i] term): low i in
        // sub-cube 0's first LDS layer (colex rank of {i} is i), high i pushed
        // to sub-cube {i} at row idx 0 (the empty low part)
        // (layer 1 is odd: it sits at the top of the region, regv - C(L,1))
        if (tid < L) region[tiled_region_vals(L) - L + tid] = d0[tid];
        if (tid < H) c.push.store(0, (((1u << tid) * H + tid) * NL) * VB, d0[L + tid]);
        __syncthreads();

        for (uint32_t h = 0; h < (uint32_t)NH; ++h) {
            const int hc = __builtin_popcount(h);
            const int j0 = h == 0 ? 1 : 0;
            const int j1 = h == (uint32_t)(NH - 1) ? L - 1 : L;
            for (int j = j0; j <= j1; ++j) {
                tiled_dispatch<V, N, L, THREADS, R>(c, h, hc, j, tid);
                if (j < j1) lds_barrier();
            }
            // pushes of this sub-cube are read by later ones: full barrier
            __syncthreads();
        }

        // closing min (tsp.cpp:483-499): G[full][m] + d[m][0], first strict min
        if (tid < 64) {
            const int m = tid + 1;
            const bool valid = m <= N;
            V gl = V(0);
            if (valid) {
                if (m <= L)  // low layer L: one row, position m-1
                    gl = region[((L & 1) ? tiled_region_vals(L) - L : 0) + (m - 1)];
                else
                    gl = c.push.load((NL - 1) * VB, ((uint32_t)((NH - 1) * H + (m - 1 - L)) * NL) * VB);
            }
            const V cand = valid ? gl + dc[m - 1] : ValT<V>::invalid;
            const V best = ValT<V>::vmin(wave_min(cand), ValT<V>::inf);
            const unsigned long long hit = __ballot(valid && cand == best && cand < ValT<V>::inf);
            const int bestM = hit ? __ffsll(hit) : 0;
            if (tid == 0) {
                int32_t *tour = tour_out + (size_t)blk * (n + 1);
                tour[0] = 0;
                tour[n - 1] = bestM;
                tour[n] = 0;
                cost_out[blk] = bestM ? best : V(-1);
            }
        }
        __syncthreads();
    }
}

// Backtracking (tiled_backtrack): one wave per block, four per workgroup,
// persistent over the blocks of the launch.  A block's backtracking is a chain
// of dependent loads (tens of microseconds), so all resident waves run their
// chains at the same time, after the forward kernel instead of stalling it.
constexpr int kTiledBtWaves = 4;
#ifndef TSPGPU_TILED_BTWG
#define TSPGPU_TILED_BTWG 6  // backtracking workgroups per CU (register budget)
#endif
namespace {  // internal linkage: every instantiation file keeps its own (timing builds differ per file)
template <typename V, int N, int L>
__global__ __launch_bounds__(64 * kTiledBtWaves, TSPGPU_TILED_BTWG) void hk_tiled_backtrack(
    int nblocks, int blk0, const char *__restrict__ slots, uint32_t slot_bytes, const TiledInfo *__restrict__ info,
    const V *__restrict__ dist, V *__restrict__ cost_out, int32_t *__restrict__ tour_out)
{
    constexpr int NL = 1 << L, n = N + 1, VB = sizeof(V), DRV = N * kTiledDS + 16;
    __shared__ uint16_t lmask[NL], lrankb[NL];
    __shared__ int smoff[L + 2];
    __shared__ V drs[kTiledBtWaves][DRV];     // per wave: the block's inner distances, then d[0][k]
    for (int i = threadIdx.x; i < NL; i += 64 * kTiledBtWaves) {
        lmask[i] = info->mask[i];
        lrankb[i] = (uint16_t)(info->rank[i] * VB);
    }
    if (threadIdx.x < (uint32_t)(L + 2)) smoff[threadIdx.x] = info->moff[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    V *dr = drs[wave];
    TiledCtx<V, N, L, 1> c;
    c.dr = dr;
    c.lmask = lmask;
    c.lrankb = lrankb;
    c.region = nullptr;
    c.moff = smoff;
    for (int blk = blk0 + (int)(blockIdx.x * kTiledBtWaves + wave); blk < nblocks;
         blk += (int)(gridDim.x * kTiledBtWaves)) {
        const V *dsrc = dist + (size_t)blk * n * n;
        for (int i = lane; i < N * kTiledDS; i += 64) {
            const int m = i / kTiledDS, k = i % kTiledDS;
            dr[i] = k < N ? dsrc[(m + 1) * n + (k + 1)] : V(0);
        }
        if (lane < (uint32_t)N) dr[N * kTiledDS + lane] = dsrc[lane + 1];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        int32_t *tour = tour_out + (size_t)blk * (n + 1);
        const int bestM = tour[n - 1];
        if (bestM < 1) continue;  // no tour (cost already -1)
        char *slot = const_cast<char *>(slots) + (size_t)(blk - blk0) * slot_bytes;
        c.push.rs = uniform_rsrc(slot, (uint32_t)tiled_push_bytes(N, L, VB));
        c.par.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB), (uint32_t)tiled_parent_bytes(N, L));
        c.rec.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB) + tiled_parent_bytes(N, L),
                                (uint32_t)tiled_recomp_bytes(L, VB));
        if (!tiled_backtrack(c, dr + N * kTiledDS, bestM, tour, lane) && lane == 0) cost_out[blk] = V(-1);
        __builtin_amdgcn_wave_barrier();  // dr is reloaded for the next block
    }
}
}  // namespace

struct TiledArgs {
    const void *dist;
    int n, blk0, blk1;        // blocks [blk0, blk1) of this launch pair
    char *slots;              // one slot per block of [blk0, blk1)
    uint32_t slot_bytes;
    const TiledInfo *info;
    void *cost;
    int32_t *tour;
    int grid;
    int bt_grid;              // backtracking workgroups (kTiledBtWaves blocks each at a time)
    hipStream_t stream;
    hipEvent_t ev_mid;        // recorded between the two kernels when non-null (split timing)
};

template <typename V, int N, int L, int THREADS, int R, int WG>
hipError_t launch_tiled_n(const TiledArgs &a)
{
    const size_t lds = tiled_lds_bytes(N, L, R, sizeof(V), !tiled_global_tables(N, L, R, sizeof(V), WG));
    static bool raised = false;  // once per instantiation
    if (!raised) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&hk_tiled_kernel<V, N, L, THREADS, R, WG>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        raised = true;
    }
    hipLaunchKernelGGL((hk_tiled_kernel<V, N, L, THREADS, R, WG>), dim3(a.grid), dim3(THREADS), lds, a.stream,
                       static_cast<const V *>(a.dist), a.blk1, a.blk0, a.slots, a.slot_bytes, a.info,
                       static_cast<V *>(a.cost), a.tour);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && a.ev_mid) e = hipEventRecord(a.ev_mid, a.stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((hk_tiled_backtrack<V, N, L>), dim3(a.bt_grid), dim3(64 * kTiledBtWaves), 0, a.stream, a.blk1, a.blk0,
                       a.slots, a.slot_bytes, a.info, static_cast<const V *>(a.dist), static_cast<V *>(a.cost),
                       a.tour);
    return hipGetLastError();
}

}  // namespace tspgpu
