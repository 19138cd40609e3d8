// K1 variant 6 — sub-cube Held-Karp, restructured for gfx950 (MI355X).
//
// Same recurrence, same IEEE operations, same first-strict-minimum argmin and
// the same global slot layout (push area, parent words, recompute area) as
// variant 5 (hk_tiled.h), whose backtracking kernel it reuses — so the same
// cost and tour bits (tsp.cpp:424-499).  What changes is how a sub-cube's
// passes are scheduled and where a relaxation's distance comes from:
//
// * Distances touching a high city need no address arithmetic.  The inner
//   distance image in LDS has H extra rows and columns that hold, for the
//   current sub-cube h, the high rows d[hm_i][*] and columns d[*][hn_u] in
//   sub-cube order (members ascending, then non-members): a pass knows i and
//   u at compile time, so d[hm_i][k] is one ds_read with an immediate offset
//   on the lane's k, d[m][hn_u] one on the lane's m, and d[hm_i][hn_u] is
//   wave-uniform (an SGPR operand of v_add).  Only the low-low relaxations
//   (43% at n = 16) keep a per-lane v_add_u32 for the address.  The extra
//   rows/columns of sub-cube h + 1 are written by idle threads during the
//   last pass of sub-cube h (which reads only the natural image).
// * Fewer, fuller passes.  The 1- and 10-row passes at both ends of a
//   sub-cube (j = 0, 1, L-1, L: 13% of the relaxations, 20% of variant 5's
//   time) become destination-parallel: a lane per (row, destination), the
//   row's T relaxations each.  j = 0 is folded into j = 1 (each lane of row
//   {a} recomputes its own G[h+a][a] from the |h| pushed values), and j = L of
//   sub-cube h runs in the same barrier interval as j = 0/1 of sub-cube h + 1
//   (independent work).  L - 1 = 9 intervals per sub-cube instead of 11.
// * Row tables instead of bit loops.  A row's members, non-members and the
//   colex ranks of its destination rows come from one 16-byte host-built
//   entry (global, L2-resident), prefetched one pass ahead; decoding is
//   independent v_bfe ops instead of a dependent ctz chain.
#pragma once
#include "hk_tiled.h"

namespace tspgpu {

// row stride (entries) of the LDS distance image: N natural columns + H
// sub-cube-ordered high columns, odd so that the low-low gathers of a
// half-wave spread over the banks (25: 1% faster than 21 and 23 at n = 16,
// profiles/r03/k1_ab_table.log run 6)
// (L = 9, 128-thread workgroups: 23, so that twelve workgroups' LDS fits a CU)
#ifndef TSPGPU_SUB_DS
#define TSPGPU_SUB_DS 25
#endif
__host__ __device__ constexpr int sub_ds(int L) { return L >= 10 ? TSPGPU_SUB_DS : 23; }

// one entry per L-bit mask (indexed like TiledInfo::mask, L <= 10): nibbles
// 0..L-1 = the members ascending, then the non-members ascending; bytes
// 5..14 = colex rank of mask | (1 << k_q) among the masks of one more member,
// for the q-th non-member k_q
struct SubRow {
    uint32_t w[4];
};

__host__ __device__ constexpr size_t sub_img_bytes(int N, int L, int vb)
{
    return (size_t)(N + (N - L)) * sub_ds(L) * vb;
}
// One low layer in LDS at a time (TSPGPU_SUB_ONE_LAYER): a middle pass loads
// its rows' values into registers, the workgroup passes a barrier, and the
// next layer is written over the one just read — the region is the largest
// layer, C(10,5) x 5 = 1260 values (10 KB), instead of two adjacent layers
// (20 KB), so the block's LDS drops from 24.5 to 14.5 KB and occupancy is set
// by registers alone.
#ifndef TSPGPU_SUB_ONE_LAYER
#define TSPGPU_SUB_ONE_LAYER 0  // measured 5% slower (the extra barrier), profiles/r03/k1_ab_table.log run 8
#endif
__host__ __device__ constexpr int sub_region_vals(int L)
{
    if (!TSPGPU_SUB_ONE_LAYER) return tiled_region_vals(L);
    int m = 0;
    for (int j = 0; j <= L; ++j) m = tiled_layer_vals(L, j) > m ? tiled_layer_vals(L, j) : m;
    return m;
}
// where layer j starts in the region
__host__ __device__ constexpr int sub_layer_off(int L, int j)
{
    return (!TSPGPU_SUB_ONE_LAYER && (j & 1)) ? tiled_region_vals(L) - tiled_layer_vals(L, j) : 0;
}
// Overlapped edge passes (TSPGPU_SUB_OVERLAP): passes 0/1 of sub-cube h + 1
// run during the last middle pass of h and pass L of h during the first middle
// pass of h + 1, on the waves those passes leave idle, and pass L - 1's push
// values are staged into LDS during middle pass L - 3 — the separate edge
// interval A(h) and its exposed memory round trips go away (diagnostic stamps:
// the two edge intervals took 33% of a block's time for 13% of its
// relaxations).  Needs layer 2 of the next sub-cube outside the region
// (C(L,2) x 2 values) and the staged values (L rows x H).
#ifndef TSPGPU_SUB_OVERLAP
#define TSPGPU_SUB_OVERLAP 2  // 2: with the edge passes' push values staged in LDS (-3% forward, profiles/r05)
#endif
__host__ __device__ constexpr int sub_l2_vals(int L) { return cbinom(L, 2) * 2; }
__host__ __device__ constexpr size_t sub_lds_bytes(int N, int L, int vb)
{
    return sub_img_bytes(N, L, vb) + (size_t)2 * 16 * vb + (size_t)sub_region_vals(L) * vb + (size_t)16 * vb +
           (TSPGPU_SUB_OVERLAP ? (size_t)(sub_l2_vals(L) + L * (N - L)) * vb : 0) +
           (TSPGPU_SUB_OVERLAP >= 2 ? (size_t)((L + 1) * (N - L) + (N - L)) * vb : 0);
}

template <typename V, int N, int L>
struct SubCtx {
    char *img;         // LDS distance image (bytes): natural rows/columns 0..N-1, sub-cube-ordered N..N+H-1
    const V *d0;       // d[0][k], k = 1..N at [k-1]
    V *region;         // live low layers (as variant 5)
    V *layerL;         // G[h | full low][m], m low: written by pass L-1, read by pass L
    V *layer2;         // layer 2 (passes 0/1 write it, middle pass 2 reads it): the region's
                       // bottom, or its own area when the edge passes overlap (TSPGPU_SUB_OVERLAP)
    V *pst;            // pass L-1's push values staged in LDS (TSPGPU_SUB_OVERLAP): [row][i]
    V *fst;            // passes 0/1's push values (TSPGPU_SUB_OVERLAP >= 2): [i] row 0, [H + a*H + i] row {a}
    V *lst;            // pass L's push values (TSPGPU_SUB_OVERLAP >= 2): [i]
    int ov;            // the overlap level this kernel runs (TSPGPU_SUB_OVERLAP; 0 below 256 threads)
    const V *dg;       // this block's distance matrix in global memory (n x n; TSPGPU_SUB_SHH)
    Rsrc<V> push;      // this block's push area
    Rsrc<uint64_t> par;  // this block's parent words
};

template <typename V>
__device__ __forceinline__ V lds_val(const char *base, uint32_t byte_off)
{
    return *reinterpret_cast<const V *>(base + byte_off);
}
// wave-uniform LDS value -> SGPR(s)
template <typename V>
__device__ __forceinline__ V uniform_val(const char *base, uint32_t byte_off)
{
    const V v = lds_val<V>(base, byte_off);
    if constexpr (sizeof(V) == 8) {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
        return __builtin_bit_cast(V, ((uint64_t)hi << 32) | lo);
    } else {
        return (V)__builtin_amdgcn_readfirstlane((uint32_t)v);
    }
}

// relaxations whose distance is an SGPR operand (wave-uniform)
__device__ __forceinline__ void relax_min_s(double &acc, double g, double d)
{
    double t;
    asm volatile("v_add_f64 %[t], %[g], %[d]\n\tv_min_f64 %[acc], %[acc], %[t]"
                 : [acc] "+v"(acc), [t] "=&v"(t)
                 : [g] "v"(g), [d] "s"(d));
}
__device__ __forceinline__ void relax_min_s(int32_t &acc, int32_t g, int32_t d)
{
    int32_t t;
    asm volatile("v_add_u32 %[t], %[d], %[g]\n\tv_min_i32 %[acc], %[acc], %[t]"
                 : [acc] "+v"(acc), [t] "=&v"(t)
                 : [g] "v"(g), [d] "s"(d));
}
__device__ __forceinline__ void relax_argmin_s(double &acc, uint32_t &arg, double g, double d, uint32_t m)
{
    double t;
    asm volatile(
        "v_add_f64 %[t], %[g], %[d]\n\t"
        "v_cmp_lt_f64 vcc, %[t], %[acc]\n\t"
        "v_cndmask_b32 %[arg], %[arg], %[m], vcc\n\t"
        "v_min_f64 %[acc], %[acc], %[t]"
        : [acc] "+v"(acc), [arg] "+v"(arg), [t] "=&v"(t)
        : [g] "v"(g), [d] "s"(d), [m] "v"(m)
        : "vcc");
}
__device__ __forceinline__ void relax_argmin_s(int32_t &acc, uint32_t &arg, int32_t g, int32_t d, uint32_t m)
{
    int32_t t;
    asm volatile(
        "v_add_u32 %[t], %[d], %[g]\n\t"
        "v_cmp_lt_i32 vcc, %[t], %[acc]\n\t"
        "v_cndmask_b32 %[arg], %[arg], %[m], vcc\n\t"
        "v_min_i32 %[acc], %[acc], %[t]"
        : [acc] "+v"(acc), [arg] "+v"(arg), [t] "=&v"(t)
        : [g] "v"(g), [d] "s"(d), [m] "v"(m)
        : "vcc");
}

// two / four independent min-only relaxations in one block: every add is
// issued before the first min, so no min waits on the add just before it
__device__ __forceinline__ void relax_min2(double &a0, double g0, double d0, double &a1, double g1, double d1)
{
    double t0, t1;
    asm volatile(
        "v_add_f64 %[t0], %[g0], %[d0]\n\t"
        "v_add_f64 %[t1], %[g1], %[d1]\n\t"
        "v_min_f64 %[a0], %[a0], %[t0]\n\t"
        "v_min_f64 %[a1], %[a1], %[t1]"
        : [a0] "+v"(a0), [a1] "+v"(a1), [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [g0] "v"(g0), [d0] "v"(d0), [g1] "v"(g1), [d1] "v"(d1));
}
// two relaxations of ONE destination: two adds and one v_min3_i32 (1.5 VALU
// instructions per relaxation instead of 2; integer min is exact in any order)
__device__ __forceinline__ void relax_min3(int32_t &a, int32_t g0, int32_t d0, int32_t g1, int32_t d1)
{
    int32_t t0, t1;
    asm volatile(
        "v_add_u32 %[t0], %[g0], %[d0]\n\t"
        "v_add_u32 %[t1], %[g1], %[d1]\n\t"
        "v_min3_i32 %[a], %[a], %[t0], %[t1]"
        : [a] "+v"(a), [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [g0] "v"(g0), [d0] "v"(d0), [g1] "v"(g1), [d1] "v"(d1));
}
#ifndef TSPGPU_SUB_MIN3
#define TSPGPU_SUB_MIN3 1  // i32 middle passes: member pairs per destination through v_min3_i32
#endif
__device__ __forceinline__ void relax_min2(int32_t &a0, int32_t g0, int32_t d0, int32_t &a1, int32_t g1, int32_t d1)
{
    int32_t t0, t1;
    asm volatile(
        "v_add_u32 %[t0], %[g0], %[d0]\n\t"
        "v_add_u32 %[t1], %[g1], %[d1]\n\t"
        "v_min_i32 %[a0], %[a0], %[t0]\n\t"
        "v_min_i32 %[a1], %[a1], %[t1]"
        : [a0] "+v"(a0), [a1] "+v"(a1), [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [g0] "v"(g0), [d0] "v"(d0), [g1] "v"(g1), [d1] "v"(d1));
}
#ifndef TSPGPU_SUB_PAIR
#define TSPGPU_SUB_PAIR 1  // middle passes: min-only relaxations two at a time (relax_min2)
#endif
#ifndef TSPGPU_SUB_SB
#define TSPGPU_SUB_SB 1  // middle passes: a scheduling barrier after every SB relaxation pairs
#endif

// generic relaxation with a first-member initialisation (edge passes)
template <bool ARG, typename V>
__device__ __forceinline__ void relax_any(bool first, V &acc, uint32_t &arg, V g, V d, uint32_t m)
{
    if (first) {
        acc = g + d;
        arg = m;
    } else if constexpr (ARG) {
        relax_argmin(acc, arg, g, d, m);
    } else {
        relax_min(acc, g, d);
    }
}

// a copy of x the compiler must treat as unknown at this point: keeps it from
// hoisting every pass's thread-index arithmetic out of the block and
// sub-cube loops (which would keep all of it live, i.e. spilled, throughout)
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// the idx-th set bit of the low `bits` bits of x (idx wave-uniform or not)
__device__ __forceinline__ uint32_t nth_bit(uint32_t x, uint32_t idx)
{
    return (uint32_t)__builtin_ctz(pdep_u32(1u << idx, x));
}

// OR of a 64-bit word over aligned groups of QP lanes (QP a power of two)
template <int QP>
__device__ __forceinline__ uint64_t group_or(uint64_t w)
{
#pragma unroll
    for (int off = 1; off < QP; off *= 2) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)w, off);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(w >> 32), off);
        w |= ((uint64_t)hi << 32) | lo;
    }
    return w;
}

__device__ __forceinline__ uint32_t sub_nib(const uint4 &e, int i)
{
    return i < 8 ? (e.x >> (4 * i)) & 15u : (e.y >> (4 * (i - 8))) & 15u;
}
__device__ __forceinline__ uint32_t sub_rank(const uint4 &e, int q)
{
    const int b = 5 + q;  // byte index
    const uint32_t w = b < 4 ? e.x : (b < 8 ? e.y : (b < 12 ? e.z : e.w));
    return (w >> (8 * (b & 3))) & 255u;
}

// ---------------------------------------------------------------------------
// Middle pass (h, J), 2 <= J <= L-2: a thread owns row r = tid (colex rank of
// its low part l among the J-subsets), T = |h| + J members, Q = N - T
// destinations; for every destination the first strict minimum over the
// members ascending of G[T][m] + d[m][k] (tsp.cpp:457-470), argmin kept only
// in the top rows (T >= N - TSPGPU_TILED_TA_OFF).
// ---------------------------------------------------------------------------
// relaxation order of a destination chunk [C0, C0 + QN): every (member,
// destination) pair whose distance comes from LDS, member-major, then the
// high-high pairs (SGPR distances) — per destination still members ascending
template <int T, int J, int QL, int C0, int QN>
__host__ __device__ constexpr int sub_lds_count()
{
    int n = 0;
    for (int p = 0; p < T; ++p)
        for (int qq = 0; qq < QN; ++qq)
            if (!(p >= J && C0 + qq >= QL)) ++n;
    return n;
}
// QP = false: member-major (p, then the destinations q: consecutive
// relaxations have different destinations, independent min chains).  QP =
// true (integer values): member 0's row first, then member PAIRS (p, p + 1)
// destination by destination, so relaxations 2i-1 and 2i share q and fold
// into one v_min3 (acc = min3(acc, g_p + d, g_(p+1) + d')).
template <int T, int J, int QL, int C0, int QN, bool QP = false>
__host__ __device__ constexpr int sub_lds_pair(int k)
{
    int n = 0;
    if (!QP) {
        for (int p = 0; p < T; ++p)
            for (int qq = 0; qq < QN; ++qq)
                if (!(p >= J && C0 + qq >= QL)) {
                    if (n == k) return p * 64 + qq;
                    ++n;
                }
        return -1;
    }
    for (int qq = 0; qq < QN; ++qq)
        if (!(0 >= J && C0 + qq >= QL)) {
            if (n == k) return qq;
            ++n;
        }
    for (int p = 1; p < T; p += 2)
        for (int qq = 0; qq < QN; ++qq)
            for (int pp = p; pp < p + 2 && pp < T; ++pp)
                if (!(pp >= J && C0 + qq >= QL)) {
                    if (n == k) return pp * 64 + qq;
                    ++n;
                }
    return -1;
}

// QP order: 1 = relaxation k opens a same-destination member pair (k, k + 1),
// 2 = k closes one, 0 = a single relaxation (member 0, or a pair member whose
// partner is a high-high relaxation, which is not in the LDS list)
template <int T, int J, int QL, int C0, int QN>
__host__ __device__ constexpr int sub_lds_role(int k)
{
    int n = 0;
    for (int qq = 0; qq < QN; ++qq)
        if (!(0 >= J && C0 + qq >= QL)) {
            if (n == k) return 0;
            ++n;
        }
    for (int p = 1; p < T; p += 2)
        for (int qq = 0; qq < QN; ++qq) {
            int in = 0;
            for (int pp = p; pp < p + 2 && pp < T; ++pp) in += !(pp >= J && C0 + qq >= QL) ? 1 : 0;
            for (int i = 0; i < in; ++i, ++n)
                if (n == k) return in == 2 ? 1 + i : 0;
        }
    return -1;
}

// Timing-only ablations (measurement builds, tools/ab_build.sh; the results
// are WRONG): 1 = the middle passes take their high members' values from the
// LDS region instead of the push loads, 2 = no LDS distance gathers (one
// register value), 4 = no barrier between the middle passes, 8 = no push
// stores in the middle passes, 16 = the sub-cube barriers wait for LDS only,
// 32 = the middle passes' push loads all read one L2-resident row (the loads
// stay, their memory traffic goes), 64 = the middle passes' push stores all
// write one L2-resident row (likewise), 128 = both, for the lowest high city's
// columns only (a fifth of the traffic)
#ifndef TSPGPU_SUB_ABL
#define TSPGPU_SUB_ABL 0
#endif

#ifndef TSPGPU_SUB_QC
#define TSPGPU_SUB_QC 7  // destinations relaxed together (register budget)
#endif
#ifndef TSPGPU_SUB_AHEAD
#define TSPGPU_SUB_AHEAD 6  // distance loads in flight per lane
#endif

// Push columns recycled (TSPGPU_SUB_RECYCLE).  Column (h', x) is written by
// sub-cube h' \ x and read by sub-cube h' only, so in the numeric sub-cube
// order it is live over [h' \ x, h']; first-fit over those intervals gives
// 23 columns at H = 5 instead of 80 (184 KB per block instead of 640 KB), and
// the six resident blocks of a CU then touch ~280 MB of pushes instead of ~1
// GB — close to the 256 MB Infinity Cache.  (Ablations, profiles/r04: push
// loads and stores redirected to one L2-resident row -18% forward time.)
#ifndef TSPGPU_SUB_RECYCLE
#define TSPGPU_SUB_RECYCLE 0
#endif
template <int H>
struct SubColMap {
    uint32_t slot[(1 << H) * H];
    int count;
};
template <int H>
constexpr SubColMap<H> sub_col_map()
{
    SubColMap<H> m{};
    int until[(1 << H) * H] = {};  // per column slot: the consumer sub-cube of its current column
    int n = 0;
    for (int p = 0; p < (1 << H); ++p)  // producers in the forward order
        for (int x = 0; x < H; ++x) {
            if ((p >> x) & 1) continue;
            const int hp = p | (1 << x);
            int s = -1;
            for (int k = 0; k < n && s < 0; ++k)
                if (until[k] < p) s = k;  // (its consumer has finished)
            if (s < 0) s = n++;
            until[s] = hp;
            m.slot[hp * H + x] = (uint32_t)s;
        }
    m.count = n;
    return m;
}
template <int H>
__constant__ SubColMap<H> g_sub_cols = sub_col_map<H>();
// the push column of (sub-cube hp, high city x)
template <int H>
__device__ __forceinline__ uint32_t sub_col(uint32_t hp, uint32_t x)
{
    // (wave-uniform: a scalar load from the constant table)
    if constexpr (TSPGPU_SUB_RECYCLE) return g_sub_cols<H>.slot[__builtin_amdgcn_readfirstlane(hp * H + x)];
    return hp * H + x;
}

// Deferred push stores (TSPGPU_SUB_DEFER).  Vector-memory operations retire
// in issue order (one vmcnt per wave), so a pass's push loads, issued after
// the previous pass's push stores, could only be used once those stores had
// completed: every pass waited for the last one's write acknowledgements.  A
// middle pass now keeps its high-destination results in registers (at most
// H - |h| values per thread), issues the NEXT pass's push loads first and only
// then these stores — the loads no longer queue behind them.  (Ablations,
// profiles/r04: no middle push stores -18% forward time, no push loads -11%.)
#ifndef TSPGPU_SUB_DEFER
#define TSPGPU_SUB_DEFER 0  // measured slower: +14% forward time (62 VGPR spills), profiles/r04/k1_defer_ab.log
#endif
constexpr int kSubPend = 6;  // >= H - |h|

// Early push loads (TSPGPU_SUB_EARLY).  A middle pass's high members' values
// (push loads, memory latency) were issued at its start and needed after the
// first J x QC relaxations: every pass exposed most of a memory round trip.
// Thread r owns row r in every pass of a sub-cube and the high members of
// pass J + 1 are pass J's (same h), so pass J issues pass J + 1's push loads
// itself, AFTER its own relaxations and stores (registers are free there),
// and they land during the barrier and the next pass's LDS reads.
#ifndef TSPGPU_SUB_EARLY
#define TSPGPU_SUB_EARLY 0
#endif
// Diagnostic build (TSPGPU_SUB_STAMP): per wave, the shader clock spent in the
// middle-pass bodies, at their barriers, in the edge intervals and in the whole
// block, written over the block's tour words (tour_out[blk*(n+1) + 4*wave + k],
// k = body, barrier, edge, total; the backtracking kernel is skipped).  The
// results are not tours in such a build.
#ifndef TSPGPU_SUB_STAMP
#define TSPGPU_SUB_STAMP 0
#endif
__device__ __forceinline__ uint32_t sub_clock()
{
    return (uint32_t)__builtin_amdgcn_s_memtime();
}
// Wave roles rotated (TSPGPU_SUB_ROT): the rows of a pass go to the threads
// in wave order, so wave 0 of every workgroup works in every pass and wave 3
// in three of seven; with the workgroups of a CU placing wave w on SIMD w, one
// SIMD would carry all the heaviest waves.  1: the roles rotate by the
// workgroup's index, 2: by workgroup and sub-cube (every wave gets every role
// in turn).  Any bijection is valid: passes hand over only through LDS and
// memory behind barriers.
#ifndef TSPGPU_SUB_ROT
#define TSPGPU_SUB_ROT 0
#endif
#ifndef TSPGPU_SUB_SHH
#define TSPGPU_SUB_SHH 0
#endif
// one |h| dispatch per sub-cube around all middle passes (instead of one per pass)
#ifndef TSPGPU_SUB_MIDSWITCH
#define TSPGPU_SUB_MIDSWITCH 0
#endif

template <typename V, int N, int L, int T, int J>
__device__ __forceinline__ void sub_mid(const SubCtx<V, N, L> &c, uint32_t h, uint32_t tid, const uint4 &ent,
                                        V (&pend)[kSubPend], V (&pre)[kSubPend])
{
    constexpr int H = N - L;
    constexpr int Q = N - T;
    constexpr int HC = T - J;   // high members (uniform)
    constexpr int QL = L - J;   // low non-members (per lane), first
    constexpr int QH = Q - QL;  // high non-members (uniform)
    static_assert(J >= 2 && J <= L - 2 && HC >= 0 && HC <= H && QH >= 0, "bad middle pass");
    constexpr int NL = 1 << L;
    constexpr int VB = sizeof(V);
    constexpr int ROWS = cbinom(L, J);
    constexpr int BASE = tiled_moff(L, J);
    constexpr int ROWS_N = cbinom(L, J + 1);
    constexpr int CUR = sub_layer_off(L, J);
    constexpr int NXT = sub_layer_off(L, J + 1);
    constexpr bool ARG = T >= N - TSPGPU_TILED_TA_OFF;
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    constexpr uint32_t HR0 = (uint32_t)N * DSB;  // image row N: the first sub-cube-ordered high row
    constexpr uint32_t HC0 = (uint32_t)N * VB;   // image column N
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
    // high-high distances of this sub-cube: wave-uniform (TSPGPU_SUB_SHH:
    // scalar loads from the block's matrix in memory, no LDS read and no
    // v_readfirstlane; else from the LDS image)
    V hh[HC * QH > 0 ? HC * QH : 1];
#pragma unroll
    for (int i = 0; i < HC; ++i)
#pragma unroll
        for (int u = 0; u < QH; ++u)
            hh[i * QH + u] = TSPGPU_SUB_SHH ? c.dg[(L + 1 + hm[i]) * (N + 1) + (L + 1 + hn[u])]
                                            : uniform_val<V>(c.img, HR0 + i * DSB + HC0 + u * VB);
    const uint32_t r = tid;
    const bool act = r < (uint32_t)ROWS;
    V g[T];
    {
        const V *src = J == 2 ? c.layer2 : c.region + CUR;
#pragma unroll
        for (int p = 0; p < J; ++p) g[p] = act ? src[p * ROWS + r] : V(0);
    }
    // (one layer in LDS: every wave has its row's values before any of the
    // next layer overwrites them)
    if (TSPGPU_SUB_ONE_LAYER) lds_barrier();
    const uint32_t voff = (BASE + r) * VB;  // the row's offset in a push column
    constexpr bool PRE_IN = TSPGPU_SUB_EARLY && J > 2, PRE_OUT = TSPGPU_SUB_EARLY && J < L - 2;
    if (act) {
#pragma unroll
        for (int i = 0; i < HC; ++i)
            g[J + i] = (TSPGPU_SUB_ABL & 1)    ? c.region[CUR + (i % J) * ROWS + r]
                       : (TSPGPU_SUB_ABL & 32) ? c.push.load(r * VB, 0)
                       : ((TSPGPU_SUB_ABL & 128) && hm[i] == 0) ? c.push.load(r * VB, 0)
                       : PRE_IN                ? pre[i]
                                               : c.push.load(voff, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
    }
    // pass J + 1's push loads (TSPGPU_SUB_EARLY): by this thread, which owns
    // row r there too; after everything else of this pass
    auto prefetch = [&] {
        if constexpr (PRE_OUT && HC > 0) {
            constexpr int ROWS_X = cbinom(L, J + 1), BASE_X = tiled_moff(L, J + 1);
            __builtin_amdgcn_sched_barrier(0);
            if (r < (uint32_t)ROWS_X) {
#pragma unroll
                for (int i = 0; i < HC; ++i)
                    pre[i] = c.push.load((BASE_X + r) * VB, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
            }
        }
        // (every entry redefined here: none stays live through a pass)
#pragma unroll
        for (int i = PRE_OUT ? HC : kSubPend; i < kSubPend; ++i) pre[i] = V(0);
    };
    // the previous middle pass's pushes, behind this pass's loads
    constexpr bool DEFER_IN = TSPGPU_SUB_DEFER && J > 2, DEFER_OUT = TSPGPU_SUB_DEFER && J < L - 2;
    if constexpr (DEFER_IN) {
        constexpr int ROWS_P = cbinom(L, J - 1), BASE_P = tiled_moff(L, J - 1);
        if (r < (uint32_t)ROWS_P) {
#pragma unroll
            for (int u = 0; u < QH; ++u)
                c.push.store((BASE_P + r) * VB, sub_col<H>(h | (1u << hn[u]), hn[u]) * (uint32_t)(NL * VB), pend[u]);
        }
    }
    if (!act) {
        prefetch();
        return;
    }
    uint32_t mrow[J], kof[QL];
#pragma unroll
    for (int p = 0; p < J; ++p) mrow[p] = sub_nib(ent, p) * DSB;
#pragma unroll
    for (int q = 0; q < QL; ++q) kof[q] = sub_nib(ent, J + q) * VB;
    // argmin operand: the member's image row offset (low: mrow, high: L + hm)
    uint32_t hrow[HC > 0 ? HC : 1];
#pragma unroll
    for (int i = 0; i < HC; ++i) hrow[i] = (L + hm[i]) * DSB;
    uint32_t wlo = 0, whi = 0;
    constexpr int QC = TSPGPU_SUB_QC;
    static_for<(Q + QC - 1) / QC>([&](auto ci) {
        constexpr int C0 = decltype(ci)::value * QC;
        constexpr int QN = Q - C0 < QC ? Q - C0 : QC;
        constexpr int CNT = sub_lds_count<T, J, QL, C0, QN>();
        constexpr int AH = TSPGPU_SUB_AHEAD < CNT ? TSPGPU_SUB_AHEAD : CNT;
        // integer min-only rows: member pairs per destination (v_min3_i32)
        constexpr bool QP = TSPGPU_SUB_MIN3 && !ARG && std::is_same<V, int32_t>::value;
        V acc[QN];
        uint32_t arg[ARG ? QN : 1];
        // distance of LDS relaxation k (compile-time pair)
        auto dload = [&](auto kk) -> V {
            constexpr int pq = sub_lds_pair<T, J, QL, C0, QN, QP>(decltype(kk)::value);
            constexpr int p = pq / 64, q = C0 + pq % 64;
            if constexpr (TSPGPU_SUB_ABL & 2)
                return g[p] + g[0];  // (ablation: no gather)
            else if constexpr (p < J && q < QL)
                return lds_val<V>(c.img, mrow[p] + kof[q]);
            else if constexpr (p < J)
                return lds_val<V>(c.img, mrow[p] + HC0 + (q - QL) * VB);
            else
                return lds_val<V>(c.img, HR0 + (p - J) * DSB + kof[q]);
        };
        V dv[AH > 0 ? AH : 1];
        static_for<AH>([&](auto kk) { dv[decltype(kk)::value] = dload(kk); });
        // relaxation k of the chunk (its distance from the load pipeline)
        auto relax_one = [&](auto kk) {
            constexpr int k = decltype(kk)::value;
            constexpr int pq = sub_lds_pair<T, J, QL, C0, QN, QP>(k);
            constexpr int p = pq / 64, qq = pq % 64;
            const V d = dv[k % AH];
            if constexpr (k + AH < CNT) dv[k % AH] = dload(std::integral_constant<int, k + AH>{});
            const uint32_t mo = p < J ? mrow[p < J ? p : 0] : hrow[p >= J ? p - J : 0];
            if constexpr (p == 0) {
                acc[qq] = g[0] + d;
                if constexpr (ARG) arg[qq] = mo;
            } else if constexpr (ARG) {
                relax_argmin(acc[qq], arg[qq], g[p], d, mo);
            } else {
                relax_min(acc[qq], g[p], d);
            }
        };
        if constexpr (QP) {
            static_for<CNT>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                constexpr int role = sub_lds_role<T, J, QL, C0, QN>(k);
                if constexpr (role == 1) {
                    constexpr int pq0 = sub_lds_pair<T, J, QL, C0, QN, QP>(k);
                    constexpr int pq1 = sub_lds_pair<T, J, QL, C0, QN, QP>(k + 1);
                    static_assert(pq0 % 64 == pq1 % 64 && pq1 / 64 == pq0 / 64 + 1, "member pair");
                    const V d0 = dv[k % AH];
                    if constexpr (k + AH < CNT) dv[k % AH] = dload(std::integral_constant<int, k + AH>{});
                    const V d1 = dv[(k + 1) % AH];
                    if constexpr (k + 1 + AH < CNT) dv[(k + 1) % AH] = dload(std::integral_constant<int, k + 1 + AH>{});
                    if constexpr (std::is_same<V, int32_t>::value)
                        relax_min3(acc[pq0 % 64], g[pq0 / 64], d0, g[pq1 / 64], d1);
                    __builtin_amdgcn_sched_barrier(0);
                } else if constexpr (role == 0) {
                    relax_one(kk);
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
        } else if constexpr (TSPGPU_SUB_PAIR && !ARG) {
            static_for<(CNT + 1) / 2>([&](auto kk2) {
                constexpr int k0 = 2 * decltype(kk2)::value, k1 = k0 + 1;
                constexpr int pq0 = sub_lds_pair<T, J, QL, C0, QN, QP>(k0);
                constexpr int pq1 = k1 < CNT ? sub_lds_pair<T, J, QL, C0, QN, QP>(k1) : 0;
                constexpr int p0 = pq0 / 64, q0 = pq0 % 64, p1 = pq1 / 64, q1 = pq1 % 64;
                if constexpr (k1 < CNT && p0 > 0 && p1 > 0 && q0 != q1) {
                    const V d0 = dv[k0 % AH];
                    if constexpr (k0 + AH < CNT) dv[k0 % AH] = dload(std::integral_constant<int, k0 + AH>{});
                    const V d1 = dv[k1 % AH];
                    if constexpr (k1 + AH < CNT) dv[k1 % AH] = dload(std::integral_constant<int, k1 + AH>{});
                    relax_min2(acc[q0], g[p0], d0, acc[q1], g[p1], d1);
                } else {
                    relax_one(std::integral_constant<int, k0>{});
                    if constexpr (k1 < CNT) relax_one(std::integral_constant<int, k1>{});
                }
                if constexpr ((decltype(kk2)::value + 1) % TSPGPU_SUB_SB == 0) __builtin_amdgcn_sched_barrier(0);
            });
        } else {
            static_for<CNT>([&](auto kk) {
                relax_one(kk);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        // high members x high destinations: SGPR distances
#pragma unroll
        for (int i = 0; i < HC; ++i)
#pragma unroll
            for (int qq = 0; qq < QN; ++qq) {
                const int q = C0 + qq;
                if (q >= QL) {
                    if constexpr (ARG)
                        relax_argmin_s(acc[qq], arg[qq], g[J + i], hh[i * QH + (q - QL)], hrow[i]);
                    else
                        relax_min_s(acc[qq], g[J + i], hh[i * QH + (q - QL)]);
                }
            }
#pragma unroll
        for (int qq = 0; qq < QN; ++qq) {
            const int q = C0 + qq;
            if (q < QL) {
                // low k -> next LDS layer: position k - q, colex rank of l + k
                const uint32_t k = kof[q] / VB;
                const uint32_t slot = (k - (uint32_t)q) * (uint32_t)ROWS_N + sub_rank(ent, q);
                c.region[NXT + slot] = acc[qq];
            } else {
                // high k -> push column (h | k, k) of sub-cube h | k, same row index
                const uint32_t cb = hn[q - QL];
                if ((TSPGPU_SUB_ABL & 64) || ((TSPGPU_SUB_ABL & 128) && cb == 0))
                    c.push.store(r * VB, 8192u, acc[qq]);
                else if (DEFER_OUT)
                    pend[q - QL] = acc[qq];  // (stored by the next pass, after its loads)
                else if (!(TSPGPU_SUB_ABL & 8))
                    c.push.store(voff, sub_col<H>(h | (1u << cb), cb) * (uint32_t)(NL * VB), acc[qq]);
            }
            if constexpr (ARG) {
                const uint32_t pos = arg[qq] / DSB;  // image row of the argmin member = its city bit
                if (q < 8)
                    wlo |= pos << (4 * q);
                else
                    whi |= pos << (4 * (q - 8));
            }
        }
    });
    if constexpr (ARG) c.par.store((BASE + r) * 8u, h * (uint32_t)(NL * 8), ((uint64_t)whi << 32) | wlo);
    prefetch();
}

// ---------------------------------------------------------------------------
// First interval of sub-cube h (|h| = C): passes j = 0 and j = 1 in
// destination-parallel form.  Lane (a, q) < L * Q1: row {a} of sub-cube h,
// destination = its q-th non-member (low ones first); it first recomputes the
// row's own G[h + a][a] (j = 0's relaxation for destination a; at h = 0 that
// is d[0][a], tsp.cpp:435), then the row's C + 1 relaxations.  Lanes
// L * Q1 + u: j = 0's high destinations (pushes of row 0).  Min-only (T <= 6).
// ---------------------------------------------------------------------------
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_first(const SubCtx<V, N, L> &c, uint32_t h, uint32_t tid)
{
    constexpr int H = N - L, QH = H - C, Q1 = N - 1 - C;
    constexpr int NL = 1 << L, VB = sizeof(V);
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    constexpr int ROWS2 = cbinom(L, 2);
    static_assert(C + 1 < N - TSPGPU_TILED_TA_OFF, "first passes are min-only");
    if (tid >= (uint32_t)(L * Q1 + (C > 0 ? QH : 0))) return;
    uint32_t hm[C > 0 ? C : 1];
    {
        uint32_t hb = h;
#pragma unroll
        for (int i = 0; i < C; ++i) {
            hm[i] = __builtin_ctz(hb);
            hb &= hb - 1u;
        }
    }
    const uint32_t nh = ~h & ((1u << H) - 1u);
    V g0[C > 0 ? C : 1];  // G[h][hm_i]: row 0 of sub-cube h (wave-uniform)
#pragma unroll
    for (int i = 0; i < C; ++i)
        g0[i] = c.ov >= 2 ? c.fst[i] : c.push.load(0, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
    if (tid < (uint32_t)(L * Q1)) {
        const uint32_t a = tid / Q1, q = tid % Q1;
        const uint32_t kk = q < (uint32_t)(L - 1) ? q + (q >= a ? 1u : 0u) : L + nth_bit(nh, q - (L - 1));
        V gA;
        if constexpr (C == 0) {
            gA = c.d0[a];
        } else {
            gA = g0[0] + lds_val<V>(c.img, (L + hm[0]) * DSB + a * VB);
#pragma unroll
            for (int i = 1; i < C; ++i)
                gA = ValT<V>::vmin(gA, g0[i] + lds_val<V>(c.img, (L + hm[i]) * DSB + a * VB));
        }
        V acc = gA + lds_val<V>(c.img, a * DSB + kk * VB);
        const uint32_t voff = (1u + a) * VB;  // row {a}: index 1 + a in the mask list
#pragma unroll
        for (int i = 0; i < C; ++i) {
            const V g1 = c.ov >= 2 ? c.fst[H + a * H + i]
                                                 : c.push.load(voff, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
            relax_min(acc, g1, lds_val<V>(c.img, (L + hm[i]) * DSB + kk * VB));
        }
        if (kk < (uint32_t)L) {
            // layer 2 (even: bottom of the region): position of kk in {a, kk}, colex rank
            const uint32_t lo = a < kk ? a : kk, hi = a < kk ? kk : a;
            c.layer2[(kk > a ? ROWS2 : 0) + hi * (hi - 1) / 2 + lo] = acc;
        } else {
            const uint32_t x = kk - L;
            c.push.store(voff, sub_col<H>(h | (1u << x), x) * (uint32_t)(NL * VB), acc);
        }
    } else if constexpr (C > 0) {
        // pass j = 0, high destination: G[h + x][x] -> push row 0 of sub-cube h | x
        const uint32_t x = nth_bit(nh, tid - L * Q1);
        V acc = g0[0] + lds_val<V>(c.img, (L + hm[0]) * DSB + (L + x) * VB);
#pragma unroll
        for (int i = 1; i < C; ++i) relax_min(acc, g0[i], lds_val<V>(c.img, (L + hm[i]) * DSB + (L + x) * VB));
        c.push.store(0, sub_col<H>(h | (1u << x), x) * (uint32_t)(NL * VB), acc);
    }
}

// ---------------------------------------------------------------------------
// Pass j = L of sub-cube h (|h| = C): the full low set, high destinations
// only, a lane per destination (lanes 0..QP-1 of the calling group).
// ---------------------------------------------------------------------------
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_last(const SubCtx<V, N, L> &c, uint32_t h, uint32_t lane)
{
    constexpr int H = N - L, Q = H - C, T = L + C;
    static_assert(Q >= 1 && T < N, "pass L needs a high destination");
    constexpr bool ARG = T >= N - TSPGPU_TILED_TA_OFF;
    constexpr int QP = pow2_at_least(Q);
    constexpr int NL = 1 << L, VB = sizeof(V);
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    if (lane >= (uint32_t)QP) return;
    uint32_t hm[C > 0 ? C : 1];
    {
        uint32_t hb = h;
#pragma unroll
        for (int i = 0; i < C; ++i) {
            hm[i] = __builtin_ctz(hb);
            hb &= hb - 1u;
        }
    }
    const bool act = lane < (uint32_t)Q;
    const uint32_t x = nth_bit(~h & ((1u << H) - 1u), act ? lane : 0u);
    const uint32_t kk = L + x;
    V acc = V(0);
    uint32_t arg = 0;
#pragma unroll
    for (int m = 0; m < L; ++m) relax_any<ARG>(m == 0, acc, arg, c.layerL[m], lds_val<V>(c.img, m * DSB + kk * VB), (uint32_t)m);
#pragma unroll
    for (int i = 0; i < C; ++i) {
        const V g = c.ov >= 2 ? c.lst[i] : c.push.load((NL - 1) * VB, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
        relax_any<ARG>(false, acc, arg, g, lds_val<V>(c.img, (L + hm[i]) * DSB + kk * VB), L + hm[i]);
    }
    if (act) c.push.store((NL - 1) * VB, sub_col<H>(h | (1u << x), x) * (uint32_t)(NL * VB), acc);
    if constexpr (ARG) {
        const uint64_t w = group_or<QP>(act ? (uint64_t)arg << (4 * lane) : 0ull);
        if (lane == 0) c.par.store((NL - 1) * 8u, h * (uint32_t)(NL * 8), w);
    }
}

// ---------------------------------------------------------------------------
// Pass j = L - 1 of sub-cube h (|h| = C): rows full \ {b} (rank r = L-1-b),
// destinations b (-> layerL[b]) and the high non-members; a lane per (row,
// destination), QP lanes per row.
// ---------------------------------------------------------------------------
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_penult(const SubCtx<V, N, L> &c, uint32_t h, uint32_t tid)
{
    constexpr int H = N - L, QH = H - C, Q = 1 + QH, T = L - 1 + C, J = L - 1;
    constexpr bool ARG = T >= N - TSPGPU_TILED_TA_OFF;
    constexpr int QP = pow2_at_least(Q);
    constexpr int NL = 1 << L, VB = sizeof(V);
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    constexpr int ROWS = L, BASE = tiled_moff(L, J);
    constexpr int CUR = sub_layer_off(L, J);
    if (tid >= (uint32_t)(L * QP)) return;
    uint32_t hm[C > 0 ? C : 1];
    {
        uint32_t hb = h;
#pragma unroll
        for (int i = 0; i < C; ++i) {
            hm[i] = __builtin_ctz(hb);
            hb &= hb - 1u;
        }
    }
    const uint32_t r = tid / QP, q = tid % QP, b = L - 1 - r;
    const bool act = q < (uint32_t)Q;
    const uint32_t x = (act && q > 0) ? nth_bit(~h & ((1u << H) - 1u), q - 1) : 0u;
    const uint32_t kk = q == 0 ? b : L + x;
    const uint32_t voff = (BASE + r) * VB;
    V acc = V(0);
    uint32_t arg = 0;
#pragma unroll
    for (int p = 0; p < L - 1; ++p) {
        const uint32_t m = (uint32_t)p + ((uint32_t)p >= b ? 1u : 0u);
        relax_any<ARG>(p == 0, acc, arg, c.region[CUR + p * ROWS + r], lds_val<V>(c.img, m * DSB + kk * VB), m);
    }
#pragma unroll
    for (int i = 0; i < C; ++i) {
        const V g = c.ov ? c.pst[r * H + i] : c.push.load(voff, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
        relax_any<ARG>(false, acc, arg, g, lds_val<V>(c.img, (L + hm[i]) * DSB + kk * VB), L + hm[i]);
    }
    if (act) {
        if (q == 0)
            c.layerL[b] = acc;
        else
            c.push.store(voff, sub_col<H>(h | (1u << x), x) * (uint32_t)(NL * VB), acc);
    }
    if constexpr (ARG) {
        const uint64_t w = group_or<QP>(act ? (uint64_t)arg << (4 * q) : 0ull);
        if (q == 0) c.par.store((BASE + r) * 8u, h * (uint32_t)(NL * 8), w);
    }
}

// ---------------------------------------------------------------------------
// Pass L-1's push values of sub-cube h (|h| = C) into LDS (TSPGPU_SUB_OVERLAP):
// lane e < L * C loads row r = e / C (layer L-1, rank r) of push column
// (h, hm_i), i = e % C, into pst[r * H + i] — by a wave that is idle in the
// middle pass it runs beside, so the load's round trip is off the critical path.
// ---------------------------------------------------------------------------
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_stage_penult(const SubCtx<V, N, L> &c, uint32_t h, uint32_t lane)
{
    constexpr int H = N - L, NL = 1 << L, VB = sizeof(V);
    constexpr int BASE = tiled_moff(L, L - 1);
    if constexpr (C > 0) {
        if (lane >= (uint32_t)(L * C)) return;
        const uint32_t r = lane / C, i = lane % C;
        const uint32_t x = nth_bit(h, i);
        c.pst[r * H + i] = c.push.load((BASE + r) * VB, sub_col<H>(h, x) * (uint32_t)(NL * VB));
    }
}

// Passes 0/1's push values of sub-cube h (|h| = C) into LDS (TSPGPU_SUB_OVERLAP
// >= 2): lanes e < C row 0 of column (h, hm_e); lanes C + a*C + i row {a} of
// column (h, hm_i), a < L.
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_stage_first(const SubCtx<V, N, L> &c, uint32_t h, uint32_t lane)
{
    constexpr int H = N - L, NL = 1 << L, VB = sizeof(V);
    if constexpr (C > 0) {
        if (lane < (uint32_t)C) {
            c.fst[lane] = c.push.load(0, sub_col<H>(h, nth_bit(h, lane)) * (uint32_t)(NL * VB));
        } else if (lane < (uint32_t)(C + L * C)) {
            const uint32_t e = lane - C, a = e / C, i = e % C;
            c.fst[H + a * H + i] = c.push.load((1u + a) * VB, sub_col<H>(h, nth_bit(h, i)) * (uint32_t)(NL * VB));
        }
    }
}
// Pass L's push values of sub-cube h (|h| = C): lane i < C, row NL - 1 of column (h, hm_i).
template <typename V, int N, int L, int C>
__device__ __forceinline__ void sub_stage_last(const SubCtx<V, N, L> &c, uint32_t h, uint32_t lane)
{
    constexpr int H = N - L, NL = 1 << L, VB = sizeof(V);
    if constexpr (C > 0 && C < H) {
        if (lane < (uint32_t)C)
            c.lst[lane] = c.push.load((NL - 1) * VB, sub_col<H>(h, nth_bit(h, lane)) * (uint32_t)(NL * VB));
    }
}

// ---------------------------------------------------------------------------
// Sub-cube-ordered high rows/columns of sub-cube h in the image (rows and
// columns N..N+H-1): position x of sigma_h = (members ascending, then
// non-members ascending).  e in [0, H*L): x = e / L, low k = e % L; then the
// high-high block.  Each entry is one LDS read and one LDS write.
// ---------------------------------------------------------------------------
template <typename V, int N, int L>
__device__ __forceinline__ void sub_build_high(const SubCtx<V, N, L> &c, uint32_t h, uint32_t e)
{
    constexpr int H = N - L, VB = sizeof(V);
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    const uint32_t cc = (uint32_t)__builtin_popcount(h);
    const uint32_t nh = ~h & ((1u << H) - 1u);
    char *img = c.img;
    if (e < (uint32_t)(H * L)) {
        const uint32_t x = e / L, k = e % L;
        if (x < cc) {
            const uint32_t s = nth_bit(h, x);
            *reinterpret_cast<V *>(img + (N + x) * DSB + k * VB) = lds_val<V>(img, (L + s) * DSB + k * VB);
        } else {
            const uint32_t s = nth_bit(nh, x - cc);
            *reinterpret_cast<V *>(img + k * DSB + (N + x - cc) * VB) = lds_val<V>(img, k * DSB + (L + s) * VB);
        }
    } else if (e < (uint32_t)(H * L) + cc * ((uint32_t)H - cc)) {
        const uint32_t f = e - H * L, i = f / ((uint32_t)H - cc), u = f % ((uint32_t)H - cc);
        const uint32_t si = nth_bit(h, i), su = nth_bit(nh, u);
        *reinterpret_cast<V *>(img + (N + i) * DSB + (N + u) * VB) = lds_val<V>(img, (L + si) * DSB + (L + su) * VB);
    }
}

template <typename V, int N, int L, int J>
__device__ __forceinline__ void sub_dispatch_mid_j(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t tid,
                                                   const uint4 &ent, V (&pend)[kSubPend], V (&pre)[kSubPend])
{
    constexpr int H = N - L;
#define TSPGPU_SM(HC)                                                                                  \
    case HC:                                                                                           \
        if constexpr (HC <= H) sub_mid<V, N, L, J + (HC <= H ? HC : 0), J>(c, h, tid, ent, pend, pre);  \
        break;
    switch (hc) {
        TSPGPU_SM(0) TSPGPU_SM(1) TSPGPU_SM(2) TSPGPU_SM(3) TSPGPU_SM(4) TSPGPU_SM(5) TSPGPU_SM(6) TSPGPU_SM(7)
    default: break;
    }
#undef TSPGPU_SM
}

#define TSPGPU_SUB_SWITCH_C(CVAR, FN, ...)                                                  \
    switch (CVAR) {                                                                         \
    case 0: if constexpr (0 <= H) FN<V, N, L, 0>(__VA_ARGS__); break;                       \
    case 1: if constexpr (1 <= H) FN<V, N, L, (1 <= H ? 1 : 0)>(__VA_ARGS__); break;        \
    case 2: if constexpr (2 <= H) FN<V, N, L, (2 <= H ? 2 : 0)>(__VA_ARGS__); break;        \
    case 3: if constexpr (3 <= H) FN<V, N, L, (3 <= H ? 3 : 0)>(__VA_ARGS__); break;        \
    case 4: if constexpr (4 <= H) FN<V, N, L, (4 <= H ? 4 : 0)>(__VA_ARGS__); break;        \
    case 5: if constexpr (5 <= H) FN<V, N, L, (5 <= H ? 5 : 0)>(__VA_ARGS__); break;        \
    case 6: if constexpr (6 <= H) FN<V, N, L, (6 <= H ? 6 : 0)>(__VA_ARGS__); break;        \
    default: break;                                                                         \
    }

template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_first(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t tid)
{
    constexpr int H = N - L;
    TSPGPU_SUB_SWITCH_C(hc, sub_first, c, h, tid)
}
template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_penult(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t tid)
{
    constexpr int H = N - L;
    TSPGPU_SUB_SWITCH_C(hc, sub_penult, c, h, tid)
}
template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_stage(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t lane)
{
    constexpr int H = N - L;
    TSPGPU_SUB_SWITCH_C(hc, sub_stage_penult, c, h, lane)
}
template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_stage_first(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t lane)
{
    constexpr int H = N - L;
    TSPGPU_SUB_SWITCH_C(hc, sub_stage_first, c, h, lane)
}
template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_stage_last(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t lane)
{
    constexpr int H = N - L;
    TSPGPU_SUB_SWITCH_C(hc, sub_stage_last, c, h, lane)
}
template <typename V, int N, int L>
__device__ __forceinline__ void sub_dispatch_last(const SubCtx<V, N, L> &c, uint32_t h, int hc, uint32_t lane)
{
    constexpr int H = N - L;
    // (|h| = H has no pass L: the full set has no destination)
    switch (hc) {
    case 0: if constexpr (0 < H) sub_last<V, N, L, 0>(c, h, lane); break;
    case 1: if constexpr (1 < H) sub_last<V, N, L, (1 < H ? 1 : 0)>(c, h, lane); break;
    case 2: if constexpr (2 < H) sub_last<V, N, L, (2 < H ? 2 : 0)>(c, h, lane); break;
    case 3: if constexpr (3 < H) sub_last<V, N, L, (3 < H ? 3 : 0)>(c, h, lane); break;
    case 4: if constexpr (4 < H) sub_last<V, N, L, (4 < H ? 4 : 0)>(c, h, lane); break;
    case 5: if constexpr (5 < H) sub_last<V, N, L, (5 < H ? 5 : 0)>(c, h, lane); break;
    default: break;
    }
}

// Forward pass + closing min of blocks blk0 + blockIdx.x, +gridDim.x, ...;
// writes cost_out[blk] and the tour's last inner city (tour[n-1]) like
// hk_tiled_kernel; hk_tiled_backtrack completes the tour from the slot.
// (TSPGPU_SUB_WG_OVERRIDE: a measurement build's occupancy for every
// configuration; the host then sizes the grid from TSPGPU_WG_PER_CU)
#ifndef TSPGPU_SUB_WG_OVERRIDE
#define TSPGPU_SUB_WG_OVERRIDE 0
#endif
__host__ __device__ constexpr int sub_wg(int wg) { return TSPGPU_SUB_WG_OVERRIDE > 0 ? TSPGPU_SUB_WG_OVERRIDE : wg; }
template <typename V, int N, int L, int THREADS, int WG>
__global__ __launch_bounds__(THREADS, tiled_waves(THREADS, sub_wg(WG))) void hk_sub_kernel(
    const V *__restrict__ dist, int nblocks, int blk0, char *__restrict__ slots, uint32_t slot_bytes,
    const SubRow *__restrict__ rows, V *__restrict__ cost_out, int32_t *__restrict__ tour_out)
{
    constexpr int H = N - L;
    constexpr int NH = 1 << H;
    constexpr int NL = 1 << L;
    constexpr int n = N + 1;
    constexpr int VB = sizeof(V);
    constexpr uint32_t DSB = (uint32_t)(sub_ds(L) * VB);
    static_assert(H >= 1 && H <= 6 && L >= 5 && L <= 10, "variant 6 sizes");
    static_assert(sub_ds(L) >= N + H, "image stride");
    // a middle pass gives each of its rows a thread; the edge intervals loop
    // their virtual lanes (pass 0/1 lanes 0..191, pass L 192..; pass L-1
    // lanes 0..127, the next sub-cube's image rows 128..) over the workgroup
    static_assert(THREADS % 64 == 0 && THREADS >= cbinom(L, L / 2), "one row per thread in a middle pass");
    static_assert(!TSPGPU_SUB_ROT || (THREADS & (THREADS - 1)) == 0, "rotated roles: a power-of-two workgroup");
    static_assert(L * (N - 1) + H <= 192 && L * 8 <= 128, "edge intervals: virtual lane layout");
    // static LDS: image/region offsets fold into immediates (A/B against
    // dynamic LDS: equal within noise, profiles/r03/k1_ab_table.log)
    __shared__ __attribute__((aligned(16))) char smem[sub_lds_bytes(N, L, VB)];
    SubCtx<V, N, L> c;
    c.img = smem;
    V *d0 = reinterpret_cast<V *>(smem + sub_img_bytes(N, L, VB));
    V *dc = d0 + 16;
    c.d0 = d0;
    c.region = dc + 16;
    c.layerL = c.region + sub_region_vals(L);
    // (the overlapped edge passes need the idle waves of a 256-thread workgroup)
    constexpr int OV = THREADS == 256 ? TSPGPU_SUB_OVERLAP : 0;
    c.ov = OV;
    c.layer2 = OV ? c.layerL + 16 : c.region + sub_layer_off(L, 2);
    c.pst = c.layerL + 16 + sub_l2_vals(L);
    c.fst = c.pst + L * H;
    c.lst = c.fst + (L + 1) * H;
    const uint32_t tid = threadIdx.x;
    const uint4 *rowtab = reinterpret_cast<const uint4 *>(rows);

    for (int blk = blk0 + blockIdx.x; blk < nblocks; blk += gridDim.x) {
        char *slot = slots + (size_t)(blk - blk0) * slot_bytes;
        c.push.rs = uniform_rsrc(slot, (uint32_t)tiled_push_bytes(N, L, VB));
        c.par.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB), (uint32_t)tiled_parent_bytes(N, L));
        const V *dsrc = dist + (size_t)blk * n * n;
        c.dg = dsrc;
        // natural image (inner distances) and, for sub-cube 0 (no high
        // member), the high columns in order
        for (int i = tid; i < N * N; i += THREADS) {
            const int m = i / N, k = i % N;
            const V v = dsrc[(m + 1) * n + (k + 1)];
            *reinterpret_cast<V *>(smem + m * DSB + k * VB) = v;
            if (m < L && k >= L) *reinterpret_cast<V *>(smem + m * DSB + (N + k - L) * VB) = v;
        }
        if (tid < N) {
            d0[tid] = dsrc[tid + 1];
            dc[tid] = dsrc[(tid + 1) * n];
        }
        // layer 1 of the high cities: G[{x}][x] = d[0][x] (tsp.cpp:435), pushed to sub-cube {x}, row 0
        if (tid < H) c.push.store(0, (sub_col<H>(1u << tid, tid) * NL) * VB, dsrc[L + tid + 1]);
        __syncthreads();

        uint4 ent = make_uint4(0, 0, 0, 0);
        V pend[kSubPend];  // deferred push stores of the last middle pass (TSPGPU_SUB_DEFER)
        V pre[kSubPend];   // the next middle pass's push values (TSPGPU_SUB_EARLY)
#pragma unroll
        for (int u = 0; u < kSubPend; ++u) pend[u] = pre[u] = V(0);
        uint32_t st_body = 0, st_bar = 0, st_edge = 0, st_t0 = 0, st_a = 0;
        uint64_t st_rt0 = 0;
        if (TSPGPU_SUB_STAMP) {
            st_t0 = sub_clock();
            st_rt0 = __builtin_amdgcn_s_memrealtime();
        }
        for (uint32_t h = 0; h < (uint32_t)NH; ++h) {
            const int hc = __builtin_popcount(h);
            if (TSPGPU_SUB_STAMP) st_a = sub_clock();
            // this sub-cube's thread -> role map (TSPGPU_SUB_ROT; whole waves)
            const uint32_t rot = TSPGPU_SUB_ROT == 2 ? (uint32_t)blockIdx.x + h : (TSPGPU_SUB_ROT == 1 ? (uint32_t)blockIdx.x : 0u);
            const uint32_t vtid = TSPGPU_SUB_ROT ? (tid + 64u * rot) & (uint32_t)(THREADS - 1) : tid;
            // interval A(h): passes 0/1 of h (lanes < 192) beside pass L of h - 1 (lanes 192..)
            // (TSPGPU_SUB_OVERLAP: at h = 0 only; later they run inside the middle passes)
            uint32_t t = opaque_u32(vtid);
            {
                constexpr int M2 = tiled_moff(L, 2), C2 = cbinom(L, 2);
                ent = rowtab[M2 + (t < (uint32_t)C2 ? t : 0u)];
            }
            if (!OV || h == 0) {
#pragma unroll
                for (uint32_t v0 = 0; v0 < 256u; v0 += THREADS) {  // (one iteration at 256 threads)
                    const uint32_t v = t + v0;
                    if (v < 192u)
                        sub_dispatch_first<V, N, L>(c, h, hc, v);
                    else if (h > 0)
                        sub_dispatch_last<V, N, L>(c, h - 1, __builtin_popcount(h - 1), v - 192u);
                }
                if (TSPGPU_SUB_ABL & 16) lds_barrier(); else __syncthreads();
            }
            if (TSPGPU_SUB_STAMP) {
                const uint32_t tb = sub_clock();
                st_edge += tb - st_a;
                st_a = tb;
            }
            // middle passes j = 2..L-2, unrolled (every offset a compile-time
            // constant); the next pass's row entry is loaded one pass ahead
            if constexpr (TSPGPU_SUB_MIDSWITCH) {
                // one dispatch on |h| per sub-cube around all middle passes:
                // each case is one straight-line sequence (the compiler's
                // wait counters and register lifetimes see across passes)
                auto mids = [&](auto hcc) {
                    constexpr int HC = decltype(hcc)::value;
                    static_for<L - 3>([&](auto jj) {
                        constexpr int j = 2 + decltype(jj)::value;
                        const uint4 cur = ent;
                        const uint32_t tj = opaque_u32(vtid);
                        if constexpr (j + 1 <= L - 2) {
                            constexpr int MN = tiled_moff(L, j + 1), CN = cbinom(L, j + 1);
                            ent = rowtab[MN + (tj < (uint32_t)CN ? tj : 0u)];
                        }
                        sub_mid<V, N, L, j + HC, j>(c, h, tj, cur, pend, pre);
                        if (!(TSPGPU_SUB_ABL & 4)) lds_barrier();
                    });
                };
                switch (hc) {
                case 0: mids(std::integral_constant<int, 0>{}); break;
                case 1: if constexpr (H >= 1) mids(std::integral_constant<int, (H >= 1 ? 1 : 0)>{}); break;
                case 2: if constexpr (H >= 2) mids(std::integral_constant<int, (H >= 2 ? 2 : 0)>{}); break;
                case 3: if constexpr (H >= 3) mids(std::integral_constant<int, (H >= 3 ? 3 : 0)>{}); break;
                case 4: if constexpr (H >= 4) mids(std::integral_constant<int, (H >= 4 ? 4 : 0)>{}); break;
                case 5: if constexpr (H >= 5) mids(std::integral_constant<int, (H >= 5 ? 5 : 0)>{}); break;
                case 6: if constexpr (H >= 6) mids(std::integral_constant<int, (H >= 6 ? 6 : 0)>{}); break;
                default: break;
                }
            } else {
                static_for<L - 3>([&](auto jj) {
                    constexpr int j = 2 + decltype(jj)::value;
                    const uint4 cur = ent;
                    const uint32_t tj = opaque_u32(vtid);
                    if constexpr (j + 1 <= L - 2) {
                        constexpr int MN = tiled_moff(L, j + 1), CN = cbinom(L, j + 1);
                        ent = rowtab[MN + (tj < (uint32_t)CN ? tj : 0u)];
                    }
                    sub_dispatch_mid_j<V, N, L, j>(c, h, hc, tj, cur, pend, pre);
                    if constexpr (OV) {
                        // edge passes on the waves this middle pass leaves idle
                        static_assert(cbinom(L, 2) <= 64 && cbinom(L, 3) <= 128 && cbinom(L, L - 3) <= 128, "overlap: idle waves");
                        if constexpr (OV >= 2) {
                            // pass 2: the edge passes' push values into LDS (waves 1-3);
                            // pass 3: pass L of h - 1 from them (wave 3)
                            if constexpr (j == 2) {
                                if (tj >= 192u) {
                                    if (h + 1 < (uint32_t)NH)
                                        sub_dispatch_stage_first<V, N, L>(c, h + 1, __builtin_popcount(h + 1), tj - 192u);
                                } else if (tj >= 128u) {
                                    sub_dispatch_stage<V, N, L>(c, h, hc, tj - 128u);
                                } else if (tj >= 64u && h > 0) {
                                    sub_dispatch_stage_last<V, N, L>(c, h - 1, __builtin_popcount(h - 1), tj - 64u);
                                }
                            }
                            if constexpr (j == 3) {
                                if (h > 0 && tj >= 192u)
                                    sub_dispatch_last<V, N, L>(c, h - 1, __builtin_popcount(h - 1), tj - 192u);
                            }
                        } else {
                            if constexpr (j == 2) {  // pass L of h - 1 (its layerL is still in LDS)
                                if (h > 0 && tj >= 64u)
                                    sub_dispatch_last<V, N, L>(c, h - 1, __builtin_popcount(h - 1), tj - 64u);
                            }
                            if constexpr (j == L - 3) {  // pass L - 1's push values into LDS
                                if (tj >= 128u) sub_dispatch_stage<V, N, L>(c, h, hc, tj - 128u);
                            }
                        }
                        if constexpr (j == L - 2) {  // passes 0/1 of h + 1 (layer 2 in its own area)
                            if (h + 1 < (uint32_t)NH && tj >= 64u)
                                sub_dispatch_first<V, N, L>(c, h + 1, __builtin_popcount(h + 1), tj - 64u);
                        }
                    }
                    uint32_t tm = 0;
                    if (TSPGPU_SUB_STAMP) {
                        tm = sub_clock();
                        st_body += tm - st_a;
                    }
                    if (!(TSPGPU_SUB_ABL & 4)) lds_barrier();
                    if (TSPGPU_SUB_STAMP) {
                        st_a = sub_clock();
                        st_bar += st_a - tm;
                    }
                });
            }
            // pass L - 1 (lanes < 128) beside the next sub-cube's high image rows/columns (lanes 128..)
            t = opaque_u32(vtid);
#pragma unroll
            for (uint32_t v0 = 0; v0 < 256u; v0 += THREADS) {
                const uint32_t v = t + v0;
                if (v < 128u)
                    sub_dispatch_penult<V, N, L>(c, h, hc, v);
                else if (h + 1 < (uint32_t)NH)
                    sub_build_high<V, N, L>(c, h + 1, v - 128u);
            }
            if (TSPGPU_SUB_ABL & 16) lds_barrier(); else __syncthreads();
            if (TSPGPU_SUB_STAMP) st_edge += sub_clock() - st_a;
        }
        if (TSPGPU_SUB_STAMP) {
            const uint32_t tot = sub_clock() - st_t0;
            const uint64_t rt = __builtin_amdgcn_s_memrealtime() - st_rt0;  // 100 MHz constant clock
            if ((tid & 63u) == 0) {
                int32_t *w = tour_out + (size_t)blk * (n + 1) + 4 * (tid >> 6);
                w[0] = (int32_t)st_body, w[1] = (int32_t)st_bar, w[2] = (int32_t)st_edge, w[3] = (int32_t)tot;
            }
            if (tid == 0) tour_out[(size_t)blk * (n + 1) + 16] = (int32_t)rt;  // (in-kernel clock = tot / rt x 100 MHz)
            __syncthreads();
            continue;
        }

        // closing min (tsp.cpp:483-499): G[full][m] + d[m][0], first strict min
        if (tid < 64) {
            const int m = tid + 1;
            const bool valid = m <= N;
            V gl = V(0);
            if (valid) {
                if (m <= L)
                    gl = c.layerL[m - 1];
                else
                    gl = c.push.load((NL - 1) * VB, (sub_col<H>(NH - 1, m - 1 - L) * NL) * VB);
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

// ---------------------------------------------------------------------------
// Backtracking of variant 6 with recycled push columns (TSPGPU_SUB_RECYCLE:
// the forward pass no longer keeps every pushed value, so the rows below the
// parent words cannot be recomputed from them).  One wave per block:
// (1) the rows with >= N - TSPGPU_TILED_TA_OFF members: their parent words,
//     as hk_tiled_backtrack;
// (2) below: the first prefix set T0 = {t1..tK} (K = N - TA_OFF - 1 cities)
//     gets its own Held-Karp, G[S][m] for every S within T0, in the slot's
//     recompute area (2^K x K values) — the same recurrence over the same
//     IEEE adds and mins, so the forward pass's bits (G[S][m] depends on S
//     and m only; min is order-free) — and the walk continues with the first
//     strict minimum over the members ascending (tsp.cpp:457-470), cities of
//     T0 ascending = local indices ascending.
// 10 * 9 * 2^8 = 23 K relaxations per 16-city block (1.3% of the forward
// pass), against a recompute of whole sub-cube rows before.
// ---------------------------------------------------------------------------
constexpr int kSubBtWaves = 4;
__host__ __device__ constexpr int sub_bt_k(int N) { return N - TSPGPU_TILED_TA_OFF - 1; }
__host__ __device__ constexpr size_t sub_rec_bytes(int N, int vb) { return ((size_t)vb * sub_bt_k(N)) << sub_bt_k(N); }
// one block's global slot for variant 6: push area, parent words and the
// recompute area of either backtracking kernel
__host__ __device__ constexpr size_t sub_slot_bytes(int N, int L, int vb)
{
    const size_t rec = tiled_recomp_bytes(L, vb) > sub_rec_bytes(N, vb) ? tiled_recomp_bytes(L, vb) : sub_rec_bytes(N, vb);
    return tiled_push_bytes(N, L, vb) + tiled_parent_bytes(N, L) + ((rec + 255) & ~(size_t)255);
}

namespace {  // (internal linkage, like hk_tiled_backtrack)
template <typename V, int N, int L>
__global__ __launch_bounds__(64 * kSubBtWaves) void hk_sub_backtrack(int nblocks, int blk0,
                                                                     const char *__restrict__ slots, uint32_t slot_bytes,
                                                                     const TiledInfo *__restrict__ info,
                                                                     const V *__restrict__ dist,
                                                                     V *__restrict__ cost_out,
                                                                     int32_t *__restrict__ tour_out)
{
    constexpr int NL = 1 << L, n = N + 1, VB = sizeof(V), K = sub_bt_k(N), NK = 1 << K;
    static_assert(K >= 1 && K <= 12 && K < N, "prefix DP size");
    __shared__ uint16_t lrank[NL];
    __shared__ int smoff[L + 2];
    __shared__ V drs[kSubBtWaves][N * N + N];  // per wave: d[m][k] (inner cities), then d[0][k]
    for (int i = threadIdx.x; i < NL; i += 64 * kSubBtWaves) lrank[i] = info->rank[i];
    if (threadIdx.x < (uint32_t)(L + 2)) smoff[threadIdx.x] = info->moff[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    V *dr = drs[wave];
    const V *d0 = dr + N * N;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    for (int blk = blk0 + (int)(blockIdx.x * kSubBtWaves + wave); blk < nblocks;
         blk += (int)(gridDim.x * kSubBtWaves)) {
        const V *dsrc = dist + (size_t)blk * n * n;
        for (int i = lane; i < N * N; i += 64) dr[i] = dsrc[(i / N + 1) * n + (i % N + 1)];
        if (lane < (uint32_t)N) dr[N * N + lane] = dsrc[lane + 1];
        wave_sync();
        int32_t *tour = tour_out + (size_t)blk * (n + 1);
        const int bestM = tour[n - 1];
        if (bestM < 1) continue;  // no tour (cost already -1)
        char *slot = const_cast<char *>(slots) + (size_t)(blk - blk0) * slot_bytes;
        Rsrc<uint64_t> par;
        par.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB), (uint32_t)tiled_parent_bytes(N, L));
        Rsrc<V> rec;
        rec.rs = uniform_rsrc(slot + tiled_push_bytes(N, L, VB) + tiled_parent_bytes(N, L),
                              (uint32_t)sub_rec_bytes(N, VB));
        uint32_t S = (1u << N) - 1u;
        int k = bestM - 1;
        bool ok = bestM >= 1 && bestM <= N;
        int pos = n - 2;
        // (1) parent words
        for (; ok && pos >= 1 && __builtin_popcount(S) - 1 >= N - TSPGPU_TILED_TA_OFF; --pos) {
            const uint32_t T = S & ~(1u << k);
            const uint32_t hT = T >> L, lT = T & (uint32_t)(NL - 1);
            const uint32_t idx = (uint32_t)smoff[__builtin_popcount(lT)] + lrank[lT];
            const uint64_t w = par.load(idx * 8u, hT * (uint32_t)(NL * 8));
            const int q = k - __builtin_popcount(T & ((1u << k) - 1u));  // k's place among T's non-members
            const int pm = (int)((w >> (4 * q)) & 15u);
            ok = pm < N && ((T >> pm) & 1u);
            if (lane == 0) tour[pos] = ok ? pm + 1 : 0;
            S = T;
            k = pm;
        }
        if (ok && pos >= 1) {
            // (2) the prefix set's own DP, local city i = the i-th member of T0 ascending
            const uint32_t T0 = S & ~(1u << k);
            ok = __builtin_popcount(T0) == K;
            int city[K];
            {
                uint32_t b = T0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    city[i] = b ? __builtin_ctz(b) : 0;
                    b &= b - 1u;
                }
            }
            // layer 1: G[{i}][i] = d[0][city i] (tsp.cpp:435)
            if (ok && lane < (uint32_t)K) rec.store(((1u << lane) * K + lane) * VB, 0, d0[city[lane]]);
            for (int j = 2; ok && j <= K; ++j) {
                wave_sync();
                for (uint32_t M = lane; M < (uint32_t)NK; M += 64) {
                    if (__builtin_popcount(M) != j) continue;
#pragma unroll
                    for (int kk = 0; kk < K; ++kk) {
                        if (!((M >> kk) & 1u)) continue;
                        const uint32_t P = M & ~(1u << kk);
                        V acc = ValT<V>::inf;
#pragma unroll
                        for (int m = 0; m < K; ++m)
                            if ((P >> m) & 1u)
                                acc = ValT<V>::vmin(acc, rec.load((P * K + m) * VB, 0) + dr[city[m] * N + city[kk]]);
                        rec.store((M * K + kk) * VB, 0, acc);
                    }
                }
            }
            wave_sync();
            // the walk below T0: first strict minimum over the members ascending
            uint32_t Mloc = (uint32_t)NK - 1u;
            for (; ok && pos >= 1; --pos) {
                const bool mem = lane < (uint32_t)K && ((Mloc >> lane) & 1u);
                V cand = ValT<V>::invalid;
                if (mem) cand = rec.load((Mloc * K + lane) * VB, 0) + dr[city[lane < (uint32_t)K ? lane : 0] * N + k];
                const V best = wave_min(cand);
                const unsigned long long hit = __ballot(mem && cand == best);
                const int li = hit ? __ffsll(hit) - 1 : K;
                ok = li < K;
                const int pm = ok ? city[li < K ? li : 0] : N;
                if (lane == 0) tour[pos] = ok ? pm + 1 : 0;
                if (ok) Mloc &= ~(1u << li);
                k = pm;
            }
        }
        if (!ok && lane == 0) cost_out[blk] = V(-1);
        wave_sync();  // dr is reloaded for the next block
    }
}

// ---------------------------------------------------------------------------
// Backtracking of variant 6, workgroup form (TSPGPU_SUB_BT = 1).
// The walk is hk_sub_backtrack's — (1) parent words while the set has
// >= N - TSPGPU_TILED_TA_OFF members, (2) the prefix set T0 (K = N - 5 cities)
// solved by its own Held-Karp, then the first strict minimum over T0's
// members ascending (tsp.cpp:457-470) — but laid out for latency:
//   * (1) runs one LANE per block, for every block the workgroup owns, before
//     any prefix DP (its four dependent parent-word loads are paid once per
//     workgroup, not once per block);
//   * (2) runs the whole workgroup on one block with the table in LDS, compact
//     (row M keeps its |M| member values: K * 2^(K-1) values, 40 KB at f64
//     K = 10), one barrier per layer.  Thread t owns destination kk = t / TPK
//     for the whole DP, so the K distances into kk sit in registers.
// Round 4's hk_tiled_backtrack recomputed whole sub-cube rows from the pushes
// through the slot's global recompute area, one wave per block (a chain of
// global round trips per layer: 1.75 ms per 65536 16-city blocks, 6.7% of the
// step).  Values are the forward pass's bits (same candidates, IEEE min is
// order-free), ties as the reference's.
// ---------------------------------------------------------------------------
#ifndef TSPGPU_SUB_BT
#define TSPGPU_SUB_BT 0  // (measured no faster than hk_tiled_backtrack yet: off)
#endif
#ifndef TSPGPU_SUB_BT_ABL
#define TSPGPU_SUB_BT_ABL 0  // timing ablations (results wrong): 1 no prefix DP, 2 no walk, 4 no DP barriers, 8 no input loads
#endif
constexpr int kSubBtThreads = 256;
// workgroups per CU: the LDS table decides (f64 K = 10: 46 KB)
__host__ __device__ constexpr int sub_bt_wg(int vb) { return vb == 8 ? 3 : 6; }

// one layer J of the prefix DP: thread (kk, sub) computes G[P | kk][kk] for the
// (J-1)-subsets P of T0 \ {kk} numbered sub, sub + TPK, ...  (all items of a
// thread unrolled: the table lookups of every item issue before the first row
// read, so a layer costs a few LDS round trips, not one per item).  Layer j is
// stored member-major: G[M][m] at layer_off(K, j) + (m's place in M) x C(K, j)
// + colex rank of M, so lanes reading neighbouring rows hit neighbouring banks.
template <typename V, int K, int J, int TPK>
__device__ __forceinline__ void sub_bt_layer(V *g, const uint16_t *sub9, const uint16_t *rk, const V (&dcol)[K],
                                             int kk, int sub)
{
    constexpr int CNT = cbinom(K - 1, J - 1), IT = (CNT + TPK - 1) / TPK;
    constexpr int BOFF = mask_off(K - 1, J - 1);  // first (J-1)-subset in sub9
    constexpr int RIN = layer_off(K, J - 1), CIN = cbinom(K, J - 1);
    constexpr int ROUT = layer_off(K, J), COUT = cbinom(K, J);
    const uint32_t below = (1u << kk) - 1u;
    uint32_t P[IT];
    int ro[IT], wo[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int p = sub + it * TPK;
        const uint32_t p9 = p < CNT ? sub9[BOFF + p] : 0u;
        P[it] = (p9 & below) | ((p9 & ~below) << 1);  // kk's bit left out
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const uint32_t M = P[it] | (1u << kk);
        ro[it] = RIN + rk[P[it]];
        wo[it] = ROUT + __builtin_popcount(M & below) * COUT + rk[M];
    }
    // branch-free: every lane loads K values, so an item's loads issue back to
    // back and wait once (an exec-masked load per member waits once per member)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        V v[K];
#pragma unroll
        for (int m = 0; m < K; ++m)  // (a non-member reads g[0]: one broadcast address, no extra bank traffic)
            v[m] = g[((P[it] >> m) & 1u) ? ro[it] + __builtin_popcount(P[it] & ((1u << m) - 1u)) * CIN : 0];
        V acc = ValT<V>::inf;
#pragma unroll
        for (int m = 0; m < K; ++m) acc = ValT<V>::vmin(acc, ((P[it] >> m) & 1u) ? v[m] + dcol[m] : ValT<V>::inf);
        if (sub + it * TPK < CNT) g[wo[it]] = acc;
    }
}
template <typename V, int K, int J, int TPK>
__device__ __forceinline__ void sub_bt_layers(V *g, const uint16_t *sub9, const uint16_t *rk, const V (&dcol)[K],
                                              int kk, int sub)
{
    if constexpr (J <= K) {
        if (kk < K) sub_bt_layer<V, K, J, TPK>(g, sub9, rk, dcol, kk, sub);
        if (!(TSPGPU_SUB_BT_ABL & 4)) __syncthreads();
        sub_bt_layers<V, K, J + 1, TPK>(g, sub9, rk, dcol, kk, sub);
    }
}

template <typename V, int N, int L>
__global__ __launch_bounds__(kSubBtThreads) void hk_sub_bt_wg(int nblocks, int blk0, const char *__restrict__ slots,
                                                              uint32_t slot_bytes, const TiledInfo *__restrict__ info,
                                                              const V *__restrict__ dist, V *__restrict__ cost_out,
                                                              int32_t *__restrict__ tour_out)
{
    constexpr int NL = 1 << L, n = N + 1, VB = sizeof(V), K = sub_bt_k(N), NK = 1 << K;
    constexpr int T = kSubBtThreads, TPK = T / K, DLV = K * K + K;
    static_assert(K >= 2 && K <= 10 && DLV + K <= T, "prefix DP size");
    __shared__ V g[K << (K - 1)];          // layer j member-major (sub_bt_layer)
    __shared__ V dl[DLV];                  // d[city m][city kk] at m * K + kk; d[city m][k0] at K * K + m
    __shared__ uint16_t rk[NK];            // colex rank of a subset among the subsets of its size
    __shared__ int lo[K + 1], cn[K + 1];   // layer_off(K, j), C(K, j)
    __shared__ uint16_t sub9[NK / 2];      // (K-1)-bit subsets by size, then colex rank
    __shared__ uint16_t wT0[T];            // (1)'s result per owned block: T0, k0 (-1: nothing left)
    __shared__ int8_t wk0[T];
    __shared__ int8_t city[K];
    const uint32_t tid = threadIdx.x;

    __shared__ uint16_t bn[K + 1][K + 1];  // binomials (setup only)
    if (tid == 0)
        for (int a = 0; a <= K; ++a)
            for (int b = 0; b <= K; ++b) bn[a][b] = b == 0 ? 1 : (a == 0 ? 0 : bn[a - 1][b - 1] + bn[a - 1][b]);
    __syncthreads();
    for (uint32_t M = tid; M < (uint32_t)NK; M += T) {
        int r = 0, i = 0;
        for (int b = 0; b < K; ++b)
            if ((M >> b) & 1u) r += bn[b][++i];
        const int j = __builtin_popcount(M);
        int lof = 0, mo = 0;  // layer_off(K, j), mask_off(K - 1, j)
        for (int u = 0; u < j; ++u) {
            lof += bn[K][u] * u;
            mo += bn[K - 1][u];
        }
        rk[M] = (uint16_t)r;
        if (M < (uint32_t)NK / 2) sub9[mo + r] = (uint16_t)M;
        if (M == (1u << j) - 1u) {  // one thread per layer
            lo[j] = lof;
            cn[j] = bn[K][j];
        }
    }

    const int kk = (int)tid / TPK, sub = (int)tid % TPK;  // this thread's destination (kk >= K: idle in the DP)
    for (int base = blk0 + (int)blockIdx.x; base < nblocks; base += T * (int)gridDim.x) {
        // (1) parent words, one lane per block
        {
            const int blk = base + (int)tid * (int)gridDim.x;
            uint32_t T0 = 0;
            int k0 = -1;
            if (blk < nblocks) {
                int32_t *tour = tour_out + (size_t)blk * (n + 1);
                const int bestM = tour[n - 1];
                if (bestM >= 1) {
                    const uint64_t *pw = reinterpret_cast<const uint64_t *>(slots + (size_t)(blk - blk0) * slot_bytes +
                                                                            tiled_push_bytes(N, L, VB));
                    uint32_t S = (1u << N) - 1u;
                    int k = bestM - 1, pos = n - 2;
                    bool ok = bestM <= N;
                    for (; ok && pos >= 1 && __builtin_popcount(S) - 1 >= N - TSPGPU_TILED_TA_OFF; --pos) {
                        const uint32_t Tm = S & ~(1u << k);
                        const uint32_t hT = Tm >> L, lT = Tm & (uint32_t)(NL - 1);
                        const uint32_t idx = (uint32_t)info->moff[__builtin_popcount(lT)] + info->rank[lT];
                        const uint64_t w = pw[(size_t)hT * NL + idx];
                        const int q = k - __builtin_popcount(Tm & ((1u << k) - 1u));  // k's place among the non-members
                        const int pm = (int)((w >> (4 * q)) & 15u);
                        ok = pm < N && ((Tm >> pm) & 1u);
                        tour[pos] = ok ? pm + 1 : 0;
                        S = Tm;
                        k = pm;
                    }
                    if (ok && pos >= 1) {
                        T0 = S & ~(1u << k);
                        ok = pos == K && __builtin_popcount(T0) == K;
                        k0 = k;
                    }
                    if (!ok) {
                        cost_out[blk] = V(-1);
                        k0 = -1;
                    }
                }
            }
            wT0[tid] = (uint16_t)T0;
            wk0[tid] = (int8_t)k0;
        }
        __syncthreads();
        const int owned = (nblocks - base + (int)gridDim.x - 1) / (int)gridDim.x;
        const int cntw = owned < T ? owned : T;
        // this thread's staged input of owned block i: a distance of dl, or
        // (K*K+K <= tid < K*K+2K) layer 1's G[{m}][m] = d[0][city m] (tsp.cpp:435)
        auto stage = [&](int i, int *cm) -> V {
            *cm = 0;
            if ((TSPGPU_SUB_BT_ABL & 8) || i >= cntw || wk0[i] < 0 || tid >= (uint32_t)(DLV + K)) return V(0);
            const uint32_t T0 = wT0[i];
            const int k0 = wk0[i];
            auto nth = [T0](int m) {  // the m-th member of T0 ascending
                uint32_t b = T0;
                for (int r = 0; r < m; ++r) b &= b - 1u;
                return __builtin_ctz(b);
            };
            const V *dsrc = dist + (size_t)(base + i * (int)gridDim.x) * n * n;
            if (tid < (uint32_t)(K * K)) return dsrc[(nth((int)tid / K) + 1) * n + nth((int)tid % K) + 1];
            if (tid < (uint32_t)DLV) return dsrc[(nth((int)tid - K * K) + 1) * n + k0 + 1];
            *cm = nth((int)tid - DLV);
            return dsrc[*cm + 1];
        };
        auto place = [&](V v, int cm) {
            if (tid < (uint32_t)DLV) {
                dl[tid] = v;
            } else if (tid < (uint32_t)(DLV + K)) {
                g[tid - DLV] = v;  // G[{m}][m] at layer_off(K, 1) + rank m
                city[tid - DLV] = (int8_t)cm;
            }
        };
        int cm = 0;
        V pf = stage(0, &cm);
        place(pf, cm);
        __syncthreads();
        // (2) one block at a time: prefix DP over T0, then the walk; the next
        // block's inputs are loaded meanwhile
        for (int i = 0; i < cntw; ++i) {
            const bool live = wk0[i] >= 0;  // (uniform)
            pf = stage(i + 1, &cm);
            if (live) {
                V dcol[K];
#pragma unroll
                for (int m = 0; m < K; ++m) dcol[m] = dl[m * K + (kk < K ? kk : 0)];
                if (!(TSPGPU_SUB_BT_ABL & 1)) sub_bt_layers<V, K, 2, TPK>(g, sub9, rk, dcol, kk, sub);
                if (tid < 64 && !(TSPGPU_SUB_BT_ABL & 2)) {
                    const int blk = base + i * (int)gridDim.x;
                    int32_t *tour = tour_out + (size_t)blk * (n + 1);
                    const uint32_t lane = tid;
                    uint32_t Mloc = (uint32_t)NK - 1u;
                    int kl = -1;  // the current city's local index (-1: k0, outside T0)
                    bool ok = true;
                    for (int pos = K; ok && pos >= 1; --pos) {
                        const int jm = __builtin_popcount(Mloc);
                        const bool mem = lane < (uint32_t)K && ((Mloc >> lane) & 1u);
                        V cand = ValT<V>::invalid;
                        if (mem)
                            cand = g[lo[jm] + __builtin_popcount(Mloc & ((1u << lane) - 1u)) * cn[jm] + rk[Mloc]] +
                                   (kl < 0 ? dl[K * K + lane] : dl[lane * K + kl]);
                        const V best = wave_min(cand);
                        const unsigned long long hit = __ballot(mem && cand == best);
                        const int li = hit ? __ffsll(hit) - 1 : K;
                        ok = li < K;
                        if (lane == 0) tour[pos] = ok ? city[li] + 1 : 0;
                        if (ok) Mloc &= ~(1u << li);
                        kl = li;
                    }
                    if (!ok && lane == 0) cost_out[blk] = V(-1);
                }
            }
            __syncthreads();  // g, dl and city are the next block's
            place(pf, cm);
            __syncthreads();
        }
    }
}
}  // namespace

struct SubArgs {
    const void *dist;
    int n, blk0, blk1;
    char *slots;
    uint32_t slot_bytes;
    const SubRow *rows;       // row table of L
    const TiledInfo *info;    // (backtracking)
    void *cost;
    int32_t *tour;
    int grid, bt_grid;
    int cus;                  // compute units (the workgroup-form backtracking's grid)
    hipStream_t stream;
    hipEvent_t ev_mid;
};

template <typename V, int N, int L, int THREADS, int WG>
hipError_t launch_sub_n(const SubArgs &a)
{
    hipLaunchKernelGGL((hk_sub_kernel<V, N, L, THREADS, WG>), dim3(a.grid), dim3(THREADS), 0, a.stream,
                       static_cast<const V *>(a.dist), a.blk1, a.blk0, a.slots, a.slot_bytes, a.rows,
                       static_cast<V *>(a.cost), a.tour);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && a.ev_mid) e = hipEventRecord(a.ev_mid, a.stream);
    if (e != hipSuccess) return e;
    if constexpr (TSPGPU_SUB_STAMP) return hipSuccess;  // (diagnostic build: the tour words hold the stamps)
    if constexpr (TSPGPU_SUB_BT && !TSPGPU_SUB_RECYCLE) {
        const int nb = a.blk1 - a.blk0, cap = a.cus * sub_bt_wg(sizeof(V));
        const int g = nb < cap ? nb : cap;
        hipLaunchKernelGGL((hk_sub_bt_wg<V, N, L>), dim3(g), dim3(kSubBtThreads), 0, a.stream, a.blk1, a.blk0,
                           a.slots, a.slot_bytes, a.info, static_cast<const V *>(a.dist), static_cast<V *>(a.cost),
                           a.tour);
    } else if constexpr (TSPGPU_SUB_RECYCLE)
        hipLaunchKernelGGL((hk_sub_backtrack<V, N, L>), dim3(a.bt_grid), dim3(64 * kSubBtWaves), 0, a.stream, a.blk1,
                           a.blk0, a.slots, a.slot_bytes, a.info, static_cast<const V *>(a.dist),
                           static_cast<V *>(a.cost), a.tour);
    else
        hipLaunchKernelGGL((hk_tiled_backtrack<V, N, L>), dim3(a.bt_grid), dim3(64 * kTiledBtWaves), 0, a.stream,
                           a.blk1, a.blk0, a.slots, a.slot_bytes, a.info, static_cast<const V *>(a.dist),
                           static_cast<V *>(a.cost), a.tour);
    return hipGetLastError();
}

}  // namespace tspgpu
