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
// the region holds the two live low layers (tiled_region_vals): layer j at
// the bottom when j is even, at the top when odd
__host__ __device__ constexpr int sub_region_vals(int L) { return tiled_region_vals(L); }
__host__ __device__ constexpr int sub_layer_off(int L, int j)
{
    return (j & 1) ? tiled_region_vals(L) - tiled_layer_vals(L, j) : 0;
}
// Overlapped edge passes (256-thread workgroups): passes 0/1 of sub-cube h + 1
// run during the last middle pass of h and pass L of h during the first middle
// pass of h + 1, on the waves those passes leave idle; the push values of
// passes 0/1, L - 1 and L are staged into LDS one pass earlier — the separate
// edge interval and its exposed memory round trips go away (round 5: -3%
// forward, profiles/r05).  Needs layer 2 of the next sub-cube outside the
// region (C(L,2) x 2 values) and the staged values.
__host__ __device__ constexpr int sub_l2_vals(int L) { return cbinom(L, 2) * 2; }
__host__ __device__ constexpr size_t sub_lds_bytes(int N, int L, int vb)
{
    return sub_img_bytes(N, L, vb) + (size_t)2 * 16 * vb + (size_t)sub_region_vals(L) * vb + (size_t)16 * vb +
           (size_t)(sub_l2_vals(L) + L * (N - L)) * vb + (size_t)((L + 1) * (N - L) + (N - L)) * vb;
}

template <typename V, int N, int L>
struct SubCtx {
    char *img;         // LDS distance image (bytes): natural rows/columns 0..N-1, sub-cube-ordered N..N+H-1
    const V *d0;       // d[0][k], k = 1..N at [k-1]
    V *region;         // live low layers (as variant 5)
    V *layerL;         // G[h | full low][m], m low: written by pass L-1, read by pass L
    V *layer2;         // layer 2 (passes 0/1 write it, middle pass 2 reads it): the region's
                       // bottom, or its own area when the edge passes overlap
    V *pst;            // pass L-1's push values staged in LDS (overlapped edge passes): [row][i]
    V *fst;            // passes 0/1's push values: [i] row 0, [H + a*H + i] row {a}
    V *lst;            // pass L's push values: [i]
    int ov;            // 2: overlapped edge passes (256-thread workgroups), 0: separate edge intervals
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

#ifndef TSPGPU_SUB_QC
#define TSPGPU_SUB_QC 7
#endif
#ifndef TSPGPU_SUB_AHEAD
#define TSPGPU_SUB_AHEAD 6
#endif
constexpr int kSubQC = TSPGPU_SUB_QC;        // destinations relaxed together (register budget)
constexpr int kSubAhead = TSPGPU_SUB_AHEAD;  // distance loads in flight per lane

// the push column of (sub-cube hp, high city x): [hp][x] in the slot's push area
template <int H>
__device__ __forceinline__ uint32_t sub_col(uint32_t hp, uint32_t x)
{
    return hp * H + x;
}

// Measured and not kept (A/B logs under profiles/r03-r05; the switches were
// removed from this header in round 6): one low layer in LDS (+5%), push
// columns recycled into 23 slots with a prefix-set backtracking (+6%), push
// stores deferred behind the next pass's loads (+14%, spills), the next pass's
// push loads issued early (+18%: they wait behind older stores in the in-order
// vmcnt), rotated wave roles, scalar loads of the high-high distances (+60%),
// one |h| dispatch per sub-cube, a workgroup-form backtracking (no faster).

template <typename V, int N, int L, int T, int J>
__device__ __forceinline__ void sub_mid(const SubCtx<V, N, L> &c, uint32_t h, uint32_t tid, const uint4 &ent)
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
    // high-high distances of this sub-cube: wave-uniform, from the LDS image
    V hh[HC * QH > 0 ? HC * QH : 1];
#pragma unroll
    for (int i = 0; i < HC; ++i)
#pragma unroll
        for (int u = 0; u < QH; ++u) hh[i * QH + u] = uniform_val<V>(c.img, HR0 + i * DSB + HC0 + u * VB);
    const uint32_t r = tid;
    const bool act = r < (uint32_t)ROWS;
    V g[T];
    {
        const V *src = J == 2 ? c.layer2 : c.region + CUR;
#pragma unroll
        for (int p = 0; p < J; ++p) g[p] = act ? src[p * ROWS + r] : V(0);
    }
    const uint32_t voff = (BASE + r) * VB;  // the row's offset in a push column
    if (act) {
#pragma unroll
        for (int i = 0; i < HC; ++i) g[J + i] = c.push.load(voff, sub_col<H>(h, hm[i]) * (uint32_t)(NL * VB));
    }
    if (!act) return;
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
    constexpr int QC = kSubQC;
    static_for<(Q + QC - 1) / QC>([&](auto ci) {
        constexpr int C0 = decltype(ci)::value * QC;
        constexpr int QN = Q - C0 < QC ? Q - C0 : QC;
        constexpr int CNT = sub_lds_count<T, J, QL, C0, QN>();
        constexpr int AH = kSubAhead < CNT ? kSubAhead : CNT;
        // integer min-only rows: member pairs per destination (v_min3_i32)
        constexpr bool QP = !ARG && std::is_same<V, int32_t>::value;
        V acc[QN];
        uint32_t arg[ARG ? QN : 1];
        // distance of LDS relaxation k (compile-time pair)
        auto dload = [&](auto kk) -> V {
            constexpr int pq = sub_lds_pair<T, J, QL, C0, QN, QP>(decltype(kk)::value);
            constexpr int p = pq / 64, q = C0 + pq % 64;
            if constexpr (p < J && q < QL)
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
        } else if constexpr (!ARG) {
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
                __builtin_amdgcn_sched_barrier(0);
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
// Pass L-1's push values of sub-cube h (|h| = C) into LDS (overlapped edge passes):
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

// Passes 0/1's push values of sub-cube h (|h| = C) into LDS (overlapped edge
// passes): lanes e < C row 0 of column (h, hm_e); lanes C + a*C + i row {a} of
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
                                                   const uint4 &ent)
{
    constexpr int H = N - L;
#define TSPGPU_SM(HC)                                                                                  \
    case HC:                                                                                           \
        if constexpr (HC <= H) sub_mid<V, N, L, J + (HC <= H ? HC : 0), J>(c, h, tid, ent);  \
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
template <typename V, int N, int L, int THREADS, int WG>
__global__ __launch_bounds__(THREADS, tiled_waves(THREADS, WG)) void hk_sub_kernel(
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
    constexpr int OV = THREADS == 256 ? 2 : 0;
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
        for (uint32_t h = 0; h < (uint32_t)NH; ++h) {
            const int hc = __builtin_popcount(h);
            // interval A(h): passes 0/1 of h (lanes < 192) beside pass L of h - 1 (lanes 192..)
            // (overlapped: at h = 0 only; later they run inside the middle passes)
            uint32_t t = opaque_u32(tid);
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
                __syncthreads();
            }
            // middle passes j = 2..L-2, unrolled (every offset a compile-time
            // constant); the next pass's row entry is loaded one pass ahead
            static_for<L - 3>([&](auto jj) {
                constexpr int j = 2 + decltype(jj)::value;
                const uint4 cur = ent;
                const uint32_t tj = opaque_u32(tid);
                if constexpr (j + 1 <= L - 2) {
                    constexpr int MN = tiled_moff(L, j + 1), CN = cbinom(L, j + 1);
                    ent = rowtab[MN + (tj < (uint32_t)CN ? tj : 0u)];
                }
                sub_dispatch_mid_j<V, N, L, j>(c, h, hc, tj, cur);
                if constexpr (OV) {
                    // edge passes on the waves this middle pass leaves idle
                    static_assert(cbinom(L, 2) <= 64 && cbinom(L, 3) <= 128 && cbinom(L, L - 3) <= 128, "overlap: idle waves");
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
                    if constexpr (j == L - 2) {  // passes 0/1 of h + 1 (layer 2 in its own area)
                        if (h + 1 < (uint32_t)NH && tj >= 64u)
                            sub_dispatch_first<V, N, L>(c, h + 1, __builtin_popcount(h + 1), tj - 64u);
                    }
                }
                lds_barrier();
            });
            // pass L - 1 (lanes < 128) beside the next sub-cube's high image rows/columns (lanes 128..)
            t = opaque_u32(tid);
#pragma unroll
            for (uint32_t v0 = 0; v0 < 256u; v0 += THREADS) {
                const uint32_t v = t + v0;
                if (v < 128u)
                    sub_dispatch_penult<V, N, L>(c, h, hc, v);
                else if (h + 1 < (uint32_t)NH)
                    sub_build_high<V, N, L>(c, h + 1, v - 128u);
            }
            __syncthreads();
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

// one block's global slot for variant 6: variant 5's layout (push area, parent
// words, recompute area), so hk_tiled_backtrack completes the tours
__host__ __device__ constexpr size_t sub_slot_bytes(int N, int L, int vb) { return tiled_slot_bytes(N, L, vb); }

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
    hipLaunchKernelGGL((hk_tiled_backtrack<V, N, L>), dim3(a.bt_grid), dim3(64 * kTiledBtWaves), 0, a.stream, a.blk1,
                       a.blk0, a.slots, a.slot_bytes, a.info, static_cast<const V *>(a.dist), static_cast<V *>(a.cost),
                       a.tour);
    return hipGetLastError();
}

}  // namespace tspgpu
