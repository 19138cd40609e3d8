// C-ABI of libtspgpu (include/tspgpu.h): context, validation, host<->device
// staging, launch of the K1 Held-Karp kernels (heldkarp.hip).
//
// Replaces the reference's `BlockSolution tsp(vector<City>)` (tsp.cpp:405-509)
// for a whole batch of blocks in one call.  The distance matrix stays on the
// host (computeDistanceMatrix, assignment2.h:184-200) because glibc pow(x,2)
// differs from x*x in ~0.08% of inputs; the device never recomputes it.
#include "tspgpu.h"
#include "tuning.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"
#include "heldkarp.h"
#include "k1_cfg.h"
#include "xfer.h"

namespace tspgpu {

static int binom_host(int a, int b)
{
    if (b < 0 || b > a) return 0;
    long long r = 1;
    for (int i = 1; i <= b; ++i) r = r * (a - b + i) / i;
    return (int)r;
}

size_t table_doubles(int N) { return (size_t)N << (N - 1); }

void host_layer_info(int N, LayerInfo *info)
{
    std::memset(info, 0, sizeof(*info));
    for (int a = 0; a < kBinomRows; ++a)
        for (int b = 0; b < kBinomCols; ++b) info->binom[a * kBinomCols + b] = binom_host(a, b);
    // colex rank = sum over members e_i (ascending) of C(e_i, i+1), split in
    // three 7-bit digit groups whose contribution depends on the member count below
    for (int lo = 0; lo < 128; ++lo) {
        int r = 0, i = 0;
        for (int b = 0; b < 7; ++b)
            if (lo >> b & 1) r += binom_host(b, ++i);
        info->rlut[lo] = r;
    }
    for (int mid = 0; mid < 128; ++mid)
        for (int c = 0; c < 8; ++c) {
            int r = 0, i = c;
            for (int b = 0; b < 7; ++b)
                if (mid >> b & 1) r += binom_host(b + 7, ++i);
            info->rlut[kRankR1 + mid * 8 + c] = r;
        }
    for (int hi = 0; hi < 64; ++hi)
        for (int c = 0; c < 15; ++c) {
            int r = 0, i = c;
            for (int b = 0; b < 6; ++b)
                if (hi >> b & 1) r += binom_host(b + 14, ++i);
            info->rlut[kRankR1 + kRankR2 + hi * 15 + c] = r;
        }
    int off = 0, moff = 0;
    for (int t = 0; t <= N + 1 && t < 24; ++t) {
        info->count[t] = binom_host(N, t);
        info->moff[t] = moff;
        moff += info->count[t];
        if (t >= 1) {
            info->off[t] = off;
            off += info->count[t] * t;
        }
    }
}

}  // namespace tspgpu

using namespace tspgpu;


namespace {

int hip_err(hipError_t e)
{
    if (e == hipSuccess) return 0;
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return -ENODEV;
    return -EIO;
}

template <typename T>
int ensure(T **p, size_t *have, size_t need)
{
    if (*have >= need && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    size_t alloc = need < 256 ? 256 : need;
    hipError_t e = hipMalloc((void **)p, alloc);
    if (e != hipSuccess) {
        *p = nullptr;
        return hip_err(e);
    }
    *have = alloc;
    return 0;
}

// a one-time table upload on the context's stream (xfer.h: small tables skip
// the runtime's copy path and its first-use cost)
hipError_t upload_sync(tspgpu_ctx *c, void *d, const void *h, size_t bytes)
{
    hipError_t e = xcopy_async(d, h, bytes, hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}

int ensure_tables(tspgpu_ctx *c, int N)
{
    if (c->d_info[N]) return 0;
    LayerInfo info;
    host_layer_info(N, &info);
    // every N-bit mask by (popcount, value): each popcount class in ascending
    // order by Gosper's next-combination step (O(2^N), not (N+1) 2^N scans)
    std::vector<uint32_t> masks;
    masks.reserve((size_t)1 << N);
    masks.push_back(0u);
    for (int t = 1; t <= N; ++t)
        for (uint32_t m = (1u << t) - 1u; m < (1u << N);) {
            masks.push_back(m);
            const uint32_t c = m & (0u - m), r = m + c;
            m = (((r ^ m) >> 2) / c) | r;
        }
    hipError_t e = hipMalloc((void **)&c->d_info[N], sizeof(LayerInfo));
    if (e == hipSuccess) e = hipMalloc((void **)&c->d_masks[N], masks.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = upload_sync(c, c->d_info[N], &info, sizeof(info));
    if (e == hipSuccess)
        e = upload_sync(c, c->d_masks[N], masks.data(), masks.size() * sizeof(uint32_t));
    if (e != hipSuccess) {
        if (c->d_info[N]) (void)hipFree(c->d_info[N]);
        if (c->d_masks[N]) (void)hipFree(c->d_masks[N]);
        c->d_info[N] = nullptr;
        c->d_masks[N] = nullptr;
        return hip_err(e);
    }
    return 0;
}

int ensure_tiled_info(tspgpu_ctx *c, int L)
{
    if (c->d_tinfo[L]) return 0;
    auto info = std::make_unique<TiledInfo>();
    std::memset(info.get(), 0, sizeof(TiledInfo));
    int k = 0;
    for (int j = 0; j <= L; ++j) {
        info->moff[j] = k;
        info->cnt[j] = binom_host(L, j);
        int r = 0;
        for (uint32_t m = 0; m < (1u << L); ++m)
            if (__builtin_popcount(m) == j) {  // numeric order of equal-popcount masks = colex order
                info->mask[k++] = (uint16_t)m;
                info->rankb8[m] = (uint16_t)(r * 8);
                info->rankb4[m] = (uint16_t)(r * 4);
                info->rank[m] = (uint16_t)r++;
            }
    }
    info->moff[L + 1] = k;
    void *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(TiledInfo));
    if (e == hipSuccess) e = upload_sync(c, d, info.get(), sizeof(TiledInfo));
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return hip_err(e);
    }
    c->d_tinfo[L] = d;
    return 0;
}

// Variants 5/6 keep one global slot per block of a launch (1.65 MB at
// n = 16) until its backtracking kernel has run, so a launch takes blocks in
// chunks: up to 65536 (108 GB of the 288 GB at n = 16 — a persistent grid of
// 1536 workgroups then idles a third of the chip for 0.67 of 42.7 rounds
// instead of 0.67 of 10.7 at 16384), at most 3/4 of the device memory free
// at that moment (other contexts or ranks on the same GPU keep theirs),
// halved while the allocation fails, down to 64 blocks.  A slot area far
// larger than a later launch needs (> 4x and > 8 GB) is given back first.
int ensure_slots(tspgpu_ctx *c, int nblocks, size_t slot, int *chunk)
{
    int ch = std::min(nblocks, 65536);
    const size_t need = (size_t)ch * slot;
    if (c->d_tslots && c->tslots_bytes > 4 * need && c->tslots_bytes > ((size_t)8 << 30)) {
        (void)hipFree(c->d_tslots);
        c->d_tslots = nullptr;
        c->tslots_bytes = 0;
    }
    if (c->tslots_bytes < need) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const size_t usable = (free_b + c->tslots_bytes) / 4 * 3;  // (the current area is freed first)
            while (ch > 64 && (size_t)ch * slot > usable) ch /= 2;
        }
    }
    for (;;) {
        const int rc = ensure(&c->d_tslots, &c->tslots_bytes, (size_t)ch * slot);
        if (rc == 0 || rc != -ENOMEM || ch <= 64) {
            *chunk = ch;
            return rc;
        }
        (void)hipGetLastError();  // (clear the failed allocation's error)
        ch /= 2;
    }
}

// Split timing (tspgpu_k1_split_timing): three events per chunk, kept until
// tspgpu_k1_last_split_ms reads them; the first is recorded here.  *ev0 = the
// chunk's first event index (unused when split timing is off).
int split_begin(tspgpu_ctx *c, hipStream_t stream, size_t *ev0)
{
    *ev0 = 0;
    if (!c->split_timing) return 0;
    constexpr size_t kMaxEvents = 3 * 4096;
    if (c->split_used + 3 > kMaxEvents) {  // more chunks than the pool: stop recording
        c->split_overflow = true;
        c->split_timing = 0;
        return 0;
    }
    while (c->ev_split.size() < c->split_used + 3) {
        hipEvent_t ev = nullptr;
        if (hipEventCreate(&ev) != hipSuccess) return -EIO;
        c->ev_split.push_back(ev);
    }
    *ev0 = c->split_used;
    c->split_used += 3;
    return hipEventRecord(c->ev_split[*ev0], stream) == hipSuccess ? 0 : -EIO;
}

// Variant 6 row table of L (hk_sub.h SubRow): per L-bit mask, its members
// then non-members as nibbles, and the colex rank of mask | (1 << k) for every
// non-member k (the destination row of the next low layer).
int ensure_sub_rows(tspgpu_ctx *c, int L)
{
    if (L > 10) return -EINVAL;  // 8-bit ranks: C(10, 5) = 252
    if (c->d_subrows[L]) return 0;
    int rc = ensure_tiled_info(c, L);
    if (rc) return rc;
    std::vector<int> rank(1 << L, 0);
    std::vector<uint32_t> order;  // masks by (popcount, value) = TiledInfo::mask
    for (int j = 0; j <= L; ++j) {
        int r = 0;
        for (uint32_t m = 0; m < (1u << L); ++m)
            if (__builtin_popcount(m) == j) {
                rank[m] = r++;
                order.push_back(m);
            }
    }
    std::vector<SubRow> rows(order.size());
    for (size_t i = 0; i < order.size(); ++i) {
        const uint32_t m = order[i];
        uint8_t bytes[16] = {0};
        int slot = 0, q = 0;
        auto put_nib = [&](int idx, uint32_t v) { bytes[idx / 2] |= (uint8_t)(v << (4 * (idx & 1))); };
        for (int b = 0; b < L; ++b)
            if (m >> b & 1) put_nib(slot++, (uint32_t)b);
        for (int b = 0; b < L; ++b)
            if (!(m >> b & 1)) {
                put_nib(slot++, (uint32_t)b);
                bytes[5 + q++] = (uint8_t)rank[m | (1u << b)];
            }
        std::memcpy(rows[i].w, bytes, 16);
    }
    void *d = nullptr;
    hipError_t e = hipMalloc(&d, rows.size() * sizeof(SubRow));
    if (e == hipSuccess) e = upload_sync(c, d, rows.data(), rows.size() * sizeof(SubRow));
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return hip_err(e);
    }
    c->d_subrows[L] = d;
    return 0;
}

// K1 variant 6 (hk_sub.h) configuration for (N, value bytes): the one
// TSPGPU_TILED_CFG names, else the first row of the table; null if none.
const SubCfg *pick_sub(const tspgpu_ctx *c, int N, int vbytes)
{
    int cnt = 0;
    const SubCfg *t = sub_cfgs(&cnt);
    if (c->tiled_cfg >= 0) {
        for (int i = 0; i < cnt; ++i)
            if (t[i].id == c->tiled_cfg && t[i].N == N && t[i].vbytes == vbytes) return &t[i];
        return nullptr;
    }
    for (int i = 0; i < cnt; ++i)
        if (t[i].N == N && t[i].vbytes == vbytes) return &t[i];
    return nullptr;
}

int solve_sub(tspgpu_ctx *c, const SubCfg *cfg, const void *d_dist, int n, int nblocks, void *d_cost,
              int32_t *d_tour, hipStream_t stream)
{
    const int N = n - 1, L = cfg->L;
    int rc = ensure_sub_rows(c, L);
    if (rc) return rc;
    // (TSPGPU_WG_PER_CU: measurement builds with another occupancy, hk_sub.h)
    const int grid = std::min(nblocks, c->cu_count * (c->wg_per_cu > 0 ? c->wg_per_cu : cfg->wg));
    // variant 5's per-block slot (push area, parent words, recompute area,
    // large enough for either backtracking kernel), kept until the
    // backtracking kernel has run
    const size_t slot = sub_slot_bytes(N, L, cfg->vbytes);
    int chunk = 0;
    if ((rc = ensure_slots(c, nblocks, slot, &chunk))) return rc;
    for (int b0 = 0; b0 < nblocks; b0 += chunk) {
        SubArgs a{};
        size_t ev0 = 0;
        if ((rc = split_begin(c, stream, &ev0))) return rc;
        a.ev_mid = c->split_timing ? c->ev_split[ev0 + 1] : nullptr;
        a.dist = d_dist;
        a.n = n;
        a.blk0 = b0;
        a.blk1 = std::min(nblocks, b0 + chunk);
        a.slots = c->d_tslots;
        a.slot_bytes = (uint32_t)slot;
        a.rows = static_cast<const SubRow *>(c->d_subrows[L]);
        a.info = static_cast<const TiledInfo *>(c->d_tinfo[L]);
        a.cost = d_cost;
        a.tour = d_tour;
        a.grid = std::min(grid, a.blk1 - a.blk0);
        a.bt_grid = std::min((a.blk1 - a.blk0 + kTiledBtWaves - 1) / kTiledBtWaves, c->cu_count * TSPGPU_TILED_BTWG);
        a.stream = stream;
        hipError_t e = cfg->launch(a);
        if (e != hipSuccess) return hip_err(e);
        if (c->split_timing && hipEventRecord(c->ev_split[ev0 + 2], stream) != hipSuccess) return -EIO;
    }
    c->last_grid = grid;
    c->last_variant = 6;
    return 0;
}

// K1 variant 5 (sub-cube tiled, hk_tiled.h) configuration for (N, value
// bytes): TSPGPU_TILED_CFG / c->tiled_cfg, else the measured default; null if
// none exists for this size.
const TiledCfg *pick_tiled(const tspgpu_ctx *c, int N, int vbytes)
{
    int cnt = 0;
    const TiledCfg *t = tiled_cfgs(&cnt);
    if (c->tiled_cfg >= 0) {
        for (int i = 0; i < cnt; ++i)
            if (t[i].id == c->tiled_cfg && t[i].N == N && t[i].vbytes == vbytes) return &t[i];
        return nullptr;
    }
    for (int i = 0; i < cnt; ++i)  // first row of the table for this size is the default
        if (t[i].N == N && t[i].vbytes == vbytes) return &t[i];
    return nullptr;
}

int solve_tiled(tspgpu_ctx *c, const TiledCfg *cfg, const void *d_dist, int n, int nblocks, void *d_cost,
                int32_t *d_tour, hipStream_t stream)
{
    const int N = n - 1, L = cfg->L;
    int rc = ensure_tiled_info(c, L);
    if (rc) return rc;
    const int grid = std::min(nblocks, c->cu_count * cfg->wg);
    // one global slot per block (push area, parent words of the top rows,
    // backtracking recompute area: 1.65 MB at n = 16, hk_tiled.h), kept until
    // the backtracking kernel of the launch has run (ensure_slots: chunks)
    const size_t slot = tiled_slot_bytes(N, L, cfg->vbytes);
    int chunk = 0;
    if ((rc = ensure_slots(c, nblocks, slot, &chunk))) return rc;
    for (int b0 = 0; b0 < nblocks; b0 += chunk) {
        TiledArgs a{};
        size_t ev0 = 0;
        if ((rc = split_begin(c, stream, &ev0))) return rc;
        a.ev_mid = c->split_timing ? c->ev_split[ev0 + 1] : nullptr;
        a.dist = d_dist;
        a.n = n;
        a.blk0 = b0;
        a.blk1 = std::min(nblocks, b0 + chunk);
        a.slots = c->d_tslots;
        a.slot_bytes = (uint32_t)slot;
        a.info = static_cast<const TiledInfo *>(c->d_tinfo[L]);
        a.cost = d_cost;
        a.tour = d_tour;
        a.grid = std::min(grid, a.blk1 - a.blk0);
        a.bt_grid = std::min((a.blk1 - a.blk0 + kTiledBtWaves - 1) / kTiledBtWaves, c->cu_count * TSPGPU_TILED_BTWG);
        a.stream = stream;
        hipError_t e = cfg->launch(a);
        if (e != hipSuccess) return hip_err(e);
        if (c->split_timing && hipEventRecord(c->ev_split[ev0 + 2], stream) != hipSuccess) return -EIO;
    }
    c->last_grid = grid;
    c->last_variant = 5;
    return 0;
}

int check_n(int n, int strict)
{
    if (n < 2) return -EINVAL;
    if (n > (strict ? TSPGPU_REFERENCE_MAX_CITIES : TSPGPU_MAX_CITIES)) return -EINVAL;
    return 0;
}

int solve_device_unordered(tspgpu_ctx *c, const void *d_dist, int n, int nblocks, void *d_cost, int32_t *d_tour,
                           hipStream_t stream, int vbytes);

// Launches share the context's workspace (slots, push areas, parent words):
// a launch on another stream than the previous one first waits for it, and
// every launch records the completion event the next one may wait for.
int solve_device_locked(tspgpu_ctx *c, const void *d_dist, int n, int nblocks, void *d_cost, int32_t *d_tour,
                        hipStream_t stream, int vbytes)
{
    if (nblocks > 0 && hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    if (nblocks > 0 && c->k1_launched && stream != c->k1_last_stream) {
        hipError_t e = hipStreamWaitEvent(stream, c->ev_k1_done, 0);
        if (e != hipSuccess) return hip_err(e);
    }
    int rc = solve_device_unordered(c, d_dist, n, nblocks, d_cost, d_tour, stream, vbytes);
    if (rc || nblocks <= 0) return rc;
    hipError_t e = hipSuccess;
    if (!c->ev_k1_done) e = hipEventCreateWithFlags(&c->ev_k1_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(c->ev_k1_done, stream);
    if (e != hipSuccess) return hip_err(e);
    c->k1_last_stream = stream;
    c->k1_launched = true;
    return 0;
}

int solve_device_unordered(tspgpu_ctx *c, const void *d_dist, int n, int nblocks, void *d_cost, int32_t *d_tour,
                           hipStream_t stream, int vbytes)
{
    int rc = check_n(n, c->strict);
    if (rc) return rc;
    if (nblocks < 0 || (nblocks > 0 && (!d_dist || !d_cost || !d_tour))) return -EINVAL;
    if (nblocks == 0) return 0;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    const int N = n - 1;
    LaunchArgs a{};
    a.dist = d_dist;
    a.n = n;
    a.nblocks = nblocks;
    a.cost = d_cost;
    a.tour = d_tour;
    a.stream = stream;
    a.vbytes = vbytes;
    int grid = nblocks;
    if (N >= 2) {
        rc = ensure_tables(c, N);
        if (rc) return rc;
        a.masks = c->d_masks[N];
        a.info = c->d_info[N];
        a.use_lds = N <= c->lds_table_max_n;
        // per-N defaults measured on MI355X (profiles/r01/*sweep*.log): small
        // tables want many blocks in flight; at n = 15, 16 one 1024-thread slot
        // per CU keeps the live layers of the 256 resident blocks in the
        // Infinity Cache (n = 15: 1.45x over two 512-thread slots)
        // (i32 tables are half the bytes: 512-thread pairs at n = 15, 16 and
        // 8 workgroups per CU up to n = 13; profiles/r01/i32_sweep*.log)
        int def_threads = N <= 11 ? 256 : (N <= 13 ? 512 : (N <= 15 ? 1024 : 256));
        int def_wg = N <= 11 ? 8 : (N <= 13 ? 2 : (N <= 15 ? 1 : 2));
        if (vbytes == 4) {
            def_threads = N <= 13 ? 256 : (N <= 15 ? 512 : 256);
            def_wg = N <= 12 ? 8 : (N <= 13 ? 4 : 2);
        }
        a.threads = c->threads > 0 ? c->threads : def_threads;
        // ping-pong + parents pays at 16 cities (the two live middle layers of
        // all 256 resident blocks then stay in the Infinity Cache), not below
        // (with a full wave of blocks: one block alone is latency-bound and the
        // argmin's extra VALU only costs there)
        // a full wave of blocks: the sub-cube kernels — variant 6 (hk_sub.h)
        // where it has a configuration, else variant 5 (hk_tiled.h) — at
        // 13-16 cities f64 and 16 cities i32 (round 2, per 16384 blocks:
        // variant 5 n = 16 f64 7.6 vs 12.0 ms for variant 4, n = 15 3.75 vs
        // 4.59, n = 14 1.80 vs 2.20, n = 13 0.88 vs 1.06, n = 16 i32 5.72 vs
        // 7.63 for variant 2, profiles/r02/k1_tiled_v17_cfgs.log); the compact
        // layer pass (variant 2) elsewhere
        const bool tiled = vbytes == 8 ? (N >= 12 && N <= 15) : N == 15;
        a.variant = c->variant >= 0 ? c->variant : (tiled && nblocks >= c->cu_count ? 6 : 2);
        if (a.variant == 6) {
            if (const SubCfg *cfg = pick_sub(c, N, vbytes))
                return solve_sub(c, cfg, d_dist, n, nblocks, d_cost, d_tour, stream);
            a.variant = 5;  // no variant-6 configuration for this size
        }
        if (a.variant == 5) {
            if (const TiledCfg *cfg = pick_tiled(c, N, vbytes))
                return solve_tiled(c, cfg, d_dist, n, nblocks, d_cost, d_tour, stream);
            a.variant = vbytes == 8 && N == 15 ? 4 : 2;  // no tiled configuration for this size
        }
        // variant 4 at 16 cities: one 512-thread workgroup per CU at 2 waves/SIMD
        // (256 VGPRs; heldkarp_impl.h TSPGPU_K1_WAVES_512V4) beats 1024 threads at 4
        if (c->threads <= 0 && a.variant == 4 && N == 15 && vbytes == 8) a.threads = 512;
        if (a.use_lds) {
            // as many resident workgroups as the LDS allows, then persistent
            const int per_cu = (int)(160 * 1024 / lds_bytes_for(N, true, threads_for(N, true, 0), vbytes == 4 || a.variant >= 1, vbytes));
            const int cap = c->cu_count * (per_cu > 0 ? per_cu : 1);
            grid = nblocks < cap ? nblocks : cap;
        } else {
            // extension sizes (N >= 16) run at 2 waves/SIMD: two workgroups per CU
            const int wg = c->wg_per_cu > 0 ? c->wg_per_cu : def_wg;
            const int per_cu = N >= 16 ? (wg < 2 ? wg : 2) : wg;
            int slots = c->slots_opt > 0 ? c->slots_opt : c->cu_count * per_cu;
            // keep the workspace under ~8 GiB for the largest extension sizes
            const size_t per = table_doubles(N) * (size_t)vbytes;
            const size_t budget = (size_t)8 << 30;
            if ((size_t)slots * per > budget) slots = (int)(budget / per);
            if (slots < 1) slots = 1;
            grid = nblocks < slots ? nblocks : slots;
            a.slot_doubles = table_doubles(N);
            rc = ensure(&c->d_slots, &c->slots_bytes, (size_t)grid * per);
            if (rc) return rc;
            a.slots = c->d_slots;
        }
    }
    c->last_grid = grid;
    c->last_variant = N >= 2 ? a.variant : 0;
    return hip_err(launch_heldkarp(a, grid));
}

thread_local std::unique_ptr<tspgpu_ctx, int (*)(tspgpu_ctx *)> t_default(nullptr, tspgpu_ctx_destroy);

template <typename V>
int solve_host_copy(tspgpu_ctx *c, const V *dist, int n, int nblocks, V *cost_out, int32_t *tour_out);

}  // namespace

extern "C" {

int tspgpu_version(void) { return TSPGPU_VERSION; }

const char *tspgpu_strerror(int code)
{
    switch (code) {
    case 0: return "success";
    case -EINVAL: return "invalid argument";
    case -ERANGE: return "tour costs reach INT_MAX (reference behaviour undefined)";
    case -ENODEV: return "no usable HIP device";
    case -ENOMEM: return "device allocation failed";
    case -EIO: return "HIP runtime or kernel launch failure";
    case -EDEADLK: return "the reference's mergeBlocks would never terminate for these paths";
    case -EOVERFLOW: return "too many tied optimal tours to enumerate above K1-wide's 31 cities";
    case -ENOSPC: return "output buffer too small";
    case -ETIMEDOUT: return "search watchdog expired (TSPGPU_SEARCH_WALL_S)";
    default: return "unknown error";
    }
}

int tspgpu_tour_length(int n) { return n == 2 ? 2 : n + 1; }

double tspgpu_relaxations_per_block(int n)
{
    const double N = n - 1;
    return N * (N - 1) * std::ldexp(1.0, n - 3);
}

double tspgpu_table_bytes_per_block(int n)
{
    const int N = n - 1;
    return 2.0 * 8.0 * N * std::ldexp(1.0, N - 1);
}

int tspgpu_distance_matrix(const tspgpu_city *cities, int n, int nblocks, double *dist)
{
    // assignment2.h:196: sqrt(pow(dx, 2) + pow(dy, 2)), glibc pow really called
    // (a volatile pointer keeps the compiler from folding pow(x,2) to x*x).
    static double (*volatile pow_fn)(double, double) = ::pow;
    static double (*volatile sqrt_fn)(double) = ::sqrt;
    if (n < 1 || nblocks < 0 || (nblocks > 0 && (!cities || !dist))) return -EINVAL;
    auto run = [&](int b0, int b1) {
        for (int b = b0; b < b1; ++b) {
            const tspgpu_city *c = cities + (size_t)b * n;
            double *d = dist + (size_t)b * n * n;
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < n; ++j) {
                    const double dx = pow_fn(c[i].x - c[j].x, 2);
                    const double dy = pow_fn(c[i].y - c[j].y, 2);
                    d[i * n + j] = sqrt_fn(dx + dy);
                }
        }
    };
    // large batches (a whole rank's blocks) on up to 16 host threads
    const long long work = (long long)nblocks * n * n;
    int nt = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (work < (1 << 18)) nt = 1;
    if (nt > nblocks) nt = nblocks > 0 ? nblocks : 1;
    if (nt <= 1) {
        run(0, nblocks);
        return 0;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back(run, (int)((long long)nblocks * t / nt), (int)((long long)nblocks * (t + 1) / nt));
    for (auto &x : th) x.join();
    return 0;
}

int tspgpu_validate(const double *dist, int n, int nblocks, int strict)
{
    int rc = check_n(n, strict);
    if (rc) return rc;
    if (nblocks < 0 || (nblocks > 0 && !dist)) return -EINVAL;
    for (int b = 0; b < nblocks; ++b) {
        const double *d = dist + (size_t)b * n * n;
        double mx = 0.0;
        for (int i = 0; i < n * n; ++i) {
            const double v = d[i];
            if (!(v >= 0.0) || !std::isfinite(v)) return -EINVAL;
            if (v > mx) mx = v;
        }
        // Every partial tour has at most n edges: below INT_MAX the reference's
        // sentinel (tsp.cpp:411,453) never wins a comparison.
        if ((double)n * mx >= (double)INT_MAX) return -ERANGE;
    }
    return 0;
}

int tspgpu_ctx_create(const tspgpu_opts *opts, tspgpu_ctx **out)
{
    if (!out) return -EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
    auto *c = new (std::nothrow) tspgpu_ctx();
    if (!c) return -ENOMEM;
    int dev = opts ? opts->device : -1;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    if (dev >= ndev) {
        delete c;
        return -ENODEV;
    }
    c->device = dev;
    c->strict = opts ? opts->strict : 0;
    c->slots_opt = opts ? opts->slots : 0;
    if (hipSetDevice(dev) != hipSuccess) {
        delete c;
        return -ENODEV;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) {
        if (prop.multiProcessorCount > 0) c->cu_count = prop.multiProcessorCount;
        char nm[128] = {0};
        if (hipDeviceGetName(nm, sizeof nm, dev) != hipSuccess || !nm[0]) std::snprintf(nm, sizeof nm, "%s", prop.name);
        std::snprintf(c->name, sizeof c->name, "%s (%s, %d CUs)", nm[0] ? nm : "AMD GPU", prop.gcnArchName,
                      prop.multiProcessorCount);
    }
    // tuning knobs for experiments and tests (tuning.h; the defaults are the measured best)
    double kv = 0.0;
    if (tspgpu::tuned("THREADS", &kv)) c->threads = (int)kv;
    if (tspgpu::tuned("LDS_TABLE_MAX_N", &kv)) c->lds_table_max_n = (int)kv < kLdsTableMaxN ? (int)kv : kLdsTableMaxN;
    if (tspgpu::tuned("K1", &kv)) {
        const int v = (int)kv;
        c->variant = v < 0 ? 1 : (v >= 6 ? 6 : (v >= 4 ? v : (v > 2 ? 2 : v)));
    }
    if (tspgpu::tuned("TILED_CFG", &kv)) c->tiled_cfg = (int)kv;
    if (tspgpu::tuned("WG_PER_CU", &kv)) c->wg_per_cu = kv > 0 ? (int)kv : 0;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return -EIO;
    }
    *out = c;
    return 0;
}

int tspgpu_ctx_destroy(tspgpu_ctx *c)
{
    if (!c) return 0;
    {
        // searches still alive keep the context: the last one's destroy
        // releases it (ctx.h "Lifetime")
        std::lock_guard<std::mutex> g(c->mu);
        c->closing = true;
        if (c->live_searches > 0) return 0;
    }
    tspgpu_ctx_release(c);
    return 0;
}

}  // extern "C"

void tspgpu_ctx_release(tspgpu_ctx *c)
{
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int i = 0; i <= kMaxN; ++i) {
        if (c->d_masks[i]) (void)hipFree(c->d_masks[i]);
        if (c->d_info[i]) (void)hipFree(c->d_info[i]);
    }
    if (c->wide_free) c->wide_free(c->wide_cache);
    // (null while a search holds the pool: round 4's segfault was
    // pool_free(nullptr) when the context went first)
    if (c->search_pool_free && c->search_pool) c->search_pool_free(c->search_pool);
    if (c->d_slots) (void)hipFree(c->d_slots);
    for (void *p : c->d_tinfo)
        if (p) (void)hipFree(p);
    for (void *p : c->d_subrows)
        if (p) (void)hipFree(p);
    if (c->d_tslots) (void)hipFree(c->d_tslots);
    if (c->d_dist) (void)hipFree(c->d_dist);
    if (c->d_cost) (void)hipFree(c->d_cost);
    if (c->d_tour) (void)hipFree(c->d_tour);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
    if (c->ev_k1_done) (void)hipEventDestroy(c->ev_k1_done);
    for (auto ev : c->ev_split) (void)hipEventDestroy(ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" {

int tspgpu_solve_blocks_device(tspgpu_ctx *c, const double *d_dist, int n, int nblocks, double *d_cost,
                               int32_t *d_tour, void *hip_stream)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return solve_device_locked(c, d_dist, n, nblocks, d_cost, d_tour, (hipStream_t)hip_stream, 8);
}

int tspgpu_solve_blocks_i32_device(tspgpu_ctx *c, const int32_t *d_dist, int n, int nblocks, int32_t *d_cost,
                                   int32_t *d_tour, void *hip_stream)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return solve_device_locked(c, d_dist, n, nblocks, d_cost, d_tour, (hipStream_t)hip_stream, 4);
}

int tspgpu_solve_blocks(tspgpu_ctx *c, const double *dist, int n, int nblocks, double *cost_out,
                        int32_t *tour_out)
{
    if (!c) return -EINVAL;
    int rc = tspgpu_validate(dist, n, nblocks, c->strict);
    if (rc) return rc;
    return solve_host_copy(c, dist, n, nblocks, cost_out, tour_out);
}

int tspgpu_solve_blocks_i32(tspgpu_ctx *c, const int32_t *dist, int n, int nblocks, int32_t *cost_out,
                            int32_t *tour_out)
{
    if (!c) return -EINVAL;
    int rc = tspgpu_validate_i32(dist, n, nblocks, c->strict);
    if (rc) return rc;
    return solve_host_copy(c, dist, n, nblocks, cost_out, tour_out);
}

int tspgpu_validate_i32(const int32_t *dist, int n, int nblocks, int strict)
{
    int rc = check_n(n, strict);
    if (rc) return rc;
    if (nblocks < 0 || (nblocks > 0 && !dist)) return -EINVAL;
    for (int b = 0; b < nblocks; ++b) {
        const int32_t *d = dist + (size_t)b * n * n;
        int64_t mx = 0;
        for (int i = 0; i < n * n; ++i) {
            if (d[i] < 0) return -EINVAL;
            if (d[i] > mx) mx = d[i];
        }
        // n edges per tour stay below INT_MAX: no i32 overflow, and the same
        // sentinel argument as tspgpu_validate
        if ((int64_t)n * mx >= (int64_t)INT_MAX) return -ERANGE;
    }
    return 0;
}

}  // extern "C"

namespace {

template <typename V>
int solve_host_copy(tspgpu_ctx *c, const V *dist, int n, int nblocks, V *cost_out, int32_t *tour_out)
{
    int rc = 0;
    if (nblocks > 0 && (!cost_out || !tour_out)) return -EINVAL;
    if (nblocks == 0) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    const size_t db = (size_t)nblocks * n * n * sizeof(V);
    const size_t cb = (size_t)nblocks * sizeof(V);
    const size_t tb = (size_t)nblocks * (n + 1) * sizeof(int32_t);
    if ((rc = ensure(&c->d_dist, &c->dist_bytes, db))) return rc;
    if ((rc = ensure(&c->d_cost, &c->cost_bytes, cb))) return rc;
    if ((rc = ensure(&c->d_tour, &c->tour_bytes, tb))) return rc;
    hipError_t e = xcopy_async(c->d_dist, dist, db, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = xset_async(c->d_tour, 0xff, tb, c->stream);
    if (e != hipSuccess) return hip_err(e);
    rc = solve_device_locked(c, c->d_dist, n, nblocks, c->d_cost, c->d_tour, c->stream, (int)sizeof(V));
    if (rc) return rc;
    e = xcopy_async(cost_out, c->d_cost, cb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = xcopy_async(tour_out, c->d_tour, tb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(e);
    for (int b = 0; b < nblocks; ++b)
        if (cost_out[b] < V(0)) return -EIO;  // backtracking found no predecessor
    return 0;
}

}  // namespace

extern "C" {

int tspgpu_solve_cities(tspgpu_ctx *c, const tspgpu_city *cities, int n, int nblocks, double *cost_out,
                        int32_t *tour_out)
{
    if (n < 2 || nblocks < 0) return -EINVAL;
    std::vector<double> dist((size_t)nblocks * n * n);
    int rc = tspgpu_distance_matrix(cities, n, nblocks, dist.data());
    if (rc) return rc;
    return tspgpu_solve_blocks(c, dist.data(), n, nblocks, cost_out, tour_out);
}

int tspgpu_solve(const double *dist, int n, int nblocks, double *cost_out, int32_t *tour_out,
                 const tspgpu_opts *opts)
{
    if (!t_default) {
        tspgpu_ctx *c = nullptr;
        int rc = tspgpu_ctx_create(opts, &c);
        if (rc) return rc;
        t_default.reset(c);
    }
    t_default->strict = opts ? opts->strict : 0;
    return tspgpu_solve_blocks(t_default.get(), dist, n, nblocks, cost_out, tour_out);
}

int tspgpu_last_grid(const tspgpu_ctx *c) { return c ? c->last_grid : 0; }

int tspgpu_last_variant(const tspgpu_ctx *c) { return c ? c->last_variant : -1; }

int tspgpu_k1_split_timing(tspgpu_ctx *c, int enable)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->split_timing = enable ? 1 : 0;
    c->split_used = 0;
    c->split_overflow = false;
    return 0;
}

int tspgpu_k1_last_split_ms(tspgpu_ctx *c, float *forward_ms, float *backtrack_ms)
{
    if (!c || !forward_ms || !backtrack_ms) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->split_overflow) return -ENOSPC;
    if (!c->split_used) return -ENOENT;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipError_t e = hipEventSynchronize(c->ev_split[c->split_used - 1]);
    double fw = 0.0, bt = 0.0;
    for (size_t i = 0; e == hipSuccess && i < c->split_used; i += 3) {
        float f = 0.f, b = 0.f;
        e = hipEventElapsedTime(&f, c->ev_split[i], c->ev_split[i + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&b, c->ev_split[i + 1], c->ev_split[i + 2]);
        fw += f;
        bt += b;
    }
    c->split_used = 0;
    *forward_ms = (float)fw;
    *backtrack_ms = (float)bt;
    return hip_err(e);
}

int tspgpu_device_count(void)
{
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int tspgpu_device_alloc(tspgpu_ctx *c, size_t bytes, void **ptr)
{
    if (!c || !ptr) return -EINVAL;
    *ptr = nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    return hip_err(hipMalloc(ptr, bytes ? bytes : 1));
}

int tspgpu_device_free(tspgpu_ctx *c, void *ptr)
{
    if (!c) return -EINVAL;
    if (!ptr) return 0;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    return hip_err(hipFree(ptr));
}

static int copy_sync(tspgpu_ctx *c, void *dst, const void *src, size_t bytes, hipMemcpyKind kind)
{
    if (!c || (bytes && (!dst || !src))) return -EINVAL;
    if (!bytes) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipError_t e = xcopy_async(dst, src, bytes, kind, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_err(e);
}

int tspgpu_memcpy_htod(tspgpu_ctx *c, void *dst, const void *src, size_t bytes)
{
    return copy_sync(c, dst, src, bytes, hipMemcpyHostToDevice);
}

int tspgpu_memcpy_dtoh(tspgpu_ctx *c, void *dst, const void *src, size_t bytes)
{
    return copy_sync(c, dst, src, bytes, hipMemcpyDeviceToHost);
}

void *tspgpu_stream(tspgpu_ctx *c) { return c ? (void *)c->stream : nullptr; }

int tspgpu_stream_create(tspgpu_ctx *c, void **stream)
{
    if (!c || !stream) return -EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    *stream = e == hipSuccess ? (void *)s : nullptr;
    return hip_err(e);
}

int tspgpu_stream_destroy(tspgpu_ctx *c, void *stream)
{
    if (!c) return -EINVAL;
    if (!stream) return 0;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->k1_last_stream == (hipStream_t)stream) {
        // the next launch must not wait on an event of a destroyed stream's queue:
        // drain it and forget it
        (void)hipStreamSynchronize((hipStream_t)stream);
        c->k1_launched = false;
        c->k1_last_stream = nullptr;
    }
    return hip_err(hipStreamDestroy((hipStream_t)stream));
}

int tspgpu_stream_synchronize(tspgpu_ctx *c, void *stream)
{
    if (!c) return -EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    return hip_err(hipStreamSynchronize((hipStream_t)stream));
}

int tspgpu_synchronize(tspgpu_ctx *c)
{
    if (!c) return -EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    return hip_err(hipStreamSynchronize(c->stream));
}

int tspgpu_timer_start(tspgpu_ctx *c)
{
    if (!c) return -EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipError_t e = hipSuccess;
    if (!c->ev_start) e = hipEventCreate(&c->ev_start);
    if (e == hipSuccess && !c->ev_stop) e = hipEventCreate(&c->ev_stop);
    if (e == hipSuccess) e = hipEventRecord(c->ev_start, c->stream);
    return hip_err(e);
}

int tspgpu_timer_stop(tspgpu_ctx *c, float *ms)
{
    if (!c || !ms || !c->ev_start) return -EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipError_t e = hipEventRecord(c->ev_stop, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(c->ev_stop);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, c->ev_start, c->ev_stop);
    return hip_err(e);
}

int tspgpu_device_info(const tspgpu_ctx *c, int *cu_count, char *name, int namecap)
{
    if (!c) return -EINVAL;
    if (cu_count) *cu_count = c->cu_count;
    if (name && namecap > 0) std::snprintf(name, (size_t)namecap, "%s", c->name);
    return 0;
}

}  // extern "C"
