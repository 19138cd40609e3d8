// K1-wide — ONE instance's Held-Karp over the whole GPU (all CUs cooperate
// on every layer), for the single-instance time to the optimal tour and for
// instances past K1's per-workgroup sizes (n <= 31: the table of
// N*2^(N-1) doubles is 129 GB at n = 31 and fits one MI355X's 288 GB).
//
// Same recurrence and the same IEEE operations as K1 / tsp.cpp:405-509, so the
// same bits: layer s is computed from layer s-1 by one launch with a thread
// per DESTINATION state (S, k) in the position-major layout of K1
// (heldkarp_impl.h): element e = p*C(N,s) + colexrank(S), p = position of k
// in S, so the writes of a wave are one contiguous 512-B segment.  The thread
// unranks S from colexrank(S) (binomials in LDS, no 2^N mask table), drops
// k, and takes the first-strict-min-free min over the members m of T = S\k of
// G[T][m] + d[m][k] (the min itself is order independent; the tie-break
// happens in the backtracking, which picks the smallest m whose candidate
// equals the state value, as K1 does).  A one-wave kernel closes the tour
// (tsp.cpp:483-499) and backtracks.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "ctx.h"
#include "xfer.h"
#include "wave.h"
#include "tspgpu.h"
#include "tuning.h"

using tspgpu::xcopy_async;

namespace {

constexpr int kWideMaxN = 30;  // inner cities (n <= 31: a 129 GB table)
constexpr int kWideThreads = 256;
constexpr double kIntMaxD = 2147483647.0;

struct WideInfo {
    long long binom[kWideMaxN + 2][kWideMaxN + 2];  // C(a, b)
    unsigned long long off[kWideMaxN + 2];          // doubles before layer t
    unsigned long long cnt[kWideMaxN + 2];          // C(N, t)
};

__device__ __forceinline__ long long bn(const long long (*b)[kWideMaxN + 2], int a, int k)
{
    return (k < 0 || k > a) ? 0 : b[a][k];
}

// layer 1: G[{i}][i] = d[0][i+1]
__global__ void wide_layer1(const double *__restrict__ d, int n, double *__restrict__ tab)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n - 1) tab[i] = d[i + 1];
}

__global__ __launch_bounds__(kWideThreads) void wide_layer(const double *__restrict__ dist, int N,
                                                           const WideInfo *__restrict__ info, int s,
                                                           double *__restrict__ tab)
{
    __shared__ long long B[kWideMaxN + 2][kWideMaxN + 2];
    __shared__ double dl[(kWideMaxN + 1) * (kWideMaxN + 1)];
    const int n = N + 1;
    for (int i = threadIdx.x; i < (kWideMaxN + 2) * (kWideMaxN + 2); i += kWideThreads)
        (&B[0][0])[i] = (&info->binom[0][0])[i];
    for (int i = threadIdx.x; i < n * n; i += kWideThreads) dl[i] = dist[i];
    __syncthreads();
    const int t = s - 1;
    const unsigned long long cs = info->cnt[s], ct = info->cnt[t];
    const unsigned long long os = info->off[s], ot = info->off[t];
    const unsigned long long total = cs * (unsigned long long)s;
    for (unsigned long long e = blockIdx.x * (unsigned long long)kWideThreads + threadIdx.x; e < total;
         e += (unsigned long long)gridDim.x * kWideThreads) {
        const int p = (int)(e / cs);
        long long r = (long long)(e - (unsigned long long)p * cs);
        // colex unrank: members e_1 < ... < e_s with r = sum C(e_i, i)
        uint32_t S = 0;
        int c = N - 1;
        for (int i = s; i >= 1; --i) {
            while (bn(B, c, i) > r) --c;
            r -= bn(B, c, i);
            S |= 1u << c;
            --c;
        }
        // k = p-th member (ascending); T = S \ k and its colex rank
        uint32_t x = S;
        for (int q = 0; q < p; ++q) x &= x - 1u;
        const int k = __builtin_ctz(x);
        const uint32_t T = S & ~(1u << k);
        long long rT = 0;
        {
            uint32_t y = T;
            int i = 1;
            while (y) {
                const int b = __builtin_ctz(y);
                rT += bn(B, b, i++);
                y &= y - 1u;
            }
        }
        double acc = kIntMaxD;  // tsp.cpp:453 (candidates are < INT_MAX by validation)
        uint32_t y = T;
        int j = 0;
        while (y) {
            const int m = __builtin_ctz(y);
            y &= y - 1u;
            const double g = tab[ot + (unsigned long long)j * ct + (unsigned long long)rT];
            acc = fmin(acc, g + dl[(m + 1) * n + (k + 1)]);
            ++j;
        }
        tab[os + e] = acc;
    }
}

// Row-owner ("push") form of a layer, t -> t+1 (default): a thread owns a
// SOURCE row T of layer t (its t values are coalesced loads: consecutive
// threads hold consecutive colex ranks) and writes every destination
// G[T+k][k] = min_{m in T} G[T][m] + d[m][k] for the N - t cities k not in T —
// the whole min of a destination comes from that one row, so every table
// entry is read once and written once (the pull form above reads each entry
// N - t times through scattered loads).  The destination rank follows from
// prefix sums over T's members: colexrank(T+k) = sum_{m<k} C(m, i_m) +
// C(k, c+1) + sum_{m>k} C(m, i_m + 1), c = #members below k = the position of
// k in T+k.  Consecutive rows differ in their low members, so the writes of
// one k are mostly contiguous runs.  Templated on t: the row lives in VGPRs.
template <int T>
__global__ __launch_bounds__(kWideThreads) void wide_push(const double *__restrict__ dist, int N,
                                                          const WideInfo *__restrict__ info,
                                                          double *__restrict__ tab)
{
    __shared__ int B[kWideMaxN + 2][kWideMaxN + 3];  // C(a, b), b <= 31 (ranks < 2^31 for N <= 30)
    __shared__ double dl[(kWideMaxN + 1) * (kWideMaxN + 1)];
    const int n = N + 1;
    for (int i = threadIdx.x; i < (kWideMaxN + 2) * (kWideMaxN + 3); i += kWideThreads) {
        const int a = i / (kWideMaxN + 3), b = i % (kWideMaxN + 3);
        (&B[0][0])[i] = b <= kWideMaxN + 1 ? (int)info->binom[a][b] : 0;
    }
    for (int i = threadIdx.x; i < n * n; i += kWideThreads) dl[i] = dist[i];
    __syncthreads();
    const unsigned long long ct = info->cnt[T], cs = info->cnt[T + 1];
    const unsigned long long ot = info->off[T], os = info->off[T + 1];
    for (unsigned long long r0 = blockIdx.x * (unsigned long long)kWideThreads + threadIdx.x; r0 < ct;
         r0 += (unsigned long long)gridDim.x * kWideThreads) {
        // colex unrank of T: members m_1 < ... < m_T with r0 = sum C(m_i, i)
        int m[T];
        long long r = (long long)r0;
        int c = N - 1;
#pragma unroll
        for (int i = T; i >= 1; --i) {
            while (B[c][i] > r) --c;
            r -= B[c][i];
            m[i - 1] = c;
            --c;
        }
        double g[T];
#pragma unroll
        for (int j = 0; j < T; ++j) g[j] = tab[ot + (unsigned long long)j * ct + r0];
        uint32_t mask = 0;
        long long hi = 0;  // sum_j C(m_j, j+2): every member above k
#pragma unroll
        for (int j = 0; j < T; ++j) {
            mask |= 1u << m[j];
            hi += B[m[j]][j + 2];
        }
        long long lo = 0;  // sum over members below k of C(m_j, j+1) - C(m_j, j+2)
        int cb = 0;        // members below k
        for (int k = 0; k < N; ++k) {
            if ((mask >> k) & 1u) {
                lo += (long long)B[k][cb + 1] - (long long)B[k][cb + 2];
                ++cb;
                continue;
            }
            double acc = kIntMaxD;  // tsp.cpp:453 (candidates are < INT_MAX by validation)
#pragma unroll
            for (int j = 0; j < T; ++j) acc = fmin(acc, g[j] + dl[(m[j] + 1) * n + (k + 1)]);
            const long long rs = hi + lo + B[k][cb + 1];
            tab[os + (unsigned long long)cb * cs + (unsigned long long)rs] = acc;
        }
    }
}

// closing min + backtracking (one wave): lane m-1 holds candidate m
__global__ void wide_close(const double *__restrict__ dist, int N, const WideInfo *__restrict__ info,
                           const double *__restrict__ tab, double *__restrict__ cost_out, int32_t *__restrict__ tour)
{
    const int n = N + 1;
    const int lane = threadIdx.x;
    const int m = lane + 1;
    const bool valid = m <= N;
    auto rank_of = [&](uint32_t M) {
        long long r = 0;
        int i = 1;
        while (M) {
            r += info->binom[__builtin_ctz(M)][i++];
            M &= M - 1u;
        }
        return r;
    };
    const double glast = valid ? tab[info->off[N] + (unsigned long long)(m - 1) * info->cnt[N]] : 0.0;
    const double cand = valid ? glast + dist[m * n] : 1.0e300;
    double best = cand;
    best = tspgpu::wave_min_dpp(best);
    best = fmin(best, kIntMaxD);
    const unsigned long long hit = __ballot(valid && cand == best && cand < kIntMaxD);
    const int bestM = hit ? __ffsll(hit) : 0;
    bool ok = bestM != 0;
    uint32_t S = (uint32_t)((1ull << N) - 1ull);
    int k = bestM;
    int pos = n - 2;
    double target = __shfl(glast, ok ? bestM - 1 : 0);
    while (ok && __builtin_popcount(S) >= 2) {
        const uint32_t T = S & ~(1u << (k - 1));
        const int tt = __builtin_popcount(T);
        const long long rT = rank_of(T);
        const bool inT = valid && ((T >> (m - 1)) & 1u);
        double gv = 0.0, c = 0.0;
        if (inT) {
            const int j = __builtin_popcount(T & ((1u << (m - 1)) - 1u));
            gv = tab[info->off[tt] + (unsigned long long)j * info->cnt[tt] + (unsigned long long)rT];
            c = gv + dist[m * n + k];
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
        *cost_out = ok ? best : -1.0;
    }
}

int herr(hipError_t e)
{
    if (e == hipSuccess) return 0;
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    return -EIO;
}

// Device buffers of one table size, kept in the context between calls.
// (A hipGraph capture of the N launches was measured: same device time,
// the ~8 us per layer at small n is the kernel boundary itself.)
struct WideState {
    int N = 0;
    double *tab = nullptr, *dist = nullptr, *cost = nullptr;
    int32_t *tour = nullptr;
    WideInfo *info = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
};

void wide_state_free(void *p)
{
    WideState *w = static_cast<WideState *>(p);
    if (!w) return;
    if (w->e0) (void)hipEventDestroy(w->e0);
    if (w->e1) (void)hipEventDestroy(w->e1);
    for (void *q : {(void *)w->tab, (void *)w->dist, (void *)w->cost, (void *)w->tour, (void *)w->info})
        if (q) (void)hipFree(q);
    delete w;
}

void launch_push(int t, int grid, hipStream_t st, const double *dist, int N, const WideInfo *info, double *tab)
{
    switch (t) {
#define TSPGPU_PUSH(TT) \
    case TT: hipLaunchKernelGGL(wide_push<TT>, dim3(grid), dim3(kWideThreads), 0, st, dist, N, info, tab); break;
    TSPGPU_PUSH(1) TSPGPU_PUSH(2) TSPGPU_PUSH(3) TSPGPU_PUSH(4) TSPGPU_PUSH(5) TSPGPU_PUSH(6) TSPGPU_PUSH(7)
    TSPGPU_PUSH(8) TSPGPU_PUSH(9) TSPGPU_PUSH(10) TSPGPU_PUSH(11) TSPGPU_PUSH(12) TSPGPU_PUSH(13) TSPGPU_PUSH(14)
    TSPGPU_PUSH(15) TSPGPU_PUSH(16) TSPGPU_PUSH(17) TSPGPU_PUSH(18) TSPGPU_PUSH(19) TSPGPU_PUSH(20) TSPGPU_PUSH(21)
    TSPGPU_PUSH(22) TSPGPU_PUSH(23) TSPGPU_PUSH(24) TSPGPU_PUSH(25) TSPGPU_PUSH(26) TSPGPU_PUSH(27) TSPGPU_PUSH(28)
    TSPGPU_PUSH(29)
#undef TSPGPU_PUSH
    default: break;
    }
}

// layer 1, layers 2..N, closing + backtracking
void enqueue_wide(const WideState *w, const WideInfo &h, int n, int cus, hipStream_t st)
{
    const int N = n - 1;
    hipLaunchKernelGGL(wide_layer1, dim3(1), dim3(64), 0, st, w->dist, n, w->tab);
    // per-destination (pull) form up to 17 cities, where both are bound by the
    // ~8 us kernel boundary per layer and pull is a little faster; the knob
    // WIDE_PULL = 0 / 1 forces either (measured: profiles/r01/k1wide_push_vs_pull.log)
    const bool pull = tspgpu::tuned_or("WIDE_PULL", n <= 17 ? 1 : 0) != 0;
    if (!pull) {
        for (int t = 1; t < N; ++t) {
            const unsigned long long blocks = (h.cnt[t] + kWideThreads - 1) / kWideThreads;
            const unsigned long long cap = (unsigned long long)cus * 16;
            const int grid = (int)(blocks < cap ? blocks : cap);
            launch_push(t, grid, st, w->dist, N, w->info, w->tab);
        }
        hipLaunchKernelGGL(wide_close, dim3(1), dim3(64), 0, st, w->dist, N, w->info, w->tab, w->cost, w->tour);
        return;
    }
    for (int s = 2; s <= N; ++s) {
        const unsigned long long total = h.cnt[s] * (unsigned long long)s;
        const unsigned long long blocks = (total + kWideThreads - 1) / kWideThreads;
        const unsigned long long cap = (unsigned long long)cus * 16;
        const int grid = (int)(blocks < cap ? blocks : cap);
        hipLaunchKernelGGL(wide_layer, dim3(grid), dim3(kWideThreads), 0, st, w->dist, N, w->info, s, w->tab);
    }
    hipLaunchKernelGGL(wide_close, dim3(1), dim3(64), 0, st, w->dist, N, w->info, w->tab, w->cost, w->tour);
}

}  // namespace

extern "C" {

int tspgpu_solve_instance(tspgpu_ctx *c, const double *dist, int n, double *cost_out, int32_t *tour_out,
                          double *kernel_ms)
{
    if (!c || !dist || !cost_out || !tour_out) return -EINVAL;
    if (n < 3 || n > kWideMaxN + 1) return -EINVAL;
    int rc = tspgpu_validate(dist, n, 1, 0 /* n <= 20 checked below */);
    if (rc == -EINVAL && n > TSPGPU_MAX_CITIES) {
        // tspgpu_validate caps n at 20: check the values here
        double mx = 0.0;
        for (int i = 0; i < n * n; ++i) {
            if (!(dist[i] >= 0.0) || !(dist[i] < INFINITY)) return -EINVAL;
            mx = dist[i] > mx ? dist[i] : mx;
        }
        rc = (double)n * mx >= (double)INT_MAX ? -ERANGE : 0;
    }
    if (rc) return rc;
    const int N = n - 1;
    WideInfo h;
    std::memset(&h, 0, sizeof h);
    for (int a = 0; a <= kWideMaxN + 1; ++a) {
        h.binom[a][0] = 1;
        for (int b = 1; b <= a; ++b) h.binom[a][b] = h.binom[a - 1][b - 1] + (b <= a - 1 ? h.binom[a - 1][b] : 0);
    }
    unsigned long long off = 0;
    for (int t = 1; t <= N; ++t) {
        h.cnt[t] = (unsigned long long)h.binom[N][t];
        h.off[t] = off;
        off += h.cnt[t] * (unsigned long long)t;
    }
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    hipStream_t st = c->stream;
    WideState *w = static_cast<WideState *>(c->wide_cache);
    if (!w || w->N != N) {
        if (w) wide_state_free(w);
        c->wide_cache = nullptr;
        c->wide_free = nullptr;
        size_t freeb = 0, totalb = 0;
        if (hipMemGetInfo(&freeb, &totalb) == hipSuccess && off * 8 + (64u << 20) > freeb) return -ENOMEM;
        w = new (std::nothrow) WideState();
        if (!w) return -ENOMEM;
        w->N = N;
        hipError_t e = hipMalloc((void **)&w->tab, off * 8);
        if (e == hipSuccess) e = hipMalloc((void **)&w->dist, sizeof(double) * n * n);
        if (e == hipSuccess) e = hipMalloc((void **)&w->info, sizeof(WideInfo));
        if (e == hipSuccess) e = hipMalloc((void **)&w->cost, sizeof(double));
        if (e == hipSuccess) e = hipMalloc((void **)&w->tour, sizeof(int32_t) * (n + 1));
        if (e == hipSuccess) e = xcopy_async(w->info, &h, sizeof h, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventCreate(&w->e0);
        if (e == hipSuccess) e = hipEventCreate(&w->e1);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            wide_state_free(w);
            return herr(e);
        }
        // keep small tables for the next call; free >1 GB ones after use
        if (off * 8 <= ((size_t)1 << 30)) {
            c->wide_cache = w;
            c->wide_free = wide_state_free;
        }
    }
    hipError_t e = xcopy_async(w->dist, dist, sizeof(double) * n * n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        (void)hipEventRecord(w->e0, st);
        enqueue_wide(w, h, n, c->cu_count, st);
        (void)hipEventRecord(w->e1, st);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e == hipSuccess) e = xcopy_async(cost_out, w->cost, sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = xcopy_async(tour_out, w->tour, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess && kernel_ms) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, w->e0, w->e1) == hipSuccess) *kernel_ms = ms;
    }
    if (c->wide_cache != w) wide_state_free(w);
    if (e != hipSuccess) return herr(e);
    return *cost_out < 0 ? -EIO : 0;
}

}  // extern "C"
