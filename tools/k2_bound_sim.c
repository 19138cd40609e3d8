/* CPU experiment for K2's bound (development aid, no product code): DFS node
 * counts of the prefix search on one instance under different lower bounds,
 * with the incumbent at the optimum (what the GPU search has after its first
 * rounds: the 2-opt start is usually optimal or within a few percent).
 *   k2_bound_sim K < matrix.txt     (n, then n*n doubles)
 * Bounds (remaining path k -> rem -> 0, c = fold cost so far):
 *   B0  sum over rem + {0} of the cheapest edge into x        (search.hip today)
 *   B1  half the sum of the two cheapest incident edges of every rem city,
 *       + the cheapest of k and of 0 (symmetric distances)
 *   H   |rem| <= K: exact suffix table H[U][x] (path from x over U to 0), the
 *       child j of k bounded by c + d[k][j] + H[rem][j]
 * A node = one child evaluated (search.hip's node count). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int n, N, K, mode;
static double d[32][32], a[32], m1[32], m2[32], opt, thr;
static double *H; /* [1<<N][N], inner cities 1..N as bits 0..N-1 */
static unsigned long long nodes;

static double hk(void)
{
    size_t S = (size_t)1 << N;
    double *G = malloc(S * N * sizeof(double));
    for (size_t i = 0; i < S * N; ++i) G[i] = 1e300;
    for (int k = 0; k < N; ++k) G[((size_t)1 << k) * N + k] = d[0][k + 1];
    for (size_t s = 1; s < S; ++s)
        for (int k = 0; k < N; ++k) {
            if (!(s >> k & 1) || s == ((size_t)1 << k)) continue;
            size_t p = s & ~((size_t)1 << k);
            double best = 1e300;
            for (int m = 0; m < N; ++m)
                if (p >> m & 1) {
                    double c = G[p * N + m] + d[m + 1][k + 1];
                    if (c < best) best = c;
                }
            G[s * N + k] = best;
        }
    double best = 1e300;
    for (int k = 0; k < N; ++k) {
        double c = G[(S - 1) * N + k] + d[k + 1][0];
        if (c < best) best = c;
    }
    free(G);
    return best;
}

static void build_h(void)
{
    size_t S = (size_t)1 << N;
    H = malloc(S * N * sizeof(double));
    for (size_t i = 0; i < S * N; ++i) H[i] = 1e300;
    for (size_t s = 1; s < S; ++s) {
        int pc = __builtin_popcountll(s);
        if (pc > K) continue;
        for (int x = 0; x < N; ++x) {
            if (!(s >> x & 1)) continue;
            if (pc == 1) {
                H[s * N + x] = d[x + 1][0];
                continue;
            }
            size_t r = s & ~((size_t)1 << x);
            double best = 1e300;
            for (int y = 0; y < N; ++y)
                if (r >> y & 1) {
                    double c = d[x + 1][y + 1] + H[r * N + y];
                    if (c < best) best = c;
                }
            H[s * N + x] = best;
        }
    }
}

static double rest_bound(int k, unsigned rem)
{
    double b = 0;
    if (mode == 0) {
        b = a[0];
        for (int x = 1; x < n; ++x)
            if (rem >> x & 1) b += a[x];
    } else {
        b = m1[k] + m1[0];
        for (int x = 1; x < n; ++x)
            if (rem >> x & 1) b += m1[x] + m2[x];
        b *= 0.5;
    }
    return b;
}

static void dfs(int k, unsigned rem, double c, int left)
{
    for (int j = 1; j < n; ++j) {
        if (!(rem >> j & 1)) continue;
        ++nodes;
        double cj = c + d[k][j];
        unsigned r2 = rem & ~(1u << j);
        if (left == 1) continue; /* tour closed: (cj + d[j][0]) checked against the incumbent */
        if (K > 0 && left <= K) {
            /* rem (as inner bits) includes j: the child's exact completion bound */
            unsigned ib = rem >> 1;
            if (cj + H[(size_t)ib * N + (j - 1)] > thr) continue;
        } else if (cj + rest_bound(j, r2) > thr)
            continue;
        dfs(j, r2, cj, left - 1);
    }
}

int main(int argc, char **argv)
{
    K = argc > 1 ? atoi(argv[1]) : 0;
    mode = argc > 2 ? atoi(argv[2]) : 0;
    if (scanf("%d", &n) != 1) return 1;
    N = n - 1;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (scanf("%lf", &d[i][j]) != 1) return 1;
    for (int x = 0; x < n; ++x) {
        a[x] = 1e300;
        m1[x] = m2[x] = 1e300;
        for (int y = 0; y < n; ++y) {
            if (y == x) continue;
            if (d[y][x] < a[x]) a[x] = d[y][x];
            double e = d[x][y];
            if (e < m1[x]) {
                m2[x] = m1[x];
                m1[x] = e;
            } else if (e < m2[x])
                m2[x] = e;
        }
    }
    opt = hk();
    thr = (argc > 3 ? atof(argv[3]) : opt) * (1.0 + 0x1p-39);
    if (K > 0) build_h();
    double hrel = 0;
    for (int s = 1; s <= K; ++s) {
        double c = 1;
        for (int i = 0; i < s; ++i) c = c * (N - i) / (i + 1);
        hrel += c * s * (s - 1);
    }
    dfs(0, ((1u << n) - 1) & ~1u, 0.0, N);
    printf("{\"n\": %d, \"K\": %d, \"bound\": \"%s\", \"opt\": %.6f, \"nodes\": %llu, \"table_relaxations\": %.0f}\n", n, K,
           mode ? "B1 two-edge" : "B0 cheapest-in", opt, nodes, hrel);
    return 0;
}
