// Host-only parts of K2 (search_host.h): bound tour, city weights, input
// check and the tie rule over the optimal set (tsp.cpp:457-470, 483-499).
#include "search_host.h"
#include "tuning.h"

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "tspgpu.h"

namespace tspgpu {
namespace host {

// Left fold of the closed tour 0 -> t1 -> ... -> tN -> 0 (tsp.cpp's cost).
template <typename V>
V fold_tour(const V *d, int n, const int32_t *t)
{
    V c = 0;
    int prev = 0;
    for (int i = 0; i < n - 1; ++i) {
        c = c + d[prev * n + t[i]];
        prev = t[i];
    }
    return c + d[prev * n];
}

// Local search on a closed tour (cyclic, real-valued sums): 2-opt and Or-opt
// (a segment of 1..3 cities moved elsewhere, either direction) until neither
// improves.
template <typename V>
void local_search(const V *d, int n, std::vector<int> &t)
{
    auto D = [&](int a, int b) { return (double)d[a * n + b]; };
    auto len_of = [&](const std::vector<int> &u) {
        double c = 0;
        for (int i = 0; i < n; ++i) c += D(u[i], u[(i + 1) % n]);
        return c;
    };
    // a move is kept only if the whole cyclic length drops by more than the
    // tolerance (asymmetric matrices: the local deltas assume symmetry), and
    // the number of moves is capped: the loop always ends
    double cur = len_of(t);
    auto better = [&](double c) { return c < cur - 1e-9 * (1.0 + std::fabs(cur)); };
    // (scratch buffers reused by every candidate: no allocation per move)
    std::vector<int> cand, seg;
    cand.reserve(n);
    seg.reserve(4);
    auto accept = [&](std::vector<int> &cd) {
        const double c = len_of(cd);
        if (better(c)) {
            t.swap(cd);
            cur = c;
            return true;
        }
        return false;
    };
    for (int moves = 0, improved = 1; improved && moves < 64 * n; ++moves) {
        improved = 0;
        for (int i = 1; i < n - 1 && !improved; ++i)
            for (int j = i + 1; j < n && !improved; ++j) {
                const int a = t[i - 1], b = t[i], c = t[j], e = t[(j + 1) % n];
                if ((D(a, c) + D(b, e)) - (D(a, b) + D(c, e)) < 0) {
                    // the 2-opt candidate in place, undone when it does not pay
                    std::reverse(t.begin() + i, t.begin() + j + 1);
                    const double cl = len_of(t);
                    if (better(cl)) {
                        cur = cl;
                        improved = 1;
                    } else {
                        std::reverse(t.begin() + i, t.begin() + j + 1);
                    }
                }
            }
        for (int len = 1; len <= 3 && !improved && n > len + 2; ++len)
            for (int i = 0; i < n && !improved; ++i) {
                // segment t[i..i+len-1] (cyclic), between p = t[i-1] and q = t[i+len]
                const int p = t[(i - 1 + n) % n], q = t[(i + len) % n];
                const int s0 = t[i], s1 = t[(i + len - 1) % n];
                const double gain = D(p, s0) + D(s1, q) - D(p, q);
                for (int k = 0; k < n && !improved; ++k) {
                    bool touch = false;  // edge (t[k], t[k+1]) must not touch the segment
                    for (int z = -1; z < len; ++z)
                        if ((i + z + n) % n == k) touch = true;
                    if (touch) continue;
                    const int u = t[k], v = t[(k + 1) % n];
                    const double fwd = D(u, s0) + D(s1, v) - D(u, v);
                    const double rev = D(u, s1) + D(s0, v) - D(u, v);
                    const bool r = rev < fwd;
                    if ((r ? rev : fwd) - gain >= 0) continue;
                    seg.clear();
                    cand.clear();
                    for (int z = 0; z < len; ++z) seg.push_back(t[(i + z) % n]);
                    if (r) std::reverse(seg.begin(), seg.end());
                    for (int z = 0; z < n - len; ++z) {
                        const int c = t[(i + len + z) % n];
                        cand.push_back(c);
                        if (c == u) cand.insert(cand.end(), seg.begin(), seg.end());
                    }
                    improved = accept(cand);
                }
            }
    }
}

// Lagrangian city weights for the two-edge bound (symmetric matrices): with
// d'[x][y] = d[x][y] + pi_x + pi_y, every path j -> R -> 0 has d'-cost =
// d-cost + pi_j + pi_0 + 2 sum_{x in R} pi_x, so the bound "interior cities
// pay half their two cheapest d' edges, the two ends half their cheapest"
// minus those pi terms is again a lower bound on the d-cost, for ANY pi.
// pi is chosen to maximise the whole-tour version, sum_x (two cheapest d'
// edges)/2 - 2 sum pi (the degree relaxation), by subgradient ascent: a city
// picked by more than two neighbours gets dearer (Polyak steps towards a
// nearest-neighbour tour's cost, 200 iterations, O(n^2) each).  On 30 random
// cities the root bound rises from 0.81 to 0.90 of the optimum, on ulysses22
// from 0.66 to 0.87 (tools/k2_lagrange_proto.py).
void lagrange_pi(const std::vector<double> &D, int n, std::vector<double> &best_pi)
{
    double ub = 0.0;  // nearest-neighbour tour from city 0: the step target
    {
        std::vector<char> used(n, 0);
        int k = 0;
        used[0] = 1;
        for (int i = 1; i < n; ++i) {
            int b = -1;
            for (int j = 0; j < n; ++j)
                if (!used[j] && (b < 0 || D[(size_t)k * n + j] < D[(size_t)k * n + b])) b = j;
            ub += D[(size_t)k * n + b];
            used[b] = 1;
            k = b;
        }
        ub += D[(size_t)k * n];
    }
    std::vector<double> pi(n, 0.0);
    std::vector<int> cnt(n);
    double best = -INFINITY, lam = 2.0;
    int stall = 0;
    best_pi.assign(n, 0.0);
    for (int it = 0; it < 200; ++it) {
        double lb = 0.0;
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int x = 0; x < n; ++x) {
            double m1 = INFINITY, m2 = INFINITY;
            int y1 = -1, y2 = -1;
            for (int y = 0; y < n; ++y) {
                if (y == x) continue;
                const double v = D[(size_t)x * n + y] + pi[x] + pi[y];
                if (v < m1) {
                    m2 = m1, y2 = y1;
                    m1 = v, y1 = y;
                } else if (v < m2) {
                    m2 = v, y2 = y;
                }
            }
            lb += (m1 + m2) * 0.5 - 2.0 * pi[x];
            ++cnt[y1];
            ++cnt[y2];
        }
        if (lb > best) {
            best = lb;
            best_pi = pi;
            stall = 0;
        } else if (++stall >= 10) {
            lam *= 0.7;
            stall = 0;
        }
        double nn = 0.0;
        for (int x = 0; x < n; ++x) nn += (cnt[x] * 0.5 - 1.0) * (cnt[x] * 0.5 - 1.0);
        if (nn == 0.0 || !(ub > lb)) break;
        const double t = lam * (ub - lb) / nn;
        for (int x = 0; x < n; ++x) pi[x] += t * (cnt[x] * 0.5 - 1.0);
    }
}

// Held-Karp city weights: subgradient ascent on the 1-tree bound (a minimum
// spanning tree of cities 1..n-1 plus the two cheapest edges at city 0, on
// d' = d + pi_x + pi_y, minus 2 sum pi), the same Polyak steps towards a
// nearest-neighbour tour's cost as lagrange_pi, 300 iterations of an O(n^2)
// Prim.  On the hardest 32-city seeds (bench.py's k2_instance 14, 30, 35) the
// bound reaches the optimum to 5 digits, where the two-edge bound stops at
// 0.83-0.88 (tools/k2_tree_bound_proto.py).  These weights serve the tree
// bound of the expand kernel (SearchArgs::mst); the bound is valid for any pi.
void held_karp_pi(const std::vector<double> &D, int n, std::vector<double> &best_pi)
{
    double ub = 0.0;
    {
        std::vector<char> used(n, 0);
        int k = 0;
        used[0] = 1;
        for (int i = 1; i < n; ++i) {
            int b = -1;
            for (int j = 0; j < n; ++j)
                if (!used[j] && (b < 0 || D[(size_t)k * n + j] < D[(size_t)k * n + b])) b = j;
            ub += D[(size_t)k * n + b];
            used[b] = 1;
            k = b;
        }
        ub += D[(size_t)k * n];
    }
    std::vector<double> pi(n, 0.0), key(n);
    std::vector<int> deg(n), par(n), out(n);
    double best = -INFINITY, lam = 2.0;
    int stall = 0;
    best_pi.assign(n, 0.0);
    const double *Dp = D.data();
    for (int it = 0; it < 300 && n >= 3; ++it) {
        std::fill(deg.begin(), deg.end(), 0);
        double lb = 0.0;
        // Prim from city 1 over cities 1..n-1 on d' = (d + pi_x) + pi_y: the
        // cities not in the tree kept in a compact list, ascending, so every
        // scan touches only them and the first minimum is the lowest index
        // (the same tree, the same sums as the scan over all cities with an
        // in-tree flag it replaces: round 6, 32 cities ~1.3 ms)
        int m = 0;
        {
            const double *D1 = Dp + n;
            const double p1 = pi[1];
            for (int v = 2; v < n; ++v) {
                key[v] = (D1[v] + p1) + pi[v];
                par[v] = 1;
                out[m++] = v;
            }
        }
        while (m > 0) {
            int bi = 0;
            double bk = key[out[0]];
            for (int i = 1; i < m; ++i) {
                const double k = key[out[i]];
                if (k < bk) bk = k, bi = i;
            }
            const int u = out[bi];
            for (int i = bi + 1; i < m; ++i) out[i - 1] = out[i];
            --m;
            lb += bk;
            ++deg[u];
            ++deg[par[u]];
            const double *Du = Dp + (size_t)u * n;
            const double pu = pi[u];
            for (int i = 0; i < m; ++i) {
                const int v = out[i];
                const double w = (Du[v] + pu) + pi[v];
                if (w < key[v]) key[v] = w, par[v] = u;
            }
        }
        auto dp0 = [&](int v) { return (Dp[v] + pi[0]) + pi[v]; };
        int a = -1, b = -1;
        for (int v = 1; v < n; ++v) {
            if (a < 0 || dp0(v) < dp0(a))
                b = a, a = v;
            else if (b < 0 || dp0(v) < dp0(b))
                b = v;
        }
        lb += dp0(a) + dp0(b);
        deg[0] = 2;
        ++deg[a];
        ++deg[b];
        for (int x = 0; x < n; ++x) lb -= 2.0 * pi[x];
        if (lb > best) {
            best = lb;
            best_pi = pi;
            stall = 0;
        } else if (++stall >= 10) {
            lam *= 0.7;
            stall = 0;
        }
        double nn = 0.0;
        for (int x = 0; x < n; ++x) nn += (double)(deg[x] - 2) * (deg[x] - 2);
        if (nn == 0.0 || !(ub > lb)) break;
        const double t = lam * (ub - lb) / nn;
        for (int x = 0; x < n; ++x) pi[x] += t * (deg[x] - 2);
    }
}

// Multi-start upper bound: a nearest-neighbour tour from every city, each
// improved by 2-opt + Or-opt, rotated to start at city 0; the best exact fold
// (tsp.cpp's cost, either direction) is a valid bound >= OPT.  A tight start
// matters: every node the search prunes is pruned against it.
// Starts first, first + step, ... (several ranks split the starts and take the
// MIN of their costs: the same bound as all starts in one process).  From 20
// cities the starts run on up to 8 host threads (32 cities: ~2.2 ms serial,
// more than the search's kernels); the results are combined in start order by
// the same rule, so the tour is the serial one.
template <typename V>
bool heuristic(const V *d, int n, std::vector<int32_t> &best, V &cost, int first = 0, int step = 1)
{
    std::vector<int> starts;
    for (int s0 = first; s0 < n; s0 += step) starts.push_back(s0);
    // below 20 cities (one thread) four spread-out starts: each start costs
    // ~7 us at 16 cities, all sixteen were a quarter of the whole in-process
    // search, and the device's suffix tests tighten the bound within the
    // first expansion anyway (profiles/r03/k2_variants.log)
    if (n < 20 && (int)starts.size() > 4 && tuned_or("HEURISTIC_ALL_STARTS", 0) == 0) {
        std::vector<int> few;
        for (int i = 0; i < 4; ++i) few.push_back(starts[(size_t)i * starts.size() / 4]);
        starts.swap(few);
    }
    const int ns = (int)starts.size();
    std::vector<std::vector<int32_t>> tours(ns);
    std::vector<V> costs(ns);
    auto one = [&](int i) {
        const int s0 = starts[i];
        std::vector<int> t(n);
        std::vector<char> used(n, 0);
        t[0] = s0;
        used[s0] = 1;
        for (int a = 1; a < n; ++a) {
            int b = -1;
            for (int j = 0; j < n; ++j)
                if (!used[j] && (b < 0 || d[t[a - 1] * n + j] < d[t[a - 1] * n + b])) b = j;
            t[a] = b;
            used[b] = 1;
        }
        local_search(d, n, t);
        std::rotate(t.begin(), std::find(t.begin(), t.end(), 0), t.end());
        std::vector<int32_t> fw(t.begin() + 1, t.end()), bw(fw.rbegin(), fw.rend());
        const V cf = fold_tour(d, n, fw.data()), cb = fold_tour(d, n, bw.data());
        costs[i] = cb < cf ? cb : cf;
        tours[i] = cb < cf ? std::move(bw) : std::move(fw);
    };
    int nt = n >= 20 ? std::min(ns, 8) : 1;
    if (double v; tuned("HEURISTIC_THREADS", &v)) nt = std::max(1, std::min(ns, (int)v));
    bool done = false;
    if (nt > 1) {
        std::vector<std::thread> th;
        try {
            th.reserve(nt);
            for (int w = 0; w < nt; ++w)
                th.emplace_back([&, w] {
                    for (int i = w; i < ns; i += nt) one(i);
                });
            done = true;
        } catch (...) {  // no thread: the serial loop below (every start again)
        }
        for (auto &x : th) x.join();
    }
    if (!done)
        for (int i = 0; i < ns; ++i) one(i);
    bool have = false;
    for (int i = 0; i < ns; ++i)
        if (!have || costs[i] < cost) {
            best = tours[i];
            cost = costs[i];
            have = true;
        }
    return have;
}

template <typename V>
int select_tour(const V *d, int n, const tspgpu_tour_record *rec, int count, V opt, int32_t *tour_out)
{
    const int N = n - 1;
    // keep the optimal records; fold[c * N + j-1] = left fold up to the j-th inner city
    std::vector<const uint8_t *> city;
    std::vector<V> fold;
    city.reserve(count);
    fold.reserve((size_t)count * N);
    for (int r = 0; r < count; ++r) {
        const uint8_t *t = rec[r].city;
        V acc = 0;
        int prev = 0;
        const size_t base = fold.size();
        for (int j = 1; j <= N; ++j) {
            acc = acc + d[prev * n + t[j - 1]];
            fold.push_back(acc);
            prev = t[j - 1];
        }
        if (!(acc + d[prev * n] == opt)) {  // recorded against an older incumbent
            fold.resize(base);
            continue;
        }
        city.push_back(t);
    }
    if (city.empty()) return -EIO;
    std::vector<int> alive(city.size());
    for (size_t i = 0; i < city.size(); ++i) alive[i] = (int)i;
    std::vector<int32_t> tour(N + 2, 0);
    std::vector<char> seen(n);
    std::vector<V> best(n);
    V target = opt;
    int next = 0;
    for (int j = N; j >= 1; --j) {
        // t_j candidates among the tours sharing the chosen suffix: best prefix fold per city
        std::fill(seen.begin(), seen.end(), 0);
        for (int idx : alive) {
            const int m = city[idx][j - 1];
            const V f = fold[(size_t)idx * N + (j - 1)];
            if (!seen[m] || f < best[m]) best[m] = f;
            seen[m] = 1;
        }
        int pick = -1;
        for (int m = 1; m <= N; ++m)
            if (seen[m] && best[m] + d[m * n + next] == target) {
                pick = m;
                break;
            }
        if (pick < 0) return -EIO;
        std::vector<int> keep;
        for (int idx : alive)
            if (city[idx][j - 1] == pick) keep.push_back(idx);
        alive.swap(keep);
        tour[j] = pick;
        target = best[pick];
        next = pick;
    }
    std::memcpy(tour_out, tour.data(), sizeof(int32_t) * (N + 2));
    return 0;
}

// Device tie rule, host side (search.h "Device tie rule"): key <-> tour and
// the certificate that the decoded tour is the one tsp()'s argmin chain picks.
int tie_split(int N) { return N <= 20 ? N : 13; }

void tie_key(int N, const int32_t *t /* t[1..N] */, uint64_t &w0, uint64_t &w1)
{
    const int split = tie_split(N);
    uint32_t unused = (uint32_t)(((1ull << N) - 1ull) << 1);
    w0 = w1 = 0;
    for (int p = 0; p < N; ++p) {
        const int c = t[N - p];
        const uint64_t dig = (uint64_t)__builtin_popcount(unused & ((1u << c) - 1u));
        unused &= ~(1u << c);
        if (p < split)
            w0 = w0 * (uint64_t)(N - p) + dig;
        else
            w1 = w1 * (uint64_t)(N - p) + dig;
    }
}

// digits of the key -> t[1..N]; false if a digit is out of range
bool tie_decode(int N, uint64_t w0, uint64_t w1, int32_t *t)
{
    const int split = tie_split(N);
    std::vector<uint64_t> dig(N);
    for (int p = N - 1; p >= 0; --p) {
        uint64_t &w = p < split ? w0 : w1;
        const uint64_t r = (uint64_t)(N - p);
        dig[p] = w % r;
        w /= r;
    }
    if (w0 != 0 || w1 != 0) return false;
    std::vector<int> left;
    for (int c = 1; c <= N; ++c) left.push_back(c);
    for (int p = 0; p < N; ++p) {
        t[N - p] = left[dig[p]];
        left.erase(left.begin() + (long)dig[p]);
    }
    return true;
}

// G[{t1..tj}][tj] of the reference's DP (the minimum left fold of a path from
// city 0 over t1..tj ending at tj), by Held-Karp over those j cities
constexpr int kTieDpMax = 16;
double prefix_min(const double *d, int n, const int32_t *t, int j)
{
    const int J = j;
    const uint32_t full = (1u << J) - 1u;
    std::vector<double> G((size_t)J << J, INFINITY);
    for (int a = 0; a < J; ++a) G[((size_t)1u << a) * J + a] = d[t[a + 1]];
    for (uint32_t S = 1; S <= full; ++S)
        for (int k = 0; k < J; ++k) {
            if (!((S >> k) & 1u) || S == (1u << k)) continue;
            const uint32_t P = S & ~(1u << k);
            double best = INFINITY;
            for (int m = 0; m < J; ++m)
                if ((P >> m) & 1u) {
                    const double v = G[(size_t)P * J + m] + d[t[m + 1] * n + t[k + 1]];
                    best = v < best ? v : best;
                }
            G[(size_t)S * J + k] = best;
        }
    return G[(size_t)full * J + (J - 1)];
}

int records_prefix(void *user, const double *d, int n, const int32_t *t, int j, double *g)
{
    const auto *rp = static_cast<const RecordsPrefix *>(user);
    const auto *recs = static_cast<const tspgpu_tour_record *>(rp->recs);
    const int N = n - 1;
    double best = INFINITY;
    bool have_t = false;  // t itself among the optimal records (else they are not all of O)
    for (int r = 0; r < rp->count; ++r) {
        const tspgpu_tour_record &R = recs[r];
        if (R.cost != rp->opt_bits) continue;
        bool same_tail = true;  // positions j..N: the same prefix set and the same end t_j
        for (int i = j; i <= N && same_tail; ++i) same_tail = R.city[i - 1] == t[i];
        if (!same_tail) continue;
        double f = 0.0;  // the left fold of the prefix, as tsp()'s DP folds it
        int prev = 0;
        bool same = true;
        for (int i = 1; i <= j; ++i) {
            f = f + d[prev * n + R.city[i - 1]];
            prev = R.city[i - 1];
            same = same && R.city[i - 1] == t[i];
        }
        have_t = have_t || same;
        best = f < best ? f : best;
    }
    if (have_t) {
        *g = best;
        return 0;
    }
    if (rp->next) return rp->next(rp->next_user, d, n, t, j, g);
    return -EAGAIN;
}

// 0: t (t[0] = 0, t[1..N]) folds to opt and every prefix fold is minimal
// (no value one ulp lower could round to the same next fold); -EAGAIN: the
// fold matches but that is not proven; -EINVAL: not a tour of cost opt
template <typename V>
int tie_certify(const V *d, int n, const int32_t *t, V opt, bool allow_dp, PrefixDp dp, void *user, int host_max)
{
    const int N = n - 1;
    std::vector<V> F(N + 2);
    V acc = 0;
    int prev = 0;
    for (int j = 1; j <= N; ++j) {
        acc = acc + d[prev * n + t[j]];
        F[j] = acc;
        prev = t[j];
    }
    F[N + 1] = acc + d[prev * n];
    if (!(F[N + 1] == opt)) return -EINVAL;
    if constexpr (std::is_same<V, double>::value) {
        // every fold exact (all distances multiples of one power of two 2^e
        // and n * max below 2^(e+53), e.g. integer-valued or coincident
        // cities): the arithmetic is the integers', nothing to prove
        int emin = INT_MAX;
        double mx = 0.0;
        for (int i = 0; i < n * n; ++i) {
            const double v = d[i];
            if (v == 0.0) continue;
            uint64_t b;
            std::memcpy(&b, &v, 8);
            const int be = (int)((b >> 52) & 0x7FF);
            uint64_t m = b & ((1ull << 52) - 1ull);
            if (be) m |= 1ull << 52;
            const int low = (be ? be - 1075 : -1074) + __builtin_ctzll(m);
            emin = std::min(emin, low);
            mx = std::max(mx, v);
        }
        if (emin == INT_MAX || (double)n * mx < std::ldexp(1.0, emin + 53)) return 0;
        for (int j = 2; j <= N; ++j) {
            const double dj = j < N ? d[t[j] * n + t[j + 1]] : d[t[N] * n];
            const volatile double below = std::nextafter(F[j], -INFINITY);
            const volatile double next = below + dj;
            if (next < F[j + 1]) continue;
            // a fold just below F[j] would round to the same next fold: the
            // prefix is proven minimal only by the DP over its own cities
            if (!allow_dp) return -EAGAIN;
            double g = 0.0;
            if (j <= std::min(host_max, kTieDpMax))
                g = prefix_min(d, n, t, j);
            else if (!dp || dp(user, d, n, t, j, &g) != 0)
                return -EAGAIN;
            if (!(g == F[j])) return -EAGAIN;
        }
    }
    return 0;
}

int validate_search(const void *dist, int dtype, int n)
{
    if (!dist || n < 3 || n > TSPGPU_SEARCH_MAX_CITIES) return -EINVAL;
    if (dtype == TSPGPU_F64) {
        const double *d = static_cast<const double *>(dist);
        double mx = 0.0;
        for (int i = 0; i < n * n; ++i) {
            if (!(d[i] >= 0.0) || !std::isfinite(d[i])) return -EINVAL;
            mx = std::max(mx, d[i]);
        }
        if ((double)n * mx >= (double)INT_MAX) return -ERANGE;  // tsp.cpp:411,453 sentinel
        return 0;
    }
    if (dtype == TSPGPU_I32) {
        const int32_t *d = static_cast<const int32_t *>(dist);
        long long mx = 0;
        for (int i = 0; i < n * n; ++i) {
            if (d[i] < 0) return -EINVAL;
            mx = std::max<long long>(mx, d[i]);
        }
        if ((long long)n * mx >= (1ll << 30)) return -ERANGE;
        return 0;
    }
    return -EINVAL;
}

int tie_tour(const void *dist, int dtype, int n, uint64_t w0, uint64_t w1, uint64_t cost_bits, int32_t *tour_out,
             bool allow_dp, PrefixDp dp, void *user, int host_max)
{
    int rc = validate_search(dist, dtype, n);
    if (rc) return rc;
    if (!tour_out) return -EINVAL;
    std::vector<int32_t> t(n + 1, 0);
    if (!tie_decode(n - 1, w0, w1, t.data())) return -EINVAL;
    if (dtype == TSPGPU_F64) {
        double opt;
        std::memcpy(&opt, &cost_bits, 8);
        rc = tie_certify(static_cast<const double *>(dist), n, t.data(), opt, allow_dp, dp, user, host_max);
    } else {
        rc = tie_certify(static_cast<const int32_t *>(dist), n, t.data(), (int32_t)(uint32_t)cost_bits, allow_dp, dp,
                         user, host_max);
    }
    if (rc != -EINVAL) std::memcpy(tour_out, t.data(), sizeof(int32_t) * (n + 1));
    return rc;
}

}  // namespace host
}  // namespace tspgpu

using namespace tspgpu::host;

extern "C" {

int tspgpu_heuristic_tour(const void *dist, int dtype, int n, double *cost_out, int32_t *tour_out)
{
    return tspgpu_heuristic_tour_starts(dist, dtype, n, 0, 1, cost_out, tour_out);
}

int tspgpu_heuristic_tour_starts(const void *dist, int dtype, int n, int first, int step, double *cost_out,
                                 int32_t *tour_out)
{
    int rc = validate_search(dist, dtype, n);
    if (rc) return rc;
    if (first < 0 || step < 1) return -EINVAL;
    if (first >= n) return -ENOENT;  // no start city in this range
    std::vector<int32_t> t;
    if (dtype == TSPGPU_F64) {
        double c = 0.0;
        heuristic(static_cast<const double *>(dist), n, t, c, first, step);
        if (cost_out) *cost_out = c;
    } else {
        int32_t c = 0;
        heuristic(static_cast<const int32_t *>(dist), n, t, c, first, step);
        if (cost_out) *cost_out = c;
    }
    if (tour_out) {
        tour_out[0] = 0;
        for (int i = 0; i < n - 1; ++i) tour_out[i + 1] = t[i];
        tour_out[n] = 0;
    }
    return 0;
}

int tspgpu_select_tour(const void *dist, int dtype, int n, const tspgpu_tour_record *records, int count,
                       uint64_t cost_bits, int32_t *tour_out)
{
    int rc = validate_search(dist, dtype, n);
    if (rc) return rc;
    if (count <= 0 || !records || !tour_out) return -EINVAL;
    if (dtype == TSPGPU_F64) {
        double opt;
        std::memcpy(&opt, &cost_bits, 8);
        return select_tour(static_cast<const double *>(dist), n, records, count, opt, tour_out);
    }
    return select_tour(static_cast<const int32_t *>(dist), n, records, count, (int32_t)(uint32_t)cost_bits,
                       tour_out);
}

int tspgpu_tie_key(int n, const int32_t *tour, uint64_t *w0, uint64_t *w1)
{
    if (!tour || !w0 || !w1 || n < 3 || n > TSPGPU_SEARCH_MAX_CITIES) return -EINVAL;
    uint32_t seen = 0;
    for (int j = 1; j < n; ++j) {
        if (tour[j] < 1 || tour[j] >= n || ((seen >> tour[j]) & 1u)) return -EINVAL;
        seen |= 1u << tour[j];
    }
    uint64_t a, b;
    tie_key(n - 1, tour, a, b);
    *w0 = a;
    *w1 = b;
    return 0;
}

int tspgpu_tie_tour(const void *dist, int dtype, int n, uint64_t w0, uint64_t w1, uint64_t cost_bits,
                    int32_t *tour_out)
{
    return tie_tour(dist, dtype, n, w0, w1, cost_bits, tour_out, true);
}

}  // extern "C"
