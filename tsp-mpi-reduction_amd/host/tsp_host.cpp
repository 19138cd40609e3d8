// Host parity layer (include/tsp_host.h): the reference's program logic around
// the block search, so that the drop-in `tsp` prints what `mpirun -np P ./tsp`
// prints.  Pure host C++; the GPU is not involved here.
#include "tsp_host.h"

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

// glibc pow is called for real (assignment2.h:143): a volatile pointer stops
// the compiler from folding pow(x,2) into x*x, which rounds differently.
double (*volatile g_pow)(double, double) = ::pow;
double (*volatile g_sqrt)(double) = ::sqrt;

inline double city_dist(const tspgpu_city &a, const tspgpu_city &b)
{
    const double dx = g_pow(a.x - b.x, 2);
    const double dy = g_pow(a.y - b.y, 2);
    return g_sqrt(dx + dy);
}

struct Solution {
    std::vector<tspgpu_city> path;
    double cost = 0.0;
};

// mergeBlocks (tsp.cpp:202-269).  The reference rotates both lists inside its
// search; the pair examined at step (i, j) is (c1[i], c1[i+1 mod L1]) x
// (c2[j], c2[j+1 mod L2]), so index arithmetic gives the same first strict
// minimum (start value INT_MAX, tsp.cpp:204) in O(L1*L2).
bool merge_into(Solution &s1, const tspgpu_city *c2, int L2, double cost2)
{
    const std::vector<tspgpu_city> &c1 = s1.path;
    const int L1 = (int)c1.size();
    double best = (double)INT_MAX;
    int bi = 0, bj = 0;
    for (int i = 0; i < L1; ++i) {
        const tspgpu_city &A = c1[i], &B = c1[(i + 1) % L1];
        const double ab = city_dist(A, B);
        for (int j = 0; j < L2; ++j) {
            const tspgpu_city &C = c2[j], &D = c2[(j + 1) % L2];
            // swapPairCost, tsp.cpp:197-200: ((d(A,D) + d(B,C)) - d(A,B)) - d(C,D)
            const double sc = city_dist(A, D) + city_dist(B, C) - ab - city_dist(C, D);
            if (sc < best) {
                best = sc;
                bi = i;
                bj = j;
            }
        }
    }
    const int idA = c1[bi].id, idB = c1[(bi + 1) % L1].id, idC = c2[bj].id;
    // splice: c2 minus its closing city, rotated so C is first, then once more,
    // inserted reversed after the first c1 city that is A or B (tsp.cpp:229-259)
    const int M = L2 - 1;
    int start = 0;
    while (start < M && c2[start].id != idC) ++start;
    if (start == M) return false;  // reference loops forever (tsp.cpp:236-239)
    start = (start + 1) % M;
    std::vector<tspgpu_city> out;
    out.reserve((size_t)L1 + (size_t)M);
    bool pending = true;
    for (int i = 0; i < L1; ++i) {
        out.push_back(c1[i]);
        if (pending && (c1[i].id == idA || c1[i].id == idB)) {
            pending = false;
            for (int j = M - 1; j >= 0; --j) out.push_back(c2[(start + j) % M]);
        }
    }
    s1.cost = s1.cost + cost2 + best;  // tsp.cpp:263
    s1.path.swap(out);
    return true;
}

void append_log(std::string &log, int recv, int ncities, int from)
{
    char line[128];
    std::snprintf(line, sizeof line, "process %i is about to receive %i cities from process %i\n", recv, ncities,
                  from);
    log += line;
}

}  // namespace

extern "C" {

void tsphost_blocks_per_dim(int nblocks, int *rows, int *cols)
{
    // ISSQUARE (assignment2.h:11), else the smallest divisor >= 2 (tsp.cpp:147-154)
    const double r = std::sqrt((double)nblocks);
    if (r - std::floor(r) == 0) {
        *rows = *cols = (int)r;
        return;
    }
    int div = 2;
    while (nblocks % div != 0) ++div;
    *rows = div;
    *cols = nblocks / div;
}

int tsphost_generate(int n, int nblocks, int grid_x, int grid_y, tspgpu_city *out)
{
    int R, C;
    tsphost_blocks_per_dim(nblocks, &R, &C);
    std::srand(0);  // tsp.cpp:273
    return tsphost_generate_grid(n, R, C, grid_x, grid_y, out);
}

int tsphost_generate_grid(int n, int R, int C, int grid_x, int grid_y, tspgpu_city *out)
{
    // block extents are float (tsp.cpp:378-379): the float products below are
    // what the reference passes (promoted) to fRand
    const float xspan = grid_x / (float)R;
    const float yspan = grid_y / (float)C;
    int id = 0;
    for (int b = 0; b < R * C; ++b) {
        const int row = (b - b % R) / R;
        const int col = (C - b % C) - 1;
        const float x_lo = row * xspan, x_hi = (row + 1) * xspan;
        const float y_lo = col * yspan, y_hi = (col + 1) * yspan;
        for (int j = 0; j < n; ++j) {
            tspgpu_city &c = out[(size_t)b * n + j];
            c.id = id++;
            // fRand (assignment2.h:86-91), x then y
            const double fx = (double)std::rand() / RAND_MAX;
            c.x = (double)x_lo + fx * ((double)x_hi - (double)x_lo);
            const double fy = (double)std::rand() / RAND_MAX;
            c.y = (double)y_lo + fy * ((double)y_hi - (double)y_lo);
        }
    }
    return R * C;
}

void tsphost_distribution_counts(int nblocks, int nprocs, int *counts)
{
    for (int r = 0; r < nprocs; ++r) counts[r] = 0;
    for (int b = nblocks; b > 0; --b) counts[b % nprocs]++;
}

int tsphost_merge(const tspgpu_city *p1, int L1, double c1, const tspgpu_city *p2, int L2, double c2,
                  tspgpu_city *out, double *cost_out)
{
    Solution s;
    s.path.assign(p1, p1 + L1);
    s.cost = c1;
    if (!merge_into(s, p2, L2, c2)) return -1;
    std::memcpy(out, s.path.data(), s.path.size() * sizeof(tspgpu_city));
    *cost_out = s.cost;
    return (int)s.path.size();
}

int tsphost_reduce(const tspgpu_city *paths, int L, const double *costs, int nblocks, int nprocs,
                   double *final_cost, char *log, int logcap)
{
    if (log && logcap > 0) log[0] = 0;
    if (nblocks < 1 || nprocs < 1 || nblocks < nprocs || L < 2) return -1;
    std::vector<int> cnt(nprocs);
    tsphost_distribution_counts(nblocks, nprocs, cnt.data());

    // each logical rank: its contiguous block range, folded left (tsp.cpp:348-352)
    std::vector<Solution> rank(nprocs);
    int next = 0;
    for (int r = 0; r < nprocs; ++r) {
        rank[r].path.assign(paths + (size_t)next * L, paths + (size_t)(next + 1) * L);
        rank[r].cost = costs[next];
        ++next;
        for (int j = 1; j < cnt[r]; ++j, ++next)
            if (!merge_into(rank[r], paths + (size_t)next * L, L, costs[next])) return -1;
    }

    // MPI_ManualReduce: the receiver appends every received path to one
    // function-local list and merges with the WHOLE list (tsp.cpp:67,93-98,115-120)
    std::vector<std::vector<tspgpu_city>> received(nprocs);
    std::string text;
    auto receive = [&](int to, int from) {
        const Solution &snd = rank[from];
        received[to].insert(received[to].end(), snd.path.begin(), snd.path.end());
        return merge_into(rank[to], received[to].data(), (int)received[to].size(), snd.cost);
    };
    const int lastpower = 1 << (int)std::log2((double)nprocs);
    for (int i = 0; i < nprocs - lastpower; ++i) {
        append_log(text, i, (int)rank[i + lastpower].path.size(), i + lastpower);
        if (!receive(i, i + lastpower)) return -1;
    }
    for (int d = 0; d < (int)std::log2((double)lastpower); ++d)
        for (int k = 0; k < lastpower; k += 1 << (d + 1))
            if (!receive(k, k + (1 << d))) return -1;

    *final_cost = rank[0].cost;
    if (log && logcap > 0) {
        const size_t m = text.size() < (size_t)logcap - 1 ? text.size() : (size_t)logcap - 1;
        std::memcpy(log, text.data(), m);
        log[m] = 0;
    }
    return 0;
}

}  // extern "C"
