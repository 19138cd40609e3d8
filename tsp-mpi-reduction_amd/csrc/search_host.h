// Host-only parts of K2 (no HIP): the initial bound (multi-start 2-opt /
// Or-opt tour), the Lagrangian and Held-Karp (1-tree) city weights of the
// search bounds, the input check, and the selection of tsp()'s own tour from
// the optimal set O (why that selection is exact: search_abi.cpp's header).
// Split from search_abi.cpp so the host ASan/UBSan check (make check-asan)
// builds it with plain g++.
#pragma once
#include <stdint.h>

#include <vector>

namespace tspgpu {
namespace host {
// 0, -EINVAL (null, n outside 3..32, negative / non-finite entries, dtype) or
// -ERANGE (a tour could reach the reference's INT_MAX sentinel, tsp.cpp:411,453)
int validate_search(const void *dist, int dtype, int n);
// subgradient ascent on the degree relaxation: city weights for the two-edge bound
void lagrange_pi(const std::vector<double> &D, int n, std::vector<double> &best_pi);
// Held-Karp 1-tree weights (the tree bound of the expand kernel)
void held_karp_pi(const std::vector<double> &D, int n, std::vector<double> &best_pi);
// G[{t1..tj}][tj] of the reference's DP for the certificate's prefix checks
// above the host's own limit (e.g. K1-wide on the GPU): 0 and *g, or an error
// (the certificate then stays unproven)
typedef int (*PrefixDp)(void *user, const double *d, int n, const int32_t *t, int j, double *g);
// tspgpu_tie_tour; allow_dp = false skips the prefix DP of the certificate
// (a cheap check when the records can decide anyway); prefixes of up to
// host_max cities by Held-Karp on the host, longer ones through dp (if any)
int tie_tour(const void *dist, int dtype, int n, uint64_t w0, uint64_t w1, uint64_t cost_bits, int32_t *tour_out,
             bool allow_dp, PrefixDp dp = nullptr, void *user = nullptr, int host_max = 16);
// G[{t1..tj}][tj] from the COMPLETE set O of the search's optimal tours
// instead of a DP (round 6): an ordering P' of the prefix set {t1..tj} ending
// at tj with fold(P') <= F[j] makes P' + (t_{j+1}..t_N) a tour of cost <= OPT
// (rounding is monotone), i.e. a member of O; so the least prefix fold over
// the tours of O that share positions j..N with t is min(G, F[j]) = G.
// Every tour of cost <= the incumbent at the time is recorded and no tour of
// cost OPT is ever pruned, so O is complete whenever the records did not
// overflow — the caller's guarantee (count = every record of the search).
// user = RecordsPrefix; when t itself is not among the records (they are not
// the whole set after all) it defers to next (or fails: -EAGAIN).
struct RecordsPrefix {
    const void *recs;  // tspgpu_tour_record[count]: cost word, then cities t1..tN
    int count;
    uint64_t opt_bits;
    PrefixDp next;     // fallback DP (may be null)
    void *next_user;
};
int records_prefix(void *user, const double *d, int n, const int32_t *t, int j, double *g);
}  // namespace host
}  // namespace tspgpu
