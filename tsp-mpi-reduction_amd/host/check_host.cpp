// Host-code check under AddressSanitizer + UBSan (`make check-asan`): the
// CPU halves of the product — the host parity layer (host/tsp_host.cpp:
// generator, distribution, mergeBlocks, reduction-tree replay) and K2's host
// algorithms (csrc/search_host.cpp: input check, multi-start tour, Lagrangian
// and 1-tree weights, the tie rule over the optimal set) — driven over a grid
// of sizes and edge cases, with the results compared against the CPU oracle
// (oracle/oracle.c, the checker, compiled into this test binary only).  Any
// sanitizer report aborts (-fno-sanitize-recover=all); a mismatch exits 1.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../oracle/oracle.h"
#include "../csrc/search_host.h"
#include "tsp_host.h"
#include "tspgpu.h"

namespace {

int failures = 0;

void expect(bool ok, const char *what, int a = 0, int b = 0, int c = 0)
{
    if (!ok) {
        std::fprintf(stderr, "MISMATCH %s (%d %d %d)\n", what, a, b, c);
        ++failures;
    }
}

uint64_t rng_state = 0x9e3779b97f4a7c15ull;
double urand()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (double)(rng_state >> 11) * 0x1p-53;
}

// generator, counts, merge tree: host layer == oracle for (n, B, P)
void check_pipeline(int n, int B, int P)
{
    std::vector<tspgpu_city> h((size_t)n * B);
    std::vector<oracle_city> o((size_t)n * B);
    tsphost_generate(n, B, 1000, 1000, h.data());
    oracle_generate(n, B, 1000, 1000, o.data());
    for (size_t i = 0; i < h.size(); ++i)
        expect(h[i].id == o[i].id && h[i].x == o[i].x && h[i].y == o[i].y, "generate", n, B, (int)i);
    std::vector<int> ch(P), co(P);
    tsphost_distribution_counts(B, P, ch.data());
    oracle_distribution_counts(B, P, co.data());
    expect(ch == co, "distribution counts", B, P);
    // every block solved by the oracle, then the host layer's fold + tree
    const int L = n == 2 ? 2 : n + 1;  // tspgpu_tour_length (the n = 2 quirk, tsp.cpp:483-502)
    std::vector<tspgpu_city> paths((size_t)B * L);
    std::vector<double> costs(B);
    std::vector<double> d((size_t)n * n);
    std::vector<int32_t> tour(n + 1);
    for (int b = 0; b < B; ++b) {
        oracle_distance_matrix(&o[(size_t)b * n], n, d.data());
        oracle_solve_block(d.data(), n, &costs[b], tour.data());
        for (int i = 0; i < L; ++i) paths[(size_t)b * L + i] = h[(size_t)b * n + tour[i]];
    }
    double fh = 0.0, fo = 0.0;
    std::vector<char> lh(1 << 16), lo(1 << 16);
    const int rh = tsphost_reduce(paths.data(), L, costs.data(), B, P, &fh, lh.data(), (int)lh.size());
    const int ro = oracle_pipeline(n, B, 1000, 1000, P, &fo, lo.data(), (int)lo.size());
    expect(rh == ro, "reduce rc", n, B, P);
    if (rh == 0 && ro == 0) {
        expect(fh == fo, "reduce final cost", n, B, P);
        expect(std::strcmp(lh.data(), lo.data()) == 0, "reduce log", n, B, P);
    }
}

// mergeBlocks on two random closed paths
void check_merge(int L1, int L2)
{
    std::vector<tspgpu_city> a(L1), b(L2);
    std::vector<oracle_city> oa(L1), ob(L2);
    for (int i = 0; i < L1; ++i) a[i] = {i, 1000 * urand(), 1000 * urand()};
    for (int i = 0; i < L2; ++i) b[i] = {100 + i, 1000 * urand(), 1000 * urand()};
    a[L1 - 1] = a[0];
    b[L2 - 1] = b[0];
    for (int i = 0; i < L1; ++i) oa[i] = {a[i].id, a[i].x, a[i].y};
    for (int i = 0; i < L2; ++i) ob[i] = {b[i].id, b[i].x, b[i].y};
    std::vector<tspgpu_city> out(L1 + L2 - 1);
    std::vector<oracle_city> oout(L1 + L2 - 1);
    double ch = 0.0, co = 0.0;
    const int rh = tsphost_merge(a.data(), L1, 10.0, b.data(), L2, 20.0, out.data(), &ch);
    const int ro = oracle_merge_blocks(oa.data(), L1, 10.0, ob.data(), L2, 20.0, oout.data(), &co);
    expect(rh == ro || rh < 0, "merge length", L1, L2);
    if (rh == ro && rh > 0) {
        expect(ch == co, "merge cost", L1, L2);
        for (int i = 0; i < rh; ++i) expect(out[i].id == oout[i].id, "merge path", L1, L2, i);
    }
}

// K2 host algorithms on random instances: the multi-start tour is a
// permutation whose cost is its left fold, >= the optimum; the tie rule on the
// optimal tour alone returns that tour; the weights are finite
void check_search_host(int n, bool integer)
{
    std::vector<double> xy(2 * n);
    for (auto &v : xy) v = 1000 * urand();
    std::vector<double> d((size_t)n * n);
    std::vector<int32_t> di((size_t)n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            d[(size_t)i * n + j] = std::sqrt(std::pow(xy[2 * i] - xy[2 * j], 2) + std::pow(xy[2 * i + 1] - xy[2 * j + 1], 2));
            di[(size_t)i * n + j] = (int32_t)std::lround(d[(size_t)i * n + j]);
            if (integer) d[(size_t)i * n + j] = di[(size_t)i * n + j];
        }
    const void *dist = integer ? (const void *)di.data() : (const void *)d.data();
    const int dtype = integer ? TSPGPU_I32 : TSPGPU_F64;
    expect(tspgpu::host::validate_search(dist, dtype, n) == 0, "validate", n);
    std::vector<int32_t> t(n + 1);
    double ub = 0.0;
    expect(tspgpu_heuristic_tour(dist, dtype, n, &ub, t.data()) == 0, "heuristic rc", n);
    std::vector<int> seen(n, 0);
    double fold = 0.0;
    for (int i = 0; i < n; ++i) {
        seen[t[i]]++;
        fold = fold + d[(size_t)t[i] * n + t[i + 1]];
    }
    for (int i = 0; i < n; ++i) expect(seen[i] == 1, "heuristic permutation", n, i);
    expect(t[0] == 0 && t[n] == 0 && fold == ub, "heuristic cost", n);
    double ub2 = 0.0;
    expect(tspgpu_heuristic_tour_starts(dist, dtype, n, 1, 3, &ub2, nullptr) == 0 && ub2 >= 0.0, "starts", n);
    std::vector<double> pi;
    tspgpu::host::lagrange_pi(d, n, pi);
    for (double v : pi) expect(std::isfinite(v), "lagrange finite", n);
    tspgpu::host::held_karp_pi(d, n, pi);
    for (double v : pi) expect(std::isfinite(v), "held-karp finite", n);
    if (n <= 12) {  // the exact optimum (oracle DP) as the only record
        double opt = 0.0;
        std::vector<int32_t> ot(n + 1);
        oracle_solve_block(d.data(), n, &opt, ot.data());
        expect(opt <= ub, "bound above optimum", n);
        tspgpu_tour_record r{};
        uint64_t bits = 0;
        if (integer) {
            bits = (uint32_t)(int32_t)opt;
        } else {
            std::memcpy(&bits, &opt, 8);
        }
        r.cost = bits;
        for (int i = 1; i < n; ++i) r.city[i - 1] = (uint8_t)ot[i];
        std::vector<int32_t> sel(n + 1);
        expect(tspgpu_select_tour(dist, dtype, n, &r, 1, bits, sel.data()) == 0, "select rc", n);
        expect(sel == ot, "select tour", n);
    }
    // invalid inputs are refused, not read out of bounds
    expect(tspgpu::host::validate_search(dist, dtype, 2) != 0, "validate n=2", n);
    expect(tspgpu_select_tour(dist, dtype, n, nullptr, 0, 0, t.data()) != 0, "select empty", n);
}

}  // namespace

int main()
{
    for (int n : {2, 3, 5, 8, 12})
        for (int B : {1, 2, 4, 7, 16})
            for (int P : {1, 2, 3, 4, 8})
                if (B >= P) check_pipeline(n, B, P);
    for (int L1 : {3, 5, 9, 17})
        for (int L2 : {3, 6, 13}) check_merge(L1, L2);
    for (int n = 3; n <= 32; n += (n < 12 ? 1 : 5))
        for (bool integer : {false, true}) check_search_host(n, integer);
    std::printf("check_host: %s (%d mismatches)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
