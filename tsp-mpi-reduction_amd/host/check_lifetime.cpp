// Handle lifetimes of the C ABI under host AddressSanitizer, on the GPU
// (`make check-lifetime-asan`; tests/test_lifetime_gpu.py runs it).  The
// library's host code (tspgpu.cpp, search_abi.cpp, search_host.cpp,
// tuning.cpp) is compiled with -Xarch_host -fsanitize=address; the kernels
// are the product's.  Checked:
//   * round 4's segfault: tspgpu_ctx_destroy while searches are alive (the
//     context freed the search pool through a null pointer, and a search
//     destroyed afterwards dereferenced the freed context).  Now the context
//     is only marked closing; the searches keep working and the last
//     tspgpu_search_destroy releases it.  No search may be created on a
//     closing context (-EINVAL).
//   * the natural leak order: searches never run, context destroyed first.
//   * a chain's readback after the caller lowered the incumbent word through
//     tspgpu_search_incumbent_device: counters and tie_slot report the device
//     word (a stale readback let a shard report its own incumbent
//     after the all-reduce).
// Any ASan report aborts; a wrong answer exits 1.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "tspgpu.h"

namespace {

int failures = 0;

void expect(bool ok, const char *what, long long a = 0, long long b = 0)
{
    if (!ok) {
        std::fprintf(stderr, "FAIL %s (%lld %lld)\n", what, a, b);
        ++failures;
    }
}

std::vector<double> instance(int n, uint64_t seed)
{
    std::vector<tspgpu_city> c(n);
    uint64_t x = seed * 0x9e3779b97f4a7c15ull + 1;
    for (int i = 0; i < n; ++i) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        c[i].id = i;
        c[i].x = (double)(x >> 11) * 0x1p-53 * 1000.0;
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        c[i].y = (double)(x >> 11) * 0x1p-53 * 1000.0;
    }
    std::vector<double> d((size_t)n * n);
    tspgpu_distance_matrix(c.data(), n, 1, d.data());
    return d;
}

uint64_t bits(double v)
{
    uint64_t b;
    std::memcpy(&b, &v, 8);
    return b;
}

}  // namespace

int main()
{
    if (tspgpu_device_count() < 1) {
        std::printf("check_lifetime: no GPU, skipped\n");
        return 0;
    }
    const int n = 16;
    const std::vector<double> d = instance(n, 7);
    // the optimum from K1 (the oracle of this program: K1 is pinned elsewhere)
    double opt = 0.0;
    std::vector<int32_t> tour(n + 1);
    tspgpu_ctx *k1 = nullptr;
    expect(tspgpu_ctx_create(nullptr, &k1) == 0, "ctx_create (K1)");
    expect(tspgpu_solve_blocks(k1, d.data(), n, 1, &opt, tour.data()) == 0, "solve_blocks");
    expect(tspgpu_ctx_destroy(k1) == 0, "ctx_destroy (K1)");

    // 1. context destroyed while three searches are alive (one has run)
    {
        tspgpu_ctx *c = nullptr;
        expect(tspgpu_ctx_create(nullptr, &c) == 0, "ctx_create");
        tspgpu_search *s[3] = {};
        for (int g = 0; g < 3; ++g) {
            expect(tspgpu_search_create(c, d.data(), TSPGPU_F64, n, g, 3, 0, &s[g]) == 0, "search_create", g);
            double ub = 0.0;
            expect(tspgpu_heuristic_tour(d.data(), TSPGPU_F64, n, &ub, nullptr) == 0, "heuristic");
            expect(tspgpu_search_set_bound(s[g], ub) == 0, "set_bound", g);
        }
        int done = 0;
        expect(tspgpu_search_chain(s[0], 0, nullptr, nullptr, &done) == 0, "chain");
        expect(tspgpu_ctx_destroy(c) == 0, "ctx_destroy with live searches");
        // a closing context takes no new search
        tspgpu_search *late = nullptr;
        expect(tspgpu_search_create(c, d.data(), TSPGPU_F64, n, 0, 1, 0, &late) == -EINVAL && !late,
               "search_create on a closing context");
        // the live searches still run on it
        for (int g = 1; g < 3; ++g) {
            int dn = 0;
            expect(tspgpu_search_chain(s[g], 0, nullptr, nullptr, &dn) == 0, "chain after ctx_destroy", g);
            if (!dn) expect(tspgpu_search_run_all(s[g]) == 0, "run_all after ctx_destroy", g);
        }
        uint64_t best = ~0ull;
        for (int g = 0; g < 3; ++g) {
            uint64_t inc = 0, nodes = 0, rec = 0;
            expect(tspgpu_search_counters(s[g], &inc, &nodes, &rec) == 0, "counters", g);
            best = inc < best ? inc : best;
        }
        expect(best == bits(opt), "MIN over shards == K1 optimum", (long long)best, (long long)bits(opt));
        for (int g = 0; g < 3; ++g) expect(tspgpu_search_destroy(s[g]) == 0, "search_destroy", g);  // the last releases c
    }

    // 2. searches never run, context first, then the searches in reverse order
    {
        tspgpu_ctx *c = nullptr;
        expect(tspgpu_ctx_create(nullptr, &c) == 0, "ctx_create 2");
        tspgpu_search *a = nullptr, *b = nullptr;
        expect(tspgpu_search_create(c, d.data(), TSPGPU_F64, n, 0, 1, 0, &a) == 0, "search_create a");
        expect(tspgpu_search_create(c, d.data(), TSPGPU_F64, n, 0, 1, 0, &b) == 0, "search_create b");
        tspgpu_ctx_destroy(c);
        tspgpu_search_destroy(b);
        tspgpu_search_destroy(a);
    }

    // 3. the chain's readback vs a caller-written incumbent word
    {
        tspgpu_ctx *c = nullptr;
        expect(tspgpu_ctx_create(nullptr, &c) == 0, "ctx_create 3");
        tspgpu_search *s = nullptr;
        expect(tspgpu_search_create(c, d.data(), TSPGPU_F64, n, 0, 1, 0, &s) == 0, "search_create 3");
        double ub = 0.0;
        tspgpu_heuristic_tour(d.data(), TSPGPU_F64, n, &ub, nullptr);
        tspgpu_search_set_bound(s, ub);
        int done = 0;
        expect(tspgpu_search_chain(s, 0, nullptr, nullptr, &done) == 0 && done == 1, "chain 3", done);
        uint64_t inc = 0, nodes = 0, rec = 0;
        tspgpu_search_counters(s, &inc, &nodes, &rec);
        expect(inc == bits(opt), "chain optimum", (long long)inc, (long long)bits(opt));
        tspgpu_tie_slot ts;
        expect(tspgpu_search_tie_slot(s, inc, &ts) == 0 && ts.found == 1, "tie slot at the optimum");
        // what an all-reduce MIN with a (pretend) better shard leaves in word 1
        const uint64_t lower = bits(opt * 0.5);
        void *w = tspgpu_search_incumbent_device(s);
        expect(w && hipMemcpy(w, &lower, 8, hipMemcpyHostToDevice) == hipSuccess, "write word 1");
        uint64_t inc2 = 0;
        expect(tspgpu_search_counters(s, &inc2, &nodes, &rec) == 0, "counters after write");
        expect(inc2 == lower, "counters read the device word", (long long)inc2, (long long)lower);
        expect(tspgpu_search_tie_slot(s, inc2, &ts) == 0 && ts.found == 0, "no tour at the lowered cost");
        tspgpu_search_destroy(s);
        tspgpu_ctx_destroy(c);
    }
    if (failures) {
        std::fprintf(stderr, "check_lifetime: %d failures\n", failures);
        return 1;
    }
    std::printf("check_lifetime: ok (context before searches, leaked order, readback after an incumbent write)\n");
    return 0;
}
