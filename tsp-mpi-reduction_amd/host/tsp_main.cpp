// `tsp` — drop-in for the reference program (tsp.cpp:270-368):
//
//     ./tsp numCitiesPerBlock numBlocks gridDimX gridDimY
//
// Same arguments, same stdout (except the measured milliseconds).  Every block
// is solved exactly on the MI355X in one batched call (libtspgpu); the
// reference's distribution, local fold and reduction tree are replayed on the
// host for the LOGICAL rank count P, which fixes the printed answer:
//   P = PMI_SIZE / OMPI_COMM_WORLD_SIZE when started under mpirun (only rank 0
//       prints and solves; other ranks exit 0), else TSP_NPROCS, else 1.
// Physical GPUs (TSP_GPUS, default 1; devices 0..TSP_GPUS-1) only change speed:
// the blocks are split into contiguous ranges, one host thread per GPU.  The
// merges (local folds + reduction tree) run on the GPU too (K3, tspgpu_reduce);
// TSP_HOST_MERGE=1 replays them on the host instead.
//
// Deviations (documented in DESIGN.md), all where the reference is undefined:
// n < 2, numBlocks < 1 or numBlocks < P exit 2 with a message on stderr
// instead of crashing or hanging (tsp.cpp:326-330, 355).
#include <time.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "tsp_host.h"
#include "tspgpu.h"

namespace {

int env_int(const char *name, int dflt)
{
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

int logical_ranks(int *my_rank)
{
    *my_rank = env_int("PMI_RANK", env_int("OMPI_COMM_WORLD_RANK", 0));
    const int launched = env_int("PMI_SIZE", env_int("OMPI_COMM_WORLD_SIZE", 0));
    if (launched > 0) return launched;
    return env_int("TSP_NPROCS", 1);
}

// All blocks on `gpus` devices: contiguous ranges, one context + thread each.
int solve_all(const std::vector<tspgpu_city> &cities, int n, int B, int gpus, std::vector<double> &cost,
              std::vector<int32_t> &tour)
{
    cost.assign(B, 0.0);
    tour.assign((size_t)B * (n + 1), -1);
    if (gpus < 1) gpus = 1;
    if (gpus > B) gpus = B;
    std::vector<int> rcs(gpus, 0);
    std::vector<std::thread> th;
    for (int g = 0; g < gpus; ++g) {
        th.emplace_back([&, g] {
            const int lo = (int)((long long)B * g / gpus), hi = (int)((long long)B * (g + 1) / gpus);
            tspgpu_opts o;
            std::memset(&o, 0, sizeof o);
            o.device = gpus == 1 ? env_int("TSP_GPU", 0) : g;
            o.strict = 1;
            tspgpu_ctx *ctx = nullptr;
            int rc = tspgpu_ctx_create(&o, &ctx);
            if (!rc)
                rc = tspgpu_solve_cities(ctx, cities.data() + (size_t)lo * n, n, hi - lo, cost.data() + lo,
                                         tour.data() + (size_t)lo * (n + 1));
            if (ctx) tspgpu_ctx_destroy(ctx);
            rcs[g] = rc;
        });
    }
    for (auto &t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

}  // namespace

int main(int argc, char **argv)
{
    struct timespec start, end;
    clock_gettime(CLOCK_MONOTONIC_RAW, &start);  // tsp.cpp:275-276, before any setup

    int my_rank = 0;
    const int P = logical_ranks(&my_rank);
    if (argc != 5) {
        // every rank prints the usage (tsp.cpp:280-284)
        const int copies = my_rank == 0 && !std::getenv("PMI_SIZE") && !std::getenv("OMPI_COMM_WORLD_SIZE") ? P : 1;
        for (int i = 0; i < copies; ++i) std::printf("Usage:  ./tsp numCitiesPerBlock numBlocks gridDimX gridDimY\n");
        return 1;
    }
    const int n = std::atoi(argv[1]);
    const int B = std::atoi(argv[2]);
    const int X = std::atoi(argv[3]);
    const int Y = std::atoi(argv[4]);
    if (n > TSPGPU_REFERENCE_MAX_CITIES) {
        if (my_rank == 0)
            std::printf("Come on... We don't want to wait forever so lets just have you retry that with less than "
                        "16 cities per block...\n");
        return 1337;  // exit(1337): status 57 (tsp.cpp:294)
    }
    if (my_rank != 0) return 0;  // under mpirun, rank 0 does the whole job

    std::printf("We have %i cities for each of our %i blocks\n", n, B);  // tsp.cpp:307
    if (n < 2 || B < 1 || B < P) {
        std::fflush(stdout);
        std::fprintf(stderr, "tsp: needs numCitiesPerBlock >= 2 and numBlocks >= max(1, ranks=%d); the reference "
                             "crashes or hangs here\n", P);
        return 2;
    }
    int R, C;
    tsphost_blocks_per_dim(B, &R, &C);
    std::printf("%i blocks in X %i in Y\n", R, C);  // tsp.cpp:377
    std::vector<tspgpu_city> cities((size_t)B * n);
    tsphost_generate(n, B, X, Y, cities.data());

    std::vector<double> cost;
    std::vector<int32_t> tour;
    const int rc = solve_all(cities, n, B, env_int("TSP_GPUS", 1), cost, tour);
    if (rc) {
        std::fflush(stdout);
        std::fprintf(stderr, "tsp: GPU block search failed: %s (%d)\n", tspgpu_strerror(rc), rc);
        return 3;
    }

    // convPathToCityPath (assignment2.h:76-84) for every block
    const int L = tspgpu_tour_length(n);
    std::vector<tspgpu_city> paths((size_t)B * L);
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < L; ++i) paths[(size_t)b * L + i] = cities[(size_t)b * n + tour[(size_t)b * (n + 1) + i]];

    // the fold + reduction tree: K3 on the GPU (default), or the host replay
    // (TSP_HOST_MERGE=1); both reproduce the reference's mergeBlocks exactly
    double final_cost = 0.0;
    std::vector<char> log(1 << 20);
    int red = 0;
    if (env_int("TSP_HOST_MERGE", 0)) {
        red = tsphost_reduce(paths.data(), L, cost.data(), B, P, &final_cost, log.data(), (int)log.size()) ? -EDEADLK
                                                                                                          : 0;
    } else {
        tspgpu_opts o;
        std::memset(&o, 0, sizeof o);
        o.device = env_int("TSP_GPU", 0);
        tspgpu_ctx *ctx = nullptr;
        red = tspgpu_ctx_create(&o, &ctx);
        if (!red) red = tspgpu_reduce(ctx, paths.data(), L, cost.data(), B, P, &final_cost, log.data(), (int)log.size());
        if (ctx) tspgpu_ctx_destroy(ctx);
    }
    if (red) {
        std::fflush(stdout);
        if (red == -EDEADLK)
            std::fprintf(stderr, "tsp: the reference's merge would not terminate for these blocks\n");
        else
            std::fprintf(stderr, "tsp: GPU merge failed: %s (%d)\n", tspgpu_strerror(red), red);
        return 2;
    }
    std::fputs(log.data(), stdout);

    clock_gettime(CLOCK_MONOTONIC_RAW, &end);
    const uint64_t ms = (uint64_t)((1000000000L * (end.tv_sec - start.tv_sec) + end.tv_nsec - start.tv_nsec) / 1e6);
    std::printf("TSP ran in %llu ms for %lu cities and the trip cost %f\n", (unsigned long long)ms,
                (unsigned long)(unsigned int)(B * n), final_cost);
    return 0;
}
