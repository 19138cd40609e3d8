// C++ shim: the reference's assignment2.h entry points over libtspgpu and the
// host parity layer.  See include/assignment2_gpu.h.
#include "assignment2_gpu.h"

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "tsp_host.h"

int procNum __attribute__((weak)) = 0;

namespace {

tspgpu_ctx *shim_ctx()
{
    static tspgpu_ctx *ctx = nullptr;
    if (!ctx) {
        tspgpu_opts o;
        std::memset(&o, 0, sizeof o);
        const char *dev = std::getenv("TSP_GPU");
        o.device = dev ? std::atoi(dev) : -1;
        const int rc = tspgpu_ctx_create(&o, &ctx);
        if (rc) {
            std::fprintf(stderr, "tspgpu: cannot create a GPU context: %s\n", tspgpu_strerror(rc));
            std::exit(3);
        }
    }
    return ctx;
}

}  // namespace

std::vector<BlockSolution> tspBatch(const std::vector<std::vector<City>> &blocks)
{
    std::vector<BlockSolution> out;
    if (blocks.empty()) return out;
    const int n = (int)blocks[0].size();
    const int B = (int)blocks.size();
    std::vector<tspgpu_city> flat((size_t)B * n);
    for (int b = 0; b < B; ++b) {
        if ((int)blocks[b].size() != n) {
            std::fprintf(stderr, "tspBatch: blocks must have equal size\n");
            std::exit(3);
        }
        std::memcpy(&flat[(size_t)b * n], blocks[b].data(), sizeof(tspgpu_city) * n);
    }
    std::vector<double> cost(B);
    std::vector<int32_t> tour((size_t)B * (n + 1));
    const int rc = tspgpu_solve_cities(shim_ctx(), flat.data(), n, B, cost.data(), tour.data());
    if (rc) {
        std::fprintf(stderr, "tspgpu_solve_cities: %s\n", tspgpu_strerror(rc));
        std::exit(3);
    }
    const int L = tspgpu_tour_length(n);
    out.resize(B);
    for (int b = 0; b < B; ++b) {
        out[b].blockId = procNum;
        out[b].cost = cost[b];
        out[b].path.resize(L);
        for (int i = 0; i < L; ++i) out[b].path[i] = blocks[b][tour[(size_t)b * (n + 1) + i]];
    }
    return out;
}

BlockSolution tsp(std::vector<City> cities)
{
    std::vector<std::vector<City>> one(1, std::move(cities));
    return tspBatch(one)[0];
}

// mergeBlocks (tsp.cpp:202-269): K3 on the GPU once the swap search is big
// enough to pay for the launches (a growing fold), the host search for small
// pairs of paths; both give the reference's result bit for bit.
BlockSolution mergeBlocks(BlockSolution s1, BlockSolution s2)
{
    BlockSolution m;
    m.blockId = procNum;
    m.path.resize(s1.path.size() + s2.path.size() - 1);
    const auto *p1 = reinterpret_cast<const tspgpu_city *>(s1.path.data());
    const auto *p2 = reinterpret_cast<const tspgpu_city *>(s2.path.data());
    auto *out = reinterpret_cast<tspgpu_city *>(m.path.data());
    const int L1 = (int)s1.path.size(), L2 = (int)s2.path.size();
    int L;
    if ((long long)L1 * L2 >= (1 << 14)) {
        L = tspgpu_merge(shim_ctx(), p1, L1, s1.cost, p2, L2, s2.cost, out, &m.cost);
        if (L < 0 && L != -EDEADLK) {
            std::fprintf(stderr, "tspgpu_merge: %s\n", tspgpu_strerror(L));
            std::exit(3);
        }
    } else {
        L = tsphost_merge(p1, L1, s1.cost, p2, L2, s2.cost, out, &m.cost);
    }
    if (L < 0) {
        std::fprintf(stderr, "mergeBlocks: the reference would not terminate on these paths\n");
        std::exit(3);
    }
    m.path.resize(L);
    return m;
}

__attribute__((weak)) std::vector<int> getBlocksPerDim(int numBlocks)
{
    int r, c;
    tsphost_blocks_per_dim(numBlocks, &r, &c);
    return {r, c};
}

__attribute__((weak)) std::vector<std::vector<City>> distributeCities(int numCitiesPerBlock, int numBlocksInRow,
                                                                      int numBlocksInCol, int gridDimX, int gridDimY)
{
    const int B = numBlocksInRow * numBlocksInCol;
    std::vector<tspgpu_city> flat((size_t)B * numCitiesPerBlock);
    std::printf("%i blocks in X %i in Y\n", numBlocksInRow, numBlocksInCol);  // tsp.cpp:377
    tsphost_generate_grid(numCitiesPerBlock, numBlocksInRow, numBlocksInCol, gridDimX, gridDimY, flat.data());
    std::vector<std::vector<City>> blocks(B);
    for (int b = 0; b < B; ++b) {
        blocks[b].resize(numCitiesPerBlock);
        std::memcpy(blocks[b].data(), &flat[(size_t)b * numCitiesPerBlock], sizeof(City) * numCitiesPerBlock);
    }
    return blocks;
}
