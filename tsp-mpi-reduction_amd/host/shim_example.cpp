// The reference's single-rank program flow (tsp.cpp:270-368 with P = 1),
// written against the drop-in C++ interface (include/assignment2_gpu.h)
// exactly as a maintainer of the reference would call it: distributeCities,
// tsp() per block (or tspBatch), the local fold with mergeBlocks.  Prints the
// reference's final line minus the timing.  Used by tests/test_shim_gpu.py.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "assignment2_gpu.h"

int procNum = 0;

int main(int argc, char **argv)
{
    if (argc < 5) {
        std::printf("usage: shim_example numCitiesPerBlock numBlocks gridDimX gridDimY [batch]\n");
        return 1;
    }
    const int n = std::atoi(argv[1]), B = std::atoi(argv[2]), X = std::atoi(argv[3]), Y = std::atoi(argv[4]);
    const bool batch = argc > 5 && std::atoi(argv[5]);
    std::srand(0);  // tsp.cpp:273
    std::vector<int> dims = getBlocksPerDim(B);
    std::vector<std::vector<City>> blocks = distributeCities(n, dims[0], dims[1], X, Y);
    std::vector<BlockSolution> sols;
    if (batch) {
        sols = tspBatch(blocks);
    } else {
        for (auto &b : blocks) sols.push_back(tsp(b));  // tsp.cpp:320
    }
    BlockSolution acc = sols[0];  // tsp.cpp:348-352
    for (size_t i = 1; i < sols.size(); ++i) acc = mergeBlocks(acc, sols[i]);
    std::printf("%lu cities and the trip cost %f\n", (unsigned long)acc.path.size(), acc.cost);
    return 0;
}
