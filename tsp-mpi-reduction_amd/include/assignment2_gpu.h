// Drop-in C++ interface for programs written against the reference's
// assignment2.h: the same data types and the same entry-point names, with the
// block search running on the MI355X through libtspgpu.
//
//   City, PathCost, BlockSolution      assignment2.h:13-31 (same layout)
//   BlockSolution tsp(vector<City>)    assignment2.h:56 / tsp.cpp:405-509
//   mergeBlocks                        assignment2.h:54 / tsp.cpp:202-269
//   distributeCities                   assignment2.h:58 / tsp.cpp:373-403
//   getBlocksPerDim                    tsp.cpp:136-157
// plus tspBatch(), which hands every block of a rank to the GPU in one call
// (the form the call sites at tsp.cpp:318-321 and 334-345 should migrate to).
#ifndef ASSIGNMENT2_GPU_H
#define ASSIGNMENT2_GPU_H

#include <vector>

#include "tspgpu.h"

// typedef'd anonymous structs exactly like the reference, so that the mangled
// names of tsp(vector<City>) and mergeBlocks(BlockSolution, BlockSolution)
// are the reference's own (the drop-in link of tsp.cpp relies on it)
typedef struct
{
    int id;
    double x;
    double y;
} City;

typedef struct
{
    double cost;
    std::vector<int> path;
} PathCost;

typedef struct
{
    int blockId;
    std::vector<City> path;
    double cost;
} BlockSolution;

static_assert(sizeof(City) == sizeof(tspgpu_city), "City must keep the reference's 24-byte layout");

// blockId of results, like the reference's global `procNum` (tsp.cpp:19,507).
// Weak so that a program that defines its own procNum (as tsp.cpp does) wins.
extern int procNum;

// The GPU versions of the reference's tsp() and mergeBlocks().  Strong
// symbols: linked together with the reference's tsp.cpp whose own two
// definitions were made weak (objcopy --weaken-symbol, oracle/Makefile
// _ref/tsp_dropin), these are the ones the reference's call sites reach.
// distributeCities and getBlocksPerDim are weak here: the reference's own
// definitions (tsp.cpp:136-157, 373-403) win when both are linked.
//
// One block on the GPU. Aborts with a message on a library error (the
// reference has no error channel; a silent CPU fallback is never taken).
BlockSolution tsp(std::vector<City> cities);

// All blocks in one GPU launch; same results as calling tsp() per block.
std::vector<BlockSolution> tspBatch(const std::vector<std::vector<City>> &blocks);

BlockSolution mergeBlocks(BlockSolution solution1, BlockSolution solution2);

std::vector<std::vector<City>> distributeCities(int numCitiesPerBlock, int numBlocksInRow, int numBlocksInCol,
                                                int gridDimX, int gridDimY);

std::vector<int> getBlocksPerDim(int numBlocks);

#endif
