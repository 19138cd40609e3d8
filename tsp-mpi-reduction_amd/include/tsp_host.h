/*
 * Host parity layer: the reference's CPU-side program logic around the block
 * search, re-implemented so the drop-in `tsp` binary prints exactly what the
 * reference prints for any logical rank count P.  No GPU code here; the block
 * search itself is libtspgpu (include/tspgpu.h).
 *
 *   generation     getBlocksPerDim tsp.cpp:136-157, distributeCities tsp.cpp:373-403, fRand assignment2.h:86-91
 *   distribution   distributeBlocks count formula tsp.cpp:167-192
 *   local fold     tsp.cpp:348-352
 *   merge          mergeBlocks tsp.cpp:197-269 (O(L1*L2) search, same first-strict-min pair)
 *   reduction      MPI_ManualReduce tsp.cpp:52-134, replayed for logical P,
 *                  including the receiver's growing `path` list (tsp.cpp:67,93-95,115-117)
 */
#ifndef TSP_HOST_H
#define TSP_HOST_H

#include <stdint.h>

#include "tspgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

void tsphost_blocks_per_dim(int nblocks, int *rows, int *cols);

/* srand(0) + distributeCities: nblocks*n cities, block-major. Returns rows*cols (== nblocks). */
int tsphost_generate(int n, int nblocks, int grid_x, int grid_y, tspgpu_city *out);

/* distributeCities itself for an explicit rows x cols grid: continues the
 * current rand() sequence (no reseed), like the reference. */
int tsphost_generate_grid(int n, int rows, int cols, int grid_x, int grid_y, tspgpu_city *out);

void tsphost_distribution_counts(int nblocks, int nprocs, int *counts);

/* mergeBlocks. out holds L1+L2-1 cities. Returns that length, or -1 when the
 * reference's rotation loop (tsp.cpp:236-239) would never terminate. */
int tsphost_merge(const tspgpu_city *p1, int L1, double c1, const tspgpu_city *p2, int L2, double c2,
                  tspgpu_city *out, double *cost_out);

/* Distribution + local fold + reduction tree for logical P, given every
 * block's solution (paths of L = tspgpu_tour_length(n) cities each,
 * block-major, in generation order).  Writes the final cost and the
 * "process %i is about to receive %i cities from process %i" lines
 * (tsp.cpp:88) into log.  Returns 0, -1 if the reference would not finish. */
int tsphost_reduce(const tspgpu_city *paths, int L, const double *costs, int nblocks, int nprocs,
                   double *final_cost, char *log, int logcap);

#ifdef __cplusplus
}
#endif
#endif
