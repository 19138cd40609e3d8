/*
 * ORACLE — CPU restatement of the reference's TSP block search and its host
 * pipeline, used ONLY as the checker by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  Nothing in the product (libtspgpu, the `tsp`
 * binary) links, loads or calls it.
 *
 * Pinned against the reference itself: tests/golden/ holds fixtures produced
 * by oracle/_ref (the unmodified reference compiled here, see oracle/Makefile
 * and tests/golden/make_golden.py); tests/test_oracle.py checks this oracle
 * against every one of them.
 */
#ifndef TSP_ORACLE_H
#define TSP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same memory layout as the reference's City (assignment2.h:13-18): 24 bytes. */
typedef struct
{
    int id;
    double x;
    double y;
} oracle_city;

/* computeDistanceMatrix, assignment2.h:184-200 (glibc pow/sqrt, not folded). */
void oracle_distance_matrix(const oracle_city *cities, int n, double *d);

/* tsp(), tsp.cpp:405-509, as an array Held-Karp with first-argmin backtracking.
 * d is n*n row-major. Writes the optimal cost and the local-index tour
 * (n+1 entries, or the 2-entry [1,0] quirk at n==2). Returns the tour length,
 * or -1 if n < 2. */
int oracle_solve_block(const double *d, int n, double *cost, int32_t *tour);

/* getBlocksPerDim, tsp.cpp:136-157. */
void oracle_blocks_per_dim(int B, int *rows, int *cols);

/* distributeCities, tsp.cpp:373-403 (srand(0) first, as main does at tsp.cpp:273).
 * Writes B*n cities, block-major. */
void oracle_generate(int n, int B, int X, int Y, oracle_city *out);

/* distributeBlocks' count formula, tsp.cpp:167-171. */
void oracle_distribution_counts(int B, int P, int *cnt);

/* mergeBlocks, tsp.cpp:197-269. out must hold L1+L2-1 cities. Returns that length. */
int oracle_merge_blocks(const oracle_city *p1, int L1, double c1, const oracle_city *p2, int L2, double c2,
                        oracle_city *out, double *cost);

/* Whole-program replay for logical rank count P (tsp.cpp:270-368 with
 * MPI_ManualReduce tsp.cpp:52-134): generate, solve every block with
 * oracle_solve_block, distribute, fold locally, reduce over the tree with the
 * stale `path` accumulator. Appends the "process %i is about to receive ..."
 * lines (tsp.cpp:88) to log (NUL-terminated, truncated at logcap).
 * Returns 0, or -1 when the reference would hang/crash (B < P, n < 2, B < 1). */
int oracle_pipeline(int n, int B, int X, int Y, int P, double *final_cost, char *log, int logcap);

#ifdef __cplusplus
}
#endif
#endif
