/*
 * tspgpu — MI355X (gfx950) exact TSP block search behind a C ABI.
 *
 * Drop-in for the reference's per-block solver
 *     BlockSolution tsp(vector<City> cities)        (assignment2.h:56, tsp.cpp:405-509)
 * and its helper computeDistanceMatrix               (assignment2.h:184-200).
 * Results are bit-identical to the reference: the same FP64 optimal cost and
 * the same tour (the reference's first-strict-minimum tie rule, tsp.cpp:457-470,
 * 484-498).  Plain C types only; no HIP or torch types cross this boundary
 * (HIP streams are passed as void*).  See INTEGRATION.md for the C++/ctypes
 * bindings a maintainer of the reference would add.
 *
 * Return codes: 0 on success, otherwise a negative errno value
 *   -EINVAL  bad argument (n outside [2, TSPGPU_MAX_CITIES] (strict: 16), nblocks < 0,
 *            NULL pointer, non-finite or negative distance)
 *   -ERANGE  n * max(d) >= INT_MAX: the reference's INT_MAX sentinel
 *            (tsp.cpp:411,453) would leave its tour undefined
 *   -ENODEV  no HIP device / device ordinal out of range
 *   -ENOMEM  device allocation failed
 *   -EIO     a HIP runtime call or kernel launch failed
 *   -EDEADLK (K3) the reference's mergeBlocks would never terminate for these paths
 *            (its rotation loop, tsp.cpp:236-239, looks for a city that is not there)
 *   -EOVERFLOW (K2) more optimal tours than can be enumerated, n > 31
 */
#ifndef TSPGPU_H
#define TSPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSPGPU_VERSION 100          /* 1.0.0 */
#define TSPGPU_MAX_CITIES 20        /* extension limit (N = n-1 <= 19) */
#define TSPGPU_REFERENCE_MAX_CITIES 16 /* tsp.cpp:289 rejects more */

/* Memory layout identical to the reference's City (assignment2.h:13-18):
 * int id at offset 0, double x at 8, double y at 16; 24 bytes. */
typedef struct
{
    int32_t id;
    double x;
    double y;
} tspgpu_city;

typedef struct
{
    int device;      /* HIP device ordinal; -1 = the calling thread's current device */
    int strict;      /* 1: accept n <= 16 only (the reference's cap, tsp.cpp:289) */
    int slots;       /* resident DP workspaces (persistent grid size); 0 = auto */
    int reserved[5]; /* must be zero */
} tspgpu_opts;

typedef struct tspgpu_ctx tspgpu_ctx;

int tspgpu_version(void);
const char *tspgpu_strerror(int code);

/* Length of the tour written per block: n+1 (0, t1..tN, 0), except the
 * reference's n==2 quirk [1,0] (tsp.cpp:483-502 with one inner city). */
int tspgpu_tour_length(int n);

/* computeDistanceMatrix (assignment2.h:184-200) on the host with glibc pow/sqrt,
 * bit-exact with the reference.  dist: nblocks*n*n row-major. */
int tspgpu_distance_matrix(const tspgpu_city *cities, int n, int nblocks, double *dist);

/* Host-side validation applied by the host-pointer entry points. */
int tspgpu_validate(const double *dist, int n, int nblocks, int strict);

int tspgpu_ctx_create(const tspgpu_opts *opts, tspgpu_ctx **out);
/* Destroy order is free: every tspgpu_search holds a reference on its
 * context, so destroying the context while searches are alive only marks it
 * closing (no new search may be created on it: -EINVAL) and the last
 * tspgpu_search_destroy releases it.  Searches never destroyed keep their
 * context (a leak, never a use-after-free). */
int tspgpu_ctx_destroy(tspgpu_ctx *ctx);

/* Batched replacement for tsp() on host buffers; synchronous.
 *   dist     nblocks*n*n doubles (host), from tspgpu_distance_matrix
 *   cost_out nblocks doubles: the block's tour cost (BlockSolution.cost)
 *   tour_out nblocks*(n+1) int32: local city indices of BlockSolution.path
 *            (tspgpu_tour_length(n) valid entries; the rest is -1) */
int tspgpu_solve_blocks(tspgpu_ctx *ctx, const double *dist, int n, int nblocks, double *cost_out,
                        int32_t *tour_out);

/* Same, from cities (distance matrix computed on the host, then solved). */
int tspgpu_solve_cities(tspgpu_ctx *ctx, const tspgpu_city *cities, int n, int nblocks, double *cost_out,
                        int32_t *tour_out);

/* Device-pointer form, asynchronous on `hip_stream` (hipStream_t, NULL = default).
 * The caller guarantees the data satisfy tspgpu_validate (not re-checked).
 * d_dist/d_cost/d_tour are device pointers on the context's device.
 * Calls on one context may use different streams: they share the context's
 * DP workspace, so a launch on a stream other than the previous launch's
 * waits (hipStreamWaitEvent) for that launch first; use one context per
 * stream for concurrent batches. */
int tspgpu_solve_blocks_device(tspgpu_ctx *ctx, const double *d_dist, int n, int nblocks, double *d_cost,
                               int32_t *d_tour, void *hip_stream);

/* Integer-weight extension (TSPLIB-style rounded distances; no reference
 * counterpart — the reference computes f64 Euclidean distances only): the same
 * DP, tie rule and tour layout on int32 distances.  Results equal
 * tspgpu_solve_blocks on the same matrix converted to double (every partial
 * sum is an exact integer below 2^31); the table and its HBM traffic are half
 * the size.  Validation: d >= 0 and n * max(d) < INT_MAX (else -ERANGE). */
int tspgpu_validate_i32(const int32_t *dist, int n, int nblocks, int strict);
int tspgpu_solve_blocks_i32(tspgpu_ctx *ctx, const int32_t *dist, int n, int nblocks, int32_t *cost_out,
                            int32_t *tour_out);
int tspgpu_solve_blocks_i32_device(tspgpu_ctx *ctx, const int32_t *d_dist, int n, int nblocks, int32_t *d_cost,
                                   int32_t *d_tour, void *hip_stream);

/* Context-free convenience form (uses a per-thread default context on the
 * current device, created on first use). */
int tspgpu_solve(const double *dist, int n, int nblocks, double *cost_out, int32_t *tour_out,
                 const tspgpu_opts *opts);

/* Device memory, stream and timing helpers for callers that have no HIP
 * runtime of their own (ctypes / cgo / JNI users, bench.py): everything on the
 * context's device; copies are synchronous; the timer is a pair of HIP events
 * recorded on the context's stream (the stream the kernels run on when
 * hip_stream == tspgpu_stream(ctx)). */
int tspgpu_device_alloc(tspgpu_ctx *ctx, size_t bytes, void **ptr);
int tspgpu_device_free(tspgpu_ctx *ctx, void *ptr);
int tspgpu_memcpy_htod(tspgpu_ctx *ctx, void *dst, const void *src, size_t bytes);
int tspgpu_memcpy_dtoh(tspgpu_ctx *ctx, void *dst, const void *src, size_t bytes);
void *tspgpu_stream(tspgpu_ctx *ctx);
/* Extra non-blocking streams on the context's device (for callers without a
 * HIP runtime of their own), and a host wait on any stream. */
int tspgpu_stream_create(tspgpu_ctx *ctx, void **stream);
int tspgpu_stream_destroy(tspgpu_ctx *ctx, void *stream);
int tspgpu_stream_synchronize(tspgpu_ctx *ctx, void *stream);
int tspgpu_synchronize(tspgpu_ctx *ctx);
int tspgpu_timer_start(tspgpu_ctx *ctx);
int tspgpu_timer_stop(tspgpu_ctx *ctx, float *elapsed_ms);
/* CU count and device name of the context's device. */
int tspgpu_device_info(const tspgpu_ctx *ctx, int *cu_count, char *name, int namecap);

/* Device-side information for measurement: number of persistent workgroups
 * the last launch used and the DP relaxations per block for n cities,
 * N(N-1)2^(N-2) with N = n-1 (tsp.cpp:442-471). */
int tspgpu_last_grid(const tspgpu_ctx *ctx);
/* K1 variant the last batched launch used: 6 = sub-cube restructured
 * (hk_sub_kernel), 5 = sub-cube tiled (hk_tiled_kernel), 4 = ping-pong +
 * parent words, 2 = compact + prefetch, ... (heldkarp_kernel). */
int tspgpu_last_variant(const tspgpu_ctx *ctx);
/* Measurement aid for variants 5 and 6, which run two kernels per chunk of at
 * most 16384 blocks (the forward pass, then hk_tiled_backtrack): with split
 * timing enabled every chunk also records HIP events before, between and
 * after the two kernels, on the launch's stream.  tspgpu_k1_last_split_ms
 * waits for the last of them and returns both kernels' durations SUMMED over
 * every chunk of every launch since the previous read (or since enabling),
 * then starts a new sum: -ENOENT if nothing was recorded, -ENOSPC if more
 * than 4096 chunks were (recording stopped).  Enabling resets the sum. */
int tspgpu_k1_split_timing(tspgpu_ctx *ctx, int enable);
int tspgpu_k1_last_split_ms(tspgpu_ctx *ctx, float *forward_ms, float *backtrack_ms);
/* Number of visible HIP devices (0 when none). */
int tspgpu_device_count(void);
double tspgpu_relaxations_per_block(int n);
/* Algorithmic table bytes per block: every DP entry written once and read
 * once, 2 * 8 * N * 2^(N-1). */
double tspgpu_table_bytes_per_block(int n);

/* ---------------------------------------------------------------------------
 * K1-wide: ONE instance's Held-Karp with every CU of the GPU on each layer
 * (K1 gives each block one workgroup).  The single-instance time to the
 * optimal tour, and exact instances up to n = 31 (table N*2^(N-1) doubles:
 * 129 GB at n = 31).  Same cost and tour bits as K1 / tsp().  dist: n*n f64
 * (host); tour_out: n+1 entries; kernel_ms (optional): device time.
 * ------------------------------------------------------------------------- */
#define TSPGPU_WIDE_MAX_CITIES 31
int tspgpu_solve_instance(tspgpu_ctx *ctx, const double *dist, int n, double *cost_out, int32_t *tour_out,
                          double *kernel_ms);

/* ---------------------------------------------------------------------------
 * K2: exact search of ONE instance, prefix-parallel branch and bound over the
 * whole GPU (one instance per call instead of one block per workgroup), the
 * north_star's search shape for the reference's per-block problem
 * (tsp.cpp:405-509).  Same answer as tsp()/K1: the optimal left-fold cost and
 * the DP's tie-broken tour (see tspgpu_select_tour), for n <= 32 cities.
 * Distances: f64 (the reference's computeDistanceMatrix output) or i32 (the
 * integer-matrix extension: d >= 0, n * max(d) < 2^30).
 * ------------------------------------------------------------------------- */
#define TSPGPU_SEARCH_MAX_CITIES 32
#define TSPGPU_F64 0
#define TSPGPU_I32 1

/* One recorded complete tour: cost (IEEE bits of the f64 cost, or the
 * integer cost) and the inner cities t1..tN (N = n-1) in visiting order. */
typedef struct
{
    uint64_t cost;
    uint8_t city[32];
} tspgpu_tour_record;

typedef struct
{
    uint64_t nodes;         /* search nodes: child extensions cost + d[last][next] with their bound test */
    uint64_t records;       /* complete tours recorded at cost <= incumbent (last phase) */
    uint64_t optimal_tours; /* |O|: tours whose cost equals the optimum */
    uint64_t items;         /* prefixes (work items) N!/(N-D)! */
    int depth;              /* prefix depth D */
    int phases;             /* 1, or 2 when the record buffer overflowed (second search, bound = optimum) */
    int fallback;           /* 1: |O| too large to enumerate, the answer came from K1-wide (n <= 31) */
    int rounds;             /* search rounds of the last phase (items split and re-queued between rounds) */
    double kernel_ms;       /* device time of the search launches */
    uint64_t lane_steps;    /* lane slots of the search loop (64 per wave step) */
    uint64_t active_steps;  /* ... of which a lane worked on an item (lane utilisation = active/lane) */
    uint64_t item_loads;    /* items loaded by lanes (seeds and hand-backs) */
    int tie;                /* 1: the tour is the device tie rule's (tspgpu_tie_tour certified it) */
    int tie_checked;        /* 1: the records were also read and their host rule gave the same tour */
} tspgpu_search_stats;

/* Device tie rule (K2): the kernels keep, per recorded cost, the least
 * reverse-lexicographic key (t_N most significant) of the tours offered at
 * that cost; digit p = rank of t_(N-p) among the cities not placed yet, radix
 * N-p, in w0 for N <= 20, else digits 0..12 in w0 and the rest in w1.  This
 * decodes the key of the optimum's slot into tour_out (n+1 entries) and
 * certifies it as tsp()'s tour (tsp.cpp:457-470, 484-499): its fold must equal
 * cost_bits and, for f64, no fold one ulp below any of its prefixes may round
 * to the same next prefix (then every prefix fold is minimal and the DP's
 * backward argmin chain picks exactly this tour).  0: certified; -EAGAIN:
 * valid but not certified (use the records); -EINVAL: not a tour of that cost. */
int tspgpu_tie_tour(const void *dist, int dtype, int n, uint64_t w0, uint64_t w1, uint64_t cost_bits,
                    int32_t *tour_out);
/* The same certificate with the prefix DPs it may need run on the context's
 * GPU (K1-wide over the prefix's cities, up to 26; the host DP stops at 16),
 * so binade crossings late in long tours are proven too. */
int tspgpu_tie_tour_gpu(tspgpu_ctx *ctx, const void *dist, int dtype, int n, uint64_t w0, uint64_t w1,
                        uint64_t cost_bits, int32_t *tour_out);
/* tspgpu_tie_tour with the certificate's prefix minima taken from the
 * search's optimal records instead of a Held-Karp DP: records[0..count) must
 * be EVERY tour the search recorded (tspgpu_search_records with no overflow,
 * all shards), so that they hold the whole optimal set O; a prefix the records
 * cannot decide falls back to the DP on ctx's GPU (ctx may be NULL: then not
 * certified, -EAGAIN). */
int tspgpu_tie_tour_records(tspgpu_ctx *ctx, const void *dist, int dtype, int n, uint64_t w0, uint64_t w1,
                            uint64_t cost_bits, const tspgpu_tour_record *records, int count, int32_t *tour_out);
/* the key of a tour (tour[0] = 0, tour[1..n-1] = t1..tN): test helper */
int tspgpu_tie_key(int n, const int32_t *tour, uint64_t *w0, uint64_t *w1);

typedef struct tspgpu_search tspgpu_search; /* one instance (or one shard of it) on one context */

/* One-shot: whole instance on the context's GPU.  cost_out: the optimal cost
 * (an integer value for TSPGPU_I32); tour_out: n+1 entries 0,t1..tN,0.
 * When more tours tie for the optimum than can be enumerated (coincident
 * cities), n <= 31 is answered by K1-wide (stats->fallback = 1), larger n
 * return -EOVERFLOW. */
int tspgpu_search_solve(tspgpu_ctx *ctx, const void *dist, int dtype, int n, double *cost_out,
                        int32_t *tour_out, tspgpu_search_stats *stats);

/* Exhaustive enumeration (BASELINE config 2: "14-city exhaustive enumeration
 * on 1 MI355X"): the same search with the bound switched off — every one of
 * the (n-1)! tours is folded (the left fold of tsp.cpp), the tours within the
 * incumbent are recorded and the DP's tie rule picks among the optimal ones,
 * so the result equals tspgpu_search_solve / tsp().  stats->nodes counts every
 * partial path (about e*(n-1)!).  Practical up to ~15 cities. */
int tspgpu_search_enumerate(tspgpu_ctx *ctx, const void *dist, int dtype, int n, double *cost_out,
                            int32_t *tour_out, tspgpu_search_stats *stats);

/* Sharded form for multi-GPU drivers (one process or thread per GPU): shard s
 * of S seeds the depth-D prefixes p with p mod S == s (static interleave).
 * Inside the GPU the work runs in rounds: lanes take items from a device
 * queue, and an item that exceeds its iteration budget is split into the
 * untried siblings of each level of its stack, re-queued for the next round.
 * A driver calls start, then step until pending == 0, exchanging the
 * incumbent word between steps (e.g. RCCL all-reduce MIN of the u64 read with
 * tspgpu_search_counters, written back with tspgpu_search_set_bound); at the
 * end it all-reduces the incumbent, gathers the records whose cost equals it
 * from every shard and calls tspgpu_select_tour.  depth 0 = automatic. */
int tspgpu_search_create(tspgpu_ctx *ctx, const void *dist, int dtype, int n, int shard, int nshards, int depth,
                         tspgpu_search **out);
/* tspgpu_search_create with flags.  TSPGPU_SEARCH_DEVICE_BOUND: the create
 * launch also computes the initial incumbent on the device (nearest neighbour
 * from spread start cities + 2-opt, the cheaper left fold of either
 * direction; every shard of an instance gets the same bound), so a driver
 * needs no host heuristic and no tspgpu_search_set_bound before the search. */
#define TSPGPU_SEARCH_DEVICE_BOUND 1
int tspgpu_search_create_ex(tspgpu_ctx *ctx, const void *dist, int dtype, int n, int shard, int nshards, int depth,
                            int flags, tspgpu_search **out);
int tspgpu_search_destroy(tspgpu_search *s);
int tspgpu_search_info(const tspgpu_search *s, int *depth, uint64_t *items, uint64_t *local_items);
/* initial incumbent (a real tour's cost, e.g. tspgpu_heuristic_tour) */
int tspgpu_search_set_bound(tspgpu_search *s, double bound);
/* seed this shard's live prefixes (synchronous) */
int tspgpu_search_start(tspgpu_search *s);
/* one round over the pending items (synchronous); *pending = items left for the next round */
int tspgpu_search_step(tspgpu_search *s, uint64_t *pending);
/* start + steps until nothing is pending */
int tspgpu_search_run_all(tspgpu_search *s);
/* device time of all seed/round launches so far, and the rounds run */
int tspgpu_search_timing(const tspgpu_search *s, double *kernel_ms, int *rounds);
/* device address of the 64-bit incumbent word (f64 bits or integer cost).
 * The caller may write it (an RCCL all-reduce MIN in place): from this call
 * on tspgpu_search_counters / tspgpu_search_tie_slot read the device, not the
 * last chain's readback. */
void *tspgpu_search_incumbent_device(tspgpu_search *s);
int tspgpu_search_counters(tspgpu_search *s, uint64_t *incumbent_bits, uint64_t *nodes, uint64_t *records);
/* forget the records (and grow the buffer to `capacity` if larger) */
int tspgpu_search_reset_records(tspgpu_search *s, unsigned int capacity);
/* the recorded tours whose cost bits equal cost_bits; -EOVERFLOW if records
 * were lost (rerun with the optimum as the bound), -ENOSPC if cap is short */
int tspgpu_search_records(tspgpu_search *s, uint64_t cost_bits, tspgpu_tour_record *out, int cap, int *count);

/* Chained run of this shard (any shard count): the seeds,
 * every frontier level and the tail fold enqueued back to back on the
 * context's stream, ONE synchronisation, and the counters, this shard's tie
 * slot at its incumbent and its first records read back with it.  Between
 * levels, every `exchange_every` levels (0: never), hook(user, stream,
 * incumbent word) is called to enqueue an exchange of the device incumbent on
 * that stream — e.g. ncclAllReduce(word, word, 1, ncclUint64, ncclMin, comm,
 * stream): the same number of calls on every shard, chained or not.
 * *done = 1: the shard's search is complete.  *done = 0: the search is not
 * a chain — too large (a level overflowed, or n is above the chain's limit;
 * it is back at its starting state: incumbent restored, no records) or too
 * small to have a frontier level (below ~15 cities the seed depth, one prefix
 * per lane of the grid, already reaches the register tails: e.g. 13 cities,
 * seed depth 7 >= 12 - 6) — continue with tspgpu_search_start /
 * tspgpu_search_step.  The hooks are enqueued either way (same count). */
typedef void (*tspgpu_level_hook)(void *user, void *stream, void *incumbent_word);
int tspgpu_search_chain(tspgpu_search *s, int exchange_every, tspgpu_level_hook hook, void *user, int *done);

/* The device tie rule's least key among the tours this shard recorded at
 * cost cost_bits (tspgpu_tie_tour's w0/w1).  A driver of S shards takes the
 * all-reduce MIN of the incumbents (the optimum), then the MIN of w0 over the
 * shards (~0 where !found), then of w1 over the holders of that w0, and
 * certifies the winner once with tspgpu_tie_tour — the DP's tour without
 * gathering any record; overflow != 0 on any shard: the
 * records decide instead (tspgpu_search_records, tspgpu_select_tour). */
typedef struct
{
    uint64_t w0, w1; /* the key (w1 = 0 when n - 1 <= 20) */
    int found;       /* 1: a recorded tour of this shard has that cost */
    int overflow;    /* 1: the tie table lost an offer, the key may not be least */
} tspgpu_tie_slot;
int tspgpu_search_tie_slot(tspgpu_search *s, uint64_t cost_bits, tspgpu_tie_slot *out);

/* Host helpers.  A nearest-neighbour + 2-opt tour and its left-fold cost (an
 * upper bound); and the DP's tie rule applied to the optimal set O: walking
 * from the last city backwards, take the smallest m that ends a tour of O with
 * the chosen suffix and whose best prefix fold + d[m][next] equals the state
 * value (tsp.cpp:457-470, 483-499) — the tour tsp() returns. */
int tspgpu_heuristic_tour(const void *dist, int dtype, int n, double *cost_out, int32_t *tour_out);
/* the same over the start cities first, first + step, ... < n only (-ENOENT
 * when first >= n): R ranks taking first = r, step = R and the MIN of their
 * costs get the bound of all starts, each doing 1/R of the work */
int tspgpu_heuristic_tour_starts(const void *dist, int dtype, int n, int first, int step, double *cost_out,
                                 int32_t *tour_out);
int tspgpu_select_tour(const void *dist, int dtype, int n, const tspgpu_tour_record *records, int count,
                       uint64_t cost_bits, int32_t *tour_out);

/* ---------------------------------------------------------------------------
 * K3: the reference's mergeBlocks (tsp.cpp:197-269) and its reduction tree
 * (MPI_ManualReduce tsp.cpp:52-134 + the local fold tsp.cpp:348-352) with the
 * paths on the GPU.  Same result as the reference bit for bit: the L1 x L2
 * swap search runs on the device, near-minimal candidates are re-evaluated
 * on the host with glibc pow (assignment2.h:141-144), the splice is a device
 * gather.  Cities are the reference's City structs, paths include the
 * closing city like BlockSolution.path.
 * ------------------------------------------------------------------------- */
/* mergeBlocks(p1, p2): out (L1+L2-1 cities), *cost_out = c1 + c2 + best swap.
 * Returns the merged length, or a negative code. */
int tspgpu_merge(tspgpu_ctx *ctx, const tspgpu_city *p1, int L1, double c1, const tspgpu_city *p2, int L2, double c2,
                 tspgpu_city *out, double *cost_out);
/* The distribution counts, every logical rank's left fold and the reduction
 * tree for logical rank count nprocs, given each block's solution (paths of
 * L cities, block-major).  Writes the final cost and the "process %i is about
 * to receive %i cities from process %i" lines (tsp.cpp:88) into log. */
int tspgpu_reduce(tspgpu_ctx *ctx, const tspgpu_city *paths, int L, const double *costs, int nblocks, int nprocs,
                  double *final_cost, char *log, int logcap);

/* ---------------------------------------------------------------------------
 * Tuning and test knobs.  The defaults are the measured best; a knob changes
 * how the kernels run (K1 variant / configuration, buffer sizes, a bound
 * switched off for an A/B run, a fallback forced by a test), never the
 * answer.  Process-wide, read where each is used (K1 knobs at context
 * creation, K2 knobs at search creation).  The library reads no environment
 * variable of its own: the documented TSP_* variables belong to bin/tsp.
 * Names: K1, TILED_CFG, WG_PER_CU, THREADS, LDS_TABLE_MAX_N, WIDE_PULL,
 * SEARCH_{KERNEL, HUNGRY, MIN_SPLIT, WALL_S, RING_LOG2, REFILL, TAIL, SUFFIX,
 * TWO_EDGE, CHAIN, LAGRANGE, MST, MST_MINREM, TAIL_CAP_LOG2, EXPAND_LOG2,
 * BUDGET, TIE, PAGEABLE, TAILS, CHAIN_CAP_LOG2, CHAIN_POISON, DEBUG, DEPTH,
 * RECORD_CAP}, CHAIN_FPB, CHAIN_GRID, ENUM_KERNEL, ENUM_WG_PER_CU,
 * HEURISTIC_THREADS, HEURISTIC_ALL_STARTS (csrc/tuning.cpp).
 * ------------------------------------------------------------------------- */
/* 0, -ENOENT (no such knob) or -EINVAL (not finite) */
int tspgpu_tuning_set(const char *name, double value);
/* back to the default (name NULL: every knob) */
int tspgpu_tuning_clear(const char *name);

#ifdef __cplusplus
}
#endif
#endif
