/* libtspcomm — RCCL communicator and in-stream incumbent exchange for the
 * one-process-per-GPU K2 driver (tsp-mpi-reduction_amd/search_dist.py).
 *
 * Replaces, for the one reduction the search needs (the global best tour:
 * tsp.cpp:483-499's closing min across shards), the reference's hand-rolled
 * MPI_Send/MPI_Recv binary tree MPI_ManualReduce (tsp.cpp:52-134).  Separate
 * from libtspgpu so that single-GPU programs never load RCCL.
 *
 * Bootstrap: rank 0 calls tspcomm_unique_id, the caller broadcasts the bytes
 * over its own process group (torch.distributed), every rank calls
 * tspcomm_create with its rank and device.  Errors: 0 or a negative errno. */
#ifndef TSPCOMM_H
#define TSPCOMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tspcomm tspcomm;

/* size of the unique id (ncclUniqueId, 128 bytes) */
int tspcomm_unique_id_bytes(void);
int tspcomm_unique_id(unsigned char *out, int cap);
int tspcomm_create(const unsigned char *id, int nranks, int rank, int device, tspcomm **out);
int tspcomm_destroy(tspcomm *c);

/* A tspgpu_level_hook (include/tspgpu.h, tspgpu_search_chain) with
 * user = the tspcomm*: enqueues ncclAllReduce(word, word, 1, ncclUint64,
 * ncclMin) on `stream` — the incumbent word exchanged between two frontier
 * levels inside the chain, no host round trip.  Counts its calls. */
void tspcomm_level_hook(void *user, void *stream, void *word);
/* hooks enqueued (and failed to enqueue) since the last reset */
int tspcomm_hook_stats(tspcomm *c, int *calls, int *errors, int reset);

/* words[0..count) <- all-reduce MIN over the ranks (count <= 8), through
 * device memory on `stream`; synchronous */
int tspcomm_allreduce_min_u64(tspcomm *c, uint64_t *words, int count, void *stream);

#ifdef __cplusplus
}
#endif
#endif
