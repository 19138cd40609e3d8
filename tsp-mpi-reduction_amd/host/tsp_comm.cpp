// libtspcomm: the RCCL side of the one-process-per-GPU K2 driver
// (search_dist.py), kept out of libtspgpu so that single-GPU users never load
// RCCL.  Exported (include/tspcomm.h):
//   * a communicator over the ranks of a torch.distributed group, bootstrapped
//     from an ncclUniqueId that rank 0 creates and the group broadcasts;
//   * tspcomm_level_hook: a tspgpu_level_hook (include/tspgpu.h) that enqueues
//     an in-place ncclAllReduce(MIN, uint64) of the search's incumbent word ON
//     THE SEARCH'S STREAM between two frontier levels — the periodic incumbent
//     exchange of north_star / SURVEY.md §8(e), with no host round trip;
//   * a device all-reduce MIN of a few u64 words (the final winner's key).
// This replaces, for the one reduction the search needs, the reference's
// blocking MPI_Send/MPI_Recv tree (tsp.cpp:52-134).
#include "tspcomm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cerrno>
#include <cstring>
#include <new>

struct tspcomm {
    ncclComm_t comm = nullptr;
    int device = 0;
    int rank = 0, nranks = 1;
    int calls = 0;   // hooks enqueued since the last tspcomm_hook_stats(reset)
    int errors = 0;  // hooks whose ncclAllReduce did not enqueue
    unsigned long long *scratch = nullptr;  // tspcomm_allreduce_min's device words
};

extern "C" {

int tspcomm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int tspcomm_unique_id(unsigned char *out, int cap)
{
    if (!out || cap < (int)sizeof(ncclUniqueId)) return -EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -EIO;
    std::memcpy(out, &id, sizeof id);
    return 0;
}

int tspcomm_create(const unsigned char *id, int nranks, int rank, int device, tspcomm **out)
{
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    auto *c = new (std::nothrow) tspcomm();
    if (!c) return -ENOMEM;
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    if (ncclCommInitRank(&c->comm, nranks, uid, rank) != ncclSuccess) {
        delete c;
        return -EIO;
    }
    if (hipMalloc((void **)&c->scratch, 8 * sizeof(unsigned long long)) != hipSuccess) {
        ncclCommDestroy(c->comm);
        delete c;
        return -ENOMEM;
    }
    *out = c;
    return 0;
}

int tspcomm_destroy(tspcomm *c)
{
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->comm) ncclCommDestroy(c->comm);
    delete c;
    return 0;
}

void tspcomm_level_hook(void *user, void *stream, void *word)
{
    auto *c = static_cast<tspcomm *>(user);
    ++c->calls;
    if (ncclAllReduce(word, word, 1, ncclUint64, ncclMin, c->comm, (hipStream_t)stream) != ncclSuccess) ++c->errors;
}

int tspcomm_hook_stats(tspcomm *c, int *calls, int *errors, int reset)
{
    if (!c) return -EINVAL;
    if (calls) *calls = c->calls;
    if (errors) *errors = c->errors;
    if (reset) c->calls = c->errors = 0;
    return 0;
}

int tspcomm_allreduce_min_u64(tspcomm *c, uint64_t *words, int count, void *stream)
{
    if (!c || !words || count < 1 || count > 8) return -EINVAL;
    (void)hipSetDevice(c->device);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(c->scratch, words, count * sizeof(uint64_t), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return -EIO;
    if (ncclAllReduce(c->scratch, c->scratch, count, ncclUint64, ncclMin, c->comm, st) != ncclSuccess) return -EIO;
    e = hipMemcpyAsync(words, c->scratch, count * sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e == hipSuccess ? 0 : -EIO;
}

}  // extern "C"
