// `tsp` — drop-in for the reference program (tsp.cpp:270-368):
//
//     ./tsp numCitiesPerBlock numBlocks gridDimX gridDimY
//
// Same arguments, same stdout (except the measured milliseconds).  Every block
// is solved exactly on the MI355X in one batched call (libtspgpu); the
// reference's distribution, local fold and reduction tree are replayed on the
// host for the LOGICAL rank count P, which fixes the printed answer:
//   P = PMI_SIZE / OMPI_COMM_WORLD_SIZE when started under mpirun, else
//       TSP_NPROCS, else 1.
// Under mpirun -np P (P > 1) every rank solves its own blocks, exactly the
// reference's share (cnt[r] contiguous blocks, tsp.cpp:167-192), on GPU
// r mod (visible devices) (TSP_GPU overrides), and hands its costs and tours
// to rank 0 through a file in a per-job directory (no MPI library is linked:
// TSP_GATHER_DIR, else /tmp/tspgpu-<uid>-<job key>); rank 0 waits for all of
// them, replays the reduction and prints.  One node only.  The job key hashes
// the launcher's job id (PMIX_NAMESPACE, OMPI_MCA_ess_base_jobid,
// SLURM_JOB_ID.SLURM_STEP_ID) or, under MPICH's hydra (which exports none),
// the parent process — the node's proxy, shared by its ranks — with its start
// time, plus the four arguments; every rank file carries it, so a file left by
// an earlier run is recognised as stale and ignored.  A worker that fails
// publishes a failure record, so rank 0 stops waiting at once.
// Without mpirun, physical GPUs (TSP_GPUS, default 1; device g mod visible
// devices for g < TSP_GPUS) only change speed: the blocks are split into
// contiguous ranges, one host thread per GPU.  The merges (local folds +
// reduction tree) run on the GPU too (K3, tspgpu_reduce); TSP_HOST_MERGE=1
// replays them on the host instead.
//
// TSP_STATS=1 adds one statistics line on stderr (phase times, relaxations/s).
//
// Deviations (documented in DESIGN.md), all where the reference is undefined:
// n < 2, numBlocks < 1 or numBlocks < P exit 2 with a message on stderr
// instead of crashing or hanging (tsp.cpp:326-330, 355).
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

// (P, this process's rank, launched by mpirun)
int logical_ranks(int *my_rank, bool *launched)
{
    *my_rank = env_int("PMI_RANK", env_int("OMPI_COMM_WORLD_RANK", 0));
    const int np = env_int("PMI_SIZE", env_int("OMPI_COMM_WORLD_SIZE", 0));
    *launched = np > 0;
    if (np > 0) return np;
    return env_int("TSP_NPROCS", 1);
}

int visible_devices()
{
    const int n = tspgpu_device_count();
    return n > 0 ? n : 1;
}

// Blocks [lo, lo + count) on `gpus` devices: contiguous ranges, one context +
// thread each; device (first_dev + g) mod visible devices.
// (keep: the context of device first_dev stays open and is returned, for the
// merges that follow on it — a second context costs a HIP stream and device
// queries; null: every context is destroyed)
int solve_range(const std::vector<tspgpu_city> &cities, int n, int lo, int count, int gpus, int first_dev,
                double *cost, int32_t *tour, tspgpu_ctx **keep = nullptr)
{
    const int B = count;
    if (B <= 0) return 0;
    if (gpus < 1) gpus = 1;
    if (gpus > B) gpus = B;
    const int ndev = visible_devices();
    std::vector<int> rcs(gpus, 0);
    std::vector<std::thread> th;
    for (int g = 0; g < gpus; ++g) {
        th.emplace_back([&, g] {
            const int a = (int)((long long)B * g / gpus), b = (int)((long long)B * (g + 1) / gpus);
            tspgpu_opts o;
            std::memset(&o, 0, sizeof o);
            o.device = (first_dev + g) % ndev;
            o.strict = 1;
            tspgpu_ctx *ctx = nullptr;
            int rc = tspgpu_ctx_create(&o, &ctx);
            if (!rc)
                rc = tspgpu_solve_cities(ctx, cities.data() + (size_t)(lo + a) * n, n, b - a, cost + a,
                                         tour + (size_t)a * (n + 1));
            if (ctx && g == 0 && keep && !rc)
                *keep = ctx;
            else if (ctx)
                tspgpu_ctx_destroy(ctx);
            rcs[g] = rc;
        });
    }
    for (auto &t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

// ---- rank-per-GPU mode: every rank's block results to rank 0 through files ----
struct RankFileHeader {
    uint32_t magic, rank, count, n;
    int32_t B, X, Y, status;  // status 0: results follow; < 0: the rank failed with this code
    uint64_t job;             // job key (job_key): equal in every rank of one run
};
constexpr uint32_t kMagic = 0x32505354;  // "TSP2"

uint64_t fnv1a(const std::string &s)
{
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

// Start time (clock ticks since boot) of process `pid`, 0 if unknown: with the
// pid it names one process, even after the pid is reused.
unsigned long long proc_start_ticks(int pid)
{
    char path[64], buf[1024];
    std::snprintf(path, sizeof path, "/proc/%d/stat", pid);
    FILE *f = std::fopen(path, "r");
    if (!f) return 0;
    const size_t len = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[len] = 0;
    const char *p = std::strrchr(buf, ')');  // the command name may contain spaces
    if (!p) return 0;
    unsigned long long v = 0;
    int field = 2;
    for (const char *q = p + 1; *q; ++q)
        if (*q == ' ' && ++field == 22) {
            v = std::strtoull(q + 1, nullptr, 10);
            break;
        }
    return v;
}

// One key per job and arguments, the same in every rank of that job.
uint64_t job_key(int n, int B, int X, int Y)
{
    std::string id;
    const char *slurm = std::getenv("SLURM_JOB_ID");
    if (const char *v = std::getenv("PMIX_NAMESPACE"))
        id = std::string("pmix:") + v;
    else if (const char *v2 = std::getenv("OMPI_MCA_ess_base_jobid"))
        id = std::string("ompi:") + v2;
    else if (slurm)
        id = std::string("slurm:") + slurm + "." + (std::getenv("SLURM_STEP_ID") ? std::getenv("SLURM_STEP_ID") : "");
    else
        id = "ppid:" + std::to_string((int)getppid()) + "@" + std::to_string(proc_start_ticks((int)getppid()));
    char args[96];
    std::snprintf(args, sizeof args, "|%d %d %d %d|%u", n, B, X, Y, (unsigned)getuid());
    return fnv1a(id + args);
}

std::string gather_dir(uint64_t key)
{
    if (const char *d = std::getenv("TSP_GATHER_DIR")) return d;
    char buf[256];
    std::snprintf(buf, sizeof buf, "/tmp/tspgpu-%u-%016llx", (unsigned)getuid(), (unsigned long long)key);
    return buf;
}

// status 0: this rank's results; status < 0: it failed (no payload)
int write_rank_file(const std::string &dir, uint64_t key, int rank, int n, int B, int X, int Y, int count,
                    const double *cost, const int32_t *tour, int status = 0)
{
    mkdir(dir.c_str(), 0700);  // may exist already
    const std::string tmp = dir + "/rank" + std::to_string(rank) + ".tmp";
    const std::string fin = dir + "/rank" + std::to_string(rank) + ".bin";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return -errno;
    RankFileHeader h{kMagic, (uint32_t)rank, (uint32_t)count, (uint32_t)n, B, X, Y, status, key};
    if (status) count = 0;
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1;
    ok = ok && (count == 0 || std::fwrite(cost, sizeof(double), (size_t)count, f) == (size_t)count);
    ok = ok && (count == 0 || std::fwrite(tour, sizeof(int32_t), (size_t)count * (n + 1), f) == (size_t)count * (n + 1));
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) return -EIO;
    return std::rename(tmp.c_str(), fin.c_str()) == 0 ? 0 : -errno;  // atomic publish
}

// Rank 0: wait (up to TSP_GATHER_TIMEOUT_S, default 600 s) for every other
// rank's file and place its blocks at their offsets.  A file of another job
// (key or arguments differ: left by an earlier run) is removed and waited past;
// a failure record of this job ends the wait with that rank's error.
int read_rank_files(const std::string &dir, uint64_t key, int P, int n, int B, int X, int Y,
                    const std::vector<int> &cnt, const std::vector<int> &off, double *cost, int32_t *tour,
                    int *failed_rank)
{
    const double limit = env_int("TSP_GATHER_TIMEOUT_S", 600);
    struct timespec t0, t;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 1; r < P; ++r) {
        const std::string fin = dir + "/rank" + std::to_string(r) + ".bin";
        for (;;) {
            FILE *f = std::fopen(fin.c_str(), "rb");
            if (!f) {
                clock_gettime(CLOCK_MONOTONIC, &t);
                if ((t.tv_sec - t0.tv_sec) + 1e-9 * (t.tv_nsec - t0.tv_nsec) > limit) return -ETIMEDOUT;
                usleep(1000);
                continue;
            }
            RankFileHeader h{};
            const bool hdr = std::fread(&h, sizeof h, 1, f) == 1 && h.magic == kMagic;
            if (!hdr || h.job != key || h.B != B || h.X != X || h.Y != Y || (int)h.n != n || (int)h.rank != r) {
                // stale (an earlier run's) or foreign: drop it, keep waiting for
                // this job's — but only if the path still names the file just
                // read: the worker may have rename()d its fresh file over it
                // meanwhile, and that one must not be deleted
                struct stat open_st {}, path_st {};
                const bool same = fstat(fileno(f), &open_st) == 0 && stat(fin.c_str(), &path_st) == 0 &&
                                  open_st.st_ino == path_st.st_ino && open_st.st_dev == path_st.st_dev;
                std::fclose(f);
                if (same) std::remove(fin.c_str());
                continue;
            }
            if (h.status != 0) {
                std::fclose(f);
                std::remove(fin.c_str());
                *failed_rank = r;
                return h.status;
            }
            bool ok = (int)h.count == cnt[r];
            ok = ok && (cnt[r] == 0 || std::fread(cost + off[r], sizeof(double), cnt[r], f) == (size_t)cnt[r]);
            ok = ok && (cnt[r] == 0 || std::fread(tour + (size_t)off[r] * (n + 1), sizeof(int32_t),
                                                  (size_t)cnt[r] * (n + 1), f) == (size_t)cnt[r] * (n + 1));
            std::fclose(f);
            std::remove(fin.c_str());
            if (!ok) return -EIO;
            break;
        }
    }
    if (!std::getenv("TSP_GATHER_DIR")) rmdir(dir.c_str());  // the per-job default directory
    return 0;
}

}  // namespace

int main(int argc, char **argv)
{
    struct timespec start, end;
    clock_gettime(CLOCK_MONOTONIC_RAW, &start);  // tsp.cpp:275-276, before any setup

    int my_rank = 0;
    bool launched = false;
    const int P = logical_ranks(&my_rank, &launched);
    const bool multi = launched && P > 1;  // one process per rank (mpirun)
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
    if (my_rank != 0 && !multi) return 0;
    const bool bad = n < 2 || B < 1 || B < P;
    if (my_rank != 0) {
        // a worker rank: solve this rank's share of the blocks and hand it to rank 0
        if (bad) return 0;  // rank 0 reports the error
        std::vector<tspgpu_city> cities((size_t)B * n);
        tsphost_generate(n, B, X, Y, cities.data());
        std::vector<int> cnt(P), off(P, 0);
        tsphost_distribution_counts(B, P, cnt.data());
        for (int r = 1; r < P; ++r) off[r] = off[r - 1] + cnt[r - 1];
        std::vector<double> cost(cnt[my_rank]);
        std::vector<int32_t> tour((size_t)cnt[my_rank] * (n + 1), -1);
        const int ndev = visible_devices();
        const int dev = env_int("TSP_GPU", my_rank % ndev);
        const uint64_t key = job_key(n, B, X, Y);
        const std::string dir = gather_dir(key);
        // TSP_INJECT_FAIL_RANK (fault injection for the tests): that rank fails
        int rc = env_int("TSP_INJECT_FAIL_RANK", -1) == my_rank
                     ? -EIO
                     : solve_range(cities, n, off[my_rank], cnt[my_rank], env_int("TSP_GPUS", 1), dev, cost.data(),
                                   tour.data());
        if (rc) {
            // tell rank 0 at once instead of leaving it waiting for this file
            (void)write_rank_file(dir, key, my_rank, n, B, X, Y, 0, nullptr, nullptr, rc);
        } else {
            rc = write_rank_file(dir, key, my_rank, n, B, X, Y, cnt[my_rank], cost.data(), tour.data());
        }
        if (rc) {
            std::fprintf(stderr, "tsp: rank %d failed: %s (%d)\n", my_rank, tspgpu_strerror(rc), rc);
            return 3;
        }
        return 0;
    }

    std::printf("We have %i cities for each of our %i blocks\n", n, B);  // tsp.cpp:307
    if (bad) {
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

    std::vector<double> cost(B, 0.0);
    std::vector<int32_t> tour((size_t)B * (n + 1), -1);
    int rc;
    timespec ts_solve0, ts_solve1, ts_merge1;
    tspgpu_ctx *kept = nullptr;  // the block search's context on TSP_GPU, reused by the merges
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts_solve0);
    // (the HIP runtime's own start-up, the analogue of the reference's
    // MPI_Init inside its clock: reported apart by TSP_STATS)
    timespec ts_rt;
    (void)tspgpu_device_count();
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts_rt);
    if (multi) {
        // rank 0's own share here, the other ranks' shares from their files
        std::vector<int> cnt(P), off(P, 0);
        tsphost_distribution_counts(B, P, cnt.data());
        for (int r = 1; r < P; ++r) off[r] = off[r - 1] + cnt[r - 1];
        const uint64_t key = job_key(n, B, X, Y);
        int failed = 0;
        rc = solve_range(cities, n, 0, cnt[0], env_int("TSP_GPUS", 1), env_int("TSP_GPU", 0), cost.data(), tour.data(),
                         &kept);
        if (!rc) rc = read_rank_files(gather_dir(key), key, P, n, B, X, Y, cnt, off, cost.data(), tour.data(), &failed);
        if (rc && failed) {
            std::fflush(stdout);
            std::fprintf(stderr, "tsp: rank %d failed: %s (%d)\n", failed, tspgpu_strerror(rc), rc);
            return 3;
        }
    } else {
        rc = solve_range(cities, n, 0, B, env_int("TSP_GPUS", 1), env_int("TSP_GPU", 0), cost.data(), tour.data(),
                         &kept);
    }
    if (rc) {
        std::fflush(stdout);
        std::fprintf(stderr, "tsp: GPU block search failed: %s (%d)\n", tspgpu_strerror(rc), rc);
        return 3;
    }

    clock_gettime(CLOCK_MONOTONIC_RAW, &ts_solve1);
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
        if (kept) tspgpu_ctx_destroy(kept);
        kept = nullptr;
        red = tsphost_reduce(paths.data(), L, cost.data(), B, P, &final_cost, log.data(), (int)log.size()) ? -EDEADLK
                                                                                                          : 0;
    } else {
        tspgpu_opts o;
        std::memset(&o, 0, sizeof o);
        o.device = env_int("TSP_GPU", 0);
        red = kept ? 0 : tspgpu_ctx_create(&o, &kept);
        if (!red) red = tspgpu_reduce(kept, paths.data(), L, cost.data(), B, P, &final_cost, log.data(), (int)log.size());
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
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts_merge1);

    clock_gettime(CLOCK_MONOTONIC_RAW, &end);
    const uint64_t ms = (uint64_t)((1000000000L * (end.tv_sec - start.tv_sec) + end.tv_nsec - start.tv_nsec) / 1e6);
    std::printf("TSP ran in %llu ms for %lu cities and the trip cost %f\n", (unsigned long long)ms,
                (unsigned long)(unsigned int)(B * n), final_cost);
    // the device context is torn down after the clock, like the reference's
    // MPI_Finalize after its end time (tsp.cpp:358-366)
    std::fflush(stdout);
    if (kept) tspgpu_ctx_destroy(kept);
    kept = nullptr;
    // opt-in statistics on stderr (SURVEY.md §5 "Metrics": stdout stays the
    // reference's byte for byte): phase times and the block search's rate
    if (env_int("TSP_STATS", 0)) {
        auto sec = [](const timespec &a, const timespec &b) {
            return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
        };
        const double solve_s = sec(ts_solve0, ts_solve1);
        const double relax = tspgpu_relaxations_per_block(n) * (multi ? 0.0 : (double)B);
        std::fprintf(stderr,
                     "tsp stats: n %d blocks %d ranks %d | setup %.3f ms, block search %.3f ms (HIP runtime start-up "
                     "%.3f ms of it; %s), merge %.3f ms, total %.3f ms | %.4g DP relaxations/s\n",
                     n, B, P, 1e3 * sec(start, ts_solve0), 1e3 * solve_s, 1e3 * sec(ts_solve0, ts_rt),
                     multi ? "rank 0's share + the rank files" : "all blocks, one process",
                     1e3 * sec(ts_solve1, ts_merge1), 1e3 * sec(start, end),
                     solve_s > 0 && relax > 0 ? relax / solve_s : 0.0);
    }
    return 0;
}
