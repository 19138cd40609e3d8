// The knob table behind tspgpu_tuning_set (tuning.h).
#include "tuning.h"

#include <cerrno>
#include <cmath>
#include <cstring>
#include <mutex>

#include "tspgpu.h"

namespace {

struct Knob {
    const char *name;
    bool set;
    double value;
};

// every knob the library reads (name, meaning at its one read site)
Knob g_knobs[] = {
    // K1 (tspgpu.cpp, read at context creation)
    {"K1", false, 0},              // force a variant (2, 4, 5, 6; 5 needs a K1_SWEEP build)
    {"TILED_CFG", false, 0},       // variant 5/6 configuration id (k1_cfg.h)
    {"WG_PER_CU", false, 0},       // workgroups per CU of the layer kernels
    {"THREADS", false, 0},         // threads per workgroup of the layer kernels
    {"LDS_TABLE_MAX_N", false, 0}, // largest N whose whole table lives in LDS
    // K1-wide (hkwide.hip)
    {"WIDE_PULL", false, 0},       // 1: per-destination layer form everywhere, 0: row-owner form
    // K2 (search_abi.cpp, read at search creation / run)
    {"SEARCH_KERNEL", false, 0},   // round kernel: 1 branching DFS, 2 lock-step DFS, 3 persistent
    {"SEARCH_HUNGRY", false, 0},
    {"SEARCH_MIN_SPLIT", false, 0},
    {"SEARCH_WALL_S", false, 0},
    {"SEARCH_RING_LOG2", false, 0},
    {"SEARCH_REFILL", false, 0},
    {"SEARCH_TAIL", false, 0},     // frontier tail length 5/6, 0: DFS rounds
    {"SEARCH_SUFFIX", false, 0},
    {"SEARCH_TWO_EDGE", false, 0},
    {"SEARCH_CHAIN", false, 0},    // 0: no chained search (step by step)
    {"SEARCH_LAGRANGE", false, 0},
    {"SEARCH_MST", false, 0},      // 0: no Held-Karp tree bound
    {"SEARCH_MST_MINREM", false, 0},
    {"SEARCH_TAIL_CAP_LOG2", false, 0},
    {"SEARCH_EXPAND_LOG2", false, 0},
    {"SEARCH_BUDGET", false, 0},
    {"SEARCH_TIE", false, 0},      // 0: no device tie rule (records only)
    {"SEARCH_PAGEABLE", false, 0}, // 1: pageable instead of pinned host words
    {"SEARCH_DEVICE_BOUND", false, 0},  // 0: search_solve below 20 cities takes the host heuristic's bound
    {"SEARCH_DEVICE_BOUND_MAXN", false, 0},  // search_solve takes the device bound from 13 cities up to below this (20)
    {"SEARCH_HEUR_ITERS", false, 0},         // device heuristic: 2-opt moves at most per start (default 8 n)
    {"SEARCH_TAILS", false, 0},
    {"SEARCH_CHAIN_CAP_LOG2", false, 0},  // chained level buffers (tests force the overflow rerun)
    {"SEARCH_CHAIN_POISON", false, 0},    // 1: fill the chain's level buffers with 0xFF first (tests)
    {"CHAIN_FPB", false, 0},
    {"CHAIN_GRID", false, 0},
    {"CHAIN_TAIL_GRID", false, 0},  // chained tail_kernel workgroups per CU
    {"CHAIN_FUSE_SEEDS", false, 0}, // 0: the chain's first level in its own launch (not in the seeds')
    {"CHAIN_LOCAL", false, 0},      // 0: a launch per chained level (no block-local levels)
    {"CHAIN_LOCAL_FPB", false, 0},
    {"SEARCH_DEBUG", false, 0},    // host phase times on stderr
    {"SEARCH_DEPTH", false, 0},
    {"SEARCH_RECORD_CAP", false, 0},  // tests: force the second phase
    {"ENUM_KERNEL", false, 0},     // 0: enumeration through the round kernels
    {"ENUM_WG_PER_CU", false, 0},
    // K3 (merge.hip)
    {"K3_PERSIST", false, 0},      // 0: per-merge fold launches instead of the persistent per-rank fold
    // host heuristics (search_host.cpp)
    {"HEURISTIC_THREADS", false, 0},
    {"HEURISTIC_ALL_STARTS", false, 0},
};
std::mutex g_mu;

Knob *find(const char *name)
{
    for (Knob &k : g_knobs)
        if (name && std::strcmp(k.name, name) == 0) return &k;
    return nullptr;
}

}  // namespace

namespace tspgpu {
bool tuned(const char *name, double *v)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const Knob *k = find(name);
    if (!k || !k->set) return false;
    if (v) *v = k->value;
    return true;
}
double tuned_or(const char *name, double dflt)
{
    double v;
    return tuned(name, &v) ? v : dflt;
}
}  // namespace tspgpu

extern "C" {
int tspgpu_tuning_set(const char *name, double value)
{
    if (!std::isfinite(value)) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    Knob *k = find(name);
    if (!k) return -ENOENT;
    k->set = true;
    k->value = value;
    return 0;
}
int tspgpu_tuning_clear(const char *name)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!name) {
        for (Knob &k : g_knobs) k.set = false;
        return 0;
    }
    Knob *k = find(name);
    if (!k) return -ENOENT;
    k->set = false;
    return 0;
}
}
