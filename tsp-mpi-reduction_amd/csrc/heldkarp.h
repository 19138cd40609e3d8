// Internal launch interface of the K1 Held-Karp kernels (heldkarp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tspgpu {

constexpr int kMaxN = 19;         // inner cities (n <= 20)
constexpr int kLdsTableMaxN = 11; // LDS-table kernels exist up to N = 11 (88 KiB)
constexpr int kLdsTableDefaultMaxN = 9; // used by default up to N = 9 (18 KiB): beyond, more blocks in flight win
constexpr int kBinomRows = 21;
constexpr int kBinomCols = 24;
// colex-rank lookup (compact kernels): rank(mask) = R1[mask & 127]
//   + R2[(mask >> 7) & 127][popcount(mask & 127)] + R3[mask >> 14][popcount(mask & 0x3fff)]
constexpr int kRankR1 = 128, kRankR2 = 128 * 8, kRankR3 = 64 * 15;
constexpr int kRankLutInts = kRankR1 + kRankR2 + kRankR3;

// Per-N constants, resident in device memory (uploaded once per context).
struct LayerInfo {
    int binom[kBinomRows * kBinomCols];  // C(a, b)
    int off[24];                         // doubles offset of layer t (off[N+1] = table size)
    int count[24];                       // C(N, t) rows in layer t
    int moff[24];                        // offset of layer t in the colex mask list
    int rlut[kRankLutInts];              // colex-rank lookup (R1 | R2 | R3), see above
};

struct LaunchArgs {
    const void *dist;       // nblocks * n * n (device), f64 or i32 (vbytes)
    int n;
    int nblocks;
    void *slots;            // grid * slot_doubles values (device), unused when use_lds
    size_t slot_doubles;    // table values per slot
    const uint32_t *masks;  // all N-bit masks sorted by (popcount, value)
    const LayerInfo *info;  // device copy
    void *cost;             // nblocks values (f64 or i32)
    int32_t *tour;
    int vbytes;             // 8: f64 distances, 4: i32 distances
    bool use_lds;
    int threads;            // 256 / 512 / 1024 threads per workgroup (global-table kernels)
    int variant;            // layer pass: 0 = member sweep over all N cities, 1 = compact (non-members only),
                            // 2 = compact with the next row prefetched
    hipStream_t stream;
};

void host_layer_info(int N, LayerInfo *info);
size_t table_doubles(int N);
hipError_t launch_heldkarp(const LaunchArgs &a, int grid);
size_t lds_bytes_for(int N, bool lds_table, int threads, bool compact, int vbytes = 8);
int threads_for(int N, bool lds_table, int requested);

}  // namespace tspgpu
