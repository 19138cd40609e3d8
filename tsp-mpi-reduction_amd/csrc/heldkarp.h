// Internal launch interface of the K1 Held-Karp kernels (heldkarp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tspgpu {

constexpr int kMaxN = 19;         // inner cities (n <= 20)
constexpr int kLdsTableMaxN = 11; // whole table in LDS: 11 * 2^10 * 8 B = 88 KiB
constexpr int kBinomRows = 21;
constexpr int kBinomCols = 24;

// Per-N constants, resident in device memory (uploaded once per context).
struct LayerInfo {
    int binom[kBinomRows * kBinomCols];  // C(a, b)
    int off[24];                         // doubles offset of layer t (off[N+1] = table size)
    int count[24];                       // C(N, t) rows in layer t
    int moff[24];                        // offset of layer t in the colex mask list
};

struct LaunchArgs {
    const double *dist;     // nblocks * n * n (device)
    int n;
    int nblocks;
    double *slots;          // grid * slot_doubles (device), unused when use_lds
    size_t slot_doubles;
    const uint32_t *masks;  // all N-bit masks sorted by (popcount, value)
    const LayerInfo *info;  // device copy
    double *cost;
    int32_t *tour;
    bool use_lds;
    int threads;            // 256 / 512 / 1024 threads per workgroup (global-table kernels)
    hipStream_t stream;
};

void host_layer_info(int N, LayerInfo *info);
size_t table_doubles(int N);
hipError_t launch_heldkarp(const LaunchArgs &a, int grid);
size_t lds_bytes_for(int N, bool lds_table, int threads);
int threads_for(int N, bool lds_table, int requested);

}  // namespace tspgpu
