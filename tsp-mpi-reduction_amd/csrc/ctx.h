// Internal definition of the opaque tspgpu_ctx (include/tspgpu.h): one HIP
// device, one stream, the K1 tables/workspaces and the K2 search state cache.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "heldkarp.h"
#include "tspgpu.h"

struct tspgpu_ctx {
    // (members are used by tspgpu.cpp for K1 and search_abi.cpp for K2)
    int device = 0;
    int strict = 0;
    int slots_opt = 0;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    uint32_t *d_masks[tspgpu::kMaxN + 1] = {};
    tspgpu::LayerInfo *d_info[tspgpu::kMaxN + 1] = {};
    double *d_slots = nullptr;
    size_t slots_bytes = 0;
    double *d_dist = nullptr;
    size_t dist_bytes = 0;
    double *d_cost = nullptr;
    size_t cost_bytes = 0;
    int32_t *d_tour = nullptr;
    size_t tour_bytes = 0;
    int last_grid = 0;
    int last_variant = -1;
    int threads = 0;     // workgroup size of the global-table kernels; 0 = per-N default
    int wg_per_cu = 0;   // resident slots per CU (auto grid); 0 = per-N default
    int lds_table_max_n = tspgpu::kLdsTableDefaultMaxN;  // largest N whose whole table stays in LDS
    int variant = -1;    // K1 layer pass (-1: per-n default): 6 = sub-cube, restructured (hk_sub.h),
                         // 5 = sub-cube tiled (hk_tiled.h),
                         // 4 = 2 + ping-pong values + parent words,
                         // 2 = compact + next-row prefetch, 1 = compact, 0 = member sweep
    int tiled_cfg = -1;  // K1 variant 5/6 configuration id (k1_cfg.h); -1 = per-(n, type) default
    void *d_tinfo[16] = {};        // TiledInfo per L (variants 5, 6)
    void *d_subrows[16] = {};      // SubRow table per L (variant 6)
    char *d_tslots = nullptr;      // variant 5/6 slots (one per block of a launch)
    size_t tslots_bytes = 0;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    // K1 workspace ordering across caller streams: the slots / push areas are
    // per context, so a launch on a stream other than the previous one waits
    // for the previous launch (event recorded after every K1 launch)
    hipEvent_t ev_k1_done = nullptr;
    // variant-5/6 split timing (tspgpu_k1_split_timing): per chunk launched
    // since the last read, three events (before the forward kernel, between
    // it and the backtracking kernel, after that); read and reset by
    // tspgpu_k1_last_split_ms
    int split_timing = 0;
    std::vector<hipEvent_t> ev_split;
    size_t split_used = 0;
    bool split_overflow = false;
    hipStream_t k1_last_stream = nullptr;
    bool k1_launched = false;
    char name[256] = {0};
    std::mutex mu;
    // K1-wide per-context cache (buffers + captured launch graph of the last n), hkwide.hip
    void *wide_cache = nullptr;
    void (*wide_free)(void *) = nullptr;
    // K2 device buffers kept between searches (search_abi.cpp); null while a
    // live search holds them
    void *search_pool = nullptr;
    void (*search_pool_free)(void *) = nullptr;
    // Lifetime: every tspgpu_search holds a reference on its context (it uses
    // the stream, the device, the mutex and the pool).  tspgpu_ctx_destroy
    // with searches still alive only marks the context closing; the last
    // tspgpu_search_destroy then releases it.  Both under mu.
    int live_searches = 0;
    bool closing = false;
};

// frees every resource of c and c itself (no live search may remain)
void tspgpu_ctx_release(tspgpu_ctx *c);
