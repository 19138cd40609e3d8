// Small transfers without the HIP runtime's copy path (round 5).
//
// The first hipMemcpy of a process costs ~8 ms (the runtime's blit set-up)
// and the first pageable copy above a few KB another ~8 ms, i.e. ~16 ms of a
// 16-city `./tsp 16 1` whose search takes 0.2 ms (profiles/r05/startup_probe.txt).
// Copies up to kXferSlotBytes go instead through a small pool of mapped,
// pinned host slots and one copy kernel of our own (its code object loads in
// ~0.3 ms); device-to-device copies and fills are that kernel too. Larger
// copies use hipMemcpyAsync / hipMemsetAsync as before.
//
// Semantics match the calls they replace: an H2D copy has read the host
// buffer when it returns (the bytes sit in a slot the stream's copy kernel
// reads; the slot is not reused before an event behind that kernel has
// fired); a D2H copy is complete when it returns (stream synchronised), so
// callers that synchronise afterwards lose nothing.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace tspgpu {

constexpr size_t kXferSlotBytes = (size_t)256 << 10;

hipError_t xcopy_async(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t st);
hipError_t xset_async(void *dst, int value, size_t bytes, hipStream_t st);

}  // namespace tspgpu
