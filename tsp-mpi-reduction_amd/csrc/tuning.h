// Tuning / test knobs of libtspgpu (include/tspgpu.h "Tuning"): a fixed table
// of named values that change HOW the kernels run — variant and configuration
// choice, buffer sizes, bounds switched off for A/B runs, forced fallbacks for
// the tests — never what they compute.  Set only through the C ABI
// (tspgpu_tuning_set); the library reads no environment variable of its own.
// Host-only (no HIP), so the ASan build links it too.
#pragma once

namespace tspgpu {
// true and *v when `name` has been set (tspgpu_tuning_set); false otherwise
bool tuned(const char *name, double *v);
// the value, or dflt when unset
double tuned_or(const char *name, double dflt);
inline int tuned_int(const char *name, int dflt) { return (int)tuned_or(name, (double)dflt); }
}  // namespace tspgpu
