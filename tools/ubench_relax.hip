// Relaxation instruction-form micro-benchmark (gfx950): how many SIMD cycles
// one DP relaxation (cand = g + d; first strict argmin; running minimum) costs
// in each candidate instruction form, with Q = 8 independent destinations per
// "row" (as in the K1 layer pass) and a given number of waves per SIMD.
//   ubench_relax <waves_per_simd>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int ITERS = 1024;
constexpr int Q = 8;

template <int MODE>
__device__ __forceinline__ void relax(double &acc, unsigned &arg, double g, double d, unsigned m)
{
    double t;
    if constexpr (MODE == 0)  // add, cmp(vcc), cndmask arg, min
        asm volatile(
            "v_add_f64 %[t], %[g], %[d]\n\tv_cmp_lt_f64 vcc, %[t], %[acc]\n\t"
            "v_cndmask_b32 %[arg], %[arg], %[m], vcc\n\tv_min_f64 %[acc], %[acc], %[t]"
            : [acc] "+v"(acc), [arg] "+v"(arg), [t] "=&v"(t)
            : [g] "v"(g), [d] "v"(d), [m] "v"(m)
            : "vcc");
    if constexpr (MODE == 2)  // add, min: no argmin (lower bound)
        asm volatile("v_add_f64 %[t], %[g], %[d]\n\tv_min_f64 %[acc], %[acc], %[t]"
                     : [acc] "+v"(acc), [t] "=&v"(t)
                     : [g] "v"(g), [d] "v"(d));
    if constexpr (MODE == 3)  // add, cmp -> SGPR pair chosen by the compiler, cndmask, min
    {
        t = g + d;
        arg = t < acc ? m : arg;
        acc = __builtin_fmin(acc, t);
    }
}

template <int MODE>
__global__ void relax_kernel(double *out, const double *dd, unsigned seed)
{
    __shared__ double dl[512];
    for (int i = threadIdx.x; i < 512; i += blockDim.x) dl[i] = dd[i];
    __syncthreads();
    double acc[Q];
    unsigned arg[Q];
    for (int q = 0; q < Q; ++q) {
        acc[q] = 1e30;
        arg[q] = 0;
    }
    unsigned lane = threadIdx.x & 63;
    unsigned a = (lane * 7 + seed) & 255;
    for (int it = 0; it < ITERS; ++it) {
        const double g = dl[(a + it) & 511];
        // d values: one LDS gather per relaxation, like the kernel
        double dv[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) dv[q] = dl[(a * 3 + q * 17 + it) & 511];
#pragma unroll
        for (int q = 0; q < Q; ++q) relax<MODE>(acc[q], arg[q], g, dv[q], (unsigned)it);
    }
    double s = 0;
    for (int q = 0; q < Q; ++q) s += acc[q] + arg[q];
    if (s == 1.2345) out[0] = s;
}

template <int MODE>
void run(const char *name, int waves, hipDeviceProp_t &p, double *out, double *dd)
{
    // waves per SIMD via workgroups of 256 threads (1 wave per SIMD each) and a
    // dynamic LDS reservation that admits exactly `waves` of them per CU
    const int lds = 160 * 1024 / waves - 4096 - 64;
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(&relax_kernel<MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int blocks = p.multiProcessorCount * waves * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(relax_kernel<MODE>, dim3(blocks), dim3(256), lds, 0, out, dd, 1u);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(relax_kernel<MODE>, dim3(blocks), dim3(256), lds, 0, out, dd, 1u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double relax = (double)blocks * 256 * ITERS * Q;
    const double simd_cycles = (double)p.multiProcessorCount * 4 * 2.4e9 * best * 1e-3;
    printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"relax_per_s\": %.4e, "
           "\"simd_cycles_per_wave_relax_at_2.4GHz\": %.2f}\n",
           name, waves, best, relax / (best * 1e-3), simd_cycles / (relax / 64));
}

int main(int argc, char **argv)
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    double *out, *dd;
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMalloc(&dd, 512 * 8));
    double h[512];
    for (int i = 0; i < 512; ++i) h[i] = 1.0 + (i * 37 % 101);
    CHECK(hipMemcpy(dd, h, sizeof h, hipMemcpyHostToDevice));
    for (int w : {1, 2, 3, 4, 8}) {
        run<0>("add,cmp,cndmask,min", w, p, out, dd);
        run<2>("add,min (no argmin)", w, p, out, dd);
        run<3>("compiler (cmp to SGPR pairs)", w, p, out, dd);
    }
    return 0;
}
