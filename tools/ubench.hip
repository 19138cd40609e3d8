// Micro-benchmarks for the roofline peaks the bench line is priced against
// (gfx950, one MI355X): issue rates of the VALU instructions the Held-Karp
// relaxation is made of, and a byte-count calibration of the rocprofv3
// FETCH_SIZE / WRITE_SIZE counters for 8-byte-per-lane loads and stores (the
// access width of the K1 table), once from a buffer far larger than the
// Infinity Cache and once from one that fits it.
//
//   ubench valu            -> one line per instruction mix: lane-ops/s
//   ubench mem <MiB> <reps> -> streams <MiB> once per rep (8-B loads + 8-B stores)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int ITERS = 2048;
constexpr int CHAINS = 8;

// MODE 0 v_add_f64, 1 v_min_f64, 2 v_cmp_lt_f64 + v_cndmask_b32, 3 v_add_u32,
// 4 v_min_i32, 5 the f64 relaxation with argmin (add, cmp, cndmask, min),
// 6 the i32 relaxation with argmin, 7 v_cndmask_b32 alone, 8 the f64
// relaxation without argmin (add, min: K1 variant 5's passes below the top rows),
// 9 the i32 relaxation without argmin
template <int MODE>
__global__ __launch_bounds__(256) void valu_kernel(double *out, double seed)
{
    double a[CHAINS], b = seed * 1e-3;
    int ia[CHAINS], ib = (int)threadIdx.x;
    unsigned arg[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        a[c] = seed + c + threadIdx.x;
        ia[c] = c + threadIdx.x;
        arg[c] = c;
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (MODE == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (MODE == 1) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (MODE == 2)
                asm volatile("v_cmp_lt_f64 vcc, %1, %2\n\tv_cndmask_b32 %0, %0, %3, vcc"
                             : "+v"(arg[c])
                             : "v"(a[c]), "v"(b), "v"(it)
                             : "vcc");
            if constexpr (MODE == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ia[c]) : "v"(ib));
            if constexpr (MODE == 4) asm volatile("v_min_i32 %0, %0, %1" : "+v"(ia[c]) : "v"(ib));
            if constexpr (MODE == 5) {
                double t;
                asm volatile(
                    "v_add_f64 %1, %2, %3\n\t"
                    "v_cmp_lt_f64 vcc, %1, %0\n\t"
                    "v_cndmask_b32 %4, %4, %5, vcc\n\t"
                    "v_min_f64 %0, %0, %1"
                    : "+v"(a[c]), "=&v"(t)
                    : "v"(b), "v"(a[(c + 1) % CHAINS]), "v"(arg[c]), "v"(it)
                    : "vcc");
                arg[c] = arg[c];
            }
            if constexpr (MODE == 6) {
                int t;
                asm volatile(
                    "v_add_u32 %1, %2, %3\n\t"
                    "v_cmp_lt_i32 vcc, %1, %0\n\t"
                    "v_cndmask_b32 %4, %4, %5, vcc\n\t"
                    "v_min_i32 %0, %0, %1"
                    : "+v"(ia[c]), "=&v"(t)
                    : "v"(ib), "v"(ia[(c + 1) % CHAINS]), "v"(arg[c]), "v"(it)
                    : "vcc");
            }
            if constexpr (MODE == 7)
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(arg[c]) : "v"(it) : "vcc");
            if constexpr (MODE == 8) {
                double t;
                asm volatile("v_add_f64 %1, %2, %3\n\tv_min_f64 %0, %0, %1"
                             : "+v"(a[c]), "=&v"(t)
                             : "v"(b), "v"(a[(c + 1) % CHAINS]));
            }
            if constexpr (MODE == 9) {
                int t;
                asm volatile("v_add_u32 %1, %2, %3\n\tv_min_i32 %0, %0, %1"
                             : "+v"(ia[c]), "=&v"(t)
                             : "v"(ib), "v"(ia[(c + 1) % CHAINS]));
            }
        }
    }
    double s = 0;
    for (int c = 0; c < CHAINS; ++c) s += a[c] + ia[c] + arg[c];
    if (s == 12345.678) out[0] = s;  // keeps the chains alive
}

template <int MODE>
static void run_valu(const char *name, int insts_per_op, hipDeviceProp_t &p)
{
    double *out;
    CHECK(hipMalloc(&out, 64));
    const int blocks = p.multiProcessorCount * 8, threads = 256;  // 8 waves per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(valu_kernel<MODE>, dim3(blocks), dim3(threads), 0, 0, out, 1.0);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(valu_kernel<MODE>, dim3(blocks), dim3(threads), 0, 0, out, 1.0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double ops = (double)blocks * threads * ITERS * CHAINS;  // lane-ops (one per chain step)
    const double insts = ops * insts_per_op;
    printf("{\"mix\": \"%s\", \"ms\": %.4f, \"lane_ops_per_s\": %.4e, \"lane_insts_per_s\": %.4e, "
           "\"cycles_per_wave_inst_at_2.4GHz\": %.3f}\n",
           name, best, ops / (best * 1e-3), insts / (best * 1e-3),
           (double)p.multiProcessorCount * 4 * 2.4e9 / (insts / 64.0 / (best * 1e-3)));
    CHECK(hipFree(out));
}

__global__ __launch_bounds__(256) void stream_kernel(const double *__restrict__ src, double *__restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i] + 1.0;
}

int main(int argc, char **argv)
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    if (argc >= 2 && !strcmp(argv[1], "valu")) {
        printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount,
               p.clockRate);
        run_valu<0>("v_add_f64", 1, p);
        run_valu<1>("v_min_f64", 1, p);
        run_valu<2>("v_cmp_lt_f64+v_cndmask_b32", 2, p);
        run_valu<3>("v_add_u32", 1, p);
        run_valu<4>("v_min_i32", 1, p);
        run_valu<7>("v_cndmask_b32", 1, p);
        run_valu<5>("f64 relaxation+argmin (add,cmp,cndmask,min)", 4, p);
        run_valu<8>("f64 relaxation min-only (add,min)", 2, p);
        run_valu<6>("i32 relaxation+argmin (add,cmp,cndmask,min)", 4, p);
        run_valu<9>("i32 relaxation min-only (add,min)", 2, p);
        return 0;
    }
    if (argc >= 4 && !strcmp(argv[1], "mem")) {
        const size_t mib = strtoull(argv[2], 0, 10);
        const int reps = atoi(argv[3]);
        const size_t n = mib * 1024 * 1024 / 8;
        double *a, *b;
        CHECK(hipMalloc(&a, n * 8));
        CHECK(hipMalloc(&b, n * 8));
        CHECK(hipMemset(a, 0, n * 8));
        CHECK(hipMemset(b, 0, n * 8));
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(stream_kernel, dim3(p.multiProcessorCount * 8), dim3(256), 0, 0, a, b, n);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"mem_mib\": %zu, \"rep\": %d, \"ms\": %.4f, \"read_bytes\": %zu, \"write_bytes\": %zu, "
                   "\"GBps_rw\": %.1f}\n",
                   mib, r, ms, n * 8, n * 8, 2.0 * n * 8 / (ms * 1e-3) / 1e9);
        }
        return 0;
    }
    fprintf(stderr, "usage: ubench valu | ubench mem <MiB> <reps>\n");
    return 1;
}
