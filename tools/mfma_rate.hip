// Microbenchmark: issue rate of v_mfma_f64_16x16x4_f64 (1..8 independent
// accumulators, 1..4 waves per SIMD) and of v_fma_f64 on the VALU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) (void)(x)
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void __launch_bounds__(256) k_rate(double *out, int iters) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_fma(double *out, int iters) {
    double x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3 + i;
    const double a = 0.999999, b = 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = fma(x[i], a, b);
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NACC>
void run(double *d, int iters, int wps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = 256 * wps;
    hipLaunchKernelGGL(k_rate<NACC>, dim3(grid), dim3(256), 0, 0, d, 10);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate<NACC>, dim3(grid), dim3(256), 0, 0, d, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double per_simd = (double)iters * NACC * wps;
    double flops = 1024.0 * per_simd * 2048;
    printf("mfma NACC=%d waves/SIMD=%d: %.3f ms, %.1f TF/s, %.0f cyc per MFMA per SIMD @2.4GHz\n", NACC, wps, ms,
           flops / ms / 1e9, ms * 1e6 / per_simd * 2.4);
}
void run_fma(double *d, int iters, int wps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = 256 * wps;
    hipLaunchKernelGGL(k_fma, dim3(grid), dim3(256), 0, 0, d, 10);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_fma, dim3(grid), dim3(256), 0, 0, d, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double per_simd = (double)iters * 16 * wps;
    double flops = 1024.0 * per_simd * 64 * 2;
    printf("v_fma_f64 waves/SIMD=%d: %.3f ms, %.1f TF/s, %.1f cyc per wave-FMA per SIMD\n", wps, ms,
           flops / ms / 1e9, ms * 1e6 / per_simd * 2.4);
}
int main() {
    double *d; CK(hipMalloc(&d, 1024 * 256 * 8));
    run<1>(d, 20000, 1); run<2>(d, 10000, 1); run<4>(d, 5000, 1); run<8>(d, 2500, 1);
    run<2>(d, 5000, 2); run<4>(d, 2500, 2); run<4>(d, 1250, 4);
    run_fma(d, 20000, 1); run_fma(d, 10000, 2); run_fma(d, 5000, 4);
    return 0;
}
