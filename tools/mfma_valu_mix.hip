// Microbenchmark: can v_fma_f64 on the VALU run beside v_mfma_f64_16x16x4_f64
// on the matrix core of the same SIMD?  Per loop iteration each wave issues
// NM MFMAs (independent accumulators) and NV wave-wide v_fma_f64 (independent
// chains); total fp64 flop rate over every CU.  Operands are non-trivial
// (lane-dependent, not zero) so the clock is the loaded one.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NM, int NV>
__global__ void __launch_bounds__(256) k_mix(double *out, int iters) {
    d4 acc[NM > 0 ? NM : 1];
    double x[NV > 0 ? NV : 1];
    for (int i = 0; i < (NM > 0 ? NM : 1); ++i) acc[i] = (d4){0, 0, 0, 0};
    for (int i = 0; i < (NV > 0 ? NV : 1); ++i) x[i] = threadIdx.x * 1e-3 + i;
    double a = 0.5 + threadIdx.x * 1.37e-3, b = 1.0 + threadIdx.x * 1.1e-4;
    const double fa = 0.999999 - threadIdx.x * 1e-9, fb = 1e-9 * threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NM; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NV; ++i) x[i] = fma(x[i], fa, fb);
    }
    double s = 0;
    for (int i = 0; i < NM; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < NV; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NM, int NV>
void run(double *d, int iters, int wps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int grid = 256 * wps;
    hipLaunchKernelGGL((k_mix<NM, NV>), dim3(grid), dim3(256), 0, 0, d, iters / 4);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_mix<NM, NV>), dim3(grid), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    double waves = 1024.0 * wps;
    double fm = waves * iters * NM * 2048.0, fv = waves * iters * NV * 128.0;
    printf("NM=%d NV=%2d waves/SIMD=%d: %7.3f ms  mfma %5.1f + valu %5.1f = %5.1f TF/s\n", NM, NV, wps, ms,
           fm / ms / 1e9, fv / ms / 1e9, (fm + fv) / ms / 1e9);
}
int main() {
    double *d; (void)hipMalloc(&d, 8 * 1024 * 256 * 8);
    run<4, 0>(d, 4000, 1); run<4, 0>(d, 4000, 2); run<4, 0>(d, 2000, 4);
    run<0, 16>(d, 8000, 1); run<0, 16>(d, 4000, 2);
    run<4, 4>(d, 4000, 1); run<4, 8>(d, 4000, 1); run<4, 16>(d, 4000, 1); run<4, 32>(d, 4000, 1);
    run<4, 8>(d, 4000, 2); run<4, 16>(d, 4000, 2); run<2, 16>(d, 4000, 2); run<4, 32>(d, 2000, 2);
    run<8, 16>(d, 2000, 2); run<8, 32>(d, 2000, 2);
    return 0;
}
