// Microbenchmark of the C-Krylov orthogonalisation kernels (BCGS-PIP pass:
// k_pipz -> k_pipr -> k_pips -> k_pipa) at C3 sizes, each timed alone over
// repeated launches, plus k_pips cut after its phases (STOP 1/2).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I tadpole_amd/csrc tools/pip_bench.hip -o tools/pip_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tp_krylov_kernels.cuh"

using namespace tp;
#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void k_rand(double *p, size_t n, unsigned long long seed) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long z = seed + 0x9E3779B97F4A7C15ULL * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    p[i] = ((double)(z >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 7729;
    const int reps = 50;
    const int Dmax = 1056;
    double *K, *W, *Z, *part, *hh, *Ri, *out;
    int *info;
    double *apart;
    unsigned *cnt;
    CK(hipMalloc(&apart, (size_t)((n + 63) / 64) * 4 * 64 * KP * 8));
    CK(hipMalloc(&cnt, (size_t)((n + 63) / 64) * 4));
    CK(hipMemset(cnt, 0, (size_t)((n + 63) / 64) * 4));
    CK(hipMalloc(&K, (size_t)n * (Dmax + KP) * 8));
    CK(hipMalloc(&out, (size_t)n * KP * 8));
    CK(hipMalloc(&Z, (size_t)(Dmax + KP) * KP * 8));
    CK(hipMalloc(&part, (size_t)((n + 63) / 64) * (Dmax + KP) * KP * 8));
    CK(hipMalloc(&hh, (size_t)((Dmax + 63) / 64 + 1) * KP * KP * 8));
    CK(hipMalloc(&Ri, KP * KP * 8));
    CK(hipMalloc(&info, 64));
    const size_t tot = (size_t)n * (Dmax + KP);
    hipLaunchKernelGGL(k_rand, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, 0, K, tot, 1ULL);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        for (int r = 0; r < 3; ++r) launch();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f us\n", name, ms * 1e3 / reps);
    };
    for (int D : {256, 1024}) {
        W = K + (size_t)D * n;   // the block right after K's D columns
        const int ldz = D + KP;
        char nm[128];
        for (int chunk : {128, 256, 512}) {
            const int S = (n + chunk - 1) / chunk, dt = (ldz + PZ_COLS - 1) / PZ_COLS;
            const size_t pstride = (size_t)ldz * KP;
            snprintf(nm, sizeof nm, "D=%d k_pipz chunk %d (%d wg)", D, chunk, dt * S);
            timeit(nm, [&] { hipLaunchKernelGGL(k_pipz, dim3((unsigned)(dt * S)), dim3(256), 0, 0, K, D, W, n, chunk, part, pstride); });
            const int nsl = (ldz + PR - 1) / PR;
            snprintf(nm, sizeof nm, "D=%d k_pipr S=%d (%d wg)", D, S, nsl);
            timeit(nm, [&] { hipLaunchKernelGGL(k_pipr, dim3((unsigned)nsl), dim3(PR_TB), 0, 0, part, pstride, S, D, Z, hh); });
        }
        const int nh = (D + PR - 1) / PR;
        // a well-conditioned Zw: Z rows D.. = 64 I-ish via the hh = 0 path
        CK(hipMemset(hh, 0, (size_t)nh * KP * KP * 8));
        std::vector<double> zh((size_t)ldz * KP, 0.0);
        for (int j = 0; j < KP; ++j)
            for (int i = 0; i < ldz; ++i) zh[i + (size_t)j * ldz] = (i >= D && i - D == j) ? 64.0 : (i >= D ? 0.01 : 0.001 * (i % 7));
        CK(hipMemcpy(Z, zh.data(), zh.size() * 8, hipMemcpyHostToDevice));
        snprintf(nm, sizeof nm, "D=%d k_pips STOP1 (sums)", D);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pips<1>, dim3(1), dim3(512), 0, 0, Z, D, hh, nh, 1e-14, Ri, info, 0); });
        snprintf(nm, sizeof nm, "D=%d k_pips (Cholesky + inverse)", D);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pips<3>, dim3(1), dim3(512), 0, 0, Z, D, hh, nh, 1e-14, Ri, info, 0); });
        snprintf(nm, sizeof nm, "D=%d k_pips (Lowdin request, far from I)", D);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pips<3>, dim3(1), dim3(512), 0, 0, Z, D, hh, nh, 1e-14, Ri, info, 1); });
        const int tiles = (n + PA_ROWS - 1) / PA_ROWS;
        snprintf(nm, sizeof nm, "D=%d k_pipa (%d wg)", D, tiles * PA_SPLIT);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pipa, dim3((unsigned)(tiles * PA_SPLIT)), dim3(256), 0, 0, K, D, n, Z, apart); });
        snprintf(nm, sizeof nm, "D=%d k_pipc (%d wg)", D, tiles);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pipc, dim3((unsigned)tiles), dim3(256), 0, 0, apart, Ri, n, W, out); });
    }
    printf("empty-kernel reference: ");
    timeit("k_pips<1> with D=0, nh=0", [&] { hipLaunchKernelGGL(k_pips<1>, dim3(1), dim3(512), 0, 0, Z, 0, hh, 0, 1e-14, Ri, info, 0); });
    return 0;
}
