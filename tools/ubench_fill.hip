// Per-CU fill-rate microbenchmark (measurement tool, not product code):
// 256 x R workgroups of 512 threads stream `bytes` of a buffer of `span` bytes
// (span 4 MB: L2-resident; 128 MB: Infinity-Cache-resident; 2 GB: HBM) with
//   mode 0: global_load_dwordx4 into registers, D loads in flight a wave
//   mode 1: global_load_lds_dwordx4 into a 64 KiB LDS ring, D in flight a wave
// and prints GB/s overall and per CU.  Each workgroup reads whole 1 KiB pieces
// (one per wave-instruction) at a stride that walks the span.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_fill.hip -o tools/ubench_fill
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ void __launch_bounds__(512) k_fill_reg(const int8_t *buf, size_t span, int iters, int *sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t nwave = (size_t)gridDim.x * 8, gw = (size_t)blockIdx.x * 8 + w;
    i32x4 acc = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        i32x4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const size_t piece = ((size_t)(it * D + d) * nwave + gw) * 1024 % span;
            v[d] = *(const i32x4 *)(buf + piece + 16 * lane);
        }
#pragma unroll
        for (int d = 0; d < D; ++d) acc ^= v[d];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) sink[0] = 1;
}

template <int D>
__global__ void __launch_bounds__(512) k_fill_lds(const int8_t *buf, size_t span, int iters, int *sink) {
    __shared__ __attribute__((aligned(16))) int8_t L[64 * 1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t nwave = (size_t)gridDim.x * 8, gw = (size_t)blockIdx.x * 8 + w;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const size_t piece = ((size_t)(it * D + d) * nwave + gw) * 1024 % span;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(buf + piece + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(L + ((w * D + d) % 64) * 1024),
                                             16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (L[threadIdx.x] == 123 && L[threadIdx.x + 1] == 45) sink[0] = 1;
}

template <int D>
static float run(int mode, const int8_t *buf, size_t span, int grid, int iters, int *sink) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(k_fill_reg<D>, dim3(grid), dim3(512), 0, 0, buf, span, iters, sink);
        else hipLaunchKernelGGL(k_fill_lds<D>, dim3(grid), dim3(512), 0, 0, buf, span, iters, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char **argv) {
    const size_t spans[4] = {(size_t)256 << 10, (size_t)1 << 20, (size_t)4 << 20, (size_t)128 << 20};
    int8_t *buf;
    int *sink;
    if (hipMalloc(&buf, spans[3]) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, spans[3]);
    for (int wg : {1, 2, 4})
    for (int mode = 0; mode < 2; ++mode)
        for (int si = 0; si < 4; ++si)
            for (int D : {4, 16}) {
                const int grid = 256 * wg;   // wg workgroups (8 waves each) a CU
                const int iters = 4096 / D;
                float ms = 0;
                switch (D) {
                    case 2: ms = run<2>(mode, buf, spans[si], grid, iters, sink); break;
                    case 4: ms = run<4>(mode, buf, spans[si], grid, iters, sink); break;
                    case 8: ms = run<8>(mode, buf, spans[si], grid, iters, sink); break;
                    default: ms = run<16>(mode, buf, spans[si], grid, iters, sink); break;
                }
                const double bytes = (double)grid * 8 * 4096 * 1024;
                printf("wg/CU %d mode %s span %6zu KB D %2d: %8.1f GB/s  %6.1f GB/s/CU  (%.3f ms)\n", wg, mode ? "lds-dma" : "reg    ",
                       spans[si] >> 10, D, bytes / ms / 1e6, bytes / ms / 1e6 / 256, ms);
                fflush(stdout);
            }
    return 0;
}
