// Microbenchmark of the banded T*Y product (k_band_ty in tp_pca.hip) and
// variants at the Krylov small problem's shape (D = 1024, b = 256, P = 64).
// hipcc --offload-arch=gfx950 -O3 -o tools/band_bench tools/band_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4b __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// V: 0 as tp_pca.hip, 1 no loads (registers from indices), 2 no epilogue reads,
// 3 XCD-contiguous (block row, column tile) chunks
template <int P, int V>
__global__ void __launch_bounds__(12 * P) kb(const double *__restrict__ T, const double *__restrict__ Y, double *Out,
                                             int D, double a, double bc, const double *Yc, double cc, const double *Yp,
                                             int ldt, int ldy) {
    constexpr int NRW = P / 16;
    __shared__ double tile[3][P][17];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, fr = l & 15, fk = l >> 4;
    const int rw = w % NRW, kbk = w / NRW;
    int ib = blockIdx.x, c0 = blockIdx.y * 16;
    if (V == 3) {
        const int W = gridDim.x * gridDim.y, L = blockIdx.x + blockIdx.y * gridDim.x;
        const int id = (W % 8) ? L : (L % 8) * (W / 8) + L / 8;
        ib = id / gridDim.y;
        c0 = (id % gridDim.y) * 16;
    }
    const int r0 = ib * P + 16 * rw;
    const int kc = ib - 1 + kbk;
    d4b acc = (d4b){0.0, 0.0, 0.0, 0.0};
    if (kc >= 0 && kc * P < D) {
        const double *tp = T + (size_t)(r0 + fr) + (size_t)(kc * P + fk) * ldt;
        const double *yp = Y + (size_t)(kc * P + fk) + (size_t)(c0 + fr) * ldy;
        double af[P / 4], bf[P / 4];
#pragma unroll
        for (int u = 0; u < P / 4; ++u) {
            if (V == 1) { af[u] = (double)(u + fr); bf[u] = (double)(u * fk); }
            else { af[u] = tp[(size_t)(4 * u) * ldt]; bf[u] = yp[4 * u]; }
        }
#pragma unroll
        for (int u = 0; u < P / 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(af[u], bf[u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[kbk][16 * rw + fk + 4 * r][fr] = acc[r];
    __syncthreads();
    if (threadIdx.x >= 4 * P) return;
    const int j = threadIdx.x / (P / 4), q = threadIdx.x % (P / 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int rl = q + e * (P / 4);
        const size_t idx = (size_t)(ib * P + rl) + (size_t)(c0 + j) * D;
        double v = (tile[0][rl][j] + tile[1][rl][j]) + tile[2][rl][j];
        if (V != 2) {
            v = a * v + bc * Yc[idx];
            if (Yp) v = v + cc * Yp[idx];
        }
        Out[idx] = v;
    }
}

__global__ void k_empty(double *o) { if (threadIdx.x == 1023) o[0] = 1.0; }

int main() {
    const int D = 1024, b = 256, P = 64;
    std::vector<double> h((size_t)D * D);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
    double *T, *Y, *O, *Yc, *Yp;
    CK(hipMalloc(&T, (size_t)(D + 64) * D * 8)); CK(hipMalloc(&Y, (size_t)(D + 64) * b * 8)); CK(hipMalloc(&O, (size_t)D * b * 8));
    CK(hipMalloc(&Yc, (size_t)D * b * 8)); CK(hipMalloc(&Yp, (size_t)D * b * 8));
    CK(hipMemcpy(T, h.data(), (size_t)D * D * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Y, h.data(), (size_t)D * b * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Yc, h.data(), (size_t)D * b * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Yp, h.data(), (size_t)D * b * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const dim3 grid(D / P, b / 16), blk(12 * P);
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 20; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 200; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %8.2f us\n", name, ms * 1000 / 200);
    };
    run("empty kernel (256 x 768)", [&] { hipLaunchKernelGGL(k_empty, grid, blk, 0, 0, O); });
    run("band v0 (as library)", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D); });
    run("band v1 no operand loads", [&] { hipLaunchKernelGGL((kb<64, 1>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D); });
    run("band v2 no epilogue reads", [&] { hipLaunchKernelGGL((kb<64, 2>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D); });
    run("band v3 XCD chunks", [&] { hipLaunchKernelGGL((kb<64, 3>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D); });
    run("band v0 ldT = ldY = D + 16", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D + 16, D + 16); });
    run("band v0 ldT = D + 16", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D + 16, D); });
    run("band v0 ldY = D + 16", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D + 16); });
    run("band v0 ldT = ldY = D + 8", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D + 8, D + 8); });
    run("band v0 (again)", [&] { hipLaunchKernelGGL((kb<64, 0>), grid, blk, 0, 0, T, Y, O, D, 0.5, 0.25, Yc, 0.1, Yp, D, D); });
    return 0;
}
