// Latency microbenchmarks for the CONISS merge chain (one workgroup, 1-2 waves
// alone on the CU): dependent LDS loads, dependent VALU f64 ops, DPP min steps,
// readfirstlane -> scalar chains, barrier ping-pong between two waves, and the
// HBM load latency.  Cycles from s_memtime.  Build: hipcc --offload-arch=gfx950
// -O3 tools/lat_bench.hip -o tools/lat_bench (diagnostics only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm volatile("v_min_f64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <int CTRL> __device__ __forceinline__ double dpp_d(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

constexpr int ITERS = 2000;

__global__ void k_lat(long long *out, const int *gidx, double seed) {
    __shared__ int chase[1024];
    __shared__ double dv[64];
    __shared__ int flag[4];
    const int t = threadIdx.x, lane = t & 63;
    const bool w0 = __builtin_amdgcn_readfirstlane(t) < 64;
    for (int i = t; i < 1024; i += blockDim.x) chase[i] = (i * 37 + 11) & 1023;
    if (t < 64) dv[t] = seed + t;
    if (t < 4) flag[t] = 0;
    __syncthreads();
    long long t0, t1;
    if (w0) {
        // 1. dependent LDS loads, all lanes one address (broadcast)
        int idx = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) idx = chase[idx];
        asm volatile("" ::"v"(idx));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[0] = (t1 - t0);
        // 2. dependent v_add_f64
        double x = seed + lane;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(seed));
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[1] = (t1 - t0);
        // 3. DPP min steps (2 movs + v_min + nop)
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) x = vmin(x, dpp_d<0xB1>(x));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[2] = (t1 - t0);
        // 4. readfirstlane -> scalar add -> back to vector, dependent
        int v = lane;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            int s = __builtin_amdgcn_readfirstlane(v);
            v = v + s + 1;
        }
        asm volatile("" ::"v"(v));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[3] = (t1 - t0);
        // 5. LDS store then dependent load of the same word (one lane stores)
        int q = 1;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            if (lane == 0) chase[5] = q;
            q = chase[5] + 1;
        }
        asm volatile("" ::"v"(q));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[4] = (t1 - t0);
        // 6. same with all 64 lanes storing
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            chase[6] = q;
            q = chase[6] + 1;
        }
        asm volatile("" ::"v"(q));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[5] = (t1 - t0);
        // 7. ballot + ctz on a compare (vector compare -> scalar)
        int pos = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            unsigned long long m = __ballot(lane >= (pos & 63));
            pos = (int)__builtin_ctzll(m) + 1;
        }
        asm volatile("" ::"s"(pos));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[6] = (t1 - t0);
        // 8. dependent global loads (HBM / L2 chase)
        int g = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 200; ++i) g = gidx[g];
        asm volatile("" ::"v"(g));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[7] = (t1 - t0) * (ITERS / 200);
        // 9. s_memtime back to back
        t0 = __builtin_amdgcn_s_memtime();
        long long acc = 0;
        for (int i = 0; i < ITERS; ++i) acc += __builtin_amdgcn_s_memtime();
        asm volatile("" ::"s"(acc));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[8] = (t1 - t0);
    }
    __syncthreads();
    // 10. barrier ping-pong: both waves, ITERS barriers with one LDS word each way
    t0 = __builtin_amdgcn_s_memtime();
    int val = 0;
    for (int i = 0; i < ITERS; ++i) {
        if (w0) { if (lane == 0) flag[0] = i + val; }
        else { if (lane == 0) flag[1] = i; }
        __syncthreads();
        val = w0 ? flag[1] : flag[0];
    }
    asm volatile("" ::"v"(val));
    t1 = __builtin_amdgcn_s_memtime();
    if (t == 0) out[9] = (t1 - t0);
    // 11. v_cndmask chain (int select, dependent)
    if (w0) {
        int z = lane;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_cmp_gt_i32 vcc, %0, 5\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(z) : "v"(lane) : "vcc");
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[10] = (t1 - t0);
        // 12. (unused: a SALU asm chain would clobber SCC under the loop branch)
        if (lane == 0) out[11] = 0;
        // 13. exec-mask region, condition true in every lane (branch not taken)
        int y = lane;
        const int lim = __builtin_amdgcn_readfirstlane(-5) + lane * 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            if (y > lim) asm volatile("v_add_u32 %0, %0, 1" : "+v"(y));
            asm volatile("" : "+v"(y));
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[12] = (t1 - t0);
        // 14. exec-mask region, condition false everywhere (branch taken)
        const int lim2 = lim + 1000000;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            if (y > lim2) asm volatile("v_add_u32 %0, %0, 1" : "+v"(y));
            asm volatile("" : "+v"(y));
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[13] = (t1 - t0) + 0 * y;
        // 15. dependent v_add_u32 (integer VALU latency)
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(y));
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[14] = (t1 - t0);
        // 16. independent v_add_f64 x4 (issue rate)
        double a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_add_f64 %0, %0, %4\n\tv_add_f64 %1, %1, %4\n\tv_add_f64 %2, %2, %4\n\tv_add_f64 %3, %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed));
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[15] = (t1 - t0) / 4 + 0 * (long long)(a0 + a1 + a2 + a3);
        // 17-19. 100 LDS double stores then lgkmcnt(0): all lanes one address,
        // all lanes distinct addresses, one lane (exec mask)
        double *dst = reinterpret_cast<double *>(chase);
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 100; ++i) {
            asm volatile("ds_write_b64 %0, %1" ::"v"((i & 7) * 8), "v"(a0) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[16] = (t1 - t0) * ITERS / 100;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 100; ++i) {
            asm volatile("ds_write_b64 %0, %1" ::"v"(lane * 8), "v"(a0) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[17] = (t1 - t0) * ITERS / 100;
        t0 = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            for (int i = 0; i < 100; ++i) {
                asm volatile("ds_write_b64 %0, %1" ::"v"((i & 7) * 8), "v"(a0) : "memory");
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[18] = (t1 - t0) * ITERS / 100;
        (void)dst;
    }
}

int main() {
    fprintf(stderr, "start\n");
    const int G = 1 << 22;
    std::vector<int> h(G);
    unsigned x = 12345;
    for (int i = 0; i < G; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int)(x % (unsigned)G); }
    int *dg;
    long long *dout;
    hipMalloc(&dg, G * sizeof(int));
    hipMemcpy(dg, h.data(), G * sizeof(int), hipMemcpyHostToDevice);
    hipMalloc(&dout, 32 * sizeof(long long));
    long long ho[32];
    fprintf(stderr, "buffers ready\n");
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(128), 0, 0, dout, dg, 1.0);
        hipDeviceSynchronize();
        fprintf(stderr, "run %d done\n", rep);
    }
    hipMemcpy(ho, dout, 32 * sizeof(long long), hipMemcpyDeviceToHost);
    const char *names[] = {"LDS dependent load (broadcast)", "v_add_f64 dependent", "DPP min step (2 mov+min+nop)",
                           "readfirstlane->scalar->vector", "LDS store(1 lane)+load same word",
                           "LDS store(64 lanes)+load same word", "ballot+ctz dependent", "global dependent load (HBM)",
                           "s_memtime", "barrier ping-pong (2 waves)", "v_cmp+v_cndmask dependent",
                           "(unused)", "exec region, taken by all lanes",
                           "exec region, skipped (branch taken)", "v_add_u32 dependent", "v_add_f64 independent x4 (per op)",
                           "LDS store b64, 64 lanes same address", "LDS store b64, 64 lanes distinct",
                           "LDS store b64, one lane"};
    for (int i = 0; i < 19; ++i) printf("%-40s %8.1f cycles\n", names[i], (double)ho[i] / ITERS);
    return 0;
}
