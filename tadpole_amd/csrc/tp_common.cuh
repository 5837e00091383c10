// Device helpers shared by the kernels.  Every .hip file of the library is
// compiled with -ffp-contract=off: the few fused multiply-adds the canonical
// arithmetic wants are written as fma() explicitly (oracle/tp_oracle.c does the
// same), so GPU and oracle round identically.
#pragma once
#include <cassert>

// Device-side bounds checks for debug builds (make DEVICE_ASSERTS=1): compiled
// out of the product library.
#ifdef TP_DEVICE_ASSERTS
#define TP_DASSERT(cond) assert(cond)
#else
#define TP_DASSERT(cond) ((void)0)
#endif
#include <hip/hip_runtime.h>
#include <cstdint>

namespace tp {

__device__ __forceinline__ double r_na() { return __longlong_as_double(0x7FF00000000007A2LL); }
__device__ __forceinline__ double r_nan() { return __longlong_as_double(0x7FF8000000000000LL); }

// DPP lane moves on a double (two 32-bit halves, no "old" operand, so no
// zero-fill moves).  CTRL: 0xB1 = quad_perm [1,0,3,2] (xor 1), 0x4E =
// quad_perm [2,3,0,1] (xor 2), 0x141 = row_half_mirror, 0x140 = row_mirror,
// 0x142 = row_bcast:15 (lane 15 of row r-1 -> row r), 0x143 = row_bcast:31
// (lane 31 -> rows 2 and 3).  Lanes without a source read 0 (bound_ctrl).
template <int CTRL> __device__ __forceinline__ double dpp_d(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// IEEE minNum of two doubles in one instruction: a quiet-NaN operand is
// ignored (fmin() would add two canonicalising v_max per call).  The s_nop
// covers the VALU-write -> DPP-read hazard the compiler cannot see through asm.
__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm volatile("v_min_f64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Canonical wave sum = xor butterfly (masks 1,2,4,8,16,32) of the oracle's
// butterfly64().  Steps 1-2 are the xor-1/xor-2 quad permutes; after them every
// lane of a quad holds the same bits, so row_half_mirror pairs l with a lane of
// quad l^4 (same value as lane l^4) and, one step later, row_mirror pairs l
// with a lane of the 8-group l^8: every lane of row r then holds R_r.  The 16-
// and 32-lane levels are the two row broadcasts: lane 63 ends with
// (R3 + R2) + (R1 + R0), the butterfly's (R0 + R1) + (R2 + R3) bit for bit
// (IEEE addition is commutative).  Returned wave-uniform (lane 63).
__device__ __forceinline__ double wave_sum(double v) {
    v = v + dpp_d<0xB1>(v);
    v = v + dpp_d<0x4E>(v);
    v = v + dpp_d<0x141>(v);
    v = v + dpp_d<0x140>(v);
    v = v + dpp_d<0x142>(v);
    v = v + dpp_d<0x143>(v);
    return readlane_d(v, 63);
}
// minimum over the wave ignoring NaN lanes (NaN only if every lane is NaN)
__device__ __forceinline__ double wave_min(double v) {
    v = vmin(v, dpp_d<0xB1>(v));
    v = vmin(v, dpp_d<0x4E>(v));
    v = vmin(v, dpp_d<0x141>(v));
    v = vmin(v, dpp_d<0x140>(v));
    v = vmin(v, dpp_d<0x142>(v));
    v = vmin(v, dpp_d<0x143>(v));
    return readlane_d(v, 63);
}

// double-double accumulation (oracle: dd_add_d / dd_div_d)
__device__ __forceinline__ void two_sum(double a, double b, double &s, double &e) {
    double x = a + b;
    double bv = x - a;
    double av = x - bv;
    s = x;
    e = (a - av) + (b - bv);
}
__device__ __forceinline__ void dd_add_d(double &hi, double &lo, double x) {
    double s, e;
    two_sum(hi, x, s, e);
    e = e + lo;
    double h2 = s + e;
    lo = e - (h2 - s);
    hi = h2;
}
__device__ __forceinline__ void dd_add_dd(double &hi, double &lo, double hi2, double lo2) {
    double s, e;
    two_sum(hi, hi2, s, e);
    e = e + (lo + lo2);
    double h2 = s + e;
    lo = e - (h2 - s);
    hi = h2;
}
__device__ __forceinline__ double dd_div_d(double hi, double lo, double d) {
    double q1 = hi / d;
    double r = fma(-q1, d, hi);
    r = r + lo;
    return q1 + r / d;
}
// wave-wide double-double sum (butterfly on pairs)
__device__ __forceinline__ void wave_dd_sum(double &hi, double &lo) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        double h2 = __shfl_xor(hi, m, 64);
        double l2 = __shfl_xor(lo, m, 64);
        dd_add_dd(hi, lo, h2, l2);
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its outstanding global stores (__syncthreads' release
// fence waits for those too -- a full HBM write latency per barrier in loops
// that stream results out).  Only for data exchanged through LDS; global data
// written before it is NOT visible to other waves after it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// total order on doubles as unsigned keys (radix select)
__device__ __forceinline__ uint64_t dkey(double x) {
    uint64_t u = (uint64_t)__double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double dkey_inv(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
    return __longlong_as_double((long long)u);
}

}  // namespace tp
