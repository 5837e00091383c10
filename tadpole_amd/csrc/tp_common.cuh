// Device helpers shared by the kernels.  Every .hip file of the library is
// compiled with -ffp-contract=off: the few fused multiply-adds the canonical
// arithmetic wants are written as fma() explicitly (oracle/tp_oracle.c does the
// same), so GPU and oracle round identically.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace tp {

__device__ __forceinline__ double r_na() { return __longlong_as_double(0x7FF00000000007A2LL); }
__device__ __forceinline__ double r_nan() { return __longlong_as_double(0x7FF8000000000000LL); }

// DPP lane moves on a double (two 32-bit halves).  CTRL: 0xB1 = quad_perm
// [1,0,3,2] (xor 1), 0x4E = quad_perm [2,3,0,1] (xor 2), 0x141 = row_half_mirror,
// 0x140 = row_mirror.
template <int CTRL> __device__ __forceinline__ double dpp_d(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// Canonical wave sum = xor butterfly (masks 1,2,4,8,16,32) of the oracle's
// butterfly64().  Steps 1-2 are the xor-1/xor-2 quad permutes; after them every
// lane of a quad holds the same bits, so row_half_mirror pairs l with a lane of
// quad l^4 (same value as lane l^4) and, one step later, row_mirror pairs l
// with a lane of the 8-group l^8.  The 16- and 32-lane steps are done on the
// four row values read with readlane: (R0 + R1) + (R2 + R3), exactly the
// butterfly's last two levels.  All lanes return the same bits.
__device__ __forceinline__ double wave_sum(double v) {
    v = v + dpp_d<0xB1>(v);
    v = v + dpp_d<0x4E>(v);
    v = v + dpp_d<0x141>(v);
    v = v + dpp_d<0x140>(v);
    double r0 = readlane_d(v, 0), r1 = readlane_d(v, 16), r2 = readlane_d(v, 32), r3 = readlane_d(v, 48);
    return (r0 + r1) + (r2 + r3);
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
