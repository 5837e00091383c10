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

// xor butterfly (masks 1,2,4,...,32): every lane gets the same bits, and the
// pairing equals the oracle's butterfly64().
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = v + __shfl_xor(v, m, 64);
    return v;
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
