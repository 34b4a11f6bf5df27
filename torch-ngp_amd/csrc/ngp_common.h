// Shared device helpers for the gfx950 (CDNA4) instant-ngp hot path.
//
// Numerics policy (see DESIGN.md "Bit-exactness"): every kernel in this library
// is compiled with -ffp-contract=off, so a fused multiply-add happens ONLY where
// the source writes fmaf()/fma() explicitly. The C oracle (oracle/ngp_oracle.c)
// places its fmaf() calls at exactly the same points (the points where nvcc's
// default contraction would fuse the reference's expressions), which is what
// makes the integer outputs (sample counts, offsets, Morton indices, bitfields)
// and the grid-encoder / marching float outputs bit-identical between the HIP
// path and the oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ngp_hip.h"
#include "ngp_error.h"

#define NGP_DEV __device__ __forceinline__

// float -> half of an already rounded float. The backend folds
// fptrunc(fmul(a, b)) into v_fma_mix*_f16 (one rounding of the exact product
// instead of the float product's two), which torch's `.half()` of a float
// tensor does not do; the empty asm pins the float first.
NGP_DEV _Float16 ngp_f2h(float x) {
    asm volatile("" : "+v"(x));
    return (_Float16)x;
}

typedef _Float16 ngp_half;
typedef _Float16 ngp_half2 __attribute__((ext_vector_type(2)));

__host__ __device__ static inline uint32_t ngp_div_up(uint32_t a, uint32_t b) { return (a + b - 1) / b; }
static inline hipStream_t ngp_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Compute units of the current device (persistent-grid sizing).
static inline uint32_t ngp_num_cus() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        return 256;
    return (uint32_t)n;
}

// scalar_t-generic arithmetic used by the templated encoder kernels.
//   S = storage type, F = compute type of one product.
// For half storage these reproduce c10::Half semantics of `Half += float`:
// the float operand is rounded to half first, then the sum is rounded
// (reference gridencoder.cu:184 with scalar_t = at::Half).
template <typename T> struct Acc;
template <> struct Acc<float> {
    using S = float;
    using F = float;
    NGP_DEV static F load(const float* p) { return *p; }
    NGP_DEV static S zero() { return 0.0f; }
    NGP_DEV static S mac(S res, F a, F b) { return fmaf(a, b, res); }  // nvcc contracts res += a*b
    NGP_DEV static F to_f(S v) { return v; }
};
template <> struct Acc<ngp_half> {
    using S = ngp_half;
    using F = float;
    NGP_DEV static F load(const ngp_half* p) { return (float)*p; }
    NGP_DEV static S zero() { return (ngp_half)0.0f; }
    NGP_DEV static S mac(S res, F a, F b) {
        ngp_half prod = (ngp_half)(a * b);
        return (ngp_half)((float)res + (float)prod);
    }
    NGP_DEV static F to_f(S v) { return (float)v; }
};
template <> struct Acc<double> {
    using S = double;
    using F = double;
    NGP_DEV static F load(const double* p) { return *p; }
    NGP_DEV static S zero() { return 0.0; }
    NGP_DEV static S mac(S res, F a, F b) { return fma(a, b, res); }
    NGP_DEV static F to_f(S v) { return v; }
};
