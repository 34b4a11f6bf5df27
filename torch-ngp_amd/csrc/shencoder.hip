// Real spherical-harmonics direction encoding (degree 1..8), gfx950.
//
// Reference: shencoder/src/shencoder.cu kernel_sh :27-355 (values :49-121,
// analytic d/dx,d/dy,d/dz :122-355), kernel_sh_backward :358-382.
//
// The basis polynomials are evaluated by ONE templated routine over a number
// type V: with V = float/double it produces the values in the reference's
// exact operation order; with V = Dual3 (value + 3 partials, forward-mode AD)
// the same routine yields the Jacobian, so the 192 hand-written derivative
// lines of the reference collapse into the product rule. For degree 4 (the
// NeRF path) the row width is a compile-time constant so each lane's 64-byte
// row leaves as four dwordx4 stores.
#include "ngp_common.h"

#include "sh_basis.h"

namespace {

using ngp_sh::Dual3;
using ngp_sh::sh_basis;

constexpr uint32_t kShBlock = 256;

// One lane per direction. Degree 4 (the NeRF path, C*C = 16 fp32 = 64 B per
// row) is instantiated with the row count known at compile time so the stores
// vectorise to dwordx4.
template <typename T, uint32_t CC>
__global__ void __launch_bounds__(kShBlock)
k_sh_fwd(const T* __restrict__ inputs, T* __restrict__ outputs, uint32_t B, uint32_t D,
         uint32_t C, T* __restrict__ dy_dx) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t C2 = CC ? CC : C * C;
    const T x = inputs[(size_t)b * D + 0], y = inputs[(size_t)b * D + 1], z = inputs[(size_t)b * D + 2];
    T* out = outputs + (size_t)b * C2;
    if constexpr (CC != 0) {
        T row[CC];
        sh_basis<T>(x, y, z, C, [&](uint32_t i, T v) { row[i] = v; });
#pragma unroll
        for (uint32_t i = 0; i < CC; ++i) out[i] = row[i];
    } else {
        sh_basis<T>(x, y, z, C, [&](uint32_t i, T v) { out[i] = v; });
    }
    if (dy_dx) {
        T* ddx = dy_dx + (size_t)b * D * C2;
        T* ddy = ddx + C2;
        T* ddz = ddy + C2;
        using Dl = Dual3<T>;
        sh_basis<Dl>(Dl(x, 1, 0, 0), Dl(y, 0, 1, 0), Dl(z, 0, 0, 1), C, [&](uint32_t i, Dl v) {
            ddx[i] = v.dx;
            ddy[i] = v.dy;
            ddz[i] = v.dz;
        });
    }
}

template <typename T>
__global__ void __launch_bounds__(kShBlock)
k_sh_bwd(const T* __restrict__ grad, uint32_t B, uint32_t D, uint32_t C,
         const T* __restrict__ dy_dx, T* __restrict__ grad_inputs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = t / D;
    if (b >= B) return;
    const uint32_t d = t - b * D;
    const uint32_t C2 = C * C;
    const T* g = grad + (size_t)b * C2;
    const T* dd = dy_dx + (size_t)b * D * C2 + (size_t)d * C2;
    T acc = grad_inputs[t];
    for (uint32_t ch = 0; ch < C2; ch++) acc += g[ch] * dd[ch];
    grad_inputs[t] = acc;
}

template <typename T>
int sh_fwd(const void* inputs, void* outputs, uint32_t B, uint32_t D, uint32_t C, void* dy_dx,
           hipStream_t st) {
    const uint32_t grid = ngp_div_up(B, kShBlock);
    const T* in = (const T*)inputs;
    T* out = (T*)outputs;
    T* dd = (T*)dy_dx;
    switch (C) {
        case 4: k_sh_fwd<T, 16><<<grid, kShBlock, 0, st>>>(in, out, B, D, C, dd); break;
        default: k_sh_fwd<T, 0><<<grid, kShBlock, 0, st>>>(in, out, B, D, C, dd); break;
    }
    return ngp_check_launch("sh_encode_forward");
}

}  // namespace

extern "C" int ngp_sh_encode_forward(const void* inputs, void* outputs, uint32_t B, uint32_t D,
                                     uint32_t C, void* dy_dx, int32_t dtype, void* stream) {
    NGP_REQUIRE(D == 3, NGP_ERR_ARG, "SH encoder only support input dim == 3");
    NGP_REQUIRE(C >= 1 && C <= 8, NGP_ERR_ARG, "SH encoder only supports degree in [1, 8]");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    switch (dtype) {
        case NGP_DTYPE_F32: return sh_fwd<float>(inputs, outputs, B, D, C, dy_dx, st);
        case NGP_DTYPE_F64: return sh_fwd<double>(inputs, outputs, B, D, C, dy_dx, st);
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "sh_encode_forward: inputs must be float32 or float64 (the wrapper casts to float32)");
    }
}

extern "C" int ngp_sh_encode_backward(const void* grad, const void* inputs, uint32_t B, uint32_t D,
                                      uint32_t C, const void* dy_dx, void* grad_inputs,
                                      int32_t dtype, void* stream) {
    (void)inputs;
    NGP_REQUIRE(D == 3, NGP_ERR_ARG, "SH encoder only support input dim == 3");
    NGP_REQUIRE(C >= 1 && C <= 8, NGP_ERR_ARG, "SH encoder only supports degree in [1, 8]");
    NGP_REQUIRE(dy_dx && grad_inputs, NGP_ERR_ARG, "sh_encode_backward: dy_dx and grad_inputs are required");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    const uint32_t grid = ngp_div_up(B * D, kShBlock);
    switch (dtype) {
        case NGP_DTYPE_F32:
            k_sh_bwd<float><<<grid, kShBlock, 0, st>>>((const float*)grad, B, D, C, (const float*)dy_dx, (float*)grad_inputs);
            break;
        case NGP_DTYPE_F64:
            k_sh_bwd<double><<<grid, kShBlock, 0, st>>>((const double*)grad, B, D, C, (const double*)dy_dx, (double*)grad_inputs);
            break;
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "sh_encode_backward: float32 or float64 only");
    }
    return ngp_check_launch("sh_encode_backward");
}
