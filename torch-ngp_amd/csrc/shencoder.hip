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

namespace {

template <typename T>
struct Dual3 {
    T v, dx, dy, dz;
    NGP_DEV Dual3() = default;
    NGP_DEV Dual3(T c) : v(c), dx(0), dy(0), dz(0) {}
    NGP_DEV Dual3(T a, T b, T c, T d) : v(a), dx(b), dy(c), dz(d) {}
};
template <typename T> NGP_DEV Dual3<T> operator+(Dual3<T> a, Dual3<T> b) { return {a.v + b.v, a.dx + b.dx, a.dy + b.dy, a.dz + b.dz}; }
template <typename T> NGP_DEV Dual3<T> operator-(Dual3<T> a, Dual3<T> b) { return {a.v - b.v, a.dx - b.dx, a.dy - b.dy, a.dz - b.dz}; }
template <typename T> NGP_DEV Dual3<T> operator-(Dual3<T> a) { return {-a.v, -a.dx, -a.dy, -a.dz}; }
template <typename T> NGP_DEV Dual3<T> operator*(Dual3<T> a, Dual3<T> b) {
    return {a.v * b.v, a.dx * b.v + a.v * b.dx, a.dy * b.v + a.v * b.dy, a.dz * b.v + a.v * b.dz};
}
template <typename T> NGP_DEV Dual3<T> operator*(float c, Dual3<T> b) { return {(T)c * b.v, (T)c * b.dx, (T)c * b.dy, (T)c * b.dz}; }
template <typename T> NGP_DEV Dual3<T> operator+(Dual3<T> a, float c) { return {a.v + (T)c, a.dx, a.dy, a.dz}; }
template <typename T> NGP_DEV Dual3<T> operator+(float c, Dual3<T> a) { return {(T)c + a.v, a.dx, a.dy, a.dz}; }
template <typename T> NGP_DEV Dual3<T> operator-(Dual3<T> a, float c) { return {a.v - (T)c, a.dx, a.dy, a.dz}; }
template <typename T> NGP_DEV Dual3<T> operator-(float c, Dual3<T> a) { return {(T)c - a.v, -a.dx, -a.dy, -a.dz}; }

// Evaluates the first C*C real SH basis functions at (x, y, z) into o[].
// Operation order matches the reference expressions term by term.
template <typename V, typename Sink>
NGP_DEV void sh_basis(V x, V y, V z, uint32_t C, Sink&& o) {
    const V xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    const V x4 = x2 * x2, y4 = y2 * y2, z4 = z2 * z2;
    const V x6 = x4 * x2, y6 = y4 * y2, z6 = z4 * z2;
    o(0, V(0.28209479177387814f));
    if (C <= 1) return;
    o(1, -0.48860251190291987f * y);
    o(2, 0.48860251190291987f * z);
    o(3, -0.48860251190291987f * x);
    if (C <= 2) return;
    o(4, 1.0925484305920792f * xy);
    o(5, -1.0925484305920792f * yz);
    o(6, 0.94617469575755997f * z2 - 0.31539156525251999f);
    o(7, -1.0925484305920792f * xz);
    o(8, 0.54627421529603959f * x2 - 0.54627421529603959f * y2);
    if (C <= 3) return;
    o(9, 0.59004358992664352f * y * (-3.0f * x2 + y2));
    o(10, 2.8906114426405538f * xy * z);
    o(11, 0.45704579946446572f * y * (1.0f - 5.0f * z2));
    o(12, 0.3731763325901154f * z * (5.0f * z2 - 3.0f));
    o(13, 0.45704579946446572f * x * (1.0f - 5.0f * z2));
    o(14, 1.4453057213202769f * z * (x2 - y2));
    o(15, 0.59004358992664352f * x * (-x2 + 3.0f * y2));
    if (C <= 4) return;
    o(16, 2.5033429417967046f * xy * (x2 - y2));
    o(17, 1.7701307697799304f * yz * (-3.0f * x2 + y2));
    o(18, 0.94617469575756008f * xy * (7.0f * z2 - 1.0f));
    o(19, 0.66904654355728921f * yz * (3.0f - 7.0f * z2));
    o(20, -3.1735664074561294f * z2 + 3.7024941420321507f * z4 + 0.31735664074561293f);
    o(21, 0.66904654355728921f * xz * (3.0f - 7.0f * z2));
    o(22, 0.47308734787878004f * (x2 - y2) * (7.0f * z2 - 1.0f));
    o(23, 1.7701307697799304f * xz * (-x2 + 3.0f * y2));
    o(24, -3.7550144126950569f * x2 * y2 + 0.62583573544917614f * x4 + 0.62583573544917614f * y4);
    if (C <= 5) return;
    o(25, 0.65638205684017015f * y * (10.0f * x2 * y2 - 5.0f * x4 - y4));
    o(26, 8.3026492595241645f * xy * z * (x2 - y2));
    o(27, -0.48923829943525038f * y * (3.0f * x2 - y2) * (9.0f * z2 - 1.0f));
    o(28, 4.7935367849733241f * xy * z * (3.0f * z2 - 1.0f));
    o(29, 0.45294665119569694f * y * (14.0f * z2 - 21.0f * z4 - 1.0f));
    o(30, 0.1169503224534236f * z * (-70.0f * z2 + 63.0f * z4 + 15.0f));
    o(31, 0.45294665119569694f * x * (14.0f * z2 - 21.0f * z4 - 1.0f));
    o(32, 2.3967683924866621f * z * (x2 - y2) * (3.0f * z2 - 1.0f));
    o(33, -0.48923829943525038f * x * (x2 - 3.0f * y2) * (9.0f * z2 - 1.0f));
    o(34, 2.0756623148810411f * z * (-6.0f * x2 * y2 + x4 + y4));
    o(35, 0.65638205684017015f * x * (10.0f * x2 * y2 - x4 - 5.0f * y4));
    if (C <= 6) return;
    o(36, 1.3663682103838286f * xy * (-10.0f * x2 * y2 + 3.0f * x4 + 3.0f * y4));
    o(37, 2.3666191622317521f * yz * (10.0f * x2 * y2 - 5.0f * x4 - y4));
    o(38, 2.0182596029148963f * xy * (x2 - y2) * (11.0f * z2 - 1.0f));
    o(39, -0.92120525951492349f * yz * (3.0f * x2 - y2) * (11.0f * z2 - 3.0f));
    o(40, 0.92120525951492349f * xy * (-18.0f * z2 + 33.0f * z4 + 1.0f));
    o(41, 0.58262136251873131f * yz * (30.0f * z2 - 33.0f * z4 - 5.0f));
    o(42, 6.6747662381009842f * z2 - 20.024298714302954f * z4 + 14.684485723822165f * z6 - 0.31784601133814211f);
    o(43, 0.58262136251873131f * xz * (30.0f * z2 - 33.0f * z4 - 5.0f));
    o(44, 0.46060262975746175f * (x2 - y2) * (11.0f * z2 * (3.0f * z2 - 1.0f) - 7.0f * z2 + 1.0f));
    o(45, -0.92120525951492349f * xz * (x2 - 3.0f * y2) * (11.0f * z2 - 3.0f));
    o(46, 0.50456490072872406f * (11.0f * z2 - 1.0f) * (-6.0f * x2 * y2 + x4 + y4));
    o(47, 2.3666191622317521f * xz * (10.0f * x2 * y2 - x4 - 5.0f * y4));
    o(48, 10.247761577878714f * x2 * y4 - 10.247761577878714f * x4 * y2 + 0.6831841051919143f * x6 - 0.6831841051919143f * y6);
    if (C <= 7) return;
    o(49, 0.70716273252459627f * y * (-21.0f * x2 * y4 + 35.0f * x4 * y2 - 7.0f * x6 + y6));
    o(50, 5.2919213236038001f * xy * z * (-10.0f * x2 * y2 + 3.0f * x4 + 3.0f * y4));
    o(51, -0.51891557872026028f * y * (13.0f * z2 - 1.0f) * (-10.0f * x2 * y2 + 5.0f * x4 + y4));
    o(52, 4.1513246297620823f * xy * z * (x2 - y2) * (13.0f * z2 - 3.0f));
    o(53, -0.15645893386229404f * y * (3.0f * x2 - y2) * (13.0f * z2 * (11.0f * z2 - 3.0f) - 27.0f * z2 + 3.0f));
    o(54, 0.44253269244498261f * xy * z * (-110.0f * z2 + 143.0f * z4 + 15.0f));
    o(55, 0.090331607582517306f * y * (-135.0f * z2 + 495.0f * z4 - 429.0f * z6 + 5.0f));
    o(56, 0.068284276912004949f * z * (315.0f * z2 - 693.0f * z4 + 429.0f * z6 - 35.0f));
    o(57, 0.090331607582517306f * x * (-135.0f * z2 + 495.0f * z4 - 429.0f * z6 + 5.0f));
    o(58, 0.07375544874083044f * z * (x2 - y2) * (143.0f * z2 * (3.0f * z2 - 1.0f) - 187.0f * z2 + 45.0f));
    o(59, -0.15645893386229404f * x * (x2 - 3.0f * y2) * (13.0f * z2 * (11.0f * z2 - 3.0f) - 27.0f * z2 + 3.0f));
    o(60, 1.0378311574405206f * z * (13.0f * z2 - 3.0f) * (-6.0f * x2 * y2 + x4 + y4));
    o(61, -0.51891557872026028f * x * (13.0f * z2 - 1.0f) * (-10.0f * x2 * y2 + x4 + 5.0f * y4));
    o(62, 2.6459606618019f * z * (15.0f * x2 * y4 - 15.0f * x4 * y2 + x6 - y6));
    o(63, 0.70716273252459627f * x * (-35.0f * x2 * y4 + 21.0f * x4 * y2 - x6 + 7.0f * y6));
}

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
