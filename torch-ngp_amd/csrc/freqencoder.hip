// NeRF positional (frequency) encoding, gfx950.
//
// Reference: freqencoder/src/freqencoder.cu kernel_freq :30-59 (forward),
// kernel_freq_backward :63-94, host entries :97-131; freqencoder/freq.py.
//   outputs [B, C], C = D + 2 D deg:
//     out[b][d]                  = x[b][d]
//     out[b][D + 2Df + d]        = sin(2^f x[b][d])
//     out[b][D + 2Df + D + d]    = sin(2^f x[b][d] + pi/2)      (cos)
//   grad_inputs[b][d] = grad[b][d]
//       + sum_f 2^f (grad_sin * out_cos - grad_cos * out_sin)   (uses the saved outputs)
// Like the reference (__sinf), the sine is the hardware approximation
// (v_sin_f32 after the 1/(2 pi) scale): its absolute error grows with the
// argument's magnitude, about |arg| * 2^-23 (tests/test_gpu_freq.py states the bound).
//
// MI355X layout: the forward is a pure HBM write stream (C * 4 bytes per
// point against 4 D read), so each thread produces a 16-byte group of
// consecutive output floats of the row-major [B, C] tensor: one dwordx4
// store per lane, consecutive lanes on consecutive 16 bytes (an unaligned
// output falls back to one float per lane). The backward reads a row's
// 2 deg terms per coordinate (one lane per (b, d)).
#include "ngp_common.h"

namespace {

constexpr uint32_t kFreqBlock = 256;
constexpr float kHalfPi = 1.5707963267948966f;  // (PI() / 2) in float, freqencoder.cu:21,55

NGP_DEV float freq_value(const float* __restrict__ row, uint32_t c, uint32_t D) {
    if (c < D) return row[c];
    const uint32_t col = c / D - 1, d = c - (col + 1) * D;
    const uint32_t f = col >> 1;
    const float phase = (col & 1u) ? kHalfPi : 0.0f;
    return __sinf(scalbnf(row[d], (int)f) + phase);
}

// one output element per thread (unaligned outputs)
__global__ void __launch_bounds__(kFreqBlock)
k_freq_fwd(const float* __restrict__ inputs, uint32_t B, uint32_t D, uint32_t C, float* __restrict__ outputs) {
    const uint32_t e = blockIdx.x * kFreqBlock + threadIdx.x;
    if (e >= B * C) return;
    const uint32_t b = e / C, c = e - b * C;
    outputs[e] = freq_value(inputs + (size_t)b * D, c, D);
}

// Rows are C = D (1 + 2 deg) floats (odd for D = 3), so the aligned path
// treats [B, C] as one flat stream: thread t writes floats 4t .. 4t + 3 as
// one 16-byte store, stepping (b, c) across row ends itself
__global__ void __launch_bounds__(kFreqBlock)
k_freq_fwd_vec4(const float* __restrict__ inputs, uint32_t B, uint32_t D, uint32_t C, float* __restrict__ outputs) {
    const uint32_t total = B * C;
    const uint32_t e0 = (blockIdx.x * kFreqBlock + threadIdx.x) * 4;
    if (e0 >= total) return;
    uint32_t b = e0 / C, c = e0 - b * C;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t bb = b < B ? b : B - 1u;  // lanes past the end compute a row they drop
        v[j] = freq_value(inputs + (size_t)bb * D, c, D);
        if (++c == C) {
            c = 0;
            ++b;
        }
    }
    if (e0 + 4 <= total) {
        *reinterpret_cast<float4*>(outputs + e0) = float4{v[0], v[1], v[2], v[3]};
    } else {
        for (uint32_t j = 0; e0 + j < total; ++j) outputs[e0 + j] = v[j];
    }
}

__global__ void __launch_bounds__(kFreqBlock)
k_freq_bwd(const float* __restrict__ grad, const float* __restrict__ outputs, uint32_t B, uint32_t D,
           uint32_t deg, uint32_t C, float* __restrict__ grad_inputs) {
    const uint32_t t = blockIdx.x * kFreqBlock + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    const float* g = grad + (size_t)b * C;
    const float* o = outputs + (size_t)b * C;
    float result = g[d];
    for (uint32_t f = 0; f < deg; ++f) {
        const uint32_t s = D + 2 * D * f + d;
        // nvcc contracts a*b - c*d into fma(a, b, -(c*d)); the power-of-two
        // scale makes result + 2^f * x one rounding either way
        const float x = fmaf(g[s], o[s + D], -(g[s + D] * o[s]));
        result += scalbnf(1.0f, (int)f) * x;
    }
    grad_inputs[t] = result;
}

}  // namespace

extern "C" int ngp_freq_encode_forward(const float* inputs, uint32_t B, uint32_t D, uint32_t deg, uint32_t C,
                                       float* outputs, void* stream) {
    NGP_REQUIRE(D > 0 && C == D + 2 * D * deg, NGP_ERR_ARG,
                "freq_encode_forward: output_dim must be input_dim * (1 + 2 * degree), got %u for D=%u deg=%u", C, D, deg);
    NGP_REQUIRE(deg <= 64, NGP_ERR_ARG, "freq_encode_forward: degree %u too large", deg);
    if (B == 0) return NGP_OK;
    const uint64_t total = (uint64_t)B * C;
    NGP_REQUIRE(total + 4 * kFreqBlock < (1ull << 32), NGP_ERR_ARG,
                "freq_encode_forward: B * output_dim must stay below 2^32, got %llu", (unsigned long long)total);
    hipStream_t st = ngp_stream(stream);
    if (((uintptr_t)outputs & 15u) == 0) {
        k_freq_fwd_vec4<<<(uint32_t)((total + 4 * kFreqBlock - 1) / (4 * kFreqBlock)), kFreqBlock, 0, st>>>(
            inputs, B, D, C, outputs);
    } else {
        k_freq_fwd<<<(uint32_t)((total + kFreqBlock - 1) / kFreqBlock), kFreqBlock, 0, st>>>(inputs, B, D, C, outputs);
    }
    return ngp_check_launch("freq_encode_forward");
}

extern "C" int ngp_freq_encode_backward(const float* grad, const float* outputs, uint32_t B, uint32_t D,
                                        uint32_t deg, uint32_t C, float* grad_inputs, void* stream) {
    NGP_REQUIRE(D > 0 && C == D + 2 * D * deg, NGP_ERR_ARG,
                "freq_encode_backward: output_dim must be input_dim * (1 + 2 * degree), got %u for D=%u deg=%u", C, D, deg);
    if (B == 0) return NGP_OK;
    NGP_REQUIRE((uint64_t)B * C < (1ull << 32), NGP_ERR_ARG, "freq_encode_backward: B * output_dim must stay below 2^32");
    hipStream_t st = ngp_stream(stream);
    k_freq_bwd<<<ngp_div_up(B * D, kFreqBlock), kFreqBlock, 0, st>>>(grad, outputs, B, D, deg, C, grad_inputs);
    return ngp_check_launch("freq_encode_backward");
}
