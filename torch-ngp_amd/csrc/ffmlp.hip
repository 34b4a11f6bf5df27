// Fully fused MLP on gfx950 fp16 MFMA (v_mfma_f32_16x16x32_f16, fp32 accumulate).
//
// Reference: ffmlp/src/ffmlp.cu — kernel_mlp_fused :331-407 (forward),
// kernel_mlp_fused_backward :410-518 + CUTLASS split-K dW GEMMs :749-895.
// Layer semantics: bias-free, per-layer weights row-major [out, in] packed
// back to back (nn.Linear layout, ffmlp.py:115), hidden activation after every
// layer but the last, output activation after the last (always None in FFMLP),
// backward ignores the output activation (ffmlp.cu:783).
//
// MI355X design:
//   * "transposed" products: a layer computes Y^T[out, S] = W[out, in] · X^T,
//     so the MFMA accumulator (lane = sample column, 4 output units per lane)
//     feeds the next layer's B operand directly, without LDS, by permuting
//     the K order (cdna_hip_programming.md §3 "accumulator as next operand").
//     The weight fragments are permuted to match once per workgroup, in LDS,
//     lane-linear so every fragment read is a conflict-free ds_read_b128.
//   * the backward recomputes activations instead of streaming them through
//     HBM (the reference stores num_layers x B x hidden fp16 forward + backward
//     buffers), propagates deltas the same register-resident way through
//     W^T fragments, and reduces dW = delta^T · H over every sample the
//     workgroup sees with MFMAs whose K dimension is the sample index (the
//     one transposition goes through a per-wave LDS tile). Per-workgroup
//     partial dW land in a slab and one reduce kernel sums them in fixed
//     order: no atomics, bit-reproducible weight gradients.
#include "ngp_common.h"

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kNB = 2;          // 16-sample column blocks per wave step (32 samples)
constexpr int kOut = 16;        // padded output width (FFMLP pads to 16)
constexpr int kScratchLd = 40;  // halves per row of the per-wave transpose tile (32 + pad)
constexpr uint32_t kMaxBwdBlocks = 256;

NGP_DEV f32x4 mfma(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Activation enum of ffmlp.py:89-96 / utils.h:29-37.
enum Act : uint32_t { kReLU = 0, kExp = 1, kSine = 2, kSigmoid = 3, kSquareplus = 4, kSoftplus = 5, kNone = 6 };
constexpr float kKAct = 10.0f;

NGP_DEV float act_fwd(uint32_t a, float x) {
    switch (a) {
        case kReLU: return x > 0.0f ? x : 0.0f;
        case kExp: return expf(x);
        case kSine: return sinf(x);
        case kSigmoid: return 1.0f / (1.0f + expf(-x));
        case kSquareplus: { const float y = x * kKAct; return 0.5f * (y + sqrtf(y * y + 4)) / kKAct; }
        case kSoftplus: return logf(expf(x * kKAct) + 1.0f) / kKAct;
        default: return x;
    }
}
// derivative expressed through the post-activation value y (utils.h:536-580)
NGP_DEV float act_bwd(uint32_t a, float g, float y) {
    switch (a) {
        case kReLU: return y > 0.0f ? g : 0.0f;
        case kExp: return g * y;
        case kSigmoid: return g * (y * (1.0f - y));
        case kSquareplus: { const float t = y * kKAct; return g * (t * t / (t * t + 1)); }
        case kSoftplus: return g * (1.0f - expf(-y * kKAct));
        default: return g;  // None; Sine has no backward in the reference (utils.h:552-556)
    }
}

// K-slot permutation produced by packing two 16-row accumulator tiles into
// one 32-deep B operand: slot (g, j) of K-step s holds unit 32s + perm(g, j).
NGP_DEV int perm_unit(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

// ---- weight fragments in LDS ------------------------------------------------
// Matmul q of the network (q = 0 first, 1..NH hidden, NH+1 = last) has weight
// W_q [out_q, in_q] at flat offset off_q. A "forward" fragment set is the A
// operand of W_q (M = out_q, K = in_q); a "backward" set is the A operand of
// W_q^T (M = in_q, K = out_q). Fragment (mt, s) = 64 lanes x 8 halves.
struct MatDesc {
    uint32_t off, out, in;   // weight slice
    uint32_t mt, ks;         // fragment grid of the A operand
    uint32_t frag0;          // first fragment index in LDS
    bool kperm;              // K order of the B operand it multiplies is permuted
};

NGP_DEV void build_frags(half8* lds, const ngp_half* __restrict__ w, const MatDesc& m, bool transposed) {
    const uint32_t n = m.mt * m.ks * 64;  // lanes to fill
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
        const uint32_t lane = t & 63, f = t >> 6;
        const uint32_t mt = f / m.ks, s = f - mt * m.ks;
        const int g = lane >> 4, c = lane & 15;
        half8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t row = 16 * mt + c;                                  // M index
            const uint32_t k = 32 * s + (m.kperm ? perm_unit(g, j) : 8 * g + j);  // K index
            // forward: A[row=o][k=i] = W[o][i]; transposed: A[row=i][k=o] = W[o][i]
            const uint32_t o = transposed ? k : row, i = transposed ? row : k;
            v[j] = (o < m.out && i < m.in) ? w[m.off + o * m.in + i] : (ngp_half)0.0f;
        }
        lds[(m.frag0 + f) * 64 + lane] = v;
    }
}

// Network geometry (all compile-time except in_dim, which only changes
// fragment contents). IN_KS = ceil(in_dim / 32), NH = hidden matmuls.
template <int W, int IN_KS, int NH>
struct Net {
    static constexpr int MTW = W / 16;             // M tiles of a hidden-width output
    static constexpr int KSW = (W + 31) / 32;      // K steps over a hidden-width input
    static constexpr int NMAT = NH + 2;            // matmuls
    static constexpr int IN_MT = IN_KS * 2;        // M tiles over the (padded) input width
    // forward fragments: first W x in, hidden W x W, last 16 x W
    static constexpr int FWD_FRAGS = MTW * IN_KS + NH * MTW * KSW + 1 * KSW;
    // backward fragments: W_q^T for q = 0..NH+1
    static constexpr int BWD_FRAGS = IN_MT * KSW + NH * MTW * KSW + MTW * 1;
};

template <int W, int IN_KS, int NH>
NGP_DEV MatDesc fwd_desc(int q, uint32_t in_dim) {
    using N = Net<W, IN_KS, NH>;
    MatDesc m;
    if (q == 0) {
        m = {0u, (uint32_t)W, in_dim, (uint32_t)N::MTW, (uint32_t)IN_KS, 0u, false};
    } else if (q <= NH) {
        m = {W * in_dim + (uint32_t)(q - 1) * W * W, (uint32_t)W, (uint32_t)W, (uint32_t)N::MTW,
             (uint32_t)N::KSW, (uint32_t)(N::MTW * IN_KS + (q - 1) * N::MTW * N::KSW), true};
    } else {
        m = {W * in_dim + (uint32_t)NH * W * W, (uint32_t)kOut, (uint32_t)W, 1u, (uint32_t)N::KSW,
             (uint32_t)(N::MTW * IN_KS + NH * N::MTW * N::KSW), true};
    }
    return m;
}

template <int W, int IN_KS, int NH>
NGP_DEV MatDesc bwd_desc(int q, uint32_t in_dim) {
    using N = Net<W, IN_KS, NH>;
    MatDesc m;
    if (q == 0) {  // W_0^T: M over input features, K over hidden units (permuted deltas)
        m = {0u, (uint32_t)W, in_dim, (uint32_t)N::IN_MT, (uint32_t)N::KSW, 0u, true};
    } else if (q <= NH) {
        m = {W * in_dim + (uint32_t)(q - 1) * W * W, (uint32_t)W, (uint32_t)W, (uint32_t)N::MTW,
             (uint32_t)N::KSW, (uint32_t)(N::IN_MT * N::KSW + (q - 1) * N::MTW * N::KSW), true};
    } else {  // last: K over the 16 outputs, natural order (grad loaded from memory)
        m = {W * in_dim + (uint32_t)NH * W * W, (uint32_t)kOut, (uint32_t)W, (uint32_t)N::MTW, 1u,
             (uint32_t)(N::IN_MT * N::KSW + NH * N::MTW * N::KSW), false};
    }
    return m;
}

// acc[nb][mt] = A(frags) · B[nb]
template <int MT, int KS>
NGP_DEV void dense(const half8* __restrict__ lds, uint32_t frag0, const half8 (&b)[kNB][KS],
                   f32x4 (&acc)[kNB][MT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[nb][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const half8 a = lds[(frag0 + mt * KS + s) * 64 + lane];
#pragma unroll
            for (int nb = 0; nb < kNB; ++nb) acc[nb][mt] = mfma(a, b[nb][s], acc[nb][mt]);
        }
    }
}

// accumulator tiles -> activation -> permuted B operand of the next product
template <int MT, int KS>
NGP_DEV void pack_act(const f32x4 (&acc)[kNB][MT], uint32_t act, half8 (&out)[kNB][KS]) {
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int mt = 2 * s + (j >> 2);
                v[j] = mt < MT ? (ngp_half)act_fwd(act, acc[nb][mt][j & 3]) : (ngp_half)0.0f;
            }
            out[nb][s] = v;
        }
}

// load a [rows, width] fp16 row-major block as natural-K B operands
template <int KS>
NGP_DEV void load_rows(const ngp_half* __restrict__ src, uint32_t width, uint32_t row0, uint32_t B,
                       half8 (&out)[kNB][KS]) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) {
        const uint32_t row = row0 + nb * 16 + c;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint32_t col = 32 * s + 8 * g;
            half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
            if (row < B && col < width) v = *reinterpret_cast<const half8*>(src + (size_t)row * width + col);
            out[nb][s] = v;
        }
    }
}

// store accumulator tiles (optionally activated) as fp16 rows [row][16 mt + 4g .. +3]
template <int MT>
NGP_DEV void store_tiles(ngp_half* __restrict__ dst, uint32_t width, uint32_t row0, uint32_t B,
                         const f32x4 (&acc)[kNB][MT], uint32_t act) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) {
        const uint32_t row = row0 + nb * 16 + c;
        if (row >= B) continue;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const uint32_t col = 16 * mt + 4 * g;
            if (col >= width) continue;
            half4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (ngp_half)act_fwd(act, acc[nb][mt][r]);
            *reinterpret_cast<half4*>(dst + (size_t)row * width + col) = v;
        }
    }
}

// ---- forward ----------------------------------------------------------------
template <int W, int IN_KS, int NH>
__global__ void __launch_bounds__(kThreads)
k_mlp_fwd(const ngp_half* __restrict__ inputs, const ngp_half* __restrict__ weights,
          ngp_half* __restrict__ outputs, ngp_half* __restrict__ fwd_buf, uint32_t B,
          uint32_t in_dim, uint32_t act, uint32_t out_act) {
    using N = Net<W, IN_KS, NH>;
    extern __shared__ half8 lds[];
    for (int q = 0; q < N::NMAT; ++q) build_frags(lds, weights, fwd_desc<W, IN_KS, NH>(q, in_dim), false);
    __syncthreads();

    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    for (uint32_t chunk = blockIdx.x * kWaves + wave; chunk < nchunks; chunk += gridDim.x * kWaves) {
        const uint32_t row0 = chunk * 16 * kNB;
        half8 x[kNB][IN_KS];
        load_rows<IN_KS>(inputs, in_dim, row0, B, x);

        f32x4 acc[kNB][N::MTW];
        half8 h[kNB][N::KSW];
        dense<N::MTW, IN_KS>(lds, fwd_desc<W, IN_KS, NH>(0, in_dim).frag0, x, acc);
        if (fwd_buf) store_tiles<N::MTW>(fwd_buf, W, row0, B, acc, act);
        pack_act<N::MTW, N::KSW>(acc, act, h);
#pragma unroll
        for (int q = 1; q <= NH; ++q) {
            dense<N::MTW, N::KSW>(lds, fwd_desc<W, IN_KS, NH>(q, in_dim).frag0, h, acc);
            if (fwd_buf) store_tiles<N::MTW>(fwd_buf + (size_t)q * B * W, W, row0, B, acc, act);
            pack_act<N::MTW, N::KSW>(acc, act, h);
        }
        f32x4 o[kNB][1];
        dense<1, N::KSW>(lds, fwd_desc<W, IN_KS, NH>(NH + 1, in_dim).frag0, h, o);
        if (outputs) store_tiles<1>(outputs, kOut, row0, B, o, out_act);
    }
}

// ---- backward ---------------------------------------------------------------
// Per-wave transpose tile: rows = units, 32 samples per row (+pad).
template <int KS, bool PERM>
NGP_DEV void write_transposed(ngp_half* __restrict__ tile, const half8 (&v)[kNB][KS], uint32_t rows) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t u = 32 * s + (PERM ? perm_unit(g, j) : 8 * g + j);
                if (u < rows) tile[u * kScratchLd + nb * 16 + c] = v[nb][s][j];
            }
}

// dW[o][i] (MO x MI tiles of 16x16) += dT^T-rows · hT-rows over the 32 samples
template <int MO, int MI>
NGP_DEV void dw_accum(const ngp_half* __restrict__ dT, const ngp_half* __restrict__ hT,
                      f32x4 (&acc)[MO][MI]) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    half8 a[MO], b[MI];
#pragma unroll
    for (int m = 0; m < MO; ++m) a[m] = *reinterpret_cast<const half8*>(dT + (16 * m + c) * kScratchLd + 8 * g);
#pragma unroll
    for (int n = 0; n < MI; ++n) b[n] = *reinterpret_cast<const half8*>(hT + (16 * n + c) * kScratchLd + 8 * g);
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int n = 0; n < MI; ++n) acc[m][n] = mfma(a[m], b[n], acc[m][n]);
}

// delta (C layout, MT tiles) * act'(post-activation h, permuted B form) -> permuted B form
template <int MT, int KS>
NGP_DEV void pack_delta(const f32x4 (&acc)[kNB][MT], const half8 (&h)[kNB][KS], uint32_t act,
                        half8 (&out)[kNB][KS]) {
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int mt = 2 * s + (j >> 2);
                v[j] = mt < MT ? (ngp_half)act_bwd(act, acc[nb][mt][j & 3], (float)h[nb][s][j]) : (ngp_half)0.0f;
            }
            out[nb][s] = v;
        }
}

// Sum the workgroup's per-wave dW tiles (LDS fp32 atomics) and publish one slab row.
template <int MO, int MI>
NGP_DEV void flush_dw(const f32x4 (&acc)[MO][MI], float* __restrict__ red, uint32_t in_w,
                      uint32_t out_w, float* __restrict__ slab_row) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const uint32_t n = out_w * in_w;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) red[t] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int k = 0; k < MI; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t o = 16 * m + 4 * g + r, i = 16 * k + c;
                if (o < out_w && i < in_w) atomicAdd(&red[o * in_w + i], acc[m][k][r]);
            }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) slab_row[t] = red[t];
}

template <int W, int IN_KS, int NH>
struct BwdLds {
    using N = Net<W, IN_KS, NH>;
    static constexpr int FRAGS = N::FWD_FRAGS + N::BWD_FRAGS;
    static constexpr int TILE_ROWS = (W > 32 * IN_KS ? W : 32 * IN_KS);
    static constexpr size_t frag_bytes = (size_t)FRAGS * 64 * 16;
    static constexpr size_t tile_bytes = (size_t)kWaves * 2 * TILE_ROWS * kScratchLd * 2;
    static constexpr size_t red_bytes = (size_t)W * (W > 32 * IN_KS ? W : 32 * IN_KS) * 4;
    static constexpr size_t scratch_bytes = tile_bytes > red_bytes ? tile_bytes : red_bytes;
    static constexpr size_t total = frag_bytes + scratch_bytes;
};

// Shared state of one backward launch.
struct BwdCtx {
    const ngp_half* grad;
    const ngp_half* inputs;
    ngp_half* grad_inputs;
    const half8* fr;
    ngp_half* dT;
    ngp_half* hT;
    float* red;
    float* slab_row;
    uint32_t B, in_dim, act, nchunks;
};

// One pass for matmul P (compile-time): recompute the forward, propagate the
// deltas down to matmul P, accumulate dW_P over every chunk this wave owns,
// then publish the workgroup's dW_P. Recurses to P-1.
template <int W, int IN_KS, int NH, int P>
NGP_DEV void bwd_pass(const BwdCtx& cx) {
    using N = Net<W, IN_KS, NH>;
    constexpr int LAST = N::NMAT - 1;
    constexpr int MO = P == LAST ? 1 : N::MTW;    // 16-row tiles over matmul P's outputs
    constexpr int MI = P == 0 ? N::IN_MT : N::MTW; // 16-col tiles over matmul P's inputs
    const uint32_t wave = threadIdx.x >> 6;

    f32x4 dw[MO][MI];
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int k = 0; k < MI; ++k) dw[m][k] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (uint32_t chunk = blockIdx.x * kWaves + wave; chunk < cx.nchunks; chunk += gridDim.x * kWaves) {
        const uint32_t row0 = chunk * 16 * kNB;
        half8 x[kNB][IN_KS];
        load_rows<IN_KS>(cx.inputs, cx.in_dim, row0, cx.B, x);
        // recompute the post-activations of every hidden layer
        half8 h[NH + 1][kNB][N::KSW];
        f32x4 acc[kNB][N::MTW];
        dense<N::MTW, IN_KS>(cx.fr, fwd_desc<W, IN_KS, NH>(0, cx.in_dim).frag0, x, acc);
        pack_act<N::MTW, N::KSW>(acc, cx.act, h[0]);
#pragma unroll
        for (int q = 1; q <= NH; ++q) {
            dense<N::MTW, N::KSW>(cx.fr, fwd_desc<W, IN_KS, NH>(q, cx.in_dim).frag0, h[q - 1], acc);
            pack_act<N::MTW, N::KSW>(acc, cx.act, h[q]);
        }
        // output gradient (output activation ignored, ffmlp.cu:783): natural K order
        half8 dout[kNB][1];
        load_rows<1>(cx.grad, kOut, row0, cx.B, dout);

        if constexpr (P == LAST) {
            write_transposed<1, false>(cx.dT, dout, kOut);
            write_transposed<N::KSW, true>(cx.hT, h[NH], W);
            dw_accum<MO, MI>(cx.dT, cx.hT, dw);
        } else {
            half8 d[kNB][N::KSW];  // delta of a matmul's (pre-activation) output, permuted B form
            dense<N::MTW, 1>(cx.fr, bwd_desc<W, IN_KS, NH>(LAST, cx.in_dim).frag0 + N::FWD_FRAGS, dout, acc);
            pack_delta<N::MTW, N::KSW>(acc, h[NH], cx.act, d);
#pragma unroll
            for (int q = NH; q > P; --q) {
                dense<N::MTW, N::KSW>(cx.fr, bwd_desc<W, IN_KS, NH>(q, cx.in_dim).frag0 + N::FWD_FRAGS, d, acc);
                pack_delta<N::MTW, N::KSW>(acc, h[q - 1], cx.act, d);
            }
            write_transposed<N::KSW, true>(cx.dT, d, W);
            if constexpr (P == 0) write_transposed<IN_KS, false>(cx.hT, x, 32 * IN_KS);
            else write_transposed<N::KSW, true>(cx.hT, h[P - 1], W);
            dw_accum<MO, MI>(cx.dT, cx.hT, dw);
            if constexpr (P == 0) {
                if (cx.grad_inputs) {
                    f32x4 gi[kNB][N::IN_MT];
                    dense<N::IN_MT, N::KSW>(cx.fr, bwd_desc<W, IN_KS, NH>(0, cx.in_dim).frag0 + N::FWD_FRAGS, d, gi);
                    store_tiles<N::IN_MT>(cx.grad_inputs, cx.in_dim, row0, cx.B, gi, kNone);
                }
            }
        }
    }
    const MatDesc mf = fwd_desc<W, IN_KS, NH>(P, cx.in_dim);
    flush_dw<MO, MI>(dw, cx.red, mf.in, mf.out, cx.slab_row + mf.off);
    __syncthreads();
    if constexpr (P > 0) bwd_pass<W, IN_KS, NH, P - 1>(cx);
}

template <int W, int IN_KS, int NH>
__global__ void __launch_bounds__(kThreads)
k_mlp_bwd(const ngp_half* __restrict__ grad, const ngp_half* __restrict__ inputs,
          const ngp_half* __restrict__ weights, ngp_half* __restrict__ grad_inputs,
          float* __restrict__ slab, uint32_t nparams, uint32_t B, uint32_t in_dim, uint32_t act) {
    using N = Net<W, IN_KS, NH>;
    using L = BwdLds<W, IN_KS, NH>;
    extern __shared__ half8 lds[];
    ngp_half* scratch = reinterpret_cast<ngp_half*>(reinterpret_cast<char*>(lds) + L::frag_bytes);

    for (int q = 0; q < N::NMAT; ++q) {
        build_frags(lds, weights, fwd_desc<W, IN_KS, NH>(q, in_dim), false);
        MatDesc mb = bwd_desc<W, IN_KS, NH>(q, in_dim);
        mb.frag0 += N::FWD_FRAGS;
        build_frags(lds, weights, mb, true);
    }
    __syncthreads();

    const uint32_t wave = threadIdx.x >> 6;
    BwdCtx cx;
    cx.grad = grad;
    cx.inputs = inputs;
    cx.grad_inputs = grad_inputs;
    cx.fr = lds;
    cx.dT = scratch + (size_t)wave * 2 * L::TILE_ROWS * kScratchLd;
    cx.hT = cx.dT + (size_t)L::TILE_ROWS * kScratchLd;
    cx.red = reinterpret_cast<float*>(scratch);
    cx.slab_row = slab + (size_t)blockIdx.x * nparams;
    cx.B = B;
    cx.in_dim = in_dim;
    cx.act = act;
    cx.nchunks = ngp_div_up(B, 16 * kNB);
    bwd_pass<W, IN_KS, NH, N::NMAT - 1>(cx);
}

template <typename OUT>
__global__ void __launch_bounds__(256)
k_slab_reduce(const float* __restrict__ slab, uint32_t rows, uint32_t n, OUT* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.0f;
    for (uint32_t r = 0; r < rows; ++r) s += slab[(size_t)r * n + i];
    out[i] = (OUT)s;
}

// ---- host dispatch ----------------------------------------------------------
uint32_t num_params(uint32_t in_dim, uint32_t hidden, uint32_t num_layers) {
    return hidden * (in_dim + hidden * (num_layers - 1) + kOut);
}

uint32_t bwd_blocks(uint32_t B) {
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t nb = ngp_div_up(nchunks, kWaves);
    return nb < kMaxBwdBlocks ? nb : kMaxBwdBlocks;
}

int check_shape(uint32_t B, uint32_t in_dim, uint32_t out_dim, uint32_t hidden, uint32_t num_layers) {
    NGP_REQUIRE(hidden == 32 || hidden == 64, NGP_ERR_UNSUPPORTED,
                "hidden_dim should in [32, 64] on this build, got %u", hidden);
    NGP_REQUIRE(in_dim > 0 && in_dim % 16 == 0 && in_dim <= 64, NGP_ERR_UNSUPPORTED,
                "FFMLP input_dim should be 16 * m (m > 0) and <= 64, got %u", in_dim);
    NGP_REQUIRE(out_dim == kOut, NGP_ERR_UNSUPPORTED, "FFMLP padded output_dim must be 16, got %u", out_dim);
    NGP_REQUIRE(num_layers >= 2 && num_layers <= 4, NGP_ERR_UNSUPPORTED,
                "FFMLP num_layers must be in [2, 4] on this build, got %u", num_layers);
    (void)B;
    return NGP_OK;
}

template <int W, int IN_KS, int NH>
int launch_fwd(const void* in, const void* w, uint32_t B, uint32_t in_dim, uint32_t act,
               uint32_t out_act, void* fwd_buf, void* out, hipStream_t st) {
    using N = Net<W, IN_KS, NH>;
    const size_t lds = (size_t)N::FWD_FRAGS * 64 * 16;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t blocks = ngp_div_up(nchunks, kWaves);
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) return NGP_OK;
    hipLaunchKernelGGL((k_mlp_fwd<W, IN_KS, NH>), dim3(blocks), dim3(kThreads), lds, st,
                       (const ngp_half*)in, (const ngp_half*)w, (ngp_half*)out, (ngp_half*)fwd_buf,
                       B, in_dim, act, out_act);
    return ngp_check_launch("ffmlp_forward");
}

template <int W, int IN_KS, int NH>
int launch_bwd(const void* grad, const void* in, const void* w, uint32_t B, uint32_t in_dim,
               uint32_t act, void* grad_in, void* gw, int32_t gw_dtype, float* slab,
               hipStream_t st) {
    using L = BwdLds<W, IN_KS, NH>;
    const uint32_t blocks = bwd_blocks(B);
    const uint32_t np = num_params(in_dim, W, NH + 1);
    if (blocks == 0) return NGP_OK;
    hipLaunchKernelGGL((k_mlp_bwd<W, IN_KS, NH>), dim3(blocks), dim3(kThreads), L::total, st,
                       (const ngp_half*)grad, (const ngp_half*)in, (const ngp_half*)w,
                       (ngp_half*)grad_in, slab, np, B, in_dim, act);
    if (gw_dtype == NGP_DTYPE_F16) {
        hipLaunchKernelGGL((k_slab_reduce<ngp_half>), dim3(ngp_div_up(np, 256)), dim3(256), 0, st,
                           (const float*)slab, blocks, np, (ngp_half*)gw);
    } else {
        hipLaunchKernelGGL((k_slab_reduce<float>), dim3(ngp_div_up(np, 256)), dim3(256), 0, st,
                           (const float*)slab, blocks, np, (float*)gw);
    }
    return ngp_check_launch("ffmlp_backward");
}

#define NGP_MLP_DISPATCH(FN, ...)                                                              \
    do {                                                                                        \
        const int ks = (int)((in_dim + 31) / 32);                                                \
        const int nh = (int)num_layers - 1;                                                     \
        switch (hidden_dim) {                                                                   \
            case 32:                                                                            \
                if (ks == 1) { if (nh == 1) return FN<32, 1, 1>(__VA_ARGS__); if (nh == 2) return FN<32, 1, 2>(__VA_ARGS__); return FN<32, 1, 3>(__VA_ARGS__); } \
                else { if (nh == 1) return FN<32, 2, 1>(__VA_ARGS__); if (nh == 2) return FN<32, 2, 2>(__VA_ARGS__); return FN<32, 2, 3>(__VA_ARGS__); } \
            case 64:                                                                            \
                if (ks == 1) { if (nh == 1) return FN<64, 1, 1>(__VA_ARGS__); if (nh == 2) return FN<64, 1, 2>(__VA_ARGS__); return FN<64, 1, 3>(__VA_ARGS__); } \
                else { if (nh == 1) return FN<64, 2, 1>(__VA_ARGS__); if (nh == 2) return FN<64, 2, 2>(__VA_ARGS__); return FN<64, 2, 3>(__VA_ARGS__); } \
            default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "unsupported hidden_dim");       \
        }                                                                                       \
    } while (0)

}  // namespace

extern "C" int ngp_ffmlp_forward(const void* inputs, const void* weights, uint32_t B,
                                 uint32_t in_dim, uint32_t output_dim, uint32_t hidden_dim,
                                 uint32_t num_layers, uint32_t activation,
                                 uint32_t output_activation, void* forward_buffer, void* outputs,
                                 void* stream) {
    if (int e = check_shape(B, in_dim, output_dim, hidden_dim, num_layers)) return e;
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    NGP_MLP_DISPATCH(launch_fwd, inputs, weights, B, in_dim, activation, output_activation,
                     forward_buffer, outputs, st);
}

extern "C" int ngp_ffmlp_inference(const void* inputs, const void* weights, uint32_t B,
                                   uint32_t input_dim, uint32_t output_dim, uint32_t hidden_dim,
                                   uint32_t num_layers, uint32_t activation,
                                   uint32_t output_activation, void* inference_buffer,
                                   void* outputs, void* stream) {
    (void)inference_buffer;
    return ngp_ffmlp_forward(inputs, weights, B, input_dim, output_dim, hidden_dim, num_layers,
                             activation, output_activation, nullptr, outputs, stream);
}

extern "C" size_t ngp_ffmlp_backward_workspace_bytes(uint32_t B, uint32_t input_dim,
                                                     uint32_t output_dim, uint32_t hidden_dim,
                                                     uint32_t num_layers) {
    (void)output_dim;
    return (size_t)bwd_blocks(B) * num_params(input_dim, hidden_dim, num_layers) * sizeof(float);
}

extern "C" int ngp_ffmlp_backward(const void* grad, const void* inputs, const void* weights,
                                  const void* forward_buffer, uint32_t B, uint32_t in_dim,
                                  uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                                  uint32_t activation, uint32_t output_activation,
                                  int32_t calc_grad_inputs, void* backward_buffer,
                                  void* grad_inputs, void* grad_weights, int32_t gw_dtype,
                                  void* workspace, size_t workspace_bytes, void* stream) {
    (void)forward_buffer;
    (void)backward_buffer;
    (void)output_activation;
    if (int e = check_shape(B, in_dim, output_dim, hidden_dim, num_layers)) return e;
    NGP_REQUIRE(gw_dtype == NGP_DTYPE_F16 || gw_dtype == NGP_DTYPE_F32, NGP_ERR_ARG,
                "grad_weights must be float16 or float32");
    if (B == 0) return NGP_OK;
    const size_t need = ngp_ffmlp_backward_workspace_bytes(B, in_dim, output_dim, hidden_dim, num_layers);
    NGP_REQUIRE(workspace && workspace_bytes >= need, NGP_ERR_ARG,
                "ffmlp_backward: workspace of %zu bytes required, got %zu", need, workspace_bytes);
    hipStream_t st = ngp_stream(stream);
    void* gi = calc_grad_inputs ? grad_inputs : nullptr;
    NGP_MLP_DISPATCH(launch_bwd, grad, inputs, weights, B, in_dim, activation, gi, grad_weights,
                     gw_dtype, (float*)workspace, st);
}

extern "C" int ngp_ffmlp_allocate_splitk(size_t size) { (void)size; return NGP_OK; }
extern "C" int ngp_ffmlp_free_splitk(void) { return NGP_OK; }
