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
#include "ffmlp_pack.h"
#include "ngp_common.h"
#include "ngp_reduce.h"
#include "sh_basis.h"

#include <cstdlib>
#include <type_traits>

namespace {

using ngp_pack::half8;
using ngp_pack::MatDesc;
using ngp_pack::PackJob;
using ngp_pack::PackJobs;
using ngp_pack::build_frags;
using ngp_pack::kMaxPackJobs;
using ngp_pack::perm_unit;
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;  // forward: waves per workgroup (sharing one fragment copy)
constexpr int kThreads = kWaves * 64;
// Backward: waves per workgroup sharing one fragment image. The dW tiles
// live in registers for the whole chunk loop (176 of them for the colour
// network), which leaves room for one wave per SIMD: at 8 waves per workgroup
// (two per SIMD, 256 registers each) the compiler spills 362 (colour) / 78
// (sigma) VGPRs.
constexpr int kBwdWaves = 4;
constexpr int kBwdThreads = kBwdWaves * 64;
static_assert(kBwdWaves % 2 == 0 && kBwdWaves <= 16, "the dW fold pairs waves (two LDS images)");
constexpr int kNB = 2;          // 16-sample column blocks per wave step (32 samples)
static_assert(16 * kNB == ngp_reduce::kBwdChunkRows, "the reduce's live-row slab count assumes 32-row chunks");
constexpr int kOut = 16;        // padded output width (FFMLP pads to 16)
// Per-wave staging tiles of the dW products: [32 samples][units], row pitch
// 80 halves (40 dwords: the 8 rows one 32-lane half of a transposed read
// touches land on 8 distinct 8-dword bank groups, i.e. conflict-free).
constexpr int kTileLd = 80;
constexpr int kTileRows = 32;
constexpr uint32_t kMaxBwdBlocks = 256;

// Workgroup barrier that orders LDS only: unlike __syncthreads() it does not
// wait for the wave's outstanding global loads (the next chunk's prefetch).
NGP_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

NGP_DEV f32x4 mfma(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Fragment image -> LDS with every load of a thread issued before its first
// store (a load/store pair per iteration exposed the load latency ~12 times).
// The loads are unconditional (a partial last round reads a clamped index):
// a load under a divergent branch leaves the compiler unsure how many memory
// operations are outstanding, so it waited vmcnt(0) after each one and the
// copy took one round trip per load (~9 K cycles, tools/fwd_stamps.py).
template <int FRAGS, int THREADS>
NGP_DEV void copy_frags(half8* __restrict__ lds, const half8* __restrict__ image) {
    constexpr int TOTAL = FRAGS * 64, PER = (TOTAL + THREADS - 1) / THREADS;
    half8 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        v[k] = image[(k + 1) * THREADS <= TOTAL ? t : min(t, TOTAL - 1)];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        if ((k + 1) * THREADS <= TOTAL || t < TOTAL) lds[t] = v[k];
    }
}

// An image copied by `nthr` threads of the workgroup (tid in [0, nthr)), four
// loads of a thread in flight per round: the NeRF backward's idle waves copy
// the sigma image during the colour pass.
template <int FRAGS>
NGP_DEV void copy_frags_part(half8* __restrict__ lds, const half8* __restrict__ image, uint32_t tid, uint32_t nthr) {
    constexpr uint32_t TOTAL = FRAGS * 64;
    for (uint32_t i0 = tid; i0 < TOTAL; i0 += 4 * nthr) {
        half8 v[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) v[k] = image[min(i0 + k * nthr, TOTAL - 1)];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (i0 + k * nthr < TOTAL) lds[i0 + k * nthr] = v[k];
    }
}

// Two images copied with every load of both issued before the first LDS
// store: one round trip instead of two (the NeRF backward's prologue).
template <int F1, int F2, int THREADS>
NGP_DEV void copy_frags2(half8* __restrict__ lds1, const half8* __restrict__ image1, half8* __restrict__ lds2,
                         const half8* __restrict__ image2) {
    constexpr int T1 = F1 * 64, P1 = (T1 + THREADS - 1) / THREADS;
    constexpr int T2 = F2 * 64, P2 = (T2 + THREADS - 1) / THREADS;
    half8 v1[P1], v2[P2];
#pragma unroll
    for (int k = 0; k < P1; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        v1[k] = image1[(k + 1) * THREADS <= T1 ? t : min(t, T1 - 1)];
    }
#pragma unroll
    for (int k = 0; k < P2; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        v2[k] = image2[(k + 1) * THREADS <= T2 ? t : min(t, T2 - 1)];
    }
#pragma unroll
    for (int k = 0; k < P1; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        if ((k + 1) * THREADS <= T1 || t < T1) lds1[t] = v1[k];
    }
#pragma unroll
    for (int k = 0; k < P2; ++k) {
        const int t = k * THREADS + (int)threadIdx.x;
        if ((k + 1) * THREADS <= T2 || t < T2) lds2[t] = v2[k];
    }
}

// a row index that is always readable (rows past B read row B - 1 and the
// caller zeroes the value): loads without branches, see copy_frags
NGP_DEV uint32_t clamp_row(uint32_t row, uint32_t B) { return row < B ? row : (B ? B - 1 : 0u); }
// A row list (the live rows of a step, see ngp_nerf_composite_loss_live): row r of
// the B rows an MLP call processes is map[r]; null: r itself.
NGP_DEV uint32_t map_row(const int32_t* map, uint32_t r) { return map ? (uint32_t)map[r] : r; }

// Activation enum of ffmlp.py:89-96 / utils.h:29-37.
enum Act : uint32_t { kReLU = 0, kExp = 1, kSine = 2, kSigmoid = 3, kSquareplus = 4, kSoftplus = 5, kNone = 6 };
constexpr float kKAct = 10.0f;

__device__ __attribute__((noinline)) float act_fwd(uint32_t a, float x) {
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
__device__ __attribute__((noinline)) float act_bwd(uint32_t a, float g, float y) {
    switch (a) {
        case kReLU: return y > 0.0f ? g : 0.0f;
        case kExp: return g * y;
        case kSigmoid: return g * (y * (1.0f - y));
        case kSquareplus: { const float t = y * kKAct; return g * (t * t / (t * t + 1)); }
        case kSoftplus: return g * (1.0f - expf(-y * kKAct));
        default: return g;  // None; Sine has no backward in the reference (utils.h:552-556)
    }
}

// Activation policies: the NeRF networks use ReLU hidden / no output
// activation, which compile to inline VALU; any other enum value goes through
// the out-of-line generic functions above (keeps the unrolled tile loops small:
// inlining every activation into every element made the kernels ~45k
// instructions and I-cache bound).
struct ActReLU {
    NGP_DEV float fwd(float x) const { return x > 0.0f ? x : 0.0f; }
    NGP_DEV float bwd(float g, float y) const { return y > 0.0f ? g : 0.0f; }
};
struct ActNone {
    NGP_DEV float fwd(float x) const { return x; }
    NGP_DEV float bwd(float g, float) const { return g; }
};
struct ActAny {
    uint32_t a;
    NGP_DEV float fwd(float x) const { return act_fwd(a, x); }
    NGP_DEV float bwd(float g, float y) const { return act_bwd(a, g, y); }
};

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
__host__ __device__ inline MatDesc fwd_desc(int q, uint32_t in_dim) {
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
__host__ __device__ inline MatDesc bwd_desc(int q, uint32_t in_dim) {
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
template <int MT, int KS, int NB>
NGP_DEV void dense(const half8* __restrict__ lds, uint32_t frag0, const half8 (&b)[NB][KS],
                   f32x4 (&acc)[NB][MT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[nb][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const half8 a = lds[(frag0 + mt * KS + s) * 64 + lane];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) acc[nb][mt] = mfma(a, b[nb][s], acc[nb][mt]);
        }
    }
}

// accumulator tiles -> activation -> permuted B operand of the next product
template <int MT, int KS, typename ACT, int NB>
NGP_DEV void pack_act(const f32x4 (&acc)[NB][MT], ACT act, half8 (&out)[NB][KS]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int mt = 2 * s + (j >> 2);
                v[j] = mt < MT ? (ngp_half)act.fwd(acc[nb][mt][j & 3]) : (ngp_half)0.0f;
            }
            out[nb][s] = v;
        }
}

// ReLU policy: round each pair of accumulators to fp16 (RNE, one packed
// conversion), then a packed signed 16-bit max with 0: every negative value,
// -0 included, has the sign bit set and becomes +0. That is max(x, 0) rounded,
// for every non-NaN x (a NaN with the sign bit clear stays NaN, as torch's
// ReLU keeps it), at 2 VALU per 2 values; the fp32 compare/select before the
// conversion was ~2 per value (a fifth of k_nerf_fwd's instructions).
typedef short ngp_short2 __attribute__((ext_vector_type(2)));
typedef float ngp_float2 __attribute__((ext_vector_type(2)));
template <int MT, int KS, int NB>
NGP_DEV void pack_act(const f32x4 (&acc)[NB][MT], ActReLU, half8 (&out)[NB][KS]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int mt = 2 * s + (j >> 1), r = 2 * (j & 1);
                ngp_short2 q = ngp_short2{0, 0};
                if (mt < MT) {
                    const ngp_half2 h = __builtin_convertvector(ngp_float2{acc[nb][mt][r], acc[nb][mt][r + 1]}, ngp_half2);
                    q = __builtin_elementwise_max(__builtin_bit_cast(ngp_short2, h), ngp_short2{0, 0});
                }
                const ngp_half2 h = __builtin_bit_cast(ngp_half2, q);
                v[2 * j] = h[0];
                v[2 * j + 1] = h[1];
            }
            out[nb][s] = v;
        }
}

// load a [rows, width] fp16 row-major block as natural-K B operands
template <int KS, int NB>
NGP_DEV void load_rows(const ngp_half* __restrict__ src, uint32_t width, uint32_t row0, uint32_t B,
                       half8 (&out)[NB][KS], const int32_t* map = nullptr) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        const uint32_t row = row0 + nb * 16 + c;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint32_t col = 32 * s + 8 * g;
            const bool ok = row < B && col < width;
            const half8 v = *reinterpret_cast<const half8*>(src + (size_t)map_row(map, clamp_row(row, B)) * width +
                                                            (col < width ? col : 0u));
            const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            out[nb][s] = ok ? v : z;
        }
    }
}

// First-layer input loaders (natural-K B operands).
struct InRowMajor {  // [B, width] row-major
    const int32_t* map = nullptr;  // row list, or null
    template <int KS, int NB>
    NGP_DEV void operator()(const ngp_half* __restrict__ src, uint32_t width, uint32_t row0, uint32_t B,
                            half8 (&out)[NB][KS]) const {
        load_rows<KS>(src, width, row0, B, out, map);
    }
};
// [width / 2][ld][2]: column pairs stored pair-major, the hash grid's
// [L, B, C = 2] layout, so the grid kernels read and write whole lines per
// level. Lane (g, c) gathers its 8 columns as 4 pairs; the 16 lanes of a
// group read 64 contiguous bytes per pair.
struct InPairMajor {
    uint32_t ld;  // allocated rows
    const int32_t* map = nullptr;  // row list, or null
    template <int KS, int NB>
    NGP_DEV void operator()(const ngp_half* __restrict__ src, uint32_t width, uint32_t row0, uint32_t B,
                            half8 (&out)[NB][KS]) const {
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            const uint32_t row = row0 + nb * 16 + c;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint32_t col = 32 * s + 8 * g;
                const bool ok = row < B && col < width;
                const uint32_t rr = map_row(map, clamp_row(row, B)), cc = col < width ? col : 0u;
                half8 v;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const ngp_half2 h = *reinterpret_cast<const ngp_half2*>(src + ((size_t)(cc / 2 + p) * ld + rr) * 2);
                    v[2 * p] = ok ? h[0] : (ngp_half)0.0f;
                    v[2 * p + 1] = ok ? h[1] : (ngp_half)0.0f;
                }
                out[nb][s] = v;
            }
        }
    }
};

// The forward kernels' pair-major loads (k_density_fwd, k_nerf_fwd): one
// buffer descriptor over the [width / 2][ld] pairs, the lane's pair row in the
// 32-bit voffset and each pair's distance (p ld 4 bytes) in an SGPR soffset:
// no 64-bit address, clamp or select per load (InPairMajor spent ~30 VALU per
// 32-row chunk on them). Rows are not masked: a forward's columns (samples)
// are independent and its epilogues store rows < B only, so a row in [B, ld)
// may hold anything, and a row past the allocation reads 0 (range check).
struct InPairMajorFwd {
    uint32_t ld;  // allocated rows
    template <int KS, int NB>
    NGP_DEV void operator()(const ngp_half* __restrict__ src, uint32_t width, uint32_t row0, uint32_t,
                            half8 (&out)[NB][KS]) const {
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<ngp_half*>(src), (short)0, (int)(width / 2 * ld * 4u), 0x00020000);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint32_t col = 32 * s + 8 * g;
                const int voff = (int)(((col / 2) * ld + row0 + nb * 16 + c) * 4u);
                uint32_t w[4];
#pragma unroll
                for (int p = 0; p < 4; ++p) w[p] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, (int)(p * ld * 4u), 0);
                const half8 v = __builtin_bit_cast(half8, (uint4{w[0], w[1], w[2], w[3]}));
                out[nb][s] = col < width ? v : half8{0, 0, 0, 0, 0, 0, 0, 0};
            }
        }
    }
};

// store accumulator tiles (optionally activated) as fp16 rows [row][16 mt + 4g .. +3]
template <int MT, typename ACT, int NB>
NGP_DEV void store_tiles(ngp_half* __restrict__ dst, uint32_t width, uint32_t row0, uint32_t B,
                         const f32x4 (&acc)[NB][MT], ACT act) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        const uint32_t row = row0 + nb * 16 + c;
        if (row >= B) continue;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const uint32_t col = 16 * mt + 4 * g;
            if (col >= width) continue;
            half4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (ngp_half)act.fwd(acc[nb][mt][r]);
            *reinterpret_cast<half4*>(dst + (size_t)row * width + col) = v;
        }
    }
}

// ---- forward ----------------------------------------------------------------
// Output epilogues: the plain [B, 16] store, or the NeRF sigma network's
// glue (nerf/network_ff.py:61-68): h [B,16] half, sigma = density_scale *
// trunc_exp(h[:,0]) (activation.py, fp32 exp of the half value) and
// color_in [B,32] = [half(SH4(dir)) | h[:,1:16] | 0] for the color network.
struct EpiStore {
    ngp_half* out;
    template <typename FO>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], FO out_act) const {
        if (out) store_tiles<1>(out, kOut, row0, B, o, out_act);
    }
};

#ifdef NGP_STAMPS  // diagnostic build only (tools/accum_stamps.py, tools/fwd_stamps.py): per-wave phase clocks
__device__ unsigned long long* g_mlp_stamps;
// k_nerf_fwd: 16 slots per wave after the backward's 2 x 2048 waves; W-suffixed
// stamps first wait for the wave's outstanding memory operations
#define FSTAMP(slot, v) do { if (g_mlp_stamps && (threadIdx.x & 63) == 0) g_mlp_stamps[(size_t)2 * 2048 * 16 + ((size_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * 16 + (slot)] = (v); } while (0)
#define FSTAMPW(slot) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); FSTAMP(slot, __builtin_amdgcn_s_memtime()); } while (0)
#define FRSTAMP(slot) FSTAMP(slot, __builtin_amdgcn_s_memrealtime())
#else
#define FSTAMPW(slot) do { } while (0)
#define FRSTAMP(slot) do { } while (0)
#endif
// (kWaves: the forward's waves per workgroup)

struct EpiNerfSigma {
    ngp_half* h;
    float* sigma;
    ngp_half* color_in;
    const float* dirs;
    float density_scale;
    template <typename FO>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], FO out_act) const {
        half8 unused[kNB][1];
        float dv[kNB][3];
        load_dirs(row0, B, dv);
        run<false>(row0, B, o, out_act, unused, dv);
    }
    // the chunk's view directions (row c of lane group g: every group loads
    // its row's), issued early so the SH does not wait a memory round trip
    NGP_DEV void load_dirs(uint32_t row0, uint32_t B, float (&dv)[kNB][3]) const {
        const int c = threadIdx.x & 15;
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) {
            const uint32_t row = row0 + nb * 16 + c;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float d = dirs[(size_t)clamp_row(row, B) * 3 + k];
                dv[nb][k] = row < B ? d : 0.0f;
            }
        }
    }
    // OPERAND: also hand back color_in's rows as the colour network's
    // first-layer B operand (load_rows' layout: lane (g, c) holds columns
    // 8g .. 8g+7 of row c), the same fp16 values the store writes.
    template <bool OPERAND, typename FO>
    NGP_DEV void run(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], FO out_act, half8 (&xc)[kNB][1],
                     const float (&dv)[kNB][3]) const {
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) {
            const uint32_t row = row0 + nb * 16 + c;
            half4 v;  // h[row][4g .. 4g+3]
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (ngp_half)out_act.fwd(o[nb][0][r]);
            // h[row][4g+4] from the next lane group (color_in shifts h by one column)
            const uint32_t nx = __shfl((uint32_t)__builtin_bit_cast(uint16_t, v[0]), lane + 16, 64);
            const ngp_half next = g < 3 ? __builtin_bit_cast(ngp_half, (uint16_t)nx) : (ngp_half)0.0f;
            const half4 q = half4{v[1], v[2], v[3], next};  // color_in[row][16 + 4g .. 16 + 4g + 3]
            uint2 qq[2];  // lane groups 2 and 3 take color_in columns 16..23 / 24..31 from groups 0,1 / 2,3
            if constexpr (OPERAND) {
                const uint2 qm = __builtin_bit_cast(uint2, q);
                const int src = (g >= 2 ? 2 * (g - 2) : 0) * 16 + c;
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    qq[k] = uint2{(uint32_t)__shfl((int)qm.x, src + 16 * k, 64), (uint32_t)__shfl((int)qm.y, src + 16 * k, 64)};
                xc[nb][0] = half8{0, 0, 0, 0, 0, 0, 0, 0};
                if (nb == 0) FSTAMPW(10);
            }
            if (row >= B) continue;
            *reinterpret_cast<half4*>(h + (size_t)row * kOut + 4 * g) = v;
            if (g == 0) sigma[row] = density_scale * expf((float)v[0]);
            ngp_half* ci = color_in + (size_t)row * 32;
            *reinterpret_cast<half4*>(ci + 16 + 4 * g) = q;
            if (OPERAND && nb == 0) FSTAMPW(11);
            float sh[16];
            ngp_sh::sh_basis<float>(dv[nb][0], dv[nb][1], dv[nb][2], 4u, [&](uint32_t k, float x) { sh[k] = x; });
            // static indices only: sh[4 * g + k] put the array in scratch memory
            // (a store and a dependent load round trip per value)
            half4 s4;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                s4[k] = ngp_f2h(g == 0 ? sh[k] : g == 1 ? sh[4 + k] : g == 2 ? sh[8 + k] : sh[12 + k]);
            *reinterpret_cast<half4*>(ci + 4 * g) = s4;
            if constexpr (OPERAND) {
                half8 x;
                if (g < 2) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) x[k] = ngp_f2h(g == 0 ? sh[k] : sh[8 + k]);
                } else {
                    const half4 a = __builtin_bit_cast(half4, qq[0]), b = __builtin_bit_cast(half4, qq[1]);
                    x = half8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
                }
                xc[nb][0] = x;
                if (nb == 0) FSTAMPW(12);
            }
        }
    }
};

// Density-grid query (renderer.update_extra_state, renderer.py:533-538): the
// sigma network's density = trunc_exp(h[:, 0]) * density_scale (fp32 exp of
// the half value), scattered into tmp_grid[index[row]]. The grid is written
// as a max (float bits as int: densities are >= 0, the grid is reset to -1):
// a cell queried twice in one partial update keeps its larger density, where
// the reference's index_put keeps an arbitrary one of them.
struct EpiDensity {
    float* tmp_grid;
    const int32_t* index;
    float density_scale;
    float* sigma_out;  // non-null: the density of row r stored at sigma_out[r] (no index, no atomic)
    template <typename FO>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], FO out_act) const {
        int32_t ix[kNB];
        load_index(row0, B, ix);
        run(row0, B, o, out_act, ix);
    }
    // the chunk's cell indices (lane group 0: row c of each column block)
    NGP_DEV void load_index(uint32_t row0, uint32_t B, int32_t (&ix)[kNB]) const {
        const int c = threadIdx.x & 15;
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) ix[nb] = sigma_out ? 0 : index[clamp_row(row0 + nb * 16 + c, B)];
    }
    // k_density_fwd's form: lanes 0..31 take one row each (row0 + lane; the
    // second column block's log densities move from lane group 0 to lanes
    // 16..31 with one permute), so the exp and the atomic run once per lane
    // instead of twice in a quarter of the wave
    NGP_DEV int32_t load_index1(uint32_t row0, uint32_t B) const {
        const uint32_t lane = threadIdx.x & 63;
        return sigma_out ? 0 : index[clamp_row(row0 + (lane & 31), B)];
    }
    NGP_DEV void run1(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], int32_t ix) const {
        static_assert(kNB == 2, "two column blocks of 16 rows");
        const int lane = threadIdx.x & 63;
        const float v1 = __shfl(o[1][0][0], lane - 16, 64);  // lanes 16..31 <- lanes 0..15
        const float v = lane < 16 ? o[0][0][0] : v1;
        const uint32_t row = row0 + (uint32_t)lane;
        if (lane >= 32 || row >= B) return;
        const float s = expf((float)(ngp_half)v) * density_scale;
        if (sigma_out)
            sigma_out[row] = s;
        else
            atomicMax(reinterpret_cast<int*>(tmp_grid) + ix, __float_as_int(s));
    }
    template <typename FO>
    NGP_DEV void run(uint32_t row0, uint32_t B, const f32x4 (&o)[kNB][1], FO out_act, const int32_t (&ix)[kNB]) const {
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
        if (g != 0) return;  // column 0 (the log density) lives in lane group 0, register 0
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) {
            const uint32_t row = row0 + nb * 16 + c;
            if (row >= B) continue;
            const float s = expf((float)(ngp_half)out_act.fwd(o[nb][0][0])) * density_scale;
            if (sigma_out)
                sigma_out[row] = s;
            else
                atomicMax(reinterpret_cast<int*>(tmp_grid) + ix[nb], __float_as_int(s));
        }
    }
};

template <int W, int IN_KS, int NH, typename FA, typename FO, typename XL, typename EPI>
__global__ void __launch_bounds__(kThreads)
k_mlp_fwd(const ngp_half* __restrict__ inputs, const ngp_half* __restrict__ weights,
          const half8* __restrict__ image, ngp_half* __restrict__ fwd_buf, uint32_t B,
          uint32_t in_dim, FA act, FO out_act, const int32_t* __restrict__ count, XL xl, EPI epi) {
    using N = Net<W, IN_KS, NH>;
    if (count) B = *count <= 0 ? 0u : min(B, (uint32_t)*count);  // rows past the sample count
    extern __shared__ half8 lds[];
    if (image) {  // prepacked (ngp_ffmlp_pack): straight 16-byte copies
        copy_frags<N::FWD_FRAGS, kThreads>(lds, image);
    } else {
        for (int q = 0; q < N::NMAT; ++q) build_frags(lds, weights, fwd_desc<W, IN_KS, NH>(q, in_dim), false);
    }
    __syncthreads();

    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    for (uint32_t chunk = blockIdx.x * kWaves + wave; chunk < nchunks; chunk += gridDim.x * kWaves) {
        const uint32_t row0 = chunk * 16 * kNB;
        half8 x[kNB][IN_KS];
        xl.template operator()<IN_KS>(inputs, in_dim, row0, B, x);

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
        epi(row0, B, o, out_act);
    }
}


// The density query's sigma network (update_extra_state, renderer.py:533-538)
// on the pair-major encodings of the grid forward, from the prepacked image.
// The grid is sized to the workgroups resident at once (the occupancy query in
// launch_fwd_density); each wave keeps its next kDensityPf chunks' encodings
// and cell indices in flight while it computes the current one. The kernel is
// bound by vector-instruction issue, not by the bytes in flight (DESIGN.md §4:
// 2-4 chunks ahead measured no faster than one, which keeps 4 waves per SIMD).
// Same values as k_mlp_fwd<EpiDensity>.
#ifndef NGP_DENSITY_PF
#define NGP_DENSITY_PF 1
#endif
constexpr int kDensityPf = NGP_DENSITY_PF;
#ifndef NGP_DENSITY_WPE
#define NGP_DENSITY_WPE 2
#endif
template <int W, int NH>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(NGP_DENSITY_WPE)))
k_density_fwd(const ngp_half* __restrict__ enc, const half8* __restrict__ img, uint32_t B, EpiDensity epi) {
    using N = Net<W, 1, NH>;
    const InPairMajorFwd xl{B};
    extern __shared__ half8 lds[];
    const ActReLU act;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB), stride = gridDim.x * kWaves;
    uint32_t chunk = blockIdx.x * kWaves + wave;
    half8 xn[kDensityPf][kNB][1];
    int32_t in_[kDensityPf];
#pragma unroll
    for (int s = 0; s < kDensityPf; ++s) {  // clamped rows past the batch: no branch
        xl.template operator()<1>(enc, 32u, (chunk + s * stride) * 16 * kNB, B, xn[s]);
        in_[s] = epi.load_index1((chunk + s * stride) * 16 * kNB, B);
    }
    copy_frags<N::FWD_FRAGS, kThreads>(lds, img);
    __syncthreads();
    for (; chunk < nchunks; chunk += kDensityPf * stride) {
#pragma unroll
        for (int s = 0; s < kDensityPf; ++s) {
            const uint32_t c = chunk + s * stride;
            if (c >= nchunks) break;  // uniform in the wave
            const uint32_t row0 = c * 16 * kNB;
            half8 x[kNB][1];
#pragma unroll
            for (int nb = 0; nb < kNB; ++nb) x[nb][0] = xn[s][nb][0];
            const int32_t ix = in_[s];
            // the chunk kDensityPf strides ahead into the freed slot
            const uint32_t ahead = (c + kDensityPf * stride) * 16 * kNB;
            xl.template operator()<1>(enc, 32u, ahead, B, xn[s]);
            in_[s] = epi.load_index1(ahead, B);
            f32x4 acc[kNB][N::MTW];
            half8 h[kNB][N::KSW];
            dense<N::MTW, 1>(lds, fwd_desc<W, 1, NH>(0, 32u).frag0, x, acc);
            pack_act<N::MTW, N::KSW>(acc, act, h);
#pragma unroll
            for (int q = 1; q <= NH; ++q) {
                dense<N::MTW, N::KSW>(lds, fwd_desc<W, 1, NH>(q, 32u).frag0, h, acc);
                pack_act<N::MTW, N::KSW>(acc, act, h);
            }
            f32x4 o[kNB][1];
            dense<1, N::KSW>(lds, fwd_desc<W, 1, NH>(NH + 1, 32u).frag0, h, o);
            epi.run1(row0, B, o, ix);
        }
    }
}

// The NeRF forward in one launch (network_ff.py:51-74): per 32-sample chunk
// the sigma network on the pair-major encodings, its epilogue (h, sigma,
// color_in stored for the composite and the backward), then the colour network
// on color_in's rows straight from registers, rgb logits stored [B, 16]. Each
// row's values are the two launches' bit for bit; the colour launch's
// color_in read and its fragment copy and launch tail go away. Both networks
// are W wide with 32 inputs; the images are the ngp_ffmlp_pack ones.
template <int W, int NHS, int NHC>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
k_nerf_fwd(const ngp_half* __restrict__ enc, const half8* __restrict__ img_s, const half8* __restrict__ img_c,
           uint32_t B, const int32_t* __restrict__ count, EpiNerfSigma es, ngp_half* __restrict__ color_out) {
    using NS = Net<W, 1, NHS>;
    using NC = Net<W, 1, NHC>;
    const InPairMajorFwd xl{B};  // the encodings' allocated rows
    FRSTAMP(8);
    FSTAMPW(0);
    if (count) B = *count <= 0 ? 0u : min(B, (uint32_t)*count);
    extern __shared__ half8 lds[];
    half8* lds_c = lds + NS::FWD_FRAGS * 64;
    const ActReLU act;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB), stride = gridDim.x * kWaves;
    // the first chunk's encodings and directions are requested before the
    // fragment copy, each later chunk's at the end of the previous one
    uint32_t chunk = blockIdx.x * kWaves + wave;
    half8 xn[kNB][1];
    float dn[kNB][3];
    xl.template operator()<1>(enc, 32u, chunk * 16 * kNB, B, xn);
    es.load_dirs(chunk * 16 * kNB, B, dn);
    copy_frags<NS::FWD_FRAGS, kThreads>(lds, img_s);
    copy_frags<NC::FWD_FRAGS, kThreads>(lds_c, img_c);
    __syncthreads();
    FSTAMPW(1);
    for (; chunk < nchunks; chunk += stride) {
        const uint32_t row0 = chunk * 16 * kNB;
        half8 x[kNB][1];
        float dv[kNB][3];
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) {
            x[nb][0] = xn[nb][0];
#pragma unroll
            for (int k = 0; k < 3; ++k) dv[nb][k] = dn[nb][k];
        }
        FSTAMPW(2);
        f32x4 acc[kNB][NS::MTW];
        half8 h[kNB][NS::KSW];
        dense<NS::MTW, 1>(lds, fwd_desc<W, 1, NHS>(0, 32u).frag0, x, acc);
        pack_act<NS::MTW, NS::KSW>(acc, act, h);
#pragma unroll
        for (int q = 1; q <= NHS; ++q) {
            dense<NS::MTW, NS::KSW>(lds, fwd_desc<W, 1, NHS>(q, 32u).frag0, h, acc);
            pack_act<NS::MTW, NS::KSW>(acc, act, h);
        }
        f32x4 o[kNB][1];
        dense<1, NS::KSW>(lds, fwd_desc<W, 1, NHS>(NHS + 1, 32u).frag0, h, o);
        FSTAMPW(3);
        es.template run<true>(row0, B, o, ActNone{}, x, dv);
        FSTAMPW(4);
        dense<NC::MTW, 1>(lds_c, fwd_desc<W, 1, NHC>(0, 32u).frag0, x, acc);
        pack_act<NC::MTW, NC::KSW>(acc, act, h);
#pragma unroll
        for (int q = 1; q <= NHC; ++q) {
            dense<NC::MTW, NC::KSW>(lds_c, fwd_desc<W, 1, NHC>(q, 32u).frag0, h, acc);
            pack_act<NC::MTW, NC::KSW>(acc, act, h);
        }
        dense<1, NC::KSW>(lds_c, fwd_desc<W, 1, NHC>(NHC + 1, 32u).frag0, h, o);
        FSTAMPW(5);
        store_tiles<1>(color_out, kOut, row0, B, o, ActNone{});
        FSTAMPW(6);
        // the next chunk's inputs (clamped rows: no branch, see copy_frags)
        xl.template operator()<1>(enc, 32u, row0 + stride * 16 * kNB, B, xn);
        es.load_dirs(row0 + stride * 16 * kNB, B, dn);
    }
    FRSTAMP(9);
}

// ---- backward ---------------------------------------------------------------
// dW = delta^T . input over a 32-sample chunk is an MFMA whose K is the
// sample index: both operands need "8 samples of one unit" per lane, while
// the chunk's activations sit as "4 units of one sample" per lane. The wave
// stores them sample-major ([sample][unit], 8- or 16-byte row segments) and
// reads the operands back with ds_read_b64_tr_b16 (gfx950's transposing LDS
// read: per 16-lane group a 4-row x 16-column block arrives column-major).
// K slot j of lane group g holds sample perm_unit(g, j) in BOTH operands.
typedef short short4v __attribute__((ext_vector_type(4)));

template <int KS, bool PERM, int NB>
NGP_DEV void write_rows(ngp_half* __restrict__ tile, const half8 (&v)[NB][KS], uint32_t units) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        ngp_half* row = tile + (nb * 16 + c) * kTileLd;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (PERM) {  // elements 0..3: units 32s+4g.., 4..7: units 32s+16+4g..
                const half4 lo = {v[nb][s][0], v[nb][s][1], v[nb][s][2], v[nb][s][3]};
                const half4 hi = {v[nb][s][4], v[nb][s][5], v[nb][s][6], v[nb][s][7]};
                *reinterpret_cast<half4*>(row + 32 * s + 4 * g) = lo;
                *reinterpret_cast<half4*>(row + 32 * s + 16 + 4 * g) = hi;
            } else {     // units 32s+8g .. +7 (zeros past `units`)
                const uint32_t u0 = 32 * s + 8 * g;
                const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
                if (u0 < (uint32_t)(32 * KS)) *reinterpret_cast<half8*>(row + u0) = u0 < units ? v[nb][s] : z;
            }
        }
    }
}

// operand fragment of units 16m..16m+15 over the chunk's 32 samples
NGP_DEV half8 read_tr(const ngp_half* __restrict__ tile, int m) {
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const ngp_half* a = tile + (4 * g + q) * kTileLd + 16 * m + 4 * p;
    const ngp_half* b = a + 16 * kTileLd;
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) short4v*)(a));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) short4v*)(b));
    return __builtin_shufflevector(__builtin_bit_cast(half4, lo), __builtin_bit_cast(half4, hi),
                                   0, 1, 2, 3, 4, 5, 6, 7);
}

// dW[o][i] (MO x MI tiles of 16x16) += dT^T . hT over the chunk
template <int MO, int MI>
NGP_DEV void dw_accum(const ngp_half* __restrict__ dT, const ngp_half* __restrict__ hT,
                      f32x4 (&acc)[MO][MI]) {
    half8 a[MO], b[MI];
    // the transposed reads are opaque intrinsics on an LDS address-space cast:
    // keep the compiler from moving them across the wave's own tile stores
    // (LDS itself executes one wave's operations in order)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < MO; ++m) a[m] = read_tr(dT, m);
#pragma unroll
    for (int n = 0; n < MI; ++n) b[n] = read_tr(hT, n);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int n = 0; n < MI; ++n) acc[m][n] = mfma(a[m], b[n], acc[m][n]);
}

// delta (C layout, MT tiles) * act'(post-activation h, permuted B form) -> permuted B form
template <int MT, int KS, typename ACT, int NB>
NGP_DEV void pack_delta(const f32x4 (&acc)[NB][MT], const half8 (&h)[NB][KS], ACT act,
                        half8 (&out)[NB][KS]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            half8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int mt = 2 * s + (j >> 2);
                v[j] = mt < MT ? (ngp_half)act.bwd(acc[nb][mt][j & 3], (float)h[nb][s][j]) : (ngp_half)0.0f;
            }
            out[nb][s] = v;
        }
}

// ReLU policy: the delta pairs rounded to fp16 (one packed conversion), then
// masked where the post-activation is 0. The recomputed activations come from
// pack_act's ReLU, so they are +0 or positive (bits in (0, 0x7fff] as signed
// 16-bit values): 0 - y is negative exactly where y > 0, and its sign spread
// over the half (>> 15) is the mask. Equal to (y > 0 ? g : 0) rounded, at 4
// VALU per 2 values against ~8 (an fp32 conversion of y, a compare and a
// select per value, and single conversions).
template <int MT, int KS, int NB>
NGP_DEV void pack_delta(const f32x4 (&acc)[NB][MT], const half8 (&h)[NB][KS], ActReLU, half8 (&out)[NB][KS]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint4 hv = __builtin_bit_cast(uint4, h[nb][s]);
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int mt = 2 * s + (j >> 1), r = 2 * (j & 1);
                o[j] = 0u;
                if (mt < MT) {
                    const ngp_half2 g2 =
                        __builtin_convertvector(ngp_float2{acc[nb][mt][r], acc[nb][mt][r + 1]}, ngp_half2);
                    // (the compiler rewrites the C form into two compares and
                    // selects; op_sel_hi:[0,1]: both halves shift by the
                    // constant's low half)
                    uint32_t m;
                    asm("v_pk_sub_i16 %0, 0, %1\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(m) : "v"(hv[j]));
                    o[j] = __builtin_bit_cast(uint32_t, g2) & m;
                }
            }
            out[nb][s] = __builtin_bit_cast(half8, (uint4{o[0], o[1], o[2], o[3]}));
        }
}

// Fold image: tile-major [tile][lane] f32x4 (one 1 KB slot per 16x16 dW
// tile), so a wave stores / adds a tile with one conflict-free 16-byte LDS
// access per lane (the [out][in] layout took four scalar accesses per tile
// element group). FIRST stores; otherwise every read of the wave is issued
// before its first add.
template <bool FIRST, int MO, int MI>
NGP_DEV void fold_tiles(const f32x4 (&t)[MO][MI], float* __restrict__ img) {
    f32x4* p = reinterpret_cast<f32x4*>(img) + (threadIdx.x & 63);
    if (FIRST) {
#pragma unroll
        for (int m = 0; m < MO; ++m)
#pragma unroll
            for (int k = 0; k < MI; ++k) p[(m * MI + k) * 64] = t[m][k];
        return;
    }
    f32x4 v[MO][MI];
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int k = 0; k < MI; ++k) v[m][k] = p[(m * MI + k) * 64];
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int k = 0; k < MI; ++k) p[(m * MI + k) * 64] = v[m][k] + t[m][k];
}

template <int MO, int MI>
NGP_DEV void zero_tiles(f32x4 (&t)[MO][MI]) {
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int k = 0; k < MI; ++k) t[m][k] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int W, int IN_KS, int NH>
struct BwdLds {
    using N = Net<W, IN_KS, NH>;
    static constexpr int FRAGS = N::FWD_FRAGS + N::BWD_FRAGS;
    static constexpr size_t frag_bytes = (size_t)FRAGS * 64 * 16;
    static constexpr size_t tile_bytes = (size_t)kBwdWaves * 2 * kTileRows * kTileLd * 2;
    static constexpr size_t nparams_max = (size_t)W * (32 * IN_KS) + (size_t)NH * W * W + (size_t)kOut * W;
    // one fold image: 1 KB per 16x16 dW tile (see fold_tiles)
    static constexpr size_t acc_bytes = (size_t)(N::MTW * N::IN_MT + NH * N::MTW * N::MTW + N::MTW) * 1024;
    // the two dW images of the epilogue reuse the fragment + tile space once
    // the chunk loop is done
    static constexpr size_t total =
        frag_bytes + tile_bytes > 2 * acc_bytes ? frag_bytes + tile_bytes : 2 * acc_bytes;
};

// Single-pass fused backward: per 32-sample chunk a wave recomputes the
// forward (activations stay in registers), walks the deltas down through
// W^T fragments, and for every matmul forms dW += delta^T . input over the
// chunk with MFMAs whose K is the sample index. The dW tiles live in the
// wave's registers (accumulation VGPRs) for the whole chunk loop; only at the
// end do the waves fold them, in fixed order, into an LDS image of dW that
// the workgroup publishes as its slab row.
// grad_inputs epilogues: the plain [B, in_dim] store, or the NeRF color
// network's (nerf/network_ff.py:67-68, the cat's backward): only the geo
// columns 16..30 of the input gradient are kept, written to columns 1..15 of
// the sigma network's output gradient [B, 16] (column 0 holds the density
// gradient, written by the composite kernel).
struct GiStore {
    ngp_half* gi;
    template <int IN_MT, int NB>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, uint32_t in_dim, const f32x4 (&t)[NB][IN_MT]) const {
        store_tiles<IN_MT>(gi, in_dim, row0, B, t, ActNone{});
    }
};

struct GiNerfGeo {
    ngp_half* gh;
    const int32_t* map = nullptr;  // row list, or null
    template <int IN_MT, int NB>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, uint32_t, const f32x4 (&t)[NB][IN_MT]) const {
        static_assert(IN_MT == 2, "the color network input is 32 wide");  // see launch_bwd
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            // lane group g holds input columns 16 + 4g .. +3 (tile 1); output
            // columns 4g .. 4g+3 take input columns 15 + 4g .. 18 + 4g
            const ngp_half r0 = (ngp_half)t[nb][1][0], r1 = (ngp_half)t[nb][1][1], r2 = (ngp_half)t[nb][1][2];
            const uint32_t pv = __shfl((uint32_t)__builtin_bit_cast(uint16_t, (ngp_half)t[nb][1][3]), lane - 16, 64);
            const uint32_t row = row0 + nb * 16 + c;
            if (row >= B) continue;
            ngp_half* d = gh + (size_t)map_row(map, row) * kOut + 4 * g;
            if (g == 0) {
                d[1] = r0;
                d[2] = r1;
                d[3] = r2;
            } else {
                *reinterpret_cast<half4*>(d) = half4{__builtin_bit_cast(ngp_half, (uint16_t)pv), r0, r1, r2};
            }
        }
    }
};

// [in_dim / 2][ld][2] pair-major input gradient (see InPairMajor)
struct GiPairMajor {
    ngp_half* gi;
    uint32_t ld;
    const int32_t* map = nullptr;  // row list, or null
    template <int IN_MT, int NB>
    NGP_DEV void operator()(uint32_t row0, uint32_t B, uint32_t in_dim, const f32x4 (&t)[NB][IN_MT]) const {
        const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            const uint32_t row = row0 + nb * 16 + c;
            if (row >= B) continue;
            const uint32_t pr = map_row(map, row);
#pragma unroll
            for (int mt = 0; mt < IN_MT; ++mt) {
                const uint32_t col = 16 * mt + 4 * g;
                if (col >= in_dim) continue;
                const uint32_t p = col / 2;
                *reinterpret_cast<ngp_half2*>(gi + ((size_t)p * ld + pr) * 2) =
                    ngp_half2{(ngp_half)t[nb][mt][0], (ngp_half)t[nb][mt][1]};
                *reinterpret_cast<ngp_half2*>(gi + ((size_t)(p + 1) * ld + pr) * 2) =
                    ngp_half2{(ngp_half)t[nb][mt][2], (ngp_half)t[nb][mt][3]};
            }
        }
    }
};

#ifdef NGP_STAMPS  // diagnostic build only (tools/accum_stamps.py): per-wave phase clocks
#define MSTAMP(slot) do { if (g_mlp_stamps && (threadIdx.x & 63) == 0) g_mlp_stamps[((size_t)(NH - 1) * 2048 + blockIdx.x * kBwdWaves + (threadIdx.x >> 6)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define MSTAMP(slot) do { } while (0)
#endif

// One backward pass over the 32-sample chunks a wave takes (map(k): the
// wave's k-th chunk; a chunk >= the chunk count ends the loop), then the
// wave's half chunk if it has one (half(): the first row of a 16-sample half
// of a chunk no wave took whole, or kNoHalf), then the fold of the waves' dW
// tiles and the workgroup's slab row. fr: the network's fragment image in
// LDS; tiles: the per-wave staging tiles; img: where the two fold images go
// (they may overlay fr and tiles, dead by then). pre() runs once the first
// chunk's loads are issued (a standalone launch copies its fragment image
// there, so the two latencies overlap).
constexpr uint32_t kNoHalf = 0xffffffffu;
struct NoHalf {
    NGP_DEV uint32_t operator()() const { return kNoHalf; }
};
struct NoIdle {
    NGP_DEV void operator()() const {}
};

template <int W, int IN_KS, int NH, bool GI_SYNC, typename FA, typename XL, typename GI, typename MAP, typename PRE,
          typename HALF = NoHalf, typename IDLE = NoIdle>
NGP_DEV void bwd_phase(const half8* __restrict__ fr, ngp_half* __restrict__ tiles, float* __restrict__ img_base,
                       const ngp_half* __restrict__ grad, const ngp_half* __restrict__ inputs, XL xl, GI gi_out,
                       bool want_gi, float* __restrict__ slab, uint32_t nparams, uint32_t B, uint32_t in_dim,
                       FA act, MAP map, PRE pre, HALF half = HALF{}, IDLE idle = IDLE{}) {
    using N = Net<W, IN_KS, NH>;
    constexpr int LAST = N::NMAT - 1;
    MSTAMP(0);
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t chunk = map(0u);
    // a wave whose only work is a half chunk (the live-row regime's common
    // case) requests the half's rows here instead, beside the prologue
    const uint32_t hrow = half();
    const bool half_first = chunk >= nchunks && hrow != kNoHalf;  // wave-uniform
    const uint32_t first_row = half_first ? hrow : chunk * 16 * kNB;
    half8 xn[kNB][IN_KS], dn[kNB][1];
    xl.template operator()<IN_KS>(inputs, in_dim, first_row, B, xn);
    load_rows<1>(grad, kOut, first_row, B, dn, xl.map);  // output activation ignored (ffmlp.cu:783)
    pre();
    MSTAMP(1);
    [[maybe_unused]] uint32_t nst = 0;

    ngp_half* dT = tiles + (size_t)wave * 2 * kTileRows * kTileLd;
    ngp_half* hT = dT + (size_t)kTileRows * kTileLd;

    f32x4 dw_last[1][N::MTW], dw_hid[NH][N::MTW][N::MTW], dw_first[N::MTW][N::IN_MT];
    zero_tiles(dw_last);
#pragma unroll
    for (int q = 0; q < NH; ++q) zero_tiles(dw_hid[q]);
    zero_tiles(dw_first);

    // one chunk of NBC 16-sample blocks from row0 (inputs x, output grads
    // dout): recompute, delta chain, dW accumulation, input grads
    auto body = [&](auto nbc, uint32_t row0, const auto& x, const auto& dout) {
        constexpr int NBC = decltype(nbc)::value;
        // recompute the post-activations of every hidden layer
        half8 h[NH + 1][NBC][N::KSW];
        f32x4 a[NBC][N::MTW];
        dense<N::MTW, IN_KS>(fr, fwd_desc<W, IN_KS, NH>(0, in_dim).frag0, x, a);
        pack_act<N::MTW, N::KSW>(a, act, h[0]);
#pragma unroll
        for (int q = 1; q <= NH; ++q) {
            dense<N::MTW, N::KSW>(fr, fwd_desc<W, IN_KS, NH>(q, in_dim).frag0, h[q - 1], a);
            pack_act<N::MTW, N::KSW>(a, act, h[q]);
        }
        // Per matmul: the transposing tiles are stored, then the next delta's
        // product (register operands + fragment reads) is issued BEFORE the
        // dW product that reads the tiles back, so its MFMAs cover the tile
        // round trip (LDS executes one wave's operations in order, the reads
        // see the stores).
        // last matmul: dW += dout^T . h[NH]
        write_rows<1, false>(dT, dout, kOut);
        write_rows<N::KSW, true>(hT, h[NH], W);
        dense<N::MTW, 1>(fr, bwd_desc<W, IN_KS, NH>(LAST, in_dim).frag0 + N::FWD_FRAGS, dout, a);
        dw_accum<1, N::MTW>(dT, hT, dw_last);
        half8 d[NBC][N::KSW];  // delta of a matmul's pre-activation output, permuted B form
        pack_delta<N::MTW, N::KSW>(a, h[NH], act, d);
#pragma unroll
        for (int q = NH; q >= 1; --q) {
            write_rows<N::KSW, true>(dT, d, W);
            write_rows<N::KSW, true>(hT, h[q - 1], W);
            dense<N::MTW, N::KSW>(fr, bwd_desc<W, IN_KS, NH>(q, in_dim).frag0 + N::FWD_FRAGS, d, a);
            dw_accum<N::MTW, N::MTW>(dT, hT, dw_hid[q - 1]);
            pack_delta<N::MTW, N::KSW>(a, h[q - 1], act, d);
        }
        // first matmul: dW += d^T . x, and grad_inputs = W_0^T d
        write_rows<N::KSW, true>(dT, d, W);
        write_rows<IN_KS, false>(hT, x, in_dim);
        f32x4 gi[NBC][N::IN_MT];
        if (want_gi) dense<N::IN_MT, N::KSW>(fr, bwd_desc<W, IN_KS, NH>(0, in_dim).frag0 + N::FWD_FRAGS, d, gi);
        dw_accum<N::MTW, N::IN_MT>(dT, hT, dw_first);
        if (want_gi) gi_out(row0, B, in_dim, gi);
    };

    // inputs and output gradients of the next chunk are prefetched while the
    // current one computes (one wave per SIMD: nothing else hides the latency)
    for (uint32_t kc = 1; chunk < nchunks; ++kc) {
        const uint32_t row0 = chunk * 16 * kNB;
        half8 x[kNB][IN_KS], dout[kNB][1];
#pragma unroll
        for (int nb = 0; nb < kNB; ++nb) {
#pragma unroll
            for (int s = 0; s < IN_KS; ++s) x[nb][s] = xn[nb][s];
            dout[nb][0] = dn[nb][0];
        }
        const uint32_t next = map(kc);
        xl.template operator()<IN_KS>(inputs, in_dim, next * 16 * kNB, B, xn);
        load_rows<1>(grad, kOut, next * 16 * kNB, B, dn, xl.map);
        body(std::integral_constant<int, kNB>{}, row0, x, dout);
        MSTAMP(2 + min(nst, 9u));
        ++nst;
        chunk = next;
    }
    // the wave's half chunk: 16 samples in rows 0..15 of the transposing
    // tiles, rows 16..31 zero (the dW products' K runs over all 32 rows)
    if (hrow != kNoHalf) {
        half8 x1[1][IN_KS], d1[1][1];
        if (half_first) {  // requested at the start
#pragma unroll
            for (int s2 = 0; s2 < IN_KS; ++s2) x1[0][s2] = xn[0][s2];
            d1[0][0] = dn[0][0];
        } else {
            xl.template operator()<IN_KS>(inputs, in_dim, hrow, B, x1);
            load_rows<1>(grad, kOut, hrow, B, d1, xl.map);
        }
        asm volatile("" ::: "memory");  // after the last chunk's transposed reads
        const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t lane = threadIdx.x & 63;
        for (uint32_t i = lane; i < 16 * kTileLd / 8; i += 64) {
            reinterpret_cast<half8*>(dT + 16 * kTileLd)[i] = z;
            reinterpret_cast<half8*>(hT + 16 * kTileLd)[i] = z;
        }
        asm volatile("" ::: "memory");
        body(std::integral_constant<int, 1>{}, hrow, x1, d1);
    }
    MSTAMP(12);
    // fold the waves' register tiles into two LDS dW images (round r: waves
    // 2r and 2r + 1 store (r = 0) or add into images 0 and 1), then publish
    // image0 + image1 as the slab row: a fixed summation order, so dW is
    // bit-reproducible. Images are tile-major (fold_tiles): first layer's
    // MTW x IN_MT tiles, each hidden layer's MTW x MTW, the last layer's 1 x MTW.
    // A later round whose two waves took no rows adds only zeros: it is
    // skipped (x + 0.0 == x, so the row is the same bit for bit).
    constexpr int T_FIRST = N::MTW * N::IN_MT, T_HID = N::MTW * N::MTW, T_LAST = N::MTW;
    constexpr int NT = T_FIRST + NH * T_HID + T_LAST;
        float* img = img_base + (size_t)(wave & 1) * NT * 256;
    auto fold = [&](auto first) {
        constexpr bool F = decltype(first)::value;
        fold_tiles<F>(dw_first, img);
#pragma unroll
        for (int q = 1; q <= NH; ++q) fold_tiles<F>(dw_hid[q - 1], img + (T_FIRST + (q - 1) * T_HID) * 256);
        fold_tiles<F>(dw_last, img + (T_FIRST + NH * T_HID) * 256);
    };
    __shared__ uint32_t s_took[kBwdWaves];  // each wave writes its own slot before the barrier below
    if ((threadIdx.x & 63) == 0) s_took[wave] = nst != 0 || hrow != kNoHalf ? 1u : 0u;
    if (nst == 0 && hrow == kNoHalf) idle();  // a wave without rows (wave-uniform)
    // fragments and tiles are dead from here on. GI_SYNC (the NeRF backward's
    // colour pass, whose input gradients the sigma pass reads): a full barrier,
    // the waves' input-gradient stores complete for the workgroup; otherwise
    // (nothing in the workgroup reads them) an LDS-only one, so the fold does
    // not wait for the stores to land. The later barriers order LDS only.
    if constexpr (GI_SYNC)
        __syncthreads();
    else
        lds_barrier();
    if (wave < 2) fold(std::true_type{});
    lds_barrier();
#pragma unroll 1
    for (uint32_t r = 1; r < (uint32_t)kBwdWaves / 2; ++r) {
        if ((s_took[2 * r] | s_took[2 * r + 1]) == 0u) continue;  // workgroup-uniform
        if ((wave >> 1) == r) fold(std::false_type{});
        lds_barrier();
    }
    MSTAMP(13);
    // slab row = image0 + image1 in the unpadded [out][in] layout: per tile a
    // lane adds its two 16-byte slots and stores its 4 outputs (rows 16m + 4g +
    // r, column 16k + c: 64-byte segments per row)
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const f32x4* i0 = reinterpret_cast<const f32x4*>(img_base);
    const f32x4* i1 = i0 + NT * 64;
    float* slab_row = slab + (size_t)blockIdx.x * nparams;
    // all of the wave's image reads first (one LDS wait), then its stores back
    // to back; each tile's geometry from compile-time divisors
    constexpr int TPW = (NT + kBwdWaves - 1) / kBwdWaves;
    f32x4 sv[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int tt = min((int)wave + q * kBwdWaves, NT - 1);
        sv[q] = i0[tt * 64 + lane] + i1[tt * 64 + lane];
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int tt = (int)wave + q * kBwdWaves;
        if (tt >= NT) break;
        uint32_t m, k, in_w, out_w, off;
        if (tt < T_FIRST) {
            m = (uint32_t)tt / N::IN_MT; k = (uint32_t)tt % N::IN_MT; in_w = in_dim; out_w = W; off = 0;
        } else if (tt < T_FIRST + NH * T_HID) {
            const uint32_t h = (uint32_t)(tt - T_FIRST) / T_HID, local = (uint32_t)(tt - T_FIRST) - h * T_HID;
            m = local / N::MTW; k = local % N::MTW; in_w = W; out_w = W;
            off = fwd_desc<W, IN_KS, NH>((int)h + 1, in_dim).off;
        } else {
            const uint32_t local = (uint32_t)(tt - T_FIRST - NH * T_HID);
            m = local / N::MTW; k = local % N::MTW; in_w = W; out_w = kOut;
            off = fwd_desc<W, IN_KS, NH>(LAST, in_dim).off;
        }
        const uint32_t i = 16 * k + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t o = 16 * m + 4 * g + r;
            if (o < out_w && i < in_w) slab_row[off + o * in_w + i] = sv[q][r];
        }
    }
    MSTAMP(14);
}


template <int W, int IN_KS, int NH, typename FA, typename XL, typename GI>
__global__ void __launch_bounds__(kBwdThreads)
k_mlp_bwd(const ngp_half* __restrict__ grad, const ngp_half* __restrict__ inputs,
          const half8* __restrict__ image, XL xl, GI gi_out, bool want_gi,
          float* __restrict__ slab, uint32_t nparams, uint32_t B, uint32_t in_dim, FA act,
          const int32_t* __restrict__ count) {
    using N = Net<W, IN_KS, NH>;
    using L = BwdLds<W, IN_KS, NH>;
    static_assert((size_t)2 * (N::MTW * N::IN_MT + NH * N::MTW * N::MTW + N::MTW) * 1024 <= L::total,
                  "fold images exceed the workgroup's LDS");
    if (count) B = *count <= 0 ? 0u : min(B, (uint32_t)*count);  // rows past the sample count
    extern __shared__ half8 lds[];
    ngp_half* tiles = reinterpret_cast<ngp_half*>(reinterpret_cast<char*>(lds) + L::frag_bytes);
    const uint32_t stride = gridDim.x * kBwdWaves, c0 = blockIdx.x * kBwdWaves + (threadIdx.x >> 6);
    bwd_phase<W, IN_KS, NH, false>(lds, tiles, reinterpret_cast<float*>(lds), grad, inputs, xl, gi_out, want_gi, slab,
                            nparams, B, in_dim, act, [=](uint32_t k) { return c0 + k * stride; },
                            [&]() {
                                copy_frags<L::FRAGS, kBwdThreads>(lds, image);
                                __syncthreads();
                            });
}

// The NeRF step's two backward networks in one launch (ngp_nerf_backward):
// the colour network (its geo-feature grads into g_h's columns 1..15), then,
// after a workgroup barrier, the sigma network over the same workgroup's
// chunks (its output grad g_h is complete for them). Workgroup b takes chunks
// b, b + G, b + 2G, ... (G workgroups) for both networks; its j-th chunk goes
// to wave j % 4 in the colour pass and to wave 3 - j % 4 in the sigma pass, so
// a wave with an extra colour chunk has one sigma chunk less. (Two launches:
// 2,528 Lego chunks over 1,024 waves gave the same waves the third chunk of
// both networks.) Both fragment images are copied at the start; the sigma
// one lies past everything the colour pass uses (its fragments, tiles and
// fold images), and the sigma pass's tiles and fold images overlay the
// colour pass's.
struct NerfBwdArgs {
    const ngp_half* g_color_out;   // [B, 16]
    const ngp_half* color_in;      // [B, 32]
    const half8* color_image;
    ngp_half* g_h;                 // [B, 16]: column 0 (density grad) given, columns 1..15 written
    const ngp_half* enc;           // [16][B][2] pair-major grid encoding
    const half8* sigma_image;
    ngp_half* g_enc;               // [16][B][2]
    float* slab_color;
    float* slab_sigma;
    uint32_t np_color, np_sigma, B;
    const int32_t* count;
    const int32_t* rows;  // the rows to run (*count of them), or null: rows [0, *count)
    // the grid backward's timing ring (NGP_GRID_TIMING, include/ngp_hip.h), or
    // null: workgroup b stores its end (after its last store) in end slot
    // MAX_WG - 1 - b of the call the next bin launch opens (the accumulate's
    // workgroups fill the slots from 0), so the grid backward's span can start
    // where this launch ended. Plain stores: one contended atomic per
    // workgroup cost ~2 us at the launch's end.
    uint32_t* timing;
};

template <int NHS, int NHC>
struct NerfBwdLds {
    using LC = BwdLds<64, 1, NHC>;
    using LS = BwdLds<64, 1, NHS>;
    static constexpr size_t sigma_frags = LC::total;  // the sigma image's offset
    static constexpr size_t total = sigma_frags + LS::frag_bytes;
    static constexpr bool fits = total <= 160 * 1024 && LS::total <= sigma_frags;
};
template <int NHS, int NHC>
__global__ void __launch_bounds__(kBwdThreads)
k_nerf_bwd(NerfBwdArgs a) {
    using LC = BwdLds<64, 1, NHC>;
    using LS = BwdLds<64, 1, NHS>;
    using NL = NerfBwdLds<NHS, NHC>;
    static_assert(NL::fits, "nerf backward LDS budget exceeded");
    uint32_t B = a.B;
    if (a.count) B = *a.count <= 0 ? 0u : min(B, (uint32_t)*a.count);
    extern __shared__ half8 lds[];
    half8* sfr = reinterpret_cast<half8*>(reinterpret_cast<char*>(lds) + NL::sigma_frags);
    const uint32_t G = gridDim.x, b = blockIdx.x, w = threadIdx.x >> 6;
    const uint32_t tcall = a.timing && threadIdx.x == 0 ? a.timing[0] : 0u;  // requested early
    // this workgroup's chunks b, b + G, ...: n of them, the j-th in slot j % 4.
    // When the last round holds r = 1 or 2 chunks (2 or 3 of the 4 waves idle
    // for a whole chunk), they are split into 2r halves of 16 samples, one per
    // slot, so the round takes a half chunk's time
    const uint32_t nch = ngp_div_up(B, 16 * kNB);
    const uint32_t n = b < nch ? (nch - b + G - 1) / G : 0u, r = n % kBwdWaves;
    const uint32_t nf = r == 1 || r == 2 ? n - r : n;  // chunks taken whole
    auto map_of = [=](uint32_t slot) {
        return [=](uint32_t k) { const uint32_t j = slot + k * kBwdWaves; return j < nf ? b + j * G : nch; };
    };
    auto half_of = [=](uint32_t slot) {
        return [=]() { return nf < n && slot < 2 * r ? (b + (nf + slot / 2) * G) * 16 * kNB + 16 * (slot & 1) : kNoHalf; };
    };
    // With 1 or 3 chunks the colour pass leaves the last waves without rows
    // (waves 2-3: two halves; wave 3: three whole chunks): they copy the sigma
    // image meanwhile, off the colour pass's critical path
    const bool idle_copy = n == 1 || n == 3;
    const uint32_t idle0 = n == 1 ? 2u : 3u;
    // live rows: the workgroups past the slab rows the reduce reads have no
    // chunk and skip both passes (ngp_reduce::live_slab_rows)
    if (!a.rows || b < ngp_reduce::live_slab_rows((int32_t)B, G)) {
    bwd_phase<64, 1, NHC, true>(lds, reinterpret_cast<ngp_half*>(reinterpret_cast<char*>(lds) + LC::frag_bytes),
                          reinterpret_cast<float*>(lds), a.g_color_out, a.color_in, InRowMajor{a.rows},
                          GiNerfGeo{a.g_h, a.rows},
                          true, a.slab_color, a.np_color, B, 32u, ActReLU{}, map_of(w),
                          [&]() {
                              copy_frags<LC::FRAGS, kBwdThreads>(lds, a.color_image);
                              if (!idle_copy) copy_frags<LS::FRAGS, kBwdThreads>(sfr, a.sigma_image);
                              __syncthreads();
                          }, half_of(w),
                          [&]() {  // the colour pass's idle waves copy the sigma image (done by the fold's barrier)
                              if (idle_copy)
                                  copy_frags_part<LS::FRAGS>(sfr, a.sigma_image, threadIdx.x - idle0 * 64,
                                                             (kBwdWaves - idle0) * 64);
                          });
    // the colour pass's geo grads (global stores of every wave) are complete
    // (the fold's first barrier) and its fold images read before the sigma
    // pass loads g_h and reuses LDS: an LDS-only barrier, so the colour slab
    // row's stores need not land first
    lds_barrier();
    bwd_phase<64, 1, NHS, false>(sfr, reinterpret_cast<ngp_half*>(lds), reinterpret_cast<float*>(lds), a.g_h, a.enc,
                          InPairMajor{a.B, a.rows}, GiPairMajor{a.g_enc, a.B, a.rows}, true, a.slab_sigma, a.np_sigma,
                          B, 32u, ActReLU{}, map_of(kBwdWaves - 1 - w), []() {}, half_of(kBwdWaves - 1 - w));
    }
    if (a.timing && b < NGP_GRID_TIMING_MAX_WG / 4) {
        __syncthreads();
        if (threadIdx.x == 0)
            a.timing[64 + 4 * NGP_GRID_TIMING_RING + (tcall % NGP_GRID_TIMING_RING) * NGP_GRID_TIMING_MAX_WG +
                     NGP_GRID_TIMING_MAX_WG - 1 - b] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
}

// grad_weights[p] = sum over workgroup rows of the slab, in a fixed order
// (deterministic; ngp_reduce.h). Block = 64 parameters x 16 row phases.
// Several networks' slabs in one launch (jobs).
using ngp_reduce::kMaxReduceJobs;
using ngp_reduce::kReducePhases;
using ngp_reduce::ReduceJobs;

template <typename OUT>
__global__ void __launch_bounds__(64 * kReducePhases)
k_slab_reduce(ReduceJobs jobs) {
    __shared__ float part[kReducePhases][64];
    ngp_reduce::slab_reduce_block<OUT, 64 * kReducePhases>(jobs, blockIdx.x, part);
}

__global__ void __launch_bounds__(256)
k_mlp_pack_jobs(PackJobs jobs) {
    const PackJob& j = jobs.job[blockIdx.x];
    build_frags(j.image, j.w, j.m, j.transposed != 0);
}

// ---- host dispatch ----------------------------------------------------------
uint32_t num_params(uint32_t in_dim, uint32_t hidden, uint32_t num_layers) {
    return hidden * (in_dim + hidden * (num_layers - 1) + kOut);
}

uint32_t bwd_blocks(uint32_t B) {
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t nb = ngp_div_up(nchunks, kBwdWaves);
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

// Forward launch: w (built per workgroup) or a prepacked image; epilogue EPI.
template <int W, int IN_KS, int NH, typename FA, typename FO, typename EPI, typename XL = InRowMajor>
int launch_fwd_t(const void* in, const void* w, const void* image, uint32_t B, uint32_t in_dim, FA act,
                 FO out_act, void* fwd_buf, const int32_t* count, EPI epi, hipStream_t st, XL xl = XL{}) {
    using N = Net<W, IN_KS, NH>;
    const size_t lds = (size_t)N::FWD_FRAGS * 64 * 16;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t blocks = ngp_div_up(nchunks, kWaves);
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) return NGP_OK;
    hipLaunchKernelGGL((k_mlp_fwd<W, IN_KS, NH, FA, FO, XL, EPI>), dim3(blocks), dim3(kThreads), lds, st,
                       (const ngp_half*)in, (const ngp_half*)w, (const half8*)image, (ngp_half*)fwd_buf,
                       B, in_dim, act, out_act, count, xl, epi);
    return ngp_check_launch("ffmlp_forward");
}

template <int W, int IN_KS, int NH>
int launch_fwd(const void* in, const void* w, const void* image, uint32_t B, uint32_t in_dim, uint32_t act,
               uint32_t out_act, void* fwd_buf, void* out, const int32_t* count, hipStream_t st) {
    const EpiStore epi{static_cast<ngp_half*>(out)};
    if (act == kReLU && out_act == kNone)
        return launch_fwd_t<W, IN_KS, NH>(in, w, image, B, in_dim, ActReLU{}, ActNone{}, fwd_buf, count, epi, st);
    return launch_fwd_t<W, IN_KS, NH>(in, w, image, B, in_dim, ActAny{act}, ActAny{out_act}, fwd_buf, count,
                                      epi, st);
}

template <int W, int IN_KS, int NH>
int launch_fwd_nerf(const void* in, const void* w, const void* image, uint32_t B, uint32_t in_dim,
                    const int32_t* count, const EpiNerfSigma& epi, bool pair_major, hipStream_t st) {
    if (pair_major)
        return launch_fwd_t<W, IN_KS, NH>(in, w, image, B, in_dim, ActReLU{}, ActNone{}, nullptr, count, epi, st,
                                          InPairMajor{B});
    return launch_fwd_t<W, IN_KS, NH>(in, w, image, B, in_dim, ActReLU{}, ActNone{}, nullptr, count, epi, st);
}

template <int W, int IN_KS, int NH>
int launch_fwd_density(const void* in, const void* w, const void* image, uint32_t B, uint32_t in_dim,
                       const EpiDensity& epi, hipStream_t st) {
    if (IN_KS == 1 && image) {  // the streaming kernel (prepacked image, 32 inputs)
        using N = Net<W, 1, NH>;
        const size_t lds = (size_t)N::FWD_FRAGS * 64 * 16;
        // the workgroups resident at once (occupancy x CUs, queried once per
        // device and shape): each wave then streams its share of the chunks
        static int resident[16] = {0};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16)
            return ngp_set_error(NGP_ERR_HIP, "nerf_density_forward: no current device");
        if (resident[dev] == 0) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_density_fwd<W, NH>, kThreads, lds) !=
                    hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                return ngp_set_error(NGP_ERR_HIP, "nerf_density_forward: occupancy query failed");
            resident[dev] = std::max(1, per_cu) * std::max(1, cus);
        }
        const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
        const uint32_t blocks = std::min<uint32_t>(ngp_div_up(nchunks, kWaves), (uint32_t)resident[dev]);
        if (blocks == 0) return NGP_OK;
        hipLaunchKernelGGL((k_density_fwd<W, NH>), dim3(blocks), dim3(kThreads), lds, st, (const ngp_half*)in,
                           (const half8*)image, B, epi);
        return ngp_check_launch("nerf_density_forward");
    }
    return launch_fwd_t<W, IN_KS, NH>(in, w, image, B, in_dim, ActReLU{}, ActNone{}, nullptr, nullptr, epi, st,
                                      InPairMajor{B});
}

template <int W, int NHS, int NHC>
int launch_nerf_fwd(const void* enc, const void* img_s, const void* img_c, uint32_t B, const int32_t* count,
                    const EpiNerfSigma& es, void* color_out, hipStream_t st) {
    const size_t lds = (size_t)(Net<W, 1, NHS>::FWD_FRAGS + Net<W, 1, NHC>::FWD_FRAGS) * 64 * 16;
    const uint32_t nchunks = ngp_div_up(B, 16 * kNB);
    uint32_t blocks = ngp_div_up(nchunks, kWaves);
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) return NGP_OK;
    hipLaunchKernelGGL((k_nerf_fwd<W, NHS, NHC>), dim3(blocks), dim3(kThreads), lds, st, (const ngp_half*)enc,
                       (const half8*)img_s, (const half8*)img_c, B, count, es, (ngp_half*)color_out);
    return ngp_check_launch("nerf_forward");
}

constexpr size_t kImageBytes = 128 * 1024;  // fragment image slot at the head of the workspace

template <int W, int IN_KS, int NH>
size_t image_bytes_t() {
    using N = Net<W, IN_KS, NH>;
    return (size_t)(N::FWD_FRAGS + N::BWD_FRAGS) * 64 * sizeof(half8);
}

// Pack jobs of one network: forward fragments of every matmul, then the
// transposed (backward) ones, into one image.
template <int W, int IN_KS, int NH>
int add_pack_jobs(PackJobs& jobs, const void* w, uint32_t in_dim, void* image) {
    using N = Net<W, IN_KS, NH>;
    NGP_REQUIRE(jobs.n + 2 * N::NMAT <= kMaxPackJobs, NGP_ERR_ARG, "ffmlp_pack: too many networks");
    for (int q = 0; q < N::NMAT; ++q) {
        jobs.job[jobs.n++] = PackJob{(const ngp_half*)w, (half8*)image, fwd_desc<W, IN_KS, NH>(q, in_dim), 0u};
        MatDesc mb = bwd_desc<W, IN_KS, NH>(q, in_dim);
        mb.frag0 += N::FWD_FRAGS;
        jobs.job[jobs.n++] = PackJob{(const ngp_half*)w, (half8*)image, mb, 1u};
    }
    return NGP_OK;
}

template <int W, int IN_KS, int NH, typename FA, typename GI, typename XL = InRowMajor>
int launch_bwd_t(const void* grad, const void* in, const void* w, const void* image, uint32_t B,
                 uint32_t in_dim, FA act, GI gi, bool want_gi, void* gw, int32_t gw_dtype, bool defer,
                 void* ws, const int32_t* count, hipStream_t st, XL xl = XL{}) {
    using L = BwdLds<W, IN_KS, NH>;
    static_assert(L::frag_bytes <= kImageBytes, "fragment image exceeds its workspace slot");
    static_assert(L::total <= 160 * 1024, "backward LDS budget exceeded");
    const uint32_t blocks = bwd_blocks(B);
    const uint32_t np = num_params(in_dim, W, NH + 1);
    if (blocks == 0) return NGP_OK;
    float* slab = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + kImageBytes);
    if (!image) {
        PackJobs jobs{};
        add_pack_jobs<W, IN_KS, NH>(jobs, w, in_dim, ws);
        hipLaunchKernelGGL(k_mlp_pack_jobs, dim3(jobs.n), dim3(256), 0, st, jobs);
        image = ws;
    }
    hipLaunchKernelGGL((k_mlp_bwd<W, IN_KS, NH, FA, XL, GI>), dim3(blocks), dim3(kBwdThreads), L::total, st,
                       (const ngp_half*)grad, (const ngp_half*)in, (const half8*)image, xl, gi, want_gi, slab,
                       np, B, in_dim, act, count);
    if (!defer) {
        ReduceJobs rj{};
        rj.n = 1;
        rj.slab[0] = slab;
        rj.out[0] = gw;
        rj.rows[0] = blocks;
        rj.np[0] = np;
        rj.block0[0] = 0;
        rj.block0[1] = ngp_div_up(np, 64);
        if (gw_dtype == NGP_DTYPE_F16)
            hipLaunchKernelGGL(k_slab_reduce<ngp_half>, dim3(rj.block0[1]), dim3(64 * kReducePhases), 0, st, rj);
        else
            hipLaunchKernelGGL(k_slab_reduce<float>, dim3(rj.block0[1]), dim3(64 * kReducePhases), 0, st, rj);
    }
    return ngp_check_launch("ffmlp_backward");
}

template <int W, int IN_KS, int NH>
int launch_bwd(const void* grad, const void* in, const void* w, const void* image, uint32_t B,
               uint32_t in_dim, uint32_t act, void* grad_in, bool nerf_geo, void* gw, int32_t gw_dtype,
               bool defer, void* ws, const int32_t* count, hipStream_t st, bool pair_major = false) {
    const bool want = grad_in != nullptr;
    ngp_half* gi = static_cast<ngp_half*>(grad_in);
    if (pair_major) {
        NGP_REQUIRE(!nerf_geo && act == kReLU, NGP_ERR_UNSUPPORTED,
                    "ffmlp_backward: pair-major inputs need ReLU and a plain grad_inputs store");
        return launch_bwd_t<W, IN_KS, NH>(grad, in, w, image, B, in_dim, ActReLU{}, GiPairMajor{gi, B}, want, gw,
                                          gw_dtype, defer, ws, count, st, InPairMajor{B});
    }
    if (nerf_geo) {
        NGP_REQUIRE(act == kReLU && IN_KS == 1 && in_dim == 32, NGP_ERR_UNSUPPORTED,
                    "ffmlp_backward: NeRF geo-feature gradients need ReLU and a 32-wide input");
        if constexpr (IN_KS == 1)
            return launch_bwd_t<W, IN_KS, NH>(grad, in, w, image, B, in_dim, ActReLU{}, GiNerfGeo{gi}, want, gw,
                                              gw_dtype, defer, ws, count, st);
    }
    if (act == kReLU)
        return launch_bwd_t<W, IN_KS, NH>(grad, in, w, image, B, in_dim, ActReLU{}, GiStore{gi}, want, gw,
                                          gw_dtype, defer, ws, count, st);
    return launch_bwd_t<W, IN_KS, NH>(grad, in, w, image, B, in_dim, ActAny{act}, GiStore{gi}, want, gw,
                                      gw_dtype, defer, ws, count, st);
}

template <int NHS, int NHC>
int launch_nerf_bwd(const NerfBwdArgs& a, hipStream_t st) {
    if constexpr (!NerfBwdLds<NHS, NHC>::fits) {
        return ngp_set_error(NGP_ERR_UNSUPPORTED, "nerf_backward: networks too large for one launch's LDS");
    } else {
        const uint32_t blocks = bwd_blocks(a.B);
        if (blocks == 0) return NGP_OK;
        constexpr size_t lds_bytes = NerfBwdLds<NHS, NHC>::total;
        hipLaunchKernelGGL((k_nerf_bwd<NHS, NHC>), dim3(blocks), dim3(kBwdThreads), lds_bytes, st, a);
        return ngp_check_launch("nerf_backward");
    }
}

#define MLP_DISPATCH(FN, ...)                                                              \
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

size_t image_bytes(uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers) {
    MLP_DISPATCH(image_bytes_t);
}

int pack_one(PackJobs& jobs, const void* w, uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers,
             void* image) {
    MLP_DISPATCH(add_pack_jobs, jobs, w, in_dim, image);
}

}  // namespace

extern "C" int ngp_ffmlp_forward(const void* inputs, const void* weights, uint32_t B,
                                 uint32_t in_dim, uint32_t output_dim, uint32_t hidden_dim,
                                 uint32_t num_layers, uint32_t activation,
                                 uint32_t output_activation, void* forward_buffer, void* outputs,
                                 void* stream) {
    if (int e = check_shape(B, in_dim, output_dim, hidden_dim, num_layers)) return e;
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    MLP_DISPATCH(launch_fwd, inputs, weights, nullptr, B, in_dim, activation, output_activation,
                     forward_buffer, outputs, nullptr, st);
}

/* Fused-step variant: rows at or past *count are not computed (count may be
 * null); image (nullable) is the network's ngp_ffmlp_pack image. */
extern "C" int ngp_ffmlp_forward_rows(const void* inputs, const void* weights, const void* image,
                                      uint32_t B, const int32_t* count, uint32_t in_dim,
                                      uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                                      uint32_t activation, uint32_t output_activation, void* outputs,
                                      void* stream) {
    if (int e = check_shape(B, in_dim, output_dim, hidden_dim, num_layers)) return e;
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    MLP_DISPATCH(launch_fwd, inputs, weights, image, B, in_dim, activation, output_activation,
                     nullptr, outputs, count, st);
}

extern "C" int ngp_nerf_sigma_forward(const void* inputs, const void* weights, const void* image, uint32_t B,
                                      const int32_t* count, uint32_t in_dim, uint32_t hidden_dim,
                                      uint32_t num_layers, void* h_out, float* sigma, void* color_in,
                                      const float* dirs, float density_scale, uint32_t flags, void* stream) {
    if (int e = check_shape(B, in_dim, kOut, hidden_dim, num_layers)) return e;
    NGP_REQUIRE(h_out && sigma && color_in && dirs, NGP_ERR_ARG, "nerf_sigma_forward: null output");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    const EpiNerfSigma epi{static_cast<ngp_half*>(h_out), sigma, static_cast<ngp_half*>(color_in), dirs,
                           density_scale};
    MLP_DISPATCH(launch_fwd_nerf, inputs, weights, image, B, in_dim, count, epi,
                     (flags & NGP_FFMLP_PAIR_MAJOR) != 0, st);
}

extern "C" int ngp_nerf_forward(const void* enc, const void* sigma_image, const void* color_image, uint32_t B,
                                const int32_t* count, uint32_t hidden_dim, uint32_t num_layers,
                                uint32_t hidden_dim_color, uint32_t num_layers_color, void* h_out, float* sigma,
                                void* color_in, const float* dirs, float density_scale, void* color_out,
                                void* stream) {
    NGP_REQUIRE(hidden_dim == 64 && hidden_dim_color == 64, NGP_ERR_UNSUPPORTED,
                "nerf_forward: 64-wide networks only on this build, got %u / %u", hidden_dim, hidden_dim_color);
    NGP_REQUIRE(num_layers >= 2 && num_layers <= 3 && num_layers_color >= 2 && num_layers_color <= 4,
                NGP_ERR_UNSUPPORTED, "nerf_forward: num_layers in [2, 3] (sigma) / [2, 4] (color), got %u / %u",
                num_layers, num_layers_color);
    NGP_REQUIRE(enc && sigma_image && color_image && h_out && sigma && color_in && dirs && color_out, NGP_ERR_ARG,
                "nerf_forward: null pointer");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    const EpiNerfSigma es{static_cast<ngp_half*>(h_out), sigma, static_cast<ngp_half*>(color_in), dirs,
                          density_scale};
    const uint32_t key = (num_layers - 1) * 8 + (num_layers_color - 1);
    switch (key) {
        case 1 * 8 + 1: return launch_nerf_fwd<64, 1, 1>(enc, sigma_image, color_image, B, count, es, color_out, st);
        case 1 * 8 + 2: return launch_nerf_fwd<64, 1, 2>(enc, sigma_image, color_image, B, count, es, color_out, st);
        case 1 * 8 + 3: return launch_nerf_fwd<64, 1, 3>(enc, sigma_image, color_image, B, count, es, color_out, st);
        case 2 * 8 + 1: return launch_nerf_fwd<64, 2, 1>(enc, sigma_image, color_image, B, count, es, color_out, st);
        case 2 * 8 + 2: return launch_nerf_fwd<64, 2, 2>(enc, sigma_image, color_image, B, count, es, color_out, st);
        default: return launch_nerf_fwd<64, 2, 3>(enc, sigma_image, color_image, B, count, es, color_out, st);
    }
}

/* Both networks' backward of the fused step in one launch: the colour
 * network's (grad g_color_out [B,16], inputs color_in [B,32]; its input
 * gradient's geo columns into g_h[:, 1:16], as ngp_ffmlp_backward_rows with
 * NGP_FFMLP_NERF_GEO), then the sigma network's (grad g_h [B,16], inputs enc
 * pair-major [16][B][2], input gradient g_enc pair-major, as
 * NGP_FFMLP_PAIR_MAJOR). Both networks' dW partials are left in their
 * workspaces (ngp_ffmlp_backward_workspace_bytes of each network) for
 * ngp_ffmlp_reduce, as NGP_FFMLP_DEFER_REDUCE. Input gradients equal the two
 * calls bit for bit; dW is summed in another order. */
static int nerf_backward_impl(const void* g_color_out, const void* color_in, const void* color_image,
                              void* g_h, const void* enc, const void* sigma_image, void* g_enc, uint32_t B,
                              const int32_t* count, const int32_t* rows, uint32_t hidden_dim, uint32_t num_layers,
                              uint32_t hidden_dim_color, uint32_t num_layers_color, void* sigma_workspace,
                              size_t sigma_workspace_bytes, void* color_workspace, size_t color_workspace_bytes,
                              uint32_t* timing, void* stream) {
    NGP_REQUIRE(!rows || count, NGP_ERR_ARG, "nerf_backward_live: a row list needs its count");
    NGP_REQUIRE(hidden_dim == 64 && hidden_dim_color == 64, NGP_ERR_UNSUPPORTED,
                "nerf_backward: 64-wide networks only on this build, got %u / %u", hidden_dim, hidden_dim_color);
    NGP_REQUIRE(num_layers >= 2 && num_layers <= 3 && num_layers_color >= 2 && num_layers_color <= 3,
                NGP_ERR_UNSUPPORTED, "nerf_backward: num_layers in [2, 3] (sigma) / [2, 3] (color), got %u / %u",
                num_layers, num_layers_color);
    NGP_REQUIRE(g_color_out && color_in && color_image && g_h && enc && sigma_image && g_enc, NGP_ERR_ARG,
                "nerf_backward: null pointer");
    if (B == 0) return NGP_OK;
    const size_t need_s = ngp_ffmlp_backward_workspace_bytes(B, 32, kOut, hidden_dim, num_layers);
    const size_t need_c = ngp_ffmlp_backward_workspace_bytes(B, 32, kOut, hidden_dim_color, num_layers_color);
    NGP_REQUIRE(sigma_workspace && sigma_workspace_bytes >= need_s && color_workspace &&
                    color_workspace_bytes >= need_c,
                NGP_ERR_ARG, "nerf_backward: workspaces of %zu / %zu bytes required, got %zu / %zu", need_s, need_c,
                sigma_workspace_bytes, color_workspace_bytes);
    NerfBwdArgs a{};
    a.g_color_out = static_cast<const ngp_half*>(g_color_out);
    a.color_in = static_cast<const ngp_half*>(color_in);
    a.color_image = static_cast<const half8*>(color_image);
    a.g_h = static_cast<ngp_half*>(g_h);
    a.enc = static_cast<const ngp_half*>(enc);
    a.sigma_image = static_cast<const half8*>(sigma_image);
    a.g_enc = static_cast<ngp_half*>(g_enc);
    a.slab_color = reinterpret_cast<float*>(static_cast<char*>(color_workspace) + kImageBytes);
    a.slab_sigma = reinterpret_cast<float*>(static_cast<char*>(sigma_workspace) + kImageBytes);
    a.np_color = num_params(32, 64, num_layers_color);
    a.np_sigma = num_params(32, 64, num_layers);
    a.B = B;
    a.count = count;
    a.timing = timing;
    a.rows = rows;
    hipStream_t st = ngp_stream(stream);
    const uint32_t key = (num_layers - 1) * 8 + (num_layers_color - 1);
    switch (key) {
        case 1 * 8 + 1: return launch_nerf_bwd<1, 1>(a, st);
        case 1 * 8 + 2: return launch_nerf_bwd<1, 2>(a, st);
        case 2 * 8 + 1: return launch_nerf_bwd<2, 1>(a, st);
        default: return launch_nerf_bwd<2, 2>(a, st);
    }
}

extern "C" int ngp_nerf_backward(const void* g_color_out, const void* color_in, const void* color_image,
                                 void* g_h, const void* enc, const void* sigma_image, void* g_enc, uint32_t B,
                                 const int32_t* count, uint32_t hidden_dim, uint32_t num_layers,
                                 uint32_t hidden_dim_color, uint32_t num_layers_color, void* sigma_workspace,
                                 size_t sigma_workspace_bytes, void* color_workspace, size_t color_workspace_bytes,
                                 uint32_t* timing, void* stream) {
    return nerf_backward_impl(g_color_out, color_in, color_image, g_h, enc, sigma_image, g_enc, B, count, nullptr,
                              hidden_dim, num_layers, hidden_dim_color, num_layers_color, sigma_workspace,
                              sigma_workspace_bytes, color_workspace, color_workspace_bytes, timing, stream);
}

extern "C" int ngp_nerf_backward_live(const void* g_color_out, const void* color_in, const void* color_image,
                                      void* g_h, const void* enc, const void* sigma_image, void* g_enc, uint32_t B,
                                      const int32_t* live_rows, const int32_t* live_count, uint32_t hidden_dim,
                                      uint32_t num_layers, uint32_t hidden_dim_color, uint32_t num_layers_color,
                                      void* sigma_workspace, size_t sigma_workspace_bytes, void* color_workspace,
                                      size_t color_workspace_bytes, uint32_t* timing, void* stream) {
    NGP_REQUIRE(live_rows && live_count, NGP_ERR_ARG, "nerf_backward_live: null row list or count");
    return nerf_backward_impl(g_color_out, color_in, color_image, g_h, enc, sigma_image, g_enc, B, live_count,
                              live_rows, hidden_dim, num_layers, hidden_dim_color, num_layers_color, sigma_workspace,
                              sigma_workspace_bytes, color_workspace, color_workspace_bytes, timing, stream);
}

extern "C" int ngp_nerf_density_forward(const void* inputs, const void* weights, const void* image, uint32_t B,
                                        uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers,
                                        float density_scale, const int32_t* indices, float* tmp_grid,
                                        void* stream) {
    if (int e = check_shape(B, in_dim, kOut, hidden_dim, num_layers)) return e;
    NGP_REQUIRE(indices && tmp_grid, NGP_ERR_ARG, "nerf_density_forward: null indices / tmp_grid");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    const EpiDensity epi{tmp_grid, indices, density_scale, nullptr};
    MLP_DISPATCH(launch_fwd_density, inputs, weights, image, B, in_dim, epi, st);
}

extern "C" int ngp_nerf_density_forward_rows(const void* inputs, const void* image, uint32_t B, uint32_t hidden_dim,
                                             uint32_t num_layers, float density_scale, float* sigma, void* stream) {
    const uint32_t in_dim = 32;
    if (int e = check_shape(B, in_dim, kOut, hidden_dim, num_layers)) return e;
    NGP_REQUIRE(image && sigma, NGP_ERR_ARG, "nerf_density_forward_rows: null image / sigma");
    if (B == 0) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    const EpiDensity epi{nullptr, nullptr, density_scale, sigma};
    const void* weights = nullptr;
    MLP_DISPATCH(launch_fwd_density, inputs, weights, image, B, in_dim, epi, st);
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
    return kImageBytes + (size_t)bwd_blocks(B) * num_params(input_dim, hidden_dim, num_layers) * sizeof(float);
}

extern "C" size_t ngp_ffmlp_image_bytes(uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers) {
    if (check_shape(0, in_dim, kOut, hidden_dim, num_layers)) return 0;
    return image_bytes(in_dim, hidden_dim, num_layers);
}

int ngp_pack::build_jobs(int32_t n, const void* const* weights, const uint32_t* in_dims,
                         const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* images,
                         PackJobs& jobs) {
    NGP_REQUIRE(n >= 1 && weights && in_dims && hidden_dims && num_layers && images, NGP_ERR_ARG,
                "ffmlp_pack: bad arguments");
    for (int k = 0; k < n; ++k) {
        if (int e = check_shape(0, in_dims[k], kOut, hidden_dims[k], num_layers[k])) return e;
        NGP_REQUIRE(weights[k] && images[k], NGP_ERR_ARG, "ffmlp_pack: null weights or image %d", k);
        if (int e = pack_one(jobs, weights[k], in_dims[k], hidden_dims[k], num_layers[k], images[k])) return e;
    }
    return NGP_OK;
}

extern "C" int ngp_ffmlp_pack(int32_t n, const void* const* weights, const uint32_t* in_dims,
                              const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* images,
                              void* stream) {
    PackJobs jobs{};
    if (int e = ngp_pack::build_jobs(n, weights, in_dims, hidden_dims, num_layers, images, jobs)) return e;
    hipLaunchKernelGGL(k_mlp_pack_jobs, dim3(jobs.n), dim3(256), 0, ngp_stream(stream), jobs);
    return ngp_check_launch("ffmlp_pack");
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
    MLP_DISPATCH(launch_bwd, grad, inputs, weights, nullptr, B, in_dim, activation, gi, false, grad_weights,
                     gw_dtype, false, workspace, nullptr, st);
}

/* Fused-step variant: rows at or past *count contribute nothing (their
 * grad_inputs are not written). image: the ngp_ffmlp_pack image (nullable:
 * packed into the workspace). flags: NGP_FFMLP_DEFER_REDUCE leaves the
 * per-workgroup dW partial sums in the workspace for ngp_ffmlp_reduce;
 * NGP_FFMLP_NERF_GEO writes the input gradient's columns 16..30 into columns
 * 1..15 of grad_inputs [B, 16] (the NeRF color network's geo features). */
extern "C" int ngp_ffmlp_backward_rows(const void* grad, const void* inputs, const void* weights,
                                       const void* image, uint32_t B, const int32_t* count, uint32_t in_dim,
                                       uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                                       uint32_t activation, void* grad_inputs, void* grad_weights,
                                       int32_t gw_dtype, uint32_t flags, void* workspace,
                                       size_t workspace_bytes, void* stream) {
    if (int e = check_shape(B, in_dim, output_dim, hidden_dim, num_layers)) return e;
    NGP_REQUIRE(gw_dtype == NGP_DTYPE_F16 || gw_dtype == NGP_DTYPE_F32, NGP_ERR_ARG,
                "grad_weights must be float16 or float32");
    if (B == 0) return NGP_OK;
    const size_t need = ngp_ffmlp_backward_workspace_bytes(B, in_dim, output_dim, hidden_dim, num_layers);
    NGP_REQUIRE(workspace && workspace_bytes >= need, NGP_ERR_ARG,
                "ffmlp_backward: workspace of %zu bytes required, got %zu", need, workspace_bytes);
    hipStream_t st = ngp_stream(stream);
    const bool geo = (flags & NGP_FFMLP_NERF_GEO) != 0, defer = (flags & NGP_FFMLP_DEFER_REDUCE) != 0;
    const bool pm = (flags & NGP_FFMLP_PAIR_MAJOR) != 0;
    MLP_DISPATCH(launch_bwd, grad, inputs, weights, image, B, in_dim, activation, grad_inputs, geo,
                     grad_weights, gw_dtype, defer, workspace, count, st, pm);
}

/* Sums the deferred dW partials of n backward calls (same B / shapes as
 * those calls) into grad_weights[k], one launch. */
uint32_t ngp_reduce::build_reduce_jobs(int32_t n, void* const* workspaces, const uint32_t* Bs,
                                       const uint32_t* in_dims, const uint32_t* hidden_dims,
                                       const uint32_t* num_layers, void* const* grad_weights, int32_t* nonfinite,
                                       ReduceJobs& rj) {
    rj = ReduceJobs{};
    rj.nonfinite = nonfinite;
    uint32_t blocks = 0;
    for (int k = 0; k < n && k < kMaxReduceJobs; ++k) {
        const uint32_t rows = bwd_blocks(Bs[k]);
        if (rows == 0) continue;
        const int j = rj.n++;
        rj.slab[j] = reinterpret_cast<const float*>(static_cast<const char*>(workspaces[k]) + kImageBytes);
        rj.out[j] = grad_weights[k];
        rj.rows[j] = rows;
        rj.np[j] = num_params(in_dims[k], hidden_dims[k], num_layers[k]);
        rj.block0[j] = blocks;
        blocks += ngp_div_up(rj.np[j], 64);
    }
    rj.block0[rj.n] = blocks;
    return blocks;
}

int ngp_reduce::launch_slab_reduce(const ReduceJobs& rj, uint32_t blocks, void* stream) {
    if (blocks == 0) return NGP_OK;
    hipLaunchKernelGGL(k_slab_reduce<ngp_half>, dim3(blocks), dim3(64 * kReducePhases), 0, ngp_stream(stream), rj);
    return ngp_check_launch("ffmlp_reduce");
}

extern "C" int ngp_ffmlp_reduce(int32_t n, void* const* workspaces, const uint32_t* Bs, const uint32_t* in_dims,
                                const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* grad_weights,
                                int32_t gw_dtype, int32_t* nonfinite, void* stream) {
    NGP_REQUIRE(n >= 1 && n <= kMaxReduceJobs, NGP_ERR_ARG, "ffmlp_reduce: 1..%d networks", kMaxReduceJobs);
    NGP_REQUIRE(gw_dtype == NGP_DTYPE_F16 || gw_dtype == NGP_DTYPE_F32, NGP_ERR_ARG,
                "grad_weights must be float16 or float32");
    ReduceJobs rj{};
    const uint32_t blocks = ngp_reduce::build_reduce_jobs(n, workspaces, Bs, in_dims, hidden_dims, num_layers,
                                                          grad_weights, nonfinite, rj);
    if (blocks == 0) return NGP_OK;
    if (gw_dtype == NGP_DTYPE_F16)
        hipLaunchKernelGGL(k_slab_reduce<ngp_half>, dim3(blocks), dim3(64 * kReducePhases), 0, ngp_stream(stream), rj);
    else
        hipLaunchKernelGGL(k_slab_reduce<float>, dim3(blocks), dim3(64 * kReducePhases), 0, ngp_stream(stream), rj);
    return ngp_check_launch("ffmlp_reduce");
}

extern "C" int ngp_ffmlp_allocate_splitk(size_t size) { (void)size; return NGP_OK; }
extern "C" int ngp_ffmlp_free_splitk(void) { return NGP_OK; }

#ifdef NGP_STAMPS
extern "C" int ngp_debug_mlp_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_mlp_stamps), &buf, sizeof(buf)) == hipSuccess ? NGP_OK : NGP_ERR_HIP;
}
#endif
