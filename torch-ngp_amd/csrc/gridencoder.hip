// Multiresolution hash-grid encoder, forward / backward / TV-grad, for gfx950.
//
// Semantics follow the reference kernels line by line:
//   fast_hash           gridencoder/src/gridencoder.cu:50-63
//   get_grid_index      gridencoder.cu:66-84
//   kernel_grid         gridencoder.cu:87-242   -> k_grid_fwd
//   kernel_grid_backward gridencoder.cu:245-337 -> k_grid_bwd
//   kernel_input_backward gridencoder.cu:340-366 -> k_grid_input_bwd
//   kernel_grad_tv      gridencoder.cu:503-607  -> k_grid_tv
//
// MI355X design:
//   * level-major scheduling: blockIdx.y = level, so the whole chip walks one
//     level's table slice at a time. The largest hashed level is 2^19 entries =
//     2 MiB in fp16, which fits one XCD's 4 MiB L2: the 8 random corner gathers
//     per (point, level) are L2 hits instead of Infinity-Cache hits.
//   * one lane per (point, level) handles all C channels of a corner with one
//     vector access (C=2 fp16: one dword gather, one global_atomic_pk_add_f16).
//   * out_layout 1 writes [B, L*C] directly (what the MLP consumes), removing
//     the reference's permute copy (grid.py:69) and its grad permute (grid.py:87).
//   * per-level scale/resolution are computed once on the host (exp2 in double,
//     rounded to float) and passed as kernel arguments.
//   * a hashed level's size is a power of two: the modulo becomes a mask.
#include "ngp_common.h"

#include <cmath>

namespace {

constexpr uint32_t kMaxLevels = 64;

struct GridLevels {
    float scale[kMaxLevels];
    uint32_t res[kMaxLevels];
};

// reference semantics: scale = exp2f(level * S) * H - 1.0f;
// resolution = (uint32_t)ceil(scale) + 1   (gridencoder.cu:138-139)
static void make_levels(GridLevels& lv, uint32_t L, float S, uint32_t H) {
    for (uint32_t l = 0; l < L; ++l) {
        float ls = (float)l * S;
        float e = (float)std::exp2((double)ls);
        float scale = e * (float)H - 1.0f;
        lv.scale[l] = scale;
        lv.res[l] = (uint32_t)std::ceil(scale) + 1u;
    }
}

template <uint32_t D>
NGP_DEV uint32_t fast_hash(const uint32_t pos_grid[D]) {
    constexpr uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                    2097192037u, 1434869437u, 2165219737u};
    uint32_t result = 0;
#pragma unroll
    for (uint32_t i = 0; i < D; ++i) result ^= pos_grid[i] * primes[i];
    return result;
}

// Returns the entry index (not multiplied by C). `hs_mask` is hs-1 when hs is
// a power of two, else 0 (then a true modulo is taken).
template <uint32_t D>
NGP_DEV uint32_t grid_index(uint32_t gridtype, bool align_corners, uint32_t hs, uint32_t hs_mask,
                            uint32_t resolution, const uint32_t pos_grid[D]) {
    uint32_t stride = 1;
    uint32_t index = 0;
#pragma unroll
    for (uint32_t d = 0; d < D && stride <= hs; d++) {
        index += pos_grid[d] * stride;
        stride *= align_corners ? resolution : (resolution + 1);
    }
    if (gridtype == 0 && stride > hs) index = fast_hash<D>(pos_grid);
    return hs_mask ? (index & hs_mask) : (index % hs);
}

NGP_DEV float smoothstep(float v) { return v * v * (3.0f - 2.0f * v); }
NGP_DEV float smoothstep_derivative(float v) { return 6 * v * (1.0f - v); }

// Vector load/store of the C channels of one entry (entries are aligned to
// C*sizeof(T) because offsets are multiples of 8 entries).
template <typename T, uint32_t C>
NGP_DEV void load_entry(const T* __restrict__ p, typename Acc<T>::F out[C]) {
    struct alignas(sizeof(T) * C) V { T v[C]; };
    V x = *reinterpret_cast<const V*>(p);
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) out[c] = (typename Acc<T>::F)x.v[c];
}
// Entry stored as E, computed as T: (F)(T)e, i.e. the reference's
// embeddings.half() applied on the fly to an fp32 table.
template <typename T, typename E, uint32_t C>
NGP_DEV void load_entry_as(const E* __restrict__ p, typename Acc<T>::F out[C]) {
    struct alignas(sizeof(E) * C) V { E v[C]; };
    V x = *reinterpret_cast<const V*>(p);
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) out[c] = (typename Acc<T>::F)(T)x.v[c];
}

// Optional input mapping of the fused train step: x = (raw + shift) * scale
// (GridEncoder.forward's (inputs + bound) / (2 * bound), which torch evaluates
// as a multiply by the fp32 reciprocal), and a device-side row count that
// clips B (rows past the marcher's sample count are not touched).
struct InMap {
    float shift, scale;  // scale == 0: inputs are used as given
    const int32_t* count;
};
NGP_DEV uint32_t rows_of(uint32_t B, const InMap& m) {
    if (!m.count) return B;
    const int32_t c = *m.count;
    return c <= 0 ? 0u : min(B, (uint32_t)c);
}

template <typename T, uint32_t C>
NGP_DEV void store_entry(T* __restrict__ p, const T in[C]) {
    struct alignas(sizeof(T) * C) V { T v[C]; };
    V x;
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) x.v[c] = in[c];
    *reinterpret_cast<V*>(p) = x;
}

template <typename T, typename E, uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_fwd(const float* __restrict__ inputs, const E* __restrict__ grid,
           const int32_t* __restrict__ offsets, T* __restrict__ outputs, uint32_t B, uint32_t L,
           GridLevels lv, T* __restrict__ dy_dx, uint32_t gridtype, bool align_corners,
           uint32_t interp, int32_t out_layout, InMap im) {
    using A = Acc<T>;
    using F = typename A::F;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= rows_of(B, im)) return;
    const uint32_t level = blockIdx.y;

    T* out = out_layout == 0 ? outputs + ((size_t)level * B + b) * C
                             : outputs + ((size_t)b * L + level) * C;

    float x[D];
    bool oob = false;
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = inputs[(size_t)b * D + d];
        if (im.scale != 0.0f) x[d] = (x[d] + im.shift) * im.scale;
        if (x[d] < 0 || x[d] > 1) oob = true;
    }
    if (oob) {
        T z[C];
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) z[c] = A::zero();
        store_entry<T, C>(out, z);
        if (dy_dx) {
            T* g = dy_dx + (size_t)b * D * L * C + level * D * C;
#pragma unroll
            for (uint32_t i = 0; i < D * C; ++i) g[i] = A::zero();
        }
        return;
    }

    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t hs_mask = (hs & (hs - 1)) == 0 ? hs - 1 : 0;
    const E* __restrict__ g = grid + (size_t)off0 * C;
    const float scale = lv.scale[level];
    const uint32_t resolution = lv.res[level];

    float pos[D], pos_deriv[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
        pos_deriv[d] = 1.0f;  // reference bug at :143 zero-inits d >= 1; see DESIGN.md
        if (interp == 1) {
            pos_deriv[d] = smoothstep_derivative(pos[d]);
            pos[d] = smoothstep(pos[d]);
        }
    }

    typename A::S res[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) res[c] = A::zero();

#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); idx++) {
        float w = 1;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) {
                w *= 1 - pos[d];
                pl[d] = pg[d];
            } else {
                w *= pos[d];
                pl[d] = pg[d] + 1;
            }
        }
        const uint32_t e = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl);
        F v[C];
        load_entry_as<T, E, C>(g + (size_t)e * C, v);
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) res[c] = A::mac(res[c], (F)w, v[c]);
    }
    store_entry<T, C>(out, res);

    if (dy_dx) {
        T* dd = dy_dx + (size_t)b * D * L * C + level * D * C;
#pragma unroll
        for (uint32_t gd = 0; gd < D; gd++) {
            typename A::S rg[C];
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) rg[c] = A::zero();
#pragma unroll
            for (uint32_t idx = 0; idx < (1u << (D - 1)); idx++) {
                float w = scale;
                uint32_t pl[D];
#pragma unroll
                for (uint32_t nd = 0; nd < D - 1; nd++) {
                    const uint32_t d = (nd >= gd) ? (nd + 1) : nd;
                    if ((idx & (1u << nd)) == 0) {
                        w *= 1 - pos[d];
                        pl[d] = pg[d];
                    } else {
                        w *= pos[d];
                        pl[d] = pg[d] + 1;
                    }
                }
                pl[gd] = pg[gd];
                const uint32_t il = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl);
                pl[gd] = pg[gd] + 1;
                const uint32_t ir = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl);
                F vl[C], vr[C];
                load_entry_as<T, E, C>(g + (size_t)il * C, vl);
                load_entry_as<T, E, C>(g + (size_t)ir * C, vr);
#pragma unroll
                for (uint32_t c = 0; c < C; ++c)
                    rg[c] = A::mac(rg[c], (F)w * (vr[c] - vl[c]), (F)pos_deriv[gd]);
            }
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) dd[gd * C + c] = rg[c];
        }
    }
}

// Forward without dy_dx: two lanes per (point, level). The lane with x bit b
// gathers the 2^(D-1) corners whose x offset is b, which neighbour its
// partner's (x prime 1 / dense stride 1): each gather instruction touches one
// cache line per lane PAIR. The partner's values arrive by one shuffle and
// both lanes accumulate all 2^D corners in the reference's order, so the
// result is bit-identical to k_grid_fwd; the even lane stores it.
template <typename T, typename E, uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_fwd_pair(const float* __restrict__ inputs, const E* __restrict__ grid,
                const int32_t* __restrict__ offsets, T* __restrict__ outputs, uint32_t B, uint32_t L,
                GridLevels lv, uint32_t gridtype, bool align_corners, uint32_t interp,
                int32_t out_layout, InMap im) {
    using A = Acc<T>;
    using F = typename A::F;
    const uint32_t b = blockIdx.x * (blockDim.x / 2) + (threadIdx.x >> 1);
    const uint32_t xbit = threadIdx.x & 1;
    const uint32_t level = blockIdx.y;
    const bool live = b < rows_of(B, im);
    if (__ballot(live) == 0) return;  // wave-uniform exit; pairs stay together below

    float x[D];
    bool oob = !live;
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = live ? inputs[(size_t)b * D + d] : 0.5f;
        if (im.scale != 0.0f) x[d] = (x[d] + im.shift) * im.scale;
        if (x[d] < 0 || x[d] > 1) oob = true;
    }
    T* out = out_layout == 0 ? outputs + ((size_t)level * B + b) * C
                             : outputs + ((size_t)b * L + level) * C;

    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t hs_mask = (hs & (hs - 1)) == 0 ? hs - 1 : 0;
    const E* __restrict__ g = grid + (size_t)off0 * C;
    const float scale = lv.scale[level];
    const uint32_t resolution = lv.res[level];

    float pos[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
        if (interp == 1) pos[d] = smoothstep(pos[d]);
    }
    // this lane's corners: idx = (rest << 1) | xbit
    F mine[1u << (D - 1)][C];
#pragma unroll
    for (uint32_t rest = 0; rest < (1u << (D - 1)); rest++) {
        const uint32_t idx = (rest << 1) | xbit;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) pl[d] = (idx & (1u << d)) ? pg[d] + 1 : pg[d];
        if (!oob) {
            const uint32_t e = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl);
            load_entry_as<T, E, C>(g + (size_t)e * C, mine[rest]);
        } else {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) mine[rest][c] = 0;
        }
    }
    typename A::S res[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) res[c] = A::zero();
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); idx++) {
        float w = 1;
#pragma unroll
        for (uint32_t d = 0; d < D; d++) w *= (idx & (1u << d)) ? pos[d] : 1 - pos[d];
        const uint32_t rest = idx >> 1;
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) {
            const F other = (F)__shfl_xor((float)mine[rest][c], 1, 64);
            const F v = ((idx & 1u) == xbit) ? mine[rest][c] : other;
            res[c] = A::mac(res[c], (F)w, v);
        }
    }
    if (live && xbit == 0) {
        if (oob) {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) res[c] = A::zero();
        }
        store_entry<T, C>(out, res);
    }
}

// ---- scatter-add of one corner's C channels (values already weighted) -----
template <typename T, uint32_t C> struct Scatter;
template <uint32_t C> struct Scatter<float, C> {
    NGP_DEV static void add(float* p, const float v[C]) {
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) atomicAdd(p + c, v[c]);
    }
};
template <uint32_t C> struct Scatter<double, C> {
    NGP_DEV static void add(double* p, const double v[C]) {
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) atomicAdd(p + c, v[c]);
    }
};
template <uint32_t C> struct Scatter<ngp_half, C> {
    NGP_DEV static void add(ngp_half* p, const float v[C]) {
        if constexpr (C % 2 == 0) {
#pragma unroll
            for (uint32_t c = 0; c < C; c += 2) {
                ngp_half2 h = {(ngp_half)v[c], (ngp_half)v[c + 1]};
                __builtin_amdgcn_global_atomic_fadd_v2f16(reinterpret_cast<ngp_half2*>(p + c), h);
            }
        } else {
            // C == 1: packed add of (v, 0) into the aligned dword holding the entry.
            const uintptr_t a = reinterpret_cast<uintptr_t>(p);
            ngp_half2* base = reinterpret_cast<ngp_half2*>(a & ~uintptr_t(3));
            const ngp_half hv = (ngp_half)v[0];
            ngp_half2 h = (a & 2) ? ngp_half2{(ngp_half)0.0f, hv} : ngp_half2{hv, (ngp_half)0.0f};
            __builtin_amdgcn_global_atomic_fadd_v2f16(base, h);
        }
    }
};

// Scatter-add with corner pairing and wave-level merging of identical targets.
//
// Float atomics execute at the memory side, one 64-B request per distinct
// 64-B segment a wave instruction touches (MI355X_MICROARCH.md "Global float
// atomics"), so the request count, not the add count, sets the time. Two
// lanes per (point, level): lane pair (2s, 2s+1) handles the corners with
// x = floor and x = floor + 1 of point s, which are neighbouring entries on
// dense levels and on hashed ones (the x prime of the hash is 1), i.e. one
// request per pair instead of two. Each lane then walks the 2^(D-1) corners
// of the remaining dimensions.
//
// Samples arrive ordered along rays, so on the coarse levels consecutive
// points hit the same cell: per corner, lanes whose target equals that of the
// lane two to the left (same x parity) form a run; a segmented inclusive scan
// (stride-2 shuffles) sums each run into its last lane, which issues ONE
// atomic for the whole run. A ballot skips the scan when nothing collides
// (the fine hashed levels). For fp16 tables each run adds (half)(sum of w*g)
// instead of rounding every term (the reference rounds each term,
// gridencoder.cu:325), i.e. the same values with fewer roundings.
template <typename T, uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_bwd(const T* __restrict__ grad, const float* __restrict__ inputs,
           const int32_t* __restrict__ offsets, T* __restrict__ grad_grid, uint32_t B, uint32_t L,
           GridLevels lv, uint32_t gridtype, bool align_corners, uint32_t interp,
           int32_t grad_layout, InMap im, uint32_t level0) {
    using A = Acc<T>;
    using F = typename A::F;
    const uint32_t b = blockIdx.x * (blockDim.x / 2) + (threadIdx.x >> 1);
    const uint32_t xbit = threadIdx.x & 1;
    const uint32_t level = level0 + blockIdx.y;
    const int lane = (int)(threadIdx.x & 63);

    bool valid = b < rows_of(B, im);
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = valid ? inputs[(size_t)b * D + d] : 0.5f;
        if (valid && im.scale != 0.0f) x[d] = (x[d] + im.shift) * im.scale;
        if (x[d] < 0 || x[d] > 1) valid = false;  // grad is zero-initialised
    }
    if (__ballot(valid) == 0) return;  // whole wave idle (wave-uniform)

    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t hs_mask = (hs & (hs - 1)) == 0 ? hs - 1 : 0;
    T* __restrict__ gg = grad_grid + (size_t)off0 * C;
    const float scale = lv.scale[level];
    const uint32_t resolution = lv.res[level];

    float pos[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
        if (interp == 1) pos[d] = smoothstep(pos[d]);
    }

    F gcur[C];
    if (valid) {
        const T* gp = grad_layout == 0 ? grad + ((size_t)level * B + b) * C
                                       : grad + ((size_t)b * L + level) * C;
        load_entry<T, C>(gp, gcur);
    } else {
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) gcur[c] = 0;
    }

#pragma unroll
    for (uint32_t rest = 0; rest < (1u << (D - 1)); rest++) {
        const uint32_t idx = (rest << 1) | xbit;  // corner bits, dimension 0 = x from the lane
        float w = 1;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) {
                w *= 1 - pos[d];
                pl[d] = pg[d];
            } else {
                w *= pos[d];
                pl[d] = pg[d] + 1;
            }
        }
        const uint32_t key = valid ? grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl)
                                   : 0xffffffffu;
        F v[C];
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) v[c] = (F)w * gcur[c];

        const uint32_t kprev = __shfl_up(key, 2, 64);
        const bool same = lane > 1 && kprev == key;
        if (__ballot(same) == 0) {
            if (valid) Scatter<T, C>::add(gg + (size_t)key * C, v);
            continue;
        }
        // run start (same parity) = inclusive max-scan of head positions
        int start = same ? 0 : lane;
#pragma unroll
        for (int o = 2; o < 64; o <<= 1) {
            const int t = __shfl_up(start, o, 64);
            if (lane >= o) start = max(start, t);
        }
#pragma unroll
        for (int o = 2; o < 64; o <<= 1) {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) {
                const F t = __shfl_up(v[c], o, 64);
                if (lane - o >= start) v[c] += t;
            }
        }
        const uint32_t knext = __shfl_down(key, 2, 64);
        const bool tail = lane >= 62 || knext != key;
        if (valid && tail) Scatter<T, C>::add(gg + (size_t)key * C, v);
    }
}

// ---- binned backward for the hashed levels (fused train step) ----------------
// Scattered atomics on the hashed levels cost one memory-side request per
// (point, corner pair) whatever is done (no reuse between points at those
// resolutions), ~180 us per Lego step. Instead, the corner contributions of a
// hashed level are sorted into bins of 2^13 table entries: each workgroup
// (256 points of one level) ranks its 2048 contributions per bin in LDS,
// reserves space per bin with one atomic, and writes each bin's run
// contiguously; then one workgroup per bin sums its contributions in an LDS
// fp32 image of the bin's entries and adds that image to the fp16 table with
// plain loads/stores (every entry has one owner). Contributions are rounded
// to half per term, like the reference's Half += float (gridencoder.cu:325),
// and summed in fp32. Bins that overflow their capacity fall back to atomics.
constexpr uint32_t kBinShift = 13;
constexpr uint32_t kBinEntries = 1u << kBinShift;
constexpr uint32_t kMaxBinsPerLevel = 256;

struct BinPlan {
    uint32_t first_level;            // levels [first_level, L) are binned
    uint32_t total_bins;
    uint32_t cap;                    // contributions per bin
    uint32_t nbins[kMaxLevels];
    uint32_t bin0[kMaxLevels];
};

struct BinItem {
    uint32_t e;                      // entry within the bin (| bin << 16 while staged)
    ngp_half2 v;
};

template <uint32_t D>
__global__ void __launch_bounds__(256)
k_grid_bwd_bin(const ngp_half* __restrict__ grad, const float* __restrict__ inputs,
               const int32_t* __restrict__ offsets, ngp_half* __restrict__ grad_grid, uint32_t B,
               uint32_t L, GridLevels lv, uint32_t gridtype, bool align_corners, uint32_t interp,
               InMap im, BinPlan bp, uint32_t* __restrict__ cursor, BinItem* __restrict__ items) {
    constexpr uint32_t C = 2, NC = 1u << D;
    __shared__ uint32_t cnt[kMaxBinsPerLevel], base[kMaxBinsPerLevel], soff[kMaxBinsPerLevel + 1];
    __shared__ BinItem stage[256 * NC];
    const uint32_t level = bp.first_level + blockIdx.y;
    const uint32_t nb = bp.nbins[level];
    for (uint32_t t = threadIdx.x; t < nb; t += 256) cnt[t] = 0;
    __syncthreads();

    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    bool valid = b < rows_of(B, im);
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = valid ? inputs[(size_t)b * D + d] : 0.5f;
        if (valid && im.scale != 0.0f) x[d] = (x[d] + im.shift) * im.scale;
        if (x[d] < 0 || x[d] > 1) valid = false;
    }
    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t hs_mask = (hs & (hs - 1)) == 0 ? hs - 1 : 0;
    const float scale = lv.scale[level];
    const uint32_t resolution = lv.res[level];
    float pos[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
        if (interp == 1) pos[d] = smoothstep(pos[d]);
    }
    float g0 = 0.0f, g1 = 0.0f;
    if (valid) {
        const ngp_half2 gv = *reinterpret_cast<const ngp_half2*>(grad + ((size_t)b * L + level) * C);
        g0 = (float)gv[0];
        g1 = (float)gv[1];
    }
    if (g0 == 0.0f && g1 == 0.0f) valid = false;  // nothing to add (e.g. samples past the early stop)

    uint32_t key[NC], rank[NC];
    ngp_half2 val[NC];
#pragma unroll
    for (uint32_t idx = 0; idx < NC; idx++) {
        float w = 1;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) {
                w *= 1 - pos[d];
                pl[d] = pg[d];
            } else {
                w *= pos[d];
                pl[d] = pg[d] + 1;
            }
        }
        key[idx] = valid ? grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pl) : 0u;
        val[idx] = ngp_half2{(ngp_half)(w * g0), (ngp_half)(w * g1)};
        rank[idx] = valid ? atomicAdd(&cnt[key[idx] >> kBinShift], 1u) : 0u;
    }
    __syncthreads();
    // reserve each bin's run; exclusive scan of the counts for the staging layout
    for (uint32_t t = threadIdx.x; t < nb; t += 256) {
        const uint32_t c = cnt[t];
        uint32_t bs = 0;
        if (c) {
            bs = atomicAdd(&cursor[bp.bin0[level] + t], c);
            if (bs + c > bp.cap) bs = 0xffffffffu;  // overflow: this block's items of bin t go atomic
        }
        base[t] = bs;
    }
    {   // block-wide exclusive scan of cnt[0..nb) (nb <= 256 = blockDim)
        __shared__ uint32_t wsum[4];
        const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
        const uint32_t v = t < nb ? cnt[t] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) {
            before += w < wv ? wsum[w] : 0u;
            all += wsum[w];
        }
        if (t < nb) soff[t] = before + incl - v;
        if (t == 0) soff[nb] = all;
    }
    __syncthreads();
    if (valid) {
        ngp_half* gg = grad_grid + (size_t)off0 * C;
#pragma unroll
        for (uint32_t idx = 0; idx < NC; idx++) {
            const uint32_t bin = key[idx] >> kBinShift;
            if (base[bin] == 0xffffffffu) {
                __builtin_amdgcn_global_atomic_fadd_v2f16(reinterpret_cast<ngp_half2*>(gg + (size_t)key[idx] * C),
                                                          val[idx]);
            } else {
                stage[soff[bin] + rank[idx]] = BinItem{(key[idx] & (kBinEntries - 1)) | (bin << 16), val[idx]};
            }
        }
    }
    __syncthreads();
    const uint32_t total = soff[nb];
    for (uint32_t k = threadIdx.x; k < total; k += 256) {
        const BinItem it = stage[k];
        const uint32_t bin = it.e >> 16;
        if (base[bin] == 0xffffffffu) continue;
        BinItem* dst = items + (size_t)(bp.bin0[level] + bin) * bp.cap + base[bin] + (k - soff[bin]);
        *dst = BinItem{it.e & 0xffffu, it.v};
    }
}

__global__ void __launch_bounds__(256)
k_grid_bin_accum(const int32_t* __restrict__ offsets, ngp_half* __restrict__ grad_grid, uint32_t L,
                 BinPlan bp, uint32_t* __restrict__ cursor, const BinItem* __restrict__ items) {
    constexpr uint32_t C = 2;
    __shared__ float acc[kBinEntries * C];
    const uint32_t g = blockIdx.x;
    uint32_t level = bp.first_level;
    while (level + 1 < L && g >= bp.bin0[level + 1]) ++level;
    const uint32_t lbin = g - bp.bin0[level];
    for (uint32_t t = threadIdx.x; t < kBinEntries * C; t += 256) acc[t] = 0.0f;
    __syncthreads();
    const uint32_t n = min(cursor[g], bp.cap);
    const BinItem* src = items + (size_t)g * bp.cap;
    for (uint32_t k = threadIdx.x; k < n; k += 256) {
        const BinItem it = src[k];
        atomicAdd(&acc[it.e * C], (float)it.v[0]);
        atomicAdd(&acc[it.e * C + 1], (float)it.v[1]);
    }
    __syncthreads();
    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t e0 = lbin * kBinEntries;
    const uint32_t ne = min(kBinEntries, hs - e0);
    ngp_half2* tbl = reinterpret_cast<ngp_half2*>(grad_grid + ((size_t)off0 + e0) * C);
    for (uint32_t e = threadIdx.x; e < ne; e += 256) {
        const float a0 = acc[e * C], a1 = acc[e * C + 1];
        if (a0 == 0.0f && a1 == 0.0f) continue;
        const ngp_half2 old = tbl[e];
        tbl[e] = ngp_half2{(ngp_half)((float)old[0] + a0), (ngp_half)((float)old[1] + a1)};
    }
    if (threadIdx.x == 0) cursor[g] = 0;  // ready for the next step
}

// Host-side plan from a host copy of the offsets: the binned levels are the
// hashed suffix whose tables hold at least 8 bins.
static BinPlan make_bin_plan(const int32_t* offsets_host, uint32_t L, uint32_t D, const GridLevels& lv,
                             bool align_corners, uint32_t B) {
    BinPlan bp{};
    bp.first_level = L;
    for (int l = (int)L - 1; l >= 0; --l) {
        const uint32_t hs = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        const double side = (double)(align_corners ? lv.res[l] : lv.res[l] + 1);
        const bool hashed = std::pow(side, (double)D) > (double)hs;
        const uint32_t nb = (hs + kBinEntries - 1) / kBinEntries;
        if (!hashed || nb < 8 || nb > kMaxBinsPerLevel) break;
        bp.first_level = (uint32_t)l;
    }
    uint32_t total = 0, maxnb = 1;
    for (uint32_t l = bp.first_level; l < L; ++l) {
        const uint32_t hs = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        bp.nbins[l] = (hs + kBinEntries - 1) / kBinEntries;
        bp.bin0[l] = total;
        total += bp.nbins[l];
        maxnb = bp.nbins[l] > maxnb ? bp.nbins[l] : maxnb;
    }
    for (uint32_t l = L; l < kMaxLevels; ++l) bp.bin0[l] = total;
    bp.total_bins = total;
    // twice the mean load of a bin (corners spread uniformly by the hash) + slack
    bp.cap = (uint32_t)(2ull * ((uint64_t)B * (1u << D) + maxnb - 1) / maxnb + 2048);
    return bp;
}

static size_t bin_workspace_bytes(const BinPlan& bp) {
    const size_t cur = ((size_t)bp.total_bins * 4 + 255) / 256 * 256;
    return cur + (size_t)bp.total_bins * bp.cap * sizeof(BinItem);
}

template <typename T, uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_input_bwd(const T* __restrict__ grad, const T* __restrict__ dy_dx,
                 T* __restrict__ grad_inputs, uint32_t B, uint32_t L, int32_t grad_layout) {
    using A = Acc<T>;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D;
    const uint32_t d = t - b * D;
    const T* dd = dy_dx + (size_t)b * L * D * C;
    typename A::S result = A::zero();
    for (uint32_t l = 0; l < L; l++) {
#pragma unroll
        for (uint32_t ch = 0; ch < C; ch++) {
            const size_t gi = grad_layout == 0 ? ((size_t)l * B + b) * C + ch
                                               : ((size_t)b * L + l) * C + ch;
            result = A::mac(result, A::load(grad + gi), A::load(dd + l * D * C + d * C + ch));
        }
    }
    grad_inputs[t] = result;
}

// TV gradient (reference gridencoder.cu:503-607). float / double only: the
// reference's half instantiation calls an empty at::Half atomicAdd stub
// (gridencoder.cu:22-26) and so never writes anything.
template <typename T, uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_tv(const T* __restrict__ inputs, const T* __restrict__ grid, T* __restrict__ grad,
          const int32_t* __restrict__ offsets, float weight, uint32_t B, uint32_t L, GridLevels lv,
          uint32_t gridtype, bool align_corners) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t level = blockIdx.y;
    T x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) return;
    }
    const uint32_t off0 = (uint32_t)offsets[level];
    const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
    const uint32_t hs_mask = (hs & (hs - 1)) == 0 ? hs - 1 : 0;
    const T* g = grid + (size_t)off0 * C;
    T* gr = grad + (size_t)off0 * C;
    const float scale = lv.scale[level];
    const uint32_t resolution = lv.res[level];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        float pos;
        if constexpr (sizeof(T) == 8) pos = (float)fma(x[d], (double)scale, align_corners ? 0.0 : 0.5);
        else pos = fmaf((float)x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos);
    }
    T results[C], idelta[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) { results[c] = 0; idelta[c] = 0; }
    const uint32_t index = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pg) * C;
    const T w = (T)(weight / (2 * D));
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        const uint32_t cur_d = pg[d];
        if (cur_d < resolution) {
            pg[d] = cur_d + 1;
            const uint32_t ir = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pg) * C;
#pragma unroll
            for (uint32_t c = 0; c < C; c++) {
                const T gv = g[index + c] - g[ir + c];
                results[c] += gv;
                idelta[c] += gv * gv;
            }
        }
        if (cur_d > 0) {
            pg[d] = cur_d - 1;
            const uint32_t il = grid_index<D>(gridtype, align_corners, hs, hs_mask, resolution, pg) * C;
#pragma unroll
            for (uint32_t c = 0; c < C; c++) {
                const T gv = g[index + c] - g[il + c];
                results[c] += gv;
                idelta[c] += gv * gv;
            }
        }
        pg[d] = cur_d;
    }
#pragma unroll
    for (uint32_t c = 0; c < C; c++)
        atomicAdd(&gr[index + c], w * results[c] * (T)rsqrtf((float)(idelta[c] + (T)1e-9f)));
}

// ---- dispatch ---------------------------------------------------------------
template <typename T, typename E, uint32_t D>
int fwd_c(const float* inputs, const void* emb, const int32_t* offsets, void* out, uint32_t B,
          uint32_t C, uint32_t L, const GridLevels& lv, void* dy_dx, uint32_t gridtype,
          bool ac, uint32_t interp, int32_t layout, const InMap& im, hipStream_t st) {
    const dim3 grid(ngp_div_up(B, 256), L);
    const E* e = (const E*)emb;
    T* o = (T*)out;
    T* dd = (T*)dy_dx;
    if (!dd && (sizeof(T) <= 4)) {
        const dim3 gp(ngp_div_up(B, 128), L);
        switch (C) {
            case 1: k_grid_fwd_pair<T, E, D, 1><<<gp, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, gridtype, ac, interp, layout, im); break;
            case 2: k_grid_fwd_pair<T, E, D, 2><<<gp, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, gridtype, ac, interp, layout, im); break;
            case 4: k_grid_fwd_pair<T, E, D, 4><<<gp, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, gridtype, ac, interp, layout, im); break;
            case 8: k_grid_fwd_pair<T, E, D, 8><<<gp, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, gridtype, ac, interp, layout, im); break;
            default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: C must be 1, 2, 4, or 8.");
        }
        return ngp_check_launch("grid_encode_forward");
    }
    switch (C) {
        case 1: k_grid_fwd<T, E, D, 1><<<grid, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, dd, gridtype, ac, interp, layout, im); break;
        case 2: k_grid_fwd<T, E, D, 2><<<grid, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, dd, gridtype, ac, interp, layout, im); break;
        case 4: k_grid_fwd<T, E, D, 4><<<grid, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, dd, gridtype, ac, interp, layout, im); break;
        case 8: k_grid_fwd<T, E, D, 8><<<grid, 256, 0, st>>>(inputs, e, offsets, o, B, L, lv, dd, gridtype, ac, interp, layout, im); break;
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: C must be 1, 2, 4, or 8.");
    }
    return ngp_check_launch("grid_encode_forward");
}

template <typename T, typename E = T>
int fwd_t(const float* inputs, const void* emb, const int32_t* offsets, void* out, uint32_t B,
          uint32_t D, uint32_t C, uint32_t L, const GridLevels& lv, void* dy_dx,
          uint32_t gridtype, bool ac, uint32_t interp, int32_t layout, hipStream_t st,
          const InMap& im = InMap{0.0f, 0.0f, nullptr}) {
    switch (D) {
        case 2: return fwd_c<T, E, 2>(inputs, emb, offsets, out, B, C, L, lv, dy_dx, gridtype, ac, interp, layout, im, st);
        case 3: return fwd_c<T, E, 3>(inputs, emb, offsets, out, B, C, L, lv, dy_dx, gridtype, ac, interp, layout, im, st);
        case 4: return fwd_c<T, E, 4>(inputs, emb, offsets, out, B, C, L, lv, dy_dx, gridtype, ac, interp, layout, im, st);
        case 5: return fwd_c<T, E, 5>(inputs, emb, offsets, out, B, C, L, lv, dy_dx, gridtype, ac, interp, layout, im, st);
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: D must be 2, 3, 4, or 5.");
    }
}

template <typename T, uint32_t D, uint32_t C>
int bwd_one(const void* grad, const float* inputs, const int32_t* offsets, void* gemb,
            uint32_t B, uint32_t L, const GridLevels& lv, const void* dy_dx, void* grad_inputs,
            uint32_t gridtype, bool ac, uint32_t interp, int32_t layout, hipStream_t st,
            const InMap& im) {
    const dim3 grid(ngp_div_up(B, 128), L);  // two lanes per point (corner pairs)
    k_grid_bwd<T, D, C><<<grid, 256, 0, st>>>((const T*)grad, inputs, offsets, (T*)gemb, B, L, lv,
                                               gridtype, ac, interp, layout, im, 0u);
    if (dy_dx && grad_inputs) {
        k_grid_input_bwd<T, D, C><<<ngp_div_up(B * D, 256), 256, 0, st>>>(
            (const T*)grad, (const T*)dy_dx, (T*)grad_inputs, B, L, layout);
    }
    return ngp_check_launch("grid_encode_backward");
}

template <typename T, uint32_t D>
int bwd_c(const void* grad, const float* inputs, const int32_t* offsets, void* gemb, uint32_t B,
          uint32_t C, uint32_t L, const GridLevels& lv, const void* dy_dx, void* gi,
          uint32_t gridtype, bool ac, uint32_t interp, int32_t layout, hipStream_t st,
          const InMap& im) {
    switch (C) {
        case 1: return bwd_one<T, D, 1>(grad, inputs, offsets, gemb, B, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 2: return bwd_one<T, D, 2>(grad, inputs, offsets, gemb, B, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 4: return bwd_one<T, D, 4>(grad, inputs, offsets, gemb, B, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 8: return bwd_one<T, D, 8>(grad, inputs, offsets, gemb, B, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: C must be 1, 2, 4, or 8.");
    }
}

template <typename T>
int bwd_t(const void* grad, const float* inputs, const int32_t* offsets, void* gemb, uint32_t B,
          uint32_t D, uint32_t C, uint32_t L, const GridLevels& lv, const void* dy_dx, void* gi,
          uint32_t gridtype, bool ac, uint32_t interp, int32_t layout, hipStream_t st,
          const InMap& im = InMap{0.0f, 0.0f, nullptr}) {
    switch (D) {
        case 2: return bwd_c<T, 2>(grad, inputs, offsets, gemb, B, C, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 3: return bwd_c<T, 3>(grad, inputs, offsets, gemb, B, C, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 4: return bwd_c<T, 4>(grad, inputs, offsets, gemb, B, C, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        case 5: return bwd_c<T, 5>(grad, inputs, offsets, gemb, B, C, L, lv, dy_dx, gi, gridtype, ac, interp, layout, st, im);
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: D must be 2, 3, 4, or 5.");
    }
}

template <typename T, uint32_t D>
int tv_c(const void* inputs, const void* emb, void* grad, const int32_t* offsets, float weight,
         uint32_t B, uint32_t C, uint32_t L, const GridLevels& lv, uint32_t gridtype, bool ac,
         hipStream_t st) {
    const dim3 grid(ngp_div_up(B, 256), L);
    const T* in = (const T*)inputs;
    const T* e = (const T*)emb;
    T* g = (T*)grad;
    switch (C) {
        case 1: k_grid_tv<T, D, 1><<<grid, 256, 0, st>>>(in, e, g, offsets, weight, B, L, lv, gridtype, ac); break;
        case 2: k_grid_tv<T, D, 2><<<grid, 256, 0, st>>>(in, e, g, offsets, weight, B, L, lv, gridtype, ac); break;
        case 4: k_grid_tv<T, D, 4><<<grid, 256, 0, st>>>(in, e, g, offsets, weight, B, L, lv, gridtype, ac); break;
        case 8: k_grid_tv<T, D, 8><<<grid, 256, 0, st>>>(in, e, g, offsets, weight, B, L, lv, gridtype, ac); break;
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: C must be 1, 2, 4, or 8.");
    }
    return ngp_check_launch("grad_total_variation");
}

template <typename T>
int tv_t(const void* inputs, const void* emb, void* grad, const int32_t* offsets, float weight,
         uint32_t B, uint32_t D, uint32_t C, uint32_t L, const GridLevels& lv, uint32_t gridtype,
         bool ac, hipStream_t st) {
    switch (D) {
        case 2: return tv_c<T, 2>(inputs, emb, grad, offsets, weight, B, C, L, lv, gridtype, ac, st);
        case 3: return tv_c<T, 3>(inputs, emb, grad, offsets, weight, B, C, L, lv, gridtype, ac, st);
        case 4: return tv_c<T, 4>(inputs, emb, grad, offsets, weight, B, C, L, lv, gridtype, ac, st);
        case 5: return tv_c<T, 5>(inputs, emb, grad, offsets, weight, B, C, L, lv, gridtype, ac, st);
        default: return ngp_set_error(NGP_ERR_UNSUPPORTED, "GridEncoding: D must be 2, 3, 4, or 5.");
    }
}

int check_common(uint32_t L, const void* a, const void* b, const void* c) {
    NGP_REQUIRE(L >= 1 && L <= kMaxLevels, NGP_ERR_ARG, "GridEncoding: L must be in [1, %u], got %u", kMaxLevels, L);
    NGP_REQUIRE(a && b && c, NGP_ERR_ARG, "GridEncoding: null tensor pointer");
    return NGP_OK;
}

}  // namespace

extern "C" int ngp_grid_encode_forward(const float* inputs, const void* embeddings,
                                       const int32_t* offsets, void* outputs, uint32_t B,
                                       uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                       void* dy_dx, uint32_t gridtype, int32_t align_corners,
                                       uint32_t interp, int32_t dtype, int32_t out_layout,
                                       void* stream) {
    if (int e = check_common(L, embeddings, offsets, outputs)) return e;
    if (B == 0) return NGP_OK;
    NGP_REQUIRE(inputs, NGP_ERR_ARG, "GridEncoding: null inputs");
    GridLevels lv;
    make_levels(lv, L, S, H);
    const bool ac = align_corners != 0;
    hipStream_t st = ngp_stream(stream);
    switch (dtype) {
        case NGP_DTYPE_F32: return fwd_t<float>(inputs, embeddings, offsets, outputs, B, D, C, L, lv, dy_dx, gridtype, ac, interp, out_layout, st);
        case NGP_DTYPE_F16: return fwd_t<ngp_half>(inputs, embeddings, offsets, outputs, B, D, C, L, lv, dy_dx, gridtype, ac, interp, out_layout, st);
        case NGP_DTYPE_F64: return fwd_t<double>(inputs, embeddings, offsets, outputs, B, D, C, L, lv, dy_dx, gridtype, ac, interp, out_layout, st);
        default: return ngp_set_error(NGP_ERR_ARG, "embeddings must be a floating tensor");
    }
}

extern "C" int ngp_grid_encode_backward(const void* grad, const float* inputs,
                                        const void* embeddings, const int32_t* offsets,
                                        void* grad_embeddings, uint32_t B, uint32_t D, uint32_t C,
                                        uint32_t L, float S, uint32_t H, const void* dy_dx,
                                        void* grad_inputs, uint32_t gridtype,
                                        int32_t align_corners, uint32_t interp, int32_t dtype,
                                        int32_t grad_layout, void* stream) {
    (void)embeddings;
    if (int e = check_common(L, grad, offsets, grad_embeddings)) return e;
    if (B == 0) return NGP_OK;
    NGP_REQUIRE(inputs, NGP_ERR_ARG, "GridEncoding: null inputs");
    GridLevels lv;
    make_levels(lv, L, S, H);
    const bool ac = align_corners != 0;
    hipStream_t st = ngp_stream(stream);
    switch (dtype) {
        case NGP_DTYPE_F32: return bwd_t<float>(grad, inputs, offsets, grad_embeddings, B, D, C, L, lv, dy_dx, grad_inputs, gridtype, ac, interp, grad_layout, st);
        case NGP_DTYPE_F16: return bwd_t<ngp_half>(grad, inputs, offsets, grad_embeddings, B, D, C, L, lv, dy_dx, grad_inputs, gridtype, ac, interp, grad_layout, st);
        case NGP_DTYPE_F64: return bwd_t<double>(grad, inputs, offsets, grad_embeddings, B, D, C, L, lv, dy_dx, grad_inputs, gridtype, ac, interp, grad_layout, st);
        default: return ngp_set_error(NGP_ERR_ARG, "grad must be a floating tensor");
    }
}

extern "C" int ngp_grad_total_variation(const void* inputs, const void* embeddings, void* grad,
                                        const int32_t* offsets, float weight, uint32_t B,
                                        uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                        uint32_t gridtype, int32_t align_corners, int32_t dtype,
                                        void* stream) {
    if (int e = check_common(L, embeddings, offsets, grad)) return e;
    if (B == 0) return NGP_OK;
    GridLevels lv;
    make_levels(lv, L, S, H);
    const bool ac = align_corners != 0;
    hipStream_t st = ngp_stream(stream);
    switch (dtype) {
        case NGP_DTYPE_F32: return tv_t<float>(inputs, embeddings, grad, offsets, weight, B, D, C, L, lv, gridtype, ac, st);
        case NGP_DTYPE_F64: return tv_t<double>(inputs, embeddings, grad, offsets, weight, B, D, C, L, lv, gridtype, ac, st);
        case NGP_DTYPE_F16:
            return ngp_set_error(NGP_ERR_UNSUPPORTED, "grad_total_variation: half embeddings are not supported (call it outside autocast, as GridEncoder.grad_total_variation does)");
        default: return ngp_set_error(NGP_ERR_ARG, "embeddings must be a floating tensor");
    }
}

/* Fused train-step entry points (DESIGN.md "fused step"): world-space inputs
 * normalised in-kernel exactly as GridEncoder.forward does, an fp32 table
 * read as half (the reference's embeddings.half()), fp16 [B, L*C] outputs /
 * output grads, fp16 grad table, rows clipped at *count. */
extern "C" int ngp_grid_encode_forward_fused(const float* xyz, float bound, const float* embeddings,
                                             const int32_t* offsets, void* outputs, uint32_t B,
                                             const int32_t* count, uint32_t D, uint32_t C, uint32_t L,
                                             float S, uint32_t H, uint32_t gridtype,
                                             int32_t align_corners, uint32_t interp, void* stream) {
    if (int e = check_common(L, embeddings, offsets, outputs)) return e;
    NGP_REQUIRE(xyz && bound > 0.0f, NGP_ERR_ARG, "grid_encode_forward_fused: null xyz or bound <= 0");
    if (B == 0) return NGP_OK;
    GridLevels lv;
    make_levels(lv, L, S, H);
    const InMap im{bound, 1.0f / (2.0f * bound), count};
    return fwd_t<ngp_half, float>(xyz, embeddings, offsets, outputs, B, D, C, L, lv, nullptr, gridtype,
                                  align_corners != 0, interp, 1, ngp_stream(stream), im);
}

extern "C" size_t ngp_grid_encode_backward_fused_workspace_bytes(uint32_t B, uint32_t D, uint32_t C,
                                                                uint32_t L, float S, uint32_t H,
                                                                int32_t align_corners,
                                                                const int32_t* offsets_host) {
    if (!offsets_host || C != 2 || D < 2 || D > 5 || L == 0 || L > kMaxLevels) return 0;
    GridLevels lv;
    make_levels(lv, L, S, H);
    const BinPlan bp = make_bin_plan(offsets_host, L, D, lv, align_corners != 0, B);
    return bp.total_bins ? bin_workspace_bytes(bp) : 0;
}

extern "C" int ngp_grid_encode_backward_fused(const void* grad, const float* xyz, float bound,
                                              const int32_t* offsets, void* grad_embeddings,
                                              uint32_t B, const int32_t* count, uint32_t D,
                                              uint32_t C, uint32_t L, float S, uint32_t H,
                                              uint32_t gridtype, int32_t align_corners,
                                              uint32_t interp, const int32_t* offsets_host,
                                              void* workspace, size_t workspace_bytes,
                                              void* stream) {
    if (int e = check_common(L, grad, offsets, grad_embeddings)) return e;
    NGP_REQUIRE(xyz && bound > 0.0f, NGP_ERR_ARG, "grid_encode_backward_fused: null xyz or bound <= 0");
    if (B == 0) return NGP_OK;
    GridLevels lv;
    make_levels(lv, L, S, H);
    const InMap im{bound, 1.0f / (2.0f * bound), count};
    hipStream_t st = ngp_stream(stream);
    const bool ac = align_corners != 0;
    BinPlan bp{};
    bp.first_level = L;
    if (workspace && offsets_host && C == 2 && D == 3) {
        bp = make_bin_plan(offsets_host, L, D, lv, ac, B);
        if (bp.total_bins) {
            NGP_REQUIRE(workspace_bytes >= bin_workspace_bytes(bp), NGP_ERR_ARG,
                        "grid_encode_backward_fused: workspace of %zu bytes required, got %zu",
                        bin_workspace_bytes(bp), workspace_bytes);
        } else {
            bp.first_level = L;
        }
    }
    // dense (and any unbinned) levels: merged atomics
    if (bp.first_level > 0) {
        const dim3 grid(ngp_div_up(B, 128), bp.first_level);
        switch (D) {
            case 3:
                if (C == 2) {
                    k_grid_bwd<ngp_half, 3, 2><<<grid, 256, 0, st>>>((const ngp_half*)grad, xyz, offsets,
                        (ngp_half*)grad_embeddings, B, L, lv, gridtype, ac, interp, 1, im, 0u);
                    break;
                }
                [[fallthrough]];
            default:
                return bwd_t<ngp_half>(grad, xyz, offsets, grad_embeddings, B, D, C, L, lv, nullptr, nullptr,
                                       gridtype, ac, interp, 1, st, im);
        }
    }
    if (bp.first_level < L) {
        uint32_t* cursor = static_cast<uint32_t*>(workspace);
        BinItem* items = reinterpret_cast<BinItem*>(static_cast<char*>(workspace) +
                                                    ((size_t)bp.total_bins * 4 + 255) / 256 * 256);
        const dim3 grid(ngp_div_up(B, 256), L - bp.first_level);
        k_grid_bwd_bin<3><<<grid, 256, 0, st>>>((const ngp_half*)grad, xyz, offsets, (ngp_half*)grad_embeddings,
                                                B, L, lv, gridtype, ac, interp, im, bp, cursor, items);
        k_grid_bin_accum<<<bp.total_bins, 256, 0, st>>>(offsets, (ngp_half*)grad_embeddings, L, bp, cursor, items);
    }
    return ngp_check_launch("grid_encode_backward_fused");
}
