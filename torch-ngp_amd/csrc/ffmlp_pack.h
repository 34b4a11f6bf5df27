// Weight-fragment images of the fused MLP (ffmlp.hip), shared with the fused
// train step's head kernel (nerf_fused.hip), which packs both NeRF networks'
// images in the same launch as the ray sampler and the deferred GradScaler
// update. Device helpers are inline; build_jobs is defined in ffmlp.hip.
#pragma once
#include "ngp_common.h"

namespace ngp_pack {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

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

// One lane's 8-element slot of fragment f of matrix m.
NGP_DEV half8 frag_slot(const ngp_half* __restrict__ w, const MatDesc& m, bool transposed,
                        uint32_t f, uint32_t lane) {
    const uint32_t mt = f / m.ks, s = f - mt * m.ks;
    const int g = lane >> 4, c = lane & 15;
    const uint32_t row = 16 * mt + c;  // M index
    half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!transposed) {
        // A[row=o][k=i] = W[o][i]: contiguous runs of the weight row -> vector loads
        if (row >= m.out) return v;
        const ngp_half* wr = w + m.off + row * m.in;
        if (!m.kperm) {
            const uint32_t i0 = 32 * s + 8 * g;  // 8 contiguous, all in or all out (in % 16 == 0)
            if (i0 < m.in) v = *reinterpret_cast<const half8*>(wr + i0);
        } else {
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            const uint32_t i0 = 32 * s + 4 * g, i1 = 32 * s + 16 + 4 * g;
            h4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
            if (i0 < m.in) a = *reinterpret_cast<const h4*>(wr + i0);
            if (i1 < m.in) b = *reinterpret_cast<const h4*>(wr + i1);
            v = half8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        }
        return v;
    }
    // A[row=i][k=o] = W[o][i]: a column of W (strided gathers)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t o = 32 * s + (m.kperm ? perm_unit(g, j) : 8 * g + j);
        v[j] = (o < m.out && row < m.in) ? w[m.off + o * m.in + row] : (ngp_half)0.0f;
    }
    return v;
}

NGP_DEV void build_frags(half8* lds, const ngp_half* __restrict__ w, const MatDesc& m, bool transposed) {
    const uint32_t n = m.mt * m.ks * 64;  // lanes to fill
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x)
        lds[m.frag0 * 64 + t] = frag_slot(w, m, transposed, t >> 6, t & 63);
}

// Fragment images of several networks in one launch: one block per (network,
// matmul, direction) job, descriptors computed on the host.
constexpr int kMaxPackJobs = 32;
struct PackJob {
    const ngp_half* w;
    half8* image;
    MatDesc m;
    uint32_t transposed;
};
struct PackJobs {
    int n;
    PackJob job[kMaxPackJobs];
};

// Host: append the pack jobs of n networks (forward + transposed fragment
// sets of every matmul) to `jobs`; returns an NGP_* code.
int build_jobs(int32_t n, const void* const* weights, const uint32_t* in_dims, const uint32_t* hidden_dims,
               const uint32_t* num_layers, void* const* images, PackJobs& jobs);

}  // namespace ngp_pack
