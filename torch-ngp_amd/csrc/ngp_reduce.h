// The deterministic dW slab reduce of the fused MLP backward (ffmlp.hip
// deferred dW partials, one slab row per backward workgroup), shared by its
// own launch (k_slab_reduce) and the grid backward's bin launch, which can
// carry it as extra blocks (gridencoder.hip): both sum in the same fixed order,
// so the weight gradients are bit-identical either way.
#pragma once
#include "ngp_common.h"


namespace ngp_reduce {

constexpr int kReducePhases = 16;  // row phases of one 64-parameter block
constexpr int kMaxReduceJobs = 4;
constexpr uint32_t kBwdChunkRows = 32;  // rows of one backward chunk (ffmlp.hip: 16 * kNB)
// The slab rows a live-row backward (ngp_nerf_backward_live) writes: its
// workgroup b takes chunks b, b + G, ..., so with nch chunks only rows < nch
// hold partials; rows up to the next multiple of 4 phases are written too
// (zeros), so the reduce's sums keep their association and its result is the
// all-rows sum bit for bit (the rows skipped would add +0.0).
NGP_DEV uint32_t live_slab_rows(int32_t live_count, uint32_t rows) {
    const uint32_t nch = live_count <= 0 ? 0u : ((uint32_t)live_count + kBwdChunkRows - 1) / kBwdChunkRows;
    const uint32_t g = 4u * kReducePhases;
    return min(rows, (nch + g - 1) / g * g);
}
struct ReduceJobs {
    int n;
    const float* slab[kMaxReduceJobs];
    void* out[kMaxReduceJobs];
    uint32_t rows[kMaxReduceJobs], np[kMaxReduceJobs];
    uint32_t block0[kMaxReduceJobs + 1];
    int32_t* nonfinite;  // nullable: set when a written grad is inf/nan (GradScaler's check)
    const int32_t* live;  // nullable: the live-row count of a live-row backward (live_slab_rows)
};

// grad_weights[p] = sum over the slab rows, in a fixed order: row phase ph
// (rows ph, ph + 16, ...) keeps 4 independent partial sums (its loads stay in
// flight), then the 16 phase sums are added in phase order. Block `blk` owns
// 64 parameters; a block of THREADS (64 x 16 or 64 x 8) threads runs 16 /
// (THREADS / 64) phases per thread. part: 16 x 64 floats of LDS.
template <typename OUT, int THREADS>
NGP_DEV void slab_reduce_block(const ReduceJobs& jobs, uint32_t blk, float (*part)[64]) {
    constexpr int WAVES = THREADS / 64, PPT = kReducePhases / WAVES;
    static_assert(kReducePhases % WAVES == 0, "whole phases per thread");
    int j = 0;
    while (j + 1 < jobs.n && blk >= jobs.block0[j + 1]) ++j;
    const float* __restrict__ slab = jobs.slab[j];
    const uint32_t rows = jobs.live ? live_slab_rows(*jobs.live, jobs.rows[j]) : jobs.rows[j], n = jobs.np[j];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t p = (blk - jobs.block0[j]) * 64 + lane;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
        const uint32_t ph = wv + (uint32_t)q * WAVES;
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
        if (p < n) {
            uint32_t r = ph;
            for (; r + 3 * kReducePhases < rows; r += 4 * kReducePhases) {
                s0 += *(slab + (size_t)r * n + p);
                s1 += *(slab + (size_t)(r + kReducePhases) * n + p);
                s2 += *(slab + (size_t)(r + 2 * kReducePhases) * n + p);
                s3 += *(slab + (size_t)(r + 3 * kReducePhases) * n + p);
            }
            for (; r < rows; r += kReducePhases) s0 += *(slab + (size_t)r * n + p);
        }
        part[ph][lane] = (s0 + s1) + (s2 + s3);
    }
    __syncthreads();
    if (wv == 0 && p < n) {
        float t = 0.0f;
#pragma unroll
        for (int k = 0; k < kReducePhases; ++k) t += part[k][lane];
        const OUT o = (OUT)t;
        static_cast<OUT*>(jobs.out[j])[p] = o;
        if (jobs.nonfinite && !__builtin_isfinite((float)o)) atomicOr(jobs.nonfinite, 1);
    }
}

// ReduceJobs of n deferred backward calls (ffmlp.hip; the arguments of
// ngp_ffmlp_reduce). Returns the number of 64-parameter blocks (0: nothing).
uint32_t build_reduce_jobs(int32_t n, void* const* workspaces, const uint32_t* Bs, const uint32_t* in_dims,
                           const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* grad_weights,
                           int32_t* nonfinite, ReduceJobs& rj);
// The reduce of built jobs as its own launch (fp16 grads); NGP_OK or an error code.
int launch_slab_reduce(const ReduceJobs& rj, uint32_t blocks, void* stream);

}  // namespace ngp_reduce
