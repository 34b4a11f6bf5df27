/*
 * ngp_hip.h — C ABI of the MI355X (gfx950) instant-ngp hot path.
 *
 * One shared library (libngp_hip.so) exports every entry point below. The
 * signatures take plain device pointers, sizes and a hipStream_t (passed as
 * void*), never torch types, so any host language can bind them (ctypes,
 * cgo, JNI, N-API). Each entry replaces one pybind11 function of the reference
 * extension; the reference declaration it stands in for is cited per function
 * (paths relative to the reference repository root).
 *
 * Conventions shared by every function:
 *   - The caller allocates every output and scratch buffer; nothing here calls
 *     hipMalloc/hipFree or synchronises, so each call can be captured into a
 *     hipGraph. Work is enqueued on `stream` (NULL = the legacy null stream).
 *   - Return value: NGP_OK (0) on success, a negative NGP_ERR_* code otherwise.
 *     NGP_ERR_ARG / NGP_ERR_UNSUPPORTED mirror the reference's TORCH_CHECK /
 *     std::runtime_error("... must be ...") failures; the Python shims raise
 *     RuntimeError with the reference's wording.
 *   - dtype codes: NGP_DTYPE_F32 = 0, NGP_DTYPE_F16 = 1, NGP_DTYPE_F64 = 2.
 */
#ifndef NGP_HIP_H
#define NGP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGP_OK 0
#define NGP_ERR_ARG (-1)
#define NGP_ERR_HIP (-2)
#define NGP_ERR_UNSUPPORTED (-3)

#define NGP_DTYPE_F32 0
#define NGP_DTYPE_F16 1
#define NGP_DTYPE_F64 2

/* Library identification: ABI version (bumped on any signature change). */
int ngp_abi_version(void);
/* Human-readable message for the last NGP_ERR_* returned on this thread. */
const char* ngp_last_error(void);

/* ------------------------------------------------------------------------ */
/* gridencoder                                                              */
/* ------------------------------------------------------------------------ */

/* Replaces grid_encode_forward, gridencoder/src/gridencoder.h:12 and
 * gridencoder/src/gridencoder.cu:445-468.
 *   inputs  f32 [B, D] in [0,1]; embeddings dtype [sum_T, C];
 *   offsets i32 [L+1] (device); dy_dx dtype [B, L*D*C] or NULL.
 *   out_layout 0: outputs [L, B, C] (the reference layout);
 *   out_layout 1: outputs [B, L*C] (the layout the MLP consumes, no permute).
 *   D in {2,3,4,5}, C in {1,2,4,8}, L <= 64. */
int ngp_grid_encode_forward(const float* inputs, const void* embeddings, const int32_t* offsets,
                            void* outputs, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                            float S, uint32_t H, void* dy_dx, uint32_t gridtype,
                            int32_t align_corners, uint32_t interp, int32_t dtype,
                            int32_t out_layout, void* stream);

/* Replaces grid_encode_backward, gridencoder/src/gridencoder.h:13 and
 * gridencoder/src/gridencoder.cu:470-500. grad_embeddings must be zeroed by
 * the caller (scatter-add target). grad_layout as out_layout above. */
int ngp_grid_encode_backward(const void* grad, const float* inputs, const void* embeddings,
                             const int32_t* offsets, void* grad_embeddings, uint32_t B, uint32_t D,
                             uint32_t C, uint32_t L, float S, uint32_t H, const void* dy_dx,
                             void* grad_inputs, uint32_t gridtype, int32_t align_corners,
                             uint32_t interp, int32_t dtype, int32_t grad_layout, void* stream);

/* Replaces grad_total_variation, gridencoder/src/gridencoder.h:15 and
 * gridencoder/src/gridencoder.cu:636-642 (inputs are dtype, like the reference). */
int ngp_grad_total_variation(const void* inputs, const void* embeddings, void* grad,
                             const int32_t* offsets, float weight, uint32_t B, uint32_t D,
                             uint32_t C, uint32_t L, float S, uint32_t H, uint32_t gridtype,
                             int32_t align_corners, int32_t dtype, void* stream);

/* ------------------------------------------------------------------------ */
/* raymarching (all float32, like the reference wrappers' cast_inputs)      */
/* ------------------------------------------------------------------------ */

/* raymarching/src/raymarching.h:7, raymarching.cu:148-156 */
int ngp_near_far_from_aabb(const float* rays_o, const float* rays_d, const float* aabb, uint32_t N,
                           float min_near, float* nears, float* fars, void* stream);
/* raymarching.h:8, raymarching.cu:201-209 */
int ngp_sph_from_ray(const float* rays_o, const float* rays_d, float radius, uint32_t N,
                     float* coords, void* stream);
/* raymarching.h:9, raymarching.cu:229-232 */
int ngp_morton3D(const int32_t* coords, uint32_t N, int32_t* indices, void* stream);
/* raymarching.h:10, raymarching.cu:257-260 */
int ngp_morton3D_invert(const int32_t* indices, uint32_t N, int32_t* coords, void* stream);
/* raymarching.h:11, raymarching.cu:292-300 */
int ngp_packbits(const float* grid, uint32_t N, float density_thresh, uint8_t* bitfield,
                 void* stream);

/* Replaces march_rays_train, raymarching.h:13 and raymarching.cu:311-492.
 * Offsets are a deterministic exclusive prefix sum in ray order (a valid
 * execution of the reference's atomicAdd ordering): rays[i] = (i, off_i, n_i).
 * counter[0] += total samples, counter[1] += N (same as the reference).
 * Samples of rays with off_i + n_i > M are dropped (reference :416); the
 * caller zero-fills xyzs/dirs/deltas like the reference wrapper does.
 * workspace: 16-byte aligned device scratch of at least
 * ngp_march_rays_train_workspace_bytes (one float per possible sample,
 * N * max_steps, plus an occupancy image of ~C * H^3 / 6 bytes), e.g. from
 * the caller's caching allocator. */
size_t ngp_march_rays_train_workspace_bytes(uint32_t N, uint32_t max_steps, uint32_t C, uint32_t H);
/* Byte offset, inside that workspace, of a u32 error word the fused march +
 * Adam launch's in-launch emit sets when one of its bounded cross-workgroup
 * waits ran out (bit 0: a lower block's sample total, bit 1: the block's own
 * offsets); the offsets it wrote are then wrong. Sticky; the caller reads and
 * clears it (FusedTrainer.device_errors). No reference counterpart: the
 * reference's march (raymarching.cu:405-406) takes its offsets with atomics. */
size_t ngp_march_rays_train_error_offset(uint32_t N, uint32_t max_steps, uint32_t C, uint32_t H);
int ngp_march_rays_train(const float* rays_o, const float* rays_d, const uint8_t* grid,
                         float bound, float dt_gamma, uint32_t max_steps, uint32_t N, uint32_t C,
                         uint32_t H, uint32_t M, const float* nears, const float* fars,
                         float* xyzs, float* dirs, float* deltas, int32_t* rays, int32_t* counter,
                         const float* noises, void* workspace, size_t workspace_bytes,
                         void* stream);

/* The occupancy image march_rays_train builds from `grid` on every call can be
 * built once per bitfield change instead: ngp_march_occupancy_build into the
 * workspace, then ngp_march_rays_train_prebuilt (same arguments) as long as
 * grid's contents are unchanged. */
int ngp_march_occupancy_build(const uint8_t* grid, uint32_t C, uint32_t H, uint32_t N,
                              uint32_t max_steps, void* workspace, size_t workspace_bytes,
                              void* stream);
int ngp_march_rays_train_prebuilt(const float* rays_o, const float* rays_d, const uint8_t* grid,
                                  float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                                  uint32_t C, uint32_t H, uint32_t M, const float* nears,
                                  const float* fars, float* xyzs, float* dirs, float* deltas,
                                  int32_t* rays, int32_t* counter, const float* noises,
                                  void* workspace, size_t workspace_bytes, void* stream);
/* ngp_march_rays_train_prebuilt plus the tail of a fused step whose optimizer
 * update was launched by ngp_fused_optimizer_update_head: the deferred
 * GradScaler / LR / loss bookkeeping (scaler arguments as
 * ngp_fused_optimizer_step; loss_ray: the previous batch's N per-ray losses)
 * and ngp_ffmlp_pack of n_nets networks, as an extra row of blocks of the
 * emit launch. */
int ngp_march_rays_train_prebuilt_tail(const float* rays_o, const float* rays_d, const uint8_t* grid,
                                       float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                                       uint32_t C, uint32_t H, uint32_t M, const float* nears,
                                       const float* fars, float* xyzs, float* dirs, float* deltas,
                                       int32_t* rays, int32_t* counter, const float* noises,
                                       void* workspace, size_t workspace_bytes, void* state,
                                       float growth_factor, float backoff_factor, int32_t growth_interval,
                                       int32_t scaler_enabled, const float* loss_ray, int32_t n_nets,
                                       const void* const* mlp_weights, const uint32_t* in_dims,
                                       const uint32_t* hidden_dims, const uint32_t* num_layers,
                                       void* const* images, void* stream);

/* ngp_march_rays_train_prebuilt_tail whose march launch also carries a
 * deferred optimizer update (world 1, fused step): the march's workgroups
 * split into march waves and Adam waves that sweep the parameters while the
 * march waves probe the occupancy image (a latency-bound LDS chain beside an
 * HBM stream). job: ngp_fused_optimizer_update's arguments; its scaler check
 * must already be done (NGP_SCALER_PRECHECKED: the backward's kernels set the
 * found-inf flag). The batch must come from ngp_fused_step_head (n_nets 0);
 * the deferred bookkeeping and the MLP packs stay in the emit launch. */
#define NGP_ADAM_JOB_MAX_TENSORS 8
typedef struct ngp_adam_job {
    int32_t n_tensors;
    float* params[NGP_ADAM_JOB_MAX_TENSORS];
    void* grads[NGP_ADAM_JOB_MAX_TENSORS];       /* fp16 */
    float* exp_avg[NGP_ADAM_JOB_MAX_TENSORS];
    float* exp_avg_sq[NGP_ADAM_JOB_MAX_TENSORS];
    void* half_params[NGP_ADAM_JOB_MAX_TENSORS]; /* fp16 shadows or NULL */
    uint64_t sizes[NGP_ADAM_JOB_MAX_TENSORS];
    float lr, beta1, beta2, eps;
    int32_t iters, zero_grads;
    float grad_mult;
    void* clear;            /* zeroed by the launch too (the grid backward's bin cursors), or NULL */
    uint32_t clear_bytes;   /* multiple of 16, clear 16-byte aligned */
    uint32_t flags;         /* NGP_ADAM_JOB_TAIL_LATER | NGP_ADAM_JOB_EMIT_LAUNCH (below) or 0 */
} ngp_adam_job;
/* ... and the emit launch's whole tail row (bookkeeping + MLP fragment packs) is
 * left to ngp_grid_encode_forward_fused_tail: with the samples emitted by the
 * march launch itself, the march is then ONE launch */
#define NGP_ADAM_JOB_TAIL_LATER 2u
/* ... and the samples are emitted by the march's own emit launch instead of
 * inside the march + Adam launch (the in-launch emit's equivalence tests) */
#define NGP_ADAM_JOB_EMIT_LAUNCH 4u
int ngp_march_rays_train_prebuilt_adam(const float* rays_o, const float* rays_d, const uint8_t* grid,
                                       float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                                       uint32_t C, uint32_t H, uint32_t M, const float* nears,
                                       const float* fars, float* xyzs, float* dirs, float* deltas,
                                       int32_t* rays, int32_t* counter, const float* noises,
                                       void* workspace, size_t workspace_bytes, void* state,
                                       float growth_factor, float backoff_factor, int32_t growth_interval,
                                       int32_t scaler_enabled, const float* loss_ray, int32_t n_nets,
                                       const void* const* mlp_weights, const uint32_t* in_dims,
                                       const uint32_t* hidden_dims, const uint32_t* num_layers,
                                       void* const* images, const ngp_adam_job* job, void* stream);

/* raymarching.h:14, raymarching.cu:580-588 */
int ngp_composite_rays_train_forward(const float* sigmas, const float* rgbs, const float* deltas,
                                     const int32_t* rays, uint32_t M, uint32_t N, float T_thresh,
                                     float* weights_sum, float* depth, float* image, void* stream);
/* raymarching.h:15, raymarching.cu:694-702. grad_sigmas / grad_rgbs are
 * zeroed by the caller (entries past a ray's early stop are not written). */
int ngp_composite_rays_train_backward(const float* grad_weights_sum, const float* grad_depth,
                                      const float* grad_image, const float* sigmas,
                                      const float* rgbs, const float* deltas, const int32_t* rays,
                                      const float* weights_sum, const float* depth,
                                      const float* image, uint32_t M, uint32_t N, float T_thresh,
                                      float* grad_sigmas, float* grad_rgbs, void* stream);
/* raymarching.h:17, raymarching.cu:817-825 */
int ngp_march_rays(uint32_t n_alive, uint32_t n_step, const int32_t* rays_alive,
                   const float* rays_t, const float* rays_o, const float* rays_d, float bound,
                   float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H, const uint8_t* grid,
                   const float* nears, const float* fars, float* xyzs, float* dirs, float* deltas,
                   const float* noises, void* stream);
/* raymarching.h:18, raymarching.cu:917-923 (in place; rays_alive[n] = -1 on termination) */
int ngp_composite_rays(uint32_t n_alive, uint32_t n_step, float T_thresh, int32_t* rays_alive,
                       float* rays_t, const float* sigmas, const float* rgbs, const float* deltas,
                       float* weights_sum, float* depth, float* image, void* stream);

/* Device-driven inference render loop (the alive-ray loop of run_cuda with
 * training off, renderer.py:376-426, without its host round trip per
 * iteration). The loop state is a two-slot device record (state_bytes);
 * iteration i reads slot i & 1 and prepares slot (i + 1) & 1:
 *   render_init: alive list 0 = arange(N), rays_t = nears, outputs zeroed;
 *   render_march: kernel_march_rays (raymarching.cu:709-814) for the
 *     iteration's n_alive and n_step = max(min(N / n_alive, 8), 1), unused
 *     sample slots zeroed, noise in the first iteration only; writes the
 *     iteration's sample count (render_count) for the grid / MLP kernels;
 *   render_composite: kernel_composite_rays (raymarching.cu:827-914) on
 *     sigmas [n_alive * n_step] and the colour network's fp16 logits
 *     color_out [*, 16] (rgb = half(sigmoid)), appending surviving rays to
 *     rays_alive_next (order within the list is unspecified; per-ray results
 *     do not depend on it).
 * Once step >= max_steps or no ray is alive, every launch is a no-op. */
size_t ngp_render_state_bytes(void);
int32_t* ngp_render_count(void* state, uint32_t iter);
int ngp_render_init(uint32_t N, const float* nears, int32_t* rays_alive, float* rays_t, float* weights_sum,
                    float* depth, float* image, void* state, void* stream);
int ngp_render_march(uint32_t N, uint32_t iter, void* state, const int32_t* rays_alive, const float* rays_t,
                     const float* rays_o, const float* rays_d, float bound, float dt_gamma, uint32_t max_steps,
                     uint32_t C, uint32_t H, const uint8_t* grid, const float* fars, float* xyzs, float* dirs,
                     float* deltas, const float* noises, void* stream);
int ngp_render_composite(uint32_t N, uint32_t iter, uint32_t max_steps, void* state, float T_thresh,
                         const int32_t* rays_alive, int32_t* rays_alive_next, float* rays_t, const float* sigmas,
                         const void* color_out, const float* deltas, float* weights_sum, float* depth,
                         float* image, void* stream);

/* ------------------------------------------------------------------------ */
/* shencoder                                                                */
/* ------------------------------------------------------------------------ */

/* shencoder/src/shencoder.h:9, shencoder.cu:420-439. dtype F32 or F64.
 * C is the degree (1..8), outputs [B, C*C]; dy_dx [B, D*C*C] or NULL. */
int ngp_sh_encode_forward(const void* inputs, void* outputs, uint32_t B, uint32_t D, uint32_t C,
                          void* dy_dx, int32_t dtype, void* stream);
/* shencoder.h:10, shencoder.cu:441-454. grad_inputs zeroed by the caller. */
int ngp_sh_encode_backward(const void* grad, const void* inputs, uint32_t B, uint32_t D,
                           uint32_t C, const void* dy_dx, void* grad_inputs, int32_t dtype,
                           void* stream);

/* ------------------------------------------------------------------------ */
/* freqencoder                                                              */
/* ------------------------------------------------------------------------ */

/* freqencoder/src/freqencoder.h:7, freqencoder.cu:97-111
 * (kernel_freq :30-59). inputs f32 [B, D], outputs f32 [B, C] with
 * C = D (1 + 2 deg): [x, sin(2^0 x), cos(2^0 x), ..., cos(2^(deg-1) x)]. */
int ngp_freq_encode_forward(const float* inputs, uint32_t B, uint32_t D, uint32_t deg, uint32_t C,
                            float* outputs, void* stream);
/* freqencoder.h:10, freqencoder.cu:114-131 (kernel_freq_backward :63-94). grad f32 [B, C],
 * outputs the forward's; grad_inputs f32 [B, D] is written (not added to). */
int ngp_freq_encode_backward(const float* grad, const float* outputs, uint32_t B, uint32_t D,
                             uint32_t deg, uint32_t C, float* grad_inputs, void* stream);

/* ------------------------------------------------------------------------ */
/* ffmlp (fp16 storage, fp16 MFMA with fp32 accumulation)                   */
/* ------------------------------------------------------------------------ */

/* ffmlp/src/ffmlp.h:8, ffmlp.cu:635-671. inputs f16 [B, input_dim], weights
 * f16 flat (per layer row-major [out, in], nn.Linear layout), outputs f16
 * [B, output_dim]. forward_buffer f16 [num_layers, B, hidden] or NULL (the
 * backward below recomputes activations and never reads it).
 * Supported on this build: hidden_dim in {32, 64}, input_dim % 16 == 0 and
 * <= 64, output_dim == 16 (FFMLP pads outputs to 16), num_layers 2..4, any B.
 * Other shapes return NGP_ERR_UNSUPPORTED with the reason in ngp_last_error. */
int ngp_ffmlp_forward(const void* inputs, const void* weights, uint32_t B, uint32_t input_dim,
                      uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                      uint32_t activation, uint32_t output_activation, void* forward_buffer,
                      void* outputs, void* stream);
/* ffmlp.h:9, ffmlp.cu:673-709 */
int ngp_ffmlp_inference(const void* inputs, const void* weights, uint32_t B, uint32_t input_dim,
                        uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                        uint32_t activation, uint32_t output_activation, void* inference_buffer,
                        void* outputs, void* stream);
/* Workspace (bytes) ngp_ffmlp_backward needs for its per-workgroup dW slabs. */
size_t ngp_ffmlp_backward_workspace_bytes(uint32_t B, uint32_t input_dim, uint32_t output_dim,
                                          uint32_t hidden_dim, uint32_t num_layers);
/* ffmlp.h:11, ffmlp.cu:749-895. grad f16 [B, output_dim]; grad_inputs f16
 * [B, input_dim] (written when calc_grad_inputs); grad_weights flat, dtype
 * gw_dtype (F16 like the reference, or F32), overwritten (not accumulated).
 * forward_buffer / backward_buffer may be NULL. */
int ngp_ffmlp_backward(const void* grad, const void* inputs, const void* weights,
                       const void* forward_buffer, uint32_t B, uint32_t input_dim,
                       uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                       uint32_t activation, uint32_t output_activation, int32_t calc_grad_inputs,
                       void* backward_buffer, void* grad_inputs, void* grad_weights,
                       int32_t gw_dtype, void* workspace, size_t workspace_bytes, void* stream);
/* ffmlp.h:12-13, ffmlp.cu:711-740. The side-stream split-K pool of the
 * reference is not needed (dW is reduced in-kernel); kept as no-ops so the
 * FFMLP module's construction sequence is unchanged. */
int ngp_ffmlp_allocate_splitk(size_t size);
int ngp_ffmlp_free_splitk(void);

/* ------------------------------------------------------------------------ */
/* optimizer (next row of SURVEY §8f): fused Adam over a flat f32 param set */
/* ------------------------------------------------------------------------ */

/* torch.optim.Adam semantics (main_nerf.py:194; betas (0.9,0.99), eps 1e-15):
 * m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g;
 * p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps), g = grad (f32 or f16) * grad_scale.
 * step is the 1-based step count after increment. */
int ngp_adam_step(float* params, const void* grads, int32_t grad_dtype, float* exp_avg,
                  float* exp_avg_sq, size_t n, float lr, float beta1, float beta2, float eps,
                  float weight_decay, int32_t step, float grad_scale, void* stream);

/* ---------------------------------------------------------------------------
 * Fused train step (DESIGN.md "fused step"). No reference counterpart as C
 * functions: together they replace the elementwise torch glue of one
 * reference training iteration (nerf/utils.py train_step :453-497 with
 * GradScaler/Adam :194-217, renderer.run_cuda :257-375, network_ff.forward
 * :69-105, gridencoder/grid.py:61-89 casts) with fused kernels. `count`
 * arguments are device pointers to the marcher's sample count: rows at or
 * past it are not computed. `state` is a device StepState
 * (ngp_fused_state_bytes). */
/* embeddings: the fp32 table (emb_dtype NGP_DTYPE_F32, rounded to half on
 * load) or its fp16 copy (NGP_DTYPE_F16, e.g. the one the fused optimizer
 * refreshes after every update): identical results, half the gather bytes. */
int ngp_grid_encode_forward_fused(const float* xyz, float bound, const void* embeddings,
                                  int32_t emb_dtype, const int32_t* offsets, void* outputs, uint32_t B,
                                  const int32_t* count, uint32_t D, uint32_t C, uint32_t L, float S,
                                  uint32_t H, uint32_t gridtype, int32_t align_corners,
                                  uint32_t interp, int32_t out_layout, void* stream);
/* Binned backward (hashed levels without scattered atomics) when workspace is
 * given: offsets_host is a host copy of offsets; the workspace (size from
 * ngp_grid_encode_backward_fused_workspace_bytes, 0 if nothing is binned) must
 * be zero-filled before its first use and is left ready for the next call.
 * nonfinite (nullable; needs offsets_host): set to 1 when a grad entry this
 * call leaves in grad_embeddings is inf/nan: GradScaler's check (torch
 * amp _amp_foreach_non_finite_check_and_unscale_) made by the kernels that
 * write the values (binned levels) or a scan of the other levels. */
size_t ngp_grid_encode_backward_fused_workspace_bytes(uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                                      float S, uint32_t H, int32_t align_corners,
                                                      const int32_t* offsets_host);
/* grad_layout | NGP_GRID_GRAD_ZEROED: grad_embeddings is all zeros on entry
 * (the fused optimizer clears it), so bins that own their table slice store
 * their sums instead of reading the slice back first. */
#define NGP_GRID_GRAD_ZEROED 0x10
/* grad_layout | NGP_GRID_CURSORS_EXTERNAL: the caller zeroes the workspace's
 * first ngp_grid_encode_backward_fused_counter_bytes bytes (the bin cursors and
 * the 512-byte area after them) between calls (the fused step's march launch
 * does), so the call does not leave them zeroed itself. With
 * NGP_GRID_GRAD_ZEROED too, the hashed levels' bins are summed one per wave
 * (same sums, same bits as the workgroup image path; round 7). */
#define NGP_GRID_CURSORS_EXTERNAL 0x20
/* grad_layout | NGP_GRID_TIMING: the binned launches time themselves on the
 * chip's 100 MHz constant clock (s_memrealtime) into a ring in the workspace
 * (ngp_grid_encode_backward_fused_timing_offset; u32 words): [0] calls so
 * far; the head of call c at word 64 + 4 (c % NGP_GRID_TIMING_RING) holds
 * {start (bin launch, block (0, 0)), samples, accumulate workgroups n, 0};
 * its ends at word 64 + 4 NGP_GRID_TIMING_RING + (c % RING) MAX_WG + w, one
 * per accumulate workgroup w < n. A call's span is max_w(end_w - start)
 * (mod 2^32 ticks of 10 ns). Plain stores only: the timed kernels keep their
 * critical path. Zero word 0 to restart. */
#define NGP_GRID_TIMING 0x40
#define NGP_GRID_TIMING_RING 256
#define NGP_GRID_TIMING_MAX_WG 1024
size_t ngp_grid_encode_backward_fused_timing_offset(uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S,
                                                    uint32_t H, int32_t align_corners, const int32_t* offsets_host);
size_t ngp_grid_encode_backward_fused_counter_bytes(uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S,
                                                    uint32_t H, int32_t align_corners,
                                                    const int32_t* offsets_host);
int ngp_grid_encode_backward_fused(const void* grad, const float* xyz, float bound,
                                   const int32_t* offsets, void* grad_embeddings, uint32_t B,
                                   const int32_t* count, uint32_t D, uint32_t C, uint32_t L, float S,
                                   uint32_t H, uint32_t gridtype, int32_t align_corners,
                                   uint32_t interp, const int32_t* offsets_host, void* workspace,
                                   size_t workspace_bytes, int32_t grad_layout, int32_t* nonfinite,
                                   void* stream);
/* ngp_grid_encode_backward_fused plus ngp_ffmlp_reduce of n_nets deferred MLP
 * backward calls (its arguments, fp16 grad_weights, mlp_nonfinite as its
 * nonfinite) carried by the bin launch as an extra column of blocks: the same
 * sums in the same order, one launch less. Without binned levels the reduce
 * runs on its own first. */
int ngp_grid_encode_backward_fused_reduce(const void* grad, const float* xyz, float bound, const int32_t* offsets,
                                          void* grad_embeddings, uint32_t B, const int32_t* count, uint32_t D,
                                          uint32_t C, uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                          int32_t align_corners, uint32_t interp, const int32_t* offsets_host,
                                          void* workspace, size_t workspace_bytes, int32_t grad_layout,
                                          int32_t* nonfinite, int32_t n_nets, void* const* mlp_workspaces,
                                          const uint32_t* mlp_Bs, const uint32_t* in_dims,
                                          const uint32_t* hidden_dims, const uint32_t* num_layers,
                                          void* const* grad_weights, int32_t* mlp_nonfinite, void* stream);
/* The fused step's next batch (ngp_fused_step_head's sampler arguments),
 * drawn by ngp_grid_encode_backward_fused_reduce_batch while this batch's
 * backward runs: the batch buffers are dead once the composite has read its
 * targets. The draw records this batch's counts (step_counter) without
 * resetting the counter, which the backward still reads; the accumulate
 * resets it. */
typedef struct ngp_batch_job {
    const float* poses;
    uint32_t n_poses;
    const float* intrinsics4;
    uint32_t H, W, N;
    const float* boxes;
    int32_t nboxes;
    const float* aabb6;
    float min_near;
    uint32_t seed;
    void* state;
    float *rays_o, *rays_d, *rgba, *bg, *nears, *fars, *noises;
    int32_t *counter, *step_counter;
} ngp_batch_job;
/* ngp_grid_encode_backward_fused_reduce + the next batch (job) as another
 * column of blocks of the bin launch. Requires a binned plan. */
int ngp_grid_encode_backward_fused_reduce_batch(const void* grad, const float* xyz, float bound,
                                                const int32_t* offsets, void* grad_embeddings, uint32_t B,
                                                const int32_t* count, uint32_t D, uint32_t C, uint32_t L,
                                                float S, uint32_t H, uint32_t gridtype, int32_t align_corners,
                                                uint32_t interp, const int32_t* offsets_host, void* workspace,
                                                size_t workspace_bytes, int32_t grad_layout, int32_t* nonfinite,
                                                int32_t n_nets, void* const* mlp_workspaces, const uint32_t* mlp_Bs,
                                                const uint32_t* in_dims, const uint32_t* hidden_dims,
                                                const uint32_t* num_layers, void* const* grad_weights,
                                                int32_t* mlp_nonfinite, const ngp_batch_job* job, void* stream);
/* ngp_grid_encode_backward_fused_reduce_batch over the rows live_rows[0 ..
 * *live_count) (the sample rows of xyz and of the [L, B, C] grad). */
int ngp_grid_encode_backward_fused_reduce_batch_live(
    const void* grad, const float* xyz, float bound, const int32_t* offsets, void* grad_embeddings, uint32_t B,
    const int32_t* live_rows, const int32_t* live_count, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int32_t align_corners, uint32_t interp, const int32_t* offsets_host, void* workspace,
    size_t workspace_bytes, int32_t grad_layout, int32_t* nonfinite, int32_t n_nets, void* const* mlp_workspaces,
    const uint32_t* mlp_Bs, const uint32_t* in_dims, const uint32_t* hidden_dims, const uint32_t* num_layers,
    void* const* grad_weights, int32_t* mlp_nonfinite, const ngp_batch_job* job, void* stream);
/* ngp_grid_encode_forward_fused (out_layout 0) with the fused step's tail as
 * extra workgroups dispatched first: the deferred GradScaler / LambdaLR / loss
 * bookkeeping of the update the march launch applied (state; when pending) and
 * the MLP fragment packs (ngp_ffmlp_pack's arguments; n_nets 0: none). For the
 * march launch of an ngp_adam_job with NGP_ADAM_JOB_TAIL_LATER. */
int ngp_grid_encode_forward_fused_tail(const float* xyz, float bound, const void* embeddings, int32_t emb_dtype,
                                       const int32_t* offsets, void* outputs, uint32_t B, const int32_t* count,
                                       uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                       int32_t align_corners, uint32_t interp, void* state, float growth_factor,
                                       float backoff_factor, int32_t growth_interval, int32_t scaler_enabled,
                                       const float* loss_ray, uint32_t n_rays, int32_t n_nets,
                                       const void* const* mlp_weights, const uint32_t* in_dims,
                                       const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* images,
                                       void* stream);
/* Weight-fragment images (forward + transposed, per matmul) of n networks in
 * one launch; image k needs ngp_ffmlp_image_bytes of its network. The
 * forward/backward *_rows calls below take the image (nullable: the weights
 * are packed per call). */
size_t ngp_ffmlp_image_bytes(uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers);
int ngp_ffmlp_pack(int32_t n, const void* const* weights, const uint32_t* in_dims,
                   const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* images,
                   void* stream);
int ngp_ffmlp_forward_rows(const void* inputs, const void* weights, const void* image, uint32_t B,
                           const int32_t* count, uint32_t in_dim, uint32_t output_dim,
                           uint32_t hidden_dim, uint32_t num_layers, uint32_t activation,
                           uint32_t output_activation, void* outputs, void* stream);
/* The NeRF sigma network with its glue as the epilogue (network_ff.py:61-68):
 * h_out [B,16] half, sigma [B] = density_scale * exp(h[:,0]) fp32, color_in
 * [B,32] half = [SH4(dirs) | h[:,1:16] | 0]. */
int ngp_nerf_sigma_forward(const void* inputs, const void* weights, const void* image, uint32_t B,
                           const int32_t* count, uint32_t in_dim, uint32_t hidden_dim,
                           uint32_t num_layers, void* h_out, float* sigma, void* color_in,
                           const float* dirs, float density_scale, uint32_t flags, void* stream);
/* The whole NeRF forward in one launch (network_ff.py:51-74): the sigma
 * network on pair-major encodings enc [16][B][2] (rows < *count), the
 * ngp_nerf_sigma_forward epilogue (h_out, sigma, color_in, same values), and
 * the colour network on color_in, rgb logits color_out [B,16] half. Images:
 * the two networks' ngp_ffmlp_pack images. 64-wide networks with 32 inputs. */
int ngp_nerf_forward(const void* enc, const void* sigma_image, const void* color_image, uint32_t B,
                     const int32_t* count, uint32_t hidden_dim, uint32_t num_layers,
                     uint32_t hidden_dim_color, uint32_t num_layers_color, void* h_out, float* sigma,
                     void* color_in, const float* dirs, float density_scale, void* color_out,
                     void* stream);
#define NGP_FFMLP_DEFER_REDUCE 1u /* leave dW partials for ngp_ffmlp_reduce */
#define NGP_FFMLP_NERF_GEO 2u     /* grad_inputs [B,16]: input-grad cols 16..30 -> cols 1..15 */
#define NGP_FFMLP_PAIR_MAJOR 4u   /* inputs and grad_inputs as [in_dim/2][B][2] (the grid's [L,B,2]) */
int ngp_ffmlp_backward_rows(const void* grad, const void* inputs, const void* weights,
                            const void* image, uint32_t B, const int32_t* count, uint32_t in_dim,
                            uint32_t output_dim, uint32_t hidden_dim, uint32_t num_layers,
                            uint32_t activation, void* grad_inputs, void* grad_weights,
                            int32_t gw_dtype, uint32_t flags, void* workspace,
                            size_t workspace_bytes, void* stream);
/* Fused-step: both FFMLP backwards of NeRFNetwork (nerf/network_ff.py:
 * color_net then sigma_net, each ffmlp.cu kernel_mlp_fused_backward :410-518)
 * in one launch. Equals ngp_ffmlp_backward_rows of the colour network
 * (flags NGP_FFMLP_NERF_GEO | NGP_FFMLP_DEFER_REDUCE, input width 32, writing
 * g_h[:, 1:16]) followed by that of the sigma network (grad g_h, inputs enc
 * [16][B][2], flags NGP_FFMLP_PAIR_MAJOR | NGP_FFMLP_DEFER_REDUCE, input
 * gradient g_enc): the input gradients bit for bit, the dW partials summed in
 * another order. Workspaces as ngp_ffmlp_backward_workspace_bytes of each
 * network; reduce with ngp_ffmlp_reduce. 64-wide networks, num_layers 2..3.
 * timing (nullable): the grid backward's NGP_GRID_TIMING ring (the fused grid
 * workspace at ngp_grid_encode_backward_fused_timing_offset): workgroup b's
 * end goes into end slot NGP_GRID_TIMING_MAX_WG - 1 - b of the next call, and
 * the grid backward's span then starts at the latest of them. */
int ngp_nerf_backward(const void* g_color_out, const void* color_in, const void* color_image, void* g_h,
                      const void* enc, const void* sigma_image, void* g_enc, uint32_t B, const int32_t* count,
                      uint32_t hidden_dim, uint32_t num_layers, uint32_t hidden_dim_color,
                      uint32_t num_layers_color, void* sigma_workspace, size_t sigma_workspace_bytes,
                      void* color_workspace, size_t color_workspace_bytes, uint32_t* timing, void* stream);
/* ngp_nerf_backward over the rows live_rows[0 .. *live_count) only (see
 * ngp_nerf_composite_loss_live): input gradients are written for those rows,
 * the others are left as they were. */
int ngp_nerf_backward_live(const void* g_color_out, const void* color_in, const void* color_image, void* g_h,
                           const void* enc, const void* sigma_image, void* g_enc, uint32_t B,
                           const int32_t* live_rows, const int32_t* live_count, uint32_t hidden_dim,
                           uint32_t num_layers, uint32_t hidden_dim_color, uint32_t num_layers_color,
                           void* sigma_workspace, size_t sigma_workspace_bytes, void* color_workspace,
                           size_t color_workspace_bytes, uint32_t* timing, void* stream);
/* Sums the deferred dW partials of n backward calls (same B and shapes as
 * those calls) into grad_weights[k], in one launch (n <= 4). nonfinite
 * (nullable): set to 1 when a written grad is inf/nan (GradScaler's check). */
int ngp_ffmlp_reduce(int32_t n, void* const* workspaces, const uint32_t* Bs, const uint32_t* in_dims,
                     const uint32_t* hidden_dims, const uint32_t* num_layers,
                     void* const* grad_weights, int32_t gw_dtype, int32_t* nonfinite, void* stream);
size_t ngp_fused_state_bytes(void);
int ngp_fused_state_init(void* state, float init_scale, void* stream);
/* Synthetic Lego batch (nerf/provider.py SyntheticLego): boxes = nboxes x
 * (lo[3], hi[3], rgb[3]); poses [n_poses, 4, 4]; intrinsics (fx, fy, cx, cy).
 * The batch index is the state's own draw counter. Also records the previous
 * batch's counter[0..1] into step_counter[(draw - 1) % 16] (nullable; the
 * reference's per-step record for update_extra_state) and zeroes counter for
 * the marcher. Touches no state the optimizer uses, so it may run beside
 * ngp_fused_optimizer_step of the previous step. */
int ngp_lego_rays(const float* poses, uint32_t n_poses, const float* intrinsics4, uint32_t H,
                  uint32_t W, uint32_t N, const float* boxes, int32_t nboxes, const float* aabb6,
                  float min_near, uint32_t seed, void* state, float* rays_o, float* rays_d,
                  float* rgba, float* bg, float* nears, float* fars, float* noises,
                  int32_t* counter, int32_t* step_counter, void* stream);
int ngp_nerf_glue_forward(const void* h_sigma, const float* dirs, float density_scale, float* sigma,
                          void* color_in, uint32_t B, const int32_t* count, void* stream);
int ngp_nerf_glue_backward(const void* grad_color_in, void* grad_h_sigma, uint32_t B,
                           const int32_t* count, void* stream);
int ngp_nerf_composite_loss(const float* sigma, const void* color_out, const void* h_sigma,
                            const float* deltas, const int32_t* rays, uint32_t M, uint32_t N,
                            float T_thresh, float density_scale, const float* gt,
                            uint32_t gt_channels, const float* bg, void* state,
                            void* grad_color_out, void* grad_h_sigma, float* out_image,
                            float* out_ws, float* loss_ray, void* stream);
/* ngp_nerf_composite_loss plus the step's live rows: every row whose written
 * gradient (the colour logits' and the density's) is nonzero in some
 * component, listed in ray order in live_rows [M] (live_total[0] of them);
 * ray_rows [M] and live_cnt [N] are scratch (each ray's live rows in its own
 * row range, and their count). The other rows' gradients are exactly zero, so
 * the backwards may skip them (ngp_nerf_backward_live,
 * ngp_grid_encode_backward_fused_reduce_batch_live): the products with a zero
 * row are zeros (instant-ngp compacts its samples before the backward the same
 * way). Two launches. */
int ngp_nerf_composite_loss_live(const float* sigma, const void* color_out, const void* h_sigma,
                                 const float* deltas, const int32_t* rays, uint32_t M, uint32_t N, float T_thresh,
                                 float density_scale, const float* gt, uint32_t gt_channels, const float* bg,
                                 void* state, void* grad_color_out, void* grad_h_sigma, float* out_image,
                                 float* out_ws, float* loss_ray, int32_t* ray_rows, int32_t* live_cnt,
                                 int32_t* live_rows, int32_t* live_total, void* stream);
/* scaler_enabled of the optimizer entries: GradScaler off; on, with its inf
 * check as a sweep over the grads; on, with the check already made by the
 * kernels that wrote the grads into the state's flag (ngp_fused_inf_flag). */
#define NGP_SCALER_OFF 0
#define NGP_ADAM_SHADOW_ALL 2
#define NGP_SCALER_SCAN 1
#define NGP_SCALER_PRECHECKED 2
/* The state's GradScaler flag (local == 0: the found-inf flag the optimizer
 * reads; local != 0: the data-parallel guard's per-rank flag), for the
 * nonfinite arguments of the grid backward and the MLP reduce. */
int32_t* ngp_fused_inf_flag(void* state, int32_t local);
/* Adam (+ GradScaler inf check/unscale/update, LambdaLR 0.1^(epoch/iters))
 * over n_tensors fp32 params with fp16 grads; half_params[k] (nullable) is
 * refreshed with half(p) where the update changed p (every value with
 * zero_grads | NGP_ADAM_SHADOW_ALL: a shadow written only now and then);
 * grads are zeroed when zero_grads & 1;
 * grads are multiplied by grad_mult as well as unscaled (data-parallel mean).
 * step_counter (nullable; pass null when ngp_lego_rays records it) gets
 * counter[0..1] at slot iter % 16. */
int ngp_fused_optimizer_step(int32_t n_tensors, float* const* params, void* const* grads,
                             float* const* exp_avg, float* const* exp_avg_sq,
                             void* const* half_params, const uint64_t* sizes, float lr, float beta1,
                             float beta2, float eps, int32_t iters, int32_t zero_grads,
                             float grad_mult, float growth_factor, float backoff_factor,
                             int32_t growth_interval,
                             int32_t scaler_enabled, uint32_t num_rays, const int32_t* counter,
                             int32_t* step_counter, const float* loss_ray, void* state,
                             void* stream);
/* ngp_fused_optimizer_step without its bookkeeping launch: the GradScaler
 * update, LR epoch, step counts and loss of this update are marked pending in
 * `state` and done by the next ngp_fused_step_head (the fused step's first
 * launch), saving one latency-bound single-block launch per step. */
int ngp_fused_optimizer_update(int32_t n_tensors, float* const* params, void* const* grads,
                               float* const* exp_avg, float* const* exp_avg_sq, void* const* half_params,
                               const uint64_t* sizes, float lr, float beta1, float beta2, float eps,
                               int32_t iters, int32_t zero_grads, float grad_mult, int32_t scaler_enabled,
                               void* state, void* stream);
/* The fused step's first launch: ngp_lego_rays's batch (same arguments), the
 * pending bookkeeping of the last ngp_fused_optimizer_update if any (scaler
 * arguments as ngp_fused_optimizer_step; loss_ray holds the previous batch's
 * per-ray losses, N rays), and ngp_ffmlp_pack of n_nets networks (n_nets may
 * be 0), as disjoint block ranges of one kernel; it also zeroes clear_bytes
 * (a multiple of 16) at clear (nullable: the grid backward's bin cursors). */
int ngp_fused_step_head(const float* poses, uint32_t n_poses, const float* intrinsics4, uint32_t H,
                        uint32_t W, uint32_t N, const float* boxes, int32_t nboxes, const float* aabb6,
                        float min_near, uint32_t seed, void* state, float* rays_o, float* rays_d,
                        float* rgba, float* bg, float* nears, float* fars, float* noises, int32_t* counter,
                        int32_t* step_counter, float growth_factor, float backoff_factor,
                        int32_t growth_interval, int32_t scaler_enabled, const float* loss_ray,
                        int32_t n_nets, const void* const* mlp_weights, const uint32_t* in_dims,
                        const uint32_t* hidden_dims, const uint32_t* num_layers, void* const* images,
                        void* clear, uint32_t clear_bytes, void* stream);
/* ngp_fused_optimizer_update (bookkeeping deferred) and the batch + clear
 * parts of ngp_fused_step_head (same arguments) as block ranges of one launch;
 * the deferred bookkeeping and the MLP packs then go to
 * ngp_march_rays_train_prebuilt_tail. */
int ngp_fused_optimizer_update_head(int32_t n_tensors, float* const* params, void* const* grads,
                                    float* const* exp_avg, float* const* exp_avg_sq,
                                    void* const* half_params, const uint64_t* sizes, float lr, float beta1,
                                    float beta2, float eps, int32_t iters, int32_t zero_grads,
                                    float grad_mult, int32_t scaler_enabled, void* state,
                                    const float* poses, uint32_t n_poses, const float* intrinsics4,
                                    uint32_t H, uint32_t W, uint32_t N, const float* boxes, int32_t nboxes,
                                    const float* aabb6, float min_near, uint32_t seed, float* rays_o,
                                    float* rays_d, float* rgba, float* bg, float* nears, float* fars,
                                    float* noises, int32_t* counter, int32_t* step_counter, void* clear,
                                    uint32_t clear_bytes, void* stream);

/* Data-parallel GradScaler guard for the sharded optimizer (nerf/fused.py,
 * world > 1), run on each rank's own fp16 gradient before the averaging
 * reduce-scatter: if any of its n elements is inf/nan, a NaN is written to
 * grad[r * chunk] for r in [0, world), so every rank's shard of the reduced
 * gradient carries it and every rank's ngp_fused_optimizer_step skips.
 * n % 8 == 0, grad 16-byte aligned, world * chunk <= n. No reference
 * counterpart (the reference trains on one GPU; GradScaler.unscale_ checks
 * the whole gradient, torch/amp/grad_scaler.py). */
int ngp_grad_guard(void* grad_half, uint64_t n, uint64_t chunk, int32_t world, void* state,
                   void* stream);
/* (n == 0: no scan; the per-rank flag ngp_fused_inf_flag(state, 1) was set by
 * the kernels that wrote the gradient.) */

/* Touched-entry gradient exchange of the replicated data-parallel step
 * (nerf/exchange.py; DESIGN.md §7 option B). Replaces the reference's DDP
 * gradient all-reduce (nerf/utils.py:325-327) for the fused engine: each rank
 * lists its nonzero fp16 channel pairs, the lists (fixed size, so the step
 * captures whole) are all-gathered, and every rank sums all of them exactly
 * (int64, 2^-24 fixed point) into the same flat gradient, then runs the full
 * Adam (world 1's step).
 *   list: grad_half[n_values] (16-byte aligned, n_values % 8 == 0) -> send,
 *     ngp_grad_exchange_words(n_values, cap) int64 words: header (int32
 *     count, int32 flags: bit 0 a non-finite value or *inf_flag (nullable)
 *     set; the header must be zero before the call), a table of
 *     bins(n_values) words ((count << 32) | start) and up to cap items
 *     ((half2 bits << 32) | pair index). The gradient is not changed.
 *   reduce: recv = world lists back to back -> grad_half = fp16(sum / world)
 *     over every value (dense); any rank's flag -> *inf_flag |= 1; a list over
 *     cap -> *inf_flag |= 2 (the update is skipped without a scale back-off)
 *     and grad_half zeroed; stats[0] += 1 per overflowed exchange, stats[1] =
 *     max(stats[1], the largest count); send (nullable): this rank's list,
 *     whose header is cleared for the next list call. */
uint32_t ngp_grad_exchange_bins(uint64_t n_values);
uint64_t ngp_grad_exchange_words(uint64_t n_values, uint32_t cap);
int ngp_grad_exchange_list(const void* grad_half, uint64_t n_values, const int32_t* inf_flag, void* send,
                           uint32_t cap, void* stream);
int ngp_grad_exchange_reduce(const void* recv, int32_t world, uint32_t cap, void* grad_half, uint64_t n_values,
                             int32_t* inf_flag, int32_t* stats, void* send, void* stream);

/* ------------------------------------------------------------------------ */
/* Density-grid update (replaces the torch glue of NeRFRenderer.             */
/* update_extra_state, nerf/renderer.py:498-598, and its packbits call,      */
/* raymarching.h:11)                                                          */
/* ------------------------------------------------------------------------ */

/* The query points of one update, P = C * ppc ordered by cascade. coords
 * int32 [P,3] cell coordinates (renderer.py:552-561), or NULL for every cell
 * of each cascade in meshgrid(x, y, z, 'ij') order (ppc = H^3, :516-523);
 * noise f32 [P,3] uniform [0,1) (the reference's rand_like, :533 / :569).
 * Writes xyzs f32 [P,3] = (2c/(H-1) - 1)(bound_c - hgs) + (2 noise - 1) hgs
 * with the reference's fp32 operations, and indices i32 [P] = cascade * H^3 +
 * morton3D(c). */
int ngp_density_grid_points(const int32_t* coords, const float* noise, uint32_t P, uint32_t ppc, uint32_t C,
                            uint32_t H, float bound, float* xyzs, int32_t* indices, void* stream);
/* The points [lo, hi) of the same draws (coords required), written to xyzs /
 * indices [0, hi - lo) in brick order: bucketed by cascade and morton3D(c) >>
 * shift (bricks of >= 512 cells, at most 8192 buckets), in unspecified order
 * inside a bucket. The densities' max into tmp_grid does not depend on the
 * order, so an update gives the same grid as with ngp_density_grid_points,
 * while a wave's points share the coarse levels' cache lines in the query.
 * ws: ngp_density_grid_sort_workspace_bytes(C, H) bytes (cleared here). */
size_t ngp_density_grid_sort_workspace_bytes(uint32_t C, uint32_t H);
int ngp_density_grid_points_sorted(const int32_t* coords, const float* noise, uint32_t P, uint32_t ppc, uint32_t C,
                                   uint32_t H, float bound, uint32_t lo, uint32_t hi, void* ws, size_t ws_bytes,
                                   float* xyzs, int32_t* indices, void* stream);
/* The densities of the points: sigma network forward on their encodings
 * (pair-major [L][B][2] half, ngp_grid_encode_forward_fused out_layout 0),
 * density = exp(h[:,0]) * density_scale (renderer.py:535-536), written as a
 * max into tmp_grid[indices[b]] (tmp_grid f32 [C * H^3], -1 where unset;
 * a cell drawn twice keeps the larger density). image: ngp_ffmlp_pack image
 * of the network or NULL. */
int ngp_nerf_density_forward(const void* inputs, const void* weights, const void* image, uint32_t B,
                             uint32_t in_dim, uint32_t hidden_dim, uint32_t num_layers, float density_scale,
                             const int32_t* indices, float* tmp_grid, void* stream);
/* The same densities stored per row, sigma[b] (no index, no atomic): the full
 * update's Morton-ordered queries (row = cell) and the brick-ordered partial
 * queries (then ngp_density_grid_run_max). 32 inputs, image required. */
int ngp_nerf_density_forward_rows(const void* inputs, const void* image, uint32_t B, uint32_t hidden_dim,
                                  uint32_t num_layers, float density_scale, float* sigma, void* stream);
/* EMA (renderer.py:582-583: where grid >= 0 and tmp >= 0, grid = max(grid *
 * decay, tmp)), tmp reset to -1, stats[0] = sum(clamp(grid, 0)) as a double
 * (mean_density = float(stats[0] / (C H^3)), :584), and the bitfield at
 * min(mean_density, density_thresh) (:589-590), all on the device. stats:
 * NGP_DENSITY_STATS_LEN doubles (the sum, then per-block partial sums added
 * in a fixed order: no atomics, no clear). */
#define NGP_DENSITY_STATS_LEN 1025
int ngp_density_grid_ema_pack(float* grid, float* tmp_grid, uint32_t C, uint32_t H, float decay,
                              double density_thresh, double* stats, uint8_t* bitfield, void* stream);
/* Device-side draws of an update (no host sync, graph-capturable): partial=0:
 * the noise of every cell (coords unused); partial=1: per cascade H^3/4
 * uniform cells then H^3/4 cells drawn from the cascade's occupied cells
 * (grid > 0, listed in cell order as torch.nonzero does, :555-558), with
 * their noise. Counter RNG over (seed ^ 0xd3a5b1c7, update, point): its own
 * domain, apart from the training sampler's draws of the same seed. */
size_t ngp_density_grid_draw_workspace_bytes(uint32_t C, uint32_t H);
int ngp_density_grid_draw(const float* grid, uint32_t C, uint32_t H, uint32_t partial, uint32_t seed,
                          uint32_t update, int32_t* coords, float* noise, void* ws, size_t ws_bytes,
                          void* stream);
/* A partial update's draws for the fused trainer, generated in Morton order:
 * per cascade N = H^3/4 uniform cells and N cells out of the occupied list
 * (grid > 0), i.i.d. with replacement as the reference draws them
 * (renderer.py:548-558), made as uniform order statistics (prefix sums of N+1
 * exponentials from the counter RNG, exact 2^-32 fixed point), so each half's
 * cells come out sorted by Morton code with no sort; the points [lo, hi) of
 * the C * 2N draws (cascade-major, uniform half first) are written to xyzs /
 * indices [0, hi - lo) with k_density_points' arithmetic. H a power of two.
 * draw_ws: ngp_density_grid_draw_workspace_bytes; ostat_ws:
 * ngp_density_grid_ostat_workspace_bytes. */
size_t ngp_density_grid_ostat_workspace_bytes(uint32_t C, uint32_t H);
int ngp_density_grid_draw_sorted(const float* grid, uint32_t C, uint32_t H, uint32_t seed, uint32_t update,
                                 float bound, uint32_t lo, uint32_t hi, void* draw_ws, size_t draw_ws_bytes,
                                 void* ostat_ws, size_t ostat_ws_bytes, float* xyzs, int32_t* indices, void* stream);
/* tmp_grid from the densities sigma[0, hi - lo) of ngp_density_grid_draw_sorted's
 * points [lo, hi): a cell's draws are adjacent within a half, so each run's
 * max is folded in by its first point with one integer atomic max (exact, in
 * any order). tmp_grid holds -1 where nothing was drawn (as the EMA leaves
 * it); densities are >= 0. */
int ngp_density_grid_run_max(const float* sigma, const int32_t* indices, uint32_t C, uint32_t H, uint32_t lo,
                             uint32_t hi, float* tmp_grid, void* stream);
/* mean_count after an update (renderer.py:593-595: int(mean of the last
 * min(16, local_step) batches' sample counts)) on the device: *out = floor(sum
 * / total) over the fused trainer's step-counter ring (int32 [16][2], slot =
 * batch % 16; *draw = batches drawn; ahead: the newest batch is in the ring,
 * else in counter[0]). */
int ngp_density_mean_count(const int32_t* step_counter, const int32_t* draw, const int32_t* counter,
                           uint32_t total, uint32_t ahead, int64_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NGP_HIP_H */
