/*
 * codenerf.h -- C ABI of the MI355X (gfx950) CodeNeRF render/train hot path.
 *
 * The reference (yuliangguo/code-nerf) has no FFI: its hot path is a set of
 * Python calls made by both loops (src/trainer.py:65-84, src/optimizer.py:
 * 75-94).  Each entry point below replaces one of them; the comment names the
 * reference interface (file:line) it stands in for.
 *
 * Conventions
 *   - All buffers are DEVICE pointers owned by the caller (plain float32 unless
 *     stated), all sizes are element counts, every call is asynchronous on the
 *     given HIP stream (hipStream_t passed as void*; NULL = default stream).
 *   - Return 0 on success, a negative code on error; cn_last_error() gives a
 *     thread-local message.  No C++ exception crosses the ABI; no call
 *     allocates device memory (workspaces are caller-provided, sized by the
 *     cn_*_bytes queries).
 *   - Parameters are addressed through a device array of float* in the
 *     reference state_dict order (encoding_xyz.0.weight, encoding_xyz.0.bias,
 *     shape_latent_layer_1.0.weight, ... rgb.2.bias; src/model.py:20-34);
 *     gradients likewise (accumulated, like autograd's .grad).
 *   - Sample index m = ray * n_samples + s (reference layout (R, N, ...)).
 *     Per-sample outputs must be sized for cn_pad_samples(plan, M) samples.
 */
#ifndef CODENERF_H
#define CODENERF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CN_ABI_VERSION 3
#define CN_FP32 0 /* exact-fp32 MFMA path (parity) */
#define CN_BF16 1 /* bf16 operands, fp32 accumulate (throughput) */
/* error-compensated bf16: weights and chain operands as bf16 hi + lo pairs,
 * three MFMAs per block into fp32 (~16-bit operands); dW as CN_BF16 */
#define CN_BF16X3 2
/* the CN_BF16X3 forward chains (rendered rgb at fp32 class) with the CN_BF16
 * backward (dX chain and dW on bf16 operands); the training forward stores the
 * CN_BF16 planes (hi parts only) */
#define CN_BF16X3F 3
/* Largest sample count (M, act_M, R * N) one call accepts: the kernels index
 * samples with 32-bit integers (3 m, 4 m).  Larger images are rendered in
 * ray parts (codenerf_amd.render.ImageStep / CodeNeRF.forward split
 * automatically); a call above the limit returns -1 with cn_last_error().
 * The activation planes have no 4 GB limit: every wave addresses its own
 * 32-sample slab through a 64-bit descriptor base. */
#define CN_MAX_SAMPLES (1 << 28)

typedef struct cn_plan cn_plan;

int cn_abi_version(void);
const char *cn_last_error(void);

/* Measurement hook (no reference counterpart; ABI 3): the next chain, dW or
 * bias-sum kernel the calling thread launches records start_event /
 * stop_event (hipEvent_t, created by the caller) from its own dispatch
 * packet (hipExtLaunchKernel), so a per-kernel timer adds no marker packets
 * between kernels.  Give both or neither (NULL, NULL clears). */
int cn_time_next_launch(void *start_event, void *stop_event);

/* Stream dependency on one device (ABI 3): `waiter` waits for the work queued
 * so far on `signaller`, through an event WITHOUT the system-scope fence a
 * default event record performs (an L2 write-back of everything the last
 * kernel dirtied: ~15 us behind a chain or dW launch).  For the dX / dW
 * pipelining of one step (render.ImageStep); host-visible results still need
 * the stream's own synchronisation. */
int cn_stream_wait(void *waiter_stream, void *signaller_stream);

/* Clock probe (measurement only, no reference counterpart): n_workgroups
 * workgroups of 4 waves issue `iters` x 4 back-to-back bf16 MFMAs
 * (v_mfma_f32_32x32x16_bf16) on hashed operands; wave 0 of each stamps the
 * shader-cycle counter and the 100 MHz real-time counter around the loop:
 * d_out[3 g + 0] = cycles, [3 g + 1] = 100 MHz ticks, [3 g + 2] = a checksum.
 * Effective clock = cycles / ticks x 100 MHz (bench.py records it beside a
 * step time, so box-to-box clock differences can be told from regressions). */
int cn_clock_probe(unsigned int *d_out, int n_workgroups, int iters, unsigned int seed, void *stream);

/* ---- plan: static layout for one network configuration and precision.
 * Replaces CodeNeRF.__init__ (src/model.py:11-34).  Creating a plan and the
 * size queries need no device (tables go up with the first cn_pack_weights).
 * Supported:
 * W = latent_dim = 256, num_xyz_freq = 10, num_dir_freq = 4,
 * (shape_blocks, texture_blocks) in {(3,1), (2,1)}. */
int cn_plan_create(int shape_blocks, int texture_blocks, int W, int num_xyz_freq,
                   int num_dir_freq, int latent_dim, int precision, cn_plan **out);
void cn_plan_destroy(cn_plan *plan);
int cn_plan_num_params(const cn_plan *plan);        /* tensors in the state_dict */
int cn_plan_num_inject(const cn_plan *plan);        /* shape + texture blocks */
int cn_pad_samples(const cn_plan *plan, int M);     /* M rounded to the tile (-1: M invalid) */
int cn_max_samples(void);                           /* CN_MAX_SAMPLES */
size_t cn_act_bytes_per_sample(const cn_plan *plan); /* workspace bytes per sample (splitting) */
size_t cn_packed_bytes(const cn_plan *plan, int bwd); /* packed weights */
size_t cn_blob_floats(const cn_plan *plan);         /* per-call bias blob */
size_t cn_act_bytes(const cn_plan *plan, int M);    /* training activations */
size_t cn_dw_ws_bytes(const cn_plan *plan, int M);  /* weight-grad partials */
/* Layout introspection of the training workspace laid out for M samples
 * (tests and debugging): byte offset of a plane (-1 if it does not exist);
 * *width = its elements per sample (masks: bytes per sample).  Plane
 * element layout: code-nerf_amd/csrc/cn_layout.h (slab_off / plane_off). */
#define CN_PLANE_Y 0     /* index: forward layer whose output it is */
#define CN_PLANE_DA 1    /* index: forward layer whose pre-activation gradient it is */
#define CN_PLANE_PE 2
#define CN_PLANE_DIR 3
#define CN_PLANE_MASKS 4
/* bf16x3 plans only (-1 otherwise): the lo parts rn(x - rn(x)) of the dW
 * pass's X operands, stored by the training forward beside the hi planes */
#define CN_PLANE_YLO 5   /* index: forward layer whose output it is */
#define CN_PLANE_PELO 6
long long cn_act_plane(const cn_plan *plan, int M, int kind, int index, int *width);

/* ---- weights: pack the parameters into the chain kernels' fragment order
 * (fwd: W, bwd: W^T).  Call after every optimiser step. */
int cn_pack_weights(const cn_plan *plan, const float *const *d_params, void *d_pack_fwd,
                    void *d_pack_bwd, void *stream);

/* ---- per-object latent layers, src/model.py:41,49: z_j = ReLU(L_j c + c_j),
 * folded into the next layer's bias (b + W z).  d_blob: cn_blob_floats floats,
 * d_zvec: num_inject x 256. */
int cn_latent_fwd(const cn_plan *plan, const float *const *d_params, const float *d_shape_code,
                  const float *d_texture_code, float *d_blob, float *d_zvec, void *stream);

/* ---- CodeNeRF.forward (src/model.py:36-53) for M samples.
 * mode A (d_xyz != NULL): explicit points xyz/viewdir [M][3];
 * mode B (d_xyz == NULL): samples of rays, xyz = rays_o + rays_d * z
 *   (src/utils.py:30), z = d_z[ray * z_stride + s] (z_stride 0: one z vector
 *   shared by all rays as in the reference, n_samples: per-ray z).
 * d_sigma [Mp], d_rgb [Mp][3].  d_act != NULL stores what the backward
 * needs: the workspace holds cn_act_bytes(plan, act_M) bytes (act_M <= 0:
 * act_M = M) and this call fills its sample rows [act_row0, act_row0 + Mp)
 * (act_row0 a multiple of cn_pad_samples' granule, 256), so the coarse and
 * the fine pass of one image share one workspace and one backward. */
int cn_mlp_fwd(const cn_plan *plan, const void *d_pack_fwd, const float *d_blob, int M,
               const float *d_xyz, const float *d_viewdir, const float *d_rays_o,
               const float *d_rays_d, const float *d_z, int z_stride, int n_samples,
               float *d_sigma, float *d_rgb, void *d_act, int act_M, int act_row0,
               void *stream);

/* ---- autograd of CodeNeRF.forward (src/trainer.py:82): dX chain. */
int cn_mlp_bwd(const cn_plan *plan, const void *d_pack_bwd, const float *d_blob, int M,
               const float *d_dsigma, const float *d_drgb, void *d_act, void *stream);

/* ---- the same over rows [act_row0, act_row0 + pad(M)) of a workspace laid
 * out for act_M samples (act_row0 a multiple of 256); d_dsigma / d_drgb point
 * at the range's first row.  The coarse and fine rows of one training step
 * (src/trainer.py:82 over both passes) are back-propagated by two launches so
 * the weight gradients of the first range (cn_mlp_dw_rows, on a second
 * stream) overlap the dX chain of the second. */
int cn_mlp_bwd_rows(const cn_plan *plan, const void *d_pack_bwd, const float *d_blob, int M,
                    const float *d_dsigma, const float *d_drgb, void *d_act, int act_M, int act_row0,
                    void *stream);

/* ---- codes-only optimisation (src/optimizer.py:75-98: the model is fixed,
 * only the latent codes are updated).  Same arguments as cn_mlp_fwd /
 * cn_mlp_bwd_rows (d_act required); the forward stores only what the backward
 * needs (ReLU masks, sigma pre-activations), the backward only the gradient
 * planes of the layers fed by a code -- what cn_mlp_dbias reads -- and none of
 * the weight-gradient operands. */
int cn_mlp_fwd_codes(const cn_plan *plan, const void *d_pack_fwd, const float *d_blob, int M,
                     const float *d_xyz, const float *d_viewdir, const float *d_rays_o,
                     const float *d_rays_d, const float *d_z, int z_stride, int n_samples,
                     float *d_sigma, float *d_rgb, void *d_act, int act_M, int act_row0,
                     void *stream);
int cn_mlp_bwd_codes(const cn_plan *plan, const void *d_pack_bwd, const float *d_blob, int M,
                     const float *d_dsigma, const float *d_drgb, void *d_act, int act_M,
                     int act_row0, void *stream);

/* ---- weight / bias gradients, accumulated into d_grads; d_dbuf
 * (num_inject x 256) receives this call's bias gradient of every layer fed by
 * a latent code (input of cn_latent_bwd).  d_params: the parameter tensors the
 * forward used (the table given to cn_pack_weights): encoding_shape's planes
 * are not stored, its gradients and those of the layers reading its output
 * (sigma head, encoding_viewdir) are folded through its weights. */
int cn_mlp_dw(const cn_plan *plan, void *d_act, int M, const float *d_zvec,
              const float *const *d_params, float *const *d_grads, float *d_dbuf, void *d_ws,
              void *stream);

/* ---- cn_mlp_dw over rows [act_row0, act_row0 + pad(M)) of a workspace laid
 * out for act_M samples (act_row0 a multiple of 256).  db_accum != 0 adds
 * this range's bias gradients into d_dbuf instead of overwriting it (the
 * later ranges of a step).  Grads accumulate as in cn_mlp_dw.
 * n_workgroups: persistent workgroups of the pass (0 = one per CU, 256);
 * fewer leave CUs to a dX chain running beside it on another stream (at
 * least 26: a workgroup's share must not span more than two layers). */
int cn_mlp_dw_rows(const cn_plan *plan, void *d_act, int act_M, int act_row0, int M,
                   const float *d_zvec, const float *const *d_params, float *const *d_grads,
                   float *d_dbuf, int db_accum, int n_workgroups, void *d_ws, void *stream);

/* ---- bias gradients of the layers after each code injection only (d_dbuf
 * [n_inject][256], as cn_mlp_dw writes them), for codes-only optimisation
 * (src/optimizer.py:92: the model is fixed, only the codes are updated, so
 * no weight gradients are needed), over rows [0, pad(M)) of a workspace laid
 * out for act_M samples (act_M <= 0: M).  d_ws: cn_dw_ws_bytes(plan, M) bytes. */
int cn_mlp_dbias(const cn_plan *plan, void *d_act, int act_M, int M, float *d_dbuf, void *d_ws,
                 void *stream);

/* ---- latent layers + code gradients (+ the code regulariser of
 * src/trainer.py:76-78 when reg_coef != 0; *d_reg_out = reg value:
 * written, not accumulated; 0 when reg_coef == 0).
 * d_scratch: num_inject x 256 floats.  d_dshape / d_dtex accumulate. */
int cn_latent_bwd(const cn_plan *plan, const float *const *d_params, float *const *d_grads,
                  const float *d_shape_code, const float *d_texture_code, const float *d_zvec,
                  const float *d_dbuf, float *d_scratch, float *d_dshape, float *d_dtex,
                  float reg_coef, float *d_reg_out, void *stream);

/* ---- geometry / rendering --------------------------------------------- */
/* get_rays, src/utils.py:10-19.  d_c2w: 4x4 row-major.  focal_is_f64: the
 * reference receives focal as a float64 tensor from default_collate and forms
 * the camera directions in float64 (type promotion) before casting. */
int cn_get_rays(int H, int W, double focal, int focal_is_f64, const float *d_c2w,
                float *d_rays_o, float *d_viewdirs, void *stream);
/* sample_from_rays point expansion, src/utils.py:30-31 */
int cn_sample_points(const float *d_rays_o, const float *d_viewdirs, const float *d_z, int z_stride,
                     int R, int N, float *d_xyz, float *d_viewdir_rep, void *stream);
/* volume_rendering, src/utils.py:34-47 (N <= 256).  d_weights may be NULL. */
int cn_composite_fwd(const float *d_sigma, const float *d_rgb, const float *d_z, int z_stride,
                     int R, int N, int white_bg, float *d_out_rgb, float *d_out_depth,
                     float *d_weights, void *stream);
/* autograd of volume_rendering; d_grad_depth may be NULL */
int cn_composite_bwd(const float *d_sigma, const float *d_rgb, const float *d_z, int z_stride,
                     int R, int N, int white_bg, const float *d_grad_rgb,
                     const float *d_grad_depth, float *d_dsigma, float *d_drgb, void *stream);
/* training: composite + chunk-mean MSE (src/trainer.py:69,75; chunk = batch
 * size B) + its gradient w.r.t. sigma / rgb.  d_chunk_loss: ceil(R/chunk). */
int cn_render_loss(const float *d_sigma, const float *d_rgb, const float *d_z, int z_stride,
                   int R, int N, int white_bg, const float *d_gt, int chunk, float *d_out_rgb,
                   float *d_ray_se, float *d_chunk_loss, float *d_dsigma, float *d_drgb,
                   void *stream);

/* ---- hierarchical sampling (BASELINE configs' "64 coarse + 64 fine"; the
 * reference has no fine pass -- NeRF's sample_pdf restated, oracle
 * oracle/ref_cpu.py:sample_pdf).  Per ray: bins = midpoints of the coarse z,
 * pdf = weights[1:-1] + 1e-5 normalised, u_j = (j + d_rand[ray][j]) / Nf,
 * d_z_f [R][Nf] = inverse cdf (ascending). */
int cn_sample_pdf(const float *d_sigma_c, const float *d_z_c, int zc_stride, int R, int Nc,
                  const float *d_rand, int Nf, float *d_z_f, void *stream);

/* fine composite over the union of each ray's coarse and fine samples
 * (merged by z) + chunk-mean MSE + backward.  d_dsig_c / d_drgb_c are
 * accumulated into (they hold the coarse loss's gradient from
 * cn_render_loss); d_dsig_f / d_drgb_f [R*Nf] are written. */
int cn_render_loss_fine(const float *d_sigma_c, const float *d_rgb_c, const float *d_z_c,
                        int zc_stride, int Nc, const float *d_sigma_f, const float *d_rgb_f,
                        const float *d_z_f, int Nf, int R, int white_bg, const float *d_gt,
                        int chunk, float *d_out_rgb, float *d_ray_se, float *d_chunk_loss,
                        float *d_dsig_c, float *d_drgb_c, float *d_dsig_f, float *d_drgb_f,
                        void *stream);

/* ---- torch.optim.AdamW step (src/trainer.py:116-120) over nseg tensors
 * (host arrays of device pointers), step = 1-based count of this update. */
int cn_adamw_step(int nseg, float *const *p, const float *const *g, float *const *m,
                  float *const *v, const int *n, const double *lr, double weight_decay,
                  double beta1, double beta2, double eps, int step, void *stream);
/* the same step, and every gradient element is set to 0 once read: the next
 * step's optimizer.zero_grad() (src/trainer.py:64) without a launch of its own */
int cn_adamw_step_zero_grad(int nseg, float *const *p, float *const *g, float *const *m,
                            float *const *v, const int *n, const double *lr, double weight_decay,
                            double beta1, double beta2, double eps, int step, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CODENERF_H */
