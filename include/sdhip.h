/*
 * sdhip.h -- C ABI of the MI355X (gfx950) SceneDINO render hot path.
 *
 * libsdhip.so is a plain C-ABI shared library: raw device pointers, sizes and a
 * hipStream_t (passed as void*), int status returns (0 = ok, <0 = error; text via
 * sd_last_error()).  No torch types cross the boundary.  The caller owns and
 * allocates every buffer; launches are asynchronous on the given stream; the
 * library keeps no mutable global state beyond the per-thread error string.
 *
 * The reference (tum-vision/scenedino) is pure Python/PyTorch: its boundary for
 * this path is the Python plugin API (scenedino.renderer.NeRFRenderer,
 * scenedino.models.BTSNet, scenedino.common.ray_sampler.ImageRaySampler).  Each
 * entry point below replaces the reference computation cited next to it; the
 * Python mirror in scenedino_amd/ binds them with ctypes.
 *
 * Layouts (all row-major, float32 unless stated):
 *   rays        (R, ray_dim>=8)  [o(3), d(3), near, far, (frame_id, x, y)]
 *   z           (R, K)
 *   camera rec  SD_CAM_WORDS (36) floats: w2c rows 0..2 (12 floats, 3x4), K (9 floats,
 *               3x3), 3 zeros, then the fused projection P = K . w2c[:3] (12 floats,
 *               3x4, rounded once from an exact product) that the 16-bit render kernels
 *               use in place of the two-step pts_into_camera / project_to_image
 *   grid        (B, Hf, Wf, C) NHWC, element type = the FIELD dtype of the MLP dtype:
 *               sd_field_dtype(SD_F32) = SD_F32, sd_field_dtype(SD_BF16) =
 *               sd_field_dtype(SD_F16) = SD_F16 -- the bf16 mode keeps every operand
 *               upstream of sigma (grid, W_in, projected grid, taps, code) in f16 and
 *               only the DINO output layer in bf16.  The render / field
 *               entry points check the caller's grid_dtype against it (ABI 10).
 *   colour img  (B, nv, Hc, Wc, 4) NHWC4 float32 (rgb + pad)
 */
#ifndef SDHIP_H
#define SDHIP_H

#include <stdint.h>

#define SD_CAM_WORDS 36  /* floats per camera record (see layout above) */
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sd_dtype { SD_F32 = 0, SD_BF16 = 1, SD_F16 = 2 };

/* Last error text of the calling thread ("" if none). */
const char *sd_last_error(void);

/* Library / ABI version (bumped on any signature change).  10: grid_dtype fields in
 * sd_render_args / sd_field_args, sd_field_dtype.  11: sd_seg_head.frag_layout. */
int sd_abi_version(void);

/* Element type of the grids the field / render kernels read for an MLP of `dtype`
 * (sd_mlp.dtype / sd_head.dtype): SD_F32 -> SD_F32, SD_BF16 and SD_F16 -> SD_F16.
 * Returns -1 for an unknown dtype.  Pack a grid for sd_render_fused / sd_field_query with
 * sd_pack_grid / sd_cast_grid(dtype = sd_field_dtype(mlp dtype)); sd_project_grid* write
 * the projected grid in sd_field_dtype(mlp->dtype). */
int sd_field_dtype(int dtype);

/* Leave n CUs of the device to other kernels: the persistent one-workgroup-per-CU grids
 * (projection, tile render and its fallback, field query, ...) launch on the device's CUs
 * minus n, rounded down to a multiple of 8.  For the multi-GPU step, whose RCCL all-gather of
 * the previous frame (one workgroup per channel, NCCL_MAX_NCHANNELS) runs beside the render:
 * a persistent workgroup whose CU that kernel holds would start only after it.  Process-wide;
 * set it before sizing sd_render_proj's work (sd_render_proj_work_bytes depends on it).
 * Returns the previous value. */
int32_t sd_reserve_cus(int32_t n);

/* Diagnostic: nblocks single-wave workgroups spinning for `us` microseconds on the stream
 * (stands in for another stream's kernel holding CUs, tools/contention_ab.py). */
int sd_spin(int32_t nblocks, float us, void *stream);

/* Frustum ray generation, bit-exact with the reference's fp32 arithmetic.
 * Replaces util.unproj_map + util.gen_rays + ImageRaySampler.sample
 *   (scenedino/common/util.py:113-158, util.py:253-285,
 *    scenedino/common/ray_sampler.py:439-513).
 * poses_c2w (n_views,4,4), Ks (n_views,3,3) normalised intrinsics,
 * frame_ids (n_views); rays_out (n_views, H, W, 11). */
int sd_gen_rays(const float *poses_c2w, const float *Ks, const float *frame_ids,
                int64_t n_views, int64_t H, int64_t W, float z_near, float z_far,
                float *rays_out, void *stream);

/* Patch ray sampling (training batches): PatchRaySampler.sample with snap_to_grid
 * (scenedino/common/ray_sampler.py:136-287).  The caller draws the patch positions with the
 * reference's own RNG calls (host) and passes them as patches (B, n_patches, 4) int32:
 * [view, top-left y, top-left x, DINO cell row * dino_w + col].  Only the sampled pixels'
 * rays are generated (bit-exact with sd_gen_rays / util.gen_rays); the rgb target
 * (images (B, V, channels, H, W)) and the DINO target (dino (B, V, dino_c, dino_h, dino_w):
 * per pixel if dino_upscaled, else one row per patch) are gathered alongside.
 * Outputs: rays (B, n_patches*ph*pw, 11), rgb_out (B, n_patches*ph*pw, channels),
 * dino_out (B, n_patches*ph*pw, dino_c) or (B, n_patches, dino_c); rgb_out / dino_out may
 * be NULL.  All pointers are device pointers except the struct itself. */
typedef struct sd_patch_args {
    const float *poses;      /* (B, V, 4, 4) camera-to-world                               */
    const float *Ks;         /* (B, V, 3, 3) normalised intrinsics                         */
    const float *frame_ids;  /* (V) ray frame-id column                                    */
    const int32_t *patches;  /* (B, n_patches, 4)                                          */
    const float *images;     /* (B, V, channels, H, W) or NULL                             */
    const float *dino;       /* (B, V, dino_c, dino_h, dino_w) or NULL                     */
    float *rays;
    float *rgb_out;
    float *dino_out;
    int64_t B, V, H, W;
    int32_t n_patches, ph, pw, channels;
    int32_t dino_c, dino_h, dino_w, dino_upscaled;
    float z_near, z_far;
} sd_patch_args;

int sd_patch_rays(const sd_patch_args *args, void *stream);

/* Channels-last f32 grid (n elements, n % 4 == 0) -> element type dtype (SD_BF16 / SD_F16),
 * same layout: the NHWC gather operand of sd_render_fused / sd_field_query when the grid
 * already is channels-last (sd_pack_grid transposes an NCHW one).  A plain conversion: for
 * the render / field kernels pass dtype = sd_field_dtype(mlp dtype) (f16 in both 16-bit
 * modes) and set grid_dtype to the same value. */
int sd_cast_grid(const float *grid_nhwc, int64_t n, int dtype, void *out, void *stream);

/* Stratified inverse-depth (lindisp) or linear z sampling.
 * Replaces NeRFRenderer.sample_coarse (scenedino/renderer/nerf.py:121-141).
 * u == NULL: jitter drawn from a counter-based RNG keyed by (seed, offset);
 * u != NULL: jitter read from u (R, K) -> bit-exact with the reference. */
int sd_sample_z(const float *rays, int64_t R, int64_t ray_dim, int64_t K, int lindisp,
                const float *u, uint64_t seed, uint64_t offset, float *z_out, void *stream);

/* NCHW float32 feature grid (B,C,H,W) -> NHWC (B,H,W,C) in element type dtype (a plain
 * conversion; the render / field kernels read sd_field_dtype(mlp dtype), see above).
 * Layout step for F.grid_sample over BTSNet.grid_f_features (bts.py:299-309). */
int sd_pack_grid(const float *grid_nchw, int64_t B, int64_t C, int64_t H, int64_t W,
                 int dtype, void *out_nhwc, void *stream);

/* NCHW colour images (B*nv, 3, H, W) -> NHWC4 float32 (B*nv, H, W, 4).
 * Layout step for BTSNet.sample_colors' F.grid_sample (bts.py:348-358). */
int sd_pack_image(const float *img_nchw, int64_t N, int64_t H, int64_t W, float *out_nhwc4,
                  void *stream);

/* Camera records of n views: out (n, 36) = [w2c rows 0..2 (3x4) | K (3x3) | 0 0 0 | K.w2c (3x4)], the
 * operands of pts_into_camera / project_to_image (pinhole.py:40-84) as the field
 * kernels read them.  w2c: (n, 4, 4) with element stride s_w (>= 16) between views,
 * inner 4x4 contiguous; Ks: (n, 3, 3), stride s_k (>= 9). */
int sd_cam_records(const float *w2c, int64_t s_w, const float *Ks, int64_t s_k, int64_t n,
                   float *out, void *stream);

/* sd_pack_image + sd_cam_records in one launch (the per-frame render inputs of
 * BTSNet.encode's colour images and encoder cameras; same outputs as the two calls). */
int sd_frame_inputs(const float *img_nchw, int64_t N, int64_t H, int64_t W, float *out_nhwc4,
                    const float *w2c, int64_t s_w, const float *Ks, int64_t s_k, int64_t n,
                    float *out_cam, void *stream);

/* The operands of sd_frame_inputs, for sd_project_grid_nhwc_inputs below. */
typedef struct sd_frame_args {
    const float *img_nchw; int64_t N, H, W; float *out_nhwc4;
    const float *w2c; int64_t s_w; const float *Ks; int64_t s_k; int64_t n; float *out_cam;
} sd_frame_args;

/* Per-point MLP parameters, pre-packed (by the host) into MFMA fragment order.
 * ResnetFC(n_blocks=0): out = W_out relu(W_in x + b_in) + b_out
 *   (scenedino/models/prediction_heads/resnetfc.py:135-203). */
typedef struct sd_mlp {
    const void *w_in;      /* [C/16+3][4][64][8] of dtype (layer-1 A fragments)            */
    const float *b_in_h;   /* [4][2][16] hidden bias, accumulator-row order                */
    const float *w_sig_h;  /* [4][2][16] W_out row 0 (sigma), accumulator-row order        */
    float b_sigma;         /* b_out[0]                                                     */
    const void *w_out;     /* layer-2 A fragments for the D dino rows (dtype-specific)     */
    const float *b_dino;   /* b_out[1:1+D]                                                 */
    int32_t C;             /* grid channels (multiple of 32)                               */
    int32_t D;             /* dino dims (multiple of 32)                                   */
    int32_t dtype;         /* SD_F32 (exact-f32 MFMA), SD_BF16 or SD_F16 (16-bit MFMA,   */
                           /* f32 accumulate); grids and w_in are in sd_field_dtype(dtype) */
                           /* (f16 for SD_BF16 too), the dino output layer in dtype        */
    int32_t d_hidden;      /* must be 128                                                  */
    const float *b_empty_h; /* learn_empty (bts.py:311-319), NULL if off: [4][2][16]       */
                           /* b_in + W_in[:, :C] . empty_feature in accumulator-row order:  */
                           /* the layer-1 pre-code activation of a point outside the       */
                           /* encoder frustum (sd_render_fused / sd_field_query only)       */
    int32_t proj_flags;    /* sd_project_grid*: bit 0 (SD_PROJ_EXACT_GRID) = the f32 grid   */
                           /* enters the MFMA as a hi + lo f16 pair (hi = f16(g), lo =      */
                           /* f16(g - hi)): P within ~2^-12 of W16 . G instead of W16 . G16 */
                           /* -- twice the MFMAs; configs[3]'s K = 128 renders need it for  */
                           /* the 1e-2 m depth bound.  0 = one f16 rounding.    */
    int32_t pad_mlp;
} sd_mlp;

#define SD_PROJ_EXACT_GRID 1

/* Fused coarse render of R rays x K samples: point generation, projection into the
 * encoder view, positional code, bilinear feature gather, MFMA MLP, softplus,
 * colour sampling in nv render views, alpha compositing (sequential
 * transmittance per ray) of depth / DINO features / colour.
 * Replaces NeRFRenderer.composite + BTSNet.forward + sample_features + sample_colors
 *   (nerf.py:230-449, bts.py:271-441, bts.py:476-595).
 * Optional per-sample outputs may be NULL. */
typedef struct sd_render_args {
    const float *rays; int64_t ray_dim; int64_t R; int64_t rays_per_sb; int32_t K;
    const float *z;                       /* (R, K)                                */
    const void *grid; int32_t Hf, Wf;     /* (B, Hf, Wf, C) NHWC                   */
    const float *cam_f;                   /* (B, 36)                               */
    const float *img; int32_t nv, Hc, Wc; /* (B, nv, Hc, Wc, 4) or NULL if nv==0   */
    const float *cam_c;                   /* (B, nv, 36); may alias cam_f (nv == 1, */
                                          /* colour view = encoder view): the render */
                                          /* kernels then re-use the encoder taps    */
                                          /* for the colours at equal resolution     */
    int32_t hard_alpha_cap;
    /* required outputs */
    float *depth;      /* (R)        */
    float *dino;       /* (R, D)     */
    float *rgb;        /* (R, 3 nv)  */
    /* optional outputs (NULL = not wanted) */
    float *weights;    /* (R, K)         */
    float *alphas;     /* (R, K)         */
    float *invalid;    /* (R, K, nv)     */
    uint8_t *invalid_f;/* (R, K)         */
    float *rgb_samps;  /* (R, K, 3 nv)   */
    /* In-kernel z sampling (sd_render_proj only): with z == NULL the kernel draws
     * each ray's depths itself exactly as sd_sample_z(rays, R, ray_dim, K, z_lindisp,
     * NULL, z_seed, z_offset) would (NeRFRenderer.sample_coarse, nerf.py:121-141),
     * so the (R, K) depth array never goes through HBM.  Ignored when z != NULL. */
    int32_t z_lindisp;
    uint64_t z_seed, z_offset;
    /* Scratch of sd_render_proj_work_bytes(R, D) bytes (sd_render_proj only; NULL when
     * that is 0): for wide DINO heads the kernel composites the 128-d hidden vectors,
     * sum_k w_k relu(h_k), and applies W_dino once per ray afterwards (the output layer is
     * linear: sum_k w_k (W h_k + b) = W sum_k w_k h_k + b sum_k w_k, nerf.py:394 over
     * resnetfc.py:199). */
    float *work;
    /* Row strides (in floats) of depth / dino / rgb; 0 = dense (1, D, 3 nv).  Lets the caller
     * render straight into one packed [dino | depth | rgb] row per ray, e.g. the send buffer
     * of the multi-GPU all-gather (sd_render_proj only; sd_render_fused requires 0). */
    int64_t ld_depth, ld_dino, ld_rgb;
    /* Element type of `grid`, checked against what the kernel reads (ABI 10): sd_render_fused
     * sd_field_dtype(mlp->dtype); sd_render_proj SD_F16 (the projected grid of both 16-bit
     * modes).  A mismatch returns -1 instead of reading the bits as another type. */
    int32_t grid_dtype;
    int32_t pad1;
} sd_render_args;

int sd_render_fused(const sd_render_args *args, const sd_mlp *mlp, void *stream);

/* ---- projected-grid render (16-bit modes) ----------------------------------
 * F.grid_sample is linear in the grid and its bilinear weights sum to one, so the
 * grid part of ResnetFC's first layer commutes with the feature gather
 * (bts.py:299-328 then resnetfc.py:163):
 *     W_in[:, :C] . sample(G, xy) + b_in  ==  sample(W_in[:, :C] . G + b_in, xy).
 * sd_project_grid evaluates P = W_in[:, :C] . G + b_in once per grid PIXEL (an MFMA
 * GEMM over C); sd_render_proj then gathers 128-channel P taps per sample and adds
 * the positional-code columns by MFMA.  Same outputs as sd_render_fused up to
 * rounding order (16-bit modes only; the f32 parity mode keeps sd_render_fused). */

/* grid_nchw (B, C, Hf, Wf) float32 -> out (B, Hf, Wf, 128) in sd_field_dtype(mlp->dtype)
 * (f16 for both 16-bit modes; mlp->dtype must be SD_BF16 or SD_F16),
 * plain NHWC: out[b][y][x][n] = P[y][x][n], 256 B per grid pixel.
 * Uses mlp->w_in chunks 0..C/16-1 and mlp->b_in_h. */
int sd_project_grid(const float *grid_nchw, int64_t B, int64_t Hf, int64_t Wf,
                    const sd_mlp *mlp, void *out, void *stream);

/* Same from a channels-last grid (B, Hf, Wf, C) float32 -- the layout the native encoder's
 * DPT writes (its NCHW-shaped grid_f_features is a permuted view of it). */
int sd_project_grid_nhwc(const float *grid_nhwc, int64_t B, int64_t Hf, int64_t Wf,
                         const sd_mlp *mlp, void *out, void *stream);

/* sd_project_grid_nhwc + sd_frame_inputs(*frame) -- a new frame's render inputs -- in ONE
 * launch where the streaming projection kernel takes the grid (C = 256): its workgroups
 * pack the image and write the camera records before their grid sweep (one kernel
 * boundary fewer per frame).  Same outputs as the two calls (which it makes otherwise). */
int sd_project_grid_nhwc_inputs(const float *grid_nhwc, int64_t B, int64_t Hf, int64_t Wf,
                                const sd_mlp *mlp, void *out, const sd_frame_args *frame,
                                void *stream);

/* Head of the projected render: code columns of W_in and the output layer, packed
 * for 16x16x32 MFMA (scenedino_amd/mlp_pack.py documents the fragment maps). */
typedef struct sd_head {
    const void *w_pe;      /* [8][64][8] ++ [8][64][4] code-column A fragments, dtype */
    const void *w_sig;     /* [4][64][8]    W_out row 0 (sigma) A fragments, dtype    */
    const void *w_out;     /* [D/16][4][64][8] W_out rows 1..D A fragments, dtype     */
    const float *b_dino;   /* b_out[1:1+D]                                            */
    float b_sigma;         /* b_out[0]                                                */
    int32_t D;             /* multiple of 16, <= 512                                  */
    int32_t dtype;         /* SD_BF16 or SD_F16: w_out (the DINO head) in dtype; w_pe and */
                           /* w_sig in sd_field_dtype(dtype) = f16 in both modes          */
} sd_head;

/* args->grid = the projected grid (B, Hf, Wf, 128) f16 from sd_project_grid (grid_dtype
 * SD_F16); K % 16 == 0.
 * Outputs as sd_render_fused; args->z may be NULL (in-kernel z sampling, see above). */
int sd_render_proj(const sd_render_args *args, const sd_head *head, void *stream);

/* Bytes of args->work sd_render_proj needs for R rays and a D-dim DINO head (0: none). */
int64_t sd_render_proj_work_bytes(int64_t R, int32_t D);

/* Test hook: cap the tile kernel's tile buffers at `bytes` (rounded down to KiB; 0 = no cap;
 * below 16 KiB the per-ray kernel renders everything), so a test can force tap boxes into
 * the per-workgroup overflow lists and the per-ray fallback behind the tile kernel.  Returns
 * the previous cap.  Process-wide, not thread-safe; the shipped path never sets it. */
int32_t sd_render_tile_cap(int32_t bytes);

/* Per-point field query without compositing (BTSNet.forward on raw points,
 * bts.py:476-595; SSCBench predict_grid / demo inference_3d).  Points are
 * (B, P, 3); outputs sigma (B,P), dino (B,P,D); colour outputs optional. */
typedef struct sd_field_args {
    const float *xyz; int64_t B; int64_t P;
    const void *grid; int32_t Hf, Wf;
    const float *cam_f;                   /* (B, 36)            */
    const float *img; int32_t nv, Hc, Wc; /* may be NULL / nv=0 */
    const float *cam_c;                   /* (B, nv, 36)        */
    float *sigma;      /* (B, P)             */
    float *dino;       /* (B, P, D)          */
    float *rgb;        /* (B, P, 3 nv) or NULL */
    float *invalid;    /* (B, P, nv) or NULL   */
    uint8_t *invalid_f;/* (B, P) or NULL       */
    int32_t dino_dtype;/* SD_F32 (0), or SD_BF16: dino written as bf16 (the input a
                        * following sd_seg_query rounds to bf16 anyway: half the bytes) */
    int32_t grid_dtype;/* element type of grid (ABI 10): sd_field_dtype(mlp->dtype); checked */
    /* Visiting order of the ceil(B P / 32) tiles of 32 consecutive points, or NULL (natural
     * order).  Speed only (every output stays at its point's index): an order in which
     * consecutive tiles project onto neighbouring texels keeps the grid taps in the XCD's
     * L2 (the SSCBench voxel columns sorted by projected pixel, BTSNet.query). */
    const int32_t *tile_order;
} sd_field_args;

int sd_field_query(const sd_field_args *args, const sd_mlp *mlp, void *stream);

/* Standalone alpha compositing for an arbitrary (non-fused) field model.
 * Replaces nerf.py:343-405.  sigma,z (R,K); feat (R,K,F) optional, rgb (R,K,Cc). */
int sd_composite(const float *z, const float *sigma, const float *feat, int64_t F,
                 const float *rgb, int64_t Cc, int64_t R, int32_t K, int32_t hard_alpha_cap,
                 float *weights, float *alphas, float *depth, float *feat_out, float *rgb_out,
                 void *stream);

/* ---- Differentiable (training) field path (sdhip_train.hip) ----------------- */

/* MLP input rows of the training path: per point the projection / frustum mask
 * (pinhole.py:40-112), the bilinear border gather of the C grid channels
 * (bts.py:299-309, F.grid_sample align_corners=False) and the 39-d positional code
 * (positional_encoding.py:13-80), written as x_out (B*P, C+40) = [feat | code | 1]
 * (bts.py:321-328; the constant 1 column carries the ResnetFC biases through its GEMMs).  grid_nhwc (B, Hf, Wf, C) f32.  Colour samples / masks as
 * sd_field_query (bts.py:330-441; rgb, invalid, img, cam_c may be NULL / nv = 0).
 * x_out element type x_dtype: SD_F32, or SD_F16 / SD_BF16 (the MLP's autocast dtype). */
int sd_field_gather(const float *xyz, int64_t B, int64_t P, const float *grid_nhwc,
                    int32_t C, int32_t Hf, int32_t Wf, const float *cam_f,
                    const float *img, int32_t nv, int32_t Hc, int32_t Wc,
                    const float *cam_c, void *x_out, int32_t x_dtype /* sd_dtype */,
                    uint8_t *invalid_f, float *rgb, float *invalid, void *stream);

/* Backward of the feature gather (grid_sample input gradient, bts.py:299-309):
 * dgrid_nhwc (B, Hf, Wf, C) += bilinear scatter of dx[:, :C] (row stride ldx).
 * Accumulates with f32 atomics: the caller zeroes dgrid_nhwc. */
int sd_field_gather_bwd(const float *xyz, int64_t B, int64_t P, const void *dx,
                        int32_t dx_dtype /* sd_dtype */, int64_t ldx, int32_t C, int32_t Hf,
                        int32_t Wf, const float *cam_f, float *dgrid_nhwc, void *stream);

/* NHWC f32 (B, H, W, C) -> NCHW f32 (B, C, H, W): the grid gradient of the training path
 * back in the encoder's layout (inverse of sd_pack_grid with dtype SD_F32). */
int sd_unpack_grid(const float *grid_nhwc, int64_t B, int64_t C, int64_t H, int64_t W,
                   float *grid_nchw, void *stream);

/* Backward of sd_composite (alpha compositing, nerf.py:376-405): upstream gradients
 * of depth (R), feat_out (R,F), rgb_out (R,Cc), weights (R,K), alphas (R,K) (any may be
 * NULL) -> d_sigma (R,K) and, when non-NULL, d_feat (R,K,F) / d_rgb (R,K,Cc).
 * K <= 512.  Division-free reverse transmittance recurrence (sdhip_train.hip). */
int sd_composite_bwd(const float *z, const float *sigma, const float *feat, int64_t F,
                     const float *rgb, int64_t Cc, int64_t R, int32_t K,
                     int32_t hard_alpha_cap, const float *g_depth, const float *g_feat,
                     const float *g_rgb, const float *g_weights, const float *g_alphas,
                     float *d_sigma, float *d_feat, float *d_rgb, void *stream);

/* ---- SSCBench voxel query (sdhip_seg.hip) ---------------------------------- */

/* Voxel-centre grid of nx*ny*nz voxels, flat index (ix*ny + iy)*nz + iz (meshgrid ij),
 * centre_j = f32(f64(f32 origin_j) + vox*coord_j + vox*0.5), moved by the rigid transform
 * T (rows 0..2 of a 4x4, fp64) and stored as f32 (pts_out (n, 3), device).  Bit-exact with
 * generate_point_grid -> TSDFVolume.vox2world -> rigid_transform -> .float()
 *   (sscbench/point_utils.py:17-82, sscbench/fusion.py:203-219,407-411,
 *    sscbench/evaluate_model_sscbench.py:270-278).
 * origin (3) and T (12, row-major rows 0..2) are HOST pointers read during the call. */
int sd_voxel_points(const double *origin, double vox, int64_t nx, int64_t ny, int64_t nz,
                    const double *T, float *pts_out, void *stream);

/* Folded MlpDimReduction.transform_expand + SemanticHead("stego_kmeans"), pre-packed by
 * the host into 32x32x16 MFMA fragment order (scenedino_amd/seg_pack.py documents every
 * map).  W1/W2: dim_reduction linear_in / linear_out; L = Wl W2, M = Wn1 W2 with Wl, Wn1,
 * Wn2 the StegoClusterHead 1x1 convolutions; centres = normalised cluster centres. */
typedef struct sd_seg_head {
    const void *w1;        /* bf16 [d_latent/32][d_in/16][64][8]                      */
    const float *b1;       /* [d_latent/32][2][16] accumulator-row order              */
    const void *w2;        /* bf16 [d_full/32][d_latent/16][64][8]                    */
    const float *b2;       /* [d_full/32][2][16]                                      */
    const void *wl;        /* bf16 [d_code/32][d_latent/16][64][8]  L = Wl W2         */
    const float *bl;       /* [d_code/32][2][16]  Wl b2                               */
    const float *bo;       /* [d_code/32][2][16]  bl + bn2                            */
    const void *wm;        /* bf16 [d_full/32][d_latent/16][64][8]  M = Wn1 W2        */
    const float *bm;       /* [d_full/32][2][16]  Wn1 b2                              */
    const float *bn1;      /* [d_full/32][2][16]                                      */
    const void *wn2;       /* bf16 [d_code/32][d_full/16][64][8]                      */
    const void *centres;   /* normalised centres as bf16 A fragments, hi and lo halves:
                            * [ceil(n_clusters/32)][2][d_code/16][64][8], rows = clusters
                            * (zero rows pad the last tile), permuted k order          */
    const int32_t *assign; /* [n_clusters] pseudo_assignment                           */
    int32_t n_clusters;    /* 1..256                                                   */
    int32_t d_in;          /* 64  (reduced DINO dims)                                  */
    int32_t d_latent;      /* 128                                                      */
    int32_t d_full;        /* multiple of 32 (768)                                     */
    int32_t d_code;        /* 64                                                       */
    /* optional fp8 norm product (NULL: bf16 w2).  OCP e4m3 fragments of W2 * 2^-e_w for
     * v_mfma_scale_f32_32x32x64_f8f6f4, [d_full/32][d_latent/64][64][32] bytes, k order
     * the fp8 accumulator-as-operand permutation (scenedino_amd/seg_pack.py); used for
     * |W2 h + b2| of the labels/seg outputs (dino_full keeps the bf16 w2)            */
    const void *w2_f8;
    float w2_f8_scale;     /* 2^e_w                                                    */
    int32_t pad0;
    /* the norm by the Gram form |e|^2 = h^T G h + 2 g.h + |b2|^2 (every bf16 launch):
     * G = W2^T W2 as bf16 hi + lo fragments, tile t = 16 fragments (hi k-steps 0..7,
     * lo 0..7), [d_latent/32][16][64][8], permuted k order                           */
    const void *wg;
    const float *g2;       /* [d_latent/32][2][16]  2 W2^T b2                         */
    float b2sq;            /* |b2|^2                                                   */
    /* SD_SEG_FRAG32 (0): the maps above, v_mfma_f32_32x32x16_bf16 fragments (needed by
     * the fp8 norm, w2_f8).  SD_SEG_FRAG16 (1, ABI 11, the default record): the same
     * products on v_mfma_f32_16x16x32_bf16 (lane l: row / column l & 15, k = 8 (l >> 4) + j;
     * accumulator register i of lane group g = l >> 4 holds row 4 g + i), every map with
     * 16-row tiles and 32-deep k-steps:
     *   w1 [d_latent/16][d_in/32][64][8]  W1[16 t + (l&15)][32 s + 8 (l>>4) + j]
     *   w2, wm [d_full/16][d_latent/32][64][8], wl [d_code/16][d_latent/32][64][8],
     *   wn2 [d_code/16][d_full/32][64][8]  W[16 t + (l&15)][perm16(q, l>>4, j)],
     *     perm16(q, g, j) = 32 q + 16 (j >> 2) + 4 g + (j & 3)
     *   wg [d_latent/32][16][64][8]: fragment i of tile t = G hi (i & 4 == 0) or lo of
     *     row tile 2 t + (i >> 3), k-step i & 3
     *   centres [ceil(n_clusters/16)][2][d_code/32][64][8]
     *   row vectors (b1, b2, bl, bo, bm, bn1, g2) [d/16][4][4]: vec[16 t + 4 g + i]
     * (scenedino_amd/seg_pack.py builds both)                                           */
    int32_t frag_layout;
} sd_seg_head;

#define SD_SEG_FRAG32 0
#define SD_SEG_FRAG16 1

/* Grow: out = 3x3x3 max filter of the (nx, ny, nz) f32 density grid in (z fastest),
 * F.max_pool3d(kernel_size=3, stride=1, padding=1) as evaluate_model_sscbench.py:755-756
 * applies it (NaN propagates; out-of-grid neighbours never win).  in != out,
 * nx * ny * nz < 2^31. */
int sd_grow3(const float *in, int64_t nx, int64_t ny, int64_t nz, float *out, void *stream);

/* Per-point segmentation head on P DINO codes dino (P, d_in), SD_F32 or SD_BF16 (16-B
 * aligned; the kernel's first MFMA takes them as bf16 either way).
 * Replaces BTSNet.forward(predict_segmentation=True)'s encoder.expand_dim +
 * downstream_head(..., "stego_kmeans") (bts.py:584-592, dim_reduction.py:22-25,
 * semantic_head.py:107-111,285-373) and, with seg, the SSCBench alpha-weighted class pick
 * (evaluate_model_sscbench.py:727-742, factor 1).  Outputs (device, NULL = not wanted):
 *   labels    (P) int32  pseudo_assignment[argmax_k cos(stego, c_k)]
 *   seg       (P) uint8  alpha > 0 ? label : 0, alpha = 1 - exp(-voxel_size * sigma)
 *                        (needs sigma (P) f32)
 *   dino_full (P, d_full) f32  transform_expand output (L2-normalised)
 * At least one output; labels/seg need the stego fields of h. */
int sd_seg_query(const void *dino, int32_t dino_dtype, int64_t P, const sd_seg_head *h,
                 const float *sigma, float voxel_size, int32_t *labels, uint8_t *seg,
                 float *dino_full, void *stream);

/* ---- DINO / DINOv2 ViT encoder (sdhip_vit.hip) -------------------------------
 * Replaces timm's VisionTransformer forward as the reference runs it
 * (scenedino/models/backbones/dino/vit.py:48-62,112-189 via DINOv2Encoder.forward,
 * dinov2_module.py:230-288): patch embedding, pre-LN blocks (qkv + softmax attention +
 * proj, GELU MLP, optional DINOv2 layer scale), final norm.  Residual stream fp32,
 * GEMM operands bf16, fp32 accumulation. */

enum sd_epilogue {
    SD_EPI_BF16 = 0,   /* out bf16 (M, ldo) = acc + bias                                  */
    SD_EPI_GELU = 1,   /* out bf16 = gelu_erf(acc + bias)           (timm Mlp fc1 + act)   */
    SD_EPI_F32 = 2,    /* out f32 = acc + bias                                             */
    SD_EPI_RESID = 3,  /* out f32 += gamma * (acc + bias)  (residual add, ls1/ls2 gamma)   */
    SD_EPI_QKV = 4,    /* scatter qkv columns into q (B,H,T,hd), k (B,H,Tp,hd),            */
                       /* vt (B,H,hd,Tp) bf16 (timm Attention reshape/permute)             */
    SD_EPI_PATCH = 5,  /* out f32 (B, patches+1, N): row b*(patches+1)+1+p = acc+bias+pos  */
    SD_EPI_SHUF = 6,   /* ConvTranspose2d(k, stride k): row m = input pixel (b, y, x),      */
                       /* column n = (dy k + dx) Cout + co -> out bf16 NHWC                 */
                       /* (B, in_h k, in_w k, Cout)[b, y k + dy, x k + dx, co] = acc + bias[n] */
    SD_EPI_NCHW = 7    /* out f32 NCHW (B, N, plane): row m = b * plane + p (plane = tokens) */
};

/* C = A (M, K) . W (N, K)^T (+ bias) with the epilogue above; A, W bf16 row-major
 * (W = nn.Linear weight layout), K % 32 == 0, lda % 8 == 0. */
typedef struct sd_gemm_args {
    const void *a; int64_t lda;
    const void *w;
    const float *bias;          /* (N) or NULL                                           */
    int64_t M, N, K;
    int32_t epi;
    void *out; int64_t ldo;     /* output / residual, element stride between rows        */
    const float *gamma;         /* SD_EPI_RESID layer scale (N) or NULL (= 1)            */
    void *q, *k, *vt;           /* SD_EPI_QKV destinations; SD_EPI_RESID: q (or NULL) =
                                 * a bf16 (B, tokens - 1, N) copy of the updated rows
                                 * without each image's first (class) token -- the
                                 * timm intermediate-layer grid, tokens_to_nhwc's output;
                                 * k (or NULL) = an f32 copy of the updated rows (row
                                 * stride ldo: sd_vit_mlp's LayerNorm input)              */
    int32_t tokens, heads, head_dim, tokens_pad;
    const float *pos;           /* SD_EPI_PATCH position embedding (patches+1, N)        */
    int32_t patches;
    /* residuals added by the BF16 / F32 epilogues: bf16 (M, N) row stride ldo, or NULL     */
    const void *res, *res2;
    /* implicit 3x3 convolution, padding 1 (conv != 0): a = NHWC bf16 input (B, H, W, Cin),
     * rows m = output pixels (B, OH, OW), k = (ky, kx, ci) (K = 9 Cin, Cin % 64 == 0),
     * w = (Cout, 3, 3, Cin); relu_in applies ReLU to the input as it is loaded (the
     * pre-activation of DPT's residual conv units) */
    int32_t conv, H, W, Cin, stride, OH, OW, relu_in;
    int32_t shuf_k, in_h, in_w; /* SD_EPI_SHUF geometry                                  */
} sd_gemm_args;

int sd_gemm(const sd_gemm_args *args, void *stream);

/* sd_gemm with SD_EPI_RESID, plus the LayerNorm of the updated residual rows (the next
 * block norm, timm Block norm1 / norm2, vit.py:112-189) in the same launch: ln_out (M, N)
 * bf16 = LayerNorm(N, eps) of the updated out rows, bit-equal to sd_layernorm on them.
 * The last workgroup to finish a row band normalises it (write-through residual stores,
 * a ticket per band).  ln_ws: ceil(M / 32) zeroed uint32 tickets, left zeroed (one
 * workspace per concurrently running call).  N <= 1024, N % 4 == 0; no conv. */
int sd_gemm_resid_ln(const sd_gemm_args *args, const float *ln_w, const float *ln_b, float eps,
                     void *ln_out, uint32_t *ln_ws, void *stream);

/* One ViT block's MLP half in one launch (timm Block: x = x + ls2 * (fc2(gelu(fc1(norm2(x))))),
 * scenedino/models/backbones/dino/vit.py:112-189) for C = 384: x (M, C) f32 is updated in place
 * by f32 atomics (the partial fc2 products of the 256-wide hidden chunks meet there, in arrival
 * order); x_ln (M, C) f32 is a copy of x taken before the call (sd_gemm SD_EPI_RESID writes one
 * to args->k), from which the LayerNorm (ln_w, ln_b, eps) is computed.  fc1_w (hidden, C) and
 * fc2_w (C, hidden) bf16, fc1_b (hidden), fc2_b (C) or NULL, gamma (C) layer scale or NULL.
 * hidden % 256 == 0. */
int sd_vit_mlp(const float *x_ln, float *x, int64_t M, int32_t C, int32_t hidden,
               const float *ln_w, const float *ln_b, float eps, const void *fc1_w,
               const float *fc1_b, const void *fc2_w, const float *fc2_b, const float *gamma,
               void *stream);

/* nn.LayerNorm(K, eps) fused into the prologue of a GEMM (timm Block: norm1 -> attn.qkv,
 * norm2 -> mlp.fc1, vit.py:112-189 over timm's VisionTransformer): out = EPI(LN(x) W^T + b)
 * for x (M, K) f32 rows, dense with row stride K (K = C in {384, 768}), W = args->w (N, K)
 * bf16; args->a is unused.  SD_EPI_QKV needs head_dim % 8 == 0 and tokens_pad % 8 == 0.
 * epi SD_EPI_QKV / SD_EPI_GELU / SD_EPI_BF16 with the sd_gemm fields they read.  The
 * normalised rows are the bf16 ones sd_layernorm would write (same arithmetic). */
int sd_ln_gemm(const sd_gemm_args *args, const float *x, const float *ln_w, const float *ln_b,
               float eps, void *stream);

/* softmax(q k^T * scale) v per (batch, head); q (B,H,T,64), k (B,H,Tp,64),
 * vt (B,H,64,Tp) bf16 with rows/columns T..Tp-1 zero; out (B, T, H*64) bf16. */
int sd_attention(const void *q, const void *k, const void *vt, int32_t B, int32_t heads,
                 int32_t tokens, int32_t tokens_pad, int32_t head_dim, float scale, void *out,
                 void *stream);

/* nn.LayerNorm(C, eps) over rows of x (rows, C) f32 -> out (rows, C) bf16 (out_f32 = 0,
 * the next GEMM's operand) or f32 (out_f32 = 1, the encoder's final norm). */
int sd_layernorm(const float *x, int64_t rows, int32_t C, const float *w, const float *b,
                 float eps, void *out, int32_t out_f32, void *stream);

/* The encoder's final norm into the DPT's last token grid (vit.py:188 over timm's
 * VisionTransformer.norm, then the prefix tokens dropped and the optional L2 normalisation
 * of dinov2_module.py:270-287): x (B, T, C) f32 rows -> out (B, npix, C) bf16 for tokens
 * n_prefix .. n_prefix + npix - 1 = sd_layernorm (out_f32 = 1) followed by
 * sd_tokens_to_nhwc, bit for bit, in one launch. */
int sd_layernorm_nhwc(const float *x, int32_t B, int32_t T, int32_t C, const float *w,
                      const float *b, float eps, int32_t n_prefix, int32_t npix, int32_t l2norm,
                      void *out, void *stream);

/* img (B,3,H,W) in [-1,1] -> normalised ((x/2+0.5 - mean)/std) im2col patches
 * (B*Np, Kp) bf16 (zero-padded columns >= 3 p p), and class-token rows of x (B, Np+1, C):
 * x[b,0,:] = cls + pos[0,:].  mean3/std3: HOST pointers (3). */
int sd_patchify(const float *img, int32_t B, int32_t H, int32_t W, int32_t p, int32_t Kp,
                const float *mean3, const float *std3, void *patches, const float *cls,
                const float *pos, float *x, int32_t C, void *stream);

/* x (B, T, C) f32 -> out (B, C, gh, gw): tokens n_prefix .. n_prefix+gh*gw-1 as a grid,
 * optionally L2-normalised over C (F.normalize, eps 1e-12). */
int sd_tokens_to_grid(const float *x, int32_t B, int32_t T, int32_t C, int32_t n_prefix,
                      int32_t gh, int32_t gw, int32_t l2norm, float *out, void *stream);

/* ---- DPT decoder pieces (sdhip_vit.hip; dpt_head.py:23-236) -------------------
 * The convolutions of the DPT head run through sd_gemm (1x1: plain GEMM; 3x3: conv = 1;
 * ConvTranspose2d(k, stride k): SD_EPI_SHUF; the last one writes NCHW f32 for the field
 * kernels: SD_EPI_NCHW).  Activations are NHWC bf16. */

/* x (B, T, C) f32 -> out (B, npix, C) bf16: tokens n_prefix .. n_prefix+npix-1, optionally
 * L2-normalised (the DPT inputs: ViT block outputs / normalised final tokens). */
int sd_tokens_to_nhwc(const float *x, int32_t B, int32_t T, int32_t C, int32_t n_prefix,
                      int32_t npix, int32_t l2norm, void *out, void *stream);

/* F.interpolate(scale_factor=2, mode="bilinear", align_corners=True) on NHWC bf16
 * (FeatureFusionBlock, dpt_head.py:157): in (B, H, W, C) -> out (B, 2H, 2W, C). */
int sd_upsample2x(const void *in, int32_t B, int32_t H, int32_t W, int32_t C, void *out,
                  void *stream);

/* ---- training path: fused ResnetFC MLP (sdhip_mlp.hip) ---------------------- */

/* ResnetFC(n_blocks=0) forward / backward of the training path under autocast
 * (scenedino/models/prediction_heads/resnetfc.py:135-203, bts.py:516-541 softplus,
 * scenedino/training/base_trainer.py:223,251 with_amp), on the sd_field_gather rows
 * x (N, ldx) = [feat (C) | code | 1] in dtype (SD_F16 / SD_BF16).  Fragments pre-packed by
 * the host (scenedino_amd/mlp_pack.py PackedTrainMLP documents the maps).
 * sd_mlp_train_fwd: h (N, 136) dtype = [relu(W_in x + b_in) | 1 | 0..], sigma (N) f32 =
 *   softplus(out_0), dino (N, D) f32 = out_1..D.
 * sd_mlp_train_bwd: from d_sigma (N), d_dino (N, D) f32: dy (N, 72) dtype = [d dino | d out_0
 *   | 0..], dh (N, 128) dtype = d relu-input, dx (N, lddx) dx_dtype = [dH W_in[:, :C] | 0..];
 *   the weight gradients are dh^T x and dy^T h (caller's GEMMs).  D <= 64, C % 32 == 0.
 *   Fused grid_sample backward (dgrid != NULL; replaces dx + sd_field_gather_bwd, bts.py:
 *   299-309): dX[:, :C], rounded to dtype like the autocast Linear's input gradient, is
 *   scattered with the forward gather's bilinear weights straight into the NHWC f32 grid
 *   gradient dgrid (N / P, Hf, Wf, C) (f32 atomics; the rows never reach HBM).  xyz (N, 3)
 *   are the points, P the points per encoder frame, cam_f the (N / P) encoder camera
 *   records; dx may then be NULL.  (N / P) * Hf * Wf * C < 2^31. */
typedef struct sd_mlp_train_args {
    const void *x;
    int64_t N;
    int32_t ldx, kx;       /* row length of x / dx, used columns (d_in + 1)              */
    int32_t dtype, D, C;
    int32_t lddx;          /* row length of dx (C: feature columns only; ldx: + zero columns) */
    int32_t dx_dtype;      /* SD_F32, or dtype: 16-bit dx rows (the autocast gradient dtype)  */
    int32_t pad;
    const void *w1f;       /* [4][ceil(kx/16)][64][8]  [W_in | b_in] A fragments          */
    const void *w2f;       /* [ceil((D+1)/32)][8][64][8] W_out B fragments (dino, out_0)   */
    const float *b_out;    /* (1 + D)                                                     */
    void *h;
    float *sigma, *dino;
    const float *d_sigma, *d_dino;
    const void *wtf;       /* [4][ceil((D+1)/16)][64][8] W_out^T A fragments              */
    const void *wxf;       /* [C/32][8][64][8] W_in B fragments (dX)                       */
    void *dy, *dh;
    void *dx;
    const float *xyz;      /* fused scatter (dgrid != NULL): (N, 3) points                  */
    const float *cam_f;    /* (N / P, SD_CAM_WORDS) encoder camera records                 */
    float *dgrid;          /* (N / P, Hf, Wf, C) f32, accumulated into; NULL: write dx       */
    int64_t P;
    int32_t Hf, Wf;
} sd_mlp_train_args;

/* Weight gradients of the training MLP: part[w] (Ma_pad x Nb_pad f32, pads to 32) =
 * sum over workgroup w's contiguous range of the N points of A[p]^T B[p], A (N, lda) and
 * B (N, ldb) 16-bit rows of which the first Ma / Nb columns are used (dW1 = dH^T X,
 * dW_o = dY^T [H | 1]); the caller sums the nparts partials.  Ma <= 128, Nb <= 320,
 * both multiples of 8. */
typedef struct sd_wgrad_args {
    const void *a, *b;
    int64_t N;
    int32_t lda, ldb, Ma, Nb, dtype, nparts;
    float *part;           /* (nparts, Ma_pad, Nb_pad)                                    */
} sd_wgrad_args;

int sd_wgrad(const sd_wgrad_args *args, void *stream);

/* Both weight gradients of the training MLP in one pass over the rows sd_mlp_train_fwd /
 * _bwd leave (the Linear backward of resnetfc.py:135-203 under autocast): dW1 = dh^T x
 * (x: ldx-strided rows, kx = d_in + 1 used columns, the ones column giving db_in) and
 * dW_o = dy^T [h | 1] (dy: (N, 72) = [d dino | d out_0 | 0..], h: (N, 136)).  The outputs
 * are the f32 gradients in the parameters' layout: dw_in (128, kx - 1), db_in (128),
 * dw_out (1 + D, 128) and db_out (1 + D) with row 0 = out_0 (sigma), rows 1..D = dino --
 * resnetfc.py's lin_out rows.  work: sd_mlp_train_wgrad_work(nparts) f32 of scratch for
 * the nparts partial sums (deterministic: fixed summation order).  kx <= 320, kx % 8 == 0,
 * D <= 64, D % 8 == 0. */
typedef struct sd_mlp_wgrad_args {
    const void *x, *dh, *dy, *h;
    int64_t N;
    int32_t ldx, kx, D, dtype, nparts, pad;
    float *work;
    float *dw_in, *db_in, *dw_out, *db_out;
} sd_mlp_wgrad_args;

int64_t sd_mlp_train_wgrad_work(int32_t nparts);
int sd_mlp_train_wgrad(const sd_mlp_wgrad_args *args, void *stream);

int sd_mlp_train_fwd(const sd_mlp_train_args *args, void *stream);
int sd_mlp_train_bwd(const sd_mlp_train_args *args, void *stream);

/* ---- training loss: PatchSalienceDownsampler (sdhip_down.hip) -------------- */

/* PatchSalienceDownsampler.forward_patches (scenedino/models/backbones/dino/downsampler.py:
 * 82-98): N patches of S = ph*pw feature vectors (C channels, x (N, S, C) f32): salience
 * s = w.x + b (1x1 conv), weights a = softmax(s * pw + pb) over the patch, out = sum a x,
 * L2-normalised if normalize.  sd_salience_fwd writes out (N, C), sal (N, S) and wmap (N, S)
 * (either may be NULL) and ynorm (N) (|sum a x|, needed by the backward when normalising).
 * sd_salience_bwd takes g_out (N, C) and optionally g_sal / g_wmap (N, S), reads x, out,
 * sal, wmap, ynorm, and writes gx (N, S, C) plus per-patch partial parameter gradients
 * gw_part (N, C), gpw_part / gpb_part (N, S), gb_part (N) (the caller sums over N).
 * S <= 1024, C <= 1024, C % 4 == 0; x, w, out, g_out, gx, gw_part 16-byte aligned. */
typedef struct sd_salience_args {
    const float *x;
    const float *w;        /* conv.weight (C)                                              */
    const float *b;        /* conv.bias (1, device; NULL: no bias)                          */
    const float *pw;       /* patch_weight (S)                                             */
    const float *pb;       /* patch_bias (S)                                               */
    int64_t N;
    int32_t S, C, normalize, pad;
    float *out;            /* forward output; backward input                               */
    float *sal;            /* forward output; backward input                               */
    float *wmap;           /* forward output; backward input                               */
    float *ynorm;          /* forward output; backward input                               */
    const float *g_out, *g_sal, *g_wmap;
    float *gx, *gw_part, *gpw_part, *gpb_part, *gb_part;
} sd_salience_args;

int sd_salience_fwd(const sd_salience_args *args, void *stream);
int sd_salience_bwd(const sd_salience_args *args, void *stream);

/* ---- SSCBench scoring (sdhip_ssc.hip) --------------------------------------- */

/* Camera field-of-view mask of the voxel grid (uint8 0/1, flat index as sd_voxel_points):
 * generate_point_grid's fov_mask (sscbench/point_utils.py:17-82, get_fov_mask :6-15) with
 * TSDFVolume.cam2pix (sscbench/fusion.py:222-232): fp64 camera points, pixel =
 * round-half-even(x fx / z + cx) with fx, fy, cx, cy the f32-rounded intrinsics, inside
 * [0, img_w) x [0, img_h) and z > 0.  origin (3), T (12: rows 0..2 of the 4x4) and cam_k
 * (9, row-major 3x3) are HOST pointers read during the call. */
int sd_voxel_fov(const double *origin, double vox, int64_t nx, int64_t ny, int64_t nz,
                 const double *T, const double *cam_k, int img_w, int img_h, uint8_t *fov_out,
                 void *stream);

/* Scoring configuration of sd_ssc_confusion (HOST struct, read during the call). */
typedef struct sd_ssc_args {
    float sigma_cutoff;          /* SIGMA_CUTOFF (evaluate_model_sscbench.py:57): 0.2         */
    int32_t additional_invalids; /* USE_ADDITIONAL_INVALIDS (:52)                            */
    int32_t inv_zmax;            /* identify_additional_invalids' height cut (:821): 7        */
    int32_t n_sizes;             /* evaluation ranges (SIZES, :49), at most 4                 */
    int32_t crop_x[4];           /* range s keeps x in [0, crop_x[s]) ...                     */
    int32_t crop_y0[4];          /* ... and y in [crop_y0[s], crop_y1[s]) (:496-501)          */
    int32_t crop_y1[4];
    int32_t n_pred_labels;       /* classes of the prediction (19 cityscapes classes)         */
    uint8_t pred_lut[256];       /* cityscapes_to_label (label_maps.yaml), values 0..15       */
    uint8_t target_lut[256];     /* sscbench_to_label (255 -> 255)                            */
    uint8_t target_known[256];   /* 1 where the raw target value is a key of sscbench_to_label */
    int32_t n_target_labels;     /* number of keys (informational, > 0)                       */
} sd_ssc_args;

/* One frame's SSCBench counts (evaluate_model_sscbench.py:366-367 convert_voxels,
 * :452-456 identify_additional_invalids (:814-827), :492 the density cut-off, :496-525
 * compute_occupancy_numbers / _segmentation / _recall_segmentation (:862-925)): conf
 * (n_sizes*256 + 1) uint32 on the device receives, per range s, the 16 x 16 matrix
 * conf[s][16 y_true + y_pred] over the voxels with y_true != 255 inside the FOV, and in its
 * last word the number of voxels whose label has no lookup-table entry (the reference's
 * dict lookup raises on those; the caller must too).  pred (nx,ny,nz) uint8 cityscapes
 * classes, sigma (nx,ny,nz) f32 (grown densities), target (nx,ny,nz) uint8 raw SSCBench
 * labels, fov (nx,ny,nz) uint8; all device, 16-byte aligned, nz a multiple of 16 (<= 64).
 * conf is zeroed on the stream first. */
int sd_ssc_confusion(const uint8_t *pred, const float *sigma, const uint8_t *target,
                     const uint8_t *fov, int64_t nx, int64_t ny, int64_t nz,
                     const sd_ssc_args *args, uint32_t *conf, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SDHIP_H */
