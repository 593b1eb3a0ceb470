// sdhip_rays.hip -- bit-exact frustum ray generation, z sampling and layout packs.
//
// sd_gen_rays : util.unproj_map (scenedino/common/util.py:113-158), util.gen_rays
//               (util.py:253-285), ImageRaySampler.sample (ray_sampler.py:439-513)
// sd_sample_z : NeRFRenderer.sample_coarse (scenedino/renderer/nerf.py:121-141)
// sd_pack_*   : NCHW -> NHWC layout steps feeding the fused gather kernels.
#include "sdhip_common.h"

// One frustum ray (11 floats) of pixel (x, y) in a W x H view: unproj_map + gen_rays +
// the frame id / NDC columns of the samplers, in the reference's fp32 operation order.
__device__ __forceinline__ void sd_ray_at(const float *__restrict__ P, const float *__restrict__ K,
                                          int64_t x, int64_t y, int64_t W, int64_t H, float xs,
                                          float xe, float ys, float ye, float z_near, float z_far,
                                          float frame_id, float *__restrict__ r) {
    float xi = sd_linspace_at(xs, xe, W, x);
    float yi = sd_linspace_at(ys, ye, H, y);
    float ux = (xi - K[2]) / K[0];
    float uy = (yi - K[5]) / K[4];
    float uz = 1.0f;
    // torch.norm over the last dim of 3: fma chain, then IEEE sqrt (verified bit-exact).
    float nrm = sqrtf(fmaf(uz, uz, fmaf(uy, uy, ux * ux)));
    ux = ux / nrm; uy = uy / nrm; uz = uz / nrm;
    r[0] = P[3]; r[1] = P[7]; r[2] = P[11];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float a = P[i * 4 + 0] * ux;
        float b = P[i * 4 + 1] * uy;
        float c = P[i * 4 + 2] * uz;
        r[3 + i] = (a + b) + c;  // 3x3 matmul: separately rounded, left to right
    }
    r[6] = z_near; r[7] = z_far; r[8] = frame_id;
    r[9] = xi; r[10] = yi;
}

// One thread per (view, pixel).  Output row = 11 floats.
__global__ void __launch_bounds__(256) k_gen_rays(const float *__restrict__ poses,
                                                  const float *__restrict__ Ks,
                                                  const float *__restrict__ frame_ids,
                                                  int64_t n_views, int64_t H, int64_t W,
                                                  float xs, float xe, float ys, float ye,
                                                  float z_near, float z_far,
                                                  float *__restrict__ rays) {
    int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t npix = H * W;
    if (gid >= n_views * npix) return;
    int64_t v = gid / npix, p = gid - v * npix;
    int64_t y = p / W, x = p - y * W;
    sd_ray_at(poses + v * 16, Ks + v * 9, x, y, W, H, xs, xe, ys, ye, z_near, z_far,
              frame_ids[v], rays + gid * 11);
}

// PatchRaySampler.sample (ray_sampler.py:171-287) for snap-to-grid patches: one thread per
// sampled ray (frame b, patch q, row py, column px).  patches (B, nq, 4) int32 holds the
// patch's view, top-left pixel (y, x) and its feature-grid cell index (row * Wd + col of
// the non-upscaled DINO target).  Writes the ray (only the sampled pixels are generated),
// the rgb target and, if requested, the per-pixel (upscaled) DINO target; the per-patch
// DINO target rows come from k_patch_dino.
__global__ void __launch_bounds__(256) k_patch_rays(const sd_patch_args a, float xs, float xe,
                                                    float ys, float ye) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t pp = (int64_t)a.ph * a.pw;
    const int64_t per_b = (int64_t)a.n_patches * pp;
    if (gid >= a.B * per_b) return;
    const int64_t b = gid / per_b, rem = gid - b * per_b;
    const int64_t q = rem / pp, pix = rem - q * pp;
    const int py = (int)(pix / a.pw), px = (int)(pix - (int64_t)py * a.pw);
    const int32_t *pt = a.patches + (b * a.n_patches + q) * 4;
    const int64_t v = pt[0], y = pt[1] + py, x = pt[2] + px;
    const int64_t bv = b * a.V + v;
    sd_ray_at(a.poses + bv * 16, a.Ks + bv * 9, x, y, a.W, a.H, xs, xe, ys, ye, a.z_near, a.z_far,
              a.frame_ids[v], a.rays + gid * 11);
    const int64_t plane = a.H * a.W;
    if (a.rgb_out) {
        const float *img = a.images + bv * a.channels * plane + y * a.W + x;
        for (int c = 0; c < a.channels; ++c) a.rgb_out[gid * a.channels + c] = img[c * plane];
    }
    if (a.dino_out && a.dino_upscaled) {  // dino (B, V, dc, H, W) at the pixel
        const float *d = a.dino + bv * (int64_t)a.dino_c * plane + y * a.W + x;
        for (int c = 0; c < a.dino_c; ++c) a.dino_out[gid * a.dino_c + c] = d[c * plane];
    }
}

// Per-patch DINO target rows (non-upscaled): one thread per (frame, patch, channel).
__global__ void __launch_bounds__(256) k_patch_dino(const sd_patch_args a) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_b = (int64_t)a.n_patches * a.dino_c;
    if (gid >= a.B * per_b) return;
    const int64_t b = gid / per_b, rem = gid - b * per_b;
    const int64_t q = rem / a.dino_c, c = rem - q * a.dino_c;
    const int32_t *pt = a.patches + (b * a.n_patches + q) * 4;
    const int64_t bv = b * a.V + pt[0];
    const int64_t dplane = (int64_t)a.dino_h * a.dino_w;
    a.dino_out[gid] = a.dino[(bv * a.dino_c + c) * dplane + pt[3]];
}

__global__ void __launch_bounds__(256) k_sample_z(const float *__restrict__ rays, int64_t R,
                                                  int64_t ray_dim, int64_t K, int lindisp,
                                                  const float *__restrict__ u, uint64_t seed,
                                                  uint64_t offset, float step, float t_end,
                                                  float *__restrict__ z) {
    int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= R * K) return;
    int64_t r = gid / K, k = gid - r * K;
    float near = rays[r * ray_dim + 6], far = rays[r * ray_dim + 7];
    // (u given: the reference's recipe, bit-exact; counter RNG: the render kernels' fast form)
    float zz = u ? sd_z_sample(near, far, K, k, u[gid], step, t_end, lindisp)
                 : sd_z_sample_rng(near, far, K, k, sd_uniform(seed, offset + (uint64_t)gid), step,
                                   t_end, lindisp);
    z[gid] = zz;
}

// NCHW f32 -> NHWC (f32 or bf16) through a 32x33 LDS tile; grid (W/32, C/32, B*H).
template <int DT>
__global__ void __launch_bounds__(256) k_pack_grid(const float *__restrict__ in, int64_t C,
                                                   int64_t H, int64_t W, void *__restrict__ out) {
    __shared__ float tile[32][33];
    int64_t bh = blockIdx.z;
    int64_t b = bh / H, y = bh - b * H;
    int64_t x0 = (int64_t)blockIdx.x * 32, c0 = (int64_t)blockIdx.y * 32;
    int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int j = ty; j < 32; j += 8) {
        int64_t c = c0 + j, x = x0 + tx;
        tile[j][tx] = (c < C && x < W) ? in[((b * C + c) * H + y) * W + x] : 0.f;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        int64_t x = x0 + j, c = c0 + tx;
        if (x < W && c < C) {
            int64_t o = ((b * H + y) * W + x) * C + c;
            float v = tile[tx][j];
            if (DT == SD_BF16)
                ((__bf16 *)out)[o] = (__bf16)v;
            else if (DT == SD_F16)
                ((_Float16 *)out)[o] = (_Float16)v;
            else
                ((float *)out)[o] = v;
        }
    }
}

// Vector variant (C % 4 == 0, W % 4 == 0): 64 channels x 64 pixels per block, 16-byte
// global loads along x and 16-byte (f32) / 8-byte (16-bit) stores along c, through a
// 64 x 65 LDS tile; grid (W/64, C/64, B*H).
template <int DT>
__global__ void __launch_bounds__(256) k_pack_grid4(const float *__restrict__ in, int64_t C,
                                                    int64_t H, int64_t W, void *__restrict__ out) {
    __shared__ float tile[64][65];
    const int64_t bh = blockIdx.z;
    const int64_t b = bh / H, y = bh - b * H;
    const int64_t x0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + 256 * k, ch = i >> 4, px = (i & 15) * 4;
        const int64_t c = c0 + ch, x = x0 + px;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (c < C && x < W) v = *(const f32x4 *)(in + ((b * C + c) * H + y) * W + x);
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[ch][px + j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + 256 * k, px = i >> 4, ch = (i & 15) * 4;
        const int64_t x = x0 + px, c = c0 + ch;
        if (x < W && c < C) {
            const int64_t o = ((b * H + y) * W + x) * C + c;
            const float v0 = tile[ch][px], v1 = tile[ch + 1][px], v2 = tile[ch + 2][px],
                        v3 = tile[ch + 3][px];
            if (DT == SD_BF16) {
                typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
                *(bf16x4 *)((__bf16 *)out + o) = bf16x4{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
            } else if (DT == SD_F16) {
                typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
                *(f16x4 *)((_Float16 *)out + o) =
                    f16x4{(_Float16)v0, (_Float16)v1, (_Float16)v2, (_Float16)v3};
            } else {
                *(f32x4 *)((float *)out + o) = f32x4{v0, v1, v2, v3};
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_pack_image(const float *__restrict__ in, int64_t N,
                                                    int64_t H, int64_t W,
                                                    float *__restrict__ out) {
    int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t hw = H * W;
    if (gid >= N * hw) return;
    int64_t n = gid / hw, p = gid - n * hw;
    const float *s = in + n * 3 * hw + p;
    f32x4 v = {s[0], s[hw], s[2 * hw], 0.f};
    *(f32x4 *)(out + gid * 4) = v;
}

// Camera records (SD_CAM_WORDS floats, include/sdhip.h) for n views; one thread per word
// (sd_cam_word, sdhip_common.h).
__global__ void __launch_bounds__(256) k_cam_records(const float *__restrict__ w2c, int64_t s_w,
                                                     const float *__restrict__ Ks, int64_t s_k,
                                                     int64_t n, float *__restrict__ out) {
    sd_cam_word(w2c, s_w, Ks, s_k, n, out, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// k_pack_image and k_cam_records in one launch (a frame's render inputs: every kernel
// boundary costs ~4-5 us at these sizes, rocprofv3): one work item per thread
// (sd_frame_item, sdhip_common.h)
__global__ void __launch_bounds__(256) k_frame_inputs(const sd_frame_args fa) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < sd_frame_items(fa)) sd_frame_item(fa, gid);
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" void sd_set_error(const char *msg);
#define SD_CHECK_LAUNCH(name)                                   \
    do {                                                        \
        hipError_t e_ = hipGetLastError();                      \
        if (e_ != hipSuccess) {                                 \
            sd_set_error(name ": launch failed");               \
            return -2;                                          \
        }                                                       \
    } while (0)

extern "C" int sd_gen_rays(const float *poses_c2w, const float *Ks, const float *frame_ids,
                           int64_t n_views, int64_t H, int64_t W, float z_near, float z_far,
                           float *rays_out, void *stream) {
    if (!poses_c2w || !Ks || !frame_ids || !rays_out || n_views <= 0 || H <= 0 || W <= 0) {
        sd_set_error("sd_gen_rays: invalid argument");
        return -1;
    }
    double pw = 2.0 / (double)W, ph = 2.0 / (double)H;
    float xs = (float)(-1.0 + 0.5 * pw), xe = (float)(1.0 - 0.5 * pw);
    float ys = (float)(-1.0 + 0.5 * ph), ye = (float)(1.0 - 0.5 * ph);
    int64_t n = n_views * H * W;
    hipLaunchKernelGGL(k_gen_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, poses_c2w, Ks, frame_ids, n_views, H, W, xs, xe, ys,
                       ye, z_near, z_far, rays_out);
    SD_CHECK_LAUNCH("sd_gen_rays");
    return 0;
}

extern "C" int sd_patch_rays(const sd_patch_args *a, void *stream) {
    if (!a || !a->poses || !a->Ks || !a->frame_ids || !a->patches || !a->rays || a->B <= 0 ||
        a->V <= 0 || a->H <= 0 || a->W <= 0 || a->ph <= 0 || a->pw <= 0 || a->n_patches <= 0 ||
        (a->rgb_out && (!a->images || a->channels <= 0)) ||
        (a->dino_out && (!a->dino || a->dino_c <= 0 ||
                         (a->dino_upscaled ? (a->dino_h != a->H || a->dino_w != a->W)
                                           : (a->dino_h <= 0 || a->dino_w <= 0))))) {
        sd_set_error("sd_patch_rays: invalid argument");
        return -1;
    }
    double pwd = 2.0 / (double)a->W, phd = 2.0 / (double)a->H;
    float xs = (float)(-1.0 + 0.5 * pwd), xe = (float)(1.0 - 0.5 * pwd);
    float ys = (float)(-1.0 + 0.5 * phd), ye = (float)(1.0 - 0.5 * phd);
    const int64_t n = a->B * a->n_patches * (int64_t)a->ph * a->pw;
    hipLaunchKernelGGL(k_patch_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *a, xs, xe, ys, ye);
    SD_CHECK_LAUNCH("sd_patch_rays");
    if (a->dino_out && !a->dino_upscaled) {
        const int64_t nd = a->B * a->n_patches * (int64_t)a->dino_c;
        hipLaunchKernelGGL(k_patch_dino, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, *a);
        SD_CHECK_LAUNCH("sd_patch_rays (dino)");
    }
    return 0;
}

// channels-last f32 grid -> the MLP dtype, same layout (4 elements per thread)
template <int DT>
__global__ void __launch_bounds__(256) k_cast_grid(const float4 *__restrict__ in, int64_t n4,
                                                   void *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 v = in[i];
    if (DT == SD_BF16) {
        typedef __attribute__((ext_vector_type(4))) __bf16 b4;
        ((b4 *)out)[i] = b4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    } else {
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        ((h4 *)out)[i] = h4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    }
}

extern "C" int sd_cast_grid(const float *grid_nhwc, int64_t n, int dtype, void *out, void *stream) {
    if (!grid_nhwc || !out || n < 0 || n % 4 || (dtype != SD_BF16 && dtype != SD_F16) ||
        (((uintptr_t)grid_nhwc | (uintptr_t)out) & 15)) {
        sd_set_error("sd_cast_grid: invalid argument (16-bit dtype, n % 4 == 0, aligned)");
        return -1;
    }
    if (n == 0) return 0;
    const int64_t n4 = n / 4;
    dim3 g((unsigned)((n4 + 255) / 256));
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_cast_grid<SD_BF16>, g, dim3(256), 0, (hipStream_t)stream,
                           (const float4 *)grid_nhwc, n4, out);
    else
        hipLaunchKernelGGL(k_cast_grid<SD_F16>, g, dim3(256), 0, (hipStream_t)stream,
                           (const float4 *)grid_nhwc, n4, out);
    SD_CHECK_LAUNCH("sd_cast_grid");
    return 0;
}

extern "C" int sd_sample_z(const float *rays, int64_t R, int64_t ray_dim, int64_t K, int lindisp,
                           const float *u, uint64_t seed, uint64_t offset, float *z_out,
                           void *stream) {
    if (!rays || !z_out || R < 0 || K <= 0 || ray_dim < 8) {
        sd_set_error("sd_sample_z: invalid argument");
        return -1;
    }
    if (R == 0) return 0;
    double step_d = 1.0 / (double)K;
    int64_t n = R * K;
    hipLaunchKernelGGL(k_sample_z, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, rays, R, ray_dim, K, lindisp, u, seed, offset,
                       (float)step_d, (float)(1.0 - step_d), z_out);
    SD_CHECK_LAUNCH("sd_sample_z");
    return 0;
}

extern "C" int sd_pack_grid(const float *grid_nchw, int64_t B, int64_t C, int64_t H, int64_t W,
                            int dtype, void *out_nhwc, void *stream) {
    if (!grid_nchw || !out_nhwc || B <= 0 || C <= 0 || H <= 0 || W <= 0 ||
        (dtype != SD_F32 && dtype != SD_BF16 && dtype != SD_F16) || B * H > 2147483647LL) {
        sd_set_error("sd_pack_grid: invalid argument");
        return -1;
    }
    if (C % 4 == 0 && W % 4 == 0 && ((uintptr_t)grid_nchw & 15) == 0 &&
        ((uintptr_t)out_nhwc & 15) == 0) {
        dim3 g4((unsigned)((W + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)(B * H));
        if (dtype == SD_BF16)
            hipLaunchKernelGGL(k_pack_grid4<SD_BF16>, g4, dim3(256), 0, (hipStream_t)stream,
                               grid_nchw, C, H, W, out_nhwc);
        else if (dtype == SD_F16)
            hipLaunchKernelGGL(k_pack_grid4<SD_F16>, g4, dim3(256), 0, (hipStream_t)stream,
                               grid_nchw, C, H, W, out_nhwc);
        else
            hipLaunchKernelGGL(k_pack_grid4<SD_F32>, g4, dim3(256), 0, (hipStream_t)stream,
                               grid_nchw, C, H, W, out_nhwc);
        SD_CHECK_LAUNCH("sd_pack_grid");
        return 0;
    }
    dim3 g((unsigned)((W + 31) / 32), (unsigned)((C + 31) / 32), (unsigned)(B * H));
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_pack_grid<SD_BF16>, g, dim3(256), 0, (hipStream_t)stream, grid_nchw,
                           C, H, W, out_nhwc);
    else if (dtype == SD_F16)
        hipLaunchKernelGGL(k_pack_grid<SD_F16>, g, dim3(256), 0, (hipStream_t)stream, grid_nchw,
                           C, H, W, out_nhwc);
    else
        hipLaunchKernelGGL(k_pack_grid<SD_F32>, g, dim3(256), 0, (hipStream_t)stream, grid_nchw,
                           C, H, W, out_nhwc);
    SD_CHECK_LAUNCH("sd_pack_grid");
    return 0;
}

extern "C" int sd_pack_image(const float *img_nchw, int64_t N, int64_t H, int64_t W,
                             float *out_nhwc4, void *stream) {
    if (!img_nchw || !out_nhwc4 || N <= 0 || H <= 0 || W <= 0) {
        sd_set_error("sd_pack_image: invalid argument");
        return -1;
    }
    int64_t n = N * H * W;
    hipLaunchKernelGGL(k_pack_image, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, img_nchw, N, H, W, out_nhwc4);
    SD_CHECK_LAUNCH("sd_pack_image");
    return 0;
}

extern "C" int sd_frame_inputs(const float *img_nchw, int64_t N, int64_t H, int64_t W,
                               float *out_nhwc4, const float *w2c, int64_t s_w, const float *Ks,
                               int64_t s_k, int64_t n, float *out_cam, void *stream) {
    if (!img_nchw || !out_nhwc4 || N <= 0 || H <= 0 || W <= 0 || !w2c || !Ks || !out_cam ||
        n <= 0 || s_w < 16 || s_k < 9) {
        sd_set_error("sd_frame_inputs: invalid argument");
        return -1;
    }
    const sd_frame_args fa = {img_nchw, N, H, W, out_nhwc4, w2c, s_w, Ks, s_k, n, out_cam};
    hipLaunchKernelGGL(k_frame_inputs, dim3((unsigned)((sd_frame_items(fa) + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, fa);
    SD_CHECK_LAUNCH("sd_frame_inputs");
    return 0;
}

extern "C" int sd_cam_records(const float *w2c, int64_t s_w, const float *Ks, int64_t s_k,
                              int64_t n, float *out, void *stream) {
    if (!w2c || !Ks || !out || n < 0 || s_w < 16 || s_k < 9) {
        sd_set_error("sd_cam_records: invalid argument");
        return -1;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_cam_records, dim3((unsigned)((n * SD_CAM_WORDS + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, w2c, s_w, Ks, s_k, n, out);
    SD_CHECK_LAUNCH("sd_cam_records");
    return 0;
}
