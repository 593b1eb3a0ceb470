// sdhip_ssc.hip -- SSCBench scoring on gfx950: the per-frame occupancy / semantic counts of
// sscbench/evaluate_model_sscbench.py as integer histograms on the device.
//
//   k_voxel_fov      : the camera field-of-view mask of the voxel grid
//                      (generate_point_grid's second output, point_utils.py:17-82 with
//                      TSDFVolume.cam2pix, fusion.py:222-232).  fp64 like the reference's
//                      numba loop: voxel centre (vox2world, f32 store), rigid transform in
//                      f64, pixel = round-half-even(x fx / z + cx) with the f32 intrinsics
//                      promoted to f64, inside [0, W) x [0, H) and z > 0.
//   k_ssc_confusion  : one frame's scoring pass (evaluate_model_sscbench.py:366-367,
//                      452-456, 492, 496-525): both label maps through their lookup
//                      tables (convert_voxels, :857-859; label_maps.yaml), the
//                      "additional invalids" (identify_additional_invalids, :814-827: an
//                      empty voxel below z = 7 with no labelled voxel underneath it becomes
//                      255), the density cut-off (segs[sigmas < SIGMA_CUTOFF] = 0), then the
//                      16 x 16 confusion matrix bincount(16 y_true + y_pred) over the voxels
//                      with y_true != 255 inside the FOV, once per evaluation range
//                      (12.8 / 25.6 / 51.2 m crops, :496-501).  Every count the reference
//                      keeps per frame (occupancy tp/fp/tn/fn, per-class tp/fp/tn/fn,
//                      occupancy recall) is a sum of confusion entries, formed on the host.
//
// Work unit: one thread per (x, y) voxel column, so the additional-invalid scan (a running
// count of labelled voxels along z) is a register loop; the column's bytes come in 16-B
// vector loads.  Histograms live in LDS (one 256-bin block per range + one bin counting
// labels outside the lookup tables) and are flushed with one global atomic per non-zero bin
// per workgroup.  Integer work end to end: bit-exact with the reference.
#include "sdhip_common.h"

extern "C" void sd_set_error(const char *msg);

#define SSC_MAX_SIZES 4
#define SSC_MAX_NZ 64
#define SSC_BAD 255  // lookup-table value of a label the reference's dict has no key for

struct SscConst {
    int64_t nx, ny, nz;
    float sigma_cutoff;
    int additional_invalids;
    int inv_zmax;     // identify_additional_invalids: invalids[:, :, 7:] = 0
    int n_sizes;
    int crop_x[SSC_MAX_SIZES];   // x in [0, crop_x)
    int crop_y0[SSC_MAX_SIZES];  // y in [crop_y0, crop_y1)
    int crop_y1[SSC_MAX_SIZES];
    uint8_t lut_pred[256];    // cityscapes class -> SSC label (label_maps.yaml cityscapes_to_label)
    uint8_t lut_target[256];  // SSCBench label -> SSC label (sscbench_to_label; 255 stays 255)
    uint8_t target_known[256];  // 1 if the raw target value is a key of sscbench_to_label
};

__global__ void __launch_bounds__(256) k_ssc_confusion(SscConst c, const uint8_t *__restrict__ pred,
                                                       const float *__restrict__ sigma,
                                                       const uint8_t *__restrict__ target,
                                                       const uint8_t *__restrict__ fov,
                                                       uint32_t *__restrict__ conf) {
    __shared__ uint32_t hist[SSC_MAX_SIZES * 256 + 1];
    const int nbins = c.n_sizes * 256 + 1;
    for (int i = threadIdx.x; i < nbins; i += 256) hist[i] = 0;
    __syncthreads();

    const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (col < c.nx * c.ny) {
        const int ix = (int)(col / c.ny), iy = (int)(col % c.ny);
        unsigned in_crop = 0;
        for (int s = 0; s < c.n_sizes; ++s)
            if (ix < c.crop_x[s] && iy >= c.crop_y0[s] && iy < c.crop_y1[s]) in_crop |= 1u << s;
        const int64_t base = col * c.nz;
        int seen = 0;  // labelled (not 0, not 255) voxels strictly below z
        uint32_t bad = 0;
        for (int z0 = 0; z0 < c.nz; z0 += 16) {
            const uint4 tv = *(const uint4 *)(target + base + z0);
            const uint4 pv = *(const uint4 *)(pred + base + z0);
            const uint4 fv = *(const uint4 *)(fov + base + z0);
            float sg[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)(sigma + base + z0 + 4 * q);
                sg[4 * q] = v.x; sg[4 * q + 1] = v.y; sg[4 * q + 2] = v.z; sg[4 * q + 3] = v.w;
            }
            const uint32_t tw[4] = {tv.x, tv.y, tv.z, tv.w};
            const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
            const uint32_t fw[4] = {fv.x, fv.y, fv.z, fv.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int z = z0 + j;
                const uint32_t traw = (tw[j >> 2] >> (8 * (j & 3))) & 0xff;
                const uint32_t praw = (pw[j >> 2] >> (8 * (j & 3))) & 0xff;
                const uint32_t f = (fw[j >> 2] >> (8 * (j & 3))) & 0xff;
                uint32_t t = c.lut_target[traw];
                uint32_t p = c.lut_pred[praw];
                bad += (c.target_known[traw] == 0) + (p == SSC_BAD);
                // identify_additional_invalids: the cumulative sum runs over the converted
                // target before any voxel is re-marked (:817-818)
                const int labelled = (t != 255u) & (t != 0u);
                if (c.additional_invalids && seen == 0 && z < c.inv_zmax && t == 0u) t = 255u;
                seen += labelled;
                if (sg[j] < c.sigma_cutoff) p = 0u;  // NaN keeps its class, as in numpy
                if (t != 255u && f != 0u && in_crop && t < 16u && p < 16u) {
                    const uint32_t bin = t * 16u + p;
                    for (int s = 0; s < c.n_sizes; ++s)
                        if (in_crop & (1u << s)) atomicAdd(&hist[s * 256 + bin], 1u);
                }
            }
        }
        if (bad) atomicAdd(&hist[c.n_sizes * 256], bad);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += 256) {
        const uint32_t v = hist[i];
        if (v) atomicAdd(conf + i, v);
    }
}

struct FovConst {
    double o[3];   // origin rounded to f32
    double t[12];  // rows 0..2 of the 4x4 transform
    double fx, fy, cx, cy;  // f32 intrinsics (cam2pix: intr.astype(np.float32))
    int img_w, img_h;
};

__global__ void __launch_bounds__(256) k_voxel_fov(FovConst c, double vox, int64_t nx, int64_t ny,
                                                   int64_t nz, uint8_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nx * ny * nz) return;
    const int64_t iz = i % nz;
    const int64_t q = i / nz;
    const int64_t iy = q % ny;
    const int64_t ix = q / ny;
    const double ci[3] = {(double)(float)ix, (double)(float)iy, (double)(float)iz};
    double p[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double v = c.o[j] + vox * ci[j];
        v = v + vox * 0.5;
        p[j] = (double)(float)v;  // vox2world stores f32
    }
    double cam[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double acc = c.t[4 * j] * p[0];
        acc = acc + c.t[4 * j + 1] * p[1];
        acc = acc + c.t[4 * j + 2] * p[2];
        cam[j] = acc + c.t[4 * j + 3];
    }
    // cam2pix (fusion.py:229-231): int(np.round(x fx / z + cx)); compared before the
    // integer conversion so points behind the camera cannot overflow it
    const double px = __builtin_rint(cam[0] * c.fx / cam[2] + c.cx);
    const double py = __builtin_rint(cam[1] * c.fy / cam[2] + c.cy);
    const bool in = px >= 0.0 && px < (double)c.img_w && py >= 0.0 && py < (double)c.img_h &&
                    cam[2] > 0.0;
    out[i] = in ? 1 : 0;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int sd_voxel_fov(const double *origin, double vox, int64_t nx, int64_t ny, int64_t nz,
                            const double *T, const double *cam_k, int img_w, int img_h,
                            uint8_t *fov_out, void *stream) {
    if (!origin || !T || !cam_k || !fov_out || nx <= 0 || ny <= 0 || nz <= 0 || !(vox > 0.0) ||
        img_w <= 0 || img_h <= 0 || nx * ny * nz > ((int64_t)1 << 40)) {
        sd_set_error("sd_voxel_fov: invalid argument");
        return -1;
    }
    FovConst c;
    for (int j = 0; j < 3; ++j) c.o[j] = (double)(float)origin[j];
    for (int j = 0; j < 12; ++j) c.t[j] = T[j];
    c.fx = (double)(float)cam_k[0];
    c.cx = (double)(float)cam_k[2];
    c.fy = (double)(float)cam_k[4];
    c.cy = (double)(float)cam_k[5];
    c.img_w = img_w;
    c.img_h = img_h;
    const int64_t n = nx * ny * nz;
    hipLaunchKernelGGL(k_voxel_fov, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, c, vox, nx, ny, nz, fov_out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_voxel_fov: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_ssc_confusion(const uint8_t *pred, const float *sigma, const uint8_t *target,
                                const uint8_t *fov, int64_t nx, int64_t ny, int64_t nz,
                                const sd_ssc_args *a, uint32_t *conf, void *stream) {
    if (!pred || !sigma || !target || !fov || !a || !conf || nx <= 0 || ny <= 0 || nz <= 0 ||
        nz % 16 || nz > SSC_MAX_NZ || a->n_sizes < 1 || a->n_sizes > SSC_MAX_SIZES ||
        nx * ny > ((int64_t)1 << 31) || a->n_pred_labels <= 0 || a->n_pred_labels > 255 ||
        a->n_target_labels <= 0 || a->n_target_labels > 256) {
        sd_set_error("sd_ssc_confusion: invalid argument");
        return -1;
    }
    // 16-B column loads
    if (((uintptr_t)pred | (uintptr_t)target | (uintptr_t)fov | (uintptr_t)sigma) & 15) {
        sd_set_error("sd_ssc_confusion: pred / sigma / target / fov must be 16-byte aligned");
        return -1;
    }
    SscConst c;
    c.nx = nx; c.ny = ny; c.nz = nz;
    c.sigma_cutoff = a->sigma_cutoff;
    c.additional_invalids = a->additional_invalids;
    c.inv_zmax = a->inv_zmax;
    c.n_sizes = a->n_sizes;
    for (int s = 0; s < SSC_MAX_SIZES; ++s) {
        c.crop_x[s] = s < a->n_sizes ? a->crop_x[s] : 0;
        c.crop_y0[s] = s < a->n_sizes ? a->crop_y0[s] : 0;
        c.crop_y1[s] = s < a->n_sizes ? a->crop_y1[s] : 0;
    }
    for (int v = 0; v < 256; ++v) {
        c.lut_pred[v] = v < a->n_pred_labels ? a->pred_lut[v] : SSC_BAD;
        c.lut_target[v] = a->target_lut[v];
        c.target_known[v] = a->target_known[v];
        if (c.lut_pred[v] > 15 && c.lut_pred[v] != SSC_BAD) {
            sd_set_error("sd_ssc_confusion: prediction labels must map into 0..15");
            return -1;
        }
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t nbytes = (size_t)(a->n_sizes * 256 + 1) * sizeof(uint32_t);
    if (hipMemsetAsync(conf, 0, nbytes, st) != hipSuccess) {
        sd_set_error("sd_ssc_confusion: memset failed");
        return -2;
    }
    const int64_t cols = nx * ny;
    hipLaunchKernelGGL(k_ssc_confusion, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, st, c,
                       pred, sigma, target, fov, conf);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_ssc_confusion: launch failed");
        return -2;
    }
    return 0;
}
